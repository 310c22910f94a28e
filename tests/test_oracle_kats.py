"""Known-answer tests of the reference's own unit tests, restated against the
oracle (the same KATs are re-run against the HIP path in tests/test_gpu_*.py)."""
import random

import numpy as np
import pytest

from oracle import learner as L
from oracle import replay as orc

OBS = (84, 84)


# -- rainbow_agent_test.py:178-285 --------------------------------------------
PROJ_KATS = [
    ([[0, 1, 2, 3, 4]], [[0.1, 0.2, 0.1, 0.3, 0.3]], [0, 1, 2, 3, 4], [[0.1, 0.2, 0.1, 0.3, 0.3]]),
    ([[0, 1, 2, 3, 4]], [[0.1, 0.2, 0.1, 0.3, 0.3]], [3, 4, 5, 6, 7], [[0.7, 0.3, 0.0, 0.0, 0.0]]),
    ([[4, 3, 2, 1, 0]], [[0.1, 0.2, 0.1, 0.3, 0.3]], [3, 4, 5, 6, 7], [[0.9, 0.1, 0.0, 0.0, 0.0]]),
    ([[0, 2, 4, 6, 8], [1, 3, 4, 5, 6]], [[0.1, 0.6, 0.1, 0.1, 0.1], [0.1, 0.2, 0.5, 0.1, 0.1]],
     [4, 5, 6, 7, 8], [[0.8, 0.0, 0.1, 0.0, 0.1], [0.8, 0.1, 0.1, 0.0, 0.0]]),
    ([[0, 2, 4, 6, 8], [0, 1, 2, 3, 4], [3, 4, 5, 6, 7]],
     [[0.1, 0.2, 0.3, 0.2, 0.2], [0.1, 0.2, 0.1, 0.3, 0.3], [0.1, 0.2, 0.3, 0.2, 0.2]],
     [3, 4, 5, 6, 7], [[0.3, 0.3, 0.0, 0.2, 0.2], [0.7, 0.3, 0.0, 0.0, 0.0], [0.1, 0.2, 0.3, 0.2, 0.2]]),
    ([[0, 2, 4, 6, 8], [8, 9, 10, 12, 14]], [[0.1, 0.2, 0.2, 0.2, 0.3], [0.1, 0.2, 0.4, 0.1, 0.2]],
     [0, 4, 8, 12, 16], [[0.2, 0.4, 0.4, 0.0, 0.0], [0.0, 0.0, 0.45, 0.45, 0.1]]),
]


@pytest.mark.parametrize('sup,w,tgt,exp', PROJ_KATS)
def test_project_distribution_kats(sup, w, tgt, exp):
  for dt in (np.float32, np.float64):
    got = L.project_distribution(sup, w, tgt, dtype=dt)
    np.testing.assert_allclose(got, exp, atol=1e-6)


# -- sum_tree_test.py:43-154 ---------------------------------------------------
def test_sumtree_kats():
  with pytest.raises(ValueError):
    orc.SumTree(-1)
  assert len(orc.SumTree(1).levels()) == 1
  assert len(orc.SumTree(2).levels()) == 2
  t = orc.SumTree(100)
  with pytest.raises(Exception):
    t.sample()
  with pytest.raises(ValueError):
    t.set(0, -1)
  t.set(0, 1.0)
  for lvl in t.levels():
    assert lvl[0] == 1.0 and not lvl[1:].any()
  t = orc.SumTree(100)
  t.set(2, 1.0); t.set(3, 3.0)
  assert t.sample(query_value=0.1) == 2
  with pytest.raises(ValueError):
    t.sample(query_value=1.1)
  t = orc.SumTree(100)
  for i in range(32):
    t.set(i, 1)
  assert t.stratified_sample(32) == list(range(32))
  t = orc.SumTree(100)
  t.set(0, 0)
  assert t.max_recorded_priority == 1
  for i in range(1, 32):
    t.set(i, i)
    assert t.max_recorded_priority == i


# -- circular_replay_buffer_test.py --------------------------------------------
def test_invalid_range_kats():                                   # 452-474
  np.testing.assert_array_equal(orc.invalid_range(6, 10, 4, 1), [5, 6, 7, 8, 9])
  np.testing.assert_array_equal(orc.invalid_range(9, 10, 4, 1), [8, 9, 0, 1, 2])
  np.testing.assert_array_equal(orc.invalid_range(0, 10, 4, 1), [9, 0, 1, 2, 3])
  np.testing.assert_array_equal(orc.invalid_range(6, 10, 4, 3), [3, 4, 5, 6, 7, 8, 9])


def test_is_valid_transition_kat():                              # 476-496
  m = orc.ReplayOracle(OBS, 4, 10, 2)
  z = np.zeros(OBS, np.uint8)
  m.add(z, 0, 0, 0); m.add(z, 0, 0, 0); m.add(z, 0, 0, 1)
  assert [int(m.is_valid_transition(i)) for i in range(10)] == [0, 0, 0, 1, 1, 0, 0, 0, 0, 0]


def test_nstep_reward_kat():                                     # 251-268
  m = orc.ReplayOracle(OBS, 4, 10, 32, update_horizon=5, gamma=1.0)
  for i in range(50):
    m.add(np.full(OBS, i, np.uint8), 0, 2.0, 0)
  for _ in range(20):
    assert m.sample_transition_batch()[2][0] == 10.0


def test_terminal_in_trajectory_kat():                           # 412-450
  m = orc.ReplayOracle(OBS, 1, 10, 2, update_horizon=3, gamma=1.0)
  for i in range(10):
    m.add(np.full(OBS, i, np.uint8), i * 2, i, 1 if i == 3 else 0)
  b = m.sample_transition_batch(batch_size=3, indices=[2, 3, 4])
  np.testing.assert_array_equal(b[2], [5, 3, 15])
  np.testing.assert_array_equal(b[6], [1, 1, 0])
  np.testing.assert_array_equal(b[1], [4, 6, 8])


def test_get_stack_padding_kat():                                # 270-297
  m = orc.ReplayOracle(OBS, 4, 50, 32)
  for i in range(11):
    m.add(np.full(OBS, i, np.uint8), 0, 0, 0)
  assert not m.stack_at(3).any()
  s = m.stack_at(6)
  for i in range(4):
    assert (s[:, :, i] == i).all()


# -- prioritized_replay_buffer_test.py:77-157 -----------------------------------
def test_per_kats():
  m = orc.PrioritizedOracle(OBS, 4, 10, 2)
  z = np.zeros(OBS, np.uint8)
  m.add(z, 0, 0, 0, 1.0)
  # padding transitions carry priority 0, the real one its own
  np.testing.assert_array_equal(m.get_priority(np.arange(4, dtype=np.int32)), [0, 0, 0, 1])
  with pytest.raises(AssertionError):
    m.get_priority(np.arange(4, dtype=np.int64))
  # zero-priority items are never sampled
  m = orc.PrioritizedOracle(OBS, 4, 10, 2)
  for i in range(5):
    m.add(np.full(OBS, i, np.uint8), 0, 0, 0, 0.0 if i < 4 else 1.0)
  m.add(z, 0, 0, 0, 0.0)
  m.add(z, 0, 0, 0, 0.0)
  for _ in range(20):
    assert (np.array(m.sample_index_batch(2)) == 7).all()


def test_epsilon_kat():                                          # dqn_agent_test.py:297-311
  assert L.linearly_decaying_epsilon(10, 0, 10, 0.1) == 1.0
  assert L.linearly_decaying_epsilon(10, 15, 10, 0.1) == pytest.approx(0.55)
  assert L.linearly_decaying_epsilon(10, 25, 10, 0.1) == pytest.approx(0.1)


def test_c51_grad_matches_finite_difference():
  rs = np.random.RandomState(0)
  B, A, N = 4, 3, 11
  z = L.c51_support(5.0, N, np.float64)
  ol = rs.randn(B, A, N); tl = rs.randn(B, A, N)
  act = rs.randint(0, A, B); rew = rs.randn(B); term = np.array([0, 1, 0, 0])
  probs = rs.uniform(0.1, 2, B)
  out = L.c51_loss(ol, tl, act, rew, term, z, 0.9, probs)
  eps = 1e-6
  for (b, a, i) in [(0, act[0], 3), (2, act[2], 7)]:
    p = ol.copy(); p[b, a, i] += eps
    m = ol.copy(); m[b, a, i] -= eps
    fd = (L.c51_loss(p, tl, act, rew, term, z, 0.9, probs)['mean_loss'] -
          L.c51_loss(m, tl, act, rew, term, z, 0.9, probs)['mean_loss']) / (2 * eps)
    # TF's backprop is softmax - labels; labels sum to 1 after projection.
    assert abs(fd - out['grad'][b, a, i]) < 1e-6


def test_iqn_grad_matches_finite_difference():
  rs = np.random.RandomState(1)
  B, A, N, Np, K = 3, 4, 5, 6, 7
  oq = rs.randn(N * B, A); tq = rs.randn(Np * B, A); ta = rs.randn(K * B, A)
  tau = rs.rand(N * B); act = rs.randint(0, A, B); rew = rs.randn(B); term = np.array([0, 0, 1])
  out = L.iqn_loss(oq, tq, ta, tau, act, rew, term, 0.97)
  eps = 1e-6
  for r in range(0, N * B, 4):
    a = act[r % B]
    p = oq.copy(); p[r, a] += eps
    m = oq.copy(); m[r, a] -= eps
    fd = (L.iqn_loss(p, tq, ta, tau, act, rew, term, 0.97)['mean_loss'] -
          L.iqn_loss(m, tq, ta, tau, act, rew, term, 0.97)['mean_loss']) / (2 * eps)
    assert abs(fd - out['grad'][r, a]) < 1e-6
