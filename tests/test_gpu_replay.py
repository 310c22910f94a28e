"""Parity of the HIP replay path (through the C ABI) against the CPU oracle and
the reference-generated golden vectors.  Integer/byte/index work: bit-exact."""
import random

import numpy as np
import pytest
import torch

from oracle import replay as orc
from tests.test_oracle_golden import build_from_golden

pytestmark = pytest.mark.gpu

KEYS = ['state', 'action', 'reward', 'next_state', 'next_action', 'next_reward', 'terminal', 'indices']


def _buffers():
  from dopamine_amd.replay_memory import circular_replay_buffer as crb
  from dopamine_amd.replay_memory import prioritized_replay_buffer as prb
  return crb, prb


def _device_from_golden(z, name, prioritized, rng):
  crb, prb = _buffers()
  C, n, stack, adds, B, rounds = [int(x) for x in z[name + '_meta']]
  cls = prb.OutOfGraphPrioritizedReplayBuffer if prioritized else crb.OutOfGraphReplayBuffer
  mem = cls((8, 8), stack, C, B, update_horizon=n, gamma=float(z[name + '_gamma']), rng=rng)
  obs, act, rew, term = (z[name + k] for k in ('_obs', '_act', '_rew', '_term'))
  for i in range(adds):
    if prioritized:
      mem.add(obs[i], act[i], rew[i], term[i], z[name + '_prio_in'][i])
    else:
      mem.add(obs[i], act[i], rew[i], term[i])
  return mem, B, rounds


@pytest.mark.parametrize('prioritized', [False, True])
def test_replay_matches_reference_golden(golden, prioritized):
  z = golden('replay_per.npz' if prioritized else 'replay_uniform.npz')
  keys = KEYS + (['probs'] if prioritized else [])
  for name in [str(c) for c in z['cases']]:
    seed = int(z[name + '_seed'])
    rng = random.Random(seed) if prioritized else np.random.RandomState(seed)
    mem, B, rounds = _device_from_golden(z, name, prioritized, rng)
    assert int(mem.add_count) == int(z[name + '_add_count'])
    for r in range(rounds):
      batch = mem.sample_transition_batch()
      for k, v in zip(keys, batch):
        np.testing.assert_array_equal(v, z[name + '_' + k][r], err_msg='%s %s round %d' % (name, k, r))
      if prioritized:
        mem.set_priority(z[name + '_upd_idx'][r], z[name + '_upd_val'][r])
    if prioritized:
      np.testing.assert_array_equal(np.concatenate(mem.sum_tree.nodes), z[name + '_nodes'])
      assert mem.sum_tree.max_recorded_priority == z[name + '_maxrec']
      assert rng.getstate()[1] == tuple(int(x) for x in z[name + '_rng_state'])
    else:
      st = rng.get_state()
      np.testing.assert_array_equal(np.array(st[1], np.int64), z[name + '_rng_state'])
      assert st[2] == int(z[name + '_rng_pos'])
    fixed = [i for i in range(mem._replay_capacity) if mem.is_valid_transition(i)][:5]
    fb = mem.sample_transition_batch(batch_size=len(fixed), indices=fixed)
    for k, v in zip(keys, fb):
      np.testing.assert_array_equal(v, z[name + '_fixed_' + k])


def test_sumtree_set_matches_reference_golden(golden):
  """Ordered delta-propagating float64 updates incl. duplicates, zeros, >64 per call."""
  _, prb = _buffers()
  z = golden('sumtree.npz')
  for c in z['capacities']:
    c = int(c)
    if c < 2:
      continue
    mem = prb.OutOfGraphPrioritizedReplayBuffer((1,), 1, c, 1)
    mem.set_priority(z['c%d_set_idx' % c], z['c%d_set_val' % c])
    np.testing.assert_array_equal(np.concatenate(mem.sum_tree.nodes), z['c%d_nodes' % c])
    assert mem.sum_tree.max_recorded_priority == z['c%d_maxrec' % c]


def test_reference_kats_on_device():
  crb, prb = _buffers()
  OBS = (84, 84)
  # circular_replay_buffer_test.py:412-450  terminal inside the n-step trajectory
  m = crb.OutOfGraphReplayBuffer(OBS, 1, 10, 2, update_horizon=3, gamma=1.0)
  for i in range(10):
    m.add(np.full(OBS, i, np.uint8), i * 2, i, 1 if i == 3 else 0)
  b = m.sample_transition_batch(batch_size=3, indices=[2, 3, 4])
  np.testing.assert_array_equal(b[2], [5, 3, 15])
  np.testing.assert_array_equal(b[6], [1, 1, 0])
  np.testing.assert_array_equal(b[1], [4, 6, 8])
  np.testing.assert_array_equal(b[0][:, 0, 0, 0], [2, 3, 4])
  # 251-268  n-step sum with wraparound
  m = crb.OutOfGraphReplayBuffer(OBS, 4, 10, 32, update_horizon=5, gamma=1.0)
  for i in range(50):
    m.add(np.full(OBS, i, np.uint8), 0, 2.0, 0)
  for _ in range(5):
    assert (m.sample_transition_batch()[2] == 10.0).all()
  # 476-496  validity with episode padding
  m = crb.OutOfGraphReplayBuffer(OBS, 4, 10, 2)
  zf = np.zeros(OBS, np.uint8)
  m.add(zf, 0, 0, 0); m.add(zf, 0, 0, 0); m.add(zf, 0, 0, 1)
  assert [int(m.is_valid_transition(i)) for i in range(10)] == [0, 0, 0, 1, 1, 0, 0, 0, 0, 0]
  # too few transitions
  m = crb.OutOfGraphReplayBuffer(OBS, 4, 10, 2)
  m.add(zf, 0, 0, 0)
  with pytest.raises(RuntimeError, match='Cannot sample a batch with fewer than stack size'):
    m.sample_index_batch(2)
  # prioritized_replay_buffer_test.py: zero-priority padding, int32 asserts, empty tree
  p = prb.OutOfGraphPrioritizedReplayBuffer(OBS, 4, 10, 2)
  with pytest.raises(Exception, match='Cannot sample from an empty sum tree.'):
    p.sample_index_batch(2)
  p.add(zf, 0, 0, 0, 1.0)
  np.testing.assert_array_equal(p.get_priority(np.arange(4, dtype=np.int32)), [0, 0, 0, 1])
  with pytest.raises(AssertionError):
    p.get_priority(np.arange(4, dtype=np.int64))
  with pytest.raises(ValueError, match='nonnegative'):
    p.set_priority(np.array([1], np.int32), np.array([-1.0], np.float32))
  # retry exhaustion (prioritized_replay_buffer_test.py:127-138)
  p = prb.OutOfGraphPrioritizedReplayBuffer(OBS, 4, 10, 2, max_sample_attempts=5)
  p.add(zf, 0, 0, 0, 1.0)   # only index 3 has mass and it straddles the cursor
  with pytest.raises(RuntimeError, match='Max sample attempts'):
    p.sample_index_batch(2)
  # rainbow_agent_test.py:493-519 insertion priorities
  p = prb.OutOfGraphPrioritizedReplayBuffer(OBS, 4, 20, 2)
  for pr in (p.sum_tree.max_recorded_priority, 10.0):
    p.add(zf, 0, 0, 0, pr)
  p.add(zf, 0, 0, 0, p.sum_tree.max_recorded_priority)
  np.testing.assert_array_equal(p.get_priority(np.arange(3, 6, dtype=np.int32)), [1.0, 10.0, 10.0])


def _atari_fill(C, seed=1):
  rs = np.random.RandomState(seed)
  obs = rs.randint(0, 256, size=(C, 84 * 84), dtype=np.uint8)
  act = rs.randint(0, 9, size=C).astype(np.int32)
  rew = rs.choice(np.array([-1, 0, 1], np.float32), size=C)
  term = (rs.rand(C) < 1 / 500.).astype(np.uint8)
  return obs, act, rew, term


def test_gather_f32_normalised_matches_raw_over_255():
  """Layout F32_NORM (CNN input) == float32(raw) / 255 exactly; NCHW order."""
  _, prb = _buffers()
  C = 20000
  obs, act, rew, term = _atari_fill(C)
  m = prb.OutOfGraphPrioritizedReplayBuffer((84, 84), 4, C, 32, update_horizon=3)
  m.load_arrays(torch.from_numpy(obs).cuda(), torch.from_numpy(act), torch.from_numpy(rew),
                torch.from_numpy(term), add_count=C + 1234,
                priorities=np.random.RandomState(2).uniform(0.1, 2.0, C))
  random.seed(5)
  raw = m.sample_transition_batch()
  idx = torch.from_numpy(raw[7]).cuda()
  dev = m.sample_device(32, indices=idx)
  st = dev['state'].cpu().numpy()
  exp = np.moveaxis(raw[0], -1, 1).astype(np.float32) / np.float32(255)
  np.testing.assert_array_equal(st, exp)
  np.testing.assert_array_equal(dev['next_state'].cpu().numpy(),
                                np.moveaxis(raw[3], -1, 1).astype(np.float32) / np.float32(255))
  # NHWC layout (the reference's (B, 84, 84, 4) order, channels_last for the CNN)
  from dopamine_amd import _lib
  nh = m.sample_device(32, indices=idx, layout=_lib.LAYOUT_F32_NHWC)
  assert nh['state'].is_contiguous(memory_format=torch.channels_last)
  np.testing.assert_array_equal(nh['state'].permute(0, 2, 3, 1).cpu().numpy(),
                                raw[0].astype(np.float32) / np.float32(255))
  np.testing.assert_array_equal(nh['next_state'].permute(0, 2, 3, 1).cpu().numpy(),
                                raw[3].astype(np.float32) / np.float32(255))
  for k in ('action', 'reward', 'next_action', 'next_reward', 'terminal', 'indices',
            'sampling_probabilities'):
    np.testing.assert_array_equal(nh[k].cpu().numpy(), dev[k].cpu().numpy())
  # the oracle on the same store + indices
  o = orc.PrioritizedOracle((84, 84), 4, C, 32, update_horizon=3)
  o.observation = obs.reshape(C, 84, 84); o.action = act; o.reward = rew; o.terminal = term
  o.add_count = C + 1234
  o.invalid_range = orc.invalid_range(o.cursor(), C, 4, 3)
  ob = o.sample_transition_batch(indices=[int(i) for i in raw[7]])
  for k, a, b in zip(KEYS, raw[:8], ob[:8]):
    np.testing.assert_array_equal(a, b, err_msg=k)


def test_per_sampling_full_size_matches_oracle():
  """1M-capacity PER (the benchmark configuration's tree depth 20) with small
  frames: indices, RNG consumption and tree updates bit-exact over many steps."""
  _, prb = _buffers()
  C, B, n = 1_000_000, 32, 3
  rs = np.random.RandomState(3)
  term = (rs.rand(C) < 1 / 500.).astype(np.uint8)
  leaves = rs.uniform(0.1, 2.0, C)
  obs = np.zeros((C, 4), np.uint8)
  m = prb.OutOfGraphPrioritizedReplayBuffer((4,), 4, C, B, update_horizon=n, rng=random.Random(0))
  m.load_arrays(torch.from_numpy(obs), torch.zeros(C, dtype=torch.int32), torch.zeros(C),
                torch.from_numpy(term), add_count=C + 12345)
  t = orc.SumTree.from_leaves(C, leaves)
  m.load_tree_nodes(t.nodes, t.max_recorded_priority)
  o = orc.PrioritizedOracle((4,), 4, C, B, update_horizon=n, py_rng=random.Random(0))
  o.terminal = term
  o.add_count = C + 12345
  o.invalid_range = orc.invalid_range(o.cursor(), C, 4, n)
  o.sum_tree = t
  prng = np.random.RandomState(9)
  for step in range(40):
    got = m.sample_index_batch(B)
    exp = o.sample_index_batch(B)
    assert got == exp, 'step %d' % step
    pr = prng.uniform(0.01, 3.0, B).astype(np.float32)
    ind = np.array(got, np.int32)
    m.set_priority(ind, pr)
    o.set_priority(ind, pr)
  assert m._rng.stream.getstate() == o.py_rng.getstate()
  np.testing.assert_array_equal(m._tree.cpu().numpy(), o.sum_tree.nodes)


def test_uniform_sampling_full_size_matches_oracle():
  crb, _ = _buffers()
  C, B = 1_000_000, 32
  rs = np.random.RandomState(4)
  term = (rs.rand(C) < 1 / 50.).astype(np.uint8)   # many invalid draws
  m = crb.OutOfGraphReplayBuffer((4,), 4, C, B, rng=np.random.RandomState(7))
  m.load_arrays(torch.zeros(C, 4, dtype=torch.uint8), torch.zeros(C, dtype=torch.int32),
                torch.zeros(C), torch.from_numpy(term), add_count=C + 777)
  o = orc.ReplayOracle((4,), 4, C, B, np_rng=np.random.RandomState(7))
  o.terminal = term
  o.add_count = C + 777
  o.invalid_range = orc.invalid_range(o.cursor(), C, 4, 1)
  for step in range(30):
    assert m.sample_index_batch(B) == o.sample_index_batch(B), step
  a, b = m._rng.stream.get_state(), o.np_rng.get_state()
  np.testing.assert_array_equal(a[1], b[1])
  assert a[2] == b[2]


def test_device_fast_path_rng_accounting():
  """sample_device (async, big tape) + lazy sync == synchronous oracle stream."""
  _, prb = _buffers()
  C, B = 5000, 32
  rs = np.random.RandomState(5)
  term = (rs.rand(C) < 1 / 20.).astype(np.uint8)
  m = prb.OutOfGraphPrioritizedReplayBuffer((4,), 4, C, B, update_horizon=3,
                                            rng=random.Random(1), tape_words=1 << 14)
  m.load_arrays(torch.zeros(C, 4, dtype=torch.uint8), torch.zeros(C, dtype=torch.int32),
                torch.zeros(C), torch.from_numpy(term), add_count=C + 17,
                priorities=rs.uniform(0.1, 2, C))
  o = orc.PrioritizedOracle((4,), 4, C, B, update_horizon=3, py_rng=random.Random(1))
  o.terminal = term; o.add_count = C + 17
  o.invalid_range = orc.invalid_range(o.cursor(), C, 4, 3)
  o.sum_tree = orc.SumTree(C)
  o.sum_tree.nodes[:] = m._tree.cpu().numpy()
  seen = []
  for step in range(300):   # forces several tape refills (16k words / 2064 worst case)
    out = m.sample_device(B)
    seen.append(out['indices'].clone())
    pr = torch.rand(B, device='cuda') + 0.05
    m.set_priority(out['indices'], pr)
    exp = o.sample_index_batch(B)
    o.set_priority(np.array(exp, np.int32), pr.cpu().numpy())
    assert seen[-1].cpu().tolist() == exp, step
  m.sync_rng()
  assert m._rng.stream.getstate() == o.py_rng.getstate()


@pytest.mark.parametrize('n', [37, 150])
def test_device_set_priority_matches_host_path_and_stops_at_first_negative(n):
  """Device-tensor set_priority (the learner's path: block-parallel kernel, chunks
  of 64 updates, duplicates) leaves the same float64 tree as the host-checked path,
  and at the first negative value applies exactly the updates before it."""
  _, prb = _buffers()
  C = 5000
  rs = np.random.RandomState(n)
  idx = rs.randint(0, 60, n).astype(np.int32)          # heavy duplication
  idx[::7] = rs.randint(0, C, len(idx[::7]))
  val = rs.uniform(0.0, 3.0, n).astype(np.float32)
  for bad in (None, n // 2):
    v = val.copy()
    if bad is not None:
      v[bad] = -1.0
    trees = []
    for device in (False, True):
      p = prb.OutOfGraphPrioritizedReplayBuffer((4,), 1, C, 2)
      p.set_priority(np.arange(C, dtype=np.int32), np.full(C, 0.5, np.float32))
      if device:
        p.set_priority(torch.from_numpy(idx).cuda(), torch.from_numpy(v).cuda())
        if bad is None:
          p.sync_rng()
        else:
          with pytest.raises(ValueError, match='nonnegative'):
            p.sync_rng()
      elif bad is None:
        p.set_priority(idx, v)
      else:
        with pytest.raises(ValueError, match='nonnegative'):
          p.set_priority(idx, v)
      trees.append((np.concatenate(p.sum_tree.nodes), p.sum_tree.max_recorded_priority))
    np.testing.assert_array_equal(trees[0][0], trees[1][0])
    assert trees[0][1] == trees[1][1]
