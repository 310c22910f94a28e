"""The standalone device SumTree (dopamine_amd.replay_memory.sum_tree.SumTree) and a
prioritized buffer's ``sum_tree`` view, against the reference's own outputs
(tests/golden/sumtree.npz, made by gen_golden.py from the reference's sum_tree.py)
and the reference's unit tests (tests/dopamine/replay_memory/sum_tree_test.py:30-154),
restated on the device.  Loop counts of the reference's 10,000-iteration checks are
reduced (each device sample synchronises); the assertions are the same."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _st():
  from dopamine_amd.replay_memory import sum_tree
  return sum_tree


def _check_tree_against_golden(tree, z, c):
  for i, v in zip(z['c%d_set_idx' % c], z['c%d_set_val' % c]):
    tree.set(int(i), v)                 # one call per update, as the reference's loop
  np.testing.assert_array_equal(np.concatenate(tree.nodes), z['c%d_nodes' % c])
  assert tree.max_recorded_priority == z['c%d_maxrec' % c]
  for b in (1, 7, 32):
    random.seed(1000 + c + b)
    assert tree.stratified_sample(b) == list(z['c%d_strat%d' % (c, b)])
    assert random.getstate()[1] == tuple(int(x) for x in z['c%d_strat%d_state' % (c, b)])
  random.seed(99 + c)
  assert [tree.sample() for _ in range(10)] == list(z['c%d_single' % c])
  assert [tree.sample(query_value=q) for q in (0.0, 0.25, 0.5, 0.999, 1.0)] == list(z['c%d_query' % c])


@pytest.mark.parametrize('c', [1, 2, 3, 5, 100, 1000, 1025, 4096])
def test_standalone_sumtree_matches_reference_golden(golden, c):
  """Every golden capacity incl. 1 (depth 0): heaps after the reference's set
  sequence, stratified / single / query samples and Python's random state."""
  z = golden('sumtree.npz')
  tree = _st().SumTree(c)
  assert tree.depth == int(np.ceil(np.log2(c)))
  assert len(tree.nodes) == tree.depth + 1
  _check_tree_against_golden(tree, z, c)


@pytest.mark.parametrize('c', [2, 100, 1025])
def test_buffer_sumtree_view_matches_reference_golden(golden, c):
  """The same surface on a prioritized buffer's ``sum_tree`` member (its own handle,
  heap and RNG tape over Python's random)."""
  from dopamine_amd.replay_memory.prioritized_replay_buffer import OutOfGraphPrioritizedReplayBuffer
  z = golden('sumtree.npz')
  mem = OutOfGraphPrioritizedReplayBuffer((1,), 1, c, 1)
  _check_tree_against_golden(mem.sum_tree, z, c)


def test_reference_sum_tree_unit_tests_on_device():
  st = _st()
  with pytest.raises(ValueError, match='Sum tree capacity should be positive. Got: -1'):
    st.SumTree(capacity=-1)
  tree = st.SumTree(capacity=100)
  with pytest.raises(ValueError, match='Sum tree values should be nonnegative. Got -1'):
    tree.set(node_index=0, value=-1)
  assert len(st.SumTree(capacity=1).nodes) == 1           # testSmallCapacityConstructor
  assert len(st.SumTree(capacity=2).nodes) == 2
  t1 = st.SumTree(capacity=1)                              # testSetValueSmallCapacity
  t1.set(0, 1.5)
  assert t1.get(0) == 1.5
  tree.set(node_index=0, value=1.0)                        # testSetValue
  assert tree.get(0) == 1.0
  for level in tree.nodes:
    assert level[0] == 1.0 and (level[1:] == 0.0).all()
  assert len(tree.nodes[-1]) >= 100                        # testCapacityGreaterThanRequested

  empty = st.SumTree(capacity=100)
  with pytest.raises(Exception, match='Cannot sample from an empty sum tree.'):
    empty.sample()
  with pytest.raises(Exception, match='Cannot sample from an empty sum tree.'):
    empty.stratified_sample(5)

  t = st.SumTree(capacity=100)
  t.set(node_index=5, value=1.0)
  with pytest.raises(ValueError, match=r'query_value must be in \[0, 1\].'):
    t.sample(query_value=-0.1)
  with pytest.raises(ValueError, match=r'query_value must be in \[0, 1\].'):
    t.sample(query_value=1.1)
  assert t.sample() == 5                                   # testSampleSingleton

  t = st.SumTree(capacity=100)                             # uneven pair
  t.set(node_index=2, value=1.0)
  t.set(node_index=3, value=3.0)
  for _ in range(100):
    random.seed(1)
    assert t.sample() == 2
    assert t.sample(query_value=0.1) == 2

  t = st.SumTree(capacity=100)                             # testSamplingWithSeedDoesNotAffectFutureCalls
  seed = 1
  random.seed(seed)
  r = random.random()
  max_value, delta = 100, 0.01
  total_value = max_value / (1 - r - delta)
  t.set(node_index=2, value=r * total_value + delta)
  t.set(node_index=3, value=max_value)
  for _ in range(100):
    random.seed(seed)
    assert t.sample() == 2
  counts = {2: 0, 3: 0}
  for _ in range(300):
    counts[t.sample()] += 1
  assert counts[2] < counts[3]

  t = st.SumTree(capacity=100)                             # testStratifiedSampling
  for i in range(32):
    t.set(node_index=i, value=1)
  assert t.stratified_sample(32) == list(range(32))

  t = st.SumTree(capacity=100)                             # testMaxRecordedProbability
  t.set(node_index=0, value=0)
  assert t.max_recorded_priority == 1
  for i in range(1, 32):
    t.set(node_index=i, value=i)
    assert t.max_recorded_priority == i


def test_stratified_sample_larger_than_the_tape():
  """More strata than the initial tape holds (the tape grows; draws stay in order)."""
  st = _st()
  from oracle import replay as OR
  t = st.SumTree(capacity=5000, tape_words=256)
  ref = OR.SumTree(5000)
  rs = np.random.RandomState(3)
  for i, v in zip(rs.randint(0, 5000, 3000), rs.uniform(0, 2, 3000)):
    t.set(int(i), float(v))
    ref.set(int(i), float(v))
  np.testing.assert_array_equal(np.concatenate(t.nodes), ref.nodes)
  random.seed(4)
  got = t.stratified_sample(1000)
  s1 = random.getstate()
  random.seed(4)
  exp = ref.stratified_sample(1000)
  assert got == [int(x) for x in exp]
  assert random.getstate() == s1


def test_host_sampling_after_device_sampling_continues_the_stream():
  """sample_index_batch after sample_device (no explicit sync_rng): the host draw
  follows the device's words -- no duplicate draws, and Python's random ends where
  the reference's sequential calls leave it."""
  from dopamine_amd.replay_memory.prioritized_replay_buffer import OutOfGraphPrioritizedReplayBuffer
  from oracle import replay as OR
  rs = np.random.RandomState(0)
  C, B = 400, 8
  mem = OutOfGraphPrioritizedReplayBuffer((4, 4), 4, C, B, update_horizon=3, rng=random.Random(5))
  ref = OR.PrioritizedOracle((4, 4), 4, C, B, update_horizon=3, py_rng=random.Random(5))
  for _ in range(600):
    o = rs.randint(0, 256, (4, 4)).astype(np.uint8)
    a, r, t, p = int(rs.randint(4)), np.float32(rs.randn()), int(rs.rand() < .05), np.float32(rs.rand() + .1)
    mem.add(o, a, r, t, p)
    ref.add(o, a, r, t, p)
  d = mem.sample_device(B)
  first = d['indices'].cpu().numpy()
  second = mem.sample_index_batch(B)
  np.testing.assert_array_equal(first, ref.sample_index_batch(B))
  assert second == [int(i) for i in ref.sample_index_batch(B)]
  assert mem._rng.stream.getstate() == ref.py_rng.getstate()
