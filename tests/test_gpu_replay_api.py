"""The reference's replay-buffer unit tests restated on the device buffers:
circular_replay_buffer_test.py:67-350, 725-830 and prioritized_replay_buffer_test.py:
36-220, against OutOfGraph(Prioritized)ReplayBuffer / Wrapped(Prioritized)ReplayBuffer
with their store in HBM (same constructor arguments, same methods: cursor, add,
_check_add_types, get_range, get_observation_stack, sample_transition_batch,
sample_index_batch, get/set_priority, sum_tree.get, the wrapper's transition).

Deviations: the wrapper's ``transition`` is filled by ``sample()`` (device tensors)
rather than by evaluating a TF staging op; checkpoint files (testSave/testLoad/
testWrapper*) are in tests/test_gpu_checkpoint.py; the device-free checks (non-tuple
shape, low capacity, invalid_range, the wrapper's argument errors) are in
tests/test_replay_api_cpu.py; testIsTransitionValid / testSamplingWithterminalIn
Trajectory / testSampleTransitionBatchExtra are in tests/test_gpu_replay.py and
tests/test_gpu_shapes.py."""
import numpy as np
import pytest
import torch

from dopamine_amd.replay_memory import circular_replay_buffer as crb
from dopamine_amd.replay_memory import prioritized_replay_buffer as prb

pytestmark = pytest.mark.gpu

OBS, STACK, B = (84, 84), 4, 32
EXTRAS = [crb.ReplayElement('extra1', [], np.float32), crb.ReplayElement('extra2', [2], np.int8)]


# ------------------------------------------------------ circular_replay_buffer_test
def test_constructor():
  """crb-test 67-89, with a 4-byte terminal dtype stored and sampled as such."""
  m = crb.OutOfGraphReplayBuffer(observation_shape=OBS, stack_size=STACK, replay_capacity=5,
                                 batch_size=B)
  assert m._observation_shape == OBS
  m = crb.OutOfGraphReplayBuffer(observation_shape=(4, 20), stack_size=STACK, replay_capacity=5,
                                 batch_size=B)
  assert m._observation_shape == (4, 20)
  assert m.add_count == 0
  m = crb.OutOfGraphReplayBuffer(observation_shape=OBS, stack_size=STACK, terminal_dtype=np.int32,
                                 replay_capacity=5, batch_size=B)
  assert m._terminal_dtype == np.int32


def test_int32_terminals_match_uint8():
  """terminal_dtype=np.int32 (crb-test 83-90): the same samples, terminals of that dtype,
  the stored values kept (a 7 marks a terminal, and unlike a 1 does not start a padded
  episode: crb:251 compares the stored value with 1), and a checkpoint round trip."""
  def build(dt):
    m = crb.OutOfGraphReplayBuffer((4, 4), 2, 20, 8, update_horizon=3, gamma=0.9,
                                   terminal_dtype=dt, rng=np.random.RandomState(5))
    for i in range(33):
      t = 1 if i % 7 == 6 else (7 if i % 11 == 10 else 0)
      m.add(np.full((4, 4), i, np.uint8), i % 3, float(i), t)
    return m
  a, b = build(np.uint8), build(np.int32)
  assert a.add_count == b.add_count
  np.testing.assert_array_equal(b._store['terminal'], a._store['terminal'].astype(np.int32))
  assert b._store['terminal'].dtype == np.int32 and 7 in b._store['terminal']
  for _ in range(5):
    for x, y in zip(a.sample_transition_batch(), b.sample_transition_batch()):
      np.testing.assert_array_equal(x, y)
  assert b.sample_transition_batch()[6].dtype == np.int32
  np.testing.assert_array_equal(b.get_terminal_stack(9), a.get_terminal_stack(9).astype(np.int32))


def test_int32_terminals_checkpoint(tmp_path):
  m = crb.OutOfGraphReplayBuffer((4, 4), 2, 20, 8, terminal_dtype=np.int32)
  for i in range(25):
    m.add(np.full((4, 4), i, np.uint8), 0, 0.0, 7 if i == 12 else 0)
  m.save(str(tmp_path), 0)
  f = crb.OutOfGraphReplayBuffer((4, 4), 2, 20, 8, terminal_dtype=np.int32)
  f.load(str(tmp_path), 0)
  np.testing.assert_array_equal(f._store['terminal'], m._store['terminal'])
  assert [f.is_valid_transition(i) for i in range(20)] == [m.is_valid_transition(i) for i in range(20)]
  idx = [i for i in range(20) if m.is_valid_transition(i)][:4]
  for x, y in zip(m.sample_transition_batch(4, idx), f.sample_transition_batch(4, idx)):
    np.testing.assert_array_equal(x, y)


def test_add():
  """crb-test 91-101: the first add pads stack_size - 1 zero transitions."""
  m = crb.OutOfGraphReplayBuffer(OBS, STACK, 5, B)
  assert m.cursor() == 0
  m.add(np.zeros(OBS), 0, 0, 0)
  assert m.cursor() == STACK


def test_extra_add_and_check_add_types():
  """crb-test 103-137."""
  m = crb.OutOfGraphReplayBuffer(OBS, STACK, 5, B, extra_storage_types=EXTRAS)
  assert m.cursor() == 0
  zeros = np.zeros(OBS)
  m.add(zeros, 0, 0, 0, 0, [0, 0])
  with pytest.raises(ValueError, match='Add expects'):
    m.add(zeros, 0, 0, 0)
  assert m.cursor() == STACK
  m._check_add_types(zeros, 0, 0, 0, 0, [0, 0])
  with pytest.raises(ValueError, match='Add expects'):
    m._check_add_types(zeros, 0, 0, 0)
  with pytest.raises(ValueError, match='has shape'):
    m._check_add_types(zeros, 0, 0, 0, 0, [0, 0, 0])


def test_just_enough_capacity():
  """crb-test 160-166."""
  crb.OutOfGraphReplayBuffer(OBS, 5, 10, B, update_horizon=5, gamma=1.0)


def test_get_range():
  """crb-test 168-249: argument checks, then slices without and with wraparound."""
  m = crb.OutOfGraphReplayBuffer(OBS, STACK, 10, B, update_horizon=5, gamma=1.0)
  with pytest.raises(AssertionError, match='end_index must be larger than start_index'):
    m.get_range([], 2, 1)
  with pytest.raises(AssertionError):
    m.get_range([], 1, -1)
  with pytest.raises(AssertionError):
    m.get_range([], 10, 11)
  with pytest.raises(AssertionError, match='Index 1 has not been added.'):
    m.get_range([], 1, 2)
  for _ in range(10):
    m.add(np.full(OBS, 0, dtype=np.uint8), 0, 2.0, 0)
  array = np.arange(10).reshape(10, 1) + np.ones(5)
  np.testing.assert_array_equal(m.get_range(array, 2, 5), array[2:5])
  np.testing.assert_array_equal(m.get_range(array, 8, 12), np.roll(array, 2, axis=0)[:4])


def test_nstep_reward_sum():
  """crb-test 251-268: n = 5 rewards of 2 with gamma 1, over a wrapped buffer."""
  m = crb.OutOfGraphReplayBuffer(OBS, STACK, 10, B, update_horizon=5, gamma=1.0)
  for i in range(50):
    m.add(np.full(OBS, i, dtype=np.uint8), 0, 2.0, 0)
  for _ in range(100):
    assert m.sample_transition_batch()[2][0] == 10.0


def test_get_stack():
  """crb-test 270-297: shapes, the episode-start zero padding, stored contents."""
  m = crb.OutOfGraphReplayBuffer(OBS, STACK, 50, B)
  for i in range(11):
    m.add(np.full(OBS, i, dtype=np.uint8), 0, 0, 0)
  for i in range(3, m.cursor()):
    assert m.get_observation_stack(i).shape == OBS + (4,)
  np.testing.assert_array_equal(m.get_observation_stack(3), np.zeros(OBS + (4,), np.uint8))
  stack = m.get_observation_stack(6)
  for i in range(4):
    np.testing.assert_array_equal(stack[:, :, i], np.full(OBS, i))


def test_sample_transition_batch():
  """crb-test 299-350: default / changed / reverted batch sizes, then given indices
  over a wrapped buffer with every fourth transition terminal."""
  C, num_adds = 10, 50
  m = crb.OutOfGraphReplayBuffer(OBS, 1, C, 2)
  for i in range(num_adds):
    m.add(np.full(OBS, i, np.uint8), 0, 0, i % 4)
  for bs, n in ((None, 200), (B, 200), (None, 200)):
    for _ in range(n):
      assert m.sample_transition_batch(bs)[0].shape[0] == (2 if bs is None else bs)
  indices = [1, 2, 3, 5, 8]
  expected_states = np.array([np.full(OBS + (1,), i, dtype=np.uint8) for i in indices])
  expected_next_states = (expected_states + 1) % C
  expected_states += num_adds - C
  expected_next_states += num_adds - C
  expected_terminal = np.array([min((x + num_adds - C) % 4, 1) for x in indices])
  (states, action, reward, next_states, next_action, next_reward, terminal,
   indices_batch) = m.sample_transition_batch(batch_size=len(indices), indices=indices)
  np.testing.assert_array_equal(states, expected_states)
  np.testing.assert_array_equal(action, np.zeros(len(indices)))
  np.testing.assert_array_equal(reward, np.zeros(len(indices)))
  np.testing.assert_array_equal(next_action, np.zeros(len(indices)))
  np.testing.assert_array_equal(next_reward, np.zeros(len(indices)))
  np.testing.assert_array_equal(next_states, expected_next_states)
  np.testing.assert_array_equal(terminal, expected_terminal)
  np.testing.assert_array_equal(indices_batch, indices)


def _verify_sampled_trajectories(t):
  """crb-test 694-723 on the wrapper's device transition."""
  mid = np.full((B,) + OBS + (STACK,), B, dtype=np.float64)
  # the wrapper hands the CNN float32 stacks already divided by 255 (NCHW view)
  states = t['state'].permute(0, 2, 3, 1).cpu().numpy().astype(np.float64) * 255.0
  next_states = t['next_state'].permute(0, 2, 3, 1).cpu().numpy().astype(np.float64) * 255.0
  np.testing.assert_allclose(states, mid, rtol=B)
  np.testing.assert_allclose(next_states, mid, rtol=B)
  np.testing.assert_allclose(t['action'].cpu().numpy(), np.ones(B) * 2)
  np.testing.assert_allclose(t['reward'].cpu().numpy(), np.ones(B))
  np.testing.assert_allclose(t['next_action'].cpu().numpy(), np.ones(B) * 2)
  np.testing.assert_allclose(t['next_reward'].cpu().numpy(), np.ones(B))
  np.testing.assert_allclose(t['terminal'].cpu().numpy(), np.zeros(B))
  np.testing.assert_allclose(t['indices'].cpu().numpy(), np.ones(B) * B, rtol=B)


@pytest.mark.parametrize('staging', [False, True])
def test_wrapper_sampling(staging):
  """crb-test 725-756: before any add, sampling raises; after 2B adds the transition
  holds a batch of them (staging is accepted and changes nothing on the device)."""
  replay = crb.WrappedReplayBuffer(observation_shape=OBS, stack_size=STACK, replay_capacity=100,
                                   batch_size=B, use_staging=staging)
  with pytest.raises(RuntimeError, match='Cannot sample a batch with fewer than stack size'):
    replay.sample()
  for i in range(B * 2):
    replay.add(np.full(OBS, i, dtype=np.uint8), 2, 1, 0)
  _verify_sampled_trajectories(replay.sample())


def test_wrapper_with_extra_storage_types():
  """crb-test 692-700 (+ prb-test 206-216)."""
  crb.WrappedReplayBuffer(observation_shape=OBS, stack_size=STACK, replay_capacity=1000,
                          extra_storage_types=EXTRAS)
  prb.OutOfGraphPrioritizedReplayBuffer(OBS, STACK, 100, B, extra_storage_types=EXTRAS)


def test_observation_dtypes():
  """crb-test 813-827."""
  r = crb.WrappedReplayBuffer(observation_shape=OBS, stack_size=STACK, replay_capacity=10)
  assert r.memory._store['observation'].dtype == np.uint8
  r = crb.WrappedReplayBuffer(observation_shape=OBS, stack_size=STACK, replay_capacity=10,
                              observation_dtype=np.int32)
  assert r.memory._store['observation'].dtype == np.int32


# -------------------------------------------------- prioritized_replay_buffer_test
C = 100


def _per(**kw):
  kw.setdefault('max_sample_attempts', 10)
  return prb.OutOfGraphPrioritizedReplayBuffer(OBS, STACK, C, B, **kw)


def _add_blank(m, action=0, reward=0.0, terminal=0, priority=1.0):
  m.add(np.zeros(OBS), action, reward, terminal, priority)
  return (m.cursor() - 1) % C


def test_add_with_and_without_priority():
  """prb-test 63-75."""
  m = _per()
  assert m.cursor() == 0
  _add_blank(m)
  assert m.cursor() == STACK and m.add_count == STACK
  with pytest.raises(ValueError, match='Add expects'):
    m.add(np.zeros(OBS), 0, 0, 0)


def test_dummy_screens_have_zero_priority():
  """prb-test 77-81."""
  m = _per()
  index = _add_blank(m)
  for i in range(index):
    assert m.sum_tree.get(i) == 0.0


def test_get_priority_with_invalid_indices():
  """prb-test 83-90."""
  m = _per()
  index = _add_blank(m)
  with pytest.raises(AssertionError):
    m.get_priority(index)
  with pytest.raises(AssertionError):
    m.get_priority(np.array([index]))


def test_set_and_get_priority():
  """prb-test 92-104 and (the wrapper's tf_* entry points) 176-193."""
  m = _per()
  indices = np.array([_add_blank(m) for _ in range(7)], dtype=np.int32)
  priorities = np.arange(7)
  m.set_priority(indices, priorities)
  fetched = m.get_priority(np.flip(indices, 0))
  for i in range(7):
    assert priorities[i] == fetched[6 - i]
  w = prb.WrappedPrioritizedReplayBuffer(OBS, STACK, use_staging=False, replay_capacity=C,
                                         batch_size=B, max_sample_attempts=10)
  idx = np.zeros(7, dtype=np.int32)
  for i in range(7):
    w.add(np.zeros(OBS), 0, 0, 0, 1.0)
    idx[i] = w.memory.cursor() - 1
  w.tf_set_priority(idx, priorities)
  fetched = w.tf_get_priority(np.flip(idx, 0))
  for i in range(7):
    assert priorities[i] == fetched[6 - i]


def test_new_element_has_high_priority():
  """prb-test 106-111."""
  m = _per()
  index = _add_blank(m)
  assert m.get_priority(np.array([index], dtype=np.int32))[0] == 1.0


def test_low_priority_element_not_sampled():
  """prb-test 113-125."""
  m = _per()
  _add_blank(m, terminal=0, priority=0.0)
  for _ in range(3):
    _add_blank(m, terminal=1)
  for _ in range(100):
    terminals = m.sample_transition_batch(batch_size=2)[6]
    assert (terminals == 1).all()


def test_too_many_failed_retries():
  """prb-test 127-138."""
  m = _per()
  _add_blank(m)
  with pytest.raises(RuntimeError, match='Max sample attempts: Tried 10 times but only '
                                         'sampled 1 valid indices. Batch size is 2'):
    m.sample_index_batch(2)


def test_sample_index_batch_respects_invalid_range():
  """prb-test 140-157: cursor == 1, so indices 0..3 are invalid."""
  m = _per(max_sample_attempts=C)
  for _ in range(C - STACK + 2):
    _add_blank(m)
  assert m.cursor() == 1
  for s in m.sample_index_batch(C):
    assert STACK <= s <= C - 1


def test_wrapper_sample_batch_probabilities():
  """prb-test 195-204: equal priorities -> every sampling probability is 1."""
  w = prb.WrappedPrioritizedReplayBuffer(OBS, STACK, use_staging=False, replay_capacity=C,
                                         batch_size=B, max_sample_attempts=10)
  for _ in range(64):
    w.add(np.zeros(OBS), 0, 0, 0, 1.0)
  probs = w.sample()['sampling_probabilities'].cpu().numpy()
  assert probs.shape == (B,) and (probs == 1.0).all()
