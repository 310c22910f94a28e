"""Replay checkpointing (crb:593-687) restated from the reference's own tests
(circular_replay_buffer_test.py:498-658, 758-800): file naming, stale-file GC,
non-array members, all-files-present load, load into the device store; plus a
PER round trip (sum tree, max priority, then identical samples)."""
import gzip
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

OBS = (5, 5)
STACK = 4
BATCH = 32


class CheckpointableClass(object):
  def __init__(self):
    self.attribute = 0


def _mem(capacity=5):
  from dopamine_amd.replay_memory.circular_replay_buffer import OutOfGraphReplayBuffer
  return OutOfGraphReplayBuffer(observation_shape=OBS, stack_size=STACK,
                                replay_capacity=capacity, batch_size=BATCH)


def test_save_writes_every_member_and_collects_stale(tmp_path):
  from dopamine_amd.replay_memory import circular_replay_buffer as crb
  memory = _mem()
  memory.observation = np.ones(10) * 1          # public members are checkpointed too
  memory.dummy_attribute_1 = 4753849
  memory.dummy_attribute_2 = 'String data'
  memory.dummy_attribute_3 = CheckpointableClass()
  current, stale = 5, 5 - crb.CHECKPOINT_DURATION
  memory.save(str(tmp_path), stale)
  names = [a for a in memory.__dict__ if not a.startswith('_')]
  names += ['$store$_' + n for n in ('observation', 'action', 'reward', 'terminal')]
  for a in names:
    assert (tmp_path / '{}_ckpt.{}.gz'.format(a, stale)).exists(), a
  memory.save(str(tmp_path), current)
  for a in names:
    assert (tmp_path / '{}_ckpt.{}.gz'.format(a, current)).exists(), a
    assert not (tmp_path / '{}_ckpt.{}.gz'.format(a, stale)).exists(), a


def test_save_into_missing_directory_is_a_no_op(tmp_path):
  _mem().save(str(tmp_path / 'absent'), 0)
  assert not (tmp_path / 'absent').exists()


def _write(tmp_path, arrays, suffix='3'):
  for attr, arr in arrays.items():
    with open(os.path.join(str(tmp_path), '{}_ckpt.{}.gz'.format(attr, suffix)), 'wb') as f:
      with gzip.GzipFile(fileobj=f, mode='wb') as out:
        np.save(out, arr, allow_pickle=False)


def _arrays(capacity=5):
  rs = np.random.RandomState(0)
  return {
      '$store$_observation': rs.randint(0, 256, (capacity,) + OBS).astype(np.uint8),
      '$store$_action': rs.randint(0, 6, capacity).astype(np.int32),
      '$store$_reward': rs.randn(capacity).astype(np.float32),
      '$store$_terminal': (rs.rand(capacity) < .3).astype(np.uint8),
      'add_count': np.array(7),
      'invalid_range': np.array([1., 2., 3., 4.]),
  }


def test_load_from_nonexistent_directory_raises_and_changes_nothing():
  from dopamine_amd.replay_memory.circular_replay_buffer import NotFoundError
  memory = _mem()
  with pytest.raises(NotFoundError, match='Missing file'):
    memory.load('/does/not/exist', '3')
  assert int(memory.add_count) == 0
  assert not memory._store['observation'].any()


def test_partial_load_fails_before_loading_anything(tmp_path):
  from dopamine_amd.replay_memory.circular_replay_buffer import NotFoundError
  memory = _mem()
  arrays = _arrays()
  del arrays['$store$_reward']
  _write(tmp_path, arrays)
  with pytest.raises(NotFoundError):
    memory.load(str(tmp_path), '3')
  assert int(memory.add_count) == 0
  assert not memory._store['observation'].any()
  assert not memory.invalid_range.any()


def test_load_fills_the_device_store(tmp_path):
  memory = _mem()
  arrays = _arrays()
  _write(tmp_path, arrays)
  memory.load(str(tmp_path), '3')
  for k in ('observation', 'action', 'reward', 'terminal'):
    np.testing.assert_array_equal(memory._store[k], arrays['$store$_' + k])
  assert int(memory.add_count) == 7
  np.testing.assert_array_equal(memory.invalid_range, arrays['invalid_range'])
  assert int(memory._read_meta().add_count) == 7       # device control block follows


def test_wrapper_save_load_round_trip(tmp_path):
  from dopamine_amd.replay_memory.circular_replay_buffer import WrappedReplayBuffer
  a = WrappedReplayBuffer(observation_shape=OBS, stack_size=STACK, replay_capacity=50,
                          batch_size=4, update_horizon=3)
  rs = np.random.RandomState(1)
  for i in range(37):
    a.add(rs.randint(0, 256, OBS).astype(np.uint8), i % 6, float(i), i % 11 == 10)
  a.save(str(tmp_path), 3)
  b = WrappedReplayBuffer(observation_shape=OBS, stack_size=STACK, replay_capacity=50,
                          batch_size=4, update_horizon=3)
  b.load(str(tmp_path), 3)
  for k in ('observation', 'action', 'reward', 'terminal'):
    np.testing.assert_array_equal(a.memory._store[k], b.memory._store[k])
  assert int(b.memory.add_count) == int(a.memory.add_count) == 49   # 37 adds + 4 x 3 padding
  np.random.seed(3)
  ia = a.memory.sample_index_batch(4)
  np.random.seed(3)
  ib = b.memory.sample_index_batch(4)
  np.testing.assert_array_equal(ia, ib)


def test_prioritized_round_trip_keeps_tree_and_samples(tmp_path):
  from dopamine_amd.replay_memory.prioritized_replay_buffer import (
      OutOfGraphPrioritizedReplayBuffer)
  kw = dict(observation_shape=OBS, stack_size=STACK, replay_capacity=100, batch_size=8,
            update_horizon=3)
  a = OutOfGraphPrioritizedReplayBuffer(**kw)
  rs = np.random.RandomState(2)
  for i in range(80):
    a.add(rs.randint(0, 256, OBS).astype(np.uint8), i % 4, 1.0, i % 17 == 16,
          float(rs.rand() * 3))
  a.set_priority(np.arange(10, 20, dtype=np.int32), np.linspace(5, 6, 10).astype(np.float32))
  a.save(str(tmp_path), 0)
  assert (tmp_path / 'sum_tree_ckpt.0.gz').exists()
  b = OutOfGraphPrioritizedReplayBuffer(**kw)
  b.load(str(tmp_path), 0)
  for la, lb in zip(a.sum_tree.nodes, b.sum_tree.nodes):
    np.testing.assert_array_equal(la, lb)
  assert b.sum_tree.max_recorded_priority == a.sum_tree.max_recorded_priority
  random.seed(11)
  sa = a.sample_index_batch(8)
  random.seed(11)
  sb = b.sample_index_batch(8)
  np.testing.assert_array_equal(sa, sb)


def test_loads_a_checkpoint_written_by_the_reference():
  """tests/golden/ckpt_uniform was written by the reference's own
  OutOfGraphReplayBuffer.save (tests/golden/gen_golden.py::gen_checkpoint); after
  load, the same np.random seed gives the reference's sample, element for element."""
  from dopamine_amd.replay_memory.circular_replay_buffer import OutOfGraphReplayBuffer
  here = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
  mem = OutOfGraphReplayBuffer(observation_shape=(6, 6), stack_size=4, replay_capacity=40,
                               batch_size=4, update_horizon=2, gamma=0.9)
  mem.load(os.path.join(here, 'ckpt_uniform'), 7)
  exp = np.load(os.path.join(here, 'ckpt_uniform_expected.npz'))
  np.random.seed(13)
  batch = mem.sample_transition_batch(batch_size=4)
  names = [e.name for e in mem.get_transition_elements(4)]
  assert set(names) == set(exp.files)
  for n, v in zip(names, batch):
    np.testing.assert_array_equal(np.asarray(v), exp[n], err_msg=n)


def test_loads_a_prioritized_checkpoint_written_by_the_reference():
  """tests/golden/ckpt_per was written by the reference's prioritized buffer (its
  `sum_tree` member is the reference's pickled SumTree); after load, the tree is the
  reference's and random.seed(17) gives the reference's sample, element for element."""
  from dopamine_amd.replay_memory.prioritized_replay_buffer import (
      OutOfGraphPrioritizedReplayBuffer)
  here = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
  mem = OutOfGraphPrioritizedReplayBuffer(observation_shape=(6, 6), stack_size=4,
                                          replay_capacity=40, batch_size=4, update_horizon=3,
                                          gamma=0.9)
  mem.load(os.path.join(here, 'ckpt_per'), 3)
  exp = np.load(os.path.join(here, 'ckpt_per_expected.npz'))
  np.testing.assert_array_equal(np.concatenate(mem.sum_tree.nodes), exp['nodes'])
  assert mem.sum_tree.max_recorded_priority == float(exp['maxrec'])
  random.seed(17)
  batch = mem.sample_transition_batch(batch_size=4)
  names = [e.name for e in mem.get_transition_elements(4)]
  for n, v in zip(names, batch):
    np.testing.assert_array_equal(np.asarray(v), exp[n], err_msg=n)
  assert random.getstate()[1] == tuple(int(x) for x in exp['rng_state'])


def test_agent_loads_a_checkpoint_saved_before_the_fc_bucket_padding(tmp_path):
  """tf_ckpt files written before the Nature-CNN flat buffers ended in the fc
  bucket's zero padding (networks.FC_BUCKET_ALIGN) load into the padded layout -- every
  tensor in the prefix, the padding zero -- and a checkpoint of another shape raises a
  ValueError that names the tensor."""
  import torch
  from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent
  mk = lambda: RainbowAgent(num_actions=9, replay_capacity=1000, batch_size=32,
                            min_replay_history=100, device=torch.device('cuda', 0))
  a = mk()
  d = str(tmp_path)
  assert a.bundle_and_checkpoint(d, 0)
  path = os.path.join(d, 'tf_ckpt-0')
  saved = torch.load(path, weights_only=True)
  n = max(o + (int(np.prod(sh)) + 3) // 4 * 4                 # the unpadded layout's length
          for o, sh in a.online_convnet.fp.offsets.values())
  assert n == a.online_convnet.fp.content_numel
  assert saved['online'].numel() > n
  old = {k: (v[:n].clone() if v.dim() == 1 and v.numel() == saved['online'].numel() else v)
         for k, v in saved.items()}
  torch.save(old, path)
  b = mk()
  b.online_convnet.fp.flat.fill_(7.0)
  assert b.unbundle(d, 0, {'training_steps': 0})
  for k in ('online', 'target'):
    got = b._ckpt_tensors()[k].cpu()
    assert torch.equal(got[:n], old[k]) and not got[n:].any()
  bad = dict(old, online=old['online'][:100])
  torch.save(bad, path)
  with pytest.raises(ValueError, match='online'):
    mk().unbundle(d, 0, {'training_steps': 0})
