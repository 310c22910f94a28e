"""Prioritized replay memory in HBM (reference prioritized_replay_buffer.py:36-365).

The sum tree is a flat float64 heap in device memory (see sum_tree.py); the
stratified sampler, retries, priority reads and ordered delta-propagating
priority updates are HIP kernels (dopamine_amd/csrc/replay.hip).
"""
import ctypes

import numpy as np
import torch

from dopamine_amd import _lib
from dopamine_amd.replay_memory import circular_replay_buffer
from dopamine_amd.replay_memory.circular_replay_buffer import ReplayElement
from dopamine_amd.replay_memory.sum_tree import DeviceSumTree, SumTreeState


class OutOfGraphPrioritizedReplayBuffer(circular_replay_buffer.OutOfGraphReplayBuffer):
  """prb:36-252."""

  _prioritized = True

  def _create_storage(self):
    super()._create_storage()
    depth = _lib.lib.dq_sumtree_depth(self._replay_capacity)
    self._tree = torch.zeros((2 ** (depth + 1) - 1,), dtype=torch.float64, device=self._device)
    self._depth = depth
    self.sum_tree = DeviceSumTree(self)

  def get_add_args_signature(self):
    return super().get_add_args_signature() + [ReplayElement('priority', (), np.float32)]

  def _priority_column(self, rows):
    pr = [r[-1] for r in rows]
    if any(p is circular_replay_buffer.MAX_RECORDED for p in pr):
      if len(pr) == 1:
        return circular_replay_buffer.MAX_RECORDED      # read by the add kernel itself
      m = self.sum_tree.max_recorded_priority           # padding rows too: the host value
      pr = [m if p is circular_replay_buffer.MAX_RECORDED else p for p in pr]
    return np.array(pr, dtype=np.float32)

  def get_transition_elements(self, batch_size=None):
    B = self._batch_size if batch_size is None else batch_size
    return super().get_transition_elements(batch_size) + [
        ReplayElement('sampling_probabilities', (B,), np.float32)]

  def _words_worst_case(self, batch_size):
    return 2 * (batch_size + self._max_sample_attempts)

  def set_priority(self, indices, priorities):
    """prb:203-214.  numpy inputs are checked on the host (ValueError at the
    first negative, earlier updates applied); device tensors go straight to the
    kernel and any error surfaces at the next synchronisation."""
    if isinstance(indices, torch.Tensor):
      assert indices.dtype == torch.int32, 'Indices must be integers, given: {}'.format(indices.dtype)
      n = indices.numel()
      if self._riders is not None:
        r = _lib.Rider()
        _lib.call('dq_replay_record_sumtree_set', self._h, _lib.ptr(indices),
                  _lib.ptr(priorities), n, ctypes.byref(r))
        self._riders.append(r)
        return
      _lib.call('dq_sumtree_set', self._h, _lib.ptr(indices), _lib.ptr(priorities), n, self._stream)
      return
    assert indices.dtype == np.int32, ('Indices must be integers, '
                                       'given: {}'.format(indices.dtype))
    # SumTree.set receives each priority as given (float32 from the agent, float64 from
    # a caller's float array): the float64 entry point stores both exactly
    given = np.asarray(priorities).reshape(-1)
    pr = given.astype(np.float64)
    idx = np.asarray(indices).reshape(-1)
    bad = np.nonzero(pr < 0.0)[0]
    upto = int(bad[0]) if len(bad) else len(idx)
    if upto:
      d_i = torch.from_numpy(np.ascontiguousarray(idx[:upto])).to(self._device)
      d_p = torch.from_numpy(np.ascontiguousarray(pr[:upto])).to(self._device)
      _lib.call('dq_sumtree_set_f64', self._h, _lib.ptr(d_i), _lib.ptr(d_p), upto, self._stream)
      torch.cuda.current_stream(self._device).synchronize()
    if len(bad):
      raise ValueError('Sum tree values should be nonnegative. Got {}'.format(given[upto]))

  def get_priority(self, indices):
    """prb:216-235."""
    if isinstance(indices, torch.Tensor):
      out = torch.empty(indices.shape, dtype=torch.float32, device=self._device)
      _lib.call('dq_sumtree_get', self._h, _lib.ptr(indices), indices.numel(), _lib.ptr(out), self._stream)
      return out
    assert indices.shape, 'Indices must be an array.'
    assert indices.dtype == np.int32, ('Indices must be int32s, '
                                       'given: {}'.format(indices.dtype))
    d_i = torch.from_numpy(np.ascontiguousarray(indices)).to(self._device)
    out = torch.empty((len(indices),), dtype=torch.float32, device=self._device)
    _lib.call('dq_sumtree_get', self._h, _lib.ptr(d_i), len(indices), _lib.ptr(out), self._stream)
    return out.cpu().numpy()

  def _set_tree_leaves(self, priorities):
    leaves = 2 ** self._depth
    self._tree.zero_()
    p = torch.as_tensor(priorities, dtype=torch.float64, device=self._device).reshape(-1)
    self._tree[leaves - 1:leaves - 1 + p.numel()] = p
    _lib.call('dq_sumtree_rebuild', self._h, self._stream)

  # checkpoint: the reference pickles its SumTree object (prb:98 is a public member);
  # here the member is a device view, so a SumTreeState with the reference SumTree's
  # fields (per-level ``nodes`` arrays, ``max_recorded_priority``) is pickled instead.
  def _checkpoint_value(self, attr, value):
    if attr == 'sum_tree' and isinstance(value, DeviceSumTree):
      return SumTreeState(value.nodes, value.max_recorded_priority)
    return value

  def _restore_value(self, attr, value):
    if attr == 'sum_tree':
      if isinstance(value, circular_replay_buffer._ReferenceSumTree):   # written by the reference
        value = SumTreeState(value.nodes, value.max_recorded_priority)
      if not isinstance(value, SumTreeState):
        raise ValueError('sum_tree checkpoint holds {}, expected SumTreeState'.format(type(value)))
      flat = np.concatenate([np.asarray(n, np.float64) for n in value.nodes])
      if flat.shape[0] != self._tree.numel():
        raise ValueError('sum_tree checkpoint has {} nodes, the buffer {}'.format(
            flat.shape[0], self._tree.numel()))
      self._tree.copy_(torch.from_numpy(flat))
      self._loaded_maxrec = float(value.max_recorded_priority)
      return DeviceSumTree(self)
    return value

  def _max_recorded_after_load(self):
    return getattr(self, '_loaded_maxrec', self.sum_tree.max_recorded_priority)

  def load_tree_nodes(self, nodes, max_recorded_priority):
    """Install a complete heap (e.g. an oracle-built tree) verbatim."""
    self._tree.copy_(torch.as_tensor(np.asarray(nodes, np.float64)))
    _lib.call('dq_replay_set_meta', self._h, int(self.add_count), float(max_recorded_priority),
              self._stream)


class WrappedPrioritizedReplayBuffer(circular_replay_buffer.WrappedReplayBuffer):
  """prb:255-365: the TF py_func wrappers become device calls."""

  def __init__(self,
               observation_shape,
               stack_size,
               use_staging=True,
               replay_capacity=1000000,
               batch_size=32,
               update_horizon=1,
               gamma=0.99,
               max_sample_attempts=1000,
               extra_storage_types=None,
               observation_dtype=np.uint8,
               terminal_dtype=np.uint8,
               action_shape=(),
               action_dtype=np.int32,
               reward_shape=(),
               reward_dtype=np.float32,
               device=None):
    memory = OutOfGraphPrioritizedReplayBuffer(
        observation_shape, stack_size, replay_capacity, batch_size, update_horizon, gamma,
        max_sample_attempts, extra_storage_types=extra_storage_types,
        observation_dtype=observation_dtype, terminal_dtype=terminal_dtype,
        action_shape=action_shape, action_dtype=action_dtype, reward_shape=reward_shape,
        reward_dtype=reward_dtype, device=device)
    super().__init__(observation_shape, stack_size, use_staging, replay_capacity, batch_size,
                     update_horizon, gamma, wrapped_memory=memory,
                     extra_storage_types=extra_storage_types,
                     observation_dtype=observation_dtype, terminal_dtype=terminal_dtype,
                     action_shape=action_shape, action_dtype=action_dtype,
                     reward_shape=reward_shape, reward_dtype=reward_dtype, device=device)

  def tf_set_priority(self, indices, priorities):
    """prb:338-350 -- asynchronous device update, stream-ordered after the loss."""
    return self.memory.set_priority(indices, priorities)

  def tf_get_priority(self, indices):
    """prb:352-365."""
    return self.memory.get_priority(indices)
