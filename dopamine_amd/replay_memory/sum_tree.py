"""Sum tree of a prioritized buffer, resident in HBM (reference sum_tree.py:30-205).

Layout: one float64 heap, level d at [2**d - 1, 2**(d+1) - 1), leaves at level
ceil(log2(capacity)) -- the reference's list of per-level arrays laid end to
end.  ``nodes`` returns that list (host copy) for inspection.
"""
import ctypes

import numpy as np
import torch

from dopamine_amd import _lib


class DeviceSumTree(object):
  """View over ``OutOfGraphPrioritizedReplayBuffer``'s tree with the reference
  SumTree's attribute surface (``nodes``, ``max_recorded_priority``, get/set)."""

  def __init__(self, buffer):
    self._buf = buffer

  @property
  def depth(self):
    return self._buf._depth

  @property
  def nodes(self):
    flat = self._buf._tree.cpu().numpy()
    return [flat[2 ** d - 1: 2 ** (d + 1) - 1] for d in range(self.depth + 1)]

  @property
  def max_recorded_priority(self):
    return float(self._buf._read_meta().max_recorded_priority)

  def _total_priority(self):
    return float(self._buf._tree[0].item())

  def get(self, node_index):
    return float(self._buf._tree[2 ** self.depth - 1 + int(node_index)].item())

  def set(self, node_index, value):
    self._buf.set_priority(np.array([node_index], np.int32), np.array([value], np.float32))


class SumTreeState(object):
  """Host snapshot of a sum tree with the reference SumTree's fields (st:80-89),
  the pickled ``sum_tree`` member of a prioritized buffer checkpoint."""

  def __init__(self, nodes, max_recorded_priority):
    self.nodes = [np.asarray(n, np.float64) for n in nodes]
    self.depth = len(self.nodes) - 1
    self.max_recorded_priority = float(max_recorded_priority)


def SumTree(capacity):  # noqa: N802 -- reference class name
  """A standalone device sum tree (sum_tree.py:65-89): a prioritized buffer
  with 1-byte observations whose tree is the object of interest."""
  from dopamine_amd.replay_memory.prioritized_replay_buffer import OutOfGraphPrioritizedReplayBuffer
  assert isinstance(capacity, int)
  if capacity <= 0:
    raise ValueError('Sum tree capacity should be positive. Got: {}'.format(capacity))
  buf = OutOfGraphPrioritizedReplayBuffer((1,), 1, max(capacity, 2), 1, update_horizon=1)
  return buf.sum_tree
