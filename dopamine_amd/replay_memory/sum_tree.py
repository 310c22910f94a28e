"""Sum tree resident in HBM (reference sum_tree.py:30-205).

Layout: one float64 heap, level d at [2**d - 1, 2**(d+1) - 1), leaves at level
ceil(log2(capacity)) -- the reference's list of per-level arrays laid end to
end.  ``nodes`` returns that list (host copy) for inspection.

Two objects carry the reference SumTree's surface:

* ``DeviceSumTree`` -- the ``sum_tree`` member of ``OutOfGraphPrioritizedReplayBuffer``,
  a view over the buffer's heap that samples from the buffer's RNG tape;
* ``SumTree(capacity)`` -- a standalone tree (any capacity >= 1, depth 0 for 1) with its
  own heap, control block and RNG tape, as constructed by the reference's tests.

Both sample on the device (``dq_sumtree_sample``: the same float64 descent as the PER
sampler) and draw Python ``random`` words exactly as the reference does, so the indices
AND ``random``'s state afterwards equal the reference's.
"""
import ctypes
import random as _random

import numpy as np
import torch

from dopamine_amd import _lib
from dopamine_amd.replay_memory.rng_tape import RNGTape


def _draw(store, mode, n, query=None):
  """n leaf indices from dq_sumtree_sample on ``store`` (a buffer or _TreeStore)."""
  dev = store._device
  out = torch.empty((n,), dtype=torch.int64, device=dev)
  q = None
  if mode == _lib.SUMTREE_QUERY:
    q = torch.as_tensor(np.asarray(query, np.float64).reshape(n), device=dev)
  else:
    rng = store._rng
    if rng.valid:                    # words the device already used come first
      rng.sync(store._stream)
    rng.rebuild(2 * n, store._stream)
  _lib.call('dq_sumtree_sample', store._h, mode, n, _lib.ptr(q), _lib.ptr(out), store._stream)
  meta = store._read_meta()
  if mode != _lib.SUMTREE_QUERY:
    store._rng.sync(store._stream, meta)
  store._check_status(meta, n)
  return out.cpu().numpy()


class DeviceSumTree(object):
  """The reference SumTree's surface (sum_tree.py:30-205) over a device heap."""

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
    """sum_tree.py:91-97."""
    return float(self._buf._tree[0].item())

  def sample(self, query_value=None):
    """sum_tree.py:99-141."""
    if self._total_priority() == 0.0:
      raise Exception('Cannot sample from an empty sum tree.')
    if query_value and (query_value < 0. or query_value > 1.):
      raise ValueError('query_value must be in [0, 1].')
    if query_value is None:
      return int(_draw(self._buf, _lib.SUMTREE_RANDOM, 1)[0])
    return int(_draw(self._buf, _lib.SUMTREE_QUERY, 1, [query_value])[0])

  def stratified_sample(self, batch_size):
    """sum_tree.py:143-166: one random.uniform(i/B, (i+1)/B) per stratum, in order."""
    if self._total_priority() == 0.0:
      raise Exception('Cannot sample from an empty sum tree.')
    return [int(i) for i in _draw(self._buf, _lib.SUMTREE_STRATIFIED, int(batch_size))]

  def get(self, node_index):
    """sum_tree.py:168-176."""
    return float(self._buf._tree[2 ** self.depth - 1 + int(node_index)].item())

  def set(self, node_index, value):
    """sum_tree.py:178-205 with a float64 value (delta propagation, max_recorded)."""
    if value < 0.0:
      raise ValueError('Sum tree values should be nonnegative. Got {}'.format(value))
    if not 0 <= int(node_index) < 2 ** self.depth:
      raise IndexError('index {} is out of bounds for axis 0 with size {}'.format(
          node_index, 2 ** self.depth))
    buf = self._buf
    d_i = torch.tensor([int(node_index)], dtype=torch.int32, device=buf._device)
    d_v = torch.tensor([float(value)], dtype=torch.float64, device=buf._device)
    _lib.call('dq_sumtree_set_f64', buf._h, _lib.ptr(d_i), _lib.ptr(d_v), 1, buf._stream)
    torch.cuda.current_stream(buf._device).synchronize()


class _TreeStore(object):
  """Device storage + handle of a standalone sum tree (dq_sumtree_create)."""

  def __init__(self, capacity, device, rng, tape_words):
    self._device = device
    self._depth = _lib.lib.dq_sumtree_depth(capacity)
    self._tree = torch.zeros((2 ** (self._depth + 1) - 1,), dtype=torch.float64, device=device)
    self._meta = torch.zeros((16,), dtype=torch.int64, device=device)
    self._h = None
    self._capacity = capacity
    self._rng = RNGTape(self, rng, tape_words, device)
    h = ctypes.c_void_p()
    _lib.call('dq_sumtree_create', capacity, _lib.ptr(self._tree), _lib.ptr(self._meta),
              _lib.ptr(self._rng.words), self._rng.capacity, ctypes.byref(h))
    self._h = h
    _lib.call('dq_replay_set_meta', self._h, 0, 1.0, self._stream)   # max_recorded_priority = 1.0

  @property
  def _stream(self):
    return ctypes.c_void_p(torch.cuda.current_stream(self._device).cuda_stream)

  def _read_meta(self):
    m = _lib.Meta()
    _lib.call('dq_replay_read_meta', self._h, ctypes.byref(m), self._stream)
    return m

  def _check_status(self, meta, n):
    st = int(meta.status)
    if st == _lib.ST_OK:
      return
    _lib.call('dq_replay_set_meta', self._h, 0, float(meta.max_recorded_priority), self._stream)
    if st == _lib.ST_EMPTY_TREE:
      raise Exception('Cannot sample from an empty sum tree.')
    raise RuntimeError('sum tree device status %d' % st)

  def __del__(self):
    h = getattr(self, '_h', None)
    if h is not None:
      try:
        _lib.lib.dq_replay_destroy(h)
      except Exception:  # interpreter shutdown
        pass


class SumTree(DeviceSumTree):
  """A standalone device sum tree (sum_tree.py:65-89): depth ceil(log2(capacity)),
  zero-initialised levels, max_recorded_priority = 1.0.  Samples draw from Python's
  ``random`` module, as the reference's do."""

  def __init__(self, capacity, device=None, rng=None, tape_words=1 << 16):
    assert isinstance(capacity, int)
    if capacity <= 0:
      raise ValueError('Sum tree capacity should be positive. Got: {}'.format(capacity))
    if device is None:
      if not torch.cuda.is_available():
        raise RuntimeError('dopamine_amd SumTree needs a ROCm GPU (no CPU fallback)')
      device = torch.device('cuda', torch.cuda.current_device())
    super().__init__(_TreeStore(capacity, torch.device(device), rng or _random, tape_words))

  def stratified_sample(self, batch_size):
    store = self._buf
    if 2 * int(batch_size) > store._rng.capacity:    # a longer tape for this many strata
      self._grow_tape(2 * int(batch_size))
    return super().stratified_sample(batch_size)

  def _grow_tape(self, words):
    store = self._buf
    if store._rng.valid:
      store._rng.sync(store._stream)
    store._rng = RNGTape(store, store._rng.stream, words, store._device)
    _lib.lib.dq_replay_destroy(store._h)
    h = ctypes.c_void_p()        # the control block (max_recorded_priority) is kept
    _lib.call('dq_sumtree_create', store._capacity, _lib.ptr(store._tree), _lib.ptr(store._meta),
              _lib.ptr(store._rng.words), store._rng.capacity, ctypes.byref(h))
    store._h = h


class SumTreeState(object):
  """Host snapshot of a sum tree with the reference SumTree's fields (st:80-89),
  the pickled ``sum_tree`` member of a prioritized buffer checkpoint."""

  def __init__(self, nodes, max_recorded_priority):
    self.nodes = [np.asarray(n, np.float64) for n in nodes]
    self.depth = len(self.nodes) - 1
    self.max_recorded_priority = float(max_recorded_priority)
