"""Device-resident RNG tape that continues a host MT19937 stream word for word.

The reference draws its sampling randomness from two host streams:

* the prioritized sampler uses Python's global ``random`` module
  (sum_tree.py:123 ``random.random()``, sum_tree.py:165 ``random.uniform``);
* the uniform sampler uses numpy's legacy global ``np.random``
  (circular_replay_buffer.py:466 ``np.random.randint``).

Both are MT19937.  ``random.random()`` consumes exactly two 32-bit words
(genrand_res53) and legacy ``randint`` consumes whole 32-bit words through
masked rejection, so the raw word sequence fully determines every draw.  This
class copies the *next* W raw words of the host stream onto the device; the
sampling kernels consume them and advance ``meta.tape_pos``.  At a
synchronisation point the host stream is advanced by exactly the number of
words the device consumed, so the Python/numpy RNG state is identical to the
reference's after the same calls -- including the data-dependent retries.
"""
import ctypes
import random as _random

import numpy as np
import torch

from dopamine_amd import _lib


def _np_state_of(stream):
  """(keys uint32[624], pos) of a Python Random or numpy RandomState."""
  if isinstance(stream, np.random.RandomState) or stream is np.random:
    st = stream.get_state()
    return np.asarray(st[1], np.uint32), int(st[2]), st
  st = stream.getstate()
  return np.asarray(st[1][:624], np.uint32), int(st[1][624]), st


def _set_stream(stream, full_state, keys, pos):
  if isinstance(stream, np.random.RandomState) or stream is np.random:
    stream.set_state(('MT19937', keys, pos, full_state[3], full_state[4]))
  else:
    stream.setstate((full_state[0], tuple(int(k) for k in keys) + (int(pos),), full_state[2]))


class RNGTape:
  """Keeps ``tape[0:len]`` = the next ``len`` words of ``stream`` (as of the last
  rebuild) and ``meta.tape_pos`` = words consumed since."""

  def __init__(self, replay, stream, capacity, device):
    self._replay = replay          # the owning buffer (for its handle / meta)
    self.stream = stream
    self.capacity = int(capacity)
    self.words = torch.zeros(self.capacity, dtype=torch.int32, device=device)
    self._base = None              # full host state the tape starts from
    self._len = 0
    self._budget = 0               # words guaranteed left (host-side worst-case accounting)
    self._host_synced = False      # last invalidation came from a host-side sync
    # Budget probe: the worst case (B + max_attempts retries per draw) is ~30x what a
    # PER step really uses, so instead of syncing when the worst-case budget runs low,
    # an async read of the device's tape position (pinned, stream-ordered, polled by
    # event) re-bases the budget on the words actually consumed.
    self._reserved = 0             # worst-case words reserved since the rebuild
    self._probe = None             # (event, words reserved before the probe point)
    self._probe_buf = None
    if self.words.is_cuda:
      self._probe_buf = torch.zeros(ctypes.sizeof(_lib.Meta), dtype=torch.uint8).pin_memory()

  @property
  def valid(self):
    return self._base is not None

  def invalidate(self):
    self._base = None
    self._probe = None

  def rebuild(self, nwords, stream_handle):
    """Draw the next ``nwords`` words of the host stream onto the device tape.
    The host stream itself is NOT advanced (the device owns those draws)."""
    nwords = min(int(nwords), self.capacity)
    keys, pos, full = _np_state_of(self.stream)
    rs = np.random.RandomState()
    rs.set_state(('MT19937', keys, pos))
    w = rs.randint(0, 2 ** 32, size=nwords, dtype=np.uint32).view(np.int32)
    host = torch.from_numpy(w)
    if self.words.is_cuda:
      host = host.pin_memory()
    self.words[:nwords].copy_(host, non_blocking=True)
    self._base = full
    self._len = nwords
    self._budget = nwords
    self._reserved = 0
    self._probe = None
    _lib.call('dq_replay_set_tape', self._replay._h, nwords, stream_handle)
    # keep the pinned staging buffer alive until the copy is done
    self._staging = host

  def _poll(self):
    ev, before = self._probe
    if not ev.query():
      return
    self._probe = None
    pos = int(_lib.Meta.from_address(self._probe_buf.data_ptr()).tape_pos)
    self._budget = max(self._budget, self._len - pos - (self._reserved - before))

  def reserve(self, worst_case, stream_handle):
    """Ensure ``worst_case`` more words are available without synchronising
    unless the tape might run dry; returns True if it had to sync."""
    if self.valid and self._probe is not None:
      self._poll()
    if self.valid and self._budget < worst_case and self._probe is not None:
      # The host ran further ahead of the device than the worst-case budget allows: wait
      # for the device to reach the probe point (the work queued behind it keeps the
      # device busy) and re-base, instead of draining the queue for a refill (a sync plus
      # a 1 Mi-word host rebuild: ~6 ms of device idle every ~250 uniform-replay steps)
      self._probe[0].synchronize()
      self._poll()
    if self.valid and self._budget >= worst_case:
      self._budget -= worst_case
      self._reserved += worst_case
      if (self._probe is None and self._probe_buf is not None and
          self._budget < self._len // 2):
        # enqueued before this reservation's work: it sees the earlier steps' use
        _lib.call('dq_replay_read_meta_async', self._replay._h, self._probe_buf.data_ptr(),
                  stream_handle)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.words.device))
        self._probe = (ev, self._reserved - worst_case)
      return False
    synced = False
    if self.valid:
      self.sync(stream_handle)
      synced = True
      size = self.capacity               # drained: a full tape (≈ hundreds of steps)
    elif self._host_synced:
      # the host drew from the stream (e.g. epsilon-greedy between steps): it will
      # again before long, so a short tape -- generating a full one per action
      # would cost milliseconds of host time each time
      size = 8 * worst_case
    else:
      size = self.capacity
    self._host_synced = False
    self.rebuild(max(worst_case, min(size, self.capacity)), stream_handle)
    self._budget -= worst_case
    self._reserved = worst_case
    return synced

  def sync(self, stream_handle, meta=None):
    """Advance the host stream by the words the device consumed; invalidate."""
    if not self.valid:
      return meta
    if meta is None:
      meta = self._replay._read_meta()
    used = int(meta.tape_pos)
    keys, pos, _ = _np_state_of(self.stream)
    base = self._base
    if isinstance(self.stream, np.random.RandomState) or self.stream is np.random:
      bkeys, bpos = np.asarray(base[1], np.uint32), int(base[2])
    else:
      bkeys, bpos = np.asarray(base[1][:624], np.uint32), int(base[1][624])
    rs = np.random.RandomState()
    rs.set_state(('MT19937', bkeys, bpos))
    if used:
      rs.randint(0, 2 ** 32, size=used, dtype=np.uint32)
    st = rs.get_state()
    _set_stream(self.stream, base, np.asarray(st[1], np.uint32), int(st[2]))
    self._base = None
    self._host_synced = True
    self._probe = None
    return meta


def default_stream(prioritized):
  return _random if prioritized else np.random
