"""Device-resident replay memory with the reference's out-of-graph API.

Mirrors ``dopamine.replay_memory.circular_replay_buffer`` (reference
circular_replay_buffer.py:80-915): the same constructor arguments, methods,
attributes, exceptions and messages.  Storage lives in HBM (torch tensors);
index sampling, validity checks, the frame-stack gather and the n-step reward
run in the HIP library (dopamine_amd/csrc/replay.hip) behind the C ABI of
include/dopamine_amd.h.  Numpy-returning methods (``sample_transition_batch``
etc.) synchronise and return exactly what the reference returns; the learner
uses ``sample_device`` which stays on the device and never synchronises.
"""
import codecs
import collections
import contextlib
import ctypes
import gzip
import math
import os
import pickle

import numpy as np
import torch

from dopamine_amd import _lib
from dopamine_amd.replay_memory.rng_tape import RNGTape, default_stream

ReplayElement = collections.namedtuple('shape_type', ['name', 'shape', 'type'])

STORE_FILENAME_PREFIX = '$store$_'
CHECKPOINT_DURATION = 4


class _ReferenceSumTree(object):
  """Target of a reference-written ``sum_tree`` pickle (dopamine.replay_memory.sum_tree.
  SumTree): only its fields (``nodes``, ``max_recorded_priority``) are restored."""


def _allowed_reconstructor(cls, base, state):
  """copyreg._reconstructor (protocol 0 / 1 object pickles, e.g. a Python 2-era reference's
  SumTree) restricted to the whitelisted classes built on ``object``."""
  if cls not in _CheckpointUnpickler._ALLOWED.values() or base is not object:
    raise pickle.UnpicklingError('replay checkpoint reconstructs {} on {}: not an allowed '
                                 'type'.format(cls, base))
  return object.__new__(cls)


class _CheckpointUnpickler(pickle.Unpickler):
  """Unpickles replay checkpoint members with a class whitelist: the reference's and
  this package's sum-tree snapshots and numpy's array / scalar reconstructors.
  Anything else (a callable a crafted file could name) is refused.  Every pickle
  protocol loads: 0 / 1 (copyreg._reconstructor, restricted above), 2-4 (the reference's
  default under Python 3, crb:643) and 5 (numpy arrays through _frombuffer)."""

  _ALLOWED = {
      ('dopamine.replay_memory.sum_tree', 'SumTree'): _ReferenceSumTree,
      ('numpy', 'ndarray'): np.ndarray,
      ('numpy', 'dtype'): np.dtype,
  }

  def find_class(self, module, name):
    key = (module, name)
    if key in self._ALLOWED:
      return self._ALLOWED[key]
    if key == ('dopamine_amd.replay_memory.sum_tree', 'SumTreeState'):
      from dopamine_amd.replay_memory.sum_tree import SumTreeState
      return SumTreeState
    if module in ('numpy.core.multiarray', 'numpy._core.multiarray') and name in ('_reconstruct',
                                                                                  'scalar'):
      return getattr(np._core.multiarray if hasattr(np, '_core') else np.core.multiarray, name)
    if module in ('numpy.core.numeric', 'numpy._core.numeric') and name == '_frombuffer':
      return getattr(np._core.numeric if hasattr(np, '_core') else np.core.numeric, name)
    if key in (('copyreg', '_reconstructor'), ('copy_reg', '_reconstructor')):
      return _allowed_reconstructor
    if key in (('builtins', 'object'), ('__builtin__', 'object')):
      return object
    if key == ('_codecs', 'encode'):    # bytes in protocol 0-2 pickles (numpy's raw data)
      return codecs.encode
    raise pickle.UnpicklingError('replay checkpoint names {}.{}: not an allowed type'.format(
        module, name))


class NotFoundError(FileNotFoundError):
  """Stands in for ``tf.errors.NotFoundError`` (same constructor), raised by
  ``load`` when a checkpoint file is missing (crb:671-673)."""

  def __init__(self, node_def, op, message):
    super().__init__(message)
    self.node_def, self.op, self.message = node_def, op, message


def invalid_range(cursor, replay_capacity, stack_size, update_horizon):
  """Indices around the cursor that cannot be sampled (crb:53-77)."""
  assert cursor < replay_capacity
  return np.array([(cursor - update_horizon + i) % replay_capacity
                   for i in range(stack_size + update_horizon)])


def _default_device(device):
  if device is not None:
    return torch.device(device)
  if not torch.cuda.is_available():
    raise RuntimeError('dopamine_amd replay memory needs a ROCm GPU (no CPU fallback)')
  return torch.device('cuda', torch.cuda.current_device())


class _MaxRecorded(float):
  """The priority argument meaning "SumTree.max_recorded_priority at the time of the add"
  (rainbow_agent.py:326-335 reads it on the host); the prioritized buffer resolves it on
  the device for a single transition, so the add needs no host round trip."""


MAX_RECORDED = _MaxRecorded(float('nan'))


def _stream_handle(device):
  return _lib.stream_of(device)


class OutOfGraphReplayBuffer(object):
  """Circular replay memory in HBM with uniform sampling (crb:80-687)."""

  _prioritized = False

  def __init__(self,
               observation_shape,
               stack_size,
               replay_capacity,
               batch_size,
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
               device=None,
               rng=None,
               tape_words=1 << 20):
    assert isinstance(observation_shape, tuple)
    if replay_capacity < update_horizon + stack_size:
      raise ValueError('There is not enough capacity to cover '
                       'update_horizon and stack_size.')
    # a scalar int32 action / float32 reward lives in the device store the learner kernels
    # read; any other shape or dtype is kept as its own element store
    # (dq_replay_gather_elems, crb:96-183 / 530-548)
    self._generic_action = tuple(action_shape) != () or np.dtype(action_dtype) != np.int32
    self._generic_reward = tuple(reward_shape) != () or np.dtype(reward_dtype) != np.float32
    if self._generic_reward and np.dtype(reward_dtype).name not in _lib.DT_CODES:
      raise NotImplementedError('reward_dtype {} is not supported'.format(np.dtype(reward_dtype)))
    # the samplers test one byte per terminal flag; a wider terminal_dtype (e.g. np.int32,
    # crb-test 83-90) keeps its stored values in a host mirror beside the device flags
    self._wide_terminal = np.dtype(terminal_dtype).itemsize != 1
    self._action_shape = tuple(action_shape)
    self._action_dtype = action_dtype
    self._reward_shape = tuple(reward_shape)
    self._reward_dtype = reward_dtype
    self._observation_shape = observation_shape
    self._stack_size = stack_size
    self._state_shape = self._observation_shape + (self._stack_size,)
    self._replay_capacity = replay_capacity
    self._batch_size = batch_size
    self._update_horizon = update_horizon
    self._gamma = gamma
    self._observation_dtype = observation_dtype
    self._terminal_dtype = terminal_dtype
    self._max_sample_attempts = max_sample_attempts
    self._extra_storage_types = list(extra_storage_types) if extra_storage_types else []
    self._device = _default_device(device)
    self._obs_bytes = int(np.prod(observation_shape, dtype=np.int64)) * np.dtype(observation_dtype).itemsize
    self._create_storage()
    self.add_count = np.array(0)
    self.invalid_range = np.zeros((self._stack_size))
    self._cumulative_discount_vector = np.array(
        [math.pow(self._gamma, n) for n in range(update_horizon)], dtype=np.float32)
    self._discount_dev = torch.from_numpy(self._cumulative_discount_vector).to(self._device)
    self._last_terminal = 0
    self._riders = None            # list while recording() is active
    self._rng = RNGTape(self, rng if rng is not None else default_stream(self._prioritized),
                        tape_words, self._device)
    self._create_handle()

  # ------------------------------------------------------------------ storage
  def _create_storage(self):
    C, dev = self._replay_capacity, self._device
    self._frames = torch.zeros((C, self._obs_bytes), dtype=torch.uint8, device=dev)
    self._actions = torch.zeros((C,), dtype=torch.int32, device=dev)
    self._rewards = torch.zeros((C,), dtype=torch.float32, device=dev)
    self._terminals = torch.zeros((C,), dtype=torch.uint8, device=dev)
    self._term_host = np.zeros((C,), self._terminal_dtype) if self._wide_terminal else None
    self._meta = torch.zeros((16,), dtype=torch.int64, device=dev)
    self._tree = None
    self._extras = {}
    if self._generic_action:      # (C, action bytes) rows, reinterpreted on the host
      ab = int(np.prod(self._action_shape, dtype=np.int64)) * np.dtype(self._action_dtype).itemsize
      self._act_rows = torch.zeros((C, max(ab, 1)), dtype=torch.uint8, device=dev)
    if self._generic_reward:
      self._rew_store = torch.zeros((C,) + self._reward_shape, dtype=_torch_dtype(self._reward_dtype),
                                    device=dev)
    for e in self._extra_storage_types:
      shape = (C,) + tuple(e.shape)
      self._extras[e.name] = torch.zeros(shape, dtype=_torch_dtype(e.type), device=dev)

  def _create_handle(self):
    cfg = _lib.Config()
    cfg.capacity = self._replay_capacity
    cfg.obs_bytes = self._obs_bytes
    cfg.stack_size = self._stack_size
    cfg.update_horizon = self._update_horizon
    cfg.max_sample_attempts = self._max_sample_attempts
    cfg.prioritized = int(self._prioritized)
    cfg.obs_is_u8 = int(np.dtype(self._observation_dtype) == np.uint8)
    cfg.gamma = self._gamma
    self._cfg = cfg
    self._h = None
    self._bind(self._rng.words, self._rng.capacity)
    # add_count 0, SumTree.max_recorded_priority = 1.0 (sum_tree.py:89)
    _lib.call('dq_replay_set_meta', self._h, 0, 1.0, self._stream)

  def _bind(self, tape, tape_cap):
    st = _lib.Storage()
    st.frames = self._frames.data_ptr()
    st.actions = self._actions.data_ptr()
    st.rewards = self._rewards.data_ptr()
    st.terminals = self._terminals.data_ptr()
    st.tree = self._tree.data_ptr() if self._tree is not None else None
    st.meta = self._meta.data_ptr()
    st.tape = tape.data_ptr()
    st.tape_capacity = tape_cap
    st.discount = self._discount_dev.data_ptr()
    if self._h is not None:
      _lib.call('dq_replay_destroy', self._h)
    h = ctypes.c_void_p()
    _lib.call('dq_replay_create', ctypes.byref(self._cfg), ctypes.byref(st), ctypes.byref(h))
    self._h = h

  def __del__(self):
    h = getattr(self, '_h', None)
    if h is not None:
      try:
        _lib.lib.dq_replay_destroy(h)
      except Exception:  # interpreter shutdown
        pass

  @property
  def _stream(self):
    return _stream_handle(self._device)

  def _read_meta(self):
    m = _lib.Meta()
    _lib.call('dq_replay_read_meta', self._h, ctypes.byref(m), self._stream)
    return m

  def _act_bytes(self):
    return int(np.prod(self._action_shape, dtype=np.int64)) * np.dtype(self._action_dtype).itemsize

  # ------------------------------------------------------------ signatures
  def get_add_args_signature(self):
    return self.get_storage_signature()

  def get_storage_signature(self):
    elems = [ReplayElement('observation', self._observation_shape, self._observation_dtype),
             ReplayElement('action', self._action_shape, self._action_dtype),
             ReplayElement('reward', self._reward_shape, self._reward_dtype),
             ReplayElement('terminal', (), self._terminal_dtype)]
    return elems + list(self._extra_storage_types)

  def get_transition_elements(self, batch_size=None):
    B = self._batch_size if batch_size is None else batch_size
    elems = [
        ReplayElement('state', (B,) + self._state_shape, self._observation_dtype),
        ReplayElement('action', (B,) + self._action_shape, self._action_dtype),
        ReplayElement('reward', (B,) + self._reward_shape, self._reward_dtype),
        ReplayElement('next_state', (B,) + self._state_shape, self._observation_dtype),
        ReplayElement('next_action', (B,) + self._action_shape, self._action_dtype),
        ReplayElement('next_reward', (B,) + self._reward_shape, self._reward_dtype),
        ReplayElement('terminal', (B,), self._terminal_dtype),
        ReplayElement('indices', (B,), np.int32)]
    for e in self._extra_storage_types:
      elems.append(ReplayElement(e.name, (B,) + tuple(e.shape), e.type))
    return elems

  # ----------------------------------------------------------------- adding
  def is_empty(self):
    return self.add_count == 0

  def is_full(self):
    return self.add_count >= self._replay_capacity

  def cursor(self):
    return self.add_count % self._replay_capacity

  def _check_args_length(self, *args):
    if len(args) != len(self.get_add_args_signature()):
      raise ValueError('Add expects {} elements, received {}'.format(
          len(self.get_add_args_signature()), len(args)))

  def _check_add_types(self, *args):
    self._check_args_length(*args)
    for arg, store in zip(args, self.get_add_args_signature()):
      if isinstance(arg, np.ndarray):
        shape = arg.shape
      elif isinstance(arg, (tuple, list)):
        shape = np.array(arg).shape
      else:
        shape = tuple()
      if shape != tuple(store.shape):
        raise ValueError('arg has shape {}, expected {}'.format(shape, tuple(store.shape)))

  def add(self, observation, action, reward, terminal, *args):
    """crb:234-260: pads stack_size - 1 zero transitions at episode starts."""
    self._check_add_types(observation, action, reward, terminal, *args)
    rows = []
    if self.is_empty() or self._last_terminal == 1:
      zero = [np.zeros(e.shape, dtype=e.type) for e in self.get_add_args_signature()]
      rows.extend([zero] * (self._stack_size - 1))
    rows.append([observation, action, reward, terminal] + list(args))
    self._add_rows(rows)

  def _priority_column(self, rows):
    return None

  # add() of up to _STAGE_ROWS rows goes up as ONE asynchronous copy from a ring of pinned
  # staging slots (obs | actions | rewards | terminals | priorities), so an env step never
  # waits on the device queue (five pageable copies each did: ~110 us per add behind a
  # training step); a slot is reused once its copy has run (event).
  _STAGE_ROWS = 16
  _STAGE_SLOTS = 8

  def _stage_rows(self, obs, act, rew, term, prio):
    n, ob = obs.shape[0], self._obs_bytes
    up = lambda x: (x + 15) // 16 * 16
    o_act = up(n * ob)
    o_rew = o_act + up(4 * n)
    o_term = o_rew + up(4 * n)
    o_prio = o_term + up(n)
    total = o_prio + up(4 * n)
    if getattr(self, '_stage_host', None) is None:
      R = self._STAGE_ROWS
      cap = up(R * ob) + 3 * up(4 * R) + up(R)
      self._stage_host = [torch.empty(cap, dtype=torch.uint8).pin_memory()
                          for _ in range(self._STAGE_SLOTS)]
      self._stage_ev = [None] * self._STAGE_SLOTS
      self._stage_dev = torch.empty(cap, dtype=torch.uint8, device=self._device)
      self._stage_i = 0
    k = self._stage_i % self._STAGE_SLOTS
    self._stage_i += 1
    if self._stage_ev[k] is not None:
      self._stage_ev[k].synchronize()
    h = self._stage_host[k].numpy()
    h[:n * ob] = obs.reshape(-1)
    h[o_act:o_act + 4 * n] = np.ascontiguousarray(act, np.int32).view(np.uint8)
    h[o_rew:o_rew + 4 * n] = np.ascontiguousarray(rew, np.float32).view(np.uint8)
    h[o_term:o_term + n] = np.ascontiguousarray(term).view(np.uint8).reshape(-1)
    if prio is not None:
      h[o_prio:o_prio + 4 * n] = np.ascontiguousarray(prio, np.float32).view(np.uint8)
    d = self._stage_dev
    d[:total].copy_(self._stage_host[k][:total], non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(self._device))
    self._stage_ev[k] = ev
    return (d, d[o_act:], d[o_rew:], d[o_term:], None if prio is None else d[o_prio:])

  def _add_rows(self, rows):
    n = len(rows)
    obs = np.empty((n, self._obs_bytes), np.uint8)
    for i, r in enumerate(rows):
      obs[i] = np.ascontiguousarray(np.asarray(r[0], dtype=self._observation_dtype)).view(np.uint8).reshape(-1)
    if self._generic_action:
      act = np.zeros(n, np.int32)
      act_rows = np.stack([np.ascontiguousarray(np.asarray(r[1], dtype=self._action_dtype))
                           .reshape(-1).view(np.uint8) for r in rows])
    else:
      act = np.array([r[1] for r in rows]).astype(np.int32)
    if self._generic_reward:
      rew = np.zeros(n, np.float32)
      rew_rows = np.stack([np.asarray(r[2], dtype=self._reward_dtype).reshape(self._reward_shape)
                           for r in rows])
    else:
      rew = np.array([r[2] for r in rows]).astype(np.float32)
    raw = np.array([r[3] for r in rows]).astype(self._terminal_dtype)
    base = int(self.add_count)
    if self._wide_terminal:
      self._term_host[[(base + i) % self._replay_capacity for i in range(n)]] = raw
      term = (raw != 0).astype(np.uint8)
    else:
      term = raw.view(np.uint8)
    prio = self._priority_column(rows)   # None, an array, or MAX_RECORDED (device-side max)
    if prio is MAX_RECORDED:
      prio = None                          # dq_replay_add: NULL = the max recorded priority
    dev = self._device
    generic = self._extra_storage_types or self._generic_action or self._generic_reward
    if not generic and n <= self._STAGE_ROWS and dev.type == 'cuda':
      d_obs, d_act, d_rew, d_term, d_prio = self._stage_rows(obs, act, rew, term, prio)
    else:
      d_obs = torch.from_numpy(obs).to(dev, non_blocking=False)
      d_act = torch.from_numpy(act).to(dev)
      d_rew = torch.from_numpy(rew).to(dev)
      d_term = torch.from_numpy(np.ascontiguousarray(term)).to(dev)
      d_prio = torch.from_numpy(prio).to(dev) if prio is not None else None
    if generic:
      slots = torch.tensor([(base + i) % self._replay_capacity for i in range(n)], device=dev)
      if self._generic_action and act_rows.shape[1]:
        self._act_rows[slots] = torch.from_numpy(act_rows).to(dev)
      if self._generic_reward:
        self._rew_store[slots] = torch.from_numpy(rew_rows).to(dev)
      for j, e in enumerate(self._extra_storage_types):
        vals = np.array([np.asarray(r[4 + j], dtype=e.type) for r in rows])
        self._extras[e.name][slots] = torch.from_numpy(vals).to(dev)
    _lib.call('dq_replay_add', self._h, n, _lib.ptr(d_obs), _lib.ptr(d_act), _lib.ptr(d_rew),
              _lib.ptr(d_term), _lib.ptr(d_prio), self._stream)
    self.add_count = np.array(base + n)
    self._last_terminal = int(bool(raw[-1] == 1))    # crb:251 store['terminal'][cursor-1] == 1
    self.invalid_range = invalid_range(self.cursor(), self._replay_capacity,
                                       self._stack_size, self._update_horizon)

  # -------------------------------------------------------------- inspection
  def get_range(self, array, start_index, end_index):
    """crb:338-366 on a host numpy array."""
    assert end_index > start_index, 'end_index must be larger than start_index'
    assert end_index >= 0
    assert start_index < self._replay_capacity
    if not self.is_full():
      assert end_index <= self.cursor(), 'Index {} has not been added.'.format(start_index)
    idx = [(start_index + i) % self._replay_capacity for i in range(end_index - start_index)]
    return array[idx, ...]

  def _stack_ids(self, index):
    return [(index - self._stack_size + 1 + k) % self._replay_capacity for k in range(self._stack_size)]

  def get_observation_stack(self, index):
    frames = self._frames[self._stack_ids(index)].cpu().numpy()
    frames = frames.view(self._observation_dtype).reshape((self._stack_size,) + self._observation_shape)
    return np.moveaxis(frames, 0, -1)

  def get_terminal_stack(self, index):
    if self._wide_terminal:
      return self._term_host[self._stack_ids(index)]
    return self._terminals[self._stack_ids(index)].cpu().numpy().view(self._terminal_dtype)

  def is_valid_transition(self, index):
    """crb:381-414 (host-side check, same rule as the device kernel)."""
    if index < 0 or index >= self._replay_capacity:
      return False
    if not self.is_full():
      if index >= self.cursor() - self._update_horizon:
        return False
      if index < self._stack_size - 1:
        return False
    if index in set(self.invalid_range):
      return False
    if self.get_terminal_stack(index)[:-1].any():
      return False
    return True

  # ---------------------------------------------------------------- sampling
  def _words_worst_case(self, batch_size):
    if self._prioritized:
      return 2 * (batch_size + self._max_sample_attempts)
    return 4 * (batch_size + self._max_sample_attempts) + 64

  def _check_status(self, meta, batch_size):
    st = int(meta.status)
    if st == _lib.ST_OK:
      return
    self._clear_status(meta)
    if st == _lib.ST_EMPTY_TREE:
      raise Exception('Cannot sample from an empty sum tree.')
    if st == _lib.ST_MAX_ATTEMPTS:
      raise RuntimeError('Max sample attempts: Tried {} times but only sampled {}'
                         ' valid indices. Batch size is {}'.format(
                             self._max_sample_attempts, int(meta.status_arg), batch_size))
    if st == _lib.ST_TOO_FEW:
      raise RuntimeError('Cannot sample a batch with fewer than stack size '
                         '({}) + update_horizon ({}) transitions.'.format(
                             self._stack_size, self._update_horizon))
    if st == _lib.ST_NEG_PRIORITY:
      raise ValueError('Sum tree values should be nonnegative. Got {}'.format(meta.status_value))
    if st == _lib.ST_BAD_INDEX:
      raise IndexError('index {} is out of bounds for the sum tree'.format(int(meta.status_value)))
    if st == _lib.ST_BROADCAST:
      # crb:540-541 with a trajectory length L that numpy cannot broadcast: raise numpy's
      # own error for those shapes (host shapes only, no data)
      L = int(meta.status_arg)
      prod = np.zeros(L, np.float32) * np.zeros((L,) + self._reward_shape, self._reward_dtype)
      np.empty((1,) + self._reward_shape, self._reward_dtype)[0] = np.sum(prod, axis=0)
      raise ValueError('reward of trajectory length {} does not broadcast'.format(L))
    raise RuntimeError('replay device status %d' % st)

  def _clear_status(self, meta):
    _lib.call('dq_replay_set_meta', self._h, int(meta.add_count), float(meta.max_recorded_priority),
              self._stream)

  def _precheck(self):
    if not self.is_full():
      if self.cursor() - self._update_horizon <= self._stack_size - 1:
        raise RuntimeError('Cannot sample a batch with fewer than stack size '
                           '({}) + update_horizon ({}) transitions.'.format(
                               self._stack_size, self._update_horizon))

  def _sample_indices_sync(self, batch_size):
    """Launch the device sampler and bring the host RNG stream in step."""
    if not self._prioritized:
      self._precheck()
    out = torch.empty((batch_size,), dtype=torch.int32, device=self._device)
    words = self._words_worst_case(batch_size)
    if self._rng.valid:                # words already used by device sampling come first
      self._rng.sync(self._stream)
    while True:
      self._rng.invalidate()           # a retry (tape ran dry) redraws from the same state
      self._rng.rebuild(words, self._stream)
      _lib.call('dq_replay_sample_indices', self._h, batch_size, _lib.ptr(out), self._stream)
      meta = self._read_meta()
      if int(meta.status) == _lib.ST_TAPE_EXHAUSTED and words < self._rng.capacity:
        self._clear_status(meta)       # nothing but the tape cursor moved: redo with more words
        words = min(self._rng.capacity, 4 * words)
        continue
      break
    self._rng.sync(self._stream, meta)
    self._check_status(meta, batch_size)
    return out

  def sample_index_batch(self, batch_size):
    """crb:436-477 (uniform) / prb:142-171 (prioritized); device-sampled."""
    return [int(i) for i in self._sample_indices_sync(batch_size).cpu().numpy()]

  def sample_transition_batch(self, batch_size=None, indices=None):
    """crb:479-558: numpy tuple in get_transition_elements() order."""
    if batch_size is None:
      batch_size = self._batch_size
    if indices is None:
      d_idx = self._sample_indices_sync(batch_size)
    else:
      assert len(indices) == batch_size
      d_idx = torch.as_tensor(np.asarray(indices, np.int64).astype(np.int32), device=self._device)
    out = self._gather(d_idx, batch_size, _lib.LAYOUT_RAW)
    S = self._stack_size

    def stack(t):
      a = t.cpu().numpy().view(self._observation_dtype).reshape((batch_size, S) + self._observation_shape)
      return np.moveaxis(a, 1, -1)

    if self._generic_reward:
      self._check_status(self._read_meta(), batch_size)   # a reward that did not broadcast

    def act(t):
      if self._generic_action:
        return t.cpu().numpy().reshape(batch_size, -1)[:, :self._act_bytes()].copy().view(
            self._action_dtype).reshape((batch_size,) + self._action_shape)
      return t.cpu().numpy().astype(self._action_dtype)

    def rew(t):
      return t.cpu().numpy().astype(self._reward_dtype)

    res = [stack(out['state']), act(out['action']), rew(out['reward']), stack(out['next_state']),
           act(out['next_action']), rew(out['next_reward']),
           out['terminal'].cpu().numpy().view(np.uint8).astype(self._terminal_dtype),
           out['indices'].cpu().numpy()]
    for e in self._extra_storage_types:
      res.append(out[e.name].cpu().numpy().astype(e.type))
    if self._prioritized:
      res.append(out['sampling_probabilities'].cpu().numpy())
    return tuple(res)

  def _alloc_batch(self, batch_size, layout):
    B, S, dev = batch_size, self._stack_size, self._device

    def states():
      if layout == _lib.LAYOUT_F32_NORM:
        return torch.empty((B, S) + tuple(self._observation_shape), dtype=torch.float32, device=dev)
      if layout == _lib.LAYOUT_F32_NHWC:   # (B, H, W, S) memory viewed as channels_last NCHW
        nhwc = torch.empty((B,) + tuple(self._observation_shape) + (S,), dtype=torch.float32, device=dev)
        return nhwc.permute(0, 3, 1, 2)
      raw = torch.empty((B, S, self._obs_bytes), dtype=torch.uint8, device=dev)
      if np.dtype(self._observation_dtype) != np.uint8:   # typed view of the gathered bytes
        return raw.view(_torch_dtype(self._observation_dtype)).reshape(
            (B, S) + tuple(self._observation_shape))
      return raw

    if self._generic_action:
      acts = lambda: torch.empty((B, self._act_rows.shape[1]), dtype=torch.uint8, device=dev)
    else:
      acts = lambda: torch.empty((B,), dtype=torch.int32, device=dev)
    if self._generic_reward:
      rews = lambda: torch.empty((B,) + self._reward_shape, dtype=self._rew_store.dtype, device=dev)
    else:
      rews = lambda: torch.empty((B,), dtype=torch.float32, device=dev)
    out = {'state': states(),
           'next_state': states(),
           'action': acts(),
           'reward': rews(),
           'next_action': acts(),
           'next_reward': rews(),
           'terminal': torch.empty((B,), dtype=torch.uint8, device=dev),
           'indices': torch.empty((B,), dtype=torch.int32, device=dev)}
    if self._prioritized:
      out['sampling_probabilities'] = torch.empty((B,), dtype=torch.float32, device=dev)
    return out

  def _gather(self, d_idx, batch_size, layout, out=None):
    if out is None:
      out = self._alloc_batch(batch_size, layout)
    p = _lib.ptr
    if self._riders is not None:
      if (layout != _lib.LAYOUT_F32_NHWC or self._extra_storage_types or self._generic_action or
          self._generic_reward):
        raise ValueError('only the NHWC gather (no extra storage, scalar int32 action and '
                         'float32 reward) can be recorded as a rider')
      r = _lib.Rider()
      _lib.call('dq_replay_record_gather_nhwc', self._h, p(d_idx), batch_size, p(out['state']),
                p(out['next_state']), p(out['action']), p(out['reward']), p(out['next_action']),
                p(out['next_reward']), p(out['terminal']), p(out['indices']),
                p(out.get('sampling_probabilities')), ctypes.byref(r))
      self._riders.append(r)
      return out
    ga, gr = self._generic_action, self._generic_reward
    _lib.call('dq_replay_gather', self._h, p(d_idx), batch_size, layout, p(out['state']),
              p(out['next_state']), None if ga else p(out['action']),
              None if gr else p(out['reward']), None if ga else p(out['next_action']),
              None if gr else p(out['next_reward']), p(out['terminal']), p(out['indices']),
              p(out.get('sampling_probabilities')), self._stream)
    if ga or gr:
      rs = self._rew_store if gr else None
      _lib.call('dq_replay_gather_elems', self._h, p(d_idx), batch_size,
                p(self._act_rows) if ga else None, self._act_bytes() if ga else 0,
                p(rs), int(np.prod(self._reward_shape, dtype=np.int64)) if gr else 1,
                (self._reward_shape[-1] if self._reward_shape else 0) if gr else 0,
                _lib.DT_CODES[np.dtype(self._reward_dtype).name] if gr else 0,
                int(np.result_type(np.float32, self._reward_dtype) == np.float64) if gr else 0,
                p(out['action']) if ga else None, p(out['next_action']) if ga else None,
                p(out['reward']) if gr else None, p(out['next_reward']) if gr else None,
                self._stream)
    if self._extra_storage_types:
      li = d_idx.long() % self._replay_capacity
      for e in self._extra_storage_types:
        out[e.name] = self._extras[e.name][li]
    return out

  # ------------------------------------------------------- device fast path
  def reserve_rng(self, batch_size=None, steps=1):
    """Host-side tape bookkeeping for ``steps`` upcoming device samples of ``batch_size``
    (call outside graph capture; may synchronise and refill the tape): the same budget as
    ``steps`` calls of one, in one call (a learner-loop chunk's reservation)."""
    B = self._batch_size if batch_size is None else batch_size
    if not self._prioritized:
      self._precheck()
    return self._rng.reserve(steps * self._words_worst_case(B), self._stream)

  def sample_device(self, batch_size=None, layout=_lib.LAYOUT_F32_NORM, out=None, indices=None,
                    reserve=True, groups=1):
    """Sample + gather without leaving the device or synchronising.

    Returns a dict of device tensors (``state``/``next_state`` as float32 NCHW
    normalised by 1/255 for the CNN).  The host RNG stream is brought in step
    lazily (``sync_rng``); device-latched errors surface at the next sync.
    ``reserve=False`` skips the host tape bookkeeping (the caller did it with
    ``reserve_rng``, e.g. around a HIP-graph replay).  ``groups`` > 1 (uniform buffers):
    that many consecutive batches of ``batch_size`` -- the draws of as many calls in a row
    (dq_replay_sample_indices_groups) -- gathered as one groups * batch_size batch."""
    B = self._batch_size if batch_size is None else batch_size
    n = B * groups
    if out is None:
      out = self._alloc_batch(n, layout)
    if indices is None:
      if reserve:
        for _ in range(groups):
          self.reserve_rng(B)
      if 'sample_indices' not in out:
        out['sample_indices'] = torch.empty((n,), dtype=torch.int32, device=self._device)
      p = _lib.ptr(out['sample_indices'])
      if self._riders is not None:
        r = _lib.Rider()
        if groups > 1:
          _lib.call('dq_replay_record_sample_groups', self._h, B, groups, p, ctypes.byref(r))
        else:
          _lib.call('dq_replay_record_sample', self._h, B, p, ctypes.byref(r))
        self._riders.append(r)
      elif groups > 1:
        _lib.call('dq_replay_sample_indices_groups', self._h, B, groups, p, self._stream)
      else:
        _lib.call('dq_replay_sample_indices', self._h, B, p, self._stream)
      indices = out['sample_indices']
    return self._gather(indices, n, layout, out)

  @contextlib.contextmanager
  def recording(self):
    """Inside, the device replay operations (sample_device's sample and NHWC
    gather, a prioritized buffer's device-tensor set_priority) are recorded as
    riders -- returned in the yielded list, in issue order -- instead of
    launched; HipNatureCNN.backward(riders=...) runs them inside its grouped
    launches.  Host-side bookkeeping (RNG tape reservation) is unchanged."""
    assert self._riders is None, 'recording() does not nest'
    self._riders = []
    try:
      yield self._riders
    finally:
      self._riders = None

  def rewind_last_sample(self):
    """Give back the RNG-tape words of the most recent device sample (whose
    indices are then discarded), e.g. a prefetched batch invalidated by add()."""
    _lib.call('dq_replay_rewind_last_sample', self._h, self._stream)

  def sync_rng(self, raise_errors=True):
    """Bring the host RNG stream in step with the device; raise latched errors."""
    meta = self._read_meta()
    self._rng.sync(self._stream, meta)
    if raise_errors:
      self._check_status(meta, self._batch_size)
    return meta

  # -------------------------------------------------------- bulk/synthetic
  def load_arrays(self, observations, actions, rewards, terminals, add_count, priorities=None):
    """Bulk-replace the store (used by the synthetic benchmark and tests):
    ``observations`` (C, obs_bytes) uint8 device/host tensor, etc."""
    C = self._replay_capacity
    self._frames.copy_(torch.as_tensor(observations).reshape(C, self._obs_bytes))
    self._actions.copy_(torch.as_tensor(actions))
    self._rewards.copy_(torch.as_tensor(rewards))
    terminals = torch.as_tensor(terminals)
    if self._wide_terminal:
      self._term_host[:] = terminals.cpu().numpy()
      terminals = terminals != 0
    self._terminals.copy_(terminals)
    self.add_count = np.array(int(add_count))
    self.invalid_range = invalid_range(self.cursor(), C, self._stack_size, self._update_horizon)
    self._last_terminal = self._terminal_is_one((self.cursor() - 1) % C)
    maxrec = 1.0
    if priorities is not None and self._prioritized:
      self._set_tree_leaves(priorities)
      maxrec = max(1.0, float(torch.as_tensor(priorities).max()))
    _lib.call('dq_replay_set_meta', self._h, int(add_count), maxrec, self._stream)

  # --------------------------------------------------------- checkpointing
  # crb:593-687: one gzip file per element, '<name>_ckpt.<iteration>.gz'; the store
  # arrays as '$store$_<name>' via np.save (no pickle), other ndarray attributes
  # via np.save, anything else pickled; the file CHECKPOINT_DURATION iterations
  # old is removed after each write; load() first checks that every file exists.
  # The arrays live in HBM: save is one D2H copy per array, load one H2D copy
  # into the existing device tensors (so shapes/dtypes must match the buffer).
  def _store_tensors(self):
    """Device views of the storage with the reference's ``_store`` names,
    shapes and dtypes (crb:160-171)."""
    C = self._replay_capacity
    obs = self._frames.view(_torch_dtype(self._observation_dtype)).reshape(
        (C,) + tuple(self._observation_shape))
    act, rew = self._actions, self._rewards
    if self._generic_action:
      ab = self._act_bytes()
      act = self._act_rows[:, :ab].view(_torch_dtype(self._action_dtype)).reshape(
          (C,) + self._action_shape) if ab else self._act_rows[:, :0].reshape((C,) + self._action_shape)
    if self._generic_reward:
      rew = self._rew_store
    st = collections.OrderedDict([('observation', obs), ('action', act),
                                  ('reward', rew), ('terminal', self._terminal_store())])
    for e in self._extra_storage_types:
      st[e.name] = self._extras[e.name]
    return st

  def _terminal_store(self):
    """The terminal store in terminal_dtype: a view of the device flags, or (wide types)
    a CPU tensor sharing the host mirror, which _after_load pushes to the device."""
    if self._wide_terminal:
      return torch.from_numpy(self._term_host)
    return self._terminals.view(_torch_dtype(self._terminal_dtype))

  def _terminal_is_one(self, i):
    if self._wide_terminal:
      return int(bool(self._term_host[i] == 1))
    return int(bool(self._terminal_store()[i].item() == 1))

  @property
  def _store(self):
    """Host copies of the storage arrays, keyed as the reference's ``_store``."""
    return {k: v.cpu().numpy() for k, v in self._store_tensors().items()}

  def _return_checkpointable_elements(self):
    """crb:596-610: every public member + every store array."""
    elems = collections.OrderedDict()
    for name, t in self._store_tensors().items():
      elems[STORE_FILENAME_PREFIX + name] = t
    for member_name, member in self.__dict__.items():
      if not member_name.startswith('_'):
        elems[member_name] = member
    return elems

  def _generate_filename(self, checkpoint_dir, name, suffix):
    return os.path.join(checkpoint_dir, '{}_ckpt.{}.gz'.format(name, suffix))

  def _checkpoint_value(self, attr, value):
    """What gets pickled for a non-array public member (PER overrides sum_tree)."""
    return value

  def _restore_value(self, attr, value):
    return value

  def save(self, checkpoint_dir, iteration_number):
    """crb:612-657."""
    if not os.path.exists(checkpoint_dir):
      return
    elems = self._return_checkpointable_elements()
    for attr, value in elems.items():
      filename = self._generate_filename(checkpoint_dir, attr, iteration_number)
      with open(filename, 'wb') as f:
        with gzip.GzipFile(fileobj=f, mode='wb') as outfile:
          if attr.startswith(STORE_FILENAME_PREFIX):
            np.save(outfile, value.cpu().numpy(), allow_pickle=False)
          elif isinstance(value, np.ndarray):
            np.save(outfile, value, allow_pickle=False)
          else:
            pickle.dump(self._checkpoint_value(attr, value), outfile)
      stale = iteration_number - CHECKPOINT_DURATION
      if stale >= 0:
        try:
          os.remove(self._generate_filename(checkpoint_dir, attr, stale))
        except FileNotFoundError:
          pass

  def load(self, checkpoint_dir, suffix):
    """crb:659-687.  Raises NotFoundError (nothing loaded) if any file is missing.
    Pickled members go through a whitelisting unpickler (_CheckpointUnpickler), so a
    checkpoint written by the reference loads (its pickled SumTree included)."""
    elems = self._return_checkpointable_elements()
    for attr in elems:
      filename = self._generate_filename(checkpoint_dir, attr, suffix)
      if not os.path.exists(filename):
        raise NotFoundError(None, None, 'Missing file: {}'.format(filename))
    arrays = {}
    for attr, cur in elems.items():
      filename = self._generate_filename(checkpoint_dir, attr, suffix)
      with open(filename, 'rb') as f:
        with gzip.GzipFile(fileobj=f, mode='rb') as infile:
          if attr.startswith(STORE_FILENAME_PREFIX):
            arr = np.load(infile, allow_pickle=False)
            if tuple(arr.shape) != tuple(cur.shape):
              raise ValueError('{}: checkpoint array has shape {}, the buffer stores {}'.format(
                  filename, arr.shape, tuple(cur.shape)))
            arrays[attr] = arr
          elif isinstance(cur, np.ndarray):
            self.__dict__[attr] = np.load(infile, allow_pickle=False)
          else:
            self.__dict__[attr] = self._restore_value(attr, _CheckpointUnpickler(infile).load())
    for attr, arr in arrays.items():
      t = elems[attr]
      t.copy_(torch.from_numpy(np.ascontiguousarray(arr)).to(dtype=t.dtype))
    self._after_load()

  def _after_load(self):
    """Re-derive the device control block from the loaded host state."""
    C = self._replay_capacity
    if self._wide_terminal:
      self._terminals.copy_(torch.from_numpy(self._term_host != 0))
    self._last_terminal = self._terminal_is_one((self.cursor() - 1) % C)
    _lib.call('dq_replay_set_meta', self._h, int(self.add_count), self._max_recorded_after_load(),
              self._stream)

  def _max_recorded_after_load(self):
    return 1.0


def _torch_dtype(np_dtype):
  return torch.from_numpy(np.zeros((), dtype=np_dtype)).dtype


class WrappedReplayBuffer(object):
  """crb:690-915 without TF: ``transition`` holds device tensors refreshed by
  ``sample()`` (the analogue of a session.run of the sampling py_func)."""

  def __init__(self,
               observation_shape,
               stack_size,
               use_staging=True,
               replay_capacity=1000000,
               batch_size=32,
               update_horizon=1,
               gamma=0.99,
               wrapped_memory=None,
               max_sample_attempts=1000,
               extra_storage_types=None,
               observation_dtype=np.uint8,
               terminal_dtype=np.uint8,
               action_shape=(),
               action_dtype=np.int32,
               reward_shape=(),
               reward_dtype=np.float32,
               device=None):
    if replay_capacity < update_horizon + 1:
      raise ValueError(
          'Update horizon ({}) should be significantly smaller '
          'than replay capacity ({}).'.format(update_horizon, replay_capacity))
    if not update_horizon >= 1:
      raise ValueError('Update horizon must be positive.')
    if not 0.0 <= gamma <= 1.0:
      raise ValueError('Discount factor (gamma) must be in [0, 1].')
    self.batch_size = batch_size
    # Staging (crb:840-872) hid host sampling latency; the device sampler has
    # none to hide, so the flag is accepted for API compatibility only.
    self.use_staging = use_staging
    if wrapped_memory is not None:
      self.memory = wrapped_memory
    else:
      self.memory = OutOfGraphReplayBuffer(
          observation_shape, stack_size, replay_capacity, batch_size, update_horizon, gamma,
          max_sample_attempts, observation_dtype=observation_dtype,
          terminal_dtype=terminal_dtype, extra_storage_types=extra_storage_types,
          action_shape=action_shape, action_dtype=action_dtype, reward_shape=reward_shape,
          reward_dtype=reward_dtype, device=device)
    if np.dtype(observation_dtype) != np.uint8:
      layout = _lib.LAYOUT_RAW
    elif stack_size == 4 and len(observation_shape) == 2:
      layout = _lib.LAYOUT_F32_NHWC     # Atari: CNN-ready channels_last, no transposes
    else:
      layout = _lib.LAYOUT_F32_NORM
    self._layout = layout
    self.transition = collections.OrderedDict()
    self._out = None

  def add(self, observation, action, reward, terminal, *args):
    self.memory.add(observation, action, reward, terminal, *args)

  def sample(self):
    """Refresh ``transition`` with a new device-sampled batch (no host sync)."""
    self._out = self.memory.sample_device(self.batch_size, layout=self._layout, out=self._out)
    self.unpack_transition(self._out)
    return self.transition

  def unpack_transition(self, out):
    self.transition = collections.OrderedDict()
    for e in self.memory.get_transition_elements(self.batch_size):
      if e.name in out:
        self.transition[e.name] = out[e.name]
    self.states = self.transition['state']
    self.actions = self.transition['action']
    self.rewards = self.transition['reward']
    self.next_states = self.transition['next_state']
    self.next_actions = self.transition['next_action']
    self.next_rewards = self.transition['next_reward']
    self.terminals = self.transition['terminal']
    self.indices = self.transition['indices']

  def save(self, checkpoint_dir, iteration_number):
    self.memory.save(checkpoint_dir, iteration_number)

  def load(self, checkpoint_dir, suffix):
    self.memory.load(checkpoint_dir, suffix)
