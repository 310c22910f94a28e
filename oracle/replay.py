"""CPU oracle for the replay path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / CPU baseline.  The product
path (``dopamine_amd``) never imports it.

A plain numpy / pure-Python restatement of Dopamine's replay memory algorithm:

* ``SumTree``            -- dopamine/replay_memory/sum_tree.py:30-205
* ``invalid_range``      -- dopamine/replay_memory/circular_replay_buffer.py:53-77
* ``ReplayOracle``       -- circular_replay_buffer.py:80-591 (add, validity,
                            uniform index sampling, transition gather, n-step)
* ``PrioritizedOracle``  -- prioritized_replay_buffer.py:36-252

Parity pin: ``tests/golden/*.npz`` were produced by running the reference's own
out-of-graph code in the build container (``tests/golden/gen_golden.py``);
``tests/test_oracle_golden.py`` checks this restatement against them bit for bit,
and ``tests/test_oracle_kats.py`` restates the reference unit-test KATs.

RNG streams are injectable (``py_rng`` = a ``random.Random``-like object,
``np_rng`` = a ``numpy.random.RandomState``) so the oracle can replay exactly the
draws the reference makes from the global ``random`` / ``np.random`` modules.
"""
import math
import random as _random

import numpy as np


# --------------------------------------------------------------------------
# Sum tree (sum_tree.py:30-205).  Stored as one flat float64 heap; level d
# occupies [2**d - 1, 2**(d+1) - 1).  ``levels()`` gives the reference's
# list-of-arrays view for comparison.
# --------------------------------------------------------------------------
class SumTree:
  def __init__(self, capacity):
    assert isinstance(capacity, int)
    if capacity <= 0:
      raise ValueError('Sum tree capacity should be positive. Got: {}'.format(capacity))
    self.depth = int(math.ceil(np.log2(capacity)))          # st:80
    self.nodes = np.zeros(2 ** (self.depth + 1) - 1)
    self.max_recorded_priority = 1.0                          # st:89

  def levels(self):
    return [self.nodes[2 ** d - 1: 2 ** (d + 1) - 1] for d in range(self.depth + 1)]

  def total(self):
    return self.nodes[0]

  def get(self, index):                                       # st:168-176
    return self.nodes[2 ** self.depth - 1 + index]

  def set(self, index, value):                                # st:178-205
    if value < 0.0:
      raise ValueError('Sum tree values should be nonnegative. Got {}'.format(value))
    self.max_recorded_priority = max(value, self.max_recorded_priority)
    leaf = 2 ** self.depth - 1 + index
    delta = value - self.nodes[leaf]
    # Walk leaf -> root adding the SAME delta at every level (no recompute).
    node = index
    for d in range(self.depth, -1, -1):
      self.nodes[2 ** d - 1 + node] += delta
      node //= 2

  def _descend(self, q):
    node = 0
    for d in range(1, self.depth + 1):
      left = self.nodes[2 ** d - 1 + 2 * node]
      if q < left:
        node = 2 * node
      else:
        node = 2 * node + 1
        q -= left
    return node

  def sample(self, query_value=None, py_rng=None):            # st:99-141
    if self.total() == 0.0:
      raise Exception('Cannot sample from an empty sum tree.')
    if query_value and (query_value < 0. or query_value > 1.):
      raise ValueError('query_value must be in [0, 1].')
    if query_value is None:
      query_value = (py_rng or _random).random()
    return self._descend(query_value * self.total())

  def stratified_sample(self, batch_size, py_rng=None):       # st:143-166
    if self.total() == 0.0:
      raise Exception('Cannot sample from an empty sum tree.')
    rng = py_rng or _random
    edges = np.linspace(0., 1., batch_size + 1)
    qs = [rng.uniform(edges[i], edges[i + 1]) for i in range(batch_size)]
    return [self.sample(query_value=q) for q in qs]

  @classmethod
  def from_leaves(cls, capacity, leaves):
    """Bulk construction (parents = sum of children).  Not the reference's
    delta order -- used only to give the oracle and the device the SAME tree."""
    t = cls(capacity)
    base = 2 ** t.depth - 1
    t.nodes[base:base + len(leaves)] = np.asarray(leaves, np.float64)
    for d in range(t.depth - 1, -1, -1):
      lo = 2 ** d - 1
      ch = t.nodes[2 ** (d + 1) - 1: 2 ** (d + 2) - 1]
      t.nodes[lo:lo + 2 ** d] = ch[0::2] + ch[1::2]
    if len(leaves):
      t.max_recorded_priority = max(1.0, float(np.max(leaves)))
    return t


def invalid_range(cursor, capacity, stack_size, update_horizon):
  """crb:53-77 -- the n + stack indices around the cursor that cannot be sampled."""
  assert cursor < capacity
  return np.array([(cursor - update_horizon + k) % capacity
                   for k in range(stack_size + update_horizon)])


# --------------------------------------------------------------------------
# Uniform circular buffer (crb:80-591)
# --------------------------------------------------------------------------
class ReplayOracle:
  def __init__(self, observation_shape, stack_size, replay_capacity, batch_size,
               update_horizon=1, gamma=0.99, max_sample_attempts=1000,
               observation_dtype=np.uint8, terminal_dtype=np.uint8,
               reward_dtype=np.float32, py_rng=None, np_rng=None, action_shape=(),
               action_dtype=np.int32, reward_shape=()):
    if replay_capacity < update_horizon + stack_size:
      raise ValueError('There is not enough capacity to cover '
                       'update_horizon and stack_size.')
    self.obs_shape = tuple(observation_shape)
    self.stack = stack_size
    self.C = replay_capacity
    self.B = batch_size
    self.n = update_horizon
    self.gamma = gamma
    self.max_attempts = max_sample_attempts
    self.obs_dtype = observation_dtype
    self.py_rng = py_rng or _random
    self.np_rng = np_rng or np.random
    self.observation = np.zeros((self.C,) + self.obs_shape, observation_dtype)
    self.action_shape, self.action_dtype = tuple(action_shape), action_dtype
    self.reward_shape, self.reward_dtype = tuple(reward_shape), reward_dtype
    self.action = np.zeros((self.C,) + self.action_shape, action_dtype)
    self.reward = np.zeros((self.C,) + self.reward_shape, reward_dtype)
    self.terminal = np.zeros((self.C,), terminal_dtype)
    self.add_count = 0
    self.invalid_range = np.zeros((self.stack,))
    # crb:181-183: gamma^k via math.pow in double, then cast to float32.
    self.discount = np.array([math.pow(gamma, k) for k in range(update_horizon)],
                             dtype=np.float32)

  # -- bookkeeping (crb:326-336)
  def is_empty(self):
    return self.add_count == 0

  def is_full(self):
    return self.add_count >= self.C

  def cursor(self):
    return self.add_count % self.C

  # -- adding (crb:234-287)
  def _write(self, obs, action, reward, terminal, priority=None):
    c = self.cursor()
    self.observation[c] = obs
    self.action[c] = action
    self.reward[c] = reward
    self.terminal[c] = terminal
    self.add_count += 1
    self.invalid_range = invalid_range(self.cursor(), self.C, self.stack, self.n)

  def _pad(self):
    return self.is_empty() or self.terminal[self.cursor() - 1] == 1

  def add(self, obs, action, reward, terminal):
    if np.shape(obs) != self.obs_shape:
      raise ValueError('arg has shape {}, expected {}'.format(np.shape(obs), self.obs_shape))
    if self._pad():
      for _ in range(self.stack - 1):
        self._write(np.zeros(self.obs_shape, self.obs_dtype), 0, 0, 0)
    self._write(obs, action, reward, terminal)

  # -- validity (crb:381-414)
  def _ring(self, start, count):
    return [(start + k) % self.C for k in range(count)]

  def is_valid_transition(self, index):
    if index < 0 or index >= self.C:
      return False
    if not self.is_full():
      if index >= self.cursor() - self.n:
        return False
      if index < self.stack - 1:
        return False
    if index in set(self.invalid_range):
      return False
    if self.terminal[self._ring(index - self.stack + 1, self.stack)][:-1].any():
      return False
    return True

  # -- uniform index sampling (crb:436-477)
  def _id_range(self):
    if self.is_full():
      return self.cursor() - self.C + self.stack - 1, self.cursor() - self.n
    lo, hi = self.stack - 1, self.cursor() - self.n
    if hi <= lo:
      raise RuntimeError('Cannot sample a batch with fewer than stack size '
                         '({}) + update_horizon ({}) transitions.'.format(self.stack, self.n))
    return lo, hi

  def sample_index_batch(self, batch_size):
    lo, hi = self._id_range()
    out, fails = [], 0
    while len(out) < batch_size and fails < self.max_attempts:
      idx = self.np_rng.randint(lo, hi) % self.C
      if self.is_valid_transition(idx):
        out.append(idx)
      else:
        fails += 1
    if len(out) != batch_size:
      raise RuntimeError('Max sample attempts: Tried {} times but only sampled {}'
                         ' valid indices. Batch size is {}'.format(self.max_attempts, len(out), batch_size))
    return out

  # -- gather (crb:479-558, 368-375)
  def stack_at(self, index):
    """(H, W, stack) frames [index-stack+1 .. index] mod C, stacking axis last."""
    frames = self.observation[self._ring(index - self.stack + 1, self.stack)]
    return np.moveaxis(frames, 0, -1)

  def nstep(self, idx):
    """Returns (discounted reward f32, terminal flag, trajectory length L)."""
    traj = self.terminal[self._ring(idx, self.n)]
    term = bool(traj.any())
    L = int(np.argmax(traj.astype(bool))) + 1 if term else self.n
    r = self.reward[self._ring(idx, L)]
    if self.reward_shape or np.dtype(self.reward_dtype) != np.float32:
      # crb:540-541 as written: the (L,) float32 discount broadcast against (L,) +
      # reward_shape (numpy raises where it does not), summed over axis 0
      return np.sum(self.discount[:L] * r, axis=0), term, L
    acc = np.float32(0.0)
    for k in range(L):  # float32 products summed left to right (numpy n<8 loop)
      acc = np.float32(acc + np.float32(self.discount[k] * r[k]))
    return acc, term, L

  def sample_transition_batch(self, batch_size=None, indices=None):
    B = self.B if batch_size is None else batch_size
    if indices is None:
      indices = self.sample_index_batch(B)
    assert len(indices) == B
    st = np.empty((B,) + self.obs_shape + (self.stack,), self.obs_dtype)
    nst = np.empty_like(st)
    act = np.empty((B,) + self.action_shape, self.action_dtype)
    rew = np.empty((B,) + self.reward_shape, self.reward_dtype)
    nact = np.empty_like(act)
    nrew = np.empty_like(rew)
    term = np.empty((B,), np.uint8)
    ind = np.empty((B,), np.int32)
    for b, idx in enumerate(indices):
      r, t, L = self.nstep(idx)
      nxt = (idx + L) % self.C
      st[b] = self.stack_at(idx)
      nst[b] = self.stack_at(nxt)
      act[b] = self.action[idx]
      rew[b] = r
      nact[b] = self.action[nxt]
      nrew[b] = self.reward[nxt]
      term[b] = t
      ind[b] = idx
    return [st, act, rew, nst, nact, nrew, term, ind]


# --------------------------------------------------------------------------
# Prioritized buffer (prb:36-252)
# --------------------------------------------------------------------------
class PrioritizedOracle(ReplayOracle):
  def __init__(self, *args, **kwargs):
    super().__init__(*args, **kwargs)
    self.sum_tree = SumTree(self.C)

  def add(self, obs, action, reward, terminal, priority):
    if np.shape(obs) != self.obs_shape:
      raise ValueError('arg has shape {}, expected {}'.format(np.shape(obs), self.obs_shape))
    if self._pad():
      for _ in range(self.stack - 1):
        self.sum_tree.set(self.cursor(), np.float32(0.0))
        self._write(np.zeros(self.obs_shape, self.obs_dtype), 0, 0, 0)
    self.sum_tree.set(self.cursor(), priority)
    self._write(obs, action, reward, terminal)

  def sample_index_batch(self, batch_size):                 # prb:142-171
    idxs = self.sum_tree.stratified_sample(batch_size, py_rng=self.py_rng)
    budget = self.max_attempts
    for i in range(len(idxs)):
      if self.is_valid_transition(idxs[i]):
        continue
      if budget == 0:
        raise RuntimeError('Max sample attempts: Tried {} times but only sampled {}'
                           ' valid indices. Batch size is {}'.format(self.max_attempts, i, batch_size))
      cand = idxs[i]
      while not self.is_valid_transition(cand) and budget > 0:
        cand = self.sum_tree.sample(py_rng=self.py_rng)
        budget -= 1
      idxs[i] = cand
    return idxs

  def get_priority(self, indices):                           # prb:216-235
    assert indices.dtype == np.int32
    return np.array([self.sum_tree.get(int(i)) for i in indices], np.float32)

  def set_priority(self, indices, priorities):               # prb:203-214
    assert indices.dtype == np.int32
    for i, p in zip(indices, priorities):
      self.sum_tree.set(int(i), p)

  def sample_transition_batch(self, batch_size=None, indices=None):
    out = super().sample_transition_batch(batch_size, indices)
    out.append(self.get_priority(out[7]))
    return out
