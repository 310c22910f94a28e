"""Generate golden replay vectors by running the REFERENCE's own code.

Runs only in the build container (needs /root/reference, never on the GPU box).
The reference's replay modules are imported from their files; the only
stand-ins are for non-algorithmic imports that are absent here:
``tensorflow`` (only ``tf.logging.info`` is touched by the code paths used)
and ``gin`` / ``gin.tf`` (``@gin.configurable`` treated as identity).

Outputs: tests/golden/{sumtree,replay_uniform,replay_per}.npz -- inputs and
reference outputs only (data, no reference source).

    python tests/golden/gen_golden.py
"""
import importlib.util
import os
import random
import sys
import types

import numpy as np

REF = '/root/reference/dopamine/replay_memory'
OUT = os.path.dirname(os.path.abspath(__file__))


def _load_reference():
  tf = types.ModuleType('tensorflow')
  tf.logging = types.SimpleNamespace(info=lambda *a, **k: None, warning=lambda *a, **k: None)
  gin = types.ModuleType('gin')
  gin.configurable = lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f))
  gin_tf = types.ModuleType('gin.tf')
  gin.tf = gin_tf
  for name, mod in (('tensorflow', tf), ('gin', gin), ('gin.tf', gin_tf)):
    sys.modules.setdefault(name, mod)
  pkg = types.ModuleType('dopamine'); pkg.__path__ = []
  sub = types.ModuleType('dopamine.replay_memory'); sub.__path__ = []
  sys.modules.setdefault('dopamine', pkg)
  sys.modules.setdefault('dopamine.replay_memory', sub)
  mods = {}
  for name in ('sum_tree', 'circular_replay_buffer', 'prioritized_replay_buffer'):
    spec = importlib.util.spec_from_file_location('dopamine.replay_memory.' + name,
                                                  os.path.join(REF, name + '.py'))
    m = importlib.util.module_from_spec(spec)
    sys.modules['dopamine.replay_memory.' + name] = m
    setattr(sub, name, m)
    spec.loader.exec_module(m)
    mods[name] = m
  return mods


def _pystate_words():
  st = random.getstate()[1]
  return np.array(st, dtype=np.int64)  # 624 words + position


def gen_sumtree(m):
  st_mod = m['sum_tree']
  out = {}
  rs = np.random.RandomState(7)
  caps = [1, 2, 3, 5, 100, 1000, 1025, 4096]
  out['capacities'] = np.array(caps)
  for c in caps:
    tree = st_mod.SumTree(c)
    nset = 3 * c + 5
    idx = rs.randint(0, c, size=nset).astype(np.int32)
    val = rs.uniform(0.0, 3.0, size=nset).astype(np.float32)
    val[rs.rand(nset) < 0.1] = 0.0
    for i, v in zip(idx, val):
      tree.set(int(i), v)
    out['c%d_set_idx' % c] = idx
    out['c%d_set_val' % c] = val
    out['c%d_nodes' % c] = np.concatenate(tree.nodes)
    out['c%d_maxrec' % c] = np.float64(tree.max_recorded_priority)
    for b in (1, 7, 32):
      random.seed(1000 + c + b)
      out['c%d_strat%d' % (c, b)] = np.array(tree.stratified_sample(b), np.int64)
      out['c%d_strat%d_state' % (c, b)] = _pystate_words()
    random.seed(99 + c)
    out['c%d_single' % c] = np.array([tree.sample() for _ in range(10)], np.int64)
    out['c%d_query' % c] = np.array([tree.sample(query_value=q) for q in (0.0, 0.25, 0.5, 0.999, 1.0)], np.int64)
  np.savez_compressed(os.path.join(OUT, 'sumtree.npz'), **out)


def _stream(rs, n, obs_shape, p_term, nA):
  obs = rs.randint(0, 256, size=(n,) + obs_shape).astype(np.uint8)
  act = rs.randint(0, nA, size=n).astype(np.int32)
  rew = rs.choice(np.array([-1.0, 0.0, 1.0, 0.5], np.float32), size=n)
  term = (rs.rand(n) < p_term).astype(np.uint8)
  return obs, act, rew, term


def gen_replay(m, prioritized):
  crb = m['circular_replay_buffer']
  prb = m['prioritized_replay_buffer']
  out = {}
  cases = [  # (name, capacity, n, stack, adds, gamma, B, rounds)
      ('full_n1', 200, 1, 4, 537, 0.99, 32, 12),
      ('full_n3', 200, 3, 4, 611, 0.99, 32, 12),
      ('part_n3', 300, 3, 4, 90, 0.9, 16, 8),
      ('full_n5_s1', 50, 5, 1, 173, 0.97, 8, 10),
  ]
  out['cases'] = np.array([c[0] for c in cases])
  rs = np.random.RandomState(11 if prioritized else 13)
  for name, C, n, stack, adds, gamma, B, rounds in cases:
    obs_shape = (8, 8)
    obs, act, rew, term = _stream(rs, adds, obs_shape, 0.06, 6)
    cls = prb.OutOfGraphPrioritizedReplayBuffer if prioritized else crb.OutOfGraphReplayBuffer
    mem = cls(observation_shape=obs_shape, stack_size=stack, replay_capacity=C,
              batch_size=B, update_horizon=n, gamma=gamma)
    prio_in = rs.uniform(0.05, 2.0, size=adds).astype(np.float32)
    for i in range(adds):
      if prioritized:
        mem.add(obs[i], act[i], rew[i], term[i], prio_in[i])
      else:
        mem.add(obs[i], act[i], rew[i], term[i])
    meta = np.array([C, n, stack, adds, B, rounds], np.int64)
    pre = '%s_' % name
    out[pre + 'meta'] = meta
    out[pre + 'gamma'] = np.float64(gamma)
    out[pre + 'obs'] = obs
    out[pre + 'act'] = act
    out[pre + 'rew'] = rew
    out[pre + 'term'] = term
    if prioritized:
      out[pre + 'prio_in'] = prio_in
    out[pre + 'add_count'] = np.int64(mem.add_count)
    seed = 4242 + C
    if prioritized:
      random.seed(seed)
    else:
      np.random.seed(seed)
    out[pre + 'seed'] = np.int64(seed)
    keys = ['state', 'action', 'reward', 'next_state', 'next_action', 'next_reward',
            'terminal', 'indices'] + (['probs'] if prioritized else [])
    rows = {k: [] for k in keys}
    upd_idx, upd_val = [], []
    for r in range(rounds):
      batch = mem.sample_transition_batch()
      for k, v in zip(keys, batch):
        rows[k].append(np.array(v))
      if prioritized:
        # set_priority with a few duplicate indices, as the agent would do with
        # sqrt(loss + 1e-10) (rainbow_agent.py:289-290).
        ind = np.array(batch[7], np.int32).copy()
        if B > 2:
          ind[-1] = ind[0]
        pv = rs.uniform(0.01, 3.0, size=B).astype(np.float32)
        mem.set_priority(ind, pv)
        upd_idx.append(ind)
        upd_val.append(pv)
    for k in keys:
      out[pre + k] = np.stack(rows[k])
    if prioritized:
      out[pre + 'upd_idx'] = np.stack(upd_idx)
      out[pre + 'upd_val'] = np.stack(upd_val)
      out[pre + 'nodes'] = np.concatenate(mem.sum_tree.nodes)
      out[pre + 'maxrec'] = np.float64(mem.sum_tree.max_recorded_priority)
      out[pre + 'rng_state'] = _pystate_words()
    else:
      out[pre + 'rng_state'] = np.array(np.random.get_state()[1], np.int64)
      out[pre + 'rng_pos'] = np.int64(np.random.get_state()[2])
    # explicit-index KAT on the final memory (crb:510 `indices` argument)
    fixed = [i for i in range(C) if mem.is_valid_transition(i)][:5]
    out[pre + 'valid_mask'] = np.array([mem.is_valid_transition(i) for i in range(-2, C + 2)], np.uint8)
    fb = mem.sample_transition_batch(batch_size=len(fixed), indices=fixed)
    for k, v in zip(keys, fb):
      out[pre + 'fixed_' + k] = np.array(v)
  fname = 'replay_per.npz' if prioritized else 'replay_uniform.npz'
  np.savez_compressed(os.path.join(OUT, fname), **out)


def gen_checkpoint(m):
  """A checkpoint WRITTEN BY THE REFERENCE's OutOfGraphReplayBuffer.save
  (crb:612-657) for a small wrapped uniform buffer -- its members are all numpy
  arrays, so every file is np.save data (no pickle) -- plus what the reference
  samples after loading it (np.random.seed(13))."""
  import shutil
  crb = m['circular_replay_buffer']
  tf = sys.modules['tensorflow']
  tf.gfile = types.SimpleNamespace(Exists=os.path.exists, Open=open, Remove=os.remove)
  tf.errors = types.SimpleNamespace(NotFoundError=FileNotFoundError)
  kw = dict(observation_shape=(6, 6), stack_size=4, replay_capacity=40, batch_size=4,
            update_horizon=2, gamma=0.9)
  mem = crb.OutOfGraphReplayBuffer(**kw)
  rs = np.random.RandomState(5)
  for i in range(57):
    mem.add(rs.randint(0, 256, (6, 6)).astype(np.uint8), int(rs.randint(0, 5)),
            float(rs.randn()), bool(i % 13 == 12))
  d = os.path.join(OUT, 'ckpt_uniform')
  shutil.rmtree(d, ignore_errors=True)
  os.makedirs(d)
  mem.save(d, 7)
  fresh = crb.OutOfGraphReplayBuffer(**kw)
  fresh.load(d, 7)
  np.random.seed(13)
  batch = fresh.sample_transition_batch(batch_size=4)
  names = [e.name for e in fresh.get_transition_elements(4)]
  np.savez_compressed(os.path.join(OUT, 'ckpt_uniform_expected.npz'),
                      **{n: np.asarray(v) for n, v in zip(names, batch)})


def gen_checkpoint_per(m):
  """A prioritized checkpoint written by the reference's save (crb:612-657 via
  prb:36-252): the `sum_tree` member is the reference's pickled SumTree object.  Plus
  what the reference samples after loading it (random.seed(17)).  The test loads it
  through a restricted unpickler (classes whitelisted, nothing else executes)."""
  import shutil
  prb = m['prioritized_replay_buffer']
  tf = sys.modules['tensorflow']
  tf.gfile = types.SimpleNamespace(Exists=os.path.exists, Open=open, Remove=os.remove)
  tf.errors = types.SimpleNamespace(NotFoundError=FileNotFoundError)
  kw = dict(observation_shape=(6, 6), stack_size=4, replay_capacity=40, batch_size=4,
            update_horizon=3, gamma=0.9)
  mem = prb.OutOfGraphPrioritizedReplayBuffer(**kw)
  rs = np.random.RandomState(6)
  for i in range(61):
    mem.add(rs.randint(0, 256, (6, 6)).astype(np.uint8), int(rs.randint(0, 5)),
            float(rs.randn()), bool(i % 11 == 10), np.float32(rs.uniform(0.1, 2.0)))
  mem.set_priority(np.array([5, 9, 5, 30], np.int32), np.array([0.3, 2.5, 0.7, 1.1], np.float32))
  d = os.path.join(OUT, 'ckpt_per')
  shutil.rmtree(d, ignore_errors=True)
  os.makedirs(d)
  mem.save(d, 3)
  fresh = prb.OutOfGraphPrioritizedReplayBuffer(**kw)
  fresh.load(d, 3)
  random.seed(17)
  batch = fresh.sample_transition_batch(batch_size=4)
  names = [e.name for e in fresh.get_transition_elements(4)]
  out = {n: np.asarray(v) for n, v in zip(names, batch)}
  out['nodes'] = np.concatenate(fresh.sum_tree.nodes)
  out['maxrec'] = np.float64(fresh.sum_tree.max_recorded_priority)
  out['rng_state'] = _pystate_words()
  np.savez_compressed(os.path.join(OUT, 'ckpt_per_expected.npz'), **out)


# (name, capacity, n, stack, adds, gamma, B, rounds, action (shape, dtype), reward (shape, dtype))
SHAPE_CASES = [
    ('a', 40, 1, 2, 97, 0.9, 6, 5, ((2,), 'int8'), ((3,), 'float32')),
    ('b', 40, 3, 2, 101, 0.9, 6, 0, ((), 'int64'), ((3,), 'float64')),
    ('c', 40, 3, 1, 89, 0.95, 5, 4, ((2, 2), 'float32'), ((), 'float64')),
    ('d', 40, 3, 2, 77, 0.9, 5, 4, ((), 'int32'), ((), 'int32')),
    ('e', 40, 1, 2, 66, 0.8, 4, 4, ((), 'uint8'), ((2, 3), 'float16')),
]


def gen_shapes(m):
    """Non-scalar / non-default action and reward elements (crb:96-183, 530-548): sampled
    batches (np.random, rounds > 0), an explicit-index batch over indices whose n-step
    length broadcasts, and for case b one index whose length does not (numpy's error)."""
    crb = m['circular_replay_buffer']
    out = {'cases': np.array([c[0] for c in SHAPE_CASES])}
    rs = np.random.RandomState(21)
    for name, C, n, stack, adds, gamma, B, rounds, (ash, adt), (rsh, rdt) in SHAPE_CASES:
        mem = crb.OutOfGraphReplayBuffer(observation_shape=(4, 4), stack_size=stack,
                                         replay_capacity=C, batch_size=B, update_horizon=n,
                                         gamma=gamma, action_shape=ash, action_dtype=np.dtype(adt),
                                         reward_shape=rsh, reward_dtype=np.dtype(rdt))
        obs = rs.randint(0, 256, (adds, 4, 4)).astype(np.uint8)
        act = rs.randint(-3, 100, (adds,) + ash).astype(adt)
        rew = (rs.randint(-4, 5, (adds,) + rsh) * 0.37).astype(rdt)
        term = (rs.rand(adds) < 0.12).astype(np.uint8)
        for i in range(adds):
            mem.add(obs[i], act[i], rew[i], term[i])
        pre = name + '_'
        out[pre + 'meta'] = np.array([C, n, stack, adds, B, rounds], np.int64)
        out[pre + 'gamma'] = np.float64(gamma)
        out[pre + 'obs'], out[pre + 'act'], out[pre + 'rew'], out[pre + 'term'] = obs, act, rew, term
        keys = ['state', 'action', 'reward', 'next_state', 'next_action', 'next_reward',
                'terminal', 'indices']
        np.random.seed(500 + C + n)
        out[pre + 'seed'] = np.int64(500 + C + n)
        rows = {k: [] for k in keys}
        for _ in range(rounds):
            for k, v in zip(keys, mem.sample_transition_batch()):
                rows[k].append(np.array(v))
        for k in keys:
            if rounds:
                out[pre + k] = np.stack(rows[k])
        traj_len = {}
        for i in range(C):
            if mem.is_valid_transition(i):
                t = mem._store['terminal'][[(i + j) % C for j in range(n)]]
                traj_len[i] = int(np.argmax(t.astype(bool))) + 1 if t.any() else n
        m_last = rsh[-1] if rsh else 0
        ok = [i for i, L in sorted(traj_len.items()) if not m_last or L in (m_last, 1)]
        fixed = ok[:B]
        out[pre + 'fixed_indices'] = np.array(fixed, np.int64)
        for k, v in zip(keys, mem.sample_transition_batch(batch_size=len(fixed), indices=fixed)):
            out[pre + 'fixed_' + k] = np.array(v)
        bad = [i for i, L in sorted(traj_len.items()) if m_last and L not in (m_last, 1)]
        if bad:
            try:
                mem.sample_transition_batch(batch_size=1, indices=[bad[0]])
                out[pre + 'bad_error'] = np.array('')
            except ValueError as e:
                out[pre + 'bad_error'] = np.array(str(e))
            out[pre + 'bad_index'] = np.int64(bad[0])
    np.savez_compressed(os.path.join(OUT, 'replay_shapes.npz'), **out)


if __name__ == '__main__':
  mods = _load_reference()
  if sys.argv[1:] == ['ckpt_per']:
    gen_checkpoint_per(mods)
    sys.exit(0)
  if sys.argv[1:] == ['shapes']:
    gen_shapes(mods)
    sys.exit(0)
  gen_sumtree(mods)
  gen_replay(mods, prioritized=False)
  gen_replay(mods, prioritized=True)
  gen_checkpoint(mods)
  gen_checkpoint_per(mods)
  gen_shapes(mods)
  for f in sorted(os.listdir(OUT)):
    if f.endswith('.npz'):
      print(f, os.path.getsize(os.path.join(OUT, f)))
