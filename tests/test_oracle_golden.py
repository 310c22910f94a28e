"""Pins the CPU oracle (oracle/replay.py) to vectors produced by running the
reference's own replay code (tests/golden/gen_golden.py).  Bit-exact."""
import random

import numpy as np
import pytest

from oracle import replay as orc


def _case_names(z):
  return [str(c) for c in z['cases']]


def test_sumtree_golden(golden):
  z = golden('sumtree.npz')
  for c in z['capacities']:
    c = int(c)
    t = orc.SumTree(c)
    for i, v in zip(z['c%d_set_idx' % c], z['c%d_set_val' % c]):
      t.set(int(i), v)
    np.testing.assert_array_equal(t.nodes, z['c%d_nodes' % c])
    assert t.max_recorded_priority == z['c%d_maxrec' % c]
    for b in (1, 7, 32):
      rng = random.Random()
      rng.seed(1000 + c + b)
      got = t.stratified_sample(b, py_rng=rng)
      np.testing.assert_array_equal(got, z['c%d_strat%d' % (c, b)])
      assert rng.getstate()[1] == tuple(int(x) for x in z['c%d_strat%d_state' % (c, b)])
    rng = random.Random(); rng.seed(99 + c)
    got = [t.sample(py_rng=rng) for _ in range(10)]
    np.testing.assert_array_equal(got, z['c%d_single' % c])
    got = [t.sample(query_value=q) for q in (0.0, 0.25, 0.5, 0.999, 1.0)]
    np.testing.assert_array_equal(got, z['c%d_query' % c])


def build_from_golden(z, name, prioritized, py_rng=None, np_rng=None):
  C, n, stack, adds, B, rounds = [int(x) for x in z[name + '_meta']]
  gamma = float(z[name + '_gamma'])
  cls = orc.PrioritizedOracle if prioritized else orc.ReplayOracle
  mem = cls((8, 8), stack, C, B, update_horizon=n, gamma=gamma, py_rng=py_rng, np_rng=np_rng)
  obs, act, rew, term = (z[name + k] for k in ('_obs', '_act', '_rew', '_term'))
  for i in range(adds):
    if prioritized:
      mem.add(obs[i], act[i], rew[i], term[i], z[name + '_prio_in'][i])
    else:
      mem.add(obs[i], act[i], rew[i], term[i])
  assert mem.add_count == int(z[name + '_add_count'])
  return mem, B, rounds


@pytest.mark.parametrize('prioritized', [False, True])
def test_replay_golden(golden, prioritized):
  z = golden('replay_per.npz' if prioritized else 'replay_uniform.npz')
  keys = ['state', 'action', 'reward', 'next_state', 'next_action', 'next_reward',
          'terminal', 'indices'] + (['probs'] if prioritized else [])
  for name in _case_names(z):
    py_rng = random.Random()
    np_rng = np.random.RandomState()
    seed = int(z[name + '_seed'])
    py_rng.seed(seed)
    np_rng.seed(seed)
    mem, B, rounds = build_from_golden(z, name, prioritized, py_rng, np_rng)
    for r in range(rounds):
      batch = mem.sample_transition_batch()
      for k, v in zip(keys, batch):
        np.testing.assert_array_equal(v, z[name + '_' + k][r], err_msg='%s %s round %d' % (name, k, r))
      if prioritized:
        mem.set_priority(z[name + '_upd_idx'][r], z[name + '_upd_val'][r])
    if prioritized:
      np.testing.assert_array_equal(mem.sum_tree.nodes, z[name + '_nodes'])
      assert mem.sum_tree.max_recorded_priority == z[name + '_maxrec']
      assert py_rng.getstate()[1] == tuple(int(x) for x in z[name + '_rng_state'])
    else:
      st = np_rng.get_state()
      np.testing.assert_array_equal(np.array(st[1], np.int64), z[name + '_rng_state'])
      assert st[2] == int(z[name + '_rng_pos'])
    C = mem.C
    got = np.array([mem.is_valid_transition(i) for i in range(-2, C + 2)], np.uint8)
    np.testing.assert_array_equal(got, z[name + '_valid_mask'])
    fixed = [i for i in range(C) if mem.is_valid_transition(i)][:5]
    fb = mem.sample_transition_batch(batch_size=len(fixed), indices=fixed)
    for k, v in zip(keys, fb):
      np.testing.assert_array_equal(v, z[name + '_fixed_' + k])


def test_reference_checkpoint_fixture_is_plain_npy():
  """The reference-written uniform checkpoint holds only np.save data (loadable
  with allow_pickle=False), in the '<name>_ckpt.<iteration>.gz' layout of crb:593-594."""
  import gzip
  import os
  d = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'ckpt_uniform')
  names = sorted(f for f in os.listdir(d))
  assert names == sorted('{}_ckpt.7.gz'.format(a) for a in (
      '$store$_observation', '$store$_action', '$store$_reward', '$store$_terminal',
      'add_count', 'invalid_range'))
  for f in names:
    with gzip.open(os.path.join(d, f), 'rb') as fh:
      np.load(fh, allow_pickle=False)


SHAPE_KEYS = ['state', 'action', 'reward', 'next_state', 'next_action', 'next_reward',
              'terminal', 'indices']


def shape_case(z, name):
  """(kwargs, adds) of a tests/golden/replay_shapes.npz case (gen_golden.SHAPE_CASES)."""
  C, n, stack, adds, B, rounds = [int(x) for x in z[name + '_meta']]
  act, rew = z[name + '_act'], z[name + '_rew']
  kw = dict(observation_shape=(4, 4), stack_size=stack, replay_capacity=C, batch_size=B,
            update_horizon=n, gamma=float(z[name + '_gamma']), action_shape=act.shape[1:],
            action_dtype=act.dtype, reward_shape=rew.shape[1:], reward_dtype=rew.dtype)
  return kw, adds, rounds


def test_shapes_golden(golden):
  """Non-scalar / non-default action and reward elements (crb:96-183, 530-548)."""
  z = golden('replay_shapes.npz')
  for name in _case_names(z):
    kw, adds, rounds = shape_case(z, name)
    np_rng = np.random.RandomState(int(z[name + '_seed']))
    mem = orc.ReplayOracle(kw['observation_shape'], kw['stack_size'], kw['replay_capacity'],
                           kw['batch_size'], update_horizon=kw['update_horizon'],
                           gamma=kw['gamma'], np_rng=np_rng, action_shape=kw['action_shape'],
                           action_dtype=kw['action_dtype'], reward_shape=kw['reward_shape'],
                           reward_dtype=kw['reward_dtype'])
    for i in range(adds):
      mem.add(z[name + '_obs'][i], z[name + '_act'][i], z[name + '_rew'][i], z[name + '_term'][i])
    for r in range(rounds):
      for k, v in zip(SHAPE_KEYS, mem.sample_transition_batch()):
        np.testing.assert_array_equal(v, z[name + '_' + k][r], err_msg='%s %s %d' % (name, k, r))
        assert v.dtype == z[name + '_' + k].dtype, (name, k)
    fixed = [int(i) for i in z[name + '_fixed_indices']]
    for k, v in zip(SHAPE_KEYS, mem.sample_transition_batch(len(fixed), indices=fixed)):
      np.testing.assert_array_equal(v, z[name + '_fixed_' + k], err_msg='%s fixed %s' % (name, k))
    if name + '_bad_index' in z:
      with pytest.raises(ValueError) as e:
        mem.sample_transition_batch(1, indices=[int(z[name + '_bad_index'])])
      assert str(e.value) == str(z[name + '_bad_error'])
