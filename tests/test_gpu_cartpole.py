"""BASELINE config 1 (DQN on CartPole-v0, dqn_cartpole.gin) -- Q-values and losses on
identical minibatches.

The agent is made exactly as the Runner makes it (gin_lite reads the reference's
dqn_cartpole.gin: float64 (4, 1) observations, stack 1, the 512-512 MLP of
gym_lib.py:75-132, Adam 1e-3 / 3.125e-4, batch 128, uniform replay of 50,000), its
buffer is filled by CartPole-v0 episodes of random actions, and it trains through
``_train_step`` (eager steps, then the captured HIP graph).  Every gradient step is
checked against float64 at the device's parameters of that step:
  * indices bit-exact: the oracle's numpy-legacy uniform sampler from the same state;
  * Q(s) and the target net's Q(s') within 1e-5 of scale (float64 MLP on the float32
    rescaled input the reference computes, gym_lib.py:97-100);
  * per-sample Huber losses (dqn_agent.py:283-322) within 1e-5 of scale;
  * every parameter gradient within 1e-5 per tensor; the Adam update from the device's
    state and gradient within 5e-8."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import learner as OL
from oracle import replay as OR

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIN = os.path.join(ROOT, 'dopamine_amd', 'agents', 'dqn', 'configs', 'dqn_cartpole.gin')
TOL = 1e-5


def _rel(got, ref):
  got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
  return float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))


def _mlp64(flat, offsets, state):
  """float64 cartpole_dqn_network (gym_lib.py:75-132) on the float32 rescaled input."""
  from dopamine_amd.agents.networks import CartpoleDQNNetwork as C
  P = {n: torch.tensor(flat[o:o + int(np.prod(s))].reshape(s), dtype=torch.float64,
                       requires_grad=True) for n, (o, s) in offsets.items()}
  x = np.asarray(state, np.float64).reshape(len(state), -1).astype(np.float32)
  x = np.float32(2.0) * ((x - C.MIN.astype(np.float32)) / (C.MAX - C.MIN).astype(np.float32)) \
      - np.float32(1.0)
  h = torch.from_numpy(x).double()
  i = 0
  while 'fc%d_w' % i in P:
    h = F.relu(F.linear(h, P['fc%d_w' % i], P['fc%d_b' % i]))
    i += 1
  return F.linear(h, P['out_w'], P['out_b']), P


def test_cartpole_dqn_steps_match_float64_oracle():
  from dopamine_amd import gin_lite
  from dopamine_amd.discrete_domains import gym_lib, run_experiment
  gin_lite.clear_config()
  run_experiment.load_gin_configs([GIN], [])
  env = gym_lib.create_gym_environment()
  np.random.seed(0)
  import random
  random.seed(0)
  agent = run_experiment.create_agent(None, env)
  gin_lite.clear_config()
  assert agent._batch_size == 128 and agent.observation_shape == (4, 1)
  agent.enable_trace()
  rs = np.random.RandomState(1)
  obs = env.reset()
  for _ in range(3000):                 # random-action CartPole episodes into the buffer
    a = int(rs.randint(2))
    nobs, r, done, _ = env.step(a)
    agent._replay.add(np.asarray(obs).reshape(4, 1), a, r, done)
    obs = env.reset() if done else nobs
  mem = agent._replay.memory
  C, B = mem._replay_capacity, agent._batch_size
  orc = OR.ReplayOracle((4, 1), 1, C, B, update_horizon=1, gamma=0.99,
                        observation_dtype=np.float64)
  orc.observation = mem._frames.cpu().numpy().view(np.float64).reshape(C, 4, 1)
  orc.action = mem._actions.cpu().numpy()
  orc.reward = mem._rewards.cpu().numpy()
  orc.terminal = mem._terminals.cpu().numpy()
  orc.add_count = int(mem.add_count)
  orc.invalid_range = OR.invalid_range(orc.cursor(), C, 1, 1)
  orc.np_rng = np.random.RandomState()
  orc.np_rng.set_state(np.random.get_state())
  offsets = agent.online_convnet.fp.offsets
  cg = np.float64(np.float32(agent.cumulative_gamma))
  U = agent._UNROLL
  errs = dict(q=0.0, target_q=0.0, loss=0.0, grad={}, params=0.0)
  for step in range(10):
    k = agent._opt_steps % 2
    w = agent.online_convnet.fp.flat.detach().cpu().double().numpy().copy()
    tw = agent.target_convnet.fp.flat.detach().cpu().double().numpy().copy()
    opt = agent._opt
    m, v = opt.m.cpu().double().numpy().copy(), opt.v.cpu().double().numpy().copy()
    st = opt.state.cpu().double().numpy()
    for _ in range(agent.update_period):   # one gradient step, the reference's cadence
      agent._train_step()
    torch.cuda.synchronize()
    tr = {n: t[U + k].detach().cpu().numpy() for n, t in agent._trace.items()}
    idx = orc.sample_index_batch(B)
    np.testing.assert_array_equal(tr['indices'], idx)
    s, act, rew, ns, _, _, term, _ = orc.sample_transition_batch(B, indices=idx)
    q, P = _mlp64(w, offsets, s)
    with torch.no_grad():
      tq, _ = _mlp64(tw, offsets, ns)
    errs['q'] = max(errs['q'], _rel(tr['online_out'], q.detach().numpy()))
    errs['target_q'] = max(errs['target_q'], _rel(tr['target_out'], tq.numpy()))
    ref = OL.dqn_huber(q.detach().numpy(), tq.numpy(), act, rew, term, cg, dtype=np.float64)
    errs['loss'] = max(errs['loss'], _rel(tr['loss'], ref['loss']))
    q.backward(torch.from_numpy(ref['grad']))
    for n, (o, shape) in offsets.items():
      size = int(np.prod(shape))
      errs['grad'][n] = max(errs['grad'].get(n, 0.0),
                            _rel(tr['grad'][o:o + size], P[n].grad.numpy().reshape(-1)))
    # float64 TF1 Adam from the device's state with the device's gradient
    g = tr['grad'].astype(np.float64)
    f = lambda x: np.float64(np.float32(x))
    b1, b2, lr, eps = f(opt.b1), f(opt.b2), f(opt.lr), f(opt.eps)
    b1p, b2p = st[2 * k], st[2 * k + 1]
    m += (g - m) * (1 - b1)
    v += (g * g - v) * (1 - b2)
    w -= lr * np.sqrt(1 - b2p) / (1 - b1p) * m / (np.sqrt(v) + eps)
    gw = agent.online_convnet.fp.flat.detach().cpu().double().numpy()
    errs['params'] = max(errs['params'], float(np.abs(gw - w).max()))
  print('cartpole errors', errs, flush=True)
  assert errs['q'] <= TOL and errs['target_q'] <= TOL and errs['loss'] <= TOL, errs
  assert max(errs['grad'].values()) <= TOL, errs
  assert errs['params'] <= 5e-8, errs
  assert agent._graphs is not None            # the later steps replayed the captured graph
