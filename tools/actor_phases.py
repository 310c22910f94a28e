"""Host-clock breakdown of the acting loop (agent.step with training): time spent in
_store_transition, _train_step and _select_action per env step, Rainbow vs DQN.
    python tools/actor_phases.py [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from tools.bench_actor import run  # noqa: E402,F401


def phases(kind, steps):
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent
  from dopamine_amd.agents.optimizers import AdamOptimizer
  dev = torch.device('cuda', 0)
  if kind == 'rainbow':
    agent = RainbowAgent(num_actions=9, update_horizon=3, min_replay_history=20000,
                         optimizer=AdamOptimizer(learning_rate=6.25e-5, epsilon=1.5e-4),
                         replay_capacity=1_000_000, device=dev)
  else:
    agent = DQNAgent(num_actions=6, min_replay_history=20000, replay_capacity=1_000_000, device=dev)
  bench.fill_synthetic(agent._replay.memory, agent.num_actions, seed=1)
  acc = {}
  for name in ('_store_transition', '_train_step', '_select_action'):
    f = getattr(agent, name)

    def timed(*a, _f=f, _n=name, **k):
      t = time.perf_counter()
      r = _f(*a, **k)
      acc[_n] = acc.get(_n, 0.0) + time.perf_counter() - t
      return r
    setattr(agent, name, timed)
  rs = np.random.RandomState(0)
  frames = rs.randint(0, 256, (64, 84, 84)).astype(np.uint8)
  agent.begin_episode(frames[0])
  for i in range(50):
    agent.step(0.0, frames[i % 64])
  torch.cuda.synchronize()
  acc.clear()
  t = time.perf_counter()
  for i in range(steps):
    agent.step(float(i % 3 - 1), frames[i % 64])
  torch.cuda.synchronize()
  dt = time.perf_counter() - t
  out = {k: round(1e6 * v / steps, 1) for k, v in acc.items()}
  out['total_us_per_env_step'] = round(1e6 * dt / steps, 1)
  return out


print(json.dumps({k: phases(k, 2000) for k in ('rainbow', 'dqn')}))
