"""Actor-loop throughput: agent.step(reward, observation) with Atari-shaped
84x84 uint8 frames from a synthetic source -- per env step the agent records
the observation, adds the transition to the device buffer, trains every 4th
step (HIP graph) and selects an epsilon-greedy action with the online network.
    python tools/bench_actor.py [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def run(kind, steps, train, device_egreedy=True):
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent
  from dopamine_amd.agents.optimizers import AdamOptimizer
  dev = torch.device('cuda', 0)
  if kind == 'rainbow':
    agent = RainbowAgent(num_actions=9, update_horizon=3, min_replay_history=20000,
                         optimizer=AdamOptimizer(learning_rate=6.25e-5, epsilon=1.5e-4),
                         replay_capacity=1_000_000, device=dev)
  else:
    agent = DQNAgent(num_actions=6, min_replay_history=20000, replay_capacity=1_000_000,
                     device=dev)
  bench.fill_synthetic(agent._replay.memory, agent.num_actions, seed=1)
  agent.eval_mode = not train
  agent.device_egreedy = device_egreedy
  rs = np.random.RandomState(0)
  frames = rs.randint(0, 256, (64, 84, 84)).astype(np.uint8)
  agent.begin_episode(frames[0])
  for i in range(50):
    agent.step(0.0, frames[i % 64])
  torch.cuda.synchronize()
  t = time.perf_counter()
  for i in range(steps):
    agent.step(float(i % 3 - 1), frames[i % 64])
  torch.cuda.synchronize()
  dt = time.perf_counter() - t
  return steps / dt


def main():
  steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
  for kind in ('rainbow', 'dqn'):
    print('%-8s train: %8.1f env steps/s   eval (act only): %8.1f env steps/s' % (
        kind, run(kind, steps, True), run(kind, steps, False)))
  # PER's epsilon-greedy draws on the host (sync + draw per action) instead of on the tape
  print('%-8s train: %8.1f env steps/s   eval (act only): %8.1f env steps/s  (host epsilon-greedy)' % (
      'rainbow', run('rainbow', steps, True, False), run('rainbow', steps, False, False)))


if __name__ == '__main__':
  main()
