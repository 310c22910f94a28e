"""Config 5 (IQN Breakout) with HIP stream priorities: argv[1] = 'side:-1' runs the prefetch
stream (the target network beside the online backward) at high priority, 'main:-1' runs
the learner loop itself (the online network) on a high-priority stream, 'none' neither;
prints steps/s.
    python tools/iqn_priority.py side:-1 [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import contextlib  # noqa: E402
import random  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
from dopamine_amd.agents.dqn import dqn_agent  # noqa: E402

mode = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 150
torch.cuda.set_device(0)
if mode.startswith('side:'):
  dqn_agent.DQNAgent.side_priority = int(mode.split(':')[1])
ctx = contextlib.nullcontext()
if mode.startswith('main:'):
  s = torch.cuda.Stream(priority=int(mode.split(':')[1]))
  s.wait_stream(torch.cuda.current_stream())
  ctx = torch.cuda.stream(s)
with ctx:
  agent = bench.build_iqn_breakout(torch.device('cuda', 0))
  random.seed(0)
  bench.fill_synthetic(agent._replay.memory, 4, seed=1)
  torch.cuda.synchronize()
  el, _ = bench.timed_steps(agent, steps, 10)
print('%s: %.2f steps/s' % (mode, steps / el), flush=True)
