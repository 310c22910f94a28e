"""Config 2 (DQN Pong, uniform replay): the learner loop with the chunk gather off, or with
its K * B gather riding in backward launch argv[1] (2, 3 or 4); prints steps/s.
    python tools/dqn_chunk_ab.py off|2|3|4 [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import random  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dopamine_amd.agents.dqn import dqn_agent  # noqa: E402

mode = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
if mode == 'off':
  dqn_agent.DQNAgent.chunk_gather = False
else:
  dqn_agent.DQNAgent.chunk_gather_launch = int(mode)
torch.cuda.set_device(0)
agent = bench.build_dqn_pong(torch.device('cuda', 0))
random.seed(0)
np.random.seed(0)
bench.fill_synthetic(agent._replay.memory, 6, seed=1)
torch.cuda.synchronize()
el, _ = bench.timed_steps(agent, steps, 10)
print('chunk gather %s: %.2f steps/s' % (mode, steps / el), flush=True)
