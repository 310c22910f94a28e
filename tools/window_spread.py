"""Run-to-run spread of the learner loop: many consecutive timed windows on one agent
(bench protocol, synthetic 1M buffer), for the Rainbow headline and the DQN config.
    python tools/window_spread.py [windows] [steps]"""
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import torch  # noqa: E402

import bench  # noqa: E402


def main():
  windows = int(sys.argv[1]) if len(sys.argv) > 1 else 20
  steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
  dev = torch.device('cuda', 0)
  out = {}
  for name, make, A in (('rainbow', lambda: bench.build_agent(9, 1_000_000, 32, dev), 9),
                        ('dqn', lambda: bench.build_dqn_pong(dev), 6)):
    agent = make()
    import random
    random.seed(0)
    bench.fill_synthetic(agent._replay.memory, A, seed=1)
    torch.cuda.synchronize()
    bench.timed_steps(agent, 100, 30)
    rates = []
    gc.disable()
    for _ in range(windows):
      torch.cuda.synchronize()
      t0 = time.perf_counter()
      agent.train_gradient_steps(steps)
      torch.cuda.synchronize()
      rates.append(round(steps / (time.perf_counter() - t0), 1))
    gc.enable()
    out[name] = rates
    del agent
    gc.collect()
    torch.cuda.empty_cache()
  print(json.dumps(out))


if __name__ == '__main__':
  main()
