"""Gradient-steps/s for the other single-GPU BASELINE configs, measured like
bench.py (synthetic full 1M-transition buffer in HBM, HIP graph, the reference's
_train_step cadence), for DESIGN.md -- not the bench line:

  config 2: DQN / Pong   -- 6 actions, uniform replay, n = 1, TF1 centered RMSProp, B = 32
  config 5: IQN / Breakout -- 4 actions, n = 3, Adam, B = 64 (quantile-Huber kernel)

    python tools/bench_configs.py [steps] [dqn_pong|iqn_breakout|all]
"""
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import torch  # noqa: E402

import bench  # noqa: E402


def measure(make, actions, steps, warmup=20):
  agent = make()
  import random
  random.seed(0)
  bench.fill_synthetic(agent._replay.memory, actions, seed=1)
  torch.cuda.synchronize()

  agent.train_gradient_steps(warmup)     # = update_period _train_step() calls per step
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  agent.train_gradient_steps(steps)
  torch.cuda.synchronize()
  dt = time.perf_counter() - t0
  agent._replay.memory.sync_rng()
  out = {'steps_per_s': round(steps / dt, 1), 'ms_per_step': round(1e3 * dt / steps, 4),
         'batch': agent._batch_size,
         'hip_cnn': agent._hip is not None or getattr(agent, '_iqn', None) is not None}
  del agent
  gc.collect()
  torch.cuda.empty_cache()
  return out


def main():
  steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
  which = sys.argv[2] if len(sys.argv) > 2 else 'all'
  extra = {}
  for a in sys.argv[3:]:            # agent keyword overrides, e.g. pipeline=0
    k, v = a.split('=')
    extra[k] = bool(int(v))
  dev = torch.device('cuda', 0)
  res = {}
  if which in ('all', 'dqn_pong'):
    res['dqn_pong'] = measure(lambda: bench.build_dqn_pong(dev, **extra), 6, steps)
  if which in ('all', 'iqn_breakout'):
    res['iqn_breakout'] = measure(lambda: bench.build_iqn_breakout(dev, **extra), 4,
                                  max(steps // 3, 50))
  print(json.dumps(res))


if __name__ == '__main__':
  main()
