"""Rainbow learner steps on synthetic replay; saves the online parameters and the
sampled indices (np.save) -- run under two DOPAMINE_AMD_LIB builds to check that
a kernel change is bitwise neutral.   python tools/dump_params.py out.npz [steps] [ride] [fuse]"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
  out = sys.argv[1]
  steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
  ride = bool(int(sys.argv[3])) if len(sys.argv) > 3 else True
  fuse = bool(int(sys.argv[4])) if len(sys.argv) > 4 else False
  from dopamine_amd.agents.optimizers import AdamOptimizer
  from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent
  random.seed(0); np.random.seed(0); torch.manual_seed(0)
  kw = {'fuse_optimizer': fuse}
  if not ride:
    kw['ride_replay'] = False
  a = RainbowAgent(num_actions=9, update_horizon=3, replay_capacity=100_000, batch_size=32,
                   min_replay_history=100, device=torch.device('cuda', 0),
                   optimizer=AdamOptimizer(learning_rate=6.25e-5, epsilon=1.5e-4), **kw)
  bench.fill_synthetic(a._replay.memory, 9, seed=1)
  idx = []
  for _ in range(steps):
    a._run_train_op()
    idx.append(a._replay.transition['indices'].cpu().numpy().copy())
  torch.cuda.synchronize()
  np.savez(out, params=a.online_convnet.fp.flat.cpu().numpy(), idx=np.stack(idx),
           loss=a._loss_out['loss'].cpu().numpy())


if __name__ == '__main__':
  main()
