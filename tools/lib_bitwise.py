"""Are two builds of the library bitwise the same on a config's bench path?  Runs STEPS
learner-loop gradient steps of the config (bench.py's agents, synthetic 1M buffers, seeds
fixed) once per library in a child process and compares the online parameters, the target
parameters and the Adam moments bit for bit.
    python tools/lib_bitwise.py <lib A> <lib B> [iqn_breakout|rainbow|dqn_pong] [STEPS]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(cfg, steps, out):
  import random
  import numpy as np
  import torch
  import bench
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(0)
  make, A = {'iqn_breakout': (lambda: bench.build_iqn_breakout(dev), 4),
             'rainbow': (lambda: bench.build_agent(9, 1_000_000, 32, dev), 9),
             'dqn_pong': (lambda: bench.build_dqn_pong(dev), 6)}[cfg]
  agent = make()
  random.seed(0)
  np.random.seed(0)
  bench.fill_synthetic(agent._replay.memory, A, seed=1)
  agent.train_gradient_steps(steps)
  torch.cuda.synchronize()
  d = {'online': agent.online_convnet.fp.flat, 'target': agent.target_convnet.fp.flat}
  for k, v in vars(agent._opt).items():
    if isinstance(v, torch.Tensor) and v.data_ptr() != agent.online_convnet.fp.flat.data_ptr():
      d['opt_' + k] = v
  np.savez(out, **{k: v.detach().cpu().numpy() for k, v in d.items()})


def main():
  if sys.argv[1] == '--child':
    return child(sys.argv[2], int(sys.argv[3]), sys.argv[4])
  import numpy as np
  a, b = sys.argv[1], sys.argv[2]
  cfg = sys.argv[3] if len(sys.argv) > 3 else 'iqn_breakout'
  steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
  res = []
  for i, lib in enumerate((a, b)):
    out = '/tmp/lib_bitwise_%d.npz' % i
    env = dict(os.environ, DOPAMINE_AMD_LIB=lib, DQ_DIAGNOSTIC_BUILD='1')
    p = subprocess.run([sys.executable, os.path.abspath(__file__), '--child', cfg, str(steps), out],
                       env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-1500:]
    res.append(dict(np.load(out)))
  same = True
  for k in res[0]:
    eq = np.array_equal(res[0][k].view(np.int32) if res[0][k].dtype == np.float32 else res[0][k],
                        res[1][k].view(np.int32) if res[1][k].dtype == np.float32 else res[1][k])
    d = float(np.abs(res[0][k].astype(np.float64) - res[1][k]).max())
    print('%-12s bitwise %-5s max |diff| %.3e' % (k, eq, d))
    same = same and eq
  print('%s after %d %s steps: %s' % ('BITWISE EQUAL' if same else 'DIFFERENT', steps, cfg,
                                      (a, b)))


if __name__ == '__main__':
  main()
