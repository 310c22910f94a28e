"""Why the bench's 20-step bf16 throughput row reports the same Rainbow loss as the fp32
headline to five decimals.  The bench protocol (bench.build_agent, the
synthetic 1M buffer, priming, warmup, a window of STEPS learner steps) runs once on the
product library and once on the bf16 build, each in a child process with the step trace on;
the parent compares what the last step saw and computed: sampled indices, online logits,
per-sample losses and the mean the bench prints.
    python tools/bf16_vs_fp32.py [STEPS]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(steps, out):
  import numpy as np
  import torch
  import random
  import bench
  from dopamine_amd import _lib
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(0)
  agent = bench.build_agent(9, 1_000_000, 32, dev)
  agent.enable_trace()
  random.seed(0)
  bench.fill_synthetic(agent._replay.memory, 9, seed=1)
  torch.cuda.synchronize()
  hist = []
  elapsed, prime = bench.timed_steps(agent, steps, 5)
  agent._replay.memory.sync_rng()
  loss = agent.mean_loss()
  U = agent._UNROLL
  # the last step's trace slot: a chunk's last step (slot U - 1) unless the window ended in
  # a single-step call (slot U + parity)
  last = U - 1 if steps % U == 0 else U + (agent._opt_steps - 1) % 2
  tr = {k: v[last].cpu().numpy() for k, v in agent._trace.items()}
  w = 1.0 / np.sqrt(tr['sampling_probabilities'] + np.float32(1e-10))
  traced = float((tr['loss'] * (w / w.max())).mean(dtype=np.float32))   # mean(w * CE), rb:298-301
  np.savez(out, loss_mean=np.float64(loss), step_loss=tr['loss'], logits=tr['online_out'],
           indices=tr['indices'], total_steps=agent._opt_steps, prime=prime, traced=traced)
  print(json.dumps({'library': _lib.BUILD_FLAGS, 'mean_loss': loss, 'trace_weighted_mean': traced,
                    'steps': int(agent._opt_steps)}))


def main():
  steps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1] != '--child' else 20
  if '--child' in sys.argv:
    return child(int(sys.argv[2]), sys.argv[3])
  import numpy as np
  from dopamine_amd import _build
  res = {}
  for name, lib in (('fp32', _build.PRODUCT_LIB_PATH), ('bf16', _build.BF16_LIB_PATH)):
    out = '/tmp/bf16_vs_fp32_%s.npz' % name
    env = dict(os.environ, DOPAMINE_AMD_LIB=lib)
    p = subprocess.run([sys.executable, os.path.abspath(__file__), '--child', str(steps), out],
                       env=env, capture_output=True, text=True, timeout=600)
    print(name, p.stdout.strip().splitlines()[-1] if p.stdout.strip() else p.stderr[-800:])
    res[name] = dict(np.load(out))
  a, b = res['fp32'], res['bf16']
  d = np.abs(a['logits'].astype(np.float64) - b['logits'])
  print('gradient steps taken (priming + warmup + window): %d / %d' % (a['total_steps'],
                                                                       b['total_steps']))
  print('last step: indices equal: %s' % bool(np.array_equal(a['indices'], b['indices'])))
  print('last step: online logits max |fp32 - bf16| %.3e (max |logit| %.3e, relative %.3e)' % (
      d.max(), np.abs(a['logits']).max(), d.max() / np.abs(a['logits']).max()))
  dl = np.abs(a['step_loss'].astype(np.float64) - b['step_loss'])
  print('last step: per-sample losses max |diff| %.3e (mean loss %.8f vs %.8f, diff %.3e)' % (
      dl.max(), a['loss_mean'], b['loss_mean'], abs(a['loss_mean'] - b['loss_mean'])))
  print('mean_loss() against the trace\'s last step (mean(w * CE) on the host, float32): fp32 '
        '%.3e, bf16 %.3e apart' % (abs(a['loss_mean'] - a['traced']), abs(b['loss_mean'] - b['traced'])))


if __name__ == '__main__':
  main()
