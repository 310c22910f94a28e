"""Is the short window's first-chunk cost the host's submission of a 4-step graph to an idle
device?  After bench.py's priming, alternates 20-step windows timed as bench.timed_steps
does: (a) train_gradient_steps(20) -- five chunk graphs; (b) train_gradient_steps(1) then
(19) -- a one-step graph first (12 packets to submit instead of ~48), four chunks, three
single steps.  If (b) is not slower despite its four extra graph boundaries (~5 us each),
the first chunk's extra is submission.
    python tools/window_split_probe.py [REPEATS]"""
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
  import bench
  reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(0)
  agent = bench.build_agent(9, 1_000_000, 32, dev)
  import random
  random.seed(0)
  bench.fill_synthetic(agent._replay.memory, 9, seed=1)
  torch.cuda.synchronize()
  bench.timed_steps(agent, 20, 5)          # priming
  agent.train_gradient_steps(1)             # the single-step graphs of both parities
  agent.train_gradient_steps(1)
  torch.cuda.synchronize()

  def window(split):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if split:
      agent.train_gradient_steps(1)
      agent.train_gradient_steps(19)
    else:
      agent.train_gradient_steps(20)
    torch.cuda.synchronize()
    return time.perf_counter() - t0

  res = {False: [], True: []}
  gc.disable()
  for _ in range(reps):
    for split in (False, True):
      agent.train_gradient_steps(40)        # busy device before each window, as bench's warmup
      res[split].append(window(split))
  gc.enable()
  for split, v in res.items():
    v = np.array(v) * 1e6
    print('%-34s median %.1f us (p10 %.1f, p90 %.1f) -> %.0f steps/s' % (
        'one-step graph first, then 19' if split else 'train_gradient_steps(20)',
        np.median(v), np.percentile(v, 10), np.percentile(v, 90), 20 / np.median(v) * 1e6))


if __name__ == '__main__':
  main()
