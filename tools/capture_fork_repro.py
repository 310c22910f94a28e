"""Minimal HIP-graph capture of the ZeRO-1 two-stream update pattern, with no RCCL and
none of this package's kernels: per step, main -> A (fork), A -> B (fork), B -> A (join),
A -> main (join, consumed at the next step), for `steps` steps in ONE capture.
    python tools/capture_fork_repro.py <steps> <variant>
variant 'plain': as above; 'direct': main also waits on B directly before capture end.
Prints 'ok' (and checks the replayed values) or dies in capture_end."""
import sys

import torch


def main():
  steps, variant = int(sys.argv[1]), sys.argv[2]
  torch.cuda.set_device(0)
  main_s = torch.cuda.current_stream()
  a, b = torch.cuda.Stream(), torch.cuda.Stream()
  x = torch.zeros(1 << 20, device='cuda')
  y = torch.zeros(1 << 20, device='cuda')
  cap = torch.cuda.Stream()
  cap.wait_stream(main_s)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.stream(cap):
    with torch.cuda.graph(g, stream=cap):
      pending = None
      for _ in range(steps):
        if pending is not None:
          cap.wait_event(pending)
        x.add_(1.0)                      # "head" on the origin stream
        ev = torch.cuda.Event()
        ev.record(cap)
        a.wait_event(ev)
        with torch.cuda.stream(a):
          x.mul_(2.0)                    # "reduce-scatter"
        e1 = torch.cuda.Event()
        e1.record(a)
        b.wait_event(e1)
        with torch.cuda.stream(b):
          y.add_(x)                      # "the slice's update"
        e2 = torch.cuda.Event()
        e2.record(b)
        a.wait_event(e2)
        with torch.cuda.stream(a):
          x.add_(y)                      # "all-gather"
        pending = torch.cuda.Event()
        pending.record(a)
      cap.wait_event(pending)
      if variant == 'direct':
        cap.wait_stream(b)
  print('captured', steps, variant, flush=True)
  g.replay()
  torch.cuda.synchronize()
  xr, yr = 0.0, 0.0
  for _ in range(steps):
    xr = (xr + 1) * 2
    yr += xr
    xr += yr
  assert float(x[0]) == xr and float(y[0]) == yr, (float(x[0]), xr, float(y[0]), yr)
  print('ok', flush=True)


if __name__ == '__main__':
  main()
