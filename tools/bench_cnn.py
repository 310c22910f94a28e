"""Micro-benchmark of the Rainbow Nature-CNN learner step variants on one GPU.

Times (HIP-graph replay) online fwd + target fwd + online bwd at B=32 for:
NCHW vs channels_last, flat-grad accumulation vs fresh grads.
    PYTORCH_MIOPEN_SUGGEST_NHWC=1 python tools/bench_cnn.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dopamine_amd.agents.networks import RainbowNetwork  # noqa: E402


def bench(fn, iters=200):
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):
    for _ in range(3):
      fn()
  torch.cuda.current_stream().wait_stream(s)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    fn()
  g.replay()
  torch.cuda.synchronize()
  t = time.perf_counter()
  for _ in range(iters):
    g.replay()
  torch.cuda.synchronize()
  return (time.perf_counter() - t) / iters * 1e6


def main():
  dev = torch.device('cuda')
  B = 32
  for cl in (False, True):
    on = RainbowNetwork(9, device=dev, seed=0)
    tg = RainbowNetwork(9, device=dev, seed=1)
    x = torch.rand(B, 4, 84, 84, device=dev)
    nx = torch.rand(B, 4, 84, 84, device=dev)
    if cl:
      x = x.contiguous(memory_format=torch.channels_last)
      nx = nx.contiguous(memory_format=torch.channels_last)
      for net in (on, tg):
        for n, p in net.fp.params.items():
          if p.dim() == 4:
            p.data = p.data.contiguous(memory_format=torch.channels_last)
            p.grad = None
    gout = torch.randn(B, 9, 51, device=dev)

    def fwd_only():
      with torch.no_grad():
        tg(nx)
        on(x)

    def step():
      with torch.no_grad():
        tg(nx)
      y = on(x)
      on.fp.grad.zero_()
      y.backward(gout)

    def step_fresh():
      for p in on.parameters():
        p.grad = None
      with torch.no_grad():
        tg(nx)
      y = on(x)
      y.backward(gout)

    tag = 'channels_last' if cl else 'NCHW'
    print('%-14s fwd(online+target) %7.1f us' % (tag, bench(fwd_only)))
    if not cl:
      print('%-14s step flat-grad     %7.1f us' % (tag, bench(step)))
    print('%-14s step fresh-grad    %7.1f us' % (tag, bench(step_fresh)))
    with torch.autocast('cuda', dtype=torch.bfloat16):
      print('%-14s bf16 step fresh    %7.1f us' % (tag, bench(step_fresh)))


if __name__ == '__main__':
  main()
