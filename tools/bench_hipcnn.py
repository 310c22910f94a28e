"""A/B of the learner's CNN work per step on one GPU: HIP Nature-CNN kernels vs
PyTorch/MIOpen (channels_last), each captured in a HIP graph:
target fwd + online fwd + online bwd at B=32 (Rainbow head, 459 outputs).
    python tools/bench_hipcnn.py [iters]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dopamine_amd.agents.networks import RainbowNetwork  # noqa: E402
from dopamine_amd.cnn import HipNatureCNN  # noqa: E402


def bench(fn, iters):
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
  iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
  dev = torch.device('cuda')
  B = 32
  on = RainbowNetwork(9, device=dev, seed=0)
  tg = RainbowNetwork(9, device=dev, seed=1)
  x = torch.rand(B, 84, 84, 4, device=dev)
  nx = torch.rand(B, 84, 84, 4, device=dev)
  gout = torch.randn(B, 459, device=dev)
  hon, htg = HipNatureCNN(on, B), HipNatureCNN(tg, B)

  def hip_fwd():
    htg.forward(nx)
    hon.forward(x)

  def hip_step():
    htg.forward(nx)
    hon.forward(x)
    hon.backward(gout)

  def hip_bwd():
    hon.backward(gout)

  xc, nxc = x.permute(0, 3, 1, 2), nx.permute(0, 3, 1, 2)

  def torch_step():
    for p in on.parameters():
      p.grad = None
    with torch.no_grad():
      tg(nxc)
    y = on(xc).reshape(B, -1)
    y.backward(gout)

  print('hip   fwd(online+target) %7.1f us' % bench(hip_fwd, iters))
  print('hip   bwd(online)        %7.1f us' % bench(hip_bwd, iters))
  print('hip   step               %7.1f us' % bench(hip_step, iters))
  print('torch step               %7.1f us' % bench(torch_step, iters))


if __name__ == '__main__':
  main()
