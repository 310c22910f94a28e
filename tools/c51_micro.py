"""Device time of the C51 loss kernel variants at B = 32, A = 9 (graph of 100):
stored logits, fc2 partials (fused) + d h, and the fused forward.
    python tools/c51_micro.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dopamine_amd import ops  # noqa: E402
from dopamine_amd.agents.networks import RainbowNetwork  # noqa: E402
from dopamine_amd.cnn import HipNatureCNN, forward_fused  # noqa: E402


def timed(fn, reps=100):
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):
    fn()
  torch.cuda.current_stream().wait_stream(s)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(reps):
      fn()
  g.replay()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  e0.record()
  g.replay()
  e1.record()
  torch.cuda.synchronize()
  return e0.elapsed_time(e1) * 1e3 / reps


def main():
  B, A, N = 32, 9, 51
  on, tg = RainbowNetwork(A, device='cuda', seed=1), RainbowNetwork(A, device='cuda', seed=2)
  ho, ht = HipNatureCNN(on, B), HipNatureCNN(tg, B)
  x, nx = torch.rand(B, 84, 84, 4, device='cuda'), torch.rand(B, 84, 84, 4, device='cuda')
  act = torch.randint(0, A, (B,), device='cuda', dtype=torch.int32)
  rew = torch.randn(B, device='cuda')
  term = (torch.rand(B, device='cuda') < 0.2).to(torch.uint8)
  probs = torch.rand(B, device='cuda') + 0.1
  sup = torch.linspace(-10, 10, N, device='cuda')
  yt = ht.forward(nx)
  yo = ho.forward(x)
  forward_fused(ho, x, ht)
  out = ops.c51_loss(yo.view(B, A, N), yt.view(B, A, N), act, rew, term, sup, 0.97, probs=probs)
  print('c51 stored logits       %7.2f us' % timed(lambda: ops.c51_loss(
      yo.view(B, A, N), yt.view(B, A, N), act, rew, term, sup, 0.97, probs=probs, out=out)))
  print('c51 fused + dh          %7.2f us' % timed(lambda: ops.c51_loss_fused(
      ho, ht, act, rew, term, sup, 0.97, probs=probs, out=out)))
  from dopamine_amd import _lib, cnn
  from dopamine_amd.ops import p as ptr, _stream
  po, pt = cnn.fc2_parts(ho), cnn.fc2_parts(ht)

  def nodh():
    _lib.call('dq_c51_loss_fused', ptr(po), ho._p.fc2_b, ptr(pt), ht._p.fc2_b, 16, ptr(act), ptr(rew),
              ptr(term), ptr(probs), ptr(sup), B, A, N, 0.97, ptr(out['grad']), ptr(out['loss']),
              ptr(out['priorities']), None, None, None, 512, None, None, _stream(sup))
  print('c51 fused, no dh        %7.2f us' % timed(nodh))
  print('forward_fused           %7.2f us' % timed(lambda: forward_fused(ho, x, ht)))
  print('forward_fused (no tfc1) %7.2f us' % timed(lambda: forward_fused(ho, x, ht, fc1_b=False)))
  print('forward                 %7.2f us' % timed(lambda: ho.forward(x)))


if __name__ == '__main__':
  main()
