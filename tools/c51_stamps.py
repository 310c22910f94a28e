"""Per-stage wall-clock stamps inside k_c51 (fused path, B = 32, A = 9), from a
-DDQ_C51_PROF build:  DOPAMINE_AMD_LIB=<that .so> python tools/c51_stamps.py
Stages: 0 start, 1 target softmax done, 2 first barrier, 3 PER weight,
4 loss/gradient (wave 0), 5 W2 rows landed, 6 d h done.  Units: us (100 MHz clock)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dopamine_amd import _lib, ops  # noqa: E402
from dopamine_amd.agents.networks import RainbowNetwork  # noqa: E402
from dopamine_amd.cnn import HipNatureCNN, forward_fused  # noqa: E402


SPLIT = int(os.environ.get('DQ_C51_SPLIT', '4'))   # blocks per sample of the build


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
  ht.forward(nx)
  fn = _lib.lib.dq_debug_c51_times
  fn.argtypes = [ctypes.c_void_p]
  buf = np.zeros((256, 8), np.int64)
  wfn = _lib.lib.dq_debug_c51_wave_times
  wfn.argtypes = [ctypes.c_void_p]
  wbuf = np.zeros((3, 256, 16), np.int64)
  rows, wrows = [], []
  for it in range(30):
    forward_fused(ho, x, ht)
    ops.c51_loss_fused(ho, ht, act, rew, term, sup, 0.97, probs=probs)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data) == 0
    if it >= 10:
      t = buf[:B * SPLIT, :7].astype(np.float64)
      t = (t - t[:, 0].min()) / 100.0
      rows.append(t)
      assert wfn(wbuf.ctypes.data) == 0
      wrows.append((wbuf[:, :B * SPLIT, :A].astype(np.float64) - buf[:B * SPLIT, 0].min()) / 100.0)
  r = np.median(np.stack(rows), axis=0)       # (B, 7) median over iterations
  print('stage   median-over-blocks   max-over-blocks (us from first block start)')
  for k in range(7):
    print('%d  %8.2f  %8.2f' % (k, np.median(r[:, k]), r[:, k].max()))
  d = r[:, 4] - r[:, 3]
  tm = np.repeat(term.cpu().numpy(), SPLIT)
  order = np.argsort(d)
  print('stage 3->4 per block (us, terminal):', ' '.join('%.2f%s' % (d[i], '*' if tm[i] else '') for i in order))
  d = r[:, 6] - r[:, 5]
  print('stage 5->6 per block (us, terminal):', ' '.join('%.2f%s' % (d[i], '*' if tm[i] else '') for i in np.argsort(d)))
  w = np.median(np.stack(wrows), axis=0)
  print('inputs in per wave  :', ' '.join('%.2f' % v for v in np.median(w[2], axis=0)))
  print('c(i,j) done per wave:', ' '.join('%.2f' % v for v in np.median(w[1], axis=0)))
  print('stage 1 per wave    :', ' '.join('%.2f' % v for v in np.median(w[0], axis=0)))


if __name__ == '__main__':
  main()
