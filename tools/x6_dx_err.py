"""IQN head backward's dX GEMM in isolation: from the device's own dh, emb and state, the
float64 d pre = (emb > 0) * (dh W1) * state and d state = sum_q (dh W1) * emb (before the
torso's ReLU), against what the device wrote.  Run once per library (DOPAMINE_AMD_LIB)
to compare the exact-f32 and split-bf16 GEMM forms.
    python tools/x6_dx_err.py [B nq]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dopamine_amd.agents.networks import ImplicitQuantileNetwork  # noqa: E402
from dopamine_amd.iqn import HipIqnNet, F  # noqa: E402


def main():
  B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
  nq = int(sys.argv[2]) if len(sys.argv) > 2 else 64
  A = 4
  torch.manual_seed(0)
  net = ImplicitQuantileNetwork(A, device='cuda', seed=3)
  with torch.no_grad():
    for n in ('conv1_b', 'conv2_b', 'conv3_b', 'emb_b', 'fc1_b', 'fc2_b'):
      net.fp[n].uniform_(-0.05, 0.05)
  rs = np.random.RandomState(B)
  x = torch.from_numpy(rs.randint(0, 256, (B, 84, 84, 4)).astype(np.float32) / np.float32(255))
  taus = torch.from_numpy(rs.rand(nq * B).astype(np.float32))
  ex = HipIqnNet(net, B, nq, keep=True)
  ex.forward(x.cuda(), taus.cuda())
  dq = torch.from_numpy(rs.randn(nq * B, A).astype(np.float32) / (nq * B))
  ex.backward(dq.cuda())
  torch.cuda.synchronize()
  R = B * nq
  dh = ex.grads['dh'].double().cpu().numpy()                       # (R, 512), row q B + b
  emb = ex.acts['emb'].double().cpu().numpy()                      # (R, F)
  state = ex.torso.acts['a3'].reshape(B, F).double().cpu().numpy()
  o, shape = net.fp.offsets['fc1_w']
  W1 = net.fp.flat[o:o + int(np.prod(shape))].reshape(shape).double().cpu().numpy()
  W1 = W1 if W1.shape == (512, F) else W1.T                         # h = x W1^T: W1 (512, F)
  dx = dh @ W1                                                      # (R, F)
  st = state[np.arange(R) % B]
  dpre64 = np.where(emb > 0, dx * st, 0.0)
  dtl = (dx * emb).reshape(nq, B, F).sum(0)                        # sum over q
  dpre = ex.grads['dpre'].double().cpu().numpy()
  dstate = ex.torso.dacts['a3'].reshape(B, F).double().cpu().numpy()
  mask = state > 0
  ds64 = np.where(mask, dtl, 0.0)
  rel = lambda a, b: float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))
  lib = os.environ.get('DOPAMINE_AMD_LIB') or 'in-tree'
  print('%s B=%d nq=%d  d pre rel %.3e  d state rel %.3e (masked to state > 0)  |dstate|max %.3e '
        'sum_q |dx emb| max %.3e' % (lib, B, nq, rel(dpre, dpre64), rel(dstate[mask], ds64[mask]),
                                     np.abs(ds64).max(), np.abs(dx * emb).reshape(nq, B, F).sum(0).max()))


if __name__ == '__main__':
  main()
