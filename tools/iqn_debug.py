"""Isolate the IQN head backward GEMMs at R = nq * B: each weight gradient vs float64
products of the device's own operands (dh, x, dpre, cos, dq, h)."""
import json
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch


def rel(a, b):
  return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def main(B, nq, A=4):
  from dopamine_amd.agents.networks import ImplicitQuantileNetwork
  from dopamine_amd.iqn import HipIqnNet
  net = ImplicitQuantileNetwork(A, device='cuda', seed=3)
  rs = np.random.RandomState(B)
  x = torch.from_numpy(rs.randint(0, 256, (B, 84, 84, 4)).astype(np.float32) / np.float32(255)).cuda()
  taus = torch.from_numpy(rs.rand(nq * B).astype(np.float32)).cuda()
  ex = HipIqnNet(net, B, nq, keep=True)
  ex.forward(x, taus)
  dq = torch.from_numpy(rs.randn(nq * B, A).astype(np.float32) / (nq * B)).cuda()
  ex.backward(dq)
  torch.cuda.synchronize()
  g = net.fp.grad.cpu().numpy().astype(np.float64)
  off = net.fp.offsets
  def grad(name):
    o, s = off[name]
    return g[o:o + int(np.prod(s))].reshape(s)
  d = lambda t: t.detach().cpu().numpy().astype(np.float64)
  dh, X, dpre, cos, h = d(ex.grads['dh']), d(ex.acts['x']), d(ex.grads['dpre']), d(ex.acts['cos']), d(ex.acts['h'])
  dqn = d(dq)
  out = {'B': B, 'nq': nq}
  out['fc1_w'] = rel(grad('fc1_w'), dh.T @ X)
  out['fc1_b'] = rel(grad('fc1_b'), dh.sum(0))
  out['emb_w'] = rel(grad('emb_w'), dpre.T @ cos)
  out['emb_b'] = rel(grad('emb_b'), dpre.sum(0))
  out['fc2_w'] = rel(grad('fc2_w'), dqn.T @ h)
  out['fc2_b'] = rel(grad('fc2_b'), dqn.sum(0))
  W2 = d(net.fp['fc2_w'])
  out['dh'] = rel(dh, (dqn @ W2) * (h > 0))
  # where the fc1_w error sits: rows (j) / columns (f) of the worst elements
  err = np.abs(grad('fc1_w') - dh.T @ X)
  j, f = np.unravel_index(np.argmax(err), err.shape)
  out['fc1_w_worst'] = [int(j), int(f)]
  colerr = err.max(0)
  out['fc1_w_bad_cols'] = int((colerr > 1e-4 * np.abs(dh.T @ X).max()).sum())
  rowerr = err.max(1)
  out['fc1_w_bad_rows'] = int((rowerr > 1e-4 * np.abs(dh.T @ X).max()).sum())
  print(json.dumps(out), flush=True)


if __name__ == '__main__':
  for B, nq in ((16, 8), (64, 8), (16, 64), (64, 64)):
    main(B, nq)
