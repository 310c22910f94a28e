"""The conditioning measures the GPU parity tests hold the device to (oracle/nature_cnn.py
abs_grad / iqn_abs_grad and mask_flips), checked here on CPU fp32 arithmetic: torch's own
fp32 convolutions and GEMMs must pass them, and a corrupted ReLU decision must not."""
import numpy as np
import torch
import torch.nn.functional as F

from dopamine_amd.agents import networks
from oracle import nature_cnn as ONC

GRAD_TOL = 1e-5        # tests/test_gpu_northstar.py's bar on the Σ|terms| measure
MASK_TOL = 1e-5        # ... and on a flipped unit's |z| / Σ|w||a| + |b|


def _params32(flat, offsets):
  P = ONC.Params64(flat, offsets)
  P.t = {k: v.detach().float().requires_grad_(True) for k, v in P.t.items()}
  return P


def _fp32_run(net, x, gout, taus=None):
  """fp32 forward + backward on the oracle's graph: (device-layout ReLU outputs, flat grad)."""
  P = _params32(net.fp.flat.numpy(), net.fp.offsets)
  L, names, _, top = ONC._graph(P, torch.as_tensor(x), None,
                                None if taus is None else torch.as_tensor(taus))
  act, masks = {}, {}
  for l in L:
    xs = [l.exact[i].float() if p is None else act[p.name] for i, p in enumerate(l.inputs)]
    z = l.fn(xs, P[l.name + '_w'], P[l.name + '_b'])
    if l is top:
      z.backward(torch.as_tensor(gout, dtype=torch.float32))
      break
    a = F.relu(z)
    act[l.name] = a
    name, nhwc = names[l.name]
    masks[name] = (a.permute(0, 2, 3, 1) if nhwc else a).detach().numpy()
  return masks, P.flat_grad()


def _check(net, B, n_out, taus=None, seed=0):
  rng = np.random.RandomState(seed)
  x = (rng.randint(0, 256, (B, 84, 84, 4)).astype(np.float32) / np.float32(255)).astype(np.float64)
  rows = B if taus is None else taus.shape[0]
  gout = rng.randn(rows, n_out).astype(np.float32).astype(np.float64)
  masks, g32 = _fp32_run(net, x, gout, taus)
  flat, offsets = net.fp.flat.numpy(), net.fp.offsets
  xin = torch.as_tensor(x)
  t64 = None if taus is None else torch.as_tensor(taus)
  flips = ONC.mask_flips(ONC.Params64(flat, offsets), xin, masks, t64)
  for name, f in flips.items():
    assert f['worst'] <= MASK_TOL, (name, f)
  if taus is None:
    g, ga = ONC.abs_grad(ONC.Params64(flat, offsets), xin, masks, gout, np.abs(gout))
  else:
    g, ga = ONC.iqn_abs_grad(ONC.Params64(flat, offsets), xin, t64, masks, gout, np.abs(gout))
  for name, (o, shape) in offsets.items():
    n = int(np.prod(shape))
    s = slice(o, o + n)
    den = np.maximum(ga[s], 1e-3 * np.abs(g[s]).max())
    assert (np.abs(g32[s] - g[s]) / den).max() <= GRAD_TOL, name
  return masks, flips, flat, offsets, xin, t64


def test_fp32_arithmetic_passes_the_measures_and_a_corrupted_decision_fails():
  torch.manual_seed(0)
  net = networks.RainbowNetwork(9, device='cpu', seed=3)
  masks, flips, flat, offsets, xin, _ = _check(net, 4, 9 * 51)
  assert sum(f['units'] for f in flips.values()) == 4 * (21 * 21 * 32 + 11 * 11 * 64 * 2 + 512)
  # one clearly active conv2 unit switched off: its |z| is a large fraction of its magnitude
  bad = {k: v.copy() for k, v in masks.items()}
  i = np.unravel_index(np.argmax(bad['a2']), bad['a2'].shape)
  bad['a2'][i] = 0.0
  f = ONC.mask_flips(ONC.Params64(flat, offsets), xin, bad)['a2']
  assert f['flips'] >= 1 and f['worst'] > 1e-2, f


def test_iqn_fp32_arithmetic_passes_the_measures():
  net = networks.ImplicitQuantileNetwork(4, device='cpu', seed=5)
  B, nq = 2, 4
  taus = np.random.RandomState(1).rand(nq * B).astype(np.float32).astype(np.float64)
  _, flips, *_ = _check(net, B, 4, taus=taus, seed=2)
  assert set(flips) == {'a1', 'a2', 'a3', 'emb', 'h'}
