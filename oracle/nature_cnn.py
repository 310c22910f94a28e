"""float64 Nature-CNN on the flat parameter layout -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module.  A torch-CPU float64 restatement of the
reference's networks (atari_lib.py:85-105 NatureDQNNetwork, :108-144
RainbowNetwork, :147-199 ImplicitQuantileNetwork) with TF's SAME padding and
TF's (h, w, c) flatten order, reading the same flat fp32 parameter buffer the
device kernels use (``dopamine_amd.agents.networks.FlatParams`` offsets: conv
filters stored (out, kh, kw, in), FC (out, in)).  Gradients come from torch
autograd in float64; they are returned in the same flat layout.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


class Params64(object):
  """float64 leaf tensors (torch layout) of a flat fp32/fp64 buffer."""

  def __init__(self, flat, offsets):
    flat = torch.as_tensor(np.asarray(flat), dtype=torch.float64)
    self.offsets = offsets
    self.numel = flat.numel()
    self.t = {}
    for name, (o, shape) in offsets.items():
      n = int(np.prod(shape))
      v = flat[o:o + n]
      if len(shape) == 4:
        out_c, in_c, kh, kw = shape
        v = v.view(out_c, kh, kw, in_c).permute(0, 3, 1, 2)
      else:
        v = v.view(shape)
      self.t[name] = v.clone().requires_grad_(True)

  def __getitem__(self, name):
    return self.t[name]

  def flat_grad(self):
    """The autograd gradients in the flat (out, kh, kw, in) / (out, in) layout."""
    g = torch.zeros(self.numel, dtype=torch.float64)
    for name, (o, shape) in self.offsets.items():
      x = self.t[name].grad
      if x is None:
        continue
      if len(shape) == 4:
        x = x.permute(0, 2, 3, 1)
      g[o:o + x.numel()] = x.reshape(-1)
    return g.numpy()


def _relu(z, masks, name, nhwc=False):
  """ReLU, or -- given the device's activations in ``masks`` -- z * (device output > 0):
  the float64 arithmetic on the device's own ReLU decisions.  A pre-activation within
  fp32 rounding of 0 can take the other branch in float64 and move a gradient that sums
  thousands of terms with cancellation by a whole term (mask-pinned checks isolate the
  arithmetic from those flips)."""
  if masks is None or name not in masks:
    return F.relu(z)
  m = torch.as_tensor(np.asarray(masks[name]) > 0, dtype=torch.float64)
  if nhwc:                                   # device NHWC -> torch NCHW
    m = m.reshape(z.shape[0], z.shape[2], z.shape[3], z.shape[1]).permute(0, 3, 1, 2)
  return z * m.reshape(z.shape)


def torso(P, x_nhwc, masks=None):
  """x (B, 84, 84, stack) float64, already /255 -> (B, 7744) in TF's flatten order."""
  x = x_nhwc.permute(0, 3, 1, 2)
  x = _relu(F.conv2d(F.pad(x, (2, 2, 2, 2)), P['conv1_w'], P['conv1_b'], stride=4), masks, 'a1',
            True)                                                                      # SAME 84->21
  x = _relu(F.conv2d(F.pad(x, (1, 2, 1, 2)), P['conv2_w'], P['conv2_b'], stride=2), masks, 'a2',
            True)                                                                      # SAME 21->11
  x = _relu(F.conv2d(F.pad(x, (1, 1, 1, 1)), P['conv3_w'], P['conv3_b'], stride=1), masks, 'a3',
            True)                                                                      # SAME 11->11
  return x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)


def forward(P, x_nhwc, masks=None):
  """NatureDQN q-values (B, A) or Rainbow logits (B, A*N): fc1 + ReLU, fc2.  masks: the
  device's activations (a1, a2, a3, h) to pin the ReLU decisions (see _relu)."""
  h = _relu(F.linear(torso(P, x_nhwc, masks), P['fc1_w'], P['fc1_b']), masks, 'h')
  return F.linear(h, P['fc2_w'], P['fc2_b'])


def iqn_forward(P, x_nhwc, taus, masks=None):
  """ImplicitQuantileNetwork (atari_lib.py:147-199): taus (N*B,) rows ordered
  q*B + b; returns quantile values (N*B, A).  masks: the device's activations
  (a1, a2, a3, emb, h) to pin the ReLU decisions (see _relu)."""
  state = torso(P, x_nhwc, masks)
  B = state.shape[0]
  nq = taus.shape[0] // B
  E = P['emb_w'].shape[1]
  tiled = state.repeat(nq, 1)
  # the reference forms the cosine's argument in float32 -- (float(i) * float32(pi)) * tau,
  # atari_lib.py:176-178 -- an argument up to 64 pi carries ~1e-5 of rounding that is part
  # of the reference's result; the cosine itself is taken in float64
  i_pi = (torch.arange(1, E + 1, dtype=torch.float32) * torch.tensor(math.pi, dtype=torch.float32))
  arg = (taus.to(torch.float32).reshape(-1, 1) * i_pi).double()
  emb = torch.cos(arg)
  emb = _relu(F.linear(emb, P['emb_w'], P['emb_b']), masks, 'emb')
  h = _relu(F.linear(tiled * emb, P['fc1_w'], P['fc1_b']), masks, 'h')
  return F.linear(h, P['fc2_w'], P['fc2_b'])


def iqn_masks(ex):
  """The ReLU outputs of a HipIqnNet's last forward (host copies) for iqn_forward."""
  t = ex.torso.acts
  return dict(a1=t['a1'].cpu().numpy(), a2=t['a2'].cpu().numpy(), a3=t['a3'].cpu().numpy(),
              emb=ex.acts['emb'].cpu().numpy(), h=ex.acts['h'].cpu().numpy())


def to_input(x_float32_nhwc):
  """The network input the reference computes in fp32 (uint8 / 255.), as float64."""
  return torch.as_tensor(np.asarray(x_float32_nhwc), dtype=torch.float32).double()


# ----------------------------------------------------------- Σ|terms| of every gradient
# The conditioning of a gradient element: the float64 sum of the absolute values of the
# terms its final reduction adds -- |dz| |x| over the batch (and positions) for a weight,
# |dz| for a bias, with dz the float64 gradient of the layer's pre-activation.  A bias
# gradient that sums 441 B positions of both signs can be far below its terms, and its fp32
# sum is then accurate to u times the terms, not to u times itself.  Tests compare
# |g_device - g_float64| with this sum element by element.
_CONVS = (('conv1', (2, 2, 2, 2), 4, 'a1'), ('conv2', (1, 2, 1, 2), 2, 'a2'),
          ('conv3', (1, 1, 1, 1), 1, 'a3'))


def _layers(P, x_nhwc, masks, rec):
  """The Nature-CNN torso as forward()/torso(), recording each layer's (name, kind, input,
  pre-activation) in rec (the pre-activations retain their gradients)."""
  x = x_nhwc.permute(0, 3, 1, 2)
  for name, pad, st, act in _CONVS:
    xi = F.pad(x, pad)
    z = F.conv2d(xi, P[name + '_w'], P[name + '_b'], stride=st)
    z.retain_grad()
    rec.append((name, ('conv', st), xi, z))
    x = _relu(z, masks, act, True)
  return x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)


def _linear(P, name, x, rec):
  z = F.linear(x, P[name + '_w'], P[name + '_b'])
  z.retain_grad()
  rec.append((name, ('fc',), x, z))
  return z


def _abs_sums(P, rec):
  """Σ|terms| of each recorded layer's weight and bias gradients, in the flat layout."""
  g = torch.zeros(P.numel, dtype=torch.float64)
  for name, kind, xi, z in rec:
    dz = z.grad.detach().abs()
    ax = xi.detach().abs()
    w = P[name + '_w'].detach().clone().requires_grad_(True)
    t = F.conv2d(ax, w, stride=kind[1]) if kind[0] == 'conv' else F.linear(ax, w)
    t.backward(dz)
    gw = w.grad.permute(0, 2, 3, 1) if kind[0] == 'conv' else w.grad
    gb = dz.sum(dim=(0, 2, 3)) if kind[0] == 'conv' else dz.sum(0)
    for suf, v in (('_w', gw), ('_b', gb)):
      o, shape = P.offsets[name + suf]
      g[o:o + v.numel()] = v.reshape(-1)
  return g.numpy()


def abs_grad(P, x_nhwc, masks, gout):
  """(flat float64 gradient, flat Σ|terms| of it) for forward(P, x, masks) and the loss
  gradient gout (B, n_out); P: fresh Params64 leaves.  masks: the device's activations (the
  ReLU decisions are the device's)."""
  rec = []
  h = _relu(_linear(P, 'fc1', _layers(P, x_nhwc, masks, rec), rec), masks, 'h')
  out = _linear(P, 'fc2', h, rec)
  out.backward(torch.as_tensor(np.asarray(gout), dtype=torch.float64))
  return P.flat_grad(), _abs_sums(P, rec)


def iqn_abs_grad(P, x_nhwc, taus, masks, gout):
  """abs_grad for iqn_forward (rows q B + b; masks a1, a2, a3, emb, h); the Hadamard
  product's own sum (over the N tiled rows of each state) is the fc1 gradient's reduction."""
  rec = []
  state = _layers(P, x_nhwc, masks, rec)
  B = state.shape[0]
  nq = taus.shape[0] // B
  E = P['emb_w'].shape[1]
  tiled = state.repeat(nq, 1)
  i_pi = (torch.arange(1, E + 1, dtype=torch.float32) * torch.tensor(math.pi, dtype=torch.float32))
  emb_in = torch.cos((taus.to(torch.float32).reshape(-1, 1) * i_pi).double())
  emb = _relu(_linear(P, 'emb', emb_in, rec), masks, 'emb')
  h = _relu(_linear(P, 'fc1', tiled * emb, rec), masks, 'h')
  out = _linear(P, 'fc2', h, rec)
  out.backward(torch.as_tensor(np.asarray(gout), dtype=torch.float64))
  return P.flat_grad(), _abs_sums(P, rec)
