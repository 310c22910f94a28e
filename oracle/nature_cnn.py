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
# terms its final reduction adds, each operand taken at its own one-level magnitude -- a
# layer input as Σ|w| |a| + |b| of the layer that produced it (masked), a pre-activation
# gradient as Σ|w| |dz| of the layer that consumed it (masked), the loss gradient as the sum
# of its terms' magnitudes (oracle/learner.py grad_abs), which the dense head (fc2, fc1)
# carries down: the loss gradient's cancellation (C51's softmax - projection, Huber's q -
# target, IQN's sum over N' target quantiles) reaches fc1, the embedding and conv3's inputs
# undiluted, while below it each convolution's own long reduction dominates.  fp32 arithmetic errs on every operand by a small multiple of u times
# that magnitude, so an element's error is bounded by a small multiple of u times this sum
# whatever cancellation its signed sum (or either operand's) has: a bias gradient summing
# 441 B positions of both signs, a weight reading an activation that is itself a near-zero
# difference.  Tests compare |g_device - g_float64| with it element by element.
class _Layer(object):
  def __init__(self, name, fn, inputs, exact=None, exact_abs=None):
    self.name, self.fn, self.inputs = name, fn, inputs     # inputs: producer layers / tensors
    self.exact = exact or {}                                # input index -> given tensor
    self.exact_abs = exact_abs or {}                        # ... its magnitude, if not |x|

  def in_abs(self, i):
    return self.exact_abs[i] if i in self.exact_abs else self.exact[i].abs()


def _conv(pad, stride):
  return lambda xs, w, b: F.conv2d(F.pad(xs[0], pad), w, b, stride=stride)


def _flat_nhwc(a):
  return a.permute(0, 2, 3, 1).reshape(a.shape[0], -1)


def _graph(P, x_nhwc, masks, taus=None):
  """The layers of forward() / iqn_forward() as a DAG: (layers, their ReLU masks in their
  output layouts (None: no ReLU), the output layer)."""
  x = x_nhwc.permute(0, 3, 1, 2)
  mask = lambda name, nhwc, shape: _relu(torch.ones(shape, dtype=torch.float64), masks, name, nhwc)
  L = []
  c1 = _Layer('conv1', _conv((2, 2, 2, 2), 4), [None], {0: x})
  c2 = _Layer('conv2', _conv((1, 2, 1, 2), 2), [c1])
  c3 = _Layer('conv3', _conv((1, 1, 1, 1), 1), [c2])
  L += [c1, c2, c3]
  if taus is None:
    f1 = _Layer('fc1', lambda xs, w, b: F.linear(_flat_nhwc(xs[0]), w, b), [c3])
  else:
    B = x.shape[0]
    nq = taus.shape[0] // B
    E = P['emb_w'].shape[1]
    i_pi = (torch.arange(1, E + 1, dtype=torch.float32) * torch.tensor(math.pi, dtype=torch.float32))
    cos = torch.cos((taus.to(torch.float32).reshape(-1, 1) * i_pi).double())
    # the device takes the cosine in fp32 (one rounding of |cos| <= 1): its magnitude as an
    # operand is |cos| + 2^-23, not |cos| (near a zero of the cosine the rounding dominates)
    em = _Layer('emb', lambda xs, w, b: F.linear(xs[0], w, b), [None], {0: cos},
                {0: cos.abs() + 2.0 ** -23})
    L.append(em)
    f1 = _Layer('fc1', lambda xs, w, b: F.linear(_flat_nhwc(xs[0]).repeat(nq, 1) * xs[1], w, b),
                [c3, em])
  f2 = _Layer('fc2', lambda xs, w, b: F.linear(xs[0], w, b), [f1])
  L += [f1, f2]
  names = {'conv1': ('a1', True), 'conv2': ('a2', True), 'conv3': ('a3', True), 'emb': ('emb', False),
           'fc1': ('h', False)}
  return L, names, mask, f2


def _abs_terms(P, x_nhwc, masks, gout, gout_abs, taus=None, full=False):
  L, names, mask, top = _graph(P, x_nhwc, masks, taus)
  act, z, m = {}, {}, {}
  for l in L:                                              # the float64 forward
    xs = [l.exact[i] if p is None else act[p.name] for i, p in enumerate(l.inputs)]
    z[l.name] = l.fn(xs, P[l.name + '_w'], P[l.name + '_b'])
    z[l.name].retain_grad()
    if l is not top:
      m[l.name] = mask(names[l.name][0], names[l.name][1], z[l.name].shape)
      act[l.name] = z[l.name] * m[l.name]
  z[top.name].backward(torch.as_tensor(np.asarray(gout), dtype=torch.float64))
  grad = P.flat_grad()
  aw = {l.name: P[l.name + '_w'].detach().abs() for l in L}
  ab = {l.name: P[l.name + '_b'].detach().abs() for l in L}
  # one-level forward magnitudes of every activation (from its true inputs)
  a_abs = {}
  for l in L:
    if l is top:
      continue
    xs = [(l.in_abs(i) if p is None else
           (a_abs[p.name] if full else act[p.name].detach().abs())) for i, p in enumerate(l.inputs)]
    with torch.no_grad():
      a_abs[l.name] = l.fn(xs, aw[l.name], ab[l.name]) * m[l.name]
  # one-level backward magnitudes of every pre-activation gradient (from its true upstream)
  dz_abs = {top.name: torch.as_tensor(np.asarray(gout_abs), dtype=torch.float64)}
  for l in reversed(L):
    for i, p in enumerate(l.inputs):
      if p is None:
        continue
      # the other operands of a product (IQN's fc1: state ⊙ emb) at their one-level forward
      # magnitudes: an fp32 operand errs by u times its magnitude, not its (maybe cancelled)
      # value, and that error scales the input gradient (xs[i]'s own value does not enter)
      xs = [((l.exact[j].abs() if q is None else act[q.name].abs()) if j == i else
             (l.in_abs(j) if q is None else a_abs[q.name])).detach().clone().requires_grad_(j == i)
            for j, q in enumerate(l.inputs)]
      # the dense head (fc2, fc1) passes on magnitudes carried from the loss's own terms; a
      # convolution passes on one level from its true gradient
      carried = full or l.name in ('fc1', 'fc2')
      l.fn(xs, aw[l.name], None).backward(
          dz_abs[l.name] if carried else z[l.name].grad.detach().abs())
      d = xs[i].grad * m[p.name]
      dz_abs[p.name] = dz_abs[p.name] + d if p.name in dz_abs else d
  # Σ|terms| of each weight / bias gradient: the layer's input magnitudes against its
  # pre-activation gradient's
  out = np.zeros(P.numel)
  for l in L:
    xs = [(l.in_abs(i) if p is None else a_abs[p.name]) for i, p in enumerate(l.inputs)]
    w = torch.zeros_like(aw[l.name], requires_grad=True)
    l.fn(xs, w, None).backward(dz_abs[l.name])
    gw = w.grad.permute(0, 2, 3, 1) if w.grad.dim() == 4 else w.grad
    d = dz_abs[l.name]
    gb = d.sum(dim=(0, 2, 3)) if d.dim() == 4 else d.sum(0)
    for suf, v in (('_w', gw), ('_b', gb)):
      o, _ = P.offsets[l.name + suf]
      out[o:o + v.numel()] = v.reshape(-1).numpy()
  return grad, out


def mask_flips(P, x_nhwc, masks, taus=None):
  """Where the device's ReLU decisions differ from float64's, and by how much they may.
  Layer by layer on the device's decisions upstream (so each layer is judged on its own
  inputs), the float64 pre-activation z of every ReLU unit against its one-level magnitude
  Σ|w||a| + |b|: fp32 arithmetic errs on z by a small multiple of u times that magnitude,
  so a unit whose decision is NOT within rounding of 0 must take float64's branch.  Returns
  {activation name: {'flips', 'units', 'worst'}}, worst = max |z| / magnitude over the
  flipped units (0 if none) -- a mask or tile bug flips units of O(1) ratio."""
  L, names, mask, top = _graph(P, x_nhwc, masks, taus)
  act, out = {}, {}
  with torch.no_grad():
    for l in L:
      if l is top:
        continue
      w, b = P[l.name + '_w'].detach(), P[l.name + '_b'].detach()
      xs = [l.exact[i] if p is None else act[p.name] for i, p in enumerate(l.inputs)]
      xa = [l.in_abs(i) if p is None else act[p.name].abs() for i, p in enumerate(l.inputs)]
      z = l.fn(xs, w, b)
      mag = l.fn(xa, w.abs(), b.abs())
      m = mask(names[l.name][0], names[l.name][1], z.shape)
      flip = (z > 0) != (m > 0)
      ratio = z.abs() / torch.clamp(mag, min=1e-300)
      out[names[l.name][0]] = dict(flips=int(flip.sum()), units=int(z.numel()),
                                   worst=float(ratio[flip].max()) if bool(flip.any()) else 0.0)
      act[l.name] = z * m
  return out


def abs_grad(P, x_nhwc, masks, gout, gout_abs):
  """(flat float64 gradient, flat Σ|terms| of each element) for forward(P, x, masks) with
  the loss gradient gout (B, n_out) and its magnitudes gout_abs; P: fresh Params64 leaves;
  masks: the device's activations (its ReLU decisions)."""
  return _abs_terms(P, x_nhwc, masks, gout, gout_abs)


def iqn_abs_grad(P, x_nhwc, taus, masks, gout, gout_abs):
  """abs_grad for iqn_forward (rows q B + b; masks a1, a2, a3, emb, h)."""
  return _abs_terms(P, x_nhwc, masks, gout, gout_abs, taus)
