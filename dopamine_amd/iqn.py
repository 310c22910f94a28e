"""HIP executor of ImplicitQuantileNetwork (atari_lib.py:147-199) over the network's
flat parameter buffer: the Nature-CNN torso on nature_cnn.hip (dq_cnn_forward_torso /
dq_cnn_backward_torso) and the quantile head on iqn.hip (cosine embedding, Hadamard
product, FC 7744 -> 512 -> A on the fp32 matrix cores), plus the quantile samples tau
from a counter-based device generator, so a captured HIP graph draws exactly what the
same calls draw eagerly.
"""
import ctypes

import torch

from dopamine_amd import _lib
from dopamine_amd.cnn import HipNatureCNN

_HEAD = ('emb_w', 'emb_b', 'fc1_w', 'fc1_b', 'fc2_w', 'fc2_b')
F, H = 7744, 512


def _head_struct(fp, buf, num_actions, embed_dim):
  s = _lib.IqnHead(embed_dim=embed_dim, num_actions=num_actions)
  for n in _HEAD:
    setattr(s, n, buf.data_ptr() + 4 * fp.offsets[n][0])
  return s


def _stream(device):
  return _lib.stream_of(device)


class TauSampler(object):
  """tau ~ U[0, 1) float32 (tf.random_uniform, atari_lib.py:171-172) from a
  counter-based generator: draw k of a sampler is a fixed function of (seed, k), and
  the counter lives on the device, so graph replays and eager calls agree."""

  def __init__(self, seed, device):
    self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    self.counter = torch.zeros(2, dtype=torch.int64, device=device)

  def draw(self, out):
    _lib.call('dq_uniform_draw', _lib.ptr(self.counter), ctypes.c_uint64(self.seed), out.numel(),
              _lib.ptr(out), _stream(out.device))
    return out

  def draw_cos(self, ex):
    """draw(ex.taus) fused with their cosine embedding into ex.acts['cos']
    (dq_iqn_tau_cos: the same draws, one launch); then ex.forward(x, cos_ready=True)."""
    _lib.call('dq_iqn_tau_cos', _lib.ptr(self.counter), ctypes.c_uint64(self.seed), ex.R, ex.E,
              _lib.ptr(ex.taus), _lib.ptr(ex.acts['cos']), _stream(ex.taus.device))
    return ex.taus


class HipIqnNet(object):
  """One (batch, nq) configuration of an ImplicitQuantileNetwork's parameters on the
  HIP kernels.  ``keep``: keep what the backward needs (the online network).
  ``store_x``: the online net stores x = tiled state * emb and streams it (the stored-x
  schedule, bitwise the default, which forms x in the FC1 / dW1 operand loaders)."""

  def __init__(self, net, batch_size, nq, keep=True, store_x=False):
    fp = net.fp
    self.net, self.B, self.nq, self.keep = net, int(batch_size), int(nq), bool(keep)
    self.A, self.E = int(net.A), int(net.E)
    self.R = self.B * self.nq
    dev = fp.flat.device
    self.device = dev
    mk = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)
    self.torso = HipNatureCNN(net, self.B)
    R = self.R
    # the online net keeps emb and never stores x = tiled state * emb: its FC1 forward and
    # dW1 form x from emb and the state in their operand loaders
    store_x = not keep or store_x
    self.acts = dict(cos=mk(R, self.E), emb=mk(R, F) if keep else None,
                     x=mk(R, F) if store_x else None, h=mk(R, H), q=mk(R, self.A))
    self.taus = mk(R)
    self._a = _lib.IqnActs(**{k: (v.data_ptr() if v is not None else None)
                              for k, v in self.acts.items()})
    self._p = _head_struct(fp, fp.flat, self.A, self.E)
    if keep:
      self.grads = dict(dh=mk(R, H), dpre=mk(R, F), dtl=mk(R, F))
      self._d = _lib.IqnGrads(**{k: v.data_ptr() for k, v in self.grads.items()})
      self._g = _head_struct(fp, fp.grad, self.A, self.E)
    n = int(_lib.lib.dq_iqn_workspace_floats(self.B, self.nq, self.A, self.E))
    self.ws = mk(max(n, 1) + 64)

  def forward(self, x, taus=None, cos_ready=False):
    """x: (B, 84, 84, 4) NHWC float32 (or its channels_last NCHW view); taus (R,) or
    None (use self.taus as filled by the caller); cos_ready: acts['cos'] already holds
    their embedding (TauSampler.draw_cos).  Returns (q (R, A), taus)."""
    x = self.torso._nhwc(x)
    self.torso._x = x
    t = self.torso
    _lib.check(_lib.lib.dq_cnn_forward_torso(ctypes.byref(t._p), self.B, x.data_ptr(),
                                             ctypes.byref(t._a), t.ws.data_ptr(),
                                             _stream(self.device)), 'dq_cnn_forward_torso')
    if taus is not None and taus.data_ptr() != self.taus.data_ptr():
      self.taus.copy_(taus.reshape(-1))
    _lib.check(_lib.lib.dq_iqn_head_forward(ctypes.byref(self._p), self.B, self.nq,
                                            t.acts['a3'].data_ptr(),
                                            None if cos_ready else self.taus.data_ptr(),
                                            ctypes.byref(self._a), self.ws.data_ptr(),
                                            _stream(self.device)), 'dq_iqn_head_forward')
    return self.acts['q'], self.taus

  def backward(self, dq, adam=None, slot=0, store_grads=True):
    """dq: (R, A) = d loss / d q.  Writes every parameter gradient into net.fp.grad.
    adam: an ops.TF1Adam / TF1RMSProp over net.fp.flat -- its whole step is applied in the
    torso's backward launches (dq_cnn_backward_torso_opt: the head's range as float4 riders,
    conv2 / conv1 in their split-K sums' epilogues), bitwise the separate optimizer launch;
    slot: Adam's beta-power slot; store_grads False: the fused epilogues skip the gradient
    stores they consume (no_grad_store)."""
    assert self.keep and dq.shape == (self.R, self.A) and dq.is_contiguous()
    t = self.torso
    _lib.check(_lib.lib.dq_iqn_head_backward(
        ctypes.byref(self._p), ctypes.byref(self._g), self.B, self.nq, t.acts['a3'].data_ptr(),
        ctypes.byref(self._a), dq.data_ptr(), ctypes.byref(self._d), t.dacts['a3'].data_ptr(),
        self.ws.data_ptr(), _stream(self.device)), 'dq_iqn_head_backward')
    if adam is None:
      _lib.check(_lib.lib.dq_cnn_backward_torso(ctypes.byref(t._p), ctypes.byref(t._g), self.B,
                                                t._x.data_ptr(), ctypes.byref(t._a),
                                                ctypes.byref(t._d), t.ws.data_ptr(),
                                                _stream(self.device)), 'dq_cnn_backward_torso')
      return self.net.fp.grad
    fp = self.net.fp
    t.store_grads = bool(store_grads)
    args = t._adam_args(adam, slot)
    head0 = fp.flat.data_ptr() + 4 * fp.offsets['emb_w'][0]
    head1 = fp.flat.data_ptr() + 4 * fp.flat.numel()
    _lib.check(_lib.lib.dq_cnn_backward_torso_opt(
        ctypes.byref(t._p), ctypes.byref(t._g), self.B, t._x.data_ptr(), ctypes.byref(t._a),
        ctypes.byref(t._d), t.ws.data_ptr(), ctypes.byref(args), ctypes.c_void_p(head0),
        ctypes.c_void_p(head1), _stream(self.device)), 'dq_cnn_backward_torso_opt')
    return self.net.fp.grad
