"""torch-tensor wrappers over the learner kernels of the C ABI.

Every function launches on torch's current stream (so it is captured by
``torch.cuda.graph``) and never synchronises.
"""
import ctypes

import torch

from dopamine_amd import _lib

p = _lib.ptr


def _stream(t):
  return _lib.stream_of(t.device)


def _c(t, dtype):
  assert t.is_cuda and t.dtype == dtype and t.is_contiguous(), (t.dtype, t.device, dtype)
  return t


def c51_loss(online_logits, target_logits, actions, rewards, terminals, support, cumulative_gamma,
             probs=None, out=None):
  """rainbow_agent.py:200-305.  Returns dict(grad, loss, priorities, mean_loss)."""
  B, A, N = online_logits.shape
  f32 = torch.float32
  if out is None:
    dev = online_logits.device
    out = dict(grad=torch.empty_like(online_logits), loss=torch.empty(B, dtype=f32, device=dev),
               priorities=torch.empty(B, dtype=f32, device=dev),
               mean_loss=torch.empty(1, dtype=f32, device=dev))
  _lib.call('dq_c51_loss', p(_c(online_logits, f32)), p(_c(target_logits, f32)),
            p(_c(actions, torch.int32)), p(_c(rewards, f32)), p(_c(terminals, torch.uint8)),
            p(probs if probs is None else _c(probs, f32)), p(_c(support, f32)), B, A, N,
            float(cumulative_gamma), p(out['grad']), p(out['loss']), p(out['priorities']),
            p(out['mean_loss']), _stream(online_logits))
  return out


def c51_loss_fused(online, target, actions, rewards, terminals, support, cumulative_gamma,
                   probs=None, out=None, logits_out=False):
  """c51_loss on the HIP CNN's fc2 k-band partials (cnn.forward_fused) of the
  online and target executors (``cnn.HipNatureCNN``); also writes the fc2 input
  gradient into ``online.dacts['h']``, so ``online.backward(..., groups=(1, 7))``
  can skip launch 0.  logits_out: also store both nets' logits in their
  ``acts['out']``.  Returns dict(grad, loss, priorities)."""
  from dopamine_amd import cnn
  B, NO = online.B, online.n_out
  N = int(support.numel())
  A = NO // N
  f32 = torch.float32
  dev = support.device
  if out is None:
    out = dict(grad=torch.empty((B, A, N), dtype=f32, device=dev),
               loss=torch.empty(B, dtype=f32, device=dev),
               priorities=torch.empty(B, dtype=f32, device=dev))
  po, pt = cnn.fc2_parts(online), cnn.fc2_parts(target)
  _lib.call('dq_c51_loss_fused', p(po), online._p.fc2_b, p(pt), target._p.fc2_b, po.shape[0],
            p(_c(actions, torch.int32)), p(_c(rewards, f32)), p(_c(terminals, torch.uint8)),
            p(probs if probs is None else _c(probs, f32)), p(_c(support, f32)), B, A, N,
            float(cumulative_gamma), p(out['grad']), p(out['loss']), p(out['priorities']),
            online._p.fc2_w, p(online.acts['h']), p(online.dacts['h']), 512,
            p(online.acts['out']) if logits_out else None,
            p(target.acts['out']) if logits_out else None, _stream(support))
  return out


def c51_loss_online(online, target_m, actions, probs=None, out=None, logits_out=False):
  """The online half of c51_loss_fused (dq_c51_loss_online): the target distribution
  ``target_m`` (B, N) comes from cnn.forward_fused_c51.  Bitwise c51_loss_fused's loss,
  gradient, priorities and d h.  Returns dict(grad, loss, priorities)."""
  from dopamine_amd import cnn
  B, NO = online.B, online.n_out
  N = int(target_m.shape[-1])
  A = NO // N
  f32 = torch.float32
  dev = target_m.device
  if out is None:
    out = dict(grad=torch.empty((B, A, N), dtype=f32, device=dev),
               loss=torch.empty(B, dtype=f32, device=dev),
               priorities=torch.empty(B, dtype=f32, device=dev))
  po = cnn.fc2_parts(online)
  _lib.call('dq_c51_loss_online', p(po), online._p.fc2_b, po.shape[0], p(target_m),
            p(_c(actions, torch.int32)), p(probs if probs is None else _c(probs, f32)), B, A, N,
            p(out['grad']), p(out['loss']), p(out['priorities']), online._p.fc2_w,
            p(online.acts['h']), p(online.dacts['h']), 512,
            p(online.acts['out']) if logits_out else None, _stream(target_m))
  return out


def dqn_huber_loss(online_q, target_q, actions, rewards, terminals, cumulative_gamma, out=None):
  """dqn_agent.py:283-322."""
  B, A = online_q.shape
  f32 = torch.float32
  if out is None:
    dev = online_q.device
    out = dict(grad=torch.empty_like(online_q), loss=torch.empty(B, dtype=f32, device=dev),
               mean_loss=torch.empty(1, dtype=f32, device=dev))
  _lib.call('dq_dqn_huber_loss', p(_c(online_q, f32)), p(_c(target_q, f32)),
            p(_c(actions, torch.int32)), p(_c(rewards, f32)), p(_c(terminals, torch.uint8)), B, A,
            float(cumulative_gamma), p(out['grad']), p(out['loss']), p(out['mean_loss']),
            _stream(online_q))
  return out


def dqn_huber_loss_fused(online, target, actions, rewards, terminals, cumulative_gamma, out=None,
                         q_out=False):
  """dqn_huber_loss on the HIP CNN's fc2 k-band partials (cnn.forward_fused) of the
  online and target executors: Q and Q' are summed inside the loss kernel, which also
  writes fc2's input gradient into ``online.dacts['h']`` (bitwise the backward's launch
  0), so ``online.backward(..., groups=(1, 7))`` starts at launch 1.  q_out: also store
  both nets' outputs in their ``acts['out']``.  Returns dict(grad, loss)."""
  from dopamine_amd import cnn
  B, A = online.B, online.n_out
  f32 = torch.float32
  dev = rewards.device
  if out is None:
    out = dict(grad=torch.empty((B, A), dtype=f32, device=dev),
               loss=torch.empty(B, dtype=f32, device=dev))
  po, pt = cnn.fc2_parts(online), cnn.fc2_parts(target)
  _lib.call('dq_dqn_huber_loss_fused', p(po), online._p.fc2_b, p(pt), target._p.fc2_b,
            po.shape[0], p(_c(actions, torch.int32)), p(_c(rewards, f32)),
            p(_c(terminals, torch.uint8)), B, A, float(cumulative_gamma), p(out['grad']),
            p(out['loss']), online._p.fc2_w, p(online.acts['h']), p(online.dacts['h']), 512,
            p(online.acts['out']) if q_out else None, p(target.acts['out']) if q_out else None,
            _stream(rewards))
  return out


def iqn_loss(online_qv, target_qv, target_qv_action, taus, actions, rewards, terminals,
             cumulative_gamma, kappa=1.0, out=None):
  """implicit_quantile_agent.py:190-321 (rows ordered q*B + b)."""
  B = rewards.shape[0]
  A = online_qv.shape[1]
  N, Np, K = online_qv.shape[0] // B, target_qv.shape[0] // B, target_qv_action.shape[0] // B
  f32 = torch.float32
  if out is None:
    dev = online_qv.device
    out = dict(grad=torch.empty_like(online_qv), loss=torch.empty(B, dtype=f32, device=dev),
               mean_loss=torch.empty(1, dtype=f32, device=dev))
  _lib.call('dq_iqn_loss', p(_c(online_qv, f32)), p(_c(target_qv, f32)),
            p(_c(target_qv_action, f32)), p(_c(taus.reshape(-1), f32)), p(_c(actions, torch.int32)),
            p(_c(rewards, f32)), p(_c(terminals, torch.uint8)), B, A, N, Np, K,
            float(cumulative_gamma), float(kappa), p(out['grad']), p(out['loss']),
            p(out['mean_loss']), _stream(online_qv))
  return out


class TF1Adam(object):
  """tf.train.AdamOptimizer over one flat fp32 buffer (ApplyAdam semantics)."""

  supports_multi = True

  def __init__(self, params, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8,
               segments=None):
    self.params = params
    self.lr, self.b1, self.b2, self.eps = float(learning_rate), float(beta1), float(beta2), float(epsilon)
    self.m = torch.zeros_like(params)
    self.v = torch.zeros_like(params)
    # {beta1_power, beta2_power} double-buffered: step t reads slot t % 2
    self.state = torch.tensor([beta1, beta2, 0.0, 0.0], dtype=torch.float32, device=params.device)
    self.segments = segments
    self.t = 0

  def _slot(self, slot):
    if slot is None:
      slot = self.t % 2
      self.t += 1
    return int(slot)

  def step(self, grad, slot=None):
    """Update from ONE flat gradient buffer (same layout as ``params``)."""
    _lib.call('dq_adam_tf1', p(self.params), p(_c(grad, torch.float32)), p(self.m), p(self.v),
              p(self.state), self._slot(slot), self.params.numel(), self.lr, self.b1, self.b2,
              self.eps, _stream(self.params))

  def step_part(self, grad, lo, hi, slot, bump):
    """Adam on the flat range [lo, hi) only (grad: the whole flat gradient).  One
    step may be split into parts; exactly one of them passes bump=True."""
    assert 0 <= lo <= hi <= self.params.numel() and lo % 4 == 0
    f = lambda t: t.data_ptr() + 4 * lo
    _lib.call('dq_adam_tf1_part', f(self.params), f(_c(grad, torch.float32)), f(self.m), f(self.v),
              p(self.state), int(slot), hi - lo, self.lr, self.b1, self.b2, self.eps, int(bool(bump)),
              _stream(self.params))

  def step_multi(self, grads, slot=None):
    """Update from per-parameter gradient tensors (memory order = the parameter
    slices ``segments`` of the flat buffer) in one launch."""
    assert self.segments is not None and len(grads) == len(self.segments)
    tl = _lib.TensorList()
    tl.count = len(grads)
    base_p, base_m, base_v = self.params.data_ptr(), self.m.data_ptr(), self.v.data_ptr()
    for i, ((o, n), g) in enumerate(zip(self.segments, grads)):
      assert g.numel() == n and g.dtype == torch.float32 and g.is_cuda
      tl.var[i] = base_p + 4 * o
      tl.grad[i] = g.data_ptr()
      tl.m[i] = base_m + 4 * o
      tl.v[i] = base_v + 4 * o
      tl.n[i] = n
    _lib.call('dq_adam_tf1_multi', ctypes.byref(tl), p(self.state), self._slot(slot), self.lr,
              self.b1, self.b2, self.eps, _stream(self.params))


class TF1RMSProp(object):
  """tf.train.RMSPropOptimizer (rms slot initialised to one, as TF1)."""

  def __init__(self, params, learning_rate=0.00025, decay=0.95, momentum=0.0, epsilon=1e-5,
               centered=True):
    self.params = params
    self.lr, self.decay, self.mu, self.eps = float(learning_rate), float(decay), float(momentum), float(epsilon)
    self.centered = bool(centered)
    self.ms = torch.ones_like(params)
    self.mg = torch.zeros_like(params)
    self.mom = torch.zeros_like(params)

  supports_multi = False

  def step(self, grad, slot=None):
    _lib.call('dq_rmsprop_tf1', p(self.params), p(_c(grad, torch.float32)), p(self.ms), p(self.mg),
              p(self.mom), self.params.numel(), self.lr, self.decay, self.mu, self.eps,
              int(self.centered), _stream(self.params))


def sync_copy(dst, src):
  """Online -> target copy (dqn_agent.py:324-339)."""
  assert dst.numel() == src.numel() and dst.dtype == src.dtype
  _lib.call('dq_sync_copy', p(dst), p(src), dst.numel() * dst.element_size(), _stream(dst))
