"""CPU oracle for the Q-learning update -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.

numpy restatement of the TF1 graph math on the hot path.  TensorFlow is not
installable here, so these functions cannot be run against the reference
itself; they follow the cited graph code and TF1 op semantics and are pinned
only where the reference's tests hold known answers (project_distribution:
rainbow_agent_test.py:178-285).  Huber / softmax-CE / quantile-Huber values and
the optimizer updates are "parity unpinned" (documented in DESIGN.md).

Every function takes a ``dtype`` so the float64 mode can serve as the
high-precision reference for the fp32 device kernels.
"""
import math

import numpy as np


def c51_support(vmax, num_atoms, dtype=np.float32):
  """tf.linspace(-vmax, vmax, num_atoms) (rainbow_agent.py:126)."""
  vmax = dtype(vmax)
  step = (vmax - (-vmax)) / dtype(num_atoms - 1)
  return (-vmax + step * np.arange(num_atoms, dtype=dtype)).astype(dtype)


def project_distribution(supports, weights, target_support, dtype=np.float64):
  """rainbow_agent.py:340-494 (Bellemare et al. 2017, Eq. 7)."""
  supports = np.asarray(supports, dtype)
  weights = np.asarray(weights, dtype)
  z = np.asarray(target_support, dtype)
  dz = z[1] - z[0]
  clipped = np.clip(supports, z[0], z[-1])[:, None, :]           # (B,1,N)
  quot = 1 - np.abs(clipped - z[None, :, None]) / dz              # (B,N,N)
  return (np.clip(quot, 0, 1) * weights[:, None, :]).sum(-1).astype(dtype)


def softmax(x, axis=-1):
  e = np.exp(x - x.max(axis=axis, keepdims=True))
  return e / e.sum(axis=axis, keepdims=True)


def c51_loss(online_logits, target_logits, actions, rewards, terminals, support,
             cumulative_gamma, probs=None, dtype=np.float64):
  """Rainbow target + loss (rainbow_agent.py:200-305).

  Returns dict(loss=(B,) unweighted CE, weights=(B,) PER weights or ones,
  grad=(B,A,N) d mean(w*loss) / d online_logits, priorities=sqrt(loss+1e-10),
  proj=(B,N), argmax=(B,))."""
  ol = np.asarray(online_logits, dtype)
  tl = np.asarray(target_logits, dtype)
  z = np.asarray(support, dtype)
  B, A, N = ol.shape
  gamma_t = dtype(cumulative_gamma) * (1 - np.asarray(terminals, dtype))
  tz = np.asarray(rewards, dtype)[:, None] + gamma_t[:, None] * z[None, :]
  tp = softmax(tl)
  q = (tp * z).sum(-1)
  astar = q.argmax(1)                                     # first max on ties
  proj = project_distribution(tz, tp[np.arange(B), astar], z, dtype)
  chosen = ol[np.arange(B), actions]
  sm = softmax(chosen)
  lse = np.log(np.exp(chosen - chosen.max(1, keepdims=True)).sum(1)) + chosen.max(1)
  loss = (proj * (lse[:, None] - chosen)).sum(1)
  if probs is not None:
    w = 1.0 / np.sqrt(np.asarray(probs, dtype) + dtype(1e-10))
    w = w / w.max()
  else:
    w = np.ones(B, dtype)
  grad = np.zeros_like(ol)
  # TF SoftmaxCrossEntropyWithLogits backprop = softmax - labels.
  grad[np.arange(B), actions] = (w / B)[:, None] * (sm - proj)
  # grad_abs: the magnitudes of the difference's two terms (oracle/nature_cnn.abs_grad)
  grad_abs = np.zeros_like(ol)
  grad_abs[np.arange(B), actions] = (w / B)[:, None] * (sm + proj)
  return dict(loss=loss, weights=w, grad=grad, grad_abs=grad_abs, proj=proj, argmax=astar,
              priorities=np.sqrt(loss + dtype(1e-10)), mean_loss=(w * loss).mean())


def dqn_huber(online_q, target_q, actions, rewards, terminals, cumulative_gamma,
              delta=1.0, dtype=np.float64):
  """dqn_agent.py:283-322 with tf.losses.huber_loss(reduction=NONE)."""
  oq = np.asarray(online_q, dtype)
  tq = np.asarray(target_q, dtype)
  B = oq.shape[0]
  target = (np.asarray(rewards, dtype) + dtype(cumulative_gamma) * tq.max(1) *
            (1 - np.asarray(terminals, dtype)))
  chosen = oq[np.arange(B), actions]
  err = chosen - target
  a = np.abs(err)
  quad = np.minimum(a, delta)
  loss = 0.5 * quad * quad + delta * (a - quad)
  grad = np.zeros_like(oq)
  grad[np.arange(B), actions] = np.clip(err, -delta, delta) / B
  grad_abs = np.zeros_like(oq)       # |q| + |target| of the difference err (abs_grad)
  grad_abs[np.arange(B), actions] = (np.abs(chosen) + np.abs(target)) / B
  return dict(loss=loss, grad=grad, grad_abs=grad_abs, target=target, mean_loss=loss.mean())


def iqn_loss(online_qv, target_qv, target_qv_action, taus, actions, rewards, terminals,
             cumulative_gamma, kappa=1.0, dtype=np.float64):
  """implicit_quantile_agent.py:190-321.

  online_qv: (N*B, A) rows ordered q*B + b (atari_lib.py:174 tiling), taus (N*B,)
  target_qv: (N'*B, A); target_qv_action: (K*B, A) for the argmax.
  Returns loss (B,), grad (N*B, A) of mean(loss) wrt online_qv."""
  oq = np.asarray(online_qv, dtype)
  tq = np.asarray(target_qv, dtype)
  ta = np.asarray(target_qv_action, dtype)
  B = len(rewards)
  A = oq.shape[1]
  N = oq.shape[0] // B
  Np = tq.shape[0] // B
  K = ta.shape[0] // B
  qmean = ta.reshape(K, B, A).mean(0)
  astar = qmean.argmax(1)
  gam = dtype(cumulative_gamma) * (1 - np.asarray(terminals, dtype))
  tvals = tq.reshape(Np, B, A)[:, np.arange(B), astar]              # (N', B)
  T = np.asarray(rewards, dtype)[None, :] + gam[None, :] * tvals      # (N', B)
  T = T.T                                                             # (B, N')
  theta = oq.reshape(N, B, A)[:, np.arange(B), actions].T             # (B, N)
  tau = np.asarray(taus, dtype).reshape(N, B).T                       # (B, N)
  u = T[:, :, None] - theta[:, None, :]                               # (B, N', N)
  au = np.abs(u)
  hub = np.where(au <= kappa, 0.5 * u * u, kappa * (au - 0.5 * kappa))
  ind = (u < 0).astype(dtype)
  w = np.abs(tau[:, None, :] - ind)
  rho = w * hub / kappa
  loss = rho.sum(2).mean(1)                                           # (B,)
  dh = np.where(au <= kappa, u, kappa * np.sign(u))
  dtheta = -(w * dh / kappa).sum(1) / Np / B                           # (B, N)
  grad = np.zeros_like(oq).reshape(N, B, A)
  grad[:, np.arange(B), actions] = dtheta.T
  # grad_abs: each term's magnitude, |T| + |theta| where u = T - theta enters linearly
  dabs = np.where(au <= kappa, np.abs(T)[:, :, None] + np.abs(theta)[:, None, :], kappa)
  gabs = np.zeros_like(oq).reshape(N, B, A)
  gabs[:, np.arange(B), actions] = ((w * dabs / kappa).sum(1) / Np / B).T
  return dict(loss=loss, grad=grad.reshape(N * B, A), grad_abs=gabs.reshape(N * B, A),
              mean_loss=loss.mean(), argmax=astar)


class TF1Adam:
  """tf.train.AdamOptimizer / ApplyAdam (TF1 training_ops), float32 state.

  m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
  var -= lr*sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps); b_power *= b."""

  def __init__(self, n, lr, beta1=0.9, beta2=0.999, eps=1e-8, dtype=np.float32):
    self.dt = dtype
    self.lr, self.b1, self.b2, self.eps = (dtype(x) for x in (lr, beta1, beta2, eps))
    self.m = np.zeros(n, dtype)
    self.v = np.zeros(n, dtype)
    self.b1p = dtype(beta1)
    self.b2p = dtype(beta2)

  def step(self, var, g):
    dt = self.dt
    one = dt(1)
    alpha = dt(self.lr * dt(np.sqrt(one - self.b2p)) / (one - self.b1p))
    self.m += (g - self.m) * (one - self.b1)
    self.v += (g * g - self.v) * (one - self.b2)
    var -= (self.m * alpha) / (np.sqrt(self.v) + self.eps)
    self.b1p = dt(self.b1p * self.b1)
    self.b2p = dt(self.b2p * self.b2)
    return var


class TF1CenteredRMSProp:
  """tf.train.RMSPropOptimizer(centered=True) / ApplyCenteredRMSProp.

  rms slot initialised to ONE (TF1), mg and mom to zero."""

  def __init__(self, n, lr, decay=0.9, momentum=0.0, eps=1e-10, dtype=np.float32):
    self.dt = dtype
    self.lr, self.rho, self.mu, self.eps = (dtype(x) for x in (lr, decay, momentum, eps))
    self.ms = np.ones(n, dtype)
    self.mg = np.zeros(n, dtype)
    self.mom = np.zeros(n, dtype)

  def step(self, var, g):
    one = self.dt(1)
    self.ms += (g * g - self.ms) * (one - self.rho)
    self.mg += (g - self.mg) * (one - self.rho)
    denom = self.ms - self.mg * self.mg + self.eps
    self.mom = self.mom * self.mu + (g * self.lr) / np.sqrt(denom)
    var -= self.mom
    return var


def linearly_decaying_epsilon(decay_period, step, warmup_steps, epsilon):
  """dqn_agent.py:45-67."""
  steps_left = decay_period + warmup_steps - step
  bonus = (1.0 - epsilon) * steps_left / decay_period
  bonus = np.clip(bonus, 0., 1. - epsilon)
  return epsilon + bonus


def cumulative_gamma(gamma, n):
  return math.pow(gamma, n)
