"""IQN agent (reference implicit_quantile_agent.py:36-321).

Online net on s with N tau samples, target net on s' with N' samples, greedy next
action from the mean of K target (or online, double_dqn) quantiles; the
quantile-Huber loss and its gradient are one HIP kernel (``dq_iqn_loss``).

With the Atari geometry the ImplicitQuantileNetwork runs on the HIP kernels
(dopamine_amd/iqn.py): the Nature-CNN torso on nature_cnn.hip and the quantile head
(cosine embedding, Hadamard product, FC 7744 -> 512 -> A and their backward) on the
fp32 matrix cores (iqn.hip).  The target net's N' and K quantile rows share one torso
pass and one head pass (R = (N' + K) * B rows).  Tau samples come from a device
counter-based generator (TF's tf.random_uniform stream cannot be reproduced without
TF: parity is on given taus), so a captured HIP graph draws what eager calls draw.
"""
import numpy as np
import torch

from dopamine_amd import ops
from dopamine_amd.agents import networks
from dopamine_amd.agents.optimizers import AdamOptimizer
from dopamine_amd.agents.rainbow import rainbow_agent


class ImplicitQuantileAgent(rainbow_agent.RainbowAgent):

  def __init__(self,
               sess=None,
               num_actions=None,
               network=networks.ImplicitQuantileNetwork,
               kappa=1.0,
               num_tau_samples=32,
               num_tau_prime_samples=32,
               num_quantile_samples=32,
               quantile_embedding_dim=64,
               double_dqn=False,
               summary_writer=None,
               summary_writing_frequency=500,
               **kwargs):
    self.kappa = kappa
    self.num_tau_samples = num_tau_samples
    self.num_tau_prime_samples = num_tau_prime_samples
    self.num_quantile_samples = num_quantile_samples
    self.quantile_embedding_dim = quantile_embedding_dim
    self.double_dqn = double_dqn
    kwargs.setdefault('optimizer', AdamOptimizer(learning_rate=0.00025, epsilon=0.0003125))
    super().__init__(sess=sess, num_actions=num_actions, network=network,
                     summary_writer=summary_writer,
                     summary_writing_frequency=summary_writing_frequency, **kwargs)

  _loss_name = 'QuantileLoss'
  # the act path's Q-values draw taus from the device counter, so evaluating them on every
  # action (the device epsilon-greedy does) would move the tau stream: host draws here
  device_egreedy = False

  def _make_network(self, seed):
    return self.network(self.num_actions, quantile_embedding_dim=self.quantile_embedding_dim,
                        stack_size=self.stack_size, device=self._device, seed=seed)

  def _build_networks(self):
    super()._build_networks()
    self._iqn = None
    if (self.use_hip_cnn and self.network is networks.ImplicitQuantileNetwork and
        self.observation_shape == (84, 84) and self.stack_size == 4):
      from dopamine_amd.iqn import HipIqnNet, TauSampler
      B = self._batch_size
      n_tgt = self.num_tau_prime_samples + (0 if self.double_dqn else self.num_quantile_samples)
      self._iqn = dict(
          online=HipIqnNet(self.online_convnet, B, self.num_tau_samples, keep=True),
          target=[HipIqnNet(self.target_convnet, B, n_tgt, keep=False) for _ in range(2)])
      if self.double_dqn:   # argmax from the ONLINE net on s' (iqn:205-214)
        self._iqn['online_next'] = HipIqnNet(self.online_convnet, B, self.num_quantile_samples,
                                             keep=False)
      self._taus = TauSampler(0x5EED0000 + self._seed, self._device)

  def _build_train_op(self):
    B, A, dev = self._batch_size, self.num_actions, self._device
    # mean_loss None: the summary mean is not on the gradient path (computed on demand)
    self._loss_out = dict(grad=torch.empty((self.num_tau_samples * B, A), device=dev),
                          loss=torch.empty(B, device=dev), mean_loss=None)

  def mean_loss(self):
    """mean over the batch of the quantile loss (the QuantileLoss summary, iqn:316-319)."""
    self.check_exchange()
    return float(self._loss_out['loss'].double().mean().item())

  def _needs_flat_grad(self):
    return self._iqn is not None or super()._needs_flat_grad()

  def _post_loss(self, t):
    """No priority write-back: the reference IQN's train op never calls
    set_priority (iqn:314, "TODO: Add prioritized replay functionality"), so with
    replay_scheme='prioritized' the stored priorities are the insert-time ones."""

  def _online_q(self, x):
    qv, _ = self.online_convnet(x, self.num_quantile_samples)
    return qv.view(self.num_quantile_samples, x.shape[0], -1).mean(0)

  def _q_values(self, state_np):
    """Action selection (iqn:216-228 _q_values: the mean over K quantiles of the
    online net), on the HIP executor at batch 1."""
    if self._iqn is None:
      return super()._q_values(state_np)
    if 'act' not in self._iqn:
      from dopamine_amd.iqn import HipIqnNet
      self._iqn['act'] = HipIqnNet(self.online_convnet, 1, self.num_quantile_samples, keep=False)
    ex = self._iqn['act']
    scale = 1.0 / 255.0 if np.dtype(self.observation_dtype) == np.uint8 else 1.0
    x = torch.as_tensor(np.asarray(state_np) * scale, dtype=torch.float32, device=self._device)
    self._taus.draw_cos(ex)
    q, _ = ex.forward(x.reshape(1, 84, 84, 4).contiguous(), cos_ready=True)
    return q.view(self.num_quantile_samples, 1, -1).mean(0)

  def _target_forward(self, t, slot):
    if self._iqn is not None:
      ex = self._iqn['target'][slot]
      self._taus.draw_cos(ex)           # N' tau' (iqn:197-199) then K argmax samples (:200-204)
      q, _ = ex.forward(t['next_state'], cos_ready=True)
      npb = self.num_tau_prime_samples * self._batch_size
      out = {'tq': q[:npb]}
      if not self.double_dqn:
        out['ta'] = q[npb:]
      return out
    with torch.no_grad():
      tq, _ = self.target_convnet(t['next_state'], self.num_tau_prime_samples)
      out = {'tq': tq}
      if not self.double_dqn:   # double DQN's argmax net is the online net of THIS step
        out['ta'], _ = self.target_convnet(t['next_state'], self.num_quantile_samples)
      return out

  def _online_loss(self, t, tgt):
    """implicit_quantile_agent.py:190-321."""
    ta = tgt.get('ta')
    if self._iqn is not None:
      if ta is None:
        ex = self._iqn['online_next']
        self._taus.draw_cos(ex)
        ta, _ = ex.forward(t['next_state'], cos_ready=True)
      on = self._iqn['online']
      self._taus.draw_cos(on)
      qv, taus = on.forward(t['state'], cos_ready=True)
    else:
      if ta is None:
        with torch.no_grad():
          ta, _ = self.online_convnet(t['next_state'], self.num_quantile_samples)
      qv, taus = self.online_convnet(t['state'], self.num_tau_samples)
    out = ops.iqn_loss(qv.detach(), tgt['tq'], ta, taus, t['action'], t['reward'], t['terminal'],
                       self.cumulative_gamma, self.kappa, out=self._loss_out)
    self._last_ta = ta
    return qv, out['grad']

  def _fused_opt(self):
    """The HIP executor with TF1 Adam / RMSProp, a single replica and no double DQN: the
    optimizer step runs inside the torso's backward launches (HipIqnNet.backward(adam=...),
    dq_cnn_backward_torso_opt) instead of a launch of its own after the step.  double_dqn
    reads the online network on s' on the prefetch stream during the backward, so there the
    update waits for it (the separate step after the streams join)."""
    return (self.fuse_optimizer and self._iqn is not None and self._pg is None and
            not self.double_dqn and isinstance(self._opt, (ops.TF1Adam, ops.TF1RMSProp)))

  def _backward(self, y, g, k=0):
    if self._iqn is not None:
      if self._fused_opt():
        self._iqn['online'].backward(g, adam=self._opt, slot=k, store_grads=self._store_grads())
      else:
        self._iqn['online'].backward(g)
      return
    super()._backward(y, g, k)

  def _trace_outputs(self, c):
    d = rainbow_agent.dqn_agent.DQNAgent._trace_outputs(self, c)
    if self._iqn is not None:
      on, tg = self._iqn['online'], self._iqn['target'][c]
      d['qv'] = on.acts['q']
      d['taus'] = on.taus
      d['target_q'] = tg.acts['q']
      d['target_taus'] = tg.taus
      if self.double_dqn:            # the online net's argmax quantiles on s'
        d['online_next_q'] = self._iqn['online_next'].acts['q']
        d['online_next_taus'] = self._iqn['online_next'].taus
    return d
