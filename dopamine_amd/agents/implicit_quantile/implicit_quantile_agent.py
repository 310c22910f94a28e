"""IQN agent (reference implicit_quantile_agent.py:36-321).

Online net on s with N tau samples, target net on s' with N' samples, greedy
next action from the mean of K target (or online, double_dqn) quantiles; the
quantile-Huber loss and its gradient are one HIP kernel (``dq_iqn_loss``).
Tau samples come from torch's device RNG (the reference's tf.random_uniform
stream cannot be reproduced without TF: parity is on given taus).
"""
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

  def _make_network(self, seed):
    return self.network(self.num_actions, quantile_embedding_dim=self.quantile_embedding_dim,
                        stack_size=self.stack_size, device=self._device, seed=seed)

  def _build_train_op(self):
    B, A, dev = self._batch_size, self.num_actions, self._device
    self._loss_out = dict(grad=torch.empty((self.num_tau_samples * B, A), device=dev),
                          loss=torch.empty(B, device=dev), mean_loss=torch.empty(1, device=dev))

  def _post_loss(self, t):
    """No priority write-back: the reference IQN's train op never calls
    set_priority (iqn:314, "TODO: Add prioritized replay functionality"), so with
    replay_scheme='prioritized' the stored priorities are the insert-time ones."""

  def _online_q(self, x):
    qv, _ = self.online_convnet(x, self.num_quantile_samples)
    return qv.view(self.num_quantile_samples, x.shape[0], -1).mean(0)

  def _target_forward(self, t, slot):
    with torch.no_grad():
      tq, _ = self.target_convnet(t['next_state'], self.num_tau_prime_samples)
      out = {'tq': tq}
      if not self.double_dqn:   # double DQN's argmax net is the online net of THIS step
        out['ta'], _ = self.target_convnet(t['next_state'], self.num_quantile_samples)
      return out

  def _online_loss(self, t, tgt):
    """implicit_quantile_agent.py:190-321."""
    ta = tgt.get('ta')
    if ta is None:
      with torch.no_grad():
        ta, _ = self.online_convnet(t['next_state'], self.num_quantile_samples)
    qv, taus = self.online_convnet(t['state'], self.num_tau_samples)
    out = ops.iqn_loss(qv.detach(), tgt['tq'], ta, taus, t['action'], t['reward'], t['terminal'],
                       self.cumulative_gamma, self.kappa, out=self._loss_out)
    return qv, out['grad']
