"""Rainbow / C51 agent (reference dopamine/agents/rainbow/rainbow_agent.py:52-494).

The target distribution, the Eq.-7 projection, the softmax cross-entropy, the
PER importance weights and the new priorities are ONE HIP kernel
(``dq_c51_loss``); the priority write-back is the ordered sum-tree update kernel,
stream-ordered before the optimizer exactly as the reference's
control_dependencies order it (rainbow_agent.py:289-297).
"""
import numpy as np
import torch

from dopamine_amd import ops
from dopamine_amd.agents import networks
from dopamine_amd.agents.dqn import dqn_agent
from dopamine_amd.agents.optimizers import AdamOptimizer
from dopamine_amd.replay_memory import circular_replay_buffer
from dopamine_amd.replay_memory import prioritized_replay_buffer


class InvalidArgumentError(ValueError):
  """Stands in for ``tf.errors.InvalidArgumentError``: a failed ``validate_args``
  assertion (rainbow_agent.py:388-410).  Everything here is eager, so the
  assertions fire at call time."""


def project_distribution(supports, weights, target_support, validate_args=False):
  """rainbow_agent.py:340-494 as a torch expression (used for inspection and
  by tests; the training path uses the fused HIP kernel).

  Errors follow the reference: a 0-d target support fails its ``[1:]`` slice
  ('Index out of range', rb:381), one with fewer than two rows fails ``deltas[0]``
  ('out of bounds', rb:383), inconsistent supports / weights / target shapes fail
  the static checks ('are incompatible', rb:385-387), and with ``validate_args`` a
  non-increasing or unequally spaced target support raises InvalidArgumentError
  ('assertion failed', rb:402-410)."""
  supports = torch.as_tensor(supports, dtype=torch.float32)
  weights = torch.as_tensor(weights, dtype=torch.float32, device=supports.device)
  target_support = torch.as_tensor(target_support, dtype=torch.float32, device=supports.device)
  if target_support.dim() == 0:
    raise ValueError('Index out of range using input dim 0 of the target support')
  deltas = target_support[1:] - target_support[:-1]
  if deltas.shape[0] == 0:
    raise ValueError('slice index 0 of dimension 0 out of bounds (target support of shape %s)'
                     % (tuple(target_support.shape),))
  delta_z = deltas[0]
  if tuple(supports.shape) != tuple(weights.shape):
    raise ValueError('Shapes %s and %s are incompatible' % (tuple(supports.shape),
                                                            tuple(weights.shape)))
  if tuple(supports.shape[1:]) != tuple(target_support.shape):
    raise ValueError('Shapes %s and %s are incompatible' % (tuple(supports.shape[1:]),
                                                            tuple(target_support.shape)))
  if target_support.dim() != 1:
    raise ValueError('Shape %s must have rank 1' % (tuple(target_support.shape),))
  if validate_args:
    if not bool((deltas > 0).all()):
      raise InvalidArgumentError('assertion failed: target_support is not monotonically increasing')
    if not bool((deltas == delta_z).all()):
      raise InvalidArgumentError('assertion failed: target_support is not equally spaced')
  clipped = supports.clamp(target_support[0], target_support[-1])[:, None, :]
  quot = 1 - (clipped - target_support[None, :, None]).abs() / delta_z
  return (quot.clamp(0, 1) * weights[:, None, :]).sum(-1)


class RainbowAgent(dqn_agent.DQNAgent):
  """rainbow_agent.py:52-337."""

  def __init__(self,
               sess=None,
               num_actions=None,
               observation_shape=dqn_agent.NATURE_DQN_OBSERVATION_SHAPE,
               observation_dtype=dqn_agent.NATURE_DQN_DTYPE,
               stack_size=dqn_agent.NATURE_DQN_STACK_SIZE,
               network=networks.RainbowNetwork,
               num_atoms=51,
               vmax=10.,
               gamma=0.99,
               update_horizon=1,
               min_replay_history=20000,
               update_period=4,
               target_update_period=8000,
               epsilon_fn=dqn_agent.linearly_decaying_epsilon,
               epsilon_train=0.01,
               epsilon_eval=0.001,
               epsilon_decay_period=250000,
               replay_scheme='prioritized',
               tf_device='/gpu:0',
               use_staging=True,
               optimizer=AdamOptimizer(learning_rate=0.00025, epsilon=0.0003125),
               summary_writer=None,
               summary_writing_frequency=500,
               **kwargs):
    vmax = float(vmax)
    self._num_atoms = num_atoms
    self._vmax = vmax
    self._replay_scheme = replay_scheme
    super().__init__(sess=sess, num_actions=num_actions, observation_shape=observation_shape,
                     observation_dtype=observation_dtype, stack_size=stack_size, network=network,
                     gamma=gamma, update_horizon=update_horizon,
                     min_replay_history=min_replay_history, update_period=update_period,
                     target_update_period=target_update_period, epsilon_fn=epsilon_fn,
                     epsilon_train=epsilon_train, epsilon_eval=epsilon_eval,
                     epsilon_decay_period=epsilon_decay_period, tf_device=tf_device,
                     use_staging=use_staging, optimizer=optimizer, summary_writer=summary_writer,
                     summary_writing_frequency=summary_writing_frequency, **kwargs)

  _loss_name = 'CrossEntropyLoss'

  def _build_replay_buffer(self, use_staging):
    if self._replay_scheme not in ['uniform', 'prioritized']:
      raise ValueError('Invalid replay scheme: {}'.format(self._replay_scheme))
    return prioritized_replay_buffer.WrappedPrioritizedReplayBuffer(
        observation_shape=self.observation_shape, stack_size=self.stack_size,
        use_staging=use_staging, update_horizon=self.update_horizon, gamma=self.gamma,
        observation_dtype=self.observation_dtype, replay_capacity=self._replay_capacity,
        batch_size=self._batch_size, device=self._device)

  def _make_network(self, seed):
    return self.network(self.num_actions, num_atoms=self._num_atoms, stack_size=self.stack_size,
                        device=self._device, seed=seed)

  def _build_train_op(self):
    B, A, N, dev = self._batch_size, self.num_actions, self._num_atoms, self._device
    # tf.linspace(-vmax, vmax, num_atoms) in float32 (rainbow_agent.py:126)
    step = np.float32(2 * self._vmax) / np.float32(N - 1)
    sup = (np.float32(-self._vmax) + step * np.arange(N, dtype=np.float32)).astype(np.float32)
    self._support = torch.from_numpy(sup).to(dev)
    # mean_loss=None: the summary mean is not on the gradient path (computed on demand)
    self._loss_out = dict(grad=torch.empty((B, A, N), device=dev), loss=torch.empty(B, device=dev),
                          priorities=torch.empty(B, device=dev), mean_loss=None)
    self._c51_m = torch.empty((B, N), device=dev)   # head_from 8: the projected target distribution

  def mean_loss(self):
    """mean(w * CE) of the last step (the CrossEntropyLoss summary, rb:298-301)."""
    self.check_exchange()
    loss = self._loss_out['loss']
    if self._replay_scheme == 'prioritized':
      w = 1.0 / torch.sqrt(self._replay.transition['sampling_probabilities'] + 1e-10)
      loss = loss * (w / w.max())
    return float(loss.mean().item())

  def _q_from_output(self, out):
    logits = out.reshape(out.shape[0], self.num_actions, self._num_atoms)
    return (torch.softmax(logits, -1) * self._support).sum(-1)

  def _target_dict(self, out):
    return {'logits': out.view(-1, self.num_actions, self._num_atoms)}

  def _target_forward(self, t, slot):
    return self._target_dict(self._target_net(t['next_state'], slot))

  def _online_loss(self, t, tgt):
    """rainbow_agent.py:200-305."""
    logits = self._online_forward(t['state']).view(-1, self.num_actions, self._num_atoms)
    prioritized = self._replay_scheme == 'prioritized'
    out = ops.c51_loss(logits.detach(), tgt['logits'], t['action'], t['reward'], t['terminal'],
                       self._support, self.cumulative_gamma,
                       probs=t['sampling_probabilities'] if prioritized else None,
                       out=self._loss_out)
    return logits, out['grad']

  # The C51 loss split in two (head_from 8): the target half (softmax, Q, greedy action,
  # projection: rb:200-251, 340-494) rides in the online forward's last launch, the target
  # network running one launch ahead of the online one; the loss launch keeps the online
  # half.  Bitwise the single-kernel loss (tests/test_gpu_cnn.py).  Measured (rocprof,
  # profiles/r2_c51_split_ab.txt): the loss launch 9.6 -> 6.6 us, but the target's conv2
  # beside the online conv1 takes that launch 6.4 -> 10.6 us: 7,290 vs 7,220 steps/s for
  # the one-kernel loss, so off by default.
  split_c51 = False

  def _head_from(self):
    if self._fused() and self.split_c51 and self.num_actions <= 16 and self._num_atoms <= 64:
      return 8
    return super()._head_from()

  def _forward_fused_c51(self, c, part=None):
    from dopamine_amd import cnn
    t, tg = self._pbuf[c], self._hip['target'][c]
    cnn.forward_fused_c51(self._hip['online'], t['state'], tg, t['reward'], t['terminal'],
                          self._support, self.cumulative_gamma, self._c51_m,
                          target_logits_out=tg.acts['out'] if self._trace is not None else None,
                          part=part)

  def _fused_loss(self, t, c):
    """_online_loss on the CNN's fc2 partials (cnn.forward_fused): the logits are
    summed inside the loss kernel, which also writes fc2's input gradient."""
    prioritized = self._replay_scheme == 'prioritized'
    if self._head_from() == 8:
      out = ops.c51_loss_online(self._hip['online'], self._c51_m, t['action'],
                                probs=t['sampling_probabilities'] if prioritized else None,
                                out=self._loss_out, logits_out=self._trace is not None)
      return None, out['grad']
    out = ops.c51_loss_fused(self._hip['online'], self._hip['target'][c], t['action'], t['reward'],
                             t['terminal'], self._support, self.cumulative_gamma,
                             probs=t['sampling_probabilities'] if prioritized else None,
                             out=self._loss_out, logits_out=self._trace is not None)
    return None, out['grad']

  def _trace_outputs(self, c):
    d = super()._trace_outputs(c)
    d['priorities'] = self._loss_out['priorities']
    return d

  def _post_loss(self, t):
    if self._replay_scheme == 'prioritized':
      # sqrt(loss + 1e-10) of the UNWEIGHTED loss (rb:289-290); it precedes the
      # next step's sample on the same stream, as control_dependencies order it.
      self._replay.tf_set_priority(t['indices'], self._loss_out['priorities'])

  def _store_transition(self, last_observation, action, reward, is_terminal, priority=None):
    """rainbow_agent.py:307-337.  The default prioritized-scheme priority, the sum tree's
    max_recorded_priority, is read by the add kernel on the device (no host round trip)."""
    if priority is None:
      if self._replay_scheme == 'uniform':
        priority = 1.
      else:
        priority = circular_replay_buffer.MAX_RECORDED
    if not self.eval_mode:
      self._replay.add(last_observation, action, reward, is_terminal, priority)
