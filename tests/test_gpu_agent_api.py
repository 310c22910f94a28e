"""The reference's agent unit tests restated on the device: dqn_agent_test.py,
rainbow_agent_test.py:288-489 and implicit_quantile_agent_test.py, against the
drop-in agents (same constructor arguments, same attributes: ``state``,
``_observation``, ``_last_observation``, ``training_steps``, ``_replay``,
``bundle_and_checkpoint`` / ``unbundle``).

The reference builds its mock agents by overriding ``_network_template``; here a
network is a class over one flat parameter buffer (agents/networks.py), so the
mocks are ``networks._Net`` subclasses with the same layers and initialisers
(zero inputs into a fully connected layer, ones biases: every action ties and the
argmax is action 0).  Deviations, each for test time only: the mock agents'
replay holds 10,000 transitions (the reference's default 1M would make the partial
unbundling test gzip 7 GB of zero frames); testCreateAgentWithDefaults keeps the
defaults.  The device-free tests (project_distribution, the non-tuple observation
shape, the epsilon schedule) are in tests/test_agent_api_cpu.py."""
from unittest import mock

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from dopamine_amd.agents import networks
from dopamine_amd.agents.dqn import dqn_agent
from dopamine_amd.agents.implicit_quantile import implicit_quantile_agent
from dopamine_amd.agents.rainbow import rainbow_agent

pytestmark = pytest.mark.gpu

OBS, DT, STACK = dqn_agent.NATURE_DQN_OBSERVATION_SHAPE, dqn_agent.NATURE_DQN_DTYPE, 4
SMALL = 10000


class MockReplayBuffer(object):
  """utils/test_utils.py:27-35."""

  def __init__(self):
    self.add = mock.Mock()
    self.memory = mock.Mock()
    self.memory.add_count = 0


class MockDQNNetwork(networks._Net):
  """dqn-test 57-73: fully_connected(zeros (B, stack)) with weights
  tile(arange(A, 0, -1), (stack, 1)) and ones biases."""

  def __init__(self, num_actions, stack_size=4, device='cuda', seed=0):
    self.A, self.S = num_actions, stack_size
    super().__init__(device, seed)
    with torch.no_grad():
      w = np.tile(np.arange(self.A, 0, -1), (self.S, 1))          # (stack, A), slim's layout
      self.fp['fc_w'].copy_(torch.as_tensor(w.T, dtype=torch.float32))
      self.fp['fc_b'].fill_(1.0)

  def shapes(self):
    return [('fc_w', (self.A, self.S)), ('fc_b', (self.A,))]

  def forward(self, x):
    inputs = torch.zeros((x.shape[0], self.S), device=self.fp.flat.device)
    return F.linear(inputs, self.fp['fc_w'], self.fp['fc_b'])


class MockRainbowNetwork(networks._Net):
  """rb-test 303-333: the first action's logits weighted arange(num_atoms), every
  other weight one, ones biases; logits (B, A, N)."""

  def __init__(self, num_actions, num_atoms=51, stack_size=4, device='cuda', seed=0):
    self.A, self.N, self.S = num_actions, num_atoms, stack_size
    super().__init__(device, seed)
    first = np.concatenate((np.arange(self.N), np.tile(np.ones(self.N), self.A - 1)))
    w = np.concatenate(([first], np.tile(np.ones(self.A * self.N), (self.S - 1, 1))))
    with torch.no_grad():
      self.fp['fc_w'].copy_(torch.as_tensor(w.T, dtype=torch.float32))
      self.fp['fc_b'].fill_(1.0)

  def shapes(self):
    return [('fc_w', (self.A * self.N, self.S)), ('fc_b', (self.A * self.N,))]

  def forward(self, x):
    inputs = torch.zeros((x.shape[0], self.S), device=self.fp.flat.device)
    return F.linear(inputs, self.fp['fc_w'], self.fp['fc_b']).view(-1, self.A, self.N)


class MockImplicitQuantileNetwork(networks._Net):
  """iqn-test 41-64: ones(B, A) tiled num_quantiles times, times ones quantiles,
  through fully_connected with ones weights and zero biases: every quantile value
  equals num_actions."""

  def __init__(self, num_actions, quantile_embedding_dim=64, stack_size=4, device='cuda', seed=0):
    self.A = num_actions
    super().__init__(device, seed)
    with torch.no_grad():
      self.fp['fc_w'].fill_(1.0)
      self.fp['fc_b'].zero_()

  def shapes(self):
    return [('fc_w', (self.A, self.A)), ('fc_b', (self.A,))]

  def forward(self, x, num_quantiles, taus=None):
    B, dev = x.shape[0], self.fp.flat.device
    state_net = torch.ones((B, self.A), device=dev)
    quantiles = torch.ones((num_quantiles * B, 1), device=dev)
    qv = F.linear(state_net.repeat(num_quantiles, 1) * quantiles.repeat(1, self.A),
                  self.fp['fc_w'], self.fp['fc_b'])
    return qv, quantiles


# ----------------------------------------------------------------------- DQN
def _dqn(observation_shape=OBS, observation_dtype=DT, stack_size=STACK, allow_partial_reload=False):
  """dqn-test 53-91."""
  agent = dqn_agent.DQNAgent(
      num_actions=4, observation_shape=observation_shape, observation_dtype=observation_dtype,
      stack_size=stack_size, network=MockDQNNetwork, min_replay_history=6,
      epsilon_fn=lambda w, x, y, z: 0.0, update_period=2, target_update_period=4,
      epsilon_eval=0.0, allow_partial_reload=allow_partial_reload, replay_capacity=SMALL)
  agent.eval_mode = True
  return agent


@pytest.mark.parametrize('cls', [dqn_agent.DQNAgent, rainbow_agent.RainbowAgent,
                                 implicit_quantile_agent.ImplicitQuantileAgent])
def test_create_agent_with_defaults(cls):
  """dqn-test 93-101, rb-test 341-349, iqn-test 75-83: the default (HIP) networks,
  1M-transition replay."""
  agent = cls(num_actions=4)
  observation = np.ones([84, 84, 1])
  a = agent.begin_episode(observation)
  assert 0 <= a < 4
  agent.step(reward=1, observation=observation)
  agent.end_episode(reward=1)
  assert agent._replay.memory.add_count == 2 + STACK - 1     # + the episode-start zero padding
  assert agent.training_steps == 2


def _begin_episode(agent):
  """dqn-test 103-139 / rb-test 370-406."""
  zero_state = np.zeros((1,) + OBS + (STACK,))
  agent.state.fill(9)
  first = np.ones(OBS + (1,))
  assert agent.begin_episode(first) == 0
  expected = zero_state.copy()
  expected[:, :, :, -1] = np.ones((1,) + OBS)
  np.testing.assert_array_equal(agent.state, expected)
  np.testing.assert_array_equal(agent._observation, first[:, :, 0])
  assert agent.training_steps == 0
  agent.eval_mode = False
  agent._replay.memory.add_count = 0
  second = np.ones(OBS + (1,)) * 2
  agent.begin_episode(second)
  expected[:, :, :, -1] = np.full((1,) + OBS, 2)
  np.testing.assert_array_equal(agent.state, expected)
  np.testing.assert_array_equal(agent._observation, second[:, :, 0])
  assert agent.training_steps == 1


def _step_eval(agent):
  """dqn-test 141-175 / rb-test 408-441."""
  base = np.ones(OBS + (1,))
  agent.begin_episode(base)
  agent._replay = MockReplayBuffer()
  expected = np.zeros((1,) + OBS + (STACK,))
  num_steps = 10
  for step in range(1, num_steps + 1):
    observation = base * step
    assert agent.step(reward=1, observation=observation) == 0
    stack_pos = step - num_steps - 1
    if stack_pos >= -STACK:
      expected[:, :, :, stack_pos] = np.full((1,) + OBS, step)
  np.testing.assert_array_equal(agent.state, expected)
  np.testing.assert_array_equal(agent._last_observation, np.ones(OBS) * (num_steps - 1))
  np.testing.assert_array_equal(agent._observation, observation[:, :, 0])
  assert agent.training_steps == 0
  assert agent._replay.add.call_count == 0


def _step_train(agent, shape=OBS, stack=STACK, check_args=True):
  """dqn-test 177-231 and its custom-shape form 255-305 / rb-test 443-475."""
  agent.eval_mode = False
  base = np.ones(shape + (1,))
  agent._replay = MockReplayBuffer()
  agent.begin_episode(base)
  observation = base
  expected = np.zeros((1,) + shape + (stack,))
  num_steps = 10
  for step in range(1, num_steps + 1):
    last_observation = observation
    observation = base * step
    assert agent.step(reward=1, observation=observation) == 0
    stack_pos = step - num_steps - 1
    if stack_pos >= -stack:
      expected[..., stack_pos] = np.full((1,) + shape, step)
    assert agent._replay.add.call_count == step
    if check_args:
      args, _ = agent._replay.add.call_args
      np.testing.assert_array_equal(last_observation[..., 0], args[0])
      assert args[1] == 0 and args[2] == 1 and not args[3]
  np.testing.assert_array_equal(agent.state, expected)
  np.testing.assert_array_equal(agent._last_observation, np.full(shape, num_steps - 1))
  np.testing.assert_array_equal(agent._observation, observation[..., 0])
  assert agent.training_steps == num_steps + 1
  assert agent._replay.add.call_count == num_steps
  agent.end_episode(reward=1)
  assert agent._replay.add.call_count == num_steps + 1
  if check_args:
    args, _ = agent._replay.add.call_args
    np.testing.assert_array_equal(observation[..., 0], args[0])
    assert args[1] == 0 and args[2] == 1 and args[3]


def test_dqn_begin_episode():
  _begin_episode(_dqn())


def test_dqn_step_eval():
  _step_eval(_dqn())


def test_dqn_step_train():
  _step_train(_dqn())


@pytest.mark.parametrize('shape,dtype,stack', [
    ((1,), np.uint8, 1), ((4, 4), np.uint8, 1), ((6, 1), np.uint8, 1), ((1, 6), np.uint8, 1),
    ((1, 1, 6), np.uint8, 1), ((6, 6, 6, 6), np.uint8, 1),          # dqn-test 307-310
    ((4, 4), np.float32, 1), ((4, 4), np.int64, 1),                  # dqn-test 312-315
    ((4, 4), np.uint8, 4), ((4, 4), np.uint8, 8)])                   # dqn-test 317-320
def test_dqn_step_train_custom(shape, dtype, stack):
  _step_train(_dqn(shape, dtype, stack), shape, stack)


def test_bundling_with_nonexistent_directory():
  """dqn-test 322-325."""
  assert _dqn().bundle_and_checkpoint('/does/not/exist', 1) is None


def test_unbundling_with_failing_replay_buffer(tmp_path):
  """dqn-test 327-334: no replay files to load -> False."""
  assert _dqn().unbundle(str(tmp_path), 1729, {}) is False


def test_unbundling_with_no_bundle_dictionary(tmp_path):
  """dqn-test 336-340."""
  agent = _dqn()
  agent._replay = mock.Mock()
  assert agent.unbundle(str(tmp_path), 1729, None) is False


def test_partial_unbundling(tmp_path):
  """dqn-test 342-353."""
  agent = _dqn(allow_partial_reload=True)
  agent.state = 'state'
  agent.training_steps = 'training_steps'
  agent.bundle_and_checkpoint(str(tmp_path), 1729)
  assert agent.unbundle(str(tmp_path), 1729, None) is True


def test_bundling(tmp_path):
  """dqn-test 355-368."""
  agent = _dqn()
  agent.state = 'state'
  agent._replay = mock.Mock()
  agent.training_steps = 'training_steps'
  bundle = agent.bundle_and_checkpoint(str(tmp_path), 1729)
  for key in ['state', 'training_steps']:
    assert key in bundle and bundle[key] == key


# ------------------------------------------------------------------- Rainbow
def _rainbow():
  """rb-test 298-339."""
  agent = rainbow_agent.RainbowAgent(
      num_actions=4, num_atoms=5, vmax=7., min_replay_history=32,
      epsilon_fn=lambda w, x, y, z: 0.0, epsilon_eval=0.0, epsilon_decay_period=90,
      network=MockRainbowNetwork, replay_capacity=SMALL)
  agent.eval_mode = True
  return agent


def test_rainbow_shapes_and_values():
  """rb-test 351-368: the support, and the logits / probabilities / Q-values of the
  action-selection and replayed states."""
  agent = _rainbow()
  assert agent._support.shape[0] == 5
  assert float(agent._support.min()) == -7.0 and float(agent._support.max()) == 7.0
  x = torch.zeros((1, STACK) + OBS, device='cuda')
  logits = agent.online_convnet(x)
  assert tuple(logits.shape) == (1, 4, 5)
  assert tuple(torch.softmax(logits, -1).shape) == tuple(logits.shape)
  replay = agent._online_forward(torch.zeros((32, STACK) + OBS, device='cuda'))
  assert tuple(replay.shape[1:]) == (4, 5)
  tgt = agent._target_forward({'next_state': torch.zeros((32, STACK) + OBS, device='cuda')}, 0)
  assert tuple(tgt['logits'].shape[1:]) == (4, 5)
  assert tuple(agent._q_values(agent.state).shape) == (1, 4)


def test_rainbow_begin_episode():
  _begin_episode(_rainbow())


def test_rainbow_step_eval():
  _step_eval(_rainbow())


def test_rainbow_step_train():
  _step_train(_rainbow(), check_args=False)


@pytest.mark.parametrize('scheme,expected', [('uniform', [1., 10., 1.]),
                                             ('prioritized', [1., 10., 10.])])
def test_rainbow_store_transition(scheme, expected):
  """rb-test 477-503: default priorities are 1 (uniform) or the max recorded one."""
  agent = rainbow_agent.RainbowAgent(num_actions=4, replay_scheme=scheme)
  frame = np.zeros((84, 84))
  agent._store_transition(frame, 0, 0, False)
  agent._store_transition(frame, 0, 0, False, 10.)
  agent._store_transition(frame, 0, 0, False)
  got = agent._replay.memory.get_priority(np.arange(STACK - 1, STACK + 2, dtype=np.int32))
  np.testing.assert_array_equal(got, expected)


# ----------------------------------------------------------------------- IQN
def _iqn():
  """iqn-test 39-73."""
  agent = implicit_quantile_agent.ImplicitQuantileAgent(
      num_actions=4, kappa=1.0, num_tau_samples=2, num_tau_prime_samples=3,
      num_quantile_samples=4, network=MockImplicitQuantileNetwork, replay_capacity=SMALL)
  agent.eval_mode = True
  return agent


def _iqn_replay(agent):
  """The loss-time tensors of a replayed batch (the reference's _replay_net_*)."""
  B = agent._replay.batch_size
  z = lambda dt: torch.zeros((B,), dtype=dt, device='cuda')
  t = {'state': torch.zeros((B, STACK) + OBS, device='cuda'),
       'next_state': torch.zeros((B, STACK) + OBS, device='cuda'),
       'action': z(torch.int32), 'reward': z(torch.float32), 'terminal': z(torch.uint8)}
  tgt = agent._target_forward(t, 0)
  qv, grad = agent._online_loss(t, tgt)
  return qv, tgt, grad


def test_iqn_shapes():
  """iqn-test 85-120."""
  agent = _iqn()
  B, A = 32, 4
  assert agent._replay.batch_size == B and agent.num_actions == A
  x = torch.zeros((1, STACK) + OBS, device='cuda')
  qv_act, _ = agent.online_convnet(x, agent.num_quantile_samples)
  assert tuple(qv_act.shape) == (agent.num_quantile_samples, A)
  assert tuple(agent._q_values(agent.state).shape) == (1, A)
  qv, tgt, grad = _iqn_replay(agent)
  assert tuple(qv.shape) == (agent.num_tau_samples * B, A)
  assert tuple(grad.shape) == (agent.num_tau_samples * B, A)
  assert tuple(tgt['tq'].shape) == (agent.num_tau_prime_samples * B, A)
  target_q = tgt['ta'].view(agent.num_quantile_samples, B, A).mean(0)
  assert tuple(target_q.shape) == (B, A)


def test_iqn_q_value_computation():
  """iqn-test 122-146: Q = the mean of K quantile values (= num_actions here) for
  every action, argmax 0, and the replayed target Q-values equal them."""
  agent = _iqn()
  agent.state = np.ones((1,) + OBS + (STACK,))
  q = agent._q_values(agent.state)[0].cpu().numpy()
  np.testing.assert_array_equal(q, np.full(agent.num_actions, 4.0))
  assert int(np.argmax(q)) == 0
  _, tgt, _ = _iqn_replay(agent)
  target_q = tgt['ta'].view(agent.num_quantile_samples, 32, -1).mean(0).cpu().numpy()
  np.testing.assert_array_equal(target_q, np.broadcast_to(q, target_q.shape))


def test_iqn_replay_quantile_value_computation():
  """iqn-test 148-169."""
  agent = _iqn()
  qv, tgt, _ = _iqn_replay(agent)
  B = agent._replay.batch_size
  qv = qv.detach().view(agent.num_tau_samples, B, agent.num_actions).cpu().numpy()
  tq = tgt['tq'].view(agent.num_tau_prime_samples, B, agent.num_actions).cpu().numpy()
  assert (qv[..., 0] == agent.num_actions).all()
  assert (tq[..., 0] == agent.num_actions).all()
