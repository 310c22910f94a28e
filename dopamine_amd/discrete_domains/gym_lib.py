"""Gym-domain plumbing for BASELINE config 1 (reference dopamine/discrete_domains/gym_lib.py).

``gym`` is not installed (third-party, not vendored by the reference), so
CartPole-v0 is restated here from gym's published classic-control model
(gym/envs/classic_control/cartpole.py, the version Dopamine 2.0 used): Euler
integration, tau 0.02 s, force 10 N, masses 1.0 / 0.1 kg, pole half-length
0.5 m; the episode ends when |x| > 2.4 or |theta| > 12 degrees; reward 1 per
step; reset draws the 4 state variables from U(-0.05, 0.05).  As in
``create_gym_environment`` (gym_lib.py:54-72) there is no TimeLimit wrapper: the
Runner's ``max_steps_per_episode`` caps episodes.
"""
import math

import numpy as np

from dopamine_amd import gin_lite
from dopamine_amd.agents import networks

CARTPOLE_MIN_VALS = networks.CartpoleDQNNetwork.MIN
CARTPOLE_MAX_VALS = networks.CartpoleDQNNetwork.MAX
CARTPOLE_OBSERVATION_SHAPE = (4, 1)
CARTPOLE_OBSERVATION_DTYPE = np.float64
CARTPOLE_STACK_SIZE = 1
for _n in ('CARTPOLE_OBSERVATION_SHAPE', 'CARTPOLE_OBSERVATION_DTYPE', 'CARTPOLE_STACK_SIZE'):
  gin_lite.constant('gym_lib.' + _n, globals()[_n])

# the network the gin file binds with @gym_lib.cartpole_dqn_network (gym_lib.py:113-132)
cartpole_dqn_network = gin_lite.register('gym_lib.cartpole_dqn_network',
                                         networks.CartpoleDQNNetwork)


class Discrete(object):
  def __init__(self, n):
    self.n = n

  def sample(self, rng=np.random):
    return int(rng.randint(self.n))


class Box(object):
  def __init__(self, low, high, dtype=np.float64):
    self.low, self.high, self.dtype = np.asarray(low), np.asarray(high), dtype
    self.shape = self.low.shape


class CartPoleEnv(object):
  """CartPole-v0 dynamics (gym classic control, Euler integrator)."""

  gravity = 9.8
  masscart = 1.0
  masspole = 0.1
  total_mass = masspole + masscart
  length = 0.5                          # half the pole's length
  polemass_length = masspole * length
  force_mag = 10.0
  tau = 0.02
  theta_threshold_radians = 12 * 2 * math.pi / 360
  x_threshold = 2.4

  def __init__(self, seed=None):
    high = np.array([self.x_threshold * 2, np.finfo(np.float32).max,
                     self.theta_threshold_radians * 2, np.finfo(np.float32).max])
    self.action_space = Discrete(2)
    self.observation_space = Box(-high, high)
    self.reward_range = (-float('inf'), float('inf'))
    self.metadata = {'render.modes': []}
    self.np_random = np.random.RandomState(seed)
    self.state = None
    self.steps_beyond_done = None

  def seed(self, seed=None):
    self.np_random = np.random.RandomState(seed)
    return [seed]

  def reset(self):
    self.state = self.np_random.uniform(low=-0.05, high=0.05, size=(4,))
    self.steps_beyond_done = None
    return np.array(self.state)

  def step(self, action):
    assert action in (0, 1), '%r invalid' % (action,)
    x, x_dot, theta, theta_dot = self.state
    force = self.force_mag if action == 1 else -self.force_mag
    costheta, sintheta = math.cos(theta), math.sin(theta)
    temp = (force + self.polemass_length * theta_dot * theta_dot * sintheta) / self.total_mass
    thetaacc = (self.gravity * sintheta - costheta * temp) / (
        self.length * (4.0 / 3.0 - self.masspole * costheta * costheta / self.total_mass))
    xacc = temp - self.polemass_length * thetaacc * costheta / self.total_mass
    x = x + self.tau * x_dot
    x_dot = x_dot + self.tau * xacc
    theta = theta + self.tau * theta_dot
    theta_dot = theta_dot + self.tau * thetaacc
    self.state = (x, x_dot, theta, theta_dot)
    done = bool(x < -self.x_threshold or x > self.x_threshold or
                theta < -self.theta_threshold_radians or theta > self.theta_threshold_radians)
    if not done:
      reward = 1.0
    elif self.steps_beyond_done is None:   # the pole just fell
      self.steps_beyond_done = 0
      reward = 1.0
    else:
      self.steps_beyond_done += 1
      reward = 0.0
    return np.array(self.state), reward, done, {}


_ENVS = {'CartPole-v0': CartPoleEnv}


@gin_lite.configurable('create_gym_environment')
def create_gym_environment(environment_name=None, version='v0'):
  """gym_lib.py:54-72."""
  assert environment_name is not None
  full_game_name = '{}-{}'.format(environment_name, version)
  if full_game_name not in _ENVS:
    raise ValueError('dopamine_amd provides {} (no gym here); got {}'.format(
        sorted(_ENVS), full_game_name))
  return GymPreprocessing(_ENVS[full_game_name]())


gin_lite.register('gym_lib.create_gym_environment', create_gym_environment)


class GymPreprocessing(object):
  """gym_lib.py:321-372: the Dopamine-facing wrapper (tracks game_over)."""

  def __init__(self, environment, render=False):
    self.environment = environment
    self.game_over = False
    self.render = render

  @property
  def observation_space(self):
    return self.environment.observation_space

  @property
  def action_space(self):
    return self.environment.action_space

  @property
  def reward_range(self):
    return self.environment.reward_range

  @property
  def metadata(self):
    return self.environment.metadata

  def reset(self):
    return self.environment.reset()

  def step(self, action):
    observation, reward, game_over, info = self.environment.step(action)
    self.game_over = game_over
    return observation, reward, game_over, info
