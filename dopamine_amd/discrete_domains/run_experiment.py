"""Experiment runner over the dopamine_amd agents, with the interface and behaviour of
the reference's dopamine/discrete_domains/run_experiment.py:40-560, configured by the
reference's .gin files through ``dopamine_amd.gin_lite``.

What a run does (the reference's semantics):
  * iterations [start, num_iterations): each one a training phase of at least
    ``training_steps`` environment steps and (Runner only) an evaluation phase of at
    least ``evaluation_steps``, whole episodes, the agent's eval_mode set accordingly;
  * an episode ends at game over or after ``max_steps_per_episode`` steps; a terminal
    that is not game over (an Atari life loss) ends the agent's episode and begins a
    new one inside the same game; the agent sees rewards clipped to [-1, 1], the
    statistics the raw returns;
  * after each iteration its statistics go to the Logger ('iteration_<k>'), written
    every ``log_every_n`` iterations, and the agent + runner state is checkpointed;
    a run finds the newest checkpoint in ``<base_dir>/checkpoints`` and resumes after it.

Not here: the TF session / TensorBoard summary writer (``sess``/``summary_writer`` are
accepted and ignored) and Atari environments (ALE/cv2 are not available), so
``create_environment_fn`` must be a gym domain (``gym_lib.create_gym_environment``).
"""
import logging
import os
import sys
import time

import numpy as np

from dopamine_amd import gin_lite
from dopamine_amd.agents import networks
from dopamine_amd.agents.dqn import dqn_agent
from dopamine_amd.agents.implicit_quantile import implicit_quantile_agent
from dopamine_amd.agents.optimizers import AdamOptimizer, RMSPropOptimizer
from dopamine_amd.agents.rainbow import rainbow_agent
from dopamine_amd.discrete_domains import gym_lib  # noqa: F401 -- registers gym refs/constants
from dopamine_amd.utils import checkpointer
from dopamine_amd.utils import iteration_statistics
from dopamine_amd.utils import logger

# what the reference's gin files reference by name
gin_lite.register('dqn_agent.identity_epsilon', dqn_agent.identity_epsilon)
gin_lite.register('dqn_agent.linearly_decaying_epsilon', dqn_agent.linearly_decaying_epsilon)
gin_lite.register('tf.train.AdamOptimizer',
                  lambda: AdamOptimizer(**gin_lite.query('tf.train.AdamOptimizer')))
gin_lite.register('tf.train.RMSPropOptimizer',
                  lambda: RMSPropOptimizer(**gin_lite.query('tf.train.RMSPropOptimizer')))
gin_lite.register('atari_lib.nature_dqn_network', networks.NatureDQNNetwork)
gin_lite.register('atari_lib.rainbow_network', networks.RainbowNetwork)
gin_lite.register('atari_lib.implicit_quantile_network', networks.ImplicitQuantileNetwork)


def _no_atari(*unused_args, **unused_kwargs):
  raise NotImplementedError('Atari environments (ALE) are out of scope for dopamine_amd; '
                            'use gym_lib.create_gym_environment')


gin_lite.register('atari_lib.create_atari_environment', _no_atari)


def load_gin_configs(gin_files, gin_bindings):
  """Parse the gin files, then the extra bindings (run_experiment.py:40-51)."""
  gin_lite.parse_config_files_and_bindings(gin_files, bindings=gin_bindings, skip_unknown=False)


# agent_name -> (module, class name, the replay wrapper class whose bindings it honours);
# the class is looked up when the agent is created, as the reference's create_agent does
_AGENTS = {'dqn': (dqn_agent, 'DQNAgent', 'WrappedReplayBuffer'),
           'rainbow': (rainbow_agent, 'RainbowAgent', 'WrappedPrioritizedReplayBuffer'),
           'implicit_quantile': (implicit_quantile_agent, 'ImplicitQuantileAgent',
                                 'WrappedPrioritizedReplayBuffer')}


def _agent_kwargs(agent_name):
  """Bindings of the agent's class and of the classes it derives from (gin fills a
  base class's unset constructor arguments the same way), plus the replay wrapper's
  replay_capacity / batch_size, which dopamine_amd's agents take directly."""
  module, name, wrapper = _AGENTS[agent_name]
  cls = getattr(module, name)
  kwargs = {}
  if isinstance(cls, type):                      # (not a stand-in callable)
    for klass in reversed(cls.__mro__[:-1]):     # base classes first, the agent last
      kwargs.update(gin_lite.query(klass.__name__))
  for w in ('WrappedReplayBuffer', wrapper):
    bound = gin_lite.query(w)
    kwargs.update({k: bound[k] for k in ('replay_capacity', 'batch_size') if k in bound})
  return cls, kwargs


@gin_lite.configurable('create_agent')
def create_agent(sess, environment, agent_name=None, summary_writer=None, debug_mode=False):
  """The agent named by ``agent_name`` for ``environment`` (run_experiment.py:54-95)."""
  assert agent_name is not None
  if agent_name not in _AGENTS:
    raise ValueError('Unknown agent: {}'.format(agent_name))
  cls, kwargs = _agent_kwargs(agent_name)
  return cls(sess, num_actions=environment.action_space.n,
             summary_writer=summary_writer if debug_mode else None, **kwargs)


@gin_lite.configurable('create_runner')
def create_runner(base_dir, schedule='continuous_train_and_eval'):
  """Runner for 'continuous_train_and_eval', TrainRunner for 'continuous_train'
  (run_experiment.py:99-121)."""
  assert base_dir is not None
  runners = {'continuous_train_and_eval': Runner, 'continuous_train': TrainRunner}
  if schedule not in runners:
    raise ValueError('Unknown schedule: {}'.format(schedule))
  return runners[schedule](base_dir, create_agent)


# Runner settings and their defaults (run_experiment.py:143-153)
_DEFAULTS = (('create_environment_fn', _no_atari), ('checkpoint_file_prefix', 'ckpt'),
             ('logging_file_prefix', 'log'), ('log_every_n', 1), ('num_iterations', 200),
             ('training_steps', 250000), ('evaluation_steps', 125000),
             ('max_steps_per_episode', 27000))


class Runner(object):
  """Runs an agent in an environment for num_iterations train (+ eval) iterations."""

  def __init__(self, base_dir, create_agent_fn, *args, **kwargs):
    """Runner(base_dir, create_agent_fn, create_environment_fn, checkpoint_file_prefix,
    logging_file_prefix, log_every_n, num_iterations, training_steps, evaluation_steps,
    max_steps_per_episode) -- the reference's parameters, positional or by name."""
    assert base_dir is not None
    names = [n for n, _ in _DEFAULTS]
    if len(args) > len(names):
      raise TypeError('Runner takes at most {} positional arguments'.format(2 + len(names)))
    for name, value in zip(names, args):
      if name in kwargs:
        raise TypeError("Runner got multiple values for argument '{}'".format(name))
      kwargs[name] = value
    unknown = sorted(set(kwargs) - set(names))
    if unknown:
      raise TypeError("Runner got an unexpected keyword argument '{}'".format(unknown[0]))
    # precedence: defaults < Runner bindings < the subclass's own (TrainRunner.*) < arguments
    settings = dict(_DEFAULTS)
    for klass in dict.fromkeys((Runner, type(self))):
      settings.update(gin_lite.query(klass.__name__))
    settings.update(kwargs)
    for name, _ in _DEFAULTS:
      if name not in ('create_environment_fn', 'checkpoint_file_prefix'):
        setattr(self, '_' + name, settings[name])
    self._base_dir = base_dir
    self._create_directories()
    self._environment = settings['create_environment_fn']()
    self._sess = None
    self._agent = create_agent_fn(self._sess, self._environment, summary_writer=None)
    self._refuse_exchanging_learners()
    self._initialize_checkpointer_and_maybe_resume(settings['checkpoint_file_prefix'])

  def _refuse_exchanging_learners(self):
    """Data-parallel learners (a DQNAgent family agent with a process group) exchange their
    gradients at EVERY gradient step, so every rank must take the same gradient steps in the
    same order.  The Runner's phases run whole episodes per rank (run_experiment.py:319-383),
    and each rank's episodes, and its replay's add_count gate (dqn_agent.py:418-442), differ,
    so its ranks would take different gradient steps per phase: a waiting rank times out
    (peer exchange) or pairs its collective with another kind (all-reduce).  Data-parallel
    learners train through the learner-only loop (DQNAgent.train_gradient_steps, bench.py);
    the Runner keeps per-rank checkpoints for agents that exchange nothing."""
    if getattr(self._agent, 'exchange', None) is None or self._process_group() is None:
      return
    import torch.distributed as dist
    if dist.get_world_size(self._process_group()) > 1 or getattr(self._agent, '_peer', None):
      raise ValueError('Runner: data-parallel learners (process_group with %d ranks, exchange=%r) '
                       'exchange gradients every gradient step, which whole-episode phases '
                       'cannot keep in step across ranks; train them with '
                       'train_gradient_steps (the learner-only loop)'
                       % (dist.get_world_size(self._process_group()), self._agent.exchange))

  # ------------------------------------------------------------------ setup
  def _create_directories(self):
    self._checkpoint_dir = os.path.join(self._base_dir, 'checkpoints')
    self._logger = logger.Logger(os.path.join(self._base_dir, 'logs'))

  def _runner_checkpoint_dir(self):
    """Where the runner's own ``ckpt.N`` / sentinel files go: the agent's directory for this
    learner (``_rank_dir``: ``checkpoints`` for a single replica as the reference,
    ``checkpoints/rank<r>`` for data-parallel learners, whose runner states -- the agent's
    ``state``, its step counters -- differ per rank).  A learner with a process group (even
    of one rank) therefore resumes only from a rank-directory checkpoint, not from a
    single-process one."""
    if self._process_group() is None:
      return self._checkpoint_dir
    return self._agent._rank_dir(self._checkpoint_dir)

  def _process_group(self):
    """The agent's torch.distributed process group (data-parallel learners), or None."""
    import torch.distributed as dist
    pg = getattr(self._agent, '_pg', None)
    return pg if isinstance(pg, dist.ProcessGroup) else None

  def _initialize_checkpointer_and_maybe_resume(self, checkpoint_file_prefix):
    """Resume after the newest checkpoint that the agent accepts (run_experiment.py:210-249).
    Data-parallel learners agree on the iteration: the newest one EVERY rank completed."""
    self._checkpointer = checkpointer.Checkpointer(self._runner_checkpoint_dir(),
                                                   checkpoint_file_prefix)
    self._start_iteration = 0
    newest = checkpointer.get_latest_checkpoint_number(self._runner_checkpoint_dir())
    pg = self._process_group()
    if (pg is not None and newest < 0 and
        checkpointer.get_latest_checkpoint_number(self._checkpoint_dir) >= 0):
      logging.warning('%s holds a single-process checkpoint; learners in a process group resume '
                      'only from their rank directories (%s), so this run starts afresh',
                      self._checkpoint_dir, self._runner_checkpoint_dir())
    if pg is not None:
      from dopamine_amd import parallel
      newest = parallel.agree_min(newest, pg)
    if newest < 0:
      return
    runner_state = self._checkpointer.load_checkpoint(newest)
    if not self._agent.unbundle(self._checkpoint_dir, newest, runner_state):
      return
    if runner_state is not None:
      assert 'logs' in runner_state and 'current_iteration' in runner_state
      self._logger.data = runner_state['logs']
      self._start_iteration = runner_state['current_iteration'] + 1
    logging.info('Reloaded checkpoint and will start from iteration %d', self._start_iteration)

  # --------------------------------------------------------------- episodes
  def _initialize_episode(self):
    return self._agent.begin_episode(self._environment.reset())

  def _run_one_step(self, action):
    observation, reward, is_terminal, _ = self._environment.step(action)
    return observation, reward, is_terminal

  def _end_episode(self, reward):
    self._agent.end_episode(reward)

  def _run_one_episode(self):
    """(steps, undiscounted return) of one game."""
    steps, episode_return = 0, 0.
    action = self._initialize_episode()
    agent_reward = 0.
    game_over = False
    while not game_over:
      observation, reward, is_terminal = self._run_one_step(action)
      steps += 1
      episode_return += reward
      agent_reward = np.clip(reward, -1, 1)
      game_over = self._environment.game_over or steps == self._max_steps_per_episode
      if game_over:
        continue
      if is_terminal:                  # a life lost: new agent episode, same game
        self._agent.end_episode(agent_reward)
        action = self._agent.begin_episode(observation)
      else:
        action = self._agent.step(agent_reward, observation)
    self._end_episode(agent_reward)
    return steps, episode_return

  def _run_one_phase(self, min_steps, statistics, run_mode_str):
    """Whole episodes until at least min_steps steps: (steps, sum of returns, episodes)."""
    lengths, returns = [], []
    while sum(lengths) < min_steps:
      length, ret = self._run_one_episode()
      lengths.append(length)
      returns.append(ret)
      statistics.append({run_mode_str + '_episode_lengths': length,
                         run_mode_str + '_episode_returns': ret})
      sys.stdout.write('Steps executed: {} Episode length: {} Return: {}\r'.format(
          sum(lengths), length, ret))
      sys.stdout.flush()
    return sum(lengths), float(sum(returns)), len(returns)

  def _phase(self, statistics, run_mode_str, min_steps, eval_mode):
    self._agent.eval_mode = eval_mode
    t0 = time.time()
    steps, total, episodes = self._run_one_phase(min_steps, statistics, run_mode_str)
    average = total / episodes if episodes else 0.0
    statistics.append({run_mode_str + '_average_return': average})
    logging.info('Average undiscounted return per %s episode: %.2f',
                 'training' if run_mode_str == 'train' else 'evaluation', average)
    if not eval_mode:
      logging.info('Average training steps per second: %.2f', steps / (time.time() - t0))
    return episodes, average

  def _run_train_phase(self, statistics):
    return self._phase(statistics, 'train', self._training_steps, eval_mode=False)

  def _run_eval_phase(self, statistics):
    return self._phase(statistics, 'eval', self._evaluation_steps, eval_mode=True)

  # ------------------------------------------------------------- iterations
  def _run_one_iteration(self, iteration):
    statistics = iteration_statistics.IterationStatistics()
    logging.info('Starting iteration %d', iteration)
    self._run_train_phase(statistics)
    self._run_eval_phase(statistics)
    return statistics.data_lists

  def _log_experiment(self, iteration, statistics):
    self._logger['iteration_{:d}'.format(iteration)] = statistics
    # data-parallel learners: group rank 0 writes the shared log files (every rank keeps its
    # statistics in its own runner checkpoint)
    pg = self._process_group()
    if pg is not None:
      import torch.distributed as dist
      if dist.get_rank(pg) != 0:
        return
    if iteration % self._log_every_n == 0:
      self._logger.log_to_file(self._logging_file_prefix, iteration)

  def _checkpoint_experiment(self, iteration):
    state = self._agent.bundle_and_checkpoint(self._checkpoint_dir, iteration)
    if not state:
      return
    state.update(current_iteration=iteration, logs=self._logger.data)
    self._checkpointer.save_checkpoint(iteration, state)

  def run_experiment(self):
    logging.info('Beginning training...')
    if self._start_iteration >= self._num_iterations:
      logging.warning('num_iterations (%d) < start_iteration(%d)', self._num_iterations,
                      self._start_iteration)
      return
    for iteration in range(self._start_iteration, self._num_iterations):
      statistics = self._run_one_iteration(iteration)
      self._log_experiment(iteration, statistics)
      self._checkpoint_experiment(iteration)
    # the learner's device resources (communicators, peer mappings; a no-op for one replica)
    close = getattr(self._agent, 'close', None)
    if close is not None:
      close()


class TrainRunner(Runner):
  """Training phases only, no evaluation (run_experiment.py:493-560)."""

  def _run_one_iteration(self, iteration):
    statistics = iteration_statistics.IterationStatistics()
    self._run_train_phase(statistics)
    return statistics.data_lists
