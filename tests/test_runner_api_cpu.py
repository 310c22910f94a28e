"""The reference's runner-side unit tests (the plumbing around the
hot path) restated against dopamine_amd's own modules: run_experiment_test.py:95-437
(mock agent and environment), checkpointer_test.py:36-150, logger_test.py:38-110,
iteration_statistics_test.py:28-69 and gym_lib_test.py:29-51.

Deviations: gin is ``dopamine_amd.gin_lite``; paths the reference expects to be
uncreatable ('/does/not/exist', which a root process CAN create) are a path under a
regular file here; there is no TF summary writer, so testRunExperiment's tfevents
glob is not restated."""
import os
import pickle
from unittest import mock

import pytest

from dopamine_amd import gin_lite
from dopamine_amd.agents.dqn import dqn_agent
from dopamine_amd.agents.implicit_quantile import implicit_quantile_agent
from dopamine_amd.agents.rainbow import rainbow_agent
from dopamine_amd.discrete_domains import gym_lib
from dopamine_amd.discrete_domains import run_experiment
from dopamine_amd.utils import checkpointer
from dopamine_amd.utils import iteration_statistics
from dopamine_amd.utils import logger

DATA = {'data1': 1, 'data2': 'two', 'data3': (3, 'three')}


def _uncreatable(tmp_path):
  blocker = tmp_path / 'a_file'
  blocker.write_text('x')
  return str(blocker / 'sub')


# ------------------------------------------------------------------ checkpointer
def test_checkpointer_initialization(tmp_path):
  """ckpt-test 36-52."""
  with pytest.raises(ValueError, match='No path provided to Checkpointer.'):
    checkpointer.Checkpointer('')
  bad = _uncreatable(tmp_path)
  with pytest.raises(ValueError, match='Unable to create checkpoint path: {}.'.format(bad)):
    checkpointer.Checkpointer(bad)
  checkpointer.Checkpointer(str(tmp_path / 'ok'))
  assert os.path.isdir(str(tmp_path / 'ok'))
  checkpointer.Checkpointer(str(tmp_path / 'ok'))


@pytest.mark.parametrize('prefix', [None, 'custom_prefix'])
def test_checkpointer_round_trip(tmp_path, prefix):
  """ckpt-test 54-76."""
  kw = {} if prefix is None else {'checkpoint_file_prefix': prefix}
  c = checkpointer.Checkpointer(str(tmp_path), **kw)
  c.save_checkpoint(1729, DATA)
  assert c.load_checkpoint(1729) == DATA
  assert c.load_checkpoint(1730) is None


def test_latest_checkpoint_number(tmp_path):
  """ckpt-test 78-101."""
  assert checkpointer.get_latest_checkpoint_number(_uncreatable(tmp_path)) == -1
  assert checkpointer.get_latest_checkpoint_number(str(tmp_path)) == -1
  assert checkpointer.get_latest_checkpoint_number('/ignored', override_number=1729) == 1729
  c = checkpointer.Checkpointer(str(tmp_path))
  c.save_checkpoint(1729, 1729)
  c.save_checkpoint(1730, 1730)
  assert checkpointer.get_latest_checkpoint_number(str(tmp_path)) == 1730


@pytest.mark.parametrize('frequency', [1, 3])
def test_checkpointer_garbage_collection(tmp_path, frequency):
  """ckpt-test 103-150: CHECKPOINT_DURATION checkpoints kept, every frequency-th saved."""
  c = checkpointer.Checkpointer(str(tmp_path), checkpoint_file_prefix='custom_prefix',
                                checkpoint_frequency=frequency)
  deleted = 7 if frequency == 1 else 6
  total = checkpointer.CHECKPOINT_DURATION * frequency + deleted + (0 if frequency == 1 else 1)
  for i in range(total):
    c.save_checkpoint(i, DATA)
  for i in range(total):
    for prefix in ('custom_prefix', 'sentinel_checkpoint_complete'):
      exists = os.path.exists(os.path.join(str(tmp_path), '{}.{}'.format(prefix, i)))
      if frequency == 1:
        assert exists == (i >= deleted), (prefix, i)
      else:
        assert exists == (i > deleted and i % frequency == 0), (prefix, i)


# ------------------------------------------------------------------------ logger
def test_logger_enabled_only_with_a_usable_directory(tmp_path):
  """logger-test 38-48, 69-72."""
  assert not logger.Logger('').is_logging_enabled()
  bad = logger.Logger(_uncreatable(tmp_path))
  assert not bad.is_logging_enabled()
  bad.log_to_file(None, None)
  assert logger.Logger(str(tmp_path)).is_logging_enabled()


def test_logger_set_entry(tmp_path):
  """logger-test 50-67."""
  lg = logger.Logger(str(tmp_path))
  assert len(lg.data) == 0
  lg['key'] = [1, 2, 3, 4]
  assert lg.data == {'key': [1, 2, 3, 4]}
  lg['key'] = 'new value'
  assert lg.data == {'key': 'new value'}


def test_logger_file_contents(tmp_path):
  """logger-test 74-89: the file holds the dict pickled with HIGHEST_PROTOCOL."""
  lg = logger.Logger(str(tmp_path))
  lg['key'] = [1, 2, 3, 4]
  lg.log_to_file('log', 7)
  with open(os.path.join(str(tmp_path), 'log_7'), 'rb') as f:
    assert f.read() == pickle.dumps({'key': [1, 2, 3, 4]}, protocol=pickle.HIGHEST_PROTOCOL)


def test_logger_garbage_collection(tmp_path):
  """logger-test 91-110."""
  lg = logger.Logger(str(tmp_path))
  lg['key'] = [1, 2, 3, 4]
  deleted = 7
  total = logger.CHECKPOINT_DURATION + deleted
  for i in range(total):
    lg.log_to_file('log', i)
  for i in range(total):
    assert os.path.exists(os.path.join(str(tmp_path), 'log_{}'.format(i))) == (i >= deleted)


# ---------------------------------------------------------- iteration statistics
def test_iteration_statistics():
  """itstats-test 28-69."""
  s = iteration_statistics.IterationStatistics()
  with pytest.raises(KeyError):
    _ = s.data_lists['missing_key']
  assert len(s.data_lists) == 0
  s.append({'key1': 0})
  assert s.data_lists == {'key1': [0]}
  s = iteration_statistics.IterationStatistics()
  s.append({'rewards': 0, 'nouns': 'reinforcement', 'angles': 3.14159})
  s.append({'nouns': 'learning'})
  assert s.data_lists == {'rewards': [0], 'nouns': ['reinforcement', 'learning'],
                          'angles': [3.14159]}


# ----------------------------------------------------------------------- gym_lib
class MockGymEnvironment(object):

  def __init__(self):
    self.observation_space = 'observation_space'
    self.action_space = 'action_space'
    self.reward_range = 'reward_range'
    self.metadata = 'metadata'

  def reset(self):
    return 'reset'

  def step(self, unused_action):
    return 'obs', 'rew', 'game_over', 'info'


def test_gym_preprocessing_passes_through():
  """gym_lib-test 29-51."""
  env = gym_lib.GymPreprocessing(MockGymEnvironment())
  assert env.observation_space == 'observation_space'
  assert env.action_space == 'action_space'
  assert env.reward_range == 'reward_range'
  assert env.metadata == 'metadata'
  assert env.reset() == 'reset'
  assert list(env.step(0)) == ['obs', 'rew', 'game_over', 'info']


# ---------------------------------------------------------------- run_experiment
class MockEnvironment(object):
  """re-test 46-70: observation counts steps; reward = +-observation by action."""

  def __init__(self, max_steps=10):
    self._observation = 0
    self.max_steps = max_steps
    self.game_over = False

  def reset(self):
    self._observation = 0
    return self._observation

  def step(self, action):
    self._observation += 1
    reward = self._observation * (-1 if action > 0 else 1)
    is_terminal = self._observation >= self.max_steps
    self.game_over = is_terminal
    return self._observation, reward, is_terminal, 0


class MockLogger(object):
  """re-test 73-96."""

  def __init__(self, run_asserts=True, data=None):
    self._run_asserts = run_asserts
    self._iter = 0
    self._calls_to_set = 0
    self._calls_to_log = 0
    self.data = data

  def __setitem__(self, key, val):
    if self._run_asserts:
      assert key == 'iteration_{:d}'.format(self._iter) and val == 'statistics'
      self._iter += 1
    self._calls_to_set += 1

  def log_to_file(self, filename_prefix, iteration_number):
    if self._run_asserts:
      assert '{}_{}'.format(filename_prefix, iteration_number) == 'prefix_{}'.format(self._iter - 1)
    self._calls_to_log += 1


def test_load_gin_configs():
  """re-test 101-110."""
  with mock.patch.object(gin_lite, 'parse_config_files_and_bindings') as parse:
    run_experiment.load_gin_configs(['file1', 'file2', 'file3'], ['binding1', 'binding2'])
  assert parse.call_count == 1
  args, kwargs = parse.call_args
  assert args[0] == ['file1', 'file2', 'file3']
  assert kwargs['bindings'] == ['binding1', 'binding2']
  assert kwargs['skip_unknown'] is False


def test_create_agent():
  """re-test 112-152: no agent name, and each agent class receiving num_actions."""
  with pytest.raises(AssertionError):
    run_experiment.create_agent(None, mock.Mock())
  for module, cls, name in ((dqn_agent, 'DQNAgent', 'dqn'),
                            (rainbow_agent, 'RainbowAgent', 'rainbow'),
                            (implicit_quantile_agent, 'ImplicitQuantileAgent',
                             'implicit_quantile')):
    with mock.patch.object(module, cls) as agent_cls:
      agent_cls.side_effect = lambda unused_sess, num_actions, summary_writer: num_actions * 10
      env = mock.Mock()
      env.action_space.n = 7
      assert run_experiment.create_agent(None, env, agent_name=name) == 70


def test_create_runner():
  """re-test 154-183."""
  with pytest.raises(ValueError, match='Unknown schedule'):
    run_experiment.create_runner('/tmp', 'Unknown schedule')
  for cls, schedule in (('Runner', None), ('TrainRunner', 'continuous_train')):
    with mock.patch.object(run_experiment, 'create_agent') as create, \
         mock.patch.object(run_experiment, cls) as runner:
      if schedule is None:
        run_experiment.create_runner('/tmp')
      else:
        run_experiment.create_runner('/tmp', schedule=schedule)
      assert runner.call_count == 1
      args, _ = runner.call_args
      assert args[0] == '/tmp' and args[1] is create


class _Agent(object):
  """re-test 188-201: a mock agent whose step checks the clipped reward."""

  def __init__(self):
    self.agent = mock.Mock()
    self.agent.begin_episode.side_effect = lambda x: 0
    self.agent.step.side_effect = self._step

  @staticmethod
  def _step(reward, observation):
    assert reward == (1 if observation % 2 else -1)
    return observation % 2

  def create(self, unused_sess, unused_env, summary_writer):
    return self.agent


def test_resume_when_unbundle_fails(tmp_path):
  """re-test 212-239."""
  ck = mock.Mock()
  ck.load_checkpoint.return_value = {'current_iteration': 1729, 'logs': 'logs'}
  agent = mock.Mock()
  agent.unbundle.return_value = False
  with mock.patch.object(checkpointer, 'get_latest_checkpoint_number', return_value=7), \
       mock.patch.object(checkpointer, 'Checkpointer', return_value=ck), \
       mock.patch.object(logger, 'Logger', return_value=mock.Mock()):
    runner = run_experiment.Runner(str(tmp_path), lambda x, y, summary_writer: agent, mock.Mock)
  assert runner._start_iteration == 0
  assert ck.load_checkpoint.call_count == 1 and agent.unbundle.call_count == 1
  args, _ = agent.unbundle.call_args
  assert args[0] == '{}/checkpoints'.format(str(tmp_path)) and args[1] == 7
  assert args[2] == {'current_iteration': 1729, 'logs': 'logs'}


def test_resume_when_unbundle_succeeds(tmp_path):
  """re-test 241-262."""
  data = {'current_iteration': 1729, 'logs': {'a': 1, 'b': 2}}
  ckdir = os.path.join(str(tmp_path), 'checkpoints')
  checkpointer.Checkpointer(ckdir, 'ckpt').save_checkpoint(7, data)
  agent = mock.Mock()
  agent.unbundle.return_value = True
  with mock.patch.object(checkpointer, 'get_latest_checkpoint_number', return_value=7):
    runner = run_experiment.Runner(str(tmp_path), lambda x, y, summary_writer: agent, mock.Mock)
  assert runner._start_iteration == 1730
  assert runner._logger.data == {'a': 1, 'b': 2}
  agent.unbundle.assert_called_once_with(ckdir, 7, data)


@pytest.mark.parametrize('max_steps,steps,ret', [(11, 10, -5), (2, 2, -1)])
def test_run_one_episode(tmp_path, max_steps, steps, ret):
  """re-test 264-288: sum_{i<10} (-1)^i i = -5; cut at 2 steps: 1 - 2 = -1."""
  a, env = _Agent(), MockEnvironment()
  runner = run_experiment.Runner(str(tmp_path), a.create, lambda: env,
                                 max_steps_per_episode=max_steps)
  assert runner._run_one_episode() == (steps, ret)
  assert a.agent.step.call_count == steps - 1
  assert a.agent.end_episode.call_count == 1


def test_run_one_phase(tmp_path):
  """re-test 290-315."""
  a, env = _Agent(), MockEnvironment(max_steps=2)
  runner = run_experiment.Runner(str(tmp_path), a.create, lambda: env)
  statistics = []
  steps, returns, episodes = runner._run_one_phase(10, statistics, 'test')
  assert a.agent.step.call_count == 5 and a.agent.end_episode.call_count == 5
  assert (steps, returns, episodes) == (10, -5, 5)
  assert statistics == [{'test_episode_lengths': 2, 'test_episode_returns': -1}] * 5


def test_run_one_iteration(tmp_path):
  """re-test 317-336."""
  a, env = _Agent(), MockEnvironment(max_steps=2)
  runner = run_experiment.Runner(str(tmp_path), a.create, lambda: env, training_steps=20,
                                 evaluation_steps=10)
  assert runner._run_one_iteration(1) == {
      'train_episode_lengths': [2] * 10, 'train_episode_returns': [-1] * 10,
      'train_average_return': [-1], 'eval_episode_lengths': [2] * 5,
      'eval_episode_returns': [-1] * 5, 'eval_average_return': [-1]}


def test_log_experiment(tmp_path):
  """re-test 338-354: every iteration stored, every log_every_n-th written."""
  ml = MockLogger()
  with mock.patch.object(logger, 'Logger', return_value=ml):
    runner = run_experiment.Runner(str(tmp_path), _Agent().create, mock.Mock,
                                   logging_file_prefix='prefix', log_every_n=2)
  for i in range(10):
    runner._log_experiment(i, 'statistics')
  assert ml._calls_to_set == 10 and ml._calls_to_log == 5


def test_checkpoint_experiment(tmp_path):
  """re-test 356-381."""
  ckdir = os.path.join(str(tmp_path), 'checkpoints')
  a = _Agent()

  def bundle(x, y):
    assert (x, y) == (ckdir, 1729)
    return {'test': 1}
  a.agent.bundle_and_checkpoint.side_effect = bundle
  ck = mock.Mock()
  with mock.patch.object(checkpointer, 'Checkpointer', return_value=ck), \
       mock.patch.object(logger, 'Logger', return_value=MockLogger(False, {'one': 1, 'two': 2})):
    runner = run_experiment.Runner(str(tmp_path), a.create, mock.Mock)
  runner._checkpoint_experiment(1729)
  assert ck.save_checkpoint.call_count == 1
  args, _ = ck.save_checkpoint.call_args
  assert args[0] == 1729
  assert args[1] == {'test': 1, 'logs': {'one': 1, 'two': 2}, 'current_iteration': 1729}


def test_run_experiment_with_inconsistent_range(tmp_path):
  """re-test 383-397."""
  ml, ck = MockLogger(), mock.Mock()
  with mock.patch.object(checkpointer, 'Checkpointer', return_value=ck), \
       mock.patch.object(logger, 'Logger', return_value=ml):
    runner = run_experiment.Runner(str(tmp_path), _Agent().create, mock.Mock, num_iterations=0)
  runner.run_experiment()
  assert ck.save_checkpoint.call_count == 0
  assert ml._calls_to_set == 0 and ml._calls_to_log == 0


def test_run_experiment_resumes(tmp_path):
  """re-test 399-433."""
  env, a = MockEnvironment(), _Agent()
  ml, ck = MockLogger(run_asserts=False), mock.Mock()
  ck.load_checkpoint.side_effect = lambda _: {'logs': 'log_data', 'current_iteration': 1728}
  a.agent.bundle_and_checkpoint.side_effect = lambda x, y: {'test': 1}
  a.agent.unbundle.return_value = True
  with mock.patch.object(checkpointer, 'get_latest_checkpoint_number', return_value=1729), \
       mock.patch.object(checkpointer, 'Checkpointer', return_value=ck), \
       mock.patch.object(logger, 'Logger', return_value=ml):
    runner = run_experiment.Runner(str(tmp_path), a.create, lambda: env, log_every_n=1,
                                   num_iterations=1739, training_steps=1, evaluation_steps=1)
  assert runner._start_iteration == 1729
  runner.run_experiment()
  assert ck.save_checkpoint.call_count == 10
  assert ml._calls_to_set == 10 and ml._calls_to_log == 10


def test_runner_signature():
  """Runner's arguments are the reference's (run_experiment.py:127-153): positional after
  create_agent_fn, by name, no duplicates, no unknown names."""
  with pytest.raises(TypeError, match='multiple values'):
    run_experiment.Runner('/tmp', None, mock.Mock, create_environment_fn=mock.Mock)
  with pytest.raises(TypeError, match='unexpected keyword'):
    run_experiment.Runner('/tmp', None, no_such_setting=1)
