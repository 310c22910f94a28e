"""BASELINE config 1 end to end on the device: train.py + the CartPole gin
config (through dopamine_amd.gin_lite) drives the Runner, the DQN agent with
float64 (4, 1) observations, logging, checkpointing and resume."""
import os
import pickle

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIN = os.path.join(ROOT, 'dopamine_amd', 'agents', 'dqn', 'configs', 'dqn_cartpole.gin')
SMALL = ['Runner.training_steps = 600', 'Runner.evaluation_steps = 200',
         'DQNAgent.min_replay_history = 300', 'WrappedReplayBuffer.replay_capacity = 5000',
         'WrappedReplayBuffer.batch_size = 32']


def test_cartpole_experiment_runs_logs_checkpoints_and_resumes(tmp_path):
  from dopamine_amd import gin_lite
  from dopamine_amd.discrete_domains import train
  base = str(tmp_path / 'cartpole')
  gin_lite.clear_config()
  runner = train.main(['--base_dir', base, '--gin_files', GIN] +
                      sum([['--gin_bindings', b] for b in SMALL + ['Runner.num_iterations = 2']], []))
  agent = runner._agent
  assert agent.training_steps >= 1200 and agent._replay.memory.add_count > 600
  with open(os.path.join(base, 'logs', 'log_1'), 'rb') as f:
    logs = pickle.load(f)
  it = logs['iteration_1']
  assert it['train_episode_lengths'] and it['eval_episode_lengths']
  assert np.isfinite(it['train_average_return'][0]) and np.isfinite(it['eval_average_return'][0])
  ck = os.path.join(base, 'checkpoints')
  for f in ('ckpt.1', 'sentinel_checkpoint_complete.1', 'tf_ckpt-1',
            '$store$_observation_ckpt.1.gz', 'add_count_ckpt.1.gz'):
    assert os.path.exists(os.path.join(ck, f)), f
  params = agent.online_convnet.fp.flat.detach().cpu().clone()
  steps = agent.training_steps
  # resume: a new Runner picks up at iteration 2 with the saved weights and replay
  gin_lite.clear_config()
  runner2 = train.main(['--base_dir', base, '--gin_files', GIN] +
                       sum([['--gin_bindings', b] for b in SMALL + ['Runner.num_iterations = 2']], []))
  assert runner2._start_iteration == 2
  a2 = runner2._agent
  assert a2.training_steps == steps
  assert np.array_equal(a2.online_convnet.fp.flat.detach().cpu().numpy(), params.numpy())
  assert int(a2._replay.memory.add_count) == int(agent._replay.memory.add_count)
  gin_lite.clear_config()
