"""The reference's replay-buffer unit tests whose checks fire before any device
storage exists, restated against the drop-in's own classes and functions (not the
oracle): circular_replay_buffer_test.py:61-65, 139-166, 452-474, 664-690.  The rest
of those suites run on the device in tests/test_gpu_replay_api.py."""
import numpy as np
import pytest

from dopamine_amd.replay_memory import circular_replay_buffer as crb

OBS = (84, 84)


def test_nontuple_observation_shape():
  """crb-test 61-65."""
  with pytest.raises(AssertionError):
    crb.OutOfGraphReplayBuffer(observation_shape=84, stack_size=4, replay_capacity=5, batch_size=32)


def test_low_capacity():
  """crb-test 139-166 (the raising half; the just-large-enough buffer is built on the
  device in test_gpu_replay_api.py)."""
  with pytest.raises(ValueError, match='There is not enough capacity'):
    crb.OutOfGraphReplayBuffer(OBS, 10, 10, 32, update_horizon=1, gamma=1.0)
  with pytest.raises(ValueError, match='There is not enough capacity'):
    crb.OutOfGraphReplayBuffer(OBS, 5, 10, 32, update_horizon=10, gamma=1.0)


def test_invalid_range():
  """crb-test 452-474 on the module's invalid_range."""
  np.testing.assert_array_equal(crb.invalid_range(6, 10, 4, 1), [5, 6, 7, 8, 9])
  np.testing.assert_array_equal(crb.invalid_range(9, 10, 4, 1), [8, 9, 0, 1, 2])
  np.testing.assert_array_equal(crb.invalid_range(0, 10, 4, 1), [9, 0, 1, 2, 3])
  np.testing.assert_array_equal(crb.invalid_range(6, 10, 4, 3), [3, 4, 5, 6, 7, 8, 9])


def test_wrapper_constructor_errors():
  """crb-test 664-690: the wrapper's argument checks, with the reference's messages."""
  with pytest.raises(ValueError, match=r'Update horizon \(5\) should be significantly '
                                       r'smaller than replay capacity \(5\)\.'):
    crb.WrappedReplayBuffer(observation_shape=OBS, stack_size=4, replay_capacity=5, update_horizon=5)
  with pytest.raises(ValueError, match=r'Update horizon must be positive\.'):
    crb.WrappedReplayBuffer(observation_shape=OBS, stack_size=4, update_horizon=0)
  for gamma in (-1, 1.1):
    with pytest.raises(ValueError, match=r'Discount factor \(gamma\) must be in \[0, 1\]\.'):
      crb.WrappedReplayBuffer(observation_shape=OBS, stack_size=4, gamma=gamma)
