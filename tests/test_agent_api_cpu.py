"""The reference's agent unit tests that need no device, restated against the
drop-in's own functions (not the oracle): rainbow_agent_test.py:31-290
(ProjectDistributionTest: known answers and the error behaviour) on
``dopamine_amd.agents.rainbow.rainbow_agent.project_distribution``, and
dqn_agent_test.py:249-253 (testNonTupleObservationShape).  The agents' behaviour
on the device is restated in tests/test_gpu_agent_api.py.

The reference's ``*WithPlaceholders`` variants feed shapes TF cannot check
statically, so their errors come from ``validate_args``'s runtime assertions
(tf.errors.InvalidArgumentError).  This implementation is eager: every shape is
known at call time, the static checks fire first, and both error kinds are
ValueErrors (rainbow_agent.InvalidArgumentError subclasses ValueError)."""
import numpy as np
import pytest
import torch

from dopamine_amd.agents.dqn import dqn_agent
from dopamine_amd.agents.rainbow import rainbow_agent
from tests.test_oracle_kats import PROJ_KATS

S2 = [[0, 2, 4, 6, 8], [3, 4, 5, 6, 7]]
W2 = [[0.1, 0.2, 0.3, 0.2, 0.2], [0.1, 0.2, 0.3, 0.2, 0.2]]


@pytest.mark.parametrize('sup,w,tgt,exp', PROJ_KATS)
def test_project_distribution_known_answers(sup, w, tgt, exp):
  """rb-test 178-285 (single / batched / non-monotonic supports / larger delta)."""
  for validate in (False, True):
    got = rainbow_agent.project_distribution(sup, w, tgt, validate_args=validate)
    assert isinstance(got, torch.Tensor) and got.dtype == torch.float32
    np.testing.assert_allclose(got.numpy(), exp, atol=1e-6)


def test_project_distribution_takes_tensors():
  """rb-test 261-285 (testUsingPlaceholders): tensor inputs, same answers."""
  sup, w, tgt, exp = PROJ_KATS[4]
  got = rainbow_agent.project_distribution(torch.tensor(sup, dtype=torch.float32),
                                           torch.tensor(w, dtype=torch.float32),
                                           torch.tensor(tgt, dtype=torch.float32))
  np.testing.assert_allclose(got.numpy(), exp, atol=1e-6)


@pytest.mark.parametrize('validate', [False, True])
def test_inconsistent_supports_and_weights(validate):
  """rb-test 33-61."""
  with pytest.raises(ValueError, match='are incompatible'):
    rainbow_agent.project_distribution(S2, [r[:4] for r in W2], [4, 5, 6, 7, 8],
                                       validate_args=validate)


@pytest.mark.parametrize('validate', [False, True])
def test_inconsistent_supports_and_target_support(validate):
  """rb-test 63-90."""
  with pytest.raises(ValueError, match='are incompatible'):
    rainbow_agent.project_distribution(S2, W2, [4, 5, 6], validate_args=validate)


@pytest.mark.parametrize('validate', [False, True])
def test_zero_dimensional_target_support(validate):
  """rb-test 92-118."""
  with pytest.raises(ValueError, match='Index out of range'):
    rainbow_agent.project_distribution(S2, W2, 3, validate_args=validate)


@pytest.mark.parametrize('validate', [False, True])
def test_multi_dimensional_target_support(validate):
  """rb-test 120-146."""
  with pytest.raises(ValueError, match='out of bounds'):
    rainbow_agent.project_distribution(S2, W2, [[3]], validate_args=validate)


def test_non_monotonic_target_support():
  """rb-test 148-160: caught by validate_args, not without it."""
  with pytest.raises(rainbow_agent.InvalidArgumentError, match='assertion failed'):
    rainbow_agent.project_distribution(S2, W2, [8, 7, 6, 5, 4], validate_args=True)
  rainbow_agent.project_distribution(S2, W2, [8, 7, 6, 5, 4])


def test_inconsistent_target_support_deltas():
  """rb-test 162-174."""
  with pytest.raises(rainbow_agent.InvalidArgumentError, match='assertion failed'):
    rainbow_agent.project_distribution(S2, W2, [3, 4, 6, 7, 8], validate_args=True)
  rainbow_agent.project_distribution(S2, W2, [3, 4, 6, 7, 8])


def test_non_tuple_observation_shape():
  """dqn-test 249-253 (abstract_agent.py:34): asserted before anything is built."""
  with pytest.raises(AssertionError):
    dqn_agent.DQNAgent(num_actions=4, observation_shape=84)
  with pytest.raises(AssertionError):
    rainbow_agent.RainbowAgent(num_actions=4, observation_shape=[84, 84])


def test_linearly_decaying_epsilon():
  """dqn-test 297-311 on the agent module's own function."""
  for step, expected in [(0, 1.0), (16, 0.91), (107, 0.1)]:
    assert abs(dqn_agent.linearly_decaying_epsilon(100, step, 6, 0.1) - expected) < 0.01


class _PlaceStub:
  """The attributes DQNAgent._place_riders reads (no device, no replay)."""
  _gather_plan = None
  chunk_gather_launch = 3
  sample_launch = 2

  def __init__(self, fused, at):
    self._f, self.rider_launches = fused, at

  def _fused(self):
    return self._f


def test_per_rider_placement_lists():
  """The PER riders (write-back, sample, gather) of the fused schedule go to backward launches
  rider_launches (rider i of the list rides in launch 1 + i; empty dq_riders in between); the
  plain schedule (target head from launch 3) keeps its launches 0, 1, 2 whatever the knob;
  a gather at or after the target conv1's launch 5 is refused."""
  from dopamine_amd import _lib
  wb, smp, gat = _lib.Rider(), _lib.Rider(), _lib.Rider()
  wb.words[0], smp.words[0], gat.words[0] = 11, 12, 13     # tags only (kind words unread here)
  place = dqn_agent.DQNAgent._place_riders
  tags = lambda rs: [int(r.words[0]) for r in rs]
  assert tags(place(_PlaceStub(True, (2, 3, 4)), [wb, smp, gat])) == [0, 11, 12, 13]
  assert tags(place(_PlaceStub(True, (1, 3, 4)), [wb, smp, gat])) == [11, 0, 12, 13]
  assert tags(place(_PlaceStub(True, (1, 2, 3)), [wb, smp, gat])) == [11, 12, 13]
  assert tags(place(_PlaceStub(True, None), [wb, smp, gat])) == [11, 12, 13]
  assert tags(place(_PlaceStub(False, (2, 3, 4)), [wb, smp, gat])) == [11, 12, 13]
  for bad in ((2, 3, 5), (3, 2, 4), (2, 4, 4), (0, 1, 2), (2, 3)):
    with pytest.raises(ValueError, match='rider_launches'):   # also under python -O
      place(_PlaceStub(True, bad), [wb, smp, gat])
  assert dqn_agent.DQNAgent.rider_launches == (2, 3, 4)
