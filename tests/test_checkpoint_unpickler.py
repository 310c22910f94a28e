"""The replay checkpoint unpickler (CPU): the reference's pickled SumTree loads as
its fields; any other class a checkpoint names is refused before it runs."""
import gzip
import io
import os
import pickle

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_reference_sum_tree_pickle_loads_as_fields():
  from dopamine_amd.replay_memory import circular_replay_buffer as crb
  with gzip.open(os.path.join(GOLDEN, 'ckpt_per', 'sum_tree_ckpt.3.gz'), 'rb') as f:
    t = crb._CheckpointUnpickler(f).load()
  assert isinstance(t, crb._ReferenceSumTree)
  exp = np.load(os.path.join(GOLDEN, 'ckpt_per_expected.npz'))
  np.testing.assert_array_equal(np.concatenate(t.nodes), exp['nodes'])
  assert float(t.max_recorded_priority) == float(exp['maxrec'])


class _Evil(object):
  def __reduce__(self):
    return (os.system, ('echo pwned',))


def test_other_classes_are_refused():
  from dopamine_amd.replay_memory import circular_replay_buffer as crb
  with pytest.raises(pickle.UnpicklingError, match='not an allowed type'):
    crb._CheckpointUnpickler(io.BytesIO(pickle.dumps(_Evil()))).load()


@pytest.mark.parametrize('protocol', [0, 1, 2, 4, 5])
def test_every_pickle_protocol_of_a_reference_sum_tree_loads(protocol, monkeypatch):
  """The reference pickles its SumTree with pickle's default protocol (crb:643): 4 under
  Python 3, 0 under Python 2.  Protocols 0 / 1 go through copyreg._reconstructor and 5
  sends numpy arrays through _frombuffer; all load as the tree's fields."""
  import sys
  import types
  from dopamine_amd.replay_memory import circular_replay_buffer as crb
  mod = types.ModuleType('dopamine.replay_memory.sum_tree')

  class SumTree(object):
    pass
  SumTree.__module__, SumTree.__qualname__ = mod.__name__, 'SumTree'
  mod.SumTree = SumTree
  for name in ('dopamine', 'dopamine.replay_memory'):
    monkeypatch.setitem(sys.modules, name, types.ModuleType(name))
  monkeypatch.setitem(sys.modules, mod.__name__, mod)
  t = SumTree()
  t.nodes = [np.array([3.0]), np.array([1.0, 2.0])]
  t.max_recorded_priority = 2.0
  got = crb._CheckpointUnpickler(io.BytesIO(pickle.dumps(t, protocol=protocol))).load()
  assert isinstance(got, crb._ReferenceSumTree)
  np.testing.assert_array_equal(np.concatenate(got.nodes), [3.0, 1.0, 2.0])
  assert got.max_recorded_priority == 2.0


def test_reconstructor_refuses_other_classes():
  import copyreg
  from dopamine_amd.replay_memory import circular_replay_buffer as crb
  data = pickle.dumps(copyreg._reconstructor, protocol=0)
  fn = crb._CheckpointUnpickler(io.BytesIO(data)).load()
  with pytest.raises(pickle.UnpicklingError, match='not an allowed type'):
    fn(dict, object, None)
  with pytest.raises(pickle.UnpicklingError, match='not an allowed type'):
    fn(crb._ReferenceSumTree, dict, None)
