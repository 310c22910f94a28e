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
