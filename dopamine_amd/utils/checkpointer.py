"""Experiment checkpointer (reference dopamine/utils/checkpointer.py:40-190).

``save_checkpoint(i, data)`` pickles ``data`` to ``<dir>/<prefix>.<i>`` and then
writes the sentinel ``sentinel_<id>_complete.<i>``; the newest iteration with a
sentinel is the one to resume from; files CHECKPOINT_DURATION x frequency
iterations old are removed.  The pickles are this code's own files (load only
checkpoints written by it)."""
import glob
import logging
import os
import pickle

CHECKPOINT_DURATION = 4


def get_latest_checkpoint_number(base_directory, override_number=None,
                                 sentinel_file_identifier='checkpoint'):
  """Largest iteration with a completed checkpoint, or -1 (none, or no such directory);
  ``override_number`` (a gin-bindable override) is returned as is."""
  if override_number is not None:
    return override_number
  pattern = os.path.join(base_directory, 'sentinel_{}_complete.*'.format(sentinel_file_identifier))
  nums = []
  for f in glob.glob(pattern):
    try:
      nums.append(int(f.split('.')[-1]))
    except ValueError:
      continue
  return max(nums) if nums else -1


class Checkpointer(object):

  def __init__(self, base_directory, checkpoint_file_prefix='ckpt',
               sentinel_file_identifier='checkpoint', checkpoint_frequency=1):
    if not base_directory:
      raise ValueError('No path provided to Checkpointer.')
    self._checkpoint_file_prefix = checkpoint_file_prefix
    self._sentinel_file_prefix = 'sentinel_{}_complete'.format(sentinel_file_identifier)
    self._checkpoint_frequency = checkpoint_frequency
    self._base_directory = base_directory
    try:
      os.makedirs(base_directory, exist_ok=True)
    except OSError:
      raise ValueError('Unable to create checkpoint path: {}.'.format(base_directory))

  def _generate_filename(self, file_prefix, iteration_number):
    return os.path.join(self._base_directory, '{}.{}'.format(file_prefix, iteration_number))

  def save_checkpoint(self, iteration_number, data):
    if iteration_number % self._checkpoint_frequency != 0:
      return
    with open(self._generate_filename(self._checkpoint_file_prefix, iteration_number), 'wb') as f:
      pickle.dump(data, f)
    with open(self._generate_filename(self._sentinel_file_prefix, iteration_number), 'w') as f:
      f.write('done')
    self._clean_up_old_checkpoints(iteration_number)

  def _clean_up_old_checkpoints(self, iteration_number):
    stale = iteration_number - self._checkpoint_frequency * CHECKPOINT_DURATION
    if stale >= 0:
      for prefix in (self._checkpoint_file_prefix, self._sentinel_file_prefix):
        try:
          os.remove(self._generate_filename(prefix, stale))
        except FileNotFoundError:
          logging.info('Unable to remove %s.', self._generate_filename(prefix, stale))

  def load_checkpoint(self, iteration_number):
    filename = self._generate_filename(self._checkpoint_file_prefix, iteration_number)
    if not os.path.exists(filename):
      return None
    with open(filename, 'rb') as f:
      return pickle.load(f)
