"""Per-iteration statistics log of an experiment, with the behaviour of the
reference's dopamine/utils/logger.py:29-105: statistics are collected in ``data``
(keyed 'iteration_<k>' by the Runner), and each logged iteration writes the whole dict,
pickled, to ``<logging_dir>/<prefix>_<k>``; files older than CHECKPOINT_DURATION
iterations are deleted.  A missing or uncreatable directory disables logging (with the
reference's messages) instead of raising.
"""
import logging
import os
import pathlib
import pickle

CHECKPOINT_DURATION = 4


def _usable_dir(logging_dir):
  """The directory as a Path, created if needed; None when logging must be off."""
  if not logging_dir:
    logging.info('Logging directory not specified, will not log.')
    return None
  path = pathlib.Path(logging_dir)
  try:
    path.mkdir(parents=True, exist_ok=True)
  except OSError:
    pass
  if path.is_dir():
    return path
  logging.warning('Could not create directory %s, logging will be disabled.', logging_dir)
  return None


class Logger(object):
  """Dict of statistics written to disk once per logged iteration."""

  def __init__(self, logging_dir):
    self.data = {}
    self._dir = _usable_dir(logging_dir)
    self._logging_enabled = self._dir is not None
    self._logging_dir = str(self._dir) if self._dir is not None else None

  def __setitem__(self, key, value):
    if self._logging_enabled:
      self.data[key] = value

  def _generate_filename(self, filename_prefix, iteration_number):
    return str(self._dir / '{}_{}'.format(filename_prefix, iteration_number))

  def log_to_file(self, filename_prefix, iteration_number):
    """Pickle ``data`` for this iteration (written to a temporary name, then renamed,
    so a reader never sees a partial file) and drop the expired one."""
    if not self._logging_enabled:
      logging.warning('Logging is disabled.')
      return
    target = self._generate_filename(filename_prefix, iteration_number)
    partial = target + '.partial'
    with open(partial, 'wb') as fout:
      pickle.dump(self.data, fout, protocol=pickle.HIGHEST_PROTOCOL)
    os.replace(partial, target)
    expired = iteration_number - CHECKPOINT_DURATION
    if expired >= 0:
      pathlib.Path(self._generate_filename(filename_prefix, expired)).unlink(missing_ok=True)

  def is_logging_enabled(self):
    return self._logging_enabled
