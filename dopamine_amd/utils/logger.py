"""Experiment logger (reference dopamine/utils/logger.py:29-98): a dict of
per-iteration statistics pickled to ``<dir>/<prefix>_<iteration>``, keeping the
last CHECKPOINT_DURATION files."""
import logging
import os
import pickle

CHECKPOINT_DURATION = 4


class Logger(object):

  def __init__(self, logging_dir):
    self.data = {}
    self._logging_enabled = True
    if not logging_dir:
      logging.info('Logging directory not specified, will not log.')
      self._logging_enabled = False
      return
    try:
      os.makedirs(logging_dir, exist_ok=True)
    except OSError:
      pass
    if not os.path.isdir(logging_dir):
      logging.warning('Could not create directory %s, logging will be disabled.', logging_dir)
      self._logging_enabled = False
      return
    self._logging_dir = logging_dir

  def __setitem__(self, key, value):
    if self._logging_enabled:
      self.data[key] = value

  def _generate_filename(self, filename_prefix, iteration_number):
    return os.path.join(self._logging_dir, '{}_{}'.format(filename_prefix, iteration_number))

  def log_to_file(self, filename_prefix, iteration_number):
    if not self._logging_enabled:
      logging.warning('Logging is disabled.')
      return
    with open(self._generate_filename(filename_prefix, iteration_number), 'wb') as fout:
      pickle.dump(self.data, fout, protocol=pickle.HIGHEST_PROTOCOL)
    stale = iteration_number - CHECKPOINT_DURATION
    if stale >= 0:
      try:
        os.remove(self._generate_filename(filename_prefix, stale))
      except FileNotFoundError:
        pass

  def is_logging_enabled(self):
    return self._logging_enabled
