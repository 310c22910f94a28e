"""Per-iteration metric lists (reference dopamine/utils/iteration_statistics.py:23-52)."""


class IterationStatistics(object):

  def __init__(self):
    self.data_lists = {}

  def append(self, data_pairs):
    """Appends each value to the list kept under its key."""
    for key, value in data_pairs.items():
      self.data_lists.setdefault(key, []).append(value)
