"""Step lengths by position in the learner loop's 4-step chunk graphs (rocprofv3
--kernel-trace database; steps cut at the anchor kernel): the median length of each step
position and the mean step, so a chunk-boundary cost is not hidden by a median step.
    python tools/step_phases.py run_results.db [anchor] [period]"""
import sqlite3
import statistics
import sys


def main():
  db = sqlite3.connect(sys.argv[1])
  anchor = sys.argv[2] if len(sys.argv) > 2 else 'k_c51'
  period = int(sys.argv[3]) if len(sys.argv) > 3 else 4
  rows = sorted(db.execute('select start, end, name from kernels'))
  starts = [r[0] for r in rows if anchor in r[2]]
  lens = [(b - a) / 1e3 for a, b in zip(starts[:-1], starts[1:])]
  lens = lens[40:-10]
  print('%d steps, mean %.1f us, median %.1f us' % (len(lens), statistics.mean(lens), statistics.median(lens)))
  for p in range(period):
    ph = lens[p::period]
    print('  position %d: median %.1f  mean %.1f  (n=%d)' % (p, statistics.median(ph), statistics.mean(ph), len(ph)))


if __name__ == '__main__':
  main()
