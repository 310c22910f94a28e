"""Per-kernel summary of a rocprofv3 results database (--kernel-trace).

Groups dispatches by (demangled-ish kernel name, grid), prints count, average
and total duration.   python tools/prof_summary.py gpurun_out/prof/run_results.db [N]
"""
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
  name = re.sub(r'dq::cnn::|dq::|\(anonymous namespace\)::', '', name)
  name = name.replace('void ', '')
  return name[:110]


def main():
  db = sqlite3.connect(sys.argv[1])
  top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
  agg = defaultdict(list)
  for name, gx, gy, gz, wx, dur in db.execute(
      'select name, grid_x, grid_y, grid_z, workgroup_x, duration from kernels'):
    agg[(short(name), (gx // max(wx, 1), gy, gz))].append(dur)
  rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
  print('%6s %9s %10s  %-18s %s' % ('count', 'avg_us', 'total_us', 'blocks', 'kernel'))
  for (name, grid), d in rows[:top]:
    print('%6d %9.2f %10.1f  %-18s %s' % (len(d), sum(d) / len(d) / 1e3, sum(d) / 1e3,
                                          '%dx%dx%d' % grid, name))


if __name__ == '__main__':
  main()
