"""Markdown per-kernel summary of a rocprofv3 --kernel-trace CSV of bench.py:
kernels grouped by (name, grid), with calls per gradient step, average and
per-step microseconds.  Grouped launches are named by their ops (trace_ops).
    python tools/profile_summary.py run_kernel_trace.csv STEPS [title]"""
import csv
import sys
from collections import defaultdict

from trace_ops import name_of


def main():
  rows = list(csv.DictReader(open(sys.argv[1])))
  steps = int(sys.argv[2])
  title = sys.argv[3] if len(sys.argv) > 3 else ''
  agg = defaultdict(list)
  for r in rows:
    blocks = (int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X'])) *
              int(r.get('Grid_Size_Y', 1)) * int(r.get('Grid_Size_Z', 1)))
    key = (name_of(r['Kernel_Name']), blocks, int(r['Workgroup_Size_X']))
    agg[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
  if title:
    print('# ' + title + '\n')
  print('%d dispatches, %d timed gradient steps.\n' % (len(rows), steps))
  print('| kernel | blocks x threads | calls | calls/step | avg us | total us |')
  print('|---|---|---|---|---|---|')
  for (n, b, t), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    if sum(d) < 100:
      continue
    print('| `%s` | %d x %d | %d | %.2f | %.2f | %.1f |' % (n[:110], b, t, len(d), len(d) / steps,
                                                        sum(d) / len(d), sum(d)))


if __name__ == '__main__':
  main()
