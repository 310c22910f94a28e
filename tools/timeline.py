"""Median per-step timeline from a rocprofv3 --kernel-trace CSV: steps are cut
at each launch of the anchor kernel (default k_adam, the last launch of a
step); every kernel of a step is printed with its median start offset,
duration and queue, in start order.
    python tools/timeline.py run_kernel_trace.csv [anchor] [skip_steps]"""
import csv
import statistics
import sys

from trace_ops import name_of


def main():
  rows = list(csv.DictReader(open(sys.argv[1])))
  anchor = sys.argv[2] if len(sys.argv) > 2 else 'k_adam'
  skip = int(sys.argv[3]) if len(sys.argv) > 3 else 20
  qkey = next((k for k in ('Queue_Id', 'Stream_Id', 'Queue_ID') if k in rows[0]), None)
  ev = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), name_of(r['Kernel_Name']),
                r.get(qkey, '?')) for r in rows))
  cuts = [i for i, e in enumerate(ev) if e[2].startswith(anchor)]
  steps = []
  for a, b in zip(cuts[skip:-1], cuts[skip + 1:]):
    t0 = ev[a][1]                       # step starts when the previous Adam ends
    steps.append([(s - t0, e - s, n, q) for s, e, n, q in ev[a + 1:b + 1]])
  if not steps:
    sys.exit('no complete steps')
  n = len(steps[0])
  steps = [s for s in steps if len(s) == n]
  print('%d steps of %d kernels; median step %.1f us (Adam end to Adam end)' % (
      len(steps), n, statistics.median(s[-1][0] + s[-1][1] for s in steps) / 1e3))
  print('%8s %8s %8s  %-6s %s' % ('start', 'dur', 'end', 'queue', 'kernel'))
  for j in range(n):
    st = statistics.median(s[j][0] for s in steps) / 1e3
    du = statistics.median(s[j][1] for s in steps) / 1e3
    print('%8.1f %8.1f %8.1f  %-6s %s' % (st, du, st + du, steps[0][j][3], steps[0][j][2][:100]))


if __name__ == '__main__':
  main()
