"""Per-step idle gaps of a rocprofv3 --kernel-trace database: for consecutive steps (cut at
an anchor kernel), the gap before each kernel on its queue and the GPU-idle intervals (no
kernel running on any queue) longer than a threshold, with the kernels on either side.
    python tools/step_gaps_db.py run_results.db anchor [steps] [min_gap_us]"""
import re
import sqlite3
import sys


def short(n):
  n = re.sub(r'dq::cnn::|dq::iqn::|dq::|\(anonymous namespace\)::|void ', '', n)
  if 'oneRankReduce' in n or 'ncclDevKernel' in n or 'nccl' in n.lower():
    return 'RCCL ' + n[:40]
  return n[:60]


def main():
  db = sqlite3.connect(sys.argv[1])
  anchor = sys.argv[2]
  nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
  thr = float(sys.argv[4]) if len(sys.argv) > 4 else 3.0
  rows = sorted(db.execute('select start, end, name, queue_id from kernels'))
  cuts = [i for i, r in enumerate(rows) if anchor in r[2]]
  mid = len(cuts) // 2
  a, b = cuts[mid], cuts[min(mid + nsteps, len(cuts) - 1)]
  seg = rows[a:b]
  t0 = seg[0][0]
  print('%d steps from the middle of the trace; idle gaps > %.1f us (no kernel on any queue):'
        % (nsteps, thr))
  end_max, prev = seg[0][1], seg[0]
  step = 0
  for r in seg[1:]:
    if anchor in r[2]:
      step += 1
    if r[0] - end_max > thr * 1e3:
      print('  step %2d  %8.1f -> %8.1f us  gap %6.1f  after [%s q%s]  before [%s q%s]' % (
          step, (end_max - t0) / 1e3, (r[0] - t0) / 1e3, (r[0] - end_max) / 1e3,
          short(prev[2]), prev[3], short(r[2]), r[3]))
    if r[1] > end_max:
      end_max, prev = r[1], r
  lens = [(rows[cuts[i + 1]][0] - rows[cuts[i]][0]) / 1e3 for i in range(mid, mid + nsteps)]
  print('step lengths (anchor to anchor):', ' '.join('%.1f' % v for v in lens))


if __name__ == '__main__':
  main()
