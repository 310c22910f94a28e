"""One step's kernel timeline (start offset, duration, queue) from a rocprofv3
--kernel-trace results database, steps cut at each launch of an anchor kernel;
prints the step whose length is the median.
    python tools/step_timeline_db.py run_results.db anchor [skip]"""
import re
import sqlite3
import statistics
import sys


def short(n):
  n = re.sub(r'dq::cnn::|dq::iqn::|dq::|\(anonymous namespace\)::|void ', '', n)
  return n[:95]


def main():
  db = sqlite3.connect(sys.argv[1])
  anchor = sys.argv[2]
  skip = int(sys.argv[3]) if len(sys.argv) > 3 else 20
  rows = sorted(db.execute('select start, end, name, queue_id, grid_x, workgroup_x from kernels'))
  cuts = [i for i, r in enumerate(rows) if anchor in r[2]]
  steps = [rows[a:b] for a, b in zip(cuts[skip:-1], cuts[skip + 1:])]
  lens = [s[-1][1] - s[0][0] for s in steps]
  med = statistics.median(lens)
  s = min(steps, key=lambda st: abs((st[-1][1] - st[0][0]) - med))
  t0 = s[0][0]
  print('%d steps; median step %.1f us (anchor %s)' % (len(steps), med / 1e3, anchor))
  busy, cur = 0, None                  # the union of the step's kernel intervals (any queue)
  for st, en in sorted((r[0], r[1]) for r in s):
    if cur is None or st > cur[1]:
      busy += 0 if cur is None else cur[1] - cur[0]
      cur = [st, en]
    else:
      cur[1] = max(cur[1], en)
  busy += cur[1] - cur[0]
  print('GPU busy (some kernel running) %.1f of %.1f us' % (busy / 1e3, (s[-1][1] - s[0][0]) / 1e3))
  print('   start      dur      end  q  blocks  kernel')
  for st, en, n, q, gx, wx in s:
    print('%8.1f %8.1f %8.1f %2s %7d  %s' % ((st - t0) / 1e3, (en - st) / 1e3, (en - t0) / 1e3, q,
                                            gx // max(wx, 1), short(n)))


if __name__ == '__main__':
  main()
