"""From a rocprofv3 --kernel-trace --hip-runtime-trace results database: how long after a
hipGraphLaunch call the graph's first kernel starts, for launches that find the GPU idle
(the first replay of a timed window, right after a synchronize) and for the rest (the host
running ahead); and how long the call itself takes on the host.
    python tools/launch_latency_db.py run_results.db"""
import sqlite3
import statistics
import sys


def main():
  db = sqlite3.connect(sys.argv[1])
  names = [r[0] for r in db.execute("select name from sqlite_master where type in ('table','view')")]
  api_src = None
  for n in names:
    cols = [c[1] for c in db.execute('pragma table_info("%s")' % n)]
    if {'start', 'end', 'name'} <= set(cols) and n not in ('kernels',) and 'kernel' not in n.lower():
      try:
        if db.execute('select count(*) from "%s" where name like \'%%hipGraphLaunch%%\'' % n).fetchone()[0]:
          api_src = n
          break
      except sqlite3.Error:
        continue
  if api_src is None:
    print('no hipGraphLaunch rows; tables:', names)
    return
  api = sorted(db.execute('select start, end, name from "%s"' % api_src))
  kern = sorted(db.execute('select start, end from kernels'))
  kstarts = [k[0] for k in kern]
  import bisect
  idle, busy, dur = [], [], []
  for i, (s, e, n) in enumerate(api):
    if 'hipGraphLaunch' not in n:
      continue
    dur.append((e - s) / 1e3)
    j = bisect.bisect_left(kstarts, s)
    if j >= len(kern):
      continue
    # the GPU was idle at the call if no kernel was running then
    prev_end = max((k[1] for k in kern[max(0, j - 64):j]), default=0)
    (idle if prev_end < s else busy).append((kern[j][0] - s) / 1e3)
  print('source %s: %d hipGraphLaunch calls' % (api_src, len(dur)))
  print('call duration on the host: median %.1f us, p90 %.1f' % (
      statistics.median(dur), sorted(dur)[int(0.9 * len(dur))]))
  if idle:
    print('GPU idle at the call (%d): first kernel starts %.1f us after the call (median; min '
          '%.1f, max %.1f)' % (len(idle), statistics.median(idle), min(idle), max(idle)))
  if busy:
    print('GPU busy at the call (%d): next kernel start - call %.1f us (median)' % (
        len(busy), statistics.median(busy)))


if __name__ == '__main__':
  main()
