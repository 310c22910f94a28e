"""The gather launches bench.py's ``roofline`` times, read back from a rocprofv3 kernel trace
of the same command (``rocprofv3 --kernel-trace --stats -- python3 bench.py ...``).

bench.time_gather launches k_gather_nhwc4 at the bench batch (grid 8 x B*2 blocks of 64) 10
times eagerly, then replays a graph of ``iters`` launches twice (a warm replay and the timed
one); nothing else in the run launches that kernel at that grid.  Prints, for the timed
replay's launches: mean kernel duration, first-start to last-end span / iters (what the HIP
events around the replay measure), and the frac of 8 TB/s each gives for the launch's
algorithmic bytes -- the line's ``roofline.frac`` must agree with these.

    python tools/gather_launches.py run_results.db [iters=400] [batch=32] [bench line json]
"""
import json
import sqlite3
import sys

HBM_PEAK_GBS = 8000.0


def main():
  db = sqlite3.connect(sys.argv[1])
  iters = int(sys.argv[2]) if len(sys.argv) > 2 else 400
  batch = int(sys.argv[3]) if len(sys.argv) > 3 else 32
  algo = batch * (2 * 4 * 7056 + 2 * 4 * 7056 * 4)
  # the bench batch's grid only (8 x 2B blocks): the DQN chunk gather (8 x 8B) and the
  # batch-1024 launches run the same kernel at other grids
  rows = sorted((s, e) for s, e, name, gx, wx, gy, wy in db.execute(
      'select start, end, name, grid_x, workgroup_x, grid_y, workgroup_y from kernels')
      if 'k_gather_nhwc4' in name and gx // max(wx, 1) == 8 and gy // max(wy, 1) == 2 * batch)
  print('k_gather_nhwc4 launches at grid 8 x (B = %d): %d (expected 10 + 2 x %d)' %
        (batch, len(rows), iters))
  # the timed replay: the last run of `iters` back-to-back launches (gaps < 2 ms); launches
  # of the same grid elsewhere in the run (e.g. eager priming steps) fall outside it
  runs, cur = [], [rows[0]]
  for r in rows[1:]:
    if r[0] - cur[-1][1] < 2_000_000:
      cur.append(r)
    else:
      runs.append(cur)
      cur = [r]
  runs.append(cur)
  timed = [r for r in runs if len(r) >= iters][-1][-iters:]
  dur = [(e - s) / 1e3 for s, e in timed]
  mean = sum(dur) / len(dur)
  span = (timed[-1][1] - timed[0][0]) / 1e3 / iters
  med = sorted(dur)[len(dur) // 2]
  out = {'launches': len(timed), 'algo_bytes_per_launch': algo,
         'mean_kernel_us': round(mean, 3), 'median_kernel_us': round(med, 3),
         'span_per_launch_us': round(span, 3),
         'frac_mean_kernel': round(algo / (mean * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
         'frac_span': round(algo / (span * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
  if len(sys.argv) > 4:
    line = json.loads([ln for ln in open(sys.argv[4]).read().splitlines()
                       if ln.startswith('{"metric"')][-1])   # rocprofv3 logs after the line
    r = line['roofline']
    out['bench_line_event_us'] = r['avg_launch_us']
    out['bench_line_frac'] = r['frac']
    out['event_vs_span'] = round(r['avg_launch_us'] / span - 1, 4)
  for k, v in out.items():
    print('%-24s %s' % (k, v))


if __name__ == '__main__':
  main()
