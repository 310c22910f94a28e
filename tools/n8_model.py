"""Config 4's per-rank step at N = 8 from measured one-rank parts.

Inputs: a one-rank RCCL step timeline (tools/step_timeline_db.py over a rocprof trace of
``bench.py --force-dist``; every collective executed, each a local copy) and the no-group
single-learner step.  The model replaces the one-rank collectives by 8-rank ones and asks
whether the fc bucket's exchange still fits the window the schedule gives it:

  main path   = the one-rank step, minus the one-rank conv all-reduce, plus an 8-rank
                all-reduce of the conv bucket (small: latency-bound)
  fc window   = from the fork (the first launch after backward launch 2 starts) to the join
                (the next step's fc1 launch starts), on the main queue
  fc branch   = the delay before the comm queue gets CUs (measured: it waits for backward
                launch 3's blocks) + the 8-rank collective(s) + the fc Adam part (measured)
  step_8      = main path + max(0, fc branch - fc window)

8-rank collective times: a ring all-reduce moves 2 (N-1)/N x S per GPU, a reduce-scatter or
all-gather (N-1)/N x S, at RCCL's bus bandwidth over xGMI.  MI355X: 7 xGMI links per GPU at
about 153 GB/s each (the task's figure; the local guides give none); RCCL's large-message bus
bandwidth on 8 x MI3xx is taken as 300-450 GB/s (a range, stated as an assumption -- it is not
measurable on a one-GPU box).  The small conv bucket's all-reduce is latency-bound: 10-25 us.

    python tools/n8_model.py profiles/r3_s3_dist/step_timeline.txt [single_step_us]
"""
import sys

FC_BYTES = 4_197_888 * 4          # fc1 + fc2 weights and biases (Rainbow, 9 actions)
N = 8


def parse(path):
  rows = []
  for line in open(path):
    p = line.split()
    if len(p) >= 6 and p[0].replace('.', '').isdigit() and p[1].replace('.', '').isdigit():
      rows.append((float(p[0]), float(p[1]), float(p[2]), int(p[3]), int(p[4]), ' '.join(p[5:])))
  head = open(path).readline()
  step = float(head.split('median step')[1].split('us')[0])
  return step, rows


def main():
  path = sys.argv[1]
  single = float(sys.argv[2]) if len(sys.argv) > 2 else 126.5
  step, rows = parse(path)
  main_q = max(set(r[3] for r in rows), key=lambda q: sum(1 for r in rows if r[3] == q))
  mains = [r for r in rows if r[3] == main_q]
  side = [r for r in rows if r[3] != main_q]
  ar_main = [r for r in mains if 'oneRank' in r[5] or 'nccl' in r[5].lower()]
  conv_ar = sum(r[1] for r in ar_main)
  grouped = [r for r in mains if 'k_grouped' in r[5]]
  # backward launches: the grouped launches after k_c51 up to the first forward conv1
  b2_end = grouped[1][2]                       # C, B1, B2 -> B2 is the 2nd grouped launch
  fork = next(r[0] for r in grouped if r[0] >= b2_end)
  fc1_start = [r for r in grouped if 'RowK, RowK, EpiPartial' in r[5]][-1][0]
  window = fc1_start - fork
  ar_side = [r for r in side if 'oneRank' in r[5] or 'nccl' in r[5].lower()]
  adam_side = [r for r in side if 'adam' in r[5]]
  wait = ar_side[0][0] - fork if ar_side else 0.0
  adam_part = sum(r[1] for r in adam_side)
  print('one-rank step %.1f us (single learner %.1f us: the schedule costs %.1f us, %.0f%%)'
        % (step, single, step - single, 100 * (step / single - 1)))
  print('main queue %d: conv bucket all-reduce (one rank, a copy) %.1f us' % (main_q, conv_ar))
  print('fc window: fork at %.1f -> next fc1 at %.1f = %.1f us; comm queue waits %.1f us for CUs;'
        ' fc Adam part %.1f us' % (fork, fc1_start, window, wait, adam_part))
  print()
  print('%-10s %-9s %8s %8s %8s %9s %8s %7s' % ('schedule', 'busbw', 'coll_us', 'branch', 'over',
                                                  'conv_ar', 'step_8', 'x at 8'))
  for sched in ('allreduce', 'zero1'):
    for bw in (300.0, 375.0, 450.0):
      if sched == 'allreduce':
        coll = 2 * (N - 1) / N * FC_BYTES / (bw * 1e3)     # us (GB/s = 1e3 bytes/us)
        upd = adam_part
      else:
        coll = 2 * (N - 1) / N * FC_BYTES / (bw * 1e3)     # reduce-scatter + all-gather
        upd = adam_part / N
      branch = wait + coll + upd
      for car in (10.0, 25.0):
        main_path = step - conv_ar + car
        step8 = main_path + max(0.0, branch - window)
        print('%-10s %5.0f GB/s %7.1f %8.1f %8.1f %7.1f %9.1f %7.2f' % (
            sched, bw, coll, branch, max(0.0, branch - window), car, step8, N * single / step8))


if __name__ == '__main__':
  main()
