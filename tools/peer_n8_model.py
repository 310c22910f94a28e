"""The peer-memory exchange's per-rank step at N = 8 from a measured one-rank step.

Input: a one-rank peer step timeline (tools/step_timeline_db.py over a rocprof kernel trace of
``bench.py --force-dist --schedules peer``: the exchange runs against the learner itself, every
wait passes at once, nothing crosses xGMI) and the no-group single learner's step.  At N = 8
the launches are the same; what changes is that each rank pulls 7/8 of the fc bucket's
gradients (the reduce-scatter, riding in backward launches 3-4), 7/8 of its parameters (the
all-gather: backward launch 5, or -- deferred -- the next forward's three conv launches) and 7
copies of the conv bucket's gradients (launch 6) over xGMI, and every wait costs at least a
flag round trip.  Per launch group g:

  t_g(8) = max(t_g(1), pull_g / BW + wait) + skew        (the launch ends when both are done)

t_g(1) is the one-rank duration, an upper bound on the N = 8 compute (its slice Adam covers the
whole bucket, 8x the N = 8 slice).  BW: the aggregate rate one GPU pulls from its 7 peers;
MI355X has 7 xGMI links at about 153 GB/s each (1.07 TB/s), taken here at 300-450 GB/s (28-42%,
an assumption: not measurable on a one-GPU box).  wait: one flag round trip (2 us);
skew: rank-to-rank arrival jitter per exchange point (0 or 3 us).  The learner loop defers the
all-gather (the 'split' rows: a quarter in launch 5, three quarters in the next forward's conv
launches, nature_cnn.hip AgParts); per-call steps keep it whole in launch 5.

    python tools/peer_n8_model.py profiles/r5_peer/peer_step_timeline.txt [single_step_us]
"""
import sys

N = 8
# the Rainbow Nature CNN's buckets (SAME padding: conv3 is 11 x 11 x 64 = 7744; 9 actions x
# 51 atoms): fc1 7744 x 512 + 512, fc2 512 x 459 + 459 floats; conv1..conv3 weights + biases
FC_FLOATS = 7744 * 512 + 512 + 512 * 459 + 459
CONV_FLOATS = 8 * 8 * 4 * 32 + 32 + 4 * 4 * 32 * 64 + 64 + 3 * 3 * 64 * 64 + 64
WAIT_US = 2.0


def parse(path):
  rows = []
  for line in open(path):
    p = line.split()
    if len(p) >= 6 and p[0].replace('.', '').isdigit() and p[1].replace('.', '').isdigit():
      rows.append((float(p[0]), float(p[1]), ' '.join(p[5:])))
  step = float(open(path).readline().split('median step')[1].split('us')[0])
  return step, rows


def groups(rows):
  """The launch groups of one step (anchored at k_c51): rs = backward launches 3 + 4,
  l5 = launch 5 (publish), l6 = the conv exchange, fconv = the next forward's three conv
  launches, rest = everything else."""
  names = [r[2] for r in rows]
  i3 = next(i for i, n in enumerate(names) if 'PeerPubOp' in n)
  i5 = next(i for i, n in enumerate(names) if 'PeerPubOp' in n and i > i3)
  i6 = next(i for i, n in enumerate(names) if 'PeerExchOp' in n)
  assert i5 == i3 + 2 and i6 == i5 + 1, names
  dur = [r[1] for r in rows]
  g = {'rs': dur[i3] + dur[i3 + 1], 'l5': dur[i5], 'l6': dur[i6],
       'fconv': sum(dur[i6 + 1:i6 + 4])}
  g['rest'] = sum(dur) - sum(g.values())
  return g


AG_LAUNCH5 = 4 / 16          # nature_cnn.hip kAgLaunch5: the deferred gather's share in launch 5


def model(g, bw, skew, where):
  pull = (N - 1) / N * FC_FLOATS * 4 / (bw * 1e3)          # us (GB/s = 1e3 bytes/us)
  conv = (N - 1) * CONV_FLOATS * 4 / (bw * 1e3)
  t = g['rest']
  t += max(g['rs'], pull + WAIT_US) + skew
  if where == 'l5':
    t += max(g['l5'], pull + WAIT_US) + skew + g['fconv']
  elif where == 'fconv':
    t += g['l5'] + max(g['fconv'], pull + WAIT_US) + skew
  else:                              # split: a quarter in launch 5, the rest in F1-F3
    t += max(g['l5'], AG_LAUNCH5 * pull + WAIT_US) + skew
    t += max(g['fconv'], (1 - AG_LAUNCH5) * pull + WAIT_US) + skew
  t += g['l6'] + conv + WAIT_US + skew
  return t, pull, conv


def main():
  path = sys.argv[1]
  single = float(sys.argv[2]) if len(sys.argv) > 2 else 122.5
  step, rows = parse(path)
  g = groups(rows)
  print('one-rank peer step %.1f us (single learner %.1f us: the exchange costs %.1f us at world 1)'
        % (step, single, step - single))
  print('launch groups (us): ' + ', '.join('%s %.1f' % kv for kv in g.items()))
  print('per rank at N = 8: reduce-scatter and all-gather pull %.2f MB each, the conv bucket '
        '%.2f MB' % ((N - 1) / N * FC_FLOATS * 4 / 1e6, (N - 1) * CONV_FLOATS * 4 / 1e6))
  print()
  print('%-24s %9s %6s %8s %8s %8s %10s %8s' % ('all-gather', 'BW GB/s', 'skew', 'pull_us',
                                                'conv_us', 'step_8', 'steps/s/GPU', 'x at 8'))
  label = {'l5': 'backward launch 5', 'fconv': 'next forward F1-F3',
           'split': 'launch 5 1/4, F1-F3 3/4'}
  for where in ('l5', 'fconv', 'split'):
    for bw in (300.0, 375.0, 450.0):
      for skew in (0.0, 3.0):
        t, pull, conv = model(g, bw, skew, where)
        print('%-24s %9.0f %6.1f %8.1f %8.1f %8.1f %10.0f %8.2f' % (
            label[where], bw, skew, pull, conv, t,
            1e6 / t, N * single / t))


if __name__ == '__main__':
  main()
