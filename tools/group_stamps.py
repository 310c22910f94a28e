"""What ends each grouped launch of the Rainbow learner step, from a stamp build (VERDICT r5
item 2: "open B3"):
    python tools/build_variant.py grpprof nature_cnn -DDQ_GROUP_PROF
    DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=<...>/grpprof/libdopamine_amd.so python tools/group_stamps.py
The bench's learner (1M PER buffer, B = 32, chunk graphs) is primed, then STEPS gradient steps
run with every wave of every grouped launch stamping s_memrealtime (100 MHz) at the kernel's
entry and after its op returned into its own ring slot (nature_cnn.hip GrpRec, no atomics).  Launches are separated in time
(one stream); per launch the table gives, for each op of the group (its index in the
group, the op's block count), how many waves ran it, when its first wave started and its
last wave ended (us from the launch's first wave), and the median wave duration; medians over
every occurrence of launches with the same block count.  The launch's end is its last op's end."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

STEPS = int(os.environ.get('GS_STEPS', '12'))   # every wave position's ring holds 128 launches
REC = np.dtype([('t0', '<u8'), ('t1', '<u8'), ('total', '<u4'), ('op_blk', '<u4')])
# the learner step's grouped launches, by their op lists (nature_cnn.hip
# backward_grouped<..., head_from 6> with riders, forward_fused)
NAMES = {
    'B1': ['PER set rider', 'dX fc1'],
    'B2': ['PER set rider', 'dW fc1 + Adam', 'dX conv3', 'dW fc2 + Adam'],
    'B3': ['PER sample rider', 'dW conv3 slabs', 'dX conv2 sp00', 'sp01', 'sp10', 'sp11',
           'dW conv2 slabs'],
    'B4': ['gather rider', 'sum conv3', 'dW conv1 slabs'],
    'B5': ['target conv1 rider?', 'sum conv2 + Adam', 'sum conv1 + Adam', 'Adam conv3', 'target conv1'],
}


def main():
  import bench
  from dopamine_amd import _lib
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(0)
  L = _lib.lib
  L.dq_debug_group_reset.argtypes = []
  L.dq_debug_group_read.argtypes = [ctypes.c_void_p] * 3
  pg, kw = None, {}
  if os.environ.get('GS_PEER') == '1':      # the one-rank peer schedule (bench --force-dist)
    import torch.distributed as dist
    from dopamine_amd import parallel
    parallel.FORCE_COLLECTIVES = True
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29534')
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    pg, kw = dist.group.WORLD, {'exchange': 'peer'}
  agent = bench.build_agent(9, 1_000_000, 32, dev, pg=pg, **kw)
  import random
  random.seed(0)
  bench.fill_synthetic(agent._replay.memory, 9, seed=1)
  torch.cuda.synchronize()
  prime = 0
  while not agent.graphs_primed() or prime < 100:
    agent.train_gradient_steps(9)
    prime += 9
  torch.cuda.synchronize()
  assert L.dq_debug_group_reset() == 0
  agent.train_gradient_steps(STEPS)
  torch.cuda.synchronize()
  dims = np.zeros(2, np.uint32)
  P, R = 1024 * 16, 128
  recs = np.zeros((P, R), REC)
  seq = np.zeros(P, np.uint32)
  assert L.dq_debug_group_read(recs.ctypes.data, seq.ctypes.data, dims.ctypes.data) == 0
  assert tuple(dims) == (P, R), dims
  assert seq.max() <= R, 'a ring wrapped: fewer steps (GS_STEPS)'
  r = np.concatenate([recs[p, :seq[p]] for p in np.flatnonzero(seq)])
  r = np.sort(r, order='t0')
  print('stamp build %r; %d gradient steps; %d wave records' % (_lib.BUILD_FLAGS, STEPS, len(r)))
  # launches: a new one starts when a wave starts after every earlier wave ended, or the grid
  # size changes
  launches, cur, tmax = [], [0], r['t1'][0]
  for i in range(1, len(r)):
    if r['t0'][i] > tmax or r['total'][i] != r['total'][i - 1]:
      launches.append(cur)
      cur = []
    cur.append(i)
    tmax = max(tmax, r['t1'][i])
  launches.append(cur)
  # every gradient step runs the same sequence of grouped launches: key them by position
  period = int(round(len(launches) / float(STEPS)))
  by_total = {}
  for li, ix in enumerate(launches):
    x = r[ix]
    t0 = int(x['t0'].min())
    ops = {}
    for k in np.unique(x['op_blk'] >> 24):
      y = x[(x['op_blk'] >> 24) == k]
      ops[int(k)] = (len(y), int(((y['op_blk'] >> 8) & 0xffff).max()) + 1,
                     (int(y['t0'].min()) - t0) / 100.0, (int(y['t1'].max()) - t0) / 100.0,
                     float(np.median(y['t1'] - y['t0'])) / 100.0)
    by_total.setdefault((li % period, int(x['total'][0])), []).append(
        ((int(x['t1'].max()) - t0) / 100.0, ops))
  gaps = [(int(r[launches[i + 1]]['t0'].min()) - int(r[launches[i]]['t1'].max())) / 100.0
          for i in range(len(launches) - 1)]
  print('launches %d; boundary (last wave end -> next first wave start) median %.2f us, p90 %.2f'
        % (len(launches), np.median(gaps), np.percentile(gaps, 90)))
  print('%d grouped launches per gradient step' % period)
  for (pos, total), occ in sorted(by_total.items()):
    dur = np.array([o[0] for o in occ])
    print('\nlaunch %d of the step, %d blocks: %d occurrences, duration median %.2f us (p10 %.2f, '
          'p90 %.2f)' % (pos, total, len(occ), np.median(dur), np.percentile(dur, 10),
                         np.percentile(dur, 90)))
    keys = sorted(set(k for o in occ for k in o[1]))
    last = [max(o[1], key=lambda k: o[1][k][3]) for o in occ]
    print('  %-4s %7s %7s %9s %9s %11s  %s' % ('op', 'blocks', 'waves', 'first in', 'last out',
                                               'wave (med)', 'ends the launch'))
    for k in keys:
      v = np.array([o[1][k] for o in occ if k in o[1]])
      print('  %-4d %7d %7d %9.2f %9.2f %11.2f  %d/%d' % (
          k, int(np.median(v[:, 1])), int(np.median(v[:, 0])), np.median(v[:, 2]),
          np.median(v[:, 3]), np.median(v[:, 4]), last.count(k), len(occ)))

  if pg is not None:                         # the exchange launch's phases (PeerExchOp)
    L.dq_debug_peer_phases.argtypes = [ctypes.c_void_p] * 2
    ph = np.zeros((16, 128, 5), np.uint64)
    sq = np.zeros(16, np.uint32)
    assert L.dq_debug_peer_phases(ph.ctypes.data, sq.ctypes.data) == 0
    n = int(min(sq.min(), 128))
    ph = ph[:, :n].astype(np.int64)
    start = ph[:, :, 0].min(axis=0)          # per occurrence: the first block's entry
    rel = (ph - start[None, :, None]) / 100.0
    print('\nexchange launch phases (us from its first exchange block\'s entry; %d occurrences, '
          'median over occurrences of the blocks\' max / min):' % n)
    for k, what in enumerate(['entry', 'published (blocks < 16)', 'wait passed', 'conv Adam done',
                              'ticket taken']):
      print('  %-26s max %.2f  min %.2f' % (what, np.median(rel[:, :, k].max(axis=0)),
                                            np.median(rel[:, :, k].min(axis=0))))


if __name__ == '__main__':
  main()
