"""Phase breakdown of the standalone gather launch (k_gather_nhwc4, B = 32) from a stamp
build:
    python tools/build_variant.py gprof replay -DDQ_GATHER_PROF
    DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=ab/gprof/libdopamine_amd.so python tools/gather_stamps.py
The launches are the bench's (bench.time_gather): ITERS back-to-back graph launches, each on
a fresh random index batch of a 1M-transition buffer.  Every wave stamps s_memrealtime
(100 MHz, 10 ns) at its start, with its index in, with its four frames in and with its
stores acknowledged, into its own slot of a ring of the last 64 launches.  Per launch, times
in us from its first wave start; 'boundary' = a launch's first wave start - the previous
launch's last store acknowledgement."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

ITERS = int(os.environ.get('GP_ITERS', '400'))


def pct(v):
  return '%7.2f %7.2f %7.2f %7.2f' % (np.percentile(v, 10), np.median(v), np.percentile(v, 90),
                                      v.max())


def main():
  import bench
  from dopamine_amd import _lib
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(0)
  agent = bench.build_agent(9, 1_000_000, 32, dev)
  import random
  random.seed(0)
  bench.fill_synthetic(agent._replay.memory, 9, seed=1)
  torch.cuda.synchronize()
  L = _lib.lib
  L.dq_debug_gather_reset.argtypes = [ctypes.c_int32]
  L.dq_debug_gather_read.argtypes = [ctypes.c_void_p] * 3
  assert L.dq_debug_gather_reset(0) == 0
  us, algo, name = bench.time_gather(agent, ITERS)
  torch.cuda.synchronize()
  dims = np.zeros(2, np.uint32)
  ring = np.zeros((64, 2048, 4), np.uint64)
  seq = np.zeros(2048, np.uint32)
  assert L.dq_debug_gather_read(ring.ctypes.data, seq.ctypes.data, dims.ctypes.data) == 0
  R, W = int(dims[0]), int(dims[1])
  n = int(seq.max())
  assert (seq == n).all(), 'waves saw different launch counts'
  print('stamp build %r; %s; launches %d; event-timed avg launch %.3f us (stamp build)' % (
      _lib.BUILD_FLAGS, name, n, us))
  order = [(l % R) for l in range(n - R, n)]          # the last R launches, in order
  st = ring[order].astype(np.float64) / 100.0          # (R, W, 4) us
  frame = st[:, :, 1] > 0                              # the frame waves (not the scalar column)
  t0 = st[:, :, 0].min(axis=1)
  rows = []
  for i in range(R):
    f = frame[i]
    s = st[i]
    rows.append([s[:, 0].max() - t0[i], s[f, 1].max() - t0[i], s[f, 2].min() - t0[i],
                 s[f, 2].max() - t0[i], s[:, 3].max() - t0[i], s[~f, 3].max() - t0[i],
                 np.median(s[f, 1] - s[f, 0]), np.median(s[f, 2] - s[f, 1]),
                 np.median(s[f, 3] - s[f, 2])])
  rows = np.array(rows)
  labs = ['last wave start (dispatch ramp)', 'last index in', 'first frames in', 'last frames in',
          'last store acked (launch end)', 'scalar column end', 'wave: index latency (median)',
          'wave: frame latency (median)', 'wave: store phase (median)']
  print('%-36s %7s %7s %7s %7s' % ('per launch (us from first wave start)', 'p10', 'median', 'p90',
                                   'max'))
  for k, lab in enumerate(labs):
    print('%-36s %s' % (lab, pct(rows[:, k])))
  end = t0 + rows[:, 4]
  b = t0[1:] - end[:-1]
  print('%-36s %s' % ('boundary (prev end -> this start)', pct(b)))
  print('%-36s %s' % ('start-to-start period', pct(np.diff(t0))))
  # one launch in detail: waves by start time
  i = R // 2
  s, f = st[i], frame[i]
  for lab, v in (('wave start', s[:, 0] - t0[i]), ('index in', s[f, 1] - t0[i]),
                 ('frames in', s[f, 2] - t0[i]), ('stores acked', s[:, 3] - t0[i])):
    print('  launch %d %-14s %s' % (i, lab, pct(v)))


if __name__ == '__main__':
  main()
