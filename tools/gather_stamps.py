"""Phase breakdown of the standalone gather launch (k_gather_nhwc4, B = 32) from a stamp
build:
    python tools/build_variant.py gprof replay -DDQ_GATHER_PROF
    DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=ab/gprof/libdopamine_amd.so python tools/gather_stamps.py
The launches are the bench's (bench.time_gather): ITERS back-to-back graph launches, each on
a fresh random index batch of a 1M-transition buffer.  Every wave stamps s_memrealtime
(100 MHz) at its start, with its index in, with its four frames in, and with its stores
acknowledged; per launch the first / last of each are kept.  Times in us from the launch's
first wave start; 'boundary' = this launch's first wave start - the previous one's last store."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

ITERS = int(os.environ.get('GP_ITERS', '400'))


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
  nl, nw = 1024, 4096
  target = ITERS // 2
  # warm-up / event timing exactly as the bench line's (the stamps add their waits)
  us, algo, name = bench.time_gather(agent, ITERS)
  assert L.dq_debug_gather_reset(target) == 0
  us2, _, _ = bench.time_gather(agent, ITERS)
  torch.cuda.synchronize()
  launches = np.zeros((nl, 8), np.uint64)
  waves = np.zeros((nw, 4), np.uint64)
  count = np.zeros(1, np.uint32)
  assert L.dq_debug_gather_read(launches.ctypes.data, waves.ctypes.data, count.ctypes.data) == 0
  n = int(count[0])
  print('stamp build %r; launches stamped %d; event-timed avg launch %.3f us (%.3f with the '
        'stamps reset between, same build)' % (_lib.BUILD_FLAGS, n, us, us2))
  # time_gather runs 10 eager launches, then the graph replayed twice: the last ITERS
  # launches are the timed replay
  Lr = launches[:min(n, nl)].astype(np.float64)
  tl = Lr[-ITERS:] if n >= ITERS else Lr
  t0 = tl[:, 0]
  rel = (tl - t0[:, None]) / 100.0
  cols = [('last wave start (dispatch ramp)', 1), ('last index in', 2), ('first frames in', 3),
          ('last frames in', 4), ('last store acked (launch end)', 5), ('scalar column end', 6)]
  print('%-34s %8s %8s %8s' % ('per launch, us from first wave start', 'p10', 'median', 'p90'))
  for lab, k in cols:
    v = rel[:, k]
    print('%-34s %8.2f %8.2f %8.2f' % (lab, np.percentile(v, 10), np.median(v), np.percentile(v, 90)))
  b = (tl[1:, 0] - tl[:-1, 5]) / 100.0
  print('%-34s %8.2f %8.2f %8.2f' % ('boundary (prev end -> this start)', np.percentile(b, 10),
                                     np.median(b), np.percentile(b, 90)))
  per = (tl[1:, 0] - tl[:-1, 0]) / 100.0
  print('%-34s %8.2f %8.2f %8.2f' % ('start-to-start period', np.percentile(per, 10),
                                     np.median(per), np.percentile(per, 90)))
  # the target launch (launch index `target` of the run: in the first replay)
  w = waves.astype(np.float64)
  live = w[:, 0] > 0
  w = w[live]
  s0 = w[:, 0].min()
  fr = w[:, 1] > 0
  print('target launch %d: %d waves (%d frame waves)' % (target, len(w), int(fr.sum())))
  for lab, v in (('wave start', (w[:, 0] - s0) / 100.0),
                 ('index latency (start -> index in)', (w[fr, 1] - w[fr, 0]) / 100.0),
                 ('frame latency (index in -> frames in)', (w[fr, 2] - w[fr, 1]) / 100.0),
                 ('store phase (frames in -> stores acked)', (w[fr, 3] - w[fr, 2]) / 100.0),
                 ('wave end', (w[:, 3] - s0) / 100.0)):
    print('  %-42s p10 %6.2f  median %6.2f  p90 %6.2f  max %6.2f' % (
        lab, np.percentile(v, 10), np.median(v), np.percentile(v, 90), v.max()))


if __name__ == '__main__':
  main()
