"""Where a short timed window's time goes (the driver's 20-step window read
2-3% below 300-step windows of the same build).  After bench.py's priming, times windows of
K steps exactly as bench.timed_steps does (synchronize, perf_counter, train_gradient_steps,
synchronize) and splits each into: host time before the first chunk graph is handed to the
GPU, host submission time of the whole window, and the GPU's time from an event recorded at
the window start to one recorded at its end.

    python tools/window_probe.py [K ...]
"""
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
  if os.environ.get('DQ_SPIN') == '1':      # host waits spin instead of yielding (HIP flag)
    import ctypes
    hip = ctypes.CDLL('libamdhip64.so')
    assert hip.hipSetDeviceFlags(1) == 0    # hipDeviceScheduleSpin, before the context exists
  import bench
  ks = [int(x) for x in sys.argv[1:]] or [20, 300]
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(0)
  agent = bench.build_agent(9, 1_000_000, 32, dev)
  import random
  random.seed(0)
  bench.fill_synthetic(agent._replay.memory, 9, seed=1)
  torch.cuda.synchronize()
  bench.timed_steps(agent, 20, 5)          # bench's priming (graphs captured, clocks up)
  if os.environ.get('DQ_UPLOAD') == '1':    # hipGraphUpload of the chunk graphs' executables
    import ctypes
    hip = ctypes.CDLL('libamdhip64.so')
    hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    for key, g in agent._graph_sets.items():
      if isinstance(key, tuple) and key[0] == 'chunk':
        rc = hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
    torch.cuda.synchronize()
  first = {}

  def wrap(g):
    orig = g.replay

    def replay():
      if 't' not in first:
        first['t'] = time.perf_counter()
      orig()
    g.replay = replay
  for key, g in agent._graph_sets.items():
    if isinstance(key, tuple) and key[0] == 'chunk':
      wrap(g)
  stream = torch.cuda.current_stream()
  rows = {k: [] for k in ks}
  gc.disable()
  for rep in range(6):
    for k in ks:
      first.clear()
      e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      torch.cuda.synchronize()
      t0 = time.perf_counter()
      e0.record(stream)
      agent.train_gradient_steps(k)
      ts = time.perf_counter()
      e1.record(stream)
      torch.cuda.synchronize()
      t1 = time.perf_counter()
      rows[k].append((first.get('t', ts) - t0, ts - t0, e0.elapsed_time(e1) * 1e-3, t1 - t0))
  # host time of each piece of the first chunk's path (one window, wrapped methods)
  import collections
  spent = collections.defaultdict(float)
  mem = agent._replay.memory

  def timed(obj, name, label):
    f = getattr(obj, name)

    def w(*a, **k):
      t = time.perf_counter()
      try:
        return f(*a, **k)
      finally:
        spent[label] += time.perf_counter() - t
    setattr(obj, name, w)
  timed(agent, '_chunk_ok', '_chunk_ok')
  timed(agent, '_join_fc', '_join_fc')
  timed(mem, 'reserve_rng', 'reserve_rng (x4)')
  timed(agent, '_run_train_ops_chunk', '_run_train_ops_chunk (incl. replay)')
  for k, g in agent._graph_sets.items():
    if isinstance(k, tuple) and k[0] == 'chunk':
      timed(g, 'replay', 'replay call')
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  agent.train_gradient_steps(4)
  tot = time.perf_counter() - t0
  torch.cuda.synchronize()
  # GPU time per chunk of a 20-step window (is the first chunk after the idle slower?)
  evs = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
  per = []
  for rep in range(6):
    torch.cuda.synchronize()
    evs[0].record(stream)
    for j in range(5):
      agent.train_gradient_steps(4)
      evs[j + 1].record(stream)
    torch.cuda.synchronize()
    per.append([evs[j].elapsed_time(evs[j + 1]) * 1e3 for j in range(5)])
  print('GPU us per 4-step chunk of a 20-step window (median of 6):',
        ' '.join('%.1f' % v for v in np.median(np.array(per), axis=0)))
  # the first chunk against the idle time before the window (host sleep after the sync)
  for idle_us in (0, 100, 1000, 10000, 100000):
    per = []
    for rep in range(6):
      torch.cuda.synchronize()
      if idle_us:
        time.sleep(idle_us * 1e-6)
      evs[0].record(stream)
      for j in range(5):
        agent.train_gradient_steps(4)
        evs[j + 1].record(stream)
      torch.cuda.synchronize()
      per.append([evs[j].elapsed_time(evs[j + 1]) * 1e3 for j in range(5)])
    print('idle %6d us before the window: GPU us per chunk (median of 6):' % idle_us,
          ' '.join('%.1f' % v for v in np.median(np.array(per), axis=0)))
  gc.enable()
  print('host us, one 4-step chunk from an idle device: total %.1f; ' % (tot * 1e6) +
        '; '.join('%s %.1f' % (k, v * 1e6) for k, v in spent.items()))
  print('K   pre-first-replay us   host submit us   GPU e0->e1 us   wall us   steps/s wall   '
        'steps/s GPU   (medians of 6)')
  for k in ks:
    a = np.median(np.array(rows[k]), axis=0) * 1e6
    print('%4d %12.1f %16.1f %15.1f %10.1f %12.1f %14.1f' % (k, a[0], a[1], a[2], a[3],
                                                             k / a[3] * 1e6, k / a[2] * 1e6))


if __name__ == '__main__':
  main()
