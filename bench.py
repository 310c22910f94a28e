"""Benchmark: Rainbow gradient-steps/sec, batch 32, 1M-transition PER buffer
(BASELINE.json metric, configs[2]: Rainbow/C51 Asterix, 9 actions, n=3).

One step = one reference ``_train_op``: prioritized stratified sample (+retries)
-> frame-stack gather + /255 + n-step reward -> online fwd/bwd + target fwd ->
C51 target/projection/cross-entropy -> priority write-back -> TF1 Adam, plus the
target sync at its reference cadence (every 8000 agent steps = 2000 gradient
steps).  Synthetic 1M-transition buffer resident in HBM (no Atari frames
offline).  Multi-GPU (torchrun): one learner + one 1M buffer per GPU, flat
gradient all-reduced over RCCL each step (weak scaling).

    python bench.py [--gpus N --steps K --warmup W]
"""
import argparse
import ctypes
import gc
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')   # as dopamine_amd/__init__.py; before HIP init

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md, HBM3E spec peak


def parse(argv=None):
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--steps', type=int, default=300)
  ap.add_argument('--warmup', type=int, default=30)
  ap.add_argument('--capacity', type=int, default=1_000_000)
  ap.add_argument('--batch', type=int, default=32)
  ap.add_argument('--actions', type=int, default=9)
  ap.add_argument('--no-graph', action='store_true')
  ap.add_argument('--cpu-seconds', type=float, default=12.0)
  ap.add_argument('--skip-cpu-baseline', action='store_true')
  ap.add_argument('--skip-configs', action='store_true',
                  help='do not time BASELINE configs 2 and 5 after the headline (N = 1)')
  ap.add_argument('--per-call', action='store_true',
                  help='drive the agent by update_period _train_step() calls per gradient '
                       'step (one graph replay per step) instead of train_gradient_steps')
  ap.add_argument('--gather-iters', type=int, default=400)
  ap.add_argument('--schedules', default=None,
                  help='N > 1 (or --force-dist): comma-separated data-parallel schedules to time, '
                       'one after the other on fresh agents, the headline from the fastest -- '
                       'peer (the exchange over peer memory inside the backward, one stream: '
                       'DQNAgent exchange=\'peer\'), allreduce (the gradient buckets\' '
                       'all-reduce on a second stream), zero1 (its reduce-scatter / slice Adam / '
                       'all-gather form).  Default: peer, and allreduce only if peer failed on '
                       'some rank (a failed construction or self-test, a latched exchange '
                       'error, replicas that differ) -- the first N > 1 run on a node does '
                       'not stake its line on a second schedule once one has run cleanly')
  ap.add_argument('--comm', choices=('native', 'torch'), default='native',
                  help='N > 1 over RCCL: the learner\'s own communicators (parallel.RcclComm) '
                       'or torch.distributed\'s collectives')
  ap.add_argument('--skip-bf16', action='store_true',
                  help='do not time the separate bf16 throughput row (N = 1)')
  ap.add_argument('--bf16-child', action='store_true', help=argparse.SUPPRESS)
  ap.add_argument('--force-dist', action='store_true',
                  help='one rank only: run the N > 1 learner schedule over a one-rank RCCL group '
                       'with every collective executed (a hardware check of the data-parallel '
                       'path on a one-GPU box; not the bench line)')
  return ap.parse_args(argv)


def fill_synthetic(mem, A, seed, priority=None):
  """SURVEY 8(d) synthetic inputs, generated on the device (priority: one priority for
  every transition, e.g. 1.0 as a 'uniform' scheme inserts; default random in [0.1, 2))."""
  C = mem._replay_capacity
  dev = mem._device
  g = torch.Generator(device=dev).manual_seed(seed)
  frames = torch.randint(0, 256, (C, mem._obs_bytes), dtype=torch.uint8, device=dev, generator=g)
  actions = torch.randint(0, A, (C,), dtype=torch.int32, device=dev, generator=g)
  rewards = (torch.randint(0, 3, (C,), device=dev, generator=g) - 1).float()
  terminals = (torch.rand(C, device=dev, generator=g) < 1.0 / 500).to(torch.uint8)
  prios = torch.rand(C, device=dev, generator=g, dtype=torch.float64) * 1.9 + 0.1
  if priority is not None:
    prios.fill_(priority)
  mem.load_arrays(frames, actions, rewards, terminals, add_count=C + 12345, priorities=prios)
  del frames


def build_agent(actions, capacity, batch, device, pg=None, **kw):
  """The benchmarked learner: Rainbow as rainbow.gin binds it (n = 3, Adam 6.25e-5 /
  1.5e-4, target period 8000, update period 4, PER), on the device's 1M buffer.
  Every rank builds the same networks (seed 0; rank 0's are broadcast anyway)."""
  from dopamine_amd.agents.optimizers import AdamOptimizer
  from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent
  agent = RainbowAgent(num_actions=actions, update_horizon=3, gamma=0.99,
                       replay_scheme='prioritized', min_replay_history=20000, update_period=4,
                       target_update_period=8000,
                       optimizer=AdamOptimizer(learning_rate=0.0000625, epsilon=0.00015),
                       replay_capacity=capacity, batch_size=batch, device=device, seed=0,
                       process_group=pg, **kw)
  # the fused optimizer consumes the gradient in registers; no flat gradient buffer is
  # written (the reference keeps none either; the traced parity tests still write it)
  agent.keep_gradients = False
  return agent


def build_dqn_pong(device, **kw):
  """BASELINE config 2: DQN as dqn.gin binds it (6 actions, uniform replay, n = 1, TF1
  centered RMSProp 2.5e-4 / 0.95 / 1e-5, target period 8000, update period 4), B = 32."""
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  agent = DQNAgent(num_actions=6, min_replay_history=20000, update_period=4,
                   target_update_period=8000, replay_capacity=1_000_000, batch_size=32,
                   device=device, seed=0, **kw)
  agent.keep_gradients = False      # as build_agent
  return agent


def build_iqn_breakout(device, **kw):
  """BASELINE config 5: IQN as implicit_quantile.gin binds it (4 actions, N = N' = 64,
  K = 32, n = 3, uniform replay, Adam 5e-5 / 3.125e-4, kappa 1, embedding 64), B = 64."""
  from dopamine_amd.agents.implicit_quantile.implicit_quantile_agent import ImplicitQuantileAgent
  from dopamine_amd.agents.optimizers import AdamOptimizer
  return ImplicitQuantileAgent(
      num_actions=4, num_tau_samples=64, num_tau_prime_samples=64, num_quantile_samples=32,
      update_horizon=3, replay_scheme='uniform', min_replay_history=20000, update_period=4,
      target_update_period=8000, optimizer=AdamOptimizer(learning_rate=0.00005, epsilon=0.0003125),
      replay_capacity=1_000_000, batch_size=64, device=device, seed=0, **kw)


MIN_PRE_STEPS = 100
# N > 1: every blocking phase (rendezvous, learner construction with its rank-0 broadcast,
# the barriers and collectives of the timed steps) must complete within DEADLINE_S seconds,
# else the rank reports which one and exits (parallel.Deadline): a cross-rank ordering bug
# or a dead peer ends the run instead of hanging it
DEADLINE_S = float(os.environ.get('DQ_DEADLINE_S', '600'))
# rehearsal only (DQ_BENCH_REHEARSE=1, gloo on one GPU): this group rank withholds the barrier
# before the timed window, so the other ranks' deadline fires (tests/test_gpu_rccl.py)
WITHHOLD_RANK = (int(os.environ['DQ_BENCH_WITHHOLD_RANK'])
                 if os.environ.get('DQ_BENCH_REHEARSE') == '1'
                 and 'DQ_BENCH_WITHHOLD_RANK' in os.environ else None)


def timed_steps(agent, steps, warmup, per_call=False, pg=None, deadline=None, probe=None):
  """The bench protocol on one agent: untimed priming, whatever ``warmup`` is, until every
  graph the timed loop replays is captured (both step parities, the 4-step chunk graphs of
  both starting parities) and the device has been busy for at least MIN_PRE_STEPS steps
  (its clocks ramp under load: a 20-step window after 5 warmup steps read 7% low); then
  the warmup; then exactly ``steps`` gradient steps between barriers + synchronize.  No
  cyclic-garbage collection pass inside the window (a full pass over a torch process's
  objects takes milliseconds).  deadline (N > 1): a parallel.Deadline armed for each
  blocking phase.  probe: called with 'before' / 'after' just outside the window (the device
  idle; e.g. the peer exchange's wait counters).  Returns (elapsed seconds, priming steps)."""
  def phase(label):
    if deadline is not None:
      deadline.phase(label, DEADLINE_S)

  def grad_steps(n):
    if per_call:
      for _ in range(n):
        for _ in range(agent.update_period):   # the reference's _train_step cadence
          agent._train_step()
    else:   # the same calls, consecutive steps replayed K per HIP graph (learner-only loop)
      agent.train_gradient_steps(n)

  gc.collect()
  gc.disable()
  try:
    prime = 0
    phase('priming (graph capture, steps with their fc / conv bucket all-reduces)')
    while ((not agent.graphs_primed() or prime + warmup < MIN_PRE_STEPS) and prime < 400):
      grad_steps(9)     # two chunks and a single step per call: every graph the window replays
      prime += 9
    grad_steps(warmup)
    torch.cuda.synchronize()
    if pg is not None:
      phase('the barrier before the timed window')
      if WITHHOLD_RANK == dist.get_rank(pg):
        time.sleep(DEADLINE_S + 60)     # rehearsal only: this rank never joins the barrier
      dist.barrier()
    torch.cuda.synchronize()
    if probe is not None:
      probe('before')
    phase('the timed window (%d steps, each with its fc / conv bucket all-reduces)' % steps)
    t0 = time.perf_counter()
    grad_steps(steps)
    torch.cuda.synchronize()
    if pg is not None:
      phase('the barrier after the timed window')
      dist.barrier()
    elapsed = time.perf_counter() - t0
    if probe is not None:
      probe('after')
    if deadline is not None:
      deadline.done()
  finally:
    gc.enable()
  return elapsed, prime


def other_configs(device, steps):
  """Supplementary, rank 0 at N = 1: BASELINE configs 2 and 5 on their own synthetic 1M
  buffers, same protocol as the headline (so the driver's run clocks them too)."""
  res = {}
  for name, make, A, n in (('dqn_pong', build_dqn_pong, 6, max(steps, 1000)),
                           ('iqn_breakout', build_iqn_breakout, 4, max(steps // 3, 50))):
    agent = make(device)
    import random
    random.seed(0)
    fill_synthetic(agent._replay.memory, A, seed=1)
    torch.cuda.synchronize()
    elapsed, prime = timed_steps(agent, n, 10)
    agent._replay.memory.sync_rng()
    loss = agent.mean_loss()
    assert np.isfinite(loss), 'non-finite loss (%s)' % name
    res[name] = {'value': round(n / elapsed, 2), 'unit': 'gradient-steps/s', 'steps': n,
                 'ms_per_step': round(1e3 * elapsed / n, 4), 'batch': agent._batch_size,
                 'final_mean_loss': round(loss, 8)}
    if name == 'dqn_pong' and agent._chunk_gathers():
      # the learner loop's chunk gather: one K * B launch per chunk (K = 4), timed as the
      # headline's gather is (standalone launches, fresh random indices, HIP events)
      kb = agent._UNROLL * agent._batch_size
      us, algo, gname = time_gather(agent, 100, batch=kb)
      gbs = algo / (us * 1e-6) / 1e9
      res[name]['chunk_gather_roofline'] = {
          'kernel': gname + ' (chunk gather, batch %d)' % kb, 'bound': 'hbm',
          'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
          'frac': round(gbs / HBM_PEAK_GBS, 4), 'algo_bytes_per_launch': algo,
          'avg_launch_us': round(us, 3)}
    del agent
    gc.collect()
    torch.cuda.empty_cache()
  res['dqn_pong']['workload'] = ('config 2: DQN Pong (6 actions), uniform replay, n=1, TF1 '
                                 'centered RMSProp, 1M-transition buffer')
  res['iqn_breakout']['workload'] = ('config 5: IQN Breakout (4 actions), N=N\'=64, K=32, n=3, '
                                     'uniform replay, Adam, 1M-transition buffer')
  # the quantile heads' big GEMMs run the split-bf16 matrix-core form (fp32 operands as
  # exact hi + mid + lo bf16 sums, six products: fp32 to rounding, not a bf16 GEMM)
  res['iqn_breakout']['gemm_form'] = ('split-bf16 x6 (fp32 to rounding) for the embedding, FC1 '
                                      'and dW1/dWe; exact f32 MFMA for dX and the torso')
  return res


def replica_verdict(agent):
  """N > 1, after a schedule's window (collective): (every replicated tensor bit-identical
  across the ranks, DQNAgent.replica_report's per-tensor report)."""
  rep = agent.replica_report()
  return all(v['in_sync'] for v in rep.values()), rep


def diagnostics(agent, waits, steps, pg, rehearse, dev):
  """N > 1: what the first multi-GPU run needs to explain itself.  Peer exchange: the
  construction-time self-test's verdict and, per rank, the microseconds per step its
  waiting blocks spent at each exchange point in the window (block 0 of each waiting op,
  100 MHz device clock) and the XCDs the last publication covered."""
  if agent._peer is None:
    return {}
  w = {}
  if 'before' in waits and 'after' in waits:
    for k in waits['after']:
      dt = waits['after'][k][0] - waits['before'][k][0]
      dn = waits['after'][k][1] - waits['before'][k][1]
      w[k] = (round(dt * 0.01 / steps, 3), round(dn / steps, 2))    # 100 MHz ticks -> us
  mine = {'wait_us_per_step': {k: v[0] for k, v in w.items()},
          'waits_per_step': {k: v[1] for k, v in w.items()},
          'xcds_seen': int(agent._peer.flags[agent._peer._lib.PEER_PUB_XCDS].item())}
  allv = [None] * dist.get_world_size(pg)
  dist.all_gather_object(allv, mine, group=pg)
  st = agent._peer.selftest
  return {'peer_wait_us_per_step': {k: [v['wait_us_per_step'].get(k) for v in allv]
                                    for k in ('grad', 'param', 'conv')},
          'peer_waits_per_step': allv[0]['waits_per_step'],
          'peer_publish_xcds': [v['xcds_seen'] for v in allv],
          'peer_selftest': ({'ok': st['ok'], 'words_per_rank': st['words_per_rank'],
                             'ms': [r['ms'] for r in st['ranks']],
                             'xcds_seen': [r['xcds_seen'] for r in st['ranks']]}
                            if 'ok' in st else st)}


def pick_headline(schedules):
  """The fastest schedule that ran on every rank with its replicas in sync (a failed or
  diverged schedule carries 'error' and no '_elapsed')."""
  timed = [k for k in schedules if '_elapsed' in schedules[k] and 'error' not in schedules[k]]
  if not timed:
    raise RuntimeError('every data-parallel schedule failed: %r' % schedules)
  return min(timed, key=lambda k: schedules[k]['_elapsed'])


def time_gather(agent, iters, batch=None):
  """Average duration of the gather kernel, HIP events on the launch stream,
  back-to-back launches captured in a HIP graph (no host launch gaps).  batch: the launch's
  batch (default the agent's; the DQN learner loop's chunk gather launches K * B)."""
  from dopamine_amd import _lib
  mem = agent._replay.memory
  B = batch or agent._batch_size
  out = agent._replay._out if B == agent._batch_size else mem._alloc_batch(B, agent._replay._layout)
  layout = agent._replay._layout
  stream = torch.cuda.current_stream()
  # a fresh random index batch per launch: 400 x 1.8 MB of frames (> the 256 MB
  # Infinity Cache), so every launch reads cold frames as in the learner step
  C = mem._replay_capacity
  gen = torch.Generator(device='cpu').manual_seed(11)
  sets = torch.randint(mem._stack_size, C - mem._update_horizon - 1, (iters, B), generator=gen,
                       dtype=torch.int32).to(torch.cuda.current_device())
  idx = sets[0]
  for _ in range(10):
    mem._gather(idx, B, layout, out)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for i in range(iters):
      mem._gather(sets[i], B, layout, out)
  g.replay()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  e0.record(stream)
  g.replay()
  e1.record(stream)
  e1.synchronize()
  graph_us = e0.elapsed_time(e1) * 1e3 / iters
  # (no eager comparison loop: under rocprofv3 --stats this kernel's rows are then exactly
  # the 10 warm-up launches and the 2 x iters graph launches timed here)
  S, obs = mem._stack_size, mem._obs_bytes
  algo_bytes = B * (2 * S * obs + 2 * S * obs * 4)   # u8 frames read + fp32 NCHW written
  name = {_lib.LAYOUT_F32_NHWC: 'k_gather_nhwc4', _lib.LAYOUT_F32_NORM: 'k_gather_f32'}[layout]
  return graph_us, algo_bytes, name


def time_gather_large(agent, batch=1024, iters=50):
  """Supplementary: the same gather kernel at batch 1024 (distinct random valid
  indices), where it is no longer launch/latency bound -- what the kernel design
  reaches on HBM.  Not the bench workload; reported beside ``roofline``."""
  mem = agent._replay.memory
  layout = agent._replay._layout
  C = mem._replay_capacity
  gen = torch.Generator(device='cpu').manual_seed(7)
  idx = torch.randint(mem._stack_size, C - mem._update_horizon - 1, (batch,), generator=gen,
                      dtype=torch.int32).to(torch.cuda.current_device())
  out = mem._alloc_batch(batch, layout)
  stream = torch.cuda.current_stream()
  for _ in range(3):
    mem._gather(idx, batch, layout, out)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(iters):
      mem._gather(idx, batch, layout, out)
  g.replay()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  e0.record(stream)
  g.replay()
  e1.record(stream)
  e1.synchronize()
  us = e0.elapsed_time(e1) * 1e3 / iters
  S, obs = mem._stack_size, mem._obs_bytes
  algo = batch * (2 * S * obs + 2 * S * obs * 4)
  del out
  return {'batch': batch, 'avg_launch_us': round(us, 3), 'algo_bytes_per_launch': algo,
          'achieved_GBs': round(algo / (us * 1e-6) / 1e9, 1),
          'frac': round(algo / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}


def gather_traffic(batch):
  """HBM bytes per gather launch from the committed PMC passes (rocprofv3 --pmc
  FETCH_SIZE / WRITE_SIZE, calibrated as MI355X_MICROARCH.md prescribes;
  tools/gpu_gather_pmc.sh + tools/gather_traffic.py): the newest of
  profiles/r<N>_gather_traffic.json, or None."""
  import glob
  paths = sorted(glob.glob(os.path.join(ROOT, 'profiles', 'r*_gather_traffic.json')),
                 key=lambda q: int(os.path.basename(q)[1:].split('_')[0]))
  for path in reversed(paths):
    try:
      d = json.load(open(path))
      return round(float(d['traffic_bytes_per_launch'][str(batch)])), os.path.relpath(path, ROOT)
    except (OSError, KeyError, ValueError):
      continue
  return None, None


FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense


def step_mfma(actions, batch, sec_per_step):
  """Algorithmic FLOPs of one Rainbow step's Nature-CNN work -- online forward + backward
  (conv1's input gradient is never formed) + the target forward -- per second, against
  the fp32 matrix peak."""
  macs = [21 * 21 * 32 * 8 * 8 * 4, 11 * 11 * 64 * 4 * 4 * 32, 11 * 11 * 64 * 3 * 3 * 64,
          7744 * 512, 512 * actions * 51]
  fwd = 2 * sum(macs) * batch
  bwd = 2 * (2 * sum(macs) - macs[0]) * batch
  flops = 2 * fwd + bwd
  achieved = flops / sec_per_step / 1e12
  return {'flops_per_step': flops, 'achieved': round(achieved, 2), 'peak': FP32_MFMA_PEAK_TFLOPS,
          'unit': 'TFLOP/s', 'frac': round(achieved / FP32_MFMA_PEAK_TFLOPS, 4)}


def bf16_child(args):
  """In a child process on the bf16 build (DOPAMINE_AMD_LIB = the bf16 library): the
  headline's Rainbow agent and config 5's IQN, same protocol; one JSON line."""
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(0)
  from dopamine_amd import _lib
  res = {'library': os.path.relpath(_lib.LIB_PATH, ROOT)}
  import random
  for name, make, A, n in (
      ('rainbow', lambda: build_agent(args.actions, args.capacity, args.batch, dev), args.actions,
       args.steps),
      ('iqn_breakout', lambda: build_iqn_breakout(dev), 4, max(args.steps // 3, 50))):
    agent = make()
    random.seed(0)
    fill_synthetic(agent._replay.memory, A, seed=1)
    torch.cuda.synchronize()
    elapsed, _ = timed_steps(agent, n, 10 if name != 'rainbow' else args.warmup)
    agent._replay.memory.sync_rng()
    loss = agent.mean_loss()
    res[name] = {'value': round(n / elapsed, 2), 'unit': 'gradient-steps/s', 'steps': n,
                 'ms_per_step': round(1e3 * elapsed / n, 4), 'final_mean_loss': round(loss, 8),
                 'finite': bool(np.isfinite(loss))}
    del agent
    gc.collect()
    torch.cuda.empty_cache()
  print(json.dumps(res), flush=True)


def bf16_throughput(args):
  """BASELINE.md §4's separate throughput row, timed by the driver's run of this script:
  the same agents on the bf16 build (dopamine_amd/libdopamine_amd_bf16.so, built by
  __graft_entry__.build()), in a child process after this one has released the GPU.
  NOT the headline and NOT fp32 parity: one bf16 product per MFMA (fp32 accumulate)
  fails the 1e-5 tests by construction."""
  import subprocess
  from dopamine_amd import _build
  base = {'dtype': 'bf16 (fp32 accumulate)',
          'parity': 'fails the fp32 1e-5 parity tests by construction; a throughput row '
                    'beside the fp32 headline, not a supported mode',
          'gemm_form': 'one v_mfma_f32_32x32x16_bf16 product (hi.hi) in every Nature-CNN '
                       'wave-private tile and the IQN heads\' split GEMMs '
                       '(-DDQ_CNN_X6=1 -DDQ_X6_PAIRS=1)'}
  if not os.path.exists(_build.BF16_LIB_PATH):
    return dict(base, error='bf16 library not built (__graft_entry__.build())')
  env = dict(os.environ, DOPAMINE_AMD_LIB=_build.BF16_LIB_PATH)
  cmd = [sys.executable, os.path.abspath(__file__), '--bf16-child', '--steps', str(args.steps),
         '--warmup', str(args.warmup), '--capacity', str(args.capacity), '--batch',
         str(args.batch), '--actions', str(args.actions)]
  try:
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else ''
    return dict(base, **json.loads(line)) if out.returncode == 0 else dict(
        base, error='child rc %d: %s' % (out.returncode, out.stderr[-500:]))
  except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
    return dict(base, error=repr(e)[:500])


def host_cores():
  """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota."""
  n = len(os.sched_getaffinity(0))
  try:
    quota, period = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
    if quota != 'max':
      n = min(n, max(1, -(-int(quota) // int(period))))
  except (OSError, ValueError):
    pass
  return n


def cpu_model():
  try:
    for line in open('/proc/cpuinfo'):
      if line.startswith('model name'):
        return line.split(':', 1)[1].strip()
  except OSError:
    pass
  return platform.processor() or platform.machine()


def cpu_baseline(seconds, A, batch):
  from oracle.cpu_step import CpuRainbowStep
  threads = host_cores()
  torch.set_num_threads(threads)
  step = CpuRainbowStep(capacity=1_000_000, batch_size=batch, num_actions=A)
  rate, k, dt = step.time(seconds=seconds)
  return {'value': round(rate, 3), 'unit': 'gradient-steps/s', 'cores': threads, 'kind': 'port',
          'sample': '%d Rainbow steps (%.1f s): oracle numpy PER sampler on a 1M buffer + torch-CPU '
                    'Nature-CNN fwd/bwd (%d threads) + oracle C51 loss + oracle TF1 Adam; host: %s, '
                    '%d CPUs available to this process (affinity/cgroup), %d online' %
                    (k, dt, threads, cpu_model(), threads, os.cpu_count() or 0)}


# constructor overrides of the benchmarked agent and a note of changed agent-class
# attributes: both empty for the bench line (the product defaults); tools/bench_ab.py sets
# schedule experiments here and on the agent classes
AGENT_OVERRIDES = {}
CLASS_OVERRIDES = {}


def main(argv=None):
  args = parse(argv)
  if args.bf16_child:
    return bf16_child(args)
  world = int(os.environ.get('WORLD_SIZE', '1'))
  rank = int(os.environ.get('RANK', '0'))
  local = int(os.environ.get('LOCAL_RANK', '0'))
  # DQ_BENCH_REHEARSE=1: every rank on cuda:0 over gloo -- a one-GPU rehearsal of
  # the N-rank code path (schedule, barriers, max-over-ranks timing), not a measurement
  rehearse = os.environ.get('DQ_BENCH_REHEARSE') == '1'
  if rehearse:
    local = 0
  torch.cuda.set_device(local)
  dev = torch.device('cuda', local)
  pg = deadline = None
  if world > 1 or args.force_dist:
    from dopamine_amd import parallel
    deadline = parallel.Deadline(rank)
    deadline.phase('init_process_group (rendezvous at %s:%s)' % (
        os.environ.get('MASTER_ADDR', '127.0.0.1'), os.environ.get('MASTER_PORT', '?')), DEADLINE_S)
  if world > 1:
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    if rehearse:
      dist.init_process_group('gloo')
    else:
      dist.init_process_group('nccl', device_id=dev)
    pg = dist.group.WORLD
  elif args.force_dist:
    parallel.FORCE_COLLECTIVES = True
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29533')
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    pg = dist.group.WORLD
  # N > 1: the data-parallel schedules are timed one after the other on fresh
  # agents, and the headline is the fastest (every one is reported)
  names = ['single'] if pg is None else (args.schedules or 'peer,allreduce').split(',')
  first_clean = pg is not None and args.schedules is None   # the default: stop at the first clean one
  kwargs_of = {'single': {}, 'peer': {'exchange': 'peer'}, 'allreduce': {},
               'zero1': {'shard_optimizer': True}}
  assert all(n in kwargs_of for n in names), names
  schedules = {}
  agent = None
  for name in names:
    if first_clean and any('_elapsed' in v for v in schedules.values()):
      schedules[name] = {'skipped': 'an earlier schedule ran cleanly on every rank'}
      continue
    if agent is not None:
      agent.close()                   # its RCCL communicators (N > 1) before the next pair
      del agent
      gc.collect()
      torch.cuda.empty_cache()
    if deadline is not None:
      deadline.phase('building the %s learner (RCCL communicators or peer mappings, rank-0 '
                     'broadcast)' % name, DEADLINE_S)
    try:
      agent = build_agent(args.actions, args.capacity, args.batch, dev, pg=pg,
                          use_hip_graph=not args.no_graph, native_comm=args.comm == 'native',
                          **AGENT_OVERRIDES, **kwargs_of[name])
    except RuntimeError as e:
      # the peer exchange's placement check (PeerExchange.available) is collective: every
      # rank gets the same answer, so every rank skips the schedule together
      if name != 'peer' or len(names) == 1:
        raise
      agent = None
      schedules[name] = {'error': str(e)}
      print('bench: rank %d: schedule peer unavailable: %s' % (rank, e), file=sys.stderr)
      if deadline is not None:
        deadline.done()
      continue
    import random
    random.seed(0 + rank)
    fill_synthetic(agent._replay.memory, args.actions, seed=1 + rank)
    torch.cuda.synchronize()
    if pg is not None:       # the ranks fill their buffers at their own pace; start together
      deadline.phase('the barrier after the replay fill', DEADLINE_S)
      dist.barrier()
      deadline.done()
    waits = {}

    def probe(when):
      if agent._peer is not None:
        waits[when] = agent._peer.wait_counters()
    elapsed, prime = timed_steps(agent, args.steps, args.warmup, args.per_call, pg, deadline,
                                 probe)
    per_rank = [elapsed]
    if pg is not None:
      deadline.phase('the all_reduce of the per-rank times', DEADLINE_S)
      t = torch.zeros(dist.get_world_size(pg), dtype=torch.float64,
                      device='cpu' if rehearse else dev)
      t[dist.get_rank(pg)] = elapsed
      dist.all_reduce(t, op=dist.ReduceOp.SUM)
      per_rank = [float(x) for x in t.cpu()]
      elapsed = max(per_rank)
      deadline.done()
    agent._replay.memory.sync_rng()   # raises if the device latched a sampling error
    try:
      loss, err = agent.mean_loss(), None     # raises if a peer-exchange wait timed out
    except RuntimeError as e:
      loss, err = float('nan'), str(e)
    if pg is not None and len(names) > 1:
      # every rank drops a schedule that failed on any rank (each rank's bounded waits end
      # its window, so all ranks reach this point) and the next one is timed
      deadline.phase('agreeing on the %s schedule\'s errors' % name, DEADLINE_S)
      f = torch.tensor([0 if err is None else 1], dtype=torch.int32,
                       device='cpu' if rehearse else dev)
      dist.all_reduce(f, op=dist.ReduceOp.MAX)
      deadline.done()
      if int(f.item()):
        schedules[name] = {'error': err or 'failed on another rank'}
        print('bench: rank %d: schedule %s failed: %s' % (rank, name, schedules[name]['error']),
              file=sys.stderr)
        continue
    if err is not None:
      raise RuntimeError(err)
    assert np.isfinite(loss), 'non-finite loss'
    entry = {
        'value': round(world * args.steps / elapsed, 2), 'ms_per_step': round(1e3 * elapsed / args.steps, 4),
        'per_rank_ms_per_step': [round(1e3 * e / args.steps, 4) for e in per_rank],
        'prime_steps': prime, 'final_mean_loss': round(loss, 8), '_elapsed': elapsed,
        'comm': ('peer memory (one stream)' if agent._peer is not None else
                 args.comm if agent._rccl is not None or args.comm == 'torch' else 'torch')
        if pg is not None else None}
    if pg is not None:
      # the replicas must be bit-identical after the window: a schedule whose
      # replicas differ is a failed schedule, never the headline (every rank sees the report)
      deadline.phase('comparing the %s schedule\'s replicas bit for bit' % name, DEADLINE_S)
      ok, rep = replica_verdict(agent)
      entry.update(diagnostics(agent, waits, args.steps, pg, rehearse, dev))
      deadline.done()
      entry['replicas_in_sync'] = ok
      entry['replicas_compared'] = {k: v['differing'] for k, v in rep.items()}
      if not ok:
        entry['error'] = 'replicas diverged: elements differing from rank 0, per rank: %r' % {
            k: v['differing'] for k, v in rep.items() if not v['in_sync']}
        entry.pop('_elapsed')
        print('bench: rank %d: schedule %s failed: %s' % (rank, name, entry['error']),
              file=sys.stderr)
    schedules[name] = entry
  best = pick_headline(schedules)
  elapsed, prime, loss = (schedules[best]['_elapsed'], schedules[best]['prime_steps'],
                          schedules[best]['final_mean_loss'])
  for v in schedules.values():
    v.pop('_elapsed', None)

  if agent is None:                 # the last schedule could not be built: time the gather on the best's
    agent = build_agent(args.actions, args.capacity, args.batch, dev, pg=pg,
                        use_hip_graph=not args.no_graph, native_comm=args.comm == 'native',
                        **AGENT_OVERRIDES, **kwargs_of[best])
    fill_synthetic(agent._replay.memory, args.actions, seed=1 + rank)
  graph_us, algo_bytes, gname = time_gather(agent, args.gather_iters)
  large = time_gather_large(agent)
  traffic, traffic_src = gather_traffic(args.batch)
  achieved = algo_bytes / (graph_us * 1e-6) / 1e9

  configs = None
  if rank == 0 and world == 1 and not args.skip_configs and not args.force_dist:
    del agent
    gc.collect()
    torch.cuda.empty_cache()
    configs = other_configs(dev, args.steps)

  bf16 = None
  if rank == 0 and world == 1 and not args.force_dist and not args.skip_bf16:
    agent = None
    gc.collect()
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    bf16 = bf16_throughput(args)

  cpu = None
  if rank == 0 and world == 1 and not args.skip_cpu_baseline:
    cpu = cpu_baseline(args.cpu_seconds, args.actions, args.batch)

  if rank == 0:
    from dopamine_amd import _lib
    value = world * args.steps / elapsed
    line = {
        'metric': 'gradient-steps/sec (Rainbow, batch=32, 1M-transition buffer)',
        'value': round(value, 2), 'unit': 'gradient-steps/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'prime_steps': prime,
        'ms_per_step': round(1e3 * elapsed / args.steps, 4), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'fp32', 'data': 'synthetic',
        'config': {'workload': 'Rainbow/C51 Asterix (9 actions), prioritized sum-tree replay, '
                               'n=3, 1M-transition 84x84x4 uint8 buffer per GPU',
                   'global_batch': args.batch * world, 'per_gpu_batch': args.batch,
                   'replay_capacity': args.capacity,
                   'parallelism': 'dp%d' % world + (' (one-rank RCCL group, --force-dist)'
                                                    if args.force_dist and world == 1 else '')
                                  + {'zero1': ', ZeRO-1 fc bucket over RCCL',
                                     'allreduce': ', all-reduce over RCCL',
                                     'peer': ', peer-memory exchange on one stream'}.get(best, ''),
                   'hip_graph': not args.no_graph},
        'roofline': {'kernel': gname + ' (frame-stack gather + /255, state+next_state)',
                     'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4),
                     'traffic': traffic, 'traffic_source': traffic_src,
                     'algo_bytes_per_launch': algo_bytes,
                     'avg_launch_us': round(graph_us, 3),
                     'same_kernel_batch_1024': large},
        # supplementary: the whole step against the fp32 matrix peak (the CNN's fp32 MFMA
        # work; the step is launch- and latency-bound at B = 32, not MFMA-bound)
        'step_mfma': step_mfma(args.actions, args.batch, elapsed / args.steps),
        'cpu_baseline': cpu,
        'final_mean_loss': round(loss, 8),
        'gc_disabled_in_timed_window': True,
        # the library that ran: its recorded -D flags ("" = the product build; _lib refuses
        # any other unless DQ_DIAGNOSTIC_BUILD=1)
        'build': {'library': os.path.relpath(_lib.LIB_PATH, ROOT), 'flags': _lib.BUILD_FLAGS,
                  'overrides': {k: str(v) for k, v in
                                dict(AGENT_OVERRIDES, **CLASS_OVERRIDES).items()} or None},
        # N > 1 (or --force-dist): every data-parallel schedule timed, the headline the faster
        'schedules': schedules if pg is not None else None,
        # supplementary: BASELINE configs 2 and 5 (N = 1), same protocol, not the metric
        'other_configs': configs,
        # BASELINE.md §4's separate bf16 row (N = 1): NOT fp32 parity, not the headline
        'throughput_mode': bf16,
    }
    print(json.dumps(line), flush=True)
  if pg is not None:
    deadline.phase('destroy_process_group', DEADLINE_S)
    dist.destroy_process_group()
    deadline.close()


if __name__ == '__main__':
  main()
