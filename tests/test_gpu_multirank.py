"""The agent's multi-learner path end to end (BASELINE config 4's schedule:
graph replays around the gradient all-reduce), exercised on ONE GPU with two
ranks sharing cuda:0 over gloo (which all-reduces CUDA tensors).

* identical seeds on both ranks: the mean gradient equals each rank's own
  ((g + g) / 2 is exact in fp32), so after K steps the parameters must equal a
  single-process agent's BIT FOR BIT -- this pins the whole N > 1 schedule;
* different seeds: the replicas stay bit-identical (checksum broadcast);
* the learner-only loop (train_gradient_steps), whose fc all-reduce + update is
  joined in the next step, between its conv and fc launches: bitwise the same."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

STEPS = 12
CAP = 30000


def _agent(pg, seed, net_seed=0, capacity=CAP, **kw):
  from dopamine_amd.agents.optimizers import AdamOptimizer
  from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent
  import bench
  import random
  agent = RainbowAgent(num_actions=9, update_horizon=3, gamma=0.99, replay_scheme='prioritized',
                       min_replay_history=100, update_period=4, target_update_period=40,
                       optimizer=AdamOptimizer(learning_rate=6.25e-5, epsilon=1.5e-4),
                       replay_capacity=capacity, batch_size=32, device=torch.device('cuda', 0),
                       seed=net_seed, process_group=pg, **kw)
  random.seed(seed)
  bench.fill_synthetic(agent._replay.memory, 9, seed=1 + seed)
  return agent


def _run(agent, loop=False, steps=None):
  steps = STEPS if steps is None else steps
  if loop:
    agent.train_gradient_steps(steps)
  else:
    for _ in range(steps):
      for _ in range(agent.update_period):
        agent._train_step()
  torch.cuda.synchronize()
  return agent.online_convnet.fp.flat.detach().cpu().clone()


def _worker(rank, world, port, same_seed, q, loop=False, net_seed_per_rank=False, shard=False):
  import sys
  sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  torch.cuda.set_device(0)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd import parallel
  agent = _agent(dist.group.WORLD, 0 if same_seed else rank,
                 net_seed=1000 * rank if net_seed_per_rank else 0, shard_optimizer=shard)
  assert agent._sharded() == shard
  flat = _run(agent, loop)
  assert agent.graphs_primed()      # the later steps replayed the captured split graphs
  ok = parallel.replicas_in_sync(agent.online_convnet.fp.flat)
  ok = ok and parallel.replicas_in_sync(agent.target_convnet.fp.flat)
  agent._gather_opt_state()         # ZeRO-1: the moments of every slice, as a checkpoint sees them
  ok = ok and parallel.replicas_in_sync(agent._opt.m) and parallel.replicas_in_sync(agent._opt.v)
  if rank == 0:
    q.put((ok, flat.numpy(), agent._opt.m.cpu().numpy(), agent._opt.v.cpu().numpy()))
  dist.barrier()
  dist.destroy_process_group()


def _free_port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _two_ranks(same_seed, loop=False, net_seed_per_rank=False, shard=False, moments=False):
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_worker, args=(r, 2, port, same_seed, q, loop, net_seed_per_rank,
                                             shard))
           for r in range(2)]
  for p in procs:
    p.start()
  ok, flat, m, v = q.get(timeout=400)
  for p in procs:
    p.join(timeout=120)
    assert p.exitcode == 0
  return (ok, flat, m, v) if moments else (ok, flat)


@pytest.mark.timeout(600)
def test_two_ranks_same_seed_equal_single_learner_bitwise():
  ok, flat = _two_ranks(same_seed=True)
  assert ok
  single = _run(_agent(None, 0)).numpy()
  assert np.array_equal(flat, single)


@pytest.mark.timeout(600)
def test_two_ranks_different_seeds_stay_in_sync():
  ok, _ = _two_ranks(same_seed=False)
  assert ok


@pytest.mark.timeout(600)
def test_two_ranks_learner_loop_equal_single_learner_bitwise():
  ok, flat = _two_ranks(same_seed=True, loop=True)
  assert ok
  single = _run(_agent(None, 0)).numpy()
  assert np.array_equal(flat, single)


def _mean_gradient_reference(loop=False, moments=False, world=2, capacity=CAP, n_steps=None):
  """Every rank's learner in ONE process, no collective: each _train_step computes its
  own gradient (the optimizer deferred), the flat gradients are averaged in group-rank
  order ((((g0 + g1) + g2) + ...) * (1 / N), parallel.allreduce_mean_'s gloo order), and
  the TF1 Adam step is applied to that mean on every replica; target syncs run after the
  update, as in _train_step.  SURVEY 8(e): the multi-GPU gradient = the mean of the
  ranks' single-GPU gradients on their own minibatches (PER weights per rank)."""
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  import random
  agents = []
  for r in range(world):
    ag = _agent(None, r, use_hip_graph=False, fuse_optimizer=False, capacity=capacity)
    ag._replay.memory._rng.stream = random.Random(r)   # each rank's own `random`, as its process
    agents.append(ag)
  steps = []
  for ag in agents:
    ag._device_opt_step = lambda k, ag=ag: steps.append((ag, k))
    ag._sync_target = lambda ag=ag: steps.append((ag, 'sync'))
  for _ in range((STEPS if n_steps is None else n_steps) * agents[0].update_period):
    steps.clear()
    for ag in agents:
      ag._train_step()
    opt = [(ag, k) for ag, k in steps if k != 'sync']
    if opt:
      assert len(opt) == world and all(k == opt[0][1] for _, k in opt)
      g = agents[0].online_convnet.fp.grad.clone()
      for ag in agents[1:]:
        g.add_(ag.online_convnet.fp.grad)
      g.mul_(1.0 / world)
      for ag, k in opt:
        ag.online_convnet.fp.grad.copy_(g)
        ag._opt.step(ag.online_convnet.fp.grad, slot=k)
    for ag, k in steps:
      if k == 'sync':
        DQNAgent._sync_target(ag)
  torch.cuda.synchronize()
  flats = [ag.online_convnet.fp.flat.cpu().numpy() for ag in agents]
  a = flats[0]
  assert all(np.array_equal(a, b) for b in flats[1:])
  if moments:
    return a, agents[0]._opt.m.cpu().numpy(), agents[0]._opt.v.cpu().numpy()
  return a


@pytest.mark.timeout(900)
@pytest.mark.parametrize('loop', [False, True])
def test_two_ranks_different_data_equal_mean_gradient_reference(loop):
  """Different buffers AND different network seeds per rank (rank 0's networks are
  broadcast at construction): after 12 steps the parameters equal -- bit for bit --
  a single process applying TF1 Adam to the mean of the two ranks' gradients.  An
  unreduced, double-counted or mis-ordered all-reduce changes the result."""
  ok, flat = _two_ranks(same_seed=False, loop=loop, net_seed_per_rank=True)
  assert ok
  ref = _mean_gradient_reference(loop)
  assert np.array_equal(flat, ref)
  lone = _run(_agent(None, 0)).numpy()        # rank 0 alone differs: the reduction did something
  assert not np.array_equal(flat, lone)


@pytest.mark.timeout(900)
@pytest.mark.parametrize('loop', [False, True])
def test_two_ranks_sharded_optimizer_equal_mean_gradient_reference(loop):
  """ZeRO-1 (shard_optimizer): the fc bucket reduce-scattered, each rank's TF1 Adam on its
  half only, the parameters all-gathered -- different buffers and network seeds per rank:
  parameters AND (gathered) Adam moments bitwise those of the replicated mean-gradient
  update."""
  ok, flat, m, v = _two_ranks(same_seed=False, loop=loop, net_seed_per_rank=True, shard=True,
                              moments=True)
  assert ok
  ref, rm, rv = _mean_gradient_reference(loop, moments=True)
  assert np.array_equal(flat, ref)
  assert np.array_equal(m, rm) and np.array_equal(v, rv)


# ---------------------------------------------------------------- world 8 (config 4)
# BASELINE config 4 runs 8 learners, each with its own 1M-transition buffer.  One GPU holds
# all eight (8 x 7.06 GB of frames), so the world-8 path -- ZeRO-1's 8-way slicing of the
# fc bucket (a head of < 32 floats joining the conv bucket), the per-rank PER `w /= max(w)`
# (rainbow_agent.py:279-280) on 8 different buffers, the 8-rank mean -- runs here over
# gloo with every rank on cuda:0 (RCCL needs one GPU per rank).

WORLD8 = 8
CAP8 = 1_000_000


def _worker8(rank, world, port, q, variants):
  import gc
  import sys
  sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  torch.cuda.set_device(0)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd import parallel
  for shard, loop in variants:
    agent = _agent(dist.group.WORLD, rank, net_seed=1000 * rank, capacity=CAP8,
                   shard_optimizer=shard)
    assert agent._sharded() == shard
    if shard:
      lo, n = agent._shard_bounds()
      assert (n - lo) % (4 * world) == 0 and lo >= n - agent._grad_buckets()[0].numel()
    flat = _run(agent, loop)
    ok = parallel.replicas_in_sync(agent.online_convnet.fp.flat)
    ok = ok and parallel.replicas_in_sync(agent.target_convnet.fp.flat)
    agent._gather_opt_state()
    ok = ok and parallel.replicas_in_sync(agent._opt.m) and parallel.replicas_in_sync(agent._opt.v)
    if rank == 0:
      q.put((shard, loop, ok, flat.numpy(), agent._opt.m.cpu().numpy(),
             agent._opt.v.cpu().numpy()))
      print('world 8: shard=%s loop=%s done' % (shard, loop), flush=True)   # progress (-s)
    del agent
    gc.collect()
    torch.cuda.empty_cache()
    dist.barrier()
  dist.destroy_process_group()


@pytest.mark.timeout(1200)
def test_world8_on_one_gpu_equals_mean_gradient_reference():
  """Config 4's world size on one GPU: 8 gloo ranks sharing cuda:0, each with a 1M buffer,
  its own data and network seed; the replicated all-reduce and ZeRO-1 schedules, per-call
  and learner-loop drives, 12 gradient steps each.  Parameters and gathered Adam moments
  equal, bit for bit, ONE process applying TF1 Adam to the rank-ordered mean of the 8
  ranks' gradients, and the replicas stay in sync."""
  variants = [(False, False), (False, True), (True, False), (True, True)]
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_worker8, args=(r, WORLD8, port, q, variants))
           for r in range(WORLD8)]
  for p in procs:
    p.start()
  got = {}
  for _ in variants:
    shard, loop, ok, flat, m, v = q.get(timeout=900)
    got[(shard, loop)] = (ok, flat, m, v)
  for p in procs:
    p.join(timeout=120)
    assert p.exitcode == 0
  ref, rm, rv = _mean_gradient_reference(moments=True, world=WORLD8, capacity=CAP8)
  for key in variants:
    ok, flat, m, v = got[key]
    assert ok, key
    assert np.array_equal(flat, ref), key
    assert np.array_equal(m, rm) and np.array_equal(v, rv), key


# ------------------------------------------------------- N > 1 checkpoints (rank-safe)
CKPT_CAP = 5000


def _ckpt_worker(rank, world, port, ckdir, q, shard):
  import random
  import sys
  sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  torch.cuda.set_device(0)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd import parallel

  def steps(agent, n):
    for _ in range(n * agent.update_period):
      agent._train_step()
    torch.cuda.synchronize()
    return agent.online_convnet.fp.flat.detach().cpu().numpy().copy()

  agent = _agent(dist.group.WORLD, rank, net_seed=1000 * rank, capacity=CKPT_CAP,
                 shard_optimizer=shard)
  steps(agent, 6)
  bundle = agent.bundle_and_checkpoint(ckdir, 3)
  files = sorted(os.listdir(os.path.join(ckdir, 'rank%d' % rank)))
  # the continuation: the same RNG state as a resumed process will set
  agent._discard_prefetch()
  agent._replay.memory.sync_rng()
  random.seed(500 + rank)
  cont = steps(agent, 6)
  cont_ok = parallel.replicas_in_sync(agent.online_convnet.fp.flat)
  del agent
  # a fresh learner with other data and networks, resumed from this rank's files
  agent = _agent(dist.group.WORLD, 100 + rank, net_seed=7 + rank, capacity=CKPT_CAP,
                 shard_optimizer=shard)
  assert agent.unbundle(ckdir, 3, bundle)
  random.seed(500 + rank)
  res = steps(agent, 6)
  res_ok = parallel.replicas_in_sync(agent.online_convnet.fp.flat)
  q.put((rank, files, bundle['training_steps'], cont, res, cont_ok and res_ok))
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.timeout(900)
@pytest.mark.parametrize('shard', [False, True])
def test_two_ranks_checkpoint_resume_is_rank_safe(tmp_path, shard):
  """bundle_and_checkpoint at world 2 writes each rank's files under checkpoint_dir/rank<r>
  (each rank's own 1M buffer and sum tree; the replicas' networks and Adam state, gathered
  first under ZeRO-1); fresh learners built with other data and networks unbundle from
  there and then train bit for bit as the original learners continue."""
  ckdir = str(tmp_path)
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_ckpt_worker, args=(r, 2, port, ckdir, q, shard)) for r in range(2)]
  for p in procs:
    p.start()
  res = dict((r, rest) for r, *rest in (q.get(timeout=600) for _ in range(2)))
  for p in procs:
    p.join(timeout=120)
    assert p.exitcode == 0
  assert sorted(os.listdir(ckdir)) == ['rank0', 'rank1']
  for r in range(2):
    files, tsteps, cont, resumed, ok = res[r]
    assert ok
    assert 'tf_ckpt-3' in files and any(f.startswith('$store$_observation_ckpt.3') for f in files)
    assert tsteps == 6 * 4
    assert np.array_equal(cont, resumed), r
  # the two ranks' buffers differ (their own data), and their replicas agree
  assert np.array_equal(res[0][2], res[1][2])
  import gzip
  obs = [gzip.open(os.path.join(ckdir, 'rank%d' % r, '$store$_observation_ckpt.3.gz')).read()
         for r in range(2)]
  assert obs[0] != obs[1]
