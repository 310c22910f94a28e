"""Multi-learner data-parallel path on CPU with gloo, world_size 2 (config 4's
exchange step).  Parity definition: the multi-GPU gradient is the
mean over ranks of each rank's single-learner gradient on its own minibatch
(PER weights normalised per rank); identical TF1 Adam updates keep the
replicas bit-identical."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import learner as OL

B, A, N = 8, 9, 51


def _rank_grad(rank, net):
  rs = np.random.RandomState(100 + rank)
  st = torch.from_numpy(rs.rand(B, 4, 84, 84).astype(np.float32))
  tl = rs.randn(B, A, N).astype(np.float32)
  logits = net(st)
  out = OL.c51_loss(logits.detach().numpy(), tl, rs.randint(0, A, B), rs.randn(B).astype(np.float32),
                    (rs.rand(B) < 0.2).astype(np.uint8), OL.c51_support(10.0, N), np.float32(0.97),
                    rs.uniform(0.1, 2, B).astype(np.float32), dtype=np.float32)
  net.fp.grad.zero_()
  logits.backward(torch.from_numpy(out['grad'].astype(np.float32)))
  return net.fp.grad.clone()


def _worker(rank, world, port, q):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  torch.set_num_threads(1)
  from dopamine_amd import parallel
  from dopamine_amd.agents.networks import RainbowNetwork
  net = RainbowNetwork(A, device='cpu', seed=0)          # same init on every rank
  adam = OL.TF1Adam(net.fp.numel, 6.25e-5, eps=1.5e-4)
  params = net.fp.flat.numpy()
  for step in range(2):
    g = _rank_grad(rank + 10 * step, net)
    net.fp.grad.copy_(g)
    parallel.allreduce_mean_(net.fp.grad)
    adam.step(params, net.fp.grad.numpy())
  in_sync = parallel.replicas_in_sync(net.fp.flat)
  if rank == 0:
    q.put((in_sync, net.fp.flat.numpy().copy()))    # by value: the child may exit first
  dist.barrier()
  dist.destroy_process_group()


def _free_port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


@pytest.mark.timeout(300)
def test_two_rank_allreduce_matches_mean_gradient():
  world = 2
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
  for p in procs:
    p.start()
  in_sync, flat = q.get(timeout=240)
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  assert in_sync
  # single-process restatement: mean of the two ranks' gradients, same Adam
  from dopamine_amd.agents.networks import RainbowNetwork
  net = RainbowNetwork(A, device='cpu', seed=0)
  adam = OL.TF1Adam(net.fp.numel, 6.25e-5, eps=1.5e-4)
  params = net.fp.flat.numpy()
  for step in range(2):
    g = sum(_rank_grad(r + 10 * step, net) for r in range(world)) / world
    adam.step(params, g.numpy())
  np.testing.assert_allclose(flat, params, rtol=1e-6, atol=1e-9)


def _shard_worker(rank, world, port, q):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd import parallel
  n = 4 * world * 5
  g = torch.arange(n, dtype=torch.float32) * (rank + 1)
  parallel.reduce_scatter_mean_(g)
  S = n // world
  mine = g[rank * S:(rank + 1) * S].clone()          # this rank's slice of the mean
  p = torch.full((n,), -1.0)
  p[rank * S:(rank + 1) * S] = mine * 10 + rank       # the owner's update of its slice
  parallel.all_gather_(p)
  q.put((rank, mine.numpy(), p.numpy()))     # by value: the child may exit before the read
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_reduce_scatter_and_all_gather_slices():
  """The ZeRO-1 pair (parallel.reduce_scatter_mean_ / all_gather_): rank r holds the mean
  of slice r, and after each owner rewrites its slice every rank holds all of them."""
  world = 2
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
  for p in procs:
    p.start()
  res = dict((r, (m, p)) for r, m, p in (q.get(timeout=240) for _ in range(world)))
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  n = 4 * world * 5
  S = n // world
  mean = torch.arange(n, dtype=torch.float32) * sum(r + 1 for r in range(world)) / world
  want = torch.cat([mean[r * S:(r + 1) * S] * 10 + r for r in range(world)])
  for r in range(world):
    assert np.array_equal(res[r][0], mean[r * S:(r + 1) * S].numpy())
    assert np.array_equal(res[r][1], want.numpy())


def _order_worker(rank, world, port, q):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd import parallel
  g = torch.from_numpy(np.random.RandomState(rank).standard_normal(4099).astype(np.float32) *
                       np.float32(10.0 ** (rank - 2)))
  parallel.allreduce_mean_(g)
  q.put((rank, g.numpy().copy()))
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_mean_is_the_rank_ordered_sum_bitwise():
  """Over gloo (the multi-rank tests' backend) the mean is (((g0 + g1) + g2) + g3) * 1/4 on
  every rank -- the order a single-process reference restates bit for bit at any world size
  (tests/test_gpu_multirank.py's world-8 test depends on it)."""
  world = 4
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_order_worker, args=(r, world, port, q)) for r in range(world)]
  for p in procs:
    p.start()
  res = dict(q.get(timeout=240) for _ in range(world))
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  gs = [np.random.RandomState(r).standard_normal(4099).astype(np.float32) *
        np.float32(10.0 ** (r - 2)) for r in range(world)]
  acc = gs[0].copy()
  for g in gs[1:]:
    acc = acc + g
  want = acc * np.float32(1.0 / world)
  for r in range(world):
    assert np.array_equal(res[r], want)
  other = ((gs[3] + gs[2]) + gs[1]) + gs[0]          # the order matters for these inputs
  assert not np.array_equal(other * np.float32(1.0 / world), want)


def _rank_dir_worker(rank, world, port, q):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  import types
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  got = DQNAgent._rank_dir(types.SimpleNamespace(_pg=dist.group.WORLD), '/ck')
  alone = DQNAgent._rank_dir(types.SimpleNamespace(_pg=None), '/ck')
  q.put((rank, got, alone))
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_data_parallel_checkpoints_go_to_rank_directories():
  """bundle_and_checkpoint / unbundle's directory (DQNAgent._rank_dir): a data-parallel rank
  writes under checkpoint_dir/rank<r> (its own buffer; the reference's names would collide
  in a shared directory), a single replica into checkpoint_dir itself as the reference."""
  world = 2
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_rank_dir_worker, args=(r, world, port, q)) for r in range(world)]
  for p in procs:
    p.start()
  res = dict((r, (g, a)) for r, g, a in (q.get(timeout=240) for _ in range(world)))
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  for r in range(world):
    assert res[r] == (os.path.join('/ck', 'rank%d' % r), '/ck')


# ---------------------------------------------------------------- N > 1 deadline
def _deadline_worker(rank, world, port, path, withhold):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd import parallel
  import time
  if rank == withhold:            # this rank never enters the collective
    time.sleep(30)
    os._exit(0)
  dl = parallel.Deadline(rank, out=open(path % rank, 'w'))
  dl.phase('the fc bucket all_reduce of step 7', 3)
  t = torch.ones(4)
  dist.all_reduce(t)              # blocks: the peer withholds it; the deadline ends us
  os._exit(0)                     # not reached


@pytest.mark.timeout(120)
def test_deadline_reports_rank_and_collective_and_exits(tmp_path):
  """parallel.Deadline (bench.py's N > 1 phases): a rank blocked in a collective that a
  peer withholds reports which rank and which phase, and exits with DEADLINE_EXIT instead
  of hanging."""
  from dopamine_amd import parallel
  ctx = mp.get_context('spawn')
  port = _free_port()
  path = str(tmp_path / 'dl_%d.txt')
  procs = [ctx.Process(target=_deadline_worker, args=(r, 2, port, path, 1)) for r in range(2)]
  for p in procs:
    p.start()
  procs[0].join(timeout=90)
  assert procs[0].exitcode == parallel.DEADLINE_EXIT
  msg = open(path % 0).read()
  assert 'rank 0: the fc bucket all_reduce of step 7 did not complete within 3 s' in msg, msg
  procs[1].kill()
  procs[1].join(timeout=30)


def test_deadline_disarmed_never_fires():
  import time
  from dopamine_amd import parallel
  dl = parallel.Deadline(0, poll=0.01)
  dl.phase('short phase', 0.05)
  dl.done()
  time.sleep(0.2)                 # would have expired had it stayed armed
  dl.close()


# ------------------------------------------------- rank-aware Runner checkpoints
class _StubAgent(object):
  """The agent interface the Runner uses (bundle / unbundle / step), with a process group:
  per-rank state, files under checkpoint_dir/rank<r> as DQNAgent._rank_dir."""

  def __init__(self, pg):
    self._pg = pg
    self.eval_mode = False
    self.state = np.zeros(1)
    self.training_steps = 0

  def _rank_dir(self, d):
    return os.path.join(d, 'rank%d' % dist.get_rank(self._pg))

  def begin_episode(self, obs):
    return 0

  def step(self, r, obs):
    self.training_steps += 1 + dist.get_rank(self._pg)    # ranks diverge
    return 0

  def end_episode(self, r):
    pass

  def bundle_and_checkpoint(self, d, it):
    os.makedirs(self._rank_dir(d), exist_ok=True)
    return {'training_steps': self.training_steps}

  def unbundle(self, d, it, bundle):
    if bundle is None:
      return False
    self.training_steps = bundle['training_steps']
    return True


class _Env(object):
  game_over = False

  class action_space(object):
    n = 2

  def reset(self):
    return np.zeros(4)

  def step(self, a):
    return np.zeros(4), 1.0, False, {}


def _runner_worker(rank, world, port, base, q, iters, drop_last_on):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd.discrete_domains import run_experiment
  pg = dist.group.WORLD
  mk = lambda sess, env, summary_writer=None: _StubAgent(pg)
  r = run_experiment.Runner(base, mk, _Env, num_iterations=iters, training_steps=5,
                            evaluation_steps=0, max_steps_per_episode=5)
  start = r._start_iteration
  r.run_experiment()
  ck = os.path.join(base, 'checkpoints', 'rank%d' % rank)
  if rank == drop_last_on:          # this rank "crashed" before its last sentinel landed
    os.remove(os.path.join(ck, 'sentinel_checkpoint_complete.%d' % (iters - 1)))
  q.put((rank, start, r._agent.training_steps, sorted(os.listdir(ck)),
         sorted(os.listdir(os.path.join(base, 'checkpoints')))))
  dist.barrier()
  dist.destroy_process_group()


def _runner_round(base, iters, drop_last_on=-1):
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_runner_worker, args=(r, 2, port, base, q, iters, drop_last_on))
           for r in range(2)]
  for p in procs:
    p.start()
  res = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in range(2)))
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  return res


@pytest.mark.timeout(300)
def test_two_rank_runner_checkpoints_are_per_rank_and_resume_together(tmp_path):
  """Runner with data-parallel learners: each rank's ckpt.N and sentinel go to
  checkpoints/rank<r> (its own runner state), logs only from rank 0, and on resume the
  ranks agree on the newest iteration EVERY rank completed."""
  base = str(tmp_path / 'run')
  res = _runner_round(base, 3, drop_last_on=1)
  for r in (0, 1):
    start, steps, files, top = res[r]
    assert start == 0 and top == ['rank0', 'rank1']
    assert 'ckpt.2' in files
  assert res[0][1] != res[1][1]                       # per-rank states differ
  assert 'sentinel_checkpoint_complete.2' not in res[1][2]
  # resume: rank 1 lacks iteration 2's sentinel, so both ranks restart after iteration 1
  res2 = _runner_round(base, 4)
  assert res2[0][0] == 2 and res2[1][0] == 2
  logs = sorted(os.listdir(os.path.join(base, 'logs')))
  assert logs and all(f.startswith('log_') for f in logs)


# ------------------------------------------------- replica verdict of the N > 1 bench
def _replica_worker(rank, world, port, q):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd import parallel
  g = torch.Generator().manual_seed(3)
  a = torch.randn(1000, generator=g)
  b = torch.randn(333, generator=g).double()
  same = parallel.replica_report({'online': a, 'opt_state': b})
  a2 = a.clone()
  if rank == 1:
    a2[417] = float('nan')        # a diverged replica (NaN-safe: bits compared, not values)
    a2[5] += 1e-7
  diverged = parallel.replica_report({'online': a2, 'opt_state': b})
  q.put((rank, same, diverged))
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_replica_report_finds_a_diverged_replica_bit_for_bit():
  """after each N > 1 schedule's window bench.py compares every replicated
  tensor with group rank 0's bit for bit; a replica that differs in two elements (one of them a
  NaN) is reported on every rank with its per-rank counts."""
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_replica_worker, args=(r, 2, port, q)) for r in range(2)]
  for p in procs:
    p.start()
  res = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in range(2)))
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  for r in (0, 1):
    same, diverged = res[r]
    assert all(v['in_sync'] and v['differing'] == [0, 0] for v in same.values())
    assert not diverged['online']['in_sync'] and diverged['online']['differing'] == [0, 2]
    assert diverged['online']['max_abs_diff'][1] == float('inf')
    assert diverged['opt_state']['in_sync']


def test_bench_headline_skips_failed_and_diverged_schedules():
  """bench.py's headline is the fastest schedule that ran with its replicas in sync: a faster
  schedule whose replicas diverged (or that failed on a rank) is never the headline."""
  import bench
  s = {'peer': {'value': 9.0, 'error': 'replicas diverged: ...', 'replicas_in_sync': False},
       'allreduce': {'value': 6.0, '_elapsed': 2.0, 'replicas_in_sync': True},
       'zero1': {'error': 'failed on another rank'}}
  assert bench.pick_headline(s) == 'allreduce'
  s['peer'] = {'value': 9.0, '_elapsed': 1.0, 'replicas_in_sync': True}
  assert bench.pick_headline(s) == 'peer'
  with pytest.raises(RuntimeError):
    bench.pick_headline({'peer': {'error': 'x'}})


class _ExchangingStub(_StubAgent):
  exchange = 'collective'


def _refuse_worker(rank, world, port, base, q):
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd.discrete_domains import run_experiment
  pg = dist.group.WORLD
  try:
    run_experiment.Runner(base, lambda sess, env, summary_writer=None: _ExchangingStub(pg), _Env,
                          num_iterations=1, training_steps=5, evaluation_steps=0)
    q.put((rank, None))
  except ValueError as e:
    q.put((rank, str(e)))
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_runner_refuses_data_parallel_learners(tmp_path):
  """the Runner's whole-episode phases cannot keep data-parallel learners' gradient
  steps in step across ranks, so it refuses them at construction on every rank (instead of
  a wait timing out or collectives pairing up wrongly mid-run)."""
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_refuse_worker, args=(r, 2, port, str(tmp_path / 'run'), q))
           for r in range(2)]
  for p in procs:
    p.start()
  res = dict(q.get(timeout=120) for _ in range(2))
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  assert all(res[r] and 'train_gradient_steps' in res[r] for r in (0, 1)), res
