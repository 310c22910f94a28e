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


def _agent(pg, seed, net_seed=0, **kw):
  from dopamine_amd.agents.optimizers import AdamOptimizer
  from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent
  import bench
  import random
  agent = RainbowAgent(num_actions=9, update_horizon=3, gamma=0.99, replay_scheme='prioritized',
                       min_replay_history=100, update_period=4, target_update_period=40,
                       optimizer=AdamOptimizer(learning_rate=6.25e-5, epsilon=1.5e-4),
                       replay_capacity=CAP, batch_size=32, device=torch.device('cuda', 0),
                       seed=net_seed, process_group=pg, **kw)
  random.seed(seed)
  bench.fill_synthetic(agent._replay.memory, 9, seed=1 + seed)
  return agent


def _run(agent, loop=False):
  if loop:
    agent.train_gradient_steps(STEPS)
  else:
    for _ in range(STEPS):
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


def _mean_gradient_reference(loop=False, moments=False):
  """Both ranks' learners in ONE process, no collective: each _train_step computes
  its own gradient (the optimizer deferred), the two flat gradients are averaged
  ((gA + gB) * 0.5, what gloo's sum + scale gives), and the TF1 Adam step is applied
  to that mean on both replicas; target syncs run after the update, as in
  _train_step.  SURVEY 8(e): the multi-GPU gradient = the mean of the ranks'
  single-GPU gradients on their own minibatches (PER weights per rank)."""
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  import random
  agents = []
  for r in range(2):
    ag = _agent(None, r, use_hip_graph=False, fuse_optimizer=False)
    ag._replay.memory._rng.stream = random.Random(r)   # each rank's own `random`, as its process
    agents.append(ag)
  steps = []
  for ag in agents:
    ag._device_opt_step = lambda k, ag=ag: steps.append((ag, k))
    ag._sync_target = lambda ag=ag: steps.append((ag, 'sync'))
  for _ in range(STEPS * agents[0].update_period):
    steps.clear()
    for ag in agents:
      ag._train_step()
    opt = [(ag, k) for ag, k in steps if k != 'sync']
    if opt:
      assert len(opt) == 2 and opt[0][1] == opt[1][1]
      g = (agents[0].online_convnet.fp.grad + agents[1].online_convnet.fp.grad) * 0.5
      for ag, k in opt:
        ag.online_convnet.fp.grad.copy_(g)
        ag._opt.step(ag.online_convnet.fp.grad, slot=k)
    for ag, k in steps:
      if k == 'sync':
        DQNAgent._sync_target(ag)
  torch.cuda.synchronize()
  a, b = (ag.online_convnet.fp.flat.cpu().numpy() for ag in agents)
  assert np.array_equal(a, b)
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
