"""The data-parallel exchange over peer memory on ONE stream (exchange='peer',
parallel.PeerExchange, dq_cnn_backward_peer), on one GPU:

* world 1 (a one-rank group, the protocol run with itself): parameters, Adam moments and beta
  powers bitwise those of the single learner's fused schedule, per call and in the learner
  loop's captured chunks;
* two ranks sharing cuda:0 (two processes, each mapping the other's buffers through IPC
  handles), different buffers and network seeds: parameters and (gathered) moments bitwise
  those of one process applying TF1 Adam to the rank-ordered mean of the two gradients
  (test_gpu_multirank._mean_gradient_reference);
* a rank that never trains: the other's bounded waits time out, latch the error word and the
  learner raises -- no hang."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.test_gpu_multirank import STEPS, _agent, _free_port, _mean_gradient_reference, _run

pytestmark = pytest.mark.gpu


# the two-rank learner-loop test's steps: enough for two chunks in one train_gradient_steps call
# between target syncs, so a chunk starts with its predecessor's deferred gather
LOOP_STEPS = 24


def _peer_worker(rank, world, port, q, loop, same_seed=False, idle_rank=-1, max_polls=None,
                 n_steps=None, stall=None, capacity=None):
  import sys
  sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
  import torch.distributed as dist
  os.environ['MASTER_ADDR'] = '127.0.0.1'
  os.environ['MASTER_PORT'] = str(port)
  torch.cuda.set_device(0)
  dist.init_process_group('gloo', rank=rank, world_size=world)
  from dopamine_amd import parallel
  if max_polls is not None and (stall is None or rank == stall[1]):
    parallel.PeerExchange.MAX_POLLS = max_polls
  agent = _agent(dist.group.WORLD, 0 if same_seed else rank,
                 net_seed=0 if same_seed else 1000 * rank, exchange='peer',
                 **({} if capacity is None else {'capacity': capacity}))
  assert agent._peer is not None and agent._sharded() and not agent._collective()
  if rank == idle_rank:
    q.put((rank, 'idle'))
    dist.barrier()          # the others' host barrier before their first exchange step
    dist.barrier()          # and their closing one
    dist.destroy_process_group()
    return
  if stall is not None:
    # rank stall[0] sleeps between two gradient steps; rank stall[1] (short max_polls) times
    # out waiting for it, latches its error and publishes nothing more
    import time
    t0 = time.time()
    for i in range(4):
      if rank == stall[0] and i == 2:
        time.sleep(3.0)
      for _ in range(agent.update_period):
        agent._train_step()
    torch.cuda.synchronize()
    t1 = time.time()
    try:
      agent.mean_loss()
      msg = None
    except RuntimeError as e:
      msg = str(e)
    try:
      agent.check_exchange(collective=True)
      cmsg = None
    except RuntimeError as e:
      cmsg = str(e)
    q.put((rank, msg, cmsg, agent._peer.error(), t1 - t0))
    dist.barrier()
    dist.destroy_process_group()
    return
  try:
    flat = _run(agent, loop, n_steps)
    err = None
    agent.mean_loss()
  except RuntimeError as e:
    q.put((rank, 'error', str(e)))
    if idle_rank >= 0:
      dist.barrier()
      dist.destroy_process_group()
      return
    raise
  assert agent._graph_sets.get(True) is not None    # the later steps replayed captured graphs
  assert not loop or any(isinstance(k, tuple) and k[0] == 'chunk' for k in agent._graph_sets)
  # world > 1: a chunk that started with its predecessor's deferred gather ran too
  assert not loop or world == 1 or any(isinstance(k, tuple) and k[0] == 'chunk' and k[-1] is True
                                       for k in agent._graph_sets), list(agent._graph_sets)
  ok = parallel.replicas_in_sync(agent.online_convnet.fp.flat)
  ok = ok and parallel.replicas_in_sync(agent.target_convnet.fp.flat)
  rep = agent.replica_report()      # gathers every slice's moments, as a checkpoint sees them
  ok = ok and parallel.replicas_in_sync(agent._opt.m) and parallel.replicas_in_sync(agent._opt.v)
  ok = ok and all(v['in_sync'] for v in rep.values())
  st = agent._opt.state.cpu().numpy()
  if rank == 0:
    q.put((rank, ok, flat.numpy(), agent._opt.m.cpu().numpy(), agent._opt.v.cpu().numpy(), st,
           int(agent._peer.flags[0].item()), err,
           {'selftest': agent._peer.selftest, 'waits': agent._peer.wait_counters(),
            'replicas': sorted(rep), 'xcds': agent._peer.desc.xcds,
            'pub_xcds': int(agent._peer.flags[agent._peer._lib.PEER_PUB_XCDS].item())}))
  agent.close()
  dist.barrier()
  dist.destroy_process_group()


def _spawn(world, loop, **kw):
  ctx = mp.get_context('spawn')
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_peer_worker, args=(r, world, port, q, loop), kwargs=kw)
           for r in range(world)]
  for p in procs:
    p.start()
  res = []
  import queue
  import time
  try:
    want = world if kw.get('idle_rank', -1) >= 0 or kw.get('stall') else 1
    t0 = time.time()
    while len(res) < want and time.time() - t0 < 400:
      try:
        res.append(q.get(timeout=5))
      except queue.Empty:          # a worker that died (its traceback is on stderr) ends the wait
        assert not any(p.exitcode not in (None, 0) for p in procs), [p.exitcode for p in procs]
    assert len(res) == want, 'workers did not report'
  finally:
    for p in procs:
      p.join(timeout=120)
      if p.exitcode is None:
        p.kill()
  return res, [p.exitcode for p in procs]


@pytest.mark.timeout(600)
@pytest.mark.parametrize('loop', [False, True])
def test_peer_world1_equals_single_learner_bitwise(loop):
  """World 1: the exchange's reduce-scatter, slice Adam, conv bucket and (empty) all-gather
  run against the learner itself -- bitwise the single learner (parameters, moments, beta
  powers), and the step counter counts the gradient steps."""
  res, codes = _spawn(1, loop)
  _, ok, flat, m, v, st, steps, _, info = res[0]
  assert codes == [0] and ok
  single = _agent(None, 0)
  sflat = _run(single, loop).numpy()
  assert np.array_equal(flat, sflat)
  assert np.array_equal(m, single._opt.m.cpu().numpy())
  assert np.array_equal(v, single._opt.v.cpu().numpy())
  assert np.array_equal(st, single._opt.state.cpu().numpy())
  assert steps == single._opt_steps == STEPS


@pytest.mark.timeout(900)
@pytest.mark.parametrize('loop', [False, True])
def test_peer_two_ranks_equal_mean_gradient_reference(loop):
  """Two processes on cuda:0, different buffers and network seeds (rank 0's broadcast at
  construction): parameters and gathered moments bitwise the rank-ordered mean-gradient
  TF1 Adam reference; the replicas stay bit-identical."""
  n = LOOP_STEPS if loop else STEPS
  res, codes = _spawn(2, loop, n_steps=n)
  _, ok, flat, m, v, st, steps, _, info = res[0]
  assert codes == [0, 0] and ok and steps == n
  ref, rm, rv = _mean_gradient_reference(loop, moments=True, n_steps=n)
  assert np.array_equal(flat, ref)
  assert np.array_equal(m, rm) and np.array_equal(v, rv)
  # the construction-time self-test passed on both ranks, every publication
  # covered every XCD, and the wait counters counted each exchange point's waits
  st = info['selftest']
  assert st['ok'] and [r['mismatched_words'] for r in st['ranks']] == [0, 0], st
  assert [r['xcds_seen'] for r in st['ranks']] == [info['xcds']] * 2 and info['xcds'] == 8, info
  assert info['pub_xcds'] == 8
  w = info['waits']
  assert w['grad'][1] == 2 * n and w['conv'][1] == n and w['param'][1] >= n, w
  assert sorted(info['replicas']) == ['online', 'opt_m', 'opt_state', 'opt_v', 'target']
  print('selftest', st, 'waits', w)


@pytest.mark.timeout(900)
@pytest.mark.parametrize('world', [4, 8])
def test_peer_world_n_equal_mean_gradient_reference(world):
  """4 and 8 processes on cuda:0 in the learner loop (world - 1 remote slices per gather,
  the rank-ordered mean of world gradients, the deferred gather across chunks; world 8 is
  config 4's): bitwise the mean-gradient TF1 Adam reference, parameters and gathered
  moments."""
  res, codes = _spawn(world, True, n_steps=LOOP_STEPS)
  _, ok, flat, m, v, st, steps, _, info = res[0]
  assert codes == [0] * world
  assert steps == LOOP_STEPS, steps
  ref, rm, rv = _mean_gradient_reference(True, moments=True, world=world, n_steps=LOOP_STEPS)
  d = np.abs(flat - ref)
  assert np.array_equal(flat, ref), ('replicas in sync: %s; params differ at %d of %d, first %s, '
                                     'max %g' % (ok, int((d > 0).sum()), d.size,
                                                 np.flatnonzero(d)[:8], float(d.max())))
  assert ok
  assert np.array_equal(m, rm) and np.array_equal(v, rv)


@pytest.mark.timeout(1200)
def test_peer_world8_at_config4_capacity_equals_mean_gradient_reference():
  """Config 4's shape (the peer tests ran at 30k transitions): 8 processes on
  cuda:0, each with its own 1M-transition buffer and network seed, in the learner loop --
  parameters and gathered moments bitwise the rank-ordered mean-gradient TF1 Adam reference
  over the same eight 1M buffers, the self-test passed on every rank."""
  res, codes = _spawn(8, True, n_steps=LOOP_STEPS, capacity=1_000_000)
  _, ok, flat, m, v, st, steps, _, info = res[0]
  assert codes == [0] * 8 and ok and steps == LOOP_STEPS
  assert info['selftest']['ok'] and len(info['selftest']['ranks']) == 8
  ref, rm, rv = _mean_gradient_reference(True, moments=True, world=8, capacity=1_000_000,
                                         n_steps=LOOP_STEPS)
  assert np.array_equal(flat, ref)
  assert np.array_equal(m, rm) and np.array_equal(v, rv)


@pytest.mark.timeout(600)
def test_peer_wait_times_out_instead_of_hanging():
  """Rank 1 builds its learner (the handles are exchanged) but never trains: rank 0's waits
  for its gradients give up after max_polls, latch the error word, and mean_loss raises."""
  res, codes = _spawn(2, False, idle_rank=1, max_polls=20000)
  by_rank = {r[0]: r for r in res}
  assert by_rank[1][1] == 'idle'
  assert by_rank[0][1] == 'error' and 'timed out' in by_rank[0][2], by_rank[0]
  assert codes == [0, 0]


@pytest.mark.timeout(600)
def test_peer_error_on_one_rank_stops_every_rank():
  """rank 1 (short max_polls) times out while rank 0 sleeps between two steps;
  rank 1 latches its error and publishes nothing more, and rank 0, once it resumes, finds
  rank 1's error word while waiting (within 64 polls, not after its own max_polls) and gives
  up too.  Each rank's local check names its cause; the collective check raises on both."""
  res, codes = _spawn(2, False, max_polls=20000, stall=(0, 1))
  by_rank = {r[0]: r[1:] for r in res}
  msg0, cmsg0, e0, dt0 = by_rank[0]
  msg1, cmsg1, e1, dt1 = by_rank[1]
  assert codes == [0, 0]
  assert 2 <= e1 <= 4 and 'timed out' in msg1, by_rank[1]
  assert e0 == 16 + 1 and 'rank 1 had latched an error' in msg0, by_rank[0]
  assert dt0 < 30, dt0            # rank 0 gave up at once (its own bound is ~1 min)
  assert cmsg0 and cmsg1
