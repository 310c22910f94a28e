"""The data-parallel learner path over RCCL itself (torch.distributed backend "nccl"
= RCCL on ROCm), on a one-GPU box: a one-rank RCCL group with every collective
executed (parallel.FORCE_COLLECTIVES).  The whole N > 1 schedule runs -- rank-0
replica broadcast, split head | tail | optimizer graphs, the fc bucket's all-reduce
(ReduceOp.AVG) on the comm stream with its Adam part behind it, the conv bucket over
the second communicator, the deferred join in the learner-only loop -- and an average
over one rank changes nothing, so the parameters must equal a single learner's BIT
FOR BIT.  (Multi-rank ordering is pinned by tests/test_gpu_multirank.py over gloo;
two RCCL ranks cannot share one device.)"""
import os
import socket

import numpy as np
import pytest
import torch

from tests.test_gpu_multirank import _agent, _run

pytestmark = pytest.mark.gpu


def _free_port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


@pytest.fixture
def rccl_group():
  import torch.distributed as dist
  from dopamine_amd import parallel
  torch.cuda.set_device(0)
  dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % _free_port(), rank=0,
                          world_size=1, device_id=torch.device('cuda', 0))
  assert dist.get_backend() == 'nccl'
  old, parallel.FORCE_COLLECTIVES = parallel.FORCE_COLLECTIVES, True
  try:
    yield dist.group.WORLD
  finally:
    parallel.FORCE_COLLECTIVES = old
    torch.cuda.synchronize()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize('loop', [False, True])
def test_rccl_one_rank_schedule_equals_single_learner_bitwise(rccl_group, loop):
  from dopamine_amd import parallel
  agent = _agent(rccl_group, 0)
  assert agent._split_allreduce()
  flat = _run(agent, loop).numpy()
  assert agent._graph_sets.get(True) is not None   # the split graphs were captured and replayed
  assert parallel.replicas_in_sync(agent.online_convnet.fp.flat, rccl_group)
  if loop:
    # the conv bucket went over the second communicator (the agent's own RcclComm pair)
    assert agent._rccl is not None and agent._pg_conv is None
    # ... and the learner loop replayed chunk graphs with the all-reduces captured in them
    assert any(k[0] == 'chunk' for k in agent._graph_sets if isinstance(k, tuple))
  single = _run(_agent(None, 0), loop).numpy()
  assert np.array_equal(flat, single)


@pytest.mark.timeout(600)
@pytest.mark.parametrize('loop', [False, True])
def test_rccl_one_rank_sharded_optimizer_equals_single_learner_bitwise(rccl_group, loop):
  """ZeRO-1 over RCCL (in-place reduce-scatter, TF1 Adam on the rank's slice, in-place
  all-gather; captured in the chunk graphs in the learner loop): one rank owns every
  slice, so the parameters equal a single learner's bit for bit."""
  agent = _agent(rccl_group, 0, shard_optimizer=True)
  assert agent._sharded()
  flat = _run(agent, loop).numpy()
  if loop:
    assert any(k[0] == 'chunk' for k in agent._graph_sets if isinstance(k, tuple))
  single = _run(_agent(None, 0), loop).numpy()
  assert np.array_equal(flat, single)


def test_collective_capture_probe(rccl_group):
  """The probe that gates captured all-reduces in the learner loop: yes for the learner's
  own RCCL communicators, no for torch.distributed's collectives (their watchdog polls
  events on the stream a capture would take over: parallel.collectives_capturable)."""
  from dopamine_amd import parallel
  parallel._CAPTURABLE.clear()
  assert not parallel.collectives_capturable(rccl_group, torch.device('cuda', 0))
  assert not parallel.collectives_capturable(rccl_group, torch.device('cuda', 0), sharded=True)
  comms = (parallel.RcclComm(rccl_group, 'cuda:0'), parallel.RcclComm(rccl_group, 'cuda:0'))
  try:
    for sharded in (False, True):
      assert parallel.collectives_capturable(rccl_group, torch.device('cuda', 0), sharded=sharded,
                                             comms=comms)
  finally:
    parallel.forget_capture_probes(comms)
    for c in comms:
      c.destroy()


def test_allreduce_mean_over_rccl_is_identity_for_one_rank(rccl_group):
  from dopamine_amd import parallel
  x = torch.randn(4_278_891, device='cuda')
  ref = x.clone()
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):                # as the agent's comm stream issues it
    parallel.allreduce_mean_(x, rccl_group)
  torch.cuda.current_stream().wait_stream(s)
  torch.cuda.synchronize()
  assert torch.equal(x, ref)


@pytest.mark.timeout(600)
@pytest.mark.parametrize('loop', [False, True])
def test_rccl_torch_collectives_schedule_equals_single_learner_bitwise(rccl_group, loop):
  """The same schedule with torch.distributed's collectives (native_comm=False): the
  learner's own communicators and the process group's give the same bits."""
  agent = _agent(rccl_group, 0, native_comm=False)
  assert agent._rccl is None
  flat = _run(agent, loop).numpy()
  # never captured: per-step graphs with the collectives issued between them
  assert not any(k[0] == 'chunk' for k in agent._graph_sets if isinstance(k, tuple))
  single = _run(_agent(None, 0), loop).numpy()
  assert np.array_equal(flat, single)


def test_native_comm_is_used_and_collectives_are_identity_for_one_rank(rccl_group):
  """parallel.RcclComm (dq_comm_*): the agent owns a pair over RCCL; in-place all-reduce,
  reduce-scatter and all-gather of one rank leave the values as they are, eagerly and
  replayed from a captured graph on a side stream."""
  from dopamine_amd import parallel
  agent = _agent(rccl_group, 0)
  assert agent._rccl is not None and len(agent._rccl) == 2
  c = agent._rccl[0]
  x = torch.randn(4_278_892, device='cuda')
  ref = x.clone()
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):
    c.allreduce_mean_(x)
    c.reduce_scatter_mean_(x)
    c.all_gather_(x)
  torch.cuda.current_stream().wait_stream(s)
  torch.cuda.synchronize()
  assert torch.equal(x, ref)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g, stream=s):
    c.allreduce_mean_(x)
    x.mul_(2.0)
  for _ in range(2):
    g.replay()
  torch.cuda.synchronize()
  assert torch.equal(x, ref * 4.0)
  parallel._CAPTURABLE.clear()
  assert parallel.collectives_capturable(rccl_group, torch.device('cuda', 0), sharded=True,
                                         comms=agent._rccl)
  # close(): the communicators destroyed, the graphs that captured them dropped
  agent.close()
  assert agent._rccl is None and not agent._graph_sets
  with pytest.raises(RuntimeError, match='closed'):
    agent.train_gradient_steps(1)
