"""Data-parallel learners, one process per GPU (BASELINE config 4).

Each rank owns a full 1M-transition buffer, its own PER priorities and RNG
streams, and a model replica.  Sampling, gather, targets, losses, priority
write-back and target sync are rank-local; the only exchange is ONE all-reduce
of the flat fp32 gradient per step (4,278,891 floats = 17.1 MB for
Rainbow/Asterix) over RCCL/xGMI, then every rank applies the identical TF1
Adam update, so replicas stay bit-identical.  PER's `w /= max(w)` stays
per-rank (rainbow_agent.py:280): the multi-GPU gradient is the mean of the
ranks' single-GPU gradients, not a single B*N batch.
"""
import os

import torch
import torch.distributed as dist

# Run the collectives even in a one-rank group (DQ_FORCE_COLLECTIVES=1): a one-GPU box
# can then drive the RCCL path itself (bench.py --force-dist, tests/test_gpu_rccl.py);
# an average over one rank leaves the values unchanged.
FORCE_COLLECTIVES = os.environ.get('DQ_FORCE_COLLECTIVES') == '1'


def allreduce_mean_(flat_grad, group=None):
  """In-place mean of a flat gradient buffer across the ranks of ``group``."""
  world = dist.get_world_size(group)
  if world == 1 and not FORCE_COLLECTIVES:
    return flat_grad
  if dist.get_backend(group) == 'nccl':     # RCCL averages in the collective (no extra kernel)
    dist.all_reduce(flat_grad, op=dist.ReduceOp.AVG, group=group)
    return flat_grad
  dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=group)
  flat_grad.mul_(1.0 / world)
  return flat_grad


def replicas_in_sync(flat_params, group=None):
  """Checksum-broadcast check that every rank holds identical parameters."""
  s = torch.stack([flat_params.double().sum(), (flat_params.double() ** 2).sum()])
  ref = s.clone()
  dist.broadcast(ref, src=0, group=group)
  ok = torch.tensor([1.0 if torch.equal(s, ref) else 0.0], dtype=torch.float64, device=s.device)
  dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
  return bool(ok.item() == 1.0)
