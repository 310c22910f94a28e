"""Sum-tree update (dq_sumtree_set, batch 32) and prioritized index sampling
(dq_replay_sample_indices) on a 1M-transition buffer: average per-launch time of
100 back-to-back launches captured in a HIP graph.
    python tools/bench_sumtree.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import torch  # noqa: E402

import bench  # noqa: E402
from dopamine_amd import _lib  # noqa: E402
from dopamine_amd.replay_memory.prioritized_replay_buffer import (  # noqa: E402
    OutOfGraphPrioritizedReplayBuffer)


def graph_us(fn, reset, iters=100):
  fn()
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(iters):
      fn()
  best = 1e9
  for _ in range(5):
    reset()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
  return best


def main():
  dev = torch.device('cuda', 0)
  B = 32
  mem = OutOfGraphPrioritizedReplayBuffer(observation_shape=(84, 84), stack_size=4,
                                          replay_capacity=1_000_000, batch_size=B,
                                          update_horizon=3, gamma=0.99, device=dev)
  bench.fill_synthetic(mem, 9, seed=1)
  mem._rng.rebuild(1 << 20, mem._stream)
  out = torch.empty(B, dtype=torch.int32, device=dev)
  _lib.call('dq_replay_sample_indices', mem._h, B, _lib.ptr(out), mem._stream)
  torch.cuda.synchronize()
  idx = out.clone()
  prio = torch.rand(B, device=dev) + 0.5
  nop = lambda: None   # noqa: E731
  t_set = graph_us(lambda: _lib.call('dq_sumtree_set', mem._h, _lib.ptr(idx), _lib.ptr(prio), B, mem._stream), nop)
  reset = lambda: _lib.call('dq_replay_set_tape', mem._h, 1 << 20, mem._stream)   # noqa: E731
  t_smp = graph_us(lambda: _lib.call('dq_replay_sample_indices', mem._h, B, _lib.ptr(out), mem._stream), reset)
  print('sumtree_set B=%d: %.2f us   per_sample B=%d: %.2f us' % (B, t_set, B, t_smp))


if __name__ == '__main__':
  main()
