"""Is the learner step host-bound?  Times, for the bench's Rainbow agent:
  step_total : K grad steps incl. final sync (what bench.py measures)
  step_host  : the same loop's host time before the final sync
  replay_only: K bare graph replays (alternating parity), no Python agent logic
    python tools/host_time.py [K] [eager]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import torch  # noqa: E402

import bench  # noqa: E402
from dopamine_amd.agents.optimizers import AdamOptimizer  # noqa: E402
from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent  # noqa: E402


def main():
  K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
  dev = torch.device('cuda', 0)
  agent = RainbowAgent(num_actions=9, update_horizon=3, gamma=0.99, replay_scheme='prioritized',
                       min_replay_history=20000, update_period=4, target_update_period=8000,
                       optimizer=AdamOptimizer(learning_rate=0.0000625, epsilon=0.00015),
                       replay_capacity=1000000, batch_size=32, device=dev,
                       use_hip_graph=not (len(sys.argv) > 2 and sys.argv[2] == 'eager'))
  bench.fill_synthetic(agent._replay.memory, 9, seed=1)
  torch.cuda.synchronize()

  def grad_step():
    for _ in range(agent.update_period):
      agent._train_step()

  for _ in range(30):
    grad_step()
  torch.cuda.synchronize()
  # host-only cost: the Python step loop with the GPU idle in between (sync each step)
  t0 = time.perf_counter()
  host = 0.0
  for _ in range(200):
    h0 = time.perf_counter()
    grad_step()
    host += time.perf_counter() - h0
    torch.cuda.synchronize()
  print('host_alone  %7.1f us  (submission per step, GPU drained between steps)' % (host / 200 * 1e6))
  t0 = time.perf_counter()
  for _ in range(K):
    grad_step()
  t1 = time.perf_counter()
  torch.cuda.synchronize()
  t2 = time.perf_counter()
  print('step_total  %7.1f us' % ((t2 - t0) / K * 1e6))
  print('step_host   %7.1f us' % ((t1 - t0) / K * 1e6))
  g = agent._graphs
  if g is None:
    return
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for i in range(K):
    g[i % 2].replay()
  t1 = time.perf_counter()
  torch.cuda.synchronize()
  t2 = time.perf_counter()
  print('replay_only %7.1f us (host %7.1f us)' % ((t2 - t0) / K * 1e6, (t1 - t0) / K * 1e6))
  # the same steps with S consecutive steps captured in ONE graph: the graph
  # boundary's cost per step (what a multi-step learner graph would save)
  for S in (2, 4, 8):
    gs = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(gs, pool=agent._graph_pool):
      for j in range(S):
        agent._grad_step(j % 2, j % 2, True)
        agent._device_opt_step(j % 2)
    torch.cuda.synchronize()
    n = K // S
    t0 = time.perf_counter()
    for _ in range(n):
      gs.replay()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print('multi_step  S=%d %7.1f us per step' % (S, (t2 - t0) / (n * S) * 1e6))


if __name__ == '__main__':
  main()
