import sys, os, time, gc, json
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '/root/repo'))
import torch, bench, random
dev = torch.device('cuda', 0)
res = {}
for trial in range(2):
  for steps in (300, 1000):
    a = bench.build_dqn_pong(dev)
    random.seed(0)
    bench.fill_synthetic(a._replay.memory, 6, seed=1)
    torch.cuda.synchronize()
    el, prime = bench.timed_steps(a, steps, 10)
    res['bench_protocol_%d_%d' % (steps, trial)] = round(steps / el, 1)
    a.train_gradient_steps(20); torch.cuda.synchronize()
    t0 = time.perf_counter(); a.train_gradient_steps(steps); torch.cuda.synchronize()
    res['again_%d_%d' % (steps, trial)] = round(steps / (time.perf_counter() - t0), 1)
    del a; gc.collect(); torch.cuda.empty_cache()
print(json.dumps(res))
