"""A/B on one box: IQN config 5 with the fused tau + cosine draw (default) and with the
separate draw / bump / embedding launches (monkeypatched back), alternating runs."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import torch  # noqa: E402

import bench  # noqa: E402
from dopamine_amd import iqn  # noqa: E402
from tools.bench_configs import measure  # noqa: E402

fused_draw, fused_fwd = iqn.TauSampler.draw_cos, iqn.HipIqnNet.forward


def separate(on):
  if on:
    iqn.TauSampler.draw_cos = lambda self, ex: self.draw(ex.taus)
    iqn.HipIqnNet.forward = lambda self, x, taus=None, cos_ready=False: fused_fwd(self, x, taus)
  else:
    iqn.TauSampler.draw_cos, iqn.HipIqnNet.forward = fused_draw, fused_fwd


dev = torch.device('cuda', 0)
res = {'fused': [], 'separate': []}
for rep in range(2):
  for name in ('fused', 'separate'):
    separate(name == 'separate')
    r = measure(lambda: bench.build_iqn_breakout(dev), 4, 150)
    res[name].append(r['steps_per_s'])
print(json.dumps(res))
