"""Count RNG-tape refills / syncs / probes in the learner loop (uniform DQN vs PER Rainbow)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('HIP_FORCE_DEV_KERNARG', '1')
import torch  # noqa: E402

import bench  # noqa: E402
from dopamine_amd.replay_memory import rng_tape  # noqa: E402

ev = []
_rebuild, _sync, _poll = rng_tape.RNGTape.rebuild, rng_tape.RNGTape.sync, rng_tape.RNGTape._poll


def rebuild(self, nwords, h):
  t = time.perf_counter()
  _rebuild(self, nwords, h)
  ev.append(('rebuild', int(nwords), round(1e3 * (time.perf_counter() - t), 3)))


def sync(self, h, meta=None):
  t = time.perf_counter()
  r = _sync(self, h, meta)
  ev.append(('sync', round(1e3 * (time.perf_counter() - t), 3)))
  return r


def poll(self):
  b = self._budget
  _poll(self)
  if self._probe is None:
    ev.append(('probe', b, self._budget, self._len))


rng_tape.RNGTape.rebuild, rng_tape.RNGTape.sync, rng_tape.RNGTape._poll = rebuild, sync, poll
dev = torch.device('cuda', 0)
out = {}
for name, make, A in (('dqn', lambda: bench.build_dqn_pong(dev), 6),
                      ('rainbow', lambda: bench.build_agent(9, 1_000_000, 32, dev), 9)):
  agent = make()
  import random
  random.seed(0)
  bench.fill_synthetic(agent._replay.memory, A, seed=1)
  torch.cuda.synchronize()
  ev.clear()
  agent.train_gradient_steps(1000)
  torch.cuda.synchronize()
  out[name] = list(ev)
  del agent
print(json.dumps(out))
