"""CPU restatement of one Rainbow gradient step -- TEST INFRASTRUCTURE / CPU BASELINE.

Only ``bench.py``'s ``cpu_baseline`` leg and tests import this.  It times the
reference's algorithm on host cores: the numpy replay oracle (oracle/replay.py,
a line-for-line restatement of the reference's sampler, which is what the
reference itself runs on the CPU inside its py_func) + a torch-CPU Nature-CNN
forward/backward + the oracle C51 loss + the oracle TF1 Adam.  TensorFlow is not
available anywhere in this pipeline, so this "port" stands in for the
reference's own _train_step.
"""
import random
import time

import numpy as np
import torch

from oracle import learner as OL
from oracle import replay as OR


class CpuRainbowStep(object):
  def __init__(self, capacity=1_000_000, batch_size=32, num_actions=9, n=3, seed=0):
    from dopamine_amd.agents.networks import RainbowNetwork  # torch module definition only
    rs = np.random.RandomState(seed)
    self.B, self.A = batch_size, num_actions
    self.mem = OR.PrioritizedOracle((84, 84), 4, capacity, batch_size, update_horizon=n,
                                    py_rng=random.Random(seed))
    # Frames are zero pages: the numpy gather's cost does not depend on pixel values.
    self.mem.action = rs.randint(0, num_actions, capacity).astype(np.int32)
    self.mem.reward = rs.choice(np.array([-1, 0, 1], np.float32), capacity)
    self.mem.terminal = (rs.rand(capacity) < 1 / 500.).astype(np.uint8)
    self.mem.add_count = capacity + 12345
    self.mem.invalid_range = OR.invalid_range(self.mem.cursor(), capacity, 4, n)
    self.mem.sum_tree = OR.SumTree.from_leaves(capacity, rs.uniform(0.1, 2.0, capacity))
    self.online = RainbowNetwork(num_actions, device='cpu', seed=seed)
    self.target = RainbowNetwork(num_actions, device='cpu', seed=seed + 1)
    self.support = OL.c51_support(10.0, 51)
    self.cg = np.float32(0.99 ** n)
    self.opt = OL.TF1Adam(self.online.fp.numel, 6.25e-5, eps=1.5e-4)
    self.params = self.online.fp.flat.numpy()   # shares memory with the torch params

  def step(self):
    b = self.mem.sample_transition_batch()
    st = torch.from_numpy(np.moveaxis(b[0], -1, 1).astype(np.float32) / np.float32(255))
    nst = torch.from_numpy(np.moveaxis(b[3], -1, 1).astype(np.float32) / np.float32(255))
    with torch.no_grad():
      tl = self.target(nst).numpy()
    logits = self.online(st)
    out = OL.c51_loss(logits.detach().numpy(), tl, b[1] % self.A, b[2], b[6], self.support,
                      self.cg, b[8], dtype=np.float32)
    self.mem.set_priority(b[7], out['priorities'].astype(np.float32))
    self.online.fp.grad.zero_()
    logits.backward(torch.from_numpy(out['grad'].astype(np.float32)))
    with torch.no_grad():
      self.opt.step(self.params, self.online.fp.grad.numpy())

  def time(self, seconds=10.0, min_steps=3, max_steps=500):
    self.step()  # warm-up (allocations, first-touch)
    t0 = time.perf_counter()
    k = 0
    while k < min_steps or (time.perf_counter() - t0 < seconds and k < max_steps):
      self.step()
      k += 1
    dt = time.perf_counter() - t0
    return k / dt, k, dt
