"""Learner kernels (C ABI) vs the numpy oracle (oracle/learner.py).

Tolerance: 1e-5 (fp32 parity bar of BASELINE.json north_star) on losses,
projections, gradients and optimizer updates, vs the float64 oracle.
"""
import numpy as np
import pytest
import torch

from oracle import learner as L

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _t(x, dt=torch.float32):
  return torch.as_tensor(np.ascontiguousarray(x)).to('cuda', dt)


@pytest.mark.parametrize('B,A,prio', [(32, 9, True), (32, 6, False), (5, 3, True), (64, 18, True)])
def test_c51_loss(B, A, prio):
  from dopamine_amd import ops
  rs = np.random.RandomState(B + A)
  N = 51
  z = L.c51_support(10.0, N, np.float32)
  ol = rs.randn(B, A, N).astype(np.float32) * 2
  tl = rs.randn(B, A, N).astype(np.float32) * 2
  act = rs.randint(0, A, B).astype(np.int32)
  rew = rs.choice([-1.0, 0.0, 1.0, 2.5], B).astype(np.float32)
  term = (rs.rand(B) < 0.2).astype(np.uint8)
  probs = rs.uniform(0.05, 2.0, B).astype(np.float32) if prio else None
  cg = 0.99 ** 3
  exp = L.c51_loss(ol, tl, act, rew, term, z, np.float32(cg), probs)
  got = ops.c51_loss(_t(ol), _t(tl), _t(act, torch.int32), _t(rew), _t(term, torch.uint8), _t(z),
                     np.float32(cg), None if probs is None else _t(probs))
  np.testing.assert_allclose(got['loss'].cpu().numpy(), exp['loss'], rtol=TOL, atol=TOL)
  np.testing.assert_allclose(got['grad'].cpu().numpy(), exp['grad'], rtol=TOL, atol=TOL)
  np.testing.assert_allclose(got['priorities'].cpu().numpy(), exp['priorities'], rtol=TOL, atol=TOL)
  np.testing.assert_allclose(got['mean_loss'].cpu().numpy()[0], exp['mean_loss'], rtol=TOL, atol=TOL)


def test_c51_projection_kats():
  """rainbow_agent_test.py:178-285 through the device kernel: a target net whose
  greedy action has the KAT weights, rewards/gamma giving the KAT supports."""
  from dopamine_amd import ops
  # supports = r + g * z with z = target support  -> choose r, g per KAT row
  cases = [([0, 1, 2, 3, 4], [0.1, 0.2, 0.1, 0.3, 0.3], [0, 1, 2, 3, 4], [0.1, 0.2, 0.1, 0.3, 0.3]),
           ([0, 1, 2, 3, 4], [0.1, 0.2, 0.1, 0.3, 0.3], [3, 4, 5, 6, 7], [0.7, 0.3, 0.0, 0.0, 0.0]),
           ([3, 4, 5, 6, 7], [0.1, 0.2, 0.3, 0.2, 0.2], [3, 4, 5, 6, 7], [0.1, 0.2, 0.3, 0.2, 0.2])]
  for sup, w, tgt, expected in cases:
    tgt = np.array(tgt, np.float32)
    sup = np.array(sup, np.float32)
    g = (sup[-1] - sup[0]) / (tgt[-1] - tgt[0])
    r = sup[0] - g * tgt[0]
    tl = np.log(np.array(w, np.float32))[None, None, :]
    ol = np.zeros((1, 1, 5), np.float32)
    out = ops.c51_loss(_t(ol), _t(tl), _t(np.zeros(1, np.int32), torch.int32), _t([r]),
                       _t(np.zeros(1, np.uint8), torch.uint8), _t(tgt), float(g))
    # grad = softmax(0) - proj  => proj = 1/N - grad
    proj = 1.0 / 5 - out['grad'].cpu().numpy()[0, 0]
    np.testing.assert_allclose(proj, expected, atol=1e-6)


@pytest.mark.parametrize('B,A', [(32, 6), (7, 4), (300, 18)])
def test_dqn_huber(B, A):
  from dopamine_amd import ops
  rs = np.random.RandomState(B)
  oq = (rs.randn(B, A) * 3).astype(np.float32)
  tq = (rs.randn(B, A) * 3).astype(np.float32)
  act = rs.randint(0, A, B).astype(np.int32)
  rew = rs.randn(B).astype(np.float32)
  term = (rs.rand(B) < 0.3).astype(np.uint8)
  exp = L.dqn_huber(oq, tq, act, rew, term, np.float32(0.99))
  got = ops.dqn_huber_loss(_t(oq), _t(tq), _t(act, torch.int32), _t(rew), _t(term, torch.uint8), 0.99)
  np.testing.assert_allclose(got['loss'].cpu().numpy(), exp['loss'], rtol=TOL, atol=TOL)
  np.testing.assert_allclose(got['grad'].cpu().numpy(), exp['grad'], rtol=TOL, atol=TOL)
  np.testing.assert_allclose(got['mean_loss'].cpu().numpy()[0], exp['mean_loss'], rtol=TOL, atol=TOL)


@pytest.mark.parametrize('B,A,N,Np,K', [(64, 4, 64, 64, 32), (5, 3, 7, 9, 11), (32, 18, 100, 70, 32)])
def test_iqn_loss(B, A, N, Np, K):
  from dopamine_amd import ops
  rs = np.random.RandomState(N)
  oq = rs.randn(N * B, A).astype(np.float32)
  tq = rs.randn(Np * B, A).astype(np.float32)
  ta = rs.randn(K * B, A).astype(np.float32)
  tau = rs.rand(N * B).astype(np.float32)
  act = rs.randint(0, A, B).astype(np.int32)
  rew = rs.randn(B).astype(np.float32)
  term = (rs.rand(B) < 0.3).astype(np.uint8)
  exp = L.iqn_loss(oq, tq, ta, tau, act, rew, term, np.float32(0.99 ** 3))
  got = ops.iqn_loss(_t(oq), _t(tq), _t(ta), _t(tau), _t(act, torch.int32), _t(rew),
                     _t(term, torch.uint8), np.float32(0.99 ** 3))
  np.testing.assert_allclose(got['loss'].cpu().numpy(), exp['loss'], rtol=TOL, atol=TOL)
  np.testing.assert_allclose(got['grad'].cpu().numpy(), exp['grad'], rtol=TOL, atol=1e-7)
  np.testing.assert_allclose(got['mean_loss'].cpu().numpy()[0], exp['mean_loss'], rtol=TOL, atol=TOL)


def test_adam_tf1_matches_oracle():
  from dopamine_amd import ops
  rs = np.random.RandomState(0)
  n = 4_278_891   # Rainbow/Asterix parameter count (odd -> exercises the tail)
  var = rs.randn(n).astype(np.float32) * 0.05
  dvar = _t(var)
  opt = ops.TF1Adam(dvar, 6.25e-5, epsilon=1.5e-4)
  ref = L.TF1Adam(n, 6.25e-5, eps=1.5e-4)
  rvar = var.copy()
  for step in range(5):
    g = (rs.randn(n) * 1e-2).astype(np.float32)
    opt.step(_t(g))
    ref.step(rvar, g)
  np.testing.assert_allclose(dvar.cpu().numpy(), rvar, rtol=1e-5, atol=1e-7)


def test_rmsprop_tf1_matches_oracle():
  from dopamine_amd import ops
  rs = np.random.RandomState(1)
  n = 100_003
  var = rs.randn(n).astype(np.float32) * 0.05
  dvar = _t(var)
  opt = ops.TF1RMSProp(dvar, 2.5e-4, decay=0.95, momentum=0.0, epsilon=1e-5, centered=True)
  ref = L.TF1CenteredRMSProp(n, 2.5e-4, decay=0.95, momentum=0.0, eps=1e-5)
  rvar = var.copy()
  for _ in range(5):
    g = (rs.randn(n) * 1e-2).astype(np.float32)
    opt.step(_t(g))
    ref.step(rvar, g)
  np.testing.assert_allclose(dvar.cpu().numpy(), rvar, rtol=1e-5, atol=1e-7)


def test_sync_copy():
  from dopamine_amd import ops
  a = torch.randn(4_278_891, device='cuda')
  b = torch.zeros_like(a)
  ops.sync_copy(b, a)
  assert torch.equal(a, b)


def test_adam_multi_tensor_equals_flat():
  """One launch over per-parameter gradients == the flat-buffer update."""
  from dopamine_amd import ops
  from dopamine_amd.agents.networks import RainbowNetwork
  net = RainbowNetwork(9, device='cuda', seed=0)
  segs = net.fp.segments()
  flat0 = net.fp.flat.clone()
  a = ops.TF1Adam(net.fp.flat, 6.25e-5, epsilon=1.5e-4, segments=segs)
  ref_p = flat0.clone()
  b = ops.TF1Adam(ref_p, 6.25e-5, epsilon=1.5e-4)
  for step in range(3):
    grads = [torch.randn_like(prm) for prm in net.parameters()]   # param-like strides
    flat_g = torch.zeros_like(ref_p)
    for (o, n), g, v in zip(segs, grads, net.fp.grad_views):
      v.copy_(g)
    flat_g.copy_(net.fp.grad)
    a.step_multi(grads)
    b.step(flat_g)
  assert torch.equal(net.fp.flat, ref_p)
  assert torch.equal(a.state, b.state)
