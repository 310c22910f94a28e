"""The IQN network on the HIP kernels (dopamine_amd/iqn.py: torso on nature_cnn.hip,
quantile head on iqn.hip) against a float64 restatement of ImplicitQuantileNetwork
(oracle/nature_cnn.py, atari_lib.py:147-199) on the same flat parameters and taus:
quantile values within 1e-5 of their scale, and every parameter gradient of a given
d loss / d q within 1e-5 of its tensor's scale."""
import numpy as np
import pytest
import torch

from oracle import nature_cnn as ONC

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _rel(got, ref):
  got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
  return float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))


@pytest.mark.parametrize('B,nq,A', [(3, 5, 4), (64, 64, 4), (16, 8, 18)])
def test_iqn_executor_matches_float64(B, nq, A):
  from dopamine_amd.agents.networks import ImplicitQuantileNetwork
  from dopamine_amd.iqn import HipIqnNet
  torch.manual_seed(0)
  net = ImplicitQuantileNetwork(A, device='cuda', seed=3)
  with torch.no_grad():     # non-zero biases so every term is exercised
    for n in ('conv1_b', 'conv2_b', 'conv3_b', 'emb_b', 'fc1_b', 'fc2_b'):
      net.fp[n].uniform_(-0.05, 0.05)
  rs = np.random.RandomState(B)
  x = torch.from_numpy(rs.randint(0, 256, (B, 84, 84, 4)).astype(np.float32) / np.float32(255))
  taus = torch.from_numpy(rs.rand(nq * B).astype(np.float32))
  ex = HipIqnNet(net, B, nq, keep=True)
  q, _ = ex.forward(x.cuda(), taus.cuda())
  q = q.cpu().numpy().copy()
  P = ONC.Params64(net.fp.flat.cpu().numpy(), net.fp.offsets)
  ref = ONC.iqn_forward(P, x.double(), taus.double())
  assert _rel(q, ref.detach().numpy()) <= TOL
  # the no-backward form (target nets) gives the same values, bit for bit
  ex2 = HipIqnNet(net, B, nq, keep=False)
  q2, _ = ex2.forward(x.cuda(), taus.cuda())
  np.testing.assert_array_equal(q2.cpu().numpy(), q)
  # backward of a given d loss / d q
  dq = torch.from_numpy(rs.randn(nq * B, A).astype(np.float32) / (nq * B))
  net.fp.grad.fill_(np.nan)           # every gradient element must be written
  ex.backward(dq.cuda())
  g = net.fp.grad.cpu().numpy()
  # gradients on the device's own ReLU decisions (see oracle/nature_cnn._relu): at R = 4096
  # a few of the 2M + 32M pre-activations sit within fp32 rounding of 0 and take the other
  # branch in float64, moving a cancelling 4096-term weight-gradient sum by a whole term
  Pm = ONC.Params64(net.fp.flat.cpu().numpy(), net.fp.offsets)
  ONC.iqn_forward(Pm, x.double(), taus.double(), masks=ONC.iqn_masks(ex)).backward(dq.double())
  g64 = Pm.flat_grad()
  errs = {}
  for name, (o, shape) in net.fp.offsets.items():
    n = int(np.prod(shape))
    assert np.isfinite(g[o:o + n]).all(), name
    errs[name] = _rel(g[o:o + n], g64[o:o + n])
  print('iqn executor grad errors (mask-pinned)', B, nq, errs, flush=True)
  assert max(errs.values()) <= TOL, errs


@pytest.mark.parametrize('B,nq', [(64, 64), (3, 5)])
def test_loader_formed_x_equals_stored_x_bitwise(B, nq):
  """The online net never stores x = tiled state * emb: the FC1 forward and dW1 loaders
  form it from emb and the state.  Same quantile values and every gradient, bit for bit,
  as the schedule that stores x and streams it (store_x=True)."""
  from dopamine_amd import iqn
  from dopamine_amd.agents.networks import ImplicitQuantileNetwork
  torch.manual_seed(0)
  net = ImplicitQuantileNetwork(4, device='cuda', seed=5)
  with torch.no_grad():
    for n in ('emb_b', 'fc1_b', 'fc2_b'):
      net.fp[n].uniform_(-0.05, 0.05)
  rs = np.random.RandomState(7)
  x = torch.from_numpy(rs.randint(0, 256, (B, 84, 84, 4)).astype(np.float32) / np.float32(255)).cuda()
  taus = torch.from_numpy(rs.rand(nq * B).astype(np.float32)).cuda()
  dq = torch.from_numpy(rs.randn(nq * B, 4).astype(np.float32) / (nq * B)).cuda()
  out = {}
  for store in (True, False):
    ex = iqn.HipIqnNet(net, B, nq, keep=True, store_x=store)
    assert (ex.acts['x'] is None) != store
    q, _ = ex.forward(x, taus)
    h = ex.acts['h'].clone()
    net.fp.grad.fill_(np.nan)
    ex.backward(dq)
    torch.cuda.synchronize()
    out[store] = (q.cpu().numpy().copy(), h.cpu().numpy(), net.fp.grad.cpu().numpy().copy())
  for a, b in zip(out[True], out[False]):
    np.testing.assert_array_equal(a, b)


def test_tau_sampler_is_uniform_and_replays_in_graphs():
  from dopamine_amd.iqn import TauSampler
  a = TauSampler(7, torch.device('cuda', 0))
  out = torch.empty(4096, device='cuda')
  eager = [a.draw(out).cpu().numpy().copy() for _ in range(3)]
  assert all(((e >= 0) & (e < 1)).all() for e in eager)
  assert abs(float(np.mean(np.concatenate(eager))) - 0.5) < 0.01
  assert not np.array_equal(eager[0], eager[1])
  b = TauSampler(7, torch.device('cuda', 0))
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    b.draw(out)
  got = []
  for _ in range(3):
    g.replay()
    got.append(out.cpu().numpy().copy())
  for e, r in zip(eager, got):
    np.testing.assert_array_equal(e, r)


@pytest.mark.parametrize('kind', ['adam', 'rmsprop_centered', 'rmsprop'])
@pytest.mark.parametrize('store', [True, False])
def test_fused_optimizer_torso_backward_equals_backward_then_adam(store, kind):
  """dq_cnn_backward_torso_opt (the IQN learner's optimizer inside the torso's grouped
  backward launches: the head as float4 riders, conv3 after its sum, conv2 / conv1 in their
  split-K sums' epilogues) == head + torso backward followed by the separate optimizer
  launch (dq_adam_tf1, or dq_rmsprop_tf1 centered and not: the RmsOp riders and GradEpi<2>
  epilogues) over the whole flat buffer, bitwise, over two steps (both beta-power slots);
  store False: the fused epilogues skip the gradient stores, the parameters and optimizer
  state unchanged."""
  from dopamine_amd import ops
  from dopamine_amd.agents.networks import ImplicitQuantileNetwork
  from dopamine_amd.iqn import HipIqnNet
  B, nq, A = 16, 8, 4
  nets = [ImplicitQuantileNetwork(A, device='cuda', seed=7) for _ in range(2)]
  exs = [HipIqnNet(n, B, nq, keep=True) for n in nets]
  if kind == 'adam':
    opts = [ops.TF1Adam(n.fp.flat, learning_rate=5e-5, epsilon=3.125e-4) for n in nets]
    names = ('params', 'm', 'v', 'state')
  else:
    opts = [ops.TF1RMSProp(n.fp.flat, learning_rate=2.5e-4, decay=0.95, momentum=0.0,
                           epsilon=1e-5, centered=kind == 'rmsprop_centered') for n in nets]
    names = ('params', 'ms', 'mom') + (('mg',) if kind == 'rmsprop_centered' else ())
  rs = np.random.RandomState(1)
  for step in range(2):
    x = torch.from_numpy(rs.rand(B, 84, 84, 4).astype(np.float32)).cuda()
    taus = torch.from_numpy(rs.rand(nq * B).astype(np.float32)).cuda()
    dq = torch.from_numpy(rs.randn(nq * B, A).astype(np.float32) / (nq * B)).cuda()
    for ex in exs:
      ex.forward(x, taus)
    exs[0].backward(dq, adam=opts[0], slot=step % 2, store_grads=store)
    exs[1].backward(dq)
    opts[1].step(nets[1].fp.grad, slot=step % 2)
    torch.cuda.synchronize()
    for n in names:
      assert torch.equal(getattr(opts[0], n), getattr(opts[1], n)), (step, n)
    if store:
      assert torch.equal(nets[0].fp.grad, nets[1].fp.grad)


@pytest.mark.parametrize('kind', ['adam', 'rmsprop'])
def test_iqn_agent_fused_optimizer_equals_separate_step_bitwise(kind):
  """The IQN agent with fuse_optimizer on (the optimizer inside the torso's backward, the
  pipelined two-stream schedule, graph capture, keep_gradients off as the bench drives it)
  and off (the separate optimizer launch after the step): parameters and optimizer state
  bitwise equal after graph-captured steps."""
  from dopamine_amd.agents.implicit_quantile.implicit_quantile_agent import ImplicitQuantileAgent
  from dopamine_amd.agents.optimizers import AdamOptimizer, RMSPropOptimizer
  import bench
  import random

  def make(fused):
    opt = (AdamOptimizer(learning_rate=5e-5, epsilon=3.125e-4) if kind == 'adam' else
           RMSPropOptimizer(learning_rate=2.5e-4, decay=0.95, momentum=0.0, epsilon=1e-5,
                            centered=True))
    ag = ImplicitQuantileAgent(num_actions=4, num_tau_samples=16, num_tau_prime_samples=16,
                               num_quantile_samples=8, update_horizon=3, min_replay_history=100,
                               update_period=4, target_update_period=40, optimizer=opt,
                               replay_capacity=20000, batch_size=16, device=torch.device('cuda', 0),
                               seed=3, fuse_optimizer=fused)
    ag.keep_gradients = False
    random.seed(5)
    bench.fill_synthetic(ag._replay.memory, 4, seed=9)
    return ag
  agents = [make(True), make(False)]
  assert agents[0]._fused_opt() and not agents[1]._fused_opt()
  for ag in agents:
    ag.train_gradient_steps(10)
  torch.cuda.synchronize()
  assert agents[0]._graph_sets and agents[1]._graph_sets    # captured steps were replayed
  a, b = agents[0]._opt, agents[1]._opt
  names = ('params', 'm', 'v', 'state') if kind == 'adam' else ('params', 'ms', 'mom', 'mg')
  for n in names:
    assert torch.equal(getattr(a, n), getattr(b, n)), n
