"""HIP Nature-CNN (fp32 MFMA implicit GEMM) vs the PyTorch network on the same
flat parameters: forward outputs and every parameter gradient.  Tolerance is
relative to each tensor's scale (fp32 with different summation orders)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=2e-5):
  a, b = a.double(), b.double()
  scale = b.abs().max().item() + 1e-30
  err = (a - b).abs().max().item()
  assert err <= rtol * scale, 'max err %.3g vs scale %.3g' % (err, scale)


@pytest.mark.parametrize('kind,B,A', [('rainbow', 32, 9), ('dqn', 32, 6), ('rainbow', 7, 4)])
def test_hip_cnn_matches_torch(kind, B, A):
  from dopamine_amd.agents.networks import NatureDQNNetwork, RainbowNetwork
  from dopamine_amd.cnn import HipNatureCNN
  torch.manual_seed(0)
  net = RainbowNetwork(A, device='cuda', seed=3) if kind == 'rainbow' else NatureDQNNetwork(A, device='cuda', seed=3)
  with torch.no_grad():     # non-zero biases so the bias paths are exercised
    for n, prm in net.fp.params.items():
      if n.endswith('_b'):
        prm.uniform_(-0.05, 0.1)
  x_nhwc = torch.rand(B, 84, 84, 4, device='cuda')
  x = x_nhwc.permute(0, 3, 1, 2)            # channels_last view, as the gather produces
  y_ref = net(x).reshape(B, -1)
  gout = torch.randn_like(y_ref)
  for prm in net.parameters():
    prm.grad = None
  y_ref.backward(gout)
  g_ref = [prm.grad.detach().clone() for prm in net.parameters()]

  hip = HipNatureCNN(net, B)
  y = hip.forward(x)
  _close(y, y_ref.detach())
  grads = {}
  for parallel in (True, False):       # weight grads on a second stream / one stream
    net.fp.grad.fill_(float('nan'))
    hip.backward(gout, parallel=parallel)
    torch.cuda.synchronize()
    grads[parallel] = torch.cat([v.reshape(-1) for v in net.fp.grad_views])  # skips alignment pads
    for (name, view), gr in zip(zip(net.fp.params.keys(), net.fp.grad_views), g_ref):
      try:
        _close(view, gr, rtol=5e-5)
      except AssertionError as e:
        raise AssertionError('%s (parallel=%s): %s' % (name, parallel, e))
  assert torch.equal(grads[True], grads[False])


def test_hip_cnn_graph_capturable_and_deterministic():
  from dopamine_amd.agents.networks import RainbowNetwork
  from dopamine_amd.cnn import HipNatureCNN
  net = RainbowNetwork(9, device='cuda', seed=1)
  hip = HipNatureCNN(net, 32)
  x = torch.rand(32, 84, 84, 4, device='cuda')
  gout = torch.randn(32, 459, device='cuda')
  hip.forward(x); hip.backward(gout)
  ref_y, ref_g = hip.acts['out'].clone(), net.fp.grad.clone()
  g = torch.cuda.CUDAGraph()
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):
    hip.forward(x); hip.backward(gout)
  torch.cuda.current_stream().wait_stream(s)
  with torch.cuda.graph(g):
    hip.forward(x); hip.backward(gout)
  net.fp.grad.zero_()
  g.replay()
  torch.cuda.synchronize()
  assert torch.equal(hip.acts['out'], ref_y)
  assert torch.equal(net.fp.grad, ref_g)     # split-K reduced in fixed order: bitwise stable


def test_fused_adam_backward_equals_backward_then_adam():
  """dq_cnn_backward_adam == dq_cnn_backward + dq_adam_tf1, bitwise, over two
  steps (both beta-power slots): same gradient, same ApplyAdam arithmetic."""
  from dopamine_amd import ops
  from dopamine_amd.agents.networks import RainbowNetwork
  from dopamine_amd.cnn import HipNatureCNN
  nets = [RainbowNetwork(9, device='cuda', seed=5) for _ in range(2)]
  hips = [HipNatureCNN(n, 32) for n in nets]
  opts = [ops.TF1Adam(n.fp.flat, learning_rate=6.25e-5, epsilon=1.5e-4) for n in nets]
  torch.manual_seed(1)
  for step in range(2):
    x = torch.rand(32, 84, 84, 4, device='cuda')
    gout = torch.randn(32, 459, device='cuda')
    for h in hips:
      h.forward(x)
    hips[0].backward(gout, adam=opts[0], slot=step % 2)
    hips[1].backward(gout)
    opts[1].step(nets[1].fp.grad, slot=step % 2)
    torch.cuda.synchronize()
    for a, b in zip(nets[0].fp.grad_views, nets[1].fp.grad_views):
      assert torch.equal(a, b)
    for n in ('params', 'm', 'v', 'state'):
      assert torch.equal(getattr(opts[0], n), getattr(opts[1], n)), (step, n)


@pytest.mark.parametrize('B', [32, 7])
def test_forward_pair_equals_two_forwards(B):
  from dopamine_amd.agents.networks import RainbowNetwork
  from dopamine_amd.cnn import HipNatureCNN, forward_pair
  on, tg = RainbowNetwork(9, device='cuda', seed=1), RainbowNetwork(9, device='cuda', seed=2)
  ho, ht = HipNatureCNN(on, B), HipNatureCNN(tg, B)
  x, nx = torch.rand(B, 84, 84, 4, device='cuda'), torch.rand(B, 84, 84, 4, device='cuda')
  ref_o, ref_t = ho.forward(x).clone(), ht.forward(nx).clone()
  ho.acts['out'].zero_()
  ht.acts['out'].zero_()
  yo, yt = forward_pair(ho, x, ht, nx)
  torch.cuda.synchronize()
  assert torch.equal(yo, ref_o) and torch.equal(yt, ref_t)


@pytest.mark.parametrize('B', [32, 5])
def test_forward_head_and_tail_equal_forward(B):
  """Head (eager, or riding in another net's backward) + tail (in the other net's
  forward) == forward(), bit for bit; the backward's own gradients are unchanged
  by the riding head."""
  from dopamine_amd.agents.networks import RainbowNetwork
  from dopamine_amd.cnn import HipNatureCNN, forward_with_tail
  on, tg = RainbowNetwork(9, device='cuda', seed=1), RainbowNetwork(9, device='cuda', seed=2)
  ho, ht = HipNatureCNN(on, B), HipNatureCNN(tg, B)
  x, nx = torch.rand(B, 84, 84, 4, device='cuda'), torch.rand(B, 84, 84, 4, device='cuda')
  ref_o, ref_t = ho.forward(x).clone(), ht.forward(nx).clone()
  dout = torch.randn(B, ho.n_out, device='cuda')
  ho.backward(dout)
  ref_g = torch.cat([v.reshape(-1) for v in on.fp.grad_views])   # skips alignment pads
  ht.acts['out'].zero_()
  ht.forward_head(nx)
  yo, yt = forward_with_tail(ho, x, ht)
  torch.cuda.synchronize()
  assert torch.equal(yo, ref_o) and torch.equal(yt, ref_t)
  # the head riding in the online backward, then the tail in the next forward
  ht.acts['out'].zero_()
  on.fp.grad.zero_()
  ho.backward(dout, head=(ht, nx))
  torch.cuda.synchronize()
  assert torch.equal(torch.cat([v.reshape(-1) for v in on.fp.grad_views]), ref_g)
  yo, yt = forward_with_tail(ho, x, ht)
  torch.cuda.synchronize()
  assert torch.equal(yo, ref_o) and torch.equal(yt, ref_t)


@pytest.mark.parametrize('B,A', [(32, 9), (7, 4)])
def test_fused_forward_and_c51_equal_separate_path(B, A):
  """The Rainbow fast path: forward_fused's fc2 k-band partials summed by
  c51_loss_fused give bitwise dq_cnn_forward's logits (written out on request)
  and therefore bitwise dq_c51_loss's gradient, loss and priorities; its fused fc2
  input gradient equals the backward's dX_fc2 within fp32 reordering; the
  backward from launch 1 then matches the full backward within tolerance."""
  from dopamine_amd import ops
  from dopamine_amd.agents.networks import RainbowNetwork
  from dopamine_amd.cnn import HipNatureCNN, forward_fused
  N = 51
  on, tg = RainbowNetwork(A, device='cuda', seed=1), RainbowNetwork(A, device='cuda', seed=2)
  with torch.no_grad():
    for net in (on, tg):
      for n, prm in net.fp.params.items():
        if n.endswith('_b'):
          prm.uniform_(-0.05, 0.1)
  ho, ht = HipNatureCNN(on, B), HipNatureCNN(tg, B)
  torch.manual_seed(3)
  x, nx = torch.rand(B, 84, 84, 4, device='cuda'), torch.rand(B, 84, 84, 4, device='cuda')
  act = torch.randint(0, A, (B,), device='cuda', dtype=torch.int32)
  rew = torch.randn(B, device='cuda')
  term = (torch.rand(B, device='cuda') < 0.2).to(torch.uint8)
  probs = torch.rand(B, device='cuda') + 0.1
  sup = torch.linspace(-10, 10, N, device='cuda')
  ref_t = ht.forward(nx).clone()
  ref_o = ho.forward(x).clone()
  ref_h = ho.acts['h'].clone()
  ref = ops.c51_loss(ref_o.view(B, A, N), ref_t.view(B, A, N), act, rew, term, sup, 0.970299,
                     probs=probs)
  ref = {k: v.clone() for k, v in ref.items()}
  ho.backward(ref['grad'].view(B, -1))
  ref_dh = ho.dacts['h'].clone()
  ref_g = torch.cat([v.reshape(-1) for v in on.fp.grad_views]).clone()
  # fused: the target's head (conv1..conv3) stays from its forward above; fc1 slabs redone
  for t in (ho.acts['out'], ht.acts['out'], ho.acts['h'], ho.dacts['h']):
    t.fill_(float('nan'))
  forward_fused(ho, x, ht)
  got = ops.c51_loss_fused(ho, ht, act, rew, term, sup, 0.970299, probs=probs, logits_out=True)
  torch.cuda.synchronize()
  assert torch.equal(ho.acts['h'], ref_h)
  assert torch.equal(ho.acts['out'], ref_o) and torch.equal(ht.acts['out'], ref_t)
  for k in ('grad', 'loss', 'priorities'):
    assert torch.equal(got[k], ref[k]), k
  _close(ho.dacts['h'], ref_dh, rtol=1e-5)
  on.fp.grad.fill_(float('nan'))
  ho.backward(got['grad'].view(B, -1), groups=(1, 7))
  torch.cuda.synchronize()
  g7 = torch.cat([v.reshape(-1) for v in on.fp.grad_views]).clone()
  _close(g7, ref_g, rtol=2e-5)
  # the five-launch schedule (head_from = 5): the same gradient bit for bit, the target
  # head's conv1/conv2 riding in launches 4/5 and its conv3 + fc1 slabs in forward_fused
  # (head_from 6 / 7: its conv2 / conv1 too beside the online net's in forward_fused)
  nx2 = torch.rand(B, 84, 84, 4, device='cuda')
  ref_t2 = HipNatureCNN(tg, B).forward(nx2).clone()
  dh0 = ho.dacts['h'].clone()      # the backward's input; each pass's loss rewrites it
  for hf in (5, 6, 7):
    ho.dacts['h'].copy_(dh0)
    on.fp.grad.fill_(float('nan'))
    for t in (ht.acts['a1'], ht.acts['a2'], ht.acts['a3'], ht.acts['out']):
      t.fill_(float('nan'))
    ho.backward(got['grad'].view(B, -1), groups=(1, 7), head=(ht, nx2), head_from=hf)
    forward_fused(ho, x, ht, conv3_b=True, conv2_b=hf >= 6, xb=nx2 if hf == 7 else None)
    ops.c51_loss_fused(ho, ht, act, rew, term, sup, 0.970299, probs=probs, logits_out=True)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([v.reshape(-1) for v in on.fp.grad_views]), g7), hf
    assert torch.equal(ht.acts['out'], ref_t2) and torch.equal(ho.acts['out'], ref_o), hf
  # head_from = 8: the target net one launch ahead (conv1 in the backward as for 6) and
  # the C51 loss split -- its target half riding beside the online fused head, the loss
  # launch the online half: loss, gradient, priorities and d h bitwise the one kernel's
  from dopamine_amd.cnn import forward_fused_c51
  ho.dacts['h'].copy_(dh0)
  ho.backward(got['grad'].view(B, -1), groups=(1, 7), head=(ht, nx2), head_from=6)
  forward_fused(ho, x, ht, conv3_b=True, conv2_b=True)
  ref6 = {k: v.clone() for k, v in ops.c51_loss_fused(ho, ht, act, rew, term, sup, 0.970299,
                                                       probs=probs).items()}
  dh6 = ho.dacts['h'].clone()
  ho.dacts['h'].copy_(dh0)
  on.fp.grad.fill_(float('nan'))
  for t in (ht.acts['a1'], ht.acts['a2'], ht.acts['a3'], ht.acts['out']):
    t.fill_(float('nan'))
  ho.backward(got['grad'].view(B, -1), groups=(1, 7), head=(ht, nx2), head_from=6)
  for t in (ht.acts['a2'], ht.acts['a3'], ho.acts['out'], ho.acts['h']):   # the forward's outputs
    t.fill_(float('nan'))
  m = torch.full((B, N), float('nan'), device='cuda')
  forward_fused_c51(ho, x, ht, rew, term, sup, 0.970299, m, target_logits_out=ht.acts['out'])
  got8 = ops.c51_loss_online(ho, m, act, probs=probs, logits_out=True)
  torch.cuda.synchronize()
  assert torch.equal(torch.cat([v.reshape(-1) for v in on.fp.grad_views]), g7)
  assert torch.equal(ht.acts['out'], ref_t2) and torch.equal(ho.acts['out'], ref_o)
  assert torch.equal(ho.acts['h'], ref_h)
  for k in ('grad', 'loss', 'priorities'):
    assert torch.equal(got8[k], ref6[k]), k
  assert torch.equal(ho.dacts['h'], dh6)


@pytest.mark.parametrize('centered', [True, False])
def test_fused_rmsprop_backward_equals_backward_then_rmsprop(centered):
  """The backward with TF1 RMSProp spread over its launches (dq_adam_args kind
  DQ_OPT_RMSPROP) == dq_cnn_backward + dq_rmsprop_tf1, bitwise, over two steps, for
  the seven-launch schedule and the fused head's six-launch one (head_from 6)."""
  from dopamine_amd import ops
  from dopamine_amd.agents.networks import NatureDQNNetwork
  from dopamine_amd.cnn import HipNatureCNN
  nets = [NatureDQNNetwork(6, device='cuda', seed=5) for _ in range(2)]
  hips = [HipNatureCNN(n, 32) for n in nets]
  opts = [ops.TF1RMSProp(n.fp.flat, learning_rate=2.5e-4, decay=0.95, momentum=0.1,
                         epsilon=1e-5, centered=centered) for n in nets]
  torch.manual_seed(1)
  for step, groups in enumerate([None, (0, 7), None]):
    x = torch.rand(32, 84, 84, 4, device='cuda')
    gout = torch.randn(32, 6, device='cuda')
    for h in hips:
      h.forward(x)
    if groups is None:
      hips[0].backward(gout, adam=opts[0])
    else:   # the ride form: dq_cnn_backward_riders with no riders (head_from 6)
      hips[0].backward(gout, adam=opts[0], groups=groups, head_from=6)
    hips[1].backward(gout)
    opts[1].step(nets[1].fp.grad)
    torch.cuda.synchronize()
    for a, b in zip(nets[0].fp.grad_views, nets[1].fp.grad_views):
      assert torch.equal(a, b), step
    for n in ('params', 'ms', 'mg', 'mom'):       # on the parameters (k_rmsprop also
      for o, m in nets[0].fp.segments():          # moves ms of the alignment pads)
        assert torch.equal(getattr(opts[0], n)[o:o + m], getattr(opts[1], n)[o:o + m]), (step, n)


@pytest.mark.parametrize('B,A', [(32, 6), (7, 18)])
def test_fused_forward_and_dqn_loss_equal_separate_path(B, A):
  """The DQN fast path: forward_fused's fc2 partials summed by dqn_huber_loss_fused give
  bitwise dq_cnn_forward's Q-values and therefore bitwise dq_dqn_huber_loss's gradient
  and loss; its fused fc2 input gradient is bitwise the backward's launch 0 (one
  nonzero product per element), so the backward from launch 1 equals the full one."""
  from dopamine_amd import ops
  from dopamine_amd.agents.networks import NatureDQNNetwork
  from dopamine_amd.cnn import HipNatureCNN, forward_fused
  on, tg = NatureDQNNetwork(A, device='cuda', seed=1), NatureDQNNetwork(A, device='cuda', seed=2)
  with torch.no_grad():
    for net in (on, tg):
      for n, prm in net.fp.params.items():
        if n.endswith('_b'):
          prm.uniform_(-0.05, 0.1)
  ho, ht = HipNatureCNN(on, B), HipNatureCNN(tg, B)
  torch.manual_seed(3)
  x, nx = torch.rand(B, 84, 84, 4, device='cuda'), torch.rand(B, 84, 84, 4, device='cuda')
  act = torch.randint(0, A, (B,), device='cuda', dtype=torch.int32)
  rew = torch.randn(B, device='cuda') * 3     # some |TD error| > 1: both Huber branches
  term = (torch.rand(B, device='cuda') < 0.2).to(torch.uint8)
  ref_t = ht.forward(nx).clone()
  ref_o = ho.forward(x).clone()
  ref_h = ho.acts['h'].clone()
  ref = ops.dqn_huber_loss(ref_o, ref_t, act, rew, term, 0.99)
  ref = {k: v.clone() for k, v in ref.items()}
  ho.backward(ref['grad'])
  ref_dh = ho.dacts['h'].clone()
  ref_g = torch.cat([v.reshape(-1) for v in on.fp.grad_views]).clone()
  for t in (ho.acts['out'], ht.acts['out'], ho.acts['h'], ho.dacts['h']):
    t.fill_(float('nan'))
  forward_fused(ho, x, ht)
  got = ops.dqn_huber_loss_fused(ho, ht, act, rew, term, 0.99, q_out=True)
  torch.cuda.synchronize()
  assert torch.equal(ho.acts['h'], ref_h)
  assert torch.equal(ho.acts['out'], ref_o) and torch.equal(ht.acts['out'], ref_t)
  for k in ('grad', 'loss'):
    assert torch.equal(got[k], ref[k]), k
  assert torch.equal(ho.dacts['h'], ref_dh)
  assert abs(float(got['loss'].double().mean()) - float(ref['mean_loss'])) <= 1e-6 * (
      1 + abs(float(ref['mean_loss'])))
  on.fp.grad.fill_(float('nan'))
  ho.backward(got['grad'], groups=(1, 7), head_from=6)
  torch.cuda.synchronize()
  assert torch.equal(torch.cat([v.reshape(-1) for v in on.fp.grad_views]), ref_g)


def test_grouped_torso_backward_equals_per_layer_bitwise():
  """dq_cnn_backward_torso (IQN's torso: conv3 .. conv1 from d a3) in its four grouped
  launches == the per-layer launches of the same tiles (dq_cnn_backward_layer), bit for bit:
  every conv weight / bias gradient and the input gradients d a2, d a1."""
  import ctypes
  from dopamine_amd import _lib
  from dopamine_amd.agents.networks import RainbowNetwork
  from dopamine_amd.cnn import HipNatureCNN
  torch.manual_seed(3)
  net = RainbowNetwork(9, device='cuda', seed=2)
  hip = HipNatureCNN(net, 32)
  x = torch.rand(32, 84, 84, 4, device='cuda')
  hip.forward(x)
  da3 = torch.randn_like(hip.dacts['a3']) * (hip.acts['a3'] > 0)
  stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
  names = [n for n in net.fp.offsets if n.startswith('conv')]

  def run(grouped):
    net.fp.grad.fill_(float('nan'))
    hip.dacts['a3'].copy_(da3)
    hip.dacts['a2'].fill_(float('nan'))
    hip.dacts['a1'].fill_(float('nan'))
    if grouped:
      _lib.check(_lib.lib.dq_cnn_backward_torso(
          ctypes.byref(hip._p), ctypes.byref(hip._g), 32, hip._x.data_ptr(), ctypes.byref(hip._a),
          ctypes.byref(hip._d), hip.ws.data_ptr(), stream), 'dq_cnn_backward_torso')
    else:
      for layer, part in ((2, 1), (2, 0), (3, 1), (3, 0), (4, 1)):
        _lib.check(_lib.lib.dq_cnn_backward_layer(
            ctypes.byref(hip._p), ctypes.byref(hip._g), 32, hip._x.data_ptr(),
            ctypes.byref(hip._a), hip.dacts['a3'].data_ptr(), ctypes.byref(hip._d),
            hip.ws.data_ptr(), layer, part, stream), 'dq_cnn_backward_layer')
    torch.cuda.synchronize()
    import math
    g = {n: net.fp.grad[net.fp.offsets[n][0]:net.fp.offsets[n][0] +
                        math.prod(net.fp.offsets[n][1])].clone() for n in names}
    return g, hip.dacts['a2'].clone(), hip.dacts['a1'].clone()

  ga, a2a, a1a = run(True)
  gb, a2b, a1b = run(False)
  for n in names:
    assert torch.isfinite(ga[n]).all(), n
    assert torch.equal(ga[n], gb[n]), n
  assert torch.equal(a2a, a2b) and torch.equal(a1a, a1b)
