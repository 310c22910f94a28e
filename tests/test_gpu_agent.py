"""End-to-end learner step on the device vs a CPU restatement of the same step
(same sampled batch, same weights): loss, priorities, gradients and the TF1
Adam update.  Also: HIP-graph replay == eager execution."""
import random

import numpy as np
import pytest
import torch

from oracle import learner as OL

pytestmark = pytest.mark.gpu


def _fill(mem, A, seed):
  C = mem._replay_capacity
  rs = np.random.RandomState(seed)
  mem.load_arrays(torch.from_numpy(rs.randint(0, 256, (C, 84 * 84), dtype=np.uint8)),
                  torch.from_numpy(rs.randint(0, A, C).astype(np.int32)),
                  torch.from_numpy(rs.choice(np.array([-1, 0, 1], np.float32), C)),
                  torch.from_numpy((rs.rand(C) < 0.01).astype(np.uint8)), add_count=C + 77,
                  priorities=rs.uniform(0.1, 2.0, C) if mem._prioritized else None)


def _rainbow(**kw):
  from dopamine_amd.agents.optimizers import AdamOptimizer
  from dopamine_amd.agents.rainbow.rainbow_agent import RainbowAgent
  a = RainbowAgent(num_actions=9, update_horizon=3, replay_capacity=3000, batch_size=32,
                   min_replay_history=100, optimizer=AdamOptimizer(6.25e-5, epsilon=1.5e-4), **kw)
  _fill(a._replay.memory, 9, 3)
  return a


def test_rainbow_step_matches_cpu_restatement():
  random.seed(11)
  a = _rainbow(use_hip_graph=False)
  w0 = a.online_convnet.fp.flat.detach().cpu().clone()
  tw = a.target_convnet.fp.flat.detach().cpu().clone()
  a._run_train_op()
  torch.cuda.synchronize()
  t = {k: v.detach().cpu() for k, v in a._replay.transition.items()}
  # CPU restatement on the same batch and weights
  from dopamine_amd.agents.networks import RainbowNetwork
  on = RainbowNetwork(9, device='cpu'); on.fp.flat.copy_(w0)
  tg = RainbowNetwork(9, device='cpu'); tg.fp.flat.copy_(tw)
  with torch.no_grad():
    tl = tg(t['next_state']).double().numpy()
  logits = on(t['state'])
  exp = OL.c51_loss(logits.detach().double().numpy(), tl, t['action'].numpy(), t['reward'].numpy(),
                    t['terminal'].numpy(), OL.c51_support(10.0, 51, np.float32), np.float32(0.99 ** 3),
                    t['sampling_probabilities'].numpy())
  np.testing.assert_allclose(a._loss_out['loss'].cpu().numpy(), exp['loss'], rtol=1e-4, atol=1e-5)
  on.fp.grad.zero_()
  logits.backward(torch.from_numpy(exp['grad'].astype(np.float32)))
  np.testing.assert_allclose(a.online_convnet.fp.gather_grads().cpu().numpy(), on.fp.grad.numpy(),
                             rtol=1e-3, atol=1e-6)
  adam = OL.TF1Adam(on.fp.numel, 6.25e-5, eps=1.5e-4)
  w = w0.numpy().copy()
  adam.step(w, a.online_convnet.fp.gather_grads().cpu().numpy())
  np.testing.assert_allclose(a.online_convnet.fp.flat.cpu().numpy(), w, rtol=1e-5, atol=1e-7)
  # the priorities written back are sqrt(loss + 1e-10) of this step
  pri = a._replay.memory.get_priority(t['indices'].numpy().astype(np.int32))
  np.testing.assert_allclose(pri, np.sqrt(exp['loss'] + 1e-10), rtol=1e-4)


@pytest.mark.parametrize('kind', ['rainbow', 'dqn', 'iqn'])
def test_hip_graph_replay_matches_eager(kind):
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  from dopamine_amd.agents.implicit_quantile.implicit_quantile_agent import ImplicitQuantileAgent

  def make(graph):
    random.seed(5); np.random.seed(5); torch.manual_seed(5)
    if kind == 'rainbow':
      return _rainbow(use_hip_graph=graph)
    if kind == 'dqn':
      a = DQNAgent(num_actions=6, replay_capacity=3000, batch_size=32, min_replay_history=100,
                   use_hip_graph=graph)
    else:
      a = ImplicitQuantileAgent(num_actions=4, replay_capacity=3000, batch_size=16,
                                num_tau_samples=8, num_tau_prime_samples=8, num_quantile_samples=4,
                                min_replay_history=100, update_horizon=3, replay_scheme='uniform',
                                use_hip_graph=graph)
    _fill(a._replay.memory, a.num_actions, 3)
    return a

  res = []
  for graph in (False, True):
    a = make(graph)
    idx = []
    for _ in range(8):
      a._run_train_op()
      idx.append(a._replay.transition['indices'].cpu().numpy().copy())
    a._replay.memory.sync_rng()
    res.append((np.stack(idx), a.online_convnet.fp.flat.cpu().numpy(), a.mean_loss()))
    assert (a._graphs is not None) == graph
  np.testing.assert_array_equal(res[0][0], res[1][0])
  # IQN's taus come from the device counter-based sampler: the graph draws what eager draws
  np.testing.assert_allclose(res[0][1], res[1][1], rtol=1e-4, atol=1e-6)


def test_pipelined_prefetch_is_invalidated_by_adds_and_host_draws():
  """The two-stream prefetch of step t+1's batch must not change what is drawn:
  add() and the agent's own random draws between steps rewind and redraw it."""
  res = []
  for pipe in (False, True):
    random.seed(3); np.random.seed(3); torch.manual_seed(3)
    a = _rainbow(use_hip_graph=False, pipeline=pipe)
    seq = []
    for step in range(8):
      a._run_train_op()
      seq.append(a._replay.transition['indices'].cpu().numpy().copy())
      if step % 2 == 0:
        a._store_transition(np.full((84, 84), step, np.uint8), 1, 0.5, False)
      if step % 3 == 1:
        a._select_action()            # epsilon = 1 here: draws from Python's random
    a._discard_prefetch()
    a._replay.memory.sync_rng()
    res.append((np.stack(seq), random.getstate(), a.online_convnet.fp.flat.cpu().numpy()))
  np.testing.assert_array_equal(res[0][0], res[1][0])
  assert res[0][1] == res[1][1]
  np.testing.assert_allclose(res[0][2], res[1][2], rtol=1e-5, atol=1e-7)


def test_iqn_with_prioritized_replay_keeps_insert_priorities():
  """IQN inherits Rainbow's replay_scheme default ('prioritized'); its train op
  never writes priorities back (iqn:314), so training must run and leave the
  sum tree's leaves untouched."""
  from dopamine_amd.agents.implicit_quantile.implicit_quantile_agent import ImplicitQuantileAgent
  random.seed(2); np.random.seed(2); torch.manual_seed(2)
  a = ImplicitQuantileAgent(num_actions=4, replay_capacity=3000, batch_size=16, num_tau_samples=8,
                            num_tau_prime_samples=8, num_quantile_samples=4, min_replay_history=100,
                            update_horizon=3)
  _fill(a._replay.memory, a.num_actions, 3)
  before = a._replay.memory.sum_tree.nodes[-1].copy()
  for _ in range(6):
    a._run_train_op()
  a._replay.memory.sync_rng()
  np.testing.assert_array_equal(a._replay.memory.sum_tree.nodes[-1], before)
  assert np.isfinite(a.mean_loss())


@pytest.mark.parametrize('kind', ['dqn', 'rainbow'])
def test_action_q_values_on_the_hip_cnn_match_torch(kind):
  """_select_action's Q-values (batch-1 HIP CNN graph) vs the PyTorch network on
  the same parameters, before and after an in-place parameter update."""
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  torch.manual_seed(3)
  a = (_rainbow(use_hip_graph=True) if kind == 'rainbow' else
       DQNAgent(num_actions=6, replay_capacity=3000, batch_size=32, min_replay_history=100))
  rs = np.random.RandomState(4)
  for _ in range(2):
    st = rs.randint(0, 256, (1, 84, 84, 4)).astype(np.float64)
    q_hip = a._q_values(st).clone()
    with torch.no_grad():
      x = torch.as_tensor(st, dtype=torch.float32, device='cuda').permute(0, 3, 1, 2) / 255.0
      q_ref = a._online_q(x.contiguous())
    torch.cuda.synchronize()
    scale = q_ref.abs().max().item() + 1e-30
    assert (q_hip - q_ref).abs().max().item() <= 2e-5 * scale
    with torch.no_grad():
      a.online_convnet.fp.flat.mul_(1.1)        # the graph reads the parameters in place


@pytest.mark.parametrize('kind', ['rainbow', 'dqn'])
@pytest.mark.parametrize('graph', [False, True])
def test_replay_riders_match_the_two_stream_schedule(kind, graph):
  """ride_replay (priority write-back -> sample -> gather as riders of the
  backward's grouped launches, one stream) draws the same batches and produces
  the same parameters and sum tree, bit for bit, as the two-stream prefetch
  (Rainbow's fused head off: it sums fc2's input gradient in another order)."""
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  res = []
  for ride in (False, True):
    random.seed(7); np.random.seed(7); torch.manual_seed(7)
    if kind == 'rainbow':
      a = _rainbow(use_hip_graph=graph, ride_replay=ride, fused_head=False)
    else:
      a = DQNAgent(num_actions=6, replay_capacity=3000, batch_size=32, min_replay_history=100,
                   use_hip_graph=graph, ride_replay=ride)
      _fill(a._replay.memory, 6, 3)
    idx = []
    for _ in range(9):
      a._run_train_op()
      idx.append(a._replay.transition['indices'].cpu().numpy().copy())
    a._discard_prefetch()
    a._replay.memory.sync_rng()
    leaves = a._replay.memory.sum_tree.nodes[-1].copy() if kind == 'rainbow' else None
    res.append((np.stack(idx), a.online_convnet.fp.flat.cpu().numpy(), leaves,
                a._replay.transition['state'].cpu().numpy()))
    assert (a._graphs is not None) == graph
  np.testing.assert_array_equal(res[0][0], res[1][0])
  np.testing.assert_array_equal(res[0][1], res[1][1])
  np.testing.assert_array_equal(res[0][3], res[1][3])
  if kind == 'rainbow':
    np.testing.assert_array_equal(res[0][2], res[1][2])


@pytest.mark.parametrize('graph', [False, True])
def test_fused_head_matches_the_plain_schedule(graph):
  """Rainbow's fused head (fc1 sum + fc2 partials in one launch, logits summed and
  fc2's input gradient formed in the loss kernel, backward from launch 1, the
  target head shifted one launch) draws the same batches and keeps parameters
  and priorities within fp32 reordering of the plain ride schedule over 9 steps."""
  res = []
  for fused in (False, True):
    random.seed(7); np.random.seed(7); torch.manual_seed(7)
    a = _rainbow(use_hip_graph=graph, ride_replay=True, fused_head=fused)
    assert a._fused() == fused
    idx = []
    for _ in range(9):
      a._run_train_op()
      idx.append(a._replay.transition['indices'].cpu().numpy().copy())
    a._discard_prefetch()
    a._replay.memory.sync_rng()
    res.append((np.stack(idx), a.online_convnet.fp.flat.cpu().numpy().astype(np.float64),
                a._replay.memory.sum_tree.nodes[-1].copy(), a._loss_out['loss'].cpu().numpy()))
  np.testing.assert_array_equal(res[0][0], res[1][0])
  np.testing.assert_allclose(res[1][1], res[0][1], rtol=0, atol=1e-6)
  np.testing.assert_allclose(res[1][2], res[0][2], rtol=1e-4)
  np.testing.assert_allclose(res[1][3], res[0][3], rtol=1e-4)


@pytest.mark.parametrize('kind', ['rainbow', 'dqn'])
def test_learner_loop_chunks_equal_per_call_loop(kind):
  """train_gradient_steps(n) (K consecutive steps per graph replay) == n *
  update_period _train_step() calls: same batches, parameters, sum tree, RNG state
  and training_steps, with target syncs falling inside and at the end of chunks."""
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  res = []
  for chunked in (False, True):
    random.seed(5); np.random.seed(5); torch.manual_seed(5)
    if kind == 'rainbow':
      a = _rainbow(target_update_period=28)
    else:
      a = DQNAgent(num_actions=6, replay_capacity=3000, batch_size=32, min_replay_history=100,
                   target_update_period=28)
      _fill(a._replay.memory, 6, 3)
    idx = []
    for n in (6, 5, 9, 3, 8):
      if chunked:
        a.train_gradient_steps(n)
      else:
        for _ in range(n * a.update_period):
          a._train_step()
      idx.append(a._replay.transition['indices'].cpu().numpy().copy())
    a._discard_prefetch()
    a._replay.memory.sync_rng()
    leaves = a._replay.memory.sum_tree.nodes[-1].copy() if kind == 'rainbow' else None
    ns = np.random.get_state()
    res.append((np.stack(idx), a.online_convnet.fp.flat.cpu().numpy(),
                a.target_convnet.fp.flat.cpu().numpy(), leaves, a.training_steps,
                a._opt_steps, random.getstate(), ns[1].copy(), ns[2]))
    if chunked:
      # a uniform replay's chunks draw and gather their batches at once (chunk gather)
      want = 'gchunk' if kind == 'dqn' else 'chunk'
      assert any(k[0] == want for k in a._graph_sets if isinstance(k, tuple)), 'no chunk ran'
  for x, y in zip(res[0], res[1]):
    if isinstance(x, np.ndarray):
      np.testing.assert_array_equal(x, y)
    else:
      assert x == y


@pytest.mark.parametrize('chunked', [False, True])
def test_per_rider_launch_placements_are_bitwise_the_same(chunked):
  """The PER riders' backward launches (write-back, sample, gather) are a schedule choice
  only: (1, 2, 3), (2, 3, 4), (1, 3, 4) and (2, 2, 3) (write-back and sample chained in one
  block of launch 2) give the same batches, parameters, target net, sum tree and RNG state,
  bit for bit, per call and in the learner loop (target syncs inside chunks)."""
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  res = []
  for at in ((1, 2, 3), (2, 3, 4), (1, 3, 4), (2, 2, 3)):
    random.seed(5); np.random.seed(5); torch.manual_seed(5)
    old = DQNAgent.rider_launches
    DQNAgent.rider_launches = at
    try:
      a = _rainbow(target_update_period=28)
      idx = []
      for n in (6, 5, 9):
        if chunked:
          a.train_gradient_steps(n)
        else:
          for _ in range(n * a.update_period):
            a._train_step()
        idx.append(a._replay.transition['indices'].cpu().numpy().copy())
      a._discard_prefetch()
      a._replay.memory.sync_rng()
      res.append((np.stack(idx), a.online_convnet.fp.flat.cpu().numpy(),
                  a.target_convnet.fp.flat.cpu().numpy(), a._replay.memory.sum_tree.nodes[-1].copy(),
                  a._replay.transition['next_state'].cpu().numpy(), random.getstate()))
    finally:
      DQNAgent.rider_launches = old
  for r in res[1:]:
    for x, y in zip(res[0], r):
      if isinstance(x, np.ndarray):
        np.testing.assert_array_equal(x, y)
      else:
        assert x == y


def test_chunk_gather_equals_per_step_gather_chunks():
  """DQN (uniform replay) learner loop: chunks whose K batches are drawn by one grouped
  sample and gathered by one K*B launch (chunk_gather) == chunks that sample and gather per
  step, bit for bit (batches, parameters, numpy RNG state), through chunk-to-chunk,
  chunk-to-per-call and target-sync transitions and a prefetch discarded by an add()."""
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  res = []
  for cg in (False, True):
    random.seed(7); np.random.seed(7); torch.manual_seed(7)
    a = DQNAgent(num_actions=6, replay_capacity=3000, batch_size=32, min_replay_history=100,
                 target_update_period=36)
    a.chunk_gather = cg
    _fill(a._replay.memory, 6, 3)
    idx = []
    for n in (9, 12, 2, 8, 4):
      a.train_gradient_steps(n)
      idx.append(a._replay.transition['indices'].cpu().numpy().copy())
    a._replay.add(np.zeros((84, 84), np.uint8), 1, 0.5, False)   # invalidates the prefetch
    for _ in range(8):
      a._train_step()
    idx.append(a._replay.transition['indices'].cpu().numpy().copy())
    a.train_gradient_steps(8)
    idx.append(a._replay.transition['indices'].cpu().numpy().copy())
    a._discard_prefetch()
    a._replay.memory.sync_rng()
    ns = np.random.get_state()
    res.append((np.stack(idx), a.online_convnet.fp.flat.cpu().numpy(),
                a.target_convnet.fp.flat.cpu().numpy(), a.training_steps, ns[1].copy(), ns[2]))
    keys = [k[0] for k in a._graph_sets if isinstance(k, tuple)]
    assert ('gchunk' in keys) == cg and ('chunk' in keys) != cg
  for x, y in zip(res[0], res[1]):
    if isinstance(x, np.ndarray):
      np.testing.assert_array_equal(x, y)
    else:
      assert x == y


@pytest.mark.parametrize('kind', ['rainbow'])
def test_device_epsilon_greedy_consumes_random_as_the_host_path(kind):
  """_select_action with a prioritized replay: the epsilon test, the explore draw and the
  greedy argmax as one kernel on the replay's RNG tape (dq_replay_egreedy) give the same
  actions, batches, parameters and Python `random` state as the host path (sync + draw),
  over 64 actions at epsilon 0.5 interleaved with adds and gradient steps."""
  from dopamine_amd.agents.implicit_quantile.implicit_quantile_agent import ImplicitQuantileAgent
  res = []
  for dev in (False, True):
    random.seed(13); np.random.seed(13); torch.manual_seed(13)
    if kind == 'rainbow':
      a = _rainbow(use_hip_graph=True)
    else:
      a = ImplicitQuantileAgent(num_actions=4, replay_capacity=3000, batch_size=16,
                                num_tau_samples=8, num_tau_prime_samples=8, num_quantile_samples=4,
                                min_replay_history=100, update_horizon=3)
      _fill(a._replay.memory, 4, 3)
    a.device_egreedy = dev
    a.epsilon_fn = lambda *args: 0.5
    rs = np.random.RandomState(0)
    acts, idx = [], []
    for i in range(64):
      a.state = rs.randint(0, 256, (1, 84, 84, 4)).astype(np.float64)
      acts.append(a._select_action())
      if i % 4 == 3:
        a._store_transition(np.full((84, 84), i, np.uint8), acts[-1], 0.5, False)
        a._run_train_op()
        idx.append(a._replay.transition['indices'].cpu().numpy().copy())
    a._discard_prefetch()
    a._replay.memory.sync_rng()
    res.append((acts, np.stack(idx), random.getstate(), a.online_convnet.fp.flat.cpu().numpy()))
  assert res[0][0] == res[1][0]
  assert len(set(res[1][0])) > 1
  np.testing.assert_array_equal(res[0][1], res[1][1])
  assert res[0][2] == res[1][2]
  np.testing.assert_array_equal(res[0][3], res[1][3])


@pytest.mark.parametrize('kind', ['rainbow', 'dqn'])
def test_fused_optimizer_without_gradient_stores_is_bitwise_the_same(kind):
  """keep_gradients=False (the bench's drive: the fused TF1 Adam / RMSProp consumes the
  gradient in registers, dq_adam_args.no_grad_store) leaves parameters, optimizer state
  and sum tree bitwise those of the gradient-storing backward, over graph-replayed chunks."""
  from dopamine_amd.agents.dqn.dqn_agent import DQNAgent
  res = []
  for keep in (True, False):
    random.seed(7); np.random.seed(7); torch.manual_seed(7)
    if kind == 'rainbow':
      a = _rainbow(target_update_period=40)
    else:
      a = DQNAgent(num_actions=6, replay_capacity=3000, batch_size=32, min_replay_history=100,
                   target_update_period=40)
      _fill(a._replay.memory, 6, 3)
    a.keep_gradients = keep
    assert a._fused_opt()
    a.train_gradient_steps(3)
    a.train_gradient_steps(12)
    a._discard_prefetch()
    torch.cuda.synchronize()
    slots = (a._opt.m, a._opt.v) if kind == 'rainbow' else (a._opt.ms, a._opt.mom, a._opt.mg)
    st = [t.cpu().clone() for t in slots]
    leaves = a._replay.memory.sum_tree.nodes[-1].copy() if kind == 'rainbow' else None
    res.append((a.online_convnet.fp.flat.cpu().clone(), st, leaves, a._opt_steps))
  assert torch.equal(res[0][0], res[1][0])
  for x, y in zip(res[0][1], res[1][1]):
    assert torch.equal(x, y)
  if kind == 'rainbow':
    np.testing.assert_array_equal(res[0][2], res[1][2])
  assert res[0][3] == res[1][3]
  # the captured graphs bake the choice in: changing it afterwards is refused
  with pytest.raises(RuntimeError, match='keep_gradients'):
    a.keep_gradients = True
  a.keep_gradients = False                   # unchanged: allowed
