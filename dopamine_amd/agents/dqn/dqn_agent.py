"""DQN agent with the reference's API (dopamine/agents/dqn/dqn_agent.py:76-551).

Graph-mode TF1 is replaced by: device-resident replay (HIP sampler + gather),
PyTorch-ROCm Nature-CNN forward/backward over a flat parameter buffer, the
Bellman target + Huber loss as one HIP kernel, and the TF1 optimizer as one
HIP kernel.  After a few eager warm-up steps the whole gradient step
(sample -> gather -> online/target forward -> loss -> backward -> optimizer)
is captured into a HIP graph and replayed.  ``sess`` and ``tf_device`` are
accepted for signature compatibility.
"""
import ctypes
import math
import os
import random

import numpy as np
import torch

from dopamine_amd import _lib
from dopamine_amd import ops
from dopamine_amd import parallel
from dopamine_amd.agents import networks
from dopamine_amd.agents.optimizers import RMSPropOptimizer
from dopamine_amd.replay_memory import circular_replay_buffer

NATURE_DQN_OBSERVATION_SHAPE = (84, 84)
NATURE_DQN_DTYPE = np.uint8
NATURE_DQN_STACK_SIZE = 4
nature_dqn_network = networks.NatureDQNNetwork


def linearly_decaying_epsilon(decay_period, step, warmup_steps, epsilon):
  """dqn_agent.py:45-67."""
  steps_left = decay_period + warmup_steps - step
  bonus = (1.0 - epsilon) * steps_left / decay_period
  bonus = np.clip(bonus, 0., 1. - epsilon)
  return epsilon + bonus


def identity_epsilon(unused_decay_period, unused_step, unused_warmup_steps, epsilon):
  return epsilon


def _device_of(tf_device, device):
  if device is not None:
    return torch.device(device)
  if tf_device and 'gpu' in tf_device.lower():
    try:
      return torch.device('cuda', int(tf_device.rsplit(':', 1)[-1]))
    except ValueError:
      pass
  return torch.device('cuda', torch.cuda.current_device())


class DQNAgent(object):
  """dqn_agent.py:76-551."""

  def __init__(self,
               sess=None,
               num_actions=None,
               observation_shape=NATURE_DQN_OBSERVATION_SHAPE,
               observation_dtype=NATURE_DQN_DTYPE,
               stack_size=NATURE_DQN_STACK_SIZE,
               network=networks.NatureDQNNetwork,
               gamma=0.99,
               update_horizon=1,
               min_replay_history=20000,
               update_period=4,
               target_update_period=8000,
               epsilon_fn=linearly_decaying_epsilon,
               epsilon_train=0.01,
               epsilon_eval=0.001,
               epsilon_decay_period=250000,
               tf_device='/gpu:0',
               eval_mode=False,
               use_staging=True,
               max_tf_checkpoints_to_keep=4,
               optimizer=RMSPropOptimizer(learning_rate=0.00025, decay=0.95, momentum=0.0,
                                          epsilon=0.00001, centered=True),
               summary_writer=None,
               summary_writing_frequency=500,
               allow_partial_reload=False,
               replay_capacity=1000000,
               batch_size=32,
               use_hip_graph=True,
               pipeline=True,
               use_hip_cnn=True,
               fuse_optimizer=True,
               pair_forward=False,
               ride_replay=True,
               fused_head=True,
               device=None,
               seed=0,
               process_group=None,
               shard_optimizer=False,
               native_comm=True,
               exchange='collective'):
    assert num_actions is not None
    assert isinstance(observation_shape, tuple)      # abstract_agent.py:34
    self.num_actions = num_actions
    self.observation_shape = tuple(observation_shape)
    self.observation_dtype = observation_dtype
    self.stack_size = stack_size
    self.network = network
    self.gamma = gamma
    self.update_horizon = update_horizon
    self.cumulative_gamma = math.pow(gamma, update_horizon)
    self.min_replay_history = min_replay_history
    self.target_update_period = target_update_period
    self.epsilon_fn = epsilon_fn
    self.epsilon_train = epsilon_train
    self.epsilon_eval = epsilon_eval
    self.epsilon_decay_period = epsilon_decay_period
    self.update_period = update_period
    self.eval_mode = eval_mode
    self.training_steps = 0
    self.optimizer = optimizer
    self.summary_writer = summary_writer
    self.summary_writing_frequency = summary_writing_frequency
    self.allow_partial_reload = allow_partial_reload
    self.max_tf_checkpoints_to_keep = max_tf_checkpoints_to_keep
    self._replay_capacity = replay_capacity
    self._batch_size = batch_size
    self._device = _device_of(tf_device, device)
    self._seed = seed
    self._pg = process_group
    # N > 1 with TF1 Adam: ZeRO-1 for the fc bucket (reduce-scatter, each rank's Adam on
    # its 1/N slice, all-gather of the parameters) instead of all-reduce + a full update
    self.shard_optimizer = bool(shard_optimizer)
    # N > 1 over RCCL: the gradient buckets go over the learner's own communicators
    # (parallel.RcclComm, issued on the stream each bucket runs on) instead of
    # torch.distributed's collectives (each forked onto the process group's own stream)
    self.native_comm = bool(native_comm)
    # N > 1: 'collective' -- the gradient buckets' all-reduce (RCCL / gloo) on a second stream
    # beside the backward (_split_step); 'peer' -- the exchange over peer memory inside the
    # backward's own launches on ONE stream (parallel.PeerExchange): one node,
    # the HIP Nature CNN with the fused Rainbow schedule and TF1 Adam
    if exchange not in ('collective', 'peer'):
      raise ValueError("exchange must be 'collective' or 'peer'")
    self.exchange = exchange
    self._peer = None
    self._rccl = None
    self._pg_conv = None           # a second communicator for the conv bucket (see _split_step)
    self._fc_pending = None        # event: the previous step's fc all-reduce + update are done
    self._defer_fc = False         # set by train_gradient_steps (learner-only loop)
    self.use_hip_graph = use_hip_graph
    self.pipeline = pipeline
    self.use_hip_cnn = use_hip_cnn
    self.fuse_optimizer = fuse_optimizer
    self.pair_forward = pair_forward
    self.ride_replay = ride_replay
    self.fused_head = fused_head
    self._graph_sets = {}          # pipe -> (graphs per parity, optimizer graphs per parity)
    self._graph_pool = None
    self._eager_steps = {True: 0, False: 0}
    self._last_train_add_count = -1
    self._selects_since_train = 0
    self._act = None
    self._opt_steps = 0
    self._slot = 0
    self._pbuf = [None, None]
    self._ptgt = [None, None]
    self._has_prefetch = False
    self._prefetch_add_count = -1
    self._cb = None                # chunk gather: 2 sets of _UNROLL batches (see _chunk_gathers)
    self._cb_ready = None          # set p: the prefetched batch is set p's last one
    self._gather_plan = None       # (set, step) while a chunk-gather graph is captured
    self._online_ready = None
    self._head = None              # (target net, input) whose forward head rides in the backward
    self._tail_head = None         # ... in the N > 1 tail graph
    self._sess = sess
    self._trace = None             # enable_trace(): per-step copies for the parity tests

    state_shape = (1,) + self.observation_shape + (stack_size,)
    self.state = np.zeros(state_shape)
    with torch.cuda.device(self._device):
      self._replay = self._build_replay_buffer(use_staging)
      self._build_networks()
      self._build_train_op()
      self._opt = self.optimizer.build(self.online_convnet.fp.flat,
                                       segments=self.online_convnet.fp.segments())
      self._side = torch.cuda.Stream(self._device, priority=self.side_priority)
      # N > 1: the fc bucket's all-reduces (comm_priority -1: a high-priority queue, whose
      # workgroups are dispatched ahead of the main queue's pending ones)
      self._comm = torch.cuda.Stream(self._device, priority=self.comm_priority)
      self._comm_opt = torch.cuda.Stream(self._device)    # ... and the Adam parts behind them
      if self._pg is not None:
        self._broadcast_replica()
        if self.exchange == 'peer':
          self._peer = self._make_peer_exchange()
        self._rccl = self._make_native_comms()
    self._observation = None
    self._last_observation = None
    self.last_loss = None

  def _replica_tensors(self):
    """Everything a replica's updates depend on: parameters and optimizer state."""
    ts = [self.online_convnet.fp.flat, self.target_convnet.fp.flat]
    ts += [v for k, v in sorted(vars(self._opt).items())
           if isinstance(v, torch.Tensor) and v.data_ptr() != self.online_convnet.fp.flat.data_ptr()]
    return ts

  def _make_native_comms(self):
    """(fc bucket, conv bucket) RcclComm pair for the split schedule over RCCL, or None
    (gloo, or a schedule without buckets).  Collective: every rank constructs its agent."""
    import torch.distributed as dist
    if not (self.native_comm and self._split_allreduce() and dist.get_backend(self._pg) == 'nccl'):
      return None
    if not parallel.native_comm_available(self._pg, self._device):
      return None        # every rank agreed: torch.distributed's collectives instead
    return (parallel.RcclComm(self._pg, self._device), parallel.RcclComm(self._pg, self._device))

  def _make_peer_exchange(self):
    """The peer-memory exchange (exchange='peer').  Collective: every rank constructs its
    agent.  Raises if the learner's schedule or placement cannot run it."""
    if not (self._hip is not None and isinstance(self._opt, ops.TF1Adam) and self._fused()
            and self._head_from() == 6 and self.fuse_optimizer):
      raise ValueError("exchange='peer' needs the HIP Nature CNN's fused schedule (ride_replay, "
                       "fused_head, fuse_optimizer) and TF1 Adam")
    if not parallel.PeerExchange.available(self._pg, self._device):
      raise RuntimeError("exchange='peer': the learners are not on one node with peer access "
                         "between their devices")
    lo, n = self._shard_bounds()
    if lo != n - self._grad_buckets()[0].numel():
      # a head of fc1 floats would join the replicated conv bucket, which the peers read in
      # the exchange launch after this learner may have rewritten it (dq_cnn_backward_peer)
      raise ValueError("exchange='peer': the fc bucket does not split into %d equal 16-byte "
                       'slices (networks.FC_BUCKET_ALIGN)' % self._world())
    return parallel.PeerExchange(self._pg, self._device, self.online_convnet.fp.grad,
                                 self.online_convnet.fp.flat, lo, n)

  def _collective(self):
    """N > 1 with the gradient exchange outside the backward (collectives between graphs or
    on a second stream); False for a single replica and for the peer exchange, whose
    learners run the single-replica schedule on one stream."""
    return self._pg is not None and self._peer is None

  def close(self):
    """Releases the learner's RCCL communicators (each holds proxy threads and device
    buffers until destroyed) or peer mappings: waits for the device, drops the HIP graphs
    that captured their collectives, then destroys them.  The agent cannot train
    afterwards.  A no-op for a single replica.  With the peer exchange it is collective: the
    learners meet at a host barrier before unmapping, so none frees buffers another's last
    launches still read."""
    self._join_fc()
    torch.cuda.synchronize(self._device)
    if self._peer is not None:
      import torch.distributed as dist
      dist.barrier(group=self._pg)
      self._graph_sets = {}
      self._graph_pool = None
      self._peer.close()
      self._peer = None
      self._closed = True
    if self._rccl is not None:
      self._graph_sets = {}
      self._graph_pool = None
      parallel.forget_capture_probes(self._rccl)
      for c in self._rccl:
        c.destroy()
      self._rccl = None
      self._closed = True

  _closed = False

  def _ar_fc(self, t):
    """The fc bucket's all-reduce (mean), on the current (comm) stream."""
    if self._rccl is not None:
      return self._rccl[0].allreduce_mean_(t)
    return parallel.allreduce_mean_(t, self._pg)

  def _ar_conv(self, t, second):
    """The conv bucket's all-reduce (mean), on the current (main) stream: over the second
    communicator when the fc bucket's may still be in flight on the first."""
    if self._rccl is not None:
      return self._rccl[1].allreduce_mean_(t)
    return parallel.allreduce_mean_(t, self._conv_group() if second else self._pg)

  def _broadcast_replica(self):
    """Data-parallel replicas start from group rank 0's networks and optimizer state
    (whatever seed each rank was built with), so the identical all-reduced updates
    keep them bit-identical (parallel.replicas_in_sync)."""
    import torch.distributed as dist
    src = dist.get_process_group_ranks(self._pg)[0]
    for t in self._replica_tensors():
      dist.broadcast(t, src=src, group=self._pg)
    torch.cuda.synchronize(self._device)

  # ---------------------------------------------------------------- tracing
  # Parity tests compare every step of the bench path (graph replays, chunks) with a
  # float64 CPU restatement.  enable_trace() (before the first step, so captured graphs
  # include it) makes each step copy its batch, network outputs, loss outputs and flat
  # gradient into ring slot j of self._trace: chunk step j -> slot j (< _UNROLL), a
  # single-step graph or eager step of parity k -> slot _UNROLL + k.  Copies only: the
  # step's own kernels and arithmetic are those of the untraced path.
  def enable_trace(self):
    assert not self._graph_sets, 'enable_trace() must precede the first gradient step'
    self._trace = {}

  def _trace_outputs(self, c):
    """name -> device tensor of step slot c's results (subclasses add theirs)."""
    t = self._pbuf[c]
    d = {k: t[k] for k in ('indices', 'action', 'reward', 'terminal', 'next_action',
                           'next_reward', 'state', 'next_state', 'sampling_probabilities')
         if k in t}
    d['loss'] = self._loss_out['loss']
    d['grad_out'] = self._loss_out['grad']
    if self._needs_flat_grad():
      d['grad'] = self.online_convnet.fp.grad
    else:   # the optimizer reads autograd's per-parameter tensors: copy them into the flat one
      d['grad'] = self.online_convnet.fp.gather_grads()
    if self._hip is not None:
      d['online_out'] = self._hip['online'].acts['out']
      d['target_out'] = self._hip['target'][c].acts['out']
      for k in ('a1', 'a2', 'a3', 'h'):    # the online forward's ReLU outputs (mask pinning)
        d['act_' + k] = self._hip['online'].acts[k]
    elif getattr(self, '_last_online_out', None) is not None and 'q' in (self._ptgt[c] or {}):
      d['online_out'] = self._last_online_out       # the PyTorch-network path (e.g. CartPole)
      d['target_out'] = self._ptgt[c]['q']
    return d

  def _trace_step(self, slot, c):
    if self._trace is None:
      return
    n = self._UNROLL + 2
    for k, v in self._trace_outputs(c).items():
      if k not in self._trace:
        self._trace[k] = torch.zeros((n,) + tuple(v.shape), dtype=v.dtype, device=v.device)
      self._trace[k][slot].copy_(v.detach())

  # ------------------------------------------------------------ graph parts
  def _build_replay_buffer(self, use_staging):
    return circular_replay_buffer.WrappedReplayBuffer(
        observation_shape=self.observation_shape, stack_size=self.stack_size,
        use_staging=use_staging, update_horizon=self.update_horizon, gamma=self.gamma,
        observation_dtype=self.observation_dtype, replay_capacity=self._replay_capacity,
        batch_size=self._batch_size, device=self._device)

  def _make_network(self, seed):
    if self.network is networks.CartpoleDQNNetwork:
      return self.network(self.num_actions, device=self._device, seed=seed)
    return self.network(self.num_actions, stack_size=self.stack_size, device=self._device, seed=seed)

  def _build_networks(self):
    self.online_convnet = self._make_network(self._seed)
    self.target_convnet = self._make_network(self._seed + 1)
    # Nature-CNN nets run on the HIP implicit-GEMM kernels (dopamine_amd/cnn.py);
    # the torch modules keep the parameters (flat buffer) and serve action selection.
    self._hip = None
    if (self.use_hip_cnn and self.network in (networks.NatureDQNNetwork, networks.RainbowNetwork)
        and self.observation_shape == NATURE_DQN_OBSERVATION_SHAPE and self.stack_size == 4):
      from dopamine_amd.cnn import HipNatureCNN
      B = self._batch_size
      self._hip = dict(online=HipNatureCNN(self.online_convnet, B),
                       target=[HipNatureCNN(self.target_convnet, B) for _ in range(2)])

  def _online_forward(self, x):
    """Online network output for the loss (keeps what the backward needs)."""
    if self._hip is not None:
      ready, self._online_ready = self._online_ready, None
      if ready is not None:             # already computed by _forward_pair
        return ready
      return self._hip['online'].forward(x)
    return self.online_convnet(self._state_input(x))

  def _target_net(self, x, slot):
    """Target network output (no gradient) into pipeline slot ``slot``."""
    if self._hip is not None:
      return self._hip['target'][slot].forward(x)
    with torch.no_grad():
      return self.target_convnet(self._state_input(x))

  def _build_train_op(self):
    B, A, dev = self._batch_size, self.num_actions, self._device
    self._loss_out = dict(grad=torch.empty((B, A), device=dev), loss=torch.empty(B, device=dev),
                          mean_loss=torch.empty(1, device=dev))

  def _state_input(self, x):
    """(B, stack, ...) device tensor from the gather -> network input."""
    if self.observation_shape == NATURE_DQN_OBSERVATION_SHAPE:
      return x
    return x.reshape(x.shape[0], -1)

  # The gradient step is split so it can be pipelined:
  #   _target_forward(t)      target-network outputs the loss needs (no grad)
  #   _online_loss(t, tgt)    online forward + the loss kernel -> (output, d loss/d output)
  #   _backward(y, g)         backward into the flat gradient
  def _target_forward(self, t, slot):
    return {'q': self._target_net(t['next_state'], slot)}

  def _online_loss(self, t, tgt):
    """dqn_agent.py:283-322."""
    q = self._online_forward(t['state'])
    self._last_online_out = q.detach()
    out = ops.dqn_huber_loss(q.detach(), tgt['q'], t['action'], t['reward'], t['terminal'],
                             self.cumulative_gamma, out=self._loss_out)
    return q, out['grad']

  def _fused_opt(self):
    """fuse_optimizer + single replica + HIP CNN + TF1 Adam or RMSProp: the optimizer
    step is spread over the backward's grouped launches (dq_cnn_backward_adam / _riders:
    float4 optimizer ops on each parameter range once its gradient is final, conv1's
    split-K sum applying it in its epilogue).  Bitwise identical to the separate
    k_adam / k_rmsprop step and 3.5% faster on MI355X for Adam (5,500 vs 5,315
    steps/s).  (Earlier forms were slower: the whole update in the last launch -1.5%;
    Adam in every gradient epilogue -12%, scalar RMW of 4M fc1 parameters.)"""
    return (self.fuse_optimizer and self._hip is not None and not self._collective() and
            isinstance(self._opt, (ops.TF1Adam, ops.TF1RMSProp)))

  def _store_grads(self):
    """Whether the fused-optimizer backward also writes the gradients it consumes to the
    flat gradient buffer: for ``keep_gradients`` (the agent's attribute; TF keeps no
    such buffer, so the bench drives the agent with it off) and while tracing.  The
    parameters and optimizer state are bitwise the same either way."""
    return bool(self.keep_gradients or self._trace is not None)

  def _backward(self, y, g, k=0):
    if self._peer is not None:      # the exchange inside the backward (non-pipelined steps too)
      self._hip['online'].backward_peer(g, self._opt, k, self._peer.desc)
      return
    if self._hip is not None:       # all gradients stored into the flat buffer
      groups = (1, 7) if self._fused() else None    # fused: d h came with the loss
      if self._fused_opt():
        self._hip['online'].store_grads = self._store_grads()
        self._hip['online'].backward(g, adam=self._opt, slot=k, groups=groups)
      else:
        self._hip['online'].backward(g, groups=groups)
      return
    # Fresh per-parameter gradients (no flat-buffer zeroing + accumulate kernels);
    # the multi-tensor TF1 Adam reads them in place.
    for prm in self.online_convnet.parameters():
      prm.grad = None
    y.backward(g)
    if self._needs_flat_grad():
      self.online_convnet.fp.gather_grads()

  def _needs_flat_grad(self):
    return (self._hip is not None or self._pg is not None or
            not getattr(self._opt, 'supports_multi', False))

  # Pipelined step.  Slot c holds step t's batch and its target-net outputs.
  # After step t's loss kernel (and priority write-back) a second HIP stream
  # samples + gathers step t+1's batch into slot 1-c and runs the target net on
  # it, concurrently with step t's backward and optimizer on the main stream.
  # Step t+1's sample still follows step t's set_priority, so draws and indices
  # are exactly the reference's; a prefetch made stale by add() or host RNG use
  # is rewound (dq_replay_rewind_last_sample) and redrawn.
  def _target_dict(self, out):
    """The target network's raw output as the loss kernel's inputs."""
    return {'q': out}

  def _rides(self):
    """ride_replay: HIP-CNN steps run on ONE stream (plus, with N > 1 replicas, the
    all-reduce's comm stream).  The next
    batch's priority write-back -> sample -> gather are recorded as riders of the
    backward's first grouped launches (dq_cnn_backward_riders), the target net's
    forward head on that batch rides in its last four, and the step after finishes
    the target forward in the online forward's last two launches
    (dq_cnn_forward_with_tail).  No second stream: the graph has no cross-queue
    fork/join edges (they cost ~28 us of a ~190 us step on MI355X), and the
    target forward adds no launches of its own."""
    return self.ride_replay and self._hip is not None

  def _fused(self):
    """fused_head: the loss kernel consumes the CNN's fc2 k-band partials and writes
    fc2's input gradient (cnn.forward_fused + _fused_loss), so the forward and the
    backward each lose a launch (the Nature-CNN agents: DQN's Huber here, Rainbow's C51
    in its subclass)."""
    return self.fused_head and self._rides()

  def _fused_loss(self, t, c):
    """_online_loss on the CNN's fc2 partials: Q / Q' summed in the loss kernel
    (dq_dqn_huber_loss_fused), which also writes fc2's input gradient."""
    out = ops.dqn_huber_loss_fused(self._hip['online'], self._hip['target'][c], t['action'],
                                   t['reward'], t['terminal'], self.cumulative_gamma,
                                   out=self._loss_out, q_out=self._trace is not None)
    return None, out['grad']

  def _loss(self, t, c):
    """(output, d loss / d output) of step slot c, by the fused or the plain path."""
    if self._fused():
      return self._fused_loss(t, c)
    return self._online_loss(t, self._ptgt[c])

  def _forward_ride(self, c, part=None):
    """The online forward of slot c with the target network's tail (ride mode).
    part: 'convs' / 'fcs' -- the fused path's conv / fc launches only."""
    from dopamine_amd import cnn
    if self._fused():
      hf = self._head_from()
      if hf == 8:                   # the target net one launch ahead, its C51 half riding
        self._forward_fused_c51(c, part)
        return
      cnn.forward_fused(self._hip['online'], self._pbuf[c]['state'], self._hip['target'][c],
                        conv3_b=hf >= 5, conv2_b=hf >= 6, part=part,
                        xb=self._pbuf[c]['next_state'] if hf == 7 else None,
                        **self._peer_fwd_gather())
      return
    assert part is None
    on, tg = cnn.forward_with_tail(self._hip['online'], self._pbuf[c]['state'], self._hip['target'][c])
    self._online_ready = on
    self._ptgt[c] = self._target_dict(tg)

  def _place_riders(self, riders):
    """Rider i of the returned list rides in backward launch first + i.  The PER riders
    (write-back, sample, gather, in that order) of the fused schedule go to rider_launches
    (default (2, 3, 4); the other placements measured are in DESIGN.md 4.2; all are bitwise
    the same).  A chunk gather's K * B gather (a chunk's first step) rides in backward launch
    chunk_gather_launch (it must precede the next batch's target head, launch 5)."""
    if self._gather_plan is not None and len(riders) == 2 and self.chunk_gather_launch > 2:
      empty = [_lib.Rider() for _ in range(self.chunk_gather_launch - 2)]
      return riders[:1] + empty + riders[1:]
    if len(riders) == 3 and self._fused():            # PER: write-back, sample, gather
      # (the fused head's backward starts at launch 1 and its target conv1 rides in launch 5;
      # the plain schedule's starts at 0 with the target head from launch 3, so there the
      # riders keep launches 0, 1, 2)
      at = self.rider_launches or (1, self.sample_launch, self.sample_launch + 1)
      if tuple(at) != (1, 2, 3):
        # the target conv1 (launch 5) reads the gather; write-back and sample in ONE launch
        # run chained in one block (dq_rider_chain: the draw after the write-back).  Any
        # other order would race (e.g. the gather beside the conv1 that reads it): an error
        # under python -O too
        if not (len(at) == 3 and 1 <= at[0] <= at[1] < at[2] <= 4):
          raise ValueError('rider_launches %r: need 1 <= write-back <= sample < gather <= 4'
                           % (tuple(at),))
        placed = [_lib.Rider() for _ in range(at[2])]
        if at[0] == at[1]:
          chained = _lib.Rider()
          _lib.call('dq_rider_chain', ctypes.byref(riders[0]), ctypes.byref(riders[1]),
                    ctypes.byref(chained))
          riders, at = [chained, riders[2]], at[1:]
        for r, i in zip(riders, at):
          placed[i - 1] = r
        return placed
    return riders

  chunk_gather_launch = 3
  # the backward launch the PER sample rides in (the gather in the next one; the target
  # head, from launch 5 on, needs the gathered batch): 2, or 3 (a schedule experiment)
  sample_launch = 2
  # (write-back, sample, gather) launches of the PER riders, overriding sample_launch; None =
  # (1, sample_launch, sample_launch + 1).  (2, 3, 4): launch 1 (dX fc1) carries no rider,
  # the sample leaves launch 3 its gather blocks' slots, the gather rides in launch 4
  # (+1.3%, same box: DESIGN 4.2)
  rider_launches = (2, 3, 4)

  def _forward_fused_c51(self, c, part=None):
    raise NotImplementedError

  # The peer exchange's all-gather inside the learner loop's chunk graphs: every step
  # publishes its updated slice and gathers a quarter of the others' in backward launch 5, the
  # next step's three conv forward launches gather the rest (they read no fc parameter; fc1's
  # launch follows) -- across chunk boundaries too: a chunk after another in the same
  # train_gradient_steps call starts with the gather its predecessor left (_peer_pending), and
  # the call ends with one dq_peer_all_gather launch (_peer_flush), as does anything inside it
  # that reads the parameters (a target sync, a per-call step).  Per-call steps keep the whole
  # gather in launch 5.  Bitwise the same parameters either way.
  _peer_defer_ag = False     # the backward being recorded defers its gather
  _peer_fwd_ag = False       # the forward being recorded gathers the previous step's
  _peer_pending = False      # the parameters await the last replayed step's deferred gather

  _peer_synced = False       # the learners met at a host barrier before this exchange began

  def resync_exchange(self):
    """The next gradient step of the peer exchange starts behind a host-side barrier of the
    process group (collective: every learner calls it at the same point, e.g. at the start of
    a training phase).  The exchange's device-side waits are bounded (they latch an error
    after PeerExchange.MAX_POLLS polls, tens of seconds), so learners that reach their first
    step far apart -- one still filling its replay or finishing an evaluation phase -- meet
    on the host first.  No-op without the peer exchange."""
    self._peer_synced = False

  def _peer_ready(self):
    if self._peer is not None and not self._peer_synced:
      import torch.distributed as dist
      torch.cuda.synchronize(self._device)
      dist.barrier(group=self._pg)
      self._peer_synced = True

  def _peer_flush(self):
    """Completes a deferred all-gather (one launch) so every parameter is current."""
    if self._peer_pending:
      self._peer.all_gather(self._opt.params, _lib.stream_of(self._device))
      self._peer_pending = False

  def _peer_fwd_gather(self):
    """forward_fused* keyword arguments of the deferred gather ({} when none rides)."""
    if not self._peer_fwd_ag:
      return {}
    return {'peer': self._peer.desc, 'var': self._opt.params}

  def _bwd_head_from(self):
    """head_from for the backward: 8 places the target's conv1 as 6 does."""
    hf = self._head_from()
    return 6 if hf == 8 else hf

  def _bwd_first(self):
    return 1 if self._fused() else 0

  def _head_from(self):
    """The backward's schedule: 7 launches with the target head from launch 3, or
    (fused) 5 launches from launch 1 with the target's conv1 in the last one and its
    conv2 / conv3 beside the online conv2 / conv3 of the next forward (measured: +1.4%
    over conv1, conv2 in the backward's launches 4, 5 (head_from 5); -0.7% with conv1
    in the next forward too (7))."""
    return 6 if self._fused() else 3

  def _pairs(self):
    return self.pair_forward and self._hip is not None and not self._rides()

  def _forward_pair(self, c):
    """pair_forward: the online net on s and the target net on s' of slot c in ONE
    pass (dq_cnn_forward_pair, 6 grouped launches) at the start of the step,
    instead of the target forward riding on the prefetch stream.  Measured slower
    (4938 vs 5260 steps/s): the prefetch-stream target forward is mostly hidden
    under the backward, while the pair lengthens the critical path."""
    from dopamine_amd.cnn import forward_pair
    t = self._pbuf[c]
    on, tg = forward_pair(self._hip['online'], t['state'], self._hip['target'][c], t['next_state'])
    self._online_ready = on
    self._ptgt[c] = self._target_dict(tg)

  def _prefetch(self, i):
    mem = self._replay.memory
    if self._gather_plan is not None:   # capturing a chunk-gather graph (_run_gather_chunk)
      p, j = self._gather_plan
      if j == 0:                        # the chunk's K next batches: one sample + one gather
        mem.sample_device(self._batch_size, layout=self._replay._layout, out=self._cb_sets()[p],
                          reserve=False, groups=self._UNROLL)
      t = self._cbv[p][j]               # the batch of the chunk's step j + 1
      self._pbuf[i] = t
      self._head = (self._hip['target'][i], t['next_state'])
      return
    t = mem.sample_device(self._batch_size, layout=self._replay._layout, out=self._pbuf[i],
                          reserve=False)
    self._pbuf[i] = t
    if self._rides():               # the target head now (or riding in the backward), tail in the step
      if mem._riders is not None:
        self._head = (self._hip['target'][i], t['next_state'])
      else:
        self._hip['target'][i].forward_head(t['next_state'])
      return
    if self._pairs():               # the target forward runs with the online one (_forward_pair)
      return
    tg = self._target_forward(t, i)
    if self._hip is not None:       # persistent per-slot output buffers: no copy
      self._ptgt[i] = tg
      return
    if self._ptgt[i] is None:
      self._ptgt[i] = {k: torch.empty_like(v) for k, v in tg.items()}
    for k, v in tg.items():
      self._ptgt[i][k].copy_(v)

  def _grad_step(self, c, k=0, pipe=None):
    pipe = self.pipeline if pipe is None else pipe
    if not pipe:
      self._prefetch(c)
    if self._rides():
      self._forward_ride(c)
    elif self._pairs():
      self._forward_pair(c)
    y, g = self._loss(self._pbuf[c], c)
    if pipe and self._rides():
      self._head = None
      with self._replay.memory.recording() as riders:
        self._post_loss(self._pbuf[c])
        self._prefetch(1 - c)
      riders = self._place_riders(riders)
      if self._peer is not None:      # the exchange inside the backward's launches (one stream)
        self._hip['online'].backward_peer(g, self._opt, k, self._peer.desc, riders=riders,
                                          head=self._head, defer_ag=self._peer_defer_ag)
        self._head = None
        return
      adam = self._opt if self._fused_opt() else None
      f = self._bwd_first()
      self._hip['online'].store_grads = self._store_grads()
      self._hip['online'].backward(g, riders=riders, adam=adam, slot=k, head=self._head,
                                   groups=(f, 7), head_from=self._bwd_head_from())
      self._head = None
    elif pipe:
      main = torch.cuda.current_stream(self._device)
      ev = torch.cuda.Event()
      ev.record(main)
      self._side.wait_event(ev)
      with torch.cuda.stream(self._side):
        self._post_loss(self._pbuf[c])
        self._prefetch(1 - c)
      self._backward(y, g, k)
      main.wait_stream(self._side)
    else:
      self._post_loss(self._pbuf[c])
      self._backward(y, g, k)

  # Data-parallel learners (N > 1) with the HIP CNN: the gradient all-reduce is
  # bucketed and overlapped.  The backward's first _SPLIT grouped launches leave
  # fc1/fc2's gradients final (93% of the 17.1 MB); their all-reduce runs on a
  # comm stream while the prefetch branch and the remaining launches run, then
  # the conv bucket is all-reduced and the optimizer applied.  Three graphs per
  # step parity: head | tail | optimizer, the collectives between them.
  _SPLIT = 3

  def _split_allreduce(self):
    return self._collective() and self._hip is not None and not self._fused_opt()

  def _head_splits(self):
    """The N > 1 head graph splits before fc1's forward (fused Rainbow path), so the
    previous step's fc all-reduce + update may still run under the conv launches."""
    return self._fused() and self._rides()

  def _grad_step_head(self, c, k, pipe=None, part=None):
    """part None: the whole head; 'a': up to the conv forward; 'b': the rest."""
    pipe = self.pipeline if pipe is None else pipe
    if part != 'b':
      if not pipe:
        self._prefetch(c)
      if part == 'a':
        self._forward_ride(c, part='convs')
        return
    if self._rides():
      self._forward_ride(c, part='fcs' if part == 'b' else None)
    elif self._pairs():
      self._forward_pair(c)
    y, g = self._loss(self._pbuf[c], c)
    f = self._bwd_first()
    self._tail_riders = None
    if pipe and self._rides():      # priority write-back -> sample -> gather ride in launches f..2
      self._head = None
      with self._replay.memory.recording() as riders:
        self._post_loss(self._pbuf[c])
        self._prefetch(1 - c)
      riders = self._place_riders(riders)
      n = self._SPLIT - f
      self._hip['online'].backward(g, groups=(f, self._SPLIT), riders=riders[:n])
      self._tail_riders = riders[n:] or None     # the fused path's gather rides in launch 3
      self._tail_head, self._head = self._head, None
    else:
      self._hip['online'].backward(g, groups=(f, self._SPLIT))
    self._dout = g

  def _grad_step_tail(self, c, k, pipe=None):
    pipe = self.pipeline if pipe is None else pipe
    g = self._dout
    if self._rides():               # the target head on the gathered batch rides in launches 3-6
      if not pipe:
        self._post_loss(self._pbuf[c])
      f = self._bwd_first()
      self._hip['online'].backward(g, groups=(self._SPLIT, 7),
                                   head=self._tail_head if pipe else None,
                                   riders=self._tail_riders if pipe else None, head_from=self._bwd_head_from())
      self._tail_head = self._tail_riders = None
    elif pipe:
      main = torch.cuda.current_stream(self._device)
      ev = torch.cuda.Event()
      ev.record(main)
      self._side.wait_event(ev)
      with torch.cuda.stream(self._side):
        self._post_loss(self._pbuf[c])
        self._prefetch(1 - c)
      self._hip['online'].backward(g, groups=(self._SPLIT, 7))
      main.wait_stream(self._side)
    else:
      self._post_loss(self._pbuf[c])
      self._hip['online'].backward(g, groups=(self._SPLIT, 7))

  def _grad_buckets(self):
    fp = self.online_convnet.fp
    o = fp.offsets['fc1_w'][0]
    return fp.grad[o:], fp.grad[:o]           # fc1 + fc2 (final after the head), convs

  # fc-bucket all-reduce pieces (N > 1).  4 pieces pipeline each piece's Adam part
  # behind its all-reduce, but with a one-rank RCCL group (bench --force-dist) they
  # cost 174 -> 212 us per step in launches; 1 until an 8-GPU measurement says otherwise.
  _FC_PIECES = 1

  def _fc_pieces(self, lo, hi):
    """[lo, hi) in _FC_PIECES ranges, every boundary a multiple of 4 floats."""
    n = self._FC_PIECES
    step = -(-(hi - lo) // (4 * n)) * 4
    return [(a, min(a + step, hi)) for a in range(lo, hi, step)]

  def _join_fc(self):
    """The main stream waits for a deferred fc all-reduce + update (_split_step)."""
    if self._fc_pending is not None:
      torch.cuda.current_stream(self._device).wait_event(self._fc_pending)
      self._fc_pending = None

  def _conv_group(self):
    """A second communicator over the same ranks: its all-reduce is not queued behind
    the fc bucket's on the first one's internal stream.  Created on first use, which
    every rank reaches at the same step."""
    if self._pg_conv is None:
      import torch.distributed as dist
      self._pg_conv = dist.new_group(ranks=dist.get_process_group_ranks(self._pg),
                                     backend=dist.get_backend(self._pg))
    return self._pg_conv

  def _sharded(self):
    """shard_optimizer in effect: N > 1 (or forced collectives) with TF1 Adam."""
    if self._peer is not None:      # each learner keeps its own slice's moments
      return True
    return (self.shard_optimizer and self._pg is not None and isinstance(self._opt, ops.TF1Adam)
            and (self._world() > 1 or parallel.FORCE_COLLECTIVES))

  def _world(self):
    import torch.distributed as dist
    return dist.get_world_size(self._pg)

  def _shard_bounds(self):
    """(lo, n): the sharded range [lo, n) of the flat buffer -- the fc bucket minus a head
    of fewer than 4N floats, so that it splits into N equal 16-byte-aligned slices; the
    head joins the conv bucket (all-reduced, replicated update)."""
    n = self.online_convnet.fp.grad.numel()
    o = n - self._grad_buckets()[0].numel()
    return o + (n - o) % (4 * self._world()), n

  # with the optimizer fused into the backward (single replica), also write the gradients
  # it consumes to the flat gradient buffer (``_store_grads``); bench.py turns it off.
  # Captured graphs bake the choice in, so it is fixed once the first graph exists.
  _keep_gradients = True

  @property
  def keep_gradients(self):
    return self._keep_gradients

  @keep_gradients.setter
  def keep_gradients(self, value):
    value = bool(value)
    if value != self._keep_gradients and self._graph_sets:
      raise RuntimeError('keep_gradients must be set before the first captured gradient step '
                         '(the HIP graphs already captured bake in the gradient stores)')
    self._keep_gradients = value
  # HIP stream priority of the N > 1 comm stream (-1 high: its collective and update are
  # dispatched ahead of the main queue's pending blocks; with the update's grid capped at 256
  # blocks, one-rank RCCL 6,044-6,047 -> 6,172-6,211 steps/s, profiles/r4_dist/one_rank_ab.log)
  comm_priority = -1
  # HIP stream priority of the prefetch stream (the pipelined non-rider schedule, e.g. IQN's
  # target network beside the online backward): 0 normal, -1 high
  side_priority = 0
  # N > 1: capture the fc bucket's branch before the backward tail instead of after it
  branch_first = False

  def _gather_opt_state(self):
    """ZeRO-1: every rank's Adam moments of the sharded range, slice r from rank r (a
    collective: every rank calls it, e.g. from bundle_and_checkpoint)."""
    if not self._sharded():
      return
    lo, n = self._shard_bounds()
    torch.cuda.synchronize(self._device)
    for t in (self._opt.m, self._opt.v):
      parallel.all_gather_(t[lo:n], self._pg)
    torch.cuda.synchronize(self._device)

  def _split_step(self, head_a, head_b, tail, opt, k=0):
    """head | tail on the main stream with the fc bucket's all-reduce on the comm
    stream beside the tail; with TF1 Adam the fc parameters' update follows their
    all-reduce on the comm stream (hidden under the conv bucket's all-reduce) and
    only the conv parameters' update (which advances the beta powers) is left
    after the join: same arithmetic, split in two launches (dq_adam_tf1_part).
    In the learner-only loop (_defer_fc, fused Rainbow head split in head_a | head_b)
    the join moves to the next step, between its conv and fc forward launches: the
    fc all-reduce then runs under this step's tail AND the next step's convs, and
    the conv bucket goes over a second communicator so it does not wait behind it.
    Every launch keeps its inputs: the next step's convs read no fc parameter, its
    fc launches wait for the update, and Adam's beta-power slots alternate (the fc
    part reads slot k while the conv part writes slot 1 - k)."""
    main = torch.cuda.current_stream(self._device)
    fc, conv = self._grad_buckets()
    split_opt = isinstance(self._opt, ops.TF1Adam)
    defer = self._defer_fc and split_opt and head_a is not None
    grad = self.online_convnet.fp.grad
    o = grad.numel() - fc.numel()
    if head_a is not None:
      head_a()
    self._join_fc()
    head_b()
    ev = torch.cuda.Event()
    ev.record(main)
    # the tail is issued (captured) before the comm branch, so in a captured graph it is the
    # first child of the head's last launch and stays on that launch's hardware queue -- the
    # all-reduce branch takes the other one (a fork to another queue costs ~10 us on the
    # critical path, measured with the branch captured first; branch_first re-measures it)
    if not self.branch_first:
      tail()
    last, conv, o = self._fc_branch(ev, grad, conv, o, k, split_opt)
    if self.branch_first:
      tail()
    if defer:
      self._ar_conv(conv, True)
      self._fc_pending = torch.cuda.Event()
      self._fc_pending.record(last)
    else:
      self._ar_conv(conv, False)
      main.wait_stream(last)
    if split_opt:
      self._opt.step_part(grad, 0, o, slot=k, bump=True)
    else:
      opt()

  def _fc_branch(self, ev, grad, conv, o, k, split_opt):
    """The fc bucket's exchange and update on the comm stream (forked at event ev, after
    the backward launch that leaves fc1 / fc2's gradients final).  Returns (the stream to
    join, the conv bucket, its end offset)."""
    self._comm.wait_event(ev)
    # The fc bucket as _FC_PIECES all-reduces back to back on the comm stream; each
    # piece's Adam part runs on a second stream behind its own all-reduce, under the
    # next piece's (an HBM-bound update beside a link-bound collective).  Elementwise
    # ops: bitwise the one-bucket result.  (Blocking collectives + events rather than
    # async work handles, which graph capture does not survive.)
    last = self._comm
    if self._sharded():
      # ZeRO-1: reduce-scatter the fc bucket, TF1 Adam on this rank's slice only (1/N of
      # the fc update's 112 MB), all-gather the updated parameters -- the same bytes over
      # the links as the all-reduce; the other slices' moments live on their owners
      lo, n = self._shard_bounds()
      S = (n - lo) // self._world()
      r = torch.distributed.get_rank(self._pg)
      # all three on the comm stream: they are dependent, so a second stream for the
      # update buys no overlap -- and that arrangement (comm -> second stream -> comm) made
      # the captured chunk graphs segfault in hipStreamEndCapture on ROCm 7.2 (DESIGN §6;
      # the repro is tools/capture_fork_repro.py, outside the product)
      with torch.cuda.stream(self._comm):
        if self._rccl is not None:
          self._rccl[0].reduce_scatter_mean_(grad[lo:n])
        else:
          parallel.reduce_scatter_mean_(grad[lo:n], self._pg)
        self._opt.step_part(grad, lo + r * S, lo + (r + 1) * S, slot=k, bump=False)
        if self._rccl is not None:
          self._rccl[0].all_gather_(self._opt.params[lo:n])
        else:
          parallel.all_gather_(self._opt.params[lo:n], self._pg)
      conv, o = grad[:lo], lo                 # the head of the fc bucket joins the conv bucket
    else:
      pieces = self._fc_pieces(o, grad.numel()) if split_opt else [(o, grad.numel())]
      # one piece: its update right behind it on the comm stream (measured equal to the
      # second stream at one rank, 6,040 / 6,007 vs 6,027 / 6,014 steps/s, and one queue
      # hop fewer in the captured graphs)
      one = len(pieces) == 1
      for lo, hi in pieces:
        with torch.cuda.stream(self._comm):
          self._ar_fc(grad[lo:hi])
          if split_opt and one:
            self._opt.step_part(grad, lo, hi, slot=k, bump=False)
        if split_opt and not one:
          e = torch.cuda.Event()
          e.record(self._comm)
          self._comm_opt.wait_event(e)
          with torch.cuda.stream(self._comm_opt):
            self._opt.step_part(grad, lo, hi, slot=k, bump=False)
          last = self._comm_opt
    return last, conv, o

  def _post_loss(self, t):
    """Work that needs the loss but not the gradient (PER priority write-back)."""

  def _device_opt_step(self, k):
    """Optimizer step k (k = gradient-step parity: TF1 Adam's beta-power slot)."""
    if self._fused_opt():
      return                          # applied inside the backward
    if self._needs_flat_grad():
      self._opt.step(self.online_convnet.fp.grad, slot=k)
    else:
      self._opt.step_multi([prm.grad for prm in self.online_convnet.parameters()], slot=k)

  def _allreduce_grads(self):
    if not self._collective():
      return
    parallel.allreduce_mean_(self.online_convnet.fp.grad, self._pg)

  def _discard_prefetch(self):
    if self._has_prefetch:
      # (after a chunk-gather chunk the rewind cursor is its last batch's: exactly the
      # prefetched one is given back)
      self._replay.memory.rewind_last_sample()
      self._has_prefetch = False
      self._cb_ready = None

  # ----------------------------------------------------- chunk gather (uniform)
  # In the learner-only loop a uniform replay's batches do not depend on priorities, so
  # the K batches of a chunk (steps 1..K-1 and the next chunk's step 0) are drawn by ONE
  # grouped sample and gathered by ONE K*B launch, riding in the chunk's first backward
  # (crb:436-558: the same draws, RNG words and batches as K per-step samples).  Two sets
  # of K batches alternate between consecutive chunks: a chunk's first step still reads
  # the previous set's last batch while its riders fill the other set.
  chunk_gather = True

  def _chunk_gathers(self):
    return (self.chunk_gather and self._fused() and not self._collective() and
            not self._replay.memory._prioritized)

  def _cb_sets(self):
    if self._cb is None:
      mem, K, B = self._replay.memory, self._UNROLL, self._batch_size
      self._cb = []
      for _ in range(2):
        d = mem._alloc_batch(K * B, self._replay._layout)
        d['sample_indices'] = torch.empty((K * B,), dtype=torch.int32, device=self._device)
        self._cb.append(d)
      self._cbv = [[{k: v[i * B:(i + 1) * B] for k, v in d.items()} for i in range(K)]
                   for d in self._cb]
    return self._cb

  def _prefetched(self):
    """The batch the next gradient step trains on (prefetched)."""
    if self._cb_ready is not None:
      return self._cbv[self._cb_ready][self._UNROLL - 1]
    return self._pbuf[self._slot]

  def _materialize_cb(self):
    """A chunk's prefetched batch into the per-call pipeline slot (the per-call graphs read
    _pbuf); its target head already ran into the slot's target executor."""
    src, dst = self._prefetched(), self._pbuf[self._slot]
    for k, v in dst.items():
      if k in src:
        v.copy_(src[k])
    self._cb_ready = None

  def _run_gather_chunk(self, K):
    """K gradient steps as one chunk-gather graph replay (captured per starting parity,
    three variants: entering from the per-call pipeline, and the two alternating sets)."""
    mem = self._replay.memory
    k0 = self._opt_steps % 2
    steady = self._cb_ready is not None
    p = 1 - self._cb_ready if steady else 0
    key = ('gchunk', K, k0, p, steady)
    if key not in self._graph_sets:
      torch.cuda.synchronize(self._device)
      self._cb_sets()
      saved = list(self._pbuf)
      try:
        for st, q in ((False, 0), (True, 0), (True, 1)):
          g = torch.cuda.CUDAGraph()
          with torch.cuda.graph(g, pool=self._graph_pool):
            for j in range(K):
              k = (k0 + j) % 2
              if j == 0:                # the prefetched batch
                self._pbuf[k] = self._cbv[1 - q][K - 1] if st else saved[k0]
              self._gather_plan = (q, j)
              self._grad_step(k, k, True)
              self._device_opt_step(k)
              self._trace_step(j, k)
            self._gather_plan = None
          self._graph_pool = g.pool()
          self._graph_sets[('gchunk', K, k0, q, st)] = g
      finally:
        self._gather_plan = None
        self._pbuf[:] = saved
    mem.reserve_rng(self._batch_size, steps=K)
    self._graph_sets[key].replay()
    self._opt_steps += K
    last = self._cbv[p][K - 2]          # the batch the chunk's last step trained on
    self._replay._out = last
    self._replay.unpack_transition(last)
    self._slot = (k0 + K) % 2
    self._cb_ready = p
    self._has_prefetch = True
    self._prefetch_add_count = int(mem.add_count)
    self._last_train_add_count = int(mem.add_count)
    self._selects_since_train = 0

  # The prefetch of step t+1 (drawn right after step t's priority write-back) is
  # only usable if nothing touches the replay RNG stream or the buffer before
  # step t+1 -- true for a learner-only loop (the benchmark), never for an agent
  # acting in an environment, where add() and (with PER) epsilon-greedy draws
  # come between steps.  Such steps use a second, non-pipelined graph family
  # instead of prefetching work that would be thrown away.
  def _interleaved(self):
    mem = self._replay.memory
    if int(mem.add_count) != self._last_train_add_count:
      return True
    return self._selects_since_train > 0 and mem._rng.stream is random

  def _run_train_op(self):
    """One gradient step (the body of sess.run(self._train_op))."""
    mem = self._replay.memory
    k = self._opt_steps % 2
    c = k                                 # pipeline slot == step parity (graphs bake it in)
    pipe = self.pipeline and not self._interleaved()
    if self._has_prefetch and (not pipe or self._prefetch_add_count != int(mem.add_count)):
      self._discard_prefetch()            # transitions were added after the prefetch
    if self._cb_ready is not None:        # a chunk's prefetch, for the per-call graphs
      self._materialize_cb()
    if pipe and not self._has_prefetch:
      mem.reserve_rng(self._batch_size)
      self._prefetch(c)
    mem.reserve_rng(self._batch_size)
    graphs = self._graph_sets.get(pipe)
    if self._split_allreduce():
      if graphs is not None:
        self._split_step(*[None if g is None else g.replay for g in graphs[0][k]], k=k)
      elif self._head_splits():
        self._split_step(lambda: self._grad_step_head(c, k, pipe, 'a'),
                         lambda: self._grad_step_head(c, k, pipe, 'b'),
                         lambda: self._grad_step_tail(c, k, pipe),
                         lambda: self._device_opt_step(k), k=k)
        self._eager_steps[pipe] += 1
      else:
        self._split_step(None, lambda: self._grad_step_head(c, k, pipe),
                         lambda: self._grad_step_tail(c, k, pipe),
                         lambda: self._device_opt_step(k), k=k)
        self._eager_steps[pipe] += 1
    elif graphs is not None:
      graphs[0][k].replay()
      if self._collective():
        self._allreduce_grads()
        graphs[1][k].replay()
    else:
      self._grad_step(c, k, pipe)
      self._allreduce_grads()
      self._device_opt_step(k)
      self._trace_step(self._UNROLL + k, c)
      self._eager_steps[pipe] += 1
    self._opt_steps += 1
    self._replay._out = self._pbuf[c]
    self._replay.unpack_transition(self._pbuf[c])
    self._slot = 1 - c
    self._has_prefetch = pipe
    self._prefetch_add_count = int(mem.add_count)
    self._last_train_add_count = int(mem.add_count)
    self._selects_since_train = 0
    if graphs is None and self.use_hip_graph and self._eager_steps[pipe] >= 3:
      self._capture(pipe)

  @property
  def _graphs(self):
    g = self._graph_sets.get(self.pipeline)
    return None if g is None else g[0]

  def _capture(self, pipe=None):
    """Two graphs, one per gradient-step parity k (pipeline slot and Adam
    beta-power slot both alternate with k); with one GPU the optimizer is in the
    same graph, with N GPUs it is a second graph after the RCCL all-reduce."""
    pipe = self.pipeline if pipe is None else pipe
    torch.cuda.synchronize(self._device)
    graphs, graphs_opt, pool = [], [], self._graph_pool
    if self._split_allreduce():
      for k in (0, 1):
        c = k
        if self._head_splits():
          fns = (lambda: self._grad_step_head(c, k, pipe, 'a'),
                 lambda: self._grad_step_head(c, k, pipe, 'b'))
        else:
          fns = (None, lambda: self._grad_step_head(c, k, pipe))
        fns += (lambda: self._grad_step_tail(c, k, pipe), lambda: self._device_opt_step(k))
        parts = []
        for fn in fns:
          gr = None
          if fn is not None:
            gr = torch.cuda.CUDAGraph()
            # thread_local: torch's process-group watchdog thread polls the events of the
            # collectives issued just before (global mode would fail its queries)
            with torch.cuda.graph(gr, pool=pool, capture_error_mode='thread_local'):
              fn()
            pool = gr.pool()
          parts.append(gr)
        graphs.append(parts)
      self._graph_pool = pool
      self._graph_sets[pipe] = (graphs, [])
      return
    for k in (0, 1):
      c = k
      g = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g, pool=pool, capture_error_mode='thread_local'):
        self._grad_step(c, k, pipe)
        if not self._collective():
          self._device_opt_step(k)
          self._trace_step(self._UNROLL + k, c)
      pool = g.pool()
      graphs.append(g)
      if self._collective():
        go = torch.cuda.CUDAGraph()
        with torch.cuda.graph(go, pool=pool, capture_error_mode='thread_local'):
          self._device_opt_step(k)
        graphs_opt.append(go)
    # capture records without executing: tape cursor and buffers are unchanged
    self._graph_pool = pool
    self._graph_sets[pipe] = (graphs, graphs_opt)

  def _sync_target(self):
    self._join_fc()
    ops.sync_copy(self.target_convnet.fp.flat, self.online_convnet.fp.flat)
    if self.pipeline and self._has_prefetch and self._rides():   # the prefetched head is stale
      self._hip['target'][self._slot].forward_head(self._prefetched()['next_state'])
    elif self.pipeline and self._has_prefetch and not self._pairs():   # prefetched target outputs are stale
      tg = self._target_forward(self._pbuf[self._slot], self._slot)
      for k, v in tg.items():
        if v.data_ptr() != self._ptgt[self._slot][k].data_ptr():
          self._ptgt[self._slot][k].copy_(v)

  # ------------------------------------------------------------- agent API
  def begin_episode(self, observation):
    self._reset_state()
    self._record_observation(observation)
    if not self.eval_mode:
      self._train_step()
    self.action = self._select_action()
    return self.action

  def step(self, reward, observation):
    self._last_observation = self._observation
    self._record_observation(observation)
    if not self.eval_mode:
      self._store_transition(self._last_observation, self.action, reward, False)
      self._train_step()
    self.action = self._select_action()
    return self.action

  def end_episode(self, reward):
    if not self.eval_mode:
      self._store_transition(self._observation, self.action, reward, True)

  def _q_values(self, state_np):
    if self._hip is not None and self.use_hip_graph:
      return self._act_q(state_np)
    # (1, *observation_shape, stack) -> (1, stack, *observation_shape): the layout the
    # replay's gather hands the network in training (float32 / 255 for uint8 frames,
    # the observation dtype otherwise; the network casts, as the reference's do)
    s = np.moveaxis(np.asarray(state_np), -1, 1)
    if np.dtype(self.observation_dtype) == np.uint8:
      x = torch.as_tensor(s, dtype=torch.float32, device=self._device) / 255.0
    else:
      x = torch.as_tensor(s.astype(self.observation_dtype), device=self._device)
    with torch.no_grad():
      return self._online_q(self._state_input(x.contiguous()))

  def _q_from_output(self, out):
    """Network output -> Q-values (B, A)."""
    return out

  def _online_q(self, x):
    return self._q_from_output(self.online_convnet(x))

  def _act_q(self, state_np):
    """Q-values for action selection on the HIP CNN at batch 1: the forward and
    the Q reduction are one captured graph; the state goes up through a pinned
    staging buffer.  The executor reads the online parameters in place."""
    if self._act is None:
      from dopamine_amd.cnn import HipNatureCNN
      exe = HipNatureCNN(self.online_convnet, 1)
      x = torch.zeros((1, 84, 84, self.stack_size), dtype=torch.float32, device=self._device)
      pin = torch.empty(x.shape, dtype=torch.float32).pin_memory()
      main = torch.cuda.current_stream(self._device)
      warm = torch.cuda.Stream(self._device)
      warm.wait_stream(main)
      with torch.cuda.stream(warm):
        self._q_from_output(exe.forward(x))
      main.wait_stream(warm)
      g = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g):
        q = self._q_from_output(exe.forward(x))
      self._act = (exe, x, pin, g, q)
    exe, x, pin, g, q = self._act
    scale = 1.0 / 255.0 if np.dtype(self.observation_dtype) == np.uint8 else 1.0
    np.multiply(state_np, scale, out=pin.numpy(), casting='unsafe')
    x.copy_(pin, non_blocking=True)
    g.replay()
    return q

  # Words reserved on the replay's RNG tape per device action: random.random() takes 2,
  # randint's getrandbits rejection at most 2 per try (P(reject) < 1/2); 64 more cover it
  # but for a (2^-64-rare) run, which falls back to the host draw.
  _EGREEDY_WORDS = 66
  device_egreedy = True

  def _select_action(self):
    """dqn_agent.py:394-416.  With a prioritized replay, whose sampler draws from Python's
    `random` as epsilon-greedy does, the draws come from the replay's RNG tape on the
    device (dq_replay_egreedy): the stream is consumed exactly as by the reference with no
    host synchronisation per action.  Otherwise (or if the tape runs out) the tape is
    brought in step and the host draws."""
    mem = self._replay.memory
    if self.eval_mode:
      epsilon = self.epsilon_eval
    else:
      epsilon = self.epsilon_fn(self.epsilon_decay_period, self.training_steps,
                                self.min_replay_history, self.epsilon_train)
    if mem._rng.stream is random:   # PER samples from Python's `random`, as epsilon-greedy does
      self._selects_since_train += 1
      self._discard_prefetch()      # its draws would precede ours: give them back first
      if self.device_egreedy:
        a = self._select_action_device(mem, epsilon)
        if a >= 0:
          return a
      mem.sync_rng()
    if random.random() <= epsilon:
      return random.randint(0, self.num_actions - 1)
    return int(torch.argmax(self._q_values(self.state), dim=1)[0].item())

  def _select_action_device(self, mem, epsilon):
    """The epsilon test, the explore draw and the greedy argmax as one kernel on the
    tape (dq_replay_egreedy) after the Q-values; -1 if the tape ran out."""
    mem._rng.reserve(self._EGREEDY_WORDS, mem._stream)
    q = self._q_values(self.state).reshape(-1)
    if q.dtype != torch.float32 or not q.is_contiguous():
      q = q.float().contiguous()
    if getattr(self, '_act_out', None) is None:
      self._act_out = torch.empty(1, dtype=torch.int32, device=self._device)
    _lib.call('dq_replay_egreedy', mem._h, _lib.ptr(q), self.num_actions, float(epsilon),
              _lib.ptr(self._act_out), mem._stream)
    return int(self._act_out.item())

  # ------------------------------------------------------ learner-only loop
  _UNROLL = 4

  def train_gradient_steps(self, n):
    """What ``n * update_period`` consecutive ``_train_step()`` calls do when nothing is
    added or acted between them -- a learner-only loop over a fixed buffer (the
    benchmark; Dopamine's fixed-replay / offline training phases).  Where the
    pipelined single-replica HIP-graph path applies, _UNROLL consecutive gradient
    steps are ONE graph replay (the graph-to-graph gap, ~5 us on MI355X, is paid
    once per chunk); the steps, their order, RNG use and target syncs are exactly
    those of the per-call loop (tests/test_gpu_agent.py)."""
    n = int(n)
    if self._closed:
      raise RuntimeError('the agent was closed (its communicators are destroyed)')
    self._peer_ready()
    self._defer_fc = True
    try:
      self._train_gradient_steps(n)
    finally:
      self._defer_fc = False
      self._join_fc()
      self._peer_flush()
    self._maybe_check_replicas()

  def _train_gradient_steps(self, n):
    while n > 0:
      K = self._UNROLL
      if n >= K and self._chunk_ok():
        self._run_train_ops_chunk(K)
        t0 = self.training_steps
        self.training_steps += K * self.update_period
        # a sync falling on the chunk's last gradient step or after it (see _chunk_ok)
        for t in range(t0, self.training_steps):
          if t % self.target_update_period == 0:
            self._peer_flush()
            self._sync_target()
        n -= K
        continue
      self._peer_flush()
      for _ in range(self.update_period):
        self._train_step()
      n -= 1

  def graphs_primed(self):
    """True once every HIP graph the learner loop replays is captured: the per-step
    graphs and, where chunking applies, the chunk graphs of both starting parities."""
    if not self.use_hip_graph:
      return True
    if self._graph_sets.get(True) is None:
      return False
    if not self._chunks_apply():
      return True
    if self._chunk_gathers():
      return all(('gchunk', self._UNROLL, k, 0, False) in self._graph_sets for k in (0, 1))
    if self._peer is not None and self._peer.world > 1 and self._fused():
      # the chunk graphs with and without the predecessor's deferred gather (a learner-loop
      # call of two chunks or more captures the latter)
      return all(('chunk', self._UNROLL, k, p) in self._graph_sets for k in (0, 1)
                 for p in (False, True))
    return all(('chunk', self._UNROLL, k) in self._graph_sets for k in (0, 1))

  def _captures_collectives(self):
    """N > 1 over the learner's own RCCL communicators with the split fused-head schedule:
    the gradient all-reduces are captured inside the learner loop's chunk graphs (gloo's
    host-side collectives cannot be, torch.distributed's are not)."""
    if not self._collective():
      return False
    import torch.distributed as dist
    # (torch.distributed's own collectives are never captured: parallel.collectives_capturable)
    return (dist.get_backend(self._pg) == 'nccl' and self._rccl is not None and
            self._split_allreduce() and self._head_splits() and
            isinstance(self._opt, ops.TF1Adam) and
            parallel.collectives_capturable(self._pg, self._device, self._comm,
                                            sharded=self._sharded(), comms=self._rccl))

  def _chunks_apply(self):
    return (self._hip is not None and self.pipeline and
            (not self._collective() or self._captures_collectives()))

  def _chunk_ok(self):
    K, U = self._UNROLL, self.update_period
    t0 = self.training_steps
    if not (self.pipeline and self.use_hip_graph and self._chunks_apply()
            and self.summary_writer is None
            and self._has_prefetch and not self._interleaved()
            and self._graph_sets.get(True) is not None and t0 % U == 0
            and self._replay.memory.add_count > self.min_replay_history):
      return False
    if self._prefetch_add_count != int(self._replay.memory.add_count):
      return False
    # a target sync must not fall between two of the chunk's gradient steps
    last = t0 + U * (K - 1)
    return not any(t % self.target_update_period == 0 for t in range(t0, last))

  def _run_train_ops_chunk(self, K):
    """K pipelined gradient steps as one replay of a K-step graph (captured per
    starting parity on first use)."""
    if self._chunk_gathers():
      return self._run_gather_chunk(K)
    mem = self._replay.memory
    k0 = self._opt_steps % 2
    defer = (not self._collective() and self._peer is not None and self._peer.world > 1 and
             self._fused())
    pending = defer and self._peer_pending
    key = ('chunk', K, k0) + ((pending,) if defer else ())
    g = self._graph_sets.get(key)
    if g is None:
      self._join_fc()                 # nothing outside the capture may be pending
      torch.cuda.synchronize(self._device)
      g = torch.cuda.CUDAGraph()
      if not self._collective():
        try:
          with torch.cuda.graph(g, pool=self._graph_pool):
            for j in range(K):
              k = (k0 + j) % 2
              self._peer_fwd_ag, self._peer_defer_ag = defer and (j > 0 or pending), defer
              self._grad_step(k, k, True)
              self._device_opt_step(k)
              self._trace_step(j, k)
        finally:
          self._peer_fwd_ag = self._peer_defer_ag = False
      else:
        # N > 1: each step's split schedule with its RCCL all-reduces captured (the comm
        # stream and RCCL's own streams fork from and join back into the capture; each
        # step's fc all-reduce + update is joined in the next step, the last one at the
        # end of the chunk).  thread_local: the process group's watchdog thread keeps
        # querying its events while this thread captures.
        with torch.cuda.graph(g, pool=self._graph_pool, capture_error_mode='thread_local'):
          for j in range(K):
            k = (k0 + j) % 2
            self._split_step(lambda k=k: self._grad_step_head(k, k, True, 'a'),
                             lambda k=k: self._grad_step_head(k, k, True, 'b'),
                             lambda k=k: self._grad_step_tail(k, k, True),
                             lambda k=k: self._device_opt_step(k), k=k)
          self._join_fc()
      self._graph_pool = g.pool()
      self._graph_sets[key] = g
    else:
      self._join_fc()
    mem.reserve_rng(self._batch_size, steps=K)
    g.replay()
    self._peer_pending = defer        # the last step's gather is left to the next chunk / flush
    self._opt_steps += K
    c = (k0 + K - 1) % 2
    self._replay._out = self._pbuf[c]
    self._replay.unpack_transition(self._pbuf[c])
    self._slot = 1 - c
    self._has_prefetch = True
    self._prefetch_add_count = int(mem.add_count)
    self._last_train_add_count = int(mem.add_count)
    self._selects_since_train = 0

  def _train_step(self):
    """dqn_agent.py:418-442."""
    if self._closed:
      raise RuntimeError('the agent was closed (its communicators are destroyed)')
    if self._replay.memory.add_count > self.min_replay_history:
      if self.training_steps % self.update_period == 0:
        self._peer_ready()
        self._run_train_op()
        if (self.summary_writer is not None and self.training_steps > 0 and
            self.training_steps % self.summary_writing_frequency == 0):
          self.summary_writer.add_summary({self._loss_name: self.mean_loss()}, self.training_steps)
      if self.training_steps % self.target_update_period == 0:
        self._sync_target()
    self.training_steps += 1

  _loss_name = 'HuberLoss'

  def check_exchange(self, collective=False):
    """Raises if the peer exchange's error word is latched (a wait timed out: another learner
    stopped or fell out of step; or another rank's error; or a publication that missed an
    XCD); a synchronising read.  collective: the ranks first agree on the worst error word,
    so every rank raises together (call it at the same point on every rank).  No-op without
    the peer exchange."""
    if self._peer is not None:
      self._peer.check(collective=collective)

  def replica_report(self):
    """Collective (every rank of the group calls it at the same point): every replicated
    tensor -- online and target parameters, the optimizer's moments (the sharded ranges'
    slices gathered first, _gather_opt_state) and its state -- compared bit for bit with
    group rank 0's (parallel.replica_report).  SURVEY 8e: identical updates keep the replicas
    bit-identical; this is the check that they did."""
    assert self._pg is not None, 'replica_report needs a process group'
    self._join_fc()
    torch.cuda.synchronize(self._device)
    self._gather_opt_state()
    named = {'online': self.online_convnet.fp.flat, 'target': self.target_convnet.fp.flat}
    for k, v in sorted(vars(self._opt).items()):
      if isinstance(v, torch.Tensor) and v.data_ptr() != self.online_convnet.fp.flat.data_ptr():
        named['opt_' + k.lstrip('_')] = v
    return parallel.replica_report(named, self._pg)

  # data-parallel learner loop: every replica_check_period gradient steps (crossed inside a
  # train_gradient_steps call, which every rank makes with the same n), the replicas are
  # compared bit for bit and a divergence raises on every rank (0: never)
  replica_check_period = 100_000
  _next_replica_check = None

  def _maybe_check_replicas(self):
    if self._pg is None or not self.replica_check_period:
      return
    if self._next_replica_check is None:
      self._next_replica_check = self._opt_steps + self.replica_check_period
    if self._opt_steps < self._next_replica_check:
      return
    self._next_replica_check = self._opt_steps + self.replica_check_period
    self.check_exchange(collective=True)
    rep = self.replica_report()
    bad = {k: v['differing'] for k, v in rep.items() if not v['in_sync']}
    if bad:
      raise RuntimeError('data-parallel replicas diverged after %d gradient steps: elements '
                         'differing from rank 0, per rank: %r' % (self._opt_steps, bad))

  def mean_loss(self):
    """Mean loss of the last gradient step (the summary scalar, dqn:318-321); the fused
    head's loss kernel leaves the mean to this call (it is not on the gradient path).
    With the peer exchange it also raises if a wait of it timed out (check_exchange)."""
    self.check_exchange()
    if self._fused():
      return float(self._loss_out['loss'].double().mean().item())
    return float(self._loss_out['mean_loss'].item())

  def _record_observation(self, observation):
    self._observation = np.reshape(observation, self.observation_shape)
    self.state = np.roll(self.state, -1, axis=-1)
    self.state[0, ..., -1] = self._observation

  def _store_transition(self, last_observation, action, reward, is_terminal):
    self._replay.add(last_observation, action, reward, is_terminal)

  def _reset_state(self):
    self.state.fill(0)

  # ---------------------------------------------------------- checkpoints
  def _ckpt_tensors(self):
    d = {'online': self.online_convnet.fp.flat, 'target': self.target_convnet.fp.flat}
    for k, v in vars(self._opt).items():
      if isinstance(v, torch.Tensor) and v.data_ptr() != self.online_convnet.fp.flat.data_ptr():
        d['opt_' + k] = v
    return d

  def _rank_dir(self, checkpoint_dir):
    """Where this learner's files go.  A single replica: ``checkpoint_dir`` itself, as the
    reference (dqn_agent.py:482-551; crb:593-687).  Data-parallel learners (a process
    group): ``checkpoint_dir/rank<r>`` per group rank -- each rank owns a different buffer
    and sum tree, and the reference's file names (``$store$_*_ckpt.N.gz``, ``tf_ckpt-N``)
    would otherwise collide in a shared run directory."""
    if self._pg is None:
      return checkpoint_dir
    import torch.distributed as dist
    return os.path.join(checkpoint_dir, 'rank%d' % dist.get_rank(self._pg))

  def bundle_and_checkpoint(self, checkpoint_dir, iteration_number):
    """dqn_agent.py:482-510 (torch tensors instead of a tf.train.Saver).  With a process
    group every rank calls it (ZeRO-1 gathers the moments first) and writes under
    ``checkpoint_dir/rank<r>`` (_rank_dir)."""
    self._join_fc()
    # ZeRO-1: complete moments on every rank -- a collective, so every rank reaches it
    # before any rank-local early return
    self._gather_opt_state()
    if not os.path.isdir(checkpoint_dir):
      return None
    checkpoint_dir = self._rank_dir(checkpoint_dir)
    os.makedirs(checkpoint_dir, exist_ok=True)
    torch.save({k: v.detach().cpu() for k, v in self._ckpt_tensors().items()},
               os.path.join(checkpoint_dir, 'tf_ckpt-{}'.format(iteration_number)))
    stale = iteration_number - self.max_tf_checkpoints_to_keep
    if stale >= 0:
      try:
        os.remove(os.path.join(checkpoint_dir, 'tf_ckpt-{}'.format(stale)))
      except OSError:
        pass
    self._replay.save(checkpoint_dir, iteration_number)
    # _opt_steps: TF1 Adam's beta powers are double-buffered by step parity
    return {'state': self.state, 'training_steps': self.training_steps,
            '_opt_steps': self._opt_steps}

  def unbundle(self, checkpoint_dir, iteration_number, bundle_dictionary):
    """dqn_agent.py:512-551 (with a process group: from ``checkpoint_dir/rank<r>``)."""
    checkpoint_dir = self._rank_dir(checkpoint_dir)
    self._discard_prefetch()          # the buffer (and its RNG use) is replaced below
    self._replay.memory.sync_rng(raise_errors=False)
    try:
      self._replay.load(checkpoint_dir, iteration_number)
    except (FileNotFoundError, NotImplementedError):
      if not self.allow_partial_reload:
        return False
    if bundle_dictionary is not None:
      for key in self.__dict__:
        if key in bundle_dictionary:
          self.__dict__[key] = bundle_dictionary[key]
    elif not self.allow_partial_reload:
      return False
    path = os.path.join(checkpoint_dir, 'tf_ckpt-{}'.format(iteration_number))
    saved = torch.load(path, weights_only=True)
    for k, v in self._ckpt_tensors().items():
      s = saved[k]
      if s.shape == v.shape:
        v.copy_(s.to(v.device))
      elif (s.dim() == 1 and v.numel() == self.online_convnet.fp.numel and
            s.numel() == self.online_convnet.fp.content_numel):
        # a flat buffer saved before the Nature-CNN layouts ended in the fc bucket's zero
        # padding (networks.FC_BUCKET_ALIGN): every tensor sits in the prefix, the padding
        # stays zero (its gradient is zero, so no optimizer ever moves it)
        v.zero_()
        v[:s.numel()].copy_(s.to(v.device))
      else:
        raise ValueError('tf_ckpt-{}: {} has shape {}, this agent expects {} (a checkpoint of '
                         'another network or layout)'.format(iteration_number, k,
                                                             tuple(s.shape), tuple(v.shape)))
    return True
