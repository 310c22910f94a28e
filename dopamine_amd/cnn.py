"""HIP Nature-CNN executor over a network's flat parameter buffer.

Forward and backward of the DQN / Rainbow Nature-CNN (atari_lib.py:85-144) run
as 6 + 14 fused implicit-GEMM / reduce launches on the fp32 matrix cores
(dopamine_amd/csrc/nature_cnn.hip) instead of ~20 + 30 PyTorch/MIOpen kernels.
The backward writes every weight/bias gradient straight into the flat gradient
buffer (plain stores), which the TF1 optimizer kernel then consumes.
"""
import ctypes

import torch

from dopamine_amd import _lib


CnnParams, CnnActs = _lib.CnnParams, _lib.CnnActs

_NAMES = ('conv1_w', 'conv1_b', 'conv2_w', 'conv2_b', 'conv3_w', 'conv3_b', 'fc1_w', 'fc1_b',
          'fc2_w', 'fc2_b')


def _params_struct(fp, buf, n_out, in_ch):
  s = CnnParams(in_channels=in_ch, n_out=n_out)
  base = buf.data_ptr()
  for n in _NAMES:
    o, _ = fp.offsets[n]
    setattr(s, n, base + 4 * o)
  return s


class HipNatureCNN(object):
  """Executes a ``NatureDQNNetwork`` / ``RainbowNetwork``'s parameters with the
  HIP kernels.  ``forward`` keeps its activations for ``backward``; use one
  executor per concurrent stream (online vs target)."""

  def __init__(self, net, batch_size):
    fp = net.fp
    self.net = net
    self.B = int(batch_size)
    shape = fp.offsets['fc2_w'][1]
    self.n_out = int(shape[0])
    self.in_ch = int(fp.offsets['conv1_w'][1][1])
    assert self.in_ch == 4 and fp.offsets['fc1_w'][1] == (512, 7744), 'Nature-CNN geometry only'
    dev = fp.flat.device
    B = self.B
    mk = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)
    self.acts = dict(a1=mk(B, 21, 21, 32), a2=mk(B, 11, 11, 64), a3=mk(B, 7744), h=mk(B, 512),
                     out=mk(B, self.n_out))
    self.dacts = dict(a1=mk(B, 21, 21, 32), a2=mk(B, 11, 11, 64), a3=mk(B, 7744), h=mk(B, 512),
                      out=mk(1))
    nws = int(_lib.lib.dq_cnn_workspace_floats(B, self.n_out)) + 64
    self.ws = mk(nws)
    self.ws_dw = mk(nws)       # split-K slabs of the weight gradients on the second stream
    self._dw_stream = None
    self._events = None
    self._p = _params_struct(fp, fp.flat, self.n_out, self.in_ch)
    self._g = _params_struct(fp, fp.grad, self.n_out, self.in_ch)
    self._a = CnnActs(**{k: v.data_ptr() for k, v in self.acts.items()})
    self._d = CnnActs(**{k: v.data_ptr() for k, v in self.dacts.items()})
    self._x = None

  @staticmethod
  def _stream(t):
    return _lib.stream_of(t.device)

  def _nhwc(self, x):
    if x.dim() == 4 and x.shape[1] == self.in_ch and x.shape[-1] != self.in_ch:
      x = x.permute(0, 2, 3, 1)              # channels_last NCHW view -> NHWC
    assert x.shape == (self.B, 84, 84, 4) and x.is_contiguous() and x.dtype == torch.float32
    return x

  def forward(self, x):
    """x: (B, 84, 84, 4) NHWC float32, or its (B, 4, 84, 84) channels_last view.
    Returns the (B, n_out) output buffer (overwritten by the next call)."""
    x = self._nhwc(x)
    self._x = x
    _lib.check(_lib.lib.dq_cnn_forward(ctypes.byref(self._p), self.B, x.data_ptr(),
                                       ctypes.byref(self._a), self.ws.data_ptr(), self._stream(x)),
               'dq_cnn_forward')
    return self.acts['out']

  def forward_head(self, x):
    """The head of forward(x): conv1..conv3 and fc1's split-K partial sums (into
    self.ws); ``forward_with_tail`` finishes it.  Bitwise the same as forward()."""
    x = self._nhwc(x)
    self._x = x
    _lib.check(_lib.lib.dq_cnn_forward_head(ctypes.byref(self._p), self.B, x.data_ptr(),
                                            ctypes.byref(self._a), self.ws.data_ptr(),
                                            self._stream(x)), 'dq_cnn_forward_head')

  def cnn_net(self, x):
    """dq_cnn_net of this network on input x (for a head run elsewhere)."""
    x = self._nhwc(x)
    self._x = x
    return _lib.CnnNet(p=ctypes.cast(ctypes.pointer(self._p), ctypes.c_void_p), x=x.data_ptr(),
                       a=ctypes.cast(ctypes.pointer(self._a), ctypes.c_void_p), ws=self.ws.data_ptr())

  # with the optimizer fused into a gradient epilogue, also write that gradient to
  # net.fp.grad (False: it is consumed in registers -- dq_adam_args.no_grad_store)
  store_grads = True

  def _adam_args(self, adam, slot):
    """dq_adam_args of an ops.TF1Adam or ops.TF1RMSProp over net.fp.flat."""
    assert adam.params.data_ptr() == self.net.fp.flat.data_ptr(), 'adam must own net.fp.flat'
    ngs = 0 if self.store_grads else 1
    if hasattr(adam, 'ms'):          # TF1RMSProp: ms / mom / mg slots (kind DQ_OPT_RMSPROP)
      return _lib.AdamArgs(var=adam.params.data_ptr(), m=adam.ms.data_ptr(), v=adam.mom.data_ptr(),
                           lr=adam.lr, epsilon=adam.eps, kind=_lib.OPT_RMSPROP,
                           centered=int(adam.centered), mg=adam.mg.data_ptr(), decay=adam.decay,
                           momentum=adam.mu, no_grad_store=ngs)
    return _lib.AdamArgs(var=adam.params.data_ptr(), m=adam.m.data_ptr(), v=adam.v.data_ptr(),
                         state=adam.state.data_ptr(), slot=int(slot), lr=adam.lr,
                         beta1=adam.b1, beta2=adam.b2, epsilon=adam.eps, no_grad_store=ngs)

  def backward_peer(self, dout, adam, slot, peer, riders=None, head=None, defer_ag=False):
    """The fused Rainbow schedule's backward (head_from 6, from launch 1) with the data-
    parallel exchange over peer memory (dq_cnn_backward_peer; ``peer``: a _lib.Peer) in
    place of the fused optimizer's updates: the gradients are stored, this rank's slice of
    the fc bucket is reduce-scattered and updated inside launches 3-4, published with the
    others' slices gathered in launch 5 (defer_ag: gathered by the next step's
    ``forward_fused*(..., peer=)`` or ``PeerExchange.all_gather`` instead), the conv bucket
    in launch 6.  Rider i rides in launch 1 + i."""
    dout = dout.reshape(self.B, self.n_out)
    assert dout.is_contiguous() and self._x is not None
    args = self._adam_args(adam, slot)
    args.no_grad_store = 0
    riders = riders or []
    arr = (_lib.Rider * max(1, len(riders)))(*riders)
    hn = None
    if head is not None:
      assert head[0] is not self
      hn = ctypes.byref(head[0].cnn_net(head[1]))
    _lib.check(_lib.lib.dq_cnn_backward_peer(
        ctypes.byref(self._p), ctypes.byref(self._g), self.B, self._x.data_ptr(),
        ctypes.byref(self._a), dout.data_ptr(), ctypes.byref(self._d), self.ws.data_ptr(),
        arr, len(riders), ctypes.byref(args), hn, ctypes.byref(peer), int(bool(defer_ag)),
        self._stream(dout)),
        'dq_cnn_backward_peer')
    return self.net.fp.grad

  def backward(self, dout, parallel=False, adam=None, slot=0, groups=None, riders=None, head=None,
               head_from=3):
    """dout: (B, n_out).  Writes all parameter gradients into net.fp.grad.

    riders: replay operations recorded with ``ReplayBuffer.recording()`` (the
    next batch's priority write-back, sample and gather); rider i runs as extra
    blocks of grouped launch i (dq_cnn_backward_riders), in order, on this
    stream.  Combines with ``adam``.  head: (net, x) -- that network's forward head
    on x runs in launches 4..7 (with riders; e.g. the target net on the batch the
    riders gather); its forward_with_tail then finishes it.

    groups=(first, last): only launches [first, last) of the 7 grouped launches
    (a data-parallel learner all-reduces fc1/fc2's gradients after launch 3);
    rider i rides in launch first + i.  first = 1 skips fc2's input gradient
    (dacts['h'] already written, by ``c51_loss_fused``).  head_from = 4: the
    head's conv1..conv3 ride in launches 4..6 and its fc1 slabs are left to
    ``forward_fused`` (the Rainbow fast path).  head_from = 5: a five-launch
    backward (from launch 1), the head's conv1/conv2 in launches 4/5 and its conv3
    left to ``forward_fused(..., conv3_b=True)``.

    adam: an ops.TF1Adam over net.fp.flat -- its step (beta-power slot ``slot``)
    is applied inside the gradient epilogues (dq_cnn_backward_adam), so no
    separate optimizer launch is needed.  Single replica only: N > 1 GPUs must
    all-reduce the gradient before the optimizer.

    parallel: the weight gradients run on a second stream, each forked after
    the input gradient it needs and joined before returning (stream-ordered,
    HIP-graph capturable).  Measured SLOWER on MI355X inside a graph (141.6 vs
    95.9 us per backward, tools/bench_hipcnn.py): the cross-queue edges cost
    more than the overlap buys, and the 135-147 KB-LDS blocks cannot share a CU
    with the other stream's.  Kept for experimentation; off by default."""
    dout = dout.reshape(self.B, self.n_out)
    assert dout.is_contiguous() and self._x is not None
    if riders or head is not None or (groups is not None and adam is not None):
      args = None if adam is None else ctypes.byref(self._adam_args(adam, slot))
      riders = riders or []
      arr = (_lib.Rider * max(1, len(riders)))(*riders)
      hn = None
      if head is not None:
        assert head[0] is not self
        hn = ctypes.byref(head[0].cnn_net(head[1]))
      first, last = (0, 7) if groups is None else groups
      _lib.check(_lib.lib.dq_cnn_backward_riders(
          ctypes.byref(self._p), ctypes.byref(self._g), self.B, self._x.data_ptr(),
          ctypes.byref(self._a), dout.data_ptr(), ctypes.byref(self._d), self.ws.data_ptr(),
          arr, len(riders), args, hn, int(head_from), int(first), int(last), self._stream(dout)),
          'dq_cnn_backward_riders')
      return self.net.fp.grad
    if groups is not None:          # a sub-range of the 7 grouped launches
      _lib.check(_lib.lib.dq_cnn_backward_groups(
          ctypes.byref(self._p), ctypes.byref(self._g), self.B, self._x.data_ptr(),
          ctypes.byref(self._a), dout.data_ptr(), ctypes.byref(self._d), self.ws.data_ptr(),
          int(groups[0]), int(groups[1]), self._stream(dout)), 'dq_cnn_backward_groups')
      return self.net.fp.grad
    if adam is not None:
      args = self._adam_args(adam, slot)
      _lib.check(_lib.lib.dq_cnn_backward_adam(
          ctypes.byref(self._p), ctypes.byref(self._g), self.B, self._x.data_ptr(),
          ctypes.byref(self._a), dout.data_ptr(), ctypes.byref(self._d), self.ws.data_ptr(),
          ctypes.byref(args), self._stream(dout)), 'dq_cnn_backward_adam')
      return self.net.fp.grad
    if not parallel:
      _lib.check(_lib.lib.dq_cnn_backward(ctypes.byref(self._p), ctypes.byref(self._g), self.B,
                                          self._x.data_ptr(), ctypes.byref(self._a),
                                          dout.data_ptr(), ctypes.byref(self._d),
                                          self.ws.data_ptr(), self._stream(dout)),
                 'dq_cnn_backward')
      return self.net.fp.grad
    main = torch.cuda.current_stream(dout.device)
    if self._dw_stream is None:
      self._dw_stream = torch.cuda.Stream(dout.device)
      self._events = [torch.cuda.Event() for _ in range(5)]
    side, ev = self._dw_stream, self._events

    def layer(i, part, stream, ws):
      _lib.check(_lib.lib.dq_cnn_backward_layer(
          ctypes.byref(self._p), ctypes.byref(self._g), self.B, self._x.data_ptr(),
          ctypes.byref(self._a), dout.data_ptr(), ctypes.byref(self._d), ws.data_ptr(), i, part,
          ctypes.c_void_p(stream.cuda_stream)), 'dq_cnn_backward_layer')

    # ev[i] marks "input gradient of layer i-1 done" (ev[0]: dout ready)
    ev[0].record(main)
    for i in range(4):                     # fc2, fc1, conv3, conv2
      side.wait_event(ev[i])
      layer(i, 1, side, self.ws_dw)
      layer(i, 0, main, self.ws)
      if i < 3:
        ev[i + 1].record(main)
    layer(4, 1, main, self.ws)             # conv1 weight gradient: last on the chain
    ev[4].record(side)
    main.wait_event(ev[4])
    return self.net.fp.grad


def forward_pair(a, xa, b, xb):
  """``a.forward(xa)`` and ``b.forward(xb)`` (e.g. the online net on s and the
  target net on s') in one pass: 6 grouped launches instead of 12, bitwise the
  same outputs.  Returns the two output buffers."""
  assert a.B == b.B and a is not b
  xa, xb = a._nhwc(xa), b._nhwc(xb)
  a._x, b._x = xa, xb
  _lib.check(_lib.lib.dq_cnn_forward_pair(
      ctypes.byref(a._p), xa.data_ptr(), ctypes.byref(a._a), a.ws.data_ptr(),
      ctypes.byref(b._p), xb.data_ptr(), ctypes.byref(b._a), b.ws.data_ptr(), a.B,
      a._stream(xa)), 'dq_cnn_forward_pair')
  return a.acts['out'], b.acts['out']


def forward_with_tail(a, xa, b):
  """``a.forward(xa)`` with ``b``'s tail (after ``b.forward_head`` or a backward
  ``head=``) in its last two launches.  Returns the two output buffers."""
  assert a.B == b.B and a is not b
  xa = a._nhwc(xa)
  a._x = xa
  _lib.check(_lib.lib.dq_cnn_forward_with_tail(
      ctypes.byref(a._p), xa.data_ptr(), ctypes.byref(a._a), a.ws.data_ptr(),
      ctypes.byref(b._p), ctypes.byref(b._a), b.ws.data_ptr(), a.B, a._stream(xa)),
      'dq_cnn_forward_with_tail')
  return a.acts['out'], b.acts['out']


def fc2_parts(net):
  """The (16, B, n_out) view of ``net``'s fc2 k-band partials (forward_fused)."""
  off = int(_lib.lib.dq_cnn_fc2_parts_offset(net.B))
  n = 16 * net.B * net.n_out
  return net.ws[off:off + n].view(16, net.B, net.n_out)


def forward_fused(a, xa, b, fc1_b=True, conv3_b=False, part=None, conv2_b=False, xb=None,
                  peer=None, var=None):
  """The Rainbow fast path's forward (dq_cnn_forward_fused): ``a`` (online) on
  ``xa`` through fc1, ``b`` (target; conv1..conv3 already run, e.g. riding in the
  previous backward with head_from=4) from its fc1 slabs (if ``fc1_b``; with
  ``conv3_b`` its conv3 too, beside ``a``'s conv3: head_from=5), then one
  launch summing both nets' fc1 slabs and forming fc2's 16 k-band partials.
  Neither net's logits are stored: ``ops.c51_loss_fused`` sums the partials
  (bitwise the logits of ``forward``).  part='convs' / 'fcs': only the three conv
  launches / only the fc launches (the same launches in two calls).  conv2_b / xb:
  ``b``'s conv2 beside ``a``'s conv2 (head_from=6) / ``b``'s conv1 on ``xb`` beside
  ``a``'s conv1 (head_from=7: no target head in the backward).  peer / var (head_from 6, the
  whole forward): the data-parallel exchange's deferred all-gather (the previous step's
  ``backward_peer(..., defer_ag=True)``) into ``a``'s flat parameters ``var`` rides in the
  three conv launches (dq_cnn_forward_fused_peer).  Returns the two partial views."""
  assert a.B == b.B and a is not b
  xa = a._nhwc(xa)
  a._x = xa
  if peer is not None:
    assert conv2_b and part is None and xb is None
    _lib.check(_lib.lib.dq_cnn_forward_fused_peer(
        ctypes.byref(a._p), xa.data_ptr(), ctypes.byref(a._a), a.ws.data_ptr(),
        ctypes.byref(b._p), None, ctypes.byref(b._a), b.ws.data_ptr(), a.B,
        int(bool(fc1_b)) | 2 * int(bool(conv3_b)) | 16, ctypes.byref(peer), var.data_ptr(),
        a._stream(xa)), 'dq_cnn_forward_fused_peer')
    return fc2_parts(a), fc2_parts(b)
  _lib.check(_lib.lib.dq_cnn_forward_fused(
      ctypes.byref(a._p), xa.data_ptr(), ctypes.byref(a._a), a.ws.data_ptr(),
      ctypes.byref(b._p), None if xb is None else b._nhwc(xb).data_ptr(), ctypes.byref(b._a),
      b.ws.data_ptr(), a.B,
      int(bool(fc1_b)) | 2 * int(bool(conv3_b)) | {None: 0, 'convs': 4, 'fcs': 8}[part] |
      16 * int(bool(conv2_b)) | 32 * int(xb is not None),
      a._stream(xa)), 'dq_cnn_forward_fused')
  return fc2_parts(a), fc2_parts(b)


def forward_fused_c51(a, xa, b, rewards, terminals, support, cumulative_gamma, m_out,
                      target_logits_out=None, part=None):
  """dq_cnn_forward_fused_c51 (head_from = 8): ``a`` (online) on ``xa`` as
  ``forward_fused``, ``b`` (target; its conv1 already run, by the previous backward) one
  launch ahead -- its conv2 / conv3 / fc1 slabs / fused head beside ``a``'s conv1 / conv2
  / conv3 / fc1 -- and the target half of the C51 loss beside ``a``'s fused head, writing
  the projected target distribution into ``m_out`` (B, N).  part: as forward_fused."""
  assert a.B == b.B and a is not b
  xa = a._nhwc(xa)
  a._x = xa
  t = _lib.C51Target(rewards=rewards.data_ptr(), terminals=terminals.data_ptr(),
                     support=support.data_ptr(), num_atoms=int(support.numel()),
                     cumulative_gamma=float(cumulative_gamma), m_out=m_out.data_ptr(),
                     target_logits_out=None if target_logits_out is None
                     else target_logits_out.data_ptr())
  _lib.check(_lib.lib.dq_cnn_forward_fused_c51(
      ctypes.byref(a._p), xa.data_ptr(), ctypes.byref(a._a), a.ws.data_ptr(),
      ctypes.byref(b._p), ctypes.byref(b._a), b.ws.data_ptr(), a.B, ctypes.byref(t),
      {None: 0, 'convs': 4, 'fcs': 8}[part], a._stream(xa)), 'dq_cnn_forward_fused_c51')
  return fc2_parts(a), m_out
