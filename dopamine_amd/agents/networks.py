"""Q-networks of the reference (atari_lib.py:85-199, gym_lib.py:75-132) in
PyTorch-ROCm, with every parameter a view into ONE flat fp32 buffer.

The flat layout is the MI355X-side design choice: the TF1 Adam / RMSProp
update, the online->target sync and the multi-GPU gradient all-reduce are each
a single kernel / copy / RCCL call over the whole model (4.28 M floats for
Rainbow/Asterix) instead of one per variable.

Input convention: states arrive from the gather kernel as float32 NCHW
(B, stack, 84, 84) already divided by 255 (atari_lib.py:96-97 is fused into the
gather).  TF "SAME" padding is reproduced exactly (conv2 needs the asymmetric
(1, 2) pad).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


class FlatParams(object):
  """Allocates named parameter views inside one contiguous fp32 buffer (each
  slice 16-byte aligned) plus a matching flat gradient buffer.  tail_align = (name,
  multiple): zero padding at the end so that the range from parameter ``name`` to the end
  is a whole number of ``multiple`` floats (the Nature-CNN nets: the fc bucket splits into
  world equal 16-byte slices for every world size 1..8 -- the data-parallel exchanges'
  shards, DQNAgent._shard_bounds; the padding keeps zero gradients, so every optimizer
  leaves it zero)."""

  def __init__(self, shapes, device, tail_align=None):
    self.offsets = {}
    off = 0
    for name, shape in shapes:
      n = int(np.prod(shape))
      self.offsets[name] = (off, tuple(shape))
      off += (n + 3) // 4 * 4
    self.content_numel = off          # the tensors' floats, before the tail padding
    if tail_align is not None:
      name, multiple = tail_align
      off += -(off - self.offsets[name][0]) % multiple
    self.numel = off
    self.flat = torch.zeros(off, dtype=torch.float32, device=device)
    self.grad = torch.zeros(off, dtype=torch.float32, device=device)
    self.params = {}
    for name, (o, shape) in self.offsets.items():
      n = int(np.prod(shape))
      p = torch.nn.Parameter(self._view(self.flat, o, shape))
      p.grad = self._view(self.grad, o, shape)
      self.params[name] = p

    self.grad_views = [self._view(self.grad, o, s) for o, s in self.offsets.values()]

  def segments(self):
    """(offset, numel) of every parameter inside the flat buffer, in order."""
    return [(o, int(np.prod(s))) for o, s in self.offsets.values()]

  def gather_grads(self):
    """Copy autograd's per-parameter gradients into the flat gradient buffer
    (one multi-tensor copy kernel); returns the flat buffer."""
    ps = list(self.params.values())
    if all(p.grad is not None and p.grad.data_ptr() == v.data_ptr()
           for p, v in zip(ps, self.grad_views)):
      return self.grad
    torch._foreach_copy_(self.grad_views, [p.grad for p in ps])
    return self.grad

  @staticmethod
  def _view(buf, o, shape):
    n = int(np.prod(shape))
    if len(shape) == 4:   # conv filters stored (out, kh, kw, in): channels_last for MIOpen NHWC
      out_c, in_c, kh, kw = shape
      return buf[o:o + n].view(out_c, kh, kw, in_c).permute(0, 3, 1, 2)
    return buf[o:o + n].view(shape)

  def __getitem__(self, name):
    return self.params[name]

  def count(self):
    return sum(int(np.prod(s)) for _, s in self.offsets.values())


def _variance_scaling_uniform(shape, fan_in, factor, gen):
  # tf.contrib.slim.variance_scaling_initializer(factor, 'FAN_IN', uniform=True)
  limit = math.sqrt(3.0 * factor / fan_in)
  return (torch.rand(shape, generator=gen) * 2 - 1) * limit


def _xavier_uniform(shape, fan_in, fan_out, gen):
  # slim default initializer: xavier_initializer(uniform=True)
  limit = math.sqrt(6.0 / (fan_in + fan_out))
  return (torch.rand(shape, generator=gen) * 2 - 1) * limit


TORSO = [('conv1', (32, None, 8, 8), 4), ('conv2', (64, 32, 4, 4), 2), ('conv3', (64, 64, 3, 3), 1)]


class _Net(object):
  """Base: owns FlatParams; subclasses define shapes() and forward()."""

  tail_align = None

  def __init__(self, device, seed, init='rainbow'):
    self.fp = FlatParams(self.shapes(), device, self.tail_align)
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
      for name, (o, shape) in self.fp.offsets.items():
        if name.endswith('_b'):
          continue  # biases: zeros (slim default)
        if len(shape) == 4:
          fan_in, fan_out = shape[1] * shape[2] * shape[3], shape[0] * shape[2] * shape[3]
        else:
          fan_in, fan_out = shape[1], shape[0]
        if init == 'rainbow':
          w = _variance_scaling_uniform(shape, fan_in, 1.0 / np.sqrt(3.0), gen)
        else:
          w = _xavier_uniform(shape, fan_in, fan_out, gen)
        self.fp[name].copy_(w.to(device))

  def parameters(self):
    return list(self.fp.params.values())

  def __call__(self, *a, **k):
    return self.forward(*a, **k)


def _torso(fp, x):
  """Nature-CNN torso with TF SAME padding: 84 -> 21 -> 11 -> 11; 7744 features.

  Activations are channels_last (NHWC in memory: MIOpen's NHWC kernels run
  without layout transposes) and the flatten is in (h, w, c) order, i.e. exactly
  TF's slim.flatten of the reference's NHWC tensors (atari_lib.py:101)."""
  x = x.contiguous(memory_format=torch.channels_last)
  x = F.relu(F.conv2d(x, fp['conv1_w'], fp['conv1_b'], stride=4, padding=2))
  x = F.relu(F.conv2d(F.pad(x, (1, 2, 1, 2)), fp['conv2_w'], fp['conv2_b'], stride=2))
  x = F.relu(F.conv2d(x, fp['conv3_w'], fp['conv3_b'], stride=1, padding=1))
  return x.permute(0, 2, 3, 1).flatten(1)


def _torso_shapes(stack):
  return [('conv1_w', (32, stack, 8, 8)), ('conv1_b', (32,)),
          ('conv2_w', (64, 32, 4, 4)), ('conv2_b', (64,)),
          ('conv3_w', (64, 64, 3, 3)), ('conv3_b', (64,))]


# the fc bucket (fc1_w .. the end) in 4 * lcm(1..8) floats: equal 16-byte slices at any world
# size up to 8 (parallel.PeerExchange, ZeRO-1)
FC_BUCKET_ALIGN = ('fc1_w', 4 * 840)


class NatureDQNNetwork(_Net):
  """atari_lib.py:85-105 -> q_values (B, A)."""
  tail_align = FC_BUCKET_ALIGN

  def __init__(self, num_actions, stack_size=4, device='cuda', seed=0):
    self.A, self.S = num_actions, stack_size
    super().__init__(device, seed, init='xavier')

  def shapes(self):
    return _torso_shapes(self.S) + [('fc1_w', (512, 7744)), ('fc1_b', (512,)),
                                    ('fc2_w', (self.A, 512)), ('fc2_b', (self.A,))]

  def forward(self, x):
    h = F.relu(F.linear(_torso(self.fp, x), self.fp['fc1_w'], self.fp['fc1_b']))
    return F.linear(h, self.fp['fc2_w'], self.fp['fc2_b'])


class RainbowNetwork(_Net):
  """atari_lib.py:108-144 -> logits (B, A, N); q/probabilities derived."""
  tail_align = FC_BUCKET_ALIGN

  def __init__(self, num_actions, num_atoms=51, stack_size=4, device='cuda', seed=0):
    self.A, self.N, self.S = num_actions, num_atoms, stack_size
    super().__init__(device, seed, init='rainbow')

  def shapes(self):
    return _torso_shapes(self.S) + [('fc1_w', (512, 7744)), ('fc1_b', (512,)),
                                    ('fc2_w', (self.A * self.N, 512)), ('fc2_b', (self.A * self.N,))]

  def forward(self, x):
    h = F.relu(F.linear(_torso(self.fp, x), self.fp['fc1_w'], self.fp['fc1_b']))
    return F.linear(h, self.fp['fc2_w'], self.fp['fc2_b']).view(-1, self.A, self.N)


class ImplicitQuantileNetwork(_Net):
  """atari_lib.py:147-199: quantile_values (N*B, A), rows ordered q*B + b."""

  def __init__(self, num_actions, quantile_embedding_dim=64, stack_size=4, device='cuda', seed=0):
    self.A, self.E, self.S = num_actions, quantile_embedding_dim, stack_size
    super().__init__(device, seed, init='rainbow')
    self._i_pi = (torch.arange(1, self.E + 1, dtype=torch.float32, device=device) * math.pi)

  def shapes(self):
    return _torso_shapes(self.S) + [('emb_w', (7744, self.E)), ('emb_b', (7744,)),
                                    ('fc1_w', (512, 7744)), ('fc1_b', (512,)),
                                    ('fc2_w', (self.A, 512)), ('fc2_b', (self.A,))]

  def forward(self, x, num_quantiles, taus=None):
    B = x.shape[0]
    state = _torso(self.fp, x)                                   # (B, 7744)
    tiled = state.repeat(num_quantiles, 1)                       # tf.tile -> row q*B + b
    if taus is None:
      taus = torch.rand(num_quantiles * B, 1, device=x.device)   # tf.random_uniform
    emb = torch.cos(taus * self._i_pi)                           # (N*B, E)
    emb = F.relu(F.linear(emb, self.fp['emb_w'], self.fp['emb_b']))
    h = F.relu(F.linear(tiled * emb, self.fp['fc1_w'], self.fp['fc1_b']))
    return F.linear(h, self.fp['fc2_w'], self.fp['fc2_b']), taus


class CartpoleDQNNetwork(_Net):
  """gym_lib.py:75-132: rescale to [-1, 1] then FC 512-512-A."""

  MIN = np.array([-2.4, -5., -math.pi / 12., -math.pi * 2.])
  MAX = np.array([2.4, 5., math.pi / 12., math.pi * 2.])

  def __init__(self, num_actions, device='cuda', seed=0, network_size=(512, 512)):
    self.A, self.sizes = num_actions, tuple(network_size)
    super().__init__(device, seed, init='xavier')
    self._min = torch.tensor(self.MIN, dtype=torch.float32, device=device)
    self._rng = torch.tensor(self.MAX - self.MIN, dtype=torch.float32, device=device)

  def shapes(self):
    dims = [4] + list(self.sizes)
    s = []
    for i in range(len(self.sizes)):
      s += [('fc%d_w' % i, (dims[i + 1], dims[i])), ('fc%d_b' % i, (dims[i + 1],))]
    return s + [('out_w', (self.A, dims[-1])), ('out_b', (self.A,))]

  def forward(self, x):
    h = x.reshape(x.shape[0], -1).float()
    h = 2.0 * ((h - self._min) / self._rng) - 1.0
    for i in range(len(self.sizes)):
      h = F.relu(F.linear(h, self.fp['fc%d_w' % i], self.fp['fc%d_b' % i]))
    return F.linear(h, self.fp['out_w'], self.fp['out_b'])
