"""Data-parallel learners, one process per GPU (BASELINE config 4).

Each rank owns a full 1M-transition buffer, its own PER priorities and RNG
streams, and a model replica.  Sampling, gather, targets, losses, priority
write-back and target sync are rank-local; the only exchange is ONE all-reduce
of the flat fp32 gradient per step (4,278,891 floats = 17.1 MB for
Rainbow/Asterix) over RCCL/xGMI, then every rank applies the identical TF1
Adam update, so replicas stay bit-identical.  PER's `w /= max(w)` stays
per-rank (rainbow_agent.py:280): the multi-GPU gradient is the mean of the
ranks' single-GPU gradients, not a single B*N batch.
"""
import ctypes
import os
import sys
import threading
import time

import torch
import torch.distributed as dist

# Run the collectives even in a one-rank group (DQ_FORCE_COLLECTIVES=1): a one-GPU box
# can then drive the RCCL path itself (bench.py --force-dist, tests/test_gpu_rccl.py);
# an average over one rank leaves the values unchanged.
FORCE_COLLECTIVES = os.environ.get('DQ_FORCE_COLLECTIVES') == '1'


def allreduce_mean_(flat_grad, group=None):
  """In-place mean of a flat gradient buffer across the ranks of ``group``."""
  world = dist.get_world_size(group)
  if world == 1 and not FORCE_COLLECTIVES:
    return flat_grad
  if dist.get_backend(group) == 'nccl':     # RCCL averages in the collective (no extra kernel)
    dist.all_reduce(flat_grad, op=dist.ReduceOp.AVG, group=group)
    return flat_grad
  # gloo (the CPU tests and one-GPU rehearsals of N ranks): every rank's gradient gathered,
  # summed in group-rank order, then scaled -- (((g0 + g1) + g2) + ...) * (1 / N) on every
  # rank, a fixed order a single-process reference can restate bit for bit at any N
  # (gloo's own all-reduce sums in a ring/chunk order that depends on N; with 2 ranks the
  # two agree, a + b being commutative)
  parts = [torch.empty_like(flat_grad) for _ in range(world)]
  dist.all_gather(parts, flat_grad, group=group)
  flat_grad.copy_(parts[0])
  for p in parts[1:]:
    flat_grad.add_(p)
  flat_grad.mul_(1.0 / world)
  return flat_grad


def _active(group):
  return dist.get_world_size(group) > 1 or FORCE_COLLECTIVES


def reduce_scatter_mean_(flat, group=None):
  """In place: slice r of ``flat`` (numel divisible by the group size; slice r = the r-th
  equal part) becomes the mean of that slice over the ranks, on group rank r.  RCCL
  reduce-scatters in place (output = input + r * count, ReduceOp.AVG); over gloo the
  whole range is all-reduced (every slice holds its mean: the replicated path's bits)."""
  world = dist.get_world_size(group)
  if not _active(group):
    return flat
  assert flat.numel() % world == 0
  if dist.get_backend(group) == 'nccl':
    n = flat.numel() // world
    r = dist.get_rank(group)
    dist.reduce_scatter_tensor(flat[r * n:(r + 1) * n], flat, op=dist.ReduceOp.AVG, group=group)
    return flat
  return allreduce_mean_(flat, group)


def all_gather_(flat, group=None):
  """In place: slice r of ``flat`` (as reduce_scatter_mean_) on every rank becomes group
  rank r's slice.  RCCL all-gathers in place; over gloo, one broadcast per slice."""
  world = dist.get_world_size(group)
  if not _active(group):
    return flat
  assert flat.numel() % world == 0
  n = flat.numel() // world
  if dist.get_backend(group) == 'nccl':
    r = dist.get_rank(group)
    dist.all_gather_into_tensor(flat, flat[r * n:(r + 1) * n], group=group)
    return flat
  ranks = dist.get_process_group_ranks(group) if group is not None else list(range(world))
  for i, src in enumerate(ranks):
    dist.broadcast(flat[i * n:(i + 1) * n], src=src, group=group)
  return flat


class RcclComm(object):
  """One RCCL communicator over ``group``'s ranks, owned by the learner (dq_comm_*,
  dopamine_amd/csrc/comm.hip): each collective is issued on the CURRENT stream, in place,
  with no internal stream of its own -- so inside a captured HIP graph a bucket costs the
  queue it runs on and nothing else (torch's ProcessGroupNCCL forks every collective onto
  its own stream and joins it back: two more cross-queue edges per collective).  The
  ncclUniqueId of group rank 0 reaches every rank by a broadcast over ``group``; every rank
  must construct its RcclComm at the same point (ncclCommInitRank is collective)."""

  def __init__(self, group, device):
    from dopamine_amd import _lib
    # RCCL's implicit launch order (on by default in this RCCL) chains the kernels of every
    # communicator of the process in host call order: inside the captured step the fc
    # bucket's all-reduce, issued first on the comm stream, then started only after the conv
    # bucket's, ~45 us late (rocprof, profiles/r3_dist).  The two buckets' kernels are small
    # grids that fit on the GPU together, so no cross-communicator order is needed for progress.
    # This package dlopens /opt/rocm/lib/librccl.so.1 by path: a second RCCL instance beside
    # the torch/lib/librccl.so torch links (two mappings in /proc/self/maps,
    # tests/test_cabi.py), with its own parameter cache, read at its first communicator init
    # here.  The variable is process-wide, but torch's instance has created its
    # communicators and run its first collectives (replica broadcast, the availability
    # check) before this point, and it serves one communicator per process group.
    os.environ.setdefault('NCCL_LAUNCH_ORDER_IMPLICIT', '0')
    self._lib = _lib
    self.world = dist.get_world_size(group)
    self.rank = dist.get_rank(group)
    uid = torch.zeros(128, dtype=torch.uint8)
    if self.rank == 0:
      _lib.call('dq_comm_unique_id', ctypes.c_void_p(uid.data_ptr()))
    on_dev = dist.get_backend(group) == 'nccl'
    t = uid.to(device) if on_dev else uid
    dist.broadcast(t, src=dist.get_process_group_ranks(group)[0], group=group)
    uid.copy_(t.cpu())
    h = ctypes.c_void_p()
    _lib.call('dq_comm_create', ctypes.c_void_p(uid.data_ptr()), self.world, self.rank,
              torch.device(device).index or 0, ctypes.byref(h))
    self._h = h
    self.device = torch.device(device)

  def _stream(self):
    return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

  def _active(self):
    return self.world > 1 or FORCE_COLLECTIVES

  def allreduce_mean_(self, flat):
    """As allreduce_mean_, on the current stream."""
    assert flat.is_contiguous() and flat.dtype == torch.float32
    if self._active():
      self._lib.call('dq_comm_allreduce_mean', self._h, ctypes.c_void_p(flat.data_ptr()),
                     flat.numel(), self._stream())
    return flat

  def reduce_scatter_mean_(self, flat):
    """As reduce_scatter_mean_, on the current stream."""
    assert flat.is_contiguous() and flat.numel() % self.world == 0
    if self._active():
      self._lib.call('dq_comm_reduce_scatter_mean', self._h, ctypes.c_void_p(flat.data_ptr()),
                     flat.numel() // self.world, self._stream())
    return flat

  def all_gather_(self, flat):
    """As all_gather_, on the current stream."""
    assert flat.is_contiguous() and flat.numel() % self.world == 0
    if self._active():
      self._lib.call('dq_comm_all_gather', self._h, ctypes.c_void_p(flat.data_ptr()),
                     flat.numel() // self.world, self._stream())
    return flat

  def destroy(self):
    if self._h:
      torch.cuda.synchronize(self.device)
      self._lib.call('dq_comm_destroy', self._h)
      self._h = None


def native_comm_available(group, device):
  """Whether EVERY rank of ``group`` can open RCCL for RcclComm (dq_comm_version): the ranks
  agree (MIN all-reduce) before any of them enters the collective communicator init, so a
  rank that cannot does not leave the others blocked in it."""
  from dopamine_amd import _lib
  ok = 1.0 if int(_lib.lib.dq_comm_version()) > 0 else 0.0
  t = torch.tensor([ok], device=device if dist.get_backend(group) == 'nccl' else 'cpu')
  dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
  return bool(t.item() == 1.0)


def agree_min(value, group):
  """The smallest of an integer every rank of ``group`` holds (e.g. the newest checkpoint
  iteration every rank completed)."""
  dev = torch.device('cuda', torch.cuda.current_device()) if dist.get_backend(group) == 'nccl' \
      else 'cpu'
  t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
  dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
  return int(t.item())


class PeerExchange(object):
  """The data-parallel exchange over peer memory (include/dopamine_amd.h dq_peer; DESIGN.md
  6): every learner maps every other learner's flat gradient, parameter and flag buffers
  (IPC handles exchanged over ``group``, a host-side collective), and the backward's grouped
  launches run the reduce-scatter + slice Adam, the conv bucket's mean + Adam and the all-
  gather as extra blocks on the learner's ONE stream (cnn.HipNatureCNN.backward_peer).

  ``[lo, n)``: the sharded range of the flat buffers (the fc bucket, minus a head of < 4N
  floats that joins the conv bucket); every rank keeps the Adam moments of its own slice
  only (ZeRO-1: DQNAgent._gather_opt_state gathers them for a checkpoint).  group None: one
  learner running the same protocol with itself (world 1).  Requires every learner on one
  node with peer access between their devices (``available``).

  Construction ends with a self-test of the exchange's memory path (dq_peer_selftest): every
  rank stores a pattern over its gradient buffer from every XCD, publishes it through the
  product publication, and reads every rank's buffer through the exchange's loads.  Any
  mismatched word, timeout or short XCD coverage on any rank raises RuntimeError on every
  rank (the ranks agree), so a learner never trains over an exchange that reads stale memory."""

  MAX_POLLS = 30_000_000     # per wait (~1-2 us per poll): a dead peer latches an error in < 1 min,
  # a live one may lag by tens of seconds (first-use code loads, host noise) without one
  SELFTEST_POLLS = 30_000_000   # the self-test's wait, whatever max_polls the exchange uses

  def __init__(self, group, device, grad, params, lo, n, max_polls=None):
    from dopamine_amd import _lib
    self._lib = _lib
    self.group = group
    self.world = 1 if group is None else dist.get_world_size(group)
    self.rank = 0 if group is None else dist.get_rank(group)
    self.device = torch.device(device)
    assert self.world <= _lib.PEER_MAX, 'the peer exchange holds at most %d ranks' % _lib.PEER_MAX
    assert lo % 4 == 0 and (n - lo) % (4 * self.world) == 0
    self.lo, self.n = int(lo), int(n)
    self.flags = torch.zeros(_lib.PEER_FLAG_WORDS, dtype=torch.int64, device=device)
    self._grad = grad
    self._opened = []
    bufs = (grad, params, self.flags)
    ptrs = [[0] * 3 for _ in range(self.world)]
    ptrs[self.rank] = [b.data_ptr() for b in bufs]
    tag = int.from_bytes(os.urandom(4), 'little')
    if self.world > 1:
      mine = []
      for b in bufs:
        h = _lib.IpcHandle()
        _lib.call('dq_peer_ipc_get', ctypes.c_void_p(b.data_ptr()), ctypes.byref(h))
        mine.append(bytes(ctypes.string_at(ctypes.addressof(h), ctypes.sizeof(h))))
      allh = [None] * self.world
      dist.all_gather_object(allh, (mine, tag), group=group)
      tag = allh[0][1]                     # group rank 0's self-test tag
      torch.cuda.synchronize(device)
      err = None
      try:
        for q in range(self.world):
          if q == self.rank:
            continue
          for k in range(3):
            h = _lib.IpcHandle.from_buffer_copy(allh[q][0][k])
            ptr, base = ctypes.c_void_p(), ctypes.c_void_p()
            _lib.call('dq_peer_ipc_open', ctypes.byref(h), ctypes.byref(ptr), ctypes.byref(base))
            self._opened.append(base.value)
            ptrs[q][k] = ptr.value
      except _lib.DQError as e:
        err = str(e)
      # every rank learns whether every mapping opened: all raise together or none does
      errs = [None] * self.world
      dist.all_gather_object(errs, err, group=group)
      if any(e is not None for e in errs):
        self.close()
        raise RuntimeError('peer exchange: mapping the other learners\' buffers failed: %s'
                           % next(e for e in errs if e is not None))
    d = _lib.Peer(world=self.world, rank=self.rank, lo=self.lo, n=self.n,
                  max_polls=int(max_polls or self.MAX_POLLS), xcds=xcd_count(device))
    for q in range(self.world):
      d.grad[q], d.param[q], d.flags[q] = ptrs[q]
    self.desc = d
    self.selftest = self._selftest(tag)

  def _selftest(self, tag):
    """dq_peer_selftest, the ranks agreeing on the verdict; raises RuntimeError (on every
    rank) if any rank saw a mismatched word, a timeout or too few XCDs.  Returns the verdict.
    (DQ_PEER_SKIP_SELFTEST=1 skips it in a diagnostic build only -- so that the replica
    checks after a bench window can be shown to catch what the self-test would have.)"""
    L = self._lib
    if os.environ.get('DQ_PEER_SKIP_SELFTEST') == '1' and L.BUILD_FLAGS:
      return {'skipped': True, 'build': L.BUILD_FLAGS}
    out = torch.zeros(1, dtype=torch.int32, device=self.device)
    t0 = time.perf_counter()
    d = L.Peer.from_buffer_copy(self.desc)
    d.max_polls = max(int(d.max_polls), self.SELFTEST_POLLS)
    L.call('dq_peer_selftest', ctypes.byref(d), ctypes.c_uint32(tag & 0xffffffff),
           ctypes.c_void_p(out.data_ptr()), L.stream_of(self.device))
    torch.cuda.synchronize(self.device)
    mine = {'rank': self.rank, 'mismatched_words': int(out.item()),
            'error': int(self.flags[L.PEER_ERR].item()),
            'xcds_seen': int(self.flags[L.PEER_PUB_XCDS].item()), 'xcds_needed': self.desc.xcds,
            'ms': round(1e3 * (time.perf_counter() - t0), 2)}
    allv = [mine]
    if self.group is not None:
      allv = [None] * self.world
      dist.all_gather_object(allv, mine, group=self.group)   # every rank's reads are done
    self._grad.zero_()                 # the pattern leaves this rank's gradient buffer
    verdict = {'ok': all(v['mismatched_words'] == 0 and v['error'] == 0 for v in allv),
               'words_per_rank': self.n * self.world, 'ranks': allv}
    if not verdict['ok']:
      self.close()
      bad = [v for v in allv if v['mismatched_words'] or v['error']]
      raise RuntimeError('peer exchange: the self-test of the exchange\'s memory path failed '
                         '(%s)' % '; '.join('rank %d: %d stale or wrong words of %d read, %s'
                                            % (v['rank'], v['mismatched_words'],
                                               self.n * self.world, self.describe(v['error']))
                                            for v in bad))
    return verdict

  @staticmethod
  def available(group, device):
    """Whether every learner of ``group`` can run the exchange: one host, and for every other
    learner's GPU (identified by its PCI address, not by a process-local ordinal) either the
    same GPU or one this process sees with peer access to it.  Collective; every rank gets
    the same answer."""
    import socket
    from dopamine_amd import _lib
    me = (socket.gethostname(), pci_address(device))
    allm = [None] * dist.get_world_size(group)
    dist.all_gather_object(allm, me, group=group)
    ok = all(h == me[0] for h, _ in allm) and dist.get_world_size(group) <= _lib.PEER_MAX
    if ok:
      visible = {pci_address(i): i for i in range(torch.cuda.device_count())}
      mine = torch.device(device).index or 0
      for _, addr in allm:
        if addr == me[1]:
          continue                       # the same GPU (learners sharing one device)
        j = visible.get(addr)
        if j is None or int(_lib.lib.dq_peer_can_access(mine, j)) != 1:
          ok = False                     # a GPU this process cannot see or map
    flags = [None] * dist.get_world_size(group)
    dist.all_gather_object(flags, bool(ok), group=group)
    return all(flags)

  def all_gather(self, var, stream):
    """The deferred all-gather in a launch of its own (dq_peer_all_gather): every other
    rank's slice of ``var`` (this learner's flat parameters) as of its last published step
    (the learner loop's last step, so every parameter is current when the loop returns)."""
    self._lib.call('dq_peer_all_gather', ctypes.byref(self.desc), ctypes.c_void_p(var.data_ptr()),
                   stream)

  def error(self):
    """0, or the latched error word (a synchronising read; describe())."""
    return int(self.flags[self._lib.PEER_ERR].item())

  def describe(self, e):
    L = self._lib
    if e == 0:
      return 'no error'
    if e >= L.PEER_ERR_XCD:
      return ('a publication\'s blocks ran on %d XCD(s), fewer than the %d whose L2 write-back '
              'it needs' % (e - L.PEER_ERR_XCD, self.desc.xcds))
    if e >= L.PEER_ERR_PEER:
      return 'rank %d had latched an error, so this one stopped' % (e - L.PEER_ERR_PEER)
    names = {1 + L.PEER_GRAD: 'gradients', 1 + L.PEER_PARAM: 'parameters',
             1 + L.PEER_CONV: 'conv gradients', 1 + L.PEER_TEST: 'self-test pattern'}
    return ('timed out waiting for the other learners\' %s (a learner stopped or fell out of '
            'step)' % names.get(e, e))

  def check(self, collective=False):
    """Raises RuntimeError if this learner's error word is latched.  collective: the ranks
    first agree (MAX all-reduce of the error words over the group), so every rank raises
    together -- call it at the same point on every rank."""
    e = self.error()
    worst = e
    if collective and self.group is not None:
      t = torch.tensor([e], dtype=torch.int64,
                       device=self.device if dist.get_backend(self.group) == 'nccl' else 'cpu')
      dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
      worst = int(t.item())
    if e:
      raise RuntimeError('peer exchange: rank %d: %s' % (self.rank, self.describe(e)))
    if worst:
      raise RuntimeError('peer exchange: rank %d: another learner latched an error (%s)'
                         % (self.rank, self.describe(worst)))

  def wait_counters(self):
    """This rank's cumulative waits at the three exchange points: {point: (ticks of the
    100 MHz clock, waits counted)} (block 0 of each waiting op; a synchronising read)."""
    f = self.flags.cpu().tolist()
    L = self._lib
    return {name: (int(f[L.PEER_WAIT_TICKS + i]), int(f[L.PEER_WAIT_COUNT + i]))
            for i, name in enumerate(('grad', 'param', 'conv'))}

  def close(self):
    for base in self._opened:
      self._lib.call('dq_peer_ipc_close', ctypes.c_void_p(base))
    self._opened = []


def pci_address(device):
  """(domain, bus, device) PCI address of a GPU: the same physical GPU has the same address
  in every process, whatever HIP_VISIBLE_DEVICES numbers it."""
  p = torch.cuda.get_device_properties(device)
  return (int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))


def xcd_count(device):
  """XCDs of the device (32 CUs each on MI355X: 8 for a whole GPU, 1 in a CPX partition)."""
  cus = torch.cuda.get_device_properties(device).multi_processor_count
  return max(1, min(8, cus // 32))


# exit status of a process whose deadline expired (Deadline)
DEADLINE_EXIT = 3


class Deadline(object):
  """Host-side deadline for the blocking phases of an N > 1 run (rendezvous, the barriers
  around the timed window, the window's captured collectives, the final exchanges).

  ``phase(label, seconds)`` names what the process is about to wait for and arms the
  deadline; ``done()`` disarms it.  A watcher thread that finds an armed deadline expired
  prints ``rank R: <label> did not complete within S s`` to stderr and ends the process with
  DEADLINE_EXIT (os._exit: no in-process retry, nothing after it runs; the launcher sees a
  non-zero status instead of a hang).  A peer that died or withheld a collective leaves the
  other ranks blocked inside RCCL / gloo, where no Python exception can reach them -- the
  watcher is what bounds it."""

  def __init__(self, rank=None, out=None, poll=0.2):
    self.rank = int(os.environ.get('RANK', '0')) if rank is None else rank
    self._out = out
    self._poll = poll
    self._lock = threading.Lock()
    self._label, self._expires, self._seconds = None, None, None
    self._stop = threading.Event()
    self._thread = threading.Thread(target=self._watch, name='dq-deadline', daemon=True)
    self._thread.start()

  def phase(self, label, seconds):
    with self._lock:
      self._label, self._seconds = label, float(seconds)
      self._expires = time.monotonic() + float(seconds)

  def done(self):
    with self._lock:
      self._label = self._expires = None

  def close(self):
    self.done()
    self._stop.set()

  def _watch(self):
    while not self._stop.wait(self._poll):
      with self._lock:
        expired = self._expires is not None and time.monotonic() > self._expires
        label, seconds = self._label, self._seconds
      if expired:
        out = self._out or sys.stderr
        out.write('dopamine_amd deadline: rank %d: %s did not complete within %.0f s; '
                  'exiting with status %d\n' % (self.rank, label, seconds, DEADLINE_EXIT))
        out.flush()
        os._exit(DEADLINE_EXIT)


def replica_report(tensors, group=None):
  """Collective: every rank compares each of ``tensors`` ({name: tensor}, the same names on
  every rank) with group rank 0's copy, bit for bit (broadcast, then the elements whose bits
  differ).  Returns {name: {'in_sync': bool, 'differing': [elements differing from rank 0's,
  per group rank], 'max_abs_diff': [per group rank]}} -- the same dict on every rank."""
  nccl = dist.get_backend(group) == 'nccl'
  src = dist.get_process_group_ranks(group)[0] if group is not None else 0
  world = dist.get_world_size(group)
  rows = []
  for name in sorted(tensors):
    x = tensors[name].detach().contiguous().reshape(-1)
    if not nccl:
      x = x.cpu()
    ref = x.clone()
    dist.broadcast(ref, src=src, group=group)
    ib = {4: torch.int32, 8: torch.int64}[x.element_size()]
    diff = x.view(ib) != ref.view(ib)
    n = int(diff.sum().item())
    mad = 0.0
    if n:
      d = (x.double() - ref.double()).abs()
      mad = float(torch.nan_to_num(d, nan=float('inf')).max().item())
    rows.append((n, mad))
  t = torch.tensor([v for r in rows for v in r], dtype=torch.float64,
                   device=torch.device('cuda', torch.cuda.current_device()) if nccl else 'cpu')
  parts = [torch.empty_like(t) for _ in range(world)]
  dist.all_gather(parts, t, group=group)
  out = {}
  for i, name in enumerate(sorted(tensors)):
    n = [int(p[2 * i].item()) for p in parts]
    m = [float(p[2 * i + 1].item()) for p in parts]
    out[name] = {'in_sync': not any(n), 'differing': n, 'max_abs_diff': m}
  return out


def replicas_in_sync(flat_params, group=None):
  """Checksum-broadcast check that every rank holds identical parameters."""
  s = torch.stack([flat_params.double().sum(), (flat_params.double() ** 2).sum()])
  ref = s.clone()
  dist.broadcast(ref, src=0, group=group)
  ok = torch.tensor([1.0 if torch.equal(s, ref) else 0.0], dtype=torch.float64, device=s.device)
  dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
  return bool(ok.item() == 1.0)


_CAPTURABLE = {}


def forget_capture_probes(comms):
  """Drops the cached probe results of a communicator pair about to be destroyed (the
  cache is keyed by object identity, which a later pair may reuse)."""
  ids = tuple(id(c) for c in comms)
  for key in [k for k in _CAPTURABLE if k[3] == ids]:
    del _CAPTURABLE[key]


def collectives_capturable(group, device, stream=None, sharded=False, group2=None, comms=None):
  """Whether every rank of ``group`` can capture the learner's collectives into a HIP
  graph and replay them correctly -- probed once per communicator pair on a small tensor,
  the ranks agreeing (eager MIN all-reduces) after each phase so no rank replays a
  collective the others did not capture.  comms: the learner's RcclComm pair (fc bucket on
  the comm stream, conv bucket on the origin).  False for gloo (host-side collectives) and
  for torch.distributed's own collectives (comms None; see below).  The learner loop
  captures its collectives only where this holds, else it replays per-step graphs with the
  collectives issued between them.  (group2: accepted for the old call form; unused.)"""
  key = (id(group), bool(sharded), id(group2) if group2 is not None else None,
         None if comms is None else tuple(id(c) for c in comms))
  if key in _CAPTURABLE:
    return _CAPTURABLE[key]
  if dist.get_backend(group) != 'nccl' or comms is None:
    # gloo: host-side collectives.  torch.distributed's RCCL collectives: never captured.
    # Capturing them once aborted the process from torch's process-group watchdog (round 3;
    # ROCm 7.2, torch 2.10), which keeps every eager work on a list and polls its events from
    # its own thread until it retires it.  Measured on HIP 7.2 (tools/micro/
    # event_query_capture.hip, profiles/r4_dist/event_query_capture.log): a thread-local
    # capture fails -- hipErrorStreamCaptureUnsupported, and the capture is invalidated --
    # on ANY hipEventQuery made by the capturing thread, while queries from other threads
    # return success even for events recorded inside the capture.  So whether a capture
    # survives depends on what torch's collective path and its watchdog do with their event
    # lists at that moment -- state this package cannot see or wait on (a sleep only made
    # the race rarer).  Only the learner's own communicators (RcclComm: no internal
    # stream, no work list, no watchdog) are captured; with torch's collectives the learner
    # loop replays per-step graphs with the collectives issued between them.
    _CAPTURABLE[key] = False
    return False

  def agree(ok):
    t = torch.tensor([1.0 if ok else 0.0], device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item() == 1.0)

  rank = dist.get_rank(group)
  world = dist.get_world_size(group)
  x = torch.full((1024 * world,), float(rank + 1), device=device)
  y = torch.full((1024,), float(rank + 1), device=device)
  comm = stream or torch.cuda.Stream(device)
  cap = torch.cuda.Stream(device)

  def collectives(origin):
    """As the learner loop captures them: the fc bucket's collectives on the comm stream
    forked from the origin stream and joined back (sharded: the ZeRO-1 pair as well),
    the second communicator's all-reduce on the origin stream meanwhile."""
    e = torch.cuda.Event()
    e.record(origin)
    comm.wait_event(e)
    with torch.cuda.stream(comm):
      comms[0].allreduce_mean_(x)
      if sharded:
        comms[0].reduce_scatter_mean_(x)
        comms[0].all_gather_(x)
    with torch.cuda.stream(origin):
      comms[1].allreduce_mean_(y)
    e = torch.cuda.Event()
    e.record(comm)
    origin.wait_event(e)

  g = torch.cuda.CUDAGraph()
  ok = True
  # the communicators are warm before capture; eager collectives outside the try, so a
  # failure there is fatal on every rank instead of one rank leaving the others blocked
  collectives(torch.cuda.current_stream(device))
  torch.cuda.synchronize(device)
  try:
    cap.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(cap):
      with torch.cuda.graph(g, stream=cap, capture_error_mode='thread_local'):
        collectives(cap)
  except Exception:                               # noqa: BLE001 -- any failure means "no"
    ok = False
  ok = agree(ok)
  if ok:
    try:
      x.fill_(float(rank + 1))
      y.fill_(float(rank + 1))
      g.replay()
      torch.cuda.synchronize(device)
      want = sum(range(1, world + 1)) / world if (world > 1 or FORCE_COLLECTIVES) else 1.0
      ok = bool(torch.allclose(x, torch.full_like(x, want)))
      ok = ok and bool(torch.allclose(y, torch.full_like(y, want)))
    except Exception:                             # noqa: BLE001
      ok = False
    ok = agree(ok)
  _CAPTURABLE[key] = ok
  return ok
