"""ctypes binding of the C ABI declared in include/dopamine_amd.h.

The HIP library is the ONLY compute path: if ``libdopamine_amd.so`` is missing
this module raises at import time -- there is no CPU fallback.
"""
import ctypes
import os

from dopamine_amd import _build
from dopamine_amd._build import HEADER, LIB_PATH  # noqa: F401

ABI_VERSION = 9
OK = 0
(ST_OK, ST_EMPTY_TREE, ST_MAX_ATTEMPTS, ST_TAPE_EXHAUSTED, ST_NEG_PRIORITY, ST_TOO_FEW, ST_BAD_INDEX,
 ST_BROADCAST) = range(8)
# DQ_DT_*: element types of dq_replay_gather_elems' reward store
DT_CODES = {'float32': 0, 'float64': 1, 'float16': 2, 'int8': 3, 'uint8': 4, 'int16': 5,
            'int32': 6, 'int64': 7}
LAYOUT_RAW, LAYOUT_F32_NORM, LAYOUT_F32_NHWC = 0, 1, 2
SUMTREE_QUERY, SUMTREE_RANDOM, SUMTREE_STRATIFIED = 0, 1, 2


class Meta(ctypes.Structure):
  _fields_ = [('add_count', ctypes.c_int64), ('tape_pos', ctypes.c_int64),
              ('tape_len', ctypes.c_int64), ('max_recorded_priority', ctypes.c_double),
              ('status', ctypes.c_int32), ('status_arg', ctypes.c_int32),
              ('status_value', ctypes.c_double), ('reserved', ctypes.c_int64 * 2)]


class Config(ctypes.Structure):
  _fields_ = [('capacity', ctypes.c_int64), ('obs_bytes', ctypes.c_int64),
              ('stack_size', ctypes.c_int32), ('update_horizon', ctypes.c_int32),
              ('max_sample_attempts', ctypes.c_int32), ('prioritized', ctypes.c_int32),
              ('obs_is_u8', ctypes.c_int32), ('pad_', ctypes.c_int32), ('gamma', ctypes.c_double)]


class Storage(ctypes.Structure):
  _fields_ = [('frames', ctypes.c_void_p), ('actions', ctypes.c_void_p),
              ('rewards', ctypes.c_void_p), ('terminals', ctypes.c_void_p),
              ('tree', ctypes.c_void_p), ('meta', ctypes.c_void_p), ('tape', ctypes.c_void_p),
              ('tape_capacity', ctypes.c_int64), ('discount', ctypes.c_void_p)]


MAX_TENSORS = 16


class AdamArgs(ctypes.Structure):
  _fields_ = [('var', ctypes.c_void_p), ('m', ctypes.c_void_p), ('v', ctypes.c_void_p),
              ('state', ctypes.c_void_p), ('slot', ctypes.c_int32), ('lr', ctypes.c_float),
              ('beta1', ctypes.c_float), ('beta2', ctypes.c_float), ('epsilon', ctypes.c_float),
              ('kind', ctypes.c_int32), ('centered', ctypes.c_int32), ('mg', ctypes.c_void_p),
              ('decay', ctypes.c_float), ('momentum', ctypes.c_float),
              ('no_grad_store', ctypes.c_int32)]


OPT_ADAM, OPT_RMSPROP = 0, 1


class TensorList(ctypes.Structure):
  _fields_ = [('count', ctypes.c_int32), ('pad_', ctypes.c_int32),
              ('var', ctypes.c_void_p * MAX_TENSORS), ('grad', ctypes.c_void_p * MAX_TENSORS),
              ('m', ctypes.c_void_p * MAX_TENSORS), ('v', ctypes.c_void_p * MAX_TENSORS),
              ('n', ctypes.c_int64 * MAX_TENSORS)]


class CnnParams(ctypes.Structure):
  _fields_ = [('in_channels', ctypes.c_int32), ('n_out', ctypes.c_int32)] + [
      (n, ctypes.c_void_p) for n in ('conv1_w', 'conv1_b', 'conv2_w', 'conv2_b', 'conv3_w',
                                     'conv3_b', 'fc1_w', 'fc1_b', 'fc2_w', 'fc2_b')]


class CnnActs(ctypes.Structure):
  _fields_ = [(n, ctypes.c_void_p) for n in ('a1', 'a2', 'a3', 'h', 'out')]


class C51Target(ctypes.Structure):
  _fields_ = [('rewards', ctypes.c_void_p), ('terminals', ctypes.c_void_p),
              ('support', ctypes.c_void_p), ('num_atoms', ctypes.c_int32),
              ('cumulative_gamma', ctypes.c_float), ('m_out', ctypes.c_void_p),
              ('target_logits_out', ctypes.c_void_p)]


class CnnNet(ctypes.Structure):
  _fields_ = [('p', ctypes.c_void_p), ('x', ctypes.c_void_p), ('a', ctypes.c_void_p),
              ('ws', ctypes.c_void_p)]


class IqnHead(ctypes.Structure):
  _fields_ = [('embed_dim', ctypes.c_int32), ('num_actions', ctypes.c_int32)] + [
      (n, ctypes.c_void_p) for n in ('emb_w', 'emb_b', 'fc1_w', 'fc1_b', 'fc2_w', 'fc2_b')]


class IqnActs(ctypes.Structure):
  _fields_ = [(n, ctypes.c_void_p) for n in ('cos', 'emb', 'x', 'h', 'q')]


class IqnGrads(ctypes.Structure):
  _fields_ = [(n, ctypes.c_void_p) for n in ('dh', 'dpre', 'dtl')]


class Rider(ctypes.Structure):
  """dq_rider: a recorded replay operation (opaque)."""
  _fields_ = [('words', ctypes.c_int64 * 40)]


PEER_MAX = 8            # DQ_PEER_MAX
PEER_FLAG_WORDS = 16    # DQ_PEER_FLAG_WORDS
(PEER_STEP, PEER_GRAD, PEER_PARAM, PEER_CONV, PEER_ERR, PEER_TICKET, PEER_PUB_COUNT,
 PEER_TEST) = range(8)
PEER_WAIT_TICKS = 8     # flags[8..10]: 100 MHz ticks waited at the grad / param / conv points
PEER_WAIT_COUNT = 11    # flags[11..13]: waits counted there
PEER_PUB_XCDS = 14      # flags[14]: XCDs the last publication's blocks ran on
PEER_ERR_PEER = 16      # error word: 16 + q -- rank q had latched an error
PEER_ERR_XCD = 32       # error word: 32 + k -- a publication saw only k XCDs


class IpcHandle(ctypes.Structure):
  _fields_ = [('handle', ctypes.c_uint8 * 64), ('offset', ctypes.c_int64)]


class Peer(ctypes.Structure):
  """dq_peer: the data-parallel exchange over peer memory."""
  _fields_ = [('world', ctypes.c_int32), ('rank', ctypes.c_int32), ('lo', ctypes.c_int64),
              ('n', ctypes.c_int64), ('grad', ctypes.c_void_p * PEER_MAX),
              ('param', ctypes.c_void_p * PEER_MAX), ('flags', ctypes.c_void_p * PEER_MAX),
              ('max_polls', ctypes.c_int64), ('xcds', ctypes.c_int32), ('reserved', ctypes.c_int32)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F = ctypes.c_float
_D = ctypes.c_double

# name -> argtypes (restype int unless noted); mirrors include/dopamine_amd.h
SIGNATURES = {
    'dq_abi_version': [],
    'dq_build_flags': [],
    'dq_last_error': [],
    'dq_sumtree_depth': [_I64],
    'dq_replay_create': [ctypes.POINTER(Config), ctypes.POINTER(Storage), ctypes.POINTER(_P)],
    'dq_replay_destroy': [_P],
    'dq_sumtree_create': [_I64, _P, _P, _P, _I64, ctypes.POINTER(_P)],
    'dq_replay_add': [_P, _I64, _P, _P, _P, _P, _P, _P],
    'dq_replay_sample_indices': [_P, _I32, _P, _P],
    'dq_replay_gather': [_P, _P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    'dq_replay_gather_elems': [_P, _P, _I32, _P, _I32, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _P,
                               _P],
    'dq_sumtree_set': [_P, _P, _P, _I64, _P],
    'dq_sumtree_set_f64': [_P, _P, _P, _I64, _P],
    'dq_sumtree_sample': [_P, _I32, _I32, _P, _P, _P],
    'dq_sumtree_get': [_P, _P, _I64, _P, _P],
    'dq_sumtree_rebuild': [_P, _P],
    'dq_replay_set_meta': [_P, _I64, _D, _P],
    'dq_replay_set_tape': [_P, _I64, _P],
    'dq_replay_read_meta': [_P, ctypes.POINTER(Meta), _P],
    'dq_replay_read_meta_async': [_P, _P, _P],
    'dq_replay_rewind_last_sample': [_P, _P],
    'dq_replay_egreedy': [_P, _P, _I32, _D, _P, _P],
    'dq_replay_record_sumtree_set': [_P, _P, _P, _I64, ctypes.POINTER(Rider)],
    'dq_replay_record_sample': [_P, _I32, _P, ctypes.POINTER(Rider)],
    'dq_replay_record_sample_groups': [_P, _I32, _I32, _P, ctypes.POINTER(Rider)],
    'dq_replay_sample_indices_groups': [_P, _I32, _I32, _P, _P],
    'dq_rider_chain': [ctypes.POINTER(Rider), ctypes.POINTER(Rider), ctypes.POINTER(Rider)],
    'dq_replay_record_gather_nhwc': [_P, _P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                     ctypes.POINTER(Rider)],
    'dq_c51_loss': [_P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _F, _P, _P, _P, _P, _P],
    'dq_dqn_huber_loss': [_P, _P, _P, _P, _P, _I32, _I32, _F, _P, _P, _P, _P],
    'dq_dqn_huber_loss_fused': [_P, _P, _P, _P, _I32, _P, _P, _P, _I32, _I32, _F, _P, _P, _P, _P,
                                _P, _I32, _P, _P, _P],
    'dq_iqn_loss': [_P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _F, _F, _P, _P, _P, _P],
    'dq_adam_tf1': [_P, _P, _P, _P, _P, _I32, _I64, _F, _F, _F, _F, _P],
    'dq_adam_tf1_part': [_P, _P, _P, _P, _P, _I32, _I64, _F, _F, _F, _F, _I32, _P],
    'dq_adam_tf1_multi': [ctypes.POINTER(TensorList), _P, _I32, _F, _F, _F, _F, _P],
    'dq_rmsprop_tf1': [_P, _P, _P, _P, _P, _I64, _F, _F, _F, _F, _I32, _P],
    'dq_sync_copy': [_P, _P, _I64, _P],
    'dq_cnn_forward': [ctypes.POINTER(CnnParams), _I32, _P, ctypes.POINTER(CnnActs), _P, _P],
    'dq_cnn_forward_pair': [ctypes.POINTER(CnnParams), _P, ctypes.POINTER(CnnActs), _P,
                            ctypes.POINTER(CnnParams), _P, ctypes.POINTER(CnnActs), _P, _I32, _P],
    'dq_cnn_backward': [ctypes.POINTER(CnnParams), ctypes.POINTER(CnnParams), _I32, _P,
                        ctypes.POINTER(CnnActs), _P, ctypes.POINTER(CnnActs), _P, _P],
    'dq_cnn_backward_adam': [ctypes.POINTER(CnnParams), ctypes.POINTER(CnnParams), _I32, _P,
                             ctypes.POINTER(CnnActs), _P, ctypes.POINTER(CnnActs), _P,
                             ctypes.POINTER(AdamArgs), _P],
    'dq_cnn_backward_groups': [ctypes.POINTER(CnnParams), ctypes.POINTER(CnnParams), _I32, _P,
                               ctypes.POINTER(CnnActs), _P, ctypes.POINTER(CnnActs), _P, _I32,
                               _I32, _P],
    'dq_cnn_backward_riders': [ctypes.POINTER(CnnParams), ctypes.POINTER(CnnParams), _I32, _P,
                               ctypes.POINTER(CnnActs), _P, ctypes.POINTER(CnnActs), _P,
                               ctypes.POINTER(Rider), _I32, ctypes.POINTER(AdamArgs),
                               ctypes.POINTER(CnnNet), _I32, _I32, _I32, _P],
    'dq_cnn_forward_fused': [ctypes.POINTER(CnnParams), _P, ctypes.POINTER(CnnActs), _P,
                             ctypes.POINTER(CnnParams), _P, ctypes.POINTER(CnnActs), _P, _I32,
                             _I32, _P],
    'dq_cnn_fc2_parts_offset': [_I32],
    'dq_cnn_forward_fused_c51': [ctypes.POINTER(CnnParams), _P, ctypes.POINTER(CnnActs), _P,
                                 ctypes.POINTER(CnnParams), ctypes.POINTER(CnnActs), _P, _I32,
                                 ctypes.POINTER(C51Target), _I32, _P],
    'dq_c51_loss_online': [_P, _P, _I32, _P, _P, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _I32,
                           _P, _P],
    'dq_c51_loss_fused': [_P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _I32, _I32, _I32, _F, _P, _P,
                          _P, _P, _P, _P, _I32, _P, _P, _P],
    'dq_cnn_forward_head': [ctypes.POINTER(CnnParams), _I32, _P, ctypes.POINTER(CnnActs), _P, _P],
    'dq_cnn_forward_with_tail': [ctypes.POINTER(CnnParams), _P, ctypes.POINTER(CnnActs), _P,
                                 ctypes.POINTER(CnnParams), ctypes.POINTER(CnnActs), _P, _I32, _P],
    'dq_cnn_backward_layer': [ctypes.POINTER(CnnParams), ctypes.POINTER(CnnParams), _I32, _P,
                              ctypes.POINTER(CnnActs), _P, ctypes.POINTER(CnnActs), _P, _I32, _I32,
                              _P],
    'dq_cnn_workspace_floats': [_I32, _I32],
    'dq_cnn_forward_torso': [ctypes.POINTER(CnnParams), _I32, _P, ctypes.POINTER(CnnActs), _P, _P],
    'dq_cnn_backward_torso': [ctypes.POINTER(CnnParams), ctypes.POINTER(CnnParams), _I32, _P,
                              ctypes.POINTER(CnnActs), ctypes.POINTER(CnnActs), _P, _P],
    'dq_cnn_backward_torso_opt': [ctypes.POINTER(CnnParams), ctypes.POINTER(CnnParams), _I32, _P,
                                  ctypes.POINTER(CnnActs), ctypes.POINTER(CnnActs), _P,
                                  ctypes.POINTER(AdamArgs), _P, _P, _P],
    'dq_iqn_head_forward': [ctypes.POINTER(IqnHead), _I32, _I32, _P, _P, ctypes.POINTER(IqnActs),
                            _P, _P],
    'dq_iqn_head_backward': [ctypes.POINTER(IqnHead), ctypes.POINTER(IqnHead), _I32, _I32, _P,
                             ctypes.POINTER(IqnActs), _P, ctypes.POINTER(IqnGrads), _P, _P, _P],
    'dq_iqn_workspace_floats': [_I32, _I32, _I32, _I32],
    'dq_uniform_draw': [_P, ctypes.c_uint64, _I64, _P, _P],
    'dq_iqn_tau_cos': [_P, ctypes.c_uint64, _I32, _I32, _P, _P, _P],
    'dq_comm_unique_id': [_P],
    'dq_comm_create': [_P, _I32, _I32, _I32, ctypes.POINTER(_P)],
    'dq_comm_destroy': [_P],
    'dq_comm_allreduce_mean': [_P, _P, _I64, _P],
    'dq_comm_reduce_scatter_mean': [_P, _P, _I64, _P],
    'dq_comm_all_gather': [_P, _P, _I64, _P],
    'dq_comm_version': [],
    'dq_peer_ipc_get': [_P, ctypes.POINTER(IpcHandle)],
    'dq_peer_ipc_open': [ctypes.POINTER(IpcHandle), ctypes.POINTER(ctypes.c_void_p),
                         ctypes.POINTER(ctypes.c_void_p)],
    'dq_peer_ipc_close': [_P],
    'dq_peer_can_access': [_I32, _I32],
    'dq_cnn_backward_peer': [ctypes.POINTER(CnnParams), ctypes.POINTER(CnnParams), _I32, _P,
                             ctypes.POINTER(CnnActs), _P, ctypes.POINTER(CnnActs), _P,
                             ctypes.POINTER(Rider), _I32, ctypes.POINTER(AdamArgs),
                             ctypes.POINTER(CnnNet), ctypes.POINTER(Peer), _I32, _P],
    'dq_cnn_forward_fused_peer': [ctypes.POINTER(CnnParams), _P, ctypes.POINTER(CnnActs), _P,
                                  ctypes.POINTER(CnnParams), _P, ctypes.POINTER(CnnActs), _P,
                                  _I32, _I32, ctypes.POINTER(Peer), _P, _P],
    'dq_peer_all_gather': [ctypes.POINTER(Peer), _P, _P],
    'dq_peer_selftest': [ctypes.POINTER(Peer), ctypes.c_uint32, _P, _P],
}
RESTYPES = {'dq_last_error': ctypes.c_char_p, 'dq_build_flags': ctypes.c_char_p, 'dq_cnn_workspace_floats': ctypes.c_size_t,
            'dq_iqn_workspace_floats': ctypes.c_size_t,
            'dq_cnn_fc2_parts_offset': ctypes.c_size_t}


class DQError(RuntimeError):
  pass


def _load():
  if not os.path.exists(LIB_PATH):
    raise ImportError(
        'dopamine_amd: HIP library %s not built (run __graft_entry__.build() or '
        'python -m dopamine_amd._build). There is no CPU fallback.' % LIB_PATH)
  lib = ctypes.CDLL(LIB_PATH)
  for name, args in SIGNATURES.items():
    fn = getattr(lib, name)
    fn.argtypes = args
    fn.restype = RESTYPES.get(name, ctypes.c_int)
  if lib.dq_abi_version() != ABI_VERSION:
    raise ImportError('dopamine_amd ABI mismatch: lib %d, python %d' % (lib.dq_abi_version(), ABI_VERSION))
  flags = lib.dq_build_flags().decode()
  # the product library carries no extra flags; the bf16 throughput build (bench.py's
  # separate row) its own; anything else (a timing or stamp build) only when asked for
  allowed = {_build.flags_string(_build.PRODUCT_FLAGS): os.path.realpath(_build.PRODUCT_LIB_PATH),
             _build.flags_string(_build.BF16_FLAGS): os.path.realpath(_build.BF16_LIB_PATH)}
  if (allowed.get(flags) != os.path.realpath(LIB_PATH)
      and os.environ.get('DQ_DIAGNOSTIC_BUILD') != '1'):
    raise ImportError('dopamine_amd: %s was built with flags %r, not a product or bf16 '
                      'throughput build (set DQ_DIAGNOSTIC_BUILD=1 for a diagnostic run)'
                      % (LIB_PATH, flags))
  return lib, flags


lib, BUILD_FLAGS = _load()


def check(rc, what=''):
  if rc != OK:
    raise DQError('%s failed (%d): %s' % (what, rc, lib.dq_last_error().decode()))


def call(name, *args):
  check(getattr(lib, name)(*args), name)


def stream_of(device):
  """The current HIP stream of ``device`` (a torch.device or index) as a void* for the C ABI:
  torch's raw getter, without building a torch.cuda.Stream object per call (the learner loop
  calls this on its host path several times per step)."""
  import torch
  idx = device if isinstance(device, int) else device.index
  if idx is None:
    idx = torch.cuda.current_device()
  return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(idx))


def ptr(t):
  """Raw device pointer of a torch tensor (or None)."""
  return None if t is None else ctypes.c_void_p(t.data_ptr())

