"""CPU-side checks of the drop-in boundary: the HIP library loads, exports every
symbol include/dopamine_amd.h declares, and the ctypes structs match the C ABI."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'dopamine_amd.h')


def _declared():
  src = open(HEADER).read()
  return sorted(set(re.findall(r'^\s*(?:int|size_t|const char\*)\s+(dq_\w+)\(', src, re.M)))


def test_library_exports_every_declared_symbol():
  from dopamine_amd import _lib
  names = _declared()
  assert len(names) >= 18
  for n in names:
    assert hasattr(_lib.lib, n), n
    assert n in _lib.SIGNATURES, 'no ctypes signature for %s' % n
  assert set(_lib.SIGNATURES) == set(names)
  assert _lib.lib.dq_abi_version() == _lib.ABI_VERSION


def test_struct_layouts_match_c():
  from dopamine_amd import _lib
  prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "dopamine_amd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(dq_replay_meta),
         sizeof(dq_replay_config), sizeof(dq_replay_storage), offsetof(dq_replay_meta, status),
         offsetof(dq_replay_config, gamma), offsetof(dq_replay_storage, discount),
         sizeof(dq_adam_args), offsetof(dq_adam_args, epsilon), sizeof(dq_iqn_head),
         offsetof(dq_iqn_head, fc2_b), sizeof(dq_iqn_acts), sizeof(dq_iqn_grads),
         sizeof(dq_cnn_params), offsetof(dq_adam_args, mg), offsetof(dq_adam_args, momentum));
  return 0;
}
'''
  with tempfile.TemporaryDirectory() as d:
    c = os.path.join(d, 'sz.c')
    open(c, 'w').write(prog)
    exe = os.path.join(d, 'sz')
    subprocess.run(['gcc', '-I', os.path.join(ROOT, 'include'), '-o', exe, c], check=True)
    got = [int(x) for x in subprocess.check_output([exe]).split()]
  exp = [ctypes.sizeof(_lib.Meta), ctypes.sizeof(_lib.Config), ctypes.sizeof(_lib.Storage),
         _lib.Meta.status.offset, _lib.Config.gamma.offset, _lib.Storage.discount.offset,
         ctypes.sizeof(_lib.AdamArgs), _lib.AdamArgs.epsilon.offset, ctypes.sizeof(_lib.IqnHead),
         _lib.IqnHead.fc2_b.offset, ctypes.sizeof(_lib.IqnActs), ctypes.sizeof(_lib.IqnGrads),
         ctypes.sizeof(_lib.CnnParams), _lib.AdamArgs.mg.offset, _lib.AdamArgs.momentum.offset]
  assert got == exp


def test_host_side_argument_errors_without_gpu():
  """Argument validation happens on the host and never touches the device."""
  from dopamine_amd import _lib
  cfg = _lib.Config(capacity=3, obs_bytes=4, stack_size=4, update_horizon=1)
  st = _lib.Storage()
  h = ctypes.c_void_p()
  rc = _lib.lib.dq_replay_create(ctypes.byref(cfg), ctypes.byref(st), ctypes.byref(h))
  assert rc == -1
  assert b'not enough capacity' in _lib.lib.dq_last_error()
  assert _lib.lib.dq_sumtree_depth(1_000_000) == 20
  assert [_lib.lib.dq_sumtree_depth(c) for c in (1, 2, 3, 4, 5, 1025)] == [0, 1, 2, 2, 3, 11]


def test_sumtree_depth_matches_reference_formula():
  import math
  import numpy as np
  from dopamine_amd import _lib
  for c in [1, 2, 3, 7, 8, 9, 100, 1000, 4096, 4097, 50000, 1_000_000]:
    assert _lib.lib.dq_sumtree_depth(c) == int(math.ceil(np.log2(c)))


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
  import importlib
  import dopamine_amd._build as b
  monkeypatch.setattr(b, 'LIB_PATH', str(tmp_path / 'nope.so'))
  import dopamine_amd._lib as L
  with pytest.raises(ImportError, match='no CPU fallback'):
    importlib.reload(L)
  monkeypatch.undo()
  importlib.reload(L)


def test_learner_rccl_is_a_separate_instance_of_the_header_version():
  """RcclComm's RCCL (dlopened by path in comm.hip) is a second instance beside the one torch
  links, so its parameters (NCCL_LAUNCH_ORDER_IMPLICIT, parallel.RcclComm) are its own
  cache; and its version is the rccl.h comm.hip compiles against (major.minor)."""
  code = r'''
import torch, re
from dopamine_amd import _lib
v = int(_lib.lib.dq_comm_version())
hdr = open('/opt/rocm/include/rccl/rccl.h').read()
code = int(re.search(r'#define NCCL_VERSION_CODE (\d+)', hdr).group(1))
assert v // 100 == code // 100, (v, code)
maps = set(l.split()[-1] for l in open('/proc/self/maps') if 'librccl' in l)
assert len(maps) == 2, maps
print('ok')
'''
  if not os.path.exists('/opt/rocm/include/rccl/rccl.h'):
    pytest.skip('no rccl.h')
  out = subprocess.run(['python', '-c', code], cwd=ROOT, capture_output=True, text=True)
  assert out.returncode == 0 and out.stdout.strip().endswith('ok'), out.stderr[-2000:]


def test_loaded_library_is_the_product_build():
  """The library the package loads records the flags it was built with (dq_build_flags): the
  product build has none (no experiment or ablation build may pass as it)."""
  from dopamine_amd import _build, _lib
  if os.environ.get('DOPAMINE_AMD_LIB'):
    pytest.skip('an alternate build was asked for')
  assert os.path.realpath(_lib.LIB_PATH) == os.path.realpath(_build.PRODUCT_LIB_PATH)
  assert _lib.BUILD_FLAGS == '' == _build.flags_string(_build.PRODUCT_FLAGS)
  assert _lib.lib.dq_build_flags().decode() == ''


def _load_in_child(env_lib, diagnostic=False):
  env = dict(os.environ, DOPAMINE_AMD_LIB=env_lib)
  env.pop('DQ_DIAGNOSTIC_BUILD', None)
  if diagnostic:
    env['DQ_DIAGNOSTIC_BUILD'] = '1'
  code = 'from dopamine_amd import _lib; print(repr(_lib.BUILD_FLAGS))'
  return subprocess.run(['python', '-c', code], cwd=ROOT, env=env, capture_output=True, text=True)


def test_non_product_builds_are_refused():
  """A library whose recorded flags do not belong to its path (here the bf16 build under
  another name) loads only with DQ_DIAGNOSTIC_BUILD=1; a library outside the tree never."""
  import shutil
  from dopamine_amd import _build
  if not os.path.exists(_build.BF16_LIB_PATH):
    pytest.skip('bf16 build absent')
  ok = _load_in_child(_build.BF16_LIB_PATH)
  assert ok.returncode == 0 and ok.stdout.strip() == repr(' '.join(_build.BF16_FLAGS)), ok.stderr[-800:]
  d = os.path.join(ROOT, 'dopamine_amd', 'build')
  os.makedirs(d, exist_ok=True)
  copy = os.path.join(d, 'test_copy_of_bf16.so')
  shutil.copyfile(_build.BF16_LIB_PATH, copy)
  try:
    bad = _load_in_child(copy)
    assert bad.returncode != 0 and 'not a product or bf16 throughput build' in bad.stderr
    diag = _load_in_child(copy, diagnostic=True)
    assert diag.returncode == 0, diag.stderr[-800:]
  finally:
    os.remove(copy)
  with tempfile.TemporaryDirectory() as t:
    out = os.path.join(t, 'libdopamine_amd.so')
    shutil.copyfile(_build.PRODUCT_LIB_PATH, out)
    far = _load_in_child(out, diagnostic=True)
    assert far.returncode != 0 and 'only in-tree builds' in far.stderr


def test_product_sources_carry_only_the_bf16_build_switches():
  """the rejected A/B knobs and the result-dropping ablations are gone from
  the product sources; the compile-time switches left are the bf16 throughput build's two
  (dopamine_amd/_build.py BF16_FLAGS).  #ifdef DQ_C51_PROF / DQ_GATHER_PROF are stamp
  builds, as DQ_GROUP_PROF (they write timing words to buffers of their own, never results);
  DQ_PEER_DROP_XCD_FENCE / DQ_PEER_HIDE_XCD / DQ_PEER_FAULT_REPLICA are fault injections for the peer exchange's
  checks (a variant that drops one XCD's write-back must be reported as a
  failed schedule), built only by tools/build_variant.py; _lib loads such a library only with
  DQ_DIAGNOSTIC_BUILD=1."""
  csrc = os.path.join(ROOT, 'dopamine_amd', 'csrc')
  knobs, ifdefs = set(), set()
  for f in os.listdir(csrc):
    src = open(os.path.join(csrc, f)).read()
    knobs |= set(re.findall(r'^#ifndef (DQ_\w+)', src, re.M))
    ifdefs |= set(re.findall(r'^#if(?:def)?\s+(DQ_\w+)', src, re.M))
  assert knobs == {'DQ_CNN_X6', 'DQ_X6_PAIRS'}, knobs
  assert ifdefs <= {'DQ_C51_PROF', 'DQ_GATHER_PROF', 'DQ_GROUP_PROF', 'DQ_BUILD_FLAGS',
                    'DQ_PEER_DROP_XCD_FENCE', 'DQ_PEER_HIDE_XCD', 'DQ_PEER_FAULT_REPLICA'}, ifdefs
