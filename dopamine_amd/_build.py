"""Builds the in-tree HIP library (gfx950).  Importing this module never loads it."""
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
PRODUCT_LIB_PATH = os.path.join(_HERE, 'libdopamine_amd.so')


def _lib_path():
  """DOPAMINE_AMD_LIB: another in-tree build of the same sources (the bf16 throughput row,
  diagnostic builds under tools/); _lib checks the build flags it records before use."""
  p = os.environ.get('DOPAMINE_AMD_LIB')
  if not p:
    return PRODUCT_LIB_PATH
  p = os.path.realpath(p)
  if os.path.commonpath([p, os.path.realpath(_ROOT)]) != os.path.realpath(_ROOT):
    raise ImportError('DOPAMINE_AMD_LIB=%s: only in-tree builds of this package load' % p)
  return p


LIB_PATH = _lib_path()
SOURCES = [os.path.join(_HERE, 'csrc', f) for f in ('replay.hip', 'learner.hip', 'nature_cnn.hip', 'iqn.hip', 'comm.hip', 'peer.hip')]
HEADER = os.path.join(os.path.dirname(_HERE), 'include', 'dopamine_amd.h')
ARCH = os.environ.get('DQ_OFFLOAD_ARCH', 'gfx950')


# The bf16 throughput build (BASELINE.md §4's separate row; NOT fp32 parity): the same
# sources with every Nature-CNN wave-private tile and the IQN heads' split GEMMs on ONE bf16
# product (hi.hi, fp32 accumulate) -- bench.py times it beside the fp32 headline.
BF16_LIB_PATH = os.path.join(_HERE, 'libdopamine_amd_bf16.so')
BF16_FLAGS = ['-DDQ_CNN_X6=1', '-DDQ_X6_PAIRS=1']
PRODUCT_FLAGS = []


def flags_string(extra):
  """What dq_build_flags() of a library built with these extra flags returns."""
  return ' '.join(extra)


def build_bf16(verbose=False):
  return build(verbose=verbose, out=BF16_LIB_PATH, extra=BF16_FLAGS)


def build_all(verbose=False):
  """The product library, then bench.py's bf16 throughput build (compiled concurrently with
  it).  The product is linked and installed first; a bf16 failure is reported, not raised
  (bench.py then reports that row as unavailable)."""
  prod = _start(verbose, PRODUCT_LIB_PATH, None, PRODUCT_FLAGS)
  bf16 = _start(verbose, BF16_LIB_PATH, None, BF16_FLAGS)
  out = [_finish(verbose, *prod)]
  try:
    out.append(_finish(verbose, *bf16))
  except (subprocess.CalledProcessError, OSError) as e:
    print('dopamine_amd: the bf16 throughput build failed (%r); the product library is built' % e)
  return out


def build(verbose=False, out=None, sources=None, extra=PRODUCT_FLAGS):
  """Compile the HIP sources into libdopamine_amd.so next to this file: one hipcc per
  translation unit, in parallel, then one link."""
  return _finish(verbose, *_start(verbose, out, sources, extra))


def _start(verbose, out, sources, extra):
  out = out or PRODUCT_LIB_PATH
  # every translation unit records the extra flags (dq_build_flags(); _lib checks them)
  flags = ['--offload-arch=' + ARCH, '-O3', '-fPIC', '-std=c++17', '-ffp-contract=off', '-Wall',
           '-I', os.path.join(_HERE, 'csrc')] + list(extra) + [
               '-DDQ_BUILD_FLAGS="%s"' % flags_string(extra)]
  objs, procs = [], []
  bdir = os.path.join(_HERE, 'build')
  os.makedirs(bdir, exist_ok=True)
  csrc = os.path.join(_HERE, 'csrc')
  headers = [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith('.h')] + [HEADER]
  newest_h = max(os.path.getmtime(h) for h in headers)
  # objects built with other flags (or before flags were recorded) are rebuilt
  stamp = os.path.join(bdir, os.path.basename(out) + '.flags')
  same_flags = os.path.exists(stamp) and open(stamp).read() == ' '.join(flags)
  for src in sources or SOURCES:
    obj = os.path.join(bdir, '%s.%s.o' % (os.path.basename(out), os.path.splitext(os.path.basename(src))[0]))
    objs.append(obj)
    if (same_flags and os.path.exists(obj) and os.path.exists(out) and
        os.path.getmtime(obj) >= max(os.path.getmtime(src), newest_h)):
      continue                       # object up to date (incremental rebuild)
    cmd = ['hipcc'] + flags + ['-c', '-o', obj, src]
    if verbose:
      print(' '.join(cmd))
    procs.append((subprocess.Popen(cmd), cmd))
  return out, objs, procs, (stamp, ' '.join(flags))


def _finish(verbose, out, objs, procs, stamp):
  for p, cmd in procs:
    if p.wait() != 0:
      raise subprocess.CalledProcessError(p.returncode, cmd)
  with open(stamp[0], 'w') as f:
    f.write(stamp[1])
  tmp = out + '.tmp'            # linked aside, then renamed: a reader never sees half a file
  cmd = ['hipcc', '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', tmp] + objs + ['-ldl']
  if verbose:
    print(' '.join(cmd))
  subprocess.run(cmd, check=True)
  os.replace(tmp, out)
  return out


if __name__ == '__main__':
  build_all(verbose=True)
