"""Builds the in-tree HIP library (gfx950).  Importing this module never loads it."""
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# DOPAMINE_AMD_LIB: an alternate in-tree build of the same library (A/B experiments)
LIB_PATH = os.environ.get('DOPAMINE_AMD_LIB') or os.path.join(_HERE, 'libdopamine_amd.so')
SOURCES = [os.path.join(_HERE, 'csrc', f) for f in ('replay.hip', 'learner.hip', 'nature_cnn.hip', 'iqn.hip', 'comm.hip')]
HEADER = os.path.join(os.path.dirname(_HERE), 'include', 'dopamine_amd.h')
ARCH = os.environ.get('DQ_OFFLOAD_ARCH', 'gfx950')


# The bf16 throughput build (BASELINE.md §4's separate row; NOT fp32 parity): the same
# sources with every Nature-CNN wave-private tile and the IQN heads' split GEMMs on ONE bf16
# product (hi.hi, fp32 accumulate) -- bench.py times it beside the fp32 headline.
BF16_LIB_PATH = os.path.join(_HERE, 'libdopamine_amd_bf16.so')
BF16_FLAGS = ['-DDQ_CNN_X6=1', '-DDQ_X6_PAIRS=1']


def build_bf16(verbose=False):
  return build(verbose=verbose, out=BF16_LIB_PATH, extra=BF16_FLAGS)


def build_all(verbose=False):
  """Both libraries (the product and the bf16 throughput build): every translation unit of
  the two compiled concurrently, then the two links."""
  jobs = [_start(verbose, LIB_PATH, None, ()), _start(verbose, BF16_LIB_PATH, None, BF16_FLAGS)]
  return [_finish(verbose, *j) for j in jobs]


def build(verbose=False, out=None, sources=None, extra=()):
  """Compile the HIP sources into libdopamine_amd.so next to this file: one hipcc per
  translation unit, in parallel, then one link."""
  return _finish(verbose, *_start(verbose, out, sources, extra))


def _start(verbose, out, sources, extra):
  out = out or LIB_PATH
  flags = ['--offload-arch=' + ARCH, '-O3', '-fPIC', '-std=c++17', '-ffp-contract=off', '-Wall',
           '-I', os.path.join(_HERE, 'csrc')] + list(extra)
  objs, procs = [], []
  bdir = os.path.join(_HERE, 'build')
  os.makedirs(bdir, exist_ok=True)
  csrc = os.path.join(_HERE, 'csrc')
  headers = [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith('.h')] + [HEADER]
  newest_h = max(os.path.getmtime(h) for h in headers)
  for src in sources or SOURCES:
    obj = os.path.join(bdir, '%s.%s.o' % (os.path.basename(out), os.path.splitext(os.path.basename(src))[0]))
    objs.append(obj)
    if (os.path.exists(obj) and os.path.exists(out) and
        os.path.getmtime(obj) >= max(os.path.getmtime(src), newest_h)):
      continue                       # object up to date (incremental rebuild)
    cmd = ['hipcc'] + flags + ['-c', '-o', obj, src]
    if verbose:
      print(' '.join(cmd))
    procs.append((subprocess.Popen(cmd), cmd))
  return out, objs, procs


def _finish(verbose, out, objs, procs):
  for p, cmd in procs:
    if p.wait() != 0:
      raise subprocess.CalledProcessError(p.returncode, cmd)
  tmp = out + '.tmp'            # linked aside, then renamed: a reader never sees half a file
  cmd = ['hipcc', '--offload-arch=' + ARCH, '-shared', '-fPIC', '-o', tmp] + objs + ['-ldl']
  if verbose:
    print(' '.join(cmd))
  subprocess.run(cmd, check=True)
  os.replace(tmp, out)
  return out


if __name__ == '__main__':
  build_all(verbose=True)
