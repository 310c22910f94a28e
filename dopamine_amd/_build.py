"""Builds the in-tree HIP library (gfx950).  Importing this module never loads it."""
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# DOPAMINE_AMD_LIB: an alternate in-tree build of the same library (A/B experiments)
LIB_PATH = os.environ.get('DOPAMINE_AMD_LIB') or os.path.join(_HERE, 'libdopamine_amd.so')
SOURCES = [os.path.join(_HERE, 'csrc', f) for f in ('replay.hip', 'learner.hip', 'nature_cnn.hip')]
HEADER = os.path.join(os.path.dirname(_HERE), 'include', 'dopamine_amd.h')
ARCH = os.environ.get('DQ_OFFLOAD_ARCH', 'gfx950')


def build(verbose=False, out=None, sources=None):
  """Compile the HIP sources into libdopamine_amd.so next to this file."""
  out = out or LIB_PATH
  cmd = ['hipcc', '--offload-arch=' + ARCH, '-O3', '-fPIC', '-shared', '-std=c++17',
         '-ffp-contract=off', '-Wall', '-I', os.path.join(_HERE, 'csrc'), '-o', out] + (sources or SOURCES)
  if verbose:
    print(' '.join(cmd))
  subprocess.run(cmd, check=True)
  return out


if __name__ == '__main__':
  build(verbose=True)
