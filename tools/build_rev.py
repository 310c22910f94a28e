"""Build the library from another git revision's HIP sources (same-box A/B against an earlier
commit): python tools/build_rev.py <rev> <name>  ->  $DQ_VARIANT_ROOT (default ab)/<name>/
libdopamine_amd.so, loading with DQ_DIAGNOSTIC_BUILD=1 (its recorded flags name the revision).
The revision's C ABI must be the current Python's (dq_abi_version is checked at load)."""
import os
import subprocess
import sys
import tarfile
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dopamine_amd import _build  # noqa: E402


def main():
  rev, name = sys.argv[1], sys.argv[2]
  out_dir = os.path.join(ROOT, os.environ.get('DQ_VARIANT_ROOT', 'ab'), name)
  os.makedirs(out_dir, exist_ok=True)
  src = tempfile.mkdtemp(prefix='dq_rev_')
  arch = subprocess.run(['git', '-C', ROOT, 'archive', rev, 'dopamine_amd/csrc', 'include'],
                        check=True, capture_output=True).stdout
  tar_path = os.path.join(src, 'src.tar')
  with open(tar_path, 'wb') as f:
    f.write(arch)
  with tarfile.open(tar_path) as t:
    t.extractall(src)
  csrc = os.path.join(src, 'dopamine_amd', 'csrc')
  flags = ['--offload-arch=' + _build.ARCH, '-O3', '-fPIC', '-std=c++17', '-ffp-contract=off',
           '-I', csrc, '-DDQ_BUILD_FLAGS="revision %s"' % rev]
  objs, procs = [], []
  for s in _build.SOURCES:
    f = os.path.join(csrc, os.path.basename(s))
    obj = os.path.join(out_dir, os.path.splitext(os.path.basename(s))[0] + '.o')
    procs.append(subprocess.Popen(['hipcc'] + flags + ['-c', '-o', obj, f]))
    objs.append(obj)
  for p in procs:
    assert p.wait() == 0
  out = os.path.join(out_dir, 'libdopamine_amd.so')
  subprocess.run(['hipcc', '--offload-arch=' + _build.ARCH, '-shared', '-fPIC', '-o', out] + objs +
                 ['-ldl'], check=True)
  print(out)


if __name__ == '__main__':
  main()
