"""Build an A/B variant of the library: recompile the named translation units with extra
flags into ab/<name>/, link them with the in-tree objects of the others.
  python tools/build_variant.py <name> <tu[,tu..]> [-DFLAG ...]
e.g.  python tools/build_variant.py c51prof learner -DDQ_C51_PROF
The variant loads through DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=ab/<name>/libdopamine_amd.so.
DQ_VARIANT_ROOT=<dir> puts it under <dir>/<name> instead (e.g. variants/, which -- unlike ab/ --
travels to the GPU box with gpurun; both are git-ignored)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dopamine_amd import _build  # noqa: E402


def main():
  name, extra = sys.argv[1], sys.argv[3:]
  # "tu" recompiles the in-tree source, "tu=path" another file in its place (e.g. a git show)
  tus = dict((t.split('=') + [None])[:2] for t in sys.argv[2].split(','))
  out_dir = os.path.join(ROOT, os.environ.get('DQ_VARIANT_ROOT', 'ab'), name)
  os.makedirs(out_dir, exist_ok=True)
  bdir = os.path.join(ROOT, 'dopamine_amd', 'build')
  # the variant records what it is (dq_build_flags); replay.hip, which exports it, is always
  # recompiled, so a variant never reports the product's empty flags.  It loads only with
  # DQ_DIAGNOSTIC_BUILD=1 (dopamine_amd/_lib.py).
  tus.setdefault('replay', None)
  note = 'variant %s: %s %s' % (name, ','.join(sorted(tus)), ' '.join(extra))
  flags = ['--offload-arch=' + _build.ARCH, '-O3', '-fPIC', '-std=c++17', '-ffp-contract=off',
           '-I', os.path.join(ROOT, 'dopamine_amd', 'csrc')] + extra + [
               '-DDQ_BUILD_FLAGS="%s"' % note.replace('"', "'")]
  objs, procs = [], []
  for src in _build.SOURCES:
    tu = os.path.splitext(os.path.basename(src))[0]
    if tu in tus:
      obj = os.path.join(out_dir, tu + '.o')
      cmd = ['hipcc'] + flags + ['-c', '-o', obj, tus[tu] or src]
      procs.append(subprocess.Popen(cmd))
    else:
      obj = os.path.join(bdir, 'libdopamine_amd.so.%s.o' % tu)
      assert os.path.exists(obj), 'build the in-tree library first: ' + obj
    objs.append(obj)
  for p in procs:
    assert p.wait() == 0
  out = os.path.join(out_dir, 'libdopamine_amd.so')
  subprocess.run(['hipcc', '--offload-arch=' + _build.ARCH, '-shared', '-fPIC', '-o', out] + objs +
                 ['-ldl'], check=True)
  print(out)


if __name__ == '__main__':
  main()
