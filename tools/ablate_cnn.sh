cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in BASE NOLOAD NOMFMA NOSTAGE NOREDUCE NOALL; do
  lib=""; [ $v != BASE ] && lib=ab/$v/libdopamine_amd.so
  DOPAMINE_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abl_$v -o run -- python3 tools/bench_hipcnn.py 100 > gpurun_out/abl_$v.log 2>&1 || exit 1
done
