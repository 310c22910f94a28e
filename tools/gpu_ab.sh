# A/B of alternate builds on one box (tools/build_variant.py ab/<name>/libdopamine_amd.so):
# chosen GPU tests on each build, then the bench (or CFG=iqn_breakout|dqn_pong through
# tools/bench_configs.py) alternating in-tree / builds twice, then (DQ_TIMELINE=1) a rocprof
# step timeline of each (DQ_NOAB=1: the timelines only).
#   gpurun -- 'DQ_TESTS="tests/test_gpu_cnn.py ..." CFG=rainbow DQ_TIMELINE=1 \
#     bash tools/gpu_ab.sh <out-name> ab/X/libdopamine_amd.so "args:--split-c51 1" ...'
# (the environment is set inside the gpurun command: gpurun does not forward it).  "args:"
# flags are tools/bench_ab.py's schedule experiments; variant builds load with
# DQ_DIAGNOSTIC_BUILD=1 (their recorded flags are not the product's).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab}
shift
mkdir -p $OUT
if [ -n "$DQ_TESTS" ]; then
  # DQ_TESTS_INTREE=1: the in-tree build's run first
  for spec in $([ -n "$DQ_TESTS_INTREE" ] && echo dopamine_amd/libdopamine_amd.so) "$@"; do
    # the build a spec runs on: "args:<flags>" the in-tree one, "<lib>|<flags>" that lib
    lib=$spec
    case "$spec" in args:*) continue;; *"|"*) lib=${spec%%|*};; esac
    n=$(basename $(dirname $lib))
    DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=$lib timeout -k 10 600 python -u -m pytest $DQ_TESTS -m gpu -v \
      --timeout 300 --timeout-method thread > $OUT/tests_$n.log 2>&1
    rc=$?; echo "[$n] tests rc=$rc"; tail -1 $OUT/tests_$n.log; grep FAILED $OUT/tests_$n.log | head
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
fi
for rep in $([ -z "$DQ_NOAB" ] && echo 1 2); do
  for spec in "" "$@"; do
    # a build (ab/X/libdopamine_amd.so), "args:<bench flags>" on the in-tree build, or
    # "ab/X/libdopamine_amd.so|<bench flags>"
    lib=$spec; extra=
    case "$spec" in args:*) lib=; extra=${spec#args:};; *"|"*) lib=${spec%%|*}; extra=${spec#*|};; esac
    if [ "${CFG:-rainbow}" = rainbow ]; then
      line=$(DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=$lib timeout -k 10 240 python tools/bench_ab.py $extra -- --steps ${STEPS:-2000} --skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20 2>>$OUT/err.log | tail -1) || exit 1
      v=$(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')
    else
      v=$(DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=$lib timeout -k 10 240 python tools/bench_configs.py ${STEPS:-300} $CFG $extra 2>>$OUT/err.log | tail -1) || exit 1
    fi
    echo "[${spec:-in-tree}] $v" | tee -a $OUT/ab.log
  done
done
if [ -n "$DQ_TIMELINE" ]; then
  i=0
  for spec in "" "$@"; do
    i=$((i + 1))
    lib=$spec; extra=
    case "$spec" in args:*) lib=; extra=${spec#args:};; *"|"*) lib=${spec%%|*}; extra=${spec#*|};; esac
    n=t$i
    DQ_DIAGNOSTIC_BUILD=1 DOPAMINE_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r_$n -o run -- python3 tools/bench_ab.py $extra -- --skip-cpu-baseline --skip-bf16 --skip-configs --gather-iters 20 > $OUT/prof_$n.log 2>&1 || exit 1
    echo "== [$n] ${spec:-in-tree}" >> $OUT/timelines.txt
    python3 tools/step_timeline_db.py /tmp/r_$n/run_results.db k_c51 30 > $OUT/timeline_$n.txt
    cat $OUT/timeline_$n.txt >> $OUT/timelines.txt
    python3 tools/prof_summary.py /tmp/r_$n/run_results.db 30 > $OUT/kernels_$n.txt
    echo "[$n] ${spec:-in-tree}"; head -2 $OUT/timeline_$n.txt
  done
fi
