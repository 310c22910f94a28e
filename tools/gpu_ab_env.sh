# A/B of an environment knob on the bench line:  AB_VAR=NAME AB_VALUES="0 1" bash tools/gpu_ab_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_${AB_VAR}
mkdir -p $OUT
for rep in 1 2; do
  for v in $AB_VALUES; do
    env $AB_VAR=$v timeout -k 10 200 python -u bench.py --skip-cpu-baseline --steps 800 --gather-iters 20 ${AB_ARGS:-} > $OUT/$v.$rep.log 2>&1 || exit $?
    echo "$AB_VAR=$v $(python -c "import json,sys; d=json.loads(open('$OUT/$v.$rep.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
