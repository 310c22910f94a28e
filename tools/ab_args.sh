#!/bin/bash
# A/B the bench under different command-line flags, one process per setting, twice.
#   bash tools/ab_args.sh "--ride 0" "--ride 1" ...
for rep in 1 2; do
  for cfg in "$@"; do
    line=$(timeout -k 10 240 python bench.py --steps 400 --skip-cpu-baseline $cfg 2>/dev/null | tail -1)
    v=$(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_mean_loss"])' 2>/dev/null)
    echo "[$cfg] -> $v"
  done
done
