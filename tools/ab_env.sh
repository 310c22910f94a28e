#!/bin/bash
# A/B the bench under HIP runtime environment settings, one process per setting.
#   bash tools/ab_env.sh "A=1 B=2" "C=3" ...
for cfg in "$@"; do
  line=$(env $cfg timeout -k 10 240 python bench.py --steps 400 --skip-cpu-baseline 2>/dev/null | tail -1)
  v=$(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)
  echo "[$cfg] -> $v"
done
