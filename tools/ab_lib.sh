#!/bin/bash
# A/B the bench between the in-tree library and alternate builds (same box, one
# process per run, alternating):   bash tools/ab_lib.sh ab/A/libdopamine_amd.so ...
for rep in 1 2; do
  for lib in "" "$@"; do
    line=$(DOPAMINE_AMD_LIB=$lib timeout -k 10 240 python bench.py --steps 400 --skip-cpu-baseline 2>/dev/null | tail -1)
    v=$(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], "gather_us=%s frac=%s b1024=%s" % (r["avg_launch_us"], r["frac"], r["same_kernel_batch_1024"]))' 2>/dev/null)
    echo "[${lib:-in-tree}] -> $v"
  done
done
