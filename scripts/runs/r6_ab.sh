#!/bin/bash
# same-box A/B of trees: each side is label:dir (a copy of another commit or variant built in place under _ab/, or
# "." for this tree); every config's bench line alternated over the sides three times
#   CFGS="c2 c3_up" SIDES="old:_ab/old new:." TAG=x bash scripts/runs/r6_ab.sh
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6ab${TAG:-}; mkdir -p $out
cfgs=${CFGS:-"c2 c2_outlier c3_up c3_down c4_shard"}
sides=${SIDES:-"old:_ab/old new:."}
for rep in 1 2 3; do
  for c in $cfgs; do
    for sd in $sides; do
      label=${sd%%:*}; dir=${sd#*:}
      timeout -k 10 200 python $dir/bench.py --config $c --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/${c}_${label}_$rep.log 2>&1 || { tail $out/${c}_${label}_$rep.log; exit 1; }
      echo "$rep $c $label $(grep -o '"value": [0-9.]*' $out/${c}_${label}_$rep.log | head -1) $(grep -o '"gemm_kernel_ms": [0-9.e-]*' $out/${c}_${label}_$rep.log | head -1)"
    done
  done
done
echo done
