#!/bin/bash
# same-box A/B of trees with kernel traces: SIDES="label:dir ..." CFGS="..."; per config and side one bench line
# (3 alternations) and one rocprofv3 kernel-trace summary
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6abp${TAG:-}; mkdir -p $out
cfgs=${CFGS:-"c2_outlier"}
sides=${SIDES:-"r05:_ab/r05 new:."}
for rep in 1 2 3; do
  for c in $cfgs; do
    for sd in $sides; do
      label=${sd%%:*}; dir=${sd#*:}
      timeout -k 10 200 python $dir/bench.py --config $c --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/${c}_${label}_$rep.log 2>&1 || { tail $out/${c}_${label}_$rep.log; exit 1; }
      echo "$rep $c $label $(grep -o '"value": [0-9.]*' $out/${c}_${label}_$rep.log | head -1) $(grep -o '"gemm_kernel_ms": [0-9.e-]*' $out/${c}_${label}_$rep.log | head -1)"
    done
  done
done
for c in $cfgs; do
  for sd in $sides; do
    label=${sd%%:*}; dir=${sd#*:}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_${c}_${label} -o run --output-format csv -- python3 $dir/bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-error-stats --node-reps 0 --cold-steps 0 > $out/prof_${c}_${label}.log 2>&1 || exit $?
  done
done
echo done
