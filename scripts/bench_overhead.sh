set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
B=quantized-gemm-for-transformer-inference_amd/build
timeout -k 10 120 $B/timing_quantize -m 4096 -n 4096 -k 4096 -r 1 > gpurun_out/ovh_timing.log 2>&1 || exit $?
tail -1 gpurun_out/ovh_timing.log
timeout -k 10 120 $B/chain2_lab 10 > gpurun_out/ovh_chain.log 2>&1 || exit $?
tail -2 gpurun_out/ovh_chain.log
for t in none ext; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 --gemm-timing $t > gpurun_out/ovh_bench_$t.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ovh_bench_$t.log').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'], d.get('gemm_kernel_ms'))"
done
