#!/bin/bash
# round-5 first GPU call: is the shipped build/ up to date for make on the box (mtimes), the GPU suite, smoke,
# the default bench line (launcher/hash changes), FFN-down kSync A/B (lab/c3d_lab.hip), bench c3_down
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5first; mkdir -p $out
echo "make would run $(make -n -C quantized-gemm-for-transformer-inference_amd all 2>/dev/null | grep -c hipcc) hipcc lines" | tee $out/make_dry.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_c2.log 2>&1 || { tail $out/bench_c2.log; exit 1; }
grep -o '"value": [0-9.]*' $out/bench_c2.log | head -1
timeout -k 10 300 lab/build/c3d_lab 2048 4096 16384 9 sync > $out/c3d_sync.log 2>&1 || { tail $out/c3d_sync.log; exit 1; }
cat $out/c3d_sync.log
timeout -k 10 300 python bench.py --config c3_down --no-cpu-baseline > $out/bench_c3_down.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $out/bench_c3_down.log | head -1
echo done
