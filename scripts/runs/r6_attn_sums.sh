#!/bin/bash
# round 6: attention softmax sums four rows per wave -- lab stamps, encoder parity tests, same-box C5 A/B against
# the tree before it (_ab/ln)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/attn_sums; mkdir -p $out
timeout -k 10 120 lab/build/attn_lab > $out/attn_lab.log 2>&1 || { tail $out/attn_lab.log; exit 1; }
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
CFGS="c5_encoder" SIDES="ln:_ab/ln new:." TAG=attn bash scripts/runs/r6_ab.sh || exit 1
cat $out/attn_lab.log | tail -20
