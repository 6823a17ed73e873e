#!/bin/bash
# the whole -m gpu suite, then a same-box A/B with kernel traces (scripts/runs/r6_ab_prof.sh; CFGS, SIDES, TAG)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6abp${TAG:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r6abp${TAG:-}/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6abp${TAG:-}/pytest.log
case $rc in 0) ;; *) exit $rc;; esac
bash scripts/runs/r6_ab_prof.sh
