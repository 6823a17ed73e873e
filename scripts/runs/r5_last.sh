#!/bin/bash
# round 5, last check of the committed tree as the driver runs it: GPU suite, smoke, the default bench line
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5last; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 || { tail $out/bench.log; exit 1; }
grep -o '"value": [0-9.]*' $out/bench.log | head -1
echo done
