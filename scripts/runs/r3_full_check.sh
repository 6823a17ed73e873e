#!/bin/bash
# full GPU suite, smoke, default bench (the driver's round-end steps)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/full; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit 1
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $out/bench.log | head -1
