#!/usr/bin/env python3
"""One line per bench.py log: config, value, ms per step, GEMM-kernel ms (in-region events), roofline frac."""
import json
import sys

for path in sys.argv[1:]:
    lines = [l for l in open(path) if l.startswith('{')]
    if not lines:
        print(f"{path}: no JSON line")
        continue
    d = json.loads(lines[-1])
    r = d.get('roofline', {})
    print(f"{path}: value {d['value']} {d['unit']}  ms/step {d['ms_per_step']}  gemm_ms {d.get('gemm_kernel_ms')}  "
          f"frac {r.get('frac')}")
