#!/bin/bash
set -o pipefail
out=gpurun_out/power; mkdir -p $out
timeout -k 10 300 python -u scripts/power_probe.py > $out/power.log 2>&1 || { cat $out/power.log; exit 1; }
cat $out/power.log
