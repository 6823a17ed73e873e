#!/bin/bash
# 8-column single-pass calls (C4 shard, C2) with non-temporal input loads (lab/c4_lab.hip)
set -o pipefail
mkdir -p gpurun_out/r4c4nt
timeout -k 10 150 lab/build/c4_lab 8192 4096 4096 7 > gpurun_out/r4c4nt/c4.log 2>&1 &&
timeout -k 10 150 lab/build/c4_lab 4096 4096 4096 7 > gpurun_out/r4c4nt/c2.log 2>&1
