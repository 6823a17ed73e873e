#!/bin/bash
# FFN-down GEMM: its time after different predecessors (lab/c3g_lab.hip); the FFN-down call with non-temporal
# pass-2 loads (lab/c3d_lab.hip); the FFN-up call with non-temporal W loads (lab/up_lab.hip)
set -o pipefail
mkdir -p gpurun_out/r4c3g
timeout -k 10 150 lab/build/c3g_lab 3 > gpurun_out/r4c3g/c3g_lab.log 2>&1 &&
timeout -k 10 150 lab/build/c3d_lab 2048 4096 16384 7 > gpurun_out/r4c3g/c3d_nt.log 2>&1 &&
timeout -k 10 150 lab/build/up_lab 2048 16384 4096 7 > gpurun_out/r4c3g/up_nt.log 2>&1
