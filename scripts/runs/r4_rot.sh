#!/bin/bash
# store-row order variants of gemm_i8_fm (lab/rot_lab.hip)
set -o pipefail
mkdir -p gpurun_out/r4rot
timeout -k 10 200 lab/build/rot_lab 7 > gpurun_out/r4rot/rot.log 2>&1
