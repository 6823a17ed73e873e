#!/bin/bash
# FFN-up pack: block-count tail of the single pass (lab/up_lab.hip)
set -o pipefail
mkdir -p gpurun_out/r4up
timeout -k 10 120 lab/build/up_lab 2048 16384 4096 10 > gpurun_out/r4up/up_lab.log 2>&1
