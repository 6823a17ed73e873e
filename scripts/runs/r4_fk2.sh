#!/bin/bash
# FFN-down call with the non-temporal pass 2: split-K inside the CU (gemm_i8_fk) vs the product's ticket-first split
set -o pipefail
mkdir -p gpurun_out/r4fk2
timeout -k 10 200 lab/build/c3d_lab 2048 4096 16384 9 > gpurun_out/r4fk2/c3d.log 2>&1
