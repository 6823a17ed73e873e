#!/bin/bash
# round 4: in-CU split-K (gemm_i8_fk) vs the product's cross-CU split-K (gemm_i8_fm<split>), and the FFN-down
# call with the pack sweep orders as variables (lab/c3d_lab.hip)
set -o pipefail
mkdir -p gpurun_out
cd lab
timeout -k 10 150 ./build/t2_lab 2048 4096 16384 9 fm,fms,fk > ../gpurun_out/r4_fk_lab.log 2>&1 &&
timeout -k 10 150 ./build/t2_lab 2048 4096 4096 9 fm,fms,fk >> ../gpurun_out/r4_fk_lab.log 2>&1 &&
timeout -k 10 150 ./build/t2_lab 2048 4096 8192 9 fm,fms,fk >> ../gpurun_out/r4_fk_lab.log 2>&1 &&
timeout -k 10 200 ./build/c3d_lab 2048 4096 16384 7 > ../gpurun_out/r4_c3d_lab.log 2>&1
