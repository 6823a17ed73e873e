#!/bin/bash
# round 4: two-team GEMM lab (lab/gemm_t2.h) vs the product gemm_i8_fm -- bit check, interleaved timing, stamps
set -o pipefail
mkdir -p gpurun_out
cd lab
timeout -k 10 150 ./build/t2_lab 4096 4096 4096 7 fm,t2,t2plain,t2np,t2late,t2s:8,t2s:16,t2s:24,t2s:32,t2p:8,t2p:16,t2p:32,t2ns,t2nl > ../gpurun_out/r4_t2_lab.log 2>&1 &&
timeout -k 10 150 ./build/t2_lab 8192 4096 4096 5 fm,t2,t2s:16,t2p:16 >> ../gpurun_out/r4_t2_lab.log 2>&1 &&
timeout -k 10 200 ./build/t2_lab 4096 4096 4096 1 t2,t2s:16,t2s:32,t2p:16,t2ns,t2nl clock > ../gpurun_out/r4_t2_clock.log 2>&1
