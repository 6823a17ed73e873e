#!/bin/bash
# round 4: XCD-pair map for the ticket-first split-K (each XCD one K half of a 4 x 8 tile patch)
set -o pipefail
mkdir -p gpurun_out
cd lab
timeout -k 10 150 ./build/t2_lab 2048 4096 16384 9 fms,fmf31,fmf31p > ../gpurun_out/r4_pairxcd_lab.log 2>&1 &&
timeout -k 10 150 ./build/t2_lab 2048 4096 4096 9 fms,fmf31,fmf31p >> ../gpurun_out/r4_pairxcd_lab.log 2>&1 &&
timeout -k 10 250 ./build/c3d_lab 2048 4096 16384 7 > ../gpurun_out/r4_pairxcd_c3d.log 2>&1
