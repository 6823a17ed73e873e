#!/bin/bash
# round 4: ticket-first split-K (one slab, uneven K split) vs both-slab split-K, alone and inside the FFN-down call
set -o pipefail
mkdir -p gpurun_out
cd lab
timeout -k 10 150 ./build/t2_lab 2048 4096 16384 9 fms,fmf28,fmf30,fmf31,fmf32,fk > ../gpurun_out/r4_splitfirst_lab.log 2>&1 &&
timeout -k 10 150 ./build/t2_lab 2048 4096 8192 9 fms,fmf30,fmf31,fk >> ../gpurun_out/r4_splitfirst_lab.log 2>&1 &&
timeout -k 10 250 ./build/c3d_lab 2048 4096 16384 7 > ../gpurun_out/r4_splitfirst_c3d.log 2>&1
