#!/bin/bash
# round 6: workgroup tile shapes (lab/make_tile_fm.py) at FFN up, the C4 shard and C2 -- bit-checked against the product
# kernel, GEMM alone and whole call, interleaved rounds (lab/epi_lab.hip)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/tile; mkdir -p $out
timeout -k 10 240 lab/build/epi_lab 2048 16384 4096 5 prod,t256_g8_img,t128x512_g4_img,t128x512_g8_img,t128x512_g16_img,t128x512_g4_pairs,t128x512_g8_pairs,t128x512_g16_pairs,t512x128_g4_pairs > $out/ffn_up.log 2>&1 || { tail $out/ffn_up.log; exit 1; }
timeout -k 10 240 lab/build/epi_lab 8192 4096 4096 5 prod,t256_g4_pairs,t128x512_g4_pairs,t128x512_g8_pairs,t512x128_g2_pairs,t512x128_g4_pairs > $out/c4_shard.log 2>&1 || { tail $out/c4_shard.log; exit 1; }
timeout -k 10 240 lab/build/epi_lab 4096 4096 4096 5 prod,t128x512_g4_pairs,t128x512_g8_pairs,t512x128_g4_pairs > $out/c2.log 2>&1 || { tail $out/c2.log; exit 1; }
grep -h -E "mismatches [1-9]|median" $out/*.log
grep -h -c "mismatches 0" $out/*.log
