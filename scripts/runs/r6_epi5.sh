set -e
mkdir -p gpurun_out/r6epi5
timeout -k 10 240 lab/build/epi_lab 2048 16384 4096 9 prod,rot0,rot1,rot2,rot3,rot4 > gpurun_out/r6epi5/c3u.log 2>&1
timeout -k 10 240 lab/build/epi_lab 2048 16384 4096 9 rot4,rot3,rot2,rot1,rot0,prod > gpurun_out/r6epi5/c3u_rev.log 2>&1
