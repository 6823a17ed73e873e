set -e
mkdir -p gpurun_out/r6epi4
timeout -k 10 240 lab/build/epi_lab 2048 16384 4096 9 prod,img_m1,row1k,row1k_m1,nostore > gpurun_out/r6epi4/c3u.log 2>&1
timeout -k 10 240 lab/build/epi_lab 2048 16384 4096 9 row1k_m1,row1k,img_m1,prod > gpurun_out/r6epi4/c3u_rev.log 2>&1
timeout -k 10 240 lab/build/epi_lab 4096 4096 4096 9 prod,ldsb0,ldsb1,ldsb2 > gpurun_out/r6epi4/c2_ldsb.log 2>&1
timeout -k 10 240 lab/build/epi_lab 8192 4096 4096 9 prod,ldsb0,ldsb1,ldsb2 > gpurun_out/r6epi4/c4_ldsb.log 2>&1
timeout -k 10 240 lab/build/epi_lab 4096 4096 4096 9 ldsb2,ldsb1,ldsb0,prod > gpurun_out/r6epi4/c2_ldsb_rev.log 2>&1
timeout -k 10 60 rocprofv3 -L > gpurun_out/r6epi4/counters.txt 2>&1 || true
