set -e
mkdir -p gpurun_out/r6epi2
V=prod,img_m1,img_m4,img_m5,pairs_m4,pairs_m5,oct_m1,oct_m4,oct_m5,quad_m1,quad_m4,nostore
timeout -k 10 240 lab/build/epi_lab 2048 16384 4096 9 $V > gpurun_out/r6epi2/c3u.log 2>&1
timeout -k 10 240 lab/build/epi_lab 2048 16384 4096 9 nostore,quad_m4,oct_m4,pairs_m4,img_m4,img_m1,prod > gpurun_out/r6epi2/c3u_rev.log 2>&1
