set -e
mkdir -p gpurun_out/r6epi
V=prod,pairs,nostore,pairs_plain,pairs_sc1,pairs_ntsc1,pairs_sc0sc1,pairs_ntsc0sc1,quad,oct,img_m1,img_m2,img_m3,pairs_m1,pairs_m2,quad_m2,oct_m2,nostore_m2
timeout -k 10 240 lab/build/epi_lab 2048 16384 4096 7 $V > gpurun_out/r6epi/c3u.log 2>&1
timeout -k 10 240 lab/build/epi_lab 8192 4096 4096 7 $V > gpurun_out/r6epi/c4.log 2>&1
timeout -k 10 240 lab/build/epi_lab 4096 4096 4096 7 prod,nostore,pairs_plain,quad,oct,pairs_m2,quad_m2,oct_m2 > gpurun_out/r6epi/c2.log 2>&1
