set -e
cd quantized-gemm-for-transformer-inference_amd
mkdir -p ../gpurun_out
timeout -k 10 120 build/pp_lab 4096 4096 4096 9 > ../gpurun_out/pp_c2.log 2>&1
timeout -k 10 120 build/pp_lab 8192 4096 4096 5 >> ../gpurun_out/pp_c2.log 2>&1
timeout -k 10 120 build/pp_lab 2048 16384 4096 5 >> ../gpurun_out/pp_c2.log 2>&1
timeout -k 10 60 build/pp_lab 0 0 0 0 peak >> ../gpurun_out/pp_c2.log 2>&1
cat ../gpurun_out/pp_c2.log
