// timing_quantize.cpp -- counterpart of the reference harness /root/reference/src/timing_quantize.cu
// (which does not compile upstream: unresolved merge markers at :76-80 and :115-120).
//
// Behaviour reproduced: per iteration, fresh U(-1,1) X[m,k] and W[k,n] (:17-20), the unquantized
// op_mm timed with gettimeofday + device sync (:27-35), the quantized chain timed the same way
// (:38-65), the signed mean error (:67-70), the per-iteration "t qt" line (:108) and the averages
// under "Final times" (:112-113; the reference's accumulators are uninitialised, ours start at 0).
// Default shape 2048^3 (the "upstream" side of the conflict, :77).
//
// Added: -r <iterations> (default 50, :106), and a final JSON line with an event-timed
// back-to-back measurement of op_quantized_mm (warm workspace) and of the fp32 op_mm, as
// GEMMs/s and int8 TOPS.
#include <getopt.h>
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "ops/op_mm_quantize.cuh"

unsigned long long randgen_seed = 0;  // timing_quantize.cu:9

static double now_us() {
    timeval tv;
    gettimeofday(&tv, nullptr);
    return tv.tv_sec * 1e6 + tv.tv_usec;
}

static void test_matmul(int m, int n, int k, double *times) {
    Tensor<float> X{m, k, true};
    op_uniform_init(X, -1.0f, 1.0f);
    Tensor<float> W{k, n, true};
    op_uniform_init(W, -1.0f, 1.0f);
    Tensor<float> C{m, n, true};
    Tensor<float> qC{m, n, true};

    double t0 = now_us();
    op_mm(X, W, C);
    hipAssert(hipDeviceSynchronize());
    double t = now_us() - t0;
    std::cout << "Time taken for matmul: " << std::endl << t / 1000 << std::endl;
    times[0] = t / 1000;

    const float range = 127.0f;
    t0 = now_us();
    op_quantized_mm(X, W, qC, range);
    hipAssert(hipDeviceSynchronize());
    double t2 = now_us() - t0;
    std::cout << "Time taken for quantized matmul: " << std::endl << t2 / 1000 << std::endl;
    times[1] = t2 / 1000;

    Tensor<float> c = C.toHost(), q = qC.toHost(), e{m, n, false};
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j) Index(e, i, j) = Index(c, i, j) - Index(q, i, j);
    std::cout << "Mean Quantization error: " << std::endl << e.mean() << std::endl;
}

static double event_ms(int m, int n, int k, bool quantized, int reps) {
    Tensor<float> X{m, k, true}, W{k, n, true}, O{m, n, true};
    op_uniform_init(X, -1.0f, 1.0f);
    op_uniform_init(W, -1.0f, 1.0f);
    for (int i = 0; i < 3; ++i) quantized ? op_quantized_mm(X, W, O, 127.0f) : op_mm(X, W, O);
    hipEvent_t a, b;
    hipAssert(hipEventCreate(&a));
    hipAssert(hipEventCreate(&b));
    hipAssert(hipEventRecord(a, nullptr));
    for (int i = 0; i < reps; ++i) quantized ? op_quantized_mm(X, W, O, 127.0f) : op_mm(X, W, O);
    hipAssert(hipEventRecord(b, nullptr));
    hipAssert(hipEventSynchronize(b));
    float ms = 0;
    hipAssert(hipEventElapsedTime(&ms, a, b));
    hipAssert(hipEventDestroy(a));
    hipAssert(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char *argv[]) {
    bool test_gpu = true;
    int test_m = 2048, test_n = 2048, test_k = 2048, iters = 50;
    for (;;) {
        const int c = getopt(argc, argv, "s:cm:n:k:r:");
        if (c == -1) break;
        switch (c) {
            case 's': randgen_seed = std::atoll(optarg); break;
            case 'c': test_gpu = false; break;
            case 'm': test_m = std::atoi(optarg); break;
            case 'n': test_n = std::atoi(optarg); break;
            case 'k': test_k = std::atoi(optarg); break;
            case 'r': iters = std::atoi(optarg); break;
            default: break;
        }
    }
    if (!test_gpu) {
        std::cerr << "no CPU path: op_quantized_mm requires device tensors (reference op_mm.cuh:72)" << std::endl;
        return 2;
    }
    double times[2] = {0, 0}, time = 0, qtime = 0;
    for (int i = 0; i < iters; ++i) {
        test_matmul(test_m, test_n, test_k, times);
        std::cout << times[0] << " " << times[1] << std::endl;
        time += times[0];
        qtime += times[1];
    }
    std::cout << "Final times" << std::endl;
    std::cout << time / iters << " " << qtime / iters << std::endl;

    const double ops = 2.0 * test_m * (double)test_n * test_k;
    const double fp_ms = event_ms(test_m, test_n, test_k, false, 10);
    const double q_ms = event_ms(test_m, test_n, test_k, true, 100);
    std::printf("{\"m\": %d, \"n\": %d, \"k\": %d, \"fp32_ms\": %.6f, \"quantized_ms\": %.6f, "
                "\"quantized_gemms_per_s\": %.1f, \"quantized_tops\": %.2f, \"fp32_tflops\": %.2f, "
                "\"library\": \"%s\"}\n",
                test_m, test_n, test_k, fp_ms, q_ms, 1e3 / q_ms, ops / (q_ms * 1e9), ops / (fp_ms * 1e9),
                qgemm_version());
    return 0;
}
