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
// GEMMs/s and int8 TOPS.  -g <ngpus>: the multi-GPU driver of SURVEY.md s8(b)/(e) -- the m rows
// sharded over ngpus devices of this node (per-rank pointer offsets A + m0*k, C + m0*n,
// op_mm_quantize_shard), then the in-place RCCL all-gather of C over xGMI (qgemm_allgather_rows),
// timed separately, checked bit for bit against the one-GPU call; a "node" JSON line.
#include <getopt.h>
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>

#include <vector>
#include <cstring>

#include "ops/op_mm_quantize.cuh"
#include "../../include/qgemm_dist.h"

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

#define DIST_CHECK(x)                                                                   \
    do {                                                                                \
        const int rc_ = (x);                                                            \
        if (rc_) {                                                                      \
            std::fprintf(stderr, "%s failed: %d (%s:%d)\n", #x, rc_, __FILE__, __LINE__); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

// -g: whole-node step.  Every device holds the full A (same seed: the replicated input of one node)
// and B, and a full-size C; device r computes its row shard, then C is all-gathered in place.
static void node_run(int m, int n, int k, int ngpus, int reps) {
    int avail = 0;
    hipAssert(hipGetDeviceCount(&avail));
    if (ngpus > avail) {
        std::fprintf(stderr, "-g %d: only %d devices visible\n", ngpus, avail);
        std::exit(2);
    }
    std::vector<int> devs(ngpus);
    std::vector<float *> A(ngpus), B(ngpus), C(ngpus);
    std::vector<hipStream_t> st(ngpus);
    std::vector<hipEvent_t> e0(ngpus), e1(ngpus), e2(ngpus);
    std::vector<void *> comms(ngpus, nullptr);
    for (int r = 0; r < ngpus; ++r) {
        devs[r] = r;
        hipAssert(hipSetDevice(r));
        hipAssert(hipMalloc(&A[r], (size_t)m * k * 4));
        hipAssert(hipMalloc(&B[r], (size_t)k * n * 4));
        hipAssert(hipMalloc(&C[r], (size_t)m * n * 4));
        hipAssert(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
        hipAssert(hipEventCreate(&e0[r]));
        hipAssert(hipEventCreate(&e1[r]));
        hipAssert(hipEventCreate(&e2[r]));
        DIST_CHECK(qgemm_fill_uniform(A[r], (int64_t)m * k, 2 * randgen_seed, -1.0f, 1.0f, st[r]));
        DIST_CHECK(qgemm_fill_uniform(B[r], (int64_t)k * n, 2 * randgen_seed + 1, -1.0f, 1.0f, st[r]));
        hipAssert(hipMemsetAsync(C[r], 0xff, (size_t)m * n * 4, st[r]));  // poisoned: NaN until written
    }
    DIST_CHECK(qgemm_comm_init_all(comms.data(), ngpus, devs.data()));
    std::vector<void *> sv(st.begin(), st.end());
    // warm-up (workspaces, RCCL channels), then reps timed steps: shard compute | all-gather
    for (int w = 0; w < 2; ++w)
        DIST_CHECK(qgemm_node_mm_quantize(A.data(), B.data(), C.data(), m, n, k, ngpus, devs.data(), comms.data(),
                                          sv.data(), 1));
    double comp_ms = 0, gath_ms = 0, step_ms = 0;
    for (int it = 0; it < reps; ++it) {
        for (int r = 0; r < ngpus; ++r) {
            hipAssert(hipSetDevice(r));
            hipAssert(hipStreamSynchronize(st[r]));
            hipAssert(hipEventRecord(e0[r], st[r]));
        }
        for (int r = 0; r < ngpus; ++r) {
            hipAssert(hipSetDevice(r));
            DIST_CHECK(op_mm_quantize_shard(A[r], B[r], C[r], m, n, k, ngpus, r, st[r]));
            hipAssert(hipEventRecord(e1[r], st[r]));
        }
        DIST_CHECK(qgemm_node_mm_quantize(A.data(), B.data(), C.data(), m, n, k, ngpus, devs.data(), comms.data(),
                                          sv.data(), 2));  // the all-gather alone
        for (int r = 0; r < ngpus; ++r) {
            hipAssert(hipSetDevice(r));
            hipAssert(hipEventRecord(e2[r], st[r]));
        }
        double cmax = 0, gmax = 0, smax = 0;
        for (int r = 0; r < ngpus; ++r) {
            hipAssert(hipSetDevice(r));
            hipAssert(hipEventSynchronize(e2[r]));
            float a = 0, b = 0;
            hipAssert(hipEventElapsedTime(&a, e0[r], e1[r]));
            hipAssert(hipEventElapsedTime(&b, e1[r], e2[r]));
            cmax = a > cmax ? a : cmax;
            gmax = b > gmax ? b : gmax;
            smax = a + b > smax ? a + b : smax;
        }
        comp_ms += cmax;
        gath_ms += gmax;
        step_ms += smax;
    }
    comp_ms /= reps;
    gath_ms /= reps;
    step_ms /= reps;
    // check: every device's gathered C == the one-GPU op_mm_quantize of the whole problem on device 0
    float *ref = nullptr;
    hipAssert(hipSetDevice(0));
    hipAssert(hipMalloc(&ref, (size_t)m * n * 4));
    DIST_CHECK(op_mm_quantize_ex(A[0], k, 1, B[0], n, 1, ref, n, 1, m, n, k, 127.0f, st[0]));
    hipAssert(hipStreamSynchronize(st[0]));
    std::vector<uint32_t> h0((size_t)m * n), h1((size_t)m * n);
    hipAssert(hipMemcpy(h0.data(), ref, h0.size() * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (int r = 0; r < ngpus; ++r) {
        hipAssert(hipSetDevice(r));
        hipAssert(hipMemcpy(h1.data(), C[r], h1.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < h0.size(); ++i) bad += h0[i] != h1[i];
    }
    const double ops = 2.0 * m * (double)n * k;
    std::printf("{\"node\": {\"gpus\": %d, \"m\": %d, \"n\": %d, \"k\": %d, \"reps\": %d, \"shard_rows\": %d, "
                "\"compute_ms\": %.6f, \"allgather_ms\": %.6f, \"step_ms\": %.6f, "
                "\"sharded_gemms_per_s\": %.2f, \"node_gemms_per_s_with_gather\": %.2f, \"node_tops\": %.1f, "
                "\"allgather_GBps_per_gpu\": %.1f, \"bit_identical_to_one_gpu\": %s, \"mismatches\": %zu}}\n",
                ngpus, m, n, k, reps, (m + ngpus - 1) / ngpus, comp_ms, gath_ms, step_ms, 1e3 / comp_ms,
                1e3 / step_ms, ops / (comp_ms * 1e9),
                ngpus > 1 ? (double)m * n * 4 * (ngpus - 1) / ngpus / (gath_ms * 1e6) : 0.0, bad ? "false" : "true",
                bad);
    hipAssert(hipFree(ref));
    for (int r = 0; r < ngpus; ++r) {
        hipAssert(hipSetDevice(r));
        DIST_CHECK(qgemm_comm_destroy(comms[r]));
        hipAssert(hipFree(A[r]));
        hipAssert(hipFree(B[r]));
        hipAssert(hipFree(C[r]));
    }
    hipAssert(hipSetDevice(0));
}

int main(int argc, char *argv[]) {
    bool test_gpu = true;
    int test_m = 2048, test_n = 2048, test_k = 2048, iters = 50, ngpus = 0;
    for (;;) {
        const int c = getopt(argc, argv, "s:cm:n:k:r:g:");
        if (c == -1) break;
        switch (c) {
            case 's': randgen_seed = std::atoll(optarg); break;
            case 'c': test_gpu = false; break;
            case 'm': test_m = std::atoi(optarg); break;
            case 'n': test_n = std::atoi(optarg); break;
            case 'k': test_k = std::atoi(optarg); break;
            case 'r': iters = std::atoi(optarg); break;
            case 'g': ngpus = std::atoi(optarg); break;
            default: break;
        }
    }
    if (!test_gpu) {
        std::cerr << "no CPU path: op_quantized_mm requires device tensors (reference op_mm.cuh:72)" << std::endl;
        return 2;
    }
    if (ngpus > 0) {  // the whole-node step only (the per-iteration reference loop is the one-GPU harness)
        node_run(test_m, test_n, test_k, ngpus, iters);
        return 0;
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
