// attn_lab.hip -- development harness (not part of the library): times the fused attention kernel and
// its phase ablations (kSkip) at the encoder's config-5 shape.  Build: make -C .. attnlab
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/attention.hip"

using namespace qgemm;

__global__ void fill_lab(float *p, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (float)((i * 2654435761u) % 2001u) / 1000.0f - 1.0f;
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
    const int seq = argc > 1 ? atoi(argv[1]) : 512, d = argc > 2 ? atoi(argv[2]) : 1024, H = argc > 3 ? atoi(argv[3]) : 16;
    const int dk = d / H;
    float *qkv, *heads;
    CK(hipMalloc(&qkv, (size_t)seq * 3 * d * 4)); CK(hipMalloc(&heads, (size_t)seq * d * 4));
    fill_lab<<<1024, 256>>>(qkv, (int64_t)seq * 3 * d);
    const float scale = 1.0f / 8.0f;
    typedef void (*K)(const float *, int, int, int, float, float *);
    struct V { const char *name; K k; int tq, threads; };
    std::vector<V> vs = {{"t32 full", attention_fused_kernel<32, 256, 1024, 0>, 32, 1024},
                         {"t32 no_qk", attention_fused_kernel<32, 256, 1024, 1>, 32, 1024},
                         {"t32 no_softmax", attention_fused_kernel<32, 256, 1024, 2 | 8>, 32, 1024},
                         {"t32 no_sums", attention_fused_kernel<32, 256, 1024, 8>, 32, 1024},
                         {"t32 no_pv", attention_fused_kernel<32, 256, 1024, 4>, 32, 1024},
                         {"t32 nothing", attention_fused_kernel<32, 256, 1024, 15>, 32, 1024}};
    hipEvent_t a, z; CK(hipEventCreate(&a)); CK(hipEventCreate(&z));
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < 7; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            const dim3 g((seq + vs[i].tq - 1) / vs[i].tq, H);
            for (int w = 0; w < 3; ++w) vs[i].k<<<g, vs[i].threads>>>(qkv, d, dk, seq, scale, heads);
            CK(hipEventRecord(a));
            for (int w = 0; w < 20; ++w) vs[i].k<<<g, vs[i].threads>>>(qkv, d, dk, seq, scale, heads);
            CK(hipEventRecord(z)); CK(hipEventSynchronize(z));
            float ms; CK(hipEventElapsedTime(&ms, a, z)); t[i].push_back(ms * 1000 / 20);
        }
    for (size_t i = 0; i < vs.size(); ++i) {
        auto v = t[i]; std::sort(v.begin(), v.end());
        printf("%-16s median %8.2f us\n", vs[i].name, v[v.size() / 2]);
    }
    const dim3 g((seq + 31) / 32, H);
    // phase stamps (block-median durations, 100 MHz ticks): Q loads + K chunk 0 staged | QK | softmax |
    // V chunk 0 staged | PV
    for (int w = 0; w < 5; ++w) attention_fused_kernel<32, 256, 1024, 16><<<g, 1024>>>(qkv, d, dk, seq, scale, heads);
    CK(hipDeviceSynchronize());
    const int nb = g.x * g.y;
    std::vector<unsigned long long> st((size_t)4096 * 8);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_attn_stamp), st.size() * 8));
    const char *nm[5] = {"stage K0 + Q", "QK", "softmax", "stage V0", "PV"};
    for (int ph = 0; ph < 5; ++ph) {
        std::vector<double> v;
        for (int b = 0; b < nb; ++b) v.push_back((st[(size_t)b * 8 + ph + 1] - st[(size_t)b * 8 + ph]) * 0.01);
        std::sort(v.begin(), v.end());
        printf("  %-14s median %6.2f us  max %6.2f us\n", nm[ph], v[v.size() / 2], v.back());
    }
    const int sub[4][2] = {{2, 6}, {6, 7}, {7, 3}, {0, 0}};
    const char *snm[3] = {"  max+exp", "  sums", "  div+sync"};
    for (int q = 0; q < 3; ++q) {
        std::vector<double> v;
        for (int b = 0; b < nb; ++b) v.push_back((st[(size_t)b * 8 + sub[q][1]] - st[(size_t)b * 8 + sub[q][0]]) * 0.01);
        std::sort(v.begin(), v.end());
        printf("  %-14s median %6.2f us  max %6.2f us  (wave 0)\n", snm[q], v[v.size() / 2], v.back());
    }
    std::vector<double> tot;
    for (int b = 0; b < nb; ++b) tot.push_back((st[(size_t)b * 8 + 5] - st[(size_t)b * 8]) * 0.01);
    std::sort(tot.begin(), tot.end());
    printf("  block total median %6.2f us  max %6.2f us\n", tot[tot.size() / 2], tot.back());
    return 0;
}
