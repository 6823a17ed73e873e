// ln_lab.hip -- development check (not part of the library): add+layernorm with and without the fused
// pack must give identical Y; prints mismatch counts.  Build: make -C .. lnlab
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../csrc/encoder_ops.hip"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_lab(float *p, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (float)(((uint32_t)i * 2654435761u + seed) % 20011u) / 10000.0f - 1.0f;
}

int main(int argc, char **argv) {
    const int rows = argc > 1 ? atoi(argv[1]) : 512, w = argc > 2 ? atoi(argv[2]) : 1024;
    float *A, *B, *Y1, *Y2; void *pk;
    CK(hipMalloc(&A, (size_t)rows * w * 4)); CK(hipMalloc(&B, (size_t)rows * w * 4));
    CK(hipMalloc(&Y1, (size_t)rows * w * 4)); CK(hipMalloc(&Y2, (size_t)rows * w * 4));
    CK(hipMalloc(&pk, packed_bytes(rows, w)));
    fill_lab<<<512, 256>>>(A, (int64_t)rows * w, 1); fill_lab<<<512, 256>>>(B, (int64_t)rows * w, 7);
    CK(launch_add_layernorm_rows(A, B, Y1, rows, w, nullptr));
    CK(launch_add_layernorm_rows_pack(A, B, Y2, rows, w, 127.0f, packed_view(pk, rows, w), nullptr));
    CK(hipDeviceSynchronize());
    std::vector<float> h1((size_t)rows * w), h2((size_t)rows * w);
    CK(hipMemcpy(h1.data(), Y1, h1.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), Y2, h2.size() * 4, hipMemcpyDeviceToHost));
    size_t bad = 0; int first = -1;
    for (size_t i = 0; i < h1.size(); ++i) if (memcmp(&h1[i], &h2[i], 4)) { if (first < 0) first = (int)i; ++bad; }
    printf("rows %d w %d: Y(pack) vs Y(plain) mismatches %zu (first at row %d)\n", rows, w, bad, first < 0 ? -1 : first / w);
    return 0;
}
