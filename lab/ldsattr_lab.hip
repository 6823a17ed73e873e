// ldsattr_lab.hip -- LAB: which role of the FFN-up single pass (pack_single_pass32_kernel<204>, 2048 x 4096 X and
// 4096 x 16384 W) produces its LDS bank-conflict cycles?  Launches, 10 each, in this order (tell them apart by
// grid size in the rocprofv3 counter CSV):
//   full   : the product launch (512 W strips + 128 X row blocks of 16 rows)      grid 640 x 1024
//   wonly  : the W strips alone                                                   grid 512 x 1024
//   xonly  : the X row blocks alone (n = rows_pad, no strips)                     grid 128 x 1024
//   build/ldsattr_lab
#include <cstdio>
#include <cstdlib>

#include "../quantized-gemm-for-transformer-inference_amd/csrc/pack.hip"

using namespace qgemm;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
    const int m = 2048, n = 16384, k = 4096;
    float *X, *W; void *PX, *PW;
    CK(hipMalloc(&X, (size_t)m * k * 4)); CK(hipMalloc(&W, (size_t)k * n * 4));
    CK(hipMalloc(&PX, packed_bytes(m, k))); CK(hipMalloc(&PW, packed_bytes(n, k)));
    CK(launch_fill_uniform(X, (int64_t)m * k, 1, -1.f, 1.f, nullptr));
    CK(launch_fill_uniform(W, (int64_t)k * n, 2, -1.f, 1.f, nullptr));
    const PackedView vx = packed_view(PX, m, k), vw = packed_view(PW, n, k);
    const int nstrips = n / kW32Cols, nx = (int)(vx.rows_pad / 16);
    for (int v = 0; v < 3; ++v)
        for (int i = 0; i < 10; ++i) {
            const int g = v == 0 ? nstrips + nx : v == 1 ? nstrips : nx;
            const int ns = v == 2 ? 0 : nstrips;
            const int nn = v == 2 ? (int)vw.rows_pad : n;  // X-only: no strips and no padding strips
            pack_single_pass32_kernel<204><<<g, 1024>>>(X, k, m, k, vx.scale, vx.q, vx.rows_pad, vx.k_pad, W, n, nn,
                                                        vw.scale, vw.q, vw.rows_pad, ns, 127.f, nullptr, 0);
            CK(hipGetLastError());
        }
    CK(hipDeviceSynchronize());
    printf("ok\n");
    return 0;
}
