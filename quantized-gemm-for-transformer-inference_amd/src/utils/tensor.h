// tensor.h -- the 2-D strided tensor the reference's operator API is written against
// (/root/reference/src/utils/tensor.cuh:44-254), re-implemented on HIP for the harnesses and the
// Tensor-level adaptor (src/ops/op_mm_quantize.cuh).
//
// Same field semantics as the reference: element (r, c) is rawp[offset + r*stride_h + c*stride_w]
// (tensor.cuh:14), contiguous construction sets stride_h = w, stride_w = 1, shallow copies share
// storage through a shared_ptr, transpose() swaps shape and strides, slice() offsets a view.
// Differences: device memory comes from hipMalloc, errors go through hipAssert (print + abort, the
// reference's cudaAssert convention, assert.cuh:10-18), and toHost()/toDevice() honour `offset`
// (the reference copies from rawp and ignores it, tensor.cuh:90/111).
#pragma once

#include <hip/hip_runtime.h>

#include <cassert>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <sstream>
#include <string>
#include <type_traits>

#define hipAssert(expr) ::qgemm_tensor::hip_assert((expr), __FILE__, __LINE__)
#define Index(t, row, col) ((((t).rawp)[(t).offset + (row) * (t).stride_h + (col) * (t).stride_w]))

namespace qgemm_tensor {

inline void hip_assert(hipError_t err, const char *file, int line) {
    if (err != hipSuccess) {
        std::fprintf(stderr, "%s:%d HIP Error %s\n", file, line, hipGetErrorString(err));
        std::abort();
    }
}

template <typename T>
struct DeviceFree {
    void operator()(T *p) const {
        if (p) (void)hipFree(p);
    }
};

template <typename T>
struct HostFree {
    void operator()(T *p) const { std::free(p); }
};

}  // namespace qgemm_tensor

template <typename T>
class Tensor {
   public:
    int32_t h = 0, w = 0;
    int32_t stride_h = 0, stride_w = 0;
    int32_t offset = 0;
    T *rawp = nullptr;
    std::shared_ptr<T> ref;
    bool on_device = false;

    Tensor() = default;

    Tensor(int32_t h_, int32_t w_, bool on_device_ = false)
        : h(h_), w(w_), stride_h(w_), stride_w(1), offset(0), on_device(on_device_) {
        const size_t bytes = sizeof(T) * (size_t)h * (size_t)w;
        if (on_device) {
            hipAssert(hipMalloc(reinterpret_cast<void **>(&rawp), bytes ? bytes : sizeof(T)));
            ref = std::shared_ptr<T>(rawp, qgemm_tensor::DeviceFree<T>());
        } else {
            rawp = static_cast<T *>(std::malloc(bytes ? bytes : sizeof(T)));
            ref = std::shared_ptr<T>(rawp, qgemm_tensor::HostFree<T>());
        }
    }

    bool contiguous() const { return stride_w == 1 && stride_h == w; }
    T *data() const { return rawp + offset; }

    Tensor<T> toHost() const {
        if (!on_device) return *this;
        assert(contiguous());
        Tensor<T> t{h, w, false};
        hipAssert(hipMemcpy(t.rawp, data(), sizeof(T) * (size_t)h * w, hipMemcpyDeviceToHost));
        return t;
    }

    Tensor<T> toDevice() const {
        if (on_device) return *this;
        assert(contiguous());
        Tensor<T> t{h, w, true};
        hipAssert(hipMemcpy(t.rawp, data(), sizeof(T) * (size_t)h * w, hipMemcpyHostToDevice));
        return t;
    }

    Tensor<T> transpose() const {
        Tensor<T> t = *this;
        t.h = w;
        t.w = h;
        t.stride_h = stride_w;
        t.stride_w = stride_h;
        return t;
    }

    Tensor<T> slice(int start_h, int end_h, int start_w, int end_w) const {
        assert(start_h < end_h && end_h <= h);
        assert(start_w < end_w && end_w <= w);
        Tensor<T> t = *this;
        t.h = end_h - start_h;
        t.w = end_w - start_w;
        t.offset = offset + start_h * stride_h + start_w * stride_w;
        return t;
    }

    // Same text layout as the reference's str() (tensor.cuh:167-199): fixed, 6 decimals,
    // space-separated, one line per row; int8 printed as integers.
    std::string str() const {
        const Tensor<T> t = on_device ? toHost() : *this;
        std::stringstream ss;
        ss.precision(6);
        ss << std::fixed;
        for (int i = 0; i < h; ++i) {
            for (int j = 0; j < w; ++j) {
                if constexpr (std::is_same_v<T, int8_t> || std::is_same_v<T, char> || std::is_same_v<T, unsigned char>)
                    ss << (int)Index(t, i, j) << " ";
                else
                    ss << Index(t, i, j) << " ";
            }
            ss << "\n";
        }
        return ss.str();
    }

    // Signed mean, summed sequentially in T and divided by h*w (tensor.cuh:201-211): the
    // reference's "Mean quantization error" metric.
    T mean() const {
        assert(!on_device);
        T sum = 0;
        for (int i = 0; i < h; ++i)
            for (int j = 0; j < w; ++j) sum += Index(*this, i, j);
        return sum / (h * w);
    }
};
