// SourceTransform on the device: system.numbers_mt partitions.
//
// The reference regenerates each 10,000-row block on the CPU
// (NumbersStream::poll_next, src/datasources/system/numbers_stream.rs:65-83:
// `(begin..=end).collect::<Vec<u64>>()`).  Here one launch writes a whole
// partition range into HBM with 16-byte stores; the scan kernels then read it
// back at HBM speed.  A splitmix64 column is the anti-closed-form control.
#include <hip/hip_runtime.h>

#include <string>

#include "fq_common.h"
#include "fq_device.h"

namespace fqk {

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__host__ __device__ inline uint64_t splitmix64(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <bool RANDOM>
__global__ void __launch_bounds__(256)
    fill_u64_vec_kernel(uint64_t *__restrict__ out, uint64_t begin, uint64_t seed, int64_t npairs) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    u64x2 *__restrict__ vp = reinterpret_cast<u64x2 *>(out);
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += T) {
        const uint64_t i0 = begin + 2 * (uint64_t)p;
        u64x2 v;
        if constexpr (RANDOM) {
            v.x = splitmix64(seed, i0);
            v.y = splitmix64(seed, i0 + 1);
        } else {
            v.x = i0;
            v.y = i0 + 1;
        }
        vp[p] = v;
    }
}

template <bool RANDOM>
__global__ void __launch_bounds__(256)
    fill_u64_scalar_kernel(uint64_t *__restrict__ out, uint64_t begin, uint64_t seed, int64_t n) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += T)
        out[i] = RANDOM ? splitmix64(seed, begin + (uint64_t)i) : begin + (uint64_t)i;
}

template <bool RANDOM>
static fq_status fill(uint64_t *d_out, uint64_t begin, uint64_t seed, uint64_t count, hipStream_t st) {
    if (count == 0) return FQ_OK;
    if (!d_out) return fqc::fail(FQ_E_INVALID, "fill: NULL output");
    if ((uintptr_t)d_out & 7u) return fqc::fail(FQ_E_INVALID, "fill: output not 8-byte aligned");
    // one workgroup per CU streams writes fastest (tools/tune_scan.py --write,
    // profiles/r01_tune_write_10gb.json: 6.0 TB/s vs 4.8 at 8 per CU)
    const int max_grid = fqc::device_cu_count();
    uint64_t head = ((uintptr_t)d_out & 15u) ? 1 : 0;
    if (head > count) head = count;
    if (head) {
        hipLaunchKernelGGL((fill_u64_scalar_kernel<RANDOM>), dim3(1), dim3(64), 0, st, d_out, begin, seed,
                           (int64_t)head);
        FQ_HIP_TRY(hipGetLastError());
    }
    const uint64_t rest = count - head;
    const int64_t npairs = (int64_t)(rest / 2);
    if (npairs > 0) {
        int64_t grid = (npairs + 255) / 256;
        if (grid > max_grid) grid = max_grid;
        hipLaunchKernelGGL((fill_u64_vec_kernel<RANDOM>), dim3((int)grid), dim3(256), 0, st, d_out + head,
                           begin + head, seed, npairs);
        FQ_HIP_TRY(hipGetLastError());
    }
    if (rest & 1) {
        const uint64_t last = head + 2 * (uint64_t)npairs;
        hipLaunchKernelGGL((fill_u64_scalar_kernel<RANDOM>), dim3(1), dim3(64), 0, st, d_out + last,
                           begin + last, seed, (int64_t)1);
        FQ_HIP_TRY(hipGetLastError());
    }
    return FQ_OK;
}

}  // namespace fqk

extern "C" {

fq_status fq_fill_numbers_u64(uint64_t *d_out, uint64_t begin, uint64_t count, void *stream) {
    return fqk::fill<false>(d_out, begin, 0, count, (hipStream_t)stream);
}

fq_status fq_fill_splitmix64(uint64_t *d_out, uint64_t seed, uint64_t first_index, uint64_t count,
                             void *stream) {
    return fqk::fill<true>(d_out, first_index, seed, count, (hipStream_t)stream);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// DataValue::to_array(size): scalar broadcast (data_value.rs:77-111)
// ---------------------------------------------------------------------------
namespace fqk {

template <typename T>
__global__ void __launch_bounds__(256) fill_value_kernel(T *__restrict__ out, int64_t n, T v) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = v;
}

template <typename T>
static fq_status fill_value(void *out, int64_t n, T v, hipStream_t st) {
    if (n <= 0) return FQ_OK;
    const int max_grid = fqc::device_cu_count() * 8;
    int64_t grid = (n + 255) / 256;
    if (grid > max_grid) grid = max_grid;
    hipLaunchKernelGGL((fill_value_kernel<T>), dim3((int)grid), dim3(256), 0, st, (T *)out, n, v);
    FQ_HIP_TRY(hipGetLastError());
    return FQ_OK;
}

}  // namespace fqk

extern "C" fq_status fq_fill_value(void *d_out, int64_t n, int32_t dtype, uint64_t bits, void *stream) {
    using namespace fqk;
    hipStream_t st = (hipStream_t)stream;
    if (n < 0) return fqc::fail(FQ_E_INVALID, "fq_fill_value: negative length");
    if (n > 0 && !d_out) return fqc::fail(FQ_E_INVALID, "fq_fill_value: NULL output");
    switch (dtype) {
        case FQ_DT_BOOLEAN: {
            const int64_t words = (n + 63) / 64;
            fq_status s = fill_value<uint64_t>(d_out, words, bits ? ~0ull : 0ull, st);
            if (s != FQ_OK || !bits || (n & 63) == 0) return s;
            const uint64_t last = (1ull << (n & 63)) - 1;  // clear bits past n
            return fill_value<uint64_t>((uint64_t *)d_out + words - 1, 1, last, st);
        }
        case FQ_DT_INT8:
        case FQ_DT_UINT8: return fill_value<uint8_t>(d_out, n, (uint8_t)bits, st);
        case FQ_DT_INT16:
        case FQ_DT_UINT16: return fill_value<uint16_t>(d_out, n, (uint16_t)bits, st);
        case FQ_DT_INT32:
        case FQ_DT_UINT32: return fill_value<uint32_t>(d_out, n, (uint32_t)bits, st);
        case FQ_DT_FLOAT32: {
            const float f = (float)__builtin_bit_cast(double, bits);
            return fill_value<uint32_t>(d_out, n, __builtin_bit_cast(uint32_t, f), st);
        }
        case FQ_DT_INT64:
        case FQ_DT_UINT64:
        case FQ_DT_FLOAT64: return fill_value<uint64_t>(d_out, n, bits, st);
        default: return fqc::fail(FQ_E_UNSUPPORTED, std::string("fq_fill_value: ") + fqc::dtype_name(dtype));
    }
}
