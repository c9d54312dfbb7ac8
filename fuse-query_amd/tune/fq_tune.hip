// Tuning variants of the C3 scan (identity u64, sum/max/min/count, no
// predicate) for tools/tune_scan.py.  Not used by the product path: the
// winning configuration is folded into agg_flat_kernel (fq_aggregate.hip).
// Built into lib/libfq_tune.so (make tune), not into the product library.
#include <hip/hip_runtime.h>

#include "fq_common.h"
#include "fq_device.h"

namespace fqk {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ u32x4_t ld16(const u32x4_t *p) {
    if constexpr (NT == 1) return __builtin_nontemporal_load(p);
    else return *p;
}

struct TAcc {
    uint64_t sum, mx, mn, cnt;
};

__device__ __forceinline__ void tacc(TAcc &a, uint64_t x) {
    a.sum += x;
    a.mx = x > a.mx ? x : a.mx;
    a.mn = x < a.mn ? x : a.mn;
}

__device__ __forceinline__ void tstore(TAcc a, Partial *out) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a.sum += shfl_xor64(a.sum, off);
        uint64_t m = shfl_xor64(a.mx, off);
        a.mx = m > a.mx ? m : a.mx;
        m = shfl_xor64(a.mn, off);
        a.mn = m < a.mn ? m : a.mn;
        a.cnt += shfl_xor64(a.cnt, off);
    }
    __shared__ TAcc s[16];
    const int w = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0) s[w] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        TAcc r = s[0];
        for (int i = 1; i < (int)(blockDim.x / 64); ++i) {
            r.sum += s[i].sum;
            r.mx = s[i].mx > r.mx ? s[i].mx : r.mx;
            r.mn = s[i].mn < r.mn ? s[i].mn : r.mn;
            r.cnt += s[i].cnt;
        }
        Partial p{};
        p.sum = r.sum;
        p.max = r.mx;
        p.min = r.mn;
        p.count = r.cnt;
        p.dtype = FQ_DT_UINT64;
        *out = p;
    }
}

// MAP 0: grid-stride over vectors (production); MAP 1: each workgroup owns a
// contiguous chunk; MAP 2: grid-stride in units of a workgroup-wide tile of
// U vectors per lane (tile-contiguous per WG); MAP 3: MAP 2 within one
// contiguous eighth of the tiles per XCD.
template <int U, int NT, int MAP>
__global__ void tune_scan_kernel(const uint64_t *__restrict__ col, int64_t n, Partial *__restrict__ parts) {
    TAcc a{0, 0, ~0ull, 0};
    const u32x4_t *vp = reinterpret_cast<const u32x4_t *>(col);
    const int64_t nvec = n / 2;
    const int64_t B = blockDim.x;
    if constexpr (MAP == 0) {
        const int64_t T = (int64_t)gridDim.x * B;
        int64_t v = (int64_t)blockIdx.x * B + threadIdx.x;
        for (; v + (int64_t)(U - 1) * T < nvec; v += (int64_t)U * T) {
            u32x4_t r[U];
#pragma unroll
            for (int k = 0; k < U; ++k) r[k] = ld16<NT>(vp + v + (int64_t)k * T);
#pragma unroll
            for (int k = 0; k < U; ++k) {
                uint64_t x0 = ((uint64_t)r[k].y << 32) | r[k].x, x1 = ((uint64_t)r[k].w << 32) | r[k].z;
                tacc(a, x0);
                tacc(a, x1);
            }
            a.cnt += 2 * U;
        }
        for (; v < nvec; v += T) {
            u32x4_t r = ld16<NT>(vp + v);
            tacc(a, ((uint64_t)r.y << 32) | r.x);
            tacc(a, ((uint64_t)r.w << 32) | r.z);
            a.cnt += 2;
        }
    } else if constexpr (MAP == 1) {
        const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
        const int64_t b0 = (int64_t)blockIdx.x * per;
        const int64_t e0 = b0 + per < nvec ? b0 + per : nvec;
        int64_t v = b0 + threadIdx.x;
        for (; v + (int64_t)(U - 1) * B < e0; v += (int64_t)U * B) {
            u32x4_t r[U];
#pragma unroll
            for (int k = 0; k < U; ++k) r[k] = ld16<NT>(vp + v + (int64_t)k * B);
#pragma unroll
            for (int k = 0; k < U; ++k) {
                tacc(a, ((uint64_t)r[k].y << 32) | r[k].x);
                tacc(a, ((uint64_t)r[k].w << 32) | r[k].z);
            }
            a.cnt += 2 * U;
        }
        for (; v < e0; v += B) {
            u32x4_t r = ld16<NT>(vp + v);
            tacc(a, ((uint64_t)r.y << 32) | r.x);
            tacc(a, ((uint64_t)r.w << 32) | r.z);
            a.cnt += 2;
        }
    } else if constexpr (MAP == 3) {
        // XCD-partitioned tiles: workgroup b runs on XCD b % 8 (round-robin
        // dispatch), XCD x streams the x-th eighth of the tiles, its
        // workgroups grid-striding through that slice
        const int64_t tile = (int64_t)U * B;
        const int64_t ntiles = nvec / tile;
        const int64_t per = (ntiles + 7) / 8;
        const int64_t x = blockIdx.x & 7, G8 = gridDim.x >> 3;
        const int64_t t1 = (x + 1) * per < ntiles ? (x + 1) * per : ntiles;
        for (int64_t t = x * per + (blockIdx.x >> 3); t < t1; t += G8) {
            const int64_t base = t * tile + threadIdx.x;
            u32x4_t r[U];
#pragma unroll
            for (int k = 0; k < U; ++k) r[k] = ld16<NT>(vp + base + (int64_t)k * B);
#pragma unroll
            for (int k = 0; k < U; ++k) {
                tacc(a, ((uint64_t)r[k].y << 32) | r[k].x);
                tacc(a, ((uint64_t)r[k].w << 32) | r[k].z);
            }
            a.cnt += 2 * U;
        }
        for (int64_t v = ntiles * tile + (int64_t)blockIdx.x * B + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * B) {
            u32x4_t r = ld16<NT>(vp + v);
            tacc(a, ((uint64_t)r.y << 32) | r.x);
            tacc(a, ((uint64_t)r.w << 32) | r.z);
            a.cnt += 2;
        }
    } else {
        const int64_t tile = (int64_t)U * B;
        const int64_t ntiles = nvec / tile;
        for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
            const int64_t base = t * tile + threadIdx.x;
            u32x4_t r[U];
#pragma unroll
            for (int k = 0; k < U; ++k) r[k] = ld16<NT>(vp + base + (int64_t)k * B);
#pragma unroll
            for (int k = 0; k < U; ++k) {
                tacc(a, ((uint64_t)r[k].y << 32) | r[k].x);
                tacc(a, ((uint64_t)r[k].w << 32) | r[k].z);
            }
            a.cnt += 2 * U;
        }
        for (int64_t v = ntiles * tile + (int64_t)blockIdx.x * B + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * B) {
            u32x4_t r = ld16<NT>(vp + v);
            tacc(a, ((uint64_t)r.y << 32) | r.x);
            tacc(a, ((uint64_t)r.w << 32) | r.z);
            a.cnt += 2;
        }
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        tacc(a, col[n - 1]);
        a.cnt += 1;
    }
    tstore(a, parts + blockIdx.x);
}

template <int U, int NT, int MAP>
static void launch(const uint64_t *col, int64_t n, int grid, int block, Partial *parts, hipStream_t st) {
    hipLaunchKernelGGL((tune_scan_kernel<U, NT, MAP>), dim3(grid), dim3(block), 0, st, col, n, parts);
}

}  // namespace fqk

// variant = U*100 + NT*10 + MAP, U in {1,2,4,8,16}
extern "C" fq_status fq_tune_scan_u64(const uint64_t *col, int64_t n, int32_t variant, int32_t grid, int32_t block,
                                      void *d_parts, void *stream) {
    using namespace fqk;
    hipStream_t st = (hipStream_t)stream;
    Partial *p = (Partial *)d_parts;
    const int U = variant / 100, NT = (variant / 10) % 10, MAP = variant % 10;
#define FQ_T(u, nt, m) \
    if (U == u && NT == nt && MAP == m) { launch<u, nt, m>(col, n, grid, block, p, st); FQ_HIP_TRY(hipGetLastError()); return FQ_OK; }
#define FQ_TU(u) FQ_T(u, 0, 0) FQ_T(u, 1, 0) FQ_T(u, 0, 1) FQ_T(u, 1, 1) FQ_T(u, 0, 2) FQ_T(u, 1, 2) FQ_T(u, 1, 3)
    FQ_TU(1) FQ_TU(2) FQ_TU(4) FQ_TU(8) FQ_TU(16)
#undef FQ_TU
#undef FQ_T
    return fqc::fail(FQ_E_INVALID, "fq_tune_scan_u64: unknown variant");
}

namespace fqk {

// ---------------------------------------------------------------------------
// Write-side variants: out[i] = base + i (fill) and out[i] = in[i] + 1 (a
// read+write stream, the shape of fq_arith), for tools/tune_scan.py --write.
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void st16(u32x4_t *p, u32x4_t v) {
    if constexpr (NT == 1) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__device__ __forceinline__ u32x4_t iota2(uint64_t i0) {
    u32x4_t v;
    v.x = (uint32_t)i0;
    v.y = (uint32_t)(i0 >> 32);
    v.z = (uint32_t)(i0 + 1);
    v.w = (uint32_t)((i0 + 1) >> 32);
    return v;
}

__device__ __forceinline__ u32x4_t add1(u32x4_t r) {
    uint64_t a = ((uint64_t)r.y << 32) | r.x, b = ((uint64_t)r.w << 32) | r.z;
    a += 1;
    b += 1;
    u32x4_t v;
    v.x = (uint32_t)a;
    v.y = (uint32_t)(a >> 32);
    v.z = (uint32_t)b;
    v.w = (uint32_t)(b >> 32);
    return v;
}

// KIND 0 fill, 1 add; MAP 0 grid-stride by vector, 2 tile-contiguous
template <int KIND, int U, int NT, int MAP>
__global__ void tune_write_kernel(const uint64_t *__restrict__ in, uint64_t *__restrict__ out, int64_t n) {
    const u32x4_t *ip = reinterpret_cast<const u32x4_t *>(in);
    u32x4_t *op = reinterpret_cast<u32x4_t *>(out);
    const int64_t nvec = n / 2;
    const int64_t B = blockDim.x;
    if constexpr (MAP == 0) {
        const int64_t T = (int64_t)gridDim.x * B;
        for (int64_t v = (int64_t)blockIdx.x * B + threadIdx.x; v < nvec; v += T) {
            if constexpr (KIND == 0) st16<NT>(op + v, iota2(2 * (uint64_t)v));
            else st16<NT>(op + v, add1(ld16<NT>(ip + v)));
        }
    } else {
        const int64_t tile = (int64_t)U * B;
        const int64_t ntiles = nvec / tile;
        for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
            const int64_t base = t * tile + threadIdx.x;
            if constexpr (KIND == 0) {
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int64_t v = base + (int64_t)k * B;
                    st16<NT>(op + v, iota2(2 * (uint64_t)v));
                }
            } else {
                u32x4_t r[U];
#pragma unroll
                for (int k = 0; k < U; ++k) r[k] = ld16<NT>(ip + base + (int64_t)k * B);
#pragma unroll
                for (int k = 0; k < U; ++k) st16<NT>(op + base + (int64_t)k * B, add1(r[k]));
            }
        }
        for (int64_t v = ntiles * tile + (int64_t)blockIdx.x * B + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * B) {
            if constexpr (KIND == 0) st16<NT>(op + v, iota2(2 * (uint64_t)v));
            else st16<NT>(op + v, add1(ld16<NT>(ip + v)));
        }
    }
}

}  // namespace fqk

// variant = KIND*1000 + U*100 + NT*10 + MAP
extern "C" fq_status fq_tune_write_u64(const uint64_t *in, uint64_t *out, int64_t n, int32_t variant, int32_t grid,
                                       int32_t block, void *stream) {
    using namespace fqk;
    hipStream_t st = (hipStream_t)stream;
    const int KIND = variant / 1000, U = (variant / 100) % 10, NT = (variant / 10) % 10, MAP = variant % 10;
#define FQ_W(kd, u, nt, m)                                                                                  \
    if (KIND == kd && U == u && NT == nt && MAP == m) {                                                     \
        hipLaunchKernelGGL((tune_write_kernel<kd, u, nt, m>), dim3(grid), dim3(block), 0, st, in, out, n); \
        FQ_HIP_TRY(hipGetLastError());                                                                      \
        return FQ_OK;                                                                                       \
    }
#define FQ_WU(kd, u) FQ_W(kd, u, 0, 0) FQ_W(kd, u, 1, 0) FQ_W(kd, u, 0, 2) FQ_W(kd, u, 1, 2)
    FQ_WU(0, 1) FQ_WU(0, 2) FQ_WU(0, 4) FQ_WU(0, 8) FQ_WU(1, 1) FQ_WU(1, 2) FQ_WU(1, 4) FQ_WU(1, 8)
#undef FQ_WU
#undef FQ_W
    return fqc::fail(FQ_E_INVALID, "fq_tune_write_u64: unknown variant");
}
