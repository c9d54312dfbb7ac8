// FilterTransform compaction on gfx950 (arrow filter_record_batch,
// src/transforms/transform_filter.rs:51): keep the rows whose predicate bit
// is set, preserving order.
//
// Three passes over tiles of 256 bitmap words (16,384 rows):
//   count   one workgroup per tile, popcount of its 256 words -> counts[tile]
//   scan    one workgroup, exclusive scan of the tile counts (+ total)
//   scatter one workgroup per tile: LDS scan of its word popcounts, then each
//           wave walks 64 words, 8 at a time; lane l moves row 64w+l to
//           base + word_offset + popcount(word & lanemask_lt(l)).
// Reads and writes are contiguous per wave; the bitmap is read twice
// (1/64 of a u64 column's bytes each time).
#include <hip/hip_runtime.h>

#include "fq_common.h"
#include "fq_device.h"

namespace fqk {

constexpr int kTileWords = 256;
constexpr int kScanThreads = 1024;

__device__ __forceinline__ uint64_t word_at(const uint64_t *bm, int64_t w, int64_t nwords, int64_t n) {
    if (w >= nwords) return 0;
    uint64_t v = bm[w];
    const int64_t rows = n - w * 64;
    if (rows < 64) v &= (1ull << rows) - 1ull;  // ignore bits past len
    return v;
}

__global__ void __launch_bounds__(kTileWords)
    compact_count_kernel(const uint64_t *__restrict__ bm, int64_t n, uint64_t *__restrict__ counts) {
    const int64_t nwords = (n + 63) / 64;
    const int64_t w = (int64_t)blockIdx.x * kTileWords + threadIdx.x;
    uint64_t c = __popcll(word_at(bm, w, nwords, n));
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) c += shfl_xor64(c, off);
    __shared__ uint64_t s[kTileWords / kWave];
    if ((threadIdx.x & (kWave - 1)) == 0) s[threadIdx.x / kWave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
#pragma unroll
        for (int i = 0; i < kTileWords / kWave; ++i) t += s[i];
        counts[blockIdx.x] = t;
    }
}

// exclusive scan of counts[0..ntiles) in place; counts[ntiles] = total.
// One workgroup of 16 waves; each wave owns a contiguous segment and walks it
// 64 entries at a time (coalesced loads, wave scan by shuffles), twice: once
// for its total, once to write prefixes after the 16 totals are scanned.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, int lane) {
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const uint64_t u = shfl_up64(v, off);
        if (lane >= off) v += u;
    }
    return v;
}

__global__ void __launch_bounds__(kScanThreads) compact_scan_kernel(uint64_t *counts, int64_t ntiles) {
    constexpr int W = kScanThreads / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t seg = (ntiles + W - 1) / W;
    const int64_t b = (int64_t)wave * seg;
    const int64_t e = (b + seg < ntiles) ? b + seg : ntiles;
    uint64_t sum = 0;
    for (int64_t i = b + lane; i < e; i += kWave) sum += counts[i];
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) sum += shfl_xor64(sum, off);
    __shared__ uint64_t s_tot[W + 1];
    if (lane == 0) s_tot[wave] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t run = 0;
        for (int w = 0; w < W; ++w) {
            const uint64_t t = s_tot[w];
            s_tot[w] = run;
            run += t;
        }
        s_tot[W] = run;
    }
    __syncthreads();
    uint64_t run = s_tot[wave];
    for (int64_t i0 = b; i0 < e; i0 += kWave) {
        const int64_t i = i0 + lane;
        const uint64_t v = i < e ? counts[i] : 0;
        const uint64_t incl = wave_incl_scan(v, lane);
        if (i < e) counts[i] = run + incl - v;
        run += shfl64(incl, kWave - 1);
    }
    if (threadIdx.x == 0) counts[ntiles] = s_tot[W];
}

template <typename T>
__global__ void __launch_bounds__(kTileWords)
    compact_scatter_kernel(const T *__restrict__ in, const uint64_t *__restrict__ bm, int64_t n,
                           const uint64_t *__restrict__ offsets, T *__restrict__ out) {
    const int64_t nwords = (n + 63) / 64;
    const int64_t w0 = (int64_t)blockIdx.x * kTileWords;
    __shared__ uint64_t s_word[kTileWords];
    __shared__ uint32_t s_off[kTileWords];
    __shared__ uint32_t s_wsum[kTileWords / kWave];
    const int t = threadIdx.x;
    const int lane = t & (kWave - 1);
    const int wave = t / kWave;
    const uint64_t word = word_at(bm, w0 + t, nwords, n);
    s_word[t] = word;
    // wave-inclusive scan of popcounts
    uint32_t c = (uint32_t)__popcll(word);
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, off, kWave);
        if (lane >= off) incl += v;
    }
    if (lane == kWave - 1) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t wave_base = 0;
    for (int i = 0; i < wave; ++i) wave_base += s_wsum[i];
    s_off[t] = wave_base + incl - c;
    __syncthreads();
    const uint64_t base = offsets[blockIdx.x];
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // 8 words per step: all loads of the step are issued before the first
    // store (8 rows per lane in flight); empty words are skipped (uniform).
    constexpr int kStep = 8;
    for (int j = 0; j < kWave; j += kStep) {
        T x[kStep];
        uint64_t wd[kStep];
#pragma unroll
        for (int k = 0; k < kStep; ++k) {
            const int wi = wave * kWave + j + k;
            wd[k] = s_word[wi];
            const int64_t row = (w0 + wi) * 64 + lane;
            x[k] = ((wd[k] >> lane) & 1ull) ? __builtin_nontemporal_load(in + row) : T(0);
        }
#pragma unroll
        for (int k = 0; k < kStep; ++k) {
            const int wi = wave * kWave + j + k;
            if ((wd[k] >> lane) & 1ull) {
                const uint64_t pos = base + s_off[wi] + (uint64_t)__popcll(wd[k] & lt_mask);
                out[pos] = x[k];
            }
        }
    }
}

// 8-byte columns, 16-byte aligned: lane l of a wave loads rows 2l and 2l+1
// of a 128-row word pair with one 16-byte load (lanes 0..31: the pair's first
// word, 32..63: its second), 4 pairs in flight per step; positions come from
// the same LDS word offsets.
typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));

template <typename T>
__global__ void __launch_bounds__(kTileWords)
    compact_scatter_vec_kernel(const T *__restrict__ in, const uint64_t *__restrict__ bm, int64_t n,
                               const uint64_t *__restrict__ offsets, T *__restrict__ out) {
    static_assert(sizeof(T) == 8, "8-byte rows");
    const int64_t nwords = (n + 63) / 64;
    const int64_t w0 = (int64_t)blockIdx.x * kTileWords;
    __shared__ uint64_t s_word[kTileWords];
    __shared__ uint32_t s_off[kTileWords];
    __shared__ uint32_t s_wsum[kTileWords / kWave];
    const int t = threadIdx.x;
    const int lane = t & (kWave - 1);
    const int wave = t / kWave;
    const uint64_t word = word_at(bm, w0 + t, nwords, n);
    s_word[t] = word;
    uint32_t c = (uint32_t)__popcll(word);
    uint32_t incl = c;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, off, kWave);
        if (lane >= off) incl += v;
    }
    if (lane == kWave - 1) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t wave_base = 0;
    for (int i = 0; i < wave; ++i) wave_base += s_wsum[i];
    s_off[t] = wave_base + incl - c;
    __syncthreads();
    const uint64_t base = offsets[blockIdx.x];
    const int half = lane >> 5;        // which word of the pair
    const int bl = (lane & 31) * 2;    // bit of this lane's first row in that word
    const uint64_t m_lt = bl == 0 ? 0ull : (~0ull >> (64 - bl));
    const u64x2_t *__restrict__ vin = reinterpret_cast<const u64x2_t *>(in);
    constexpr int kPairs = 4;
    for (int j = 0; j < kWave; j += 2 * kPairs) {
        u64x2_t x[kPairs];
        uint64_t wd[kPairs];
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
            const int wi = wave * kWave + j + 2 * k + half;
            wd[k] = s_word[wi];
            const int64_t row = (w0 + wave * kWave + j + 2 * k) * 64 + 2 * lane;
            const uint64_t bits = (wd[k] >> bl) & 3ull;
            x[k] = u64x2_t{0, 0};
            if (bits) {
                if (row + 1 < n) {
                    x[k] = __builtin_nontemporal_load(vin + (row >> 1));
                } else {
                    x[k].x = (unsigned long long)__builtin_bit_cast(uint64_t, in[row]);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kPairs; ++k) {
            const int wi = wave * kWave + j + 2 * k + half;
            const uint64_t bits = (wd[k] >> bl) & 3ull;
            if (!bits) continue;
            uint64_t pos = base + s_off[wi] + (uint64_t)__popcll(wd[k] & m_lt);
            if (bits & 1ull) out[pos++] = __builtin_bit_cast(T, (uint64_t)x[k].x);
            if (bits & 2ull) out[pos] = __builtin_bit_cast(T, (uint64_t)x[k].y);
        }
    }
}

}  // namespace fqk

extern "C" {

size_t fq_filter_workspace_bytes(int64_t len) {
    const int64_t nwords = (len + 63) / 64;
    const int64_t ntiles = (nwords + fqk::kTileWords - 1) / fqk::kTileWords;
    return (size_t)(ntiles + 1) * sizeof(uint64_t);
}

fq_status fq_filter_compact(const fq_col *in, const uint64_t *d_bitmap, void *d_out, int64_t *out_len,
                            void *d_ws, size_t ws_bytes, void *stream) {
    using namespace fqk;
    if (!in || !out_len) return fqc::fail(FQ_E_INVALID, "fq_filter_compact: NULL argument");
    const int64_t n = in->len;
    *out_len = 0;
    if (n == 0) return FQ_OK;
    if (!in->data || !d_bitmap || !d_out || !d_ws)
        return fqc::fail(FQ_E_INVALID, "fq_filter_compact: NULL buffer");
    if (ws_bytes < fq_filter_workspace_bytes(n))
        return fqc::fail(FQ_E_INVALID, "fq_filter_compact: workspace too small");
    const int esz = in->dtype == FQ_DT_BOOLEAN ? 0 : fqc::dtype_size(in->dtype);
    if (esz == 0) return fqc::fail(FQ_E_UNSUPPORTED, "fq_filter_compact: column type not supported");
    hipStream_t st = (hipStream_t)stream;
    const int64_t nwords = (n + 63) / 64;
    const int64_t ntiles = (nwords + kTileWords - 1) / kTileWords;
    uint64_t *counts = (uint64_t *)d_ws;
    hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)ntiles), dim3(kTileWords), 0, st, d_bitmap, n,
                       counts);
    FQ_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, counts, ntiles);
    FQ_HIP_TRY(hipGetLastError());
    switch (esz) {
        case 1:
            hipLaunchKernelGGL(compact_scatter_kernel<uint8_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0, st,
                               (const uint8_t *)in->data, d_bitmap, n, counts, (uint8_t *)d_out);
            break;
        case 2:
            hipLaunchKernelGGL(compact_scatter_kernel<uint16_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0, st,
                               (const uint16_t *)in->data, d_bitmap, n, counts, (uint16_t *)d_out);
            break;
        case 4:
            hipLaunchKernelGGL(compact_scatter_kernel<uint32_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0, st,
                               (const uint32_t *)in->data, d_bitmap, n, counts, (uint32_t *)d_out);
            break;
        default:
            if (((uintptr_t)in->data & 15u) == 0)
                hipLaunchKernelGGL(compact_scatter_vec_kernel<uint64_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0,
                                   st, (const uint64_t *)in->data, d_bitmap, n, counts, (uint64_t *)d_out);
            else
                hipLaunchKernelGGL(compact_scatter_kernel<uint64_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0,
                                   st, (const uint64_t *)in->data, d_bitmap, n, counts, (uint64_t *)d_out);
            break;
    }
    FQ_HIP_TRY(hipGetLastError());
    uint64_t total = 0;
    FQ_HIP_TRY(hipMemcpyAsync(&total, counts + ntiles, sizeof(total), hipMemcpyDeviceToHost, st));
    FQ_HIP_TRY(hipStreamSynchronize(st));
    *out_len = (int64_t)total;
    return FQ_OK;
}

}  // extern "C"
