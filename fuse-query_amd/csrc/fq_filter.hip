// FilterTransform compaction on gfx950 (arrow filter_record_batch,
// src/transforms/transform_filter.rs:51): keep the rows whose predicate bit
// is set, preserving order.
//
// Three passes over tiles of 256 bitmap words (16,384 rows), in groups of 16:
//   count   one workgroup per group: popcounts of its tiles -> each tile's
//           exclusive prefix inside the group, and the group's total
//   scan    one workgroup: exclusive scan of the group totals
//   scatter one workgroup per tile, LDS scan of its word popcounts, then:
//           8-byte aligned columns: two 8,192-row rounds, each loading row
//           pairs with 16-byte loads, dropping kept rows into an LDS stage
//           at their output offset and writing the round's contiguous output
//           range with aligned 16-byte stores;
//           other widths: each wave walks 64 words, 8 at a time; lane l
//           moves row 64w+l to base + word_offset + popcount(word & lt(l)).
// The bitmap is read twice (1/64 of a u64 column's bytes each time).
#include <hip/hip_runtime.h>

#include "fq_common.h"
#include "fq_device.h"
#include "fq_scan.h"

namespace fqk {

constexpr int kTileWords = 256;

__device__ __forceinline__ uint64_t word_at(const uint64_t *bm, int64_t w, int64_t nwords, int64_t n) {
    if (w >= nwords) return 0;
    uint64_t v = bm[w];
    const int64_t rows = n - w * 64;
    if (rows < 64) v &= (1ull << rows) - 1ull;  // ignore bits past len
    return v;
}

// count: workgroup g covers the kGroupTiles tiles of group g (wave w: tiles
// 4w..4w+3 of the group, all 16 word loads of a lane in flight together);
// writes each tile's exclusive prefix within the group -> intra[tile] and
// the group's total -> gpre[g].
constexpr int kGroupTiles = 16;
constexpr int kWaveTiles = kGroupTiles / (kTileWords / kWave);

__global__ void __launch_bounds__(kTileWords)
    compact_count_kernel(const uint64_t *__restrict__ bm, int64_t n, int64_t ntiles, uint64_t *__restrict__ intra,
                         uint64_t *__restrict__ gpre) {
    const int64_t nwords = (n + 63) / 64;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int64_t t0 = (int64_t)blockIdx.x * kGroupTiles + wave * kWaveTiles;
    uint64_t wd[kWaveTiles][kTileWords / kWave];
#pragma unroll
    for (int k = 0; k < kWaveTiles; ++k)
#pragma unroll
        for (int j = 0; j < kTileWords / kWave; ++j)
            wd[k][j] = bm[min((t0 + k) * kTileWords + j * kWave + lane, nwords - 1)];  // all in flight
#pragma unroll
    for (int k = 0; k < kWaveTiles; ++k)
#pragma unroll
        for (int j = 0; j < kTileWords / kWave; ++j) {
            const int64_t w = (t0 + k) * kTileWords + j * kWave + lane;
            const int64_t rows = n - w * 64;
            if (rows <= 0) wd[k][j] = 0;
            else if (rows < 64) wd[k][j] &= (1ull << rows) - 1ull;  // ignore bits past len
        }
    __shared__ uint64_t s_c[kGroupTiles];
#pragma unroll
    for (int k = 0; k < kWaveTiles; ++k) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < kTileWords / kWave; ++j) c += __popcll(wd[k][j]);
#pragma unroll
        for (int off = kWave / 2; off > 0; off >>= 1) c += shfl_xor64(c, off);
        if (lane == 0) s_c[wave * kWaveTiles + k] = c;
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < kGroupTiles) {
        uint64_t pre = 0;
        for (int i = 0; i < t; ++i) pre += s_c[i];
        const int64_t tile = (int64_t)blockIdx.x * kGroupTiles + t;
        if (tile < ntiles) intra[tile] = pre;
        if (t == kGroupTiles - 1) gpre[blockIdx.x] = pre + s_c[t];
    }
}

// exclusive scan of gpre[0..m) in place, gpre[m] = total.  One workgroup;
// the array is taken 16,384 entries per round, 16 consecutive entries per
// thread loaded together (indices clamped, values masked), so a round costs
// one memory round trip.
constexpr int kScanThreads = 1024;
constexpr int kScanPer = 16;

__global__ void __launch_bounds__(kScanThreads) compact_scan_kernel(uint64_t *gpre, int64_t m) {
    constexpr int W = kScanThreads / kWave;
    const int t = threadIdx.x;
    const int lane = t & (kWave - 1);
    const int wave = t / kWave;
    __shared__ uint64_t s_w[W];
    uint64_t run = 0;  // uniform: total of the earlier rounds
    for (int64_t r0 = 0; r0 < m; r0 += (int64_t)kScanThreads * kScanPer) {
        const int64_t i0 = r0 + (int64_t)t * kScanPer;
        uint64_t v[kScanPer];
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) v[k] = gpre[i0 + k < m ? i0 + k : m - 1];
        uint64_t tot = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            if (i0 + k >= m) v[k] = 0;
            tot += v[k];
        }
        uint64_t incl = tot;
#pragma unroll
        for (int off = 1; off < kWave; off <<= 1) {
            const uint64_t u = shfl_up64(incl, off);
            if (lane >= off) incl += u;
        }
        if (lane == kWave - 1) s_w[wave] = incl;
        __syncthreads();
        uint64_t wbase = 0, rtot = 0;
        for (int w = 0; w < W; ++w) {
            const uint64_t x = s_w[w];
            if (w < wave) wbase += x;
            rtot += x;
        }
        uint64_t p = run + wbase + incl - tot;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            if (i0 + k < m) gpre[i0 + k] = p;
            p += v[k];
        }
        run += rtot;
        __syncthreads();  // s_w reused by the next round
    }
    if (t == 0) gpre[m] = run;
}

__device__ __forceinline__ uint64_t tile_base(const uint64_t *intra, const uint64_t *gpre, int64_t tile) {
    return gpre[tile / kGroupTiles] + intra[tile];
}

template <typename T>
__global__ void __launch_bounds__(kTileWords)
    compact_scatter_kernel(const T *__restrict__ in, const uint64_t *__restrict__ bm, int64_t n,
                           const uint64_t *__restrict__ intra, const uint64_t *__restrict__ gpre, T *__restrict__ out) {
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
    const uint64_t base = tile_base(intra, gpre, blockIdx.x);
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
                               const uint64_t *__restrict__ intra, const uint64_t *__restrict__ gpre, T *__restrict__ out) {
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
    const uint64_t base = tile_base(intra, gpre, blockIdx.x);
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

// 8-byte columns, input and output 16-byte aligned: the tile is compacted in
// two 8,192-row rounds through LDS (64 KB stage, 2 workgroups per CU).  Each thread loads 8 row pairs with
// 16-byte loads (consecutive threads, consecutive pairs), drops the kept rows
// into a 32 KB LDS stage at their offset within the round, and the
// workgroup then writes the round's contiguous output range as aligned
// 16-byte stores (8-byte stores only at its two ends).
constexpr int kRoundWords = 128;
constexpr int kRoundPairs = kRoundWords * 32;

template <typename T>
__global__ void __launch_bounds__(kTileWords)
    compact_scatter_lds_kernel(const T *__restrict__ in, const uint64_t *__restrict__ bm, int64_t n,
                               const uint64_t *__restrict__ intra, const uint64_t *__restrict__ gpre, T *__restrict__ out) {
    static_assert(sizeof(T) == 8, "8-byte rows");
    const int64_t nwords = (n + 63) / 64;
    const int64_t tile = blockIdx.x;
    const int64_t w0 = tile * kTileWords;
    __shared__ uint64_t s_word[kTileWords];
    __shared__ uint32_t s_off[kTileWords + 1];
    __shared__ uint32_t s_wsum[kTileWords / kWave];
    __shared__ uint64_t s_stage[kRoundPairs * 2];
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
    if (t == kTileWords - 1) s_off[kTileWords] = wave_base + incl;
    __syncthreads();
    const uint64_t base = tile_base(intra, gpre, tile);
    const u64x2_t *__restrict__ vin = reinterpret_cast<const u64x2_t *>(in);
    u64x2_t *__restrict__ vout = reinterpret_cast<u64x2_t *>(out);
    constexpr int kPer = kRoundPairs / kTileWords;
    for (int rw = 0; rw < kTileWords; rw += kRoundWords) {
        const uint32_t rb = s_off[rw], re = s_off[rw + kRoundWords];
        if (rb == re) continue;  // nothing kept in this round (uniform)
        const int64_t row_r = (w0 + rw) * 64;
        u64x2_t x[kPer];
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int v = t + kTileWords * i;
            const int64_t row = row_r + 2 * v;
            const uint64_t bits = (s_word[rw + (v >> 5)] >> ((2 * v) & 63)) & 3ull;
            x[i] = u64x2_t{0, 0};
            if (bits) {
                if (row + 1 < n) {
                    x[i] = __builtin_nontemporal_load(vin + (row >> 1));
                } else if (row < n) {
                    x[i].x = (unsigned long long)__builtin_bit_cast(uint64_t, in[row]);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int v = t + kTileWords * i;
            const int wi = rw + (v >> 5);
            const int bl = (2 * v) & 63;
            const uint64_t wd = s_word[wi];
            const uint64_t bits = (wd >> bl) & 3ull;
            if (!bits) continue;
            const uint64_t m_lt = bl == 0 ? 0ull : (~0ull >> (64 - bl));
            uint32_t pos = s_off[wi] - rb + (uint32_t)__popcll(wd & m_lt);
            if (bits & 1ull) s_stage[pos++] = (uint64_t)x[i].x;
            if (bits & 2ull) s_stage[pos] = (uint64_t)x[i].y;
        }
        __syncthreads();
        const uint64_t g0 = base + rb, g1 = base + re;
        for (uint64_t p = (g0 >> 1) + t; p < ((g1 + 1) >> 1); p += kTileWords) {
            const uint64_t e0 = 2 * p, e1 = e0 + 1;
            if (e0 >= g0 && e1 < g1) {
                __builtin_nontemporal_store(u64x2_t{s_stage[e0 - g0], s_stage[e1 - g0]}, vout + p);
            } else if (e0 >= g0) {
                out[e0] = __builtin_bit_cast(T, s_stage[e0 - g0]);
            } else {
                out[e1] = __builtin_bit_cast(T, s_stage[e1 - g0]);
            }
        }
        __syncthreads();
    }
}

}  // namespace fqk

extern "C" {

size_t fq_filter_workspace_bytes(int64_t len) {
    const int64_t nwords = (len + 63) / 64;
    const int64_t ntiles = (nwords + fqk::kTileWords - 1) / fqk::kTileWords;
    const int64_t ngroups = (ntiles + fqk::kGroupTiles - 1) / fqk::kGroupTiles;
    return (size_t)(ntiles + ngroups + 1) * sizeof(uint64_t);
}

}  // extern "C"

namespace fqk {
namespace {

// block b of a block stream with every row kept holds min(B, n - b * B) rows
__global__ void block_lengths_kernel(int64_t *__restrict__ counts, int64_t nb, int64_t B, int64_t n) {
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (int64_t)gridDim.x * blockDim.x)
        counts[b] = b * B + B <= n ? B : n - b * B;
}

// filter_project_blocks_enqueue with a resident workspace: after the
// projection kernel, one thread moves {kept rows, flag words} to d_res (host
// memory the device writes) and zeroes the three workspace words -- one launch
// in place of the next call's memset and this call's copy.
__global__ void project_hand_off_kernel(uint64_t *__restrict__ ws, uint64_t *__restrict__ d_res) {
    if (threadIdx.x != 0) return;
    d_res[0] = ws[0];
    d_res[1] = ws[1];
    ws[0] = 0;
    ws[1] = 0;
    ws[2] = 0;
}

// ---- fq_blocks_compact: a block stream's valid rows into one array ----
// counts[b] -> exclusive offsets in three launches: per-chunk sums of
// kCompactChunk counts, one workgroup scanning the chunk sums, then each chunk
// scanning its counts from its base; a copy kernel moves block b's rows (one
// workgroup per block, lane-consecutive 8-byte rows: coalesced both sides).
constexpr int kCompactChunk = 1024;

__global__ void __launch_bounds__(kCompactChunk)
blocks_chunk_sums_kernel(const int64_t *__restrict__ counts, int64_t nb, int64_t *__restrict__ sums) {
    __shared__ int64_t red[kCompactChunk / kWave];
    const int64_t b = (int64_t)blockIdx.x * kCompactChunk + threadIdx.x;
    int64_t v = b < nb ? counts[b] : 0;
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int w = 0; w < kCompactChunk / kWave; ++w) t += red[w];
        sums[blockIdx.x] = t;
    }
}

// exclusive scan of `n` values in place by one workgroup; base[n] = the total
__global__ void __launch_bounds__(kCompactChunk) blocks_scan_sums_kernel(int64_t *__restrict__ sums, int64_t n) {
    __shared__ int64_t part[kCompactChunk];
    const int64_t per = (n + kCompactChunk - 1) / kCompactChunk;
    const int64_t lo = threadIdx.x * per, hi = lo + per < n ? lo + per : n;
    int64_t t = 0;
    for (int64_t i = lo; i < hi; ++i) t += sums[i];
    part[threadIdx.x] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t run = 0;
        for (int i = 0; i < kCompactChunk; ++i) {
            const int64_t x = part[i];
            part[i] = run;
            run += x;
        }
        sums[n] = run;
    }
    __syncthreads();
    int64_t run = part[threadIdx.x];
    for (int64_t i = lo; i < hi; ++i) {
        const int64_t x = sums[i];
        sums[i] = run;
        run += x;
    }
}

__global__ void __launch_bounds__(kCompactChunk)
blocks_offsets_kernel(const int64_t *__restrict__ counts, int64_t nb, const int64_t *__restrict__ sums,
                      int64_t *__restrict__ offs) {
    __shared__ int64_t part[kCompactChunk];
    const int64_t b = (int64_t)blockIdx.x * kCompactChunk + threadIdx.x;
    part[threadIdx.x] = b < nb ? counts[b] : 0;
    __syncthreads();
    for (int o = 1; o < kCompactChunk; o <<= 1) {  // Hillis-Steele inclusive scan
        const int64_t add = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += add;
        __syncthreads();
    }
    if (b < nb) offs[b] = sums[blockIdx.x] + part[threadIdx.x] - counts[b];
    if (b == nb - 1) offs[nb] = sums[blockIdx.x] + part[threadIdx.x];
}

struct CompactCols {
    const uint64_t *in[FQ_MAX_PROJECT];
    uint64_t *out[FQ_MAX_PROJECT];
};

__global__ void __launch_bounds__(256)
blocks_copy_kernel(CompactCols cols, int32_t n_cols, const int64_t *__restrict__ counts,
                   const int64_t *__restrict__ offs, int64_t nb, int64_t block_rows) {
    for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const int64_t c = counts[b], src = b * block_rows, dst = offs[b];
        for (int j = 0; j < n_cols; ++j)
            for (int64_t r = threadIdx.x; r < c; r += blockDim.x) cols.out[j][dst + r] = cols.in[j][src + r];
    }
}

// Workspace of fq_filter_project: [total][flag words: predicate,
// expressions][the ticket counter, a 128 B line][one look-back status word
// per tile].
struct ProjWs {
    uint64_t *total;
    uint32_t *flags, *ticket;
    uint64_t *status;
    int64_t ntiles;
};

ProjWs proj_ws(void *d_ws, int64_t n) {
    ProjWs w;
    w.ntiles = (n + select_tile_rows() - 1) / select_tile_rows();
    w.total = (uint64_t *)d_ws;
    w.flags = (uint32_t *)(w.total + 1);
    w.ticket = (uint32_t *)(w.total + 2);
    w.status = w.total + 2 + 16;
    return w;
}

fq_status flag_error(uint32_t f) {
    if (f & 0x80000000u) return fqc::fail(FQ_E_INTERNAL, "fused projection: the offset look-back did not complete");
    if (f & FQ_STATE_DIV_ZERO) return fqc::fail(FQ_E_DIVIDE_BY_ZERO, "Internal Error: Divide by zero error");
    if (f & FQ_STATE_CAST_NULL)
        return fqc::fail(FQ_E_UNSUPPORTED, "cast produced nulls (nulls are not supported on the device path)");
    return FQ_OK;
}

fq_status lower_projection(const fq_col *col, const fq_pred *pred, const fq_expr *values, int32_t n_out, void *const *d_out,
                           void *stream, ProjLaunch &P) {
    if (!col) return fqc::fail(FQ_E_INVALID, "fq_filter_project: NULL column");
    if (col->len > 0 && !col->data) return fqc::fail(FQ_E_INVALID, "fq_filter_project: NULL column data");
    if (fqc::dtype_size(col->dtype) != 8 || col->dtype == FQ_DT_BOOLEAN)
        return fqc::fail(FQ_E_UNSUPPORTED, "fused projection needs a 64-bit numeric column");
    if (n_out < 0 || n_out > FQ_MAX_PROJECT || (n_out > 0 && (!values || !d_out)))
        return fqc::fail(FQ_E_INVALID, "fq_filter_project: bad output list");
    P = ProjLaunch{};
    P.col = col->data;
    P.n = col->len;
    P.stream = (hipStream_t)stream;
    fq_status s = lower_pred(pred, col->dtype, col->len, true, P.pred);
    if (s != FQ_OK) return s;
    P.n_out = n_out;
    for (int j = 0; j < n_out; ++j) {
        if (!d_out[j] && col->len > 0) return fqc::fail(FQ_E_INVALID, "fq_filter_project: NULL output");
        int32_t dt = col->dtype;
        s = lower_expr(values[j], col->dtype, P.vals[j], dt);
        if (s != FQ_OK) return s;
        if (fqc::dtype_size(dt) != 8) return fqc::fail(FQ_E_UNSUPPORTED, "fused projection outputs are 64-bit");
        P.chain[j] = values[j].n_steps > 0;
        P.dtypes[j] = dt;
        P.out[j] = d_out[j];
    }
    return FQ_OK;
}

}  // namespace
}  // namespace fqk

extern "C" {

size_t fq_filter_project_workspace_bytes(int64_t len) {
    const fqk::ProjWs w = fqk::proj_ws(nullptr, len < 0 ? 0 : len);
    return (size_t)(2 + 16 + w.ntiles) * sizeof(uint64_t);
}

fq_status fq_filter_project(const fq_col *col, const fq_pred *pred, const fq_expr *values, int32_t n_out,
                            void *const *d_out, int64_t *out_len, void *d_ws, size_t ws_bytes, void *stream) {
    using namespace fqk;
    if (!out_len) return fqc::fail(FQ_E_INVALID, "fq_filter_project: NULL out_len");
    *out_len = 0;
    ProjLaunch P;
    fq_status s = lower_projection(col, pred, values, n_out, d_out, stream, P);
    if (s != FQ_OK) return s;
    if (n_out < 1) return fqc::fail(FQ_E_INVALID, "fq_filter_project: no outputs");
    if (!jit_project_available())
        return fqc::fail(FQ_E_UNSUPPORTED, "fq_filter_project: hipRTC unavailable or the JIT is off");
    if ((s = jit_project_prepare(col->dtype, P)) != FQ_OK) return s;
    const int64_t n = col->len;
    if (n == 0) return FQ_OK;
    if (!d_ws || ws_bytes < fq_filter_project_workspace_bytes(n))
        return fqc::fail(FQ_E_INVALID, "fq_filter_project: workspace too small");
    const ProjWs w = proj_ws(d_ws, n);
    hipStream_t st = P.stream;
    uint64_t local[2] = {0, 0};
    uint64_t *const pinned = fqc::host_staging();
    uint64_t *const host = pinned ? pinned : local;  // kept rows, flag words
    host[0] = host[1] = 0;
    if (P.pred.kind == FQ_PRED_NONE) {
        FQ_HIP_TRY(hipMemsetAsync(w.flags, 0, 2 * sizeof(uint32_t), st));
        if ((s = jit_project_map(col->dtype, P, w.flags + 1)) != FQ_OK) return s;
        FQ_HIP_TRY(hipMemcpyAsync(&host[1], w.flags, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        host[0] = (uint64_t)n;
    } else {
        FQ_HIP_TRY(hipMemsetAsync(d_ws, 0, fq_filter_project_workspace_bytes(n), st));
        if ((s = jit_project_select(col->dtype, P, P.pred.kind == FQ_PRED_BITMAP ? P.pred.bitmap : nullptr, w.status,
                                    w.ticket, w.flags, w.total)) != FQ_OK)
            return s;
        FQ_HIP_TRY(hipMemcpyAsync(host, w.total, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));  // total + flag words
    }
    FQ_HIP_TRY(hipStreamSynchronize(st));
    const uint32_t pred_flags = (uint32_t)(host[1] & 0xffffffffu), val_flags = (uint32_t)(host[1] >> 32);
    if ((s = flag_error(pred_flags)) != FQ_OK) return s;  // FilterTransform runs first
    if ((s = flag_error(val_flags)) != FQ_OK) return s;
    *out_len = (int64_t)host[0];
    return FQ_OK;
}

size_t fq_filter_project_blocks_workspace_bytes(void) { return 3 * sizeof(uint64_t); }  // total, flags, ticket

}  // extern "C"

namespace fqk {

fq_status filter_project_blocks_enqueue(const fq_col *col, int64_t block_rows, const fq_pred *pred,
                                        const fq_expr *values, int32_t n_out, void *const *d_out, int64_t *d_counts,
                                        uint64_t *h_result, uint64_t *d_result, void *d_ws, size_t ws_bytes,
                                        void *ev_start, void *ev_end, void *stream) {
    static_assert(FQ_PROJECT_MIN_BLOCK_ROWS == kProjectBlockTile, "the ABI's minimum block is the kernel's tile");
    if (!h_result) return fqc::fail(FQ_E_INVALID, "fq_filter_project_blocks: NULL result words");
    // a resident call's words are the caller's until the hand-off writes them
    // (the engine keeps a sentinel there to poll for)
    if (!d_result) h_result[0] = h_result[1] = 0;
    if (block_rows < FQ_PROJECT_MIN_BLOCK_ROWS)
        return fqc::fail(FQ_E_INVALID, "fq_filter_project_blocks: block_rows below FQ_PROJECT_MIN_BLOCK_ROWS");
    ProjLaunch P;
    fq_status s = lower_projection(col, pred, values, n_out, d_out, stream, P);
    if (s != FQ_OK) return s;
    if (n_out < 1) return fqc::fail(FQ_E_INVALID, "fq_filter_project_blocks: no outputs");
    if (!jit_project_available())
        return fqc::fail(FQ_E_UNSUPPORTED, "fq_filter_project_blocks: hipRTC unavailable or the JIT is off");
    if ((s = jit_project_prepare(col->dtype, P)) != FQ_OK) return s;
    const int64_t n = col->len;
    if (n == 0) return FQ_OK;
    if (!d_counts) return fqc::fail(FQ_E_INVALID, "fq_filter_project_blocks: NULL block counts");
    if (!d_ws || ws_bytes < fq_filter_project_blocks_workspace_bytes())
        return fqc::fail(FQ_E_INVALID, "fq_filter_project_blocks: workspace too small");
    uint64_t *const total = (uint64_t *)d_ws;
    uint32_t *const flags = (uint32_t *)(total + 1);
    uint32_t *const ticket = (uint32_t *)(total + 2);
    hipStream_t st = P.stream;
    const int64_t nb = block_rows >= n ? 1 : (n + block_rows - 1) / block_rows;
    const bool resident = d_result != nullptr;
    if (!resident) FQ_HIP_TRY(hipMemsetAsync(d_ws, 0, fq_filter_project_blocks_workspace_bytes(), st));
    if (ev_start) FQ_HIP_TRY(hipEventRecord((hipEvent_t)ev_start, st));
    if (P.pred.kind == FQ_PRED_NONE) {  // every row kept: outputs in place, counts = block lengths
        if ((s = jit_project_map(col->dtype, P, flags + 1)) != FQ_OK) return s;
        hipLaunchKernelGGL(block_lengths_kernel, dim3((unsigned)std::min<int64_t>((nb + 255) / 256, 4096)), dim3(256), 0,
                           st, d_counts, nb, std::min(block_rows, n), n);
        FQ_HIP_TRY(hipGetLastError());
        if (ev_end) FQ_HIP_TRY(hipEventRecord((hipEvent_t)ev_end, st));
        FQ_HIP_TRY(hipMemcpyAsync(&h_result[1], flags, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        h_result[0] = (uint64_t)n;
        // the map kernel used the flag words: zero again for a resident workspace
        if (resident) FQ_HIP_TRY(hipMemsetAsync(d_ws, 0, fq_filter_project_blocks_workspace_bytes(), st));
        return FQ_OK;
    }
    if ((s = jit_project_blocks(col->dtype, P, block_rows, P.pred.kind == FQ_PRED_BITMAP ? P.pred.bitmap : nullptr,
                                d_counts, flags, total, ticket)) != FQ_OK)
        return s;
    if (ev_end) FQ_HIP_TRY(hipEventRecord((hipEvent_t)ev_end, st));
    if (resident) {
        hipLaunchKernelGGL(project_hand_off_kernel, dim3(1), dim3(64), 0, st, total, d_result);
        FQ_HIP_TRY(hipGetLastError());
    } else {
        FQ_HIP_TRY(hipMemcpyAsync(h_result, total, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    }
    return FQ_OK;
}

fq_status filter_project_blocks_result(const uint64_t *h_result, int64_t *out_len) {
    if (!h_result || !out_len) return fqc::fail(FQ_E_INVALID, "fq_filter_project_blocks: NULL result");
    *out_len = 0;
    const uint32_t pred_flags = (uint32_t)(h_result[1] & 0xffffffffu), val_flags = (uint32_t)(h_result[1] >> 32);
    fq_status s;
    if ((s = flag_error(pred_flags)) != FQ_OK) return s;  // FilterTransform runs first
    if ((s = flag_error(val_flags)) != FQ_OK) return s;
    *out_len = (int64_t)h_result[0];
    return FQ_OK;
}

}  // namespace fqk

extern "C" {

fq_status fq_filter_project_blocks(const fq_col *col, int64_t block_rows, const fq_pred *pred, const fq_expr *values,
                                   int32_t n_out, void *const *d_out, int64_t *d_counts, int64_t *out_len, void *d_ws,
                                   size_t ws_bytes, void *stream) {
    if (!out_len) return fqc::fail(FQ_E_INVALID, "fq_filter_project_blocks: NULL out_len");
    *out_len = 0;
    uint64_t local[2] = {0, 0};
    uint64_t *const pinned = fqc::host_staging();
    uint64_t *const host = pinned ? pinned : local;  // kept rows, flag words
    fq_status s = fqk::filter_project_blocks_enqueue(col, block_rows, pred, values, n_out, d_out, d_counts, host,
                                                     nullptr, d_ws, ws_bytes, nullptr, nullptr, stream);
    if (s != FQ_OK) return s;
    FQ_HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return fqk::filter_project_blocks_result(host, out_len);
}

size_t fq_blocks_compact_workspace_bytes(int64_t n_blocks) {
    const int64_t nb = n_blocks < 1 ? 1 : n_blocks;
    const int64_t chunks = (nb + fqk::kCompactChunk - 1) / fqk::kCompactChunk;
    return (size_t)(nb + 1 + chunks + 1) * sizeof(int64_t);
}

fq_status fq_blocks_compact(int32_t n_cols, const void *const *d_in, int64_t len, int64_t block_rows,
                            const int64_t *d_counts, void *const *d_out, int64_t *out_len, void *d_ws, size_t ws_bytes,
                            void *stream) {
    using namespace fqk;
    if (out_len) *out_len = 0;
    if (n_cols < 0 || n_cols > FQ_MAX_PROJECT || (n_cols > 0 && (!d_in || !d_out)))
        return fqc::fail(FQ_E_INVALID, "fq_blocks_compact: bad column list");
    if (len < 0 || block_rows < 1) return fqc::fail(FQ_E_INVALID, "fq_blocks_compact: bad geometry");
    if (len == 0) return FQ_OK;
    const int64_t nb = (len + block_rows - 1) / block_rows;
    if (!d_counts || !d_ws) return fqc::fail(FQ_E_INVALID, "fq_blocks_compact: NULL buffer");
    if (ws_bytes < fq_blocks_compact_workspace_bytes(nb))
        return fqc::fail(FQ_E_INVALID, "fq_blocks_compact: workspace too small");
    CompactCols cols{};
    for (int j = 0; j < n_cols; ++j) {
        if (!d_in[j] || !d_out[j]) return fqc::fail(FQ_E_INVALID, "fq_blocks_compact: NULL column");
        cols.in[j] = (const uint64_t *)d_in[j];
        cols.out[j] = (uint64_t *)d_out[j];
    }
    hipStream_t st = (hipStream_t)stream;
    int64_t *const offs = (int64_t *)d_ws;  // nb + 1
    int64_t *const sums = offs + nb + 1;    // chunks + 1
    const int64_t chunks = (nb + kCompactChunk - 1) / kCompactChunk;
    hipLaunchKernelGGL(blocks_chunk_sums_kernel, dim3((unsigned)chunks), dim3(kCompactChunk), 0, st, d_counts, nb, sums);
    FQ_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(blocks_scan_sums_kernel, dim3(1), dim3(kCompactChunk), 0, st, sums, chunks);
    FQ_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(blocks_offsets_kernel, dim3((unsigned)chunks), dim3(kCompactChunk), 0, st, d_counts, nb, sums,
                       offs);
    FQ_HIP_TRY(hipGetLastError());
    if (n_cols > 0) {
        hipLaunchKernelGGL(blocks_copy_kernel, dim3((unsigned)std::min<int64_t>(nb, 1 << 20)), dim3(256), 0, st, cols,
                           n_cols, d_counts, offs, nb, block_rows);
        FQ_HIP_TRY(hipGetLastError());
    }
    if (!out_len) return FQ_OK;
    uint64_t local = 0;
    uint64_t *const pinned = fqc::host_staging();
    uint64_t *const total = pinned ? pinned : &local;
    FQ_HIP_TRY(hipMemcpyAsync(total, offs + nb, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    FQ_HIP_TRY(hipStreamSynchronize(st));
    *out_len = (int64_t)*total;
    return FQ_OK;
}

fq_status fq_predicate_bitmap(const fq_col *col, const fq_pred *pred, uint64_t *d_bitmap, uint32_t *d_flag,
                              void *stream) {
    using namespace fqk;
    ProjLaunch P;
    fq_status s = lower_projection(col, pred, nullptr, 0, nullptr, stream, P);
    if (s != FQ_OK) return s;
    if (P.pred.kind != FQ_PRED_EXPR && P.pred.kind != FQ_PRED_TREE)
        return fqc::fail(FQ_E_INVALID, "fq_predicate_bitmap: needs an FQ_PRED_EXPR or FQ_PRED_TREE predicate");
    if (!jit_project_available())
        return fqc::fail(FQ_E_UNSUPPORTED, "fq_predicate_bitmap: hipRTC unavailable or the JIT is off");
    P.n_out = 1;  // the module's shape needs one output; the bits kernel writes none
    P.dtypes[0] = col->dtype;
    if ((s = jit_project_prepare(col->dtype, P)) != FQ_OK) return s;
    if (col->len == 0) return FQ_OK;
    if (!d_bitmap || !d_flag) return fqc::fail(FQ_E_INVALID, "fq_predicate_bitmap: NULL buffer");
    FQ_HIP_TRY(hipMemsetAsync(d_flag, 0, sizeof(uint32_t), P.stream));
    if ((s = jit_project_bits(col->dtype, P, d_bitmap, d_flag)) != FQ_OK) return s;
    uint32_t local = 0;
    uint64_t *const pinned = fqc::host_staging();
    uint32_t *const h = pinned ? (uint32_t *)pinned : &local;
    FQ_HIP_TRY(hipMemcpyAsync(h, d_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, P.stream));
    FQ_HIP_TRY(hipStreamSynchronize(P.stream));
    return flag_error(*h);
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
    const int64_t ngroups = (ntiles + kGroupTiles - 1) / kGroupTiles;
    uint64_t *intra = (uint64_t *)d_ws;
    uint64_t *gpre = intra + ntiles;
    hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)ngroups), dim3(kTileWords), 0, st, d_bitmap, n, ntiles,
                       intra, gpre);
    FQ_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, gpre, ngroups);
    FQ_HIP_TRY(hipGetLastError());
    switch (esz) {
        case 1:
            hipLaunchKernelGGL(compact_scatter_kernel<uint8_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0, st,
                               (const uint8_t *)in->data, d_bitmap, n, intra, gpre, (uint8_t *)d_out);
            break;
        case 2:
            hipLaunchKernelGGL(compact_scatter_kernel<uint16_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0, st,
                               (const uint16_t *)in->data, d_bitmap, n, intra, gpre, (uint16_t *)d_out);
            break;
        case 4:
            hipLaunchKernelGGL(compact_scatter_kernel<uint32_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0, st,
                               (const uint32_t *)in->data, d_bitmap, n, intra, gpre, (uint32_t *)d_out);
            break;
        default:
            if (((uintptr_t)in->data & 15u) == 0 && ((uintptr_t)d_out & 15u) == 0)
                hipLaunchKernelGGL(compact_scatter_lds_kernel<uint64_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0,
                                   st, (const uint64_t *)in->data, d_bitmap, n, intra, gpre, (uint64_t *)d_out);
            else if (((uintptr_t)in->data & 15u) == 0)
                hipLaunchKernelGGL(compact_scatter_vec_kernel<uint64_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0,
                                   st, (const uint64_t *)in->data, d_bitmap, n, intra, gpre, (uint64_t *)d_out);
            else
                hipLaunchKernelGGL(compact_scatter_kernel<uint64_t>, dim3((unsigned)ntiles), dim3(kTileWords), 0,
                                   st, (const uint64_t *)in->data, d_bitmap, n, intra, gpre, (uint64_t *)d_out);
            break;
    }
    FQ_HIP_TRY(hipGetLastError());
    uint64_t local = 0;
    uint64_t *const pinned = fqc::host_staging();
    uint64_t *const total = pinned ? pinned : &local;
    FQ_HIP_TRY(hipMemcpyAsync(total, gpre + ngroups, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    FQ_HIP_TRY(hipStreamSynchronize(st));
    *out_len = (int64_t)*total;
    return FQ_OK;
}

}  // extern "C"
