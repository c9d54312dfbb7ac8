// Probe (not product code): the ceiling of Filter -> Projection on MI355X.
// Same tile shape and store pattern as fq_jit_pselect (256 threads x 32 rows
// of u64 per tile, ballots + in-tile scan, outputs x+1 and x/2 of the rows
// with x % 8 < 3 at base + rank) but every tile's base comes from a prefix
// array computed beforehand: no ticket, no look-back.  Also the plain read,
// map and copy rates of the same 10 GB column.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 select_ideal.hip -o select_ideal
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

typedef unsigned long long u64;
typedef unsigned int u32;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int TH = 256, ROWS = 32, TILE = TH * ROWS, WAVES = TH / 64;

__global__ void iota(u64 *p, long long n) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = (u64)i;
}

__global__ void __launch_bounds__(TH) tile_counts(const u64 *__restrict__ col, long long n, u32 *__restrict__ cnt) {
    const long long t = blockIdx.x;
    u32 c = 0;
    for (int k = 0; k < ROWS; ++k) {
        const long long r = t * TILE + (long long)k * TH + threadIdx.x;
        if (r < n && (col[r] % 8) < 3) ++c;
    }
    __shared__ u32 s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    atomicAdd(&s, c);
    __syncthreads();
    if (threadIdx.x == 0) cnt[t] = s;
}

// pselect's body with the base given
template <bool NT_LOAD>
__global__ void __launch_bounds__(TH) ideal_select(const u64 *__restrict__ col, long long n, const u64 *__restrict__ tbase,
                                                  u64 *__restrict__ o1, u64 *__restrict__ o2) {
    __shared__ u64 bal[ROWS][WAVES];
    __shared__ u32 off[ROWS * WAVES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long ntiles = (n + TILE - 1) / TILE;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        u64 x[ROWS];
        const long long r0 = t * TILE + tid;
#pragma unroll
        for (int k = 0; k < ROWS; ++k) {
            const long long r = r0 + (long long)k * TH;
            x[k] = r < n ? (NT_LOAD ? __builtin_nontemporal_load(col + r) : col[r]) : 0ull;
        }
        const u64 base = tbase[t];
#pragma unroll
        for (int k = 0; k < ROWS; ++k) {
            const long long r = r0 + (long long)k * TH;
            const bool p = r < n && (x[k] % 8) < 3;
            const u64 b = __ballot(p);
            if (lane == 0) {
                bal[k][wave] = b;
                off[k * WAVES + wave] = (u32)__popcll(b);
            }
        }
        __syncthreads();
        if (wave == 0) {
            constexpr int NE = ROWS * WAVES, PER = (NE + 63) / 64;
            u32 cv[PER], tot = 0;
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int i = lane * PER + q;
                cv[q] = i < NE ? off[i] : 0u;
                tot += cv[q];
            }
            u32 incl = tot;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const u32 v = (u32)__shfl_up((int)incl, o, 64);
                if (lane >= o) incl += v;
            }
            u32 run = incl - tot;
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                const int i = lane * PER + q;
                if (i < NE) off[i] = run;
                run += cv[q];
            }
        }
        __syncthreads();
        const u64 lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
        for (int k = 0; k < ROWS; ++k) {
            const u64 b = bal[k][wave];
            if ((b >> lane) & 1ull) {
                const u64 pos = base + off[k * WAVES + wave] + (u32)__popcll(b & lt);
                o1[pos] = x[k] + 1;
                o2[pos] = x[k] / 2;
            }
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) read_sum(const u64 *__restrict__ col, long long n, u64 *sink) {
    u64 acc = 0;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        acc += __builtin_nontemporal_load(col + i);
    if (acc == 0x1234567ull) sink[0] = acc;
}

typedef u64 u64x2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) map2(const u64x2 *__restrict__ col, long long npair, u64x2 *__restrict__ o1,
                                            u64x2 *__restrict__ o2) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < npair; i += (long long)gridDim.x * 256) {
        const u64x2 v = __builtin_nontemporal_load(col + i);
        o1[i] = v + (u64)1;
        o2[i] = v / (u64)2;
    }
}
__global__ void __launch_bounds__(256) copy1(const u64x2 *__restrict__ col, long long npair, u64x2 *__restrict__ o1) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < npair; i += (long long)gridDim.x * 256)
        o1[i] = __builtin_nontemporal_load(col + i);
}

int main() {
    const long long n = 1250000000;  // 10 GB of u64
    u64 *col, *o1, *o2, *tb, *sink;
    u32 *cnt;
    const long long ntiles = (n + TILE - 1) / TILE;
    CK(hipMalloc(&col, n * 8));
    CK(hipMalloc(&o1, n * 8));
    CK(hipMalloc(&o2, n * 8));
    CK(hipMalloc(&tb, ntiles * 8));
    CK(hipMalloc(&cnt, ntiles * 4));
    CK(hipMalloc(&sink, 8));
    hipLaunchKernelGGL(iota, dim3(4096), dim3(256), 0, 0, col, n);
    hipLaunchKernelGGL(tile_counts, dim3((unsigned)ntiles), dim3(TH), 0, 0, col, n, cnt);
    std::vector<u32> hc(ntiles);
    std::vector<u64> hb(ntiles);
    CK(hipMemcpy(hc.data(), cnt, ntiles * 4, hipMemcpyDeviceToHost));
    u64 run = 0;
    for (long long t = 0; t < ntiles; ++t) {
        hb[t] = run;
        run += hc[t];
    }
    const u64 kept = run;
    CK(hipMemcpy(tb, hb.data(), ntiles * 8, hipMemcpyHostToDevice));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        float best = 1e9, sum = 0;
        for (int r = 0; r < 7; ++r) {
            CK(hipEventRecord(e0));
            fn();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
            sum += ms;
        }
        return best;
    };
    const double sel_bytes = 8.0 * n + 16.0 * kept;
    printf("kept %llu of %lld (algorithmic select bytes %.2f GB)\n", kept, n, sel_bytes / 1e9);
    for (int w : {1, 2, 3, 4, 5, 6, 8}) {
        const int grid = cus * w;
        float ms = timeit([&] { hipLaunchKernelGGL(ideal_select<true>, dim3(grid), dim3(TH), 0, 0, col, n, tb, o1, o2); });
        printf("ideal select (nt loads), %d WG/CU: %.3f ms = %.2f TB/s algorithmic\n", w, ms, sel_bytes / ms / 1e9);
        ms = timeit([&] { hipLaunchKernelGGL(ideal_select<false>, dim3(grid), dim3(TH), 0, 0, col, n, tb, o1, o2); });
        printf("ideal select (plain loads), %d WG/CU: %.3f ms = %.2f TB/s algorithmic\n", w, ms, sel_bytes / ms / 1e9);
    }
    // spot check the last tile's outputs
    std::vector<u64> h1(16);
    CK(hipMemcpy(h1.data(), o1 + kept - 16, 16 * 8, hipMemcpyDeviceToHost));
    u64 want = n - 1;
    while (want % 8 >= 3) --want;
    printf("last kept row + 1: %llu (expect %llu)\n", h1[15], want + 1);
    for (int w : {2, 4, 8}) {
        float ms = timeit([&] { hipLaunchKernelGGL(read_sum, dim3(cus * w), dim3(256), 0, 0, col, n, sink); });
        printf("read only, %d WG/CU: %.3f ms = %.2f TB/s\n", w, ms, 8.0 * n / ms / 1e9);
        ms = timeit([&] { hipLaunchKernelGGL(map2, dim3(cus * w), dim3(256), 0, 0, (const u64x2 *)col, n / 2, (u64x2 *)o1, (u64x2 *)o2); });
        printf("map x -> (x+1, x/2), %d WG/CU: %.3f ms = %.2f TB/s\n", w, ms, 24.0 * n / ms / 1e9);
        ms = timeit([&] { hipLaunchKernelGGL(copy1, dim3(cus * w), dim3(256), 0, 0, (const u64x2 *)col, n / 2, (u64x2 *)o1); });
        printf("copy, %d WG/CU: %.3f ms = %.2f TB/s\n", w, ms, 16.0 * n / ms / 1e9);
    }
    return 0;
}
