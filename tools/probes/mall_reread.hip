// Probe (not product code): does a chunk read right after it was streamed from
// HBM come back from the 256 MB Infinity Cache (MALL), and how fast?
// Streams a 10 GB buffer in chunks of C MB: kernel A reads chunk i, kernel B
// re-reads chunk i (both non-temporal 16-B loads, tile-contiguous), and
// reports total time against a single pass.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) readk(const u32x4 *__restrict__ p, long long nvec, unsigned *__restrict__ sink) {
    unsigned acc = 0;
    const long long TV = 4 * 256;
    const long long ntiles = nvec / TV;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const long long base = t * TV + threadIdx.x;
        u32x4 r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = NT ? __builtin_nontemporal_load(p + base + k * 256) : p[base + k * 256];
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= r[k].x ^ r[k].y ^ r[k].z ^ r[k].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main() {
    const size_t total = 10ull << 30;
    u32x4 *buf;
    unsigned *sink;
    CK(hipMalloc(&buf, total));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(buf, 1, total));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 2;
    auto timeit = [&](auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            fn();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        return best;
    };
    const long long nvec = (long long)(total / 16);
    float one = timeit([&] { readk<true><<<grid, 256>>>(buf, nvec, sink); });
    printf("single pass 10 GB: %.3f ms (%.2f TB/s)\n", one, total / one / 1e9);
    for (int mb : {32, 64, 128, 192, 256}) {
        for (int nt2 = 0; nt2 < 2; ++nt2) {
            const long long cv = (long long)mb << 20 >> 4;
            const long long nch = nvec / cv;
            float t2 = timeit([&] {
                for (long long c = 0; c < nch; ++c) {
                    readk<false><<<grid, 256>>>(buf + c * cv, cv, sink);  // temporal: keep it in the caches
                    if (nt2) readk<true><<<grid, 256>>>(buf + c * cv, cv, sink);
                    else readk<false><<<grid, 256>>>(buf + c * cv, cv, sink);
                }
            });
            float t1 = timeit([&] {
                for (long long c = 0; c < nch; ++c) readk<false><<<grid, 256>>>(buf + c * cv, cv, sink);
            });
            printf("chunk %3d MB: read once %.3f ms, read+reread(%s) %.3f ms -> reread cost %.3f ms = %.2f TB/s\n", mb, t1,
                   nt2 ? "nt" : "temporal", t2, t2 - t1, (double)nch * cv * 16 / (t2 - t1) / 1e9);
        }
    }
    return 0;
}
