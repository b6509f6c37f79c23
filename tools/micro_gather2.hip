// micro_gather2.hip — round-2 calibration for the C3 scan redesign (not product code).
//   1. random gathers from an L2-resident table: 4-B / 8-B, plain vs nt vs sc1 (L1 bypass)
//   2. the chunk-select pattern: 64 register-resident word indices per thread, one LDS
//      chunk at a time, exec-masked reads (what a chunk-streamed filter costs per position)
//   3. streaming a 448 KiB table through a 112 KiB LDS chunk (L2 -> LDS rate per CU)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

enum { kPlain = 0, kNt = 1, kSc1 = 2 };

template <typename T, int MODE>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (MODE == kNt) return __builtin_nontemporal_load(p);
    else if constexpr (MODE == kSc1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}

template <typename T, int MODE, int B>
__global__ void k_gather(const T* __restrict__ t, uint32_t mask, uint32_t iters, uint64_t* out) {
    uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B9u + 12345u;
    uint64_t acc = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        T v[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            v[j] = ld<T, MODE>(t + (x & mask));
        }
#pragma unroll
        for (int j = 0; j < B; ++j) acc += v[j];
    }
    if (acc == 0x1234567) out[0] = acc;
}

// Chunk select: thread holds K word indices into a virtual table of C chunks x CW words;
// per chunk, exec-masked LDS reads of the indices that fall in it.
template <int K, int C>
__global__ __launch_bounds__(512) void k_select(uint32_t cw, uint32_t iters, uint32_t* out) {
    extern __shared__ uint32_t tab[];
    for (uint32_t i = threadIdx.x; i < cw; i += blockDim.x) tab[i] = i * 2654435761u;
    __syncthreads();
    uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B9u + 12345u;
    uint32_t acc = 0;
    const uint32_t span = cw << 15;
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t g[K], w[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            g[k] = (uint32_t)(((uint64_t)x * (C * cw)) >> 32) << 15;
            w[k] = 0;
        }
        for (int c = 0; c < C; ++c) {
            const uint32_t base = (uint32_t)c * span;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t d = g[k] - base;
                if (d < span) w[k] = tab[d >> 15];
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc += w[k];
    }
    if (acc == 0x1234567) out[0] = acc;
}

// Stream a table of C*cw words through one LDS chunk of cw words, `iters` passes.
__global__ __launch_bounds__(512) void k_stream(const uint4* __restrict__ t, uint32_t cw, uint32_t C, uint32_t iters,
                                                uint32_t* out) {
    extern __shared__ uint4 buf[];
    const uint32_t n4 = cw / 4;
    uint32_t acc = 0;
    for (uint32_t it = 0; it < iters; ++it)
        for (uint32_t c = 0; c < C; ++c) {
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < n4; i += blockDim.x) buf[i] = t[c * n4 + i];
            __syncthreads();
            acc += buf[(threadIdx.x * 37 + it) % n4].x;
        }
    if (acc == 0x1234567) out[0] = acc;
}

template <typename F>
static double time_ms(F&& launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipEventRecord(a));
    for (int r = 0; r < 5; ++r) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

int main() {
    uint8_t* t;
    CK(hipMalloc(&t, 64 << 20));
    CK(hipMemset(t, 1, 64 << 20));
    uint64_t* out;
    CK(hipMalloc(&out, 64));
    const int cus = 256;
    const uint32_t iters = 64;
    for (size_t tb : {512ull << 10, 2ull << 20}) {
        const int blocks = cus * 16 / 4;
        const double probes = (double)blocks * 256 * iters * 16;
#define G(T, M, name)                                                                                          \
    {                                                                                                          \
        const uint32_t mask = (uint32_t)(tb / sizeof(T) - 1);                                                  \
        double ms = time_ms([&] {                                                                              \
            hipLaunchKernelGGL((k_gather<T, M, 16>), dim3(blocks), dim3(256), 0, 0, (const T*)t, mask, iters, out); \
        });                                                                                                    \
        printf("gather %-10s table %5zu KiB: %7.1f Gprobe/s\n", name, tb >> 10, probes / ms / 1e6);           \
    }
        G(uint32_t, kPlain, "u32 plain");
        G(uint32_t, kNt, "u32 nt");
        G(uint32_t, kSc1, "u32 sc1");
        G(uint64_t, kPlain, "u64 plain");
        G(uint64_t, kNt, "u64 nt");
        G(uint64_t, kSc1, "u64 sc1");
    }
    // chunk select: 1 WG of 512 threads per CU, 112 KiB chunk
    {
        const uint32_t cw = 28672, it = 64;
        CK(hipFuncSetAttribute((const void*)k_select<64, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, cw * 4));
        CK(hipFuncSetAttribute((const void*)k_select<32, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, cw * 4));
        double ms = time_ms([&] { hipLaunchKernelGGL((k_select<64, 4>), dim3(cus), dim3(512), cw * 4, 0, cw, it, (uint32_t*)out); });
        double pos = (double)cus * 512 * it * 64;
        printf("select K=64 C=4 512 thr: %.3f ms, %.1f Gpos/s, %.2f cyc/pos/CU\n", ms, pos / ms / 1e6,
               ms * 1e-3 * 2.4e9 * cus / pos);
        ms = time_ms([&] { hipLaunchKernelGGL((k_select<32, 4>), dim3(cus), dim3(512), cw * 4, 0, cw, it, (uint32_t*)out); });
        pos = (double)cus * 512 * it * 32;
        printf("select K=32 C=4 512 thr: %.3f ms, %.1f Gpos/s, %.2f cyc/pos/CU\n", ms, pos / ms / 1e6,
               ms * 1e-3 * 2.4e9 * cus / pos);
    }
    // streaming 4 x 112 KiB chunks per pass
    {
        const uint32_t cw = 28672, C = 4, it = 32;
        CK(hipFuncSetAttribute((const void*)k_stream, hipFuncAttributeMaxDynamicSharedMemorySize, cw * 4));
        double ms = time_ms([&] { hipLaunchKernelGGL(k_stream, dim3(cus), dim3(512), cw * 4, 0, (const uint4*)t, cw, C, it, (uint32_t*)out); });
        const double bytes = (double)cus * it * C * cw * 4;
        printf("stream 4x112KiB via LDS, 1 WG/CU: %.3f ms, %.1f GB/s per CU, %.2f TB/s chip\n", ms,
               bytes / cus / ms / 1e6, bytes / ms / 1e9);
    }
    return 0;
}
