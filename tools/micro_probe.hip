// micro_probe.hip — calibration microbenchmarks for the scan design (not product code).
// Random 8-byte gathers from a global table of varying size (L2 / MALL / HBM resident),
// and random 4-byte reads from an LDS table, reported as probes/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int B>
__global__ void k_gather(const uint64_t* __restrict__ t, uint32_t mask, uint32_t iters, uint64_t* out) {
    uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B9u + 12345u;
    uint64_t acc = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        uint64_t v[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            v[j] = t[x & mask];
        }
#pragma unroll
        for (int j = 0; j < B; ++j) acc += v[j];
    }
    if (acc == 0x1234567) out[0] = acc;
}

// LDS random reads: table of `words` u32 in LDS
__global__ void k_lds(uint32_t wmask, uint32_t iters, uint32_t* out) {
    extern __shared__ uint32_t tab[];
    for (uint32_t i = threadIdx.x; i <= wmask; i += blockDim.x) tab[i] = i * 2654435761u;
    __syncthreads();
    uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B9u + 12345u;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            v[j] = tab[x & wmask];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += v[j];
    }
    if (acc == 0x1234567) out[0] = acc;
}

// xorshift-only control (same VALU work, no memory)
__global__ void k_alu(uint32_t iters, uint32_t* out) {
    uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B9u + 12345u;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; acc += x; }
    }
    if (acc == 0x1234567) out[0] = acc;
}

int main() {
    uint64_t* t;
    const size_t maxb = 256ull << 20;
    CK(hipMalloc(&t, maxb));
    CK(hipMemset(t, 1, maxb));
    uint64_t* out;
    CK(hipMalloc(&out, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int cus = 256;
    for (int wpc : {8, 16, 32}) {
        for (size_t tb : {64ull << 10, 512ull << 10, 1ull << 20, 2ull << 20, 4ull << 20, 16ull << 20, 128ull << 20}) {
            const uint32_t mask = (uint32_t)(tb / 8 - 1);
            const uint32_t iters = 64;
            const int blocks = cus * wpc / 4;
            hipLaunchKernelGGL(k_gather<16>, dim3(blocks), dim3(256), 0, 0, t, mask, iters, out);
            CK(hipEventRecord(a));
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_gather<16>, dim3(blocks), dim3(256), 0, 0, t, mask, iters, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            const double probes = 5.0 * blocks * 256.0 * iters * 16;
            printf("gather8  waves/CU %2d table %7zu KiB: %.1f Gprobe/s  (%.2f per clk per XCD @2.4GHz)\n", wpc, tb >> 10,
                   probes / ms / 1e6, probes / (ms * 1e-3) / 8 / 2.4e9);
        }
    }
    for (int wpc : {4, 8, 16}) {
        for (uint32_t kb : {16u, 64u, 128u}) {
            const uint32_t wm = kb * 256 - 1;
            const uint32_t iters = 512;
            const int blocks = cus * wpc / 4;
            hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(256), kb << 10, 0, wm, iters, (uint32_t*)out);
            CK(hipEventRecord(a));
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(256), kb << 10, 0, wm, iters, (uint32_t*)out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            const double probes = 5.0 * blocks * 256.0 * iters * 8;
            printf("lds32    waves/CU %2d (resident may be lower) table %3u KiB: %.1f Gprobe/s (%.2f per clk per CU)\n", wpc, kb,
                   probes / ms / 1e6, probes / (ms * 1e-3) / 256 / 2.4e9);
        }
    }
    {
        const uint32_t iters = 512;
        const int blocks = cus * 16 / 4;
        hipLaunchKernelGGL(k_alu, dim3(blocks), dim3(256), 0, 0, iters, (uint32_t*)out);
        CK(hipEventRecord(a));
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_alu, dim3(blocks), dim3(256), 0, 0, iters, (uint32_t*)out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double ops = 5.0 * blocks * 256.0 * iters * 8 * 7;  // 6 xorshift ops + 1 add
        printf("alu      %.1f Tlane-op/s (%.1f lane-ops per clk per CU @2.4GHz)\n", ops / ms / 1e9, ops / (ms * 1e-3) / 256 / 2.4e9);
    }
    return 0;
}
