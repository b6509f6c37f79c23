// micro_read.hip — HBM read ceiling on this box (calibration, not product code).
// Streams a 4 GiB buffer with 16-byte loads per lane, each wave reading K KiB
// contiguous per iteration (K loads in flight per lane), plain or non-temporal,
// reporting GB/s; plus the same stream with the signature's byte-sum work
// (udot4) on the loaded data to show whether light VALU work changes the rate.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int K, bool NT, bool WORK>
__global__ __launch_bounds__(256) void k_read(const uint8_t* __restrict__ buf, uint64_t nchunks, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    uint32_t acc = 0;
    for (uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < nchunks; c += nw) {
        const uint8_t* p = buf + c * (K * 1024ull) + lane * 16;
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (NT) v[k] = __builtin_nontemporal_load((const u32x4*)(p + k * 1024));
            else v[k] = *(const u32x4*)(p + k * 1024);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (WORK) {
                acc = __builtin_amdgcn_udot4(v[k].x, 0x01010101u, acc, false);
                acc = __builtin_amdgcn_udot4(v[k].y, 0x01010101u, acc, false);
                acc = __builtin_amdgcn_udot4(v[k].z, 0x01010101u, acc, false);
                acc = __builtin_amdgcn_udot4(v[k].w, 0x01010101u, acc, false);
            } else {
                acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
            }
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

template <int K, bool NT, bool WORK>
static void run(const uint8_t* d, uint64_t bytes, uint32_t* o, int grid, const char* name) {
    const uint64_t nchunks = bytes / (K * 1024ull);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_read<K, NT, WORK>), dim3(grid), dim3(256), 0, 0, d, nchunks, o);
    CK(hipEventRecord(a));
    const int it = 20;
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL((k_read<K, NT, WORK>), dim3(grid), dim3(256), 0, 0, d, nchunks, o);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= it;
    printf("%-28s grid %6d: %.3f ms  %.1f GB/s\n", name, grid, ms, bytes / (ms * 1e-3) / 1e9);
}

int main() {
    const uint64_t bytes = 4ull << 30;
    uint8_t* d;
    uint32_t* o;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&o, 64));
    CK(hipMemset(d, 0x5A, bytes));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int g : {cus * 8, cus * 16, 1 << 20 >> 2}) {
        run<1, false, false>(d, bytes, o, g, "read K=1 plain");
        run<4, false, false>(d, bytes, o, g, "read K=4 plain");
        run<4, true, false>(d, bytes, o, g, "read K=4 nt");
        run<8, true, false>(d, bytes, o, g, "read K=8 nt");
        run<4, true, true>(d, bytes, o, g, "read K=4 nt + udot4");
    }
    return 0;
}
