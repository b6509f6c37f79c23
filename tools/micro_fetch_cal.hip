// micro_fetch_cal.hip — FETCH_SIZE calibration for the access widths the scans use
// (measurement only).  Each kernel reads a known set of bytes; the host
// prints the exact number of accesses and of distinct 32/64/128-byte lines they touch, so
// FETCH_SIZE of each kernel (rocprofv3 --pmc, one pass) divides into bytes per line.
//   k_cal_stream      16 B per lane, coalesced, 1 GiB once            (the guide's calibrated case)
//   k_cal_g4_hbm      random 4-byte gathers from a 4 GiB table         (k_scan_r's level-2 word misses)
//   k_cal_g16_hbm     random 16-byte reads from a 4 GiB table          (exact-table bucket reads that miss)
//   k_cal_g4_l3       random 4-byte gathers from a 16 MiB table        (L2-missing, Infinity-Cache-resident)
//   k_cal_g16_l3      random 16-byte reads from a 16 MiB table
// The random indices come from a hash of (thread, j), replayed on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__host__ __device__ inline uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
constexpr int kG = 8;  // gathers per thread

__global__ void k_cal_stream(const uint4* __restrict__ t, uint64_t n4, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = t[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}
template <int kName>
__global__ void k_gather4(const uint32_t* __restrict__ t, uint64_t mask, uint64_t seed, uint32_t* out) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < kG; ++j) acc += t[mix(seed + g * kG + j) & mask];
    if (acc == 0x9E3779B9u) out[0] = acc;
}
template <int kName>
__global__ void k_gather16(const uint4* __restrict__ t, uint64_t mask, uint64_t seed, uint32_t* out) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < kG; ++j) {
        const uint4 v = t[mix(seed + g * kG + j) & mask];
        acc += v.x ^ v.w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}
// Both 64-byte halves of random 128-byte lines, the second read after the first returned:
// one L2 request per line if a miss fills all 128 bytes, two if it fills 64.
__global__ void k_cal_pair(const uint32_t* __restrict__ t, uint64_t lmask, uint64_t seed, uint32_t* out) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < kG; ++j) {
        const uint64_t line = mix(seed + g * kG + j) & lmask;
        // agent-scope atomic loads skip the L1, so both reach the L2
        const uint32_t v = __hip_atomic_load(t + line * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc += __hip_atomic_load(t + line * 32 + 16 + (v & 0x80000000u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}
// distinct lines of `line` bytes among the accesses (elem-byte elements, indices from mix)
static void count(const char* name, uint64_t threads, uint64_t mask, uint64_t seed, uint32_t elem) {
    std::vector<uint64_t> a(threads * kG);
    for (uint64_t g = 0; g < threads; ++g)
        for (int j = 0; j < kG; ++j) a[g * kG + j] = (mix(seed + g * kG + j) & mask) * elem;
    printf("%s accesses %llu bytes_requested %llu", name, (unsigned long long)a.size(),
           (unsigned long long)(a.size() * elem));
    for (uint32_t line : {32u, 64u, 128u}) {
        std::vector<uint64_t> l(a.size());
        for (size_t i = 0; i < a.size(); ++i) l[i] = a[i] / line;
        std::sort(l.begin(), l.end());
        printf(" lines%u %llu", line, (unsigned long long)(std::unique(l.begin(), l.end()) - l.begin()));
    }
    printf("\n");
}

int main() {
    const size_t big = 4ull << 30, small = 16ull << 20, sbytes = 1ull << 30;
    uint8_t *tb, *ts, *st;
    uint32_t* out;
    CK(hipMalloc(&tb, big));
    CK(hipMalloc(&ts, small));
    CK(hipMalloc(&st, sbytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(tb, 1, big));
    CK(hipMemset(ts, 2, small));
    CK(hipMemset(st, 3, sbytes));
    CK(hipDeviceSynchronize());
    const uint64_t threads = 1ull << 19;  // x kG = 4 Mi accesses per kernel
    const dim3 grid((uint32_t)(threads / 256)), block(256);
    hipLaunchKernelGGL(k_cal_stream, dim3(4096), block, 0, 0, (const uint4*)st, (uint64_t)(sbytes / 16), out);
    printf("k_cal_stream accesses %llu bytes_requested %llu\n", (unsigned long long)(sbytes / 16),
           (unsigned long long)sbytes);
    hipLaunchKernelGGL(k_gather4<0>, grid, block, 0, 0, (const uint32_t*)tb, (uint64_t)(big / 4 - 1), 11ull, out);
    count("k_gather4<0> (4 GiB table)", threads, big / 4 - 1, 11ull, 4);
    hipLaunchKernelGGL(k_gather16<0>, grid, block, 0, 0, (const uint4*)tb, (uint64_t)(big / 16 - 1), 22ull, out);
    count("k_gather16<0> (4 GiB table)", threads, big / 16 - 1, 22ull, 16);
    // the small table: one warm-up pass loads it into the Infinity Cache, the measured one follows
    hipLaunchKernelGGL(k_cal_stream, dim3(1024), block, 0, 0, (const uint4*)ts, (uint64_t)(small / 16), out);
    hipLaunchKernelGGL(k_gather4<1>, grid, block, 0, 0, (const uint32_t*)ts, (uint64_t)(small / 4 - 1), 33ull, out);
    count("k_gather4<1> (16 MiB table, warm)", threads, small / 4 - 1, 33ull, 4);
    hipLaunchKernelGGL(k_gather16<1>, grid, block, 0, 0, (const uint4*)ts, (uint64_t)(small / 16 - 1), 44ull, out);
    count("k_gather16<1> (16 MiB table, warm)", threads, small / 16 - 1, 44ull, 16);
    hipLaunchKernelGGL(k_cal_pair, grid, block, 0, 0, (const uint32_t*)tb, (uint64_t)(big / 128 - 1), 55ull, out);
    count("k_cal_pair (4 GiB table, line heads)", threads, big / 128 - 1, 55ull, 128);
    CK(hipDeviceSynchronize());
    printf("(the second k_cal_stream launch is the 16 MiB warm-up: %llu bytes)\n", (unsigned long long)small);
    return 0;
}
