// wsr_check.hip — not product code: wave_strong_regs (k_scan_r's in-register XXH3 of a
// 4096-byte window) against the C oracle's XXH3-64 for every window start of one wave
// tile, on random and on low-alphabet bytes.  Build: tools/wsr_check.sh; run on the GPU box.
#include "../sy_amd/csrc/sydelta_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <vector>

extern "C" uint64_t oracle_xxh3_64(const uint8_t* in, uint64_t len);

// the launch wrappers' host helpers live in sydelta_api.cpp, which this check does not link
namespace sydelta {
ProfScope::ProfScope(Profiler* p_, hipStream_t s_, const char* n) : p(p_), s(s_), name(n) {}
ProfScope::~ProfScope() {}
hipError_t dev_malloc_async(void** p, size_t bytes, hipStream_t s) { return hipMallocAsync(p, bytes, s); }
}  // namespace sydelta

namespace sydelta {
__global__ __launch_bounds__(64) void k_wsr_check(const uint8_t* buf, uint64_t len, uint32_t nofs, uint64_t* out) {
    __shared__ uint64_t kt[48];
    const uint32_t lane = threadIdx.x & 63;
    if (lane < 48)
        kt[lane] = lane < 24 ? c_tab.w[lane] : lane < 32 ? c_tab.last[lane - 24] : lane < 40 ? c_tab.init[lane - 32]
                                                                                          : c_tab.merge[lane - 40];
    __syncthreads();
    uint32_t xo[16], xi[16];
    load_chunk(buf, len, 64ull * lane, xo);
    load_chunk(buf, len, 4096ull + 64ull * lane, xi);
    for (uint32_t o = 0; o < nofs; ++o) {
        const uint64_t st = wave_strong_regs(xo, xi, o, kt);
        if (lane == 0) out[o] = st;
    }
}
}  // namespace sydelta

int main() {
    const uint64_t len = 8192 + 64;
    std::vector<uint8_t> h(len);
    int bad = 0;
    for (int pass = 0; pass < 2; ++pass) {
        uint64_t x = 0x9E3779B97F4A7C15ull + pass;
        for (auto& b : h) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            b = pass == 0 ? (uint8_t)x : (uint8_t)(x % 3);
        }
        uint8_t* d = nullptr;
        uint64_t* dout = nullptr;
        hipMalloc(&d, len + 64);
        hipMalloc(&dout, 4096 * 8);
        hipMemcpy(d, h.data(), len, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(sydelta::k_wsr_check, dim3(1), dim3(64), 0, 0, d, len, 4096u, dout);
        std::vector<uint64_t> got(4096);
        if (hipMemcpy(got.data(), dout, 4096 * 8, hipMemcpyDeviceToHost) != hipSuccess) { printf("hip error\n"); return 2; }
        int pbad = 0;
        for (uint32_t o = 0; o < 4096; ++o) {
            const uint64_t want = oracle_xxh3_64(h.data() + o, 4096);
            if (got[o] != want) {
                if (pbad < 2) printf("pass %d o=%u got %016llx want %016llx\n", pass, o, (unsigned long long)got[o],
                                     (unsigned long long)want);
                ++pbad;
            }
        }
        printf("pass %d: %d of 4096 window starts differ\n", pass, pbad);
        bad += pbad;
        hipFree(d);
        hipFree(dout);
    }
    return bad ? 1 : 0;
}
