// micro_bufoob.hip — what a raw buffer load returns past num_records on gfx950 (not
// product code).  The descriptor covers the first 4 KiB of a 4.25 GiB allocation filled
// with a marker, so every offset probed below is mapped memory whatever the range
// check does: a load that returns the marker was not range-checked.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_probe(const uint32_t* base, uint32_t nrec, int flags, const uint32_t* offs, uint32_t n, uint32_t* out) {
    const uint32_t i = threadIdx.x;
    const uint64_t b = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                                                 (int)nrec, flags);
    if (i < n) out[i] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)offs[i], 0, 0);
}

int main() {
    const size_t bytes = (17ull << 28);  // 4.25 GiB
    uint32_t* t;
    CK(hipMalloc(&t, bytes));
    CK(hipMemsetD32((hipDeviceptr_t)t, 0xA5A5A5A5u, bytes / 4));
    const uint32_t offs[] = {0, 4, 4088, 4092, 4093, 4094, 4095, 4096, 4100, 8192, 1u << 20, 0x7FFFFFF0u,
                             0xFFFFFFF0u, 0xFFFFFFFCu, 0xFFFFFFFDu, 0xFFFFFFFEu, 0xFFFFFFFFu};
    const uint32_t n = sizeof(offs) / 4;
    uint32_t *d_offs, *d_out;
    CK(hipMalloc(&d_offs, sizeof(offs)));
    CK(hipMalloc(&d_out, 4 * n));
    CK(hipMemcpy(d_offs, offs, sizeof(offs), hipMemcpyHostToDevice));
    for (int flags : {0x00020000, 0x00027000, 0x00027FAC, 0}) {
        CK(hipMemset(d_out, 0x11, 4 * n));
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, t, 4096u, flags, d_offs, n, d_out);
        CK(hipDeviceSynchronize());
        uint32_t out[64];
        CK(hipMemcpy(out, d_out, 4 * n, hipMemcpyDeviceToHost));
        printf("flags 0x%08x, num_records 4096:\n", flags);
        for (uint32_t i = 0; i < n; ++i) printf("  offset 0x%08x -> 0x%08x %s\n", offs[i], out[i], out[i] == 0 ? "(range-checked: 0)" : "");
    }
    return 0;
}
