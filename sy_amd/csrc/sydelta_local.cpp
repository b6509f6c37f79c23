// sydelta_local.cpp — sy's local-transport delta path on the device (SURVEY.md §8f
// row 3): the block-compare loop of src/transport/local.rs:541-619 / :682-760 and
// estimate_change_ratio (src/delta/ratio.rs:78-192), for files already in HBM.
#include <math.h>

#include <algorithm>
#include <vector>

#include "sydelta_host.hpp"
#include "sydelta_internal.hpp"

using namespace sydelta;

namespace {
struct DevMem {
    void* p = nullptr;
    hipStream_t s = nullptr;
    ~DevMem() {
        if (p) (void)hipFreeAsync(p, s);
    }
};
}  // namespace

// local.rs:549-619: for every block of the source, whether it differs from the same
// block of the destination; stats as the loop counts them (changed_blocks,
// literal_bytes = bytes of changed blocks, bytes_written = source size).
extern "C" int sydelta_block_compare_device(int device, const uint8_t* d_src, uint64_t src_len, const uint8_t* d_dst,
                                            uint64_t dst_len, uint64_t block_size, uint8_t* d_changed, void* stream,
                                            sydelta_block_compare_stats* out) try {
    if (!block_size) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (src_len && (!d_src || !d_changed)) return fail(SYDELTA_E_INVAL, "NULL buffer");
    if (dst_len && !d_dst) return fail(SYDELTA_E_INVAL, "NULL destination");
    if (int r = ensure_device(device)) return r;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    const uint64_t nb = (src_len + block_size - 1) / block_size;
    CallProf cp;
    HIP_TRY(launch_block_cmp(d_src, src_len, d_dst, dst_len, block_size, d_changed, s, cp.get()));
    if (out) {
        std::vector<uint8_t> h(nb);
        if (nb) HIP_TRY(hipMemcpyAsync(h.data(), d_changed, nb, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        uint64_t ch = 0, lit = 0;
        for (uint64_t k = 0; k < nb; ++k)
            if (h[k]) {
                ++ch;
                lit += std::min(block_size, src_len - k * block_size);
            }
        out->blocks = nb;
        out->changed_blocks = ch;
        out->literal_bytes = lit;
        out->bytes_written = src_len;
    }
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// ratio.rs:78-192 on device-resident bytes.  sample_count < 0 -> 20, threshold < 0 ->
// 0.75 (the defaults of :85-86).
extern "C" int sydelta_estimate_change_ratio_device(int device, const uint8_t* d_src, uint64_t src_len,
                                                    const uint8_t* d_dst, uint64_t dst_len, uint64_t block_size,
                                                    int64_t sample_count, double threshold, void* stream,
                                                    sydelta_change_ratio* out) try {
    if (!out) return fail(SYDELTA_E_INVAL, "NULL result");
    if (!block_size) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    uint64_t want = sample_count < 0 ? 20 : (uint64_t)sample_count;
    if (threshold < 0) threshold = 0.75;
    const uint64_t total_blocks = (dst_len + block_size - 1) / block_size;  // :99
    want = std::min(want, total_blocks);                                       // :102
    const double size_diff = dst_len > 0 ? fabs((double)src_len - (double)dst_len) / (double)dst_len : 1.0;
    auto finish = [&](double r, uint64_t sampled, uint64_t changed) {
        out->change_ratio = r;
        out->blocks_sampled = sampled;
        out->blocks_changed = changed;
        out->use_delta = r <= threshold ? 1 : 0;  // ChangeRatioResult::new
        out->reserved = 0;
        out->threshold = threshold;
        return SYDELTA_OK;
    };
    if (size_diff > 0.5) return finish(std::min(size_diff, 1.0), 0, 0);  // :112-124
    std::vector<uint64_t> pos(want);
    const uint64_t step = want > 1 ? total_blocks / (want - 1) : 0;     // :128-132
    for (uint64_t i = 0; i < want; ++i)                                  // :134-141
        pos[i] = want > 1 ? std::min(i * step, total_blocks ? total_blocks - 1 : 0) : 0;
    if (!want) return finish(0.0, 0, 0);
    if (int r = ensure_device(device)) return r;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    DevMem m;
    HIP_TRY(hipMallocAsync(&m.p, want * 8 * 3, s));
    m.s = s;
    uint64_t* d_pos = (uint64_t*)m.p;
    uint64_t* d_hs = d_pos + want;
    uint64_t* d_hd = d_hs + want;
    HIP_TRY(hipMemcpyAsync(d_pos, pos.data(), want * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(launch_hash_blocks(d_src, src_len, block_size, d_pos, (uint32_t)want, d_hs, s));
    HIP_TRY(launch_hash_blocks(d_dst, dst_len, block_size, d_pos, (uint32_t)want, d_hd, s));
    std::vector<uint64_t> hs(want), hd(want);
    HIP_TRY(hipMemcpyAsync(hs.data(), d_hs, want * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(hd.data(), d_hd, want * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    uint64_t changed = 0;
    for (uint64_t i = 0; i < want; ++i) {  // :150-168
        const uint64_t off = pos[i] * block_size;
        const uint64_t sr = src_len > off ? std::min(block_size, src_len - off) : 0;
        const uint64_t dr = dst_len > off ? std::min(block_size, dst_len - off) : 0;
        if (sr != dr || hs[i] != hd[i]) ++changed;
    }
    return finish((double)changed / (double)want, want, changed);  // :171-175
} catch (...) {
    return sydelta::host_exception();
}
