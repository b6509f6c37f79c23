// sydelta_integrity.cpp — whole-file XXH3-64 on the device:
// XxHash3Hasher::hash_file / hash_data (src/integrity/xxhash3.rs:17-40) for files
// already in HBM, one file or a batch (the per-file verify loop of integrity/mod.rs:104).
#include <algorithm>
#include <numeric>
#include <vector>

#include "sydelta_host.hpp"
#include "sydelta_internal.hpp"

using namespace sydelta;

extern "C" int sydelta_xxh3_batch_device(int device, const uint8_t* d_buf, uint64_t buf_len, const uint64_t* offs, const uint64_t* lens,
                                         uint64_t nfiles, void* stream, uint64_t* out) try {
    if (!nfiles) return SYDELTA_OK;
    if (!offs || !lens || !out) return fail(SYDELTA_E_INVAL, "NULL offs/lens/out");
    if (nfiles > 0xFFFFFFFFull) return fail(SYDELTA_E_INVAL, "too many files");
    uint64_t total = 0;
    for (uint64_t f = 0; f < nfiles; ++f) {
        if (offs[f] > buf_len || lens[f] > buf_len - offs[f]) return fail(SYDELTA_E_INVAL, "file range outside the buffer");
        total |= lens[f];
    }
    if (total && !d_buf) return fail(SYDELTA_E_INVAL, "NULL buffer");
    SYDELTA_ENTER_DEVICE(device);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    // host tables: block-count prefix and the size order of the chains
    std::vector<uint64_t> pfx(nfiles + 1, 0), nb(nfiles);
    for (uint64_t f = 0; f < nfiles; ++f) {
        nb[f] = lens[f] > 240 ? (lens[f] - 1) >> 10 : 0;
        pfx[f + 1] = pfx[f] + nb[f];
    }
    const uint64_t npieces = pfx[nfiles];
    // phase A's table: files with at least one full block (offset, block prefix)
    std::vector<uint64_t> aoff, apfx;
    for (uint64_t f = 0; f < nfiles; ++f)
        if (nb[f]) {
            aoff.push_back(offs[f]);
            apfx.push_back(pfx[f]);
        }
    const uint64_t nact = aoff.size();
    apfx.push_back(npieces);
    std::vector<uint32_t> order(nfiles);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return nb[a] > nb[b]; });
    const uint64_t tab = nfiles * 8 * 3 + (nfiles + 1) * 8 + nact * 8 + (nact + 1) * 8 + nfiles * 4;
    const uint64_t bytes = (tab + 255) / 256 * 256 + xxh_chain_records(npieces) * 64;
    void* ws = nullptr;
    HIP_TRY(dev_malloc_async(&ws, bytes, s));
    struct Free {
        void* p;
        hipStream_t s;
        ~Free() { (void)hipFreeAsync(p, s); }
    } fr{ws, s};
    uint64_t* d_off = (uint64_t*)ws;
    uint64_t* d_len = d_off + nfiles;
    uint64_t* d_out = d_len + nfiles;
    uint64_t* d_pfx = d_out + nfiles;
    uint64_t* d_aoff = d_pfx + nfiles + 1;
    uint64_t* d_apfx = d_aoff + nact;
    uint32_t* d_order = (uint32_t*)(d_apfx + nact + 1);
    uint64_t* d_C = (uint64_t*)((uint8_t*)ws + (tab + 255) / 256 * 256);
    HIP_TRY(hipMemcpyAsync(d_off, offs, nfiles * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_len, lens, nfiles * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_pfx, pfx.data(), (nfiles + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_order, order.data(), nfiles * 4, hipMemcpyHostToDevice, s));
    if (nact) HIP_TRY(hipMemcpyAsync(d_aoff, aoff.data(), nact * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_apfx, apfx.data(), (nact + 1) * 8, hipMemcpyHostToDevice, s));
    CallProf cp;
    HIP_TRY(launch_xxh_files(d_buf, d_off, d_len, d_pfx, d_aoff, d_apfx, nact, d_order, nfiles, npieces, d_C, d_out, s,
                             cp.get()));
    HIP_TRY(hipMemcpyAsync(out, d_out, nfiles * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_xxh3_device(int device, const uint8_t* d_buf, uint64_t len, void* stream, uint64_t* out) try {
    const uint64_t off = 0;
    return sydelta_xxh3_batch_device(device, d_buf, len, &off, &len, 1, stream, out);
} catch (...) {
    return sydelta::host_exception();
}
