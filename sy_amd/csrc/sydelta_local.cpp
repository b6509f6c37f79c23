// sydelta_local.cpp — sy's local-transport delta path on the device (SURVEY.md §8f
// row 3): the block-compare loop of src/transport/local.rs:541-619 / :682-760 and
// estimate_change_ratio (src/delta/ratio.rs:78-192), for files already in HBM.
#include <errno.h>
#include <fcntl.h>
#include <math.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

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
    SYDELTA_ENTER_DEVICE(device);
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

// The sampled block indices of ratio.rs:96-138 (dst_len's blocks; `want` already
// clamped to their count): evenly spaced, the last ones clamped to the final block.
static std::vector<uint64_t> sample_blocks(uint64_t want, uint64_t total_blocks) {
    std::vector<uint64_t> pos(want);
    const uint64_t step = want > 1 ? total_blocks / (want - 1) : 0;     // :125-129
    for (uint64_t i = 0; i < want; ++i)                                  // :131-138
        pos[i] = want > 1 ? std::min(i * step, total_blocks ? total_blocks - 1 : 0) : 0;
    return pos;
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
    const std::vector<uint64_t> pos = sample_blocks(want, total_blocks);
    if (!want) return finish(0.0, 0, 0);
    SYDELTA_ENTER_DEVICE(device);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    DevMem m;
    HIP_TRY(dev_malloc_async(&m.p, want * 8 * 3, s));
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

// ratio.rs:78-192 `estimate_change_ratio(source, dest, block_size, sample_count,
// threshold)` on two paths: the sampled blocks are read from both files (one pread
// each, as the BufReader seek + read of :145-154 returns min(block_size, bytes left)),
// packed into device memory and hashed there with XXH3-64 (sydelta_xxh3_batch_device,
// :162-168); blocks whose read sizes differ count as changed without hashing
// (:156-160).  Samples go in batches of at most 64 MiB per file.  I/O errors ->
// SYDELTA_E_IO (io::Result's Err).
extern "C" int sydelta_estimate_change_ratio(const char* source_path, const char* dest_path, uint64_t block_size,
                                             int64_t sample_count, double threshold, sydelta_change_ratio* out) try {
    if (!out || !source_path || !dest_path) return fail(SYDELTA_E_INVAL, "NULL argument");
    if (!block_size) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    struct Fd {
        int fd = -1;
        ~Fd() {
            if (fd >= 0) close(fd);
        }
    } fs, fd;
    fs.fd = open(source_path, O_RDONLY);  // :89-90
    if (fs.fd < 0) return fail(SYDELTA_E_IO, "open %s: %s", source_path, strerror(errno));
    fd.fd = open(dest_path, O_RDONLY);
    if (fd.fd < 0) return fail(SYDELTA_E_IO, "open %s: %s", dest_path, strerror(errno));
    struct stat ss, sd;
    if (fstat(fs.fd, &ss) || fstat(fd.fd, &sd)) return fail(SYDELTA_E_IO, "stat: %s", strerror(errno));
    const uint64_t src_len = (uint64_t)ss.st_size, dst_len = (uint64_t)sd.st_size;  // :93-94
    uint64_t want = sample_count < 0 ? 20 : (uint64_t)sample_count;
    if (threshold < 0) threshold = 0.75;
    const uint64_t total_blocks = (dst_len + block_size - 1) / block_size;  // :97
    want = std::min(want, total_blocks);                                       // :100
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
    if (size_diff > 0.5) return finish(std::min(size_diff, 1.0), 0, 0);  // :110-121
    if (!want) return finish(0.0, 0, 0);                                   // :172-176
    const std::vector<uint64_t> pos = sample_blocks(want, total_blocks);
    // read min(block_size, bytes left) at offset (short reads retried; EOF ends it)
    auto read_block = [&](int f, uint64_t off, uint8_t* dst, uint64_t* got) -> int {
        uint64_t n = 0;
        while (n < block_size) {
            const ssize_t r = pread(f, dst + n, block_size - n, (off_t)(off + n));
            if (r < 0) {
                if (errno == EINTR) continue;
                return fail(SYDELTA_E_IO, "read: %s", strerror(errno));
            }
            if (r == 0) break;
            n += (uint64_t)r;
        }
        *got = n;
        return SYDELTA_OK;
    };
    int dev = 0;
    if (int r = path_device(&dev)) return r;
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = thread_stream(dev);
    const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(want, (64ull << 20) / block_size));
    std::vector<uint8_t> host(2 * per * block_size);
    DevMem m;
    HIP_TRY(dev_malloc_async(&m.p, host.size(), s));
    m.s = s;
    uint64_t changed = 0;
    std::vector<uint64_t> offs, lens, hash;
    std::vector<uint64_t> rs(per), rd(per);
    for (uint64_t i0 = 0; i0 < want; i0 += per) {
        const uint64_t k = std::min(per, want - i0);
        offs.clear();
        lens.clear();
        for (uint64_t i = 0; i < k; ++i) {
            const uint64_t off = pos[i0 + i] * block_size;  // :146
            uint8_t* bs_ = host.data() + 2 * i * block_size;
            if (int r = read_block(fs.fd, off, bs_, &rs[i])) return r;
            if (int r = read_block(fd.fd, off, bs_ + block_size, &rd[i])) return r;
            if (rs[i] != rd[i]) continue;  // :156-160
            offs.push_back(2 * i * block_size);
            lens.push_back(rs[i]);
            offs.push_back((2 * i + 1) * block_size);
            lens.push_back(rd[i]);
        }
        hash.assign(offs.size(), 0);
        if (!offs.empty()) {
            HIP_TRY(hipMemcpyAsync(m.p, host.data(), 2 * k * block_size, hipMemcpyHostToDevice, s));
            if (int r = sydelta_xxh3_batch_device(-1, (const uint8_t*)m.p, 2 * k * block_size, offs.data(),
                                                  lens.data(), offs.size(), s, hash.data()))
                return r;
        }
        size_t h = 0;
        for (uint64_t i = 0; i < k; ++i) {
            if (rs[i] != rd[i]) {
                ++changed;
                continue;
            }
            if (hash[h] != hash[h + 1]) ++changed;  // :162-168
            h += 2;
        }
    }
    return finish((double)changed / (double)want, want, changed);  // :171-176
} catch (...) {
    return sydelta::host_exception();
}
