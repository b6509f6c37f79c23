// sydelta_api.cpp — C ABI (include/sydelta.h) over the gfx950 kernels.
//
// Host-side orchestration of sy's delta hot path:
//   signature  : compute_checksums (src/delta/checksum.rs:31-80)
//   index      : candidate map     (src/delta/generator.rs:75-81)
//   match      : generate_delta / generate_delta_streaming (generator.rs:67-379)
// The greedy op emission (generator.rs:116-221) is resolved on the host from the
// position-sorted list of verified device hits: walking it reproduces the
// sequential scan exactly because every full-window position p <= len-bs has
// been classified on the device (hit with its first-in-index-order block, or
// not), and the scan only ever jumps by bs after a hit or by 1 otherwise.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/sydelta.h"
#include "sydelta_internal.hpp"

using namespace sydelta;

// ---------------------------------------------------------------------------
// errors (thread-local, like io::Error propagated to the caller)
// ---------------------------------------------------------------------------
static thread_local std::string t_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) {                                                                         \
            int code_ = (e_ == hipErrorOutOfMemory) ? SYDELTA_E_OOM : SYDELTA_E_KERNEL;                 \
            return fail(code_, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__);   \
        }                                                                                               \
    } while (0)

extern "C" const char* sydelta_last_error(void) { return t_err.c_str(); }
extern "C" int sydelta_abi_version(void) { return SYDELTA_ABI_VERSION; }

// ---------------------------------------------------------------------------
// devices: call_once init per device, gfx950 only
// ---------------------------------------------------------------------------
namespace {
struct DevState {
    std::once_flag once;
    int status = SYDELTA_E_NODEV;
    std::string msg;
};
std::mutex g_dev_mu;
std::map<int, std::unique_ptr<DevState>> g_devs;

int ensure_device(int device) {
    if (device < 0) device = 0;
    DevState* st;
    {
        std::lock_guard<std::mutex> lk(g_dev_mu);
        auto& p = g_devs[device];
        if (!p) p.reset(new DevState());
        st = p.get();
    }
    std::call_once(st->once, [&] {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= device) {
            st->msg = "no HIP device " + std::to_string(device);
            return;
        }
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
            st->msg = "hipGetDeviceProperties failed";
            return;
        }
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            st->msg = std::string("device is ") + prop.gcnArchName + ", libsydelta is built for gfx950 only";
            return;
        }
        st->status = SYDELTA_OK;
    });
    if (st->status != SYDELTA_OK) return fail(st->status, "%s", st->msg.c_str());
    if (hipSetDevice(device) != hipSuccess) return fail(SYDELTA_E_NODEV, "hipSetDevice(%d) failed", device);
    return SYDELTA_OK;
}

// one non-blocking stream per (thread, device): calls on different threads never share a stream
hipStream_t thread_stream(int device) {
    static thread_local std::map<int, hipStream_t> streams;
    auto it = streams.find(device);
    if (it != streams.end()) return it->second;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    streams[device] = s;
    return s;
}

// ---------------------------------------------------------------------------
// profiling
// ---------------------------------------------------------------------------
std::atomic<int> g_prof_on{0};
std::mutex g_prof_mu;
std::map<std::string, std::pair<double, uint64_t>> g_prof;
}  // namespace

namespace sydelta {
ProfScope::ProfScope(Profiler* p_, hipStream_t s_, const char* n) : p(p_), s(s_), name(n) {
    if (!p) return;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) { p = nullptr; return; }
    (void)hipEventRecord(a, s);
}
ProfScope::~ProfScope() {
    if (!p) return;
    (void)hipEventRecord(b, s);
    p->pending.push_back({name, a, b});
}
void Profiler::resolve() {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (auto& q : pending) {
        float ms = 0;
        if (hipEventSynchronize(q.b) == hipSuccess && hipEventElapsedTime(&ms, q.a, q.b) == hipSuccess) {
            auto& e = g_prof[q.name];
            e.first += ms;
            e.second += 1;
        }
        (void)hipEventDestroy(q.a);
        (void)hipEventDestroy(q.b);
    }
    pending.clear();
}
}  // namespace sydelta

namespace {
struct CallProf {
    Profiler prof;
    Profiler* get() { return g_prof_on.load() ? &prof : nullptr; }
    ~CallProf() { prof.resolve(); }
};
}  // namespace

extern "C" void sydelta_set_profiling(int on) { g_prof_on.store(on ? 1 : 0); }

extern "C" size_t sydelta_profile_json(char* buf, size_t cap, int reset) {
    std::string s = "{";
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        bool first = true;
        for (auto& kv : g_prof) {
            char tmp[256];
            snprintf(tmp, sizeof tmp, "%s\"%s\": {\"ms\": %.6f, \"count\": %llu}", first ? "" : ", ", kv.first.c_str(),
                     kv.second.first, (unsigned long long)kv.second.second);
            s += tmp;
            first = false;
        }
        if (reset) g_prof.clear();
    }
    s += "}";
    if (buf && cap > s.size()) memcpy(buf, s.c_str(), s.size() + 1);
    return s.size();
}

// ---------------------------------------------------------------------------
// small utilities
// ---------------------------------------------------------------------------
extern "C" int sydelta_device_count(int* count) {
    if (!count) return fail(SYDELTA_E_INVAL, "count is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return SYDELTA_OK;
}

// mod.rs:20-23
extern "C" uint64_t sydelta_calculate_block_size(uint64_t file_size) {
    uint64_t s = (uint64_t)std::sqrt((double)file_size);
    return std::min<uint64_t>(std::max<uint64_t>(s, 512), 128 * 1024);
}

static uint32_t ceil_log2(uint64_t v) {
    uint32_t b = 0;
    while ((1ull << b) < v) ++b;
    return b;
}

// ---------------------------------------------------------------------------
// signature
// ---------------------------------------------------------------------------
extern "C" int sydelta_signature_device(int device, const uint8_t* d_buf, uint64_t len, uint64_t block_size,
                                        uint32_t* d_weak, uint64_t* d_strong, void* stream) {
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (len && (!d_buf || !d_weak || !d_strong)) return fail(SYDELTA_E_INVAL, "NULL device pointer");
    if (int r = ensure_device(device)) return r;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    CallProf cp;
    HIP_TRY(launch_signature(d_buf, len, block_size, d_weak, d_strong, s, cp.get()));
    if (!stream || cp.get()) HIP_TRY(hipStreamSynchronize(s));
    return SYDELTA_OK;
}

extern "C" int sydelta_signature_batch_device(int device, const uint8_t* d_buf, const uint64_t* off,
                                              const uint64_t* len, uint64_t nfiles, uint64_t block_size,
                                              uint32_t* d_weak, uint64_t* d_strong, void* stream) {
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (nfiles && (!off || !len)) return fail(SYDELTA_E_INVAL, "NULL segment table");
    if (int r = ensure_device(device)) return r;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    std::vector<uint64_t> fblk(nfiles + 1, 0);
    for (uint64_t f = 0; f < nfiles; ++f) fblk[f + 1] = fblk[f] + (len[f] + block_size - 1) / block_size;
    const uint64_t total = fblk[nfiles];
    if (!total) return SYDELTA_OK;
    uint64_t* d_meta = nullptr;
    HIP_TRY(hipMallocAsync((void**)&d_meta, sizeof(uint64_t) * (3 * nfiles + 1), s));
    HIP_TRY(hipMemcpyAsync(d_meta, off, 8 * nfiles, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_meta + nfiles, len, 8 * nfiles, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d_meta + 2 * nfiles, fblk.data(), 8 * (nfiles + 1), hipMemcpyHostToDevice, s));
    CallProf cp;
    hipError_t e = launch_signature_batch(d_buf, d_meta, d_meta + nfiles, d_meta + 2 * nfiles, nfiles, block_size,
                                          total, d_weak, d_strong, s, cp.get());
    (void)hipFreeAsync(d_meta, s);
    HIP_TRY(e);
    HIP_TRY(hipStreamSynchronize(s));  // the host segment table must outlive the copies
    return SYDELTA_OK;
}

// ---------------------------------------------------------------------------
// index (one or many basis signatures; arrays concatenated over files)
// ---------------------------------------------------------------------------
struct sydelta_index {
    int device = 0;
    uint64_t bs = 0;
    uint64_t nfiles = 0;
    std::vector<uint64_t> fblk;       // block prefix, nfiles+1
    std::vector<uint64_t> last_size;  // per file (0 for an empty signature)
    uint32_t* d_weak = nullptr;       // owned copies, concatenated
    uint64_t* d_strong = nullptr;
    DeviceIndex ix;
    void* d_pool = nullptr;           // one allocation for all index arrays
};

static void index_release(sydelta_index* x) {
    if (!x) return;
    if (x->d_pool) (void)hipFree(x->d_pool);
    delete x;
}

extern "C" void sydelta_index_free(sydelta_index* idx) {
    if (!idx) return;
    (void)hipSetDevice(idx->device);
    index_release(idx);
}

static int index_create_impl(int device, const uint32_t* weak, const uint64_t* strong, const uint64_t* nblk,
                             const uint64_t* last, uint64_t nfiles, uint64_t block_size, int arrays_on_device,
                             void* stream, sydelta_index** out) {
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (nfiles == 0 || nfiles >= 0xFFFFFFFFull) return fail(SYDELTA_E_INVAL, "bad file count %llu", (unsigned long long)nfiles);
    std::vector<uint64_t> fblk(nfiles + 1, 0);
    for (uint64_t f = 0; f < nfiles; ++f) {
        if (nblk[f] && (last[f] == 0 || last[f] > block_size))
            return fail(SYDELTA_E_INVAL, "file %llu: last_size must be in [1, block_size]", (unsigned long long)f);
        fblk[f + 1] = fblk[f] + nblk[f];
    }
    const uint64_t nblocks = fblk[nfiles];
    if (nblocks && (!weak || !strong)) return fail(SYDELTA_E_INVAL, "NULL signature arrays");
    if (nblocks >= 0xFFFFFFFFull) return fail(SYDELTA_E_INVAL, "too many blocks (%llu)", (unsigned long long)nblocks);
    if (int r = ensure_device(device)) return r;
    if (device < 0) device = 0;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device);
    std::unique_ptr<sydelta_index, void (*)(sydelta_index*)> x(new sydelta_index(), index_release);
    x->device = device;
    x->bs = block_size;
    x->nfiles = nfiles;
    x->fblk = fblk;
    x->last_size.resize(nfiles);
    DeviceIndex& ix = x->ix;
    ix.nfiles = nfiles;
    ix.nblocks = nblocks;
    ix.files.resize(nfiles);
    // per file: Bloom filter in 32-bit words -- up to kLdsFilterKeys keys at most 2^13
    // words (32 KiB) that the LDS-staged scan holds in LDS (>= 16 bits per key, 128 bits
    // per key for small bases), above that 16 bits per key in HBM/L2; exact table in
    // buckets of 4 keys at load <= 0.5.
    uint64_t fw = 0, sl = 0;
    for (uint64_t f = 0; f < nfiles; ++f) {
        x->last_size[f] = nblk[f] ? last[f] : 0;
        const uint64_t nk = nblk[f] ? nblk[f] : 1;
        const uint32_t lk = ceil_log2(nk);
        // <= 4 Ki keys: <= 16 KiB filter (3 scan workgroups per CU); <= 16 Ki keys: 32 KiB (2 per CU)
        const uint32_t fwbits = nk <= 4096 ? std::min<uint32_t>(12, std::max<uint32_t>(6, lk + 2))
                                : nk <= kLdsFilterKeys ? 13u
                                                       : std::min<uint32_t>(28, lk - 1);
        const uint32_t bbits = std::max<uint32_t>(2, ceil_log2((nk + 1) / 2));
        FileIx& F = ix.files[f];
        F.filt_off = fw;
        F.slot_off = sl;
        F.blk_base = fblk[f];
        F.fwshift = 32 - fwbits;
        F.bmask = (1u << bbits) - 1;
        fw += 1ull << fwbits;
        sl += 4ull << bbits;
        ix.max_fwords = std::max<uint32_t>(ix.max_fwords, 1u << fwbits);
    }
    ix.fwords = fw;
    ix.nslots = sl;
    const size_t nb = std::max<uint64_t>(nblocks, 1);
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t sz_weak = al(4 * nb), sz_strong = al(8 * nb), sz_filt = al(4 * fw), sz_t = al(4 * sl);
    const size_t sz_order = al(4 * nb), sz_slot = al(4 * nb), sz_files = al(sizeof(FileIx) * nfiles);
    const size_t sz_fblk = al(8 * (nfiles + 1)), sz_cstrong = al(8 * nb);
    const size_t total = sz_weak + sz_strong + sz_filt + 4 * sz_t + sz_order + sz_slot + sz_files + sz_fblk + sz_cstrong;
    HIP_TRY(hipMalloc(&x->d_pool, total));
    uint8_t* p = (uint8_t*)x->d_pool;
    x->d_weak = (uint32_t*)p; p += sz_weak;
    x->d_strong = (uint64_t*)p; p += sz_strong;
    ix.filt = (uint32_t*)p; p += sz_filt;
    ix.keys = (uint32_t*)p; p += sz_t;
    ix.cnt = (uint32_t*)p; p += sz_t;
    ix.start = (uint32_t*)p; p += sz_t;
    ix.fill = (uint32_t*)p; p += sz_t;
    ix.order = (uint32_t*)p; p += sz_order;
    ix.slot_of = (uint32_t*)p; p += sz_slot;
    ix.d_files = (FileIx*)p; p += sz_files;
    ix.d_fblk = (uint64_t*)p; p += sz_fblk;
    ix.cstrong = (uint64_t*)p; p += sz_cstrong;
    const hipMemcpyKind kind = arrays_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (nblocks) {
        HIP_TRY(hipMemcpyAsync(x->d_weak, weak, 4 * nblocks, kind, s));
        HIP_TRY(hipMemcpyAsync(x->d_strong, strong, 8 * nblocks, kind, s));
    }
    HIP_TRY(hipMemcpyAsync(ix.d_files, ix.files.data(), sizeof(FileIx) * nfiles, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(ix.d_fblk, x->fblk.data(), 8 * (nfiles + 1), hipMemcpyHostToDevice, s));
    CallProf cp;
    HIP_TRY(launch_index_build(x->d_weak, x->d_strong, ix, s, cp.get()));
    HIP_TRY(hipStreamSynchronize(s));  // host tables must outlive the copies
    *out = x.release();
    return SYDELTA_OK;
}

extern "C" int sydelta_index_create(int device, const uint32_t* weak, const uint64_t* strong, uint64_t nblocks,
                                    uint64_t block_size, uint64_t last_size, int arrays_on_device, void* stream,
                                    sydelta_index** out) {
    const uint64_t last = nblocks ? last_size : 0;
    return index_create_impl(device, weak, strong, &nblocks, &last, 1, block_size, arrays_on_device, stream, out);
}

extern "C" int sydelta_index_create_batch(int device, const uint32_t* weak, const uint64_t* strong,
                                          const uint64_t* nblocks, const uint64_t* last_size, uint64_t nfiles,
                                          uint64_t block_size, int arrays_on_device, void* stream,
                                          sydelta_index** out) {
    if (nfiles && (!nblocks || !last_size)) return fail(SYDELTA_E_INVAL, "NULL file table");
    return index_create_impl(device, weak, strong, nblocks, last_size, nfiles, block_size, arrays_on_device, stream,
                             out);
}

// ---------------------------------------------------------------------------
// delta object
// ---------------------------------------------------------------------------
struct sydelta_delta {
    std::vector<sydelta_op> ops;
    uint64_t source_size = 0, block_size = 0;
    sydelta_match_stats stats{};
    std::vector<uint8_t> lit;         // literal bytes (host-data entry points)
    std::vector<uint64_t> lit_off;    // per op: offset into lit, or UINT64_MAX
};

struct sydelta_delta_batch {
    std::vector<sydelta_delta> d;
    sydelta_match_stats total{};
};

extern "C" uint64_t sydelta_delta_num_ops(const sydelta_delta* d) { return d ? d->ops.size() : 0; }
extern "C" const sydelta_op* sydelta_delta_ops(const sydelta_delta* d) {
    return (d && !d->ops.empty()) ? d->ops.data() : nullptr;
}
extern "C" uint64_t sydelta_delta_source_size(const sydelta_delta* d) { return d ? d->source_size : 0; }
extern "C" uint64_t sydelta_delta_block_size(const sydelta_delta* d) { return d ? d->block_size : 0; }
extern "C" const uint8_t* sydelta_delta_literal(const sydelta_delta* d, uint64_t i) {
    if (!d || i >= d->ops.size() || d->lit_off.size() != d->ops.size()) return nullptr;
    if (d->ops[i].kind != SYDELTA_OP_DATA || d->lit_off[i] == UINT64_MAX) return nullptr;
    return d->lit.data() + d->lit_off[i];
}
extern "C" int sydelta_delta_stats(const sydelta_delta* d, sydelta_match_stats* out) {
    if (!d || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = d->stats;
    return SYDELTA_OK;
}
// generator.rs:30-55
extern "C" double sydelta_delta_compression_ratio(const sydelta_delta* d) {
    if (!d) return 1.0;
    uint64_t lit = 0, cop = 0;
    for (auto& o : d->ops) (o.kind == SYDELTA_OP_DATA ? lit : cop) += o.b;
    const uint64_t tot = lit + cop;
    return tot == 0 ? 1.0 : (double)lit / (double)tot;
}
extern "C" void sydelta_delta_free(sydelta_delta* d) { delete d; }

extern "C" uint64_t sydelta_delta_batch_count(const sydelta_delta_batch* b) { return b ? b->d.size() : 0; }
extern "C" const sydelta_delta* sydelta_delta_batch_get(const sydelta_delta_batch* b, uint64_t i) {
    return (b && i < b->d.size()) ? &b->d[i] : nullptr;
}
extern "C" int sydelta_delta_batch_stats(const sydelta_delta_batch* b, sydelta_match_stats* out) {
    if (!b || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = b->total;
    return SYDELTA_OK;
}
extern "C" void sydelta_delta_batch_free(sydelta_delta_batch* b) { delete b; }

// ---------------------------------------------------------------------------
// match
// ---------------------------------------------------------------------------
namespace {
struct DevBuf {
    void* p = nullptr;
    hipStream_t s = nullptr;
    ~DevBuf() {
        if (p) (void)hipFreeAsync(p, s);
    }
};

// Greedy op emission (generator.rs:116-221) of one file from its position-sorted
// verified hits (pos, global block).
void emit_ops(const uint64_t* pos, const uint32_t* blk, size_t nhits, uint64_t blk_base, uint64_t nblocks,
              uint64_t n, uint64_t last_size, uint64_t len, int tail_match, sydelta_delta* d) {
    uint64_t x = 0;
    auto data = [&](uint64_t a, uint64_t b) {
        if (b) {
            d->ops.push_back({SYDELTA_OP_DATA, 0, a, b});
            d->stats.data_ops++;
            d->stats.literal_bytes += b;
        }
    };
    auto copy = [&](uint64_t b) {
        const uint64_t sz = (b + 1 == nblocks) ? last_size : n;
        d->ops.push_back({SYDELTA_OP_COPY, 0, b * n, sz});
        d->stats.copy_ops++;
    };
    for (size_t i = 0; i < nhits; ++i) {
        const uint64_t p = pos[i];
        if (p < x) continue;  // inside the previous Copy: never visited
        data(x, p - x);
        copy(blk[i] - blk_base);
        x = p + n;  // generator.rs:313 / :144
    }
    if (tail_match) {  // generator.rs:324-353: only p* = len - last_size can match
        const uint64_t pstar = len - last_size;
        if (pstar >= x) {
            data(x, pstar - x);
            copy(nblocks - 1);
            x = len;
        }
    }
    data(x, len - x);
}
}  // namespace

// Match source f (d_buf[src_off[f] .. +src_len[f])) against file f of the index,
// for every f; results in b->d[f].
static int match_impl(sydelta_index* ix, const uint8_t* d_buf, const uint64_t* src_off, const uint64_t* src_len,
                      hipStream_t s, sydelta_delta_batch* b) {
    CallProf cp;
    Profiler* prof = cp.get();
    const uint64_t n = ix->bs;
    const uint64_t nf = ix->nfiles;
    b->d.assign(nf, sydelta_delta());
    for (uint64_t f = 0; f < nf; ++f) {
        b->d[f].source_size = src_len[f];
        b->d[f].block_size = n;
        if (src_len[f] && !d_buf) return fail(SYDELTA_E_INVAL, "NULL source buffer");
        if (src_len[f] && ((uintptr_t)(d_buf + src_off[f]) & 15) != 0)
            return fail(SYDELTA_E_INVAL, "source %llu must start 16-byte aligned", (unsigned long long)f);
    }
    // segments: per file, runs of <= seg_max full-window positions (generator.rs:116-155)
    const uint64_t tile = scan_tile_positions();
    const uint64_t seg_max = (1ull << 31) / tile * tile;
    std::vector<ScanSeg> segs;
    std::vector<uint32_t> seg_file;
    uint64_t ntiles = 0, tot_pos = 0;
    for (uint64_t f = 0; f < nf; ++f) {
        const uint64_t len = src_len[f];
        const uint64_t npos = len >= n ? len - n + 1 : 0;
        b->d[f].stats.positions = npos;
        tot_pos += npos;
        if (!npos || ix->fblk[f + 1] == ix->fblk[f]) continue;  // no windows, or empty signature
        for (uint64_t p0 = 0; p0 < npos; p0 += seg_max) {
            ScanSeg g{};
            g.src = src_off[f];
            g.len = len;
            g.pos_begin = p0;
            g.pos_end = std::min(npos, p0 + seg_max);
            g.tile_base = (uint32_t)ntiles;
            g.file = (uint32_t)f;
            ntiles += (g.pos_end - g.pos_begin + tile - 1) / tile;
            segs.push_back(g);
            seg_file.push_back((uint32_t)f);
        }
    }
    b->total.positions = tot_pos;
    if (ntiles >= 0xFFFFFFFFull || segs.size() >= 0x7FFFFFFFull)
        return fail(SYDELTA_E_INVAL, "batch too large (%llu tiles)", (unsigned long long)ntiles);
    const bool wide = n > scan_max_window();
    if (wide && nf != 1) return fail(SYDELTA_E_INVAL, "batched match needs block_size <= %u", scan_max_window());
    // tail rule jobs (generator.rs:156-184)
    std::vector<TailJob> tails;
    std::vector<uint32_t> tail_file;
    for (uint64_t f = 0; f < nf; ++f) {
        const uint64_t nb = ix->fblk[f + 1] - ix->fblk[f], ls = ix->last_size[f];
        if (nb && ls < n && src_len[f] >= ls) {
            tails.push_back({src_off[f] + src_len[f] - ls, ls, ix->fblk[f + 1] - 1});
            tail_file.push_back((uint32_t)f);
        }
    }
    std::vector<int> tail_flag(tails.size(), 0);
    DevBuf tail_buf;
    if (!tails.empty()) {
        const size_t bytes = tails.size() * sizeof(TailJob);
        HIP_TRY(hipMallocAsync(&tail_buf.p, bytes + tails.size() * sizeof(int), s));
        tail_buf.s = s;
        int* d_flag = (int*)((uint8_t*)tail_buf.p + bytes);
        HIP_TRY(hipMemcpyAsync(tail_buf.p, tails.data(), bytes, hipMemcpyHostToDevice, s));
        HIP_TRY(launch_tail(d_buf, (const TailJob*)tail_buf.p, (uint32_t)tails.size(), ix->d_weak, ix->d_strong, d_flag,
                            s));
        HIP_TRY(hipMemcpyAsync(tail_flag.data(), d_flag, tails.size() * sizeof(int), hipMemcpyDeviceToHost, s));
    }
    std::vector<uint64_t> hkey;
    std::vector<uint32_t> hval;
    if (!segs.empty()) {
        unsigned long long* d_counts = nullptr;
        DevBuf cnt_buf;
        HIP_TRY(hipMallocAsync((void**)&d_counts, 64, s));
        cnt_buf.p = d_counts; cnt_buf.s = s;
        DevBuf seg_buf, q_buf;
        size_t qcap = 0;
        if (!wide) {
            HIP_TRY(hipMallocAsync(&seg_buf.p, segs.size() * sizeof(ScanSeg), s));
            seg_buf.s = s;
            HIP_TRY(hipMemcpyAsync(seg_buf.p, segs.data(), segs.size() * sizeof(ScanSeg), hipMemcpyHostToDevice, s));
            qcap = scan_queue_entries();
            HIP_TRY(hipMallocAsync(&q_buf.p, qcap * sizeof(uint2), s));
            q_buf.s = s;
        }
        // verified hits: at most one per position; start from ~4 per block of positions
        uint64_t want = std::min<uint64_t>(tot_pos, tot_pos / n * 4 + (1 << 16));
        uint64_t cap = 0, nver = 0;
        unsigned long long counts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        DevBuf hit_buf;
        for (int attempt = 0; attempt < 2; ++attempt) {
            if (want > cap) {
                if (hit_buf.p) { (void)hipFreeAsync(hit_buf.p, s); hit_buf.p = nullptr; }
                cap = want;
                // keys [cap] + key scratch [cap] + values [cap] + value scratch [cap]
                HIP_TRY(hipMallocAsync(&hit_buf.p, cap * 24, s));
                hit_buf.s = s;
            }
            uint64_t* d_key = (uint64_t*)hit_buf.p;
            uint32_t* d_val = (uint32_t*)(d_key + 2 * cap);
            HIP_TRY(hipMemsetAsync(d_counts, 0, 64, s));
            if (!wide) {
                HIP_TRY(launch_scan(d_buf, (const ScanSeg*)seg_buf.p, (uint32_t)segs.size(), (uint32_t)ntiles,
                                    (uint32_t)n, ix->ix, ix->d_strong, d_key, d_val, cap, d_counts,
                                    (uint2*)q_buf.p, qcap, s, prof));
            } else {
                for (size_t g = 0; g < segs.size(); ++g)
                    HIP_TRY(launch_scan_wide(d_buf + segs[g].src, segs[g].len, segs[g].pos_begin, segs[g].pos_end,
                                             (uint32_t)g, (uint32_t)n, ix->ix, ix->d_strong, d_key, d_val, cap,
                                             d_counts, s, prof));
            }
            HIP_TRY(hipMemcpyAsync(counts, d_counts, 64, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            if (getenv("SYDELTA_PHASE_TIMING"))
                fprintf(stderr, "sydelta phase cycles (wave 0, summed over workgroups): stage %llu prefix %llu roll %llu flush %llu\n",
                        counts[4], counts[5], counts[6], counts[7]);
            if (counts[0] <= cap) break;
            want = counts[0];  // dense hits: grow once and rescan
        }
        nver = counts[0];
        b->total.weak_hits = counts[1];
        b->total.verified_hits = nver;
        if (nver) {
            uint64_t* d_key = (uint64_t*)hit_buf.p;
            uint32_t* d_val = (uint32_t*)(d_key + 2 * cap);
            uint64_t* k_out = nullptr;
            uint32_t* v_out = nullptr;
            const int end_bit = kSegShift + (int)ceil_log2(segs.size() + 1);
            {
                ProfScope ps(prof, s, "sort_hits");
                HIP_TRY(launch_sort_hits(d_key, d_val, d_key + cap, d_val + cap, nver, end_bit, s, &k_out, &v_out));
            }
            hkey.resize(nver);
            hval.resize(nver);
            HIP_TRY(hipMemcpyAsync(hkey.data(), k_out, nver * 8, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(hval.data(), v_out, nver * 4, hipMemcpyDeviceToHost, s));
        }
    }
    HIP_TRY(hipStreamSynchronize(s));
    // per-file op emission from the (segment, position)-sorted hits
    std::vector<int> tail_of(nf, 0);
    for (size_t j = 0; j < tails.size(); ++j) tail_of[tail_file[j]] = tail_flag[j];
    std::vector<uint64_t> pos;
    std::vector<uint32_t> blk;
    size_t h = 0;
    for (uint64_t f = 0; f < nf; ++f) {
        pos.clear();
        blk.clear();
        while (h < hkey.size() && seg_file[hkey[h] >> kSegShift] == f) {
            const ScanSeg& g = segs[hkey[h] >> kSegShift];
            pos.push_back(g.pos_begin + (hkey[h] & 0xFFFFFFFFull));
            blk.push_back(hval[h]);
            ++h;
        }
        sydelta_delta* d = &b->d[f];
        d->stats.verified_hits = pos.size();
        const uint64_t nb = ix->fblk[f + 1] - ix->fblk[f];
        emit_ops(pos.data(), blk.data(), pos.size(), ix->fblk[f], nb, n, ix->last_size[f], src_len[f], tail_of[f], d);
        b->total.copy_ops += d->stats.copy_ops;
        b->total.data_ops += d->stats.data_ops;
        b->total.literal_bytes += d->stats.literal_bytes;
    }
    if (nf == 1) b->d[0].stats.weak_hits = b->total.weak_hits;
    return SYDELTA_OK;
}

extern "C" int sydelta_match_device(sydelta_index* idx, const uint8_t* d_src, uint64_t len, void* stream,
                                    sydelta_delta** out) {
    if (!idx || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = nullptr;
    if (idx->nfiles != 1) return fail(SYDELTA_E_INVAL, "index holds %llu files; use sydelta_match_batch_device",
                                      (unsigned long long)idx->nfiles);
    if (len && !d_src) return fail(SYDELTA_E_INVAL, "NULL source");
    if (int r = ensure_device(idx->device)) return r;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(idx->device);
    sydelta_delta_batch b;
    const uint64_t off = 0;
    if (int r = match_impl(idx, d_src, &off, &len, s, &b)) return r;
    *out = new sydelta_delta(std::move(b.d[0]));
    return SYDELTA_OK;
}

extern "C" int sydelta_match_batch_device(sydelta_index* idx, const uint8_t* d_buf, const uint64_t* src_off,
                                          const uint64_t* src_len, uint64_t nfiles, void* stream,
                                          sydelta_delta_batch** out) {
    if (!idx || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = nullptr;
    if (nfiles != idx->nfiles) return fail(SYDELTA_E_INVAL, "index holds %llu files, %llu sources given",
                                           (unsigned long long)idx->nfiles, (unsigned long long)nfiles);
    if (nfiles && (!src_off || !src_len)) return fail(SYDELTA_E_INVAL, "NULL segment table");
    if (int r = ensure_device(idx->device)) return r;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(idx->device);
    std::unique_ptr<sydelta_delta_batch> b(new sydelta_delta_batch());
    if (int r = match_impl(idx, d_buf, src_off, src_len, s, b.get())) return r;
    *out = b.release();
    return SYDELTA_OK;
}

// ---------------------------------------------------------------------------
// host-buffer entry points
// ---------------------------------------------------------------------------
extern "C" int sydelta_compute_checksums_buf(int device, const uint8_t* buf, uint64_t len, uint64_t block_size,
                                             sydelta_block_checksum* out, uint64_t cap, uint64_t* n_out) {
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (!n_out) return fail(SYDELTA_E_INVAL, "n_out is NULL");
    const uint64_t nb = len ? (len + block_size - 1) / block_size : 0;  // checksum.rs:36-41
    *n_out = nb;
    if (!nb) return SYDELTA_OK;
    if (!buf || !out) return fail(SYDELTA_E_INVAL, "NULL buffer");
    if (cap < nb) return fail(SYDELTA_E_INVAL, "output holds %llu entries, need %llu", (unsigned long long)cap,
                              (unsigned long long)nb);
    if (int r = ensure_device(device)) return r;
    if (device < 0) device = 0;
    hipStream_t s = thread_stream(device);
    uint8_t* d_buf = nullptr;
    HIP_TRY(hipMallocAsync((void**)&d_buf, (len + 15) & ~15ull, s));
    DevBuf b1; b1.p = d_buf; b1.s = s;
    uint32_t* d_w = nullptr;
    HIP_TRY(hipMallocAsync((void**)&d_w, nb * 12 + 16, s));
    DevBuf b2; b2.p = d_w; b2.s = s;
    uint64_t* d_st = (uint64_t*)(((uintptr_t)(d_w + nb) + 7) & ~(uintptr_t)7);
    HIP_TRY(hipMemcpyAsync(d_buf, buf, len, hipMemcpyHostToDevice, s));
    CallProf cp;
    HIP_TRY(launch_signature(d_buf, len, block_size, d_w, d_st, s, cp.get()));
    std::vector<uint32_t> w(nb);
    std::vector<uint64_t> st(nb);
    HIP_TRY(hipMemcpyAsync(w.data(), d_w, 4 * nb, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(st.data(), d_st, 8 * nb, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (uint64_t i = 0; i < nb; ++i) {
        out[i].index = i;
        out[i].offset = i * block_size;
        out[i].size = std::min<uint64_t>(block_size, len - i * block_size);
        out[i].weak = w[i];
        out[i].reserved = 0;
        out[i].strong = st[i];
    }
    return SYDELTA_OK;
}

// Signatures from the caller must follow compute_checksums' layout (index order,
// offset = index*bs, full-size blocks except possibly the last).
static int check_sigs(const sydelta_block_checksum* sigs, uint64_t n, uint64_t bs, uint64_t* last_size) {
    *last_size = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (sigs[i].index != i || sigs[i].offset != i * bs)
            return fail(SYDELTA_E_INVAL, "checksum %llu is not in compute_checksums layout (index %llu, offset %llu)",
                        (unsigned long long)i, (unsigned long long)sigs[i].index, (unsigned long long)sigs[i].offset);
        const bool last = (i + 1 == n);
        if ((!last && sigs[i].size != bs) || (last && (sigs[i].size == 0 || sigs[i].size > bs)))
            return fail(SYDELTA_E_INVAL, "checksum %llu has size %llu (block size %llu)", (unsigned long long)i,
                        (unsigned long long)sigs[i].size, (unsigned long long)bs);
    }
    if (n) *last_size = sigs[n - 1].size;
    return SYDELTA_OK;
}

static int generate_from_host(int device, const uint8_t* src, uint64_t len, const sydelta_block_checksum* sigs,
                              uint64_t nsigs, uint64_t bs, sydelta_delta** out) {
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    if (bs == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (nsigs && !sigs) return fail(SYDELTA_E_INVAL, "NULL checksums");
    if (len && !src) return fail(SYDELTA_E_INVAL, "NULL source");
    uint64_t last_size = 0;
    if (int r = check_sigs(sigs, nsigs, bs, &last_size)) return r;
    if (int r = ensure_device(device)) return r;
    if (device < 0) device = 0;
    hipStream_t s = thread_stream(device);
    std::vector<uint32_t> w(nsigs);
    std::vector<uint64_t> st(nsigs);
    for (uint64_t i = 0; i < nsigs; ++i) { w[i] = sigs[i].weak; st[i] = sigs[i].strong; }
    sydelta_index* ix = nullptr;
    if (int r = sydelta_index_create(device, w.data(), st.data(), nsigs, bs, last_size, 0, s, &ix)) return r;
    std::unique_ptr<sydelta_index, void (*)(sydelta_index*)> ixg(ix, sydelta_index_free);
    uint8_t* d_src = nullptr;
    DevBuf b;
    if (len) {
        HIP_TRY(hipMallocAsync((void**)&d_src, (len + 15) & ~15ull, s));
        b.p = d_src; b.s = s;
        HIP_TRY(hipMemcpyAsync(d_src, src, len, hipMemcpyHostToDevice, s));
    }
    sydelta_delta_batch bt;
    const uint64_t off = 0;
    if (int r = match_impl(ix, d_src, &off, &len, s, &bt)) return r;
    std::unique_ptr<sydelta_delta> d(new sydelta_delta(std::move(bt.d[0])));
    // literal bytes: owned copy of each Data run (DeltaOp::Data(Vec<u8>))
    d->lit_off.assign(d->ops.size(), UINT64_MAX);
    uint64_t tot = 0;
    for (auto& o : d->ops) if (o.kind == SYDELTA_OP_DATA) tot += o.b;
    d->lit.resize(tot);
    uint64_t at = 0;
    for (size_t i = 0; i < d->ops.size(); ++i) {
        if (d->ops[i].kind != SYDELTA_OP_DATA) continue;
        memcpy(d->lit.data() + at, src + d->ops[i].a, d->ops[i].b);
        d->lit_off[i] = at;
        at += d->ops[i].b;
    }
    *out = d.release();
    return SYDELTA_OK;
}

extern "C" int sydelta_generate_delta_buf(int device, const uint8_t* src, uint64_t len,
                                          const sydelta_block_checksum* sigs, uint64_t nsigs, uint64_t block_size,
                                          sydelta_delta** out) {
    return generate_from_host(device, src, len, sigs, nsigs, block_size, out);
}

// ---------------------------------------------------------------------------
// path-level API (src/delta public functions)
// ---------------------------------------------------------------------------
static int read_file(const char* path, std::vector<uint8_t>& data) {
    if (!path) return fail(SYDELTA_E_INVAL, "path is NULL");
    FILE* f = fopen(path, "rb");
    if (!f) return fail(SYDELTA_E_IO, "%s: %s", path, strerror(errno));
    struct stat stt;
    if (fstat(fileno(f), &stt) != 0) {
        fclose(f);
        return fail(SYDELTA_E_IO, "%s: %s", path, strerror(errno));
    }
    data.resize((size_t)stt.st_size);
    size_t got = data.empty() ? 0 : fread(data.data(), 1, data.size(), f);
    const bool err = ferror(f);
    fclose(f);
    if (err || got != data.size()) return fail(SYDELTA_E_IO, "%s: short read", path);
    return SYDELTA_OK;
}

// checksum.rs:31-80
extern "C" int sydelta_compute_checksums(const char* path, uint64_t block_size, sydelta_block_checksum** out,
                                         uint64_t* n) {
    if (!out || !n) return fail(SYDELTA_E_INVAL, "NULL output");
    *out = nullptr;
    *n = 0;
    std::vector<uint8_t> data;
    if (int r = read_file(path, data)) return r;
    if (data.empty()) return SYDELTA_OK;  // checksum.rs:36-38
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    const uint64_t nb = (data.size() + block_size - 1) / block_size;
    sydelta_block_checksum* v = (sydelta_block_checksum*)malloc(sizeof(sydelta_block_checksum) * nb);
    if (!v) return fail(SYDELTA_E_OOM, "host allocation failed");
    uint64_t got = 0;
    if (int r = sydelta_compute_checksums_buf(-1, data.data(), data.size(), block_size, v, nb, &got)) {
        free(v);
        return r;
    }
    *out = v;
    *n = got;
    return SYDELTA_OK;
}

extern "C" void sydelta_checksums_free(sydelta_block_checksum* p) { free(p); }

// generator.rs:242
extern "C" int sydelta_generate_delta(const char* source_path, const sydelta_block_checksum* sigs, uint64_t nsigs,
                                      uint64_t block_size, sydelta_delta** out) {
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    std::vector<uint8_t> data;
    if (int r = read_file(source_path, data)) return r;
    return generate_from_host(-1, data.data(), data.size(), sigs, nsigs, block_size, out);
}

// generator.rs:67 — identical ops to generate_delta for block_size <= 128 KiB
// (SURVEY.md App. A R10); larger sizes are outside the production domain.
extern "C" int sydelta_generate_delta_streaming(const char* source_path, const sydelta_block_checksum* sigs,
                                                uint64_t nsigs, uint64_t block_size, sydelta_delta** out) {
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    if (block_size > 128 * 1024)
        return fail(SYDELTA_E_INVAL, "block_size %llu > 131072: streaming semantics diverge (see sydelta.h)",
                    (unsigned long long)block_size);
    return sydelta_generate_delta(source_path, sigs, nsigs, block_size, out);
}

// applier.rs:22-56 — receiver side, host I/O only.
extern "C" int sydelta_apply_delta(const char* old_file, const sydelta_delta* d, const char* new_file,
                                   sydelta_apply_stats* out) {
    if (!d || !old_file || !new_file) return fail(SYDELTA_E_INVAL, "NULL argument");
    if (d->lit_off.size() != d->ops.size())
        return fail(SYDELTA_E_INVAL, "delta has no literal bytes (device-only source)");
    FILE* old = fopen(old_file, "rb");
    if (!old) return fail(SYDELTA_E_IO, "%s: %s", old_file, strerror(errno));
    FILE* nw = fopen(new_file, "wb");
    if (!nw) {
        fclose(old);
        return fail(SYDELTA_E_IO, "%s: %s", new_file, strerror(errno));
    }
    uint64_t literal = 0, written = 0;
    std::vector<uint8_t> buf;
    int rc = SYDELTA_OK;
    for (size_t i = 0; i < d->ops.size() && rc == SYDELTA_OK; ++i) {
        const sydelta_op& o = d->ops[i];
        if (o.kind == SYDELTA_OP_COPY) {  // seek + read_exact + write_all (:31-40)
            buf.resize(o.b);
            if (fseeko(old, (off_t)o.a, SEEK_SET) != 0 || fread(buf.data(), 1, o.b, old) != o.b)
                rc = fail(SYDELTA_E_IO, "%s: failed to fill whole buffer", old_file);
            else if (fwrite(buf.data(), 1, o.b, nw) != o.b)
                rc = fail(SYDELTA_E_IO, "%s: write failed", new_file);
            written += o.b;
        } else {  // :41-46
            if (o.b && fwrite(d->lit.data() + d->lit_off[i], 1, o.b, nw) != o.b)
                rc = fail(SYDELTA_E_IO, "%s: write failed", new_file);
            literal += o.b;
            written += o.b;
        }
    }
    fclose(old);
    if (fclose(nw) != 0 && rc == SYDELTA_OK) rc = fail(SYDELTA_E_IO, "%s: flush failed", new_file);
    if (rc == SYDELTA_OK && out) {
        out->operations_count = d->ops.size();
        out->literal_bytes = literal;
        out->bytes_written = written;
    }
    return rc;
}

// rolling.rs:35-45
extern "C" uint32_t sydelta_adler32_hash(const uint8_t* data, uint64_t len) {
    uint32_t a = 1, b = 0;
    for (uint64_t i = 0; i < len; ++i) {
        a = (a + data[i]) % 65521u;
        b = (b + a) % 65521u;
    }
    return (b << 16) | a;
}

// ---------------------------------------------------------------------------
// synthetic data (bench)
// ---------------------------------------------------------------------------
extern "C" int sydelta_synth_fill(uint8_t* d_buf, uint64_t len, uint64_t seed, void* stream) {
    if (len && !d_buf) return fail(SYDELTA_E_INVAL, "NULL buffer");
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (int r = ensure_device(dev)) return r;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    HIP_TRY(launch_synth_fill(d_buf, len, seed, s));
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return SYDELTA_OK;
}

extern "C" int sydelta_synth_mutate(uint8_t* d_dst, const uint8_t* d_src, uint64_t len, uint64_t seed,
                                    uint32_t rate_ppm, void* stream) {
    if (len && (!d_dst || !d_src)) return fail(SYDELTA_E_INVAL, "NULL buffer");
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (int r = ensure_device(dev)) return r;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    HIP_TRY(launch_synth_mutate(d_dst, d_src, len, seed, rate_ppm, s));
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return SYDELTA_OK;
}
