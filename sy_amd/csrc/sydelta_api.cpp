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
// index
// ---------------------------------------------------------------------------
struct sydelta_index {
    int device = 0;
    uint64_t nblocks = 0, bs = 0, last_size = 0;
    uint32_t last_weak = 0;
    uint64_t last_strong = 0;
    uint32_t* d_weak = nullptr;   // owned copies
    uint64_t* d_strong = nullptr;
    DeviceIndex ix;
    void* d_pool = nullptr;       // one allocation for all index arrays
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

extern "C" int sydelta_index_create(int device, const uint32_t* weak, const uint64_t* strong, uint64_t nblocks,
                                    uint64_t block_size, uint64_t last_size, int arrays_on_device, void* stream,
                                    sydelta_index** out) {
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (nblocks && (!weak || !strong)) return fail(SYDELTA_E_INVAL, "NULL signature arrays");
    if (nblocks && (last_size == 0 || last_size > block_size))
        return fail(SYDELTA_E_INVAL, "last_size must be in [1, block_size]");
    if (nblocks >= 0xFFFFFFFFull) return fail(SYDELTA_E_INVAL, "too many blocks (%llu)", (unsigned long long)nblocks);
    if (int r = ensure_device(device)) return r;
    if (device < 0) device = 0;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device);
    std::unique_ptr<sydelta_index, void (*)(sydelta_index*)> x(new sydelta_index(), index_release);
    x->device = device;
    x->nblocks = nblocks;
    x->bs = block_size;
    x->last_size = nblocks ? last_size : 0;
    // sizes: Bloom filter in 32-bit words.  Up to kLdsFilterKeys keys it is at most
    // 2^13 words (32 KiB) and the LDS-staged scan holds it in LDS (>= 16 bits per key,
    // 128 bits per key for small bases); above that 16 bits per key in HBM/L2.
    // Exact table: buckets of 4 keys at load <= 0.5.
    const uint64_t nk = nblocks ? nblocks : 1;
    const uint32_t lk = ceil_log2(nk);
    const uint32_t fwbits = nk <= kLdsFilterKeys ? std::min<uint32_t>(13, std::max<uint32_t>(6, lk + 2))
                                                 : std::min<uint32_t>(28, lk - 1);
    const uint32_t bbits = std::max<uint32_t>(4, ceil_log2((nk + 1) / 2));
    const size_t nslots = ((size_t)1 << bbits) * 4;
    const size_t nb = std::max<uint64_t>(nblocks, 1);
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t sz_weak = al(4 * nb), sz_strong = al(8 * nb), sz_filt = al(((size_t)1 << fwbits) * 4);
    const size_t sz_t = al(4 * nslots), sz_order = al(4 * nb), sz_slot = al(4 * nb);
    const size_t total = sz_weak + sz_strong + sz_filt + 4 * sz_t + sz_order + sz_slot;
    HIP_TRY(hipMalloc(&x->d_pool, total));
    uint8_t* p = (uint8_t*)x->d_pool;
    x->d_weak = (uint32_t*)p; p += sz_weak;
    x->d_strong = (uint64_t*)p; p += sz_strong;
    x->ix.filt = (uint32_t*)p; p += sz_filt;
    x->ix.fwbits = fwbits;
    x->ix.keys = (uint32_t*)p; p += sz_t;
    x->ix.cnt = (uint32_t*)p; p += sz_t;
    x->ix.start = (uint32_t*)p; p += sz_t;
    x->ix.fill = (uint32_t*)p; p += sz_t;
    x->ix.order = (uint32_t*)p; p += sz_order;
    x->ix.slot_of = (uint32_t*)p; p += sz_slot;
    x->ix.bmask = (uint32_t)((1u << bbits) - 1);
    const hipMemcpyKind kind = arrays_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (nblocks) {
        HIP_TRY(hipMemcpyAsync(x->d_weak, weak, 4 * nblocks, kind, s));
        HIP_TRY(hipMemcpyAsync(x->d_strong, strong, 8 * nblocks, kind, s));
        if (arrays_on_device) {
            HIP_TRY(hipMemcpyAsync(&x->last_weak, weak + nblocks - 1, 4, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(&x->last_strong, strong + nblocks - 1, 8, hipMemcpyDeviceToHost, s));
        } else {
            x->last_weak = weak[nblocks - 1];
            x->last_strong = strong[nblocks - 1];
        }
    }
    CallProf cp;
    HIP_TRY(launch_index_build(x->d_weak, nblocks, x->ix, s, cp.get()));
    HIP_TRY(hipStreamSynchronize(s));
    *out = x.release();
    return SYDELTA_OK;
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

// Greedy op emission (generator.rs:116-221) from position-sorted verified hits.
void emit_ops(const std::vector<HitRec>& hits, const std::vector<uint64_t>& hit_pos, const sydelta_index* ix,
              uint64_t len, int tail_match, sydelta_delta* d) {
    const uint64_t n = ix->bs;
    uint64_t x = 0;
    auto data = [&](uint64_t a, uint64_t b) {
        if (b) {
            d->ops.push_back({SYDELTA_OP_DATA, 0, a, b});
            d->stats.data_ops++;
            d->stats.literal_bytes += b;
        }
    };
    auto copy = [&](uint64_t blk) {
        const uint64_t sz = (blk + 1 == ix->nblocks) ? ix->last_size : n;
        d->ops.push_back({SYDELTA_OP_COPY, 0, blk * n, sz});
        d->stats.copy_ops++;
    };
    for (size_t i = 0; i < hits.size(); ++i) {
        const uint64_t p = hit_pos[i];
        if (p < x) continue;  // inside the previous Copy: never visited
        data(x, p - x);
        copy(hits[i].slot);
        x = p + n;  // generator.rs:313 / :144
    }
    if (tail_match) {  // generator.rs:324-353: only p* = len - last_size can match
        const uint64_t pstar = len - ix->last_size;
        if (pstar >= x) {
            data(x, pstar - x);
            copy(ix->nblocks - 1);
            x = len;
        }
    }
    data(x, len - x);
}
}  // namespace

static int match_impl(sydelta_index* ix, const uint8_t* d_src, uint64_t len, hipStream_t s, sydelta_delta* d) {
    CallProf cp;
    Profiler* prof = cp.get();
    const uint64_t n = ix->bs;
    d->source_size = len;
    d->block_size = n;
    if (len == 0) return SYDELTA_OK;  // generator.rs:262-268
    if (((uintptr_t)d_src & 15) != 0) return fail(SYDELTA_E_INVAL, "device source must be 16-byte aligned");
    const uint64_t npos = (len >= n) ? len - n + 1 : 0;
    d->stats.positions = npos;
    std::vector<HitRec> all_hits;
    std::vector<uint64_t> all_pos;
    // tail check (async; read with the first sync)
    int tail_flag = 0;
    int* d_flag = nullptr;
    DevBuf flag_buf;
    const bool want_tail = ix->nblocks && ix->last_size < n && len >= ix->last_size;
    if (want_tail) {
        HIP_TRY(hipMallocAsync((void**)&d_flag, 16, s));
        flag_buf.p = d_flag; flag_buf.s = s;
        HIP_TRY(launch_tail(d_src, len, ix->last_size, ix->last_weak, ix->last_strong, d_flag, s));
        HIP_TRY(hipMemcpyAsync(&tail_flag, d_flag, sizeof(int), hipMemcpyDeviceToHost, s));
    }
    if (npos && ix->nblocks) {
        const uint64_t tile = scan_tile_positions();
        const uint64_t seg_max = (1ull << 31) / tile * tile;
        unsigned long long* d_counts = nullptr;
        DevBuf cnt_buf;
        HIP_TRY(hipMallocAsync((void**)&d_counts, 64, s));
        cnt_buf.p = d_counts; cnt_buf.s = s;
        const size_t qcap = scan_queue_entries();
        uint2* d_q = nullptr;
        DevBuf q_buf;
        HIP_TRY(hipMallocAsync((void**)&d_q, qcap * sizeof(uint2), s));
        q_buf.p = d_q; q_buf.s = s;
        uint64_t cap = 0;
        DevBuf hit_buf;
        for (uint64_t seg = 0; seg < npos; seg += seg_max) {
            const uint64_t seg_end = std::min(npos, seg + seg_max);
            const uint64_t seg_pos = seg_end - seg;
            // verified hits: at most one per position; start from ~4 per block of positions
            uint64_t want = std::max<uint64_t>(1 << 16, seg_pos / n * 4 + (1 << 16));
            want = std::min<uint64_t>(want, seg_pos);
            unsigned long long counts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int attempt = 0; attempt < 2; ++attempt) {
                if (want > cap) {
                    if (hit_buf.p) { (void)hipFreeAsync(hit_buf.p, s); hit_buf.p = nullptr; }
                    cap = want;
                    // verified hits [cap] + sort scratch [cap]
                    HIP_TRY(hipMallocAsync(&hit_buf.p, 2 * cap * sizeof(HitRec), s));
                    hit_buf.s = s;
                }
                HIP_TRY(hipMemsetAsync(d_counts, 0, 64, s));
                HIP_TRY(launch_scan(d_src, len, seg, seg_end, (uint32_t)n, ix->ix, ix->d_strong, (HitRec*)hit_buf.p,
                                    cap, d_counts, d_q, qcap, s, prof));
                HIP_TRY(hipMemcpyAsync(counts, d_counts, 64, hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                if (getenv("SYDELTA_PHASE_TIMING"))
                    fprintf(stderr, "sydelta phase cycles (wave 0, summed over workgroups): stage %llu prefix %llu roll %llu flush %llu\n",
                            counts[4], counts[5], counts[6], counts[7]);
                if (counts[0] <= cap) break;
                want = counts[0];  // dense hits: grow once and rescan
            }
            d->stats.weak_hits += counts[1];
            HitRec* d_ver = (HitRec*)hit_buf.p;
            HitRec* d_sort = d_ver + cap;
            const uint64_t nver = counts[0];
            d->stats.verified_hits += nver;
            if (nver) {
                HitRec* sorted = nullptr;
                {
                    ProfScope ps(prof, s, "sort_hits");
                    HIP_TRY(launch_sort_hits(d_ver, d_sort, nver, s, &sorted));
                }
                const size_t base = all_hits.size();
                all_hits.resize(base + nver);
                HIP_TRY(hipMemcpyAsync(all_hits.data() + base, sorted, nver * sizeof(HitRec), hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                all_pos.resize(base + nver);
                for (size_t i = base; i < base + nver; ++i) all_pos[i] = seg + all_hits[i].pos;
            }
        }
    }
    HIP_TRY(hipStreamSynchronize(s));
    emit_ops(all_hits, all_pos, ix, len, tail_flag, d);
    return SYDELTA_OK;
}

extern "C" int sydelta_match_device(sydelta_index* idx, const uint8_t* d_src, uint64_t len, void* stream,
                                    sydelta_delta** out) {
    if (!idx || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = nullptr;
    if (len && !d_src) return fail(SYDELTA_E_INVAL, "NULL source");
    if (int r = ensure_device(idx->device)) return r;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(idx->device);
    std::unique_ptr<sydelta_delta> d(new sydelta_delta());
    if (int r = match_impl(idx, d_src, len, s, d.get())) return r;
    *out = d.release();
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
    std::unique_ptr<sydelta_delta> d(new sydelta_delta());
    if (int r = match_impl(ix, d_src, len, s, d.get())) return r;
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
