// fake_device.cpp — TEST INFRASTRUCTURE, never part of libsydelta.  A host emulation
// of the device layer so that the library's host logic (classification bookkeeping,
// walks, chunked and streamed path API, batch API, change-ratio sampling) can run on a
// CPU-only machine: tests/test_host_emulated.py links the C ABI's host translation
// units against this file instead of libamdhip64 and the gfx950 kernels.
//
//   * HIP runtime calls: host memory, synchronous copies, one fake gfx950 device;
//   * the launch_* entry points of sydelta_internal.hpp: the same contracts computed
//     with the C oracle's Adler-32 / XXH3-64 (oracle/sydelta_oracle.c) and hash maps —
//     weak/strong per block, first candidate in index order with equal strong, hits
//     keyed (segment << 32 | position - pos_begin).
//
// It says nothing about the kernels themselves (the GPU tests do); it checks that the
// host code around them is right.
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <unordered_map>
#include <vector>

#include "sydelta_internal.hpp"

extern "C" uint64_t oracle_xxh3_64(const uint8_t* in, uint64_t len);

// ---------------------------------------------------------------------------
// HIP runtime
// ---------------------------------------------------------------------------
struct ihipStream_t {
    int dummy;
};
struct ihipEvent_t {
    int dummy;
};

// EMU_DEVICES=N (default 1): N emulated gfx950 devices sharing host memory; the current
// device is per thread, as in HIP.  emu_device_sets counts hipSetDevice calls per device.
static int emu_devices() {
    static const int n = [] {
        const char* e = getenv("EMU_DEVICES");
        const int v = e ? atoi(e) : 1;
        return v >= 1 && v <= 64 ? v : 1;
    }();
    return n;
}
static thread_local int t_cur_dev = 0;
static std::atomic<uint64_t> g_dev_sets[64];
extern "C" uint64_t emu_device_sets(int d) { return d >= 0 && d < 64 ? g_dev_sets[d].load() : 0; }
extern "C" {
hipError_t hipGetDeviceCount(int* n) {
    *n = emu_devices();
    return hipSuccess;
}
hipError_t hipGetDevice(int* d) {
    *d = t_cur_dev;
    return hipSuccess;
}
hipError_t hipSetDevice(int d) {
    if (d < 0 || d >= emu_devices()) return hipErrorInvalidDevice;
    t_cur_dev = d;
    ++g_dev_sets[d];
    return hipSuccess;
}
hipError_t hipDeviceCanAccessPeer(int* ok, int d, int p) {
    *ok = d != p && d < emu_devices() && p < emu_devices();
    return hipSuccess;
}
hipError_t hipDeviceEnablePeerAccess(int, unsigned int) { return hipSuccess; }
hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* p, int d) {
    if (d < 0 || d >= emu_devices()) return hipErrorInvalidDevice;
    memset(p, 0, sizeof(*p));
    strcpy(p->name, "host emulation");
    strcpy(p->gcnArchName, "gfx950:sramecc+:xnack-");
    p->multiProcessorCount = 256;
    return hipSuccess;
}
const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "no error" : "emulated HIP error"; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
    *s = new ihipStream_t();
    return hipSuccess;
}
hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned int f, int) { return hipStreamCreateWithFlags(s, f); }
hipError_t hipDeviceGetStreamPriorityRange(int* least, int* greatest) {
    *least = 0;
    *greatest = -1;
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned int) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* e) {
    *e = new ihipEvent_t();
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) {
    *ms = 0.f;
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
    delete e;
    return hipSuccess;
}
static int emu_pool_tag;
// Host profiles (tools/host_profile.py sets EMU_PROFILE=1): copies and memsets count as
// device time (DMA engines on the GPU), so memmoves a GPU run would not have on the host
// stay out of the host column.
static bool emu_profile() {
    static const bool on = [] { const char* e = getenv("EMU_PROFILE"); return e && e[0] == '1'; }();
    return on;
}
static void* emu_alloc(size_t n) {
    void* p = nullptr;
    if (posix_memalign(&p, 256, n ? n : 1)) return nullptr;
    return p;
}
static void emu_free(void* p) { free(p); }
static void emu_copy_time(uint64_t ns);
struct EmuCopyTimer {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~EmuCopyTimer() {
        if (emu_profile())
            emu_copy_time((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now() - t0).count());
    }
};
hipError_t hipMallocAsync(void** p, size_t n, hipStream_t) {
    *p = emu_alloc(n);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipMalloc(void** p, size_t n) { return hipMallocAsync(p, n, nullptr); }
hipError_t hipDeviceGetDefaultMemPool(hipMemPool_t* p, int d) {
    if (d < 0 || d >= emu_devices()) return hipErrorInvalidDevice;
    *p = (hipMemPool_t)&emu_pool_tag;
    return hipSuccess;
}
hipError_t hipMemPoolSetAttribute(hipMemPool_t, hipMemPoolAttr, void*) { return hipSuccess; }
hipError_t hipMemPoolCreate(hipMemPool_t* p, const hipMemPoolProps* props) {
    if (!props || props->location.id < 0 || props->location.id >= emu_devices()) return hipErrorInvalidDevice;
    *p = (hipMemPool_t)&emu_pool_tag;
    return hipSuccess;
}
hipError_t hipMallocFromPoolAsync(void** p, size_t n, hipMemPool_t pool, hipStream_t s) {
    if (pool != (hipMemPool_t)&emu_pool_tag) return hipErrorInvalidValue;
    // SYDELTA_EMU_POOL_CAP: pool allocations above that many bytes fail as on a full device
    if (const char* e = getenv("SYDELTA_EMU_POOL_CAP"))
        if (n > strtoull(e, nullptr, 10)) return hipErrorOutOfMemory;
    return hipMallocAsync(p, n, s);
}
hipError_t hipFreeAsync(void* p, hipStream_t) {
    emu_free(p);
    return hipSuccess;
}
hipError_t hipFree(void* p) {
    emu_free(p);
    return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned int) { return hipMallocAsync(p, n, nullptr); }
hipError_t hipHostFree(void* p) {
    emu_free(p);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
    EmuCopyTimer t;
    if (n) memmove(d, s, n);
    return hipSuccess;
}
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind k) { return hipMemcpyAsync(d, s, n, k, nullptr); }
hipError_t hipMemcpyPeerAsync(void* d, int dd, const void* s, int sd, size_t n, hipStream_t st) {
    if (dd < 0 || dd >= emu_devices() || sd < 0 || sd >= emu_devices()) return hipErrorInvalidDevice;
    return hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, st);
}
hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) {
    EmuCopyTimer t;
    memset(d, v, n);
    return hipSuccess;
}
hipError_t hipGetLastError() { return hipSuccess; }
}

// ---------------------------------------------------------------------------
// device layer
// ---------------------------------------------------------------------------
// Time spent inside the emulated launches, so a host profile can subtract it
// (tools/host_profile.py): emu_kernel_ms(reset).
static std::atomic<uint64_t> g_emu_ns{0};
static thread_local int t_emu_depth = 0;
static void emu_copy_time(uint64_t ns) {
    if (t_emu_depth == 0) g_emu_ns += ns;  // inside an emulated launch it is counted already
}
struct EmuTimer {  // the outermost launch of a nest counts
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    EmuTimer() { ++t_emu_depth; }
    ~EmuTimer() {
        if (--t_emu_depth == 0)
            g_emu_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now() - t0)
                            .count();
    }
};
extern "C" double emu_kernel_ms(int reset) {
    const double ms = g_emu_ns.load() / 1e6;
    if (reset) g_emu_ns = 0;
    return ms;
}

namespace sydelta {
namespace {
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kMod = 65521;

struct Cand {
    uint32_t blk;
    uint64_t strong;
};
struct FakeIndex {
    std::vector<std::unordered_map<uint32_t, std::vector<Cand>>> files;  // weak -> candidates in index order
    std::vector<uint64_t> any;  // 2^26-bit filter over (file, weak): a fast reject before the map
};
inline uint64_t any_bit(uint32_t file, uint32_t w) { return ((uint64_t)w * 0x9E3779B97F4A7C15ull + file * 0xC2B2AE3D27D4EB4Full) >> 38; }

// Adler-32 (zlib), the modulus deferred over 5552-byte runs
uint32_t adler(const uint8_t* p, uint64_t n) {
    uint64_t a = 1, b = 0;
    while (n) {
        const uint64_t k = n < 5552 ? n : 5552;
        for (uint64_t i = 0; i < k; ++i) {
            a += p[i];
            b += a;
        }
        a %= kMod;
        b %= kMod;
        p += k;
        n -= k;
    }
    return (uint32_t)((b << 16) | a);
}
std::mutex g_mu;
std::map<const void*, FakeIndex> g_ix;  // keyed by the index's `keys` array

const FakeIndex& find_ix(const DeviceIndex& ix) {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_ix.at(ix.keys);
}

// first candidate in index order with equal strong (generator.rs:127-133), or kNone
uint32_t lookup(const FakeIndex& F, uint32_t file, uint32_t weak, const uint8_t* win, uint64_t n, bool* weak_hit) {
    const uint64_t bit = any_bit(file, weak);
    if (!((F.any[bit >> 6] >> (bit & 63)) & 1)) return kNone;
    const auto& m = F.files[file];
    auto it = m.find(weak);
    if (it == m.end()) return kNone;
    if (weak_hit) *weak_hit = true;
    const uint64_t st = oracle_xxh3_64(win, n);
    for (const Cand& c : it->second)
        if (c.strong == st) return c.blk;
    return kNone;
}

// classify window starts [p0, p1) of src (len bytes) against file `file`; hits to the output
void scan_range(const FakeIndex& F, uint32_t file, const uint8_t* src, uint64_t p0, uint64_t p1, uint64_t n,
                uint64_t key_hi, uint64_t* key, uint32_t* val, uint64_t cap, unsigned long long* counters) {
    if (p0 >= p1) return;
    uint64_t a = 1, b = 0;  // Adler of [p0, p0+n)
    for (uint64_t i = 0; i < n; ++i) {
        a = (a + src[p0 + i]) % kMod;
        b = (b + a) % kMod;
    }
    for (uint64_t p = p0;; ++p) {
        bool wh = false;
        const uint32_t w = (uint32_t)((b << 16) | a);
        const uint32_t blk = lookup(F, file, w, src + p, n, &wh);
        if (wh) counters[1]++;
        if (blk != kNone) {
            const unsigned long long k = counters[0]++;
            if (k < cap) {
                key[k] = key_hi | (p - p0);
                val[k] = blk;
            }
        }
        if (p + 1 >= p1) break;
        const uint64_t out = src[p], in = src[p + n];  // rolling.rs:66-79
        a = (a + 2 * kMod - out + in) % kMod;
        b = (b + 3 * kMod - (n * out) % kMod + a - 1) % kMod;
    }
}
}  // namespace

hipError_t launch_signature(const uint8_t* d_buf, uint64_t len, uint64_t bs, uint32_t* d_weak, uint64_t* d_strong,
                            hipStream_t, Profiler*) {
    EmuTimer emu_t;
    const uint64_t nb = (len + bs - 1) / bs;
    for (uint64_t k = 0; k < nb; ++k) {
        const uint64_t sz = std::min(bs, len - k * bs);
        d_weak[k] = adler(d_buf + k * bs, sz);
        d_strong[k] = oracle_xxh3_64(d_buf + k * bs, sz);
    }
    return hipSuccess;
}

hipError_t launch_signature_batch(const uint8_t* d_buf, const uint64_t* d_off, const uint64_t* d_len,
                                  const uint64_t* d_fblk, uint64_t nfiles, uint64_t bs, uint64_t, uint32_t* d_weak,
                                  uint64_t* d_strong, hipStream_t s, Profiler* p) {
    EmuTimer emu_t;
    for (uint64_t f = 0; f < nfiles; ++f)
        launch_signature(d_buf + d_off[f], d_len[f], bs, d_weak + d_fblk[f], d_strong + d_fblk[f], s, p);
    return hipSuccess;
}

hipError_t launch_signature_batch_fast(const uint8_t* d_buf, const uint64_t* d_aoff, const uint64_t* d_agb,
                                       const uint64_t* d_apfx, uint64_t nact, uint64_t, const uint64_t* d_loff,
                                       const uint64_t* d_llen, const uint64_t* d_lidx, uint64_t npart, uint64_t bs,
                                       uint32_t* d_weak, uint64_t* d_strong, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    for (uint64_t f = 0; f < nact; ++f)
        for (uint64_t j = 0; j < d_apfx[f + 1] - d_apfx[f]; ++j) {
            const uint8_t* b = d_buf + d_aoff[f] + j * bs;
            d_weak[d_agb[f] + j] = adler(b, bs);
            d_strong[d_agb[f] + j] = oracle_xxh3_64(b, bs);
        }
    for (uint64_t i = 0; i < npart; ++i) {
        d_weak[d_lidx[i]] = adler(d_buf + d_loff[i], d_llen[i]);
        d_strong[d_lidx[i]] = oracle_xxh3_64(d_buf + d_loff[i], d_llen[i]);
    }
    return hipSuccess;
}

// the emulated scans test windows against the exact keys, so the level-1 filters are not built
hipError_t launch_ribbon_build(const DeviceIndex&, hipStream_t, Profiler*, const uint32_t*, uint64_t) { return hipSuccess; }

hipError_t launch_index_extras(const uint32_t*, const DeviceIndex&, hipStream_t, Profiler*) { return hipSuccess; }
hipError_t launch_index_build(const uint32_t* d_weak, const uint64_t* d_strong, DeviceIndex& ix, hipStream_t,
                              Profiler*, bool) {
    EmuTimer emu_t;
    FakeIndex F;
    F.files.resize(ix.nfiles);
    F.any.assign((1ull << 26) / 64, 0);
    for (uint64_t f = 0; f < ix.nfiles; ++f)
        for (uint64_t k = ix.d_fblk[f]; k < ix.d_fblk[f + 1]; ++k) {
            F.files[f][d_weak[k]].push_back({(uint32_t)k, d_strong[k]});
            const uint64_t bit = any_bit((uint32_t)f, d_weak[k]);
            F.any[bit >> 6] |= 1ull << (bit & 63);
        }
    std::lock_guard<std::mutex> lk(g_mu);
    g_ix[ix.keys] = std::move(F);
    return hipSuccess;
}

uint64_t scan_tile_positions() { return 16384; }
int scan_wide_mode() {
    const char* e = getenv("SYDELTA_SCAN_WIDE");
    return (e && e[0] == '0') ? 0 : 1;
}
uint32_t scan_max_window() { return 8192; }
size_t scan_queue_entries() { return 1024; }

hipError_t launch_scan(const uint8_t* d_buf, const ScanSeg* d_segs, uint32_t nsegs, uint32_t, uint32_t n,
                       const DeviceIndex& ix, const uint64_t*, uint64_t* d_hit_key, uint32_t* d_hit_val,
                       uint64_t out_cap, unsigned long long* d_counters, uint2*, size_t, hipStream_t, Profiler*,
                       DevScratch*) {
    EmuTimer emu_t;
    const FakeIndex& F = find_ix(ix);
    for (uint32_t g = 0; g < nsegs; ++g) {
        const ScanSeg& S = d_segs[g];
        scan_range(F, S.file, d_buf + S.src, S.pos_begin, S.pos_end, n, (uint64_t)g << kSegShift, d_hit_key, d_hit_val,
                   out_cap, d_counters);
    }
    return hipSuccess;
}

hipError_t launch_scan_wide(const uint8_t* d_src, uint64_t, uint64_t pos_begin, uint64_t pos_end, uint32_t seg_id,
                            uint32_t n, const DeviceIndex& ix, const uint64_t*, uint64_t* d_hit_key,
                            uint32_t* d_hit_val, uint64_t out_cap, unsigned long long* d_counters, hipStream_t,
                            Profiler*) {
    EmuTimer emu_t;
    scan_range(find_ix(ix), 0, d_src, pos_begin, pos_end, n, (uint64_t)seg_id << kSegShift, d_hit_key, d_hit_val,
               out_cap, d_counters);
    return hipSuccess;
}

hipError_t launch_sort_hits(uint64_t* key, uint32_t* val, uint64_t*, uint32_t*, uint64_t nhits, int, hipStream_t,
                            uint64_t** key_out, uint32_t** val_out) {
    EmuTimer emu_t;
    std::vector<uint64_t> idx(nhits);
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](uint64_t x, uint64_t y) { return key[x] < key[y]; });
    std::vector<uint64_t> k2(nhits);
    std::vector<uint32_t> v2(nhits);
    for (uint64_t i = 0; i < nhits; ++i) {
        k2[i] = key[idx[i]];
        v2[i] = val[idx[i]];
    }
    std::copy(k2.begin(), k2.end(), key);
    std::copy(v2.begin(), v2.end(), val);
    *key_out = key;
    *val_out = val;
    return hipSuccess;
}

hipError_t launch_probe(const uint8_t* d_base, const ProbeJob* d_jobs, uint32_t njobs, uint64_t nprobes,
                        uint32_t stride, uint32_t n, bool, const DeviceIndex& ix, uint32_t* d_pw, uint64_t* d_pst,
                        uint32_t* d_out, hipStream_t, Profiler*, int phases) {
    EmuTimer emu_t;
    for (uint32_t j = 0; j < njobs; ++j) {
        const uint64_t end = j + 1 < njobs ? d_jobs[j + 1].pfx : nprobes;
        for (uint64_t w = d_jobs[j].pfx; w < end; ++w) {
            const uint64_t k = d_jobs[j].k0 + (w - d_jobs[j].pfx) * stride;
            const uint8_t* win = d_base + d_jobs[j].src + k * n;
            if (phases & 1) {
                d_pw[w] = adler(win, n);
                d_pst[w] = oracle_xxh3_64(win, n);
            }
            if (phases & 2) {
                if (d_pw[w] != adler(win, n)) return hipErrorInvalidValue;  // looked up before it was hashed
                d_out[w] = lookup(find_ix(ix), d_jobs[j].file, d_pw[w], win, n, nullptr);
            }
        }
    }
    return hipSuccess;
}

hipError_t launch_tail(const uint8_t* d_buf, const TailJob* d_jobs, uint32_t njobs, const uint32_t* d_weak,
                       const uint64_t* d_strong, int* d_flag, hipStream_t) {
    EmuTimer emu_t;
    for (uint32_t i = 0; i < njobs; ++i) {
        const uint8_t* p = d_buf + d_jobs[i].src;
        const uint64_t L = d_jobs[i].last_size, b = d_jobs[i].blk;
        d_flag[i] = adler(p, L) == d_weak[b] && oracle_xxh3_64(p, L) == d_strong[b];
    }
    return hipSuccess;
}

hipError_t launch_apply(const ApplyPiece* d_pieces, uint64_t npieces, const uint8_t* d_basis, const uint8_t* d_lit,
                        uint8_t* d_out, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    for (uint64_t i = 0; i < npieces; ++i) {
        const ApplyPiece& p = d_pieces[i];
        memcpy(d_out + p.dst, (p.from_basis ? d_basis : d_lit) + p.src, p.len);
    }
    return hipSuccess;
}

hipError_t launch_json_len(const JsonPiece*, uint64_t, const uint8_t*, uint64_t*, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    return hipErrorNotSupported;
}
hipError_t launch_json_write(const JsonPiece*, uint64_t, const uint8_t*, const uint64_t*, uint64_t, uint8_t*,
                             hipStream_t, Profiler*) {
    EmuTimer emu_t;
    return hipErrorNotSupported;
}
// K7s: the kernels' per-thread bodies (sydelta_sigjson.hpp) tile by tile; each tile's
// text is staged in an array of exactly its length and stored chunk by chunk, the
// chunks in descending order (one schedule of the workgroup's threads).
hipError_t launch_sigjson_len(const sigjson::SigArgs& a, uint64_t* d_tile_len, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    const uint64_t nt = (a.n + sigjson::kTile - 1) / sigjson::kTile;
    for (uint64_t t = 0; t < nt; ++t) {
        uint64_t tot = 0;
        for (uint64_t i = t * sigjson::kTile; i < std::min<uint64_t>(a.n, (t + 1) * sigjson::kTile); ++i)
            tot += sigjson::entry_len(a, i);
        d_tile_len[t] = tot;
    }
    return hipSuccess;
}
hipError_t launch_sigjson_write(const sigjson::SigArgs& a, const uint64_t* d_tile_off, uint8_t* d_out, hipStream_t,
                                Profiler*) {
    EmuTimer emu_t;
    const uint64_t nt = (a.n + sigjson::kTile - 1) / sigjson::kTile;
    for (uint64_t t = 0; t < nt; ++t) {
        const uint64_t i0 = t * sigjson::kTile, i1 = std::min<uint64_t>(a.n, i0 + sigjson::kTile);
        std::vector<uint32_t> off(i1 - i0 + 1, 0);
        for (uint64_t i = i0; i < i1; ++i) off[i - i0 + 1] = off[i - i0] + sigjson::entry_len(a, i);
        const uint32_t tot = off[i1 - i0];
        std::unique_ptr<uint8_t[]> stage(new uint8_t[tot ? tot : 1]);
        for (uint64_t i = i0; i < i1; ++i)
            if (sigjson::entry_write(a, i, stage.get() + off[i - i0]) != off[i - i0 + 1] - off[i - i0])
                return hipErrorLaunchFailure;
        uint8_t* dst = d_out + d_tile_off[t];
        const uintptr_t c0 = (uintptr_t)dst & ~(uintptr_t)15, c1 = ((uintptr_t)dst + tot + 15) & ~(uintptr_t)15;
        for (uintptr_t c = c1; c > c0;) {
            c -= 16;
            sigjson::store_chunk(stage.get(), tot, dst, c);
        }
    }
    return hipSuccess;
}
// K7p: chunk_entries / chunk_parse per chunk (the chunks in descending order).
hipError_t launch_sigparse_count(const uint8_t* d_text, uint64_t len, uint64_t* d_count, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    const uint64_t nc = (len + sigjson::kParseChunk - 1) / sigjson::kParseChunk;
    for (uint64_t c = 0; c < nc; ++c) d_count[c] = sigjson::chunk_entries(d_text, len, c);
    return hipSuccess;
}
hipError_t launch_sigparse(const uint8_t* d_text, uint64_t len, const uint64_t* d_rank, sydelta_block_checksum* d_out,
                           uint64_t cap, unsigned long long* d_bad, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    const uint64_t nc = (len + sigjson::kParseChunk - 1) / sigjson::kParseChunk;
    for (uint64_t c = nc; c-- > 0;) {
        const uint64_t b = sigjson::chunk_parse(d_text, len, c, d_rank[c], d_out, cap);
        if (b < *d_bad) *d_bad = b;
    }
    return hipSuccess;
}
// K7d: sydelta_dparse.hpp's chunk bodies per chunk (parse in descending chunk order).
hipError_t launch_dparse_count(const dparse::DArgs& a, uint64_t* d_ocnt, uint64_t* d_lcnt, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    for (uint64_t c = 0; c < a.nc; ++c) dparse::chunk_count(a, c, d_ocnt[c], d_lcnt[c]);
    return hipSuccess;
}
hipError_t launch_dparse_place(const dparse::DArgs& a, const uint64_t* d_orank, uint64_t* d_pos, hipStream_t,
                               Profiler*) {
    EmuTimer emu_t;
    for (uint64_t c = 0; c < a.nc; ++c) dparse::chunk_place(a, c, d_orank[c], d_pos);
    return hipSuccess;
}
hipError_t launch_dparse(const dparse::DArgs& a, const uint64_t* d_orank, const uint64_t* d_lrank, const uint64_t* d_pos,
                         uint64_t nops, sydelta_op* d_ops, uint8_t* d_lit, unsigned long long* d_bad, hipStream_t,
                         Profiler*) {
    EmuTimer emu_t;
    for (uint64_t c = a.nc; c-- > 0;) {
        const uint64_t b = dparse::chunk_parse(a, c, d_orank, d_lrank, d_pos, nops, d_ops, d_lit);
        if (b < *d_bad) *d_bad = b;
    }
    return hipSuccess;
}
// K5b: the kernels' own per-thread bodies (sydelta_chain.hpp) in the launch order of
// sydelta_kernels.hip's launch_chain, one loop per kernel.  The marking levels run their
// threads alternately forward and backward: two of the schedules a GPU may produce for
// a launch whose threads read marks that others of the same launch write.
hipError_t launch_chain(const chain::ChainArgs& a, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    if (a.M + 2 >= (1ull << 31) || a.nblk + 1 >= (1ull << 31) || a.K == 0 || a.K > 32) return hipErrorInvalidValue;
    if ((1ull << a.K) <= a.M + 1) return hipErrorInvalidValue;
    const uint64_t W = a.M + 2;
    memset(a.res, 0, sizeof(chain::ChainResult));
    auto excl = [](const uint32_t* in, uint32_t* out, uint64_t n) {
        uint32_t acc = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t v = in[i];
            out[i] = acc;
            acc += v;
        }
    };
    if (a.probed) {
        for (uint64_t k = 0; k <= a.nblk; ++k) chain::chain_flag(a, k);
        excl(a.aflag, a.apfx, a.nblk + 1);
        for (uint64_t k = 0; k < a.nblk; ++k) chain::chain_place_aligned(a, k);
    }
    for (uint64_t h = 0; h < a.H; ++h) chain::chain_place_scan(a, h);
    for (uint64_t i = 0; i < W; ++i) chain::chain_succ(a, i);
    for (uint32_t l = 0; l + 1 < a.K; ++l)
        for (uint64_t i = 0; i < W; ++i) chain::chain_lift(a, l, i);
    memset(a.on, 0, W);
    chain::chain_entry(a);
    for (uint32_t l = a.K; l-- > 0;) {
        if (l & 1)
            for (uint64_t i = W; i-- > 0;) chain::chain_mark(a, l, i);
        else
            for (uint64_t i = 0; i < W; ++i) chain::chain_mark(a, l, i);
    }
    for (uint64_t i = 0; i <= a.M; ++i) chain::chain_count(a, i);
    excl(a.cnt, a.off, a.M + 1);
    for (uint64_t i = 0; i < a.M; ++i) {
        const uint64_t lit = chain::chain_emit(a, i);
        if (lit) {
            a.res->data_ops += 1;
            a.res->lit_bytes += lit;
        }
    }
    chain::chain_finish(a);
    return hipSuccess;
}

// K10: each unit's greedy walk (generator.rs:116-221) from its entry until it leaves
// [entry, end), every visited window classified exactly, the ops run-length coded as
// k_walk_files writes them (WalkRec), units placed in order in the compact output.  The
// aligned probe's results, when given, must agree with the exact classification.
void walk_expand(const ExpandArgs& a, uint64_t u_lo, uint64_t u_hi);  // (below)
hipError_t launch_walk_files(const WalkArgs& a, hipStream_t, Profiler*, bool slim) {
    EmuTimer emu_t;
    if (slim) return a.ahit && !a.self_nb ? hipSuccess : hipErrorInvalidValue;  // the full launch after it walks every unit
    if (a.n % 64 != 0 || a.n < 256 || a.n > kWalkMaxN || a.self_nb > kSelfIxMaxBlocks) return hipErrorInvalidValue;
    FakeIndex self;  // self-indexed (a batch's walks): the units' files' candidates from the signature
    if (a.self_nb) {
        uint32_t nfl = 0;
        for (uint32_t u = 0; u < a.nunits; ++u) nfl = std::max(nfl, a.units[u].file + 1);
        self.files.resize(nfl);
        self.any.assign((1ull << 26) / 64, 0);
        for (uint32_t f = 0; f < nfl; ++f) {
            if (a.fblk[f + 1] - a.fblk[f] > a.self_nb) return hipErrorInvalidValue;  // the kernel's LDS would overflow
            for (uint64_t k = a.fblk[f]; k < a.fblk[f + 1]; ++k) {
                self.files[f][a.weak[k]].push_back({(uint32_t)k, a.strong[k]});
                const uint64_t bit = any_bit(f, a.weak[k]);
                self.any[bit >> 6] |= 1ull << (bit & 63);
            }
        }
    }
    DeviceIndex key_ix;
    key_ix.keys = (uint32_t*)a.keys;
    const FakeIndex& F = a.self_nb ? self : find_ix(key_ix);
    const uint64_t n = a.n;
    uint64_t placed = *a.total;
    for (uint32_t u = 0; u < a.nunits; ++u) {
        const WalkUnit& U = a.units[u];
        const uint8_t* src = a.base + U.src;
        const uint64_t len = U.len, gb0 = a.fblk[U.file], nbf = a.fblk[U.file + 1] - gb0, ls = a.last_size[U.file];
        std::vector<WalkRec> rec;
        uint32_t ck = 0, ca = 0, weak_hits = 0, hits = 0;
        auto close_run = [&] {
            if (ck) rec.push_back({ck, ca, 0});
            ck = 0;
        };
        auto data = [&](uint64_t lo, uint64_t hi) {
            if (hi > lo) {
                close_run();
                rec.push_back({0, (uint32_t)(hi - lo), lo});
            }
        };
        auto copy = [&](uint32_t g) {
            if (ck && g == ca + ck) {
                ++ck;
            } else {
                close_run();
                ck = 1;
                ca = g;
            }
        };
        uint64_t wa = 0, wb = 0, wpos = UINT64_MAX;  // rolling Adler state of the window at wpos
        bool probe_ok = true;
        auto classify = [&](uint64_t x) {
            if (wpos != UINT64_MAX && x == wpos + 1) {
                const uint64_t out = src[wpos], in = src[wpos + n];
                wa = (wa + 2 * kMod - out + in) % kMod;
                wb = (wb + 3 * kMod - (n * out) % kMod + wa - 1) % kMod;
            } else {
                const uint32_t w = adler(src + x, n);
                wa = w & 0xFFFF;
                wb = w >> 16;
            }
            wpos = x;
            bool wh = false;
            const uint32_t w = (uint32_t)((wb << 16) | wa);
            const uint32_t blk = lookup(F, U.file, w, src + x, n, &wh);
            weak_hits += wh;
            if (a.ahit && x % n == 0) {
                const uint32_t h = a.ahit[x / n - U.kb];
                if (h != kNone && h >= kPreMark)  // pre-rolled: a miss here
                    probe_ok = probe_ok && blk == kNone;
                else if (h != blk || a.apw[x / n - U.kb] != w)
                    probe_ok = false;
            }
            return blk;
        };
        uint64_t x = U.entry, lit = U.entry;
        while (x < U.end) {
            const uint32_t blk = classify(x);
            if (a.ahit && blk == kNone && x % n == 0 && a.ahit[x / n - U.kb] != kNone) {  // pre-rolled
                const uint32_t h = a.ahit[x / n - U.kb];
                if (h != kPreNone) {  // its first hit must be a hit
                    const uint64_t q = x + (a.apw[x / n - U.kb] & 0x3FFF);
                    bool wh = false;
                    if (q <= x || q >= x + n || lookup(F, U.file, adler(src + q, n), src + q, n, &wh) != (h & ~kPreMark))
                        return hipErrorInvalidValue;
                }
            }
            if (blk != kNone) {
                ++hits;
                data(lit, x);
                copy(blk);
                x += n;
                lit = x;
            } else {
                ++x;
            }
        }
        if (!probe_ok) return hipErrorInvalidValue;  // the host handed over wrong probe results
        uint64_t exit;
        if (U.final_) {
            if (nbf && ls < n && len >= ls && len - ls >= lit && adler(src + len - ls, ls) == a.weak[gb0 + nbf - 1] &&
                oracle_xxh3_64(src + len - ls, ls) == a.strong[gb0 + nbf - 1]) {
                data(lit, len - ls);
                copy((uint32_t)(gb0 + nbf - 1));
                lit = len;
                ++hits;
            }
            data(lit, len);
            exit = len;
        } else {
            data(lit, U.end);
            exit = std::max(x, U.end);
        }
        close_run();
        const uint64_t cap = 2 * ((U.end - U.entry) / n) + 4;
        if (rec.size() > cap) return hipErrorInvalidValue;  // the kernel's staging region would overflow
        std::copy(rec.begin(), rec.end(), a.stage + U.rec_off);  // (the kernel stages every unit's records)
        if (!a.out) {  // records left in the staging region
            a.fout[u] = WalkFileOut{(uint32_t)U.rec_off, (uint32_t)rec.size(), weak_hits, hits, exit, 0};
            if (a.fout_dev) a.fout_dev[u] = a.fout[u];
            continue;
        }
        std::copy(rec.begin(), rec.end(), a.out + placed);
        a.fout[u] = WalkFileOut{(uint32_t)placed, (uint32_t)rec.size(), weak_hits, hits, exit, 0};
        if (a.fout_dev) a.fout_dev[u] = a.fout[u];
        placed += rec.size();
    }
    if (a.out) *a.total = placed;
    if (a.x.ops) {  // (the kernel: each file's last unit to finish) the files whose units were all in this launch
        const uint64_t u_lo = (uint64_t)(a.units - a.x.units);
        walk_expand(a.x, u_lo, u_lo + a.nunits);
    }
    return hipSuccess;
}

// k_walk_expand: each file's units' staged records chained (a unit entered past its start cut
// at the previous exit when its leading literal run reaches it, else the file is bad), Data
// ops joined across units, expanded into ops at ops + op_off[f]
std::atomic<uint64_t> g_expand_files{0};  // files expanded (emu_expand_files)
void walk_expand(const ExpandArgs& a, uint64_t u_lo, uint64_t u_hi) {
    for (uint32_t f = 0; f < a.nf; ++f) {
        if (a.fu[f] < u_lo || a.fu[f + 1] > u_hi) continue;
        ++g_expand_files;
        std::vector<WalkRec> m;
        bool bad = false;
        uint32_t wh = 0, vh = 0;
        for (uint32_t u = a.fu[f]; u < a.fu[f + 1] && !bad; ++u) {
            const WalkFileOut& o = a.fout[u];
            wh += o.weak_hits;
            vh += o.hits;
            const WalkRec* r0 = a.stage + a.units[u].rec_off;
            const WalkRec* r1 = r0 + o.count;
            std::vector<WalkRec> rs(r0, r1);
            size_t k0 = 0;
            if (u > a.fu[f]) {
                const uint64_t pe = a.fout[u - 1].exit, entry = a.units[u].entry;
                if (entry != pe) {
                    if (pe > entry && !rs.empty() && rs[0].kind == 0 && rs[0].off == entry && rs[0].off + rs[0].a >= pe) {
                        const uint64_t h = rs[0].off + rs[0].a;
                        if (h == pe) {
                            k0 = 1;
                        } else {
                            rs[0].a = (uint32_t)(h - pe);
                            rs[0].off = pe;
                        }
                    } else {
                        bad = true;
                    }
                }
            }
            for (size_t k = k0; k < rs.size() && !bad; ++k) {
                if (!rs[k].kind && !m.empty() && !m.back().kind && m.back().off + m.back().a == rs[k].off)
                    m.back().a += rs[k].a;
                else
                    m.push_back(rs[k]);
            }
        }
        uint64_t nops = 0, nd = 0, lit = 0;
        for (const WalkRec& x : m) {
            nops += x.kind ? x.kind : 1;
            if (!x.kind) {
                ++nd;
                lit += x.a;
            }
        }
        if (bad || nops > a.op_off[f + 1] - a.op_off[f]) {
            a.res[f] = ExpandOut{0, 0, 0, 0, 0, 1, 0};
            continue;
        }
        const uint64_t gb0 = a.fblk[f], nbf = a.fblk[f + 1] - gb0, ls = a.last_size[f];
        sydelta_op* w = a.ops + a.op_off[f];
        for (const WalkRec& x : m) {
            if (!x.kind) {
                *w++ = sydelta_op{SYDELTA_OP_DATA, 0, x.off, x.a};
                continue;
            }
            for (uint64_t g = x.a - gb0, e = g + x.kind; g < e; ++g)
                *w++ = sydelta_op{SYDELTA_OP_COPY, 0, g * a.n, g + 1 == nbf ? ls : (uint64_t)a.n};
        }
        a.res[f] = ExpandOut{nops, nd, lit, wh, vh, 0, 0};
    }
}

// k_chunk_write: each unit's records from the plan's `skip`, the cut first record and the
// last one's extension applied, written as ops from plan.first
std::atomic<uint64_t> g_chunk_units{0};  // units written (emu_chunk_units)
hipError_t launch_chunk_write(const WalkUnit* units, const WalkRec* stage, const CxPlan* plan, uint32_t nunits,
                              uint32_t n, uint64_t nbf, uint64_t ls, sydelta_op* ops, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    if (!nunits) return hipSuccess;
    if (!units || !stage || !plan || !ops || !n) return hipErrorInvalidValue;
    for (uint32_t u = 0; u < nunits; ++u) {
        const CxPlan& P = plan[u];
        const WalkRec* src = stage + units[u].rec_off;
        sydelta_op* w = ops + P.first;
        for (uint32_t i = P.skip; i < P.cnt; ++i) {
            WalkRec x = src[i];
            if (i == P.skip && (P.flags & 1)) {
                x.off = P.r0_off;
                x.a = P.r0_a;
            }
            if (!x.kind) {
                *w++ = sydelta_op{SYDELTA_OP_DATA, 0, x.off, (uint64_t)x.a + (i + 1 == P.cnt ? P.ext : 0)};
                continue;
            }
            for (uint64_t g = x.a, e = g + x.kind; g < e; ++g)
                *w++ = sydelta_op{SYDELTA_OP_COPY, 0, g * n, g + 1 == nbf ? ls : (uint64_t)n};
        }
        ++g_chunk_units;
    }
    return hipSuccess;
}

// K10's pre-roll: each missed aligned block's first hit in (x, min(x + n, pend)), exactly
hipError_t launch_preroll(const WalkArgs& a, uint32_t* ahit, uint32_t* apw, uint64_t kb, uint64_t b0, uint64_t b1,
                          uint64_t pend, uint64_t len, uint32_t*, unsigned long long*, uint32_t waves,
                          uint64_t max_miss, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    if (b1 <= b0) return hipSuccess;
    if (a.n % 64 != 0 || a.n < 256 || a.n > kWalkMaxN || !ahit || !apw || !waves) return hipErrorInvalidValue;
    uint64_t misses = 0;
    for (uint64_t r = b0; r < b1; ++r) misses += ahit[r] == kNone;
    if (misses > max_miss) return hipSuccess;  // nothing pre-rolled (the walk rolls what it meets)
    DeviceIndex key_ix;
    key_ix.keys = (uint32_t*)a.keys;
    const FakeIndex& F = find_ix(key_ix);
    const uint64_t n = a.n;
    for (uint64_t r = b0; r < b1; ++r) {
        if (ahit[r] != kNone) continue;
        const uint64_t x = (kb + r) * n, yend = std::min(x + n, pend);
        if (x + n > len) return hipErrorInvalidValue;  // a probed block is a full window
        uint32_t h = kPreNone, off = 0, wcnt = 0;
        for (uint64_t y = x + 1; y < yend; ++y) {
            bool wh = false;
            const uint32_t b = lookup(F, 0, adler(a.base + y, n), a.base + y, n, &wh);
            wcnt += wh;
            if (b != kNone) {
                if (b >= kPreMark) return hipErrorInvalidValue;
                h = b | kPreMark;
                off = (uint32_t)(y - x);
                break;
            }
        }
        ahit[r] = h;
        apw[r] = off | (std::min(wcnt, 0x3FFFFu) << 14);
    }
    return hipSuccess;
}

// zstd blocks: the sequential form of k_zstd_block (sydelta_zstd.hpp block_content_seq)
hipError_t zstd_phase_ticks(unsigned long long* out) {
    for (int i = 0; i < 16; ++i) out[i] = 0;
    return hipSuccess;
}

hipError_t launch_zstd_blocks(const uint8_t* d_text, uint64_t len, uint64_t b0, uint32_t nb, uint8_t* d_slots,
                              uint8_t* d_lz, uint32_t* d_size, uint32_t* d_type, uint64_t* d_len64,
                              hipStream_t, Profiler*) {
    EmuTimer emu_t;
    if (b0 * zstd::kBlockMax >= len) return hipErrorInvalidValue;
    for (uint32_t i = 0; i < nb; ++i) {
        const uint64_t p = (b0 + i) * zstd::kBlockMax;
        const uint32_t n = (uint32_t)std::min<uint64_t>(zstd::kBlockMax, len - p);
        uint32_t type = 0;
        d_size[i] = zstd::block_content_seq(d_text + p, n, d_slots + (uint64_t)i * zstd::kBlockMax,
                                            zstd::seq_scratch_at(d_lz, nb, i), &type);
        d_type[i] = type;
        d_len64[i] = 3ull + d_size[i];
    }
    return hipSuccess;
}
hipError_t launch_zstd_frame(const uint8_t* d_text, uint64_t len, uint64_t b0, uint32_t nb, uint64_t nblocks,
                             const uint8_t* d_slots, const uint32_t* d_size, const uint32_t* d_type, const uint64_t* d_off,
                             uint64_t base, uint8_t* d_out, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    for (uint32_t i = 0; i < nb; ++i) {
        const uint64_t gb = b0 + i;
        const uint32_t n = (uint32_t)std::min<uint64_t>(zstd::kBlockMax, len - gb * zstd::kBlockMax);
        uint8_t* o = d_out + base + d_off[i];
        if (gb == 0) zstd::frame_header(d_out, len);
        zstd::block_header(o, gb + 1 == nblocks, d_type[i], d_type[i] == 2 ? d_size[i] : n);
        const uint8_t* src = d_type[i] == 2 ? d_slots + (uint64_t)i * zstd::kBlockMax : d_text + gb * zstd::kBlockMax;
        memcpy(o + 3, src, d_size[i]);
    }
    return hipSuccess;
}

hipError_t launch_exclusive_sum_u64(const uint64_t* d_in, uint64_t* d_out, uint64_t n, hipStream_t) {
    EmuTimer emu_t;
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t v = d_in[i];
        d_out[i] = acc;
        acc += v;
    }
    return hipSuccess;
}

hipError_t launch_block_cmp(const uint8_t* d_src, uint64_t slen, const uint8_t* d_dst, uint64_t dlen, uint64_t bs,
                            uint8_t* d_changed, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    const uint64_t nb = (slen + bs - 1) / bs;
    for (uint64_t k = 0; k < nb; ++k) {
        const uint64_t o = k * bs, sl = std::min(bs, slen - o), dl = dlen > o ? std::min(bs, dlen - o) : 0;
        d_changed[k] = sl != dl || memcmp(d_src + o, d_dst + o, sl) != 0;
    }
    return hipSuccess;
}

hipError_t launch_hash_blocks(const uint8_t* d_buf, uint64_t len, uint64_t bs, const uint64_t* d_pos, uint32_t count,
                              uint64_t* d_out, hipStream_t) {
    EmuTimer emu_t;
    for (uint32_t i = 0; i < count; ++i) {
        const uint64_t o = d_pos[i] * bs;
        d_out[i] = oracle_xxh3_64(d_buf + o, o < len ? std::min(bs, len - o) : 0);
    }
    return hipSuccess;
}

hipError_t launch_xxh_files(const uint8_t* d_buf, const uint64_t* d_off, const uint64_t* d_len, const uint64_t*,
                            const uint64_t*, const uint64_t*, uint64_t, const uint32_t*, uint64_t nfiles, uint64_t,
                            uint64_t*, uint64_t* d_out, hipStream_t, Profiler*) {
    EmuTimer emu_t;
    for (uint64_t f = 0; f < nfiles; ++f) d_out[f] = oracle_xxh3_64(d_buf + d_off[f], d_len[f]);
    return hipSuccess;
}

hipError_t launch_synth_fill(uint8_t*, uint64_t, uint64_t, hipStream_t, uint64_t) {
    EmuTimer emu_t; return hipErrorNotSupported; }
hipError_t launch_synth_edit_blocks(uint8_t*, uint64_t, uint64_t, uint64_t, uint64_t, uint32_t, hipStream_t) {
    EmuTimer emu_t;
    return hipErrorNotSupported;
}
hipError_t launch_synth_mutate(uint8_t*, const uint8_t*, uint64_t, uint64_t, uint32_t, hipStream_t) {
    EmuTimer emu_t;
    return hipErrorNotSupported;
}
}  // namespace sydelta

// the files the emulated k_walk_expand saw (emulated_checks asserts the device-expand path ran)
extern "C" uint64_t emu_expand_files() { return sydelta::g_expand_files.load(); }
// the units the emulated k_chunk_write wrote (emulated_checks asserts the chunk path ran)
extern "C" uint64_t emu_chunk_units() { return sydelta::g_chunk_units.load(); }
