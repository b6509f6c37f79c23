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
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <immintrin.h>
#include <chrono>
#include <cmath>
#include <numeric>
#include <map>
#include <memory>
#include <new>
#include <mutex>
#include <thread>
#include <string>
#include <set>
#include <unordered_set>
#include <vector>

#include "../../include/sydelta.h"
#include "sydelta_host.hpp"
#include "sydelta_internal.hpp"

using namespace sydelta;

// ---------------------------------------------------------------------------
// errors (thread-local, like io::Error propagated to the caller)
// ---------------------------------------------------------------------------
static thread_local std::string t_err;

int sydelta::fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}


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
constexpr int kMaxPoolDevices = 64;
hipMemPool_t g_pools[kMaxPoolDevices] = {};  // written once per device under its call_once
// K10's wave slots per device: CUs x 4 SIMDs x 4 waves (k_walk_files' __launch_bounds__(64, 4));
// 4096 on MI355X's 256 CUs (written under the device's call_once, like g_pools)
uint32_t g_wave_slots[kMaxPoolDevices] = {};

int ensure_device_impl(int device) {
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
        const hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess || n <= device) {
            st->msg = "no HIP device " + std::to_string(device) + " (hipGetDeviceCount: " + hipGetErrorString(e) +
                      ", " + std::to_string(n) + " devices)";
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
        // Scratch (index arrays, hit lists, probe jobs, streamed chunks) comes from the
        // library's own stream-ordered pool on this device (never the device's default
        // pool, which other libraries in the process share).  A pool's default release
        // threshold is 0: every stream synchronization hands the freed memory back and the
        // next call maps it again, so keep up to SYDELTA_POOL_KEEP_MIB (default 4 GiB)
        // reserved across calls -- for this library's scratch only.
        if (device >= kMaxPoolDevices) {
            st->msg = "device index " + std::to_string(device) + " above the library's limit";
            return;
        }
        hipMemPoolProps props{};
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = device;
        hipMemPool_t pool = nullptr;
        if (hipMemPoolCreate(&pool, &props) != hipSuccess || !pool) {
            st->msg = "hipMemPoolCreate failed on device " + std::to_string(device);
            return;
        }
        uint64_t keep = 4096;
        if (const char* e = getenv("SYDELTA_POOL_KEEP_MIB")) keep = strtoull(e, nullptr, 10);
        keep <<= 20;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        g_pools[device] = pool;
        g_wave_slots[device] = (uint32_t)std::max(64, prop.multiProcessorCount * 16);
        st->status = SYDELTA_OK;
    });
    if (st->status != SYDELTA_OK) return fail(st->status, "%s", st->msg.c_str());
    if (hipSetDevice(device) != hipSuccess) return fail(SYDELTA_E_NODEV, "hipSetDevice(%d) failed", device);
    return SYDELTA_OK;
}

// one stream per (thread, device): calls on different threads never share a stream
hipStream_t thread_stream_impl(int device) {
    static thread_local std::map<int, hipStream_t> streams;
    auto it = streams.find(device);
    if (it != streams.end()) return it->second;
    hipStream_t s = nullptr;
    // blocking: orders against work on the legacy default stream (torch's default
    // stream), so buffers a caller filled there are complete before our kernels read them
    if (hipStreamCreateWithFlags(&s, hipStreamDefault) != hipSuccess) return nullptr;
    streams[device] = s;
    return s;
}

// A third and fourth stream per (thread, device): the chunk walk's parts alternate between
// them, so that a part's walk starts when its lookups are done even while the previous
// part's still runs.  Ordered by events only, never destroyed.  (Low-priority walk streams,
// so that the dispatcher would favour the hashing beside them, measured the same:
// `profiles/r05x_*`.)
// Threads expanding walk records into op arrays (SYDELTA_ASM_THREADS, per call; default the
// host pool and the caller)
int asm_threads_env() {
    const char* e = getenv("SYDELTA_ASM_THREADS");
    return (e && *e) ? std::max(1, atoi(e)) : (int)walk::HostPool::get().size() + 1;
}

// Where a one-file index's ribbon level-1 starts (read per call): 2 at index creation, 1 at
// the match call, 0 after the index (by the first scan)
int early_ribbon_mode() {
    const char* e = getenv("SYDELTA_EARLY_RIBBON");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : 2;
}

hipStream_t thread_walk_stream(int device, int i) {
    static thread_local std::map<int, hipStream_t> streams[3];  // [2]: the ribbon started at index creation
    auto it = streams[i].find(device);
    if (it != streams[i].end()) return it->second;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    streams[i][device] = s;
    return s;
}

// A second stream per (thread, device) for work overlapped with the caller's (the index
// build); ordered by events only, never destroyed.
hipStream_t thread_aux_stream(int device) {
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

int sydelta::ensure_device(int device) { return ensure_device_impl(device); }
hipError_t sydelta::dev_malloc_async(void** p, size_t bytes, hipStream_t s) {
    int d = 0;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess) return e;
    // every entry point runs ensure_device (which sets the device) before allocating
    if (d < 0 || d >= kMaxPoolDevices || !g_pools[d]) return hipErrorInvalidDevice;
    return hipMallocFromPoolAsync(p, bytes, g_pools[d], s);
}
int sydelta::host_exception() {
    try {
        throw;
    } catch (const std::bad_alloc&) {
        return fail(SYDELTA_E_OOM, "out of host memory");
    } catch (const std::exception& e) {
        return fail(SYDELTA_E_INVAL, "%s", e.what());
    } catch (...) {
        return fail(SYDELTA_E_INVAL, "unexpected host error");
    }
}
hipStream_t sydelta::thread_stream(int device) { return thread_stream_impl(device); }
uint32_t sydelta::wave_slots(int device) {
    return device >= 0 && device < kMaxPoolDevices && g_wave_slots[device] ? g_wave_slots[device] : 4096u;
}

namespace sydelta {
// Timing events are recycled: creating and destroying HIP events per launch costs
// runtime signal allocations (measured: tens of ms per C4 step), so a thread keeps its
// own pool (never destroyed, like the per-thread streams).
namespace {
thread_local std::map<int, std::vector<hipEvent_t>> t_event_pool;  // per device
std::vector<hipEvent_t>& event_pool() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return t_event_pool[dev];
}
// Timed launches are resolved when the profile is read (sydelta_profile_json, after the
// caller synchronized), not at the end of each call: a per-call event wait would add a
// host round trip, and an idle GPU, to every call of a profiled run.  Resolved events go
// to a shared free list per device (the resolving thread may not be the recording one).
std::vector<Profiler::Pending> g_deferred;                  // under g_prof_mu
std::map<int, std::vector<hipEvent_t>> g_free_events;       // under g_prof_mu
constexpr size_t kDeferredMax = 1 << 14;                     // beyond: resolve on the spot
// Each device's timed launches as intervals on one time line (relative to the first
// launch resolved since the last reset, whose start event is kept as the origin): their
// union is the time the device spent in timed kernels, which per-launch times overstate
// when launches of several callers' streams overlap (sydelta_profile_json's "__busy__").
std::map<int, hipEvent_t> g_origin;                                  // under g_prof_mu
std::map<int, std::vector<std::pair<double, double>>> g_intervals;   // under g_prof_mu
// Resolve the entries of v (all, waiting on their events; or, with only_done, those whose
// end event has completed, so a long profiled run keeps recycling its events).
void resolve_locked(std::vector<Profiler::Pending>& v, bool only_done = false) {
    size_t keep = 0;
    for (size_t i = 0; i < v.size(); ++i) {
        Profiler::Pending& q = v[i];
        if (only_done && hipEventQuery(q.b) != hipSuccess) {
            if (keep != i) v[keep] = std::move(q);
            ++keep;
            continue;
        }
        float ms = 0;
        bool origin = false;
        if (hipEventSynchronize(q.b) == hipSuccess && hipEventElapsedTime(&ms, q.a, q.b) == hipSuccess) {
            auto& e = g_prof[q.name];
            e.first += ms;
            e.second += 1;
            hipEvent_t& o = g_origin[q.device];
            if (!o) {
                o = q.a;
                origin = true;
            }
            float t0 = 0;
            if (hipEventElapsedTime(&t0, o, q.a) == hipSuccess) g_intervals[q.device].push_back({t0, t0 + ms});
        }
        auto& fl = g_free_events[q.device];
        if (!origin) fl.push_back(q.a);
        fl.push_back(q.b);
    }
    v.resize(keep);
}
// union length and span of the intervals of every device (ms)
std::pair<double, double> busy_locked(size_t* count) {
    double busy = 0, span = 0;
    *count = 0;
    for (auto& kv : g_intervals) {
        auto iv = kv.second;
        *count += iv.size();
        if (iv.empty()) continue;
        std::sort(iv.begin(), iv.end());
        double lo = iv[0].first, hi = iv[0].second, first = lo, last = hi;
        for (auto& x : iv) {
            last = std::max(last, x.second);
            if (x.first > hi) {
                busy += hi - lo;
                lo = x.first;
                hi = x.second;
            } else {
                hi = std::max(hi, x.second);
            }
        }
        busy += hi - lo;
        span += last - first;
    }
    return {busy, span};
}
void reset_intervals_locked() {
    for (auto& kv : g_origin)
        if (kv.second) g_free_events[kv.first].push_back(kv.second);
    g_origin.clear();
    g_intervals.clear();
}
hipEvent_t take_event() {
    auto& pool = event_pool();
    if (pool.empty()) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        std::lock_guard<std::mutex> lk(g_prof_mu);
        auto& fl = g_free_events[dev];
        while (!fl.empty() && pool.size() < 64) {
            pool.push_back(fl.back());
            fl.pop_back();
        }
    }
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}
}  // namespace
ProfScope::ProfScope(Profiler* p_, hipStream_t s_, const char* n) : p(p_), s(s_), name(n) {
    if (!p) return;
    a = take_event();
    b = take_event();
    if (!a || !b) { p = nullptr; return; }
    (void)hipGetDevice(&device);
    (void)hipEventRecord(a, s);
}
ProfScope::~ProfScope() {
    if (!p) return;
    (void)hipEventRecord(b, s);
    p->pending.push_back({name, a, b, device});
}
void Profiler::resolve() {
    if (pending.empty()) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_deferred.insert(g_deferred.end(), pending.begin(), pending.end());
    pending.clear();
    resolve_locked(g_deferred, g_deferred.size() <= kDeferredMax);
}
}  // namespace sydelta

bool sydelta::profiling_on() { return g_prof_on.load() != 0; }

extern "C" void sydelta_set_profiling(int on) { g_prof_on.store(on ? 1 : 0); }

extern "C" size_t sydelta_profile_json(char* buf, size_t cap, int reset) {
    std::string s = "{";
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        sydelta::resolve_locked(sydelta::g_deferred);
        bool first = true;
        for (auto& kv : g_prof) {
            char tmp[256];
            snprintf(tmp, sizeof tmp, "%s\"%s\": {\"ms\": %.6f, \"count\": %llu}", first ? "" : ", ", kv.first.c_str(),
                     kv.second.first, (unsigned long long)kv.second.second);
            s += tmp;
            first = false;
        }
        size_t nint = 0;
        const auto bs = sydelta::busy_locked(&nint);
        if (nint) {  // the union of the timed launches (not a kernel)
            char tmp[256];
            snprintf(tmp, sizeof tmp, "%s\"__busy__\": {\"ms\": %.6f, \"count\": %llu, \"span_ms\": %.6f}",
                     first ? "" : ", ", bs.first, (unsigned long long)nint, bs.second);
            s += tmp;
        }
        if (reset) {
            g_prof.clear();
            sydelta::reset_intervals_locked();
        }
    }
    s += "}";
    if (buf && cap > s.size()) memcpy(buf, s.c_str(), s.size() + 1);
    return s.size();
}

// ---------------------------------------------------------------------------
// small utilities
// ---------------------------------------------------------------------------
extern "C" int sydelta_device_count(int* count) try {
    if (!count) return fail(SYDELTA_E_INVAL, "count is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// ---------------------------------------------------------------------------
// the device of the path-level entry points
// ---------------------------------------------------------------------------
// sy calls compute_checksums / generate_delta(_streaming) from up to --parallel (default
// 10) spawn_blocking threads at once (sync/mod.rs:672-697, cli.rs:178-180, ssh.rs:913),
// and Rust cannot make a device current for them.  So each calling thread is bound to a
// device on its first path-level call -- the allowed device with the fewest bound threads,
// ties broken round-robin -- and stays there (its stream, pinned buffers and scratch live
// on that device); a thread's exit unbinds it.  sydelta_set_thread_device binds one
// explicitly, sydelta_set_devices restricts the automatic choice.
namespace {
std::mutex& bind_mu() {
    static std::mutex* m = new std::mutex();  // never destroyed: thread exits may come after static teardown
    return *m;
}
// heap-allocated and never destroyed, like bind_mu: a bound thread may exit after static teardown
std::vector<int>& g_allowed = *new std::vector<int>();  // under bind_mu; empty: every visible device
std::map<int, int>& g_bound = *new std::map<int, int>();  // under bind_mu; device -> bound threads
unsigned g_rr = 0;           // under bind_mu
struct ThreadBinding {
    int dev = -1;
    void set(int d) {
        std::lock_guard<std::mutex> lk(bind_mu());
        if (dev >= 0 && g_bound[dev] > 0) --g_bound[dev];
        dev = d;
        if (dev >= 0) ++g_bound[dev];
    }
    ~ThreadBinding() { set(-1); }
};
thread_local ThreadBinding t_bind;
}  // namespace

int sydelta::path_device(int* out) {
    if (t_bind.dev >= 0) {
        *out = t_bind.dev;
        return SYDELTA_OK;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(SYDELTA_E_NODEV, "no HIP device visible");
    int best = -1;
    {
        std::lock_guard<std::mutex> lk(bind_mu());
        std::vector<int> cand;
        for (int d : g_allowed)
            if (d >= 0 && d < n) cand.push_back(d);
        if (cand.empty())
            for (int d = 0; d < n; ++d) cand.push_back(d);
        const unsigned start = g_rr++;
        for (size_t k = 0; k < cand.size(); ++k) {
            const int d = cand[(start + k) % cand.size()];
            if (best < 0 || g_bound[d] < g_bound[best]) best = d;
        }
        ++g_bound[best];
    }
    t_bind.dev = best;
    *out = best;
    return SYDELTA_OK;
}

extern "C" int sydelta_set_devices(const int* devices, int n) try {
    if (n < 0 || (n > 0 && !devices)) return fail(SYDELTA_E_INVAL, "bad device list");
    int vis = 0;
    if (hipGetDeviceCount(&vis) != hipSuccess) vis = 0;
    for (int i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= vis)
            return fail(SYDELTA_E_NODEV, "device %d is not visible (%d devices)", devices[i], vis);
    std::lock_guard<std::mutex> lk(bind_mu());
    g_allowed.assign(devices, devices + n);
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_set_thread_device(int device) try {
    if (device >= 0) {
        int vis = 0;
        if (hipGetDeviceCount(&vis) != hipSuccess || device >= vis)
            return fail(SYDELTA_E_NODEV, "device %d is not visible", device);
    }
    t_bind.set(device < 0 ? -1 : device);
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_thread_device(int* device) try {
    if (!device) return fail(SYDELTA_E_INVAL, "device is NULL");
    return path_device(device);
} catch (...) {
    return sydelta::host_exception();
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
namespace {
int pinned_at_least(PinnedHits& h, size_t bytes);                              // (below)
int upload_staged(void* d_dst, const void* src, size_t bytes, hipStream_t s);  // (below)
}  // namespace

extern "C" int sydelta_signature_device(int device, const uint8_t* d_buf, uint64_t len, uint64_t block_size,
                                        uint32_t* d_weak, uint64_t* d_strong, void* stream) try {
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (len && (!d_buf || !d_weak || !d_strong)) return fail(SYDELTA_E_INVAL, "NULL device pointer");
    SYDELTA_ENTER_DEVICE(device);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    CallProf cp;
    HIP_TRY(launch_signature(d_buf, len, block_size, d_weak, d_strong, s, cp.get()));
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

namespace {
// The batched signature kernel's table for files [0, nfiles) (block_size % 64 == 0, files
// 16-byte aligned): aoff | agb | apfx (nact + 1) | loff | llen | lidx, appended to t; agb /
// lidx count blocks from gb0.
struct SigTable {
    size_t at;  // the table's first entry in t
    uint64_t nact, nfull, npart;
};
SigTable sig_batch_table(const uint64_t* off, const uint64_t* len, uint64_t nfiles, uint64_t block_size, uint64_t gb0,
                         std::vector<uint64_t>& t) {
    std::vector<uint64_t> aoff, agb, apfx{0}, loff, llen, lidx;
    uint64_t gb = gb0;
    for (uint64_t f = 0; f < nfiles; ++f) {
        const uint64_t nfull = len[f] / block_size;
        if (nfull) {
            aoff.push_back(off[f]);
            agb.push_back(gb);
            apfx.push_back(apfx.back() + nfull);
        }
        if (len[f] % block_size) {
            loff.push_back(off[f] + nfull * block_size);
            llen.push_back(len[f] % block_size);
            lidx.push_back(gb + nfull);
        }
        gb += (len[f] + block_size - 1) / block_size;
    }
    SigTable r{t.size(), aoff.size(), apfx.back(), loff.size()};
    for (auto* v : {&aoff, &agb, &apfx, &loff, &llen, &lidx}) t.insert(t.end(), v->begin(), v->end());
    return r;
}
hipError_t launch_sig_table(const uint8_t* d_buf, const uint64_t* d_t, const SigTable& T, uint64_t block_size,
                            uint32_t* d_weak, uint64_t* d_strong, hipStream_t s, Profiler* prof) {
    const uint64_t* p = d_t + T.at;
    const uint64_t* d_aoff = p; p += T.nact;
    const uint64_t* d_agb = p; p += T.nact;
    const uint64_t* d_apfx = p; p += T.nact + 1;
    const uint64_t* d_loff = p; p += T.npart;
    const uint64_t* d_llen = p; p += T.npart;
    const uint64_t* d_lidx = p;
    return launch_signature_batch_fast(d_buf, d_aoff, d_agb, d_apfx, T.nact, T.nfull, d_loff, d_llen, d_lidx, T.npart,
                                       block_size, d_weak, d_strong, s, prof);
}
}  // namespace

extern "C" int sydelta_signature_batch_device(int device, const uint8_t* d_buf, const uint64_t* off,
                                              const uint64_t* len, uint64_t nfiles, uint64_t block_size,
                                              uint32_t* d_weak, uint64_t* d_strong, void* stream) try {
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (nfiles && (!off || !len)) return fail(SYDELTA_E_INVAL, "NULL segment table");
    SYDELTA_ENTER_DEVICE(device);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    std::vector<uint64_t> fblk(nfiles + 1, 0);
    for (uint64_t f = 0; f < nfiles; ++f) fblk[f + 1] = fblk[f] + (len[f] + block_size - 1) / block_size;
    const uint64_t total = fblk[nfiles];
    if (!total) return SYDELTA_OK;
    bool fast = block_size % 64 == 0 && block_size >= 256 && block_size <= (1ull << 31);
    for (uint64_t f = 0; f < nfiles && fast; ++f) fast = !len[f] || ((uintptr_t)(d_buf + off[f]) & 15) == 0;
    if (fast) {
        std::vector<uint64_t> t;
        t.reserve(6 * nfiles + 1);
        const SigTable T = sig_batch_table(off, len, nfiles, block_size, 0, t);
        uint64_t* d_t = nullptr;
        HIP_TRY(dev_malloc_async((void**)&d_t, 8 * t.size(), s));
        if (int r = upload_staged(d_t, t.data(), 8 * t.size(), s)) {
            (void)hipFreeAsync(d_t, s);
            return r;
        }
        CallProf cp;
        hipError_t e = launch_sig_table(d_buf, d_t, T, block_size, d_weak, d_strong, s, cp.get());
        (void)hipFreeAsync(d_t, s);
        HIP_TRY(e);
        if (!stream) HIP_TRY(hipStreamSynchronize(s));  // the library's stream: done on return
        return SYDELTA_OK;
    }
    uint64_t* d_meta = nullptr;
    HIP_TRY(dev_malloc_async((void**)&d_meta, sizeof(uint64_t) * (3 * nfiles + 1), s));
    {
        std::vector<uint64_t> meta(3 * nfiles + 1);
        std::copy(off, off + nfiles, meta.begin());
        std::copy(len, len + nfiles, meta.begin() + nfiles);
        std::copy(fblk.begin(), fblk.end(), meta.begin() + 2 * nfiles);
        if (int r = upload_staged(d_meta, meta.data(), 8 * meta.size(), s)) {
            (void)hipFreeAsync(d_meta, s);
            return r;
        }
    }
    CallProf cp;
    hipError_t e = launch_signature_batch(d_buf, d_meta, d_meta + nfiles, d_meta + 2 * nfiles, nfiles, block_size,
                                          total, d_weak, d_strong, s, cp.get());
    (void)hipFreeAsync(d_meta, s);
    HIP_TRY(e);
    if (!stream) HIP_TRY(hipStreamSynchronize(s));  // the library's stream: done on return
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
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
    size_t pool_bytes = 0;
    hipStream_t stream = nullptr;     // the stream the pool was allocated on
    // the ribbon level-1 (ix.rib_l1): 0 none, 1 built by the first scan of >= kRibMinScan
    // positions, 2 by the first scan (SYDELTA_L1=ribbon); built once, on the stream of the
    // scan that builds it, which records rib_ev for scans on other streams
    int rib_mode = 0;
    std::mutex rib_mu;
    bool rib_built = false;
    hipStream_t rib_stream = nullptr;
    hipEvent_t rib_ev = nullptr;
    // An index over device arrays is built on the creating thread's aux stream (its
    // copies of the arrays stay on the caller's stream): `ready` is recorded after the
    // build and every use waits for it on its own stream (index_wait), so work the caller
    // queues meanwhile -- C5's aligned probe of the source -- overlaps the build.
    hipEvent_t ready = nullptr;
    PinnedHits stage;  // the file tables' upload (mapped; returned at release)
    uint64_t max_nblk = 0;  // the most blocks of any file
    // A batch whose walks are self-indexed (K10 builds each file's filter and table in LDS from
    // the signature, sydelta_filewalk.hip) defers its filters and tables until a match takes
    // another path (index_full): a C4 step then has no index build at all.
    bool deferred = false;
    std::mutex build_mu;
    // A single-file index's scan extras (the level-1 filter, the fat table) are filled by the
    // first scan that runs against it (scan_index): the chunk walk and the aligned probe read
    // only the Bloom filter and the exact table (C5: 1-8 Mi keys).  extras_ev orders scans on
    // other streams after them.
    bool extras_deferred = false;
    hipEvent_t extras_ev = nullptr;
    hipStream_t extras_stream = nullptr;
};

namespace {
// Order `s` after the index build (a no-op for an index built synchronously).
hipError_t index_wait(const sydelta_index* x, hipStream_t s) {
    return x->ready ? hipStreamWaitEvent(s, x->ready, 0) : hipSuccess;
}
// A deferred index's filters and tables, built on `s` (after its copies) for a match that needs
// them; later users order themselves after the build through `ready`.
int index_full(sydelta_index* x, hipStream_t s) {
    std::lock_guard<std::mutex> lk(x->build_mu);
    if (!x->deferred) return SYDELTA_OK;
    HIP_TRY(index_wait(x, s));
    CallProf cp;
    HIP_TRY(launch_index_build(x->d_weak, x->d_strong, x->ix, s, cp.get()));
    if (x->ready) HIP_TRY(hipEventRecord(x->ready, s));
    x->deferred = false;
    return SYDELTA_OK;
}
}  // namespace

// Index memory is kept for the next index: a released index's allocation is held (one
// per device) and the next index built with no more bytes (and no less than half) takes
// it over, so the usual sequence -- build, match, free, build again (a file after
// another, bench steps) -- allocates once.  A hipFreeAsync on a stream with no work
// queued blocked the host 0.3-0.6 ms for these allocations (measured, round 3: C3's 50 MB
// index, C5's 130 MB one), as for the scan's hit buffers.  The held block is homed on a
// library stream (never destroyed): an index built on a caller stream hands its block
// over with an event (record on the caller stream, wait on the library stream), so no
// handle to a caller stream outlives its index; a new owner on another stream waits for
// the home stream the same way.  No host synchronization on either side.
namespace {
struct KeptPool {
    void* p = nullptr;
    size_t bytes = 0;
    hipStream_t s = nullptr;  // a library thread stream
};
std::mutex g_kept_mu;
KeptPool g_kept[64];
// One event per (thread, device) for stream hand-offs (re-recorded freely: a wait takes
// the record that precedes it); never destroyed, like the thread streams.
hipEvent_t handoff_event(int device) {
    static thread_local std::map<int, hipEvent_t> ev;
    hipEvent_t& e = ev[device];
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
    return e;
}
// Order `to` after the work queued so far on `from` (same device, current).
hipError_t stream_after(hipStream_t to, hipStream_t from, int device) {
    if (to == from) return hipSuccess;
    hipEvent_t e = handoff_event(device);
    if (!e) return hipErrorOutOfMemory;
    hipError_t r = hipEventRecord(e, from);
    return r != hipSuccess ? r : hipStreamWaitEvent(to, e, 0);
}
}  // namespace

// Pinned host buffers of finished chunk walks and indexes, kept for the next ones (pinning
// tens of MB costs milliseconds), of two kinds: kMapped, coherent and mapped, which kernels
// write and the host then reads (a chunk walk's per-unit results and records); kStage,
// ordinary pinned memory (cached by the CPU) the host fills and the DMA engines read (unit
// tables, file tables: filling coherent memory, which the CPU does not cache, held a chunk's
// launch ~0.1 ms, `profiles/r05zs_c5_w70_step_timeline.txt`).  Released by sydelta_trim.
namespace {
enum PinKind { kMapped = 0, kStage = 1 };
std::mutex g_mapped_mu;
std::vector<PinnedHits> g_mapped[2];  // per kind: at most kMappedKeep buffers and kMappedKeepBytes
constexpr size_t kMappedKeep = 64, kMappedKeepBytes = (size_t)1 << 30;
int take_mapped(size_t bytes, PinnedHits& out, PinKind kind = kMapped) {
    {
        std::lock_guard<std::mutex> lk(g_mapped_mu);
        std::vector<PinnedHits>& g = g_mapped[kind];
        size_t best = g.size();
        for (size_t i = 0; i < g.size(); ++i)
            if (g[i].bytes >= bytes && g[i].bytes <= 4 * bytes + (1u << 20) &&
                (best == g.size() || g[i].bytes < g[best].bytes))
                best = i;  // (a small request does not take a chunk walk's large buffer)
        if (best < g.size()) {
            out = g[best];
            g.erase(g.begin() + best);
            return SYDELTA_OK;
        }
    }
    out = PinnedHits();
    const size_t want = bytes + bytes / 4;
    const unsigned flags = kind == kStage ? hipHostMallocDefault
                                          : hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent;
    HIP_TRY(hipHostMalloc((void**)&out.p, want, flags));
    out.bytes = want;
    return SYDELTA_OK;
}
void give_mapped(PinnedHits h, PinKind kind = kMapped) {  // h idle (its last use was synchronized)
    if (!h.p) return;
    PinnedHits drop;
    {
        std::lock_guard<std::mutex> lk(g_mapped_mu);
        std::vector<PinnedHits>& g = g_mapped[kind];
        g.push_back(h);
        size_t held = 0;
        for (const PinnedHits& x : g) held += x.bytes;
        if (g.size() > kMappedKeep || held > kMappedKeepBytes) {
            auto it = std::min_element(g.begin(), g.end(),
                                       [](const PinnedHits& a, const PinnedHits& b) { return a.bytes < b.bytes; });
            drop = *it;
            g.erase(it);
        }
    }
    if (drop.p) (void)hipHostFree(drop.p);
}
void release_mapped() {
    std::vector<PinnedHits> v;
    {
        std::lock_guard<std::mutex> lk(g_mapped_mu);
        for (auto& g : g_mapped) {
            v.insert(v.end(), g.begin(), g.end());
            g.clear();
        }
    }
    for (auto& h : v) (void)hipHostFree(h.p);
}
// Events that outlive one call (a chunk's, recorded by classify and waited on by walk),
// recycled per device: creating events costs runtime signal allocations.
std::mutex g_ev_mu;
std::map<int, std::vector<hipEvent_t>> g_ev_free;
hipEvent_t take_event(int device) {
    {
        std::lock_guard<std::mutex> lk(g_ev_mu);
        auto& v = g_ev_free[device];
        if (!v.empty()) {
            hipEvent_t e = v.back();
            v.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    return e;
}
void give_event(int device, hipEvent_t e) {
    if (!e) return;
    std::lock_guard<std::mutex> lk(g_ev_mu);
    g_ev_free[device].push_back(e);
}
}  // namespace

static void index_release(sydelta_index* x) {
    if (!x) return;
    // tables built on other streams (a ribbon started at creation may never have been used):
    // the pool's release below follows x->stream
    if (x->rib_ev && x->rib_stream && x->rib_stream != x->stream) (void)hipStreamWaitEvent(x->stream, x->rib_ev, 0);
    if (x->extras_ev && x->extras_stream && x->extras_stream != x->stream)
        (void)hipStreamWaitEvent(x->stream, x->extras_ev, 0);
    give_event(x->device, x->rib_ev);  // (pooled: a wait queued on an event holds its record)
    give_event(x->device, x->extras_ev);
    // the build has uploaded the file tables from `stage` (done long before, as a rule)
    if (x->ready) (void)hipEventSynchronize(x->ready);
    give_mapped(x->stage, kStage);
    x->stage = PinnedHits();
    if (x->d_pool) {
        KeptPool old;
        const hipStream_t home = thread_stream(x->device);
        if (x->device >= 0 && x->device < 64 && home && stream_after(home, x->stream, x->device) == hipSuccess &&
            index_wait(x, home) == hipSuccess) {
            std::lock_guard<std::mutex> lk(g_kept_mu);
            old = g_kept[x->device];
            g_kept[x->device] = {x->d_pool, x->pool_bytes, home};
        } else {
            old = {x->d_pool, 0, x->stream};  // released in its own stream's order
        }
        if (old.p) (void)hipFreeAsync(old.p, old.s);
    }
    if (x->ready) give_event(x->device, x->ready);
    delete x;
}

// The held allocation of `device` if it fits `bytes` (ordered after its home stream), else
// released in its home stream's order.
static void* take_kept_pool(int device, size_t bytes, hipStream_t s, size_t* got) {
    if (device < 0 || device >= 64) return nullptr;
    KeptPool k;
    {
        std::lock_guard<std::mutex> lk(g_kept_mu);
        k = g_kept[device];
        g_kept[device] = KeptPool();
    }
    if (!k.p) return nullptr;
    if (k.bytes >= bytes && k.bytes <= 2 * bytes + (64u << 20) && stream_after(s, k.s, device) == hipSuccess) {
        *got = k.bytes;
        return k.p;
    }
    (void)hipFreeAsync(k.p, k.s);
    return nullptr;
}


// Per-thread scratch of the scan (Classifier::scan): the verified-hit buffers on each
// device and the pinned host buffer the sorted hits come back into.
// A thread's scratch is released by sydelta_trim (the calling thread's, and every other
// thread's that is not inside a call: the owner holds `mu` while it uses the buffers) and
// when the thread exits (sy's spawn_blocking threads come and go; the host pool's
// workers classify chunks of sydelta_delta_multi_device).  The main thread's is left to
// the process exit (the HIP runtime may be tearing down by then).
namespace sydelta {
namespace {
struct ThreadScratch {
    std::recursive_mutex mu;  // held by the owning thread while a call uses the buffers
    std::map<int, HitScratch> hits;  // per device
    std::map<int, DevScratch> scan;  // per device: launch_scan's scratch
    std::map<int, DevScratch> probe;  // per device: the aligned probe's jobs and results
    std::map<int, DevScratch> walk;   // per device: k_walk_files' table and records
    PinnedHits pinned;     // sorted hits / the file walk's table, counts and records
    PinnedHits seg_pin;    // Classifier::scan's segment table
    PinnedHits probe_pin;  // Classifier::probe's results
    PinnedHits phase_pin;  // Classifier::phase_probe's results
    PinnedHits walk_map;   // run_walk's results: coherent, mapped (the walk kernel writes it)
    // upload_staged's ring: pinned copies of small host tables, each reused once the copy
    // that read it (its event) has run
    PinnedHits up[4];
    hipEvent_t up_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    int up_dev[4] = {0, 0, 0, 0};
    unsigned up_next = 0;
};
std::mutex& scratch_mu() {
    static std::mutex* m = new std::mutex();  // never destroyed (thread exits after static teardown)
    return *m;
}
std::vector<ThreadScratch*>& all_scratch() {  // under scratch_mu: every live thread's
    static std::vector<ThreadScratch*>* v = new std::vector<ThreadScratch*>();
    return *v;
}
const std::thread::id g_main_thread = std::this_thread::get_id();  // the thread that loaded the library

// Free t's buffers (t.mu held, t's owner outside any call: its last call synchronized the
// streams it used, so the buffers are idle).  Device memory goes back to the library's
// pool in the legacy stream's order.
void release_scratch(ThreadScratch& t) {
    DeviceScope keep_device;
    std::set<int> devs;
    auto dev_free = [&](int d, void* p) {
        if (p && hipSetDevice(d) == hipSuccess) {
            (void)hipFreeAsync(p, nullptr);
            devs.insert(d);
        }
    };
    for (auto& kv : t.hits) dev_free(kv.first, kv.second.p);
    t.hits.clear();
    for (auto* m : {&t.scan, &t.probe, &t.walk}) {
        for (auto& kv : *m) dev_free(kv.first, kv.second.p);
        m->clear();
    }
    for (int d : devs)
        if (hipSetDevice(d) == hipSuccess) (void)hipStreamSynchronize(nullptr);
    for (PinnedHits* h : {&t.pinned, &t.seg_pin, &t.probe_pin, &t.phase_pin}) {
        if (h->p) (void)hipHostFree(h->p);
        *h = PinnedHits();
    }
    if (t.walk_map.p) (void)hipHostFree(t.walk_map.p);
    t.walk_map = PinnedHits();
    for (int i = 0; i < 4; ++i) {
        if (t.up_ev[i] && hipSetDevice(t.up_dev[i]) == hipSuccess) {
            (void)hipEventSynchronize(t.up_ev[i]);
            (void)hipEventDestroy(t.up_ev[i]);
        }
        t.up_ev[i] = nullptr;
        if (t.up[i].p) (void)hipHostFree(t.up[i].p);
        t.up[i] = PinnedHits();
    }
}

struct ScratchOwner {  // thread_local: the thread's scratch, released at its exit
    ThreadScratch* t = nullptr;
    ~ScratchOwner() {
        if (!t) return;
        {
            std::lock_guard<std::mutex> lk(scratch_mu());
            auto& v = all_scratch();
            v.erase(std::remove(v.begin(), v.end(), t), v.end());
        }
        if (std::this_thread::get_id() == g_main_thread) return;  // process exit: left to the OS
        {
            std::lock_guard<std::recursive_mutex> h(t->mu);
            release_scratch(*t);
        }
        delete t;
    }
};
ThreadScratch& thread_scratch() {
    static thread_local ScratchOwner own;
    if (!own.t) {
        own.t = new ThreadScratch();
        std::lock_guard<std::mutex> lk(scratch_mu());
        all_scratch().push_back(own.t);
    }
    return *own.t;
}
}  // namespace
HitScratch& thread_hit_scratch(int device) { return thread_scratch().hits[device]; }
DevScratch& thread_scan_scratch(int device) { return thread_scratch().scan[device]; }
DevScratch& thread_probe_scratch(int device) { return thread_scratch().probe[device]; }
DevScratch& thread_walk_scratch(int device) { return thread_scratch().walk[device]; }
PinnedHits& thread_pinned_hits() { return thread_scratch().pinned; }
ScratchHold::ScratchHold() : mu(&thread_scratch().mu) { mu->lock(); }
ScratchHold::~ScratchHold() { mu->unlock(); }
}  // namespace sydelta

namespace {
PinnedHits& thread_seg_pin() { return thread_scratch().seg_pin; }
PinnedHits& thread_probe_pin() { return thread_scratch().probe_pin; }
PinnedHits& thread_phase_pin() { return thread_scratch().phase_pin; }
PinnedHits& thread_walk_map() { return thread_scratch().walk_map; }
// Copy `bytes` of host memory to d_dst in s's order without waiting for the copy: through a
// slot of the calling thread's pinned ring (a pageable source would have to outlive the
// copy, i.e. a stream synchronisation).  The current device is the stream's.
int upload_staged(void* d_dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return SYDELTA_OK;
    ScratchHold hold;
    ThreadScratch& t = thread_scratch();
    const unsigned i = t.up_next++ & 3;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (t.up_ev[i]) {
        HIP_TRY(hipEventSynchronize(t.up_ev[i]));  // the slot's previous copy (long done, as a rule)
        if (t.up_dev[i] != dev) {
            DeviceScope keep;
            (void)hipSetDevice(t.up_dev[i]);
            (void)hipEventDestroy(t.up_ev[i]);
            t.up_ev[i] = nullptr;
        }
    }
    if (!t.up_ev[i]) {
        HIP_TRY(hipEventCreateWithFlags(&t.up_ev[i], hipEventDisableTiming));
        t.up_dev[i] = dev;
    }
    if (int r = pinned_at_least(t.up[i], bytes)) return r;
    memcpy(t.up[i].p, src, bytes);
    HIP_TRY(hipMemcpyAsync(d_dst, t.up[i].p, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(t.up_ev[i], s));
    return SYDELTA_OK;
}
// a pinned host buffer of at least `bytes` (grown by a quarter; the previous call on this
// thread synchronized the streams that used it)
int pinned_at_least(PinnedHits& h, size_t bytes) {
    if (h.bytes >= bytes) return SYDELTA_OK;
    if (h.p) (void)hipHostFree(h.p);
    h = PinnedHits();
    HIP_TRY(hipHostMalloc((void**)&h.p, bytes + bytes / 4, hipHostMallocDefault));
    h.bytes = bytes + bytes / 4;
    return SYDELTA_OK;
}
}  // namespace

namespace {
void release_small_ops();  // the recycled per-file op arrays (below)
}

extern "C" void sydelta_trim(void) {
    DeviceScope keep_device;  // the frees below switch devices
    release_small_ops();
    // kept index allocations of every device, released in their (library) streams' order
    KeptPool kept[64];
    {
        std::lock_guard<std::mutex> lk(g_kept_mu);
        for (int d = 0; d < 64; ++d) {
            kept[d] = g_kept[d];
            g_kept[d] = KeptPool();
        }
    }
    for (int d = 0; d < 64; ++d)
        if (kept[d].p && hipSetDevice(d) == hipSuccess) (void)hipFreeAsync(kept[d].p, kept[d].s);
    release_mapped();
    // the scan / probe / walk scratch of this thread and of every thread not inside a call
    (void)thread_scratch();  // registers this thread's
    std::lock_guard<std::mutex> lk(scratch_mu());
    for (ThreadScratch* t : all_scratch()) {
        std::unique_lock<std::recursive_mutex> h(t->mu, std::try_to_lock);
        if (h.owns_lock()) release_scratch(*t);
    }
}

extern "C" void sydelta_index_free(sydelta_index* idx) {
    if (!idx) return;
    DeviceScope keep_device;
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipSetDevice(idx->device);
    const auto t1 = std::chrono::steady_clock::now();
    index_release(idx);
    if (host_timing)
        fprintf(stderr, "sydelta index free: set device %.3f ms, release %.3f ms\n",
                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
}

static int index_create_impl(int device, const uint32_t* weak, const uint64_t* strong, const uint64_t* nblk,
                             const uint64_t* last, uint64_t nfiles, uint64_t block_size, int arrays_on_device,
                             void* stream, sydelta_index** out) {
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (nfiles == 0 || nfiles >= 0xFFFFFFFFull) return fail(SYDELTA_E_INVAL, "bad file count %llu", (unsigned long long)nfiles);
    std::vector<uint64_t> fblk(nfiles + 1, 0);
    uint64_t max_nblk = 0;
    for (uint64_t f = 0; f < nfiles; ++f) {
        if (nblk[f] && (last[f] == 0 || last[f] > block_size))
            return fail(SYDELTA_E_INVAL, "file %llu: last_size must be in [1, block_size]", (unsigned long long)f);
        fblk[f + 1] = fblk[f] + nblk[f];
        max_nblk = std::max(max_nblk, nblk[f]);
    }
    const uint64_t nblocks = fblk[nfiles];
    if (nblocks && (!weak || !strong)) return fail(SYDELTA_E_INVAL, "NULL signature arrays");
    if (nblocks >= 0xFFFFFFFFull) return fail(SYDELTA_E_INVAL, "too many blocks (%llu)", (unsigned long long)nblocks);
    SYDELTA_ENTER_DEVICE(device);
    if (device < 0) device = 0;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device);
    std::unique_ptr<sydelta_index, void (*)(sydelta_index*)> x(new sydelta_index(), index_release);
    x->device = device;
    x->bs = block_size;
    x->nfiles = nfiles;
    x->fblk = fblk;
    x->max_nblk = max_nblk;
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
        F.fwshift = 32 - fwbits;  // 2^fwbits 32-bit words
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
    // the level-1 filter of the register-fed scans (k_scan_r at bs 4096, k_scan_g at any
    // other): one file with more keys than an LDS-resident Bloom filter takes
    const bool want_narrow = nfiles == 1 && nblocks > kLdsFilterKeys;
    // windows above the LDS-staged scans' limit, one file (the production block sizes of
    // files over 64 MiB, mod.rs:20-23): k_scan_g's level-1 filter and fat table
    const bool want_wide = nfiles == 1 && block_size > scan_max_window() && scan_wide_mode() != 0;
    const bool want_l1 = want_narrow || want_wide;
    const uint32_t l1_wshift = 1u;  // kL1WordsR words (k_scan_r / k_scan_g)
    const size_t sz_l1 = want_l1 ? al(4 * l1_total_words(l1_wshift)) : 0;
    // k_scan_r's ribbon level-1 (sydelta_internal.hpp): its key lists, counts, overflow list
    // SYDELTA_L1=bloom|ribbon forces the layout (A/B measurements, parity tests at small sizes)
    const char* l1e = getenv("SYDELTA_L1");
    const bool want_rib = want_narrow && (l1e && !strcmp(l1e, "ribbon") ? true
                                          : l1e && !strcmp(l1e, "bloom") ? false
                                                                          : nblocks >= kRibMinKeys && nblocks <= kRibMaxKeys);
    const size_t sz_rib = want_rib ? al(4ull * kL1WordsR) + al(4ull * kRibShards * kRibCap) + al(4ull * (kRibShards + 1)) +
                                         al(4 * nb)
                                   : 0;
    const size_t sz_fat = want_l1 ? al(16 * (size_t)sl) : 0;
    const size_t total = sz_weak + sz_strong + sz_filt + sz_l1 + sz_fat + 4 * sz_t + sz_order + sz_slot + sz_files +
                         sz_fblk + sz_cstrong + sz_rib;
    x->d_pool = take_kept_pool(device, total, s, &x->pool_bytes);
    if (!x->d_pool) {
        HIP_TRY(dev_malloc_async(&x->d_pool, total, s));  // stream-ordered: no device-wide synchronization
        x->pool_bytes = total;
    }
    x->stream = s;
    uint8_t* p = (uint8_t*)x->d_pool;
    x->d_weak = (uint32_t*)p; p += sz_weak;
    x->d_strong = (uint64_t*)p; p += sz_strong;
    ix.filt = (uint32_t*)p; p += sz_filt;
    if (want_l1) {
        ix.l1 = (uint32_t*)p; p += sz_l1;
        ix.l1_wshift = l1_wshift;
        if (want_rib) {  // the Bloom stays in l1; the ribbon is built on demand (scan_index)
            x->rib_mode = l1e && !strcmp(l1e, "ribbon") ? 2 : 1;
            ix.rib_l1 = (uint32_t*)p; p += al(4ull * kL1WordsR);
            ix.rib_keys = (uint32_t*)p; p += al(4ull * kRibShards * kRibCap);
            ix.rib_cnt = (uint32_t*)p; p += al(4ull * (kRibShards + 1));
            ix.rib_over = (uint32_t*)p; p += al(4 * nb);
        }
        ix.fat = (uint4*)p; p += sz_fat;
    }
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
    // device arrays: nothing waited for here.  One file is built on this thread's aux stream; a
    // batch's index, used at once by its match, in the caller's stream order (more streams per
    // caller share the process's four hardware queues with ten callers' work).
    if (arrays_on_device) {
        const size_t fb = sizeof(FileIx) * nfiles, tb = ((fb + 15) & ~(size_t)15) + 8 * (nfiles + 1);
        if (int r = take_mapped(tb, x->stage, kStage)) return r;
        memcpy(x->stage.p, ix.files.data(), fb);
        memcpy(x->stage.p + ((fb + 15) & ~(size_t)15), x->fblk.data(), 8 * (nfiles + 1));
        HIP_TRY(hipMemcpyAsync(ix.d_files, x->stage.p, fb, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(ix.d_fblk, x->stage.p + ((fb + 15) & ~(size_t)15), 8 * (nfiles + 1),
                               hipMemcpyHostToDevice, s));
        // one file: on the aux stream, beside the caller's next work; a batch: in the caller's
        // stream order, no host wait (its match follows at once on that stream)
        const hipStream_t sb = nfiles == 1 ? thread_aux_stream(device) : s;
        if (!sb) return fail(SYDELTA_E_OOM, "no stream for the index build");
        HIP_TRY(stream_after(sb, s, device));
        x->ready = take_event(device);
        if (!x->ready) return fail(SYDELTA_E_OOM, "no event for the index build");
        // a batch of small files whose walks self-index (file_walk_ok's index conditions): the
        // build waits for a match that takes another path (index_full)
        x->deferred = nfiles >= 2 && block_size % 64 == 0 && block_size >= 256 && block_size <= kWalkMaxN &&
                      max_nblk <= kSelfIxMaxBlocks && !ix.l1;
        x->extras_deferred = nfiles == 1 && ix.l1 != nullptr;
        if (!x->deferred) {
            CallProf cp;
            HIP_TRY(launch_index_build(x->d_weak, x->d_strong, ix, sb, cp.get(), !x->extras_deferred));
        }
        HIP_TRY(hipEventRecord(x->ready, sb));
        // the ribbon level-1 of a whole-file scan as large as the basis (scan_index), from the
        // signature's weak values on a stream of its own: beside the index build (queued after
        // it, the first to be needed), before the match call is made (SYDELTA_EARLY_RIBBON: 2 here, 1 at the match call, 0 after the
        // index, as in round 5).  A match that never scans has spent ~0.2 ms of a few CUs.
        if (nfiles == 1 && nblocks && early_ribbon_mode() == 2 &&
            (x->rib_mode == 2 || (x->rib_mode == 1 && nblocks * block_size >= kRibMinScan))) {
            const hipStream_t sr = thread_walk_stream(device, 2);
            if (!sr) return fail(SYDELTA_E_OOM, "no stream for the ribbon");
            HIP_TRY(stream_after(sr, s, device));
            CallProf cp;
            HIP_TRY(launch_ribbon_build(ix, sr, cp.get(), x->d_weak, nblocks));
            if (!(x->rib_ev = take_event(device))) return fail(SYDELTA_E_OOM, "no event for the ribbon");
            HIP_TRY(hipEventRecord(x->rib_ev, sr));
            x->rib_built = true;
            x->rib_stream = sr;
        }
        *out = x.release();
        return SYDELTA_OK;
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
                                    sydelta_index** out) try {
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t last = nblocks ? last_size : 0;
    const int r = index_create_impl(device, weak, strong, &nblocks, &last, 1, block_size, arrays_on_device, stream, out);
    if (host_timing)
        fprintf(stderr, "sydelta index create: %.3f ms (host)\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    return r;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_index_create_batch(int device, const uint32_t* weak, const uint64_t* strong,
                                          const uint64_t* nblocks, const uint64_t* last_size, uint64_t nfiles,
                                          uint64_t block_size, int arrays_on_device, void* stream,
                                          sydelta_index** out) try {
    if (nfiles && (!nblocks || !last_size)) return fail(SYDELTA_E_INVAL, "NULL file table");
    return index_create_impl(device, weak, strong, nblocks, last_size, nfiles, block_size, arrays_on_device, stream,
                             out);
} catch (...) {
    return sydelta::host_exception();
}

// ---------------------------------------------------------------------------
// delta object
// ---------------------------------------------------------------------------
// Recycled op arrays: a walk over a copy-heavy source emits one op per block
// (1 Mi ops = 24 MiB for 8 GiB at 8 KiB blocks); first-touch page faults of a
// fresh array cost more than the walk itself, so freed deltas hand their arrays
// back for the next walk (bounded: 16 arrays; a parallel walk takes one per segment).
namespace {
// Pinned op arrays (walk::op_arena): installed with the device walk, so the D2H of a
// device-resolved op list is a DMA into the delta's own array.  Released arrays go back
// to the pool below first; one released at process exit is left to the OS (the HIP
// runtime may already be gone).
std::atomic<bool> g_exiting{false};
std::mutex g_arena_mu;
std::unordered_set<void*>* g_arena_live = new std::unordered_set<void*>();  // never destroyed
void* arena_alloc(size_t bytes) {
    void* p = nullptr;
    if (g_exiting.load() || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_arena_mu);
    g_arena_live->insert(p);
    return p;
}
bool arena_release(void* p) {
    {
        std::lock_guard<std::mutex> lk(g_arena_mu);
        if (!g_arena_live->erase(p)) return false;
    }
    if (!g_exiting.load()) (void)hipHostFree(p);
    return true;
}
void install_op_arena() {
    static std::once_flag once;
    std::call_once(once, [] {
        atexit([] { g_exiting = true; });  // runs before the HIP runtime's own teardown
        ::op_arena().release = arena_release;
        ::op_arena().alloc = arena_alloc;
    });
}

std::atomic<uint64_t> g_device_walks{0}, g_device_walk_fallbacks{0};  // sydelta_walk_counters
std::atomic<uint64_t> g_expand_files{0}, g_expand_host{0};               // sydelta_expand_counters

struct OpSlab;
OpSlab* slab_of(const void* q);  // (below)
std::mutex g_ops_mu;
std::vector<OpVec>& g_ops_pool = *new std::vector<OpVec>();  // never destroyed (arrays may be pinned)
OpVec take_ops(size_t want) {
    // best fit: the smallest pooled array holding `want`, else the largest one when it
    // holds at least half (it grows once)
    std::lock_guard<std::mutex> lk(g_ops_mu);
    size_t best = g_ops_pool.size(), big = g_ops_pool.size();
    for (size_t i = 0; i < g_ops_pool.size(); ++i) {
        const size_t c = g_ops_pool[i].capacity();
        if (c >= want && (best == g_ops_pool.size() || c < g_ops_pool[best].capacity())) best = i;
        if (big == g_ops_pool.size() || c > g_ops_pool[big].capacity()) big = i;
    }
    if (best == g_ops_pool.size() && big < g_ops_pool.size() && g_ops_pool[big].capacity() >= want / 2) best = big;
    OpVec v;
    if (best < g_ops_pool.size()) {
        v.swap(g_ops_pool[best]);
        g_ops_pool.erase(g_ops_pool.begin() + best);
    }
    v.clear();
    return v;
}
void give_ops(OpVec&& v) {
    if (v.capacity() < 4096 || slab_of(v.data())) return;  // (a slab's array goes back to its slab)
    std::lock_guard<std::mutex> lk(g_ops_mu);
    if (g_ops_pool.size() < 16) g_ops_pool.push_back(std::move(v));
}

// The per-file op arrays of batched matches (C4: 10 000 arrays of ~6 KiB) are recycled
// whole: a freed batch hands them back and the next batch's files take them before
// their walks.  Fresh arrays cost more in allocation and first-touch page faults than
// the walks that fill them, and their release as much again (tools/walk_bench_c4.cpp,
// 10 000 C4 files on 8 threads in this container: walks 14 ms with fresh arrays, 5.3 ms
// with recycled ones, and 14 ms to free the fresh ones).  At most kSmallPoolBytes held.
std::mutex g_small_mu;
std::vector<OpVec>* g_small_pool = new std::vector<OpVec>();  // never destroyed (exit order)
size_t g_small_bytes = 0;
constexpr size_t kSmallPoolBytes = (size_t)512 << 20;
void give_small_ops(std::vector<sydelta_delta>& d) {
    std::lock_guard<std::mutex> lk(g_small_mu);
    for (auto& x : d) {
        const size_t c = x.ops.capacity() * sizeof(sydelta_op);
        if (!c || c >= kOpArenaMin || slab_of(x.ops.data())) continue;  // (a slab's arrays go back to it)
        if (g_small_bytes + c > kSmallPoolBytes) break;
        g_small_bytes += c;
        g_small_pool->push_back(std::move(x.ops));
    }
}
void release_small_ops() {
    std::vector<OpVec> v;
    {
        std::lock_guard<std::mutex> lk(g_small_mu);
        v.swap(*g_small_pool);
        g_small_bytes = 0;
    }
}
void take_small_ops(std::vector<sydelta_delta>& d) {
    std::lock_guard<std::mutex> lk(g_small_mu);
    for (auto& x : d) {
        if (g_small_pool->empty()) break;
        x.ops.swap(g_small_pool->back());
        g_small_pool->pop_back();
        g_small_bytes -= x.ops.capacity() * sizeof(sydelta_op);
        x.ops.clear();
    }
}

// Op slabs (OpSlabHooks, sydelta_walk.hpp): when the device expands a batch's op lists
// (WalkArgs::x), every file's op array is reserved from one pinned, host-mapped slab that
// the kernel writes into.  A slab counts its live arrays (+1 while the batch reserves from it)
// and is reused once they are all gone; slabs are kept for the process (at most kMaxSlabs:
// ten concurrent callers take one each), so a released array never races with a free.
struct OpSlab {
    uint8_t* p = nullptr;
    size_t bytes = 0;
    std::atomic<int64_t> live{0};
};
constexpr int kMaxSlabs = 32;
std::atomic<OpSlab*> g_slab_tab[kMaxSlabs];
std::mutex g_slab_mu;
thread_local OpSlab* t_slab = nullptr;  // the slab this thread reserves from
thread_local size_t t_slab_used = 0;
void* slab_take(size_t bytes) {
    OpSlab* sl = t_slab;
    if (!sl || t_slab_used + bytes > sl->bytes) return nullptr;
    void* q = sl->p + t_slab_used;
    t_slab_used += bytes;  // (multiples of 24 bytes: every array stays 8-byte aligned)
    sl->live.fetch_add(1);
    return q;
}
OpSlab* slab_of(const void* q) {
    for (int i = 0; i < kMaxSlabs; ++i) {
        OpSlab* sl = g_slab_tab[i].load(std::memory_order_acquire);
        if (sl && (const uint8_t*)q >= sl->p && (const uint8_t*)q < sl->p + sl->bytes) return sl;
    }
    return nullptr;
}
bool slab_give(void* q) {
    OpSlab* sl = slab_of(q);
    if (!sl) return false;
    sl->live.fetch_sub(1);
    return true;
}
// A slab of at least `bytes` for this thread's reservations (nullptr: none to be had, the host
// expands); slab_close ends them.
OpSlab* slab_open(size_t bytes) {
    static std::once_flag once;
    std::call_once(once, [] {
        op_slab().take = slab_take;
        op_slab().give = slab_give;
    });
    std::lock_guard<std::mutex> lk(g_slab_mu);
    OpSlab* best = nullptr;
    int freei = -1;
    for (int i = 0; i < kMaxSlabs; ++i) {
        OpSlab* sl = g_slab_tab[i].load(std::memory_order_acquire);
        if (!sl) {
            if (freei < 0) freei = i;
            continue;
        }
        if (sl->live.load() == 0 && sl->bytes >= bytes && (!best || sl->bytes < best->bytes)) best = sl;
    }
    if (best) {
        int64_t z = 0;
        if (!best->live.compare_exchange_strong(z, 1)) best = nullptr;  // (taken back by a late release? no: live 0 stays 0)
    }
    if (!best) {
        if (freei < 0) return nullptr;
        size_t want = (size_t)1 << 20;
        while (want < bytes) want <<= 1;  // powers of two: reuse across batch sizes
        OpSlab* sl = new OpSlab();
        if (hipHostMalloc((void**)&sl->p, want, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) !=
            hipSuccess) {
            delete sl;
            return nullptr;
        }
        sl->bytes = want;
        sl->live.store(1);
        g_slab_tab[freei].store(sl, std::memory_order_release);
        best = sl;
    }
    t_slab = best;
    t_slab_used = 0;
    return best;
}
void slab_close(OpSlab* sl) {
    t_slab = nullptr;
    t_slab_used = 0;
    if (sl) sl->live.fetch_sub(1);
}
}  // namespace


struct sydelta_delta_batch {
    std::vector<sydelta_delta> d;
    sydelta_match_stats total{};
};

extern "C" int sydelta_expand_counters(uint64_t* device_files, uint64_t* host_batches) {
    if (device_files) *device_files = g_expand_files.load();
    if (host_batches) *host_batches = g_expand_host.load();
    return SYDELTA_OK;
}

extern "C" int sydelta_walk_counters(uint64_t* device_walks, uint64_t* device_fallbacks) {
    if (device_walks) *device_walks = g_device_walks.load();
    if (device_fallbacks) *device_fallbacks = g_device_walk_fallbacks.load();
    return SYDELTA_OK;
}

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
extern "C" int sydelta_delta_stats(const sydelta_delta* d, sydelta_match_stats* out) try {
    if (!d || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = d->stats;
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}
// generator.rs:30-55
extern "C" double sydelta_delta_compression_ratio(const sydelta_delta* d) {
    if (!d) return 1.0;
    uint64_t lit = 0, cop = 0;
    for (auto& o : d->ops) (o.kind == SYDELTA_OP_DATA ? lit : cop) += o.b;
    const uint64_t tot = lit + cop;
    return tot == 0 ? 1.0 : (double)lit / (double)tot;
}
extern "C" void sydelta_delta_free(sydelta_delta* d) {
    if (!d) return;
    give_ops(std::move(d->ops));
    delete d;
}

extern "C" uint64_t sydelta_delta_batch_count(const sydelta_delta_batch* b) { return b ? b->d.size() : 0; }
extern "C" const sydelta_delta* sydelta_delta_batch_get(const sydelta_delta_batch* b, uint64_t i) {
    return (b && i < b->d.size()) ? &b->d[i] : nullptr;
}
extern "C" int sydelta_delta_batch_stats(const sydelta_delta_batch* b, sydelta_match_stats* out) try {
    if (!b || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = b->total;
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}
extern "C" void sydelta_delta_batch_free(sydelta_delta_batch* b) {
    if (!b) return;
    give_small_ops(b->d);
    delete b;
}

// ---------------------------------------------------------------------------
// match
// ---------------------------------------------------------------------------
// Classification + walk.  Every full-window position p of a source is classified
// (hit: first block in index order with equal weak and strong, or not) by one of
//   * the aligned probe (k_probe): positions k*n, one wave per window;
//   * the rolling scan (k_scan_lds / k_scan): every position of a block range.
// The greedy walk (generator.rs:116-221) then runs on the host over the sorted
// hits.  When the probe runs, the scan covers only the blocks whose aligned window
// did not hit: the walk reaches such a block's interior only through an unaligned
// hit's jump, and when it does the block is scanned on demand (Classifier::walk).
// The op list is identical whichever subset was classified first.
namespace {
struct DevBuf {
    void* p = nullptr;
    hipStream_t s = nullptr;
    ~DevBuf() {
        if (p) (void)hipFreeAsync(p, s);
    }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
};

using walk::BasisInfo;
using walk::HitBlk;
using walk::HitPos;
using walk::first_unknown;
using walk::kNoBlk;
using walk::kUnknownNone;
using walk::merge_hits;
using walk::run_parallel;
using walk::Src;
using walk::walk_src;

double ms_since(std::chrono::steady_clock::time_point t0);
void finish_stats_impl(sydelta_delta* d);
int walk_threads();
uint64_t walk_par_min();
bool device_walk_on();
uint64_t device_walk_min();


bool phase_probe_on() {
    // probe long miss runs at their phase ("0": off).  Off by default until round 4: on the
    // C4 shape the host time of the phase probes outweighed the scan they save; with the
    // host path trimmed the phase probe takes C4 (10 callers) from 19.6 to 17.3 ms/step
    // (profiles/r04p_c4c10{,ph}_bench.json)
    const char* e = getenv("SYDELTA_PHASE_PROBE");
    return !(e && e[0] == '0');
}

// The index carries k_scan_g's level-1 filter (one file, window above the LDS-staged
// scans' limit) and SYDELTA_SCAN_WIDE does not turn it off.
bool wide_scan(const sydelta_index* x) {
    return x->ix.l1 != nullptr && scan_wide_mode() != 0;
}

int probe_mode_env() {
    const char* e = getenv("SYDELTA_PROBE");  // "0" never, "1" always, unset/other: auto
    if (e && e[0] == '0') return 0;
    if (e && e[0] == '1') return 1;
    return -1;
}

struct Classifier {
    sydelta_index* ix = nullptr;
    const uint8_t* base = nullptr;  // launch base (sources at Src::off)
    hipStream_t s = nullptr;
    Profiler* prof = nullptr;
    uint64_t n = 0;
    std::vector<Src> src;
    uint64_t weak_hits = 0;
    // probed sources: their runs of blocks whose aligned window missed, [first, end)
    // local blocks, ascending; source i's are miss_runs[miss_off[i] .. miss_off[i+1])
    // (set by probe)
    std::vector<std::array<uint64_t, 2>> miss_runs;
    std::vector<size_t> miss_off;
    // the full probe pass's results on the device: source i's at d_probe_out + probe_pfx[i]
    DevBuf probe_buf;
    // a transient classifier (one match call) takes its probe buffers from the calling
    // thread's kept scratch instead (a chunk's outlives other calls on its thread)
    DevScratch* probe_scratch = nullptr;
    uint32_t* d_probe_out = nullptr;
    std::vector<uint64_t> probe_pfx;

    // Aligned probe of every block of every source (mode 1), of none (0), or, in
    // auto mode (-1), when a 1-in-16 sample finds >= 1/8 of its windows hitting.
    int probe(int mode);
    // Scan blocks [ka, kz) of source si for every (si, ka, kz); hits merged, blocks marked.
    int scan(const std::vector<std::array<uint64_t, 3>>& ranges);
    int classify(int mode);
    // Probe window starts k*n + phi for blocks [k0, k0 + cnt) of source si, for every
    // job {si, k0 (local block), cnt, phi}: hits are merged into the sources' hit lists,
    // every probed start is recorded in ppos, and the blocks that missed are appended
    // to `missed` as scan ranges.
    int phase_probe(const std::vector<std::array<uint64_t, 4>>& jobs,
                    std::vector<std::array<uint64_t, 3>>& missed);
    // Walk source i from entry, scanning on demand what the walk needs.
    int walk(size_t i, uint64_t entry, const BasisInfo& bi, bool final_src, int tail_match, sydelta_delta* d,
             uint64_t* exit);
    // The same walk split at block-aligned points over threads, each segment walked
    // speculatively from its split point; a segment whose true entry (the previous
    // segment's exit) differs is walked again from it.  Returns 0 (done, d->ops set),
    // 1 (a segment reached an unclassified block: walk sequentially), 2 (too small).
    int walk_parallel(size_t i, uint64_t entry, const BasisInfo& bi, bool final_src, int tail_match,
                      sydelta_delta* d, uint64_t* exit);
    // The same walk resolved on the device (K5b, sydelta_chain.hpp; SYDELTA_DEVICE_WALK=1).
    // Returns 0 (done, d->ops and its stats set), 1 (the path reaches an unclassified
    // position: walk on the host, which scans on demand), 2 (not applicable) or an error.
    int walk_device(size_t i, uint64_t entry, const BasisInfo& bi, bool final_src, int tail_match,
                    sydelta_delta* d, uint64_t* exit);

    // The first sources' per-block and hit lists are handed to the next classifier on
    // the same thread (emptied, capacity kept): at C3b's 1 Mi blocks and hits, fresh
    // lists cost their first-touch page faults and their release ~3 ms (measured, round
    // 3).  Bounded: kSpareSrcs sources, kSpareBytes in all.
    static constexpr size_t kSpareSrcs = 2, kSpareBytes = 512ull << 20;
    static std::vector<Src>& spare() {
        static thread_local std::vector<Src> v;
        return v;
    }
    template <class V>
    static size_t cap_bytes(const V& v) {
        return v.capacity() * sizeof(typename V::value_type);
    }
    static size_t src_bytes(const Src& c) {
        return cap_bytes(c.ahit) + cap_bytes(c.scanned) + cap_bytes(c.hpos) + cap_bytes(c.hblk) +
               cap_bytes(c.ppos) + cap_bytes(c.phit);
    }
    // after src.resize(): take the spare lists
    void adopt_spare() {
        auto& sp = spare();
        for (size_t i = 0; i < src.size() && i < sp.size(); ++i) {
            src[i].ahit.swap(sp[i].ahit);
            src[i].scanned.swap(sp[i].scanned);
            src[i].hpos.swap(sp[i].hpos);
            src[i].hblk.swap(sp[i].hblk);
            src[i].ppos.swap(sp[i].ppos);
            src[i].phit.swap(sp[i].phit);
        }
        sp.clear();
    }
    ~Classifier() {
        auto& sp = spare();
        size_t total = 0;
        sp.clear();
        for (size_t i = 0; i < src.size() && sp.size() < kSpareSrcs; ++i) {
            const size_t b = src_bytes(src[i]);
            if (total + b > kSpareBytes) break;
            total += b;
            sp.emplace_back();
            Src& k = sp.back();
            k.ahit.swap(src[i].ahit);
            k.scanned.swap(src[i].scanned);
            k.hpos.swap(src[i].hpos);
            k.hblk.swap(src[i].hblk);
            k.ppos.swap(src[i].ppos);
            k.phit.swap(src[i].phit);
            k.ahit.clear();
            k.scanned.clear();
            k.hpos.clear();
            k.hblk.clear();
            k.ppos.clear();
            k.phit.clear();
        }
    }
};

int Classifier::probe(int mode) {
    if (mode == 0) return SYDELTA_OK;
    uint64_t total = 0;
    for (auto& c : src) total += c.nblk;
    if (!total) return SYDELTA_OK;
    if (mode < 0 && total < 4096) return SYDELTA_OK;  // small inputs: one scan is cheaper
    bool fast = n % 64 == 0 && n >= 256;
    for (auto& c : src) fast = fast && ((uintptr_t)(base + c.off) & 15) == 0;
    // results land in pinned host memory (per thread, grown on demand): no zero fill and
    // no staging copy for the D2H of one u32 per probed window
    ScratchHold hold;
    PinnedHits& pin = thread_probe_pin();
    uint32_t* out = nullptr;
    uint64_t nout = 0;
    auto run = [&](uint32_t stride, std::vector<uint64_t>& pfx) -> int {
        std::vector<ProbeJob> jobs;
        pfx.assign(src.size() + 1, 0);
        uint64_t np = 0;
        for (size_t i = 0; i < src.size(); ++i) {
            const Src& c = src[i];
            pfx[i] = np;
            const uint64_t cnt = (c.nblk + stride - 1) / stride;
            if (cnt) jobs.push_back({c.off, c.kb, np, c.file, 0});
            np += cnt;
        }
        pfx[src.size()] = np;
        nout = np;
        if (!np) return SYDELTA_OK;
        if (int r = pinned_at_least(pin, np * 4)) return r;
        out = (uint32_t*)pin.p;
        // the full pass's results stay on the device for the device walk (walk_device)
        DevBuf local;
        DevBuf& jb = stride == 1 ? probe_buf : local;
        if (jb.p) { (void)hipFreeAsync(jb.p, s); jb.p = nullptr; }
        const size_t jbytes = (jobs.size() * sizeof(ProbeJob) + 255) & ~(size_t)255;
        const size_t obytes = (np * 4 + 255) & ~(size_t)255;
        const size_t need = jbytes + 2 * obytes + np * 8;
        uint8_t* jp = nullptr;
        if (probe_scratch) {  // the sample pass's results were read before the full pass reuses it
            if (probe_scratch->bytes < need) {
                if (probe_scratch->p) (void)hipFreeAsync(probe_scratch->p, s);
                *probe_scratch = DevScratch();
                HIP_TRY(dev_malloc_async(&probe_scratch->p, need + need / 4, s));
                probe_scratch->bytes = need + need / 4;
            }
            jp = (uint8_t*)probe_scratch->p;
        } else {
            HIP_TRY(dev_malloc_async(&jb.p, need, s));
            jb.s = s;
            jp = (uint8_t*)jb.p;
        }
        uint32_t* d_out = (uint32_t*)(jp + jbytes);
        uint32_t* d_pw = (uint32_t*)(jp + jbytes + obytes);
        if (stride == 1) {
            d_probe_out = d_out;
        }
        uint64_t* d_pst = (uint64_t*)(jp + jbytes + 2 * obytes);
        HIP_TRY(hipMemcpyAsync(jp, jobs.data(), jobs.size() * sizeof(ProbeJob), hipMemcpyHostToDevice, s));
        HIP_TRY(launch_probe(base, (const ProbeJob*)jp, (uint32_t)jobs.size(), np, stride, (uint32_t)n, fast,
                             ix->ix, d_pw, d_pst, d_out, s, prof));
        HIP_TRY(hipMemcpyAsync(out, d_out, np * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        return SYDELTA_OK;
    };
    std::vector<uint64_t> pfx;
    if (mode < 0) {
        const uint32_t S = 16;
        if (int r = run(S, pfx)) return r;
        uint64_t hits = 0;
        for (uint64_t i = 0; i < nout; ++i) hits += out[i] != kNoBlk;
        if (hits * 8 < nout) return SYDELTA_OK;
    }
    if (int r = run(1, pfx)) return r;
    probe_pfx = pfx;
    // Copy the results into the sources and find their miss runs (the blocks classify
    // scans) in one pass, in pieces of 64 Ki blocks on the host pool: one large source
    // (C5) is split as well as many small ones (C4).
    const size_t ns = src.size();
    constexpr uint64_t kPiece = 1 << 16;
    struct Piece {
        size_t si;
        uint64_t b0, b1;  // local blocks
    };
    std::vector<Piece> pieces;
    for (size_t i = 0; i < ns; ++i) {
        Src& c = src[i];
        c.probed = true;
        if (c.nblk > kPiece) {  // one piece per source is sized on its pool thread (C4: 10 000 sources)
            c.ahit.resize(c.nblk);
            c.scanned.assign(c.nblk, 0);
        }
        for (uint64_t b = 0; b < c.nblk; b += kPiece) pieces.push_back({i, b, std::min(c.nblk, b + kPiece)});
    }
    struct Run {
        size_t si;
        uint64_t k, e;
    };
    const size_t np = pieces.size();
    const int nthr = np > 1 ? std::min<int>(walk_threads(), (int)np) : 1;
    std::vector<std::vector<Run>> truns(nthr);
    auto fill = [&](int t) {  // pieces [np*t/nthr, np*(t+1)/nthr), in order
        std::vector<Run> runs;  // on this thread's stack: the vector headers in truns sit side by side
        for (size_t p = np * t / nthr, pe = np * (t + 1) / nthr; p < pe; ++p) {
            const Piece& q = pieces[p];
            const uint32_t* in = out + pfx[q.si];
            if (src[q.si].nblk <= kPiece) {
                src[q.si].ahit.resize(src[q.si].nblk);
                src[q.si].scanned.assign(src[q.si].nblk, 0);
            }
            memcpy(src[q.si].ahit.data() + q.b0, in + q.b0, (q.b1 - q.b0) * sizeof(uint32_t));
            uint64_t k = q.b0;
            while (k < q.b1) {
                // 16 windows at a time while none missed (a loop the compiler vectorizes)
                if (k + 16 <= q.b1) {
                    bool miss = false;
                    for (int j = 0; j < 16; ++j) miss |= in[k + j] == kNoBlk;
                    if (!miss) { k += 16; continue; }
                }
                if (in[k] != kNoBlk) { ++k; continue; }
                uint64_t e = k + 1;
                while (e < q.b1 && in[e] == kNoBlk) ++e;
                runs.push_back({q.si, k, e});
                k = e;
            }
        }
        truns[t].swap(runs);
    };
    if (!run_parallel(nthr, fill)) return fail(SYDELTA_E_OOM, "out of host memory (probe results)");
    // runs in (source, block) order; a run that crosses a piece boundary is joined
    miss_runs.clear();
    miss_off.assign(ns + 1, 0);
    size_t last_si = SIZE_MAX;
    for (auto& tr : truns)
        for (const Run& r : tr) {
            if (r.si == last_si && miss_runs.back()[1] == r.k) {
                miss_runs.back()[1] = r.e;
                continue;
            }
            miss_runs.push_back({r.k, r.e});
            ++miss_off[r.si + 1];
            last_si = r.si;
        }
    for (size_t i = 0; i < ns; ++i) miss_off[i + 1] += miss_off[i];
    for (size_t i = 0; i < ns; ++i) {
        uint64_t missed = 0;
        for (size_t j = miss_off[i]; j < miss_off[i + 1]; ++j) missed += miss_runs[j][1] - miss_runs[j][0];
        src[i].nahit = src[i].nblk - missed;
    }
    return SYDELTA_OK;
}

// The index a scan of tot_pos positions runs against: with the ribbon level-1 (built here
// by the first scan that wants it, sydelta_index::rib_mode) or as built (the Bloom).
static hipError_t scan_index(sydelta_index* x, uint64_t tot_pos, hipStream_t s, Profiler* prof, DeviceIndex& out) {
    out = x->ix;
    {  // the scan extras, filled by the first scan (sydelta_index::extras_deferred)
        std::lock_guard<std::mutex> lk(x->build_mu);
        if (x->extras_deferred) {
            if (hipError_t e = launch_index_extras(x->d_weak, x->ix, s, prof)) return e;
            if (!x->extras_ev)
                if (!(x->extras_ev = take_event(x->device))) return hipErrorOutOfMemory;
            if (hipError_t e = hipEventRecord(x->extras_ev, s)) return e;
            x->extras_deferred = false;
            x->extras_stream = s;
        } else if (x->extras_ev && x->extras_stream != s) {
            if (hipError_t e = hipStreamWaitEvent(s, x->extras_ev, 0)) return e;
        }
    }
    if (x->rib_mode == 0 || (x->rib_mode == 1 && tot_pos < kRibMinScan)) return hipSuccess;
    {
        std::lock_guard<std::mutex> lk(x->rib_mu);
        if (!x->rib_built) {
            if (hipError_t e = launch_ribbon_build(x->ix, s, prof)) return e;
            if (!x->rib_ev) {
                if (!(x->rib_ev = take_event(x->device))) return hipErrorOutOfMemory;
            }
            if (hipError_t e = hipEventRecord(x->rib_ev, s)) return e;
            x->rib_built = true;
            x->rib_stream = s;
        } else if (x->rib_stream != s) {
            if (hipError_t e = hipStreamWaitEvent(s, x->rib_ev, 0)) return e;
        }
    }
    out.l1 = out.rib_l1;
    out.l1_ribbon = 1;
    return hipSuccess;
}

int Classifier::scan(const std::vector<std::array<uint64_t, 3>>& ranges) {
    ScratchHold hold;
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    double t_kern = 0, t_d2h = 0;
    const uint64_t tile = scan_tile_positions();
    const uint64_t seg_max = (1ull << 31) / tile * tile;
    // windows above the LDS-staged layouts: k_scan_g when the index has its level-1
    // filter (single file, built with SYDELTA_SCAN_WIDE != 0), else the per-thread k_scan
    const bool wide_w = n > scan_max_window() && wide_scan(ix);
    const bool wide = n > scan_max_window() && !wide_w;
    std::vector<ScanSeg> segs;
    std::vector<uint32_t> seg_src;
    uint64_t ntiles = 0, tot_pos = 0;
    for (auto& r : ranges) {
        Src& c = src[r[0]];
        const uint64_t lo = std::max(c.p0, r[1] * n), hi = std::min(c.p1, r[2] * n);
        if (c.probed)
            for (uint64_t k = r[1]; k < r[2]; ++k) c.scanned[k - c.kb] = 1;
        if (lo >= hi) continue;
        // tiles load 16-byte granules from the segment start: start on one
        const uint64_t lo16 = wide ? lo : (lo & ~15ull);
        for (uint64_t q = lo16; q < hi; q += seg_max) {
            ScanSeg g{};
            g.src = c.off;
            g.len = c.len;
            g.pos_begin = q;
            g.pos_end = std::min(hi, q + seg_max);
            g.tile_base = (uint32_t)ntiles;
            g.file = c.file;
            ntiles += (g.pos_end - g.pos_begin + tile - 1) / tile;
            tot_pos += g.pos_end - g.pos_begin;
            segs.push_back(g);
            seg_src.push_back((uint32_t)r[0]);
        }
    }
    if (segs.empty()) return SYDELTA_OK;
    if (ntiles >= 0xFFFFFFFFull || segs.size() >= 0x7FFFFFFFull)
        return fail(SYDELTA_E_INVAL, "scan too large (%llu tiles)", (unsigned long long)ntiles);
    if (wide && ix->nfiles != 1) return fail(SYDELTA_E_INVAL, "batched match needs block_size <= %u", scan_max_window());
    unsigned long long* d_counts = nullptr;
    DevBuf cnt_buf;
    HIP_TRY(dev_malloc_async((void**)&d_counts, 128, s));
    cnt_buf.p = d_counts;
    cnt_buf.s = s;
    DevBuf seg_buf;
    if (!wide) {
        HIP_TRY(dev_malloc_async(&seg_buf.p, segs.size() * sizeof(ScanSeg), s));
        seg_buf.s = s;
        // through the thread's pinned staging buffer: a pageable H2D of C4's 68 K segments
        // (2.7 MB) is a staged, host-blocking copy.  The previous call on this thread
        // synchronized its stream, so the buffer is free.
        PinnedHits& seg_pin = thread_seg_pin();
        const size_t sbytes = segs.size() * sizeof(ScanSeg);
        if (sbytes > (64u << 10)) {
            if (int r = pinned_at_least(seg_pin, sbytes)) return r;
            memcpy(seg_pin.p, segs.data(), sbytes);
            HIP_TRY(hipMemcpyAsync(seg_buf.p, seg_pin.p, sbytes, hipMemcpyHostToDevice, s));
        } else {
            HIP_TRY(hipMemcpyAsync(seg_buf.p, segs.data(), sbytes, hipMemcpyHostToDevice, s));
        }
    }
    // verified hits: at most one per position; start from ~4 per block of positions
    DeviceIndex dix;
    HIP_TRY(scan_index(ix, tot_pos, s, prof, dix));
    uint64_t want = std::min<uint64_t>(tot_pos, tot_pos / n * 4 + (1 << 16));
    uint64_t cap = 0;
    unsigned long long counts[16] = {0};
    // The verified-hit buffers (keys [cap] + key scratch [cap] + values [cap] + value
    // scratch [cap]) stay with the calling thread between calls, grown as needed: freeing
    // them after the synchronize below -- ~100 MB at C3 -- blocked the host ~0.6 ms per
    // call (measured, round 3), reusing them costs nothing.  The previous call on this
    // thread synchronized its stream, so a buffer made on another stream is free to
    // take over (or to release in this stream's order).  One buffer per (thread, device):
    // a thread that alternates devices keeps each device's.  Released by sydelta_trim;
    // never freed at thread exit (the HIP runtime may be gone), like the per-thread streams.
    int cur_dev = 0;
    HIP_TRY(hipGetDevice(&cur_dev));
    HitScratch& hits_tl = thread_hit_scratch(cur_dev);
    struct {
        void* p = nullptr;
    } hit_buf;
    for (int attempt = 0; attempt < 2; ++attempt) {
        if (want > cap) {
            cap = want;
            if (hits_tl.bytes < cap * 24) {
                if (hits_tl.p) (void)hipFreeAsync(hits_tl.p, s);
                hits_tl = HitScratch();
                const size_t bytes = cap * 24 + (cap * 24) / 4;  // room to grow by a quarter
                HIP_TRY(dev_malloc_async(&hits_tl.p, bytes, s));
                hits_tl.bytes = bytes;
            }
            hit_buf.p = hits_tl.p;
        }
        uint64_t* d_key = (uint64_t*)hit_buf.p;
        uint32_t* d_val = (uint32_t*)(d_key + 2 * cap);
        HIP_TRY(hipMemsetAsync(d_counts, 0, 128, s));
        if (host_timing) fprintf(stderr, "sydelta scan setup: %.3f ms\n", ms_since(t0));
        if (!wide) {
            HIP_TRY(launch_scan(base, (const ScanSeg*)seg_buf.p, (uint32_t)segs.size(), (uint32_t)ntiles,
                                (uint32_t)n, dix, ix->d_strong, d_key, d_val, cap, d_counts, nullptr, 0,
                                s, prof, &thread_scan_scratch(cur_dev)));
        } else {
            for (size_t g = 0; g < segs.size(); ++g)
                HIP_TRY(launch_scan_wide(base + segs[g].src, segs[g].len, segs[g].pos_begin, segs[g].pos_end,
                                         (uint32_t)g, (uint32_t)n, ix->ix, ix->d_strong, d_key, d_val, cap, d_counts,
                                         s, prof));
        }
        if (host_timing) fprintf(stderr, "sydelta scan launched: %.3f ms\n", ms_since(t0));
        HIP_TRY(hipMemcpyAsync(counts, d_counts, 128, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (host_timing) fprintf(stderr, "sydelta scan synchronized: %.3f ms\n", ms_since(t0));
        if (getenv("SYDELTA_PHASE_TIMING"))
            fprintf(stderr, "sydelta phase cycles (wave 0, summed over workgroups): [k_scan_lds: stage prefix roll flush"
                            " lookup verify] %llu %llu %llu %llu"
                            " %llu %llu l1 passes %llu passes %llu weak %llu positions %llu\n",
                    counts[4], counts[5], counts[6], counts[7], counts[8], counts[9], counts[3], counts[2], counts[1],
                    (unsigned long long)tot_pos);
        if (counts[0] <= cap) break;
        want = counts[0];  // dense hits: grow once and rescan
    }
    const uint64_t nver = counts[0];
    weak_hits += counts[1];
    t_kern = ms_since(t0);
    if (!nver) return SYDELTA_OK;
    uint64_t* d_key = (uint64_t*)hit_buf.p;
    uint32_t* d_val = (uint32_t*)(d_key + 2 * cap);
    uint64_t* k_out = nullptr;
    uint32_t* v_out = nullptr;
    const int end_bit = kSegShift + (int)ceil_log2(segs.size() + 1);
    {
        ProfScope ps(prof, s, "sort_hits");
        HIP_TRY(launch_sort_hits(d_key, d_val, d_key + cap, d_val + cap, nver, end_bit, s, &k_out, &v_out));
    }
    // The sorted hits come back into pinned host memory kept by the calling thread (grown
    // as needed; released by sydelta_trim, and after a call that needed more than
    // kPinnedHitsKeep): fresh pageable vectors cost their page faults plus a staged copy,
    // 2-3 ms for C3b's 1 Mi hits (measured, round 3).
    PinnedHits& ph = thread_pinned_hits();
    if (ph.bytes < nver * 12) {
        if (ph.p) (void)hipHostFree(ph.p);
        ph = PinnedHits();
        const size_t bytes = nver * 12 + (nver * 12) / 4;
        HIP_TRY(hipHostMalloc((void**)&ph.p, bytes, hipHostMallocDefault));
        ph.bytes = bytes;
    }
    const uint64_t* hkey = (const uint64_t*)ph.p;
    const uint32_t* hval = (const uint32_t*)(ph.p + nver * 8);
    HIP_TRY(hipMemcpyAsync(ph.p, k_out, nver * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(ph.p + nver * 8, v_out, nver * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    t_d2h = ms_since(t0);
    // (segment, position)-sorted; segments are in (source, position) order, so each
    // source's hits are one run; runs are merged into their sources on host threads
    auto merge_range = [&](size_t h, size_t hend) {
        HitPos pos;
        HitBlk blk;
        while (h < hend) {
            const uint32_t si = seg_src[hkey[h] >> kSegShift];
            Src& c = src[si];
            size_t e = h;
            while (e < hend && seg_src[hkey[e] >> kSegShift] == si) ++e;
            // a source's first hits go straight into its lists (recycled capacity, see
            // Classifier::~Classifier); later ones are merged
            const bool direct = c.hpos.empty();
            HitPos& P = direct ? c.hpos : pos;
            HitBlk& B = direct ? c.hblk : blk;
            P.clear();
            B.clear();
            P.reserve(e - h);
            B.reserve(e - h);
            for (; h < e; ++h) {
                const uint64_t p = segs[hkey[h] >> kSegShift].pos_begin + (hkey[h] & 0xFFFFFFFFull);
                if (p >= c.p0 && p < c.p1) { P.push_back(p); B.push_back(hval[h]); }
            }
            if (!direct) merge_hits(c, pos, blk);
        }
    };
    const int nthr = nver >= (1u << 16) ? walk_threads() : 1;
    const uint32_t s_first = seg_src[hkey[0] >> kSegShift], s_last = seg_src[hkey[nver - 1] >> kSegShift];
    if (nthr > 1 && s_first == s_last && src[s_first].hpos.empty()) {
        // one source (C3, C3b): its hits are position-sorted, so the ones inside [p0, p1)
        // are one run; its lists are filled in parallel slices (was one thread, 5.8 ms for
        // C3b's 986 K hits, round 3)
        Src& c = src[s_first];
        auto pos_of = [&](size_t h) { return segs[hkey[h] >> kSegShift].pos_begin + (hkey[h] & 0xFFFFFFFFull); };
        auto first_at = [&](uint64_t p) {  // first hit at or after position p
            size_t lo = 0, hi = nver;
            while (lo < hi) {
                const size_t mid = (lo + hi) / 2;
                if (pos_of(mid) < p) lo = mid + 1; else hi = mid;
            }
            return lo;
        };
        const size_t a = first_at(c.p0), b = first_at(c.p1);
        c.hpos.resize(b - a);
        c.hblk.resize(b - a);
        const size_t per = (b - a + nthr - 1) / nthr;
        if (!run_parallel(nthr, [&](int t) {
                const size_t e = std::min(b, a + (size_t)(t + 1) * per);
                for (size_t h = a + (size_t)t * per; h < e; ++h) {
                    c.hpos[h - a] = pos_of(h);
                    c.hblk[h - a] = hval[h];
                }
            }))
            return fail(SYDELTA_E_OOM, "out of host memory (hit lists)");
    } else if (nthr > 1) {
        // split points at source boundaries
        std::vector<size_t> cut{0};
        for (int t = 1; t < nthr; ++t) {
            size_t h = std::max(cut.back(), nver * t / nthr);
            while (h < nver && h > 0 && seg_src[hkey[h] >> kSegShift] == seg_src[hkey[h - 1] >> kSegShift]) ++h;
            cut.push_back(h);
        }
        cut.push_back(nver);
        if (!run_parallel(nthr, [&](int t) { merge_range(cut[t], cut[t + 1]); }))
            return fail(SYDELTA_E_OOM, "out of host memory (hit lists)");
    } else {
        merge_range(0, nver);
    }
    if (ph.bytes > kPinnedHitsKeep) {  // a dense call's buffer is not kept (hipHostFree synchronizes)
        (void)hipHostFree(ph.p);
        ph = PinnedHits();
    }
    if (host_timing)
        fprintf(stderr, "sydelta scan: %zu segments, %llu hits: setup+kernel %.3f ms, sort+D2H %.3f ms, merge %.3f ms\n",
                segs.size(), (unsigned long long)nver, t_kern, t_d2h - t_kern, ms_since(t0) - t_d2h);
    return SYDELTA_OK;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Scan ranges of one source, merged when closer than a scan tile (aligned-hit blocks
// between them are scanned too: cheaper than another tile).
void merge_ranges(std::vector<std::array<uint64_t, 3>>& r, uint64_t gap_blocks) {
    std::vector<std::array<uint64_t, 3>> out;
    for (auto& x : r) {
        if (!out.empty() && out.back()[0] == x[0] && x[1] >= out.back()[2] && x[1] - out.back()[2] < gap_blocks)
            out.back()[2] = std::max(out.back()[2], x[2]);
        else
            out.push_back(x);
    }
    r.swap(out);
}

int Classifier::classify(int mode) {
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    if (int r = probe(mode)) return r;
    const double t_probe = ms_since(t0);
    const uint64_t gap_blocks = std::max<uint64_t>(1, scan_tile_positions() / n);
    // Runs of blocks whose aligned window missed.  A short run is scanned.  A long run
    // (an insertion or deletion shifts everything after it) gets its first block scanned;
    // its first hit there gives the phase phi the walk will continue at, so the run's
    // other blocks are probed at k*n + phi (one window each) and only the blocks whose
    // phase window misses are scanned.  Anything the walk still needs is scanned on
    // demand (Classifier::walk), so the op list does not depend on these guesses.
    constexpr uint64_t kPhaseRun = 8;
    std::vector<std::array<uint64_t, 3>> ranges;
    std::vector<std::array<uint64_t, 3>> runs;  // long runs: source, first, end (local blocks)
    for (size_t i = 0; i < src.size(); ++i) {
        const Src& c = src[i];
        if (!c.nblk) continue;
        if (!c.probed) {
            ranges.push_back({i, c.kb, c.kb + c.nblk});
            continue;
        }
        for (size_t j = miss_off[i]; j < miss_off[i + 1]; ++j) {
            const uint64_t k = miss_runs[j][0], e = miss_runs[j][1];
            if (e - k >= kPhaseRun && phase_probe_on()) {
                ranges.push_back({i, c.kb + k, c.kb + k + 2});
                runs.push_back({i, k, e});
            } else {
                ranges.push_back({i, c.kb + k, c.kb + e});
            }
        }
    }
    merge_ranges(ranges, gap_blocks);
    const auto t1 = std::chrono::steady_clock::now();
    int r = scan(ranges);
    const double t_scan1 = ms_since(t1);
    if (r || runs.empty()) {
        if (host_timing)
            fprintf(stderr, "sydelta classify: probe %.3f ms, ranges %zu (%.3f ms), scan %.3f ms\n", t_probe,
                    ranges.size(), std::chrono::duration<double, std::milli>(t1 - t0).count() - t_probe, t_scan1);
        return r;
    }
    // phase of each long run: the first hit in its first two blocks (the block holding
    // an insertion has no hit; the next one hits at the shifted phase)
    std::vector<std::array<uint64_t, 4>> jobs;
    std::vector<std::array<uint64_t, 3>> rest;
    for (auto& run : runs) {
        const Src& c = src[run[0]];
        const uint64_t k = run[1], e = run[2];
        const uint64_t b0 = (c.kb + k) * n;
        auto it = std::lower_bound(c.hpos.begin(), c.hpos.end(), b0);
        if (it == c.hpos.end() || *it >= b0 + 2 * n) {
            rest.push_back({run[0], c.kb + k + 2, c.kb + e});
            continue;
        }
        const uint64_t phi = (*it - b0) % n;
        // blocks k+2 .. whose phase window starts inside [p0, p1) (k, k+1 are scanned)
        uint64_t last = e;
        while (last > k + 2 && (c.kb + last - 1) * n + phi >= c.p1) --last;
        if (last > k + 2) jobs.push_back({run[0], k + 2, last - (k + 2), phi});
        if (last < e) rest.push_back({run[0], c.kb + std::max(last, k + 2), c.kb + e});
    }
    const auto t2 = std::chrono::steady_clock::now();
    if ((r = phase_probe(jobs, rest))) return r;
    const double t_phase = ms_since(t2);
    std::sort(rest.begin(), rest.end());
    merge_ranges(rest, gap_blocks);
    const auto t3 = std::chrono::steady_clock::now();
    r = scan(rest);
    if (host_timing)
        fprintf(stderr, "sydelta classify: probe %.3f ms, ranges %zu (%.3f ms), scan %.3f ms, phase probe %zu runs "
                "%.3f ms, scan of %zu missed ranges %.3f ms\n", t_probe, ranges.size(),
                std::chrono::duration<double, std::milli>(t1 - t0).count() - t_probe, t_scan1, jobs.size(), t_phase,
                rest.size(), ms_since(t3));
    return r;
}

int Classifier::phase_probe(const std::vector<std::array<uint64_t, 4>>& jobs,
                            std::vector<std::array<uint64_t, 3>>& missed) {
    if (jobs.empty()) return SYDELTA_OK;
    ScratchHold hold;
    std::vector<ProbeJob> pj;
    pj.reserve(jobs.size());
    uint64_t np = 0;
    bool fast = n % 64 == 0 && n >= 256;
    for (auto& j : jobs) {
        const Src& c = src[j[0]];
        pj.push_back({c.off + j[3], c.kb + j[1], np, c.file, 0});
        fast = fast && ((uintptr_t)(base + c.off + j[3]) & 15) == 0;
        np += j[2];
    }
    DevBuf jb;
    const size_t jbytes = (pj.size() * sizeof(ProbeJob) + 255) & ~(size_t)255;
    const size_t obytes = (np * 4 + 255) & ~(size_t)255;
    HIP_TRY(dev_malloc_async(&jb.p, jbytes + 2 * obytes + np * 8, s));
    jb.s = s;
    uint32_t* d_out = (uint32_t*)((uint8_t*)jb.p + jbytes);
    uint32_t* d_pw = (uint32_t*)((uint8_t*)jb.p + jbytes + obytes);
    uint64_t* d_pst = (uint64_t*)((uint8_t*)jb.p + jbytes + 2 * obytes);
    HIP_TRY(hipMemcpyAsync(jb.p, pj.data(), pj.size() * sizeof(ProbeJob), hipMemcpyHostToDevice, s));
    HIP_TRY(launch_probe(base, (const ProbeJob*)jb.p, (uint32_t)pj.size(), np, 1, (uint32_t)n, fast, ix->ix, d_pw,
                         d_pst, d_out, s, prof));
    // results into the thread's pinned buffer (a pageable D2H of C4's ~1.3 M results is a
    // staged copy); the previous call on this thread synchronized its stream
    PinnedHits& pin = thread_phase_pin();
    if (int r = pinned_at_least(pin, np * 4)) return r;
    const uint32_t* out = (const uint32_t*)pin.p;
    HIP_TRY(hipMemcpyAsync(pin.p, d_out, np * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // each source's phase arrays sized once, then the jobs filled on the host pool (jobs of
    // one source cover disjoint blocks), each job's missed blocks in its own list, joined
    // in job order
    std::vector<uint64_t> jofs(jobs.size() + 1, 0);
    for (size_t q = 0; q < jobs.size(); ++q) jofs[q + 1] = jofs[q] + jobs[q][2];
    std::vector<std::vector<std::array<uint64_t, 3>>> jmiss(jobs.size());
    const int nthr = jobs.size() >= 64 ? walk_threads() : 1;
    auto fill = [&](int t) {
        for (size_t q = jobs.size() * t / nthr; q < jobs.size() * (t + 1) / nthr; ++q) {
            const auto& j = jobs[q];
            Src& c = src[j[0]];
            if (q == 0 || jobs[q - 1][0] != j[0]) {  // the source's first job (jobs are grouped by source)
                c.ppos.assign(c.nblk, kUnknownNone);
                c.phit.assign(c.nblk, kNoBlk);
            }
        }
    };
    if (!run_parallel(nthr, fill)) return fail(SYDELTA_E_OOM, "out of host memory (phase probes)");
    auto fill2 = [&](int t) {
        for (size_t q = jobs.size() * t / nthr; q < jobs.size() * (t + 1) / nthr; ++q) {
            const auto& j = jobs[q];
            Src& c = src[j[0]];
            auto& mv = jmiss[q];
            uint64_t w = jofs[q];
            for (uint64_t t2 = 0; t2 < j[2]; ++t2, ++w) {
                const uint64_t k = j[1] + t2;  // local block
                c.ppos[k] = (c.kb + k) * n + j[3];
                c.phit[k] = out[w];
                if (out[w] != kNoBlk) continue;
                if (!mv.empty() && mv.back()[2] == c.kb + k)
                    mv.back()[2] = c.kb + k + 1;
                else
                    mv.push_back({j[0], c.kb + k, c.kb + k + 1});
            }
        }
    };
    if (!run_parallel(nthr, fill2)) return fail(SYDELTA_E_OOM, "out of host memory (phase probes)");
    for (auto& mv : jmiss)
        for (auto& r : mv) {
            if (!missed.empty() && missed.back()[0] == r[0] && missed.back()[2] == r[1])
                missed.back()[2] = r[2];
            else
                missed.push_back(r);
        }
    return SYDELTA_OK;
}

int Classifier::walk(size_t i, uint64_t entry, const BasisInfo& bi, bool final_src, int tail_match, sydelta_delta* d,
                     uint64_t* exit) {
    Src& c = src[i];
    OpVec& ops = d->ops;
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    if (ops.empty() && device_walk_on()) {
        const auto t0 = std::chrono::steady_clock::now();
        const int r = walk_device(i, entry, bi, final_src, tail_match, d, exit);
        if (host_timing && r != 2)
            fprintf(stderr, "sydelta device walk: %.3f ms, %zu ops, rc=%d\n", ms_since(t0), ops.size(), r);
        if (r == 0) {
            g_device_walks.fetch_add(1);
            return SYDELTA_OK;
        }
        if (r != 1 && r != 2) return r;
        if (r == 1) g_device_walk_fallbacks.fetch_add(1);
    }
    if (ops.empty()) {
        const auto t0 = std::chrono::steady_clock::now();
        const int r = walk_parallel(i, entry, bi, final_src, tail_match, d, exit);
        if (host_timing && r != 2)
            fprintf(stderr, "sydelta parallel walk: %.3f ms, %zu ops, rc=%d\n", ms_since(t0), ops.size(), r);
        if (r != 1 && r != 2) return r;  // done (stats counted by the join), or an error
    }
    if (ops.empty() && c.nahit + c.hpos.size() >= 4096) ops = take_ops(2 * (c.nahit + c.hpos.size()));
    for (int round = 0;; ++round) {
        uint64_t need = 0;
        const auto t0 = std::chrono::steady_clock::now();
        const int r = walk_src(c, n, entry, c.p1, bi, final_src, tail_match, ops, exit, &need);
        if (host_timing && src.size() == 1)
            fprintf(stderr, "sydelta walk round %d: %.3f ms, %zu ops, need=%d\n", round,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                    ops.size(), r);
        if (!r) break;
        // the walk jumped into a block only its aligned window was classified for
        const uint64_t k = need / n;
        if (round < 4)
            { if (int r = scan({{i, k, k + 1}})) return r; }
        else
            { if (int r = scan({{i, k, c.kb + c.nblk}})) return r; }
    }
    finish_stats_impl(d);
    return SYDELTA_OK;
}

int walk_threads() {
    const char* e = getenv("SYDELTA_WALK_THREADS");
    if (e && *e) return std::max(1, atoi(e));
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::min(8u, std::max(1u, hw));
}

uint64_t walk_par_min() {
    const char* e = getenv("SYDELTA_WALK_PAR_MIN");  // hits below which the walk stays serial
    return (e && *e) ? strtoull(e, nullptr, 10) : (1ull << 16);
}

int Classifier::walk_parallel(size_t i, uint64_t entry, const BasisInfo& bi, bool final_src, int tail_match,
                              sydelta_delta* d, uint64_t* exit) {
    const Src& c = src[i];
    const uint64_t nh = c.nahit + c.hpos.size();
    const int T0 = walk_threads();
    if (T0 < 2 || nh < walk_par_min() || c.p1 <= entry || (c.p1 - entry) / n < 2 * (uint64_t)T0) return 2;
    const std::vector<uint64_t> st = walk::split_points(c, n, entry, T0);
    struct Pool {
        OpVec take(size_t want) { return take_ops(want); }
        void give(OpVec&& v) { give_ops(std::move(v)); }
    } pool;
    const auto t0 = std::chrono::steady_clock::now();
    walk::SplitTiming tm;
    walk::OpCounts oc;
    const int r = walk::walk_split(c, n, st, bi, final_src, tail_match, d->ops, exit, pool,
                                   [&] { return ms_since(t0); }, &tm, &oc);
    if (r < 0) return fail(SYDELTA_E_OOM, "out of host memory (op lists)");
    if (r == 0) {
        d->stats.copy_ops = oc.copy_ops;
        d->stats.data_ops = oc.data_ops;
        d->stats.literal_bytes = oc.literal_bytes;
    }
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    if (host_timing && r == 0)
        fprintf(stderr,
                "sydelta parallel walk: %d segments, walk %.3f ms (segment max %.3f min %.3f), chain %.3f ms, "
                "join %.3f ms\n",
                (int)st.size() - 1, tm.walk_ms, tm.seg_max_ms, tm.seg_min_ms, tm.chain_ms, tm.join_ms);
    return r;
}

// SYDELTA_DEVICE_WALK=1: resolve walks of sources with at least SYDELTA_DEVICE_WALK_MIN
// hits (default 4096) on the device.  Off by default until measured on hardware.
bool device_walk_on() {
    const char* e = getenv("SYDELTA_DEVICE_WALK");  // read per walk, like the other knobs
    const bool on = e && e[0] == '1';
    if (on) install_op_arena();
    return on;
}
uint64_t device_walk_min() {
    const char* e = getenv("SYDELTA_DEVICE_WALK_MIN");
    return (e && *e) ? strtoull(e, nullptr, 10) : 4096;
}

int Classifier::walk_device(size_t i, uint64_t entry, const BasisInfo& bi, bool final_src, int tail_match,
                            sydelta_delta* d, uint64_t* exit) {
    const Src& c = src[i];
    if (!c.ppos.empty() || entry >= c.p1 || entry < c.p0) return 2;  // phase probes: host walk
    if (c.probed && (!d_probe_out || probe_pfx.size() <= i)) return 2;
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    // scan hits, minus those at an aligned position whose aligned window hit (the same
    // hit twice: the merge needs two disjoint lists)
    const uint64_t* hp = c.hpos.data();
    const uint32_t* hb = c.hblk.data();
    std::vector<uint64_t> fp;
    std::vector<uint32_t> fb;
    if (c.probed && !c.hpos.empty()) {
        bool dup = false;
        for (uint64_t p : c.hpos)
            if (p % n == 0 && c.ahit[p / n - c.kb] != kNoBlk) { dup = true; break; }
        if (dup) {
            fp.reserve(c.hpos.size());
            fb.reserve(c.hpos.size());
            for (size_t h = 0; h < c.hpos.size(); ++h) {
                const uint64_t p = c.hpos[h];
                if (p % n == 0 && c.ahit[p / n - c.kb] != kNoBlk) continue;
                fp.push_back(p);
                fb.push_back(c.hblk[h]);
            }
            hp = fp.data();
            hb = fb.data();
        }
    }
    const uint64_t H = hp == c.hpos.data() ? c.hpos.size() : fp.size();
    const uint64_t M = (c.probed ? c.nahit : 0) + H;
    if (M < device_walk_min() || M > (1ull << 25)) return 2;
    const uint32_t K = chain::chain_levels(M);
    const uint64_t W = M + 2, nblk = c.probed ? c.nblk : 0;
    // one allocation: known | aflag | apfx | hpos | hblk | upos | ublk | jump | on | cnt | off | ops | res
    auto al = [](uint64_t b) { return (b + 255) & ~(uint64_t)255; };
    const uint64_t o_known = 0, o_aflag = o_known + al(nblk), o_apfx = o_aflag + al(4 * (nblk + 1));
    const uint64_t o_hpos = o_apfx + al(4 * (nblk + 1)), o_hblk = o_hpos + al(8 * H), o_upos = o_hblk + al(4 * H);
    const uint64_t o_ublk = o_upos + al(8 * M), o_jump = o_ublk + al(4 * M), o_on = o_jump + al(4 * W * K);
    const uint64_t o_cnt = o_on + al(W), o_off = o_cnt + al(4 * (M + 1)), o_ops = o_off + al(4 * (M + 1));
    const uint64_t o_res = o_ops + al(sizeof(sydelta_op) * 2 * M), total = o_res + al(sizeof(chain::ChainResult));
    DevBuf buf;
    HIP_TRY(dev_malloc_async(&buf.p, total, s));
    buf.s = s;
    uint8_t* B = (uint8_t*)buf.p;
    chain::ChainArgs a{};
    a.n = n;
    a.p1 = c.p1;
    a.kb = c.kb;
    a.nblk = nblk;
    a.entry = entry;
    a.probed = c.probed ? 1u : 0u;
    a.K = K;
    a.ahit = c.probed ? d_probe_out + probe_pfx[i] : nullptr;
    a.known = B + o_known;
    a.aflag = (uint32_t*)(B + o_aflag);
    a.apfx = (uint32_t*)(B + o_apfx);
    a.hpos = (const uint64_t*)(B + o_hpos);
    a.hblk = (const uint32_t*)(B + o_hblk);
    a.H = H;
    a.M = M;
    a.upos = (uint64_t*)(B + o_upos);
    a.ublk = (uint32_t*)(B + o_ublk);
    a.jump = (uint32_t*)(B + o_jump);
    a.on = B + o_on;
    a.cnt = (uint32_t*)(B + o_cnt);
    a.off = (uint32_t*)(B + o_off);
    a.blk_base = bi.blk_base;
    a.nblocks = bi.nblocks;
    a.last_size = bi.last_size;
    a.ops = (sydelta_op*)(B + o_ops);
    a.res = (chain::ChainResult*)(B + o_res);
    if (c.probed && nblk)  // per block: all its window starts were scanned
        HIP_TRY(hipMemcpyAsync(B + o_known, c.scanned.data(), nblk, hipMemcpyHostToDevice, s));
    if (H) {
        HIP_TRY(hipMemcpyAsync(B + o_hpos, hp, 8 * H, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(B + o_hblk, hb, 4 * H, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(launch_chain(a, s, prof));
    chain::ChainResult res{};
    HIP_TRY(hipMemcpyAsync(&res, a.res, sizeof(res), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const double t_kern = ms_since(t0);
    if (res.unk) return 1;
    if (res.bad || res.nops > 2 * M || (res.first < M) != (res.last < M)) {
        // cannot happen with consistent inputs; the host walk gives the right answer anyway
        if (host_timing) fprintf(stderr, "sydelta device walk: inconsistent result, host walk\n");
        return 1;
    }
    // [entry, first hit) | the device's ops | the end of the walk (walk::finish_walk)
    OpVec& ops = d->ops;
    const bool lead = res.first < M && res.first_pos > entry;
    if (ops.capacity() < (lead ? 1 : 0) + res.nops + 3) ops = take_ops((lead ? 1 : 0) + res.nops + 3);
    ops.resize((lead ? 1 : 0) + res.nops);
    if (lead) ops[0] = sydelta_op{SYDELTA_OP_DATA, 0, entry, res.first_pos - entry};
    if (res.nops)
        HIP_TRY(hipMemcpyAsync(ops.data() + (lead ? 1 : 0), a.ops, sizeof(sydelta_op) * res.nops,
                               hipMemcpyDeviceToHost, s));
    const uint64_t x = res.first < M ? res.last_pos + n : c.p1;  // no hit: the walk runs to the end
    const uint64_t lit = res.first < M ? x : entry;
    const size_t before_end = ops.size();
    walk::finish_walk(c, n, lit, x, c.p1, bi, final_src, tail_match, ops, exit);
    HIP_TRY(hipStreamSynchronize(s));
    // stats: the device counted its Data ops and bytes
    uint64_t nd = res.data_ops + (lead ? 1 : 0), lb = res.lit_bytes + (lead ? res.first_pos - entry : 0);
    for (size_t k = before_end; k < ops.size(); ++k)
        if (ops[k].kind == SYDELTA_OP_DATA) { ++nd; lb += ops[k].b; }
    d->stats.copy_ops = ops.size() - nd;
    d->stats.data_ops = nd;
    d->stats.literal_bytes = lb;
    if (host_timing)
        fprintf(stderr, "sydelta device walk: %llu hits (%llu aligned), %u levels: kernels %.3f ms, ops to host %.3f ms\n",
                (unsigned long long)M, (unsigned long long)(M - H), K, t_kern, ms_since(t0) - t_kern);
    return 0;
}

void finish_stats_impl(sydelta_delta* d) {
    // one pass over the op array (24 MiB at 1 Mi ops): split over the host pool when large
    const size_t no = d->ops.size();
    const int T = no >= (1u << 18) ? walk_threads() : 1;
    struct Part {
        uint64_t data = 0, lit = 0;
        char pad[48];  // one cache line per part
    };
    std::vector<Part> part(T);
    auto count = [&](int t) {
        const sydelta_op* o = d->ops.data();
        uint64_t nd = 0, lit = 0;
        for (size_t i = no * t / T, e = no * (t + 1) / T; i < e; ++i) {
            const bool data = o[i].kind != SYDELTA_OP_COPY;
            nd += data;
            lit += data ? o[i].b : 0;
        }
        part[t].data = nd;
        part[t].lit = lit;
    };
    if (!run_parallel(T, count)) {  // the pool could not take the batch: count here
        part.assign(T, Part{});
        for (int t = 0; t < T; ++t) count(t);
    }
    d->stats.data_ops = d->stats.literal_bytes = 0;
    for (auto& p : part) {
        d->stats.data_ops += p.data;
        d->stats.literal_bytes += p.lit;
    }
    d->stats.copy_ops = no - d->stats.data_ops;
}

// Tail-rule flags (generator.rs:156-184) of the given sources of c (file f's last
// basis block shorter than n, source at least that long).
int tail_flags(Classifier& C, const std::vector<size_t>& which, std::vector<int>& flag) {
    sydelta_index* ix = C.ix;
    std::vector<TailJob> tails;
    std::vector<size_t> tail_of;
    flag.assign(C.src.size(), 0);
    for (size_t i : which) {
        const Src& c = C.src[i];
        const uint64_t f = c.file;
        const uint64_t nb = ix->fblk[f + 1] - ix->fblk[f], ls = ix->last_size[f];
        if (nb && ls < C.n && c.flen >= ls && c.len >= c.flen) {
            tails.push_back({c.off + c.flen - ls, ls, ix->fblk[f + 1] - 1});
            tail_of.push_back(i);
        }
    }
    if (tails.empty()) return SYDELTA_OK;
    std::vector<int> tf(tails.size(), 0);
    DevBuf tail_buf;
    const size_t bytes = (tails.size() * sizeof(TailJob) + 15) & ~(size_t)15;
    HIP_TRY(dev_malloc_async(&tail_buf.p, bytes + tails.size() * sizeof(int), C.s));
    tail_buf.s = C.s;
    int* d_flag = (int*)((uint8_t*)tail_buf.p + bytes);
    HIP_TRY(hipMemcpyAsync(tail_buf.p, tails.data(), tails.size() * sizeof(TailJob), hipMemcpyHostToDevice, C.s));
    HIP_TRY(launch_tail(C.base, (const TailJob*)tail_buf.p, (uint32_t)tails.size(), ix->d_weak, ix->d_strong, d_flag,
                        C.s));
    HIP_TRY(hipMemcpyAsync(tf.data(), d_flag, tails.size() * sizeof(int), hipMemcpyDeviceToHost, C.s));
    HIP_TRY(hipStreamSynchronize(C.s));
    for (size_t j = 0; j < tails.size(); ++j) flag[tail_of[j]] = tf[j];
    return SYDELTA_OK;
}
}  // namespace

void sydelta::finish_stats(sydelta_delta* d) { finish_stats_impl(d); }

// K10 (k_walk_files): the whole walk of every file on the device, for batches of small
// files (SYDELTA_FILE_WALK=0 turns it off; =1 takes it for any batch it can serve).
namespace {
int file_walk_mode() {
    const char* e = getenv("SYDELTA_FILE_WALK");
    return (e && e[0] == '0') ? 0 : (e && e[0] == '1') ? 1 : -1;
}
bool file_walk_ok(const sydelta_index* ix, const uint64_t* src_off, const uint64_t* src_len, const uint8_t* d_buf) {
    const int mode = file_walk_mode();
    if (mode == 0) return false;
    const uint64_t n = ix->bs, nf = ix->nfiles;
    if (ix->ix.l1 || n % 64 != 0 || n < 256 || n > kWalkMaxN || ix->max_nblk > kSelfIxMaxBlocks || nf >= (1u << 31))
        return false;
    // one workgroup walks a file: many files, none large (auto mode)
    if (mode < 0 && nf < 64) return false;
    uint64_t recs = 0;
    for (uint64_t f = 0; f < nf; ++f) {
        if (src_len[f] >= (1ull << 32) || (mode < 0 && src_len[f] > (64ull << 20))) return false;
        if (src_len[f] && (!d_buf || ((uintptr_t)(d_buf + src_off[f]) & 15) != 0)) return false;
        recs += 2 * (src_len[f] / n) + 4;
    }
    return recs < (1ull << 32);
}
}  // namespace

// One launch of K10 over `units`: the unit table up, the per-unit results and the
// run-length coded records down (two D2H: the counts, then the records).  The records stay
// in the calling thread's pinned buffer (res.rec) until its next use.
struct WalkResult {
    std::vector<WalkFileOut> out;  // per unit
    const WalkRec* rec = nullptr;  // compact records: unit u's at rec[out[u].base, + out[u].count)
    uint64_t nrec = 0;
    const ExpandOut* xres = nullptr;  // with an ExpandReq: per file (the thread's mapped buffer)
    double ms_kernel = 0, ms_d2h = 0;
};
// The op lists expanded on the device by the walk (WalkArgs::x): file f's units
// [fu[f], fu[f + 1]), its ops at ops + op_off[f] (host-mapped, capacity to op_off[f + 1]).
struct ExpandReq {
    const uint32_t* fu;
    const uint64_t* op_off;
    sydelta_op* ops;
};
// Groups of a batch walked by separate launches (sydelta_delta_pairs_device): group g's units
// [ub[g], ub[g + 1]) start once ev[g] (its files' signature) has passed, odd groups on s2, so a
// group's walk runs beside the next group's signature.
struct WalkGroups {
    std::vector<uint64_t> ub;
    std::vector<hipEvent_t> ev;
    hipStream_t s2 = nullptr;
};
static int run_walk(sydelta_index* ix, const uint8_t* base, const std::vector<WalkUnit>& units, const uint32_t* ahit,
                    const uint32_t* apw, bool lds_filter, hipStream_t s, Profiler* prof, WalkResult& res,
                    const ExpandReq* ex = nullptr, const WalkGroups* groups = nullptr) {
    ScratchHold hold;
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t nu = units.size(), nf = ix->nfiles;
    res.out.clear();
    res.rec = nullptr;
    res.nrec = 0;
    res.xres = nullptr;
    if (!nu) return SYDELTA_OK;
    int cur_dev = 0;
    HIP_TRY(hipGetDevice(&cur_dev));
    uint64_t rec_total = 0;
    for (const WalkUnit& u : units) rec_total = std::max(rec_total, u.rec_off + 2 * ((u.end - u.entry) / ix->bs) + 4);
    // pinned: the unit table and the last sizes up; the counts down (over them, once uploaded)
    const size_t ubytes = sizeof(WalkUnit) * nu, lbytes = 8 * nf, fout_bytes = sizeof(WalkFileOut) * nu;
    // one upload: the unit table, the last sizes and the zeroed record counter (+ the 16
    // SYDELTA_PHASE_TIMING tick counters) -- ten concurrent callers' extra copies showed
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t o_units = 0, o_last = ubytes, o_total = o_last + lbytes, o_fu = al(o_total + 136);
    const size_t o_opoff = o_fu + al(4 * (nf + 1)), o_xdone = o_opoff + al(8 * (nf + 1));
    const size_t up = ex ? o_xdone + 4 * nf : o_total + 136;
    PinnedHits& ph = thread_pinned_hits();
    if (int r = pinned_at_least(ph, std::max(up, fout_bytes + 16))) return r;
    memcpy(ph.p, units.data(), ubytes);
    memcpy(ph.p + o_last, ix->last_size.data(), lbytes);
    memset(ph.p + o_total, 0, 136);
    if (ex) {
        memcpy(ph.p + o_fu, ex->fu, 4 * (nf + 1));
        memcpy(ph.p + o_opoff, ex->op_off, 8 * (nf + 1));
        memset(ph.p + o_xdone, 0, 4 * nf);  // the per-file unit counters
    }
    // device: the upload, the staged records (+ the per-unit results' device copy for the
    // expansion); host (coherent, mapped; the thread's, kept): the per-unit results and the
    // compacted records, which the kernel writes there directly -- one stream synchronisation,
    // no D2H round trips (+ the expansion's per-file results)
    const size_t o_stage = al(up), o_fdev = o_stage + al(sizeof(WalkRec) * rec_total);
    const size_t need = o_fdev + (ex ? al(fout_bytes) : 0);
    const size_t m_rec = al(fout_bytes), m_res = al(m_rec + sizeof(WalkRec) * rec_total);
    const size_t m_need = m_res + (ex ? sizeof(ExpandOut) * nf : 0);
    PinnedHits& wm = thread_walk_map();
    if (wm.bytes < m_need) {
        if (wm.p) {
            HIP_TRY(hipStreamSynchronize(s));  // (the previous call on this thread synchronized its walk)
            (void)hipHostFree(wm.p);
        }
        wm = PinnedHits();
        const size_t want = m_need + m_need / 4;
        HIP_TRY(hipHostMalloc((void**)&wm.p, want, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent));
        wm.bytes = want;
    }
    DevScratch& sc = thread_walk_scratch(cur_dev);
    if (sc.bytes < need) {
        if (sc.p) (void)hipFreeAsync(sc.p, s);
        sc = DevScratch();
        HIP_TRY(dev_malloc_async(&sc.p, need + need / 4, s));
        sc.bytes = need + need / 4;
    }
    uint8_t* D = (uint8_t*)sc.p;
    HIP_TRY(hipMemcpyAsync(D, ph.p, up, hipMemcpyHostToDevice, s));
    static const bool timing = getenv("SYDELTA_PHASE_TIMING") != nullptr;
    WalkArgs a{};
    a.base = base;
    a.units = (const WalkUnit*)(D + o_units);
    a.last_size = (const uint64_t*)(D + o_last);
    a.nunits = (uint32_t)nu;
    a.n = (uint32_t)ix->bs;
    a.nm = (uint32_t)(ix->bs % 65521);
    a.self_nb = lds_filter ? (uint32_t)std::max<uint64_t>(1, ix->max_nblk) : 0u;
    a.files = ix->ix.d_files;
    a.fblk = ix->ix.d_fblk;
    a.filt = ix->ix.filt;
    a.keys = ix->ix.keys;
    a.start = ix->ix.start;
    a.cnt = ix->ix.cnt;
    a.order = ix->ix.order;
    a.cstrong = ix->ix.cstrong;
    a.weak = ix->d_weak;
    a.strong = ix->d_strong;
    a.ahit = ahit;
    a.apw = apw;
    a.stage = (WalkRec*)(D + o_stage);
    a.out = (WalkRec*)(wm.p + m_rec);
    a.fout = (WalkFileOut*)wm.p;
    a.total = (unsigned long long*)(D + o_total);
    a.ticks = timing ? a.total + 1 : nullptr;
    a.fout_dev = ex ? (WalkFileOut*)(D + o_fdev) : nullptr;
    if (ex) {  // the op lists expanded by each file's last unit (k_walk_files, expand_file)
        ExpandArgs& xa = a.x;
        xa.units = a.units;
        xa.fout = a.fout_dev;
        xa.stage = a.stage;
        xa.fu = (const uint32_t*)(D + o_fu);
        xa.fblk = ix->ix.d_fblk;
        xa.last_size = a.last_size;
        xa.op_off = (const uint64_t*)(D + o_opoff);
        xa.ops = ex->ops;
        xa.res = (ExpandOut*)(wm.p + m_res);
        xa.nf = (uint32_t)nf;
        xa.n = (uint32_t)ix->bs;
        a.xdone = (uint32_t*)(D + o_xdone);
        res.xres = xa.res;
    }
    if (groups && groups->ub.size() > 2) {
        hipEvent_t up = take_event(cur_dev), back = take_event(cur_dev);
        if (!up || !back) return fail(SYDELTA_E_OOM, "no event for the grouped walk");
        HIP_TRY(hipEventRecord(up, s));  // the upload, before the other stream's launches
        for (size_t g = 0; g + 1 < groups->ub.size(); ++g) {
            const hipStream_t sg = (g & 1) ? groups->s2 : s;
            if (sg != s) HIP_TRY(hipStreamWaitEvent(sg, up, 0));
            HIP_TRY(hipStreamWaitEvent(sg, groups->ev[g], 0));
            WalkArgs ag = a;  // (a.x stays global: the expansion indexes units and files globally)
            ag.units = a.units + groups->ub[g];
            ag.nunits = (uint32_t)(groups->ub[g + 1] - groups->ub[g]);
            ag.fout = a.fout + groups->ub[g];
            ag.fout_dev = a.fout_dev ? a.fout_dev + groups->ub[g] : nullptr;
            HIP_TRY(launch_walk_files(ag, sg, prof));
        }
        HIP_TRY(hipEventRecord(back, groups->s2));
        HIP_TRY(hipStreamWaitEvent(s, back, 0));
        HIP_TRY(hipStreamSynchronize(s));
        give_event(cur_dev, up);
        give_event(cur_dev, back);
    } else {
        HIP_TRY(launch_walk_files(a, s, prof));
    }
    if (timing) {
        unsigned long long tk[16];
        HIP_TRY(hipMemcpyAsync(tk, a.ticks, sizeof tk, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        fprintf(stderr, "sydelta file walk phases (wave ticks, 100 MHz, summed over units): setup %llu hash %llu "
                "lookup %llu stage %llu roll %llu verify %llu out %llu | passes %llu windows %llu rolls %llu "
                "verify batches %llu\n", tk[0], tk[1], tk[2], tk[3], tk[4], tk[5], tk[6], tk[8], tk[9], tk[10], tk[11]);
    }
    HIP_TRY(hipStreamSynchronize(s));
    res.ms_kernel = ms_since(t0);
    res.out.assign((const WalkFileOut*)wm.p, (const WalkFileOut*)wm.p + nu);
    uint64_t nrec = 0;
    for (const WalkFileOut& o : res.out) {
        if ((uint64_t)o.base + o.count > rec_total)
            return fail(SYDELTA_E_KERNEL, "walk: records [%u, +%u) past the capacity %llu", o.base, o.count,
                        (unsigned long long)rec_total);
        nrec += o.count;
    }
    res.rec = (const WalkRec*)(wm.p + m_rec);
    res.nrec = nrec;
    res.ms_d2h = ms_since(t0) - res.ms_kernel;
    return SYDELTA_OK;
}

// The ops of records [r0, r1) into w (Copy sizes from the basis file's blocks); returns the
// data ops and literal bytes written.
// kStream: non-temporal stores, for a large op array written once and read later (a chunk's:
// C5's 24 MiB per call); they skip each destination line's read-for-ownership.  The caller
// fences (_mm_sfence) before another thread reads the array.
template <bool kStream>
static inline void put_op(sydelta_op* w, uint32_t kind, uint64_t a, uint64_t b) {
    static_assert(sizeof(sydelta_op) == 24, "sydelta_op layout");
    if (kStream) {
        long long* q = (long long*)w;
        _mm_stream_si64(q, (long long)kind);
        _mm_stream_si64(q + 1, (long long)a);
        _mm_stream_si64(q + 2, (long long)b);
    } else {
        *w = {kind, 0, a, b};
    }
}
template <bool kStream = false>
static inline void expand_records(const WalkRec* r0, const WalkRec* r1, uint64_t n, uint64_t bb, uint64_t nbf,
                                  uint64_t ls, sydelta_op* w, uint64_t* nd, uint64_t* lb) {
    for (const WalkRec* r = r0; r < r1; ++r) {
        if (!r->kind) {
            put_op<kStream>(w++, SYDELTA_OP_DATA, r->off, r->a);
            ++*nd;
            *lb += r->a;
            continue;
        }
        for (uint64_t g = r->a - bb, e = g + r->kind; g < e; ++g)
            put_op<kStream>(w++, SYDELTA_OP_COPY, g * n, g + 1 == nbf ? ls : n);
    }
}
static inline uint64_t records_ops(const WalkRec* r0, const WalkRec* r1) {
    uint64_t k = 0;
    for (const WalkRec* r = r0; r < r1; ++r) k += r->kind ? r->kind : 1;
    return k;
}

// The batched match with the walk on the device: one unit per file.
// Segments per file of a batched device walk (SYDELTA_FILE_SEGS=G forces G): a wave walks
// its unit serially, so a batch of fewer files than the chip holds at once (4096 waves at
// four per SIMD) is cut into as many segments as keep every unit in that one round (at
// least 32 blocks each; 8 when forced).  Measured at 1250 files (`profiles/r05zz7_*`): three
// segments per file walk in 0.55 ms, four (5000 units, a second round) in 0.65.  nf counts
// the files of every batch walking at the time (concurrent callers share the chip).
std::atomic<uint64_t> g_walking_files{0};
static uint64_t file_segs(uint64_t nf, int device) {
    const char* e = getenv("SYDELTA_FILE_SEGS");  // read per call (tests switch it)
    if (e && *e) return std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    return std::max<uint64_t>(1, std::min<uint64_t>(64, wave_slots(device) / std::max<uint64_t>(nf, 1)));
}

// The batched match with the walk on the device: one unit per file, or per segment of a
// file (file_segs).  A segment is walked from its start; where the previous segment's walk
// left it later (a Copy crossing the boundary), the segment's walk still holds when its
// leading literal run reaches that exit -- the greedy walk from the exit then classifies the
// same positions the same way -- and its leading Data op is cut to start there; otherwise
// the segment is walked again from the exit (rounds, as for a chunk's segments).
// split/ev/s2: the pairs entry point's groups (files [split[g], split[g + 1]) after event ev[g])
static int match_walk_files(sydelta_index* ix, const uint8_t* d_buf, const uint64_t* src_off, const uint64_t* src_len,
                            hipStream_t s, Profiler* prof, sydelta_delta_batch* b,
                            const std::vector<uint64_t>* split = nullptr, const std::vector<hipEvent_t>* gev = nullptr,
                            hipStream_t s2 = nullptr) {
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const uint64_t n = ix->bs, nf = ix->nfiles;
    struct Walking {  // this batch's files counted while it walks
        uint64_t k, total;
        explicit Walking(uint64_t k_) : k(k_), total(g_walking_files.fetch_add(k_) + k_) {}
        ~Walking() { g_walking_files.fetch_sub(k); }
    } walking(nf);
    // callers come and go between their signature, index and match calls: the peak of the
    // last second stands for them (a heuristic; races only shift the segment count)
    static std::atomic<uint64_t> peak{0};
    static std::atomic<int64_t> peak_ms{0};
    const int64_t now_ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                               std::chrono::steady_clock::now().time_since_epoch()).count();
    if (walking.total >= peak.load() || now_ms - peak_ms.load() > 1000) {
        peak.store(walking.total);
        peak_ms.store(now_ms);
    }
    const uint64_t G = file_segs(std::max(walking.total, peak.load()), ix->device), min_seg = (getenv("SYDELTA_FILE_SEGS") && *getenv("SYDELTA_FILE_SEGS")) ? 8 : 32;
    std::vector<WalkUnit> units;
    units.reserve(nf * G);
    std::vector<uint64_t> fu(nf + 1, 0);  // file f's units: [fu[f], fu[f+1])
    uint64_t rec_off = 0;
    for (uint64_t f = 0; f < nf; ++f) {
        fu[f] = units.size();
        const uint64_t len = src_len[f], nbf = ix->fblk[f + 1] - ix->fblk[f];
        const uint64_t p1 = (nbf && len >= n) ? len - n + 1 : 0;  // an empty signature matches nothing (generator.rs:121)
        const uint64_t nb = (p1 + n - 1) / n;
        const uint64_t segb = G > 1 ? std::max<uint64_t>(min_seg, (nb + G - 1) / G) : std::max<uint64_t>(nb, 1);
        uint64_t e0 = 0;
        do {
            const uint64_t e1 = std::min(p1, e0 + segb * n);
            units.push_back(WalkUnit{src_off[f], len, e0, e1, p1, rec_off, 0, (uint32_t)f, (uint32_t)(e1 >= p1)});
            rec_off += 2 * ((e1 - e0) / n) + 4;
            e0 = e1;
        } while (e0 < p1);
    }
    fu[nf] = units.size();
    const uint64_t nu = units.size();
    // the op lists: expanded on the device into op arrays reserved from a pinned host-mapped
    // slab (each file's last unit of the walk kernel) when the host has few threads for them (SYDELTA_DEVICE_EXPAND=0|1
    // forces it off / on; per call), else on the host below
    const int asm_threads = asm_threads_env();
    const char* dxe = getenv("SYDELTA_DEVICE_EXPAND");
    const bool dexp = (dxe && *dxe) ? dxe[0] == '1' : asm_threads <= 4;
    std::vector<uint64_t> op_off;
    std::vector<uint32_t> fu32;
    ExpandReq req{};
    bool expand_dev = false;
    if (dexp) {
        op_off.assign(nf + 1, 0);
        fu32.resize(nf + 1);
        for (uint64_t f = 0; f < nf; ++f) {
            uint64_t cap = 0;  // ops per unit: a Copy per block, a Data op before each, the tail's two
            for (uint64_t u = fu[f]; u < fu[f + 1]; ++u) cap += 2 * ((units[u].end - units[u].entry) / n) + 8;
            op_off[f + 1] = op_off[f] + cap;
            fu32[f] = (uint32_t)fu[f];
        }
        fu32[nf] = (uint32_t)fu[nf];
        if (OpSlab* slab = slab_open(op_off[nf] * sizeof(sydelta_op))) {
            expand_dev = true;
            for (uint64_t f = 0; f < nf; ++f) {
                OpVec v;
                v.reserve(op_off[f + 1] - op_off[f]);  // (from the slab, in file order)
                expand_dev = expand_dev && (uint8_t*)v.data() == slab->p + op_off[f] * sizeof(sydelta_op);
                b->d[f].ops.swap(v);
            }
            req = ExpandReq{fu32.data(), op_off.data(), (sydelta_op*)slab->p};
            slab_close(slab);
        }
    }
    if (!expand_dev) take_small_ops(b->d);  // recycled per-file op arrays
    WalkGroups groups;
    if (split) {
        for (uint64_t f : *split) groups.ub.push_back(fu[f]);
        groups.ev = *gev;
        groups.s2 = s2;
    }
    WalkResult res;
    if (int r = run_walk(ix, d_buf, units, nullptr, nullptr, true, s, prof, res, expand_dev ? &req : nullptr,
                         split ? &groups : nullptr))
        return r;
    const auto t1 = std::chrono::steady_clock::now();
    if (res.xres) {  // every file expanded on the device (a file that needs a re-walk: the host path below)
        bool all = true;
        for (uint64_t f = 0; f < nf && all; ++f) all = !res.xres[f].bad;
        (all ? g_expand_files : g_expand_host) += all ? nf : 1;
        if (all) {
            for (uint64_t f = 0; f < nf; ++f) {
                const ExpandOut& x = res.xres[f];
                sydelta_delta& d = b->d[f];
                d.ops.resize(x.nops);  // (written by the device; no initialisation)
                d.stats.copy_ops = x.nops - x.data_ops;
                d.stats.data_ops = x.data_ops;
                d.stats.literal_bytes = x.lit;
                d.stats.weak_hits = x.weak_hits;
                d.stats.verified_hits = x.hits;
                b->total.copy_ops += d.stats.copy_ops;
                b->total.data_ops += x.data_ops;
                b->total.literal_bytes += x.lit;
                b->total.weak_hits += x.weak_hits;
                b->total.verified_hits += x.hits;
            }
            if (host_timing)
                fprintf(stderr, "sydelta file walk: %llu files in %llu units, ops expanded on the device: kernels %.3f ms, "
                        "results %.3f ms\n", (unsigned long long)nf, (unsigned long long)nu, res.ms_kernel, ms_since(t1));
            return SYDELTA_OK;
        }
    }
    std::vector<WalkFileOut>& out = res.out;
    std::vector<std::pair<const WalkRec*, const WalkRec*>> span(nu);
    for (uint64_t u = 0; u < nu; ++u) span[u] = {res.rec + out[u].base, res.rec + out[u].base + out[u].count};
    // chain the segments of each file
    constexpr uint64_t kNoTrim = UINT64_MAX;
    std::vector<uint64_t> tstart;  // a segment's leading Data op cut to start here
    std::vector<std::vector<WalkRec>> kept;  // records that outlive the pinned buffer
    int rounds = 0;
    if (nu > nf) {
        tstart.assign(nu, kNoTrim);
        for (;;) {
            std::vector<uint64_t> bad;
            for (uint64_t f = 0; f < nf; ++f)
                for (uint64_t u = fu[f] + 1; u < fu[f + 1]; ++u) {
                    const uint64_t pe = out[u - 1].exit;
                    tstart[u] = kNoTrim;
                    if (units[u].entry == pe) continue;
                    const WalkRec* r0 = span[u].first;
                    const uint64_t h = (r0 < span[u].second && !r0->kind) ? r0->off + r0->a : units[u].entry;
                    if (pe > units[u].entry && h >= pe)
                        tstart[u] = pe;  // the walk from pe meets this one at once
                    else
                        bad.push_back(u);
                }
            if (bad.empty()) break;
            ++rounds;
            if (kept.empty()) {  // the next launch reuses the pinned buffer: keep the records
                kept.emplace_back(res.rec, res.rec + res.nrec);
                const WalkRec* base = kept.back().data();
                for (uint64_t u = 0; u < nu; ++u)
                    span[u] = {base + (span[u].first - res.rec), base + (span[u].second - res.rec)};
            }
            std::vector<WalkUnit> again;
            uint64_t roff = 0;
            for (uint64_t u : bad) {
                units[u].entry = out[u - 1].exit;
                units[u].end = std::max(units[u].end, units[u].entry);
                WalkUnit w = units[u];
                w.rec_off = roff;
                roff += 2 * ((w.end - w.entry) / n) + 4;
                again.push_back(w);
            }
            WalkResult r1;
            if (int r = run_walk(ix, d_buf, again, nullptr, nullptr, true, s, prof, r1)) return r;
            kept.emplace_back(r1.rec, r1.rec + r1.nrec);
            const WalkRec* base = kept.back().data();
            for (size_t j = 0; j < bad.size(); ++j) {
                out[bad[j]] = r1.out[j];
                span[bad[j]] = {base + r1.out[j].base, base + r1.out[j].base + r1.out[j].count};
            }
        }
    }
    // each file's records into its op array (recycled arrays: no page faults), on the host
    // pool and the caller (SYDELTA_ASM_THREADS overrides)
    const int nthr = nf >= 64 ? (int)std::min<uint64_t>(asm_threads, (nf + 63) / 64) : 1;
    std::atomic<uint64_t> next{0};
    std::vector<sydelta_match_stats> part(nthr);
    auto worker = [&](int t) {
        sydelta_match_stats acc{};
        std::vector<WalkRec> tmp;
        for (;;) {
            const uint64_t f0 = next.fetch_add(64);
            if (f0 >= nf) break;
            for (uint64_t f = f0; f < std::min<uint64_t>(nf, f0 + 64); ++f) {
                sydelta_delta& d = b->d[f];
                const WalkRec *r0 = span[fu[f]].first, *r1 = span[fu[f]].second;
                uint32_t wh = 0, vh = 0;
                for (uint64_t u = fu[f]; u < fu[f + 1]; ++u) {
                    wh += out[u].weak_hits;
                    vh += out[u].hits;
                }
                if (fu[f + 1] - fu[f] > 1) {  // the segments' records joined: cut leading runs, merged Data ops
                    tmp.clear();
                    for (uint64_t u = fu[f]; u < fu[f + 1]; ++u)
                        for (const WalkRec* r = span[u].first; r < span[u].second; ++r) {
                            WalkRec x = *r;
                            if (r == span[u].first && tstart[u] != kNoTrim) {
                                const uint64_t h = x.off + x.a;
                                if (h <= tstart[u]) continue;
                                x.a = (uint32_t)(h - tstart[u]);
                                x.off = tstart[u];
                            }
                            if (!x.kind && !tmp.empty() && !tmp.back().kind && tmp.back().off + tmp.back().a == x.off)
                                tmp.back().a += x.a;
                            else
                                tmp.push_back(x);
                        }
                    r0 = tmp.data();
                    r1 = tmp.data() + tmp.size();
                }
                const uint64_t nops = records_ops(r0, r1);
                d.ops.resize(nops);
                uint64_t nd = 0, lb = 0;
                expand_records(r0, r1, n, ix->fblk[f], ix->fblk[f + 1] - ix->fblk[f], ix->last_size[f], d.ops.data(),
                               &nd, &lb);
                d.stats.copy_ops = nops - nd;
                d.stats.data_ops = nd;
                d.stats.literal_bytes = lb;
                d.stats.weak_hits = wh;
                d.stats.verified_hits = vh;
                acc.copy_ops += d.stats.copy_ops;
                acc.data_ops += nd;
                acc.literal_bytes += lb;
                acc.weak_hits += wh;
                acc.verified_hits += vh;
            }
        }
        part[t] = acc;
    };
    if (!run_parallel(nthr, worker)) return fail(SYDELTA_E_OOM, "out of host memory (op lists)");
    for (auto& p : part) {
        b->total.copy_ops += p.copy_ops;
        b->total.data_ops += p.data_ops;
        b->total.literal_bytes += p.literal_bytes;
        b->total.weak_hits += p.weak_hits;
        b->total.verified_hits += p.verified_hits;
    }
    PinnedHits& ph = thread_pinned_hits();
    if (ph.bytes > kPinnedHitsKeep) {
        (void)hipHostFree(ph.p);
        ph = PinnedHits();
    }
    if (host_timing)
        fprintf(stderr, "sydelta file walk: %llu files in %llu units, %d re-walk rounds, %llu records: kernel+counts "
                "%.3f ms, records D2H %.3f ms, expand %.3f ms\n", (unsigned long long)nf, (unsigned long long)nu, rounds,
                (unsigned long long)res.nrec, res.ms_kernel, res.ms_d2h, ms_since(t1));
    return SYDELTA_OK;
}

// Match source f (d_buf[src_off[f] .. +src_len[f])) against file f of the index,
// for every f; results in b->d[f].
// mode: the classifier's probe mode (-2: SYDELTA_PROBE's, probe_mode_env)
static int match_impl(sydelta_index* ix, const uint8_t* d_buf, const uint64_t* src_off, const uint64_t* src_len,
                      hipStream_t s, sydelta_delta_batch* b, int mode_hint = -2) {
    ScratchHold hold;  // the probe scratch is used until the walks end
    const auto t_begin = std::chrono::steady_clock::now();
    CallProf cp;
    HIP_TRY(index_wait(ix, s));
    const uint64_t n = ix->bs;
    const uint64_t nf = ix->nfiles;
    b->d.assign(nf, sydelta_delta());
    Classifier C;
    C.ix = ix;
    C.base = d_buf;
    C.s = s;
    C.prof = cp.get();
    C.n = n;
    C.src.resize(nf);
    C.adopt_spare();
    {
        int cur_dev = 0;
        HIP_TRY(hipGetDevice(&cur_dev));
        C.probe_scratch = &thread_probe_scratch(cur_dev);
    }
    uint64_t tot_pos = 0;
    for (uint64_t f = 0; f < nf; ++f) {
        b->d[f].source_size = src_len[f];
        b->d[f].block_size = n;
        if (src_len[f] && !d_buf) return fail(SYDELTA_E_INVAL, "NULL source buffer");
        if (src_len[f] && ((uintptr_t)(d_buf + src_off[f]) & 15) != 0)
            return fail(SYDELTA_E_INVAL, "source %llu must start 16-byte aligned", (unsigned long long)f);
        const uint64_t len = src_len[f];
        const uint64_t npos = len >= n ? len - n + 1 : 0;
        b->d[f].stats.positions = npos;
        tot_pos += npos;
        Src& c = C.src[f];
        c.file = (uint32_t)f;
        c.off = src_off[f];
        c.len = c.flen = len;
        const bool has_sig = ix->fblk[f + 1] > ix->fblk[f];
        c.p0 = 0;
        c.p1 = has_sig ? npos : 0;  // an empty signature matches nothing (generator.rs:121)
        c.kb = 0;
        c.nblk = (c.p1 + n - 1) / n;
    }
    b->total.positions = tot_pos;
    if (file_walk_ok(ix, src_off, src_len, d_buf)) return match_walk_files(ix, d_buf, src_off, src_len, s, C.prof, b);
    if (int r = index_full(ix, s)) return r;  // the classifier's probes and scans read the tables
    if (nf >= 64) take_small_ops(b->d);       // recycled per-file op arrays
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    const int mode = n > scan_max_window() && !wide_scan(ix) ? 0 : mode_hint != -2 ? mode_hint : probe_mode_env();
    if (int r = C.classify(mode)) return r;
    const double t_cls = ms_since(t0);
    std::vector<size_t> all(nf);
    for (size_t f = 0; f < nf; ++f) all[f] = f;
    std::vector<int> tail;
    if (int r = tail_flags(C, all, tail)) return r;
    const double t_tail = ms_since(t0);
    // Many sources: walk them on host threads first (a walk is pure host work over the
    // classified hits); a source whose walk reaches an unscanned block, and every source
    // of a small batch, is walked below through Classifier::walk (on-demand scans).
    std::vector<uint8_t> walked(nf, 0);
    const int nthr = walk_threads();
    if (nf >= 64 && nthr > 1) {
        std::atomic<uint64_t> next{0};
        auto worker = [&]() {
            for (;;) {
                const uint64_t f0 = next.fetch_add(32);
                if (f0 >= nf) break;
                for (uint64_t f = f0; f < std::min<uint64_t>(nf, f0 + 32); ++f) {
                    const Src& c = C.src[f];
                    if (c.nahit + c.hpos.size() >= walk_par_min()) continue;  // large: parallel walk below
                    const BasisInfo bi{ix->fblk[f], ix->fblk[f + 1] - ix->fblk[f], ix->last_size[f]};
                    uint64_t exit = 0, need = 0;
                    sydelta_delta* d = &b->d[f];
                    if (walk_src(c, n, 0, c.p1, bi, true, tail[f], d->ops, &exit, &need) == 0) {
                        walked[f] = 1;
                        d->stats.verified_hits = c.hpos.size() + c.nahit;
                        finish_stats(d);
                    }
                }
            }
        };
        if (!run_parallel(nthr, [&](int) { worker(); })) return fail(SYDELTA_E_OOM, "out of host memory (op lists)");
    }
    const double t_par = ms_since(t0);
    for (uint64_t f = 0; f < nf; ++f) {
        sydelta_delta* d = &b->d[f];
        const BasisInfo bi{ix->fblk[f], ix->fblk[f + 1] - ix->fblk[f], ix->last_size[f]};
        uint64_t exit = 0;
        if (!walked[f]) {
            if (int r = C.walk(f, 0, bi, true, tail[f], d, &exit)) return r;  // counts the ops too
            d->stats.verified_hits = C.src[f].hpos.size() + C.src[f].nahit;
        }
        b->total.verified_hits += d->stats.verified_hits;
        b->total.copy_ops += d->stats.copy_ops;
        b->total.data_ops += d->stats.data_ops;
        b->total.literal_bytes += d->stats.literal_bytes;
    }
    b->total.weak_hits = C.weak_hits;
    if (nf == 1) b->d[0].stats.weak_hits = C.weak_hits;
    if (host_timing && nf == 1) fprintf(stderr, "sydelta match: %.3f ms before the classifier's release\n", ms_since(t_begin));
    if (host_timing && nf > 1)
        fprintf(stderr,
                "sydelta match batch: %llu files, setup %.3f ms, classify %.3f ms, tail %.3f ms, threaded walks %.3f "
                "ms, rest %.3f ms\n",
                (unsigned long long)nf, ms_since(t_begin) - ms_since(t0), t_cls, t_tail - t_cls, t_par - t_tail,
                ms_since(t0) - t_par);
    return SYDELTA_OK;
}

namespace {
bool chunk_walk_ok(const sydelta_index* idx);  // (below)

// Is a single source copy-heavy, so that K10 walks it (as one chunk, sydelta_chunk_classify)
// instead of the classifier scanning every window start (k_scan_r: a literal-heavy source such
// as C3)?  Yes when 1/8 or more of a 1-in-16 sample of its aligned windows hit (the
// classifier's own probe rule), or -- a shifted source, where insertions put every later window
// off the block grid (C3b) -- when 1/4 or more of 256 consecutive blocks mid-file find a hit
// among their window starts (the walk's roll, k_preroll, on each missed block).  The index
// must be built (the caller waited for it).
int copy_heavy(sydelta_index* ix, const uint8_t* d_src, uint64_t len, hipStream_t s, Profiler* prof, bool* heavy) {
    *heavy = false;
    const uint64_t n = ix->bs, npos = len - n + 1, nblk = (npos + n - 1) / n;
    const uint32_t S = 16;
    const uint64_t np1 = (nblk + S - 1) / S, np2 = std::min<uint64_t>(256, nblk), r0 = (nblk - np2) / 2;
    ScratchHold hold;
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    DevScratch& sc = thread_probe_scratch(cur);
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t o_jobs = 0, o_out1 = 256, o_pw1 = o_out1 + al(4 * np1), o_pst1 = o_pw1 + al(4 * np1);
    const size_t o_out2 = o_pst1 + al(8 * np1), o_pw2 = o_out2 + al(4 * np2), o_pst2 = o_pw2 + al(4 * np2);
    const size_t o_list = o_pst2 + al(8 * np2), o_cnt = o_list + al(4 * np2), need = o_cnt + 256;
    if (sc.bytes < need) {
        if (sc.p) (void)hipFreeAsync(sc.p, s);
        sc = DevScratch();
        HIP_TRY(dev_malloc_async(&sc.p, need + need / 4, s));
        sc.bytes = need + need / 4;
    }
    uint8_t* D = (uint8_t*)sc.p;
    // both samples' results come back after one synchronization: h1 | h2 | the jobs' staging
    PinnedHits& pin = thread_probe_pin();
    if (int r = pinned_at_least(pin, al(4 * np1) + al(4 * np2) + 256)) return r;
    uint32_t* h1 = (uint32_t*)pin.p;
    uint32_t* h2 = (uint32_t*)(pin.p + al(4 * np1));
    ProbeJob* jobs = (ProbeJob*)(pin.p + al(4 * np1) + al(4 * np2));
    jobs[0] = ProbeJob{0, 0, 0, 0, 0};
    jobs[1] = ProbeJob{0, r0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(D + o_jobs, jobs, 2 * sizeof(ProbeJob), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(D + o_cnt, 0, 8, s));
    const bool fast = ((uintptr_t)d_src & 15) == 0;
    HIP_TRY(launch_probe(d_src, (const ProbeJob*)(D + o_jobs), 1, np1, S, (uint32_t)n, fast, ix->ix,
                         (uint32_t*)(D + o_pw1), (uint64_t*)(D + o_pst1), (uint32_t*)(D + o_out1), s, prof));
    HIP_TRY(hipMemcpyAsync(h1, D + o_out1, 4 * np1, hipMemcpyDeviceToHost, s));
    // the shifted sample: 256 consecutive aligned windows, each miss rolled for its first hit
    // (queued with the first: one round trip for both)
    uint32_t* d_out2 = (uint32_t*)(D + o_out2);
    uint32_t* d_pw2 = (uint32_t*)(D + o_pw2);
    HIP_TRY(launch_probe(d_src, (const ProbeJob*)(D + o_jobs) + 1, 1, np2, 1, (uint32_t)n, fast, ix->ix, d_pw2,
                         (uint64_t*)(D + o_pst2), d_out2, s, prof));
    const DeviceIndex& di = ix->ix;
    WalkArgs a{};
    a.base = d_src;
    a.n = (uint32_t)n;
    a.nm = (uint32_t)(n % 65521);
    a.files = di.d_files;
    a.fblk = di.d_fblk;
    a.filt = di.filt;
    a.keys = di.keys;
    a.start = di.start;
    a.cnt = di.cnt;
    a.order = di.order;
    a.cstrong = di.cstrong;
    a.weak = ix->d_weak;
    a.strong = ix->d_strong;
    if (ix->fblk[1] < kPreMark)
        HIP_TRY(launch_preroll(a, d_out2, d_pw2, r0, 0, np2, npos, len, (uint32_t*)(D + o_list),
                               (unsigned long long*)(D + o_cnt), (uint32_t)np2, np2, s, prof));
    HIP_TRY(hipMemcpyAsync(h2, d_out2, 4 * np2, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    uint64_t hits = 0;
    for (uint64_t i = 0; i < np1; ++i) hits += h1[i] != kNoBlk;
    if (hits * 8 >= np1) {
        *heavy = true;
        return SYDELTA_OK;
    }
    hits = 0;
    for (uint64_t i = 0; i < np2; ++i) hits += h2[i] != kNoBlk && h2[i] != kPreNone;
    *heavy = hits * 4 >= np2;
    return SYDELTA_OK;
}
}  // namespace

extern "C" int sydelta_match_device(sydelta_index* idx, const uint8_t* d_src, uint64_t len, void* stream,
                                    sydelta_delta** out) try {
    if (!idx || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = nullptr;
    if (idx->nfiles != 1) return fail(SYDELTA_E_INVAL, "index holds %llu files; use sydelta_match_batch_device",
                                      (unsigned long long)idx->nfiles);
    if (len && !d_src) return fail(SYDELTA_E_INVAL, "NULL source");
    SYDELTA_ENTER_DEVICE(idx->device);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(idx->device);
    sydelta_delta_batch b;
    const uint64_t off = 0;
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    int mode = -2;
    // the ribbon level-1 a whole-file scan of this many positions takes (scan_index), built now
    // from the signature's weak values -- beside the index's own build on the aux stream --
    // instead of from its exact table after it (SYDELTA_EARLY_RIBBON=0: after, as in round 5)
    const uint64_t npos_all = len >= idx->bs ? len - idx->bs + 1 : 0;
    if (early_ribbon_mode() == 1 && s == idx->stream && idx->nfiles == 1 &&
        (idx->rib_mode == 2 || (idx->rib_mode == 1 && npos_all >= kRibMinScan))) {
        std::lock_guard<std::mutex> lk(idx->rib_mu);
        if (!idx->rib_built) {
            CallProf cp;
            HIP_TRY(launch_ribbon_build(idx->ix, s, cp.get(), idx->d_weak, idx->fblk[1]));
            if (!idx->rib_ev && !(idx->rib_ev = take_event(idx->device))) return fail(SYDELTA_E_OOM, "no event");
            HIP_TRY(hipEventRecord(idx->rib_ev, s));
            idx->rib_built = true;
            idx->rib_stream = s;
        }
    }
    // the scan's extras (level-1 Bloom, fat table: scan_index) on the ribbon's stream, beside
    // the copy-heavy sample below, so that a literal-heavy source's scan finds them built (a
    // copy-heavy one has spent ~0.06 ms of a few CUs)
    if (idx->nfiles == 1 && s == idx->stream && npos_all) {
        std::lock_guard<std::mutex> lk(idx->build_mu);
        if (idx->extras_deferred && !idx->deferred) {
            const hipStream_t sx = thread_walk_stream(idx->device, 2);
            if (sx) {
                HIP_TRY(index_wait(idx, sx));
                CallProf cp;
                HIP_TRY(launch_index_extras(idx->d_weak, idx->ix, sx, cp.get()));
                if (!idx->extras_ev && !(idx->extras_ev = take_event(idx->device)))
                    return fail(SYDELTA_E_OOM, "no event");
                HIP_TRY(hipEventRecord(idx->extras_ev, sx));
                idx->extras_deferred = false;
                idx->extras_stream = sx;
            }
        }
    }
    // a copy-heavy source is walked by K10 as one chunk (generator.rs:116-221 on the device);
    // a literal-heavy one by the classifier, whose probe sample would say the same (mode 0)
    if (chunk_walk_ok(idx) && probe_mode_env() < 0 && len >= idx->bs && idx->fblk[1] > 0 &&
        ((uintptr_t)d_src & 15) == 0) {
        HIP_TRY(index_wait(idx, s));
        bool heavy = false;
        {
            CallProf cp;
            if (int r = copy_heavy(idx, d_src, len, s, cp.get(), &heavy)) return r;
        }
        if (heavy) {
            sydelta_chunk* ch = nullptr;
            if (int r = sydelta_chunk_classify(idx, d_src, 0, len, len, 0, len, s, &ch)) return r;
            uint64_t exit = 0;
            const int r = sydelta_chunk_walk(ch, 0, &exit, out);
            sydelta_chunk_free(ch);
            if (host_timing) fprintf(stderr, "sydelta match_device (K10): %.3f ms\n", ms_since(t0));
            return r;
        }
        mode = 0;
    }
    if (int r = match_impl(idx, d_src, &off, &len, s, &b, mode)) return r;
    *out = new sydelta_delta(std::move(b.d[0]));
    if (host_timing) fprintf(stderr, "sydelta match_device: %.3f ms (with the classifier's release)\n", ms_since(t0));
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_match_batch_device(sydelta_index* idx, const uint8_t* d_buf, const uint64_t* src_off,
                                          const uint64_t* src_len, uint64_t nfiles, void* stream,
                                          sydelta_delta_batch** out) try {
    if (!idx || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = nullptr;
    if (nfiles != idx->nfiles) return fail(SYDELTA_E_INVAL, "index holds %llu files, %llu sources given",
                                           (unsigned long long)idx->nfiles, (unsigned long long)nfiles);
    if (nfiles && (!src_off || !src_len)) return fail(SYDELTA_E_INVAL, "NULL segment table");
    SYDELTA_ENTER_DEVICE(idx->device);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(idx->device);
    std::unique_ptr<sydelta_delta_batch> b(new sydelta_delta_batch());
    if (int r = match_impl(idx, d_buf, src_off, src_len, s, b.get())) return r;
    *out = b.release();
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// Signature + match of many (basis, source) pairs in one call (the C4 shape): the files in two
// groups, the first's signature and walks on `stream`, the second's on the thread's aux stream,
// so the first group's walks run beside the second group's signature; no index is built (the
// walks self-index each file from the signature, sydelta_filewalk.hip).
extern "C" int sydelta_delta_pairs_device(int device, const uint8_t* d_basis, const uint64_t* basis_off,
                                          const uint64_t* basis_len, const uint8_t* d_src, const uint64_t* src_off,
                                          const uint64_t* src_len, uint64_t nfiles, uint64_t block_size, void* stream,
                                          sydelta_delta_batch** out) try {
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    if (!nfiles || nfiles >= (1ull << 31)) return fail(SYDELTA_E_INVAL, "bad file count %llu", (unsigned long long)nfiles);
    if (!basis_off || !basis_len || !src_off || !src_len) return fail(SYDELTA_E_INVAL, "NULL segment table");
    const uint64_t n = block_size;
    if (n % 64 != 0 || n < 256 || n > kWalkMaxN)
        return fail(SYDELTA_E_INVAL, "block_size %llu: the pairs call needs a multiple of 64 in [256, %u]",
                    (unsigned long long)n, kWalkMaxN);
    std::vector<uint64_t> fblk(nfiles + 1, 0), last(nfiles, 0);
    uint64_t max_nblk = 0, recs = 0;
    for (uint64_t f = 0; f < nfiles; ++f) {
        const uint64_t nb = (basis_len[f] + n - 1) / n;
        if (nb > kSelfIxMaxBlocks)
            return fail(SYDELTA_E_INVAL, "basis %llu has %llu blocks (at most %u)", (unsigned long long)f,
                        (unsigned long long)nb, kSelfIxMaxBlocks);
        if (basis_len[f] && (!d_basis || ((uintptr_t)(d_basis + basis_off[f]) & 15)))
            return fail(SYDELTA_E_INVAL, "basis %llu must start 16-byte aligned", (unsigned long long)f);
        if (src_len[f] && (!d_src || ((uintptr_t)(d_src + src_off[f]) & 15)))
            return fail(SYDELTA_E_INVAL, "source %llu must start 16-byte aligned", (unsigned long long)f);
        if (src_len[f] >= (1ull << 32)) return fail(SYDELTA_E_INVAL, "source %llu too large", (unsigned long long)f);
        fblk[f + 1] = fblk[f] + nb;
        last[f] = nb ? basis_len[f] - (nb - 1) * n : 0;
        max_nblk = std::max(max_nblk, nb);
        recs += 2 * (src_len[f] / n) + 4;
    }
    if (recs >= (1ull << 32) || fblk[nfiles] >= 0xFFFFFFFFull) return fail(SYDELTA_E_INVAL, "batch too large");
    SYDELTA_ENTER_DEVICE(device);
    if (device < 0) device = 0;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device);
    hipStream_t s2 = thread_aux_stream(device);
    if (!s2) return fail(SYDELTA_E_OOM, "no stream for the pairs call");
    const uint64_t nb = std::max<uint64_t>(1, fblk[nfiles]);
    const uint64_t G = nfiles >= 128 ? 2 : 1;
    std::vector<uint64_t> split(G + 1);
    for (uint64_t g = 0; g <= G; ++g) split[g] = nfiles * g / G;
    // one upload: the file table, then each group's signature table (the kernels' arguments
    // live in this call's own allocation: none is freed while a kernel on the other stream runs)
    std::vector<uint64_t> up(fblk.begin(), fblk.end());
    std::vector<SigTable> tabs;
    for (uint64_t g = 0; g < G; ++g)
        tabs.push_back(sig_batch_table(basis_off + split[g], basis_len + split[g], split[g + 1] - split[g], n,
                                       fblk[split[g]], up));
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t o_weak = 0, o_strong = al(4 * nb), o_fblk = o_strong + al(8 * nb), need = o_fblk + 8 * up.size();
    uint8_t* D = nullptr;
    CallProf cp;
    HIP_TRY(dev_malloc_async((void**)&D, need, s));
    struct Free {  // the arrays, in s's order (the walks on s2 are joined to s before returning)
        uint8_t* p;
        hipStream_t s;
        ~Free() { (void)hipFreeAsync(p, s); }
    } free_d{D, s};
    if (int r = upload_staged(D + o_fblk, up.data(), 8 * up.size(), s)) return r;
    // groups: two halves of a batch of >= 128 files (each half still fills the chip's wave
    // slots with its segments)
    std::vector<hipEvent_t> ev(G, nullptr);
    struct Events {
        std::vector<hipEvent_t>& v;
        int dev;
        ~Events() {
            for (hipEvent_t e : v)
                if (e) give_event(dev, e);
        }
    } ev_back{ev, device};
    hipEvent_t ready = take_event(device);  // the arrays allocated (s2 orders itself after it)
    if (!ready) return fail(SYDELTA_E_OOM, "no event for the pairs call");
    ev_back.v.push_back(ready);
    HIP_TRY(hipEventRecord(ready, s));
    for (uint64_t g = 0; g < G; ++g) {
        const hipStream_t sg = (g & 1) ? s2 : s;  // (run_walk launches group g's walks on the same stream)
        if (sg != s) HIP_TRY(hipStreamWaitEvent(sg, ready, 0));
        if (tabs[g].nfull || tabs[g].npart)
            HIP_TRY(launch_sig_table(d_basis, (const uint64_t*)(D + o_fblk), tabs[g], n, (uint32_t*)(D + o_weak),
                                     (uint64_t*)(D + o_strong), sg, cp.get()));
        ev[g] = take_event(device);
        if (!ev[g]) return fail(SYDELTA_E_OOM, "no event for the pairs call");
        HIP_TRY(hipEventRecord(ev[g], sg));
    }
    // the walks' view of the signature: no tables (each walk self-indexes its file)
    sydelta_index X;
    X.device = device;
    X.bs = n;
    X.nfiles = nfiles;
    X.fblk = fblk;
    X.last_size = last;
    X.d_weak = (uint32_t*)(D + o_weak);
    X.d_strong = (uint64_t*)(D + o_strong);
    X.ix.d_fblk = (uint64_t*)(D + o_fblk);
    X.ix.nfiles = nfiles;
    X.ix.nblocks = fblk[nfiles];
    X.max_nblk = max_nblk;
    X.deferred = true;
    std::unique_ptr<sydelta_delta_batch> b(new sydelta_delta_batch());
    b->d.assign(nfiles, sydelta_delta());
    for (uint64_t f = 0; f < nfiles; ++f) {
        b->d[f].source_size = src_len[f];
        b->d[f].block_size = n;
        b->d[f].stats.positions = src_len[f] >= n ? src_len[f] - n + 1 : 0;
        b->total.positions += b->d[f].stats.positions;
    }
    if (int r = match_walk_files(&X, d_src, src_off, src_len, s, cp.get(), b.get(), &split, &ev, s2)) return r;
    *out = b.release();
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// ---------------------------------------------------------------------------
// host-buffer entry points
// ---------------------------------------------------------------------------
extern "C" int sydelta_compute_checksums_buf(int device, const uint8_t* buf, uint64_t len, uint64_t block_size,
                                             sydelta_block_checksum* out, uint64_t cap, uint64_t* n_out) try {
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (!n_out) return fail(SYDELTA_E_INVAL, "n_out is NULL");
    const uint64_t nb = len ? (len + block_size - 1) / block_size : 0;  // checksum.rs:36-41
    *n_out = nb;
    if (!nb) return SYDELTA_OK;
    if (!buf || !out) return fail(SYDELTA_E_INVAL, "NULL buffer");
    if (cap < nb) return fail(SYDELTA_E_INVAL, "output holds %llu entries, need %llu", (unsigned long long)cap,
                              (unsigned long long)nb);
    SYDELTA_ENTER_DEVICE(device);
    if (device < 0) device = 0;
    hipStream_t s = thread_stream(device);
    uint8_t* d_buf = nullptr;
    HIP_TRY(dev_malloc_async((void**)&d_buf, (len + 15) & ~15ull, s));
    DevBuf b1; b1.p = d_buf; b1.s = s;
    uint32_t* d_w = nullptr;
    HIP_TRY(dev_malloc_async((void**)&d_w, nb * 12 + 16, s));
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
} catch (...) {
    return sydelta::host_exception();
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
    SYDELTA_ENTER_DEVICE(device);
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
        HIP_TRY(dev_malloc_async((void**)&d_src, (len + 15) & ~15ull, s));
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
                                          sydelta_delta** out) try {
    return generate_from_host(device, src, len, sigs, nsigs, block_size, out);
} catch (...) {
    return sydelta::host_exception();
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

// Streamed file input for the path API: a file is read in chunks (64 MiB, a multiple of
// lcm(block_size, 16); SYDELTA_STREAM_CHUNK overrides the size for tests) through two
// per-thread pinned buffers.  While the device works on chunk g (H2D, then its kernels),
// a reader thread fills the other buffer with chunk g+1, so host memory stays at two
// chunks whatever the file size (plus the output: checksums, ops, literal bytes).
namespace {
uint64_t stream_chunk_bytes(uint64_t bs) {
    uint64_t want = 64ull << 20;
    if (const char* e = getenv("SYDELTA_STREAM_CHUNK")) {
        const uint64_t v = strtoull(e, nullptr, 10);
        if (v) want = v;
    }
    const uint64_t unit = bs / std::gcd<uint64_t>(bs, 16) * 16;  // lcm(bs, 16)
    return std::max<uint64_t>(unit, want / unit * unit);
}

struct PinnedPair {  // per thread, grown on demand, freed at thread exit
    uint8_t* p[2] = {nullptr, nullptr};
    uint64_t cap = 0;
    ~PinnedPair() { release(); }
    void release() {
        for (auto& q : p) {
            if (q) (void)hipHostFree(q);
            q = nullptr;
        }
        cap = 0;
    }
    int ensure(uint64_t bytes) {
        if (bytes <= cap) return SYDELTA_OK;
        release();
        for (auto& q : p) HIP_TRY(hipHostMalloc((void**)&q, bytes, hipHostMallocDefault));
        cap = bytes;
        return SYDELTA_OK;
    }
};
thread_local PinnedPair t_stream_pinned;

struct InFile {
    int fd = -1;
    uint64_t len = 0;
    std::string path;
    ~InFile() {
        if (fd >= 0) close(fd);
    }
    int open_(const char* p) {
        if (!p) return fail(SYDELTA_E_INVAL, "path is NULL");
        path = p;
        fd = open(p, O_RDONLY | O_CLOEXEC);
        if (fd < 0) return fail(SYDELTA_E_IO, "%s: %s", p, strerror(errno));
        struct stat stt;
        if (fstat(fd, &stt) != 0) return fail(SYDELTA_E_IO, "%s: %s", p, strerror(errno));
        len = (uint64_t)stt.st_size;
        return SYDELTA_OK;
    }
    // exactly [off, off + n) (the file must not shrink meanwhile).  A large read is split
    // into pieces of >= 8 MiB read by the shared host pool: one thread copies from the
    // page cache at ~12 GB/s, far below the pinned H2D's 57 GB/s (round 3, the path API's
    // 4 GiB leg: 12.7 GiB/s with 1 reader, 20.0 with 8, 25.7 with 16 on the box's 16-core
    // share; profiles/r03n_*).  A failed piece repeats the whole read on this thread, so
    // sydelta_last_error() names the failure.
    int read_at(uint64_t off, uint8_t* dst, uint64_t n) const {
        const int kReaders = [] {  // SYDELTA_READ_THREADS: readers per chunk (per call)
            const char* e = getenv("SYDELTA_READ_THREADS");
            return (e && *e) ? std::max(1, atoi(e)) : 16;
        }();
        const uint64_t kPiece = [] {  // SYDELTA_READ_PIECE: smallest piece (tests)
            const char* e = getenv("SYDELTA_READ_PIECE");
            const uint64_t v = (e && *e) ? strtoull(e, nullptr, 10) : 0;
            return v ? v : 8ull << 20;
        }();
        const int np = (int)std::min<uint64_t>((uint64_t)kReaders, n / kPiece);
        if (np > 1) {
            const uint64_t per = (n / np + 4095) & ~4095ull;
            std::atomic<bool> bad{false};
            const bool ok = run_parallel(np, [&](int t) {
                const uint64_t a = std::min(n, (uint64_t)t * per), b = std::min(n, a + per);
                if (read_range(off + a, dst + a, b - a, false)) bad = true;
            });
            if (ok && !bad) return SYDELTA_OK;
        }
        return read_range(off, dst, n, true);
    }
    int read_range(uint64_t off, uint8_t* dst, uint64_t n, bool report) const {
        uint64_t got = 0;
        while (got < n) {
            const ssize_t r = pread(fd, dst + got, (size_t)std::min<uint64_t>(n - got, 1ull << 30), (off_t)(off + got));
            if (r < 0 && errno == EINTR) continue;
            if (r < 0) return report ? fail(SYDELTA_E_IO, "%s: %s", path.c_str(), strerror(errno)) : SYDELTA_E_IO;
            if (r == 0)
                return report ? fail(SYDELTA_E_IO, "%s: short read at %llu", path.c_str(), (unsigned long long)(off + got))
                              : SYDELTA_E_IO;
            got += (uint64_t)r;
        }
        return SYDELTA_OK;
    }
};

// Runs `read` (the next chunk) on a helper thread while the caller runs `work` (the
// device part of this chunk); inline after `work` when no thread can be started.  A
// failed read is repeated on the calling thread so that its sydelta_last_error() names
// the failure.
template <class R, class W>
int overlap(bool has_next, R&& read, W&& work) {
    int rr = SYDELTA_OK;
    std::thread t;
    bool threaded = false;
    if (has_next) {
        try {
            t = std::thread([&] { rr = read(); });
            threaded = true;
        } catch (...) {
        }
    }
    int wr;
    try {
        wr = work();
    } catch (...) {
        if (t.joinable()) t.join();
        throw;
    }
    if (t.joinable()) t.join();
    if (wr) return wr;
    if (has_next && (!threaded || rr)) rr = read();
    return rr;
}
}  // namespace

// checksum.rs:31-80: every block of the file, read chunk by chunk (the reference opens,
// seeks and reads each block, :46-59), signed on the device; bounded host memory.
extern "C" int sydelta_compute_checksums(const char* path, uint64_t block_size, sydelta_block_checksum** out,
                                         uint64_t* n) try {
    if (!out || !n) return fail(SYDELTA_E_INVAL, "NULL output");
    *out = nullptr;
    *n = 0;
    InFile f;
    if (int r = f.open_(path)) return r;
    const uint64_t L = f.len;
    if (L == 0) return SYDELTA_OK;  // checksum.rs:36-38
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    const uint64_t nb = (L + block_size - 1) / block_size;
    int dev = 0;
    if (int r = path_device(&dev)) return r;
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = thread_stream(dev);
    const uint64_t C = std::min<uint64_t>(stream_chunk_bytes(block_size), L);
    const uint64_t nch = (L + C - 1) / C;
    PinnedPair& pin = t_stream_pinned;
    if (int r = pin.ensure(C + 16)) return r;
    DevBuf db, dw;
    HIP_TRY(dev_malloc_async(&db.p, C + 16, s));
    db.s = s;
    HIP_TRY(dev_malloc_async(&dw.p, nb * 12 + 16, s));
    dw.s = s;
    uint32_t* d_w = (uint32_t*)dw.p;
    uint64_t* d_st = (uint64_t*)(((uintptr_t)(d_w + nb) + 7) & ~(uintptr_t)7);
    if (int r = f.read_at(0, pin.p[0], std::min(C, L))) return r;
    CallProf cp;
    for (uint64_t g = 0; g < nch; ++g) {
        const uint64_t b0 = g * C, len = std::min(C, L - b0);
        const uint64_t nb1 = b0 + C < L ? std::min(C, L - b0 - C) : 0;
        const int r = overlap(
            g + 1 < nch, [&] { return f.read_at(b0 + C, pin.p[(g + 1) & 1], nb1); },
            [&]() -> int {
                HIP_TRY(hipMemcpyAsync(db.p, pin.p[g & 1], len, hipMemcpyHostToDevice, s));
                HIP_TRY(launch_signature((const uint8_t*)db.p, len, block_size, d_w + b0 / block_size,
                                         d_st + b0 / block_size, s, cp.get()));
                HIP_TRY(hipStreamSynchronize(s));  // the device buffer and this pinned buffer are reused
                return SYDELTA_OK;
            });
        if (r) return r;
    }
    std::vector<uint32_t> w(nb);
    std::vector<uint64_t> st(nb);
    HIP_TRY(hipMemcpyAsync(w.data(), d_w, 4 * nb, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(st.data(), d_st, 8 * nb, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    sydelta_block_checksum* v = (sydelta_block_checksum*)malloc(sizeof(sydelta_block_checksum) * nb);
    if (!v) return fail(SYDELTA_E_OOM, "host allocation failed");
    for (uint64_t i = 0; i < nb; ++i) {
        v[i].index = i;
        v[i].offset = i * block_size;
        v[i].size = std::min<uint64_t>(block_size, L - i * block_size);
        v[i].weak = w[i];
        v[i].reserved = 0;
        v[i].strong = st[i];
    }
    *out = v;
    *n = nb;
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" void sydelta_checksums_free(sydelta_block_checksum* p) { free(p); }

// generator.rs:242
extern "C" int sydelta_generate_delta(const char* source_path, const sydelta_block_checksum* sigs, uint64_t nsigs,
                                      uint64_t block_size, sydelta_delta** out) try {
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    std::vector<uint8_t> data;
    if (int r = read_file(source_path, data)) return r;
    int dev = 0;
    if (int r = path_device(&dev)) return r;
    return generate_from_host(dev, data.data(), data.size(), sigs, nsigs, block_size, out);
} catch (...) {
    return sydelta::host_exception();
}

// generator.rs:67-228 — identical ops to generate_delta for block_size <= 128 KiB
// (SURVEY.md App. A R10); larger sizes are outside the production domain.  The source is
// streamed: chunk g (window starts [g*C, (g+1)*C), its bytes plus the n-1 that the last
// window needs) is copied from a pinned buffer to the device, classified
// (sydelta_chunk_classify: aligned probe, scans) and walked from the previous chunk's
// exit (sydelta_chunk_walk, on-demand scans read the chunk still on the device), and
// its Data ops take their literal bytes from the pinned chunk; the next chunk is read
// meanwhile.  The ops equal generate_delta's (the chunk-sharded walk).
extern "C" int sydelta_generate_delta_streaming(const char* source_path, const sydelta_block_checksum* sigs,
                                                uint64_t nsigs, uint64_t block_size, sydelta_delta** out) try {
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    if (block_size == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    if (block_size > 128 * 1024)
        return fail(SYDELTA_E_INVAL, "block_size %llu > 131072: streaming semantics diverge (see sydelta.h)",
                    (unsigned long long)block_size);
    if (nsigs && !sigs) return fail(SYDELTA_E_INVAL, "NULL checksums");
    uint64_t last_size = 0;
    if (int r = check_sigs(sigs, nsigs, block_size, &last_size)) return r;
    InFile f;
    if (int r = f.open_(source_path)) return r;
    int dev = 0;
    if (int r = path_device(&dev)) return r;
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = thread_stream(dev);
    const uint64_t L = f.len, n = block_size;
    std::vector<uint32_t> w(nsigs);
    std::vector<uint64_t> st(nsigs);
    for (uint64_t i = 0; i < nsigs; ++i) {
        w[i] = sigs[i].weak;
        st[i] = sigs[i].strong;
    }
    sydelta_index* ixp = nullptr;
    if (int r = sydelta_index_create(dev, w.data(), st.data(), nsigs, n, last_size, 0, s, &ixp)) return r;
    std::unique_ptr<sydelta_index, void (*)(sydelta_index*)> ix(ixp, sydelta_index_free);
    std::vector<uint32_t>().swap(w);
    std::vector<uint64_t>().swap(st);
    const uint64_t npos = L >= n ? L - n + 1 : 0;
    const uint64_t C = stream_chunk_bytes(n);
    const uint64_t nch = npos ? (npos + C - 1) / C : 1;
    auto chunk_end = [&](uint64_t g) { return g + 1 == nch ? L : std::min(L, (g + 1) * C + n - 1); };
    const uint64_t cap = std::max<uint64_t>(chunk_end(0), nch > 1 ? chunk_end(nch - 1) - (nch - 1) * C : 0);
    PinnedPair& pin = t_stream_pinned;
    if (int r = pin.ensure(cap + 16)) return r;
    DevBuf db;
    HIP_TRY(dev_malloc_async(&db.p, cap + 16, s));
    db.s = s;
    std::unique_ptr<sydelta_delta> d(new sydelta_delta());
    d->source_size = L;
    d->block_size = n;
    if (L) {
        if (int r = f.read_at(0, pin.p[0], chunk_end(0))) return r;
    }
    uint64_t entry = 0;
    for (uint64_t g = 0; g < nch; ++g) {
        const uint64_t b0 = g * C, b1 = chunk_end(g), blen = b1 - b0;
        const uint8_t* host = pin.p[g & 1];
        const int r = overlap(
            g + 1 < nch, [&] { return f.read_at(b0 + C, pin.p[(g + 1) & 1], chunk_end(g + 1) - (b0 + C)); },
            [&]() -> int {
                if (blen) HIP_TRY(hipMemcpyAsync(db.p, host, blen, hipMemcpyHostToDevice, s));
                sydelta_chunk* chp = nullptr;
                const uint64_t pe = g + 1 == nch ? std::max(npos, b0) : b0 + C;
                if (int rc = sydelta_chunk_classify(ix.get(), (const uint8_t*)db.p, b0, blen, L, b0, pe, s, &chp))
                    return rc;
                std::unique_ptr<sydelta_chunk, void (*)(sydelta_chunk*)> ch(chp, sydelta_chunk_free);
                sydelta_delta* pp = nullptr;
                uint64_t exit = 0;
                if (int rc = sydelta_chunk_walk(ch.get(), entry, &exit, &pp)) return rc;
                std::unique_ptr<sydelta_delta, void (*)(sydelta_delta*)> part(pp, sydelta_delta_free);  // recycles its ops
                HIP_TRY(hipStreamSynchronize(s));  // the device buffer and this pinned buffer are reused
                // append, merging a Data op contiguous with the previous chunk's last one, and
                // copy every Data op's bytes from this chunk's host buffer
                size_t j = 0;
                if (!d->ops.empty() && !part->ops.empty()) {
                    sydelta_op& a = d->ops.back();
                    const sydelta_op& b = part->ops.front();
                    if (a.kind == SYDELTA_OP_DATA && b.kind == SYDELTA_OP_DATA && a.a + a.b == b.a) {
                        if (b.a < b0 || b.a + b.b > b1)
                            return fail(SYDELTA_E_INVAL, "internal: literal run outside its chunk");
                        d->lit.insert(d->lit.end(), host + (b.a - b0), host + (b.a - b0) + b.b);
                        a.b += b.b;
                        j = 1;
                    }
                }
                for (; j < part->ops.size(); ++j) {
                    const sydelta_op& o = part->ops[j];
                    d->ops.push_back(o);
                    if (o.kind == SYDELTA_OP_DATA) {
                        if (o.a < b0 || o.a + o.b > b1)
                            return fail(SYDELTA_E_INVAL, "internal: literal run [%llu, +%llu) outside chunk [%llu, %llu)",
                                        (unsigned long long)o.a, (unsigned long long)o.b, (unsigned long long)b0,
                                        (unsigned long long)b1);
                        d->lit_off.resize(d->ops.size() - 1, UINT64_MAX);
                        d->lit_off.push_back(d->lit.size());
                        d->lit.insert(d->lit.end(), host + (o.a - b0), host + (o.a - b0) + o.b);
                    }
                }
                d->stats.positions += part->stats.positions;
                d->stats.weak_hits += part->stats.weak_hits;
                d->stats.verified_hits += part->stats.verified_hits;
                entry = exit;
                return SYDELTA_OK;
            });
        if (r) return r;
    }
    d->lit_off.resize(d->ops.size(), UINT64_MAX);
    finish_stats(d.get());
    *out = d.release();
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// applier.rs:22-56 — receiver side, host I/O only.
// applier.rs:22-56 on device-resident bytes: Copy{offset, size} reads basis[offset,
// +size) (read_exact: past the end is an error, applier.rs:36), Data reads its literal
// bytes from d_lit at the op's source offset (a device delta's Data ops index the
// source the delta was generated from).
extern "C" int sydelta_apply_delta_device(int device, const uint8_t* d_basis, uint64_t basis_len,
                                          const sydelta_delta* d, const uint8_t* d_lit, uint64_t lit_len,
                                          uint8_t* d_out, uint64_t out_cap, void* stream, sydelta_apply_stats* out) try {
    if (!d) return fail(SYDELTA_E_INVAL, "NULL delta");
    SYDELTA_ENTER_DEVICE(device);
    // the piece table is staged in pinned host memory (one per thread, grown on demand)
    // so its upload runs at PCIe speed
    struct Pinned {
        ApplyPiece* p = nullptr;
        size_t cap = 0;
        ~Pinned() { if (p) (void)hipHostFree(p); }
    };
    static thread_local Pinned pin;
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    constexpr uint64_t kSlice = 64 * 1024;
    // validate every op first, overflow-checked (a delta parsed from remote JSON may
    // carry any sizes): the output is not touched and nothing is allocated on an error
    uint64_t pos = 0, literal = 0, need = 0;
    for (size_t i = 0; i < d->ops.size(); ++i) {
        const sydelta_op& o = d->ops[i];
        const bool cp = o.kind == SYDELTA_OP_COPY;
        if (o.kind != SYDELTA_OP_COPY && o.kind != SYDELTA_OP_DATA)
            return fail(SYDELTA_E_INVAL, "op %zu: unknown kind %u", i, (unsigned)o.kind);
        if (cp && (o.a > basis_len || o.b > basis_len - o.a))
            return fail(SYDELTA_E_IO, "op %zu: Copy{offset %llu, size %llu} past the end of the basis (%llu bytes): "
                        "failed to fill whole buffer", i, (unsigned long long)o.a, (unsigned long long)o.b,
                        (unsigned long long)basis_len);
        if (!cp && (o.a > lit_len || o.b > lit_len - o.a))
            return fail(SYDELTA_E_INVAL, "op %zu: Data [%llu, +%llu) outside the literal buffer", i,
                        (unsigned long long)o.a, (unsigned long long)o.b);
        if (o.b > out_cap - std::min(pos, out_cap))
            return fail(SYDELTA_E_INVAL, "output needs more than its capacity of %llu bytes",
                        (unsigned long long)out_cap);
        pos += o.b;  // <= out_cap: no overflow
        if (!cp) literal += o.b;
        need += o.b / kSlice + (o.b % kSlice != 0);
    }
    if (pos && !d_out) return fail(SYDELTA_E_INVAL, "NULL output");
    if (need > pin.cap) {
        if (pin.p) { (void)hipHostFree(pin.p); pin.p = nullptr; pin.cap = 0; }
        const size_t cap = std::max<size_t>(need, 4096) * 5 / 4;
        HIP_TRY(hipHostMalloc((void**)&pin.p, cap * sizeof(ApplyPiece), hipHostMallocDefault));
        pin.cap = cap;
    }
    ApplyPiece* pieces = pin.p;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(device < 0 ? 0 : device);
    CallProf cp;
    if (need) {
        // Pipelined: the host fills batch j of the piece table while batch j-1 is
        // uploaded on a copy stream and batch j-2 is copied by k_apply on `s`.
        constexpr size_t kBatches = 8;
        // per thread and device, never destroyed (like thread_stream)
        static thread_local std::map<int, std::pair<hipStream_t, std::vector<hipEvent_t>>> copy_streams;
        auto& cs = copy_streams[device < 0 ? 0 : device];
        if (!cs.first) HIP_TRY(hipStreamCreateWithFlags(&cs.first, hipStreamNonBlocking));
        while (cs.second.size() < kBatches) {
            hipEvent_t e;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            cs.second.push_back(e);
        }
        hipStream_t cstream = cs.first;
        const std::vector<hipEvent_t>& ev = cs.second;
        // On an error after the first upload was queued: drain both streams before the
        // table (device) and the pinned staging (host, reused by the next call) go away
        // (drain is declared after pb, so it runs first).
        DevBuf pb;
        struct Drain {
            hipStream_t a, b;
            bool armed = false;
            ~Drain() {
                if (armed) { (void)hipStreamSynchronize(a); (void)hipStreamSynchronize(b); }
            }
        } drain{cstream, s};
        HIP_TRY(dev_malloc_async(&pb.p, need * sizeof(ApplyPiece), s));
        pb.s = s;
        HIP_TRY(hipEventRecord(ev[0], s));  // the table allocation is ordered before the uploads
        HIP_TRY(hipStreamWaitEvent(cstream, ev[0], 0));
        drain.armed = true;
        ApplyPiece* dp = (ApplyPiece*)pb.p;
        const size_t per = std::max<size_t>(1, (d->ops.size() + kBatches - 1) / kBatches);
        size_t np = 0, j = 0;
        uint64_t at = 0;
        for (size_t i0 = 0; i0 < d->ops.size(); i0 += per, ++j) {
            const size_t i1 = std::min(d->ops.size(), i0 + per);
            const size_t b0 = np;
            for (size_t i = i0; i < i1; ++i) {
                const sydelta_op& o = d->ops[i];
                const uint32_t cpf = o.kind == SYDELTA_OP_COPY ? 1u : 0u;
                for (uint64_t k = 0; k < o.b; k += kSlice)
                    pieces[np++] = {at + k, o.a + k, (uint32_t)std::min<uint64_t>(kSlice, o.b - k), cpf};
                at += o.b;
            }
            if (np == b0) continue;
            HIP_TRY(hipMemcpyAsync(dp + b0, pieces + b0, (np - b0) * sizeof(ApplyPiece), hipMemcpyHostToDevice,
                                   cstream));
            HIP_TRY(hipEventRecord(ev[j], cstream));
            HIP_TRY(hipStreamWaitEvent(s, ev[j], 0));
            HIP_TRY(launch_apply(dp + b0, np - b0, d_basis, d_lit, d_out, s, cp.get()));
        }
        const double t_enq = ms_since(t0);
        HIP_TRY(hipStreamSynchronize(s));  // the pinned table is reused by the next call
        drain.armed = false;
        if (host_timing)
            fprintf(stderr, "sydelta apply: %zu pieces, validate+build+enqueue %.3f ms, total %.3f ms\n", np,
                    t_enq, ms_since(t0));
    }
    if (out) {
        out->operations_count = d->ops.size();
        out->literal_bytes = literal;
        out->bytes_written = pos;
    }
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_apply_delta(const char* old_file, const sydelta_delta* d, const char* new_file,
                                   sydelta_apply_stats* out) try {
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
} catch (...) {
    return sydelta::host_exception();
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
extern "C" int sydelta_synth_fill(uint8_t* d_buf, uint64_t len, uint64_t seed, void* stream) try {
    if (len && !d_buf) return fail(SYDELTA_E_INVAL, "NULL buffer");
    int dev = 0;
    (void)hipGetDevice(&dev);
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    HIP_TRY(launch_synth_fill(d_buf, len, seed, s));
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_synth_fill_range(uint8_t* d_buf, uint64_t first, uint64_t len, uint64_t seed, void* stream) try {
    if (len && !d_buf) return fail(SYDELTA_E_INVAL, "NULL buffer");
    if (first % 8) return fail(SYDELTA_E_INVAL, "first must be a multiple of 8");
    int dev = 0;
    (void)hipGetDevice(&dev);
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    HIP_TRY(launch_synth_fill(d_buf, len, seed, s, first));
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_synth_mutate_blocks(uint8_t* d_dst, const uint8_t* d_src, uint64_t first, uint64_t len,
                                           uint64_t block_size, uint64_t seed, uint32_t rate_ppm, void* stream) try {
    if (len && (!d_dst || !d_src)) return fail(SYDELTA_E_INVAL, "NULL buffer");
    if (!block_size || first % block_size) return fail(SYDELTA_E_INVAL, "first must be a multiple of block_size");
    int dev = 0;
    (void)hipGetDevice(&dev);
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    if (len && d_dst != d_src) HIP_TRY(hipMemcpyAsync(d_dst, d_src, len, hipMemcpyDeviceToDevice, s));
    HIP_TRY(launch_synth_edit_blocks(d_dst, len, block_size, first, seed, rate_ppm, s));
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_synth_mutate(uint8_t* d_dst, const uint8_t* d_src, uint64_t len, uint64_t seed,
                                    uint32_t rate_ppm, void* stream) try {
    if (len && (!d_dst || !d_src)) return fail(SYDELTA_E_INVAL, "NULL buffer");
    int dev = 0;
    (void)hipGetDevice(&dev);
    SYDELTA_ENTER_DEVICE(dev);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(dev);
    HIP_TRY(launch_synth_mutate(d_dst, d_src, len, seed, rate_ppm, s));
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

// ---------------------------------------------------------------------------
// chunk-sharded match of one file (BASELINE C5)
// ---------------------------------------------------------------------------
// Rank g classifies the window starts of its chunk [pos_begin, pos_end) against the
// all-gathered signature; the walks are then chained: chunk g's walk starts where
// chunk g-1's left (its exit may lie up to n-1 bytes inside chunk g after a Copy),
// and the op lists concatenate with sydelta_delta_append.  The result equals the
// single-device op list because classification is a pure function of the position.
namespace {
// K10 over a chunk, launched by sydelta_chunk_classify (chunk_pipe_launch): sub-range j's
// aligned probe on the caller's stream, then its walk on the thread's aux stream after an
// event, the walk's per-unit results and records written straight into host-mapped
// memory.  sydelta_chunk_walk waits for the sub-ranges in turn and assembles each one's
// ops while the later ones still run (chunk_pipe_finish).
struct ChunkPipe {
    bool on = false;
    int device = 0;
    std::vector<WalkUnit> units;   // from the segment starts
    std::vector<uint32_t> ub;      // sub-range j: units [ub[j], ub[j+1])
    std::vector<hipEvent_t> done;  // per sub-range: its walk finished (results readable)
    void* dmem = nullptr;          // the unit table and the probe's results (device)
    hipStream_t ds = nullptr;      // dmem's stream (the caller's)
    PinnedHits pin;                // host-mapped (kMapped): per-unit results, records
    PinnedHits stage;              // the uploads' source (kStage)
    const WalkFileOut* fout = nullptr;
    const WalkRec* rec = nullptr;
    const WalkUnit* d_units = nullptr;  // the unit table and the staged records (device), for
    const WalkRec* d_stage = nullptr;   // the ops written on the device (launch_chunk_write)
    const uint32_t* ahit = nullptr;  // the probe's results (device; NULL: no probe)
    const uint32_t* apw = nullptr;
    unsigned long long* ticks = nullptr;  // SYDELTA_PHASE_TIMING: 16 counters per part (device)
    void release() {  // the chunk's device is current
        for (hipEvent_t e : done) {  // the parts' walks
            (void)hipEventSynchronize(e);
            give_event(device, e);
        }
        done.clear();
        if (dmem) (void)hipFreeAsync(dmem, ds);
        dmem = nullptr;
        give_mapped(pin);
        pin = PinnedHits();
        give_mapped(stage, kStage);
        stage = PinnedHits();
        on = false;
    }
    ~ChunkPipe() { release(); }
};
}  // namespace

struct sydelta_chunk {
    Classifier C;
    bool final_src = false;
    int tail_flag = 0;
    uint64_t file_len = 0;
    BasisInfo bi{0, 0, 0};
    bool dev_walk = false;  // K10 over the chunk's segments (ChunkPipe)
    ChunkPipe pipe;         // destroyed before C (whose buffers its launches read)
};

// K10 over a chunk (C5, and the streamed path API's chunks): the aligned probe's results
// stay on the device and the walk runs there, one wave per segment of chunk_seg_blocks()
// blocks, each from its segment's start; a segment whose true entry (the previous one's
// exit) differs is walked again from it (after a Copy that crosses the boundary).
// SYDELTA_CHUNK_WALK=0, or SYDELTA_PROBE=0, keeps the classifier + host walk.
namespace {
// blocks per segment of the last part of a pipelined chunk, whose walk ends the pipeline:
// SYDELTA_CHUNK_SEG_LAST, else as short as keeps the part within ~3300 units (one round of
// the chip's 4096 wave slots, beside the first part's last waves), at least 32.  At C5 (the
// last 30 %: 315 K blocks): 96 blocks 4.105-4.112 ms per step, 80: 4.20-4.23, 64 (two
// rounds): 4.19-4.33, 128: 4.22-4.33 (`profiles/r05zz9_*`).
uint64_t chunk_seg_blocks();
uint64_t chunk_seg_last_blocks(uint64_t last_blocks, int device) {
    const char* e = getenv("SYDELTA_CHUNK_SEG_LAST");  // (knobs are read per call: tests switch them)
    const uint64_t x = (e && *e) ? strtoull(e, nullptr, 10) : 0;
    const uint64_t forced = (x >= 8 && x <= 1024) ? x : 0;
    const uint64_t round = std::max<uint64_t>(1, wave_slots(device) * 4 / 5);  // 3276 units at 4096 slots
    const uint64_t v = forced ? forced : std::max<uint64_t>(32, (last_blocks + round - 1) / round);
    return std::min(v, chunk_seg_blocks());
}
// blocks per segment (SYDELTA_CHUNK_SEG overrides; a power of two from 8 to 1024)
uint64_t chunk_seg_blocks() {
    const char* e = getenv("SYDELTA_CHUNK_SEG");
    const uint64_t x = (e && *e) ? strtoull(e, nullptr, 10) : 128;
    return (x >= 8 && x <= 1024 && (x & (x - 1)) == 0) ? x : (uint64_t)128;
}
bool chunk_walk_ok(const sydelta_index* idx) {
    const char* e = getenv("SYDELTA_CHUNK_WALK");
    if (e && e[0] == '0') return false;
    const uint64_t n = idx->bs;
    return idx->nfiles == 1 && n % 64 == 0 && n >= 256 && n <= kWalkMaxN && probe_mode_env() != 0;
}

// The units of a chunk's walk from `from`: the segments of [from, c.p1), the last one final
// when the file ends in the chunk.
// (appended to `units`, segments of seg_blocks blocks from the chunk start's grid;
// record offsets continue from the last unit's)
void chunk_units(const sydelta_chunk* ch, uint64_t from, std::vector<WalkUnit>& units, uint64_t seg_blocks = 0) {
    const Src& c = ch->C.src[0];
    const uint64_t n = ch->C.n, seg = (seg_blocks ? seg_blocks : chunk_seg_blocks()) * n;
    uint64_t rec = units.empty() ? 0 : units.back().rec_off + 2 * ((units.back().end - units.back().entry) / n) + 4;
    const uint64_t lo = std::max(from, c.p0);
    uint64_t s0 = c.p0 + (lo > c.p0 ? (lo - c.p0) / seg * seg : 0);
    do {
        const uint64_t e = std::min(c.p1, s0 + seg), en = std::max(lo, s0);
        const bool last = e >= c.p1;
        // len: the readable end of the chunk's buffer (c.len), which bounds the walk's loads; the
        // final unit's is the file's length (its tail rule and last literal run need it)
        units.push_back(WalkUnit{0, c.len, en, std::max(e, en), c.p1, rec, c.kb, 0,
                                 (uint32_t)(last && ch->final_src)});
        rec += 2 * ((std::max(e, en) - en) / n) + 4;
        s0 = e;
    } while (s0 < c.p1);
}

// The pre-roll of a chunk's aligned misses before the last part's walk (launch_preroll): one
// wave per miss rolls it, so that walk, which ends the pipeline, takes each miss's result
// instead of rolling its misses in turn.  SYDELTA_PREROLL=0: off; 2: before every part's
// walk.  Its grid: the device's wave slots.
bool preroll_on() {
    const char* e = getenv("SYDELTA_PREROLL");
    return !e || e[0] != '0';
}
bool preroll_all() {  // SYDELTA_PREROLL=2: every part's (else the last part's: the others' walks are hidden)
    const char* e = getenv("SYDELTA_PREROLL");
    return e && e[0] == '2';
}
bool slim_walk() {  // SYDELTA_SLIM_WALK=0: a pre-rolled part walked by the full kernel alone
    const char* e = getenv("SYDELTA_SLIM_WALK");
    return !e || e[0] != '0';
}

// Sub-ranges of a chunk's walk: 2 from 512 segments (SYDELTA_CHUNK_PIPE=K).  At C5 (8192
// segments) two parts took 4.43-4.51 ms per step, one 4.82-4.88 and four 4.96-5.00: the
// second part's hashing hides the first part's walk, while each further part adds a walk
// launch whose last round runs under-filled (`profiles/r05r_*`).
int chunk_pipe_parts(size_t nu) {
    const char* e = getenv("SYDELTA_CHUNK_PIPE");
    int K = (e && *e) ? std::max(1, atoi(e)) : nu >= 512 ? 2 : 1;
    return (int)std::min<size_t>((size_t)K, nu);
}

// Launch the walk of ch from `from` (with the aligned probe first: from is c.p0), in
// sub-ranges pipelined over two streams (ChunkPipe).
int chunk_pipe_launch(sydelta_chunk* ch, uint64_t from, bool probe) {
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t_begin = std::chrono::steady_clock::now();
    Classifier& C = ch->C;
    const Src& c = C.src[0];
    ChunkPipe& P = ch->pipe;
    const uint64_t n = C.n;
    P.units.clear();
    chunk_units(ch, from, P.units);
    size_t nu = P.units.size();
    const uint64_t np = probe ? c.nblk : 0;
    const int K = probe ? chunk_pipe_parts(nu) : 1;
    P.ub.resize(K + 1);
    for (int j = 0; j <= K; ++j) P.ub[j] = (uint32_t)(nu * j / K);
    // two parts: 70 % / 30 % (the second part's hashing hides the first part's walk, and its
    // own walk, which ends the pipeline, is the shorter: 4.11-4.12 ms per step at C5 against
    // 4.26-4.43 for halves, `profiles/r05zs_*`, `r05zt_*`)
    if (K == 2) P.ub[1] = (uint32_t)std::min<uint64_t>(nu - 1, std::max<uint64_t>(1, nu * 7 / 10));
    // the last part, whose walk ends the pipeline, in shorter segments (its waves finish sooner)
    const uint64_t seg_last = K >= 2 ? chunk_seg_last_blocks((c.p1 - P.units[P.ub[K - 1]].entry + n - 1) / n, C.ix->device)
                                     : chunk_seg_blocks();
    if (K >= 2 && seg_last < chunk_seg_blocks()) {
        const uint64_t split = P.units[P.ub[K - 1]].entry;
        P.units.resize(P.ub[K - 1]);
        chunk_units(ch, split, P.units, seg_last);
        nu = P.units.size();
        P.ub[K] = (uint32_t)nu;
    }
    uint64_t rec_total = 0;
    for (const WalkUnit& u : P.units) rec_total = std::max(rec_total, u.rec_off + 2 * ((u.end - u.entry) / n) + 4);
    if (rec_total >= (1ull << 32)) return fail(SYDELTA_E_INVAL, "chunk too large for one walk");
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    // device: the probe jobs, the last size and the record counter (uploaded first, for the
    // hashing), the unit table (uploaded once the first hashing is queued), the probe's
    // results, the staged records; host: the per-unit results and the compacted records
    // (kMapped), the uploads' source (kStage, same offsets as the device's)
    // (the pre-roll's: per part a miss counter, zeroed with the record counter; the miss
    // list and the first hits)
    const bool preroll = probe && preroll_on() && C.ix->fblk[1] < kPreMark;
    const size_t o_jobs = 0, o_last = al(sizeof(ProbeJob) * K), o_total = o_last + 8, o_cnt = o_total + 8;
    static const bool timing = getenv("SYDELTA_PHASE_TIMING") != nullptr;  // per part: 16 tick counters
    const size_t o_ticks = o_cnt + 8 * K, o_zend = o_ticks + (timing ? 128 * K : 0);
    const size_t o_units = al(o_zend);
    const size_t ubytes = sizeof(WalkUnit) * nu;
    const size_t o_out = o_units + al(ubytes), o_pw = o_out + al(4 * np), o_pst = o_pw + al(4 * np);
    const size_t o_list = o_pst + al(8 * np);
    const size_t o_stage = o_list + (preroll ? al(4 * np) : 0), dneed = o_stage + al(sizeof(WalkRec) * rec_total);
    const size_t h_rec = al(sizeof(WalkFileOut) * nu), h_end = h_rec + al(sizeof(WalkRec) * rec_total);
    P.on = true;  // release() undoes whatever is set below
    P.device = C.ix->device;
    P.ds = C.s;
    if (int r = take_mapped(h_end, P.pin)) return r;
    if (int r = take_mapped(o_units + ubytes, P.stage, kStage)) return r;
    HIP_TRY(dev_malloc_async(&P.dmem, dneed, C.s));
    uint8_t* H = P.pin.p;
    uint8_t* S = P.stage.p;
    uint8_t* D = (uint8_t*)P.dmem;
    P.fout = (const WalkFileOut*)H;
    P.rec = (const WalkRec*)(H + h_rec);
    P.d_units = (const WalkUnit*)(D + o_units);
    P.d_stage = (const WalkRec*)(D + o_stage);
    uint32_t* d_out = (uint32_t*)(D + o_out);
    uint32_t* d_pw = (uint32_t*)(D + o_pw);
    uint64_t* d_pst = (uint64_t*)(D + o_pst);
    P.ahit = probe ? d_out : nullptr;
    P.apw = probe ? d_pw : nullptr;
    // the jobs, the last size and the zeroed counter up (the staging buffer outlives the copies)
    ProbeJob* jobs = (ProbeJob*)(S + o_jobs);
    auto part_block = [&](int j) -> uint64_t {  // part j's first block (relative to the chunk's)
        return j < K ? (P.units[P.ub[j]].entry - c.p0) / n : np;
    };
    for (int j = 0; j < K; ++j) jobs[j] = ProbeJob{c.off, c.kb + part_block(j), 0, 0, 0};
    *(uint64_t*)(S + o_last) = C.ix->last_size[0];
    memset(S + o_total, 0, o_zend - o_total);
    HIP_TRY(hipMemcpyAsync(D, S, o_zend, hipMemcpyHostToDevice, C.s));
    P.ticks = timing ? (unsigned long long*)(D + o_ticks) : nullptr;
    bool units_up = false;
    auto upload_units = [&]() -> int {
        if (units_up) return SYDELTA_OK;
        units_up = true;
        memcpy(S + o_units, P.units.data(), ubytes);
        HIP_TRY(hipMemcpyAsync(D + o_units, S + o_units, ubytes, hipMemcpyHostToDevice, C.s));
        return SYDELTA_OK;
    };
    // (the second: the aux stream, idle once the index is built; a fifth stream would share
    // one of the process's four hardware queues with another and serialize behind it)
    hipStream_t s2[2] = {thread_walk_stream(P.device, 0), thread_aux_stream(P.device)};
    hipEvent_t hand = handoff_event(P.device);
    if (!s2[0] || !s2[1] || !hand) return fail(SYDELTA_E_OOM, "no stream or event for the chunk walk");
    const bool fast = ((uintptr_t)(C.base + c.off) & 15) == 0;
    WalkArgs a{};
    a.base = C.base;
    a.last_size = (const uint64_t*)(D + o_last);
    a.n = (uint32_t)n;
    a.nm = (uint32_t)(n % 65521);
    a.self_nb = 0;  // the index's filter and tables from L2 (one file's are too large for LDS)
    const DeviceIndex& ix = C.ix->ix;
    a.files = ix.d_files;
    a.fblk = ix.d_fblk;
    a.filt = ix.filt;
    a.keys = ix.keys;
    a.start = ix.start;
    a.cnt = ix.cnt;
    a.order = ix.order;
    a.cstrong = ix.cstrong;
    a.weak = C.ix->d_weak;
    a.strong = C.ix->d_strong;
    a.ahit = P.ahit;
    a.apw = P.apw;
    // records staged on the device, compacted into host memory (read in order by the
    // assembly: staged there, one unit's per 4 KiB page, they cost a TLB miss each)
    a.stage = (WalkRec*)(D + o_stage);
    a.out = (WalkRec*)(H + h_rec);
    // one record counter for every part: the parts' walks run on two streams at once, and the
    // device-scope atomics give each unit a disjoint range of out; take() copies a part's
    // [lo, hi) only after that part's walk finished (ranges of a part still walking may lie
    // inside it, but are never read from the copy)
    a.total = (unsigned long long*)(D + o_total);
    a.ticks = nullptr;
    auto probe_part = [&](int j, int phases) -> hipError_t {
        const uint64_t b0 = part_block(j), b1 = std::min<uint64_t>(part_block(j + 1), np);
        return launch_probe(C.base, (const ProbeJob*)(D + o_jobs) + j, 1, b1 - b0, 1, (uint32_t)n, fast, ix,
                            d_pw + b0, d_pst + b0, d_out + b0, C.s, C.prof, phases);
    };
    // per sub-range: its windows hashed, looked up (after the index: one built from device
    // arrays may still be building on the aux stream, and the first hashing overlaps it), and
    // walked on the aux stream while the next sub-range is hashed
    for (int j = 0; j < K; ++j) {
        if (probe) HIP_TRY(probe_part(j, 1));
        if (int r = upload_units()) return r;  // after the first hashing is queued
        if (j == 0) HIP_TRY(index_wait(C.ix, C.s));
        if (probe) HIP_TRY(probe_part(j, 2));
        hipStream_t sw = s2[j & 1];
        HIP_TRY(hipEventRecord(hand, C.s));
        HIP_TRY(hipStreamWaitEvent(sw, hand, 0));
        hipEvent_t e = take_event(P.device);
        if (!e) return fail(SYDELTA_E_OOM, "no event for the chunk walk");
        P.done.push_back(e);
        a.units = (const WalkUnit*)(D + o_units) + P.ub[j];
        a.nunits = P.ub[j + 1] - P.ub[j];
        a.fout = (WalkFileOut*)P.fout + P.ub[j];
        a.ticks = P.ticks ? P.ticks + 16 * j : nullptr;
        if (preroll && (j == K - 1 || preroll_all())) {
            const uint64_t b0 = part_block(j), b1 = std::min<uint64_t>(part_block(j + 1), np);
            HIP_TRY(launch_preroll(a, d_out, d_pw, c.kb, b0, b1, c.p1, c.len,
                                   (uint32_t*)(D + o_list) + b0, (unsigned long long*)(D + o_cnt) + j, wave_slots(P.device),
                                   std::max<uint64_t>(64, (b1 - b0) / 16),
                                   sw, C.prof));
            if (slim_walk()) HIP_TRY(launch_walk_files(a, sw, C.prof, true));
        }
        HIP_TRY(launch_walk_files(a, sw, C.prof));
        HIP_TRY(hipEventRecord(e, sw));
    }
    if (host_timing) fprintf(stderr, "sydelta chunk launch: %zu segments, %d parts: %.3f ms\n", nu, K, ms_since(t_begin));
    return SYDELTA_OK;
}

// The chunk's ops from `entry`: the segments in order, each sub-range as soon as its walk
// finished.  A segment whose entry differs from the previous one's exit (a Copy crossed
// the boundary) stops the overlap: it and every later one whose entry changed are walked
// again (in one launch per round; a shifted source keeps its phase, so a round or two),
// then assembled.  A Data op ending at a segment's end is joined with the next segment's
// first Data op (literal runs stay maximal, generator.rs:186-197).
int chunk_pipe_finish(sydelta_chunk* ch, uint64_t entry, uint64_t* exit_pos, sydelta_delta* d) {
    static const bool host_timing = getenv("SYDELTA_HOST_TIMING") != nullptr;
    const auto t_begin = std::chrono::steady_clock::now();
    // the re-walks' records (run_walk's WalkResult) live in this thread's walk scratch until
    // they are copied out below: sydelta_trim must not release it in between
    ScratchHold hold;
    Classifier& C = ch->C;
    ChunkPipe& P = ch->pipe;
    const uint64_t n = C.n;
    std::vector<WalkUnit> units = P.units;  // re-walks move entries (the launch's stay for a later call)
    const size_t nu = units.size();
    size_t u0 = 0;  // the segment holding entry
    while (u0 + 1 < nu && units[u0].end <= entry) ++u0;
    uint64_t cap = 0;  // ops per unit: at most a Copy per block, a Data op before each, a tail Copy
    for (size_t u = u0; u < nu; ++u) cap += 2 * ((units[u].end - units[u].entry) / n) + 8;
    OpVec& ops = d->ops;
    // the last part's ops -- the pipeline's tail -- written on the device (launch_chunk_write:
    // the host only chains the units and plans each one's ops) into an op array reserved from
    // a pinned host-mapped slab; the other parts' assembled on the host behind the next part's
    // walk.  Writing every part on the device (SYDELTA_DEVICE_EXPAND=1) lets part 1's PCIe
    // writes slow part 2's pre-roll: the N = 8 proxy rank at 2 host threads 7.05-7.13 ms
    // against 6.83-6.84 (`profiles/r06z_*`); 0: every part on the host.
    const char* dxe = getenv("SYDELTA_DEVICE_EXPAND");
    const bool dev_set = dxe && *dxe;
    const bool dev_all = dev_set && dxe[0] == '1';
    const bool dev_last = (!dev_set || dxe[0] == '2') && P.ub.size() > 2;
    const bool want_dev = P.d_units && P.d_stage && (dev_all || dev_last);
    bool cdev = false;
    if (want_dev) {
        if (OpSlab* slab = slab_open(cap * sizeof(sydelta_op))) {
            OpVec v;
            v.reserve(cap);
            cdev = (uint8_t*)v.data() == slab->p;
            slab_close(slab);
            if (cdev) ops.swap(v);
        }
    }
    if (!cdev && ops.capacity() < cap) ops = take_ops(cap);
    ops.resize(cap);
    CxPlan* plan_h = nullptr;  // per unit (staging), and its device copy
    CxPlan* plan_d = nullptr;
    PinnedHits plan_pin;
    struct PlanFree {
        CxPlan*& d;
        PinnedHits& h;
        hipStream_t s;
        ~PlanFree() {
            if (d) (void)hipFreeAsync(d, s);
            give_mapped(h, kStage);
        }
    } plan_free{plan_d, plan_pin, C.s};
    if (cdev) {
        if (int r = take_mapped(sizeof(CxPlan) * nu, plan_pin, kStage)) return r;
        HIP_TRY(dev_malloc_async((void**)&plan_d, sizeof(CxPlan) * nu, C.s));
        plan_h = (CxPlan*)plan_pin.p;
    }
    bool dev_pending = false;  // device writes queued on C.s
    std::vector<std::pair<uint64_t, uint64_t>> patches;  // (op, bytes) added once the device's writes are done
    std::vector<const WalkRec*> orig(nu, nullptr);  // each unit's first record in the host copy
    std::vector<uint8_t> cut(nu, 0);  // its first record cut (joins)
    size_t owner = SIZE_MAX;           // the unit holding the last op planned so far
    const double ms_ops = ms_since(t_begin);
    double ms_asm = 0;
    std::vector<WalkFileOut> out(nu);
    std::vector<std::pair<const WalkRec*, const WalkRec*>> span(nu);
    std::vector<std::vector<WalkRec>> again_rec;  // re-walked units' records
    const uint64_t nbf = C.ix->fblk[1], ls = C.ix->last_size[0];
    uint64_t nops = 0, data_ops = 0, lit = 0, hits = 0, weak = 0;
    // assembly threads: SYDELTA_ASM_THREADS, else the host pool and the caller (C5's 1 Mi ops:
    // 0.46-0.58 ms on 16 + 1 threads, 0.78-0.92 on 8, `profiles/r05s_*`)
    const int pool = asm_threads_env();
    double ms_wait = 0;
    // units [a, b) after ops [0, nops)
    auto assemble = [&](size_t a, size_t b) -> int {
        if (b <= a) return SYDELTA_OK;
        const auto ta = std::chrono::steady_clock::now();
        std::vector<uint64_t> first(b - a + 1, nops);
        std::vector<uint8_t> join(b - a, 0);
        for (size_t u = a; u < b; ++u) {
            const WalkRec *r0 = span[u].first, *r1 = span[u].second;
            uint64_t k = records_ops(r0, r1);
            if (u > u0 && r0 < r1 && !r0->kind && span[u - 1].second > span[u - 1].first) {
                const WalkRec* pl = span[u - 1].second - 1;
                if (!pl->kind && pl->off + pl->a == r0->off) {
                    join[u - a] = 1;
                    --k;
                }
            }
            first[u - a + 1] = first[u - a] + k;
            hits += out[u].hits;
            weak += out[u].weak_hits;
        }
        if (first.back() > ops.size())
            return fail(SYDELTA_E_KERNEL, "chunk walk: %llu ops above the bound %llu", (unsigned long long)first.back(),
                        (unsigned long long)ops.size());
        const size_t m = b - a;
        const int nt = first.back() - nops >= (1u << 15) ? (int)std::min<size_t>(m, (size_t)pool) : 1;
        std::vector<uint64_t> nd(nt, 0), lb(nt, 0);
        if (!run_parallel(nt, [&](int t) {
                for (size_t u = a + m * t / nt; u < a + m * (t + 1) / nt; ++u) {
                    const WalkRec* r0 = span[u].first + join[u - a];
                    expand_records<true>(r0, span[u].second, n, 0, nbf, ls, ops.data() + first[u - a], &nd[t],
                                         &lb[t]);
                }
                _mm_sfence();  // the streamed ops visible before the task reports done
            }))
            return fail(SYDELTA_E_OOM, "out of host memory (op lists)");
        for (int t = 0; t < nt; ++t) {
            data_ops += nd[t];
            lit += lb[t];
        }
        for (size_t u = a; u < b; ++u)
            if (join[u - a]) {
                const uint64_t add = span[u].first->a;
                ops[first[u - a] - 1].b += add;  // the previous unit's last op
                lit += add;
            }
        nops = first.back();
        ms_asm += ms_since(ta);
        return SYDELTA_OK;
    };
    // the results of units [a, b) out of the mapped buffer: copied in two block moves
    double ms_take = 0;
    auto take = [&](size_t a, size_t b) {
        if (b <= a) return;
        const auto tt = std::chrono::steady_clock::now();
        memcpy(out.data() + a, P.fout + a, sizeof(WalkFileOut) * (b - a));
        const WalkRec* base = P.rec;
        uint64_t lo = UINT64_MAX, hi = 0;
        for (size_t u = a; u < b; ++u)
            if (out[u].count) {
                lo = std::min<uint64_t>(lo, out[u].base);
                hi = std::max<uint64_t>(hi, (uint64_t)out[u].base + out[u].count);
            }
        if (hi > lo) {
            again_rec.emplace_back(P.rec + lo, P.rec + hi);
            base = again_rec.back().data();
        } else {
            lo = 0;
        }
        for (size_t u = a; u < b; ++u) {  // (a unit with no records: an empty span anywhere)
            const WalkRec* r = out[u].count ? base + (out[u].base - lo) : base;
            span[u] = {r, r + out[u].count};
            orig[u] = r;
        }
        ms_take += ms_since(tt);
    };
    // Unit u's walk holds from pe, the true entry (the previous unit's exit, or `entry`), when
    // it started there, or earlier with a leading literal run that reaches pe: the greedy walk
    // from pe then classifies the same positions the same way (a shifted source's segments,
    // whose previous Copy crosses the boundary by the shift) -- its leading Data op is cut to
    // start at pe (dropped when it ends there).  Otherwise it is walked again from pe.
    auto joins = [&](size_t u, uint64_t pe) -> bool {
        if (units[u].entry == pe) return true;
        const WalkRec* r0 = span[u].first;
        if (pe < units[u].entry || r0 >= span[u].second || r0->kind || r0->off != units[u].entry ||
            r0->off + r0->a < pe)
            return false;
        WalkRec* w = const_cast<WalkRec*>(r0);  // (our copy of the unit's records, take())
        if (w->off + w->a == pe) {
            ++span[u].first;
        } else {
            w->a = (uint32_t)(w->off + w->a - pe);
            w->off = pe;
            cut[u] = 1;
        }
        units[u].entry = pe;
        return true;
    };
    // units [a, b) planned (the host's assemble rules, same counts) and written on the device
    auto plan_part = [&](size_t a, size_t b) -> int {
        if (b <= a) return SYDELTA_OK;
        const auto ta = std::chrono::steady_clock::now();
        for (size_t u = a; u < b; ++u) {
            const WalkRec *r0 = span[u].first, *r1 = span[u].second;
            uint64_t k = 0, nd = 0, lb = 0;
            for (const WalkRec* r = r0; r < r1; ++r) {
                if (r->kind) {
                    k += r->kind;
                } else {
                    ++k;
                    ++nd;
                    lb += r->a;
                }
            }
            bool join = false;
            if (u > u0 && r0 < r1 && !r0->kind && span[u - 1].second > span[u - 1].first) {
                const WalkRec* pl = span[u - 1].second - 1;
                join = !pl->kind && pl->off + pl->a == r0->off;
            }
            CxPlan& pu = plan_h[u];
            const uint32_t s0 = (uint32_t)(r0 - orig[u]);
            pu = CxPlan{nops, 0, 0, 0, out[u].count, s0 + (join ? 1u : 0u), 0};
            if (!join && cut[u] && s0 == 0 && r0 < r1) {
                pu.flags = 1;
                pu.r0_off = r0->off;
                pu.r0_a = r0->a;
            }
            if (join) {  // into the last op so far (a Data op): its unit's, or a patch after the writes
                --k;
                --nd;
                if (owner != SIZE_MAX && owner >= a)
                    plan_h[owner].ext += r0->a;
                else
                    patches.emplace_back(nops - 1, (uint64_t)r0->a);
            }
            data_ops += nd;
            lit += lb;
            hits += out[u].hits;
            weak += out[u].weak_hits;
            nops += k;
            if (k) owner = u;
        }
        if (nops > ops.size())
            return fail(SYDELTA_E_KERNEL, "chunk walk: %llu ops above the bound %llu", (unsigned long long)nops,
                        (unsigned long long)ops.size());
        HIP_TRY(hipMemcpyAsync(plan_d + a, plan_h + a, sizeof(CxPlan) * (b - a), hipMemcpyHostToDevice, C.s));
        HIP_TRY(launch_chunk_write(P.d_units + a, P.d_stage, plan_d + a, (uint32_t)(b - a), (uint32_t)n, nbf, ls,
                                   ops.data(), C.s, C.prof));
        dev_pending = true;
        ms_asm += ms_since(ta);
        return SYDELTA_OK;
    };
    // the device's writes done, then the joins into ops they wrote
    auto dev_finish = [&]() -> int {
        if (!dev_pending) return SYDELTA_OK;
        dev_pending = false;
        HIP_TRY(hipStreamSynchronize(C.s));
        for (const auto& pt : patches) ops[pt.first].b += pt.second;
        patches.clear();
        return SYDELTA_OK;
    };
    size_t stop = nu;  // the first unit whose entry is not the previous one's exit
    for (size_t j = 0; j + 1 < P.ub.size() && stop == nu; ++j) {
        const size_t a = std::max<size_t>(P.ub[j], u0), b = P.ub[j + 1];
        if (b <= a) continue;
        const auto tw = std::chrono::steady_clock::now();
        HIP_TRY(hipEventSynchronize(P.done[j]));
        ms_wait += ms_since(tw);
        take(a, b);
        size_t e = a;
        while (e < b && joins(e, e == u0 ? entry : out[e - 1].exit)) ++e;
        const bool part_dev = cdev && (dev_all || j + 2 == P.ub.size());
        if (int r = part_dev ? plan_part(a, e) : assemble(a, e)) return r;
        if (e < b) stop = e;
    }
    int rounds = 0;
    if (stop < nu) {
        if (int r = dev_finish()) return r;  // (the host's assembly below may join into the device's last op)
        for (hipEvent_t e : P.done) HIP_TRY(hipEventSynchronize(e));
        take(P.ub[std::upper_bound(P.ub.begin(), P.ub.end(), (uint32_t)stop) - P.ub.begin()], nu);  // later sub-ranges
        for (;;) {
            std::vector<size_t> bad;
            std::vector<WalkUnit> again;
            uint64_t roff = 0;
            for (size_t u = stop; u < nu; ++u) {
                const uint64_t ex = u == u0 ? entry : out[u - 1].exit;  // a Copy reaches < n bytes past a boundary
                if (joins(u, ex)) continue;
                units[u].entry = ex;
                units[u].end = std::max(units[u].end, ex);
                WalkUnit w = units[u];
                w.rec_off = roff;
                roff += 2 * ((w.end - w.entry) / n) + 4;
                again.push_back(w);
                bad.push_back(u);
            }
            if (bad.empty()) break;
            ++rounds;
            WalkResult r1;
            if (int r = run_walk(C.ix, C.base, again, P.ahit, P.apw, false, C.s, C.prof, r1)) return r;
            for (size_t j = 0; j < bad.size(); ++j) {
                const size_t u = bad[j];
                const WalkRec* q = r1.rec + r1.out[j].base;
                again_rec.emplace_back(q, q + r1.out[j].count);
                span[u] = {again_rec.back().data(), again_rec.back().data() + again_rec.back().size()};
                out[u] = r1.out[j];
            }
        }
        if (int r = assemble(stop, nu)) return r;
    }
    if (int r = dev_finish()) return r;
    if (P.ticks) {
        std::vector<unsigned long long> tk(16 * P.done.size());
        HIP_TRY(hipMemcpy(tk.data(), P.ticks, 8 * tk.size(), hipMemcpyDeviceToHost));
        for (size_t j = 0; j < P.done.size(); ++j) {
            const unsigned long long* t = tk.data() + 16 * j;
            fprintf(stderr, "sydelta chunk walk part %zu (%u units; wave ticks, 100 MHz, summed): setup %llu hash %llu "
                    "lookup %llu stage %llu roll %llu verify %llu out %llu | passes %llu windows %llu rolls %llu\n", j,
                    P.ub[j + 1] - P.ub[j], t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[8], t[9], t[10]);
        }
    }
    ops.resize(nops);
    d->stats.data_ops = data_ops;
    d->stats.copy_ops = nops - data_ops;
    d->stats.literal_bytes = lit;
    d->stats.verified_hits = hits;
    d->stats.weak_hits = weak;
    *exit_pos = out[nu - 1].exit;
    if (host_timing)
        fprintf(stderr, "sydelta chunk walk: %zu segments in %zu parts, %d re-walk rounds, %llu ops%s: op array %.3f ms, "
                "waits %.3f ms, results %.3f ms, assembly %.3f ms, all %.3f ms\n", nu, P.done.size(), rounds,
                (unsigned long long)nops, cdev ? " (written on the device)" : "", ms_ops, ms_wait, ms_take, ms_asm,
                ms_since(t_begin));
    return SYDELTA_OK;
}
}  // namespace

extern "C" int sydelta_chunk_classify(sydelta_index* idx, const uint8_t* d_buf, uint64_t buf_pos, uint64_t buf_len,
                                      uint64_t file_len, uint64_t pos_begin, uint64_t pos_end, void* stream,
                                      sydelta_chunk** out) try {
    if (!idx || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = nullptr;
    if (idx->nfiles != 1) return fail(SYDELTA_E_INVAL, "chunked match needs a single-file index");
    const uint64_t n = idx->bs;
    const uint64_t npos = file_len >= n ? file_len - n + 1 : 0;
    // a chunk at or past the last window start is empty (it may still own the tail)
    if (pos_begin < npos && pos_begin % n) return fail(SYDELTA_E_INVAL, "pos_begin must be a multiple of block_size");
    if (pos_end < pos_begin && pos_begin < npos) return fail(SYDELTA_E_INVAL, "pos_end < pos_begin");
    if ((buf_pos & 15) || ((uintptr_t)d_buf & 15))
        return fail(SYDELTA_E_INVAL, "d_buf and buf_pos must be 16-byte aligned");
    if (buf_pos > (std::min(pos_begin, npos) & ~15ull)) return fail(SYDELTA_E_INVAL, "buffer starts after the chunk");
    const bool final_src = pos_end >= npos;
    const uint64_t p1 = std::min(pos_end, npos), p0 = std::min(pos_begin, p1);
    const uint64_t need_end = final_src ? file_len : std::min(file_len, p1 + n - 1);
    if ((p1 > p0 || final_src) && buf_pos + buf_len < need_end)
        return fail(SYDELTA_E_INVAL, "buffer ends at %llu, chunk needs bytes up to %llu",
                    (unsigned long long)(buf_pos + buf_len), (unsigned long long)need_end);
    if (buf_len && !d_buf) return fail(SYDELTA_E_INVAL, "NULL buffer");
    SYDELTA_ENTER_DEVICE(idx->device);
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream(idx->device);
    std::unique_ptr<sydelta_chunk> ch(new sydelta_chunk());
    CallProf cp;
    Classifier& C = ch->C;
    C.ix = idx;
    C.base = d_buf - buf_pos;
    C.s = s;
    C.prof = cp.get();
    C.n = n;
    C.src.resize(1);
    C.adopt_spare();
    Src& c = C.src[0];
    c.file = 0;
    c.off = 0;
    c.len = std::min(file_len, buf_pos + buf_len);
    c.flen = file_len;
    const bool has_sig = idx->fblk[1] > 0;
    c.p0 = p0;
    c.p1 = has_sig ? p1 : p0;
    c.kb = p0 / n;
    c.nblk = c.p1 > c.p0 ? (c.p1 + n - 1) / n - c.kb : 0;
    ch->final_src = final_src;
    ch->file_len = file_len;
    ch->bi = BasisInfo{0, idx->fblk[1], idx->last_size[0]};
    if (chunk_walk_ok(idx)) {  // K10 walks the chunk on the device: probe and walk launched here
        ch->dev_walk = true;
        if (c.p1 > c.p0)  // (the index is waited for between the probe's hashing and its lookups)
            if (int r = chunk_pipe_launch(ch.get(), c.p0, true)) return r;
        C.prof = nullptr;
        *out = ch.release();
        return SYDELTA_OK;
    }
    HIP_TRY(index_wait(idx, s));
    // windows above the LDS scans' limit without k_scan_g: every position scanned (k_scan,
    // one launch per range), no probe, as match_impl does
    if (int r = C.classify(n > scan_max_window() && !wide_scan(idx) ? 0 : probe_mode_env())) return r;
    if (final_src) {
        std::vector<int> tf;
        if (int r = tail_flags(C, {0}, tf)) return r;
        ch->tail_flag = tf[0];
    }
    C.prof = nullptr;
    *out = ch.release();
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" int sydelta_chunk_walk(sydelta_chunk* ch, uint64_t entry, uint64_t* exit_pos, sydelta_delta** out) try {
    if (!ch || !exit_pos || !out) return fail(SYDELTA_E_INVAL, "NULL argument");
    *out = nullptr;
    Classifier& C = ch->C;
    const Src& c = C.src[0];
    if (entry < c.p0) return fail(SYDELTA_E_INVAL, "entry %llu precedes the chunk", (unsigned long long)entry);
    SYDELTA_ENTER_DEVICE(C.ix->device);
    CallProf cp;
    C.prof = cp.get();
    std::unique_ptr<sydelta_delta> d(new sydelta_delta());
    d->source_size = ch->file_len;
    d->block_size = C.n;
    d->stats.positions = c.p1 - c.p0;
    if (ch->dev_walk) {
        int r = SYDELTA_OK;
        if (!ch->pipe.on) r = chunk_pipe_launch(ch, entry, false);  // nothing to probe: launched now
        if (!r) r = chunk_pipe_finish(ch, entry, exit_pos, d.get());
        C.prof = nullptr;
        if (r) return r;
        *out = d.release();
        return SYDELTA_OK;
    }
    const int r = C.walk(0, entry, ch->bi, ch->final_src, ch->tail_flag, d.get(), exit_pos);
    C.prof = nullptr;
    if (r) return r;
    d->stats.verified_hits = c.hpos.size() + c.nahit;
    d->stats.weak_hits = C.weak_hits;  // op counts: C.walk
    *out = d.release();
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" void sydelta_chunk_free(sydelta_chunk* ch) {
    if (!ch) return;
    DeviceScope keep_device;
    (void)hipSetDevice(ch->C.ix->device);
    delete ch;
}

// Concatenate src's ops onto dst; a Data op that ends where src's first Data op
// starts is extended (literal runs stay maximal, generator.rs:186-197, 218-221).
extern "C" int sydelta_delta_append(sydelta_delta* dst, const sydelta_delta* src) try {
    if (!dst || !src) return fail(SYDELTA_E_INVAL, "NULL argument");
    if (!dst->lit_off.empty() || !src->lit_off.empty())
        return fail(SYDELTA_E_INVAL, "append is for device deltas (no host literal copies)");
    size_t j = 0;
    if (!dst->ops.empty() && !src->ops.empty()) {
        sydelta_op& a = dst->ops.back();
        const sydelta_op& b = src->ops.front();
        if (a.kind == SYDELTA_OP_DATA && b.kind == SYDELTA_OP_DATA && a.a + a.b == b.a) {
            a.b += b.b;
            j = 1;
        }
    }
    dst->ops.insert(dst->ops.end(), src->ops.begin() + j, src->ops.end());
    dst->stats.positions += src->stats.positions;
    dst->stats.weak_hits += src->stats.weak_hits;
    dst->stats.verified_hits += src->stats.verified_hits;
    if (!dst->block_size) dst->block_size = src->block_size;
    dst->source_size = std::max(dst->source_size, src->source_size);
    finish_stats(dst);
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}

extern "C" sydelta_delta* sydelta_delta_from_ops(const sydelta_op* ops, uint64_t n, uint64_t source_size,
                                                 uint64_t block_size) {
    if (n && !ops) return nullptr;
    for (uint64_t i = 0; i < n; ++i)  // only DeltaOp::Copy / DeltaOp::Data exist (generator.rs:10-15)
        if (ops[i].kind != SYDELTA_OP_COPY && ops[i].kind != SYDELTA_OP_DATA) {
            fail(SYDELTA_E_INVAL, "op %llu: unknown kind %u", (unsigned long long)i, (unsigned)ops[i].kind);
            return nullptr;
        }
    sydelta_delta* d = new (std::nothrow) sydelta_delta();
    if (!d) return nullptr;
    d->source_size = source_size;
    d->block_size = block_size;
    d->ops.assign(ops, ops + n);
    finish_stats(d);
    return d;
}

extern "C" sydelta_delta* sydelta_delta_new(uint64_t source_size, uint64_t block_size) {
    sydelta_delta* d = new sydelta_delta();
    d->source_size = source_size;
    d->block_size = block_size;
    return d;
}

// ---------------------------------------------------------------------------
// One file chunk-sharded over several devices of this process (BASELINE config 5,
// SURVEY.md §8e): the in-process form of bench.py's one-process-per-GPU C5 step.
// ---------------------------------------------------------------------------
// 1. each device signs its basis chunk into its slice of a whole-file signature SoA;
// 2. every device pulls the other slices with peer copies (hipMemcpyPeerAsync: xGMI
//    between MI355X devices of one node), so each holds the full signature with global
//    block indices and the lowest-index rule stays global;
// 3. each device builds the full index and classifies its source chunk (host-pool
//    threads, one per chunk: the classification's host waits overlap);
// 4. the walks run speculatively from each chunk's start, in parallel; a chunk whose
//    true entry (the previous chunk's exit) differs is walked again, in chunk order
//    (shard.py walk_chain's rule); the parts are joined with sydelta_delta_append.
// The result equals generate_delta's op list for the whole file (generator.rs:242-379):
// classification is a pure function of the position.
namespace {
std::mutex g_peer_mu;
std::set<std::pair<int, int>> g_peer_on;  // under g_peer_mu: (device, peer) with access enabled
void enable_peer(int dev, int peer) {
    if (dev == peer) return;
    DeviceScope keep_device;
    std::lock_guard<std::mutex> lk(g_peer_mu);
    if (!g_peer_on.insert({dev, peer}).second) return;
    int ok = 0;
    if (hipDeviceCanAccessPeer(&ok, dev, peer) == hipSuccess && ok && hipSetDevice(dev) == hipSuccess)
        (void)hipDeviceEnablePeerAccess(peer, 0);  // already enabled / unsupported: the copy still works
    (void)hipGetLastError();
}
}  // namespace

extern "C" int sydelta_delta_multi_device(const int* devices, int ndev, const uint8_t* const* d_basis,
                                          const uint64_t* basis_len, const uint8_t* const* d_src,
                                          const uint64_t* src_pos, const uint64_t* src_buf_len, uint64_t src_len,
                                          uint64_t block_size, sydelta_delta** out) try {
    DeviceScope keep_device;  // restored after every hipSetDevice below, on every return
    if (!out) return fail(SYDELTA_E_INVAL, "out is NULL");
    *out = nullptr;
    if (ndev < 1 || !devices || !d_basis || !basis_len || !d_src || !src_pos || !src_buf_len)
        return fail(SYDELTA_E_INVAL, "NULL argument or no device");
    const uint64_t n = block_size;
    if (n == 0) return fail(SYDELTA_E_INVAL, "block_size must be > 0");
    // basis chunks: every one but the last a whole number of blocks
    std::vector<uint64_t> nbg(ndev), bofs(ndev + 1, 0);
    uint64_t L = 0;
    for (int g = 0; g < ndev; ++g) {
        if (g + 1 < ndev && basis_len[g] % n)
            return fail(SYDELTA_E_INVAL, "basis chunk %d: length %llu is not a multiple of block_size", g,
                        (unsigned long long)basis_len[g]);
        if (basis_len[g] && !d_basis[g]) return fail(SYDELTA_E_INVAL, "basis chunk %d: NULL buffer", g);
        nbg[g] = (basis_len[g] + n - 1) / n;
        bofs[g + 1] = bofs[g] + nbg[g];
        L += basis_len[g];
    }
    const uint64_t nb = bofs[ndev];
    if (nb >= 0xFFFFFFFFull) return fail(SYDELTA_E_INVAL, "too many blocks");
    const uint64_t last_size = nb ? L - (nb - 1) * n : 0;
    // source chunks: block-aligned starts, chunk 0 from position 0
    if (src_pos[0] != 0) return fail(SYDELTA_E_INVAL, "source chunk 0 must start at position 0");
    for (int g = 1; g < ndev; ++g)
        if (src_pos[g] < src_pos[g - 1] || src_pos[g] % n)
            return fail(SYDELTA_E_INVAL, "source chunk %d: start %llu not ascending / not a multiple of block_size", g,
                        (unsigned long long)src_pos[g]);
    for (int g = 0; g < ndev; ++g)
        if (int r = ensure_device(devices[g])) return r;
    for (int g = 0; g < ndev; ++g)
        for (int h = 0; h < ndev; ++h) enable_peer(devices[g], devices[h]);
    // 1. signatures (the calling thread's stream on each device)
    std::vector<hipStream_t> s(ndev);
    std::vector<std::unique_ptr<DevBuf>> sig(ndev);
    std::vector<uint32_t*> dw(ndev);
    std::vector<uint64_t*> dst(ndev);
    std::vector<hipEvent_t> ev(ndev, nullptr);
    struct EvFree {
        std::vector<hipEvent_t>& v;
        ~EvFree() {
            for (hipEvent_t e : v)
                if (e) (void)hipEventDestroy(e);
        }
    } ev_free{ev};
    // on any return (an error below included): every stream's queued copies finish before
    // the slices in sig are released on their own streams (destroyed before sig)
    struct SyncAll {
        const int* dev;
        const std::vector<hipStream_t>& s;
        ~SyncAll() {
            for (size_t g = 0; g < s.size(); ++g)
                if (s[g] && hipSetDevice(dev[g]) == hipSuccess) (void)hipStreamSynchronize(s[g]);
        }
    } sync_all{devices, s};
    CallProf cp;
    for (int g = 0; g < ndev; ++g) {
        HIP_TRY(hipSetDevice(devices[g]));
        s[g] = thread_stream(devices[g]);
        sig[g].reset(new DevBuf());
        HIP_TRY(dev_malloc_async(&sig[g]->p, nb * 12 + 16, s[g]));
        sig[g]->s = s[g];
        dw[g] = (uint32_t*)sig[g]->p;
        dst[g] = (uint64_t*)(((uintptr_t)(dw[g] + nb) + 7) & ~(uintptr_t)7);
        HIP_TRY(launch_signature(d_basis[g], basis_len[g], n, dw[g] + bofs[g], dst[g] + bofs[g], s[g], cp.get()));
        HIP_TRY(hipEventCreateWithFlags(&ev[g], hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ev[g], s[g]));
    }
    // 2. gather: device g pulls slice h from device h
    for (int g = 0; g < ndev; ++g) {
        HIP_TRY(hipSetDevice(devices[g]));
        for (int h = 0; h < ndev; ++h) {
            if (h == g || !nbg[h]) continue;
            HIP_TRY(hipStreamWaitEvent(s[g], ev[h], 0));
            if (devices[g] == devices[h]) {
                HIP_TRY(hipMemcpyAsync(dw[g] + bofs[h], dw[h] + bofs[h], 4 * nbg[h], hipMemcpyDeviceToDevice, s[g]));
                HIP_TRY(hipMemcpyAsync(dst[g] + bofs[h], dst[h] + bofs[h], 8 * nbg[h], hipMemcpyDeviceToDevice, s[g]));
            } else {
                HIP_TRY(hipMemcpyPeerAsync(dw[g] + bofs[h], devices[g], dw[h] + bofs[h], devices[h], 4 * nbg[h], s[g]));
                HIP_TRY(hipMemcpyPeerAsync(dst[g] + bofs[h], devices[g], dst[h] + bofs[h], devices[h], 8 * nbg[h], s[g]));
            }
        }
    }
    // every device's gather done before any slice is released or read from another stream
    for (int g = 0; g < ndev; ++g) {
        HIP_TRY(hipSetDevice(devices[g]));
        HIP_TRY(hipStreamSynchronize(s[g]));
    }
    // 3. full index per device, then the chunks classified in parallel
    std::vector<std::unique_ptr<sydelta_index, void (*)(sydelta_index*)>> idx;
    for (int g = 0; g < ndev; ++g) {
        sydelta_index* x = nullptr;
        if (int r = sydelta_index_create(devices[g], dw[g], dst[g], nb, n, nb ? last_size : n, 1, s[g], &x)) return r;
        idx.emplace_back(x, sydelta_index_free);
    }
    for (int g = 0; g < ndev; ++g) {
        HIP_TRY(hipSetDevice(devices[g]));
        HIP_TRY(hipStreamSynchronize(s[g]));
    }
    std::vector<std::unique_ptr<sydelta_chunk, void (*)(sydelta_chunk*)>> ch;
    for (int g = 0; g < ndev; ++g) ch.emplace_back(nullptr, sydelta_chunk_free);
    std::vector<int> rc(ndev, SYDELTA_OK);
    std::vector<std::string> err(ndev);
    auto pos_end = [&](int g) { return g + 1 < ndev ? src_pos[g + 1] : std::max<uint64_t>(src_len, src_pos[g]) + 1; };
    if (!run_parallel(ndev, [&](int g) {
            sydelta_chunk* c = nullptr;
            rc[g] = sydelta_chunk_classify(idx[g].get(), d_src[g], src_pos[g], src_buf_len[g], src_len, src_pos[g],
                                           pos_end(g), nullptr, &c);
            if (rc[g]) err[g] = sydelta_last_error();
            ch[g].reset(c);
        }))
        return fail(SYDELTA_E_OOM, "out of host memory (chunk tasks)");
    for (int g = 0; g < ndev; ++g)
        if (rc[g]) return fail(rc[g], "chunk %d: %s", g, err[g].c_str());
    // 4. speculative walks, then the chain
    std::vector<std::unique_ptr<sydelta_delta, void (*)(sydelta_delta*)>> part;
    for (int g = 0; g < ndev; ++g) part.emplace_back(nullptr, sydelta_delta_free);
    std::vector<uint64_t> ex(ndev, 0);
    if (!run_parallel(ndev, [&](int g) {
            sydelta_delta* d = nullptr;
            rc[g] = sydelta_chunk_walk(ch[g].get(), src_pos[g], &ex[g], &d);
            if (rc[g]) err[g] = sydelta_last_error();
            part[g].reset(d);
        }))
        return fail(SYDELTA_E_OOM, "out of host memory (walk tasks)");
    for (int g = 0; g < ndev; ++g)
        if (rc[g]) return fail(rc[g], "chunk %d walk: %s", g, err[g].c_str());
    uint64_t e = 0;
    for (int g = 0; g < ndev; ++g) {
        if (e != src_pos[g]) {  // the previous chunk's last Copy reaches into this one
            sydelta_delta* d = nullptr;
            if (int r = sydelta_chunk_walk(ch[g].get(), e, &ex[g], &d)) return r;
            part[g].reset(d);
        }
        e = ex[g];
    }
    std::unique_ptr<sydelta_delta, void (*)(sydelta_delta*)> joined(sydelta_delta_new(src_len, n), sydelta_delta_free);
    for (int g = 0; g < ndev; ++g)
        if (int r = sydelta_delta_append(joined.get(), part[g].get())) return r;
    joined->source_size = src_len;
    ch.clear();
    idx.clear();
    sig.clear();
    *out = joined.release();
    return SYDELTA_OK;
} catch (...) {
    return sydelta::host_exception();
}
