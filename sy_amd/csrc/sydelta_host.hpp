// sydelta_host.hpp — host-side definitions shared by the C ABI translation units
// (sydelta_api.cpp: signature / index / match / apply; sydelta_wire.cpp: wire formats).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/sydelta.h"
#include "sydelta_internal.hpp"
#include "sydelta_walk.hpp"  // OpVec


// Delta (generator.rs:19-25): ops plus, for host-data entry points, the literal bytes.
struct sydelta_delta {
    OpVec ops;
    uint64_t source_size = 0, block_size = 0;
    sydelta_match_stats stats{};
    std::vector<uint8_t> lit;         // literal bytes (host-data entry points)
    std::vector<uint64_t> lit_off;    // per op: offset into lit, or UINT64_MAX
};

namespace sydelta {
// Record the calling thread's error text (sydelta_last_error) and return code.
int fail(int code, const char* fmt, ...);
// For the catch (...) of every int entry point (a function-try-block): no C++
// exception crosses the C ABI; std::bad_alloc -> SYDELTA_E_OOM, others -> SYDELTA_E_INVAL.
int host_exception();
// Make `device` current after its one-time gfx950 check.
int ensure_device(int device);
// Every entry point leaves the calling thread's current HIP device as it found it
// (sydelta.h, "Devices"): a guard records it on entry and restores it on every return.
// Guards nest: an inner one restores what the outer entry made current.
struct DeviceScope {
    int dev = -1;
    DeviceScope() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceScope() {
        int now = -1;
        if (dev >= 0 && hipGetDevice(&now) == hipSuccess && now != dev) (void)hipSetDevice(dev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};
// The device of the calling thread's path-level calls (bound on first use, sticky).
int path_device(int* out);
// The calling thread's stream for `device`.
hipStream_t thread_stream(int device);
// K10 wave slots of a device (CUs x 16: four waves per SIMD), from its properties at first use
uint32_t wave_slots(int device);
// Recount copy/data ops and literal bytes of d.
void finish_stats(sydelta_delta* d);
// Per-thread scan scratch (Classifier::scan): the verified-hit buffers on one device,
// and the pinned host buffer the sorted hits come back into (not kept above
// kPinnedHitsKeep).  Released by sydelta_trim.
struct HitScratch {
    void* p = nullptr;
    size_t bytes = 0;
};
struct PinnedHits {
    uint8_t* p = nullptr;
    size_t bytes = 0;
};
constexpr size_t kPinnedHitsKeep = (size_t)256 << 20;
HitScratch& thread_hit_scratch(int device);
DevScratch& thread_scan_scratch(int device);   // launch_scan's kept scratch
DevScratch& thread_probe_scratch(int device);  // Classifier::probe's (transient classifiers)
DevScratch& thread_walk_scratch(int device);   // the file walk's (match_walk_files)
PinnedHits& thread_pinned_hits();
// Held (recursively) by the calling thread while it uses its scratch: sydelta_trim on
// another thread then leaves that scratch alone.
struct ScratchHold {
    std::recursive_mutex* mu;
    ScratchHold();
    ~ScratchHold();
    ScratchHold(const ScratchHold&) = delete;
    ScratchHold& operator=(const ScratchHold&) = delete;
};
// sydelta_set_profiling state; CallProf collects one call's kernel timings.
bool profiling_on();
struct CallProf {
    Profiler prof;
    Profiler* get() { return profiling_on() ? &prof : nullptr; }
    ~CallProf() { prof.resolve(); }
};
}  // namespace sydelta

// An entry point's device: the caller's current device restored on return (DeviceScope),
// `dev` made current (ensure_device) or the error returned.
#define SYDELTA_ENTER_DEVICE(dev)              \
    ::sydelta::DeviceScope sydelta_dscope_;   \
    if (int r_ = ::sydelta::ensure_device(dev)) return r_

#define HIP_TRY(expr)                                                                                 \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) {                                                                         \
            int code_ = (e_ == hipErrorOutOfMemory) ? SYDELTA_E_OOM : SYDELTA_E_KERNEL;                 \
            return ::sydelta::fail(code_, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,     \
                                   __LINE__);                                                           \
        }                                                                                               \
    } while (0)
