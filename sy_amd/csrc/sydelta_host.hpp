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
// The device of the calling thread's path-level calls (bound on first use, sticky).
int path_device(int* out);
// The calling thread's stream for `device`.
hipStream_t thread_stream(int device);
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
PinnedHits& thread_pinned_hits();
// sydelta_set_profiling state; CallProf collects one call's kernel timings.
bool profiling_on();
struct CallProf {
    Profiler prof;
    Profiler* get() { return profiling_on() ? &prof : nullptr; }
    ~CallProf() { prof.resolve(); }
};
}  // namespace sydelta

#define HIP_TRY(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) {                                                                         \
            int code_ = (e_ == hipErrorOutOfMemory) ? SYDELTA_E_OOM : SYDELTA_E_KERNEL;                 \
            return ::sydelta::fail(code_, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,     \
                                   __LINE__);                                                           \
        }                                                                                               \
    } while (0)
