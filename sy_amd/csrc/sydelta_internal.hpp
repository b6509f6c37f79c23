// sydelta_internal.hpp — shared between the kernel TU and the host API TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <string>
#include <vector>

namespace sydelta {

constexpr uint32_t kEmptyKey = 0xFFFFFFFFu;  // never a valid weak: A = weak & 0xFFFF <= 65520
constexpr uint64_t kLdsFilterKeys = 16384;   // index sizes whose Bloom filter (<= 32 KiB) the scan keeps in LDS
constexpr uint32_t kLdsFilterWordsMax = 8192;

// One (weak or verified) hit.  pos = position relative to the segment start,
// slot = table slot (weak hit) or block index (verified hit).  pos is the low
// word so a radix sort of the record as a u64 on bits [0,32) orders by position.
struct HitRec {
    uint32_t pos;
    uint32_t slot;
};
static_assert(sizeof(HitRec) == 8, "HitRec must be 8 bytes");

// Device-resident probe table over a basis signature (SoA in HBM).
struct DeviceIndex {
    uint32_t* filt = nullptr;  // blocked Bloom filter: 2^fwbits 32-bit words (filt_hash/filt_mask)
    uint32_t fwbits = 0;
    uint32_t* keys = nullptr;   // 4-key buckets of unique weak values, kEmptyKey = free
    uint32_t* cnt = nullptr;    // candidates per slot
    uint32_t* start = nullptr;  // exclusive prefix of cnt
    uint32_t* fill = nullptr;   // scratch for the scatter
    uint32_t* order = nullptr;  // block indices grouped by slot
    uint32_t* slot_of = nullptr;
    uint32_t bmask = 0;         // buckets - 1
};

// Per-kernel HIP-event timing (enabled by sydelta_set_profiling).
struct Profiler {
    struct Pending { std::string name; hipEvent_t a, b; };
    std::vector<Pending> pending;
    void resolve();  // after the stream has been synchronised
};
struct ProfScope {
    Profiler* p;
    hipStream_t s;
    const char* name;
    hipEvent_t a{}, b{};
    ProfScope(Profiler* p_, hipStream_t s_, const char* n);
    ~ProfScope();
};

hipError_t launch_signature(const uint8_t* d_buf, uint64_t len, uint64_t bs, uint32_t* d_weak, uint64_t* d_strong,
                            hipStream_t s, Profiler* prof);
hipError_t launch_signature_batch(const uint8_t* d_buf, const uint64_t* d_off, const uint64_t* d_len,
                                  const uint64_t* d_fblk, uint64_t nfiles, uint64_t bs, uint64_t total_blocks,
                                  uint32_t* d_weak, uint64_t* d_strong, hipStream_t s, Profiler* prof);
hipError_t launch_index_build(const uint32_t* d_weak, uint64_t n, DeviceIndex& ix, hipStream_t s, Profiler* prof);
size_t scan_lds_bytes(uint32_t n, uint32_t* nchunks_out);
uint64_t scan_tile_positions();
// Scratch the scan needs: filter-pass queues, scan_queue_entries() uint2 entries
// (enough for 2 workgroups per CU on a 256-CU device; launch_scan checks).
size_t scan_queue_entries();
hipError_t launch_scan(const uint8_t* d_src, uint64_t len, uint64_t pos_begin, uint64_t pos_end, uint32_t n,
                       const DeviceIndex& ix, const uint64_t* d_strong, HitRec* d_out, uint64_t out_cap,
                       unsigned long long* d_counters, uint2* gfq, size_t gfq_cap, hipStream_t s, Profiler* prof);
hipError_t launch_sort_hits(HitRec* d_in, HitRec* d_tmp_out, uint64_t nhits, hipStream_t s, HitRec** sorted);
hipError_t launch_tail(const uint8_t* d_src, uint64_t len, uint64_t last_size, uint32_t want_weak, uint64_t want_strong,
                       int* d_flag, hipStream_t s);
hipError_t launch_synth_fill(uint8_t* d_buf, uint64_t len, uint64_t seed, hipStream_t s);
hipError_t launch_synth_mutate(uint8_t* d_dst, const uint8_t* d_src, uint64_t len, uint64_t seed, uint32_t rate_ppm,
                               hipStream_t s);

}  // namespace sydelta
