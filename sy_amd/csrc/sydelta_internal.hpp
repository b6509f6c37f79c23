// sydelta_internal.hpp — shared between the kernel TU and the host API TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <string>
#include <vector>

#include "sydelta_chain.hpp"
#include "sydelta_sigjson.hpp"
#include "sydelta_dparse.hpp"
#include "sydelta_zstd.hpp"

namespace sydelta {

// Stream-ordered device scratch from the library's own memory pool (one per device,
// created by ensure_device), so its release threshold never touches the device's
// default pool that torch or other libraries in the process may use.  Freed with
// hipFreeAsync like any pool allocation.
hipError_t dev_malloc_async(void** p, size_t bytes, hipStream_t s);

constexpr uint32_t kEmptyKey = 0xFFFFFFFFu;  // never a valid weak: A = weak & 0xFFFF <= 65520
constexpr uint64_t kLdsFilterKeys = 16384;   // index sizes whose Bloom filter (<= 32 KiB) the scan keeps in LDS
constexpr uint32_t kLdsFilterWordsMax = 8192;
// k_scan_g's small-index mode keeps one file filter per wave in LDS: up to 4096 words
// (16 KiB; files of up to 4 Ki blocks), eight waves per workgroup.
constexpr uint32_t kSmallWords = 4096;
// k_scan_r's small-index mode (n = 4096, twelve waves): one slot per wave in the level-1
// area (kL1WordsR words), so up to 3200 words; files of up to 512 blocks (1024 words).
constexpr uint32_t kSmallWordsR = 2048;
// k_scan_r's level-1 filter (one large file at n = 4096): 38400 words = 150 KiB, the LDS
// left when the tile's bytes stay in registers, word = l1r_word(q) (l1_wshift 1 marks it).
constexpr uint32_t kL1WordsR = 38400;
// k_scan_r's level-1 filter as a homogeneous ribbon (Dillinger & Walzer 2021) of width 32
// in kRibShards independent shards of kRibBits columns: a key w (probe hashes q, r) lies in
// shard q >> 22, its equation covers columns [start, start + 32) of that shard (start from
// r) with coefficients (q ^ rotl(r, 16)) | 1, and the solution z satisfies every key's
// equation c . z = 0 (mod 2); a position passes when its own window's parity is even.
// One bit of result: a non-key passes with probability ~1/2 however the bits are spent
// (0.504 measured on Adler values of 1 Mi random 4 KiB blocks, tools/ribbon_sim.c), against
// 1 - e^(-keys/1228800) for the one-hash Bloom of the same 150 KiB (0.574 at 1 Mi keys):
// allocated when the index has kRibMinKeys..kRibMaxKeys blocks (the two cross at ~852 K
// keys) and built by the first scan of at least kRibMinScan positions (its ~0.35 ms of
// listing and solving pays back ~0.17 ms per 2^30 positions: C3's whole-file scan builds
// it, C5's scan of its edited blocks does not).
// Homogeneous: every system is consistent, so no key set makes the build fail (a shard
// loaded past its columns only passes more positions).
constexpr uint32_t kRibShards = 1024;
constexpr uint32_t kRibBits = 1184;  // columns per shard: 37 words
constexpr uint32_t kRibWords = kRibShards * kRibBits / 32;  // 37888, + 1 pad word read past the last window
static_assert(kRibWords + 1 <= kL1WordsR, "the ribbon fits k_scan_r's level-1 LDS area");
constexpr uint32_t kRibCap = 2048;     // distinct keys listed per shard (mean 1024 at 1 Mi keys); more: overflow list
constexpr uint64_t kRibMinKeys = 852000;
// ... and at most kRibMaxKeys: beyond ~0.95 keys per column a shard's system is full and
// passes nearly every position (the Bloom's 1 - e^(-keys/1228800) is then lower).
constexpr uint64_t kRibMaxKeys = 1100000;
constexpr uint64_t kRibMinScan = 1ull << 31;
// words of a level-1 filter: l1_wshift 1 marks k_scan_r's scaled-word layout, any other
// value a power-of-two filter of 2^(32 - l1_wshift) words
constexpr size_t l1_total_words(uint32_t l1_wshift) {
    return l1_wshift == 1 ? (size_t)kL1WordsR : (size_t)1 << (32 - l1_wshift);
}

// Verified hits are written as key/value pairs: key = (segment << 32) | position
// relative to the segment's first position, value = global block index (into the
// index's concatenated signature).  A radix sort of the keys orders hits by
// (segment, position); segments are laid out in (file, position) order.
constexpr int kSegShift = 32;

// Probe structures of one file inside a (possibly batched) index.  All arrays
// of the index are concatenations over its files.
struct FileIx {
    uint64_t filt_off;  // first Bloom word of this file
    uint64_t slot_off;  // first exact-table slot (multiple of 4)
    uint64_t blk_base;  // first block of this file in the concatenated signature
    uint32_t fwshift;   // 32 - log2(this file's filter words)
    uint32_t bmask;     // this file's bucket count - 1
};

// One range of full-window positions of one source, scanned by one launch.
struct ScanSeg {
    uint64_t src;        // byte offset of the source in the scanned buffer
    uint64_t len;        // source length
    uint64_t pos_begin;  // first position (relative to the source)
    uint64_t pos_end;    // one past the last full-window position of this segment
    uint32_t tile_base;  // first tile of this segment within the launch
    uint32_t file;       // FileIx of the basis this source is matched against
};

// Device-resident probe table over one or more basis signatures (SoA in HBM).
struct DeviceIndex {
    uint32_t* filt = nullptr;   // blocked Bloom filters (probe_hash/filt_mask), per-file 2^k 32-bit words
    uint32_t* l1 = nullptr;     // level-1 filter: single-file indexes above kLdsFilterKeys keys at bs 4096
                                // (k_scan_r, k_scan_g) or with windows above scan_max_window() (k_scan_g)
    uint32_t l1_wshift = 1;     // 1: kL1WordsR words, l1r_word(q)
    uint32_t l1_ribbon = 0;     // with l1_wshift 1: the words hold the ribbon (kRibWords), not a Bloom filter
    // the ribbon, built on demand (launch_ribbon_build) into rib_l1 (kL1WordsR words); a
    // scan that uses it gets a copy of the index with l1 = rib_l1, l1_ribbon = 1
    uint32_t* rib_l1 = nullptr;
    uint32_t* rib_keys = nullptr;  // ribbon build: kRibShards lists of kRibCap distinct keys
    uint32_t* rib_cnt = nullptr;   // kRibShards + 1 counts (the last: the overflow list's)
    uint32_t* rib_over = nullptr;  // overflow list (capacity nblocks)
    uint4* fat = nullptr;       // with l1: per slot {key, first candidate | multi, its strong} (k_idx_fat)
    uint32_t* keys = nullptr;   // 4-key buckets of unique weak values, kEmptyKey = free
    uint32_t* cnt = nullptr;    // candidates per slot
    uint32_t* start = nullptr;  // exclusive prefix of cnt (global positions into order)
    uint32_t* fill = nullptr;   // scratch for the scatter
    uint32_t* order = nullptr;  // global block indices grouped by slot (any order within a slot)
    uint64_t* cstrong = nullptr;  // strong hash of order[j]
    uint32_t* slot_of = nullptr;
    FileIx* d_files = nullptr;  // per-file offsets (device copy of files)
    uint64_t* d_fblk = nullptr; // block prefix over files, nfiles+1 entries
    std::vector<FileIx> files;  // host copy
    uint64_t nfiles = 0, nblocks = 0, fwords = 0, nslots = 0;
    uint32_t max_fwords = 0;    // largest per-file filter (decides LDS residency)
};

// Per-kernel HIP-event timing (enabled by sydelta_set_profiling).
struct Profiler {
    struct Pending { std::string name; hipEvent_t a, b; int device; };
    std::vector<Pending> pending;
    void resolve();  // hands the call's timed launches over; read by sydelta_profile_json
};
struct ProfScope {
    Profiler* p;
    hipStream_t s;
    const char* name;
    hipEvent_t a{}, b{};
    int device = 0;
    ProfScope(Profiler* p_, hipStream_t s_, const char* n);
    ~ProfScope();
};

hipError_t launch_signature(const uint8_t* d_buf, uint64_t len, uint64_t bs, uint32_t* d_weak, uint64_t* d_strong,
                            hipStream_t s, Profiler* prof);
hipError_t launch_signature_batch(const uint8_t* d_buf, const uint64_t* d_off, const uint64_t* d_len,
                                  const uint64_t* d_fblk, uint64_t nfiles, uint64_t bs, uint64_t total_blocks,
                                  uint32_t* d_weak, uint64_t* d_strong, hipStream_t s, Profiler* prof);
// Build filters + exact tables of every file of ix from the concatenated weak
// values (ix.nblocks entries; ix.d_fblk / ix.d_files already on the device).
// extras = false leaves the scans' level-1 filter and fat table (ix.l1, ix.fat) unfilled:
// launch_index_extras fills them when a scan first needs them (the chunk walk and the aligned
// probe read only the Bloom filter and the exact table).
hipError_t launch_index_build(const uint32_t* d_weak, const uint64_t* d_strong, DeviceIndex& ix, hipStream_t s,
                              Profiler* prof, bool extras = true);
hipError_t launch_index_extras(const uint32_t* d_weak, const DeviceIndex& ix, hipStream_t s, Profiler* prof);
// The ribbon level-1 of a built single-file index (ix.rib_l1 and its key lists set):
// its distinct keys listed by shard from the exact table, then each shard solved.
// keys: the keys to list (nkeys of them, duplicates allowed: a duplicate's equation reduces to 0),
// by default the exact table's (ix.keys, ix.nslots); the signature's weak values (never
// kEmptyKey: an Adler digest's low half is below 65521) let it start before the table is built.
hipError_t launch_ribbon_build(const DeviceIndex& ix, hipStream_t s, Profiler* prof, const uint32_t* keys = nullptr,
                               uint64_t nkeys = 0);
uint64_t scan_tile_positions();  // positions per tile of the LDS-staged scan
// SYDELTA_SCAN_WIDE=0: windows above scan_max_window() take the per-thread k_scan
// instead of the register-fed k_scan_g (read when the index is built and per call)
int scan_wide_mode();
uint32_t scan_max_window();      // largest block size the LDS-staged scan handles
// Scratch the LDS-staged scan needs: filter-pass queues, scan_queue_entries() uint2
// entries (2 workgroups per CU on up to 256 CUs; launch_scan checks; with no queues
// given it takes them from its scratch).
size_t scan_queue_entries();
// A device buffer kept between calls by its owner (the calling thread), grown on demand
// in the owner's stream order.
struct DevScratch {
    void* p = nullptr;
    size_t bytes = 0;
};
// Scan all tiles of segs[0..nsegs) (device copy d_segs; block_size n <= scan_max_window()).
// scratch (may be null: allocated and freed per call) holds the register-fed scans' pass
// records, staged outputs and deferred list; the previous use of it must have completed
// (the caller synchronized its stream).
hipError_t launch_scan(const uint8_t* d_buf, const ScanSeg* d_segs, uint32_t nsegs, uint32_t ntiles, uint32_t n,
                       const DeviceIndex& ix, const uint64_t* d_strong, uint64_t* d_hit_key, uint32_t* d_hit_val,
                       uint64_t out_cap, unsigned long long* d_counters, uint2* gfq, size_t gfq_cap, hipStream_t s,
                       Profiler* prof, DevScratch* scratch = nullptr);
// Fallback for block sizes above scan_max_window(): one segment, file 0 of ix, hits
// keyed with seg_id.
hipError_t launch_scan_wide(const uint8_t* d_src, uint64_t len, uint64_t pos_begin, uint64_t pos_end, uint32_t seg_id,
                            uint32_t n, const DeviceIndex& ix, const uint64_t* d_strong, uint64_t* d_hit_key,
                            uint32_t* d_hit_val, uint64_t out_cap, unsigned long long* d_counters, hipStream_t s,
                            Profiler* prof);
// Sort nhits (key, value) pairs by key on bits [0, end_bit); sorted output in
// (*key_out, *val_out) (either the input or the tmp arrays).
hipError_t launch_sort_hits(uint64_t* key, uint32_t* val, uint64_t* key_tmp, uint32_t* val_tmp, uint64_t nhits,
                            int end_bit, hipStream_t s, uint64_t** key_out, uint32_t** val_out);
// Aligned-window probe: probe w of job j (jobs[j].pfx <= w < jobs[j+1].pfx) is the
// window at position k*n, k = k0 + (w - pfx) * stride, of the source at byte
// offset src from the launch base; out[w] = global block index of its hit
// (first candidate in index order with equal weak and strong), or 0xFFFFFFFF.
struct ProbeJob {
    uint64_t src;
    uint64_t k0;
    uint64_t pfx;
    uint32_t file;
    uint32_t pad;
};
// fast: n % 64 == 0, n >= 256 and every window 16-byte aligned.
// Scratch: d_pw[nprobes], d_pst[nprobes] (the windows' weak / strong).
// phases: 1 hash the windows (d_pw, d_pst), 2 look them up (d_out; the index must be
// built), 3 both -- split so the hashing can run before the index is ready.
hipError_t launch_probe(const uint8_t* d_base, const ProbeJob* d_jobs, uint32_t njobs, uint64_t nprobes,
                        uint32_t stride, uint32_t n, bool fast, const DeviceIndex& ix, uint32_t* d_pw,
                        uint64_t* d_pst, uint32_t* d_out, hipStream_t s, Profiler* prof, int phases = 3);
// Tail rule (generator.rs:156-184) of every listed file: flag[i] = 1 iff the
// suffix of source i hashes to (weak[blk], strong[blk]) of its last basis block.
struct TailJob {
    uint64_t src;        // byte offset of the suffix [len - last_size, len) in the buffer
    uint64_t last_size;  // 1 .. block_size - 1
    uint64_t blk;        // global index of the file's last basis block
};
hipError_t launch_tail(const uint8_t* d_buf, const TailJob* d_jobs, uint32_t njobs, const uint32_t* d_weak,
                       const uint64_t* d_strong, int* d_flag, hipStream_t s);
// K5b: the walk of one classified source resolved on the device (sydelta_chain.hpp):
// merge, successors, pointer-jumping path marking, op emission; a.res receives the
// totals.  All arrays of a are device memory sized as ChainArgs documents.
hipError_t launch_chain(const chain::ChainArgs& a, hipStream_t s, Profiler* prof);
// K10: the greedy walk (generator.rs:116-221) on the device, one wave per unit
// (k_walk_files): a unit is a whole file of a batch (C4's small files) or a segment of a
// chunk of one file (C5), walked from its entry until it leaves [entry, end).  Block sizes
// n % 64 == 0, 256 <= n <= kWalkMaxN.  A batch's walks are self-indexed: each unit builds its
// file's Bloom filter and exact candidate table in LDS from the file's signature (files of at
// most kSelfIxMaxBlocks blocks; the batch index's tables are not needed); a large single-file
// index's filter and tables are read from L2.  The ops
// come back run-length coded: a Data op, or a run of Copies of consecutive global basis
// blocks (each Copy's size follows from its block: the basis file's last block has
// last_size, every other one n).
constexpr uint32_t kSelfIxMaxBlocks = 1024;
constexpr uint32_t kWalkMaxN = 8192;
struct WalkRec {
    uint32_t kind;  // 0: Data; else the number of Copies in the run
    uint32_t a;     // Data: length; Copy run: its first global block
    uint64_t off;   // Data: offset in the source file
};
struct WalkUnit {
    uint64_t src;      // byte offset of source position 0 from the launch base
    uint64_t len;      // source file length (a final unit's tail rule and last literal run)
    uint64_t entry;    // the first position walked
    uint64_t end;      // the walk leaves the unit at its first position >= end (<= p1)
    uint64_t p1;       // full-window starts [0, p1) of the source (0 without a signature)
    uint64_t rec_off;  // staging region: stage + rec_off (2 * ((end - entry) / n) + 4 records)
    uint64_t kb;       // with probe results (WalkArgs::ahit): block k's at ahit[k - kb]
    uint32_t file;     // basis file (FileIx) of the index
    uint32_t final_;   // 1: the source ends in this unit (tail rule, last literal run to len)
};
struct WalkFileOut {
    uint32_t base, count;  // the unit's records: out[base, base + count)
    uint32_t weak_hits;    // candidate windows verified (passed the Bloom filter)
    uint32_t hits;         // windows classified as hits
    uint64_t exit;         // where the walk left the unit (>= end; a final unit: len)
    uint64_t pad;
};
// The op lists of a batch's walk expanded on the device (WalkArgs::x, k_walk_files): the
// last unit of each file to finish joins the file's units' staged records (a Data op ending at a unit's end merged with the next
// unit's first; a unit entered past its start cut at the previous unit's exit when its
// leading literal run reaches it -- match_walk_files' rules), then writes every op
// (sydelta_op, generator.rs:10-15: a Copy per block of a copy run) at ops + op_off[f], in
// host-mapped memory.  A file whose units do not chain that way (it needs a re-walk), whose
// records exceed the wave's LDS or whose ops exceed op_off[f + 1] - op_off[f] gets bad = 1 and
// no ops.
struct ExpandOut {
    uint64_t nops, data_ops, lit;
    uint32_t weak_hits, hits, bad, pad;
};
struct ExpandArgs {
    const WalkUnit* units;       // the walk's unit table (device)
    const WalkFileOut* fout;     // its per-unit results (device copy)
    const WalkRec* stage;        // its staged records (unit u's at stage + units[u].rec_off)
    const uint32_t* fu;          // nf + 1: file f's units [fu[f], fu[f + 1])
    const uint64_t* fblk;        // the index's block prefix
    const uint64_t* last_size;   // per file
    const uint64_t* op_off;      // nf + 1: file f's ops at ops + op_off[f], capacity to op_off[f + 1]
    sydelta_op* ops;
    ExpandOut* res;              // per file
    uint32_t nf, n;
};
struct WalkArgs {
    const uint8_t* base;         // launch base
    const WalkUnit* units;
    const uint64_t* last_size;   // per basis file (0: empty signature)
    uint32_t nunits, n, nm;
    uint32_t self_nb;            // self-indexed: the most blocks of any unit's file (<= kSelfIxMaxBlocks);
                                 // 0: the index's filter and tables are read from global memory
    const FileIx* files;
    const uint64_t* fblk;
    const uint32_t* filt;
    const uint32_t* keys;
    const uint32_t* start;
    const uint32_t* cnt;
    const uint32_t* order;
    const uint64_t* cstrong;
    const uint32_t* weak;        // the index's signature copies (the tail rule)
    const uint64_t* strong;
    const uint32_t* ahit;        // optional: the aligned probe's results (block k: its hit or none, or
                                 // launch_preroll's) ...
    const uint32_t* apw;         // ... and its windows' weak values
    WalkRec* stage;              // may be host-mapped memory (with out NULL)
    WalkRec* out;                // compacted records of every unit; NULL: left in stage (base = rec_off)
    WalkFileOut* fout;
    WalkFileOut* fout_dev;       // optional: a device copy of fout (the expansion reads it)
    unsigned long long* total;   // records placed in out (zeroed before the launch)
    unsigned long long* ticks;   // SYDELTA_PHASE_TIMING: 16 counters (zeroed), else null
    ExpandArgs x;                // self-indexed batches: x.ops set -> the op lists expanded on the device
    uint32_t* xdone;             // ... with per-file unit counters (zeroed)
};
// slim: the walk of units whose aligned misses were pre-rolled (launch_preroll; a.ahit set,
// the filter in global memory), for the units whose walk stays on the aligned grid; it marks
// them done (kUnitDone in WalkUnit::final_, the unit table written), and a full launch after it
// walks the others.  The unit table must not be reused for another slim launch.
constexpr uint32_t kUnitDone = 2;
hipError_t launch_walk_files(const WalkArgs& a, hipStream_t s, Profiler* prof, bool slim = false);
// A chunk's op list written on the device (chunk_pipe_finish with SYDELTA_DEVICE_EXPAND): the
// host chains the units of a part from its copy of their records (a leading literal run cut at
// the previous unit's exit, a Data op merged into the previous one) and hands each unit a plan;
// one wave per unit writes the unit's ops from its staged records (generator.rs:10-15's ops: a
// Copy per block of a copy run) into `ops` (host memory the device can write).
struct CxPlan {
    uint64_t first;   // the unit's first op (index into ops)
    uint64_t ext;     // bytes added to the unit's last op (a Data op: later units' leading Data)
    uint64_t r0_off;  // flags & 1: record `skip` cut to start here ...
    uint32_t r0_a;    // ... with this length
    uint32_t cnt;     // the unit's staged records
    uint32_t skip;    // leading records not written (cut away, or merged into the previous op)
    uint32_t flags;
};
hipError_t launch_chunk_write(const WalkUnit* units, const WalkRec* stage, const CxPlan* plan, uint32_t nunits,
                              uint32_t n, uint64_t nbf, uint64_t ls, sydelta_op* ops, hipStream_t s, Profiler* prof);
// K10's pre-roll of a chunk's aligned misses: every block r in [b0, b1) (relative to kb)
// whose aligned probe missed (ahit[r] == kNoBlock) is rolled: the first verified hit among
// the window starts (x, min(x + n, pend)), x = (kb + r) n, replaces the probe's results:
// ahit[r] = its block | kPreMark (kPreNone: none), apw[r] = its offset from x (bits 0-13)
// | the windows verified << 14.  k_walk_files takes such a miss's result instead of rolling.
// One wave per miss from a list (list[0, *count): count zeroed before, room for b1 - b0);
// `waves` waves loop over it.  a: the chunk's K10 arguments (one file; the filter from
// global memory; block ids below kPreMark).
constexpr uint32_t kPreMark = 0x80000000u, kPreNone = 0xFFFFFFFEu;
// More than max_miss misses (a shifted source): nothing is pre-rolled (the walk rolls what it meets).
hipError_t launch_preroll(const WalkArgs& a, uint32_t* ahit, uint32_t* apw, uint64_t kb, uint64_t b0, uint64_t b1,
                          uint64_t pend, uint64_t len, uint32_t* list, unsigned long long* count, uint32_t waves,
                          uint64_t max_miss, hipStream_t s, Profiler* prof);
// One slice (<= 64 KiB) of an op for the device apply: out[dst, dst+len) =
// (from_basis ? basis : lit)[src, src+len).
struct ApplyPiece {
    uint64_t dst;
    uint64_t src;
    uint32_t len;
    uint32_t from_basis;
};
hipError_t launch_apply(const ApplyPiece* d_pieces, uint64_t npieces, const uint8_t* d_basis, const uint8_t* d_lit,
                        uint8_t* d_out, hipStream_t s, Profiler* prof);
// Delta JSON on the device (K7).  A piece is a Copy op (a = offset, b = size) or a
// chunk of <= kJsonChunk literal bytes of a Data op (lit[src, src+len)).
constexpr uint32_t kJsonData = 1, kJsonFirst = 2, kJsonLast = 4, kJsonSep = 8;
constexpr uint32_t kJsonChunk = 4096;
constexpr uint32_t kJsonStage = 4 * kJsonChunk + 32;  // LDS text staging per chunk
struct JsonPiece {
    uint64_t src;
    uint64_t a, b;
    uint32_t len;
    uint32_t flags;
};
hipError_t launch_json_len(const JsonPiece* d_pieces, uint64_t npieces, const uint8_t* d_lit, uint64_t* d_len,
                           hipStream_t s, Profiler* prof);
hipError_t launch_json_write(const JsonPiece* d_pieces, uint64_t npieces, const uint8_t* d_lit,
                             const uint64_t* d_off, uint64_t base, uint8_t* d_out, hipStream_t s, Profiler* prof);
hipError_t launch_exclusive_sum_u64(const uint64_t* d_in, uint64_t* d_out, uint64_t n, hipStream_t s);
// Signature JSON (sydelta_sigjson.hpp, K7s): d_tile_len[t] = text length of entries
// [t * kTile, +kTile); then tile t's text at d_out + d_tile_off[t].
hipError_t launch_sigjson_len(const sigjson::SigArgs& a, uint64_t* d_tile_len, hipStream_t s, Profiler* prof);
hipError_t launch_sigjson_write(const sigjson::SigArgs& a, const uint64_t* d_tile_off, uint8_t* d_out, hipStream_t s,
                                Profiler* prof);
// Signature JSON parse (K7p): d_count[c] = '{' in 64-byte chunk c; then with d_rank (its
// exclusive scan) every entry parsed into d_out[rank] (d_out NULL or rank >= cap: checked
// only); *d_bad = the first bad position (atomicMin; initialised to UINT64_MAX).
hipError_t launch_sigparse_count(const uint8_t* d_text, uint64_t len, uint64_t* d_count, hipStream_t s, Profiler* prof);
hipError_t launch_sigparse(const uint8_t* d_text, uint64_t len, const uint64_t* d_rank, sydelta_block_checksum* d_out,
                           uint64_t cap, unsigned long long* d_bad, hipStream_t s, Profiler* prof);
// Delta JSON parse (K7d, sydelta_dparse.hpp): per-chunk op / literal starts, op start
// positions by rank, then ops and literal bytes (d_lit NULL: checked only); *d_bad =
// the first bad position (atomicMin; initialised to UINT64_MAX).
hipError_t launch_dparse_count(const dparse::DArgs& a, uint64_t* d_ocnt, uint64_t* d_lcnt, hipStream_t s,
                               Profiler* prof);
hipError_t launch_dparse_place(const dparse::DArgs& a, const uint64_t* d_orank, uint64_t* d_pos, hipStream_t s,
                               Profiler* prof);
hipError_t launch_dparse(const dparse::DArgs& a, const uint64_t* d_orank, const uint64_t* d_lrank, const uint64_t* d_pos,
                         uint64_t nops, sydelta_op* d_ops, uint8_t* d_lit, unsigned long long* d_bad, hipStream_t s,
                         Profiler* prof);
// zstd frame of a text in HBM (sydelta_zstd.hpp).  Blocks [b0, b0 + nb) of d_text (len
// bytes, 16-byte aligned, readable to the end of its last granule): slot i of d_slots
// (zstd::kBlockMax bytes each) gets block b0+i's content, d_size[i] its size, d_type[i]
// its type, d_len64[i] = 3 + size; d_lz holds nb * zstd::kSeqScratchBytes of literals +
// sequences scratch (zstd::seq_scratch_at).  Then launch_zstd_frame writes them behind their block
// headers at d_out + base + d_off[i] (d_off: exclusive prefix of d_len64), and the frame
// header when b0 == 0.
hipError_t zstd_phase_ticks(unsigned long long* out);  // SYDELTA_PHASE_TIMING (k_zstd_block)
hipError_t launch_zstd_blocks(const uint8_t* d_text, uint64_t len, uint64_t b0, uint32_t nb, uint8_t* d_slots,
                              uint8_t* d_lz, uint32_t* d_size, uint32_t* d_type, uint64_t* d_len64,
                              hipStream_t s, Profiler* prof);
hipError_t launch_zstd_frame(const uint8_t* d_text, uint64_t len, uint64_t b0, uint32_t nb, uint64_t nblocks,
                             const uint8_t* d_slots, const uint32_t* d_size, const uint32_t* d_type, const uint64_t* d_off,
                             uint64_t base, uint8_t* d_out, hipStream_t s, Profiler* prof);
// Local path: changed[k] = block k of src differs from block k of dst (k < ceil(slen/bs)).
hipError_t launch_block_cmp(const uint8_t* d_src, uint64_t slen, const uint8_t* d_dst, uint64_t dlen, uint64_t bs,
                            uint8_t* d_changed, hipStream_t s, Profiler* prof);
// out[i] = XXH3-64 of block pos[i] of buf (clipped at len, empty past the end).
hipError_t launch_hash_blocks(const uint8_t* d_buf, uint64_t len, uint64_t bs, const uint64_t* d_pos, uint32_t count,
                              uint64_t* d_out, hipStream_t s);
// Whole-file XXH3-64 of files (d_off[f], d_len[f]) of d_buf: d_pfx = prefix of full
// 1 KiB block counts ((len-1)/1024 for len > 240, else 0), (d_aoff, d_apfx) the same
// for the nact files with >= 1 block (d_apfx[nact] = npieces), d_order = files by block
// count descending, d_C = 8 rows of xxh_chain_records(npieces) u64 of scratch, d_out[f] = hash.
constexpr uint64_t xxh_chain_records(uint64_t npieces) { return npieces + 3 * 32; }
hipError_t launch_xxh_files(const uint8_t* d_buf, const uint64_t* d_off, const uint64_t* d_len, const uint64_t* d_pfx,
                            const uint64_t* d_aoff, const uint64_t* d_apfx, uint64_t nact, const uint32_t* d_order,
                            uint64_t nfiles, uint64_t npieces, uint64_t* d_C, uint64_t* d_out,
                            hipStream_t s, Profiler* prof);
// Batched signature when bs % 64 == 0, bs >= 256 and every file starts 16-byte aligned:
// full blocks of the nact files with >= 1 (aoff, agb = first global block, apfx = prefix
// of full-block counts, apfx[nact] = nfull) by the row kernel, then npart listed
// segments (loff, llen, output slot lidx) one wave each.
hipError_t launch_signature_batch_fast(const uint8_t* d_buf, const uint64_t* d_aoff, const uint64_t* d_agb,
                                       const uint64_t* d_apfx, uint64_t nact, uint64_t nfull, const uint64_t* d_loff,
                                       const uint64_t* d_llen, const uint64_t* d_lidx, uint64_t npart, uint64_t bs,
                                       uint32_t* d_weak, uint64_t* d_strong, hipStream_t s, Profiler* prof);
hipError_t launch_synth_fill(uint8_t* d_buf, uint64_t len, uint64_t seed, hipStream_t s, uint64_t first = 0);
hipError_t launch_synth_edit_blocks(uint8_t* d_dst, uint64_t len, uint64_t bs, uint64_t first, uint64_t seed,
                                    uint32_t rate_ppm, hipStream_t s);
hipError_t launch_synth_mutate(uint8_t* d_dst, const uint8_t* d_src, uint64_t len, uint64_t seed, uint32_t rate_ppm,
                               hipStream_t s);

}  // namespace sydelta
