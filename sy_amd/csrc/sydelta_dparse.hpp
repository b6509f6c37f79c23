// sydelta_dparse.hpp — K7d: the receiver's parse of the Delta JSON on the device,
// `serde_json::from_str::<Delta>` (sy-remote.rs:175) for text in the compact form the
// sender writes (serde_json::to_string, ssh.rs:1003; sydelta_delta_to_json_device):
//
//   {"ops":[{"Copy":{"offset":O,"size":S}},{"Data":[b0,b1,...]},...],"source_size":N,"block_size":B}
//
// The head (`{"ops":[`) and the tail (`],"source_size":N,"block_size":B}`) are checked on
// the host; the device parses the ops region R = [8, E) between them.  In the compact
// form, inside R:
//   * an op starts at each '{' at 8 or right after "},";
//   * a literal byte starts at each digit right after '[' or ',' (the Copy fields' digits
//     follow ':'), so literal k of the delta is the k-th such digit;
// so one thread per 64-byte chunk counts both, two exclusive scans rank them, the op
// starts are placed by rank, and then each thread parses the ops and literal bytes that
// start in its chunk: a Copy op whole, a Data op's head (its literal range is the count
// of literal starts between its '{' and the next op's), each literal byte with the
// character after it (',' + digit, or "]}" + the next op / the end).  The ops and the
// literals between them then chain from 8 to E, so every byte of R is checked by some
// thread.  Any other spelling is refused with its first byte; the host parser
// (sydelta_delta_from_json) takes those.
//
// Every function below is the body of one thread (sydelta_kernels.hip); the host
// emulation of the device layer (tests/csrc/fake_device.cpp) and the sanitizer build
// (tests/csrc/kernel_bodies_fuzz.cpp) run the same bodies on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sydelta.h"
#include "sydelta_sigjson.hpp"  // get_dec, get_lit

namespace sydelta {
namespace dparse {

constexpr uint32_t kChunk = 64;   // text bytes per thread
constexpr uint64_t kHead = 8;     // {"ops":[
constexpr uint64_t kNoBad = UINT64_MAX;

struct DArgs {
    const uint8_t* t;  // the whole text
    uint64_t e;        // end of the ops region (its ']')
    uint64_t nc;       // chunks of [kHead, e)
};

__host__ __device__ __forceinline__ bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
// T: the text as a byte pointer, or any type with operator[](uint64_t) -> uint8_t (the
// kernels read their wave's tile from LDS, LdsText in sydelta_kernels.hip)
template <class T>
__host__ __device__ __forceinline__ bool op_start(const T& t, uint64_t p) {
    return t[p] == '{' && (p == kHead || (t[p - 1] == ',' && t[p - 2] == '}'));
}
template <class T>
__host__ __device__ __forceinline__ bool lit_start(const T& t, uint64_t p) {
    return is_digit(t[p]) && (t[p - 1] == '[' || t[p - 1] == ',');
}
__host__ __device__ __forceinline__ uint64_t chunk_lo(const DArgs& a, uint64_t c) { return kHead + c * kChunk; }
__host__ __device__ __forceinline__ uint64_t chunk_hi(const DArgs& a, uint64_t c) {
    const uint64_t h = kHead + (c + 1) * kChunk;
    return h < a.e ? h : a.e;
}

// Op starts and literal starts in chunk c.
template <class T>
__host__ __device__ inline void chunk_count(const DArgs& a, const T& t, uint64_t c, uint64_t& nops, uint64_t& nlit) {
    nops = nlit = 0;
    for (uint64_t p = chunk_lo(a, c); p < chunk_hi(a, c); ++p) {
        nops += op_start(t, p);
        nlit += lit_start(t, p);
    }
}
__host__ __device__ inline void chunk_count(const DArgs& a, uint64_t c, uint64_t& nops, uint64_t& nlit) {
    chunk_count(a, a.t, c, nops, nlit);
}

// Position of every op start of chunk c, by rank.
template <class T>
__host__ __device__ inline void chunk_place(const DArgs& a, const T& t, uint64_t c, uint64_t rank, uint64_t* pos) {
    for (uint64_t p = chunk_lo(a, c); p < chunk_hi(a, c); ++p)
        if (op_start(t, p)) pos[rank++] = p;
}
__host__ __device__ inline void chunk_place(const DArgs& a, uint64_t c, uint64_t rank, uint64_t* pos) {
    chunk_place(a, a.t, c, rank, pos);
}

// Literal starts before position x (kHead <= x <= e): the chunk's rank plus a recount.
template <class T>
__host__ __device__ inline uint64_t lits_before(const DArgs& a, const T& t, const uint64_t* lrank, uint64_t x) {
    if (x >= a.e) return lrank[a.nc];  // lrank holds nc + 1 entries: the total last
    const uint64_t c = (x - kHead) / kChunk;
    uint64_t r = lrank[c];
    for (uint64_t p = chunk_lo(a, c); p < x; ++p) r += lit_start(t, p);
    return r;
}

// What may follow an op ending at q: ',' and the next op's '{', or the region's end.
template <class T>
__host__ __device__ __forceinline__ bool op_follow(const DArgs& a, const T& t, uint64_t q) {
    return q == a.e || (q + 1 < a.e && t[q] == ',' && t[q + 1] == '{');
}

// Chunk c's ops and literal bytes.  orank/lrank: exclusive scans (lrank with the total
// at nc), pos: op starts by rank (nops entries).  Writes ops[rank] (kind, a = literal
// offset or basis offset, b = size) and lit[rank] (lit NULL: checked only; L: a byte
// pointer, or a type with operator bool and operator[](uint64_t) -> uint8_t&, the kernel's
// LDS staging).  Returns the first bad position in the chunk or kNoBad.
template <class T, class L = uint8_t*>
__host__ __device__ inline uint64_t chunk_parse(const DArgs& a, const T& t, uint64_t c, const uint64_t* orank,
                                               const uint64_t* lrank, const uint64_t* pos, uint64_t nops,
                                               sydelta_op* ops, L lit) {
    const uint64_t len = a.e;  // no token of R reads past its ']'
    uint64_t ork = orank[c], lrk = lrank[c];
    // The chain starts at the first op: a non-empty region must open with one, or the
    // bytes before the first "},{" would be checked by no thread.
    if (c == 0 && a.e > kHead && !op_start(t, kHead)) return kHead;
    for (uint64_t p = chunk_lo(a, c); p < chunk_hi(a, c); ++p) {
        if (op_start(t, p)) {
            uint64_t q = p, o = 0, sz = 0;
            uint32_t k;
            sydelta_op op{};
            if (sigjson::get_lit(t, len, q, "{\"Copy\":{\"offset\":")) {
                if (!(k = sigjson::get_dec(t, len, q, UINT64_MAX, o))) return p;
                q += k;
                if (!sigjson::get_lit(t, len, q, ",\"size\":") || !(k = sigjson::get_dec(t, len, q, UINT64_MAX, sz)))
                    return p;
                q += k;
                if (!sigjson::get_lit(t, len, q, "}}") || !op_follow(a, t, q)) return p;
                op.kind = SYDELTA_OP_COPY;
                op.a = o;
                op.b = sz;
            } else {
                q = p;
                if (!sigjson::get_lit(t, len, q, "{\"Data\":[")) return p;
                if (q < len && t[q] == ']') {  // empty Data
                    ++q;
                    if (!sigjson::get_lit(t, len, q, "}") || !op_follow(a, t, q)) return p;
                } else if (!(q < len && is_digit(t[q]))) {
                    return p;  // the first literal (checked by its own thread) must start here
                }
                // the recounts reach other chunks' text (the next op may be anywhere): a.t
                const uint64_t l0 = lits_before(a, a.t, lrank, q);
                const uint64_t next = ork + 1 < nops ? pos[ork + 1] : a.e;
                op.kind = SYDELTA_OP_DATA;
                op.a = l0;
                op.b = lits_before(a, a.t, lrank, next) - l0;
            }
            ops[ork++] = op;
        } else if (lit_start(t, p)) {
            uint64_t v = 0;
            const uint32_t k = sigjson::get_dec(t, len, p, 255, v);
            if (!k) return p;
            uint64_t q = p + k;
            if (q < len && t[q] == ',') {
                if (!(q + 1 < len && is_digit(t[q + 1]))) return p;
            } else {
                if (!sigjson::get_lit(t, len, q, "]}") || !op_follow(a, t, q)) return p;
            }
            if (lit) lit[lrk] = (uint8_t)v;
            ++lrk;
        }
    }
    return kNoBad;
}
__host__ __device__ inline uint64_t chunk_parse(const DArgs& a, uint64_t c, const uint64_t* orank,
                                               const uint64_t* lrank, const uint64_t* pos, uint64_t nops,
                                               sydelta_op* ops, uint8_t* lit) {
    return chunk_parse<const uint8_t*, uint8_t*>(a, a.t, c, orank, lrank, pos, nops, ops, lit);
}

}  // namespace dparse
}  // namespace sydelta
