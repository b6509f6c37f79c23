// sydelta_sigjson.hpp — K7s: serde_json's compact text of a device-resident signature,
// `serde_json::to_string(&Vec<BlockChecksum>)`, the line `sy-remote checksums` prints
// (sy-remote.rs:146-147) and ssh.rs:967-973 parses on the sender.
//
//   [{"index":0,"offset":0,"size":4096,"weak":123,"strong":456},{"index":1,...}]
//
// Field order and names follow the derived Serialize of checksum.rs:9-21; numbers are
// plain decimal (serde_json's itoa).  The signature is the SoA sydelta_signature_device
// writes (weak u32, strong u64 per block, index order); index, offset = index * bs and
// size (bs, the last block last_size) are implied.
//
// Layout of the text: entry i is one separator ('[' before entry 0, ',' before the
// others), the 46 fixed characters of the keys and braces, its five numbers, and ']'
// after the last entry, so the whole text is the concatenation of the entries.  One
// workgroup writes kTile consecutive entries: k_sigjson_len sums their lengths per tile,
// an exclusive scan places the tiles, and k_sigjson_write composes each tile's text in
// LDS (a workgroup scan places the entries) and stores it with 16-byte stores on the
// aligned chunks it covers entirely, byte stores on the two edge chunks it shares with
// its neighbours.
//
// The sender's side (ssh.rs:967-973, serde_json::from_str::<Vec<BlockChecksum>>) parses
// the same text: on the device when it is exactly this compact form (K7p, parse_entry):
// every '{' starts an entry, so one thread per 64-byte chunk counts its '{', an exclusive
// scan ranks them, and each '{' is parsed by the thread whose chunk holds it, which also
// checks the characters around its entry ('[' or "},"  before, ',' + '{' or the final
// ']' after).  The entries then form one chain from byte 1 to the last, so every byte of
// the text is checked by some thread.  Any other spelling serde accepts (whitespace,
// other key orders, unknown keys) is refused with its position and goes to the host
// parser (sydelta_checksums_from_json).
//
// Every function below is the body of one thread (sydelta_kernels.hip); the host
// emulation of the device layer (tests/csrc/fake_device.cpp) and the sanitizer build
// (tests/csrc/kernel_bodies_fuzz.cpp) run the same bodies on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sydelta.h"

namespace sydelta {
namespace sigjson {

constexpr uint32_t kTile = 256;   // entries per workgroup
constexpr uint32_t kFixed = 46;   // {"index": ,"offset": ,"size": ,"weak": ,"strong": }
constexpr uint32_t kMaxEntry = 1 + kFixed + 20 + 20 + 20 + 10 + 20 + 1;  // 138
constexpr uint32_t kStage = kTile * kMaxEntry;                          // LDS bytes per tile

struct SigArgs {
    const uint32_t* weak;
    const uint64_t* strong;
    uint64_t n;      // entries
    uint64_t bs;     // block size: offset = index * bs
    uint64_t last;   // size of the last block, in (0, bs]
};

__host__ __device__ inline uint32_t digits(uint64_t v) {
    uint32_t d = 1;
    uint64_t p = 10;
    while (d < 20 && v >= p) {
        ++d;
        p *= 10;
    }
    return d;
}

// Decimal digits of v at p; returns their count.
__host__ __device__ inline uint32_t put_dec(uint8_t* p, uint64_t v) {
    const uint32_t d = digits(v);
    for (uint32_t k = d; k-- > 0;) {
        p[k] = (uint8_t)('0' + v % 10);
        v /= 10;
    }
    return d;
}

__host__ __device__ inline uint64_t size_of(const SigArgs& a, uint64_t i) { return i + 1 == a.n ? a.last : a.bs; }

// Length of entry i's text (separator and, for the last, the closing ']' included).
__host__ __device__ inline uint32_t entry_len(const SigArgs& a, uint64_t i) {
    return 1 + kFixed + digits(i) + digits(i * a.bs) + digits(size_of(a, i)) + digits(a.weak[i]) +
           digits(a.strong[i]) + (i + 1 == a.n ? 1u : 0u);
}

__host__ __device__ inline uint32_t put_str(uint8_t* p, const char* s) {
    uint32_t k = 0;
    while (s[k]) {
        p[k] = (uint8_t)s[k];
        ++k;
    }
    return k;
}

// Entry i's text at p; returns its length (== entry_len(a, i)).
__host__ __device__ inline uint32_t entry_write(const SigArgs& a, uint64_t i, uint8_t* p) {
    uint32_t k = 0;
    p[k++] = i == 0 ? '[' : ',';
    k += put_str(p + k, "{\"index\":");
    k += put_dec(p + k, i);
    k += put_str(p + k, ",\"offset\":");
    k += put_dec(p + k, i * a.bs);
    k += put_str(p + k, ",\"size\":");
    k += put_dec(p + k, size_of(a, i));
    k += put_str(p + k, ",\"weak\":");
    k += put_dec(p + k, a.weak[i]);
    k += put_str(p + k, ",\"strong\":");
    k += put_dec(p + k, a.strong[i]);
    p[k++] = '}';
    if (i + 1 == a.n) p[k++] = ']';
    return k;
}

// One thread's share of a tile's store: the 16-byte-aligned chunk at address c of the
// destination range [dst, dst + len), whose bytes are stage[0, len).  A chunk inside
// the range is one 16-byte store; an edge chunk (shared with the neighbouring tile's
// text or outside the output) gets byte stores of its bytes in the range only.
__host__ __device__ inline void store_chunk(const uint8_t* stage, uint32_t len, uint8_t* dst, uintptr_t c) {
    const uintptr_t d0 = (uintptr_t)dst, d1 = d0 + len;
    const uintptr_t lo = c < d0 ? d0 : c, hi = c + 16 < d1 ? c + 16 : d1;
    if (lo >= hi) return;
    const uint8_t* s = stage + (lo - d0);
    if (lo == c && hi == c + 16) {
        uint32_t w[4];
        for (int j = 0; j < 4; ++j)
            w[j] = (uint32_t)s[4 * j] | ((uint32_t)s[4 * j + 1] << 8) | ((uint32_t)s[4 * j + 2] << 16) |
                   ((uint32_t)s[4 * j + 3] << 24);
        *(uint4*)c = make_uint4(w[0], w[1], w[2], w[3]);
        return;
    }
    for (uintptr_t x = lo; x < hi; ++x) *(uint8_t*)x = s[x - lo];
}

// ---- parse (K7p)
constexpr uint32_t kParseChunk = 64;  // text bytes per thread

// Unsigned decimal at t[p]: digits only, no leading zero unless the number is 0, value <=
// maxv.  Returns the digits consumed (0: not a number in range).
// T: a byte pointer, or any type with operator[](uint64_t) -> uint8_t (the device parsers'
// LDS-staged text, sydelta_dparse.hpp LdsText)
template <class T>
__host__ __device__ inline uint32_t get_dec(const T& t, uint64_t len, uint64_t p, uint64_t maxv, uint64_t& v) {
    uint64_t x = 0;
    uint32_t k = 0;
    while (p + k < len && t[p + k] >= '0' && t[p + k] <= '9') {
        const uint64_t d = (uint64_t)(t[p + k] - '0');
        if (x > (maxv - d) / 10) return 0;
        x = x * 10 + d;
        ++k;
    }
    if (k == 0 || (k > 1 && t[p] == '0')) return 0;
    v = x;
    return k;
}

template <class T>
__host__ __device__ inline bool get_lit(const T& t, uint64_t len, uint64_t& p, const char* s) {
    for (uint32_t k = 0; s[k]; ++k, ++p)
        if (p >= len || t[p] != (uint8_t)s[k]) return false;
    return true;
}

// The entry whose '{' is at t[p], in exactly the compact form, with the right characters
// before and after it; fills r.  False otherwise.
__host__ __device__ inline bool parse_entry(const uint8_t* t, uint64_t len, uint64_t p, sydelta_block_checksum& r) {
    if (!(p == 1 ? t[0] == '[' : p >= 2 && t[p - 1] == ',' && t[p - 2] == '}')) return false;
    uint64_t q = p, v = 0;
    uint32_t k;
    if (!get_lit(t, len, q, "{\"index\":") || !(k = get_dec(t, len, q, UINT64_MAX, v))) return false;
    r.index = v;
    q += k;
    if (!get_lit(t, len, q, ",\"offset\":") || !(k = get_dec(t, len, q, UINT64_MAX, v))) return false;
    r.offset = v;
    q += k;
    if (!get_lit(t, len, q, ",\"size\":") || !(k = get_dec(t, len, q, UINT64_MAX, v))) return false;
    r.size = v;
    q += k;
    if (!get_lit(t, len, q, ",\"weak\":") || !(k = get_dec(t, len, q, 0xFFFFFFFFull, v))) return false;
    r.weak = (uint32_t)v;
    r.reserved = 0;
    q += k;
    if (!get_lit(t, len, q, ",\"strong\":") || !(k = get_dec(t, len, q, UINT64_MAX, v))) return false;
    r.strong = v;
    q += k;
    if (!get_lit(t, len, q, "}")) return false;
    return q < len && ((t[q] == ',' && q + 1 < len && t[q + 1] == '{') || (t[q] == ']' && q + 1 == len));
}

// '{' in chunk c of the text.
__host__ __device__ inline uint32_t chunk_entries(const uint8_t* t, uint64_t len, uint64_t c) {
    uint32_t m = 0;
    for (uint64_t p = c * kParseChunk; p < len && p < (c + 1) * kParseChunk; ++p) m += t[p] == '{';
    return m;
}

// Chunk c's entries, ranked from rank: parsed into out[rank..] (out NULL or past cap:
// checked only); returns the first bad position in the chunk or UINT64_MAX.  Chunk 0
// also checks the head: "[]" or "[{".
__host__ __device__ inline uint64_t chunk_parse(const uint8_t* t, uint64_t len, uint64_t c, uint64_t rank,
                                               sydelta_block_checksum* out, uint64_t cap) {
    if (c == 0 && !(len >= 2 && t[0] == '[' && (len == 2 ? t[1] == ']' : t[1] == '{'))) return 0;
    for (uint64_t p = c * kParseChunk; p < len && p < (c + 1) * kParseChunk; ++p) {
        if (t[p] != '{') continue;
        sydelta_block_checksum r;
        if (!parse_entry(t, len, p, r)) return p;
        if (out && rank < cap) out[rank] = r;
        ++rank;
    }
    return UINT64_MAX;
}

// sum_{i < n} digits(i * m), in O(20): digits(v) = 1 + #{d >= 1 : v >= 10^d}, and
// #{i < n : i * m >= T} = n - min(n, ceil(T / m)).
inline uint64_t sum_digits_mult(uint64_t n, uint64_t m) {
    uint64_t s = n;
    uint64_t T = 10;
    for (int d = 1; d < 20; ++d, T *= 10) {
        const uint64_t first = (T + m - 1) / m;  // smallest i with i * m >= T
        if (first < n) s += n - first;
        if (T > UINT64_MAX / 10) break;
    }
    return s;
}

// Bounds of the text length from the implied fields alone (weak takes 1-10 digits,
// strong 1-20): the host checks the device's total against them before writing.
inline void text_bounds(uint64_t n, uint64_t bs, uint64_t last, uint64_t& lo, uint64_t& hi) {
    if (n == 0) {
        lo = hi = 2;  // []
        return;
    }
    const uint64_t fixed = n * (1 + kFixed) + 1 + sum_digits_mult(n, 1) + sum_digits_mult(n, bs) +
                           (n - 1) * digits(bs) + digits(last);
    lo = fixed + n * 2;
    hi = fixed + n * 30;
}

}  // namespace sigjson
}  // namespace sydelta
