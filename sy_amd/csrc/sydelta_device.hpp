// sydelta_device.hpp — device-side primitives for the delta hot path (gfx950).
//
// Adler-32 (src/delta/rolling.rs:35-45) and XXH3-64 seed 0 (crate xxhash-rust
// 0.8.15, used at src/delta/checksum.rs:65-67 and generator.rs:128-130) laid
// out for 64-lane wavefronts:
//   * XXH3's long-path accumulation is additive inside each 1 KiB block, so a
//     lane computes the contribution of its 16 bytes and a 16-lane xor-shuffle
//     tree sums a block; the 3 scrambles and the merge are done redundantly by
//     every lane (they are per-accumulator, so lane q owns accumulators 2q,2q+1).
//   * Adler-32 is evaluated in closed form, A = 1 + sum(x), B = n + sum((n-i) x_i),
//     with v_dot4_u32_u8 doing the byte sums (weights 1 and the in-dword offsets).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sydelta {

constexpr uint32_t kMod = 65521u;  // rolling.rs:22

constexpr uint64_t P32_1 = 0x9E3779B1ull, P32_2 = 0x85EBCA77ull, P32_3 = 0xC2B2AE3Dull;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t P64_3 = 0x165667B19E3779F9ull, P64_4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t P64_5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t PMX1 = 0x165667919E3779F9ull, PMX2 = 0x9FB21C651E98DF25ull;

// XXH3 default secret (192 bytes).  Published constant of the algorithm.
struct SecretBytes { uint8_t b[192]; };
constexpr SecretBytes kSecretBytes = {{
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
}};

constexpr uint64_t sec64(int off) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | kSecretBytes.b[off + i];
    return v;
}
constexpr uint32_t sec32(int off) {
    return (uint32_t)kSecretBytes.b[off] | ((uint32_t)kSecretBytes.b[off + 1] << 8) |
           ((uint32_t)kSecretBytes.b[off + 2] << 16) | ((uint32_t)kSecretBytes.b[off + 3] << 24);
}

// Secret words used by the long path, all at compile time.
struct SecretTables {
    uint64_t w[24];     // sec64(8k): stripe keys (stripe s, lane i -> w[s+i]); scramble keys w[16..23]
    uint64_t last[8];   // sec64(121 + 8i): last-stripe keys (XXH_SECRET_LASTACC_START = 7)
    uint64_t merge[8];  // sec64(11 + 8k): mergeAccs keys (XXH_SECRET_MERGEACCS_START = 11)
    uint64_t init[8];   // initial accumulators
};
constexpr SecretTables make_tables() {
    SecretTables t{};
    for (int k = 0; k < 24; ++k) t.w[k] = sec64(8 * k);
    for (int i = 0; i < 8; ++i) t.last[i] = sec64(121 + 8 * i);
    for (int k = 0; k < 8; ++k) t.merge[k] = sec64(11 + 8 * k);
    const uint64_t ini[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    for (int i = 0; i < 8; ++i) t.init[i] = ini[i];
    return t;
}
// Device copies (this header is compiled into exactly one translation unit).
static __constant__ SecretTables c_tab = make_tables();
static __constant__ SecretBytes c_secret = kSecretBytes;
#define kTables c_tab

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t udot4(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_udot4(a, b, c, false);
}
__device__ __forceinline__ uint64_t fold64(uint64_t a, uint64_t b) { return (a * b) ^ __umul64hi(a, b); }
__device__ __forceinline__ uint64_t xxh3_aval(uint64_t h) {
    h ^= h >> 37; h *= PMX1; h ^= h >> 32; return h;
}
__device__ __forceinline__ uint64_t xxh64_aval(uint64_t h) {
    h ^= h >> 33; h *= P64_2; h ^= h >> 29; h *= P64_3; h ^= h >> 32; return h;
}
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl64(h, 49) ^ rotl64(h, 24); h *= PMX2; h ^= (h >> 35) + len; h *= PMX2; return h ^ (h >> 28);
}
__device__ __forceinline__ uint64_t scramble1(uint64_t a, uint64_t key) {
    a ^= a >> 47; a ^= key; return a * P32_1;
}
__device__ __forceinline__ uint64_t mul32x32(uint64_t dk) { return (uint64_t)(uint32_t)dk * (dk >> 32); }

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = (uint32_t)__shfl_xor((int)lo, m, 64);
    hi = (uint32_t)__shfl_xor((int)hi, m, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v += (uint32_t)__shfl_xor((int)v, m, 64);
    return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v += shfl_xor64(v, m);
    return v;
}

// Cross-lane sums without the LDS crossbar (ds_bpermute): DPP within a 16-lane row
// (quad_perm / row_ror) and the gfx950 permlane16/32 swaps across rows.  A rotation
// by 4 then 8 inside a row sums the 4 lanes of equal lane&3, like xor 4 / xor 8; a
// permlane swap of x with itself returns the row pair (or wave halves) as two
// values whose sum is the xor-16 (xor-32) sum on every lane.
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, false);
}
template <int kCtrl>
__device__ __forceinline__ uint64_t dpp_add64(uint64_t v) {
    const uint32_t lo = dpp32<kCtrl>((uint32_t)v), hi = dpp32<kCtrl>((uint32_t)(v >> 32));
    return v + (((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t swap16_sum32(uint32_t v) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return r[0] + r[1];
}
__device__ __forceinline__ uint32_t swap32_sum32(uint32_t v) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return r[0] + r[1];
}
__device__ __forceinline__ uint64_t swap16_sum64(uint64_t v) {
    const auto l = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap((uint32_t)(v >> 32), (uint32_t)(v >> 32), false, false);
    return ((((uint64_t)h[0]) << 32) | l[0]) + ((((uint64_t)h[1]) << 32) | l[1]);
}
__device__ __forceinline__ uint64_t swap32_sum64(uint64_t v) {
    const auto l = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap((uint32_t)(v >> 32), (uint32_t)(v >> 32), false, false);
    return ((((uint64_t)h[0]) << 32) | l[0]) + ((((uint64_t)h[1]) << 32) | l[1]);
}
constexpr int kDppQuadXor1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int kDppRowRor4 = 0x124;
constexpr int kDppRowRor8 = 0x128;
// sum over the 16 lanes with the same lane & 3 (= xor 4, 8, 16, 32)
__device__ __forceinline__ uint64_t sum_q16_64(uint64_t v) {
    v = dpp_add64<kDppRowRor4>(v);
    v = dpp_add64<kDppRowRor8>(v);
    v = swap16_sum64(v);
    return swap32_sum64(v);
}
// sum over the 4 lanes of a quad (= xor 1, 2)
__device__ __forceinline__ uint64_t sum_quad64(uint64_t v) {
    v = dpp_add64<kDppQuadXor1>(v);
    return dpp_add64<kDppQuadXor2>(v);
}
__device__ __forceinline__ uint32_t wave_sum32_dpp(uint32_t v) {
    v += dpp32<kDppQuadXor1>(v);
    v += dpp32<kDppQuadXor2>(v);
    v += dpp32<kDppRowRor4>(v);
    v += dpp32<kDppRowRor8>(v);
    v = swap16_sum32(v);
    return swap32_sum32(v);
}
__device__ __forceinline__ uint64_t wave_sum64_dpp(uint64_t v) {
    return sum_q16_64(sum_quad64(v));
}

// Unaligned little-endian loads for the rare scalar paths.  Every aligned word
// touched holds at least one byte of [p, p+n), so no access leaves the 16-byte
// granule of a valid byte (see sydelta.h conventions).
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t sh = (uint32_t)(a & 7) * 8;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint64_t lo = q[0];
    if (sh == 0) return lo;
    const uint64_t hi = q[1];
    return (lo >> sh) | (hi << (64 - sh));
}
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Adler-32 of a short run by one thread (closed form, exact for len < 2^16).
__device__ __forceinline__ uint32_t adler_scalar(const uint8_t* p, uint64_t len) {
    uint64_t s = 0, b = 0;
    for (uint64_t i = 0; i < len; ++i) {
        const uint32_t x = p[i];
        s += x;
        b += (len - i) * x;
    }
    const uint32_t A = (uint32_t)((1 + s) % kMod);
    const uint32_t B = (uint32_t)((len + b) % kMod);
    return (B << 16) | A;
}

// Runtime read of the raw secret (short paths only; hot paths use c_tab).
__device__ __forceinline__ uint64_t dsec64(int off) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i) v = (v << 8) | c_secret.b[off + i];
    return v;
}
__device__ __forceinline__ uint32_t dsec32(int off) {
    return (uint32_t)c_secret.b[off] | ((uint32_t)c_secret.b[off + 1] << 8) | ((uint32_t)c_secret.b[off + 2] << 16) |
           ((uint32_t)c_secret.b[off + 3] << 24);
}
__device__ __forceinline__ uint64_t mix16(const uint8_t* in, int soff) {
    return fold64(ld64u(in) ^ dsec64(soff), ld64u(in + 8) ^ dsec64(soff + 8));
}

// XXH3-64 for len <= 240 by one thread (xxh3 0-16 / 17-128 / 129-240 paths).
__device__ __noinline__ uint64_t xxh3_short(const uint8_t* in, uint64_t len) {
    if (len <= 16) {
        if (len > 8) {
            const uint64_t bf1 = dsec64(24) ^ dsec64(32), bf2 = dsec64(40) ^ dsec64(48);
            const uint64_t lo = ld64u(in) ^ bf1, hi = ld64u(in + len - 8) ^ bf2;
            const uint64_t acc = len + __builtin_bswap64(lo) + hi + fold64(lo, hi);
            return xxh3_aval(acc);
        }
        if (len >= 4) {
            const uint32_t i1 = ld32u(in), i2 = ld32u(in + len - 4);
            const uint64_t bf = dsec64(8) ^ dsec64(16);
            const uint64_t i64 = (uint64_t)i2 + ((uint64_t)i1 << 32);
            return rrmxmx(i64 ^ bf, len);
        }
        if (len) {
            const uint32_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
            const uint32_t comb = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
            const uint64_t bf = (uint64_t)(dsec32(0) ^ dsec32(4));
            return xxh64_aval((uint64_t)comb ^ bf);
        }
        return xxh64_aval(dsec64(56) ^ dsec64(64));
    }
    if (len <= 128) {
        uint64_t acc = len * P64_1;
        if (len > 32) {
            if (len > 64) {
                if (len > 96) { acc += mix16(in + 48, 96); acc += mix16(in + len - 64, 112); }
                acc += mix16(in + 32, 64); acc += mix16(in + len - 48, 80);
            }
            acc += mix16(in + 16, 32); acc += mix16(in + len - 32, 48);
        }
        acc += mix16(in, 0); acc += mix16(in + len - 16, 16);
        return xxh3_aval(acc);
    }
    uint64_t acc = len * P64_1;
    const uint32_t nb = (uint32_t)(len / 16);
    for (uint32_t i = 0; i < 8; ++i) acc += mix16(in + 16 * i, 16 * i);
    uint64_t acc_end = mix16(in + len - 16, 136 - 17);
    acc = xxh3_aval(acc);
    for (uint32_t i = 8; i < nb; ++i) acc_end += mix16(in + 16 * i, 16 * (i - 8) + 3);
    return xxh3_aval(acc + acc_end);
}

// Load 64 bytes at an arbitrary address as 16 little-endian dwords.
// `sh` = address & 3 must be uniform across the wave.
__device__ __forceinline__ void load64_unaligned(const uint8_t* p, uint32_t x[16]) {
    const uintptr_t a = (uintptr_t)p;
    if ((a & 15) == 0) {
        const uint4* q = (const uint4*)p;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 v = q[i];
            x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
        }
        return;
    }
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
    uint32_t d[17];
#pragma unroll
    for (int i = 0; i < 16; ++i) d[i] = q[i];
    d[16] = sh ? q[16] : 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
}

// Weights (4i, 4i+1, 4i+2, 4i+3) for in-stripe byte offsets of dword i.
__device__ __forceinline__ uint32_t offw(int i) {
    const uint32_t b = 4u * (uint32_t)i;
    return b | ((b + 1) << 8) | ((b + 2) << 16) | ((b + 3) << 24);
}

// Byte sources for wave_hash_long: global memory, or a scan tile's LDS rows
// (64-byte rows at a 17-dword stride, sydelta_kernels.hip k_scan_lds).
struct GlobalBytes {
    const uint8_t* p;
    __device__ __forceinline__ void load64(uint64_t off, uint32_t x[16]) const { load64_unaligned(p + off, x); }
    __device__ __forceinline__ uint32_t byte(uint64_t off) const { return p[off]; }
};
struct LdsRowBytes {
    const uint32_t* rows;  // LDS
    uint32_t base;         // tile offset of byte 0
    __device__ __forceinline__ uint32_t dword(uint32_t d) const { return rows[(d >> 4) * 17 + (d & 15)]; }
    __device__ __forceinline__ void load64(uint64_t off, uint32_t x[16]) const {
        const uint32_t o = base + (uint32_t)off;
        const uint32_t d0 = o >> 2, sh = o & 3;
        uint32_t d[17];
#pragma unroll
        for (int i = 0; i < 17; ++i) d[i] = dword(d0 + i);
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
    }
    __device__ __forceinline__ uint32_t byte(uint64_t off) const {
        const uint32_t o = base + (uint32_t)off;
        return (dword(o >> 2) >> (8 * (o & 3))) & 0xFF;
    }
};

// Wave-cooperative Adler-32 + XXH3-64 of an arbitrary segment [0, len) of `src`,
// len > 240.  Every lane of the wave must call it with the same arguments;
// every lane returns the same result.
template <class Src>
__device__ __forceinline__ void wave_hash_src(const Src& src, uint64_t len, uint32_t& weak_out, uint64_t& strong_out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nS = (len - 1) / 64;          // stripes consumed by the block loop
    const uint64_t nb_blocks = (len - 1) / 1024; // 1 KiB blocks followed by a scramble
    uint64_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = kTables.init[i];
    uint64_t asum = 0, bsum = 0;  // adler partial sums over this lane's bytes
    for (uint64_t k0 = 0; k0 < nS; k0 += 64) {
        const uint64_t s = k0 + lane;
        uint64_t c[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = 0;
        if (s < nS) {
            uint32_t x[16];
            src.load64(64 * s, x);
            const uint32_t ks = (uint32_t)(s & 15);
            uint32_t S = 0, V = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) { S = udot4(x[i], 0x01010101u, S); V = udot4(x[i], offw(i), V); }
            asum += S;
            bsum += (len - 64 * s) * (uint64_t)S - V;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint64_t v = (uint64_t)x[2 * i] | ((uint64_t)x[2 * i + 1] << 32);
                const uint64_t dk = v ^ kTables.w[ks + i];  // ks + i <= 22
                c[i ^ 1] += v;
                c[i] += mul32x32(dk);
            }
        }
        // sum each 16-lane group = one 1 KiB block
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            c[i] += shfl_xor64(c[i], 1); c[i] += shfl_xor64(c[i], 2);
            c[i] += shfl_xor64(c[i], 4); c[i] += shfl_xor64(c[i], 8);
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint64_t piece = k0 / 16 + m;
            if (16 * piece < nS) {
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[i] += shfl64(c[i], 16 * m);
                if (piece < nb_blocks) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) acc[i] = scramble1(acc[i], kTables.w[16 + i]);
                }
            }
        }
    }
    // bytes after the last full stripe, for Adler: [64*nS, len) (1..64 bytes)
    {
        const uint64_t o = 64 * nS + lane;
        if (o < len) {
            const uint32_t xb = src.byte(o);
            asum += xb;
            bsum += (len - o) * (uint64_t)xb;
        }
    }
    // last stripe (overlapping), identical in every lane
    {
        uint32_t x[16];
        src.load64(len - 64, x);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t v = (uint64_t)x[2 * i] | ((uint64_t)x[2 * i + 1] << 32);
            const uint64_t dk = v ^ kTables.last[i];
            acc[i ^ 1] += v;
            acc[i] += mul32x32(dk);
        }
    }
    uint64_t r = len * P64_1;
#pragma unroll
    for (int i = 0; i < 4; ++i) r += fold64(acc[2 * i] ^ kTables.merge[2 * i], acc[2 * i + 1] ^ kTables.merge[2 * i + 1]);
    strong_out = xxh3_aval(r);
    asum = wave_sum64(asum);
    bsum = wave_sum64(bsum);
    const uint32_t A = (uint32_t)((1 + asum) % kMod);
    const uint32_t B = (uint32_t)((len + bsum) % kMod);
    weak_out = (B << 16) | A;
}

__device__ __forceinline__ void wave_hash_long(const uint8_t* p, uint64_t len, uint32_t& weak_out,
                                               uint64_t& strong_out) {
    wave_hash_src(GlobalBytes{p}, len, weak_out, strong_out);
}

// splitmix64 finaliser used by the synthetic-data generator.
__host__ __device__ __forceinline__ uint64_t splitmix_word(uint64_t seed, uint64_t idx) {
    uint64_t z = idx * 0x9E3779B97F4A7C15ull + seed * 0xD1B54A32D192ED03ull;
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace sydelta
