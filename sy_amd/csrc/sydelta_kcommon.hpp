// sydelta_kcommon.hpp — device code shared by the kernel translation units
// (sydelta_kernels.hip, sydelta_filewalk.hip): the signature kernel's row layout (row_hash),
// the probe hashes and Bloom-filter tests of the index, the exact-table lookup and the
// DPP wave scan.  Included inside namespace sydelta, after sydelta_device.hpp and
// sydelta_internal.hpp.
#pragma once

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Row-per-block form (the production signature kernel): each 16-lane row of a wave
// hashes its own block, so a 1 KiB piece is reduced inside the row (two DPP
// rotations) and the accumulate/scramble fold (XXH3 long loop) runs in the row with
// no cross-row traffic.  Lane (slot, q) of a row takes stripes slot, slot+4,
// slot+8, slot+12 of each piece (accumulator pair q): a load instruction reads
// 256 contiguous bytes per row.  The next piece's loads are issued before the
// current piece is hashed.  bs % 64 == 0, bs >= 256, blocks 16-byte aligned.
struct RowPiece {
    uint4 v[4];
};
template <bool kAligned = true>
__device__ __forceinline__ void load_piece(const uint8_t* __restrict__ p, uint32_t slot, uint32_t q, uint32_t lim,
                                           RowPiece& r) {
    // bytes [0, lim) of the piece are valid (lim <= 1024, a multiple of 16 here); the
    // rest reads as zero.  Unaligned pieces: a 4-byte aligned 16-byte load plus one
    // dword, funnel-shifted (alignbyte) into place.
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t off = ((slot + 4 * k) << 6) + (q << 4);
        r.v[k] = make_uint4(0, 0, 0, 0);
        if (off < lim) {
            if (kAligned) {
                const u32x4 x = __builtin_nontemporal_load((const u32x4*)(p + off));
                r.v[k] = make_uint4(x.x, x.y, x.z, x.w);
            } else {
                const uintptr_t u = (uintptr_t)(p + off);
                const uint32_t sh = (uint32_t)(u & 3);
                const uint32_t* w = (const uint32_t*)(u & ~(uintptr_t)3);
                u32x4 x;
                __builtin_memcpy(&x, w, 16);
                const uint32_t d4 = sh ? w[4] : 0u;
                r.v[k] = make_uint4(__builtin_amdgcn_alignbyte(x.y, x.x, sh), __builtin_amdgcn_alignbyte(x.z, x.y, sh),
                                    __builtin_amdgcn_alignbyte(x.w, x.z, sh), __builtin_amdgcn_alignbyte(d4, x.w, sh));
            }
        }
    }
}

template <bool kLast>
__device__ __forceinline__ void hash_piece(const RowPiece& r, uint32_t slot, uint32_t q, uint32_t poff, uint32_t bs,
                                           const uint64_t (&kk0)[4], const uint64_t (&kk1)[4], uint32_t last_k,
                                           uint32_t last_slot, uint64_t k0l, uint64_t k1l, uint32_t& asum,
                                           uint32_t& vsum, uint64_t& bpos, uint64_t& c_lo, uint64_t& c_hi) {
    c_lo = 0;
    c_hi = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint4 v = r.v[k];
        const uint32_t off = poff + ((slot + 4 * k) << 6) + (q << 4);
        uint32_t s = udot4(v.x, 0x01010101u, 0);
        s = udot4(v.y, 0x01010101u, s);
        s = udot4(v.z, 0x01010101u, s);
        s = udot4(v.w, 0x01010101u, s);
        uint32_t u = udot4(v.x, 0x03020100u, 0);
        u = udot4(v.y, 0x07060504u, u);
        u = udot4(v.z, 0x0B0A0908u, u);
        u = udot4(v.w, 0x0F0E0D0Cu, u);
        asum += s;
        vsum += u;
        bpos += (uint64_t)(bs - off) * s;  // s == 0 past the end
        uint64_t k0 = kk0[k], k1 = kk1[k];
        if (kLast && k == (int)last_k && slot == last_slot) { k0 = k0l; k1 = k1l; }
        const uint64_t w0 = (uint64_t)v.x | ((uint64_t)v.y << 32);
        const uint64_t w1 = (uint64_t)v.z | ((uint64_t)v.w << 32);
        uint64_t p_lo = mul32x32(w0 ^ k0) + w1;
        uint64_t p_hi = mul32x32(w1 ^ k1) + w0;
        if (kLast && off >= bs) { p_lo = 0; p_hi = 0; }
        c_lo += p_lo;
        c_hi += p_hi;
    }
    c_lo = dpp_add64<kDppRowRor4>(c_lo);
    c_lo = dpp_add64<kDppRowRor8>(c_lo);
    c_hi = dpp_add64<kDppRowRor4>(c_hi);
    c_hi = dpp_add64<kDppRowRor8>(c_hi);
}

// Hash of the window [base, base + bs) of this lane's row; the result is valid in
// the row's first lane (lane & 15 == 0).  All four rows of the wave must call it
// (DPP inside rows only; rows may pass different windows of the same bs).
template <bool kAligned = true>
__device__ __forceinline__ void row_hash(const uint8_t* __restrict__ base, uint32_t bs, uint32_t& weak_out,
                                         uint64_t& strong_out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t q = lane & 3, slot = (lane >> 2) & 3;
    const uint32_t npieces = (bs + 1023) >> 10;
    const uint32_t ls = (bs >> 6) - 1 - ((npieces - 1) << 4);  // last stripe inside the last piece
    const uint32_t last_k = ls >> 2, last_slot = ls & 3;
    uint64_t kk0[4], kk1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        kk0[k] = c_tab.w[slot + 4 * k + 2 * q];
        kk1[k] = c_tab.w[slot + 4 * k + 2 * q + 1];
    }
    const uint64_t k0l = c_tab.last[2 * q], k1l = c_tab.last[2 * q + 1];
    const uint64_t sk0 = c_tab.w[16 + 2 * q], sk1 = c_tab.w[16 + 2 * q + 1];
    uint64_t acc_lo = c_tab.init[2 * q], acc_hi = c_tab.init[2 * q + 1];
    uint32_t asum = 0, vsum = 0;
    uint64_t bpos = 0;
    RowPiece cur, nxt;
    load_piece<kAligned>(base, slot, q, npieces > 1 ? 1024u : bs, cur);
    for (uint32_t j = 0; j + 1 < npieces; ++j) {  // full pieces, each followed by a scramble
        const uint32_t nlim = (j + 2 < npieces) ? 1024u : bs - ((j + 1) << 10);
        load_piece<kAligned>(base + ((j + 1) << 10), slot, q, nlim, nxt);
        uint64_t c_lo, c_hi;
        hash_piece<false>(cur, slot, q, j << 10, bs, kk0, kk1, 0, 0, k0l, k1l, asum, vsum, bpos, c_lo, c_hi);
        acc_lo = scramble1(acc_lo + c_lo, sk0);
        acc_hi = scramble1(acc_hi + c_hi, sk1);
        cur = nxt;
    }
    {
        uint64_t c_lo, c_hi;
        hash_piece<true>(cur, slot, q, (npieces - 1) << 10, bs, kk0, kk1, last_k, last_slot, k0l, k1l, asum, vsum,
                         bpos, c_lo, c_hi);
        acc_lo += c_lo;
        acc_hi += c_hi;
    }
    uint64_t f = fold64(acc_lo ^ c_tab.merge[2 * q], acc_hi ^ c_tab.merge[2 * q + 1]);
    f = sum_quad64(f);
    // row sums of the Adler partials (16 lanes)
    asum += dpp32<kDppQuadXor1>(asum);
    asum += dpp32<kDppQuadXor2>(asum);
    asum += dpp32<kDppRowRor4>(asum);
    asum += dpp32<kDppRowRor8>(asum);
    vsum += dpp32<kDppQuadXor1>(vsum);
    vsum += dpp32<kDppQuadXor2>(vsum);
    vsum += dpp32<kDppRowRor4>(vsum);
    vsum += dpp32<kDppRowRor8>(vsum);
    bpos = sum_quad64(bpos);
    bpos = dpp_add64<kDppRowRor4>(bpos);
    bpos = dpp_add64<kDppRowRor8>(bpos);
    const uint32_t A = (1u + asum) % kMod;
    const uint32_t B = (uint32_t)(((uint64_t)bs + bpos - vsum) % kMod);
    weak_out = (B << 16) | A;
    strong_out = xxh3_aval((uint64_t)bs * P64_1 + f);
}

// Probe hashes of a weak value w = (B << 16) | A, each two 24-bit multiplies (full
// rate; a 32-bit multiply is quarter rate and this runs once per scanned position):
//   q = A*0x9E3779 + B*0x85EBCB  -> the level-1 bit / ribbon shard and coefficients, and
//                                   the five bit positions of the level-2 word (bits 0..24)
//   r = A*0xC2B2AF + B*0x27D4EB  -> the level-2 word (top bits), the ribbon start
// Level 2 is a blocked Bloom filter of 32-bit words, 5 bits per key in the key's word
// (3 until round 3: 1.1 % false passes measured on Adler values of random 4 KiB blocks),
// 16 bits per key for large indexes (the word from r and the bits from q: taking both
// from one linear hash correlates them, 1.8 %).  Sizing (sydelta_index_create): up to 16 Ki
// keys the filter is <= 32 KiB and the LDS-staged scan copies it into LDS; above
// that it stays in HBM/L2.  FileIx::filt_off counts words; fwshift = 32 - log2(words).
struct ProbeHash {
    uint32_t q, r;
};
__device__ __forceinline__ ProbeHash probe_hash(uint32_t A, uint32_t B) {
    const uint32_t q = (uint32_t)__umul24(A, 0x9E3779u) + (uint32_t)__umul24(B, 0x85EBCBu);
    const uint32_t r = (uint32_t)__umul24(A, 0xC2B2AFu) + (uint32_t)__umul24(B, 0x27D4EBu);
    return {q, r};
}
__device__ __forceinline__ ProbeHash probe_hash(uint32_t w) { return probe_hash(w & 0xFFFFu, w >> 16); }
// Five bits per key in its 32-bit word (q's five low 5-bit fields): 0.74 % false passes at
// 16 bits per key against 1.08 % with three (Poisson keys per word), so a third fewer
// exact-table lookups behind the scans' filters (round 4; each lookup of a level-2 false
// pass misses L2 for a table line).
__device__ __forceinline__ uint32_t filt_mask(uint32_t q) {
    return (1u << (q & 31)) | (1u << ((q >> 5) & 31)) | (1u << ((q >> 10) & 31)) | (1u << ((q >> 15) & 31)) |
           (1u << ((q >> 20) & 31));
}
__device__ __forceinline__ bool filt_pass(uint32_t word, uint32_t q) {
    const uint32_t m = filt_mask(q);
    return (word & m) == m;
}
// filt_pass as 0/1 with five bit extracts (the offset operand takes bits [4:0])
__device__ __forceinline__ uint32_t filt_bit(uint32_t word, uint32_t q) {
    return __builtin_amdgcn_ubfe(word, q, 1) & __builtin_amdgcn_ubfe(word, q >> 5, 1) &
           __builtin_amdgcn_ubfe(word, q >> 10, 1) & __builtin_amdgcn_ubfe(word, q >> 15, 1) &
           __builtin_amdgcn_ubfe(word, q >> 20, 1);
}
// Level-1 filters (held in LDS by k_scan_r / k_scan_g so that only the positions they
// pass cost a level-2 request to L2): one bit per key, bit = q[0..4] (one bit extract;
// the level-2 word tests q[0..4] too, but in an unrelated word).
__device__ __forceinline__ uint32_t l1_test(uint32_t word, uint32_t q) { return __builtin_amdgcn_ubfe(word, q, 1); }
// k_scan_r's level-1 word (kL1WordsR words, not a power of two): floor(q * words / 2^32)
// from the top 24 bits of q, one shift and one v_mul_hi_u32_u24
static_assert((kL1WordsR << 8) < (1u << 24), "l1r_word's constant is a 24-bit operand");
__host__ __device__ __forceinline__ uint32_t l1r_word(uint32_t q) {
    return (uint32_t)(((uint64_t)(q >> 8) * (kL1WordsR << 8)) >> 32);
}
__device__ __forceinline__ uint32_t bucket_hash(uint32_t w) {
    uint32_t h = w ^ (w >> 15);
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h;
}

// Exact lookup: slot of weak value w, or -1.
__device__ __forceinline__ int64_t table_find(const uint32_t* __restrict__ keys, uint32_t bmask, uint32_t w) {
    uint32_t b = bucket_hash(w) & bmask;
    for (;;) {
        const uint4 k = *(const uint4*)(keys + 4 * b);
        if (k.x == w) return 4 * b;
        if (k.y == w) return 4 * b + 1;
        if (k.z == w) return 4 * b + 2;
        if (k.w == w) return 4 * b + 3;
        if (k.w == kEmptyKey) return -1;  // buckets fill in order: a free last slot ends the chain
        b = (b + 1) & bmask;
    }
}

constexpr uint32_t kNoBlock = 0xFFFFFFFFu;  // no hit

// Exclusive wave scan (lane l gets the sum over lanes < l) and the wave total: DPP
// row_shr steps inside each 16-lane row, then the row totals through SGPRs (no LDS
// crossbar round trips: the window phase runs three of these per value).
template <int K>
__device__ __forceinline__ uint32_t dpp_shr(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + K, 0xF, 0xF, true);  // out of row: 0
}
__device__ __forceinline__ uint32_t wave_scan_excl(uint32_t v, uint32_t& total) {
    uint32_t x = v;
    x += dpp_shr<1>(x);
    x += dpp_shr<2>(x);
    x += dpp_shr<4>(x);
    x += dpp_shr<8>(x);
    const uint32_t r0 = __builtin_amdgcn_readlane(x, 15), r1 = __builtin_amdgcn_readlane(x, 31);
    const uint32_t r2 = __builtin_amdgcn_readlane(x, 47), r3 = __builtin_amdgcn_readlane(x, 63);
    const uint32_t row = (threadIdx.x & 63) >> 4;
    const uint32_t off = row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r0 + r1 : r0 + r1 + r2;
    total = r0 + r1 + r2 + r3;
    return x + off - v;
}

