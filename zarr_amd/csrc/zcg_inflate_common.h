// zcg_inflate_common.h — RFC 1951 / gzip machinery shared by the serial
// (zcg_inflate.hip) and parallel (zcg_inflate_par.hip) inflate kernels:
// Huffman tables in LDS, the wave-uniform bit reader, block headers, zlib's
// post-N look-ahead, flate2's gzip header rules.
#pragma once
#include "zcg_common.h"

namespace zcg {


constexpr int INF_LBITS = 10;  // literal/length root table bits
constexpr int INF_DBITS = 8;   // distance root table bits
constexpr u32 INF_LTAB = 1536; // root 1024 + subtables (zlib enough(286,10,15) = 1334)
constexpr u32 INF_DTAB = 512;  // root 256 + subtables (enough(30,8,15) = 402)
constexpr u32 INF_RING = 32768;
constexpr u32 INF_FLUSH = 16384;

// Two-level tables: every code decodes in <= 2 LDS lookups (no bit-serial
// path: a rare per-lane slow path would stall whole 64-lane waves).
// entry: [31:28] code length | [27:24] kind | [23:16] extra bits | [15:0] value
//        K_SUB: [23:16] subtable bits, [15:0] subtable offset (code length 0)
enum : u32 { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_BAD = 3, K_DIST = 4, K_SUB = 5 };

__constant__ u16 c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ u8 c_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                   2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ u16 c_dist_base[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                    33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                    1025, 1537, 2049, 3073, 4097, 6145,  8193,  12289, 16385,
                                    24577};
__constant__ u8 c_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                                    6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ u8 c_clen_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ u32 mk_entry(u32 len, u32 kind, u32 extra, u32 val) {
    return (len << 28) | (kind << 24) | (extra << 16) | val;
}

// Canonical Huffman code description in LDS (built per block).
struct HuffLds {
    u32 count[16];
    u32 first[16];     // first canonical code of each length
    u32 cpre[5 * 16];  // per 64-symbol chunk: codes of each length in earlier chunks
};

// Entry for symbol `s` of table type `dist`.
__device__ __forceinline__ u32 sym_entry(u32 s, u32 len, bool dist) {
    if (!dist) {
        if (s < 256) return mk_entry(len, K_LIT, 0, s);
        if (s == 256) return mk_entry(len, K_EOB, 0, 0);
        if (s <= 285) return mk_entry(len, K_LEN, c_len_extra[s - 257], c_len_base[s - 257]);
        return mk_entry(len, K_BAD, 0, 0);
    }
    if (s < 30) return mk_entry(len, K_DIST, c_dist_extra[s], c_dist_base[s]);
    return mk_entry(len, K_BAD, 0, 0);
}

__device__ __forceinline__ u32 bitrev(u32 v, int n) { return __builtin_bitreverse32(v) >> (32 - n); }
// popcount of the mask bits below this lane
__device__ __forceinline__ u32 mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
}

// Build the canonical code and the two-level table from lens[0..nsym)
// (nsym <= 320; block-cooperative: every thread of the workgroup calls this
// uniformly).  Symbol-driven, like zlib's inflate_table: a symbol's rank among
// the codes of its length comes from wave ballots, a short code fills its
// 2^(root-L) root slots, each long-code prefix gets a subtable sized by its
// longest code (atomicMax) and placed by a block scan.  `cap` = table entries.
// Returns 0 ok, -1 over-subscribed or incomplete (zlib inflate_table rules:
// an incomplete code is only allowed when it is a single length-1 code).
__device__ int build_table(const u8* lens, u32 nsym, HuffLds* h, u32* table, int root, bool dist,
                           u32 cap) {
    const u32 tid = threadIdx.x, nth = blockDim.x;
    const u32 lane = tid & 63, wv = tid >> 6, nwv = nth >> 6;
    const u32 nchunk = (nsym + 63) >> 6;
    const u32 nroot = 1u << root;
    __shared__ u32 s_part[256 / 64 + 1];
    __syncthreads();
    // 1. per-chunk counts of each code length; rank of my symbol in its chunk
    constexpr u32 MAXC = 5;
    u32 myL[MAXC], myR[MAXC];
#pragma unroll
    for (u32 i = 0; i < MAXC; i++) {
        const u32 c = wv + i * nwv;
        myL[i] = 0;
        myR[i] = 0;
        if (c < nchunk) {
            const u32 s = c * 64 + lane;
            const u32 L = s < nsym ? lens[s] : 0;
            myL[i] = L;
            for (u32 l = 1; l < 16; l++) {
                const unsigned long long m = __ballot(L == l);
                if (L == l) myR[i] = mbcnt64(m);
                if (lane == 0) h->cpre[c * 16 + l] = (u32)__popcll(m);
            }
        }
    }
    for (u32 k = tid; k < nroot; k += nth) table[k] = 0;
    __syncthreads();
    if (tid < 16) {  // exclusive prefix over chunks, totals
        u32 acc = 0;
        if (tid > 0)
            for (u32 c = 0; c < nchunk; c++) {
                const u32 v = h->cpre[c * 16 + tid];
                h->cpre[c * 16 + tid] = acc;
                acc += v;
            }
        h->count[tid] = acc;
    }
    __syncthreads();
    int ok = 1, maxlen = 0;
    {
        int left = 1;
        for (int l = 1; l <= 15; l++) {
            left <<= 1;
            left -= (int)h->count[l];
            if (left < 0) ok = 0;  // over-subscribed
            if (h->count[l]) maxlen = l;
        }
        if (ok && left > 0 && maxlen > 1) ok = 0;
    }
    if (tid == 0) {
        u32 f = 0;
        for (int l = 1; l < 16; l++) {
            f = (f + h->count[l - 1]) << 1;
            h->first[l] = f;
        }
    }
    __syncthreads();
    if (!ok) return -1;
    u32 rev[MAXC];
#pragma unroll
    for (u32 i = 0; i < MAXC; i++) {
        const u32 c = wv + i * nwv, L = myL[i];
        rev[i] = 0;
        if (L) rev[i] = bitrev(h->first[L] + h->cpre[c * 16 + L] + myR[i], (int)L);
    }
    // 2. subtable size of each long-code prefix
    if (maxlen > root) {
#pragma unroll
        for (u32 i = 0; i < MAXC; i++)
            if (myL[i] > (u32)root) atomicMax(&table[rev[i] & (nroot - 1)], myL[i] - root);
        __syncthreads();
    }
    // 3. root slots: subtable heads (placed by a block scan) or invalid
    const u32 per = (nroot + nth - 1) / nth;  // contiguous slots per thread
    u32 mysum = 0;
    for (u32 k = 0; k < per; k++) {
        const u32 slot = tid * per + k;
        if (slot < nroot && table[slot]) mysum += 1u << table[slot];
    }
    u32 x = mysum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(x, d, 64);
        if ((int)lane >= d) x += y;
    }
    if (lane == 63) s_part[wv] = x;
    __syncthreads();
    u32 off = nroot, tot = 0;
    for (u32 w = 0; w < nwv; w++) {
        const u32 v = s_part[w];
        if (w < wv) off += v;
        tot += v;
    }
    off += x - mysum;
    for (u32 k = 0; k < per; k++) {
        const u32 slot = tid * per + k;
        if (slot >= nroot) break;
        const u32 sb = table[slot];
        table[slot] = sb ? mk_entry(0, K_SUB, sb, off) : mk_entry(1, K_BAD, 0, 0);
        off += sb ? (1u << sb) : 0u;
    }
    __syncthreads();
    if (nroot + tot > cap) return -1;  // cannot happen for a complete code (zlib ENOUGH)
    // 4. fill: short codes into the root, long codes into their subtable
#pragma unroll
    for (u32 i = 0; i < MAXC; i++) {
        const u32 L = myL[i];
        if (!L) continue;
        const u32 s = (wv + i * nwv) * 64 + lane;
        const u32 e = sym_entry(s, L, dist);
        if (L <= (u32)root) {
            for (u32 k = rev[i]; k < nroot; k += 1u << L) table[k] = e;
        } else {
            const u32 te = table[rev[i] & (nroot - 1)];
            const u32 base = te & 0xFFFF, sb = (te >> 16) & 0xFF;
            for (u32 k = rev[i] >> root; k < (1u << sb); k += 1u << (L - root)) table[base + k] = e;
        }
    }
    __syncthreads();
    return 0;
}

// Look up a symbol from >= 15 stream bits `v` (two levels).
__device__ __forceinline__ u32 table_lookup(const u32* tab, int root, u32 v) {
    u32 e = tab[v & ((1u << root) - 1)];
    if (((e >> 24) & 15) == K_SUB) e = tab[(e & 0xFFFF) + ((v >> root) & ((1u << ((e >> 16) & 0xFF)) - 1))];
    return e;
}

// Wave-uniform bit reader (every lane holds the same state).  Input words
// come from a 256-byte LDS cache that the whole wave refills with one
// coalesced load, so a refill costs an LDS read, not a global round trip.
constexpr u32 BI_CACHE_WORDS = 64;
struct BitIn {
    const u8* src;
    u64 n;        // input bytes
    u64 pos;      // next byte to load into the buffer (multiple of 4)
    u64 buf;      // bit buffer (LSB = next bit)
    u32 cnt;      // valid bits in buf
    u64 consumed; // bits consumed from the stream start
    u64 limit;    // bits that may be consumed (input end, or look-ahead window end)
    u32* cache;   // LDS [BI_CACHE_WORDS]
    u64 cbase;    // byte offset of cache[0]
};

__device__ __forceinline__ void bi_init(BitIn& b, const u8* src, u64 n, u32* cache) {
    b.src = src; b.n = n; b.pos = 0; b.buf = 0; b.cnt = 0; b.consumed = 0; b.limit = n * 8;
    b.cache = cache; b.cbase = ~0ull;
}

__device__ __forceinline__ u32 bi_word(BitIn& b, u64 pos) {
    if (pos < b.cbase || pos + 4 > b.cbase + 4 * BI_CACHE_WORDS) {
        const int lane = lane_id();
        const u64 q = pos + 4 * (u64)lane;
        u32 w = 0;
        if (q + 4 <= b.n) w = ld32(b.src + q);
        else
            for (u32 i = 0; i < 4; i++)
                if (q + i < b.n) w |= (u32)b.src[q + i] << (8 * i);
        __builtin_amdgcn_wave_barrier();
        b.cache[lane] = w;
        __builtin_amdgcn_wave_barrier();
        b.cbase = pos;
    }
    return __builtin_amdgcn_readfirstlane(b.cache[(pos - b.cbase) >> 2]);
}

__device__ __forceinline__ void bi_refill(BitIn& b) {
    if (b.cnt <= 32) {
        const u32 w = bi_word(b, b.pos);
        b.buf |= (u64)w << b.cnt;
        b.cnt += 32;
        b.pos += 4;
    }
}

// Position the reader at absolute stream bit `bit`.
__device__ __forceinline__ void bi_seek(BitIn& b, u64 bit) {
    b.pos = (bit >> 5) << 2;
    b.buf = 0;
    b.cnt = 0;
    b.consumed = bit & ~31ull;
    bi_refill(b);
    const u32 drop = (u32)(bit & 31);
    b.buf >>= drop;
    b.cnt -= drop;
    b.consumed += drop;
}

__device__ __forceinline__ bool bi_has(const BitIn& b, u32 k) { return b.consumed + k <= b.limit; }
__device__ __forceinline__ u32 bi_peek(BitIn& b, u32 k) { return (u32)(b.buf & ((1ull << k) - 1)); }
__device__ __forceinline__ void bi_drop(BitIn& b, u32 k) {
    b.buf >>= k;
    b.cnt -= k;
    b.consumed += k;
}
__device__ __forceinline__ u32 bi_bits(BitIn& b, u32 k) {  // k <= 32
    bi_refill(b);
    u32 v = bi_peek(b, k);
    bi_drop(b, k);
    return v;
}

struct InfOut {
    u8* ring;   // LDS ring [INF_RING]
    u64 P;      // logical bytes produced
    u64 F;      // logical bytes flushed to dst
    u8* dst;
    u64 D;
    DType t;
};

// Flush [F, upto) (upto element-aligned or == D) from the ring to dst.
__device__ void inf_flush(InfOut& o, u64 upto) {
    const int lane = lane_id();
    __syncthreads();
    const u64 F = o.F;
    for (u64 p = F + (u64)lane * 16; p < upto; p += 64 * 16) {
        if (p + 16 <= upto) {
            const u32 r = (u32)(p & (INF_RING - 1));  // 16-aligned, never wraps mid-vector
            u32x4 v = *(const u32x4*)(o.ring + r);
            st16(o.dst + p, transform16(v, o.t));
        } else {
            for (u64 q = p; q < upto; q++)
                o.dst[swap_pos(q, o.t)] = norm_byte(o.ring[q & (INF_RING - 1)], o.t);
        }
    }
    o.F = upto;
    __syncthreads();
}

__device__ __forceinline__ void inf_maybe_flush(InfOut& o) {
    if (o.P - o.F >= INF_FLUSH) inf_flush(o, o.F + INF_FLUSH);
}

__device__ __forceinline__ void put_lit(InfOut& o, u32 byte) {
    if (lane_id() == 0) o.ring[o.P & (INF_RING - 1)] = (u8)byte;
    o.P++;
}

__device__ __forceinline__ void put_match(InfOut& o, u32 len, u32 dist) {
    const int lane = lane_id();
    const u32 m = dist < 64 ? dist : 64;
    const u64 P = o.P;
    for (u32 base = 0; base < len; base += m) {
        const u32 k = base + lane;
        if ((u32)lane < m && k < len) {
            const u64 q = P + k;
            o.ring[q & (INF_RING - 1)] = o.ring[(q - dist) & (INF_RING - 1)];
        }
        __builtin_amdgcn_wave_barrier();
    }
    o.P = P + len;
}

// Result of a bit-level step: ok, ran out of bits (EOF in the main decode,
// "zlib waits for input" in the look-ahead), or corrupt.
enum : int { R_OK = 0, R_EXHAUSTED = 1, R_INVALID = 2 };

// Decode one symbol (two-level table) with the wave-uniform reader.
__device__ __forceinline__ int decode_sym(BitIn& b, const u32* tab, int root, u32* out) {
    bi_refill(b);
    const u32 e = __builtin_amdgcn_readfirstlane(table_lookup(tab, root, bi_peek(b, 15)));
    const u32 l = e >> 28;
    if (!bi_has(b, l)) return R_EXHAUSTED;
    if (((e >> 24) & 15) == K_BAD) return R_INVALID;
    bi_drop(b, l);
    *out = e;
    return R_OK;
}

// Table geometry: literal/length root bits + table capacity, distance root
// bits + capacity (defaults: the serial and 256-lane kernels' 10/8-bit roots).
// Dynamic block header (RFC 1951 3.2.7) -> tables; zlib's validity rules.
template <int LB = INF_LBITS, u32 LCAP = INF_LTAB, int DB = INF_DBITS, u32 DCAP = INF_DTAB>
__device__ __attribute__((always_inline)) int read_dynamic(BitIn& b, u8* lens, HuffLds* lh, u32* ltab, HuffLds* dh, u32* dtab) {
    const u32 tid = threadIdx.x, nth = blockDim.x;
    if (!bi_has(b, 14)) return R_EXHAUSTED;
    const u32 nlen = bi_bits(b, 5) + 257, ndist = bi_bits(b, 5) + 1, ncode = bi_bits(b, 4) + 4;
    if (nlen > 286 || ndist > 30) return R_INVALID;  // "too many length or distance symbols"
    u8 cl[19];
    for (int i = 0; i < 19; i++) cl[i] = 0;
    if (!bi_has(b, 3 * ncode)) return R_EXHAUSTED;
    for (u32 i = 0; i < ncode; i++) cl[c_clen_order[i]] = (u8)bi_bits(b, 3);
    {  // code-length code must be complete ("invalid code lengths set")
        u32 cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < 19; i++) cnt[cl[i]]++;
        int left = 1;
        for (int l = 1; l <= 7; l++) { left <<= 1; left -= cnt[l]; if (left < 0) break; }
        if (left != 0) return R_INVALID;
    }
    __syncthreads();
    for (u32 i = tid; i < 19; i += nth) lens[i] = cl[i];
    __syncthreads();
    build_table(lens, 19, lh, ltab, 7, false, LCAP);
    u32 idx = 0;
    u8 prev = 0;
    while (idx < nlen + ndist) {
        u32 e;
        int r = decode_sym(b, ltab, 7, &e);
        if (r != R_OK) return r;
        const u32 sym = e & 0xFFFF;
        if (sym < 16) {
            if (tid == 0) lens[idx] = (u8)sym;
            prev = (u8)sym;
            idx++;
            continue;
        }
        u32 rep;
        u8 v = 0;
        if (sym == 16) {
            if (idx == 0) return R_INVALID;  // "invalid bit length repeat"
            if (!bi_has(b, 2)) return R_EXHAUSTED;
            v = prev;
            rep = 3 + bi_bits(b, 2);
        } else if (sym == 17) {
            if (!bi_has(b, 3)) return R_EXHAUSTED;
            rep = 3 + bi_bits(b, 3);
        } else {
            if (!bi_has(b, 7)) return R_EXHAUSTED;
            rep = 11 + bi_bits(b, 7);
        }
        if (idx + rep > nlen + ndist) return R_INVALID;
        if (tid < 64)
            for (u32 k = tid; k < rep; k += 64) lens[idx + k] = v;
        idx += rep;
        prev = v;
    }
    __syncthreads();
    u8 dl = 0;
    if (tid < ndist) dl = lens[nlen + tid];
    __syncthreads();
    for (u32 i = nlen + tid; i < 288; i += nth) lens[i] = 0;
    if (tid < 32) lens[288 + tid] = tid < ndist ? dl : 0;
    __syncthreads();
    if (lens[256] == 0) return R_INVALID;  // "invalid code -- missing end-of-block"
    if (build_table(lens, 288, lh, ltab, LB, false, LCAP) != 0) return R_INVALID;
    if (build_table(lens + 288, 30, dh, dtab, DB, true, DCAP) != 0) return R_INVALID;
    return R_OK;
}

template <int LB = INF_LBITS, u32 LCAP = INF_LTAB, int DB = INF_DBITS, u32 DCAP = INF_DTAB>
__device__ void fixed_tables(u8* lens, HuffLds* lh, u32* ltab, HuffLds* dh, u32* dtab) {
    const u32 tid = threadIdx.x, nth = blockDim.x;
    __syncthreads();
    for (u32 i = tid; i < 320; i += nth)
        lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
    __syncthreads();
    build_table(lens, 288, lh, ltab, LB, false, LCAP);
    // all 32 five-bit distance codes (30 and 31 decode as invalid), as zlib
    // builds the fixed table: the 30-symbol code alone would be incomplete
    build_table(lens + 288, 32, dh, dtab, DB, true, DCAP);
}

// Block header: 3 bits, then stored-length check / table construction.
// *type receives BTYPE; for stored blocks *slen the LEN field.
template <int LB = INF_LBITS, u32 LCAP = INF_LTAB, int DB = INF_DBITS, u32 DCAP = INF_DTAB>
__device__ __attribute__((always_inline)) int read_block_header(BitIn& b, bool* last, u32* type, u32* slen, u8* lens, HuffLds* lh,
                                 u32* ltab, HuffLds* dh, u32* dtab) {
    if (!bi_has(b, 3)) return R_EXHAUSTED;
    const u32 hdr = bi_bits(b, 3);
    *last = hdr & 1;
    *type = hdr >> 1;
    if (*type == 0) {
        const u32 pad = (u32)((8 - (b.consumed & 7)) & 7);  // to byte boundary
        if (!bi_has(b, pad + 32)) return R_EXHAUSTED;
        bi_bits(b, pad);
        const u32 len = bi_bits(b, 16), nlen = bi_bits(b, 16);
        if ((len ^ 0xFFFF) != nlen) return R_INVALID;  // "invalid stored block lengths"
        *slen = len;
        return R_OK;
    }
    if (*type == 3) return R_INVALID;  // "invalid block type"
    if (*type == 1) { fixed_tables<LB, LCAP, DB, DCAP>(lens, lh, ltab, dh, dtab); return R_OK; }
    return read_dynamic<LB, LCAP, DB, DCAP>(b, lens, lh, ltab, dh, dtab);
}

// zlib keeps decoding after the output is full until it needs to emit a
// byte (LIT / MATCH with left == 0) or needs input it was not given: the
// next literal/length code, length extra bits, distance code, distance
// extra bits, and whole block headers are validated.  The input it was
// given is the rest of flate2's current 32 KiB BufReader window.
template <int LB = INF_LBITS, u32 LCAP = INF_LTAB, int DB = INF_DBITS, u32 DCAP = INF_DTAB>
__device__ __attribute__((always_inline)) int inf_lookahead(BitIn& b, bool last, bool at_header, u8* lens, HuffLds* lh,
                             u32* ltab, HuffLds* dh, u32* dtab) {
    for (;;) {
        if (at_header) {  // after a stored block: straight to the next header
            at_header = false;
            if (last) return R_OK;
            u32 type = 0, slen = 0;
            int r = read_block_header<LB, LCAP, DB, DCAP>(b, &last, &type, &slen, lens, lh, ltab, dh, dtab);
            if (r != R_OK) return r;
            if (type == 0) {
                if (slen != 0) return R_OK;
                at_header = true;
                continue;
            }
        }
        u32 e;
        int r = decode_sym(b, ltab, LB, &e);
        if (r != R_OK) return r;
        const u32 kind = (e >> 24) & 15;
        if (kind == K_LIT) return R_OK;
        if (kind == K_BAD) return R_INVALID;  // "invalid literal/length code"
        if (kind == K_LEN) {
            const u32 ex = (e >> 16) & 0xFF;
            if (!bi_has(b, ex)) return R_EXHAUSTED;
            if (ex) bi_bits(b, ex);
            u32 de;
            r = decode_sym(b, dtab, DB, &de);
            if (r != R_OK) return r;
            if (((de >> 24) & 15) != K_DIST) return R_INVALID;  // "invalid distance code"
            return R_OK;  // DISTEXT then MATCH: zlib leaves there (left == 0)
        }
        // end of block: the next block header is parsed without output
        for (;;) {
            if (last) return R_OK;  // stream end
            u32 type = 0, slen = 0;
            r = read_block_header<LB, LCAP, DB, DCAP>(b, &last, &type, &slen, lens, lh, ltab, dh, dtab);
            if (r != R_OK) return r;
            if (type != 0) break;         // decode symbols of the new block
            if (slen != 0) return R_OK;   // COPY with left == 0: leave
        }
    }
}


// flate2 read_gz_header (wave-uniform): returns status, *hlen = header bytes.
__device__ inline int gzip_header(const u8* s, u64 n_in, u64* hlen) {
    u64 h = 10;
    if (n_in < 10) return ZCG_ERR_UNEXPECTED_EOF;
    if (s[0] != 0x1f || s[1] != 0x8b || s[2] != 8) return ZCG_ERR_INVALID_DATA;
    const u32 flg = s[3];
    if (flg & 4) {
        if (h + 2 > n_in) return ZCG_ERR_UNEXPECTED_EOF;
        h += 2 + ((u64)s[h] | ((u64)s[h + 1] << 8));
        if (h > n_in) return ZCG_ERR_UNEXPECTED_EOF;
    }
    if (flg & 8) {
        while (h < n_in && s[h]) h++;
        if (h >= n_in) return ZCG_ERR_UNEXPECTED_EOF;
        h++;
    }
    if (flg & 16) {
        while (h < n_in && s[h]) h++;
        if (h >= n_in) return ZCG_ERR_UNEXPECTED_EOF;
        h++;
    }
    if (flg & 2) {
        if (h + 2 > n_in) return ZCG_ERR_UNEXPECTED_EOF;
        u32 crc = 0xFFFFFFFFu;
        for (u64 i = 0; i < h; i++) crc = g_crc32_table[(crc ^ s[i]) & 255] ^ (crc >> 8);
        crc ^= 0xFFFFFFFFu;
        if ((crc & 0xFFFF) != ((u32)s[h] | ((u32)s[h + 1] << 8))) return ZCG_ERR_INVALID_DATA;
        h += 2;
    }
    *hlen = h;
    return ZCG_OK;
}

}  // namespace zcg
