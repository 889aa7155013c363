// zcg_inflate_common.h — RFC 1951 / gzip machinery shared by the serial
// (zcg_inflate.hip) and parallel (zcg_inflate_par.hip) inflate kernels:
// Huffman tables in LDS, the wave-uniform bit reader, block headers, zlib's
// post-N look-ahead, flate2's gzip header rules.
#pragma once
#include "zcg_common.h"

namespace zcg {


constexpr int INF_LBITS = 10;
constexpr int INF_DBITS = 8;
constexpr u32 INF_RING = 32768;
constexpr u32 INF_FLUSH = 16384;

// entry: [31:28] codelen (0 => slow path) | [27:24] kind | [23:16] extra | [15:0] value
enum : u32 { K_LIT = 0, K_LEN = 1, K_EOB = 2, K_BAD = 3, K_DIST = 4 };

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

// Canonical Huffman code description in LDS (puff.c style).
struct HuffLds {
    u16 count[16];
    u16 sym[288];
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

// Build canonical code + primary table from lengths[0..nsym) (wave-cooperative).
// Returns 0 ok, -1 over-subscribed/incomplete (zlib inflate_table rules).
__device__ int build_table(const u8* lens, u32 nsym, HuffLds* h, u32* table, int tbits, bool dist) {
    // block-cooperative: every thread of the workgroup calls this uniformly
    const u32 tid = threadIdx.x, nth = blockDim.x;
    __shared__ u16 s_offs[16];
    __syncthreads();
    if (tid < 16) h->count[tid] = 0;
    __syncthreads();
    if (tid == 0) {
        for (u32 s = 0; s < nsym; s++) h->count[lens[s]]++;
    }
    __syncthreads();
    int ok = 1, maxlen = 0;
    {
        int left = 1;
        for (int l = 1; l <= 15; l++) {
            left <<= 1;
            left -= h->count[l];
            if (left < 0) ok = 0;  // over-subscribed
            if (h->count[l]) maxlen = l;
        }
        // incomplete codes are only allowed for a single length-1 code
        if (ok && left > 0 && maxlen > 1) ok = 0;
    }
    if (tid == 0) {
        u32 o = 0;
        s_offs[0] = 0;
        for (int l = 1; l < 16; l++) { s_offs[l] = o; o += h->count[l]; }
        for (u32 s = 0; s < nsym; s++)
            if (lens[s]) h->sym[s_offs[lens[s]]++] = (u16)s;
    }
    __syncthreads();
    // primary table: slot bits are stream-order (LSB first)
    const u32 nslots = 1u << tbits;
    for (u32 slot = tid; slot < nslots; slot += nth) {
        u32 code = 0, first = 0, index = 0, e = mk_entry(0, K_BAD, 0, 0);
        bool found = false;
        for (int l = 1; l <= tbits; l++) {
            code |= (slot >> (l - 1)) & 1;
            const u32 cnt = h->count[l];
            if (code - first < cnt) {  // unsigned compare also covers code < first
                e = sym_entry(h->sym[index + (code - first)], l, dist);
                found = true;
                break;
            }
            index += cnt;
            first += cnt;
            first <<= 1;
            code <<= 1;
        }
        if (!found) e = (maxlen > tbits) ? mk_entry(0, K_LEN, 0, 0) /* slow path */
                                         : mk_entry(0, K_BAD, 0, 0);
        table[slot] = e;
    }
    __syncthreads();
    return ok ? 0 : -1;
}

// Canonical decode of a long code from the bits of v (LSB first).
__device__ __forceinline__ u32 slow_sym(u64 v, const HuffLds* h, bool dist, u32* used) {
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; len++) {
        code |= (int)((v >> (len - 1)) & 1);
        const int cnt = h->count[len];
        if (code - cnt < first) {
            *used = len;
            return sym_entry(h->sym[index + (code - first)], len, dist);
        }
        index += cnt;
        first += cnt;
        first <<= 1;
        code <<= 1;
    }
    *used = 0;
    return mk_entry(0, K_BAD, 0, 0);
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

// Decode one symbol: primary table, else canonical bit-serial decode.
__device__ __forceinline__ int decode_sym(BitIn& b, const u32* tab, int tbits, const HuffLds* h,
                                          bool dist, u32* out) {
    bi_refill(b);
    u32 e = __builtin_amdgcn_readfirstlane(tab[bi_peek(b, tbits)]);
    u32 l = e >> 28;
    if (l != 0) {
        if (!bi_has(b, l)) return R_EXHAUSTED;
        bi_drop(b, l);
        *out = e;
        return R_OK;
    }
    if (((e >> 24) & 15) == K_BAD) {  // unused slot of an incomplete (1-bit) code
        if (!bi_has(b, 1)) return R_EXHAUSTED;
        return R_INVALID;
    }
    int code = 0, first = 0, index = 0;
    for (int len = 1; len <= 15; len++) {
        if (!bi_has(b, 1)) return R_EXHAUSTED;
        bi_refill(b);
        code |= (int)bi_peek(b, 1);
        bi_drop(b, 1);
        const int cnt = h->count[len];
        if (code - cnt < first) {
            *out = sym_entry(h->sym[index + (code - first)], len, dist);
            return R_OK;
        }
        index += cnt;
        first += cnt;
        first <<= 1;
        code <<= 1;
    }
    return R_INVALID;
}

// Dynamic block header (RFC 1951 3.2.7) -> tables; zlib's validity rules.
__device__ int read_dynamic(BitIn& b, u8* lens, HuffLds* lh, u32* ltab, HuffLds* dh, u32* dtab) {
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
    build_table(lens, 19, lh, ltab, 7, false);
    u32 idx = 0;
    u8 prev = 0;
    while (idx < nlen + ndist) {
        u32 e;
        int r = decode_sym(b, ltab, 7, lh, false, &e);
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
        if (tid == 0)
            for (u32 k = 0; k < rep; k++) lens[idx + k] = v;
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
    if (build_table(lens, 288, lh, ltab, INF_LBITS, false) != 0) return R_INVALID;
    if (build_table(lens + 288, 30, dh, dtab, INF_DBITS, true) != 0) return R_INVALID;
    return R_OK;
}

__device__ void fixed_tables(u8* lens, HuffLds* lh, u32* ltab, HuffLds* dh, u32* dtab) {
    const u32 tid = threadIdx.x, nth = blockDim.x;
    __syncthreads();
    for (u32 i = tid; i < 320; i += nth)
        lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
    __syncthreads();
    build_table(lens, 288, lh, ltab, INF_LBITS, false);
    build_table(lens + 288, 30, dh, dtab, INF_DBITS, true);
}

// Block header: 3 bits, then stored-length check / table construction.
// *type receives BTYPE; for stored blocks *slen the LEN field.
__device__ int read_block_header(BitIn& b, bool* last, u32* type, u32* slen, u8* lens, HuffLds* lh,
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
    if (*type == 1) { fixed_tables(lens, lh, ltab, dh, dtab); return R_OK; }
    return read_dynamic(b, lens, lh, ltab, dh, dtab);
}

// zlib keeps decoding after the output is full until it needs to emit a
// byte (LIT / MATCH with left == 0) or needs input it was not given: the
// next literal/length code, length extra bits, distance code, distance
// extra bits, and whole block headers are validated.  The input it was
// given is the rest of flate2's current 32 KiB BufReader window.
__device__ int inf_lookahead(BitIn& b, bool last, bool at_header, u8* lens, HuffLds* lh,
                             u32* ltab, HuffLds* dh, u32* dtab) {
    for (;;) {
        if (at_header) {  // after a stored block: straight to the next header
            at_header = false;
            if (last) return R_OK;
            u32 type = 0, slen = 0;
            int r = read_block_header(b, &last, &type, &slen, lens, lh, ltab, dh, dtab);
            if (r != R_OK) return r;
            if (type == 0) {
                if (slen != 0) return R_OK;
                at_header = true;
                continue;
            }
        }
        u32 e;
        int r = decode_sym(b, ltab, INF_LBITS, lh, false, &e);
        if (r != R_OK) return r;
        const u32 kind = (e >> 24) & 15;
        if (kind == K_LIT) return R_OK;
        if (kind == K_BAD) return R_INVALID;  // "invalid literal/length code"
        if (kind == K_LEN) {
            const u32 ex = (e >> 16) & 0xFF;
            if (!bi_has(b, ex)) return R_EXHAUSTED;
            if (ex) bi_bits(b, ex);
            u32 de;
            r = decode_sym(b, dtab, INF_DBITS, dh, true, &de);
            if (r != R_OK) return r;
            if (((de >> 24) & 15) != K_DIST) return R_INVALID;  // "invalid distance code"
            return R_OK;  // DISTEXT then MATCH: zlib leaves there (left == 0)
        }
        // end of block: the next block header is parsed without output
        for (;;) {
            if (last) return R_OK;  // stream end
            u32 type = 0, slen = 0;
            r = read_block_header(b, &last, &type, &slen, lens, lh, ltab, dh, dtab);
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
