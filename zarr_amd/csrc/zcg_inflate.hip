// zcg_inflate.hip — GzipCompression decode (src/compression/gzip.rs:49-52,
// flate2 read::GzDecoder over zlib raw inflate) on gfx950.
//
// Version 1 structure: one wave (64 lanes) per chunk.
//   * the gzip member header is parsed as flate2 does (magic, CM=8, FEXTRA,
//     FNAME, FCOMMENT, FHCRC verified), then RFC 1951 blocks are decoded;
//   * Huffman tables live in LDS: a 2^10-entry literal/length table and a
//     2^8-entry distance table, each entry one u32 (length, kind, extra bits,
//     value); codes longer than the table width take a canonical bit-serial
//     slow path (rare by construction: probability < 2^-10);
//   * the whole 32 KiB LZ77 window is an LDS ring, so every match source is
//     read from LDS; match bytes are copied by up to 64 lanes per round
//     (rounds of min(dist,64) bytes keep overlapping matches exact);
//   * decoded bytes leave the ring in 16 KiB element-aligned slabs with
//     16 B/lane coalesced stores, the '>'-type byte reversal / bool rule
//     fused into the store;
//   * decoding stops as soon as N*size bytes exist (read_exact, chunk.rs:
//     112-113): the CRC32/ISIZE trailer is not consulted on a full read,
//     exactly like flate2 (parity contract).
// The Huffman symbol decode is a wave-uniform serial chain; its throughput is
// bounded by scalar issue, not HBM.  DESIGN.md quantifies the bound.
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
    const int lane = lane_id();
    __shared__ u16 s_offs[16];
    if (lane < 16) h->count[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (lane == 0) {
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
    if (lane == 0) {
        u32 o = 0;
        s_offs[0] = 0;
        for (int l = 1; l < 16; l++) { s_offs[l] = o; o += h->count[l]; }
        for (u32 s = 0; s < nsym; s++)
            if (lens[s]) h->sym[s_offs[lens[s]]++] = (u16)s;
    }
    __syncthreads();
    // primary table: slot bits are stream-order (LSB first)
    const u32 nslots = 1u << tbits;
    for (u32 slot = lane; slot < nslots; slot += 64) {
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

struct BitIn {
    const u8* src;
    u64 n;        // input bytes
    u64 pos;      // next byte to load into the buffer
    u64 buf;      // bit buffer (LSB = next bit)
    u32 cnt;      // valid bits in buf
    u64 consumed; // bits consumed from the stream start
    u64 limit;    // bits that may be consumed (input end, or look-ahead window end)
};

__device__ __forceinline__ void bi_refill(BitIn& b) {
    if (b.cnt <= 32) {
        u32 w;
        if (b.pos + 4 <= b.n) {
            w = ld32(b.src + b.pos);
        } else {
            w = 0;
            for (u32 i = 0; i < 4; i++)
                if (b.pos + i < b.n) w |= (u32)b.src[b.pos + i] << (8 * i);
        }
        w = __builtin_amdgcn_readfirstlane(w);
        b.buf |= (u64)w << b.cnt;
        b.cnt += 32;
        b.pos += 4;
    }
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
    const int lane = lane_id();
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
    for (u32 i = lane; i < 19; i += 64) lens[i] = cl[i];
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
            if (lane == 0) lens[idx] = (u8)sym;
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
        if (lane == 0)
            for (u32 k = 0; k < rep; k++) lens[idx + k] = v;
        idx += rep;
        prev = v;
    }
    __syncthreads();
    u8 dl = 0;
    if ((u32)lane < ndist) dl = lens[nlen + lane];
    __syncthreads();
    for (u32 i = nlen + lane; i < 288; i += 64) lens[i] = 0;
    if ((u32)lane < 32) lens[288 + lane] = (u32)lane < ndist ? dl : 0;
    __syncthreads();
    if (lens[256] == 0) return R_INVALID;  // "invalid code -- missing end-of-block"
    if (build_table(lens, 288, lh, ltab, INF_LBITS, false) != 0) return R_INVALID;
    if (build_table(lens + 288, 30, dh, dtab, INF_DBITS, true) != 0) return R_INVALID;
    return R_OK;
}

__device__ void fixed_tables(u8* lens, HuffLds* lh, u32* ltab, HuffLds* dh, u32* dtab) {
    const int lane = lane_id();
    __syncthreads();
    for (u32 i = lane; i < 320; i += 64)
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

__global__ __launch_bounds__(64) void inflate_kernel(const zcg_chunk* __restrict__ chunks, u32 n,
                                                     u64 D, DType t, u32 vflags,
                                                     i32* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) u8 ring[INF_RING];
    __shared__ u32 ltab[1u << INF_LBITS];
    __shared__ u32 dtab[1u << INF_DBITS];
    __shared__ HuffLds lh, dh;
    __shared__ u8 lens[320];

    const u32 c = blockIdx.x;
    if (c >= n) return;
    const int lane = lane_id();
    const zcg_chunk ch = chunks[c];
    int st = ZCG_OK;
    if (D == 0) { if (lane == 0) status[c] = ZCG_OK; return; }
    if (ch.dst_cap < D) { if (lane == 0) status[c] = ZCG_ERR_INVALID_INPUT; return; }

    const u8* s = (const u8*)ch.src;
    const u64 n_in = ch.src_len;
    // ---- gzip member header (flate2 read_gz_header) ---------------------
    u64 h = 10;
    if (n_in < 10) st = ZCG_ERR_UNEXPECTED_EOF;
    else if (s[0] != 0x1f || s[1] != 0x8b || s[2] != 8) st = ZCG_ERR_INVALID_DATA;
    if (st == ZCG_OK) {
        const u32 flg = s[3];
        if (flg & 4) {
            if (h + 2 > n_in) st = ZCG_ERR_UNEXPECTED_EOF;
            else h += 2 + ((u64)s[h] | ((u64)s[h + 1] << 8));
            if (st == ZCG_OK && h > n_in) st = ZCG_ERR_UNEXPECTED_EOF;
        }
        if (st == ZCG_OK && (flg & 8)) {
            while (h < n_in && s[h]) h++;
            if (h >= n_in) st = ZCG_ERR_UNEXPECTED_EOF; else h++;
        }
        if (st == ZCG_OK && (flg & 16)) {
            while (h < n_in && s[h]) h++;
            if (h >= n_in) st = ZCG_ERR_UNEXPECTED_EOF; else h++;
        }
        if (st == ZCG_OK && (flg & 2)) {
            if (h + 2 > n_in) st = ZCG_ERR_UNEXPECTED_EOF;
            else {
                u32 crc = 0xFFFFFFFFu;
                for (u64 i = 0; i < h; i++) crc = g_crc32_table[(crc ^ s[i]) & 255] ^ (crc >> 8);
                crc ^= 0xFFFFFFFFu;
                if ((crc & 0xFFFF) != ((u32)s[h] | ((u32)s[h + 1] << 8))) st = ZCG_ERR_INVALID_DATA;
                h += 2;
            }
        }
    }
    if (st != ZCG_OK) { if (lane == 0) status[c] = st; return; }

    BitIn b{s + h, n_in - h, 0, 0, 0, 0, (n_in - h) * 8};
    InfOut o{ring, 0, 0, (u8*)ch.dst, D, t};
    bool last = false;
    bool boundary = false;  // output filled exactly at a symbol boundary
    bool after_stored = false;
    int r = R_OK;
    while (r == R_OK && o.P < D) {
        if (last) { r = R_EXHAUSTED; break; }  // stream ended before N bytes
        u32 type = 0, slen = 0;
        r = read_block_header(b, &last, &type, &slen, lens, &lh, ltab, &dh, dtab);
        if (r != R_OK) break;
        if (type == 0) {  // stored: drain whole bytes of the bit buffer, then copy
            u32 done = 0;
            while (done < slen && b.cnt >= 8 && o.P < D) {
                if (!bi_has(b, 8)) { r = R_EXHAUSTED; break; }
                put_lit(o, bi_bits(b, 8));
                done++;
                inf_maybe_flush(o);
            }
            if (r != R_OK) break;
            if (done < slen && o.P < D) {
                u64 in0 = b.pos;  // bit buffer is empty here
                while (done < slen && o.P < D) {
                    u32 k = slen - done;
                    const u64 room = INF_FLUSH - (o.P - o.F);
                    if (k > room) k = (u32)room;
                    if (k > 64 * 64) k = 64 * 64;
                    if ((u64)k > D - o.P) k = (u32)(D - o.P);
                    if (in0 + k > b.n) { r = R_EXHAUSTED; break; }
                    for (u32 i = lane; i < k; i += 64)
                        ring[(o.P + i) & (INF_RING - 1)] = b.src[in0 + i];
                    __builtin_amdgcn_wave_barrier();
                    o.P += k; in0 += k; done += k;
                    inf_maybe_flush(o);
                }
                b.pos = in0; b.buf = 0; b.cnt = 0; b.consumed = in0 * 8;
            }
            boundary = (done == slen);
            after_stored = true;
            continue;
        }
        // ---- Huffman block body ---------------------------------------------
        after_stored = false;
        for (;;) {
            if (o.P >= D) { boundary = true; break; }
            u32 e;
            r = decode_sym(b, ltab, INF_LBITS, &lh, false, &e);
            if (r != R_OK) break;
            const u32 kind = (e >> 24) & 15;
            if (kind == K_LIT) {
                put_lit(o, e & 0xFF);
            } else if (kind == K_LEN) {
                const u32 ex = (e >> 16) & 0xFF;
                if (!bi_has(b, ex)) { r = R_EXHAUSTED; break; }
                u32 len = (e & 0xFFFF) + (ex ? bi_bits(b, ex) : 0);
                u32 de;
                r = decode_sym(b, dtab, INF_DBITS, &dh, true, &de);
                if (r != R_OK) break;
                if (((de >> 24) & 15) != K_DIST) { r = R_INVALID; break; }
                const u32 dex = (de >> 16) & 0xFF;
                if (!bi_has(b, dex)) { r = R_EXHAUSTED; break; }
                const u32 dist = (de & 0xFFFF) + (dex ? bi_bits(b, dex) : 0);
                if (dist > o.P) { r = R_INVALID; break; }  // "invalid distance too far back"
                if (o.P + len > D) {  // MATCH leaves with left == 0: no look-ahead
                    put_match(o, (u32)(D - o.P), dist);
                    boundary = false;
                    break;
                }
                put_match(o, len, dist);
            } else if (kind == K_EOB) {
                break;
            } else {
                r = R_INVALID;
                break;
            }
            inf_maybe_flush(o);
        }
    }
    if (r == R_OK && o.P >= D && boundary) {
        // look-ahead bounded by the 32 KiB window holding the last consumed bit
        const u64 last_byte = h + (b.consumed ? (b.consumed - 1) / 8 : 0);
        u64 wend = (last_byte / 32768 + 1) * 32768;
        if (wend > n_in) wend = n_in;
        b.limit = (wend - h) * 8;
        if (b.limit >= b.consumed) {
            int la = inf_lookahead(b, last, after_stored, lens, &lh, ltab, &dh, dtab);
            if (la == R_INVALID) r = R_INVALID;
        }
    }
    if (r == R_INVALID) st = ZCG_ERR_INVALID_DATA;
    else if (r == R_EXHAUSTED || o.P < D) st = ZCG_ERR_UNEXPECTED_EOF;
    if (st == ZCG_OK) {
        while (D - o.F > INF_FLUSH) inf_flush(o, o.F + INF_FLUSH);
        inf_flush(o, D);
    }
    if (lane == 0) status[c] = st;
}

hipError_t launch_inflate(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                          int32_t* d_status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    hipLaunchKernelGGL(inflate_kernel, dim3(n), dim3(64), 0, s, d_chunks, n, D, t,
                       a->compression.flags, d_status);
    return hipGetLastError();
}

}  // namespace zcg
