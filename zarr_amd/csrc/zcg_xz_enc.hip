// zcg_xz_enc.hip — Xz encoder (write_chunk for CompressionType::Xz).
//
// Reference: xz.rs:34-43 wraps the writer in xz2's XzEncoder at `preset`
// (lzma_easy_encoder(preset, CRC64)): one .xz stream with one block, a single
// LZMA2 filter whose dictionary size is the preset's, CRC64 check, index and
// footer.  The compressed bytes are not pinned by the reference beyond the
// doc-spec vector; the contract is that liblzma (the reference's
// decoder) reproduces the serialised chunk, with xz2's container conventions
// (stream flags 00 04, block header 02 00 21 01 <dict prop> 00 00 00 + CRC32,
// LZMA2 lc=3 lp=0 pb=2 as in every liblzma preset).
//
// One wave per chunk, wave-uniform like the decoder (zcg_xz_core.h):
//   * greedy parse: at each position the rep0 candidate and a 4-byte-hash
//     candidate (4 096-entry LDS table) are measured 64 bytes per step with a
//     wave ballot; a rep0 match of >= 2 that is not shorter than the hash
//     match by more than one byte wins (LZMA codes rep0 matches cheaply);
//   * the LZMA range encoder (the decoder's model, LDS probabilities) emits
//     bytes into a lane-distributed 64-byte staging group, stored coalesced;
//   * LZMA2 chunks end before 64 KiB of compressed data (chunk header
//     patched in place), the first with dictionary + state reset and props;
//   * CRC64 of the serialised chunk by 64 lane segments (zcg_crc.h).
// '>'-types and bool are serialised on the fly (write_data, chunk.rs:118-140).
#include "zcg_common.h"
#include "zcg_crc.h"

namespace zcg {

constexpr u32 XE_HBITS = 12;
constexpr u32 XE_PROBS = 1846 + (0x300u << 3);  // lc + lp = 3
constexpr u32 XE_CMAX = 65536 - 64;             // compressed bytes per LZMA2 chunk (+ margin)
constexpr u32 XE_UMAX = (1u << 21) - 273;       // uncompressed bytes per LZMA2 chunk
constexpr u32 XE_LC = 3, XE_PB = 2;

// model layout (same as the decoder's)
enum : u32 {
    E_IS_MATCH = 0, E_IS_REP = 192, E_IS_REP_G0 = 204, E_IS_REP0_LONG = 240, E_POS_SLOT = 432,
    E_SPEC_POS = 688, E_ALIGN = 802, E_LEN = 818, E_REP_LEN = 1332, E_LITERAL = 1846
};
enum : u32 { EL_CHOICE = 0, EL_CHOICE2 = 1, EL_LOW = 2, EL_MID = 130, EL_HIGH = 258 };

// log2 of the dictionary of lzma_easy presets 0..9: 256K, 1M, 2M, 4M, 4M, 8M,
// 8M, 16M, 32M, 64M (the LZMA2 property is 2*(lg-12))
__device__ __forceinline__ u32 xe_dict_lg(int preset) {
    const int p = (preset < 0 || preset > 9) ? 6 : preset;
    return p == 0 ? 18u : (p == 1 ? 20u : (p == 2 ? 21u : (p <= 4 ? 22u : (p <= 6 ? 23u : (u32)(p + 17)))));
}

struct XeEnc {
    // serialised input
    const gu8* src;
    u64 n;
    DType t;
    // output
    gu8* dst;
    u64 cap, pos;
    u32 lbuf;
    bool over;
    // range coder
    u64 low;
    u32 range, cache;
    u64 cache_size;
    lu16* probs;
    int lane;

    __device__ __forceinline__ u32 sb(u64 p) const {  // serialised byte p
        return (u32)norm_byte(src[swap_pos(p, t)], t);
    }
    __device__ __forceinline__ void out(u32 b) {
        if (pos < cap) {
            if ((u32)lane == (pos & 63)) lbuf = b;
            if ((pos & 63) == 63) dst[(pos & ~63ull) + lane] = (u8)lbuf;
        } else {
            over = true;
        }
        pos++;
    }
    __device__ __forceinline__ void out_flush() {
        const u64 g = pos & ~63ull;
        const u64 e = pos < cap ? pos : cap;
        if (g + lane < e) dst[g + lane] = (u8)lbuf;
    }
    // byte `at` < pos, possibly still in the staging group
    __device__ __forceinline__ void patch(u64 at, u32 b) {
        if (at >= cap) return;
        if ((at >> 6) == (pos >> 6)) {
            if ((u32)lane == (at & 63)) lbuf = b;
        } else if (lane == 0) {
            dst[at] = (u8)b;
        }
    }
    __device__ __forceinline__ void rc_reset() {
        low = 0; range = 0xFFFFFFFFu; cache = 0; cache_size = 1;
    }
    __device__ __forceinline__ void shift_low() {
        if ((u32)low < 0xFF000000u || (u32)(low >> 32) != 0) {
            const u32 carry = (u32)(low >> 32);
            u32 temp = cache;
            do {
                out((temp + carry) & 0xFF);
                temp = 0xFF;
            } while (--cache_size != 0);
            cache = (u32)(low >> 24) & 0xFF;
        }
        cache_size++;
        low = (low & 0x00FFFFFFull) << 8;
    }
    __device__ __forceinline__ void bit(u32 pi, u32 b) {
        const u32 p = probs[pi];
        const u32 bound = (range >> 11) * p;
        if (b == 0) {
            range = bound;
            probs[pi] = (u16)(p + ((2048 - p) >> 5));
        } else {
            low += bound;
            range -= bound;
            probs[pi] = (u16)(p - (p >> 5));
        }
        while (range < (1u << 24)) {
            range <<= 8;
            shift_low();
        }
    }
    __device__ __forceinline__ void tree(u32 base, u32 nbits, u32 v) {
        u32 m = 1;
        for (int i = (int)nbits - 1; i >= 0; i--) {
            const u32 b = (v >> i) & 1;
            bit(base + m, b);
            m = (m << 1) | b;
        }
    }
    __device__ __forceinline__ void rtree(u32 base, u32 nbits, u32 v) {
        u32 m = 1;
        for (u32 i = 0; i < nbits; i++) {
            const u32 b = (v >> i) & 1;
            bit(base + m, b);
            m = (m << 1) | b;
        }
    }
    __device__ __forceinline__ void direct(u32 v, u32 nbits) {
        for (int i = (int)nbits - 1; i >= 0; i--) {
            range >>= 1;
            if ((v >> i) & 1) low += range;
            while (range < (1u << 24)) {
                range <<= 8;
                shift_low();
            }
        }
    }
    __device__ __forceinline__ void length(u32 lbase, u32 l, u32 ps) {  // l = len - 2
        if (l < 8) {
            bit(lbase + EL_CHOICE, 0);
            tree(lbase + EL_LOW + (ps << 3), 3, l);
        } else if (l < 16) {
            bit(lbase + EL_CHOICE, 1);
            bit(lbase + EL_CHOICE2, 0);
            tree(lbase + EL_MID + (ps << 3), 3, l - 8);
        } else {
            bit(lbase + EL_CHOICE, 1);
            bit(lbase + EL_CHOICE2, 1);
            tree(lbase + EL_HIGH, 8, l - 16);
        }
    }
    __device__ __forceinline__ void distance(u32 dist, u32 len) {
        const u32 lps = len - 2 < 3 ? len - 2 : 3;
        u32 slot;
        if (dist < 4) {
            slot = dist;
        } else {
            const u32 lg = 31 - __builtin_clz(dist);
            slot = 2 * lg + ((dist >> (lg - 1)) & 1);
        }
        tree(E_POS_SLOT + (lps << 6), 6, slot);
        if (slot >= 4) {
            const u32 nd = (slot >> 1) - 1;
            const u32 base = (2 | (slot & 1)) << nd;
            const u32 red = dist - base;
            if (slot < 14) {
                rtree(E_SPEC_POS + base - slot - 1, nd, red);
            } else {
                direct(red >> 4, nd - 4);
                rtree(E_ALIGN, 4, red & 15);
            }
        }
    }
};

// length of the common run of serialised bytes at a and b (< a), capped at `mx`
__device__ __forceinline__ u32 xe_match_len(const XeEnc& e, u64 a, u64 b, u32 mx) {
    const int lane = lane_id();
    u32 len = 0;
    while (len < mx) {
        const u32 k = len + lane;
        const bool ok = k < mx && e.sb(a + k) == e.sb(b + k);
        const u64 miss = __ballot(!ok);
        if (miss) return len + (u32)__builtin_ctzll(miss) < mx ? len + (u32)__builtin_ctzll(miss) : mx;
        len += 64;
    }
    return mx;
}

__global__ __launch_bounds__(64) void xz_encode_kernel(const zcg_chunk* __restrict__ chunks, u32 nch,
                                                       u64 D, DType t, int preset,
                                                       u64* __restrict__ out_len,
                                                       i32* __restrict__ status) {
    __shared__ u16 probs[XE_PROBS];
    __shared__ u32 htab[1u << XE_HBITS];
    const u32 c = blockIdx.x;
    if (c >= nch) return;
    const int lane = lane_id();
    const zcg_chunk ch = chunks[c];
    XeEnc e;
    e.src = (const gu8*)ch.src;
    e.n = D;
    e.t = t;
    e.dst = (gu8*)ch.dst;
    e.cap = ch.dst_cap;
    e.pos = 0;
    e.lbuf = 0;
    e.over = false;
    e.probs = (lu16*)probs;
    e.lane = lane;
    const u32 dlg = xe_dict_lg(preset);
    const u32 dprop = 2u * (dlg - 12u);
    const u64 dsize = 1ull << dlg;

    // ---- stream header: magic, flags 00 04 (CRC64), CRC32(flags) ----
    // FD 37 7A 58 5A 00 | 00 04 | E6 D6 B4 46
    for (int k = 0; k < 12; k++)
        e.out((u32)(((k < 8 ? 0xFD377A585A000004ull : 0xE6D6B446ull) >> (8 * ((k < 8 ? 7 : 11) - k))) & 0xFF));
    const u64 blk0 = e.pos;
    u64 unpadded = 0;
    const u64 n = D;
    if (n > 0) {
        // ---- block header: 02 00 21 01 <prop> 00 00 00 + CRC32 ----
        u32 hc = 0xFFFFFFFFu;
        for (int k = 0; k < 8; k++) {
            const u32 b = k == 0 ? 0x02u : (k == 2 ? 0x21u : (k == 3 ? 0x01u : (k == 4 ? dprop : 0u)));
            e.out(b);
            hc = g_crc32_table[(hc ^ b) & 0xFF] ^ (hc >> 8);
        }
        hc = ~hc;
        for (int k = 0; k < 4; k++) e.out((hc >> (8 * k)) & 0xFF);
        const u64 cdata0 = e.pos;

        for (u32 i = lane; i < XE_PROBS; i += 64) probs[i] = 1024;
        for (u32 i = lane; i < (1u << XE_HBITS); i += 64) htab[i] = 0;
        u32 state = 0, rep0 = 0;
        bool first = true;
        u64 p = 0;
        while (p < n) {
            // ---- one LZMA2 chunk ----
            const u64 hdr = e.pos;
            const u32 hlen = first ? 6 : 5;
            for (u32 k = 0; k < hlen; k++) e.out(0);
            const u64 data0 = e.pos;
            const u64 u0 = p;
            e.rc_reset();
            while (p < n && (p - u0) < XE_UMAX && (e.pos - data0) + e.cache_size + 5 < XE_CMAX) {
                const u32 ps = (u32)p & ((1u << XE_PB) - 1);
                const u32 mx = (n - p) < 273 ? (u32)(n - p) : 273u;
                u32 rl = 0, hl = 0, hd = 0;
                if (p > rep0 && mx >= 2) rl = xe_match_len(e, p, p - rep0 - 1, mx);
                if (mx >= 4) {
                    const u32 x = e.sb(p) | (e.sb(p + 1) << 8) | (e.sb(p + 2) << 16) | (e.sb(p + 3) << 24);
                    const u32 h = (x * 2654435761u) >> (32 - XE_HBITS);
                    const u32 cand = htab[h];
                    htab[h] = (u32)p + 1;
                    if (cand && (u64)p - cand < dsize) {  // within the declared dictionary
                        hd = (u32)p - cand;  // 0-based distance: p - (cand - 1) - 1
                        hl = xe_match_len(e, p, cand - 1, mx);
                        if (hl < 4) hl = 0;
                    }
                }
                if (rl >= 2 && rl + 1 >= hl) {
                    // rep0 match: is_match 1, is_rep 1, is_rep_g0 0, is_rep0_long 1
                    e.bit(E_IS_MATCH + (state << 4) + ps, 1);
                    e.bit(E_IS_REP + state, 1);
                    e.bit(E_IS_REP_G0 + state, 0);
                    e.bit(E_IS_REP0_LONG + (state << 4) + ps, 1);
                    e.length(E_REP_LEN, rl - 2, ps);
                    state = state < 7 ? 8 : 11;
                    p += rl;
                } else if (hl >= 4) {
                    e.bit(E_IS_MATCH + (state << 4) + ps, 1);
                    e.bit(E_IS_REP + state, 0);
                    e.length(E_LEN, hl - 2, ps);
                    e.distance(hd, hl);
                    rep0 = hd;
                    state = state < 7 ? 7 : 10;
                    p += hl;
                } else {
                    const u32 sym = e.sb(p);
                    const u32 prev = p ? e.sb(p - 1) : 0u;
                    const u32 base = E_LITERAL + 0x300u * (prev >> (8 - XE_LC));
                    e.bit(E_IS_MATCH + (state << 4) + ps, 0);
                    if (state < 7) {
                        e.tree(base, 8, sym);
                    } else {
                        u32 mb = e.sb(p - rep0 - 1), off = 0x100, m = 1;
                        for (int i = 7; i >= 0; i--) {
                            const u32 b = (sym >> i) & 1;
                            mb <<= 1;
                            const u32 mbit = mb & off;
                            e.bit(base + off + mbit + m, b);
                            m = (m << 1) | b;
                            off &= b ? mbit : ~mbit;
                        }
                    }
                    state = state < 4 ? 0 : (state < 10 ? state - 3 : state - 6);
                    p += 1;
                }
            }
            for (int k = 0; k < 5; k++) e.shift_low();  // range coder flush
            const u32 usz = (u32)(p - u0) - 1;
            const u32 csz = (u32)(e.pos - data0) - 1;
            e.patch(hdr, (first ? 0xE0u : 0x80u) | (usz >> 16));
            e.patch(hdr + 1, (usz >> 8) & 0xFF);
            e.patch(hdr + 2, usz & 0xFF);
            e.patch(hdr + 3, (csz >> 8) & 0xFF);
            e.patch(hdr + 4, csz & 0xFF);
            if (first) e.patch(hdr + 5, (XE_PB * 5 + 0) * 9 + XE_LC);
            first = false;
        }
        e.out(0x00);  // end of LZMA2 data
        const u64 csize = e.pos - cdata0;
        while ((e.pos - cdata0) & 3) e.out(0x00);  // block padding
        // CRC64 of the serialised chunk
        e.out_flush();
        const u64 crc = wave_crc_fn<u64, CRC64_POLY>([&e](u64 q) -> u32 { return e.sb(q); }, 0, n);
        for (int k = 0; k < 8; k++) e.out((u32)(crc >> (8 * k)) & 0xFF);
        unpadded = 12 + csize + 8;
    }
    // ---- index: 00, count, (unpadded, uncompressed), padding, CRC32 ----
    const u64 idx0 = e.pos;
    u32 ic = 0xFFFFFFFFu;
    auto iout = [&](u32 b) {
        e.out(b);
        ic = g_crc32_table[(ic ^ b) & 0xFF] ^ (ic >> 8);
    };
    auto ivli = [&](u64 v) {
        while (v >= 0x80) {
            iout((u32)(v & 0x7F) | 0x80);
            v >>= 7;
        }
        iout((u32)v);
    };
    iout(0x00);
    ivli(n > 0 ? 1 : 0);
    if (n > 0) {
        ivli(unpadded);
        ivli(n);
    }
    while ((e.pos - idx0) & 3) iout(0x00);
    ic = ~ic;
    for (int k = 0; k < 4; k++) e.out((ic >> (8 * k)) & 0xFF);
    const u64 isize = e.pos - idx0;
    // ---- stream footer: CRC32(backward size, flags), backward size, 00 04, 'YZ' ----
    const u32 bsz = (u32)(isize / 4 - 1);
    const u64 fbw = (u64)bsz | (0x0400ull << 32);  // backward size LE32, flags 00 04
    u32 fc = 0xFFFFFFFFu;
    for (int k = 0; k < 6; k++) fc = g_crc32_table[(fc ^ (u32)(fbw >> (8 * k))) & 0xFF] ^ (fc >> 8);
    fc = ~fc;
    for (int k = 0; k < 4; k++) e.out((fc >> (8 * k)) & 0xFF);
    for (int k = 0; k < 6; k++) e.out((u32)(fbw >> (8 * k)) & 0xFF);
    e.out(0x59);
    e.out(0x5A);
    e.out_flush();
    (void)blk0;
    if (lane == 0) {
        out_len[c] = e.pos;
        status[c] = e.over ? ZCG_ERR_OUTPUT_TOO_SMALL : ZCG_OK;
    }
}

hipError_t launch_xz_encode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                            uint64_t* d_out_len, int32_t* d_status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    hipLaunchKernelGGL(xz_encode_kernel, dim3(n), dim3(64), 0, s, d_chunks, n, D, t,
                       a->compression.xz_preset, d_out_len, d_status);
    return hipGetLastError();
}

}  // namespace zcg
