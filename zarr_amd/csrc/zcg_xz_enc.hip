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
// Match finding runs ahead of the coder, data-parallel over every position of
// a sub-batch (<= 128 MiB of input), so the whole chunk is the dictionary as in
// liblzma (whose presets' dictionaries cover a 1 MiB chunk):
//   * xe_keys + a hipCUB radix sort of (chunk, 20-bit hash of 4 bytes) keys
//     with the positions as values (stable: ascending positions per key);
//   * xe_chain: each position's predecessor with the same key = hash chain;
//   * xe_best: one thread per position walks its chain up to XE_DEPTH
//     candidates inside the preset's dictionary and keeps the longest match
//     (nearest on ties), up to XE_NICE bytes (then it stops walking).
// The coder is one wave per chunk, wave-uniform like the decoder (zcg_xz_core.h):
//   * parse: at each position the rep0 candidate (measured 64 bytes per step
//     with a wave ballot) and the precomputed best match; a rep0 match of >= 2
//     that is not shorter than the best match by more than one byte wins
//     (LZMA codes rep0 cheaply); one-step lazy evaluation (a literal when the
//     next position's match is longer by more than one byte);
//   * the LZMA range encoder (the decoder's model, LDS probabilities) emits
//     bytes into a lane-distributed 64-byte staging group, stored coalesced;
//   * LZMA2 chunks end before 64 KiB of compressed data (chunk header
//     patched in place), the first with dictionary + state reset and props;
//   * CRC64 of the serialised chunk by 64 lane segments (zcg_crc.h).
// '>'-types and bool are serialised on the fly (write_data, chunk.rs:118-140).
#include <hipcub/hipcub.hpp>

#include "zcg_crc.h"
#include "zcg_xz_enc.h"

namespace zcg {

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

__global__ __launch_bounds__(64) void xz_encode_kernel(const zcg_chunk* __restrict__ chunks, u32 c0, u32 cnt,
                                                       u64 D, DType t, int preset,
                                                       const u16* __restrict__ g_blen,
                                                       const u32* __restrict__ g_bdist,
                                                       u64* __restrict__ out_len,
                                                       i32* __restrict__ status) {
    __shared__ u16 probs[XE_PROBS];
    if (blockIdx.x >= cnt) return;
    const u32 c = c0 + blockIdx.x;
    const u16* blen = g_blen + (u64)blockIdx.x * D;    // best match length per position (0: none)
    const u32* bdist = g_bdist + (u64)blockIdx.x * D;  // its distance (p - q)
    const int lane = lane_id();
    const zcg_chunk ch = chunks[c];
    if (ch.src_len < D) {  // fewer serialised bytes than the chunk holds (chunk.rs:309-318)
        if (lane == 0) { out_len[c] = 0; status[c] = ZCG_ERR_INVALID_DATA; }
        return;
    }
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

        u32 state = 0, rep0 = 0;
        // liblzma's LZMA2 chunk flags (lzma2_encoder.c): a dictionary reset
        // and the properties go with the first chunk of their kind; an
        // uncompressed chunk leaves a state reset pending for the next LZMA one.
        bool need_dict = true, need_props = true, need_state = true;
        // Per-lane window of 64 consecutive positions: the serialised byte, the
        // byte rep0 + 1 back, and the precomputed best match, so literal runs
        // need no dependent memory access per position.
        u64 wb = 0;
        u32 wrep = 0xFFFFFFFFu, wbyte = 0, wrb = 0, wlen = 0, wdist = 0;
        auto refill = [&](u64 base) {
            wb = base;
            wrep = rep0;
            const u64 q = base + (u64)lane;
            const bool in = q < n;
            wbyte = in ? e.sb(q) : 0u;
            wrb = (in && q > rep0) ? e.sb(q - rep0 - 1) : 0x100u;
            wlen = in ? (u32)blen[q] : 0u;
            wdist = in ? bdist[q] : 0u;
        };
        u64 p = 0;
        while (p < n) {
            // ---- one LZMA2 chunk ----
            const u64 hdr = e.pos;
            const bool over0 = e.over;
            const u32 hlen = need_props ? 6 : 5;
            if (need_state) {  // LZMA state reset: probabilities, state, reps
                __syncthreads();
                for (u32 i = lane; i < XE_PROBS; i += 64) probs[i] = 1024;
                __syncthreads();
                state = 0;
                rep0 = 0;
            }
            for (u32 k = 0; k < hlen; k++) e.out(0);
            const u64 data0 = e.pos;
            const u64 u0 = p;
            e.rc_reset();
            while (p < n && (p - u0) < XE_UMAX && (e.pos - data0) + e.cache_size + 5 < XE_CMAX) {
                const u32 ps = (u32)p & ((1u << XE_PB) - 1);
                const u32 mx = (n - p) < 273 ? (u32)(n - p) : 273u;
                // the 64-position window [wb, wb+64) holds p-1 .. p+1 for the current rep0
                if (p + 1 >= wb + 64 || p < wb + (p ? 1 : 0) || rep0 != wrep) refill(p ? p - 1 : 0);
                const u32 i = (u32)(p - wb);
                const u32 sym = __builtin_amdgcn_readlane(wbyte, i);
                u32 rl = 0, hl = 0, hd = 0;
                if (p > rep0 && mx >= 2 && sym == (u32)__builtin_amdgcn_readlane(wrb, i) &&
                    __builtin_amdgcn_readlane(wbyte, i + 1) == __builtin_amdgcn_readlane(wrb, i + 1))
                    rl = xe_match_len(e, p, p - rep0 - 1, mx);
                if (mx >= 4) {
                    hl = __builtin_amdgcn_readlane(wlen, i);
                    if (hl >= 4) {
                        hd = __builtin_amdgcn_readlane(wdist, i) - 1;  // 0-based distance
                        if (hl > mx) hl = mx;
                        // lazy: the next position's match is longer by more than one byte
                        if (p + 1 < n && hl < XE_NICE && rl + 1 < hl) {
                            const u32 nl = __builtin_amdgcn_readlane(wlen, i + 1);
                            if (nl > hl + 1) { hl = 0; rl = 0; }
                        }
                    } else {
                        hl = 0;
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
                    const u32 prev = p ? (u32)__builtin_amdgcn_readlane(wbyte, i - 1) : 0u;
                    const u32 base = E_LITERAL + 0x300u * (prev >> (8 - XE_LC));
                    e.bit(E_IS_MATCH + (state << 4) + ps, 0);
                    if (state < 7) {
                        e.tree(base, 8, sym);
                    } else {
                        u32 mb = __builtin_amdgcn_readlane(wrb, i), off = 0x100, m = 1;
                        for (int k = 7; k >= 0; k--) {
                            const u32 b = (sym >> k) & 1;
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
            if (e.pos - data0 >= p - u0) {
                // liblzma's rule: an LZMA chunk that is not smaller than its
                // input is replaced by an uncompressed chunk (control 1 with a
                // dictionary reset, else 2; then size-1 big-endian, the bytes).
                // The input stays in the dictionary; the next LZMA chunk
                // starts with a state reset.  (usz <= XE_CMAX < 64 KiB.)
                const u32 usz = (u32)(p - u0) - 1;
                e.rewind(hdr);
                e.over = over0;
                e.out(need_dict ? 0x01u : 0x02u);
                e.out((usz >> 8) & 0xFF);
                e.out(usz & 0xFF);
                e.out_run(u0, p - u0);
                need_dict = false;
                need_state = true;
                continue;
            }
            const u32 usz = (u32)(p - u0) - 1;
            const u32 csz = (u32)(e.pos - data0) - 1;
            const u32 ctl = need_props ? (need_dict ? 0xE0u : 0xC0u) : (need_state ? 0xA0u : 0x80u);
            e.patch(hdr, ctl | (usz >> 16));
            e.patch(hdr + 1, (usz >> 8) & 0xFF);
            e.patch(hdr + 2, usz & 0xFF);
            e.patch(hdr + 3, (csz >> 8) & 0xFF);
            e.patch(hdr + 4, csz & 0xFF);
            if (need_props) e.patch(hdr + 5, (XE_PB * 5 + 0) * 9 + XE_LC);
            need_dict = need_props = need_state = false;
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

namespace {

constexpr u32 XE_KEYBITS = 20;            // hash bits of the match-finder keys
constexpr u64 XE_SUB_BYTES = 128ull << 20;  // input bytes per match-finder sub-batch (sort scratch)
constexpr u64 XE_SUPER_BYTES = 1ull << 30;  // input bytes per coder launch (match arrays kept)

struct XeLayout {
    u32 m;    // chunks per match-finder sub-batch
    u32 sm;   // chunks per coder launch (a multiple of m)
    u64 tot;  // m * D positions
    u64 cub_bytes;
    u64 off_ka, off_kb, off_va, off_vb, off_prev, off_blen, off_bdist, off_cub, total;
};

XeLayout xe_layout(u64 D, u32 n) {
    XeLayout y{};
    u64 m = D ? XE_SUB_BYTES / D : n;
    if (m < 1) m = 1;
    if (m > n) m = n;
    if (m > 4096) m = 4096;
    y.m = (u32)m;
    y.tot = m * D;
    u64 sm = D ? XE_SUPER_BYTES / D : n;
    sm = sm / m * m;
    if (sm < m) sm = m;
    if (sm > n) sm = n;
    y.sm = (u32)sm;
    size_t cb = 0;
    hipcub::DoubleBuffer<u32> k(nullptr, nullptr), v(nullptr, nullptr);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cb, k, v, (int)(y.tot ? y.tot : 1), 0, 32);
    y.cub_bytes = (cb + 511) & ~255ull;
    u64 p = 0;
    auto take = [&](u64 bytes) { const u64 o = p; p = (p + bytes + 255) & ~255ull; return o; };
    y.off_ka = take(4 * y.tot);
    y.off_kb = take(4 * y.tot);
    y.off_va = take(4 * y.tot);
    y.off_vb = take(4 * y.tot);
    y.off_prev = take(4 * y.tot);
    y.off_blen = take(2 * (u64)y.sm * D);
    y.off_bdist = take(4 * (u64)y.sm * D);
    y.off_cub = take(y.cub_bytes);
    y.total = p;
    return y;
}

__global__ void xe_keys(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, u64 tot, DType t, u32 cshift,
                        u32* __restrict__ keys, u32* __restrict__ vals) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tot) return;
    const u32 cl = (u32)(g / D);
    const u64 p = g - (u64)cl * D;
    u32 h = 0;
    if (p + 4 <= D && chunks[c0 + cl].src_len >= D) h = (xe_ser4((const u8*)chunks[c0 + cl].src, p, t) * 2654435761u) >> (32 - XE_KEYBITS);
    keys[g] = (cl << cshift) | h;
    vals[g] = (u32)g;
}

__global__ void xe_chain(u64 tot, const u32* __restrict__ keys, const u32* __restrict__ vals,
                         u32* __restrict__ prev) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= tot) return;
    prev[vals[j]] = (j > 0 && keys[j] == keys[j - 1]) ? vals[j - 1] : 0xFFFFFFFFu;
}

__global__ void xe_best(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, u64 tot, DType t, u64 dsize,
                        const u32* __restrict__ prev, u16* __restrict__ blen, u32* __restrict__ bdist) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tot) return;
    const u32 cl = (u32)(g / D);
    const u64 p = g - (u64)cl * D;
    u32 best = 0, bd = 0;
    if (p + 4 <= D && chunks[c0 + cl].src_len >= D) {  // short src: INVALID_DATA in the coder
        const u8* src = (const u8*)chunks[c0 + cl].src;
        const u64 cbase = (u64)cl * D;
        const u32 mx = (D - p) < 273 ? (u32)(D - p) : 273u;
        const u32 v0 = xe_ser4(src, p, t);
        u32 q = prev[g];
        for (u32 dep = 0; dep < XE_DEPTH && q != 0xFFFFFFFFu; dep++) {
            const u64 qp = q - cbase;
            if (p - qp >= dsize) break;  // beyond the preset's dictionary
            const u32 qn = prev[q];  // the next link, in flight during this candidate's compare
            if (xe_ser4(src, qp, t) == v0) {
                u32 k = 4;
                bool diff = false;
                while (k + 4 <= mx) {
                    const u32 x = xe_ser4(src, p + k, t) ^ xe_ser4(src, qp + k, t);
                    if (x) { k += (u32)__builtin_ctz(x) >> 3; diff = true; break; }
                    k += 4;
                }
                if (!diff)
                    while (k < mx && xe_ser1(src, p + k, t) == xe_ser1(src, qp + k, t)) k++;
                if (k > best) { best = k; bd = (u32)(p - qp); }
                if (best >= XE_NICE) break;
            }
            q = qn;
        }
    }
    blen[g] = (u16)best;
    bdist[g] = bd;
}

}  // namespace

u64 xe_sort_scratch(u64 tot) {
    size_t cb = 0;
    hipcub::DoubleBuffer<u32> k(nullptr, nullptr), v(nullptr, nullptr);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cb, k, v, (int)(tot ? tot : 1), 0, 32);
    return (cb + 511) & ~255ull;
}

hipError_t launch_xe_chains(const zcg_chunk* d_chunks, u32 c0, u64 D, u64 tot, DType t, u32 cbits, u32* ka, u32* kb,
                            u32* va, u32* vb, u32* prev, void* cub, u64 cub_bytes, hipStream_t s) {
    const u32 G = (u32)((tot + 255) / 256);
    hipLaunchKernelGGL(xe_keys, dim3(G), dim3(256), 0, s, d_chunks, c0, D, tot, t, XE_KEYBITS, ka, va);
    hipcub::DoubleBuffer<u32> dk(ka, kb), dv(va, vb);
    size_t cb = cub_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(cub, cb, dk, dv, (int)tot, 0, (int)(XE_KEYBITS + cbits), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(xe_chain, dim3(G), dim3(256), 0, s, tot, dk.Current(), dv.Current(), prev);
    return hipGetLastError();
}

uint64_t xz_encode_ws_bytes(const zcg_array* a, uint32_t n) {
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    if (n == 0) return 0;
    if (xz_uses_opt(a)) return xz_opt_ws_bytes(a, n);
    return xe_layout(D, n).total;
}

hipError_t launch_xz_encode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                            uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (xz_uses_opt(a)) return launch_xz_opt(a, d_chunks, n, d_out_len, d_status, ws, ws_bytes, s);
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const XeLayout y = xe_layout(D, n);
    if (ws_bytes < y.total || y.tot >= (1ull << 31)) return hipErrorInvalidValue;
    u8* w = (u8*)ws;
    const int preset = a->compression.xz_preset;
    const int pr = (preset < 0 || preset > 9) ? 6 : preset;
    const u32 dlg = pr == 0 ? 18u : (pr == 1 ? 20u : (pr == 2 ? 21u : (pr <= 4 ? 22u : (pr <= 6 ? 23u : (u32)(pr + 17)))));
    u32 cbits = 0;
    while ((1u << cbits) < y.m) cbits++;
    for (u32 s0 = 0; s0 < n; s0 += y.sm) {
        const u32 scnt = (n - s0) < y.sm ? (n - s0) : y.sm;
        for (u32 c0 = s0; c0 < s0 + scnt; c0 += y.m) {  // match finding, sub-batch by sub-batch
            const u32 cnt = (s0 + scnt - c0) < y.m ? (s0 + scnt - c0) : y.m;
            const u64 tot = (u64)cnt * D;
            if (!tot) continue;
            u32 *ka = (u32*)(w + y.off_ka), *kb = (u32*)(w + y.off_kb);
            u32 *va = (u32*)(w + y.off_va), *vb = (u32*)(w + y.off_vb);
            const u32 G = (u32)((tot + 255) / 256);
            hipError_t e = launch_xe_chains(d_chunks, c0, D, tot, t, cbits, ka, kb, va, vb, (u32*)(w + y.off_prev),
                                            w + y.off_cub, y.cub_bytes, s);
            if (e != hipSuccess) return e;
            const u64 mo = (u64)(c0 - s0) * D;  // this sub-batch's slice of the match arrays
            hipLaunchKernelGGL(xe_best, dim3(G), dim3(256), 0, s, d_chunks, c0, D, tot, t, 1ull << dlg,
                               (const u32*)(w + y.off_prev), (u16*)(w + y.off_blen) + mo,
                               (u32*)(w + y.off_bdist) + mo);
        }
        hipLaunchKernelGGL(xz_encode_kernel, dim3(scnt), dim3(64), 0, s, d_chunks, s0, scnt, D, t, preset,
                           (const u16*)(w + y.off_blen), (const u32*)(w + y.off_bdist), d_out_len, d_status);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace zcg
