// zcg_xz_opt.hip — Xz encoder, presets 4-9: optimal parsing (write_chunk for
// CompressionType::Xz; xz.rs:39-42 wraps xz2's XzEncoder at `preset`, whose
// presets 4-9 run liblzma's "normal" mode: a price-driven optimal parse over
// reps 0-3, short reps and every match length of a binary-tree match finder).
//
// Same container as the greedy coder (zcg_xz_enc.hip): one .xz stream, one
// block, one LZMA2 filter with the preset's dictionary, CRC64.  The bytes are
// not pinned by the reference; liblzma decodes them, and
// tests/hostcore/xz_opt_ref.cpp restates these kernels step for step so the
// GPU streams are compared byte for byte.
//
//   1. match candidates (data-parallel over every position of a sub-batch):
//      the keys / radix sort / chain kernels of zcg_xz_enc.hip build the
//      4-byte hash chains; xo_cands (one thread per position) adds the
//      nearest 2-byte repeat within 64 bytes (liblzma's hash2 role: short
//      close matches price well on numeric data) to the strictly-longer
//      chain matches (16 links, < 2^23 back) and keeps the 3 longest,
//      packed len << 23 | dist;
//   2. xo_segment (one wave per 256 KiB segment of a chunk): each segment is
//      an independent LZMA2 run — its first LZMA chunk resets the state and
//      sets the properties (lc=0 lp=0 pb=2: 2.6 K probabilities in LDS), the
//      dictionary is shared — so a 1 MiB chunk is coded by 4 waves at once.
//      The parse plans windows of <= 256 positions: node i's arcs (literal,
//      short rep, rep0-3, candidate matches; lengths 2..8 and the last three
//      of each range) are priced lane-parallel from the probabilities at the
//      window start and relaxed by 64-bit LDS atomic minima of
//      (price, source node, arc), which is the serial restatement's
//      first-best tie rule; the path is then range-coded symbol by symbol;
//   3. xo_assemble (one wave per chunk): stream and block headers, the
//      segments' LZMA2 chunks back to back, end mark, padding, CRC64 of the
//      serialised chunk, index and footer.
#include "zcg_crc.h"
#include "zcg_xz_enc.h"

namespace zcg {

namespace {

constexpr u32 XO_SEG = 1u << 18;   // bytes per independently coded segment
constexpr u32 XO_WIN = 256;        // parse window (positions)
constexpr u32 XO_K = 3;            // candidates kept per position
constexpr u32 XO_DEPTH = 16;       // hash-chain links walked
constexpr u32 XO_NICE = 64;        // stop walking at a match this long
constexpr u32 XO_W2 = 64;          // 2-byte repeat search distance
constexpr u32 XO_LENS = 8;         // lengths 2..XO_LENS of a range, then its last three
constexpr u32 XO_MAXLEN = 273;
constexpr u32 XO_PROBS = 1846 + 0x300;  // lc = lp = 0: one literal coder
constexpr u32 XO_PROPS = (2 * 5 + 0) * 9 + 0;
constexpr u64 XO_SEGCAP = XO_SEG + XO_SEG / 16 + 4096;  // a segment's LZMA2 chunks (bound)
constexpr u32 XO_KEYBITS = 20;
constexpr u64 XO_SUB_BYTES = 128ull << 20;
constexpr u64 XO_SUPER_BYTES = 1ull << 30;
constexpr u32 XO_DMAX_LG = 23;  // candidate distances < 2^23 (they pack in 23 bits)
constexpr u32 ARC_REP = 2, ARC_MATCH = 1100;  // arc ids: 0 literal, 1 short rep, 2 + r*274 + len, 1100 + len

// -log2((i*16+8)/2048) in 1/16 bit, rounded (the price of a bit of probability p is c_xo_price[p >> 4])
__constant__ u8 c_xo_price[128] = {
    128, 103, 91, 83, 77, 73, 69, 65, 63, 60, 58, 56, 54, 52, 50, 49, 47, 46, 45, 43, 42, 41, 40, 39, 38, 37,
    36,  35,  35, 34, 33, 32, 32, 31, 30, 30, 29, 28, 28, 27, 27, 26, 25, 25, 24, 24, 23, 23, 22, 22, 21, 21,
    21,  20,  20, 19, 19, 18, 18, 18, 17, 17, 17, 16, 16, 15, 15, 15, 14, 14, 14, 13, 13, 13, 12, 12, 12, 12,
    11,  11,  11, 10, 10, 10, 10, 9,  9,  9,  9,  8,  8,  8,  7,  7,  7,  7,  7,  6,  6,  6,  6,  5,  5,  5,
    5,   4,   4,  4,  4,  4,  3,  3,  3,  3,  3,  2,  2,  2,  2,  2,  1,  1,  1,  1,  1,  0,  0,  0};

__device__ __forceinline__ u32 st_lit(u32 s) { return s < 4 ? 0 : (s < 10 ? s - 3 : s - 6); }
__device__ __forceinline__ u32 st_match(u32 s) { return s < 7 ? 7 : 10; }
__device__ __forceinline__ u32 st_rep(u32 s) { return s < 7 ? 8 : 11; }
__device__ __forceinline__ u32 st_short(u32 s) { return s < 7 ? 9 : 11; }
__device__ __forceinline__ u32 slot_of(u32 d) {
    if (d < 4) return d;
    const u32 lg = 31 - __builtin_clz(d);
    return 2 * lg + ((d >> (lg - 1)) & 1);
}
__device__ __forceinline__ u32 ufl(u32 v) { return (u32)__builtin_amdgcn_readfirstlane((int)v); }

// ---------------------------------------------------------------- candidates
__global__ void xo_cands(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, u64 tot, DType t, u64 dmax,
                         const u32* __restrict__ prev, u32* __restrict__ cand) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tot) return;
    const u32 cl = (u32)(g / D);
    const u64 p = g - (u64)cl * D;
    u32 k0 = 0, k1 = 0, k2 = 0;  // the kept candidates, newest (longest) in k2
    const zcg_chunk ch = chunks[c0 + cl];
    if (ch.src_len >= D) {  // short src: INVALID_DATA in the assembler
        const u8* src = (const u8*)ch.src;
        const u32 mx = (D - p) < XO_MAXLEN ? (u32)(D - p) : XO_MAXLEN;
        auto push = [&](u32 l, u32 d) { k0 = k1; k1 = k2; k2 = (l << 23) | d; };
        // common length of the runs at p and q (< p), capped at mx
        auto common = [&](u64 q) -> u32 {
            u32 k = 0;
            while (k + 4 <= mx) {
                const u32 x = xe_ser4(src, p + k, t) ^ xe_ser4(src, q + k, t);
                if (x) return k + ((u32)__builtin_ctz(x) >> 3);
                k += 4;
            }
            while (k < mx && xe_ser1(src, p + k, t) == xe_ser1(src, q + k, t)) k++;
            return k;
        };
        u32 best = 1;
        if (p + 3 <= D) {  // the nearest 2-byte repeat within XO_W2
            const u32 b0 = xe_ser1(src, p, t) | (xe_ser1(src, p + 1, t) << 8);
            const u64 lo = p > XO_W2 ? p - XO_W2 : 0;
            u32 w = p > 0 ? xe_ser1(src, p, t) : 0u;  // byte q + 1 of the pair at q (sliding down)
            for (u64 q = p; q-- > lo;) {
                const u32 v = xe_ser1(src, q, t);
                if ((v | (w << 8)) == b0) {
                    const u32 l = common(q);
                    best = l;
                    push(l, (u32)(p - q - 1));
                    break;
                }
                w = v;
            }
        }
        if (p + 4 <= D) {
            if (best < 3) best = 3;
            const u32 v0 = xe_ser4(src, p, t);
            const u64 cbase = (u64)cl * D;
            u32 q = prev[g];
            for (u32 dep = 0; dep < XO_DEPTH && q != 0xFFFFFFFFu; dep++) {
                const u64 qp = q - cbase;
                if (p - qp > dmax) break;
                const u32 qn = prev[q];  // the next link, in flight during this compare
                u32 l = 0;
                if (xe_ser4(src, qp, t) == v0) l = common(qp);
                else {
                    const u32 x = xe_ser4(src, qp, t) ^ v0;
                    l = (u32)__builtin_ctz(x) >> 3;
                }
                if (l > mx) l = mx;
                if (l > best) {
                    best = l;
                    push(l, (u32)(p - qp - 1));
                    if (l >= XO_NICE || l == mx) break;
                }
                q = qn;
            }
        }
    }
    // lengths ascending, empty slots first-to-last as 0: k0 <= k1 <= k2 (0 = none)
    u32* c = cand + g * XO_K;
    const u32 n = (k0 != 0) + (k1 != 0) + (k2 != 0);
    c[0] = n == 3 ? k0 : (n == 2 ? k1 : k2);
    c[1] = n == 3 ? k1 : (n == 2 ? k2 : 0u);
    c[2] = n == 3 ? k2 : 0u;
}

// ---------------------------------------------------------------- segments
struct XoLds {
    u64 key[XO_WIN + 1];       // best (price << 20 | source << 11 | arc) of each window node
    u32 nrep[XO_WIN + 1][4];   // reps of each node's best path
    u32 wc[XO_WIN * XO_K];     // the window's candidates
    u32 pth[XO_WIN];           // planned path, reversed: arc | len << 11
    u32 pdist[XO_WIN];         //   and the match distance
    u16 probs[XO_PROBS];
    u8 nst[XO_WIN + 1];        // state of each node
    u8 tile[XO_WIN];           // the window's bytes
    u8 price[128];
};

__device__ __forceinline__ u32 xo_pb(const XoLds& L, u32 i, u32 b) {
    const u32 p = L.probs[i];
    return L.price[(b ? 2048 - p : p) >> 4];
}
__device__ __forceinline__ u32 xo_ptree(const XoLds& L, u32 base, u32 nb, u32 v) {
    u32 s = 0;
    for (u32 k = 0; k < nb; k++) {
        const u32 b = (v >> (nb - 1 - k)) & 1;
        s += xo_pb(L, base + ((1u << k) | (v >> (nb - k))), b);
    }
    return s;
}
__device__ __forceinline__ u32 xo_prtree(const XoLds& L, u32 base, u32 nb, u32 v) {
    u32 s = 0;
    for (u32 k = 0; k < nb; k++) {
        const u32 b = (v >> k) & 1;
        // index after k bits: 1 followed by bits 0..k-1 in reverse order of arrival
        u32 m = 1;
        for (u32 j = 0; j < k; j++) m = (m << 1) | ((v >> j) & 1);
        s += xo_pb(L, base + m, b);
    }
    return s;
}
__device__ __forceinline__ u32 xo_plen(const XoLds& L, u32 lb, u32 l, u32 ps) {
    if (l < 8) return xo_pb(L, lb + EL_CHOICE, 0) + xo_ptree(L, lb + EL_LOW + (ps << 3), 3, l);
    if (l < 16)
        return xo_pb(L, lb + EL_CHOICE, 1) + xo_pb(L, lb + EL_CHOICE2, 0) + xo_ptree(L, lb + EL_MID + (ps << 3), 3, l - 8);
    return xo_pb(L, lb + EL_CHOICE, 1) + xo_pb(L, lb + EL_CHOICE2, 1) + xo_ptree(L, lb + EL_HIGH, 8, l - 16);
}
__device__ __forceinline__ u32 xo_pdist(const XoLds& L, u32 d, u32 len) {
    const u32 lps = len - 2 < 3 ? len - 2 : 3, slot = slot_of(d);
    u32 s = xo_ptree(L, E_POS_SLOT + (lps << 6), 6, slot);
    if (slot >= 4) {
        const u32 nd = (slot >> 1) - 1, base = (2 | (slot & 1)) << nd, red = d - base;
        if (slot < 14) s += xo_prtree(L, E_SPEC_POS + base - slot - 1, nd, red);
        else s += (nd - 4) * 16 + xo_prtree(L, E_ALIGN, 4, red & 15);
    }
    return s;
}

// kept lengths of the range [a, Lr]: a..min(Lr, 8), then max(a, 9, Lr - 2)..Lr
__device__ __forceinline__ u32 xo_range_count(u32 a, u32 Lr, u32* c1, u32* hi0) {
    if (Lr < a) { *c1 = 0; *hi0 = a; return 0; }
    const u32 lo_end = Lr < XO_LENS ? Lr : XO_LENS;
    *c1 = lo_end >= a ? lo_end - a + 1 : 0;
    u32 h = Lr >= 2 ? Lr - 2 : 0;
    if (h < XO_LENS + 1) h = XO_LENS + 1;
    if (h < a) h = a;
    *hi0 = h;
    return *c1 + (Lr >= h ? Lr - h + 1 : 0);
}

// the distance of match arc `len` from node `src` (the first candidate whose clipped range holds it)
__device__ __forceinline__ u32 xo_arc_dist(const XoLds& L, u32 src, u32 len, u32 room) {
    for (u32 k = 0; k < XO_K; k++) {
        const u32 c = L.wc[src * XO_K + k], Lk = c >> 23;
        if (Lk && len <= (Lk < room ? Lk : room)) return c & 0x7FFFFFu;
    }
    return 0;
}

__global__ __launch_bounds__(64) void xo_segment(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, DType t,
                                                 u32 nseg, const u32* __restrict__ cand, u8* __restrict__ segbuf,
                                                 u32* __restrict__ seglen) {
    __shared__ XoLds L;
    const u32 sid = blockIdx.x;
    const u32 cl = sid / nseg, k = sid % nseg;
    const int lane = lane_id();
    const zcg_chunk ch = chunks[c0 + cl];
    if (ch.src_len < D) {
        if (lane == 0) seglen[sid] = 0;
        return;
    }
    for (u32 i = lane; i < 128; i += 64) L.price[i] = c_xo_price[i];
    XeEnc e;
    e.src = (const gu8*)ch.src;
    e.n = D;
    e.t = t;
    e.dst = (gu8*)(segbuf + (u64)sid * XO_SEGCAP);
    e.cap = XO_SEGCAP;
    e.pos = 0;
    e.lbuf = 0;
    e.over = false;
    e.probs = (lu16*)L.probs;
    e.lane = lane;
    const u32* cbase = cand + (u64)cl * D * XO_K;
    const u64 s0 = (u64)k * XO_SEG, s1 = (D - s0) < XO_SEG ? D : s0 + XO_SEG;
    bool need_dict = k == 0, need_props = true, need_state = true;
    u32 state = 0, r0 = 0, r1 = 0, r2 = 0, r3 = 0;
    u64 p = s0;
    auto sbyte = [&](u64 x, u64 wbase) -> u32 {  // serialised byte x (< the window end)
        return x >= wbase ? (u32)L.tile[x - wbase] : e.sb(x);
    };
    while (p < s1) {
        // ---- one LZMA2 chunk ----
        const u64 hdr = e.pos;
        const bool over0 = e.over;
        const u32 hlen = need_props ? 6 : 5;
        if (need_state) {
            __syncthreads();
            for (u32 i = lane; i < XO_PROBS; i += 64) L.probs[i] = 1024;
            __syncthreads();
            state = 0;
            r0 = r1 = r2 = r3 = 0;
        }
        for (u32 q = 0; q < hlen; q++) e.out(0);
        const u64 data0 = e.pos;
        const u64 u0 = p;
        e.rc_reset();
        u32 npath = 0;  // symbols of the planned path left (pth[npath-1] is next)
        u64 wb = 0;     // the planned window's first position
        while (p < s1 && (e.pos - data0) + e.cache_size + 5 < XE_CMAX) {
            if (npath == 0) {
                // ================= plan a window [p, we) =================
                const u64 we = (s1 - p) < XO_WIN ? s1 : p + XO_WIN;
                const u32 W = (u32)(we - p);
                wb = p;
                __syncthreads();
                for (u32 j = lane; j <= W; j += 64) L.key[j] = ~0ull;
                for (u32 j = lane; j < W; j += 64) L.tile[j] = (u8)e.sb(p + j);
                for (u32 j = lane; j < W * XO_K; j += 64) L.wc[j] = cbase[p * XO_K + j];
                __syncthreads();
                if (lane == 0) {
                    L.key[0] = 0;
                    L.nst[0] = (u8)state;
                    L.nrep[0][0] = r0; L.nrep[0][1] = r1; L.nrep[0][2] = r2; L.nrep[0][3] = r3;
                }
                __syncthreads();
                for (u32 i = 0; i < W; i++) {
                    const u64 a = L.key[i];
                    const u32 alo = ufl((u32)a), ahi = ufl((u32)(a >> 32));
                    u32 st, q0, q1, q2, q3;
                    if (i == 0) {
                        st = state; q0 = r0; q1 = r1; q2 = r2; q3 = r3;
                    } else {
                        const u32 src = (alo >> 11) & 511, arc = alo & 2047;
                        const u32 bst = ufl(L.nst[src]);
                        const u32 b0 = ufl(L.nrep[src][0]), b1 = ufl(L.nrep[src][1]), b2 = ufl(L.nrep[src][2]),
                                  b3 = ufl(L.nrep[src][3]);
                        if (arc == 0) { st = st_lit(bst); q0 = b0; q1 = b1; q2 = b2; q3 = b3; }
                        else if (arc == 1) { st = st_short(bst); q0 = b0; q1 = b1; q2 = b2; q3 = b3; }
                        else if (arc < ARC_MATCH) {
                            const u32 r = (arc - ARC_REP) / 274;
                            st = st_rep(bst);
                            q0 = r == 0 ? b0 : r == 1 ? b1 : r == 2 ? b2 : b3;
                            q1 = r == 0 ? b1 : b0;
                            q2 = r <= 1 ? b2 : b1;
                            q3 = r <= 2 ? b3 : b2;
                        } else {
                            st = st_match(bst);
                            q0 = ufl(xo_arc_dist(L, src, arc - ARC_MATCH, W - src));
                            q1 = b0; q2 = b1; q3 = b2;
                        }
                        if (lane == 0) {
                            L.nst[i] = (u8)st;
                            L.nrep[i][0] = q0; L.nrep[i][1] = q1; L.nrep[i][2] = q2; L.nrep[i][3] = q3;
                        }
                    }
                    const u32 P = (alo >> 20) | (ahi << 12);
                    const u64 at = p + i;
                    const u32 ps = (u32)at & 3;
                    const u32 room = W - i, mx = room < XO_MAXLEN ? room : XO_MAXLEN;
                    const u32 sym = L.tile[i];
                    const u32 mbyte = at > q0 ? ufl(sbyte(at - q0 - 1, p)) : 0u;
                    // ---- rep lengths: lane = rep * 16 + byte of the round ----
                    u32 rl0 = 0, rl1 = 0, rl2 = 0, rl3 = 0, open = 0xF;
                    {
                        const u32 r = (u32)lane >> 4, tb = (u32)lane & 15;
                        const u32 rd = r == 0 ? q0 : r == 1 ? q1 : r == 2 ? q2 : q3;
                        for (u32 base = 0; open; base += 16) {
                            const u32 o = base + tb;
                            bool ok = false;
                            if (((open >> r) & 1) && at > rd && o < mx)
                                ok = L.tile[i + o] == sbyte(at - rd - 1 + o, p);
                            const u64 miss = __ballot(!ok);
                            u32 done = 0;
                            for (u32 rr = 0; rr < 4; rr++) {
                                if (!((open >> rr) & 1)) continue;
                                const u32 m = (u32)(miss >> (16 * rr)) & 0xFFFFu;
                                if (m) {
                                    const u32 v = base + (u32)__builtin_ctz(m);
                                    if (rr == 0) rl0 = v; else if (rr == 1) rl1 = v; else if (rr == 2) rl2 = v; else rl3 = v;
                                    done |= 1u << rr;
                                }
                            }
                            open &= ~done;
                        }
                    }
                    // ---- literal bit prices (lanes 0-7) and flag prices (lanes 8-19) ----
                    u32 pv = 0;
                    if (lane < 8) {
                        const u32 j = (u32)lane, b = (sym >> (7 - j)) & 1, m = (1u << j) | (sym >> (8 - j));
                        u32 idx = E_LITERAL + m;
                        if (st >= 7) {
                            const u32 off = (sym >> (8 - j)) == (mbyte >> (8 - j)) ? 0x100u : 0u;
                            const u32 mbit = off ? ((mbyte >> (7 - j)) & 1) << 8 : 0u;
                            idx += off + mbit;
                        }
                        pv = xo_pb(L, idx, b);
                    } else if (lane < 20) {
                        const u32 f = (u32)lane - 8, b = f & 1;
                        const u32 idx = f < 2 ? E_IS_MATCH + (st << 4) + ps
                                      : f < 4 ? E_IS_REP + st
                                      : f < 6 ? E_IS_REP_G0 + st
                                      : f < 8 ? E_IS_REP_G1 + st
                                      : f < 10 ? E_IS_REP_G2 + st
                                      : E_IS_REP0_LONG + (st << 4) + ps;
                        pv = xo_pb(L, idx, b);
                    }
                    u32 litp = 0;
                    for (int j = 0; j < 8; j++) litp += (u32)__builtin_amdgcn_readlane((int)pv, j);
                    u32 f[12];
                    for (int j = 0; j < 12; j++) f[j] = (u32)__builtin_amdgcn_readlane((int)pv, 8 + j);
                    // ---- arcs: literal, short rep, rep ranges, candidate ranges ----
                    const bool sr = at > q0 && sym == mbyte;
                    const u32 rbase = P + f[1] + f[3];
                    const u32 rb[4] = {rbase + f[4] + f[11], rbase + f[5] + f[6], rbase + f[5] + f[7] + f[8],
                                       rbase + f[5] + f[7] + f[9]};
                    const u32 rl[4] = {rl0, rl1, rl2, rl3};
                    u32 cnt[9], ga[9], gc1[9], gh[9], gd[9];
                    cnt[0] = 1; cnt[1] = sr ? 1u : 0u;
                    for (u32 r = 0; r < 4; r++) {
                        ga[2 + r] = 2;
                        cnt[2 + r] = rl[r] >= 2 ? xo_range_count(2, rl[r], &gc1[2 + r], &gh[2 + r]) : 0u;
                        gd[2 + r] = 0;
                    }
                    u32 lprev = 1;
                    for (u32 c = 0; c < XO_K; c++) {
                        const u32 w = L.wc[i * XO_K + c], Lk = w >> 23;
                        const u32 Lr = Lk < mx ? Lk : mx;
                        const u32 a0 = lprev + 1 > 2 ? lprev + 1 : 2;
                        ga[6 + c] = a0;
                        gd[6 + c] = w & 0x7FFFFFu;
                        cnt[6 + c] = Lk ? xo_range_count(a0, Lr, &gc1[6 + c], &gh[6 + c]) : 0u;
                        if (Lk && Lr > lprev) lprev = Lr;
                    }
                    u32 N = 0;
                    for (u32 g = 0; g < 9; g++) N += cnt[g];
                    const u32 mb0 = P + f[1] + f[2];
                    for (u32 base = 0; base < N; base += 64) {
                        const u32 j = base + (u32)lane;
                        if (j < N) {
                            u32 g = 0, acc = 0;
                            while (j >= acc + cnt[g]) { acc += cnt[g]; g++; }
                            const u32 el = j - acc;
                            u32 len = 1, price, arc;
                            if (g == 0) {
                                price = P + f[0] + litp;
                                arc = 0;
                            } else if (g == 1) {
                                price = rbase + f[4] + f[10];
                                arc = 1;
                            } else {
                                len = el < gc1[g] ? ga[g] + el : gh[g] + (el - gc1[g]);
                                if (g < 6) {
                                    price = rb[g - 2] + xo_plen(L, E_REP_LEN, len - 2, ps);
                                    arc = ARC_REP + (g - 2) * 274 + len;
                                } else {
                                    price = mb0 + xo_plen(L, E_LEN, len - 2, ps) + xo_pdist(L, gd[g], len);
                                    arc = ARC_MATCH + len;
                                }
                            }
                            const u64 key = ((u64)price << 20) | ((u64)i << 11) | arc;
                            atomicMin((unsigned long long*)&L.key[i + len], (unsigned long long)key);
                        }
                    }
                    __syncthreads();
                }
                // ---- the path to the window end (reversed) ----
                {
                    u32 j = W, np = 0;
                    while (j > 0) {
                        const u64 a = L.key[j];
                        const u32 alo = ufl((u32)a);
                        const u32 src = (alo >> 11) & 511, arc = alo & 2047, len = j - src;
                        const u32 d = arc >= ARC_MATCH ? xo_arc_dist(L, src, len, W - src) : 0u;
                        if (lane == 0) {
                            L.pth[np] = arc | (len << 11);
                            L.pdist[np] = d;
                        }
                        np++;
                        j = src;
                    }
                    npath = np;
                    __syncthreads();
                }
            }
            // ---- code the next symbol of the path ----
            npath--;
            const u32 w = ufl(L.pth[npath]);
            const u32 arc = w & 2047, len = w >> 11, ps = (u32)p & 3;
            if (arc == 0) {
                const u32 sym = L.tile[p - wb];
                e.bit(E_IS_MATCH + (state << 4) + ps, 0);
                if (state < 7) {
                    e.tree(E_LITERAL, 8, sym);
                } else {
                    u32 mb = p > r0 ? ufl(sbyte(p - r0 - 1, wb)) : 0u, off = 0x100, m = 1;
                    for (int q = 7; q >= 0; q--) {
                        const u32 b = (sym >> q) & 1;
                        mb <<= 1;
                        const u32 mbit = mb & off;
                        e.bit(E_LITERAL + off + mbit + m, b);
                        m = (m << 1) | b;
                        off &= b ? mbit : ~mbit;
                    }
                }
                state = st_lit(state);
            } else if (arc == 1) {
                e.bit(E_IS_MATCH + (state << 4) + ps, 1);
                e.bit(E_IS_REP + state, 1);
                e.bit(E_IS_REP_G0 + state, 0);
                e.bit(E_IS_REP0_LONG + (state << 4) + ps, 0);
                state = st_short(state);
            } else if (arc < ARC_MATCH) {
                const u32 r = (arc - ARC_REP) / 274;
                e.bit(E_IS_MATCH + (state << 4) + ps, 1);
                e.bit(E_IS_REP + state, 1);
                if (r == 0) {
                    e.bit(E_IS_REP_G0 + state, 0);
                    e.bit(E_IS_REP0_LONG + (state << 4) + ps, 1);
                } else {
                    e.bit(E_IS_REP_G0 + state, 1);
                    if (r == 1) {
                        e.bit(E_IS_REP_G1 + state, 0);
                    } else {
                        e.bit(E_IS_REP_G1 + state, 1);
                        e.bit(E_IS_REP_G2 + state, r - 2);
                    }
                    const u32 d = r == 1 ? r1 : r == 2 ? r2 : r3;
                    if (r == 3) r3 = r2;
                    if (r >= 2) r2 = r1;
                    r1 = r0;
                    r0 = d;
                }
                e.length(E_REP_LEN, len - 2, ps);
                state = st_rep(state);
            } else {
                const u32 d = ufl(L.pdist[npath]);
                e.bit(E_IS_MATCH + (state << 4) + ps, 1);
                e.bit(E_IS_REP + state, 0);
                e.length(E_LEN, len - 2, ps);
                e.distance(d, len);
                r3 = r2; r2 = r1; r1 = r0; r0 = d;
                state = st_match(state);
            }
            p += len;
        }
        for (int q = 0; q < 5; q++) e.shift_low();
        if (e.pos - data0 >= p - u0) {
            // stored chunk (liblzma's rule; usz <= XE_CMAX < 64 KiB): the state resets next
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
        if (need_props) e.patch(hdr + 5, XO_PROPS);
        need_dict = need_props = need_state = false;
    }
    e.out_flush();
    if (lane == 0) seglen[sid] = e.over ? 0xFFFFFFFFu : (u32)e.pos;
}

// ---------------------------------------------------------------- assembly
__global__ __launch_bounds__(64) void xo_assemble(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, DType t,
                                                  u32 dprop, u32 nseg, const u8* __restrict__ segbuf,
                                                  const u32* __restrict__ seglen, u64* __restrict__ out_len,
                                                  i32* __restrict__ status) {
    const u32 cl = blockIdx.x, c = c0 + cl;
    const int lane = lane_id();
    const zcg_chunk ch = chunks[c];
    if (ch.src_len < D) {  // fewer serialised bytes than the chunk holds (chunk.rs:309-318)
        if (lane == 0) { out_len[c] = 0; status[c] = ZCG_ERR_INVALID_DATA; }
        return;
    }
    gu8* dst = (gu8*)ch.dst;
    const u64 cap = ch.dst_cap;
    auto put = [&](u64 at, u32 b) { if (at < cap) dst[at] = (u8)b; };  // (one lane)
    u64 pos = 12;
    if (lane < 12) {
        const u32 b = (u32)(((lane < 8 ? 0xFD377A585A000004ull : 0xE6D6B446ull) >> (8 * ((lane < 8 ? 7 : 11) - lane))) & 0xFF);
        put((u64)lane, b);
    }
    u64 unpadded = 0;
    bool bad = false;
    if (D > 0) {
        if (lane == 0) {  // block header: 02 00 21 01 <prop> 00 00 00 + CRC32
            u32 hc = 0xFFFFFFFFu;
            for (int k = 0; k < 8; k++) {
                const u32 b = k == 0 ? 0x02u : (k == 2 ? 0x21u : (k == 3 ? 0x01u : (k == 4 ? dprop : 0u)));
                put(12 + k, b);
                hc = g_crc32_table[(hc ^ b) & 0xFF] ^ (hc >> 8);
            }
            hc = ~hc;
            for (int k = 0; k < 4; k++) put(20 + k, (hc >> (8 * k)) & 0xFF);
        }
        pos = 24;
        const u64 cdata0 = pos;
        for (u32 k = 0; k < nseg; k++) {
            const u32 sl = seglen[(u64)cl * nseg + k];
            if (sl == 0xFFFFFFFFu) { bad = true; break; }
            const u8* sb = segbuf + ((u64)cl * nseg + k) * XO_SEGCAP;
            for (u32 q = (u32)lane; q < sl; q += 64) put(pos + q, sb[q]);
            pos += sl;
        }
        if (lane == 0) put(pos, 0x00);  // end of LZMA2 data
        pos++;
        const u64 csize = pos - cdata0;
        while ((pos - cdata0) & 3) { if (lane == 0) put(pos, 0); pos++; }
        const u64 crc = wave_crc_fn<u64, CRC64_POLY>([&](u64 q) -> u32 { return xe_ser1((const u8*)ch.src, q, t); }, 0, D);
        if (lane == 0)
            for (int k = 0; k < 8; k++) put(pos + k, (u32)(crc >> (8 * k)) & 0xFF);
        pos += 8;
        unpadded = 12 + csize + 8;
    }
    if (lane == 0) {
        // index: 00, count, (unpadded, uncompressed), padding, CRC32
        const u64 idx0 = pos;
        u32 ic = 0xFFFFFFFFu;
        auto iout = [&](u32 b) { put(pos++, b); ic = g_crc32_table[(ic ^ b) & 0xFF] ^ (ic >> 8); };
        auto ivli = [&](u64 v) {
            while (v >= 0x80) { iout((u32)(v & 0x7F) | 0x80); v >>= 7; }
            iout((u32)v);
        };
        iout(0x00);
        ivli(D > 0 ? 1 : 0);
        if (D > 0) { ivli(unpadded); ivli(D); }
        while ((pos - idx0) & 3) iout(0x00);
        ic = ~ic;
        for (int k = 0; k < 4; k++) put(pos++, (ic >> (8 * k)) & 0xFF);
        const u64 isize = pos - idx0;
        const u32 bsz = (u32)(isize / 4 - 1);
        const u64 fbw = (u64)bsz | (0x0400ull << 32);
        u32 fc = 0xFFFFFFFFu;
        for (int k = 0; k < 6; k++) fc = g_crc32_table[(fc ^ (u32)(fbw >> (8 * k))) & 0xFF] ^ (fc >> 8);
        fc = ~fc;
        for (int k = 0; k < 4; k++) put(pos++, (fc >> (8 * k)) & 0xFF);
        for (int k = 0; k < 6; k++) put(pos++, (u32)(fbw >> (8 * k)) & 0xFF);
        put(pos++, 0x59);
        put(pos++, 0x5A);
        out_len[c] = bad ? 0 : pos;
        status[c] = bad ? ZCG_ERR_RUNTIME : (pos > cap ? ZCG_ERR_OUTPUT_TOO_SMALL : ZCG_OK);
    }
}

struct XoLayout {
    u32 m, sm, nseg;
    u64 tot, cub_bytes;
    u64 off_ka, off_kb, off_va, off_vb, off_prev, off_cand, off_seg, off_len, off_cub, total;
};

XoLayout xo_layout(u64 D, u32 n) {
    XoLayout y{};
    u64 m = D ? XO_SUB_BYTES / D : n;
    if (m < 1) m = 1;
    if (m > n) m = n;
    if (m > 4096) m = 4096;
    y.m = (u32)m;
    y.tot = m * D;
    u64 sm = D ? XO_SUPER_BYTES / D : n;
    sm = sm / m * m;
    if (sm < m) sm = m;
    if (sm > n) sm = n;
    y.sm = (u32)sm;
    y.nseg = D ? (u32)((D + XO_SEG - 1) / XO_SEG) : 1;
    y.cub_bytes = xe_sort_scratch(y.tot);
    u64 p = 0;
    auto take = [&](u64 bytes) { const u64 o = p; p = (p + bytes + 255) & ~255ull; return o; };
    y.off_ka = take(4 * y.tot);
    y.off_kb = take(4 * y.tot);
    y.off_va = take(4 * y.tot);
    y.off_vb = take(4 * y.tot);
    y.off_prev = take(4 * y.tot);
    y.off_cand = take(4ull * XO_K * y.sm * D);
    y.off_seg = take(XO_SEGCAP * y.sm * y.nseg);
    y.off_len = take(4ull * y.sm * y.nseg);
    y.off_cub = take(y.cub_bytes);
    y.total = p;
    return y;
}

}  // namespace

uint64_t xz_opt_ws_bytes(const zcg_array* a, uint32_t n) {
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    if (n == 0) return 0;
    return xo_layout(D, n).total;
}

hipError_t launch_xz_opt(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n, uint64_t* d_out_len,
                         int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const XoLayout y = xo_layout(D, n);
    if (ws_bytes < y.total || y.tot >= (1ull << 31) || D >= (1ull << 32)) return hipErrorInvalidValue;
    u8* w = (u8*)ws;
    const int preset = a->compression.xz_preset;
    const int pr = (preset < 0 || preset > 9) ? 6 : preset;
    const u32 dlg = pr == 0 ? 18u : (pr == 1 ? 20u : (pr == 2 ? 21u : (pr <= 4 ? 22u : (pr <= 6 ? 23u : (u32)(pr + 17)))));
    const u64 dmax = dlg < XO_DMAX_LG ? (1ull << dlg) : (1ull << XO_DMAX_LG);
    u32 cbits = 0;
    while ((1u << cbits) < y.m) cbits++;
    for (u32 s0 = 0; s0 < n; s0 += y.sm) {
        const u32 scnt = (n - s0) < y.sm ? (n - s0) : y.sm;
        for (u32 c0 = s0; c0 < s0 + scnt; c0 += y.m) {
            const u32 cnt = (s0 + scnt - c0) < y.m ? (s0 + scnt - c0) : y.m;
            const u64 tot = (u64)cnt * D;
            if (!tot) continue;
            u32 *ka = (u32*)(w + y.off_ka), *kb = (u32*)(w + y.off_kb);
            u32 *va = (u32*)(w + y.off_va), *vb = (u32*)(w + y.off_vb);
            const u32 G = (u32)((tot + 255) / 256);
            hipError_t e = launch_xe_chains(d_chunks, c0, D, tot, t, cbits, ka, kb, va, vb, (u32*)(w + y.off_prev),
                                            w + y.off_cub, y.cub_bytes, s);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(xo_cands, dim3(G), dim3(256), 0, s, d_chunks, c0, D, tot, t, dmax,
                               (const u32*)(w + y.off_prev), (u32*)(w + y.off_cand) + (u64)(c0 - s0) * D * XO_K);
        }
        if (D > 0)
            hipLaunchKernelGGL(xo_segment, dim3(scnt * y.nseg), dim3(64), 0, s, d_chunks, s0, D, t, y.nseg,
                               (const u32*)(w + y.off_cand), w + y.off_seg, (u32*)(w + y.off_len));
        hipLaunchKernelGGL(xo_assemble, dim3(scnt), dim3(64), 0, s, d_chunks, s0, D, t, 2u * (dlg - 12u), y.nseg,
                           (const u8*)(w + y.off_seg), (const u32*)(w + y.off_len), d_out_len, d_status);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace zcg
