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
//      first-best tie rule (lanes 16 g .. 16 g + 15 price rep g's lengths,
//      then candidate g's); the path is then range-coded symbol by symbol.
//      Residency: 9.75 KB of LDS per wave (the length-price table keeps one
//      copy of the position-state-free high lengths) and 128 VGPRs (prices
//      packed two per register) admit 4 waves per SIMD, so a 1 024-chunk
//      batch (4 096 waves) is one generation; at 12.8 KB of LDS only 11
//      waves per CU were admitted;
//   3. xo_assemble (one wave per chunk): stream and block headers, the
//      segments' LZMA2 chunks back to back, end mark, padding, CRC64 of the
//      serialised chunk, index and footer.
#include "zcg_crc.h"
#include "zcg_xz_enc.h"

namespace zcg {

namespace {

#ifndef XO_SEG_KB
#define XO_SEG_KB 256
#endif
constexpr u32 XO_SEG = XO_SEG_KB << 10;  // bytes per independently coded segment (a 1 MiB chunk: 4 waves)
constexpr u32 XO_WIN = 256;        // parse window (positions)
constexpr u32 XO_K = 3;            // candidates kept per position
constexpr u32 XO_DEPTH = 16;       // hash-chain links walked
constexpr u32 XO_NICE = 64;        // stop walking at a match this long
constexpr u32 XO_W2 = 64;          // 2-byte repeat search distance
constexpr u32 XO_LENS = 8;         // lengths 2..XO_LENS of a range, then its last three
constexpr u32 XO_MAXLEN = 273;
constexpr u32 XO_HIST = 0;  // bytes before a window kept in the LDS tile (a 4 KiB history was slower: occupancy)
constexpr u32 XO_PROBS = 1846 + 0x300;  // lc = lp = 0: one literal coder
constexpr u32 XO_PROPS = (2 * 5 + 0) * 9 + 0;
constexpr u64 XO_SEGCAP = XO_SEG + XO_SEG / 16 + 4096;  // a segment's LZMA2 chunks (bound)
constexpr u32 XO_KEYBITS = 20;
constexpr u64 XO_SUB_BYTES = 128ull << 20;
constexpr u64 XO_SUPER_BYTES = 1ull << 30;
constexpr u32 XO_DMAX_LG = 23;  // candidate distances < 2^23 (they pack in 23 bits)
constexpr u32 ARC_REP = 2, ARC_MATCH = 1100;  // arc ids: 0 literal, 1 short rep, 2 + r*274 + len, 1100 + len
#ifndef XO_WPE
#define XO_WPE 4  // waves per SIMD the coder's register allocation targets (LDS admits 4)
#endif
#ifndef XO_PROF
#define XO_PROF 0  // 1 (A/B builds only): cycle and event counters, read by zcg__debug_xz_opt_counters
#endif
__device__ unsigned long long g_xo_prof[16];  // plan cycles, code cycles, nodes, symbols, windows, total cycles

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
// wave-local ordering point for LDS (and the compiler): one wave per
// workgroup, whose LDS operations are performed in issue order
__device__ __forceinline__ void wsync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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


// Range-code `cnt` (<= N) bits whose probabilities sit at distinct indices:
// every probability is loaded before the first bit is coded, so a symbol
// costs one LDS round trip instead of one per bit.
template <int N>
__device__ __forceinline__ void xo_code(XeEnc& e, const u32 (&idx)[N], const u32 (&bits)[N], u32 cnt) {
    u32 pr[N];
#pragma unroll
    for (int j = 0; j < N; j++) pr[j] = (u32)j < cnt ? (u32)e.probs[idx[j]] : 0u;
#pragma unroll
    for (int j = 0; j < N; j++) {
        if ((u32)j >= cnt) break;
        const u32 p = pr[j], bound = (e.range >> 11) * p;
        u32 np;
        if (bits[j] == 0) {
            e.range = bound;
            np = p + ((2048 - p) >> 5);
        } else {
            e.low += bound;
            e.range -= bound;
            np = p - (p >> 5);
        }
        e.probs[idx[j]] = (u16)np;
        while (e.range < (1u << 24)) {
            e.range <<= 8;
            e.shift_low();
        }
    }
}

// Like xo_code, for N fixed slots of which `use` (bit j = slot j) are coded,
// in slot order: one LDS round trip for a whole symbol's modelled bits.
template <int N>
__device__ __forceinline__ void xo_code_m(XeEnc& e, const u32 (&idx)[N], const u32 (&bits)[N], u32 use) {
    u32 pr[N];
#pragma unroll
    for (int j = 0; j < N; j++) pr[j] = (use >> j) & 1 ? (u32)e.probs[idx[j]] : 0u;
#pragma unroll
    for (int j = 0; j < N; j++) {
        if (!((use >> j) & 1)) continue;
        const u32 p = pr[j], bound = (e.range >> 11) * p;
        u32 np;
        if (bits[j] == 0) {
            e.range = bound;
            np = p + ((2048 - p) >> 5);
        } else {
            e.low += bound;
            e.range -= bound;
            np = p - (p >> 5);
        }
        e.probs[idx[j]] = (u16)np;
        while (e.range < (1u << 24)) {
            e.range <<= 8;
            e.shift_low();
        }
    }
}
// the 10 length-code slots (choice, choice2, 8 tree levels) of l = len - 2 at o
template <int N>
__device__ __forceinline__ void xo_len_slots(u32 (&idx)[N], u32 (&bits)[N], u32& use, int o, u32 lb, u32 l, u32 ps) {
    idx[o] = lb + EL_CHOICE; bits[o] = l >= 8; use |= 1u << o;
    idx[o + 1] = lb + EL_CHOICE2; bits[o + 1] = l >= 16; use |= (l >= 8 ? 1u : 0u) << (o + 1);
    const u32 tb = l < 8 ? EL_LOW + (ps << 3) : l < 16 ? EL_MID + (ps << 3) : EL_HIGH;
    const u32 tv = l < 8 ? l : l < 16 ? l - 8 : l - 16, tn = l < 16 ? 3u : 8u;
#pragma unroll
    for (u32 k = 0; k < 8; k++) {
        const bool u = k < tn;
        bits[o + 2 + k] = u ? (tv >> (tn - 1 - k)) & 1 : 0u;
        idx[o + 2 + k] = lb + tb + ((1u << k) | (u ? tv >> (tn - k) : 0u));
        use |= (u ? 1u : 0u) << (o + 2 + k);
    }
}
// an nb-bit tree symbol (MSB first) / reverse tree symbol (LSB first)
template <int N>
__device__ __forceinline__ void xo_tree(XeEnc& e, u32 base, u32 nb, u32 v) {
    u32 idx[N], bits[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
        bits[k] = (u32)k < nb ? (v >> (nb - 1 - k)) & 1 : 0u;
        idx[k] = base + ((1u << k) | ((u32)k < nb ? v >> (nb - k) : 0u));
    }
    xo_code<N>(e, idx, bits, nb);
}
template <int N>
__device__ __forceinline__ void xo_rtree(XeEnc& e, u32 base, u32 nb, u32 v) {
    u32 idx[N], bits[N], m = 1;
#pragma unroll
    for (int k = 0; k < N; k++) {
        bits[k] = (v >> k) & 1;
        idx[k] = base + m;
        m = (m << 1) | bits[k];
    }
    xo_code<N>(e, idx, bits, nb);
}
__device__ __forceinline__ void xo_literal(XeEnc& e, u32 sym, bool matched, u32 mbyte) {
    u32 idx[8], bits[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        bits[j] = (sym >> (7 - j)) & 1;
        u32 x = E_LITERAL + ((1u << j) | (sym >> (8 - j)));
        if (matched) {
            const u32 off = (sym >> (8 - j)) == (mbyte >> (8 - j)) ? 0x100u : 0u;
            x += off + (off ? ((mbyte >> (7 - j)) & 1) << 8 : 0u);
        }
        idx[j] = x;
    }
    xo_code<8>(e, idx, bits, 8);
}
__device__ __forceinline__ void xo_length(XeEnc& e, u32 lb, u32 l, u32 ps) {  // l = len - 2
    u32 idx[10], bits[10], cnt;
    if (l < 8) {
        idx[0] = lb + EL_CHOICE; bits[0] = 0;
        for (int k = 0; k < 3; k++) { bits[1 + k] = (l >> (2 - k)) & 1; idx[1 + k] = lb + EL_LOW + (ps << 3) + ((1u << k) | (l >> (3 - k))); }
        cnt = 4;
    } else if (l < 16) {
        idx[0] = lb + EL_CHOICE; bits[0] = 1; idx[1] = lb + EL_CHOICE2; bits[1] = 0;
        const u32 v = l - 8;
        for (int k = 0; k < 3; k++) { bits[2 + k] = (v >> (2 - k)) & 1; idx[2 + k] = lb + EL_MID + (ps << 3) + ((1u << k) | (v >> (3 - k))); }
        cnt = 5;
    } else {
        idx[0] = lb + EL_CHOICE; bits[0] = 1; idx[1] = lb + EL_CHOICE2; bits[1] = 1;
        const u32 v = l - 16;
        for (int k = 0; k < 8; k++) { bits[2 + k] = (v >> (7 - k)) & 1; idx[2 + k] = lb + EL_HIGH + ((1u << k) | (v >> (8 - k))); }
        cnt = 10;
    }
    for (u32 k = cnt; k < 10; k++) { idx[k] = lb; bits[k] = 0; }
    xo_code<10>(e, idx, bits, cnt);
}
__device__ __forceinline__ void xo_distance(XeEnc& e, u32 d, u32 len) {
    const u32 lps = len - 2 < 3 ? len - 2 : 3, slot = slot_of(d);
    xo_tree<6>(e, E_POS_SLOT + (lps << 6), 6, slot);
    if (slot >= 4) {
        const u32 nd = (slot >> 1) - 1, base = (2 | (slot & 1)) << nd, red = d - base;
        if (slot < 14) {
            xo_rtree<5>(e, E_SPEC_POS + base - slot - 1, nd, red);
        } else {
            e.direct(red >> 4, nd - 4);
            xo_rtree<4>(e, E_ALIGN, 4, red & 15);
        }
    }
}

// ---------------------------------------------------------------- segments
struct XoLds {
    u64 key[XO_WIN + 1];       // best (price << 20 | source << 11 | arc) of each window node
    union {
        struct {                   // planning: the window's price tables (from the probabilities at its start)
            u16 len[640];          //   match / rep length codes (xo_lenix): l = len - 2 < 16 by position
                                   //   state, l >= 16 (choice, choice2, high tree: no position state) shared
            u16 slot[4][64];       //   position slots by length state
            u16 spec[128];         //   the reverse-tree low bits of distances 4..127
            u16 align[16];         //   the 4 align bits
        } pt;
        struct {                   // coding: the planned path, reversed
            u32 pth[XO_WIN];       //   arc | len << 11
            u32 pdist[XO_WIN];     //   and the match distance
        } path;
    } nr;
    u16 probs[XO_PROBS];
    u8 tile[XO_HIST + XO_WIN]; // the window's bytes and the XO_HIST before it
    u8 price[128];
};

// index of length code l = len - 2 of coder c (0 match, 1 rep) at position state ps in XoLds::pt.len
__device__ __forceinline__ u32 xo_lenix(u32 c, u32 ps, u32 l) {
    return l < 16 ? (c << 6) + (ps << 4) + l : 128 + (c << 8) + (l - 16);
}
__device__ __forceinline__ u32 xo_pb(const XoLds& L, u32 i, u32 b) {
    const u32 p = L.probs[i];
    return L.price[(b ? 2048 - p : p) >> 4];
}
// Price of a length code (l = len - 2, coder at lb, position state ps) and,
// for a match, of distance d: every probability index is formed first (21
// slots: choice, choice2, 8 tree levels; 6 slot levels, 5 reverse-tree
// levels), then all probabilities are read, then all their prices, so the
// arc costs two LDS round trips instead of two per tree level.
__device__ __forceinline__ u32 xo_arc_price(const XoLds& L, u32 lb, u32 l, u32 ps, bool match, u32 d, u32 len) {
    u32 idx[21], bit[21], use = 0;
    idx[0] = lb + EL_CHOICE; bit[0] = l >= 8; use |= 1u;
    idx[1] = lb + EL_CHOICE2; bit[1] = l >= 16; use |= (l >= 8 ? 1u : 0u) << 1;
    const u32 tb = l < 8 ? EL_LOW + (ps << 3) : l < 16 ? EL_MID + (ps << 3) : EL_HIGH;
    const u32 tv = l < 8 ? l : l < 16 ? l - 8 : l - 16, tn = l < 16 ? 3u : 8u;
#pragma unroll
    for (u32 k = 0; k < 8; k++) {
        const bool u = k < tn;
        bit[2 + k] = u ? (tv >> (tn - 1 - k)) & 1 : 0u;
        idx[2 + k] = lb + tb + ((1u << k) | (u ? tv >> (tn - k) : 0u));
        use |= (u ? 1u : 0u) << (2 + k);
    }
    u32 extra = 0;
    {
        const u32 lps = len - 2 < 3 ? len - 2 : 3, slot = slot_of(d);
#pragma unroll
        for (u32 k = 0; k < 6; k++) {
            bit[10 + k] = (slot >> (5 - k)) & 1;
            idx[10 + k] = E_POS_SLOT + (lps << 6) + ((1u << k) | (slot >> (6 - k)));
            use |= (match ? 1u : 0u) << (10 + k);
        }
        u32 rb = 0, rn = 0, rv = 0;
        if (match && slot >= 4) {
            const u32 nd = (slot >> 1) - 1, base = (2 | (slot & 1)) << nd, red = d - base;
            if (slot < 14) { rb = E_SPEC_POS + base - slot - 1; rn = nd; rv = red; }
            else { rb = E_ALIGN; rn = 4; rv = red & 15; extra = (nd - 4) * 16; }
        }
        u32 m = 1;
#pragma unroll
        for (u32 k = 0; k < 5; k++) {
            bit[16 + k] = (rv >> k) & 1;
            idx[16 + k] = rb + m;
            m = (m << 1) | bit[16 + k];
            use |= (k < rn ? 1u : 0u) << (16 + k);
        }
    }
    u32 pr[21];
#pragma unroll
    for (u32 j = 0; j < 21; j++) pr[j] = (use >> j) & 1 ? (u32)L.probs[idx[j]] : 1024u;
    u32 sum = extra;
#pragma unroll
    for (u32 j = 0; j < 21; j++) {
        const u32 q = L.price[(bit[j] ? 2048 - pr[j] : pr[j]) >> 4];
        sum += (use >> j) & 1 ? q : 0u;
    }
    return sum;
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
__device__ __forceinline__ u32 xo_arc_dist(const u32* __restrict__ wc, u32 src, u32 len, u32 room) {
    const u32 c0 = ufl(wc[src * XO_K]), c1 = ufl(wc[src * XO_K + 1]), c2 = ufl(wc[src * XO_K + 2]);
    auto holds = [&](u32 c) { const u32 Lk = c >> 23; return Lk && len <= (Lk < room ? Lk : room); };
    return (holds(c0) ? c0 : holds(c1) ? c1 : holds(c2) ? c2 : 0u) & 0x7FFFFFu;
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(XO_WPE))) void xo_segment(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, DType t,
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
    u64 prof[5] = {0, 0, 0, 0, 0};
    u64 prof2[6] = {0, 0, 0, 0, 0, 0};
    const u64 tk0 = XO_PROF ? __builtin_readcyclecounter() : 0;
    const u64 rt0 = XO_PROF ? __builtin_amdgcn_s_memrealtime() : 0;  // 100 MHz reference clock
    // serialised byte x (< the window end): from the tile when it is inside
    auto sbyte = [&](u64 x, u64 wbase) -> u32 {
        return x + XO_HIST >= wbase ? (u32)L.tile[x + XO_HIST - wbase] : e.sb(x);
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
                const u64 tp0 = XO_PROF ? __builtin_readcyclecounter() : 0;
                // ================= plan a window [p, we) =================
                const u64 we = (s1 - p) < XO_WIN ? s1 : p + XO_WIN;
                const u32 W = (u32)(we - p);
                wb = p;
                __syncthreads();
                for (u32 j = lane; j <= W; j += 64) L.key[j] = ~0ull;
                for (u32 j = lane; j < XO_HIST + W; j += 64)
                    if (j + p >= XO_HIST) L.tile[j] = (u8)e.sb(p + j - XO_HIST);
                const u32* __restrict__ wc = cbase + p * XO_K;  // the window's candidates (read-only)
                __syncthreads();
                if (lane == 0) L.key[0] = 0;
                __syncthreads();
                // Nodes in order, software-pipelined by one: node t's literal and
                // short-rep keys (its only arcs to t + 1) are resolved in registers,
                // so node t + 1 is final before node t's longer arcs are priced;
                // node t + 1's rep-byte loads are issued before that pricing and
                // land while it runs.
                u32 cst = state, cq0 = r0, cq1 = r1, cq2 = r2, cq3 = r3, cP = 0;
                u32 i_sym = 0, i_w0 = 0, i_w1 = 0, i_w2 = 0, i_rb = 0, i_mine = 0;
                bool i_valid = false;
                auto issue = [&](u32 t, u32 q0_, u32 q1_, u32 q2_, u32 q3_) {
                    const u64 at = p + t;
                    const u32 room = W - t, mx = room < XO_MAXLEN ? room : XO_MAXLEN;
                    const u32 r = (u32)lane >> 4, tb = (u32)lane & 15;
                    const u32 rd = r == 0 ? q0_ : r == 1 ? q1_ : r == 2 ? q2_ : q3_;
                    i_sym = L.tile[XO_HIST + t];
                    i_w0 = wc[t * XO_K];
                    i_w1 = wc[t * XO_K + 1];
                    i_w2 = wc[t * XO_K + 2];
                    i_valid = at > rd && tb < mx;
                    i_rb = i_valid ? sbyte(at - rd - 1 + tb, p) : 0u;
                    i_mine = tb < mx ? (u32)L.tile[XO_HIST + t + tb] : 0u;
                };
                // The window's flag-bit prices and plain-literal prices, read
                // per node with v_readlane (no LDS round trip): lane st*4+ps
                // holds is_match / is_rep0_long of (state, pos state), lane st
                // the is_rep / rep_g0-2 pairs, lane l the literals l + 64 k.
                // (two 16-bit prices per register: bit value 0 low, 1 high; literals l and l + 64 (+ 128))
                u32 pIM, pRL, pIR, pG0, pG1, pG2, pL01, pL23;
                {
                    const u32 sp = (u32)lane < 48 ? (u32)lane : 0u, st4 = sp >> 2, ps4 = sp & 3;
                    auto pair = [&](u32 i) { return xo_pb(L, i, 0) | (xo_pb(L, i, 1) << 16); };
                    pIM = pair(E_IS_MATCH + (st4 << 4) + ps4);
                    pRL = pair(E_IS_REP0_LONG + (st4 << 4) + ps4);
                    const u32 s1 = (u32)lane < 12 ? (u32)lane : 0u;
                    pIR = pair(E_IS_REP + s1);
                    pG0 = pair(E_IS_REP_G0 + s1);
                    pG1 = pair(E_IS_REP_G1 + s1);
                    pG2 = pair(E_IS_REP_G2 + s1);
                    auto plain = [&](u32 sym) {
                        u32 sum = 0;
#pragma unroll
                        for (u32 j = 0; j < 8; j++) sum += xo_pb(L, E_LITERAL + ((1u << j) | (sym >> (8 - j))), (sym >> (7 - j)) & 1);
                        return sum;
                    };
                    pL01 = plain((u32)lane) | (plain((u32)lane + 64) << 16);
                    pL23 = plain((u32)lane + 128) | (plain((u32)lane + 192) << 16);
                }
                // length / distance price tables of the window (lane-parallel)
                for (u32 q = lane; q < 640; q += 64) {
                    const u32 coder = q < 128 ? q >> 6 : (q - 128) >> 8, ps4 = q < 128 ? (q >> 4) & 3 : 0u,
                              l = q < 128 ? q & 15 : 16 + ((q - 128) & 255);
                    L.nr.pt.len[q] = (u16)xo_arc_price(L, coder ? E_REP_LEN : E_LEN, l, ps4, false, 0, 2);
                }
                for (u32 q = lane; q < 4 * 64; q += 64) {
                    const u32 lps = q >> 6, sl = q & 63;
                    u32 sum = 0;
#pragma unroll
                    for (u32 k = 0; k < 6; k++)
                        sum += xo_pb(L, E_POS_SLOT + (lps << 6) + ((1u << k) | (sl >> (6 - k))), (sl >> (5 - k)) & 1);
                    L.nr.pt.slot[lps][sl] = (u16)sum;
                }
                for (u32 q = lane; q < 128 + 16; q += 64) {
                    u32 sum = 0, m = 1;
                    if (q < 128) {
                        if (q >= 4) {
                            const u32 sl = slot_of(q), nd = (sl >> 1) - 1, base = (2 | (sl & 1)) << nd, red = q - base;
                            for (u32 k = 0; k < nd; k++) {
                                const u32 b = (red >> k) & 1;
                                sum += xo_pb(L, E_SPEC_POS + base - sl - 1 + m, b);
                                m = (m << 1) | b;
                            }
                        }
                        L.nr.pt.spec[q] = (u16)sum;
                    } else {
                        const u32 a = q - 128;
                        for (u32 k = 0; k < 4; k++) {
                            const u32 b = (a >> k) & 1;
                            sum += xo_pb(L, E_ALIGN + m, b);
                            m = (m << 1) | b;
                        }
                        L.nr.pt.align[a] = (u16)sum;
                    }
                }
                __syncthreads();
                // Each node's state and reps live in registers: node i in lane
                // i & 63 of row i >> 6 (nodes 0..255 are the arcs' sources).
                u32 nS[4] = {0, 0, 0, 0}, nR0[4] = {0, 0, 0, 0}, nR1[4] = {0, 0, 0, 0}, nR2[4] = {0, 0, 0, 0},
                    nR3[4] = {0, 0, 0, 0};
                auto node_put = [&](u32 i, u32 st_, u32 a0, u32 a1, u32 a2, u32 a3) {
                    const u32 row = i >> 6;
                    const int ln = (int)(i & 63);
#pragma unroll
                    for (u32 rr = 0; rr < 4; rr++) {
                        if (rr != row) continue;
                        const bool me = lane == ln;
                        nS[rr] = me ? st_ : nS[rr];
                        nR0[rr] = me ? a0 : nR0[rr];
                        nR1[rr] = me ? a1 : nR1[rr];
                        nR2[rr] = me ? a2 : nR2[rr];
                        nR3[rr] = me ? a3 : nR3[rr];
                    }
                };
                auto node_get = [&](u32 i, u32& st_, u32& a0, u32& a1, u32& a2, u32& a3) {
                    const u32 row = i >> 6;
                    const int ln = (int)(i & 63);
                    const u32 vS = row == 0 ? nS[0] : row == 1 ? nS[1] : row == 2 ? nS[2] : nS[3];
                    const u32 v0 = row == 0 ? nR0[0] : row == 1 ? nR0[1] : row == 2 ? nR0[2] : nR0[3];
                    const u32 v1 = row == 0 ? nR1[0] : row == 1 ? nR1[1] : row == 2 ? nR1[2] : nR1[3];
                    const u32 v2 = row == 0 ? nR2[0] : row == 1 ? nR2[1] : row == 2 ? nR2[2] : nR2[3];
                    const u32 v3 = row == 0 ? nR3[0] : row == 1 ? nR3[1] : row == 2 ? nR3[2] : nR3[3];
                    st_ = (u32)__builtin_amdgcn_readlane((int)vS, ln);
                    a0 = (u32)__builtin_amdgcn_readlane((int)v0, ln);
                    a1 = (u32)__builtin_amdgcn_readlane((int)v1, ln);
                    a2 = (u32)__builtin_amdgcn_readlane((int)v2, ln);
                    a3 = (u32)__builtin_amdgcn_readlane((int)v3, ln);
                };
                node_put(0, state, r0, r1, r2, r3);
                issue(0, cq0, cq1, cq2, cq3);
                for (u32 t = 0; t < W; t++) {
                    u64 tq = XO_PROF >= 2 ? __builtin_readcyclecounter() : 0;
                    auto stamp = [&](int slot) {
                        if (XO_PROF >= 2) {
                            const u64 t2 = __builtin_readcyclecounter();
                            prof2[slot] += t2 - tq;
                            tq = t2;
                        }
                    };
                    const u64 at = p + t;
                    const u32 ps = (u32)at & 3;
                    const u32 room = W - t, mx = room < XO_MAXLEN ? room : XO_MAXLEN;
                    const u32 st = cst, q0 = cq0, q1 = cq1, q2 = cq2, q3 = cq3, P = cP;
                    // ---- node t: rep lengths (lane = rep * 16 + byte), first round issued ----
                    const u32 sym = ufl(i_sym);
                    const u32 wk[XO_K] = {ufl(i_w0), ufl(i_w1), ufl(i_w2)};
                    u32 rl0 = 0, rl1 = 0, rl2 = 0, rl3 = 0, open = 0xF;
                    {
                        const u32 r = (u32)lane >> 4, tb = (u32)lane & 15;
                        const u32 rd = r == 0 ? q0 : r == 1 ? q1 : r == 2 ? q2 : q3;
                        bool ok = i_valid && i_mine == i_rb;
                        for (u32 base = 0; open; base += 16) {
                            if (base) {
                                const u32 o = base + tb;
                                ok = false;
                                if (((open >> r) & 1) && at > rd && o < mx)
                                    ok = L.tile[XO_HIST + t + o] == sbyte(at - rd - 1 + o, p);
                            }
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
                    const u32 mbyte = at > q0 ? (u32)__builtin_amdgcn_readlane((int)i_rb, 0) : 0u;
                    stamp(1);
                    // ---- node t: literal price (matched literals: lanes 0-7) and flag prices ----
                    u32 litp;
                    if (st < 7) {
                        const u32 hi = sym >> 6, lo = sym & 63;
                        const u32 v = (u32)__builtin_amdgcn_readlane((int)(hi < 2 ? pL01 : pL23), (int)lo);
                        litp = (hi & 1) ? v >> 16 : v & 0xFFFFu;
                    } else {
                        u32 pv = 0;
                        if (lane < 8) {
                            const u32 j = (u32)lane, b = (sym >> (7 - j)) & 1, m = (1u << j) | (sym >> (8 - j));
                            const u32 off = (sym >> (8 - j)) == (mbyte >> (8 - j)) ? 0x100u : 0u;
                            const u32 mbit = off ? ((mbyte >> (7 - j)) & 1) << 8 : 0u;
                            pv = xo_pb(L, E_LITERAL + m + off + mbit, b);
                        }
                        litp = 0;
                        for (int j = 0; j < 8; j++) litp += (u32)__builtin_amdgcn_readlane((int)pv, j);
                    }
                    const int sps = (int)(st * 4 + ps), sst = (int)st;
                    const u32 fIM = (u32)__builtin_amdgcn_readlane((int)pIM, sps), fIR = (u32)__builtin_amdgcn_readlane((int)pIR, sst),
                              fG0 = (u32)__builtin_amdgcn_readlane((int)pG0, sst), fG1 = (u32)__builtin_amdgcn_readlane((int)pG1, sst),
                              fG2 = (u32)__builtin_amdgcn_readlane((int)pG2, sst), fRL = (u32)__builtin_amdgcn_readlane((int)pRL, sps);
                    const u32 f[12] = {fIM & 0xFFFFu, fIM >> 16, fIR & 0xFFFFu, fIR >> 16, fG0 & 0xFFFFu, fG0 >> 16,
                                       fG1 & 0xFFFFu, fG1 >> 16, fG2 & 0xFFFFu, fG2 >> 16, fRL & 0xFFFFu, fRL >> 16};
                    stamp(2);
                    // ---- node t + 1: final key (min with node t's literal / short rep), state, reps ----
                    const bool sr = at > q0 && sym == mbyte;
                    const u32 rbase = P + f[1] + f[3];
                    {
                        const u64 kl = ((u64)(P + f[0] + litp) << 20) | ((u64)t << 11);
                        const u64 ks = sr ? ((u64)(rbase + f[4] + f[10]) << 20) | ((u64)t << 11) | 1u : ~0ull;
                        u64 nk = L.key[t + 1];
                        nk = ((u64)ufl((u32)(nk >> 32)) << 32) | ufl((u32)nk);
                        nk = nk < kl ? nk : kl;
                        nk = nk < ks ? nk : ks;
                        wsync_lds();
                        if (lane == 0) L.key[t + 1] = nk;
                        cP = (u32)(nk >> 20);
                        if (t + 1 < W) {
                            const u32 alo = (u32)nk, src = (alo >> 11) & 511, arc = alo & 2047;
                            u32 bst, b0, b1, b2, b3;
                            if (src == t) {
                                bst = st; b0 = q0; b1 = q1; b2 = q2; b3 = q3;
                            } else {
                                node_get(src, bst, b0, b1, b2, b3);
                            }
                            if (arc == 0) { cst = st_lit(bst); cq0 = b0; cq1 = b1; cq2 = b2; cq3 = b3; }
                            else if (arc == 1) { cst = st_short(bst); cq0 = b0; cq1 = b1; cq2 = b2; cq3 = b3; }
                            else if (arc < ARC_MATCH) {
                                const u32 r = (arc - ARC_REP) / 274;
                                cst = st_rep(bst);
                                cq0 = r == 0 ? b0 : r == 1 ? b1 : r == 2 ? b2 : b3;
                                cq1 = r == 0 ? b1 : b0;
                                cq2 = r <= 1 ? b2 : b1;
                                cq3 = r <= 2 ? b3 : b2;
                            } else {
                                cst = st_match(bst);
                                cq0 = ufl(xo_arc_dist(wc, src, arc - ARC_MATCH, W - src));
                                cq1 = b0; cq2 = b1; cq3 = b2;
                            }
                            node_put(t + 1, cst, cq0, cq1, cq2, cq3);
                            issue(t + 1, cq0, cq1, cq2, cq3);
                        }
                    }
                    stamp(0);
                    // ---- node t: rep and candidate arcs (lengths >= 2, targets >= t + 2) ----
                    // Lanes 16 r .. 16 r + 15 price rep r's kept lengths (at most 10),
                    // then lanes 16 c .. 16 c + 15 candidate c's (c < 3); every
                    // lane's group is fixed, so no lane searches for its arc.
                    const u32 gl = (u32)lane >> 4, el = (u32)lane & 15;
                    {
                        const u32 rlg = gl == 0 ? rl0 : gl == 1 ? rl1 : gl == 2 ? rl2 : rl3;
                        const u32 rbg = rbase + (gl == 0 ? f[4] + f[11] : gl == 1 ? f[5] + f[6] : f[5] + f[7] + (gl == 2 ? f[8] : f[9]));
                        u32 c1, h;
                        const u32 cn = rlg >= 2 ? xo_range_count(2, rlg, &c1, &h) : 0u;
                        if (el < cn) {
                            const u32 len = el < c1 ? 2 + el : h + (el - c1);
                            const u32 price = rbg + L.nr.pt.len[xo_lenix(1, ps, len - 2)];
                            const u64 key = ((u64)price << 20) | ((u64)t << 11) | (ARC_REP + gl * 274 + len);
                            atomicMin((unsigned long long*)&L.key[t + len], (unsigned long long)key);
                        }
                    }
                    stamp(3);
                    {
                        // candidate c's lengths start past the longer ones before it
                        u32 a0[XO_K], lr[XO_K], lprev = 1;
#pragma unroll
                        for (u32 c = 0; c < XO_K; c++) {
                            const u32 Lk = wk[c] >> 23;
                            lr[c] = Lk < mx ? Lk : mx;
                            a0[c] = lprev + 1 > 2 ? lprev + 1 : 2;
                            if (Lk && lr[c] > lprev) lprev = lr[c];
                        }
                        const u32 wg = gl == 0 ? wk[0] : gl == 1 ? wk[1] : wk[2];
                        const u32 ag = gl == 0 ? a0[0] : gl == 1 ? a0[1] : a0[2];
                        const u32 lg = gl == 0 ? lr[0] : gl == 1 ? lr[1] : lr[2];
                        u32 c1, h;
                        const u32 cn = gl < XO_K && (wg >> 23) ? xo_range_count(ag, lg, &c1, &h) : 0u;
                        if (el < cn) {
                            const u32 len = el < c1 ? ag + el : h + (el - c1);
                            const u32 d = wg & 0x7FFFFFu, lps = len - 2 < 3 ? len - 2 : 3, sl = slot_of(d);
                            u32 dp = L.nr.pt.slot[lps][sl];
                            if (sl >= 14) dp += (((sl >> 1) - 1) - 4) * 16 + L.nr.pt.align[d & 15];
                            else if (sl >= 4) dp += L.nr.pt.spec[d];
                            const u32 price = P + f[1] + f[2] + L.nr.pt.len[xo_lenix(0, ps, len - 2)] + dp;
                            const u64 key = ((u64)price << 20) | ((u64)t << 11) | (ARC_MATCH + len);
                            atomicMin((unsigned long long*)&L.key[t + len], (unsigned long long)key);
                        }
                    }
                    wsync_lds();
                    stamp(4);
                }
                // ---- the path to the window end (reversed) ----
                {
                    u32 j = W, np = 0;
                    while (j > 0) {
                        const u64 a = L.key[j];
                        const u32 alo = ufl((u32)a);
                        const u32 src = (alo >> 11) & 511, arc = alo & 2047, len = j - src;
                        const u32 d = arc >= ARC_MATCH ? xo_arc_dist(wc, src, len, W - src) : 0u;
                        if (lane == 0) {
                            L.nr.path.pth[np] = arc | (len << 11);
                            L.nr.path.pdist[np] = d;
                        }
                        np++;
                        j = src;
                    }
                    npath = np;
                    __syncthreads();
                }
                if (XO_PROF) {
                    prof[0] += __builtin_readcyclecounter() - tp0;
                    prof[2] += W;
                    prof[4] += 1;
                }
            }
            if (XO_PROF) prof[3] += 1;
            // ---- code the next symbol of the path ----
            npath--;
            const u32 w = ufl(L.nr.path.pth[npath]);
            const u32 arc = w & 2047, len = w >> 11, ps = (u32)p & 3;
            if (arc == 0) {
                const u32 sym = L.tile[XO_HIST + p - wb];
                const bool matched = state >= 7;
                const u32 mb = matched && p > r0 ? ufl(sbyte(p - r0 - 1, wb)) : 0u;
                u32 idx[9], bits[9];
                idx[0] = E_IS_MATCH + (state << 4) + ps;
                bits[0] = 0;
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    bits[1 + j] = (sym >> (7 - j)) & 1;
                    u32 x = E_LITERAL + ((1u << j) | (sym >> (8 - j)));
                    if (matched) {
                        const u32 off = (sym >> (8 - j)) == (mb >> (8 - j)) ? 0x100u : 0u;
                        x += off + (off ? ((mb >> (7 - j)) & 1) << 8 : 0u);
                    }
                    idx[1 + j] = x;
                }
                xo_code_m<9>(e, idx, bits, 0x1FFu);
                state = st_lit(state);
            } else if (arc == 1) {
                const u32 idx[4] = {E_IS_MATCH + (state << 4) + ps, E_IS_REP + state, E_IS_REP_G0 + state,
                                    E_IS_REP0_LONG + (state << 4) + ps};
                const u32 bits[4] = {1, 1, 0, 0};
                xo_code_m<4>(e, idx, bits, 0xFu);
                state = st_short(state);
            } else if (arc < ARC_MATCH) {
                const u32 r = (arc - ARC_REP) / 274;
                // slots: is_match, is_rep, rep_g0, rep0_long (r = 0), rep_g1, rep_g2 (r >= 2), length
                u32 idx[16], bits[16], use = 0x7u;
                idx[0] = E_IS_MATCH + (state << 4) + ps; bits[0] = 1;
                idx[1] = E_IS_REP + state; bits[1] = 1;
                idx[2] = E_IS_REP_G0 + state; bits[2] = r != 0;
                idx[3] = E_IS_REP0_LONG + (state << 4) + ps; bits[3] = 1; use |= (r == 0 ? 1u : 0u) << 3;
                idx[4] = E_IS_REP_G1 + state; bits[4] = r >= 2; use |= (r >= 1 ? 1u : 0u) << 4;
                idx[5] = E_IS_REP_G2 + state; bits[5] = r >= 3; use |= (r >= 2 ? 1u : 0u) << 5;
                xo_len_slots<16>(idx, bits, use, 6, E_REP_LEN, len - 2, ps);
                xo_code_m<16>(e, idx, bits, use);
                if (r != 0) {
                    const u32 d = r == 1 ? r1 : r == 2 ? r2 : r3;
                    if (r == 3) r3 = r2;
                    if (r >= 2) r2 = r1;
                    r1 = r0;
                    r0 = d;
                }
                state = st_rep(state);
            } else {
                const u32 d = ufl(L.nr.path.pdist[npath]);
                // slots: is_match, is_rep, length, position slot; then the slot's low bits
                const u32 lps = len - 2 < 3 ? len - 2 : 3, slot = slot_of(d);
                u32 idx[18], bits[18], use = 0x3u;
                idx[0] = E_IS_MATCH + (state << 4) + ps; bits[0] = 1;
                idx[1] = E_IS_REP + state; bits[1] = 0;
                xo_len_slots<18>(idx, bits, use, 2, E_LEN, len - 2, ps);
#pragma unroll
                for (u32 k = 0; k < 6; k++) {
                    bits[12 + k] = (slot >> (5 - k)) & 1;
                    idx[12 + k] = E_POS_SLOT + (lps << 6) + ((1u << k) | (slot >> (6 - k)));
                }
                use |= 0x3Fu << 12;
                xo_code_m<18>(e, idx, bits, use);
                if (slot >= 4) {
                    const u32 nd = (slot >> 1) - 1, base = (2 | (slot & 1)) << nd, red = d - base;
                    if (slot < 14) {
                        xo_rtree<5>(e, E_SPEC_POS + base - slot - 1, nd, red);
                    } else {
                        e.direct(red >> 4, nd - 4);
                        xo_rtree<4>(e, E_ALIGN, 4, red & 15);
                    }
                }
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
    if (XO_PROF && lane == 0) {
        const u64 tot = __builtin_readcyclecounter() - tk0;
        atomicAdd(&g_xo_prof[0], (unsigned long long)prof[0]);
        atomicAdd(&g_xo_prof[1], (unsigned long long)(tot - prof[0]));
        atomicAdd(&g_xo_prof[2], (unsigned long long)prof[2]);
        atomicAdd(&g_xo_prof[3], (unsigned long long)prof[3]);
        atomicAdd(&g_xo_prof[4], (unsigned long long)prof[4]);
        atomicAdd(&g_xo_prof[5], (unsigned long long)tot);
        for (int q = 0; q < 5; q++) atomicAdd(&g_xo_prof[8 + q], (unsigned long long)prof2[q]);
        const u64 rt1 = __builtin_amdgcn_s_memrealtime();
        atomicAdd(&g_xo_prof[6], (unsigned long long)(rt1 - rt0));
        atomicMax(&g_xo_prof[7], (unsigned long long)(rt1 - rt0));   // longest wave
        atomicMax(&g_xo_prof[13], (unsigned long long)rt0);          // last wave start
        atomicMax(&g_xo_prof[14], (unsigned long long)~rt0);         // ~first wave start
        atomicMax(&g_xo_prof[15], (unsigned long long)rt1);          // last wave end
    }
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

extern "C" int zcg__debug_xz_opt_counters(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_xo_prof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_xo_prof), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}

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

const char* cfg_xz_opt() {
    return "xz_opt:SEG_KB=" ZCG_STR(XO_SEG_KB) ",WPE=" ZCG_STR(XO_WPE) ",PROF=" ZCG_STR(XO_PROF);
}

}  // namespace zcg
