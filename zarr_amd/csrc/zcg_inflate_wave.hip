// zcg_inflate_wave.hip — gzip chunk decode with ONE WAVE PER CHUNK on gfx950
// (GzipCompression decode, src/compression/gzip.rs:49-52 -> flate2 -> zlib).
//
// A deflate block body is one serial Huffman bit stream; its symbols come in
// tokens (literal, or length/distance match), 16 383 per block for zlib's
// default memLevel (a C2 chunk has 17 blocks of ~195 Kbit, ~60 KB output).
// The wave owns the chunk and works block by block:
//
//  H (Huffman) round: the block body is cut into 64 COARSE segments, one per
//    lane (~3 Kbit, ~250 tokens each, sized from the previous block).  Each
//    lane decodes its own segment from its first bit as if a token started
//    there, appending its tokens to a private list in the HBM workspace and
//    marking token starts inside the first IW_MW bits of its segment (LDS).
//    A misaligned Huffman decoder falls into step with the true one within a
//    few tokens (median 64 bits, p99 ~450 bits on zlib-6 data), so when a
//    lane runs past its segment end it soon lands on a token start the next
//    lane marked: from there that lane's list is the true path.  Lane 0 starts
//    at the true position; the chain of sync points gives every lane the
//    first valid token of its list.  Segments are long, so the resync tail
//    costs ~15 % of the decode instead of the ~60 % that 256-bit segments cost.
//    A lane that hits an invalid code or an end-of-block in its own segment
//    records it and keeps decoding after it (the record is real only if the
//    lane's valid range reaches it), so a garbage path never ends a segment
//    early.
//  L (LZ77) phase: the valid tokens, in stream order, are resolved up to IW_S
//    output bytes at a time in an LDS ring of 16-bit entries, TOKEN by token:
//    a literal writes its byte; a far match (its whole source before the
//    stage) is copied from the chunk's committed output by 16-byte pieces, one
//    far token per lane after a ballot compaction; a near match writes one
//    pointer per byte, and the near bytes are resolved in ordered batches of
//    64 by pointer jumping.  One coalesced 16-B store pass per stage commits
//    the ring with the byte-order transform fused.
//
// Everything is wave-synchronous: no s_barrier between phases, and the other
// chunks' waves on the SIMD fill the dependent-LDS latency.  Block headers,
// stored blocks and zlib's post-N look-ahead use the wave-uniform reader of
// zcg_inflate_common.h.  Results are bit-identical to the serial kernel
// (zcg_inflate.hip) and the 256-lane round kernel (zcg_inflate_par.hip);
// tests/ compare all three against the oracle.
#include <climits>
#include <type_traits>

#include "zcg_inflate_common.h"

// A/B knobs: stage entries, tokens per lane list, waves per SIMD the register
// budget targets, far-byte loads in flight per lane
#ifndef ZIW_S
#define ZIW_S 2048
#endif
#ifndef ZIW_TCAP
#define ZIW_TCAP 768
#endif
#ifndef ZIW_WPE
#define ZIW_WPE 4
#endif
#ifndef ZIW_EST_PCT
#define ZIW_EST_PCT 108
#endif
#ifndef ZIW_DBG
#define ZIW_DBG 0  // 1: debug counters compiled in (ZCG_FLAG_DEBUG_COUNTERS; tools/iw_stats.py cycle
                   // shares).  Out by default: their checks cost 1.4 % of the C2 launch (22.05 -> 21.74 ms)
#endif

namespace zcg {

constexpr u32 IW_S = ZIW_S;            // stage ring entries: 64 lane blocks of IW_BLK
constexpr u32 IW_BLK = IW_S / 64;
constexpr u32 IW_TCAP = ZIW_TCAP;
constexpr u32 IW_GK = 3;       // token groups in flight in the L phase (named slots)  // far-byte loads in flight per lane (gather)
constexpr u32 IW_SEGMIN = 128;   // bits per lane segment
constexpr u32 IW_SEGMAX = 4096;
constexpr u32 IW_K = 4;          // decode steps between staged-token / mark flushes
constexpr u32 IW_KH = 2;         // flush periods per outer step (reader loads at its top, absorbs at its bottom)
#ifndef ZIW_G
#define ZIW_G 4
#endif

constexpr u32 IW_G = ZIW_G;                      // lanes whose lists are interleaved by 16-byte blocks
constexpr u32 IW_TSTR = IW_TCAP + 2 * IW_K;      // token list stride (a flush writes up to two aligned blocks)
static_assert(IW_TSTR % 4 == 0 && 64 % IW_G == 0, "list blocks");
// word offset of token j of lane l's list: lists of IW_G consecutive lanes
// are interleaved by aligned 4-word blocks, so one flush of those lanes fills
// whole cache lines ([lane / G][j / 4][lane % G][j % 4]; G = 1: [lane][j])
__device__ __forceinline__ u32 iw_ta(u32 l, u32 j) {
    // (< 2^24 operands: the full-rate 24-bit multiply, not the quarter-rate 32-bit one)
    return __umul24(l / IW_G, IW_G * IW_TSTR) + (((j >> 2) * IW_G + (l % IW_G)) << 2) + (j & 3);
}
constexpr u32 IW_MWIN = 8;                       // mark words a lane keeps in LDS between flushes
constexpr u32 IW_EMW = 2;                        // a segment's first mark words kept in LDS for pass 2
#ifndef ZIW_MARKW
#define ZIW_MARKW 32
#endif
constexpr u32 IW_MARKW = ZIW_MARKW;  // bitmap words kept per segment (the rest is never read)
constexpr u32 IW_MWORDS = IW_MARKW + IW_MWIN;  // mark words per segment (bitmap, u32; the last window may spill past IW_MARKW)
static_assert(IW_MARKW + IW_MWIN <= IW_MWORDS, "mark window inside the bitmap");
constexpr u32 IW_EST0 = 64 * 3072;  // first block's body estimate (zlib-6 blocks: ~195 Kbit)
static_assert(IW_S == 2048 && IW_BLK == 32, "the L phase keeps one 32-entry block per lane in registers");

// token word (same layout as zcg_inflate_par.hip, plus bit lengths on markers):
//   literal  = bits << 24 | byte
//   match    = 1 << 31 | bits << 24 | (len - 3) << 16 | (dist - 1)
//   marker   = 1 << 30 | bits << 24 | code   (EOB / invalid code / input exhausted)
// bits = the token's stream bits (<= 48), so a token's start is the lane's
// segment start plus the bits of the tokens before it in the lane's list.
constexpr u32 W_MATCH = 0x80000000u;
constexpr u32 W_MARK = 0x40000000u;
enum : u32 { M_EOB = 0, M_BAD = 1, M_EXH = 2, M_END = 3 /* synthetic: no more tokens in the round */ };
__device__ __forceinline__ bool w_marker(u32 t) { return (t & 0xC0000000u) == W_MARK; }
__device__ __forceinline__ u32 w_bits(u32 t) { return (t >> 24) & 63; }
__device__ __forceinline__ u32 w_len(u32 t) { return (t & W_MATCH) ? ((t >> 16) & 0xFF) + 3 : (w_marker(t) ? 0u : 1u); }

// lane stop codes (>= 64)
constexpr u32 S_NONE = 0xFFFFFFFFu;
constexpr u32 S_ROUND_END = 64;  // reached the end of the round's range
constexpr u32 S_MARKER = 65;     // pass 2 ended on a marker (last token of the list)
constexpr u32 S_CAP = 66;        // token list full

// stage entries (u16): IE_VAL|byte = a final byte; a value below IW_S = the
// ring index of an earlier byte of the stage (a near byte not yet resolved)
constexpr u32 IE_VAL = 0xFF00u;
static_assert(IW_S <= IE_VAL, "stage entry encoding");

// Table geometry: a 9-bit literal/length root (zlib's ENOUGH_LENS = 852
// entries covers every complete code) and an 8-bit distance root, so the LDS
// footprint allows 16 chunks per CU.
constexpr int W_LB = 9;
constexpr u32 W_LCAP = 852;
constexpr int W_DB = 8;
constexpr u32 W_DCAP = 432;  // >= enough(30, 8, 15) = 402

constexpr u32 IW_NDBG = 28;
__device__ unsigned long long g_iw_dbg[32];
enum { IWD_ROUNDS, IWD_BLOCKS, IWD_STAGES, IWD_GROUPS, IWD_P1_IT, IWD_P2_IT, IWD_CHAIN, IWD_SPARE7, IWD_CAPS,
       IWD_NOEOB, IWT_HDR, IWT_P1, IWT_P2, IWT_CHAIN, IWT_CLASSIFY, IWT_FAR, IWT_NEAR, IWT_PLACE,
       IWT_COMMIT, IWT_TOTAL, IWD_FARIT, IWD_NBATCH, IWD_NPASS, IWD_NSTRAD, IWT_HTAB, IWT_REFETCH, IWT_EOB, IWT_HWALK };
static_assert(IWT_HWALK < IW_NDBG, "debug slots");

struct IwLds {
    u32 ltab[W_LCAP];
    u32 dtab[W_DCAP];
    union {
        struct {  // block headers and the look-ahead (wave-uniform reader)
            HuffLds lh, dh;
            u8 lens[320];
            u32 bcache[BI_CACHE_WORDS];
            u32 hwin[130];  // 512 stream bytes from the code-length codes on (dynamic header)
        } h;
        struct Hr {    // H round: marked extent (bits) of each segment, staged tokens, mark windows
            u32 mlim[64];
            u32 tst[2 * IW_K][64];  // ring of two aligned list blocks (slot = token index % 8)
            u32 mwin[IW_MWIN][64];
            u32 em[IW_EMW][64];     // each segment's first IW_EMW mark words (pass 2 reads them here)
        } hr;
        struct {       // L phase: the stage ring, near-token descriptors and batch markers
            u16 ptr[IW_S];
            u64 fd[64];  // far parts of the group by rank: source byte | (ring entry | length << 16) << 32
            // near batch: slot << 26 | part descriptor at the slot of each
            // part's first byte in the batch, 0 elsewhere (cleared per batch)
            u32 mk[64];
        } st;
    } u;
    u32 dbgc[IW_NDBG];
};
static_assert(sizeof(IwLds) + 32 <= 10240, "16 chunks per CU");

// wave-local ordering point for LDS (and the compiler): a wave's LDS
// operations are performed in issue order, so a fence at wavefront scope is
// enough to publish one lane's LDS writes to the other lanes
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ u32 iw_incl_scan(u32 v) {
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    // rows -> wave: lane 15 into rows 1 and 3, then lane 31 into rows 2 and 3
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

__device__ __forceinline__ u32 iw_wave_sum(u32 v) {
    const u32 x = iw_incl_scan(v);
    return (u32)__builtin_amdgcn_readlane((int)x, 63);
}

// ---- per-lane bit reader straight from HBM, refilled at wave-uniform points ----------
// The stream is read as aligned 16-byte vectors from base = ds & ~15 (an
// aligned vector holding any stream byte is readable; bytes outside the
// stream are don't-care: a token that needs bits past the end becomes the
// input-exhausted marker, and an index past the stream re-reads the last
// vector).  A 96-bit window (lo:hi) holds the next nb bits; words are
// appended from the two resident vectors A:B (8 words).
// Loads are issued only at wave-uniform points: every lane loads the two
// vectors after B at the top of an outer step (IW_K2 decode steps) and
// absorbs them at its bottom (gr_absorb), so no load is in flight across a
// loop back edge.  The memory counters are per wave, not per lane: a load
// issued in a divergent step (when one lane's vector runs out) is waited for
// by the whole wave as soon as any lane touches that register, i.e. at about
// every step; a loop-carried register in flight is copied at the loop header,
// which waits as well; and a flat (generic) load would also hold every LDS
// table lookup.
// Round 5: a bit cursor bp into the 256 bits of A:B instead of a shifted
// window.  Each step selects the three words from bp >> 5 by a 3-level
// barrel select (11 selects) and funnel-shifts them (2 v_alignbit), so a
// step costs no word appends and no 64-bit shifts; dropping bits is one add.
// Same run-dry rule as the window reader: a lane decodes while >= 48 bits of
// A:B are left (bp <= 208).
struct GRd {
    u32x4 A, B;
    u32 bp;  // bit cursor into A:B (0..256)
    u32 vc;  // vector index after B
    u64 lo;  // 64 stream bits from bp (>= 48 valid), set by gr_fill
};

typedef __attribute__((address_space(1))) u32x4 gu32x4;
__device__ __forceinline__ u32x4 gr_vec(const u8* base, u32 nvec, u32 v) {
    const u32 vc = v < nvec ? v : (nvec ? nvec - 1 : 0u);
    return *(const gu32x4*)((const gu8*)base + 16ull * vc);
}

__device__ __forceinline__ bool gr_fill(GRd& s) {
    const u32 bp = s.bp;
    if (bp > 208) return false;
    const bool b4 = (bp & 128) != 0, b2 = (bp & 64) != 0, b1 = (bp & 32) != 0;
    // word i = bp >> 5 <= 6 of R = A:B: T[k] = R[k + 4 b4], U[k] = T[k + 2 b2],
    // W[k] = U[k + b1]; R[8] (needed only as W2 at i = 6) is don't-care
    const u32 t0 = b4 ? s.B.x : s.A.x, t1 = b4 ? s.B.y : s.A.y, t2 = b4 ? s.B.z : s.A.z,
              t3 = b4 ? s.B.w : s.A.w, t4 = s.B.x, t5 = s.B.y;
    const u32 u0 = b2 ? t2 : t0, u1 = b2 ? t3 : t1, u2 = b2 ? t4 : t2, u3 = b2 ? t5 : t3;
    const u32 w0 = b1 ? u1 : u0, w1 = b1 ? u2 : u1, w2 = b1 ? u3 : u2;
    const u32 lo = __builtin_amdgcn_alignbit(w1, w0, bp & 31);
    const u32 hi = __builtin_amdgcn_alignbit(w2, w1, bp & 31);
    s.lo = ((u64)hi << 32) | lo;
    return true;
}

__device__ __forceinline__ void gr_drop(GRd& s, u32 k) { s.bp += k; }

__device__ __forceinline__ void gr_absorb(GRd& s, const u32x4& C, const u32x4& D) {
    const u32 sh = s.bp >= 256 ? 2u : s.bp >= 128 ? 1u : 0u;
    s.A = sh == 2 ? C : sh == 1 ? s.B : s.A;
    s.B = sh == 2 ? D : sh == 1 ? C : s.B;
    s.vc += sh;
    s.bp -= 128 * sh;
}

__device__ __forceinline__ void gr_init(GRd& s, const u8* base, u32 nvec, u32 qa) {
    const u32 v0 = qa >> 7;
    s.A = gr_vec(base, nvec, v0);
    s.B = gr_vec(base, nvec, v0 + 1);
    s.vc = v0 + 2;
    s.bp = qa & 127;
    s.lo = 0;
}

// Decode one token from >= 48 valid bits: both table lookups always run, so
// lanes holding different token kinds do not serialise.
__device__ __forceinline__ u32 iw_decode(const IwLds& L, u64 v, u32* adv) {
    u32 e = L.ltab[(u32)v & ((1u << W_LB) - 1)];
    if (((e >> 24) & 15) == K_SUB)
        e = L.ltab[(e & 0xFFFF) + (((u32)v >> W_LB) & ((1u << ((e >> 16) & 0xFF)) - 1))];
    const u32 l = e >> 28, kind = (e >> 24) & 15, ex = (e >> 16) & 0xFF;
    const u32 t = l + ex;
    // 32-bit fields only: the length code and its extra bits end by bit 20,
    // and the distance code and its extra bits take <= 28 bits from t
    const u32 vd = __builtin_amdgcn_alignbit((u32)(v >> 32), (u32)v, t);
    u32 de = L.dtab[vd & ((1u << W_DB) - 1)];
    if (((de >> 24) & 15) == K_SUB)
        de = L.dtab[(de & 0xFFFF) + ((vd >> W_DB) & ((1u << ((de >> 16) & 0xFF)) - 1))];
    const u32 dl = de >> 28, dex = (de >> 16) & 0xFF;
    const u32 len = (e & 0xFFFF) + (((u32)v >> l) & ((1u << ex) - 1));
    const u32 dist = (de & 0xFFFF) + ((vd >> dl) & ((1u << dex) - 1));
    const u32 madv = t + dl + dex;
    const bool dok = ((de >> 24) & 15) == K_DIST;
    u32 a = l ? l : 1;
    u32 tk = W_MARK | (a << 24) | M_BAD;
    if (kind == K_LIT) tk = (l << 24) | (e & 0xFF);
    if (kind == K_EOB) tk = W_MARK | (l << 24) | M_EOB;
    if (kind == K_LEN) {
        a = dok ? madv : t + (dl ? dl : 1);
        tk = dok ? (W_MATCH | (madv << 24) | ((len - 3) << 16) | (dist - 1)) : (W_MARK | (a << 24) | M_BAD);
    }
    *adv = a;
    return tk;
}

typedef __attribute__((address_space(1))) u32x4 gu32x4_a4 __attribute__((aligned(4)));
typedef __attribute__((address_space(1))) u32x4 gu32x4_a16 __attribute__((aligned(16)));
typedef __attribute__((address_space(1))) u64 gu64_ua __attribute__((aligned(1)));
// LDS stores at 2-byte alignment (gfx950 DS accepts unaligned addresses:
// tools/probe/lds_unaligned.hip)
typedef u32x4 u32x4_l2 __attribute__((aligned(2)));
typedef u32 __attribute__((ext_vector_type(2))) u32x2_l2 __attribute__((aligned(2)));
typedef u32 u32_l2 __attribute__((aligned(2)));
// n (1..8) stage entries e0..e7 (two per word) stored exactly at pe
__device__ __forceinline__ void iw_put(u16* pe, u32 n, u32 x, u32 y, u32 z, u32 w) {
    if (n >= 8) {
        *(u32x4_l2*)pe = u32x4{x, y, z, w};
        return;
    }
    if (n & 4u) *(u32x2_l2*)pe = u32x2{x, y};
    const u32 a = (n & 4u) ? z : x, b = (n & 4u) ? w : y;
    u16* pt = pe + (n & 4u);
    if (n & 2u) *(u32_l2*)pt = a;
    if (n & 1u) pt[n & 2u] = (u16)((n & 2u) ? b : a);
}
// two source bytes (0-1 / 2-3 of w) as two final stage entries
__device__ __forceinline__ u32 ie_lo(u32 w) { return __builtin_amdgcn_perm(0xFFFFFFFFu, w, 0x04010400u); }
__device__ __forceinline__ u32 ie_hi(u32 w) { return __builtin_amdgcn_perm(0xFFFFFFFFu, w, 0x04030402u); }

// tokens of a lane's list that start before word wi of its bitmap, plus the
// marks in `part` (the bits of word wi below the position)
__device__ __forceinline__ u32 iw_rank(const IwLds& L, u32 ks, const gu32* mw, u32 wi, u32 part) {
    u32 c = __popc(part);
#pragma unroll 8
    for (u32 w = 0; w < wi; w++) c += __popc(w < IW_EMW ? L.u.hr.em[w][ks] : mw[w]);
    return c;
}

// stream bit of token j of the list of `lm` (segment start + bits before it)
__device__ __forceinline__ u32 iw_pos(const gu32* gl, u32 lm, u32 j, u32 seg0) {
    const u32 lane = (u32)lane_id();
    u32 s = 0;
    for (u32 x = lane; x < j; x += 64) s += w_bits(gl[iw_ta(lm, x)]);
    return seg0 + iw_wave_sum(s);
}

// Flush resolved stage bytes [from, to) to dst (byte-order transform fused,
// bool deferred to the end of the chunk: the committed bytes are the window).
// The stage starting at output position S holds position q at ring entry
// q - (S & ~15): 16-byte-aligned output pieces are 16-entry-aligned in the
// ring, and a stage of at most IW_S - 16 bytes never wraps.
__device__ void iw_commit(IwLds& L, u8* dst, u64 from, u64 to, DType t) {
    const u32 lane = (u32)lane_id();
    wsync();
    const u64 base = from & ~15ull;
    const u64 a16 = (from + 15) & ~15ull, b16 = to & ~15ull;
    if (a16 < b16) {
        for (u64 p = a16 + (u64)lane * 16; p < b16; p += 64 * 16) {
            const u32 i = (u32)(p - base);
            const u32x4 lo = *(const u32x4*)(L.u.st.ptr + i);
            const u32x4 hi = *(const u32x4*)(L.u.st.ptr + i + 8);
            auto pk = [](u32 a, u32 b) -> u32 { return __builtin_amdgcn_perm(b, a, 0x06040200u); };
            const u32x4 v = u32x4{pk(lo.x, lo.y), pk(lo.z, lo.w), pk(hi.x, hi.y), pk(hi.z, hi.w)};
            st16(dst + p, transform16(v, t));
        }
    }
    const u64 e0 = a16 < b16 ? a16 : to;
    for (u64 q = from + lane; q < e0; q += 64) dst[swap_pos(q, t)] = (u8)L.u.st.ptr[q - base];
    if (a16 < b16)
        for (u64 q = b16 + lane; q < to; q += 64) dst[swap_pos(q, t)] = (u8)L.u.st.ptr[q - base];
    // the next stage's far reads come back through this CU's L1/L2: wait
    // for the stores (same-CU stores refresh the L1)
    __syncthreads();
}

__device__ void iw_bool_norm(u8* dst, u64 D) {
    __syncthreads();
    const u32 lane = (u32)lane_id();
    const bool al = (((uintptr_t)dst) & 15) == 0;
    for (u64 p = (u64)lane * 16; p < D; p += 64 * 16) {
        if (p + 16 <= D) {
            u32x4 v = al ? *(u32x4*)(dst + p) : ld16(dst + p);
            v.x = bool_norm32(v.x); v.y = bool_norm32(v.y); v.z = bool_norm32(v.z); v.w = bool_norm32(v.w);
            if (al) *(u32x4*)(dst + p) = v; else st16(dst + p, v);
        } else {
            for (u64 q = p; q < D; q++) dst[q] = dst[q] != 0;
        }
    }
}

#define IW_T(slot)                                                              \
    do {                                                                        \
        if (dbg) {                                                              \
            const u64 _t = __builtin_readcyclecounter();                        \
            if (lane == 0) L.dbgc[slot] += (u32)(_t - t_last);                  \
            t_last = _t;                                                        \
        }                                                                       \
    } while (0)
#define IW_ADD(slot, v) do { if (dbg && lane == 0) L.dbgc[slot] += (u32)(v); } while (0)

// inclusive unsigned max over the wave (DPP row shifts, then the row maxima)
__device__ __forceinline__ u32 iw_incl_umax(u32 v) {
    v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

__device__ __forceinline__ u32 swap_pos32(u32 p, const DType& t) {
    if (!t.swap) return p;
    const u32 m = t.es - 1;
    return (p & ~m) | (m - (p & m));
}

// ---- dynamic block header, wave-parallel ------------------------------------
// Same results, validity rules and order as read_dynamic
// (zcg_inflate_common.h).  The code-length symbols are decoded at 64 bit
// positions at once (lane i at window bit w0 + i: symbol, code bits, extra
// bits, repeat count), and the true chain is walked through the window with
// v_readlane on wave-uniform positions, so a symbol costs a few scalar
// instructions instead of two dependent LDS round trips.
template <int LB, u32 LCAP, int DB, u32 DCAP>
__device__ __attribute__((always_inline)) int read_dynamic_wave(BitIn& b, u8* lens, HuffLds* lh, u32* ltab,
                                                                HuffLds* dh, u32* dtab, u32* hwin, u32* tcyc) {
    const u32 lane = (u32)lane_id();
    const u64 t_hdr0 = tcyc ? __builtin_readcyclecounter() : 0ull;
    if (!bi_has(b, 14)) return R_EXHAUSTED;
    const u32 nlen = bi_bits(b, 5) + 257, ndist = bi_bits(b, 5) + 1, ncode = bi_bits(b, 4) + 4;
    if (nlen > 286 || ndist > 30) return R_INVALID;  // "too many length or distance symbols"
    if (!bi_has(b, 3 * ncode)) return R_EXHAUSTED;
    const gu8* src = (const gu8*)b.src;
    const u64 nbytes = b.n;
    // The code lengths take < 300 bytes (<= 316 symbols of <= 7 + 7 bits):
    // one coalesced load puts the 512 bytes from here in LDS, so the window
    // walk below waits on LDS, not on a global round trip per window.
    const u64 wb = (b.consumed >> 3) & ~7ull;  // window base byte
    {
        const u64 by = wb + 8ull * lane;
        u64 w = 0;
        if (by + 8 <= nbytes) {
            w = *(const gu64_ua*)(src + by);
        } else {
            for (u32 k = 0; k < 8; k++)
                if (by + k < nbytes) w |= (u64)src[by + k] << (8 * k);
        }
        hwin[2 * lane] = (u32)w;
        hwin[2 * lane + 1] = (u32)(w >> 32);
        if (lane < 2) hwin[128 + lane] = 0;
    }
    __syncthreads();
    // 32 stream bits from absolute bit q (bytes past the input read as 0)
    auto bits32 = [&](u64 q) -> u32 {
        const u32 r = (u32)(q - 8 * wb);
        const u32 wi = r >> 5;
        if (wi + 1 < 128) {  // (hwin[128..129] are padding, not stream bytes)
            const u64 x = ((u64)hwin[wi + 1] << 32) | hwin[wi];
            return (u32)(x >> (r & 31));
        }
        const u64 by = q >> 3;
        u64 w = 0;
        for (u32 k = 0; k < 8; k++)
            if (by + k < nbytes) w |= (u64)src[by + k] << (8 * k);
        return (u32)(w >> (q & 7));
    };
    // the 3-bit code-length code lengths: lane i < ncode reads its own field
    const u64 c0 = b.consumed;
    const u32 mycl = lane < ncode ? bits32(c0 + 3 * lane) & 7 : 0u;
    {  // code-length code must be complete ("invalid code lengths set")
        int left = 1;
        for (u32 l = 1; l <= 7; l++) {
            const u32 cnt = (u32)__popcll(__ballot(lane < ncode && mycl == l));
            left <<= 1;
            left -= (int)cnt;
            if (left < 0) break;
        }
        if (left != 0) return R_INVALID;
    }
    __syncthreads();
    if (lane < 19) lens[lane] = 0;
    __syncthreads();
    if (lane < ncode) lens[c_clen_order[lane]] = (u8)mycl;
    __syncthreads();
    build_table(lens, 19, lh, ltab, 7, false, LCAP);
    const u32 total = nlen + ndist;
    const u64 lim = b.limit;
    u64 pos = c0 + 3 * ncode;  // wave-uniform reader position
    u32 idx = 0, prev = 0;
    // lens[0, total) starts at zero, so only the symbols with a nonzero value
    // write (one length, or a 16's 3-6 repeats); 17 / 18 write nothing
    for (u32 i = lane; i < 320; i += 64) lens[i] = 0;
    __syncthreads();
    while (idx < total) {
        // every lane decodes at bit pos + lane: code bits l, symbol, bits
        // consumed with the extra bits (adv), lengths written (cnt)
        const u64 q = pos + lane;
        const u32 v = bits32(q);
        const u32 e = ltab[v & 127];
        const u32 l = e >> 28, sym = e & 0x1F;
        const u32 x = v >> l;
        const u32 adv = sym == 16 ? l + 2 : sym == 17 ? l + 3 : sym == 18 ? l + 7 : l;
        const u32 cnt = sym == 16 ? 3 + (x & 3) : sym == 17 ? 3 + (x & 7) : sym == 18 ? 11 + (x & 127) : 1;
        // the true symbol starts in the window: a scalar walk of adv (l >= 1)
        u64 mem = 0;
        u32 rel = 0;
        while (rel < 64) {
            mem |= 1ull << rel;
            rel += (u32)__builtin_amdgcn_readlane((int)adv, (int)rel);
        }
        // every member at once: its first length index (prefix sum of the
        // counts), valid while that is below total (later members are the
        // block body)
        const bool m = ((mem >> lane) & 1ull) != 0;
        const u32 c = m ? cnt : 0u;
        const u32 incl = iw_incl_scan(c);
        const u32 is = idx + incl - c;
        const bool valid = m && is < total;
        // zlib's checks in read_dynamic's order (code bits, repeat at 0, extra
        // bits, overflow); the first member, in stream order, that fails decides
        const u64 at = pos + lane;
        u32 err = 0;
        if (valid) {
            if (at + l > lim) err = R_EXHAUSTED;
            else if (sym == 16 && is == 0) err = R_INVALID;
            else if (at + adv > lim) err = R_EXHAUSTED;
            else if (is + cnt > total) err = R_INVALID;
        }
        const u64 eb = __ballot(err != 0);
        if (eb) return (int)__builtin_amdgcn_readlane((int)err, (int)__builtin_ctzll(eb));
        // values: a literal length, 0 for 17 / 18, and for 16 the value of the
        // last non-16 member before it (the window's, or the previous window's)
        const u32 own = sym < 16 ? sym : 0u;
        const u32 lsrc = iw_incl_umax(valid && sym != 16 ? lane + 1 : 0u);
        const u32 pv = (u32)__shfl((int)own, (int)(lsrc ? lsrc - 1 : 0u), 64);
        const u32 val = sym == 16 ? (lsrc ? pv : prev) : own;
        if (valid && val)
            for (u32 k = 0; k < cnt; k++) lens[is + k] = (u8)val;  // (cnt <= 6 here)
        const u64 vb = __ballot(valid);
        const u32 lastm = 63u - (u32)__builtin_clzll(vb);
        idx = (u32)__builtin_amdgcn_readlane((int)(is + c), (int)lastm);
        prev = (u32)__builtin_amdgcn_readlane((int)val, (int)lastm);
        // next window: after the last member, or at the first member past the
        // code lengths (the block body starts there)
        const u64 rest = mem & ~vb;
        pos += rest ? (u32)__builtin_ctzll(rest) : rel;
    }
    b.cbase = ~0ull;
    bi_seek(b, pos);
    const u64 t_tab = tcyc ? __builtin_readcyclecounter() : 0ull;
    if (tcyc && lane == 0) tcyc[IWT_HWALK - IWT_HTAB] += (u32)(t_tab - t_hdr0);
    __syncthreads();
    u8 dl = 0;
    if (lane < ndist) dl = lens[nlen + lane];
    __syncthreads();
    for (u32 i = nlen + lane; i < 288; i += 64) lens[i] = 0;
    if (lane < 32) lens[288 + lane] = lane < ndist ? dl : 0;
    __syncthreads();
    if (lens[256] == 0) return R_INVALID;  // "invalid code -- missing end-of-block"
    if (build_table(lens, 288, lh, ltab, LB, false, LCAP) != 0) return R_INVALID;
    if (build_table(lens + 288, 30, dh, dtab, DB, true, DCAP) != 0) return R_INVALID;
    if (tcyc && lane == 0) *tcyc += (u32)(__builtin_readcyclecounter() - t_tab);
    return R_OK;
}

template <int LB, u32 LCAP, int DB, u32 DCAP>
__device__ __attribute__((always_inline)) int read_block_header_wave(BitIn& b, bool* last, u32* type, u32* slen,
                                                                     u8* lens, HuffLds* lh, u32* ltab, HuffLds* dh,
                                                                     u32* dtab, u32* hwin, u32* tcyc) {
    if (!bi_has(b, 3)) return R_EXHAUSTED;
    const u32 hdr = bi_bits(b, 3);
    *last = hdr & 1;
    *type = hdr >> 1;
    if (*type != 2) {  // stored / fixed / invalid: the serial reader's rules
        b.cbase = ~0ull;
        bi_seek(b, b.consumed - 3);
        return read_block_header<LB, LCAP, DB, DCAP>(b, last, type, slen, lens, lh, ltab, dh, dtab);
    }
    return read_dynamic_wave<LB, LCAP, DB, DCAP>(b, lens, lh, ltab, dh, dtab, hwin, tcyc);
}

constexpr u32 IW_NSLOT_MAX = 8192;
constexpr u64 IW_LIST_WORDS = 64ull * IW_TSTR;              // token lists of a slot (u32)
constexpr u64 IW_MARK_WORDS = 64ull * IW_MWORDS;            // token-start bitmaps of a slot (u32)
constexpr u64 IW_SLOT_WORDS = IW_LIST_WORDS + IW_MARK_WORDS;
constexpr u64 IW_OWNER_BYTES = IW_NSLOT_MAX * 4;

__global__ __launch_bounds__(64, ZIW_WPE) void inflate_wave_kernel(const zcg_chunk* __restrict__ chunks, u32 n,
                                                                  u64 D, DType t, u32 vflags,
                                                                  i32* __restrict__ status,
                                                                  u32* __restrict__ owner, u32 nslot,
                                                                  gu32* __restrict__ pools) {
    extern __shared__ __attribute__((aligned(16))) u8 smem_raw[];
    IwLds& L = *(IwLds*)smem_raw;
    const u32 c = blockIdx.x;
    if (c >= n) return;
    const u32 lane = threadIdx.x;
    const bool dbg = ZIW_DBG && (vflags & ZCG_FLAG_DEBUG_COUNTERS) != 0;
    const zcg_chunk ch = chunks[c];
    if (D == 0) { if (lane == 0) status[c] = ZCG_OK; return; }
    if (ch.dst_cap < D) { if (lane == 0) status[c] = ZCG_ERR_INVALID_INPUT; return; }
    const u8* s = (const u8*)ch.src;
    const u64 n_in = ch.src_len;
    u64 h = 0;
    int st = gzip_header(s, n_in, &h);
    if (st == ZCG_OK && (n_in - h >= (1ull << 28) || D >= (1ull << 32))) st = ZCG_ERR_UNSUPPORTED;  // u32 positions
    if (st != ZCG_OK) { if (lane == 0) status[c] = st; return; }

    u8* dst = (u8*)ch.dst;
    const u8* ds = s + h;
    const u64 n_ds = n_in - h;
    const u32 total_bits = (u32)(n_ds * 8);
    const u8* vbase = (const u8*)((uintptr_t)ds & ~(uintptr_t)15);
    const u32 a0b = (u32)((uintptr_t)ds & 15) * 8;  // stream bit 0 relative to vbase
    const u32 nvec = (u32)(((uintptr_t)ds & 15) + n_ds + 15) / 16;
    DType tw = t;
    tw.isbool = 0;

    // workspace slot (freed at the end; every path below reaches it)
    u32 slot = 0;
    if (lane == 0) {
        u32 sl = c % nslot;
        while (atomicCAS(&owner[sl], 0u, 1u) != 0u) sl = (sl + 1) % nslot;
        slot = sl;
    }
    slot = __builtin_amdgcn_readfirstlane(slot);
    gu32* const gl = pools + (u64)slot * IW_SLOT_WORDS;                 // token lists (iw_ta layout)
    gu32* const marks = gl + IW_LIST_WORDS;                             // token-start bitmaps [lane][IW_MWORDS]
    gu32* const mk = marks + (u64)lane * IW_MWORDS;

    BitIn b;
    bi_init(b, ds, n_ds, L.u.h.bcache);
    u64 P = 0;
    bool last = false, boundary = false, after_stored = false;
    int r = R_OK;
    u32 est = IW_EST0;
    if (dbg) {
        if (lane < IW_NDBG) L.dbgc[lane] = 0;
        wsync();
    }
    u64 t_last = __builtin_readcyclecounter();
    const u64 t_start = t_last;

    while (r == R_OK && P < D) {
        // ---- block header (wave-uniform reader) ------------------------------------
        if (last) { r = R_EXHAUSTED; break; }
        u32 type = 0, slen = 0;
        b.cbase = ~0ull;  // the reader's LDS cache shares storage with the stage
        wsync();
        r = read_block_header_wave<W_LB, W_LCAP, W_DB, W_DCAP>(b, &last, &type, &slen, L.u.h.lens, &L.u.h.lh, L.ltab,
                                                               &L.u.h.dh, L.dtab, L.u.h.hwin,
                                                               dbg ? &L.dbgc[IWT_HTAB] : nullptr);
        const u32 hdr_end = (u32)b.consumed;
        IW_T(IWT_HDR);
        if (r != R_OK) break;
        IW_ADD(IWD_BLOCKS, 1);
        wsync();
        if (type == 0) {
            // ---- stored block: byte copies through the stage ------------------------
            u64 in0 = hdr_end >> 3;  // byte aligned after LEN/NLEN
            u32 done = 0;
            while (done < slen && P < D) {
                u32 k = slen - done;
                if (k > IW_S - 16) k = IW_S - 16;
                if ((u64)k > D - P) k = (u32)(D - P);
                if (in0 + k > n_ds) { r = R_EXHAUSTED; break; }
                wsync();
                for (u32 i = lane; i < k; i += 64) L.u.st.ptr[(P & 15) + i] = (u16)(IE_VAL | ds[in0 + i]);
                iw_commit(L, dst, P, P + k, tw);
                P += k; in0 += k; done += k;
            }
            if (r != R_OK) break;
            b.cbase = ~0ull;
            bi_seek(b, in0 * 8);
            boundary = (done == slen);
            after_stored = true;
            continue;
        }
        after_stored = false;
        const u32 body0 = hdr_end;
        u32 R0 = hdr_end;
        bool block_end = false;
        bool final_cut = false;
        const u32 est_pct = (vflags & ZCG_FLAG_DEBUG_INFLATE_LONG_SEG) ? 116u : (u32)ZIW_EST_PCT;
        u32 seg = (u32)(((u64)est * est_pct / 100 / 64 + 31) & ~31ull);
        seg = seg < IW_SEGMIN ? IW_SEGMIN : seg > IW_SEGMAX ? IW_SEGMAX : seg;
        while (!block_end && !final_cut && r == R_OK && P < D) {
            // ================= H round: coarse speculative Huffman decode =================
            IW_ADD(IWD_ROUNDS, 1);
            const u32 round_hi = R0 + 64 * seg;
            const u32 p = R0 + lane * seg;
            const u32 pend = p + seg;
            u32 q = p, nt = 0, nxt = S_NONE, give = 0;
            const bool active = p < total_bits;
            GRd bs;
            gr_init(bs, vbase, nvec, (active ? p : 0u) + a0b);
            if (!active) {
                if (lane == 0) {  // the block body starts at the stream end
                    gl[iw_ta(0, 0)] = W_MARK | M_EXH;
                    nt = 1;
                    nxt = S_MARKER;
                } else {
                    nxt = S_ROUND_END;  // (never on the chain: the lane before it ends in EXH)
                }
            }
            // pass 1: my segment; markers other than EXH do not stop it.  Each
            // step stages its token and sets its start bit in an LDS window of
            // IW_MWIN mark words; every IW_K steps all lanes flush both to the
            // workspace with unconditional stores and refill the reader.
            u32 it1 = 0, w0 = 0, nt0 = nt;
#pragma unroll
            for (u32 j = 0; j < IW_MWIN; j++) L.u.hr.mwin[j][lane] = 0;
            bool run = nxt == S_NONE;
            while (__ballot(run) != 0) {
              const u32x4 vC = gr_vec(vbase, nvec, bs.vc), vD = gr_vec(vbase, nvec, bs.vc + 1);
              for (u32 kh = 0; kh < IW_KH; kh++) {
                for (u32 k = 0; k < IW_K; k++) {
                    if (!run || !gr_fill(bs)) continue;
                    u32 adv;
                    u32 tk = iw_decode(L, bs.lo, &adv);
                    if (q + adv > total_bits) tk = W_MARK | M_EXH;
                    if (nt == IW_TCAP) { nxt = S_CAP; run = false; continue; }
                    L.u.hr.tst[nt & (2 * IW_K - 1)][lane] = tk;
                    nt++;
                    const u32 off = q - p;  // (<= 5 words past w0 within one flush period)
                    atomicOr(&L.u.hr.mwin[(off >> 5) - w0][lane], 1u << (off & 31));
                    if (tk == (W_MARK | M_EXH)) { nxt = S_MARKER; run = false; continue; }
                    gr_drop(bs, adv);
                    q += adv;
                    it1++;
                    if (q >= pend) run = false;
                }
                // flush: the aligned block holding token nt0 once it is complete
                // (each block is stored once: its first words stay in the ring
                // until then, <= 3 + IW_K < 8 entries); then the mark window
                // (words past my position are still zero)
                {
                    const u32 a0 = nt0 & ~3u, sb = a0 & 4u;
                    if (nt >= a0 + 4) {
                        *(gu32x4_a16*)(gl + iw_ta(lane, a0)) =
                            u32x4{L.u.hr.tst[sb][lane], L.u.hr.tst[sb + 1][lane], L.u.hr.tst[sb + 2][lane],
                                  L.u.hr.tst[sb + 3][lane]};
                        nt0 = nt;
                    }
                }
                u32 mv[IW_MWIN];
#pragma unroll
                for (u32 j = 0; j < IW_MWIN; j++) mv[j] = L.u.hr.mwin[j][lane];
                // marks are kept for the first IW_MARKW words of the segment only
                // (a misaligned decoder syncs within ~450 bits at p99); later
                // flushes store nothing (stores to a dummy slot instead cost
                // 14 GB of writes and 11 % of the time per C2 launch: the slot
                // lines do not stay in L2 under 4 096 chunks' token lists)
                // Only words w0 .. w1 (the word of my next token start) can hold
                // marks yet, and w1 - w0 < 4 in almost every period: the second
                // half of the window is stored only when the lane got that far
                // (its zero words are stored when the window has slid onto them;
                // pass 2 and iw_rank read no word past the marked extent)
                const u32 w1 = (q - p) >> 5;
                if (w0 < IW_MARKW) {
                    *(gu32x4_a4*)(mk + w0) = u32x4{mv[0], mv[1], mv[2], mv[3]};
                    if (w1 >= w0 + 4) *(gu32x4_a4*)(mk + w0 + 4) = u32x4{mv[4], mv[5], mv[6], mv[7]};
                }
                // the first IW_EMW words also into LDS (rewritten until the
                // window has moved past them: then they are final)
                static_assert(IW_EMW == 2, "early mark words");
                if (w0 == 0) {
                    L.u.hr.em[0][lane] = mv[0];
                    L.u.hr.em[1][lane] = mv[1];
                } else if (w0 == 1) {
                    L.u.hr.em[1][lane] = mv[0];
                }
                // slide the window to the word of my next token start (< 8 words on)
                const u32 dw = w1 - w0;
#pragma unroll
                for (u32 sb = 1; sb < IW_MWIN; sb <<= 1) {
                    const bool t = (dw & sb) != 0;
#pragma unroll
                    for (u32 j = 0; j < IW_MWIN; j++) mv[j] = t ? (j + sb < IW_MWIN ? mv[j + sb] : 0u) : mv[j];
                }
#pragma unroll
                for (u32 j = 0; j < IW_MWIN; j++) L.u.hr.mwin[j][lane] = mv[j];
                w0 = w1;
              }
              gr_absorb(bs, vC, vD);
            }
            static_assert(IW_K == 4 && IW_MWIN == 8, "flush layout");
            // the last, incomplete block (an inactive lane's list never went through the ring)
            if (active && nt > (nt0 & ~3u)) {
                const u32 a0 = nt0 & ~3u, sb = a0 & 4u;
                *(gu32x4_a16*)(gl + iw_ta(lane, a0)) =
                    u32x4{L.u.hr.tst[sb][lane], L.u.hr.tst[sb + 1][lane], L.u.hr.tst[sb + 2][lane],
                          L.u.hr.tst[sb + 3][lane]};
            }
            // marked extent: the whole segment, or up to where the lane stopped
            {
                const u32 ext = !active ? 0u : nxt == S_NONE ? seg : (q - p) + (nxt == S_MARKER ? 1u : 0u);
                L.u.hr.mlim[lane] = ext < 32 * IW_MARKW ? ext : 32 * IW_MARKW;
            }
            __syncthreads();  // every lane's marks and list are stored
            IW_T(IWT_P1);
            // pass 2: follow my path until it meets a token start a later lane marked
            u32 ks = lane + 1, pk = pend, it2 = 0;
            u32 lim = ks < 64 ? L.u.hr.mlim[ks] : 0u;  // (no segment past lane 63)
            u32 cwi = 0xFFFFFFFFu, cwv = 0;
            bool run2 = nxt == S_NONE;
            while (__ballot(run2) != 0) {
                const u32x4 vC = gr_vec(vbase, nvec, bs.vc), vD = gr_vec(vbase, nvec, bs.vc + 1);
                for (u32 k = 0; k < IW_K * IW_KH; k++) {
                    if (!run2) continue;
                    if (q >= round_hi) { nxt = S_ROUND_END; run2 = false; continue; }
                    if (q >= pk + seg) { ks++; pk += seg; lim = ks < 64 ? L.u.hr.mlim[ks] : 0u; cwi = 0xFFFFFFFFu; }
                    const u32 off = q - pk;
                    if (off < lim) {
                        const u32 wi = off >> 5;
                        if (wi != cwi) { cwv = wi < IW_EMW ? L.u.hr.em[wi][ks] : marks[(u64)ks * IW_MWORDS + wi]; cwi = wi; }
                        if ((cwv >> (off & 31)) & 1u) {
                            give = iw_rank(L, ks, marks + (u64)ks * IW_MWORDS, wi, cwv & ((1u << (off & 31)) - 1u));
                            nxt = ks;
                            run2 = false;
                            continue;
                        }
                    }
                    if (!gr_fill(bs)) continue;  // A:B ran dry: wait for the refill
                    u32 adv;
                    u32 tk = iw_decode(L, bs.lo, &adv);
                    if (q + adv > total_bits) tk = W_MARK | M_EXH;
                    if (nt == IW_TCAP) { nxt = S_CAP; run2 = false; continue; }
                    gl[iw_ta(lane, nt)] = tk;
                    nt++;
                    it2++;
                    if (w_marker(tk)) {
                        if (tk != (W_MARK | M_EXH)) q += adv;
                        nxt = S_MARKER;
                        run2 = false;
                        continue;
                    }
                    gr_drop(bs, adv);
                    q += adv;
                }
                gr_absorb(bs, vC, vD);
            }
            if (dbg) {
                const u32 m1 = iw_wave_sum(it1), m2 = iw_wave_sum(it2);
                const u32 m3 = iw_wave_sum(nxt == S_CAP ? 1u : 0u);
                IW_ADD(IWD_P1_IT, m1);
                IW_ADD(IWD_P2_IT, m2);
                IW_ADD(IWD_CAPS, m3);
            }
            IW_T(IWT_P2);
            // ---- chain: lane 0 is true; follow the sync targets (wave-uniform walk) ----
            // chain member m lives in lane m's chL/chS/chE (its lane, first valid
            // token, list length): a sync target is always a later lane, so a
            // chain has <= 64 members, and the wave-uniform cursor reads them
            // with v_readlane instead of dependent LDS reads
            u32 ncm = 0, cur = 0, sidx = 0;
            u32 chL = 0, chS = 0, chE = 0;
            for (;;) {
                const u32 e = (u32)__builtin_amdgcn_readlane((int)nt, (int)cur);
                const u32 nx = (u32)__builtin_amdgcn_readlane((int)nxt, (int)cur);
                if (lane == ncm) { chL = cur; chS = sidx; chE = e; }
                ncm++;
                if (nx < 64) {
                    sidx = (u32)__builtin_amdgcn_readlane((int)give, (int)cur);
                    cur = nx;
                    continue;
                }
                break;
            }
            const u32 endq = (u32)__builtin_amdgcn_readlane((int)q, (int)cur);  // after the last member's list
            if ((u32)__builtin_amdgcn_readlane((int)nxt, (int)cur) == S_CAP && seg > IW_SEGMIN)
                seg = (seg / 2 + 31) & ~31u;  // lists overflowed: shorter segments next round (this round's
                                              // positions come from p, computed with the old seg)
            IW_ADD(IWD_CHAIN, ncm);
            // token lists of other lanes are read below: their stores must be done
            __syncthreads();
            IW_T(IWT_CHAIN);

            // ================= L phase: the chain's tokens, one stage at a time =========
            // Stage: output [S, S + emit) in the ring; lane l owns the 32-entry
            // block at absolute B0 + 32 l, B0 = S & ~31 (64 blocks = the ring).
            u32 cm = 0, cj = 0;  // cursor: chain member, token index in its list
            // lane's token at the cursor + lane (a member's list may end inside a group)
            auto mL = [&](u32 m) -> u32 { return (u32)__builtin_amdgcn_readlane((int)chL, (int)m); };
            auto mE = [&](u32 m) -> u32 { return (u32)__builtin_amdgcn_readlane((int)chE, (int)m); };
            // member m's successor's first valid token, in lane m (0 past the chain)
            const u32 chSn = (u32)__shfl_down((int)chS, 1, 64);  // (every lane: a lane reads an active lane)
            const u32 chS1 = lane + 1 < ncm ? chSn : 0u;
            auto mS1 = [&](u32 m) -> u32 { return (u32)__builtin_amdgcn_readlane((int)chS1, (int)m); };
            auto advance = [&](u32& cm0, u32& cj0, u32 k) {
                // (wave-uniform: kept in scalar registers)
                u32 m = (u32)__builtin_amdgcn_readfirstlane((int)cm0), j = (u32)__builtin_amdgcn_readfirstlane((int)(cj0 + k));
                while (m < ncm) {
                    const u32 e = mE(m);
                    if (j < e) break;
                    j = j - e + mS1(m);
                    m++;
                }
                cm0 = m;
                cj0 = j;
            };
            // The token words of the next IW_GK groups are in flight while a
            // group is placed (the lists sit in MALL/HBM: ~2 K cycles away).
            // Each group slot is a named register that is loaded IW_GK groups
            // before its use, so no in-flight value is copied at the loop's
            // back edge (a copy would wait for it).  Within a stage every
            // group but the last is taken whole, so the prefetch positions
            // are exact; a new stage refetches from its cursor.
            // two chain tokens per lane per group (tokens 2l, 2l + 1): the
            // group's fixed costs (scan, ballots, cursor walk) are paid once
            // per 128 tokens
            // A slot holds the two raw loaded words and a validity mask (bit 0:
            // token 2l, bit 1: token 2l + 1; a token past the chain is M_END).
            // The words are loaded unconditionally (a dummy word otherwise) and
            // not touched until the slot is consumed: any use of a loaded
            // register, even a select, waits for it.
            auto fetch2 = [&](u32 cm0, u32 cj0, u32& ta, u32& tb, u32& ok) {
                u32 ja = cj0 + 2 * lane, jb = ja + 1, la = 0xFFFFFFFFu, lb = 0xFFFFFFFFu, pa = 0, pb = 0;
                for (u32 m = (u32)__builtin_amdgcn_readfirstlane((int)cm0); m < ncm; m++) {
                    const u32 e = mE(m), ln = mL(m), s1 = mS1(m);
                    if (la == 0xFFFFFFFFu && ja < e) { la = ln; pa = ja; }
                    if (lb == 0xFFFFFFFFu && jb < e) { lb = ln; pb = jb; }
                    if (__ballot(la == 0xFFFFFFFFu || lb == 0xFFFFFFFFu) == 0) break;
                    if (la == 0xFFFFFFFFu) ja = ja - e + s1;
                    if (lb == 0xFFFFFFFFu) jb = jb - e + s1;
                }
                ok = (la != 0xFFFFFFFFu ? 1u : 0u) | (lb != 0xFFFFFFFFu ? 2u : 0u);
                ta = gl[la != 0xFFFFFFFFu ? iw_ta(la, pa) : 0u];
                tb = gl[lb != 0xFFFFFFFFu ? iw_ta(lb, pb) : 0u];
            };
            u32 tq0a, tq0b, tq1a, tq1b, tq2a, tq2b, ok0, ok1, ok2;
            u32 pcm = 0, pcj = 0;  // prefetch cursor: IW_GK groups past the cursor (groups inside a stage are whole)
            // the IW_GK groups from the cursor in one walk over the chain
            // members (tokens cj + 128 g + 2 l + {0, 1} of group g)
            auto refetch = [&]() {
                static_assert(IW_GK == 3, "three group slots");
                u32 jt[6], lt[6], pt[6];
#pragma unroll
                for (u32 t = 0; t < 6; t++) {
                    jt[t] = cj + 128 * (t >> 1) + 2 * lane + (t & 1);
                    lt[t] = 0xFFFFFFFFu;
                    pt[t] = 0;
                }
                for (u32 m = (u32)__builtin_amdgcn_readfirstlane((int)cm); m < ncm; m++) {
                    const u32 e = mE(m), ln = mL(m), s1 = mS1(m);
                    bool open = false;
#pragma unroll
                    for (u32 t = 0; t < 6; t++) {
                        if (lt[t] == 0xFFFFFFFFu && jt[t] < e) { lt[t] = ln; pt[t] = jt[t]; }
                        open |= lt[t] == 0xFFFFFFFFu;
                    }
                    if (__ballot(open) == 0) break;
#pragma unroll
                    for (u32 t = 0; t < 6; t++)
                        if (lt[t] == 0xFFFFFFFFu) jt[t] = jt[t] - e + s1;
                }
                auto ld = [&](u32 t) -> u32 { return gl[lt[t] != 0xFFFFFFFFu ? iw_ta(lt[t], pt[t]) : 0u]; };
                auto okm = [&](u32 t) -> u32 {
                    return (lt[t] != 0xFFFFFFFFu ? 1u : 0u) | (lt[t + 1] != 0xFFFFFFFFu ? 2u : 0u);
                };
                tq0a = ld(0); tq0b = ld(1); ok0 = okm(0);
                tq1a = ld(2); tq1b = ld(3); ok1 = okm(2);
                tq2a = ld(4); tq2b = ld(5); ok2 = okm(4);
                u32 cm1 = cm, cj1 = cj;
                advance(cm1, cj1, 128 * IW_GK);
                pcm = cm1;
                pcj = cj1;
            };
            refetch();
            u32 gslot = 0;  // the group slot the next group is in
            bool round_done = false;
            while (!round_done && r == R_OK) {
                const u64 S = P;
                const u64 room = D - P;
                const u32 capS = IW_S - 16;  // (S & 15) + cap <= IW_S: the stage never wraps the ring
                const u32 cap = room < capS ? (u32)room : capS;
                const bool fin = (u64)cap == room;
                // Token-granular stage.  The ring is cleared, then every kept
                // token writes its own entries: a literal its final byte; a FAR
                // match (whole source before the stage) its final bytes, copied
                // from the committed output by 16-byte pieces, one aligned quad
                // of entries OR-ed in per source dword; a NEAR match one pointer
                // per byte (to the byte d before it), resolved in ordered
                // batches of 64 near bytes by pointer jumping.  Sources always
                // lie before their byte, so a batch only waits on itself.
                {
                    u32x4* z = (u32x4*)L.u.st.ptr;
#pragma unroll
                    for (u32 i = 0; i < IW_S / 512; i++) z[lane + 64 * i] = u32x4{0u, 0u, 0u, 0u};
                }
                wsync();
                u32 emitted = 0;
                bool rej = false;  // the stage ended before a group that did not fit whole
                bool bad = false;  // a distance before the output start
                u32 why = 0;       // 1 final cut, 2 marker / round end, 3 capacity
                u32 mcode = 0;
                const gu8* gd = (const gu8*)dst;
                // 16-byte source pieces: native byte order, and every piece of
                // a far token ends before S + 16 <= D
                const bool wide_ok = !tw.swap && room >= 16;
                const u32 S32 = (u32)S;  // (D < 2^32)
                const u32 s0 = S32 & 15u;  // ring entry of the stage's first byte
                struct Tk {
                    // kind 0 none, 1 literal (d = byte), 2 match; L clipped at cap;
                    // fl: the far part, the first bytes whose source lies before
                    // the stage (copied from the committed output); the rest of
                    // the match is its near part (source inside the stage)
                    u32 kind, o, L, d, fl;
                };
                auto classify = [&](u32 tk, u32 o, u32 len, bool keep) -> Tk {
                    Tk t{0u, o, 0u, 0u, 0u};
                    if (!keep) return t;
                    if (!(tk & W_MATCH)) {
                        t.kind = 1u;
                        t.L = 1u;
                        t.d = tk & 0xFFu;
                        return t;
                    }
                    const u32 d = (tk & 0x7FFFu) + 1u;
                    if (d > S32 + o) {
                        bad = true;
                        return t;
                    }
                    t.L = (fin && o + len > cap) ? cap - o : len;
                    t.d = d;
                    t.kind = 2u;
                    if (wide_ok && o < d) t.fl = d - o < t.L ? d - o : t.L;
                    return t;
                };
                // near parts of the group before, resolved while the far loads
                // of the current group are in flight (their sources lie in
                // earlier groups or in themselves; the far and literal entries
                // of the current group are disjoint from them)
                u32 pn_nla = 0, pn_nlb = 0, pn_na = 0, pn_nb = 0, pn_dsa = 0, pn_dsb = 0, pn_NB = 0;
                auto near_run = [&]() {
                    // near batches of 64 bytes in output order: lane i takes near
                    // byte n0 + i; its part is the last one whose first byte in
                    // the batch is at or before it.  Each part of the batch puts
                    // slot << 26 | descriptor at the slot of its first byte there
                    // (slot 0 for the part running into the batch), so one
                    // unsigned max scan over the cleared slots hands every lane
                    // its part's descriptor.
                    for (u32 n0 = 0; n0 < pn_NB; n0 += 64) {
                        L.u.st.mk[lane] = 0;
                        wsync();
                        if (pn_nla && pn_na < n0 + 64 && pn_na + pn_nla > n0) {
                            const u32 sl = pn_na > n0 ? pn_na - n0 : 0u;
                            L.u.st.mk[sl] = (sl << 26) | pn_dsa;
                        }
                        if (pn_nlb && pn_nb < n0 + 64 && pn_nb + pn_nlb > n0) {
                            const u32 sl = pn_nb > n0 ? pn_nb - n0 : 0u;
                            L.u.st.mk[sl] = (sl << 26) | pn_dsb;
                        }
                        wsync();
                        const u32 dsc = iw_incl_umax(L.u.st.mk[lane]) & 0x3FFFFFFu;
                        const u32 i = n0 + lane;
                        bool done = i >= pn_NB, strad = false;
                        u32 pos = 0, cur = 0;
                        if (!done) {
                            const u32 p = (dsc & 0x7FFu) + i;
                            const u32 d = (dsc >> 11) + 1u;
                            pos = s0 + p;
                            if (p >= d) cur = s0 + p - d;
                            else cur = IE_VAL | (u32)gd[swap_pos32(S32 + p - d, tw)];  // before the stage (!wide_ok only)
                            strad = p < d;
                            // a source that is already final settles the byte now: the
                            // read precedes this batch's writes, and an entry of this
                            // batch still reads as a pointer (zero or older), so only
                            // final values are taken
                            const u32 v0 = cur >= IE_VAL ? cur : (u32)L.u.st.ptr[cur];
                            done = v0 >= IE_VAL;
                            if (done) cur = v0;
                            L.u.st.ptr[pos] = (u16)cur;
                        }
                        wsync();
                        IW_ADD(IWD_NBATCH, 1);
                        if (dbg && __ballot(strad) != 0) IW_ADD(IWD_NSTRAD, 1);
                        for (u32 pass = 0; __ballot(!done) != 0; pass++) {
                            IW_ADD(IWD_NPASS, 1);
                            if (pass >= 8) {  // a 64-byte batch resolves in <= 7 passes
                                bad = true;
                                break;
                            }
                            u32 v = 0;
                            if (!done) v = L.u.st.ptr[cur];
                            wsync();
                            if (!done) {
                                L.u.st.ptr[pos] = (u16)v;
                                cur = v;
                                done = v >= IE_VAL;
                            }
                            wsync();
                        }
                    }
                    pn_NB = 0;
                };
                auto group2 = [&](u32& tqa, u32& tqb, u32& okq) -> bool {
                    IW_ADD(IWD_GROUPS, 1);
                    const u32 ta = (okq & 1u) ? tqa : (W_MARK | M_END), tb = (okq & 2u) ? tqb : (W_MARK | M_END);
                    const u64 ma = __ballot(w_marker(ta)), mb = __ballot(w_marker(tb));
                    const u32 fa = ma ? 2 * (u32)__builtin_ctzll(ma) : 128u, fb = mb ? 2 * (u32)__builtin_ctzll(mb) + 1 : 128u;
                    const u32 fm = fa < fb ? fa : fb;  // first marker, in token order
                    const u32 ia = 2 * lane, ib = ia + 1;
                    const u32 la = ia < fm ? w_len(ta) : 0u, lb = ib < fm ? w_len(tb) : 0u;
                    const u32 ps = la + lb;
                    const u32 incl = iw_incl_scan(ps);
                    const u32 oa = emitted + incl - ps, ob = oa + la;
                    const bool ka = ia < fm && (fin ? oa < cap : oa + la <= cap);
                    const bool kb = ib < fm && (fin ? ob < cap : ob + lb <= cap);
                    const u32 ntk = (u32)__popcll(__ballot(ka)) + (u32)__popcll(__ballot(kb));
                    // a group that does not fit whole into a stage that has
                    // bytes already starts the next stage instead: the token
                    // slots stay valid (nothing was prefetched into this one),
                    // so no refetch is needed there
                    if (!fin && emitted != 0 && ntk < fm) {
                        rej = true;
                        why = 3;
                        return true;
                    }
                    IW_T(IWT_PLACE);
                    const Tk A = classify(ta, oa, la, ka), B = classify(tb, ob, lb, kb);
                    if (A.kind == 1u) L.u.st.ptr[s0 + A.o] = (u16)(IE_VAL | A.d);
                    if (B.kind == 1u) L.u.st.ptr[s0 + B.o] = (u16)(IE_VAL | B.d);
                    IW_T(IWT_CLASSIFY);
                    // far parts, compacted one per lane (rank in token order):
                    // 16-byte source pieces from the part's first source byte,
                    // widened to entries by v_perm and stored exactly with
                    // unaligned ds_write_b128 (8 entries; a part's last < 8
                    // entries by b64 / b32 / b16), so tokens never share a store.
                    // The token words of the group IW_GK ahead are fetched right
                    // after the far loads: vmcnt is in order, so the far data can
                    // then be waited for with the prefetch still in flight.
                    {
                        const bool fA = A.fl != 0u, fB = B.fl != 0u;
                        const u64 bA = __ballot(fA), bB = __ballot(fB);
                        const u64 below = (1ull << lane) - 1ull;
                        const u32 rkA = (u32)__popcll(bA & below) + (u32)__popcll(bB & below), rkB = rkA + (fA ? 1u : 0u);
                        const u32 NF = (u32)__popcll(bA) + (u32)__popcll(bB);
                        // source byte | (ring entry of the first byte | length << 16) << 32
                        auto fdesc = [&](const Tk& t) -> u64 {
                            return (u64)(S32 + t.o - t.d) | ((u64)((s0 + t.o) | (t.fl << 16)) << 32);
                        };
                        // one batch of <= 64 far parts; the first one issues the prefetch
                        auto far_batch = [&](u32 f0, auto with_prefetch) {
                            if (fA && rkA - f0 < 64u) L.u.st.fd[rkA - f0] = fdesc(A);
                            if (fB && rkB - f0 < 64u) L.u.st.fd[rkB - f0] = fdesc(B);
                            wsync();
                            const bool fl = f0 + lane < NF;
                            const u64 fdw = L.u.st.fd[lane];
                            const u32 src = (u32)fdw, hi = (u32)(fdw >> 32);
                            const u32 qi = hi & 0xFFFFu, e = hi >> 16;
                            const u32 np = (e + 15) >> 4;
                            u32x4 V0 = u32x4{0u, 0u, 0u, 0u}, V1 = V0;
                            if (fl) {
                                V0 = *(const gu32x4_ua*)(gd + src);
                                // unconditional (a second read of the first piece when
                                // there is one piece): a load kept under a branch waited
                                // for the first one before issuing
                                V1 = *(const gu32x4_ua*)(gd + src + (np > 1 ? 16u : 0u));
                            }
                            if constexpr (decltype(with_prefetch)::value) {
                                fetch2(pcm, pcj, tqa, tqb, okq);
                                advance(pcm, pcj, 128);
                                if (pn_NB) near_run();
                            }
                            // both pieces waited for here, on every path: vmcnt(2)
                            // with the prefetch still in flight (a wait where the
                            // registers are next written would be vmcnt(0))
                            asm volatile("" ::"v"(V0), "v"(V1));
                            if (fl) {
                                auto piece = [&](const u32x4& V, u32 p) {
                                    const u32 b0 = 16 * p;  // < e
                                    iw_put(L.u.st.ptr + qi + b0, e - b0, ie_lo(V.x), ie_hi(V.x), ie_lo(V.y), ie_hi(V.y));
                                    if (e > b0 + 8)
                                        iw_put(L.u.st.ptr + qi + b0 + 8, e - b0 - 8, ie_lo(V.z), ie_hi(V.z), ie_lo(V.w),
                                               ie_hi(V.w));
                                };
                                piece(V0, 0);
                                if (np > 1) piece(V1, 1);
                                for (u32 p = 2; p < np; p++) {
                                    IW_ADD(IWD_FARIT, 1);
                                    const u32x4 Vp = *(const gu32x4_ua*)(gd + src + 16 * p);
                                    piece(Vp, p);
                                }
                            }
                            wsync();
                        };
                        far_batch(0u, std::true_type{});
                        for (u32 f0 = 64; f0 < NF; f0 += 64) far_batch(f0, std::false_type{});
                    }
                    IW_T(IWT_FAR);
                    // near parts: one pointer per byte, resolved in ordered
                    // batches of 64 by pointer jumping (index in the group's
                    // ordered list of near bytes).  (Token-level copies of whole
                    // near parts, in rounds until their sources are final, took
                    // 27.1 vs 21.6 ms per C2 launch: 8 entries at 2-byte
                    // alignment are an unaligned LDS access, 256 instead of 72
                    // cycles per read, tools/probe/lds_unaligned_perf.hip.)
                    const u32 noa = A.o + A.fl, nob = B.o + B.fl;
                    const u32 nla = A.kind == 2u ? A.L - A.fl : 0u, nlb = B.kind == 2u ? B.L - B.fl : 0u;
                    const u32 nps = nla + nlb;
                    const u32 nincl = iw_incl_scan(nps);
                    const u32 na = nincl - nps, nb = na + nla;
                    const u32 NB = (u32)__builtin_amdgcn_readlane((int)nincl, 63);
                    // a part's descriptor: (its first offset - its first near index) | (d - 1) << 11
                    const u32 dsa = (noa - na) | ((A.d - 1u) << 11), dsb = (nob - nb) | ((B.d - 1u) << 11);
                    pn_nla = nla;
                    pn_nlb = nlb;
                    pn_na = na;
                    pn_nb = nb;
                    pn_dsa = dsa;
                    pn_dsb = dsb;
                    pn_NB = NB;
                    IW_T(IWT_NEAR);
                    if (ntk) {
                        const u32 t = ntk - 1;  // the last taken token: lane t / 2, slot t % 2
                        const u32 ea = incl - ps + la;
                        emitted += (u32)__builtin_amdgcn_readlane((int)((t & 1) ? incl : ea), (int)(t >> 1));
                    }
                    advance(cm, cj, ntk);
                    if (fin && emitted >= cap) { why = 1; return true; }
                    if (ntk < 128) {
                        if (ntk == fm) {
                            why = 2;
                            mcode = (u32)__builtin_amdgcn_readlane((int)((fm & 1) ? tb : ta), (int)(fm >> 1)) & 3u;
                        } else {
                            why = 3;
                        }
                        return true;
                    }
                    return false;
                };
                for (;;) {
                    bool end;
                    if (gslot == 0) end = group2(tq0a, tq0b, ok0);
                    else if (gslot == 1) end = group2(tq1a, tq1b, ok1);
                    else end = group2(tq2a, tq2b, ok2);
                    if (!rej) gslot = gslot == IW_GK - 1 ? 0u : gslot + 1;
                    if (end) break;
                }
                if (!rej) {  // the stage ended inside a group: the next one starts at the cursor
                    refetch();  // (its loads fly during the last near batches)
                    gslot = 0;
                }
                IW_T(IWT_REFETCH);
                if (pn_NB) near_run();  // the stage's last group
                IW_T(IWT_NEAR);
                IW_ADD(IWD_STAGES, 1);
                if (__ballot(bad) != 0) { r = R_INVALID; break; }
                const u32 emit = emitted < cap ? emitted : cap;  // a token may cross N: clip
                IW_T(IWT_CLASSIFY);
                if (emit) {
                    iw_commit(L, dst, S, S + emit, tw);
                    P = S + emit;
                    IW_T(IWT_COMMIT);
                }
                if (why == 1) {
                    // output full: zlib's look-ahead continues at the first untaken token
                    boundary = emitted == cap;
                    final_cut = true;
                    round_done = true;
                    if (boundary) {
                        u32 qn = endq;
                        // (the member's segment start from this round's p: seg may
                        // already be halved for the next round, after a capped list)
                        if (cm < ncm) qn = iw_pos(gl, mL(cm), cj, (u32)__builtin_amdgcn_readlane((int)p, (int)mL(cm)));
                        b.cbase = ~0ull;
                        bi_seek(b, qn);
                    }
                } else if (why == 2) {
                    round_done = true;
                    if (mcode == M_END) {
                        R0 = endq;  // the chain ended without a marker: next round from there
                        IW_ADD(IWD_NOEOB, 1);
                        // the rest of the block is likely short: size the next round for it
                        const u32 used = R0 - body0;
                        const u32 rem = est > used ? est - used : est / 8;
                        u32 sg = (rem / 64 + 31) & ~31u;
                        seg = sg < IW_SEGMIN ? IW_SEGMIN : sg > IW_SEGMAX ? IW_SEGMAX : sg;
                    } else if (mcode == M_EOB) {
                        const u32 lm = mL(cm);
                        // after the EOB code; the member's segment start is this
                        // round's p (not R0 + lm * seg: seg may already be halved for
                        // the next round when the chain's last list was capped)
                        const u32 qe = iw_pos(gl, lm, cj + 1, (u32)__builtin_amdgcn_readlane((int)p, (int)lm));
                        IW_T(IWT_EOB);
                        block_end = true;
                        b.cbase = ~0ull;
                        bi_seek(b, qe);
                        est = qe - body0;
                    } else if (mcode == M_BAD) {
                        r = R_INVALID;
                    } else {
                        r = R_EXHAUSTED;
                    }
                }
            }
        }
    }
    // zlib's post-N look-ahead (wave-uniform); see zcg_inflate_common.h
    if (r == R_OK && P >= D && boundary) {
        const u64 last_byte = h + (b.consumed ? (b.consumed - 1) / 8 : 0);
        u64 wend = (last_byte / 32768 + 1) * 32768;
        if (wend > n_in) wend = n_in;
        b.limit = (wend - h) * 8;
        b.cbase = ~0ull;
        wsync();
        if (b.limit >= b.consumed) {
            const int la = inf_lookahead<W_LB, W_LCAP, W_DB, W_DCAP>(b, last, after_stored, L.u.h.lens, &L.u.h.lh,
                                                                     L.ltab, &L.u.h.dh, L.dtab);
            if (la == R_INVALID) r = R_INVALID;
        }
    }
    if (r == R_INVALID) st = ZCG_ERR_INVALID_DATA;
    else if (r == R_EXHAUSTED || P < D) st = ZCG_ERR_UNEXPECTED_EOF;
    if (t.isbool) iw_bool_norm(dst, P < D ? P : D);
    if (dbg) {
        if (lane == 0) L.dbgc[IWT_TOTAL] = (u32)(__builtin_readcyclecounter() - t_start);
        wsync();
        if (lane < IW_NDBG && L.dbgc[lane]) atomicAdd(&g_iw_dbg[lane], (unsigned long long)L.dbgc[lane]);
    }
    __syncthreads();  // every workspace access of this wave is done
    if (lane == 0) {
        status[c] = st;
        atomicExch(&owner[slot], 0u);
    }
}

extern "C" int zcg__debug_inflate_wave_counters(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_iw_dbg), sizeof(unsigned long long) * 32) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_iw_dbg), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}

// Slots: one per resident wave (the LDS footprint bounds residency), never
// more than the batch.
static u32 iw_nslot(uint32_t n) {
    const u32 cus = device_cu_count();
    u32 per_cu = (u32)(160 * 1024 / sizeof(IwLds));
    if (per_cu < 1) per_cu = 1;
    u64 ns = (u64)cus * per_cu;
    if (ns > n) ns = n;
    if (ns > IW_NSLOT_MAX) ns = IW_NSLOT_MAX;
    return (u32)ns;
}

const char* cfg_inflate_wave() {
    return "inflate_wave:S=" ZCG_STR(ZIW_S) ",TCAP=" ZCG_STR(ZIW_TCAP) ",WPE=" ZCG_STR(ZIW_WPE)
           ",EST_PCT=" ZCG_STR(ZIW_EST_PCT) ",MARKW=" ZCG_STR(ZIW_MARKW) ",G=" ZCG_STR(ZIW_G) ",DBG=" ZCG_STR(ZIW_DBG);
}

uint64_t inflate_wave_ws_bytes(const zcg_array* a, uint32_t n) {
    (void)a;
    if (n == 0) return 0;
    return IW_OWNER_BYTES + (u64)iw_nslot(n) * IW_SLOT_WORDS * 4;
}

hipError_t launch_inflate_wave(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                               int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (!ws || ws_bytes < inflate_wave_ws_bytes(a, n)) return hipErrorInvalidValue;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const size_t lds = sizeof(IwLds);
    if (hipError_t e = lds_attr_once((const void*)inflate_wave_kernel, (int)lds); e != hipSuccess) return e;
    const u32 nslot = iw_nslot(n);
    u32* owner = (u32*)ws;
    hipError_t e = hipMemsetAsync(owner, 0, (size_t)nslot * 4, s);
    if (e != hipSuccess) return e;
    gu32* pools = (gu32*)((u8*)ws + IW_OWNER_BYTES);
    hipLaunchKernelGGL(inflate_wave_kernel, dim3(n), dim3(64), lds, s, d_chunks, n, D, t,
                       a->compression.flags, d_status, owner, nslot, pools);
    return hipGetLastError();
}

}  // namespace zcg
