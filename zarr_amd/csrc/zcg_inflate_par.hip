// zcg_inflate_par.hip — parallel inflate of gzip chunks on gfx950
// (GzipCompression decode, src/compression/gzip.rs:49-52 -> flate2 -> zlib).
//
// A deflate block is one serial Huffman stream, so a chunk gets lane
// parallelism by SPECULATIVE, SELF-SYNCHRONISING decoding.  One workgroup of
// 256 lanes (4 waves, one per SIMD of the CU) owns one chunk:
//
//   round: the block stages the next ~8.7 KiB of the stream in LDS; lane i
//     decodes from bit R0 + i*SEG as if a symbol started there, keeping the
//     bit buffer in registers, storing every token (literal, match, or an
//     EOB / invalid-code / input-exhausted marker) and marking its start bit
//     in lane i's segment bitmap, until it leaves its segment.
//   sync:  every lane then keeps following its own path past its segment and
//     stops at the first token start that another lane MARKED (any later
//     segment): from a common start bit two Huffman paths are identical, so
//     the lane that marked it is on the true path from there.  Measured on
//     the bench data (SURVEY §8(d) "quant", zlib-6): median 50-80 bits, p99
//     ~450 bits to resynchronise.  Lane 0 is true by construction; the valid
//     chain follows the sync targets (almost always lane i+1; the rare
//     skips/stops are walked by one thread).
//   place: a block-wide prefix sum over the chain lanes' output lengths
//     positions every token; the round is cut at STAGE bytes, and at N with
//     zlib's look-ahead semantics when N falls on a token boundary.
//   LZ77:  literals land in an LDS stage; matches resolve in rounds (each
//     lane walks its own matches in order and copies one as soon as its
//     source bytes are resolved — the earliest unresolved match is always
//     resolvable, so this terminates); sources before the round come from
//     the 32 KiB LDS window ring.  Copies read B[src + k mod dist] so a
//     match's reads never depend on its own writes.
//   commit: the stage is flushed to HBM with 16 B/lane stores (byte order /
//     bool transform fused) and appended to the window ring.
// Block headers, stored blocks and the post-N look-ahead use the wave-uniform
// reader of zcg_inflate_common.h (wave 0).  Results are bit-identical to the
// serial kernel (zcg_inflate.hip); tests/ compare the two.
#include "zcg_inflate_common.h"

// tuning knobs (A/B builds): tokens prefetched into registers per lane, far
// gathers in flight per thread, waves per SIMD the register budget targets
#ifndef ZCG_INF_PF
#define ZCG_INF_PF 16
#endif
#ifndef ZCG_INF_FU
#define ZCG_INF_FU 16
#endif
#ifndef ZCG_INF_WPE
#define ZCG_INF_WPE 3
#endif

namespace zcg {

constexpr u32 PI_NL = 256;       // lanes per chunk (4 waves)
constexpr u32 PI_SEG = 256;      // bits per lane segment
constexpr u32 PI_TMAX = 96;      // tokens per lane per round (the lane stops with N_CAP)
constexpr u32 PI_STAGE = 16384;  // output bytes per round (power of 2)
constexpr u32 PI_WIN = 32768;    // LZ77 window (read back from the chunk's committed output)
constexpr u32 PI_SEGW = PI_SEG / 32;
constexpr u32 PI_IN_VEC = (PI_NL * PI_SEG + 1024) / 128 + 2;  // staged 16-B vectors
constexpr u32 PI_IN_WORDS = PI_IN_VEC * 4;
// LDS bank-conflict padding: one pad word after every 8 words, so lanes that
// read at an 8-word stride (segment starts, segment marks) hit distinct banks.
constexpr u32 PI_IN_PAD = PI_IN_WORDS + PI_IN_WORDS / 8 + 8;
__device__ __forceinline__ u32 padw(u32 w) { return w + (w >> 3); }
constexpr u32 PI_MAXSEG = 64;    // chain segments tracked per round

// token word: literal = byte value; match = 1<<31 | (len-3)<<16 | (dist-1);
// markers (bit 30): EOB, invalid code, input exhausted.
constexpr u32 T_MATCH = 0x80000000u;
constexpr u32 T_EOB = 0x40000000u;
constexpr u32 T_BAD = 0x40000001u;
constexpr u32 T_EXH = 0x40000002u;

// lane stop codes (next[] >= PI_NL)
constexpr u32 N_ROUND_END = PI_NL;  // reached the end of the round's range
constexpr u32 N_MARKER = PI_NL + 1; // last stored token is a marker
constexpr u32 N_CAP = PI_NL + 2;    // token store full before syncing

// Debug counters (flag ZCG_FLAG_DEBUG_COUNTERS): summed over all chunks.
__device__ unsigned long long g_inf_dbg[32];
enum { DBG_ROUNDS, DBG_CHAIN, DBG_END_CAP, DBG_END_EOB, DBG_END_BAD, DBG_SKIPS, DBG_MRR_IT,
       DBG_CUTS, DBG_BLOCKS, DBG_BYTES, DBG_TOKENS, DBG_END_ROUND, DBG_PASS2_TOK,
       DBG_CAP_P1, DBG_CAP_P2, DBG_P2_MAX };

// phase timers (debug): slots 16.. of g_inf_dbg
enum { TP_HDR = 16, TP_STAGE, TP_PASS1, TP_PASS2, TP_CHAIN, TP_PLACE, TP_LIT, TP_MRR, TP_COMMIT, TP_TOTAL };
#define TSTAMP(slot)                                                                 \
    do {                                                                             \
        if (dbg) {                                                                   \
            __syncthreads();                                                         \
            const u64 _t = __builtin_readcyclecounter();                             \
            if (tid == 0) L.dbgc[slot] += (u32)(_t - t_last);                     \
            t_last = _t;                                                             \
        }                                                                            \
    } while (0)

__device__ __forceinline__ bool tok_is_marker(u32 t) { return (t & 0xC0000000u) == 0x40000000u; }
__device__ __forceinline__ u32 tok_len(u32 t) { return (t & T_MATCH) ? ((t >> 16) & 0xFF) + 3 : 1; }
__device__ __forceinline__ u32 tok_dist(u32 t) { return (t & 0x7FFF) + 1; }
// stream bits of a literal/match token (bits 24..29; <= 48)
__device__ __forceinline__ u32 tok_bits(u32 t) { return (t >> 24) & 63; }

// Round-stage entries (u16): E_VAL|byte is a final byte value; a value below
// PI_STAGE points at an earlier byte of the same round (offset from the round
// start); E_FAR + k - 1 stands for the byte k (1..32768) positions before the
// round start, read back from the chunk's committed output.
constexpr u32 E_VAL = 0xFF00u;
constexpr u32 E_FAR = 0x4000u;
static_assert(PI_STAGE <= E_FAR && E_FAR + PI_WIN <= E_VAL, "stage entry encoding");
__device__ __forceinline__ bool e_val(u32 v) { return v >= E_VAL; }

// 50 KiB: three chunks' workgroups per CU (12 waves).  The token lists live in a
// per-workgroup slot of the HBM workspace (coalesced [token][lane] layout,
// L2-resident while the chunk decodes), not in LDS.
struct ParLds {
    // The staged stream and the segment marks are dead after pass 2, the round
    // bytes are first written by placement: they share storage (and the
    // dynamic-header scratch lives there between rounds).
    union {
        u16 ptr[PI_STAGE];               // round bytes (E_VAL / pointer / E_FAR entries); header scratch
        struct {
            u32 in[PI_IN_PAD];               // staged stream words (padded: in[padw(w)])
            u32 mark[PI_NL * (PI_SEGW + 1)]; // token-start bitmap of each lane's segment (+1 pad)
        };
    };
    u32 head[PI_STAGE / 32];         // token-start bitmap over the round's output bytes
    u32 ltab[INF_LTAB];
    u32 dtab[INF_DTAB];
    HuffLds lh, dh;
    u8 lens[320];
    u32 bcache[(PI_NL / 64) * BI_CACHE_WORDS];  // one bit-reader cache per wave
    u32 next[PI_NL];                 // sync target lane, or a stop code
    u32 endp[PI_NL];                 // bit where the lane stopped
    u32 give[PI_NL];                 // index of the sync token in the target's list
    u32 sidx[PI_NL];                 // first valid token of the lane
    u32 ntok[PI_NL];
    unsigned long long anom[PI_NL / 64];
    u32 seg_s[PI_MAXSEG], seg_e[PI_MAXSEG];  // chain segments [s, e] (lane ranges)
    u32 wsum[8];
    u32 ctl[16];
    u32 dbgc[32];                    // debug counters of this chunk (flushed at the end)
};
// debug counter add (LDS atomic; flushed to g_inf_dbg once per chunk)
#define DBG_ADD(slot, v) atomicAdd(&L.dbgc[slot], (u32)(v))

static_assert(sizeof(ParLds) <= 53 * 1024, "ParLds must leave room for three workgroups per CU");

// Per-workgroup token slots in the workspace: slot s holds PI_TMAX x PI_NL
// token words, token j of lane i at [j * PI_NL + i].  A workgroup takes a
// free slot when it starts (owner word 0 -> 1) and frees it when it ends; the
// launcher zeroes the owner words before each launch.
constexpr u32 PI_NSLOT = 1024;  // > the 768 workgroups three per CU (256 CUs) keep resident
constexpr u64 PI_SLOT_WORDS = (u64)PI_TMAX * PI_NL;
constexpr u64 PI_OWNER_BYTES = PI_NSLOT * 4;

// Decode one token from a bit buffer holding >= 48 valid bits: <= 2 LDS
// lookups for the literal/length code, <= 2 for the distance code.
__device__ __forceinline__ u32 decode_token(const ParLds& L, u64 v, u32* adv) {
    const u32 e = table_lookup(L.ltab, INF_LBITS, (u32)v);
    const u32 l = e >> 28;
    const u32 kind = (e >> 24) & 15;
    if (kind == K_LIT) { *adv = l; return (l << 24) | (e & 0xFF); }
    if (kind == K_EOB) { *adv = l; return T_EOB; }
    if (kind != K_LEN) { *adv = l ? l : 1; return T_BAD; }
    const u32 ex = (e >> 16) & 0xFF;
    const u32 len = (e & 0xFFFF) + ((u32)(v >> l) & ((1u << ex) - 1));
    const u32 t = l + ex;
    const u64 vd = v >> t;
    const u32 de = table_lookup(L.dtab, INF_DBITS, (u32)vd);
    const u32 dl = de >> 28;
    if (((de >> 24) & 15) != K_DIST) { *adv = t + (dl ? dl : 1); return T_BAD; }
    const u32 dex = (de >> 16) & 0xFF;
    const u32 dist = (de & 0xFFFF) + ((u32)(vd >> dl) & ((1u << dex) - 1));
    *adv = t + dl + dex;
    return T_MATCH | ((t + dl + dex) << 24) | ((len - 3) << 16) | (dist - 1);
}

// decode_token without control flow on the token kind: both table lookups
// always run (the distance one is ignored for literals), so lanes of a wave
// holding different kinds do not serialise.
__device__ __forceinline__ u32 decode_token_fast(const ParLds& L, u64 v, u32* adv) {
    u32 e = L.ltab[(u32)v & ((1u << INF_LBITS) - 1)];
    if (((e >> 24) & 15) == K_SUB)
        e = L.ltab[(e & 0xFFFF) + (((u32)v >> INF_LBITS) & ((1u << ((e >> 16) & 0xFF)) - 1))];
    const u32 l = e >> 28, kind = (e >> 24) & 15, ex = (e >> 16) & 0xFF;
    const u32 t = l + ex;
    const u64 vd = v >> t;
    u32 de = L.dtab[(u32)vd & ((1u << INF_DBITS) - 1)];
    if (((de >> 24) & 15) == K_SUB)
        de = L.dtab[(de & 0xFFFF) + (((u32)vd >> INF_DBITS) & ((1u << ((de >> 16) & 0xFF)) - 1))];
    const u32 dl = de >> 28, dex = (de >> 16) & 0xFF;
    const u32 len = (e & 0xFFFF) + ((u32)(v >> l) & ((1u << ex) - 1));
    const u32 dist = (de & 0xFFFF) + ((u32)(vd >> dl) & ((1u << dex) - 1));
    const u32 madv = t + dl + dex;
    const bool dok = ((de >> 24) & 15) == K_DIST;
    u32 tk = T_BAD, a = l ? l : 1;
    if (kind == K_LIT) { tk = (l << 24) | (e & 0xFF); a = l; }
    if (kind == K_EOB) tk = T_EOB;
    if (kind == K_LEN) {
        tk = dok ? (T_MATCH | (madv << 24) | ((len - 3) << 16) | (dist - 1)) : T_BAD;
        a = dok ? madv : t + (dl ? dl : 1);
    }
    *adv = a;
    return tk;
}

// Token j of lane i in the workgroup's slot.
__device__ __forceinline__ u32 tok_at(const gu32* gp, u32 i, u32 j) { return gp[j * PI_NL + i]; }

// Register bit buffer over the staged words: a 96-bit window (lo:hi) holding
// bits [q, q+nb) of the stream; lb_fill keeps nb >= 48 (one token's worst
// case: 15+5 bits of length, 15+13 bits of distance), so a token decodes from
// `lo` alone with no LDS read on its critical path.
struct LaneBits {
    u64 lo;
    u32 hi;
    u32 nb;
    u32 w;   // staged word after `nw`
    u32 nw;  // next staged word to append (prefetched one fill ahead)
};

__device__ __forceinline__ void lb_init(LaneBits& s, const u32* in, u32 q, u32 bit0) {
    const u32 rel = q - bit0;
    const u32 w = rel >> 5, sh = rel & 31;
    const u64 a = ((u64)in[padw(w + 1)] << 32) | in[padw(w)];
    const u32 c = in[padw(w + 2)];
    s.lo = sh ? (a >> sh) | ((u64)c << (64 - sh)) : a;
    s.hi = sh ? c >> sh : c;
    s.nb = 96 - sh;
    s.nw = in[padw(w + 3)];
    s.w = w + 4;
}
__device__ __forceinline__ void lb_fill(LaneBits& s, const u32* in) {
    if (s.nb <= 64) {
        const u32 v = s.nw;
        s.nw = in[padw(s.w++)];
        if (s.nb < 64) {
            s.lo |= (u64)v << s.nb;
            if (s.nb > 32) s.hi = v >> (64 - s.nb);
            else s.hi = 0;  // nb <= 32: v fits in lo entirely
        } else {
            s.hi = v;
        }
        s.nb += 32;
    }
}
__device__ __forceinline__ void lb_drop(LaneBits& s, u32 k) {  // 0 < k <= 48
    s.lo = (s.lo >> k) | ((u64)s.hi << (64 - k));
    s.hi = k >= 32 ? 0u : (s.hi >> k);
    s.nb -= k;
}

// Flush the resolved round bytes [from, to) to dst (byte-order transform
// fused; bool normalisation is deferred to the end of the chunk because the
// committed bytes double as the LZ77 window).  ptr[] is indexed by absolute
// pos & mask.  The trailing barrier makes the bytes visible to the next
// round's window reads (same workgroup, same CU).
__device__ void par_commit(ParLds& L, u8* dst, u64 from, u64 to, DType t) {
    const u32 tid = threadIdx.x;
    __syncthreads();
    const u64 a16 = (from + 15) & ~15ull, b16 = to & ~15ull;
    if (a16 < b16) {
        for (u64 p = a16 + (u64)tid * 16; p < b16; p += PI_NL * 16) {
            const u32 i = (u32)(p & (PI_STAGE - 1));
            const u32x4 lo = *(const u32x4*)(L.ptr + i);
            const u32x4 hi = *(const u32x4*)(L.ptr + i + 8);
            // each u32 holds two 16-bit entries; keep their low bytes
            auto pk = [](u32 a, u32 b) -> u32 {
                return __builtin_amdgcn_perm(b, a, 0x06040200u);
            };
            const u32x4 v = u32x4{pk(lo.x, lo.y), pk(lo.z, lo.w), pk(hi.x, hi.y), pk(hi.z, hi.w)};
            st16(dst + p, transform16(v, t));
        }
    }
    const u64 e0 = a16 < b16 ? a16 : to;
    for (u64 q = from + tid; q < e0; q += PI_NL) dst[swap_pos(q, t)] = (u8)L.ptr[q & (PI_STAGE - 1)];
    if (a16 < b16)
        for (u64 q = b16 + tid; q < to; q += PI_NL) dst[swap_pos(q, t)] = (u8)L.ptr[q & (PI_STAGE - 1)];
    __syncthreads();
}

// Bool arrays: byte != 0 over the whole decoded chunk, after the last round.
__device__ void par_bool_norm(u8* dst, u64 D) {
    __syncthreads();
    const u32 tid = threadIdx.x;
    const bool al = (((uintptr_t)dst) & 15) == 0;
    for (u64 p = (u64)tid * 16; p < D; p += PI_NL * 16) {
        if (p + 16 <= D) {
            u32x4 v = al ? *(u32x4*)(dst + p) : ld16(dst + p);
            v.x = bool_norm32(v.x); v.y = bool_norm32(v.y); v.z = bool_norm32(v.z); v.w = bool_norm32(v.w);
            if (al) *(u32x4*)(dst + p) = v; else st16(dst + p, v);
        } else {
            for (u64 q = p; q < D; q++) dst[q] = dst[q] != 0;
        }
    }
}

// Block-wide exclusive scan over 256 lanes; *total receives the sum.
__device__ __forceinline__ u32 block_excl_scan(ParLds& L, u32 v, u32* total) {
    const int lane = lane_id();
    const u32 wv = threadIdx.x >> 6;
    u32 x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) L.wsum[wv] = x;
    __syncthreads();
    u32 off = 0, tot = 0;
    for (u32 k = 0; k < PI_NL / 64; k++) {
        const u32 s = L.wsum[k];
        if (k < wv) off += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + x - v;
}

// ---- dynamic block header, block-parallel --------------------------------------------
// Same validity rules and result codes as read_dynamic (zcg_inflate_common.h),
// in the same order.  The code-length symbols (<= 316 of <= 14 bits) are
// decoded at EVERY bit position of the header region at once; one lane then
// walks the true chain through those records (one LDS read per symbol) and the
// block expands the repeat codes in parallel.
constexpr u32 HD_BITS = 4608;            // >= 316 symbols * 14 bits
constexpr u32 HD_WORDS = HD_BITS / 32 + 8;
static_assert(3 * HD_BITS * 2 + (HD_WORDS + 128 + 320) * 4 <= PI_STAGE * 2, "header scratch fits in ptr[]");

__device__ __attribute__((always_inline)) int read_dynamic_par(ParLds& L, BitIn& b, bool dbg) {
    const u32 tid = threadIdx.x;
    u64 hts = __builtin_readcyclecounter();
    if (!bi_has(b, 14)) return R_EXHAUSTED;
    const u32 nlen = bi_bits(b, 5) + 257, ndist = bi_bits(b, 5) + 1, ncode = bi_bits(b, 4) + 4;
    if (nlen > 286 || ndist > 30) return R_INVALID;  // "too many length or distance symbols"
    if (!bi_has(b, 3 * ncode)) return R_EXHAUSTED;
    // the 3-bit code-length code lengths: lane i < ncode reads its own field
    const u64 c0 = b.consumed;
    u32 mycl = 0;
    {
        bi_refill(b);  // >= 33 bits buffered; 3*19 = 57 may need a second word
        const u32 lane = tid & 63;
        const u64 w = b.buf;
        u32 v = 0;
        if (lane < ncode) {
            const u32 at = 3 * lane;
            v = at + 3 <= b.cnt ? (u32)(w >> at) & 7 : 0xFFFFFFFFu;
        }
        const bool need = __ballot(v == 0xFFFFFFFFu) != 0;
        if (need) {  // rare: read the rest through the word reader
            const u32 lo = b.cnt;
            bi_drop(b, lo - lo % 3);
            bi_refill(b);
            if (v == 0xFFFFFFFFu) v = (u32)(b.buf >> (3 * lane - (lo - lo % 3))) & 7;
        }
        mycl = v;
        bi_seek(b, c0 + 3 * ncode);
    }
    {  // code-length code must be complete ("invalid code lengths set")
        const u32 lane = tid & 63;
        int left = 1;
        for (u32 l = 1; l <= 7; l++) {
            const u32 cnt = (u32)__popcll(__ballot(lane < ncode && mycl == l));
            left <<= 1;
            left -= (int)cnt;
            if (left < 0) break;
        }
        if (left != 0) return R_INVALID;
        __syncthreads();
        if (tid < 19) L.lens[tid] = 0;
        __syncthreads();
        if (tid < ncode) L.lens[c_clen_order[tid]] = (u8)mycl;
    }
    // stage the region [H0, H0 + HD_BITS) of the stream (header scratch lives
    // in the round arrays, which are free between rounds)
    const u64 H0 = b.consumed;
    const u64 B0 = H0 >> 3;
    const u32 o = (u32)(H0 & 7);
    // header scratch, all inside ptr[] (bytes): rec [0, 9216), rec4 [9216, 27648),
    // hw [27648, 28256), gpos [28256, 28768), srec [28768, 30048)
    u32* hw = (u32*)(L.ptr + 3 * HD_BITS);
    for (u32 w = tid; w < HD_WORDS; w += PI_NL) {
        const u64 q = B0 + 4ull * w;
        u32 v = 0;
        if (q + 4 <= b.n) v = ld32(b.src + q);
        else
            for (u32 k = 0; k < 4; k++)
                if (q + k < b.n) v |= (u32)b.src[q + k] << (8 * k);
        hw[w] = v;
    }
    build_table(L.lens, 19, &L.lh, L.ltab, 7, false, INF_LTAB);  // barriers inside
    // one record per bit position: adv | codelen << 4 | sym << 7 (the repeat
    // count is re-derived from the stream bits by hd_cnt)
    u16* rec = L.ptr;
    auto hd_v = [&](u32 r) -> u32 {
        const u32 bit = o + r, w = bit >> 5, sh = bit & 31;
        return (u32)((((u64)hw[w + 1] << 32) | hw[w]) >> sh) & 0x3FFF;
    };
    auto hd_cnt = [&](u32 r, u32 f) -> u32 {  // f = rec[r]
        const u32 l = (f >> 4) & 7, sym = f >> 7, x = hd_v(r) >> l;
        return sym == 16 ? 3 + (x & 3) : sym == 17 ? 3 + (x & 7) : sym == 18 ? 11 + (x & 127) : 1;
    };
    for (u32 r = tid; r < HD_BITS; r += PI_NL) {
        const u32 v = hd_v(r);
        const u32 e = L.ltab[v & 127];
        const u32 l = e >> 28, sym = e & 0x1F;
        const u32 adv = sym == 16 ? l + 2 : sym == 17 ? l + 3 : sym == 18 ? l + 7 : l;
        rec[r] = (u16)(adv | (l << 4) | (sym << 7));
    }
    __syncthreads();
    // 4-symbol jumps: pos (13 bits) | summed count << 13 (positions past the
    // region read the last record, as zlib's reader would run out there)
    auto cl = [](u32 r) -> u32 { return r < HD_BITS ? r : HD_BITS - 1; };
    u32* rec4 = (u32*)(L.ptr + HD_BITS);
    for (u32 r = tid; r < HD_BITS; r += PI_NL) {
        const u32 a0 = rec[r];
        const u32 r1 = r + (a0 & 15), r1c = cl(r1);
        const u32 a1 = rec[r1c];
        const u32 r2 = cl(r1 + (a1 & 15));
        const u32 a2 = rec[r2];
        const u32 q1 = r2 + (a2 & 15), q1c = cl(q1);
        const u32 a3 = rec[q1c];
        const u32 c = hd_cnt(r, a0) + hd_cnt(r1c, a1) + hd_cnt(r2, a2) + hd_cnt(q1c, a3);
        rec4[r] = (q1 + (a3 & 15)) | (c << 13);
    }
    __syncthreads();
    // the walk over groups of 4 symbols: gpos[g] = start bit | out index << 13
    u32* gpos = hw + HD_WORDS;  // <= 79 groups (each covers >= 4 symbol indices)
    const u32 total = nlen + ndist;
    if (dbg && tid == 0) { const u64 t = __builtin_readcyclecounter(); L.dbgc[26] += (u32)(t - hts); hts = t; }
    if (tid == 0) {
        u32 r = 0, idx = 0, g = 0;
        while (idx < total) {
            const u32 f = rec4[cl(r)];
            gpos[g++] = r | (idx << 13);
            idx += f >> 13;
            r = f & 8191;
        }
        L.ctl[1] = g;
        L.ctl[0] = 0xFFFFFFFFu;  // min (symbol << 2 | error code)
        L.ctl[2] = 0;            // symbols
        L.ctl[3] = 0;            // end bit
    }
    __syncthreads();
    // expand the groups: symbol i = 4g + k while its out index < total
    u32* srec = gpos + 128;  // idx | cnt << 9 | sym << 17 (<= 316 symbols)
    {
        const u64 lim64 = b.limit - H0;
        const u32 lim = lim64 < HD_BITS ? (u32)lim64 : HD_BITS;
        const u32 ng = L.ctl[1];
        for (u32 g = tid; g < ng; g += PI_NL) {
            u32 r = gpos[g] & 8191, idx = gpos[g] >> 13;
            for (u32 k = 0; k < 4 && idx < total; k++) {
                const u32 rc = cl(r);
                const u32 f = rec[rc];
                const u32 adv = f & 15, l = (f >> 4) & 7, sym = f >> 7, cnt = hd_cnt(rc, f);
                const u32 i = 4 * g + k;
                u32 err = 0;  // zlib's checks in order: code bits, repeat at 0, extra bits, overflow
                if (r + l > lim) err = 1 + R_EXHAUSTED;
                else if (sym == 16 && idx == 0) err = 1 + R_INVALID;
                else if (r + adv > lim) err = 1 + R_EXHAUSTED;
                else if (idx + cnt > total) err = 1 + R_INVALID;
                if (err) atomicMin(&L.ctl[0], (i << 2) | (err - 1));
                srec[i] = idx | (cnt << 9) | (sym << 17);
                if (idx + cnt >= total) { L.ctl[2] = i + 1; L.ctl[3] = r + adv; }
                idx += cnt;
                r += adv;
            }
        }
    }
    __syncthreads();
    const u32 em = L.ctl[0];
    const u32 nsyms = L.ctl[2], rend = L.ctl[3];
    if (dbg && tid == 0) { const u64 t = __builtin_readcyclecounter(); L.dbgc[27] += (u32)(t - hts); hts = t; }
    if (em != 0xFFFFFFFFu) return (int)(em & 3);  // (the reader position no longer matters)
    for (u32 i = tid; i < nsyms; i += PI_NL) {
        const u32 f = srec[i];
        const u32 idx = f & 511, cnt = (f >> 9) & 255, sym = f >> 17;
        u32 val = sym < 16 ? sym : 0u;
        if (sym == 16) {  // repeat the previous length: nearest earlier non-16 symbol
            u32 j = i;
            u32 sj = 16;
            while (sj == 16 && j > 0) sj = srec[--j] >> 17;
            val = sj < 16 ? sj : 0u;
        }
        for (u32 k = 0; k < cnt; k++) L.lens[idx + k] = (u8)val;
    }
    bi_seek(b, H0 + rend);
    __syncthreads();
    u8 dl = 0;
    if (tid < ndist) dl = L.lens[nlen + tid];
    __syncthreads();
    for (u32 i = nlen + tid; i < 288; i += PI_NL) L.lens[i] = 0;
    if (tid < 32) L.lens[288 + tid] = tid < ndist ? dl : 0;
    __syncthreads();
    if (L.lens[256] == 0) return R_INVALID;  // "invalid code -- missing end-of-block"
    if (build_table(L.lens, 288, &L.lh, L.ltab, INF_LBITS, false, INF_LTAB) != 0) return R_INVALID;
    if (build_table(L.lens + 288, 30, &L.dh, L.dtab, INF_DBITS, true, INF_DTAB) != 0) return R_INVALID;
    if (dbg && tid == 0) { const u64 t = __builtin_readcyclecounter(); L.dbgc[28] += (u32)(t - hts); hts = t; }
    return R_OK;
}

// read_block_header with the block-parallel dynamic header
__device__ __attribute__((always_inline)) int read_block_header_par(ParLds& L, BitIn& b, bool* last, u32* type, u32* slen, bool dbg) {
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
    if (*type == 1) { fixed_tables(L.lens, &L.lh, L.ltab, &L.dh, L.dtab); return R_OK; }
    return read_dynamic_par(L, b, dbg);
}

__global__ __launch_bounds__(PI_NL, ZCG_INF_WPE) void inflate_par_kernel(const zcg_chunk* __restrict__ chunks,
                                                               u32 n, u64 D, DType t, u32 vflags,
                                                               i32* __restrict__ status,
                                                               u32* __restrict__ owner, gu32* __restrict__ pools) {
    extern __shared__ __attribute__((aligned(16))) u8 smem_raw[];
    ParLds& L = *(ParLds*)smem_raw;
    const u32 c = blockIdx.x;
    if (c >= n) return;
    const u32 tid = threadIdx.x;
    const bool dbg = (vflags & ZCG_FLAG_DEBUG_COUNTERS) != 0;
    const zcg_chunk ch = chunks[c];
    if (D == 0) { if (tid == 0) status[c] = ZCG_OK; return; }
    if (ch.dst_cap < D) { if (tid == 0) status[c] = ZCG_ERR_INVALID_INPUT; return; }
    const u8* s = (const u8*)ch.src;
    const u64 n_in = ch.src_len;
    u64 h = 0;
    int st = gzip_header(s, n_in, &h);
    if (st == ZCG_OK && n_in - h >= (1ull << 28)) st = ZCG_ERR_UNSUPPORTED;  // u32 bit positions
    if (st != ZCG_OK) { if (tid == 0) status[c] = st; return; }

    u8* dst = (u8*)ch.dst;
    const u8* ds = s + h;  // deflate stream
    DType tw = t;  // commit transform: bool waits for the end (the output is the window)
    tw.isbool = 0;
    // take a token slot (released at the end; every path below reaches it)
    if (tid == 0) {
        u32 sl = c % PI_NSLOT;
        while (atomicCAS(&owner[sl], 0u, 1u) != 0u) sl = (sl + 1) % PI_NSLOT;
        L.ctl[15] = sl;
    }
    __syncthreads();
    const u32 slot = L.ctl[15];
    gu32* const gp = pools + (u64)slot * PI_SLOT_WORDS;
    const u64 n_ds = n_in - h;
    const u32 total_bits = (u32)(n_ds * 8);
    // Every wave runs the wave-uniform header/look-ahead code redundantly on
    // the same data (block barriers inside), each with its own LDS cache.
    BitIn b;
    bi_init(b, ds, n_ds, L.bcache + (tid >> 6) * BI_CACHE_WORDS);
    u64 P = 0;
    bool last = false, boundary = false, after_stored = false;
    int r = R_OK;
    if (dbg) {
        if (tid < 32) L.dbgc[tid] = 0;
        if (tid == 0) L.ctl[13] = 0;
        __syncthreads();
    }
    u64 t_last = __builtin_readcyclecounter();
    const u64 t_start = t_last;

    while (r == R_OK && P < D) {
        TSTAMP(TP_COMMIT);
        // ---- block header (all waves, identical) ------------------------------------
        if (last) { r = R_EXHAUSTED; break; }
        u32 type = 0, slen = 0;
        r = read_block_header_par(L, b, &last, &type, &slen, dbg);
        const u32 hdr_end = (u32)b.consumed;
        TSTAMP(TP_HDR);
        if (r != R_OK) break;
        if (dbg && tid == 0) DBG_ADD(DBG_BLOCKS, 1);
        if (type == 0) {
            // ---- stored block: byte copies through the stage --------------------
            u64 in0 = hdr_end >> 3;  // byte aligned after LEN/NLEN
            u32 done = 0;
            while (done < slen && P < D) {
                u32 k = slen - done;
                if (k > PI_STAGE) k = PI_STAGE;
                if ((u64)k > D - P) k = (u32)(D - P);
                if (in0 + k > n_ds) { r = R_EXHAUSTED; break; }
                for (u32 i = tid; i < k; i += PI_NL)
                    L.ptr[(P + i) & (PI_STAGE - 1)] = (u16)(E_VAL | ds[in0 + i]);
                par_commit(L, dst, P, P + k, tw);
                P += k; in0 += k; done += k;
            }
            if (r != R_OK) break;
            bi_seek(b, in0 * 8);
            boundary = (done == slen);
            after_stored = true;
            continue;
        }
        after_stored = false;
        // ---- Huffman block body: speculative parallel rounds -------------------
        u32 R0 = hdr_end;
        bool block_end = false;
        while (!block_end && r == R_OK && P < D) {
            const u32 bit0 = R0 & ~127u;  // 16-byte aligned stream offset
            const u64 byte0 = bit0 >> 3;
            {
                u32x4 v[(PI_IN_VEC + PI_NL - 1) / PI_NL];
#pragma unroll
                for (u32 k = 0; k < (PI_IN_VEC + PI_NL - 1) / PI_NL; k++) {
                    const u32 vi = tid + k * PI_NL;
                    const u64 q = byte0 + 16ull * vi;
                    u32x4 x = {0u, 0u, 0u, 0u};
                    if (vi < PI_IN_VEC) {
                        if (q + 16 <= n_ds) x = ld16(ds + q);
                        else {
                            u64 lo = 0, hi = 0;
                            for (u32 i = 0; i < 16; i++)
                                if (q + i < n_ds) {
                                    const u64 b8 = (u64)ds[q + i] << (8 * (i & 7));
                                    if (i < 8) lo |= b8; else hi |= b8;
                                }
                            x = u32x4{(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
                        }
                    }
                    v[k] = x;
                }
#pragma unroll
                for (u32 k = 0; k < (PI_IN_VEC + PI_NL - 1) / PI_NL; k++) {
                    const u32 vi = tid + k * PI_NL;
                    if (vi < PI_IN_VEC) {
                        const u32 w = 4 * vi;  // 4 words never straddle a pad (pads after 8)
                        u32* d = L.in + padw(w);
                        d[0] = v[k].x; d[1] = v[k].y; d[2] = v[k].z; d[3] = v[k].w;
                    }
                }
            }
            for (u32 k = tid; k < PI_STAGE / 32; k += PI_NL) L.head[k] = 0;
            for (u32 k = tid; k < PI_NL * (PI_SEGW + 1); k += PI_NL) L.mark[k] = 0;
            __syncthreads();
            TSTAMP(TP_STAGE);

            // ---- pass 1: decode my own segment, mark token starts ----------------
            const u32 p = R0 + tid * PI_SEG;
            const u32 pend = p + PI_SEG;
            u32* mymark = L.mark + tid * (PI_SEGW + 1);
            LaneBits bs;
            lb_init(bs, L.in, p, bit0);
            u32 q = p, nt = 0, olen_all = 0;  // olen_all: output bytes of all stored tokens
            u32 nxt = 0xFFFFFFFFu;
            // append a token; false when the lane's token store is full
            auto push = [&](u32 tk) -> bool {
                if (nt == PI_TMAX) return false;
                gp[nt * PI_NL + tid] = tk;
                nt++;
                olen_all += tok_len(tk);
                return true;
            };
            while (q < pend) {
                lb_fill(bs, L.in);
                u32 adv;
                u32 tk = decode_token_fast(L, bs.lo, &adv);
                if (q + adv > total_bits) tk = T_EXH;
                if (!push(tk)) { nxt = N_CAP; break; }
                const u32 off = q - p;
                atomicOr(&mymark[off >> 5], 1u << (off & 31));
                if (tok_is_marker(tk)) {
                    if (tk == T_EOB) q += adv;
                    nxt = N_MARKER;
                    break;
                }
                lb_drop(bs, adv);
                q += adv;
            }
            __syncthreads();
            TSTAMP(TP_PASS1);
            // ---- pass 2: follow my path until it meets a marked token start -----
            const u32 round_hi = R0 + PI_NL * PI_SEG;
            u32 give = 0, p2tok = 0;
            while (nxt == 0xFFFFFFFFu) {
                if (q >= round_hi) { nxt = N_ROUND_END; break; }
                const u32 rel = q - R0;
                const u32 k = rel / PI_SEG, off = rel % PI_SEG;
                const u32* km = L.mark + k * (PI_SEGW + 1);
                const u32 mw = km[off >> 5];
                lb_fill(bs, L.in);
                u32 adv;
                u32 tk = decode_token_fast(L, bs.lo, &adv);  // (discarded on a sync)
                if (mw & (1u << (off & 31))) {
                    // sync: index of that token in lane k's list = marks below it
                    u32 cnt = __popc(mw & ((1u << (off & 31)) - 1));
                    for (u32 x = 0; x < (off >> 5); x++) cnt += __popc(km[x]);
                    nxt = k;
                    give = cnt;
                    break;
                }
                if (q + adv > total_bits) tk = T_EXH;
                if (!push(tk)) { nxt = N_CAP; break; }
                p2tok++;
                if (tok_is_marker(tk)) {
                    if (tk == T_EOB) q += adv;
                    nxt = N_MARKER;
                    break;
                }
                lb_drop(bs, adv);
                q += adv;
            }
            // prefetch the lane's first PF tokens into registers: the loads
            // overlap the chain phase's barriers (placement usually needs no more)
            constexpr u32 PF = ZCG_INF_PF;
            u32 pre[PF];
#pragma unroll
            for (u32 u = 0; u < PF; u++) pre[u] = u < nt ? tok_at(gp, tid, u) : 0u;
            L.next[tid] = nxt;
            L.endp[tid] = q;
            L.give[tid] = give;
            L.ntok[tid] = nt;
            if (dbg) {
                DBG_ADD(p2tok < 8 ? 29 : p2tok < 16 ? 30 : p2tok < 32 ? 31 : p2tok < 48 ? 13 : 14, 1);
                DBG_ADD(DBG_PASS2_TOK, p2tok);
                atomicMax(&L.ctl[13], p2tok);

            }
            __syncthreads();
            TSTAMP(TP_PASS2);

            // ---- chain: lane 0 is true; follow sync targets --------------------------
            // Common case next[i] == i+1; one thread walks only the exceptions.
            {
                const bool an = nxt != tid + 1;
                const unsigned long long bm = __ballot(an);
                if ((tid & 63) == 0) L.anom[tid >> 6] = bm;
            }
            __syncthreads();
            if (tid == 0) {
                u32 curl = 0, ns = 0, endl = 0;
                for (;;) {
                    // first anomaly >= curl
                    u32 a = PI_NL - 1;
                    for (u32 w = curl >> 6; w < PI_NL / 64; w++) {
                        unsigned long long m = L.anom[w];
                        if (w == (curl >> 6)) m &= ~0ull << (curl & 63);
                        if (m) { a = w * 64 + __builtin_ctzll(m); break; }
                    }
                    L.seg_s[ns] = curl;
                    L.seg_e[ns] = a;
                    ns++;
                    const u32 nx = L.next[a];
                    if (nx < PI_NL && ns < PI_MAXSEG) { curl = nx; continue; }
                    endl = a;
                    break;
                }
                L.ctl[5] = endl;
                L.ctl[12] = ns;
            }
            __syncthreads();
            {
                const u32 ns = L.ctl[12];
                u32 sx = 0xFFFFFFFFu;
                for (u32 k = 0; k < ns; k++) {
                    const u32 s0 = L.seg_s[k], e0 = L.seg_e[k];
                    if (tid >= s0 && tid <= e0) {
                        if (tid == 0) sx = 0;
                        else if (tid == s0) sx = L.give[L.seg_e[k - 1]];  // jump target
                        else sx = L.give[tid - 1];
                    }
                }
                L.sidx[tid] = sx;
            }
            __syncthreads();
            const u32 E = L.ctl[5];
            TSTAMP(TP_CHAIN);
            if (dbg && tid == 0) {
                DBG_ADD(DBG_ROUNDS, 1);
                DBG_ADD(DBG_P2_MAX, L.ctl[13]);
                L.ctl[13] = 0;

                DBG_ADD(DBG_CHAIN, E + 1);
                const u32 nx = L.next[E];
                DBG_ADD(nx == N_CAP ? DBG_END_CAP : nx == N_ROUND_END ? DBG_END_ROUND
                        : (tok_at(gp, E, L.ntok[E] - 1) == T_EOB ? DBG_END_EOB : DBG_END_BAD), 1);
                u32 sk = 0;
                for (u32 x = 0; x < E; x++) sk += L.next[x] != x + 1;
                DBG_ADD(DBG_SKIPS, sk);
            }
            const u32 my_s = L.sidx[tid];
            const bool on = (tid <= E) && my_s != 0xFFFFFFFFu;
            u32 vend = nt;
            u32 marker = 0;
            if (on && tid == E && nxt == N_MARKER) { vend = nt - 1; marker = tok_at(gp, tid, nt - 1); }
            // ---- placement ------------------------------------------------------------------
            // output bytes of my valid tokens [my_s, vend): the running sum minus
            // the tokens before my sync point (few) and a trailing marker
            u32 olen = 0;
            if (on) {
                olen = olen_all - (vend < nt ? 1u : 0u);
#pragma unroll
                for (u32 u = 0; u < PF; u++)
                    if (u < my_s) olen -= tok_len(pre[u]);
                for (u32 a0 = PF; a0 < my_s; a0 += 4) {
                    u32 tk4[4];
#pragma unroll
                    for (u32 u = 0; u < 4; u++) tk4[u] = a0 + u < my_s ? tok_at(gp, tid, a0 + u) : 0u;
#pragma unroll
                    for (u32 u = 0; u < 4; u++)
                        if (a0 + u < my_s) olen -= tok_len(tk4[u]);
                }
            }
            u32 total;
            const u32 base = block_excl_scan(L, olen, &total);
            const u64 room = D - P;
            const u32 cap = room < PI_STAGE ? (u32)room : PI_STAGE;
            u32 take_end = on ? vend : my_s;
            u32 emitted = total;
            u32 round_end = L.endp[E];
            if (tid == E) L.ctl[6] = marker;
            __syncthreads();
            u32 mk = L.ctl[6];
            bool final_round = false, fin_boundary = false;
            const bool cut = total > cap || (total == cap && cap == room);
            if (cut) {
                if (dbg && tid == 0) DBG_ADD(DBG_CUTS, 1);
                // the lane whose output range holds byte `cap`
                const bool mine = on && olen > 0 && base < cap && base + olen >= cap;
                if (mine) {
                    // take tokens while they fit below cap (at N: until cap is reached);
                    // the first PF come from registers
                    // sb: stream bits of tokens [0, a), summed as they are taken
                    u32 acc = base, a = my_s, sb = 0;
                    bool go = true;
#pragma unroll
                    for (u32 u = 0; u < PF; u++) {
                        if (u < my_s) sb += tok_bits(pre[u]);
                        if (go && u >= my_s && u < vend) {  // a == u here
                            const u32 len = tok_len(pre[u]);
                            if (cap == room ? acc >= cap : acc + len > cap) go = false;
                            else { acc += len; sb += tok_bits(pre[u]); a++; }
                        }
                    }
                    for (u32 j = PF; j < my_s; j++) sb += tok_bits(tok_at(gp, tid, j));  // rare
                    while (go && a < vend) {
                        u32 tk8[8];
#pragma unroll
                        for (u32 u = 0; u < 8; u++) tk8[u] = a + u < vend ? tok_at(gp, tid, a + u) : 0u;
#pragma unroll
                        for (u32 u = 0; u < 8; u++) {
                            if (go && a < vend) {  // while go holds, a == (a at the load) + u
                                const u32 len = tok_len(tk8[u]);
                                if (cap == room ? acc >= cap : acc + len > cap) go = false;
                                else { acc += len; sb += tok_bits(tk8[u]); a++; }
                            }
                        }
                    }
                    // bit position of the first token not taken: the segment start
                    // plus the stored bit lengths of tokens [0, a), or the lane's end
                    const u32 pos = a < nt ? R0 + tid * PI_SEG + sb : q;
                    L.ctl[7] = (cap == room && acc == cap) ? 1u : 0u;
                    L.ctl[8] = acc < cap ? acc : cap;  // a token may cross N: clip there
                    L.ctl[9] = tid;
                    L.ctl[10] = a;
                    L.ctl[11] = pos;
                }
                __syncthreads();
                const u32 cl = L.ctl[9];
                emitted = L.ctl[8];
                fin_boundary = L.ctl[7] != 0;
                final_round = (cap == room);
                mk = 0;
                if (tid > cl) take_end = my_s;
                if (tid == cl) take_end = L.ctl[10];
                round_end = L.ctl[11];
            }
            // ---- errors on the taken range ----------------------------------------------------
            if (mk == T_BAD) { r = R_INVALID; break; }
            if (mk == T_EXH) { r = R_EXHAUSTED; break; }
            // ---- token heads: one entry per taken token ----------------------------------
            // literal -> E_VAL|byte (final); match -> dist-1 at its first byte,
            // plus a token-start bit in head[] over the round's output bytes.
            const u64 S = P;
            bool far = false;
            {
                u32 o = base;
                u32 hw = 0xFFFFFFFFu, hbits = 0;
                auto put = [&](u32 tk) {
                    u16 v;
                    u32 len;
                    if (tk & T_MATCH) {
                        const u32 d = tok_dist(tk);
                        if (d > P + o) far = true;  // before the stream start
                        v = (u16)(d - 1);
                        len = tok_len(tk);
                    } else {
                        v = (u16)(E_VAL | (tk & 0xFF));
                        len = 1;
                    }
                    L.ptr[(S + o) & (PI_STAGE - 1)] = v;
                    if ((o >> 5) != hw) {
                        if (hbits) atomicOr(&L.head[hw], hbits);
                        hw = o >> 5;
                        hbits = 0;
                    }
                    hbits |= 1u << (o & 31);
                    o += len;
                };
#pragma unroll
                for (u32 u = 0; u < PF; u++)
                    if (u >= my_s && u < take_end) put(pre[u]);
                for (u32 a0 = my_s > PF ? my_s : PF; a0 < take_end; a0 += 8) {
                    u32 tk8[8];
#pragma unroll
                    for (u32 u = 0; u < 8; u++) tk8[u] = a0 + u < take_end ? tok_at(gp, tid, a0 + u) : 0u;
#pragma unroll
                    for (u32 u = 0; u < 8; u++)
                        if (a0 + u < take_end) put(tk8[u]);
                }
                if (hbits) atomicOr(&L.head[hw], hbits);
            }
            if (__syncthreads_or(far)) { r = R_INVALID; break; }
            TSTAMP(TP_PLACE);
            // ---- LZ77 resolution by pointer jumping ---------------------------------------
            // Every round byte gets its value (literal), a pointer to an EARLIER
            // round byte, or a far code (a byte before the round): byte k of a match
            // (start o, distance d) copies B[o - d + (k mod d)], which lies
            // before the match start.  Thread t expands the contiguous byte
            // range [x0, x1), carrying in the match that covers x0.
            {
                // range length ≡ 2 (mod 4) entries: an odd dword stride between
                // threads, so a wave's reads spread over all banks (a full 16 KiB
                // stage gives 64 entries = 32 dwords: every thread in one bank)
                const u32 c0 = (emitted + PI_NL - 1) / PI_NL;
                const u32 ch = c0 + ((2u - c0) & 3u);
                const u32 x0 = tid * ch;
                const u32 x1 = (x0 + ch < emitted) ? x0 + ch : emitted;
                u32 mo = 0, md = 0, mj = 0;  // current match: start, distance, k mod d
                if (x0 < x1 && !((L.head[x0 >> 5] >> (x0 & 31)) & 1u)) {
                    // nearest token start below x0 (a match: <= 258 bytes back)
                    u32 w = x0 >> 5;
                    u32 m = L.head[w] & ((1u << (x0 & 31)) - 1u);
                    while (!m) m = L.head[--w];
                    mo = w * 32 + 31 - __builtin_clz(m);
                    md = (u32)L.ptr[(S + mo) & (PI_STAGE - 1)] + 1;
                    const u32 k0 = x0 - mo - 1;  // the loop steps mj before use
                    mj = k0 < md ? k0 : k0 % md;
                }
                __syncthreads();  // heads are read before any thread rewrites them
                u32 hb = x0 < x1 ? L.head[x0 >> 5] : 0;
                bool in_match = md != 0;
                for (u32 x = x0; x < x1; x++) {
                    if ((x & 31) == 0) hb = L.head[x >> 5];
                    const u32 i = (u32)((S + x) & (PI_STAGE - 1));
                    if ((hb >> (x & 31)) & 1u) {
                        const u16 v = L.ptr[i];
                        if (e_val(v)) { in_match = false; continue; }  // literal: final
                        mo = x; md = (u32)v + 1; mj = 0; in_match = true;
                    } else if (!in_match) {
                        continue;  // unreachable for a well-formed round
                    } else {
                        mj = (mj + 1 == md) ? 0 : mj + 1;
                    }
                    const int sp = (int)mo - (int)md + (int)mj;
                    u16 nv;
                    if (sp < 0) nv = (u16)(E_FAR - 1 + (u32)(-sp));
                    else if ((u32)sp >= x0) nv = L.ptr[(S + (u32)sp) & (PI_STAGE - 1)];  // mine, final
                    else nv = (u16)sp;
                    L.ptr[i] = nv;
                }
            }
            __syncthreads();
            // far codes: read the bytes back from the committed output (the
            // previous rounds' bytes, L2-hot; FU loads in flight per thread)
            constexpr u32 FU = ZCG_INF_FU;  // loads in flight per thread
            for (u32 x = tid; x < emitted; x += FU * PI_NL) {
                u32 v[FU];
                u8 bv[FU];
#pragma unroll
                for (u32 u = 0; u < FU; u++) {
                    const u32 xx = x + u * PI_NL;
                    v[u] = xx < emitted ? (u32)L.ptr[(u32)((S + xx) & (PI_STAGE - 1))] : E_VAL;
                }
#pragma unroll
                for (u32 u = 0; u < FU; u++) {
                    const bool fr = !e_val(v[u]) && v[u] >= E_FAR;
                    bv[u] = fr ? ((const gu8*)dst)[swap_pos(S - (v[u] - E_FAR + 1), tw)] : (u8)0;
                }
#pragma unroll
                for (u32 u = 0; u < FU; u++)
                    if (!e_val(v[u]) && v[u] >= E_FAR)
                        L.ptr[(u32)((S + x + u * PI_NL) & (PI_STAGE - 1))] = (u16)(E_VAL | bv[u]);
            }
            __syncthreads();
            TSTAMP(TP_LIT);
            for (;;) {
                bool pending = false;
                for (u32 x = tid; x < emitted; x += 4 * PI_NL) {
                    u16 v[4], w[4];
#pragma unroll
                    for (u32 u = 0; u < 4; u++) {
                        const u32 xx = x + u * PI_NL;
                        v[u] = xx < emitted ? L.ptr[(u32)((S + xx) & (PI_STAGE - 1))] : (u16)E_VAL;
                    }
#pragma unroll
                    for (u32 u = 0; u < 4; u++)
                        w[u] = e_val(v[u]) ? v[u] : L.ptr[(u32)((S + v[u]) & (PI_STAGE - 1))];
#pragma unroll
                    for (u32 u = 0; u < 4; u++)
                        if (!e_val(v[u])) {
                            L.ptr[(u32)((S + x + u * PI_NL) & (PI_STAGE - 1))] = w[u];
                            pending |= !e_val(w[u]);
                        }
                }
                if (dbg && tid == 0) DBG_ADD(DBG_MRR_IT, 1);
                if (!__syncthreads_or(pending)) break;
            }
            TSTAMP(TP_MRR);
            // ---- commit -------------------------------------------------------------------------------
            par_commit(L, dst, S, S + emitted, tw);
            P = S + emitted;
            if (dbg) {
                if (tid == 0) DBG_ADD(DBG_BYTES, emitted);
                if (take_end > my_s) DBG_ADD(DBG_TOKENS, take_end - my_s);
            }
            if (final_round) {
                boundary = fin_boundary;
                bi_seek(b, round_end);
                break;
            }
            if (mk == T_EOB) {
                block_end = true;
                bi_seek(b, round_end);  // bit after the EOB code
            }
            R0 = round_end;
        }
    }
    // zlib's post-N look-ahead (all waves, identical); see zcg_inflate_common.h
    if (r == R_OK && P >= D && boundary) {
        const u64 last_byte = h + (b.consumed ? (b.consumed - 1) / 8 : 0);
        u64 wend = (last_byte / 32768 + 1) * 32768;
        if (wend > n_in) wend = n_in;
        b.limit = (wend - h) * 8;
        if (b.limit >= b.consumed) {
            const int la = inf_lookahead(b, last, after_stored, L.lens, &L.lh, L.ltab, &L.dh, L.dtab);
            if (la == R_INVALID) r = R_INVALID;
        }
    }
    if (r == R_INVALID) st = ZCG_ERR_INVALID_DATA;
    else if (r == R_EXHAUSTED || P < D) st = ZCG_ERR_UNEXPECTED_EOF;
    if (t.isbool) par_bool_norm(dst, P < D ? P : D);
    if (dbg) {
        if (tid == 0) L.dbgc[TP_TOTAL] = (u32)(__builtin_readcyclecounter() - t_start);
        __syncthreads();
        if (tid < 32 && L.dbgc[tid]) atomicAdd(&g_inf_dbg[tid], (unsigned long long)L.dbgc[tid]);
    }
    __syncthreads();  // every token-slot access of this workgroup is done
    if (tid == 0) {
        status[c] = st;
        atomicExch(&owner[slot], 0u);
    }
}

extern "C" int zcg__debug_inflate_counters(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_inf_dbg), sizeof(unsigned long long) * 32) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_inf_dbg), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}

uint64_t inflate_par_ws_bytes(const zcg_array* a, uint32_t n) {
    (void)a;
    if (n == 0) return 0;
    return PI_OWNER_BYTES + (u64)PI_NSLOT * PI_SLOT_WORDS * 4;
}

const char* cfg_inflate_par() {
    return "inflate_par:PF=" ZCG_STR(ZCG_INF_PF) ",FU=" ZCG_STR(ZCG_INF_FU) ",WPE=" ZCG_STR(ZCG_INF_WPE);
}

hipError_t launch_inflate_par(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                              int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (!ws || ws_bytes < inflate_par_ws_bytes(a, n)) return hipErrorInvalidValue;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const size_t lds = sizeof(ParLds);
    if (hipError_t e = lds_attr_once((const void*)inflate_par_kernel, (int)lds); e != hipSuccess) return e;
    u32* owner = (u32*)ws;  // the workspace is shared by the stream's codecs: clear the owners
    hipError_t e = hipMemsetAsync(owner, 0, PI_OWNER_BYTES, s);
    if (e != hipSuccess) return e;
    gu32* pools = (gu32*)((u8*)ws + PI_OWNER_BYTES);
    hipLaunchKernelGGL(inflate_par_kernel, dim3(n), dim3(PI_NL), lds, s, d_chunks, n, D, t,
                       a->compression.flags, d_status, owner, pools);
    return hipGetLastError();
}

}  // namespace zcg
