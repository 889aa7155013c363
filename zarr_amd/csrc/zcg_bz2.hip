// zcg_bz2.hip — Bzip2Compression decode (src/compression/bzip.rs:35-46,
// bzip2 read::BzDecoder = libbz2 BZ2_bzDecompress) on gfx950.
//
// One 256-thread workgroup per chunk; the chunk's bzip2 blocks are decoded
// one after another, each in three stages:
//   A. (wave 0, zcg_bz2_core.h) block header, selectors, code lengths,
//      Huffman + RUNA/RUNB + move-to-front -> the BWT last column L[nblock]
//      streamed to HBM 64 bytes at a time.  Serial by nature; the Huffman
//      tables are LDS lookups, the MTF list lives in one VGPR per lane and
//      a move-to-front is one DPP wave shift.
//   B. (256 threads) inverse BWT: a stable counting sort of L by wave ballots
//      gives the T^-1 links, stored packed with the sorted byte as
//      W[j] = link << 8 | F[j] (libbz2's tt[] layout; F[j] = L[link]), so one
//      4-byte gather yields both the next position and the next output byte.
//      The output order is a list ranking of the links: 1 024 power-of-two-
//      strided samples (+ the start) are walked in parallel (5 interleaved
//      walks per thread), the sample chain is ranked by one thread, and a
//      second walk writes T[] in output order.  A chain that is not one cycle
//      (corrupt data) falls back to libbz2's serial walk.
//   C. (256 threads) RLE1 as a parallel scan of the 5-state run machine,
//      output offsets by a block scan, byte stores with the '>'/bool
//      transform fused, the block CRC as 256 segment CRCs combined by
//      GF(2) x^(8n) shifts, checked against the stored CRC when the block
//      completes inside D (read_exact semantics, chunk.rs:112-113).
// Workspace: per chunk in flight (4 096) L (900 000 B) + selectors + state;
// per stage-B/C workgroup slot (1 024) T (900 000 B) + W (3.6 MB).
// Algorithmic bytes per chunk: C + D.  Bound: stage A (serial Huffman/MTF),
// not HBM.
#include "zcg_common.h"
#ifdef ZB_DEBUG_TRACE
#define ZB_TRACE(bp, nb, v) do { if (threadIdx.x == 0 && bp < 400) printf("bits bp=%llu nb=%u v=%u\n", (unsigned long long)(bp), (unsigned)(nb), (unsigned)(v)); } while (0)
#endif
#include "zcg_bz2_core.h"

namespace zcg {

constexpr u32 BZ_NMAX = 900000;
constexpr u32 BZ_NSAMP = 1024;
constexpr int BZ_WALKS = BZ_NSAMP / 256 + 1;
#ifndef ZB_KMUL
#define ZB_KMUL 4
#endif
constexpr u32 BZ_KMUL = ZB_KMUL;  // kept bytes per walk, in sample strides
static_assert(BZ_KMUL >= 1 && (BZ_KMUL & (BZ_KMUL - 1)) == 0, "power of two");  // interleaved walks per thread (+ the start)
constexpr u32 BZ_T = 256;
constexpr u64 BZ_LBYTES = 900096;  // L / T capacity (BZ_NMAX rounded up to 256)

constexpr u32 BZ_POLY = 0x04C11DB7u;
struct BzCrcTable {
    u32 t[256];
    constexpr BzCrcTable() : t() {
        for (u32 i = 0; i < 256; i++) {
            u32 c = i << 24;
            for (int k = 0; k < 8; k++) c = (c << 1) ^ ((c & 0x80000000u) ? BZ_POLY : 0u);
            t[i] = c;
        }
    }
};
__constant__ BzCrcTable g_bzcrc = BzCrcTable();

__device__ inline u32 bz_mulmod(u32 a, u32 b) {
    u32 r = 0;
    for (int i = 31; i >= 0; i--) {
        r = (r << 1) ^ ((r & 0x80000000u) ? BZ_POLY : 0u);
        if ((a >> i) & 1) r ^= b;
    }
    return r;
}
__device__ inline u32 bz_xpow8(u64 n) {
    u32 r = 1, p = 0x100;  // x^8
    while (n) {
        if (n & 1) r = bz_mulmod(p, r);
        p = bz_mulmod(p, p);
        n >>= 1;
    }
    return r;
}

// ---- stage A device IO (wave 0) ----------------------------------------------
struct BzDevIO {
    const gu8* src;
    u64 n;
    u64 cbp, bb;          // bit reader (wave-uniform): bits [cbp, cbp + 64), MSB-first
    // The compressed stream is staged in VGPRs, 2 KiB spread over the wave:
    // lane i holds bytes [vb + 16 i, +16) (wc) and [vb + 1024 + 16 i, +16)
    // (wn).  The 16-byte window refills from these with readlane (no memory
    // latency); the next KiB is prefetched when the front one is retired.
    u32x4 wc, wn;
    u64 vb;
    zb::Group* groups;
    lu8* lensb;
    lu8* seq;
    gu8* sel;
    gu8* L;
    u32 sbase, sw0, sw1, sw2, sw3;  // selector window
    u32x4 lt0, lt1, lt2, lt3, lt4, lt5, ltc;  // VGPR Huffman tables (see build_lut)
    u32 ltc_t;
    u32 mtfw;                      // MTF list bytes [4 lane, 4 lane + 4)
    u32 lbuf;                      // pending L bytes, one per lane
    int lane;

    __device__ __forceinline__ u32x4 load16(u64 q) {  // bytes past n read as 0
        if (q + 16 <= n) return *(const gu32x4_ua*)(src + q);
        u64 lo = 0, hi = 0;
        for (u32 i = 0; i < 16; i++)
            if (q + i < n) {
                const u64 b8 = (u64)src[q + i] << (8 * (i & 7));
                if (i < 8) lo |= b8; else hi |= b8;
            }
        return u32x4{(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
    }
    __device__ __forceinline__ void stage(u64 at) {  // (re)start the staged window at `at`
        vb = at & ~15ull;
        wc = load16(vb + 16ull * lane);
        wn = load16(vb + 1024 + 16ull * lane);
    }
    __device__ __forceinline__ u32 word(u32 widx) {  // staged word widx (uniform, < 512)
        const u32x4 v = widx < 256 ? wc : wn;
        const u32 c = widx & 3;
        const u32 x = c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
        return (u32)__builtin_amdgcn_readlane((int)x, (int)((widx >> 2) & 63));
    }
    __device__ __forceinline__ void release_regs() {
        const u32x4 z = u32x4{0u, 0u, 0u, 0u};
        lt0 = lt1 = lt2 = lt3 = lt4 = lt5 = ltc = wc = wn = z;
        ltc_t = 0xFFFFFFFFu;
        vb = ~0ull >> 1;         // next refill re-stages from memory
        cbp = ~0ull >> 1;        // next peek refills
    }
    // The bit reader: bb holds the 64 stream bits from bit cbp on, MSB-first
    // (bzip2's bit order), so a peek is two scalar shifts; it refills from the
    // staged window every >= 33 bits, byte-swapping the words in VGPRs before
    // they are read out (no 64-bit byte swap on the scalar path).
    __device__ __forceinline__ u32 word_be(u32 widx) {  // staged word widx, big-endian
        const u32x4 v = widx < 256 ? wc : wn;
        const u32 c = widx & 3;
        const u32 x = c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
        return (u32)__builtin_amdgcn_readlane((int)__builtin_bswap32(x), (int)((widx >> 2) & 63));
    }
    __device__ __forceinline__ void refill(u64 byte) {
        const u64 a = byte & ~3ull;
        if (a < vb || a + 12 > vb + 2048 + 1024) {
            stage(a);
        } else if (a + 12 > vb + 2048) {
            wc = wn;
            vb += 1024;
            wn = load16(vb + 1024 + 16ull * lane);
        }
        const u32 w0 = (u32)(a - vb) >> 2;
        const u64 hi = ((u64)word_be(w0) << 32) | word_be(w0 + 1);
        const u32 lo = word_be(w0 + 2);
        const u32 sh = (u32)(byte & 3) * 8;
        bb = sh ? (hi << sh) | (lo >> (32 - sh)) : hi;
        cbp = byte * 8;
    }
    __device__ __forceinline__ u32 peek(u64 bp, u32 nb) {
        u64 d = bp - cbp;
        if (d + nb > 64) {
            refill(bp >> 3);
            d = bp & 7;
        }
        return (u32)((bb << d) >> (64 - nb));
    }
    __device__ __forceinline__ zb::Group* group(u32 t) { return groups + t; }
    __device__ __forceinline__ u8* lens(u32 t) { return (u8*)(lensb + t * 260); }
    __device__ __forceinline__ u8* seqbuf() { return (u8*)seq; }
    // The fast Huffman tables live in VGPRs: lane i holds entries
    // [8 i, 8 i + 8) of each group's 512-entry table as four u16 pairs
    // (lt0..lt5); the selected group's copy `ltc` is read with one readlane
    // per symbol (no LDS round trip on the decoder's serial path).
    __device__ __forceinline__ void build_lut(u32 t, const zb::Group* g, u32) {
        static_assert(zb::LUT_BITS == 9, "VGPR table layout assumes 512 entries");
        u64 lo = 0, hi = 0;
#pragma unroll 1
        for (u32 j = 0; j < 8; j++) {
            const u64 e = (u64)zb::lut_entry(g, 8 * (u32)lane + j) << (16 * (j & 3));
            if (j < 4) lo |= e; else hi |= e;
        }
        const u32x4 v = u32x4{(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
        // (mask arithmetic, not a switch or selects: those get folded into a
        // variable-offset access of this struct, which then lives in scratch)
        auto put = [&](u32x4& dst, u32 k) {
            const u32 m = 0u - (u32)(t == k);
            dst = (v & m) | (dst & ~m);
        };
        put(lt0, 0); put(lt1, 1); put(lt2, 2); put(lt3, 3); put(lt4, 4); put(lt5, 5);
        ltc_t = 0xFFFFFFFFu;
    }
    __device__ __forceinline__ u32 lut_get(u32 t, u32 x) {
        if (t != ltc_t) {
            auto m = [&](u32 k) { return 0u - (u32)(t == k); };
            ltc = (lt0 & m(0)) | (lt1 & m(1)) | (lt2 & m(2)) | (lt3 & m(3)) | (lt4 & m(4)) | (lt5 & m(5));
            ltc_t = t;
        }
        const u32 k = (x >> 1) & 3;
        const u32 w = k == 0 ? ltc.x : (k == 1 ? ltc.y : (k == 2 ? ltc.z : ltc.w));
        const u32 r = (u32)__builtin_amdgcn_readlane((int)w, (int)(x >> 3));
        return (r >> ((x & 1) * 16)) & 0xFFFF;
    }
    __device__ __forceinline__ void sel_put(u32 i, u32 v) { sel[i] = (u8)v; }
    __device__ __forceinline__ u32 sel_get(u32 i) {
        if (i - sbase >= 16) {
            sbase = i & ~15u;
            const u32x4 v = *(const gu32x4_ua*)(sel + sbase);
            sw0 = __builtin_amdgcn_readfirstlane(v.x); sw1 = __builtin_amdgcn_readfirstlane(v.y);
            sw2 = __builtin_amdgcn_readfirstlane(v.z); sw3 = __builtin_amdgcn_readfirstlane(v.w);
        }
        const u32 d = i - sbase;
        // (values through readfirstlane: a select between the fields would be
        // folded into a variable-offset load, which keeps this whole struct
        // in scratch memory)
        const u32 a0 = __builtin_amdgcn_readfirstlane(sw0), a1 = __builtin_amdgcn_readfirstlane(sw1);
        const u32 a2 = __builtin_amdgcn_readfirstlane(sw2), a3 = __builtin_amdgcn_readfirstlane(sw3);
        const u32 w = d < 8 ? (d < 4 ? a0 : a1) : (d < 12 ? a2 : a3);
        return (w >> ((d & 3) * 8)) & 0xFF;
    }
    __device__ __forceinline__ void mtf_reset(const u8*, u32) {
        mtfw = ((const lu32*)seq)[lane];
        sbase = 0xFFFFFFF0u;  // selectors were just stored: re-read them
        __threadfence_block();
    }
    __device__ __forceinline__ u32 mtf_front() { return __builtin_amdgcn_readlane(mtfw, 0) & 0xFF; }
    __device__ __forceinline__ u32 mtf_take(u32 nn) {
        const u32 wn = nn >> 2, sh = (nn & 3) * 8;

        const u32 v = (__builtin_amdgcn_readlane(mtfw, wn) >> sh) & 0xFF;
        // lanes 0..wn shift by one lane: within DPP row 0 (row_shr:1) when
        // nn < 64, the common case; across rows through ds_bpermute
        const u32 pw = wn < 16 ? (u32)__builtin_amdgcn_update_dpp(0, (int)mtfw, 0x111, 0xf, 0xf, false)
                               : __shfl_up(mtfw, 1);
        u32 shw = (mtfw << 8) | (lane == 0 ? v : (pw >> 24));
        const u32 keep = (u32)(0xFFFFFFFFull << (sh + 8));
        u32 nw = mtfw;
        if ((u32)lane < wn) nw = shw;
        else if ((u32)lane == wn) nw = (shw & ~keep) | (mtfw & keep);
        mtfw = nw;
        return v;
    }
    __device__ __forceinline__ void l_put(u32 i, u32 b) {
        if ((u32)lane == (i & 63)) lbuf = b;
        if ((i & 63) == 63) L[(i & ~63u) + lane] = (u8)lbuf;
    }
    __device__ __forceinline__ void l_run(u32 i, u32 b, u32 cnt) {
        while (cnt > 0) {
            const u32 q = i & 63;
            const u32 take = (64 - q) < cnt ? (64 - q) : cnt;
            if ((u32)lane >= q && (u32)lane < q + take) lbuf = b;
            i += take;
            cnt -= take;
            if ((i & 63) == 0) L[i - 64 + lane] = (u8)lbuf;
        }
    }
    __device__ __forceinline__ void l_flush(u32 nb) {
        if ((nb & 63) && (u32)lane < (nb & 63)) L[(nb & ~63u) + lane] = (u8)lbuf;
    }
};

// ---- helpers for 256-thread stages ----------------------------------------------
__device__ __forceinline__ u64 eq_mask(u32 v, bool valid) {
    u64 m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const u64 bb = __ballot((v >> b) & 1);
        m &= ((v >> b) & 1) ? bb : ~bb;
    }
    return m;
}

// exclusive scan over the 256 threads (returns prefix, *total = sum)
__device__ __forceinline__ u32 block_scan_u32(u32 x, u32* tmp, u32* total) {
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u32 incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(incl, d);
        if (lane >= (u32)d) incl += y;
    }
    if (lane == 63) tmp[w] = incl;
    __syncthreads();
    u32 base = 0;
    for (u32 k = 0; k < w; k++) base += tmp[k];
    *total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
    __syncthreads();
    return base + incl - x;
}

// f(byte) over T[a0, a1) in order: 16-byte loads, the next one issued
// before the current one is consumed
template <class F>
__device__ __forceinline__ void t_bytes(const gu8* T, u32 a0, u32 a1, F&& f) {
    if (a0 >= a1) return;
    u32 kb = a0 & ~15u;
    u32x4 cur = *(const gu32x4_ua*)(T + kb);
    for (; kb < a1; kb += 16) {
        const u32x4 nxt = kb + 16 < a1 ? *(const gu32x4_ua*)(T + kb + 16) : cur;
#pragma unroll
        for (u32 j = 0; j < 16; j++) {
            const u32 k = kb + j;
            const u32 w = j < 4 ? cur.x : (j < 8 ? cur.y : (j < 12 ? cur.z : cur.w));
            if (k >= a0 && k < a1) f((w >> (8 * (j & 3))) & 0xFF);
        }
        cur = nxt;
    }
}

__device__ __forceinline__ u32 rle_trans(u32 s, u32 c, u32 pc) {
    return s == 4 ? 0u : (s == 0 ? 1u : (c == pc ? s + 1 : 1u));
}

// phase timers (always on: a few global atomics per block): A, sort, walk 1,
// rank, walk 2, RLE1/output/CRC; slot 6 counts blocks
__device__ unsigned long long g_bz_dbg[8];
#define BZ_TSTAMP(k)                                                            \
    do {                                                                        \
        if (tid == 0) {                                                         \
            const u64 _t = __builtin_readcyclecounter();                        \
            atomicAdd(&g_bz_dbg[k], (unsigned long long)(_t - t_last));         \
            t_last = _t;                                                        \
        }                                                                       \
    } while (0)

extern "C" int zcg__debug_bz2_counters(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bz_dbg), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_bz_dbg), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}

struct BzShared {
    u32 nblock, orig, stored_crc, randomised, single, done_status;
    u64 out_pos;
    u32 p0;
};

// LDS of the stage B/C workgroup
struct BzBcLds {
    u32 hist[4][256];
    u16 succ[BZ_NSAMP + 1];
    u32 slen[BZ_NSAMP + 1];
    u32 soff[BZ_NSAMP + 1];
    u32 pcap[BZ_NSAMP + 1];  // where a walk longer than CAP stood at step CAP
    u32 tstate[BZ_T];
    u32 tcrc[BZ_T];
    u32 tlen[BZ_T];
    u32 scan_tmp[8];
    u32 crct[256];  // CRC-32 (MSB-first) byte table
    BzShared sh;
};

// Stages B and C of one block (256 threads): L[nblock] -> output bytes at
// X.sh.out_pos.. of dst (bounded by D), block CRC check.  In: X.sh.{nblock,
// orig, stored_crc, randomised, out_pos}.  Out: X.sh.out_pos advanced,
// X.tcrc[0] = the block CRC; returns a final chunk status (>= 0) or -1 when
// the stream continues.
__device__ __forceinline__ int bz_block_bc(BzBcLds& X, const gu8* L, gu8* KB, u32 kcap, gu8* T, gu32* W, gu8* dst,
                                           u64 D, DType t, u32 vflags, u64& t_last) {
    const u32 tid = threadIdx.x, lane = tid & 63;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    auto& hist = X.hist;
    auto& succ = X.succ;
    auto& slen = X.slen;
    auto& pcap = X.pcap;
    auto& soff = X.soff;
    auto& tstate = X.tstate;
    auto& tcrc = X.tcrc;
    auto& tlen = X.tlen;
    auto& scan_tmp = X.scan_tmp;
    auto& crct = X.crct;
    auto& sh = X.sh;
    const u32 nblock = sh.nblock;

    // ---------------- stage B: T^-1 links by a stable counting sort ----------------
    const u32 q0 = (u32)(((u64)nblock * wave / 4) & ~63ull);
    const u32 q1 = wave == 3 ? nblock : (u32)(((u64)nblock * (wave + 1) / 4) & ~63ull);
    for (u32 v = lane; v < 256; v += 64) hist[wave][v] = 0;
    __syncthreads();
    for (u32 g = q0; g < q1; g += 64) {
        const u32 i = g + lane;
        const bool ok = i < q1;
        const u32 v = ok ? (u32)L[i] : 0u;
        const u64 m = eq_mask(v, ok);
        if (ok && (u32)__builtin_ctzll(m) == lane) hist[wave][v] += (u32)__builtin_popcountll(m);
    }
    __syncthreads();
    {
        const u32 v = tid;
        const u32 h0 = hist[0][v], h1 = hist[1][v], h2 = hist[2][v], h3 = hist[3][v];
        u32 tot;
        const u32 cf = block_scan_u32(h0 + h1 + h2 + h3, scan_tmp, &tot);
        hist[0][v] = cf;
        hist[1][v] = cf + h0;
        hist[2][v] = cf + h0 + h1;
        hist[3][v] = cf + h0 + h1 + h2;
    }
    __syncthreads();
    for (u32 g = q0; g < q1; g += 64) {
        const u32 i = g + lane;
        const bool ok = i < q1;
        const u32 v = ok ? (u32)L[i] : 0u;
        const u64 m = eq_mask(v, ok);
        const u32 b = hist[wave][v & 255];
        const u32 rank = (u32)__builtin_popcountll(m & ((1ull << lane) - 1));
        if (ok) W[b + rank] = (i << 8) | v;
        if (ok && (u32)__builtin_ctzll(m) == lane) hist[wave][v] = b + (u32)__builtin_popcountll(m);
    }
    __syncthreads();
    BZ_TSTAMP(1);

    // ---------------- stage B: list ranking of the chain p -> W[p] >> 8 ----------------
    const u32 p0 = W[sh.orig] >> 8;
    u32 lgs = 0;
    while (((u64)BZ_NSAMP << lgs) < nblock) lgs++;
    const u32 S = 1u << lgs, smask = S - 1;
    const u32 NR = (nblock + S - 1) >> lgs;
    const bool extra = (p0 & smask) != 0;
    const u32 sid0 = extra ? NR : (p0 >> lgs);
#define BZ_IS_SAMPLE(p) ((((p) & smask) == 0) || ((p) == p0))
#define BZ_SID(p) ((((p) & smask) == 0) ? ((p) >> lgs) : NR)
    for (u32 k = tid; k <= BZ_NSAMP; k += BZ_T) soff[k] = 0xFFFFFFFFu;
    // One walk per sample: step m from position p reads W[p] = next << 8 |
    // L[next], i.e. output byte soff + 1 + m.  The first CAP bytes of each
    // walk are kept (4 at a time in a register, then one u32 store) in the
    // slot's kept-byte buffer KB; a walk longer than CAP records where it was
    // at step CAP and finishes after the ranking.  Walk lengths are close to
    // exponential with mean nblock / NR <= S, so CAP = BZ_KMUL * S leaves
    // ~e^-BZ_KMUL of the bytes to the second walk (CAP = S: ~31 %).  The
    // kept-byte region is sized from the array's block-size level (kcap per
    // walk, a power of two >= 16); a stream whose blocks are larger than the
    // level says keeps fewer bytes per walk and leaves more to the second
    // walk, with the same output.
    const u32 CAP0 = S < 16 / BZ_KMUL ? 16u : BZ_KMUL * S;
    const u32 CAP = CAP0 < kcap ? CAP0 : kcap;
    gu32* buf32 = (gu32*)KB;
    const u32 Lp0 = L[p0];  // T[0] (the cycle's first byte)
    __syncthreads();
    {
        u32 ps[BZ_WALKS], ln[BZ_WALKS], sidk[BZ_WALKS], acc[BZ_WALKS];
        u32 act = 0;
#pragma unroll
        for (int k = 0; k < BZ_WALKS; k++) {
            const bool last = k == BZ_WALKS - 1;
            const u32 sd = !last ? tid + (u32)k * BZ_T : NR;
            const bool on = !last ? sd < NR : (tid == 0 && extra);
            sidk[k] = sd;
            ps[k] = !last ? (sd << lgs) : p0;
            ln[k] = 0;
            acc[k] = 0;
            if (on) act |= 1u << k;
        }
        while (act) {
            u32 w[BZ_WALKS];
#pragma unroll
            for (int k = 0; k < BZ_WALKS; k++) w[k] = (act >> k & 1) ? W[ps[k]] : 0u;
#pragma unroll
            for (int k = 0; k < BZ_WALKS; k++) {
                if (!(act >> k & 1)) continue;
                const u32 m = ln[k], nx = w[k] >> 8;
                if (m < CAP) {
                    acc[k] |= (w[k] & 0xFF) << (8 * (m & 3));
                    if ((m & 3) == 3) {
                        buf32[(sidk[k] * CAP + m) >> 2] = acc[k];
                        acc[k] = 0;
                    }
                } else if (m == CAP) {
                    pcap[sidk[k]] = ps[k];
                }
                ln[k] = m + 1;
                ps[k] = nx;
                if (BZ_IS_SAMPLE(nx)) {
                    const u32 kept = ln[k] < CAP ? ln[k] : CAP;
                    if (kept & 3) buf32[(sidk[k] * CAP + kept) >> 2] = acc[k];
                    succ[sidk[k]] = (u16)BZ_SID(nx);
                    slen[sidk[k]] = ln[k];
                    act &= ~(1u << k);
                }
            }
        }
    }
    __syncthreads();
    BZ_TSTAMP(2);
    if (tid == 0) {
        u32 sd = sid0, off = 0, cnt = 0;
        do {
            soff[sd] = off;
            off += slen[sd];
            sd = succ[sd];
            cnt++;
        } while (sd != sid0 && cnt <= NR + 1);
        sh.single = (sd == sid0 && off == nblock) ? 1u : 0u;
        sh.p0 = p0;
    }
    __syncthreads();
    BZ_TSTAMP(3);
    if (sh.single) {
        // kept bytes -> T, a wave per sample (byte m of walk s is T[soff + 1 + m]):
        // lane l moves bytes 4l..4l+3 of each 256-byte piece, so a load is one
        // coalesced dword per lane and a store instruction covers two lines
        for (u32 sd = wave; sd <= NR; sd += BZ_T / 64) {
            if (sd == NR && !extra) break;
            const u32 so = soff[sd];
            if (so == 0xFFFFFFFFu) continue;
            const u32 len = slen[sd], kept = len < CAP ? len : CAP;
            const gu32* kb = buf32 + ((sd * CAP) >> 2);
            for (u32 m = 4 * lane; m < kept; m += 256) {
                const u32 v = kb[m >> 2];
#pragma unroll
                for (u32 j = 0; j < 4; j++)
                    if (m + j < kept) {
                        const u32 idx = so + 1 + m + j;
                        T[idx < nblock ? idx : idx - nblock] = (u8)(v >> (8 * j));
                    }
            }
        }
        // walks longer than CAP: the rest, interleaved per thread
        u32 q[BZ_WALKS], rem[BZ_WALKS], of[BZ_WALKS];
        u32 act = 0;
#pragma unroll
        for (int k = 0; k < BZ_WALKS; k++) {
            const bool last = k == BZ_WALKS - 1;
            const u32 sd = !last ? tid + (u32)k * BZ_T : NR;
            const bool on = !last ? sd < NR : (tid == 0 && extra);
            q[k] = 0;
            rem[k] = 0;
            of[k] = 0;
            if (on && soff[sd] != 0xFFFFFFFFu && slen[sd] > CAP) {
                q[k] = pcap[sd];
                rem[k] = slen[sd] - CAP;
                of[k] = soff[sd] + 1 + CAP;
                act |= 1u << k;
            }
        }
        while (act) {
            u32 w[BZ_WALKS];
#pragma unroll
            for (int k = 0; k < BZ_WALKS; k++) w[k] = (act >> k & 1) ? W[q[k]] : 0u;
#pragma unroll
            for (int k = 0; k < BZ_WALKS; k++) {
                if (!(act >> k & 1)) continue;
                const u32 idx = of[k]++;
                T[idx < nblock ? idx : idx - nblock] = (u8)(w[k] & 0xFF);
                q[k] = w[k] >> 8;
                if (--rem[k] == 0) act &= ~(1u << k);
            }
        }
    } else if (tid == 0) {
        // not one cycle (corrupt): libbz2's serial tPos walk (T[k+1] = L[next] = W[p] & 0xFF)
        u32 p = p0;
        T[0] = (u8)Lp0;
        for (u32 k = 1; k < nblock; k++) {
            const u32 w = W[p];
            T[k] = (u8)(w & 0xFF);
            p = w >> 8;
        }
    }
#undef BZ_IS_SAMPLE
#undef BZ_SID
    __syncthreads();
    BZ_TSTAMP(4);
    if (sh.randomised && tid == 0) {
        // BZ_RAND_UPD_MASK: fetch F_{m+1} - 2 is XORed with 1
        u32 f = 0, rt = 0;
        for (;;) {
            f += zb::kRNums[rt];
            rt = (rt + 1) & 511;
            if (f - 2 >= nblock) break;
            T[f - 2] ^= 1;
        }
    }
    __syncthreads();

    // ---------------- stage C: RLE1 + output + block CRC ----------------
    const u32 seg = (nblock + BZ_T - 1) / BZ_T;
    const u32 a0 = tid * seg < nblock ? tid * seg : nblock;
    const u32 a1 = a0 + seg < nblock ? a0 + seg : nblock;
    const u32 pc0 = a0 ? (u32)T[a0 - 1] : 0u;
    {
        u32 st0 = 0, st1 = 1, st2 = 2, st3 = 3, st4 = 4;
        u32 pc = pc0;
        t_bytes(T, a0, a1, [&](u32 cb) {
            st0 = rle_trans(st0, cb, pc); st1 = rle_trans(st1, cb, pc);
            st2 = rle_trans(st2, cb, pc); st3 = rle_trans(st3, cb, pc);
            st4 = rle_trans(st4, cb, pc);
            pc = cb;
        });
        tstate[tid] = st0 | (st1 << 3) | (st2 << 6) | (st3 << 9) | (st4 << 12);
    }
    __syncthreads();
    if (tid == 0) {
        u32 stt = 0;
        for (u32 k = 0; k < BZ_T; k++) {
            const u32 f = tstate[k];
            tstate[k] = stt;
            stt = (f >> (3 * stt)) & 7;
        }
        sh.done_status = stt;  // state after the last byte
    }
    __syncthreads();
    u32 cnt_out = 0;
    {
        u32 stt = tstate[tid];
        u32 pc = pc0;
        t_bytes(T, a0, a1, [&](u32 cb) {
            cnt_out += (stt == 4) ? cb : 1u;
            stt = rle_trans(stt, cb, pc);
            pc = cb;
        });
    }
    u32 blk_total;
    const u32 my_off = block_scan_u32(cnt_out, scan_tmp, &blk_total);
    const u64 ob = sh.out_pos;
    const bool tail4 = sh.done_status == 4;  // a run of four without its count byte
    const bool complete = !tail4 && ob + blk_total <= D;
    {
        u32 stt = tstate[tid];
        u32 pc = pc0;
        u64 op = ob + my_off;
        u32 crc = 0xFFFFFFFFu;
        t_bytes(T, a0, a1, [&](u32 cb) {
            const u32 reps = (stt == 4) ? cb : 1u;
            const u32 val = (stt == 4) ? pc : cb;
            for (u32 r2 = 0; r2 < reps; r2++, op++) {
                if (op < D) dst[swap_pos(op, t)] = norm_byte((u8)val, t);
                if (complete) crc = (crc << 8) ^ crct[((crc >> 24) ^ val) & 0xFF];
            }
            stt = rle_trans(stt, cb, pc);
            pc = cb;
        });
        tcrc[tid] = ~crc;
        tlen[tid] = cnt_out;
    }
    __syncthreads();
    if (complete) {
        for (u32 step = 1; step < BZ_T; step <<= 1) {
            if ((tid & (2 * step - 1)) == 0) {
                const u32 o = tid + step;
                tcrc[tid] = bz_mulmod(tcrc[tid], bz_xpow8(tlen[o])) ^ tcrc[o];
                tlen[tid] += tlen[o];
            }
            __syncthreads();
        }
    }
    if (tid == 0) {
        int fs = -1;
        if (tail4) {
            // libbz2 reads the next chain byte (the cycle start) as the count,
            // emits those copies, then reports the stream corrupt
            const u32 g = (u32)T[0] ^ 0u;
            const u32 val = nblock ? (u32)T[nblock - 1] : 0u;
            u64 op = ob + blk_total;
            for (u32 r2 = 0; r2 < g && op < D; r2++, op++) dst[swap_pos(op, t)] = norm_byte((u8)val, t);
            fs = (op >= D) ? ZCG_OK : ((vflags & ZCG_FLAG_DEBUG_COUNTERS) ? 20000 : ZCG_ERR_INVALID_DATA);
        } else if (!complete) {
            fs = ZCG_OK;  // D reached inside the block
        } else if (tcrc[0] != sh.stored_crc && !(vflags & ZCG_FLAG_DEBUG_COUNTERS)) {
            fs = ZCG_ERR_INVALID_DATA;
        }
        sh.done_status = (u32)fs;
        sh.out_pos = ob + blk_total;
    }
    __syncthreads();
    BZ_TSTAMP(5);
    if (tid == 0) atomicAdd(&g_bz_dbg[6], 1ull);
    return (int)sh.done_status;
}

// ---- the per-round pipeline ---------------------------------------------------------
// Stage A is one serial wave per chunk and dominates the time, so it runs in
// its own kernel (64-thread workgroups, small LDS, its own register budget:
// many chunks in flight per CU); stages B+C run in a 256-thread kernel.  A
// round is one block per unfinished chunk; the launcher issues a fixed
// number of rounds and the monolithic kernel finishes any chunk still open.
struct BzChunkState {
    zb::BzState s;
    u64 out_pos;
    int final_status;  // -1 while open
    u32 pending;       // a block decoded by stage A awaits stages B+C
    u32 pad[2];
};
static_assert(sizeof(BzChunkState) <= 256, "chunk state");

// workspace: NA stage-A slots [L | SEL | state] + NB stage-B/C slots [T | W] + owners
constexpr u64 BZ_A_OFF_SEL = BZ_LBYTES;
constexpr u64 BZ_A_OFF_ST = BZ_LBYTES + 18176;
constexpr u64 BZ_A_SLOT = BZ_A_OFF_ST + 256;              // L, SEL, state
constexpr u64 BZ_BC_OFF_W = BZ_LBYTES;
constexpr u64 BZ_BC_OFF_K = BZ_BC_OFF_W + 4ull * BZ_NMAX + 128;
// B/C slot: T, W, then the kept walk bytes, (NSAMP + 1) walks of kcap bytes
// each; kcap follows the array's block-size level (bz_kcap), so a level-1
// array's slot is 3.6 MB smaller than a level-9 one's
__host__ __device__ constexpr u32 bz_kcap(int lvl) {
    u32 S = 1;
    while ((u64)BZ_NSAMP * S < 100000ull * (u64)lvl) S <<= 1;
    return S < 16 / BZ_KMUL ? 16u : BZ_KMUL * S;
}
__host__ __device__ constexpr u64 bz_bc_slot(u32 kcap) {
    return (BZ_BC_OFF_K + (u64)kcap * (BZ_NSAMP + 1) + 255) & ~255ull;
}
static_assert(bz_kcap(9) == BZ_KMUL * 1024 && bz_kcap(1) == BZ_KMUL * 128, "kept-byte caps");
constexpr u32 BZ_NA = 4096;  // chunks in flight (stage A occupancy: 16 waves per CU)
constexpr u32 BZ_NB = 1024;  // stage B/C workspace slots (>= resident B/C workgroups)
static_assert(BZ_A_SLOT % 256 == 0 && BZ_BC_OFF_K % 16 == 0, "slot alignment");

__device__ __forceinline__ void bz_io_init(BzDevIO& io, const zcg_chunk& ch, zb::Group* groups, u8* lensb, u8* seq,
                                           gu8* sel, gu8* L, int lane) {
    io.src = (const gu8*)ch.src;
    io.n = ch.src_len;
    io.cbp = ~0ull >> 1;
    io.bb = 0;
    io.groups = groups;
    io.lensb = (lu8*)lensb;
    io.ltc_t = 0xFFFFFFFFu;
    io.seq = (lu8*)seq;
    io.sel = sel;
    io.L = L;
    io.sbase = 0xFFFFFFF0u;
    io.sw0 = io.sw1 = io.sw2 = io.sw3 = 0;
    io.mtfw = 0;
    io.lbuf = 0;
    io.lane = lane;
    io.vb = ~0ull >> 1;  // the first refill stages the window
}

__device__ __forceinline__ void bz_state_init(zb::BzState& s, u64 n) {
    s.n = n;
    s.lim = n;
    s.bitpos = 0;
    s.level = 0;
    s.full = 0;
    s.header_done = 0;
    s.combined = 0;
    s.stored_crc = s.randomised = s.orig_ptr = s.nblock = 0;
    s.err_line = 0;
}

// status of the stream after stage A returned r (the decode loop's rules)
__device__ __forceinline__ int bz_after_a(int r, const zb::BzState& s, u32 vflags) {
    if (r == zb::R_STOP || r == zb::R_END) return s.full ? ZCG_OK : ZCG_ERR_UNEXPECTED_EOF;
    if (r != zb::R_BLOCK) {
        if ((vflags & ZCG_FLAG_DEBUG_COUNTERS) && r == zb::ST_INVALID) return 10000 + (int)s.err_line;
        return r;
    }
    if (s.full) return ZCG_OK;  // the block after N decoded (validated): nothing to emit
    return -1;
}

// after a block's stages B+C completed without a final status
__device__ __forceinline__ void bz_after_bc(zb::BzState& s, u32 bcrc, u64 out_pos, u64 D) {
    s.combined = ((s.combined << 1) | (s.combined >> 31)) ^ bcrc;
    if (out_pos == D) {
        // output full exactly at a block end: libbz2 keeps parsing the
        // current 32 KiB input window
        s.full = 1;
        const u64 used = (s.bitpos + 7) >> 3;
        const u64 ve = ((used ? used - 1 : 0) / zb::BUFREADER + 1) * zb::BUFREADER;
        s.lim = ve < s.n ? ve : s.n;
    }
}

__global__ __launch_bounds__(64) void bz2_init_kernel(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                      u8* __restrict__ wsa, u32 c_base, u32 cnt,
                                                      i32* __restrict__ status) {
    const u32 k = blockIdx.x * 64 + threadIdx.x;
    if (k >= cnt || c_base + k >= n) return;
    const u32 c = c_base + k;
    BzChunkState* st = (BzChunkState*)(wsa + (u64)k * BZ_A_SLOT + BZ_A_OFF_ST);
    const zcg_chunk ch = chunks[c];
    int fs = -1;
    if (D > 0 && ch.dst_cap < D) fs = ZCG_ERR_INVALID_INPUT;
    else if (D == 0) fs = ZCG_OK;
    bz_state_init(st->s, ch.src_len);
    st->out_pos = 0;
    st->final_status = fs;
    st->pending = 0;
    if (fs >= 0) status[c] = fs;
}

__global__ __launch_bounds__(64) void bz2_stage_a_kernel(const zcg_chunk* __restrict__ chunks, u32 n,
                                                         u8* __restrict__ wsa, u32 c_base, u32 vflags,
                                                         i32* __restrict__ status) {
    __shared__ zb::Group groups[6];
    __shared__ __attribute__((aligned(16))) u8 lensb[6 * 260];
    __shared__ __attribute__((aligned(16))) u8 seq[256];
    const u32 k = blockIdx.x;
    const u32 c = c_base + k;
    if (c >= n) return;
    u8* slot = wsa + (u64)k * BZ_A_SLOT;
    BzChunkState* st = (BzChunkState*)(slot + BZ_A_OFF_ST);
    if (__builtin_amdgcn_readfirstlane(st->final_status) >= 0 || __builtin_amdgcn_readfirstlane(st->pending)) return;
    const int lane = lane_id();
    const u64 t0 = __builtin_readcyclecounter();
    const zcg_chunk ch = chunks[c];
    BzDevIO io;
    bz_io_init(io, ch, groups, lensb, seq, (gu8*)(slot + BZ_A_OFF_SEL), (gu8*)slot, lane);
    zb::BzState s = st->s;
    const int r = zb::bz_block(io, s);
    io.l_flush(s.nblock * (r == zb::R_BLOCK ? 1u : 0u));
    const int fs = bz_after_a(r, s, vflags);
    if (lane == 0) {
        st->s = s;
        st->final_status = fs;
        st->pending = fs < 0 ? 1u : 0u;
        if (fs >= 0) status[c] = fs;
        atomicAdd(&g_bz_dbg[0], (unsigned long long)(__builtin_readcyclecounter() - t0));
    }
}

__global__ __launch_bounds__(256) void bz2_stage_bc_kernel(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                           DType t, u8* __restrict__ wsa, u8* __restrict__ wsb,
                                                           u32* __restrict__ owner, u32 nb, u32 kcap, u32 c_base,
                                                           u32 vflags, i32* __restrict__ status) {
    __shared__ BzBcLds S;
    const u32 k = blockIdx.x;
    const u32 c = c_base + k;
    if (c >= n) return;
    const u32 tid = threadIdx.x;
    u8* slot = wsa + (u64)k * BZ_A_SLOT;
    BzChunkState* st = (BzChunkState*)(slot + BZ_A_OFF_ST);
    if (!__builtin_amdgcn_readfirstlane(st->pending)) return;
    S.crct[tid] = g_bzcrc.t[tid];
    if (tid == 0) {
        u32 b = k % nb;
        while (atomicCAS(&owner[b], 0u, 1u) != 0u) b = (b + 1) % nb;
        S.sh.p0 = b;  // (p0 is rewritten by the ranking stage)
        S.sh.nblock = st->s.nblock;
        S.sh.orig = st->s.orig_ptr;
        S.sh.stored_crc = st->s.stored_crc;
        S.sh.randomised = st->s.randomised;
        S.sh.out_pos = st->out_pos;
    }
    __syncthreads();
    const u32 b = S.sh.p0;
    u8* bslot = wsb + (u64)b * bz_bc_slot(kcap);
    const zcg_chunk ch = chunks[c];
    u64 t_last = __builtin_readcyclecounter();
    const int fs = bz_block_bc(S, (const gu8*)slot, (gu8*)(bslot + BZ_BC_OFF_K), kcap, (gu8*)bslot, (gu32*)(bslot + BZ_BC_OFF_W), (gu8*)ch.dst, D, t,
                               vflags, t_last);
    __syncthreads();  // all B/C workspace accesses done
    if (tid == 0) {
        zb::BzState s = st->s;
        if (fs < 0) bz_after_bc(s, S.tcrc[0], S.sh.out_pos, D);
        st->s = s;
        st->out_pos = S.sh.out_pos;
        st->final_status = fs;
        st->pending = 0;
        if (fs >= 0) status[c] = fs;
        atomicExch(&owner[b], 0u);
    }
}

// The whole stream in one workgroup, for chunks the rounds did not finish.
__global__ __launch_bounds__(256) void bz2_decode_kernel(const zcg_chunk* __restrict__ chunks, u32 n,
                                                         u64 D, DType t, u8* __restrict__ wsa, u8* __restrict__ wsb,
                                                         u32* __restrict__ owner, u32 nb, u32 kcap, u32 c_base,
                                                         u32 vflags, i32* __restrict__ status) {
    __shared__ zb::Group groups[6];
    __shared__ __attribute__((aligned(16))) u8 lensb[6 * 260];
    __shared__ __attribute__((aligned(16))) u8 seq[256];
    __shared__ BzBcLds S;
    __shared__ int sh_r;
    __shared__ zb::BzState sh_s;
    const u32 k = blockIdx.x;
    const u32 c = c_base + k;
    if (c >= n) return;
    const u32 tid = threadIdx.x, lane = tid & 63;
    u8* slot = wsa + (u64)k * BZ_A_SLOT;
    BzChunkState* st = (BzChunkState*)(slot + BZ_A_OFF_ST);
    if (__builtin_amdgcn_readfirstlane(st->final_status) >= 0) return;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    S.crct[tid] = g_bzcrc.t[tid];
    const zcg_chunk ch = chunks[c];
    if (tid == 0) {
        u32 b = k % nb;
        while (atomicCAS(&owner[b], 0u, 1u) != 0u) b = (b + 1) % nb;
        S.sh.p0 = b;
        S.sh.out_pos = 0;
    }
    __syncthreads();
    const u32 b = S.sh.p0;
    u8* bslot = wsb + (u64)b * bz_bc_slot(kcap);
    BzDevIO io;
    zb::BzState s;
    if (wave == 0) {
        bz_io_init(io, ch, groups, lensb, seq, (gu8*)(slot + BZ_A_OFF_SEL), (gu8*)slot, lane);
        bz_state_init(s, ch.src_len);
    }
    int final_status = -1;
    u64 t_last = __builtin_readcyclecounter();
    for (;;) {
        if (wave == 0) {
            const int r = zb::bz_block(io, s);
            io.l_flush(s.nblock * (r == zb::R_BLOCK ? 1u : 0u));
            io.release_regs();
            if (lane == 0) {
                sh_r = r;
                sh_s = s;
            }
        }
        __syncthreads();
        const int fa = bz_after_a(sh_r, sh_s, vflags);
        if (fa >= 0) { final_status = fa; break; }
        if (tid == 0) {
            S.sh.nblock = sh_s.nblock;
            S.sh.orig = sh_s.orig_ptr;
            S.sh.stored_crc = sh_s.stored_crc;
            S.sh.randomised = sh_s.randomised;
        }
        __syncthreads();
        const int fs = bz_block_bc(S, (const gu8*)slot, (gu8*)(bslot + BZ_BC_OFF_K), kcap, (gu8*)bslot, (gu32*)(bslot + BZ_BC_OFF_W), (gu8*)ch.dst,
                                   D, t, vflags, t_last);
        __syncthreads();
        if (fs >= 0) { final_status = fs; break; }
        if (wave == 0) bz_after_bc(s, S.tcrc[0], S.sh.out_pos, D);
        __syncthreads();
    }
    __syncthreads();
    if (tid == 0) {
        status[c] = final_status;
        st->final_status = final_status;
        atomicExch(&owner[b], 0u);
    }
}

namespace {
u32 bz_na(uint32_t n) { return n < BZ_NA ? n : BZ_NA; }
u32 bz_nb(uint32_t n) { return n < BZ_NB ? n : BZ_NB; }
constexpr u64 BZ_OWNER_BYTES = 4ull * BZ_NB;
}  // namespace

const char* cfg_bz2() { return "bz2:KMUL=" ZCG_STR(ZB_KMUL) ",GSAFE=" ZCG_STR(ZB_GSAFE); }

// the array's block-size level (9 when the metadata does not say)
static int bz_level(const zcg_array* a) {
    const int l = a->compression.bzip2_block_size;
    return l >= 1 && l <= 9 ? l : 9;
}

uint64_t bzip2_decode_ws_bytes(const zcg_array* a, uint32_t n) {
    if (n == 0) return 0;
    return BZ_OWNER_BYTES + (u64)bz_na(n) * BZ_A_SLOT + (u64)bz_nb(n) * bz_bc_slot(bz_kcap(bz_level(a)));
}

hipError_t launch_bzip2_decode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                               int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const u32 na = bz_na(n), nb = bz_nb(n);
    if (ws_bytes < bzip2_decode_ws_bytes(a, n)) return hipErrorInvalidValue;
    u32* owner = (u32*)ws;
    u8* wsa = (u8*)ws + BZ_OWNER_BYTES;
    u8* wsb = wsa + (u64)na * BZ_A_SLOT;
    const u32 vflags = a->compression.flags;
    // rounds: the blocks a chunk of D bytes needs at the array's block size
    // (each block emits >= 4/5 of its 100 000 * level bytes), + the block
    // after N and the end-of-stream record; anything longer finishes in the
    // whole-stream kernel
    const int lvl = bz_level(a);
    const u32 kcap = bz_kcap(lvl);
    const u64 per = 80000ull * (u64)lvl;
    const u32 rounds = (u32)((D + per - 1) / per) + 2;
    hipError_t e = hipMemsetAsync(owner, 0, BZ_OWNER_BYTES, s);
    if (e != hipSuccess) return e;
    for (u32 c0 = 0; c0 < n; c0 += na) {
        const u32 cnt = (n - c0) < na ? (n - c0) : na;
        hipLaunchKernelGGL(bz2_init_kernel, dim3((cnt + 63) / 64), dim3(64), 0, s, d_chunks, n, D, wsa, c0, cnt,
                           d_status);
        for (u32 r = 0; r < rounds; r++) {
            hipLaunchKernelGGL(bz2_stage_a_kernel, dim3(cnt), dim3(64), 0, s, d_chunks, n, wsa, c0, vflags, d_status);
            hipLaunchKernelGGL(bz2_stage_bc_kernel, dim3(cnt), dim3(BZ_T), 0, s, d_chunks, n, D, t, wsa, wsb, owner,
                               nb, kcap, c0, vflags, d_status);
        }
        hipLaunchKernelGGL(bz2_decode_kernel, dim3(cnt), dim3(BZ_T), 0, s, d_chunks, n, D, t, wsa, wsb, owner, nb,
                           kcap, c0, vflags, d_status);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace zcg
