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
//      gives the T^-1 links N[]; the output order is a list ranking of N:
//      1 024 power-of-two-strided samples (+ the start) are walked in
//      parallel (5 interleaved walks per thread), the sample chain is ranked
//      by one thread, and a second walk writes T[] in output order.  A chain
//      that is not one cycle (corrupt data) falls back to libbz2's serial walk.
//   C. (256 threads) RLE1 as a parallel scan of the 5-state run machine,
//      output offsets by a block scan, byte stores with the '>'/bool
//      transform fused, the block CRC as 256 segment CRCs combined by
//      GF(2) x^(8n) shifts, checked against the stored CRC when the block
//      completes inside D (read_exact semantics, chunk.rs:112-113).
// Workspace per chunk slot: L, T (900 000 B each), N (3.6 MB), selectors.
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
constexpr u32 BZ_T = 256;
constexpr u64 BZ_OFF_L = 0;
constexpr u64 BZ_OFF_T = 900096;
constexpr u64 BZ_OFF_SEL = BZ_OFF_T + 900096;
constexpr u64 BZ_OFF_N = BZ_OFF_SEL + 18176;
constexpr u64 BZ_SLOT = BZ_OFF_N + 4ull * BZ_NMAX;  // bytes per chunk slot (multiple of 256)
constexpr u32 BZ_MAX_SLOTS = 1024;                   // chunks per launch (workspace bound)

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
    u64 wbase, wlo, whi;  // 16-byte input window (wave-uniform)
    zb::Group* groups;
    lu8* lensb;
    lu16* lut;
    lu8* seq;
    gu8* sel;
    gu8* L;
    u32 sbase, sw0, sw1, sw2, sw3;  // selector window
    u32 mtfw;                      // MTF list bytes [4 lane, 4 lane + 4)
    u32 lbuf;                      // pending L bytes, one per lane
    int lane;

    __device__ __forceinline__ void refill(u64 byte) {
        u32x4 v;
        if (byte + 16 <= n) {
            v = *(const gu32x4_ua*)(src + byte);
        } else {
            u32 t[4] = {0, 0, 0, 0};
            for (u64 q = byte; q < n && q < byte + 16; q++) t[(q - byte) >> 2] |= (u32)src[q] << (8 * ((q - byte) & 3));
            v = u32x4{t[0], t[1], t[2], t[3]};
        }
        wbase = byte;
        wlo = ((u64)(u32)__builtin_amdgcn_readfirstlane(v.y) << 32) | (u32)__builtin_amdgcn_readfirstlane(v.x);
        whi = ((u64)(u32)__builtin_amdgcn_readfirstlane(v.w) << 32) | (u32)__builtin_amdgcn_readfirstlane(v.z);
    }
    __device__ __forceinline__ u32 peek(u64 bp, u32 nb) {
        const u64 byte = bp >> 3;
        u64 o = byte - wbase;
        if (o > 8) { refill(byte); o = 0; }
        u64 v = (o == 0) ? wlo : (o == 8 ? whi : ((wlo >> (8 * o)) | (whi << (64 - 8 * o))));
        v = __builtin_bswap64(v);
        return (u32)((v << (bp & 7)) >> (64 - nb));
    }
    __device__ __forceinline__ zb::Group* group(u32 t) { return groups + t; }
    __device__ __forceinline__ u8* lens(u32 t) { return (u8*)(lensb + t * 260); }
    __device__ __forceinline__ u8* seqbuf() { return (u8*)seq; }
    __device__ __forceinline__ void build_lut(u32 t, const zb::Group* g, u32) {
        for (u32 x = lane; x < (1u << zb::LUT_BITS); x += 64) lut[(t << zb::LUT_BITS) + x] = (u16)zb::lut_entry(g, x);
    }
    __device__ __forceinline__ u32 lut_get(u32 t, u32 x) {
        return __builtin_amdgcn_readfirstlane(lut[(t << zb::LUT_BITS) + x]);
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
        const u32 w = d < 8 ? (d < 4 ? sw0 : sw1) : (d < 12 ? sw2 : sw3);
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
        const u32 pw = __shfl_up(mtfw, 1);
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
__device__ u32 block_scan_u32(u32 x, u32* tmp, u32* total) {
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

__device__ __forceinline__ u32 rle_trans(u32 s, u32 c, u32 pc) {
    return s == 4 ? 0u : (s == 0 ? 1u : (c == pc ? s + 1 : 1u));
}

struct BzShared {
    int r;
    u32 nblock, orig, stored_crc, randomised, level, full, single, done_status;
    u64 out_pos;
    u32 p0;
};

__global__ __launch_bounds__(256) void bz2_decode_kernel(const zcg_chunk* __restrict__ chunks, u32 n,
                                                         u64 D, DType t, u8* __restrict__ ws,
                                                         u32 c_base, u32 vflags,
                                                         i32* __restrict__ status) {
    __shared__ zb::Group groups[6];
    __shared__ __attribute__((aligned(16))) u8 lensb[6 * 260];
    __shared__ u16 lut[6 << zb::LUT_BITS];
    __shared__ __attribute__((aligned(16))) u8 seq[256];
    __shared__ u32 hist[4][256];
    __shared__ u16 succ[BZ_NSAMP + 1];
    __shared__ u32 slen[BZ_NSAMP + 1];
    __shared__ u32 soff[BZ_NSAMP + 1];
    __shared__ u32 tstate[BZ_T];
    __shared__ u32 tcrc[BZ_T];
    __shared__ u32 tlen[BZ_T];
    __shared__ u32 scan_tmp[8];
    __shared__ BzShared sh;

    const u32 c = c_base + blockIdx.x;
    if (c >= n) return;
    const u32 tid = threadIdx.x, lane = tid & 63;
    const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const zcg_chunk ch = chunks[c];
    if (D > 0 && ch.dst_cap < D) {
        if (tid == 0) status[c] = ZCG_ERR_INVALID_INPUT;
        return;
    }
    if (D == 0) {
        if (tid == 0) status[c] = ZCG_OK;
        return;
    }
    u8* slot = ws + (u64)blockIdx.x * BZ_SLOT;
    gu8* L = (gu8*)(slot + BZ_OFF_L);
    gu8* T = (gu8*)(slot + BZ_OFF_T);
    gu32* N = (gu32*)(slot + BZ_OFF_N);
    gu8* dst = (gu8*)ch.dst;

    BzDevIO io;
    zb::BzState s;
    if (wave == 0) {
        io.src = (const gu8*)ch.src;
        io.n = ch.src_len;
        io.wbase = ~0ull >> 1;
        io.wlo = io.whi = 0;
        io.groups = groups;
        io.lensb = (lu8*)lensb;
        io.lut = (lu16*)lut;
        io.seq = (lu8*)seq;
        io.sel = (gu8*)(slot + BZ_OFF_SEL);
        io.L = L;
        io.sbase = 0xFFFFFFF0u;
        io.sw0 = io.sw1 = io.sw2 = io.sw3 = 0;
        io.mtfw = 0;
        io.lbuf = 0;
        io.lane = lane;
        s.n = ch.src_len;
        s.lim = ch.src_len;
        s.bitpos = 0;
        s.level = 0;
        s.full = 0;
        s.header_done = 0;
        s.combined = 0;
        s.stored_crc = s.randomised = s.orig_ptr = s.nblock = 0;
        s.err_line = 0;
    }
    if (tid == 0) sh.out_pos = 0;
    int final_status = -1;

    for (;;) {
        // ---------------- stage A ----------------
        if (wave == 0) {
            const int r = zb::bz_block(io, s);
            if (lane == 0) {
                sh.r = r;
                sh.nblock = s.nblock;
                sh.orig = s.orig_ptr;
                sh.stored_crc = s.stored_crc;
                sh.randomised = s.randomised;
                sh.level = (r == zb::ST_INVALID) ? s.err_line : s.level;
                sh.full = s.full;
            }
            io.l_flush(s.nblock * (r == zb::R_BLOCK ? 1u : 0u));
        }
        __syncthreads();
        const int r = sh.r;
        if (r == zb::R_STOP || r == zb::R_END) { final_status = sh.full ? ZCG_OK : ZCG_ERR_UNEXPECTED_EOF; break; }
        if (r != zb::R_BLOCK) {
            final_status = r;
            if ((vflags & ZCG_FLAG_DEBUG_COUNTERS) && r == zb::ST_INVALID) final_status = 10000 + (int)sh.level;
            break;
        }
        if (sh.full) { final_status = ZCG_OK; break; }
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
            if (ok) N[b + rank] = i;
            if (ok && (u32)__builtin_ctzll(m) == lane) hist[wave][v] = b + (u32)__builtin_popcountll(m);
        }
        __syncthreads();

        // ---------------- stage B: list ranking of the chain p -> N[p] ----------------
        const u32 p0 = N[sh.orig];
        u32 lgs = 0;
        while (((u64)BZ_NSAMP << lgs) < nblock) lgs++;
        const u32 S = 1u << lgs, smask = S - 1;
        const u32 NR = (nblock + S - 1) >> lgs;
        const bool extra = (p0 & smask) != 0;
        const u32 sid0 = extra ? NR : (p0 >> lgs);
#define BZ_IS_SAMPLE(p) ((((p) & smask) == 0) || ((p) == p0))
#define BZ_SID(p) ((((p) & smask) == 0) ? ((p) >> lgs) : NR)
        for (u32 k = tid; k <= BZ_NSAMP; k += BZ_T) soff[k] = 0xFFFFFFFFu;
        {
            u32 ps[5], ln[5], sidk[5];
            u32 act = 0;
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const u32 sd = (k < 4) ? tid + (u32)k * BZ_T : NR;
                const bool on = (k < 4) ? sd < NR : (tid == 0 && extra);
                sidk[k] = sd;
                ps[k] = (k < 4) ? (sd << lgs) : p0;
                ln[k] = 0;
                if (on) act |= 1u << k;
            }
            while (act) {
                u32 nx[5];
#pragma unroll
                for (int k = 0; k < 5; k++) nx[k] = (act >> k & 1) ? N[ps[k]] : 0u;
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    if (!(act >> k & 1)) continue;
                    ln[k]++;
                    ps[k] = nx[k];
                    if (BZ_IS_SAMPLE(nx[k])) {
                        succ[sidk[k]] = (u16)BZ_SID(nx[k]);
                        slen[sidk[k]] = ln[k];
                        act &= ~(1u << k);
                    }
                }
            }
        }
        __syncthreads();
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
        if (sh.single) {
            u32 ps[5], ln[5], of[5];
            u32 act = 0;
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const u32 sd = (k < 4) ? tid + (u32)k * BZ_T : NR;
                const bool on = (k < 4) ? sd < NR : (tid == 0 && extra);
                ps[k] = (k < 4) ? (sd << lgs) : p0;
                of[k] = on ? soff[sd] : 0;
                ln[k] = on ? slen[sd] : 0;
                if (on && of[k] != 0xFFFFFFFFu && ln[k]) act |= 1u << k;
            }
            while (act) {
                u32 nx[5], by[5];
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    nx[k] = (act >> k & 1) ? N[ps[k]] : 0u;
                    by[k] = (act >> k & 1) ? (u32)L[ps[k]] : 0u;
                }
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    if (!(act >> k & 1)) continue;
                    T[of[k]++] = (u8)by[k];
                    ps[k] = nx[k];
                    if (--ln[k] == 0) act &= ~(1u << k);
                }
            }
        } else if (tid == 0) {
            // not one cycle (corrupt): libbz2's serial tPos walk
            u32 p = p0;
            for (u32 k = 0; k < nblock; k++) {
                T[k] = L[p];
                p = N[p];
            }
        }
#undef BZ_IS_SAMPLE
#undef BZ_SID
        __syncthreads();
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
        {
            u32 st0 = 0, st1 = 1, st2 = 2, st3 = 3, st4 = 4;
            u32 pc = a0 ? (u32)T[a0 - 1] : 0u;
            for (u32 k = a0; k < a1; k++) {
                const u32 cb = T[k];
                st0 = rle_trans(st0, cb, pc); st1 = rle_trans(st1, cb, pc);
                st2 = rle_trans(st2, cb, pc); st3 = rle_trans(st3, cb, pc);
                st4 = rle_trans(st4, cb, pc);
                pc = cb;
            }
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
            u32 pc = a0 ? (u32)T[a0 - 1] : 0u;
            for (u32 k = a0; k < a1; k++) {
                const u32 cb = T[k];
                cnt_out += (stt == 4) ? cb : 1u;
                stt = rle_trans(stt, cb, pc);
                pc = cb;
            }
        }
        u32 blk_total;
        const u32 my_off = block_scan_u32(cnt_out, scan_tmp, &blk_total);
        const u64 ob = sh.out_pos;
        const bool tail4 = sh.done_status == 4;  // a run of four without its count byte
        const bool complete = !tail4 && ob + blk_total <= D;
        {
            u32 stt = tstate[tid];
            u32 pc = a0 ? (u32)T[a0 - 1] : 0u;
            u64 op = ob + my_off;
            u32 crc = 0xFFFFFFFFu;
            for (u32 k = a0; k < a1; k++) {
                const u32 cb = T[k];
                const u32 reps = (stt == 4) ? cb : 1u;
                const u32 val = (stt == 4) ? pc : cb;
                for (u32 r2 = 0; r2 < reps; r2++, op++) {
                    if (op < D) dst[swap_pos(op, t)] = norm_byte((u8)val, t);
                    if (complete) crc = (crc << 8) ^ g_bzcrc.t[((crc >> 24) ^ val) & 0xFF];
                }
                stt = rle_trans(stt, cb, pc);
                pc = cb;
            }
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
        if ((int)sh.done_status >= 0) { final_status = (int)sh.done_status; break; }
        if (wave == 0) {
            const u32 bcrc = tcrc[0];
            s.combined = ((s.combined << 1) | (s.combined >> 31)) ^ bcrc;
            if (sh.out_pos == D) {
                s.full = 1;
                const u64 used = (s.bitpos + 7) >> 3;
                const u64 ve = ((used ? used - 1 : 0) / zb::BUFREADER + 1) * zb::BUFREADER;
                s.lim = ve < s.n ? ve : s.n;
            }
        }
        __syncthreads();
    }
    if (tid == 0) status[c] = final_status;
}

uint64_t bzip2_decode_ws_bytes(const zcg_array* a, uint32_t n) {
    (void)a;
    const u32 slots = n < BZ_MAX_SLOTS ? n : BZ_MAX_SLOTS;
    return (u64)slots * BZ_SLOT;
}

hipError_t launch_bzip2_decode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                               int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const u32 slots = n < BZ_MAX_SLOTS ? n : BZ_MAX_SLOTS;
    if (ws_bytes < (u64)slots * BZ_SLOT) return hipErrorInvalidValue;
    for (u32 c0 = 0; c0 < n; c0 += slots) {
        const u32 cnt = (n - c0) < slots ? (n - c0) : slots;
        hipLaunchKernelGGL(bz2_decode_kernel, dim3(cnt), dim3(BZ_T), 0, s, d_chunks, n, D, t,
                           (u8*)ws, c0, a->compression.flags, d_status);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace zcg
