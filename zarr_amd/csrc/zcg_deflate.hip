// zcg_deflate.hip — gzip encoder (write_chunk for CompressionType::Gzip).
//
// Reference: gzip.rs:50-56 wraps the writer in flate2's GzEncoder at the
// effective level (gzip.rs:28-39: -1 / out of [0,9] -> 6): a 10-byte header
// 1f 8b 08 00 | mtime 0 | XFL | OS 255 (XFL 2 at level >= 9, 4 at level <= 1,
// else 0), zlib raw deflate, then CRC32 and ISIZE (LE).  Encoded bytes are not
// pinned beyond the doc-spec vector; the contract is: the stream
// inflates (zlib) to exactly the serialised chunk, with those conventions.
// The block-type choice (stored / fixed / dynamic by size, fixed on a tie)
// follows zlib's _tr_flush_block, which is what reproduces the doc-spec vector.
//
// Layout (stream-ordered kernels):
//   0. match finding over whole chunks, data-parallel (<= 128 MiB per
//      sub-batch): keys (chunk, the 3 serialised bytes) sorted with the
//      positions as values (hipCUB radix sort, stable), df_chain links each
//      position to its predecessor with the same 3 bytes, df_best walks up to
//      zlib's max_chain (capped at 64) candidates within 32 KiB and keeps the
//      longest match (nearest on ties, zlib's nice_length stops the walk).
//   1. deflate_segment: one wave per 16 KiB input segment.  The segment and
//      the 32 KiB before it (deflate's window) are staged in LDS with the
//      dtype transform applied (write_data's byte order, chunk.rs:118-140).
//      Every position's longest match comes precomputed (step 0); the
//      64 lanes read 64 consecutive positions' matches and the wave walks them
//      greedily (one-step lazy evaluation at level >= 4).  Pass A runs the parse for symbol
//      frequencies; the wave builds length-limited Huffman codes (zlib's
//      bl_count overflow rule) and picks stored/fixed/dynamic; pass B re-runs
//      the same deterministic parse and emits the bits through an LDS ring
//      (wave prefix sums place 64 literal codes at once).  A non-final
//      segment ends with an empty stored block so it is byte aligned.
//      Segment k is written at its upper-bound slot of dst.
//   2. deflate_finalize: per chunk, the gzip header and segment compaction.
//   3. gzip_crc32: per chunk, 64 lanes CRC their slices, lane 0 combines them
//      with a precomputed GF(2) shift operator; CRC32 + ISIZE trailer.
#include <hipcub/hipcub.hpp>

#include "zcg_common.h"
#include "zcg_zlib_core.h"

namespace zcg {

constexpr u32 DF_SEG = 16384;               // input bytes per segment (one deflate block)
constexpr u32 DF_HIST = 32768;              // deflate window
constexpr u32 DF_WIN = DF_SEG + DF_HIST;
constexpr u32 DF_SLOT = DF_SEG + 128;       // output slot per segment (stored worst case + sync)
constexpr u32 DF_RING = 1024;               // output ring words
constexpr u32 DF_FLUSH = 512;
constexpr u32 DF_HDR = 10;

__constant__ u16 d_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ u8 d_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                   2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ u16 d_dist_base[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                    33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                    1025, 1537, 2049, 3073, 4097, 6145,  8193,  12289, 16385,
                                    24577};
__constant__ u8 d_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                                    6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ u8 d_clen_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ u32 len_code(u32 len) {  // 3..258 -> 0..28 (d_len_base)
    if (len == 258) return 28;
    const u32 x = len - 3;
    if (x < 8) return x;
    const u32 k = 31 - __builtin_clz(x);  // 3..7
    return 4 * (k - 1) + ((x >> (k - 2)) & 3);
}
__device__ __forceinline__ u32 dist_code(u32 d) {  // 1..32768 -> 0..29 (d_dist_base)
    const u32 x = d - 1;
    if (x < 4) return x;
    const u32 k = 31 - __builtin_clz(x);  // 2..14
    return 2 * k + ((x >> (k - 1)) & 1);
}
__device__ __forceinline__ u32 rev_bits(u32 v, u32 n) { return n ? __builtin_bitreverse32(v) >> (32 - n) : 0u; }

struct DefLds {
    u32 lfreq[288], dfreq[32], cfreq[20];
    u32 lcode[288], dcode[32], ccode[20];  // (length << 16) | bit-reversed code
    u32 ring[DF_RING];
    // Huffman construction scratch
    u16 sorted[288];
    u16 parent[576];
    u16 depth[576];
    u32 wq[288];               // internal node weights (two-queue construction)
    u8 clens[320];             // code lengths: litlen [0,286), dist [288,318)
    u8 clcl[20];               // code-length code lengths
    u8 seq[320];               // litlen ++ dist lengths for the RLE
    u16 rle[320];              // code-length symbols: sym | extra << 8
    u32 ctl[16];
};

// Bits into the LDS ring at absolute bit position `bp` (value < 2^n, n <= 32).
__device__ __forceinline__ void ring_put(DefLds& L, u32 bp, u32 v, u32 n) {
    if (!n) return;
    const u32 w = bp >> 5, sh = bp & 31;
    atomicOr(&L.ring[w & (DF_RING - 1)], v << sh);
    if (sh + n > 32) atomicOr(&L.ring[(w + 1) & (DF_RING - 1)], v >> (32 - sh));
}

// Flush complete ring words [*fw, upto) to out (wave-cooperative).
constexpr u32 DF_OUTCAP = DF_SLOT - 4;   // bytes a segment may write after its length word
constexpr u32 CTL_ERR = 8;               // L.ctl slot: pass B inconsistency / overrun

__device__ void ring_flush(DefLds& L, u8* out, u32* fw, u32 upto) {
    const u32 lane = lane_id();
    __syncthreads();
    for (u32 w = *fw + lane; w < upto; w += 64) {
        const u32 v = L.ring[w & (DF_RING - 1)];
        if (4 * w + 4 <= DF_OUTCAP) {
            u8* o = out + 4ull * w;
            o[0] = (u8)v; o[1] = (u8)(v >> 8); o[2] = (u8)(v >> 16); o[3] = (u8)(v >> 24);
        } else {
            L.ctl[CTL_ERR] = 1;  // would overrun the slot: the segment falls back to stored
        }
        L.ring[w & (DF_RING - 1)] = 0;
    }
    *fw = upto;
    __syncthreads();
}

// Length-limited Huffman code lengths for freq[0..n) (n <= 288), wave-wide.
// Symbols with freq 0 get length 0; if fewer than 2 symbols are used, the
// first unused of symbols 0/1 gets freq 1 (zlib build_tree forces 2 codes).
__device__ void huff_lengths(DefLds& L, u32* freq, u32 n, u32 maxbits, u8* len_out) {
    const u32 lane = lane_id();
    __syncthreads();
    if (lane == 0) {
        u32 used = 0;
        for (u32 i = 0; i < n; i++) used += freq[i] != 0;
        for (u32 i = 0; used < 2 && i < 2; i++)
            if (!freq[i]) { freq[i] = 1; used++; }
    }
    __syncthreads();
    // rank sort by (freq, symbol) ascending, zero-frequency symbols excluded
    for (u32 s = lane; s < n; s += 64) {
        const u32 f = freq[s];
        if (!f) { len_out[s] = 0; continue; }
        u32 r = 0;
        for (u32 t = 0; t < n; t++) {
            const u32 g = freq[t];
            r += (g && (g < f || (g == f && t < s))) ? 1u : 0u;
        }
        L.sorted[r] = (u16)s;
    }
    __syncthreads();
    if (lane == 0) {
        u32 m = 0;
        for (u32 i = 0; i < n; i++) m += freq[i] != 0;
        // two-queue Huffman: leaves 0..m-1 (sorted), internal nodes m..2m-2
        u32* wq = L.wq;
        u32 li = 0, ii = 0, nint = 0;
        for (u32 k = 0; k + 1 < m; k++) {
            u32 pick[2];
            u32 wsum = 0;
            for (u32 j = 0; j < 2; j++) {
                const bool leaf = li < m && (ii >= nint || freq[L.sorted[li]] <= wq[ii]);
                if (leaf) { pick[j] = li; wsum += freq[L.sorted[li]]; li++; }
                else { pick[j] = m + ii; wsum += wq[ii]; ii++; }
            }
            L.parent[pick[0]] = (u16)(m + nint);
            L.parent[pick[1]] = (u16)(m + nint);
            wq[nint++] = wsum;
        }
        // depths: root = m + nint - 1
        u32 blc[16];
        for (u32 b = 0; b < 16; b++) blc[b] = 0;
        if (m == 1) {
            blc[1] = 1;
        } else {
            // zlib gen_bitlen: depths top-down from the CLAMPED parent depth;
            // every node (internal or leaf) pushed past maxbits counts as overflow
            L.depth[m + nint - 1] = 0;
            int overflow = 0;
            for (int x = (int)(m + nint) - 2; x >= 0; x--) {
                u32 d = (u32)L.depth[L.parent[x]] + 1;
                if (d > maxbits) { d = maxbits; overflow++; }
                L.depth[x] = (u16)d;
                if ((u32)x < m) blc[d]++;
            }
            while (overflow > 0) {  // zlib gen_bitlen
                u32 b = maxbits - 1;
                while (blc[b] == 0) b--;
                blc[b]--;
                blc[b + 1] += 2;
                blc[maxbits]--;
                overflow -= 2;
            }
        }
        // least frequent symbols get the longest codes
        u32 h = 0;
        for (u32 b = maxbits; b >= 1; b--)
            for (u32 c = blc[b]; c > 0; c--) len_out[L.sorted[h++]] = (u8)b;
    }
    __syncthreads();
}

// Canonical codes (bit-reversed for LSB-first output): code[s] = len << 16 | rev.
__device__ void huff_codes(const u8* len, u32 n, u32* code) {
    if (lane_id() != 0) return;
    u32 blc[16], next[16];
    for (u32 b = 0; b < 16; b++) blc[b] = 0;
    for (u32 s = 0; s < n; s++) blc[len[s]]++;
    blc[0] = 0;
    u32 c = 0;
    for (u32 b = 1; b < 16; b++) { c = (c + blc[b - 1]) << 1; next[b] = c; }
    for (u32 s = 0; s < n; s++) {
        const u32 l = len[s];
        code[s] = l ? ((l << 16) | rev_bits(next[l]++, l)) : 0u;
    }
}

// Fixed Huffman code (RFC 1951 3.2.6).
__device__ __forceinline__ u32 fixed_lcode(u32 s) {
    if (s < 144) return (8u << 16) | rev_bits(0x30 + s, 8);
    if (s < 256) return (9u << 16) | rev_bits(0x190 + (s - 144), 9);
    if (s < 280) return (7u << 16) | rev_bits(s - 256, 7);
    return (8u << 16) | rev_bits(0xC0 + (s - 280), 8);
}

struct ParseCfg {
    bool lazy;     // one-step lazy evaluation
    bool insert;   // insert positions inside matches
};

// One pass of the segment parse over window positions [h0, wend).
// EMIT=false: symbol frequencies.  EMIT=true: bits into the ring (bp, fw).
template <bool EMIT>
__device__ void parse_pass(DefLds& L, u32 h0, u32 wend, ParseCfg cfg, u32* bp, u32* fw, u8* out,
                           const u32* __restrict__ mt, const u8* __restrict__ src, u64 w0, DType t) {
    const u32 lane = lane_id();
    u32 ip = h0;
    while (ip < wend) {
        // keep the ring from wrapping: a group adds < 2 Kbit
        if (EMIT && (*bp >> 5) >= *fw + DF_FLUSH) ring_flush(L, out, fw, *bp >> 5);
        const u32 gend = (wend - ip) < 64 ? (wend - ip) : 64u;  // positions of this group
        const u32 p = ip + lane;
        const bool valid = lane < gend && p + 3 <= wend;
        // the precomputed longest match of this position (df_best), clipped to the segment
        const u32 m = valid ? mt[p] : 0u;
        u32 bl = m & 0x1FF, br = p - ((m >> 16) + 1);
        if (bl > wend - p) bl = wend - p;
        if (bl < 3 || (bl == 3 && p - br > 4096)) bl = 0;  // zlib TOO_FAR
        const unsigned long long mask = __ballot(bl >= 3);
        // The greedy (lazy) parse of the group as a chain over its positions:
        // position p steps to p + 1 (literal), p + len (match) or, when the
        // next position holds a longer match (lazy evaluation), emits a
        // literal and that match and steps to p + 1 + len'.  The chain from 0
        // is found by pointer doubling (lane k gets its k-th member in six
        // ds_bpermute rounds), and the members emit in parallel at bit
        // offsets from a wave prefix sum: the same parse, decisions and bits
        // as a serial walk (zlib deflate_slow's order).
        (void)mask;
        const u32 bl1 = (u32)__shfl((int)bl, (int)((lane + 1) & 63), 64);
        const u32 br1 = (u32)__shfl((int)br, (int)((lane + 1) & 63), 64);
        const bool ism = bl >= 3;
        const bool lz = cfg.lazy && ism && bl < 32 && lane + 1 < gend && bl1 > bl;
        const u32 nx = !ism ? lane + 1 : lz ? lane + 1 + bl1 : lane + bl;
        u32 J[6];
        J[0] = nx;
#pragma unroll
        for (u32 k = 1; k < 6; k++) {
            const u32 t = (u32)__shfl((int)J[k - 1], (int)(J[k - 1] & 63), 64);
            J[k] = J[k - 1] < 64 ? t : J[k - 1];
        }
        u32 cur = 0;  // position of member #lane
#pragma unroll
        for (u32 k = 0; k < 6; k++) {
            const u32 t = (u32)__shfl((int)J[k], (int)(cur & 63), 64);
            if ((lane >> k) & 1u) cur = cur < 64 ? t : cur;
        }
        const bool mem = cur < gend;
        const u32 nm = (u32)__popcll(__ballot(mem));  // >= 1: position 0 is a member
        const u32 lastp = (u32)__builtin_amdgcn_readlane((int)cur, (int)(nm - 1));
        const u32 pos = (u32)__builtin_amdgcn_readlane((int)nx, (int)lastp);  // first position after the group's chain
        // my member's unit: literal, match, or literal + match (lazy)
        const u32 q = cur & 63;
        const u32 qism = (u32)__shfl((int)(ism ? 1u : 0u), (int)q, 64);
        const u32 qlz = (u32)__shfl((int)(lz ? 1u : 0u), (int)q, 64);
        const u32 qbl = (u32)__shfl((int)bl, (int)q, 64), qbr = (u32)__shfl((int)br, (int)q, 64);
        const u32 qbl1 = (u32)__shfl((int)bl1, (int)q, 64), qbr1 = (u32)__shfl((int)br1, (int)q, 64);
        const bool hlit = mem && (!qism || qlz);  // a literal at q
        const bool hmat = mem && qism;            // a match at q (or q + 1 when lazy)
        const u32 mpos = ip + q + (qlz ? 1u : 0u);
        const u32 mlen = qlz ? qbl1 : qbl;
        const u32 d = mpos - (qlz ? qbr1 : qbr);
        const u32 byte = hlit ? (u32)norm_byte(src[swap_pos(w0 + ip + q, t)], t) : 0u;
        const u32 lc = hmat ? len_code(mlen) : 0u, dc = hmat ? dist_code(d) : 0u;
        if (!EMIT) {
            if (hlit) atomicAdd(&L.lfreq[byte], 1u);
            if (hmat) { atomicAdd(&L.lfreq[257 + lc], 1u); atomicAdd(&L.dfreq[dc], 1u); }
        } else {
            const u32 cw = hlit ? L.lcode[byte] : 0u;
            const u32 nb = cw >> 16;
            const u32 lcw = hmat ? L.lcode[257 + lc] : 0u, dcw = hmat ? L.dcode[dc] : 0u;
            const u32 nl = lcw >> 16, nd = dcw >> 16;
            const u32 el = hmat ? (u32)d_len_extra[lc] : 0u, ed = hmat ? (u32)d_dist_extra[dc] : 0u;
            if ((hlit && nb == 0) || (hmat && (nl == 0 || nd == 0))) L.ctl[CTL_ERR] = 1;
            const u32 nbits = nb + nl + el + nd + ed;
            u32 x = nbits;  // wave inclusive scan of the units' bit counts
#pragma unroll
            for (int dd = 1; dd < 64; dd <<= 1) {
                const u32 y = (u32)__shfl_up((int)x, dd, 64);
                if ((int)lane >= dd) x += y;
            }
            const u32 tot = (u32)__shfl((int)x, 63, 64);
            u32 b = *bp + x - nbits;
            if (hlit) { ring_put(L, b, cw & 0xFFFF, nb); b += nb; }
            if (hmat) {
                ring_put(L, b, lcw & 0xFFFF, nl); b += nl;
                ring_put(L, b, mlen - d_len_base[lc], el); b += el;
                ring_put(L, b, dcw & 0xFFFF, nd); b += nd;
                ring_put(L, b, d - d_dist_base[dc], ed);
            }
            *bp += tot;
        }
        ip += pos;
    }
    if (EMIT && (*bp >> 5) >= *fw + DF_FLUSH) ring_flush(L, out, fw, *bp >> 5);
}

__global__ __launch_bounds__(64) void deflate_segment(const zcg_chunk* __restrict__ chunks, u32 c0, u32 n, u64 D,
                                                      u32 nseg, u64 bound, DType t, u32 level,
                                                      const u32* __restrict__ match) {
    extern __shared__ __attribute__((aligned(16))) u8 smem_raw[];
    DefLds& L = *(DefLds*)smem_raw;
    const u32 lane = threadIdx.x;
    const u32 cl = blockIdx.x / nseg, k = blockIdx.x % nseg;
    if (cl >= n) return;
    const u32 c = c0 + cl;
    const zcg_chunk ch = chunks[c];
    if (ch.dst_cap < bound || ch.src_len < D) return;
    const u8* src = (const u8*)ch.src;
    u8* slot = (u8*)ch.dst + DF_HDR + (u64)k * DF_SLOT;
    u8* out = slot + 4;
    const u64 s0 = (u64)k * DF_SEG;
    const u32 S = (u32)((D - s0) < DF_SEG ? (D - s0) : DF_SEG);
    const u32 hist = (u32)(s0 < DF_HIST ? s0 : DF_HIST);
    const u64 w0 = s0 - hist;
    const u32 wend = hist + S;
    const bool final_seg = (k + 1 == nseg);
    for (u32 q = lane; q < 288; q += 64) L.lfreq[q] = 0;
    if (lane < 32) L.dfreq[lane] = 0;
    if (lane < 20) L.cfreq[lane] = 0;
    for (u32 q = lane; q < DF_RING; q += 64) L.ring[q] = 0;
    __syncthreads();
    u32 bp = 0, fw = 0;
    int btype = 0;  // 0 stored, 1 fixed, 2 dynamic
    u32 hlit = 257, hdist = 1, hclen = 4, nrle = 0;
    if (level > 0) {
        const ParseCfg cfg{level >= 4, level >= 4};
        parse_pass<false>(L, hist, wend, cfg, &bp, &fw, out, match + (u64)cl * D + w0, src, w0, t);
        if (lane == 0) L.lfreq[256] += 1;  // end of block
        __syncthreads();
        // ---- codes and the block type (zlib _tr_flush_block) ------------------------
        huff_lengths(L, L.lfreq, 286, 15, L.clens);
        huff_lengths(L, L.dfreq, 30, 15, L.clens + 288);
        if (lane == 0) {
            hlit = 286;
            while (hlit > 257 && L.clens[hlit - 1] == 0) hlit--;
            hdist = 30;
            while (hdist > 1 && L.clens[288 + hdist - 1] == 0) hdist--;
            // code-length sequence (litlen[0..hlit) ++ dist[0..hdist)), RLE 16/17/18
            u8* seq = L.seq;
            const u32 N = hlit + hdist;
            for (u32 i = 0; i < hlit; i++) seq[i] = L.clens[i];
            for (u32 i = 0; i < hdist; i++) seq[hlit + i] = L.clens[288 + i];
            u32 i = 0;
            nrle = 0;
            while (i < N) {
                const u32 v = seq[i];
                u32 run = 1;
                while (i + run < N && seq[i + run] == v) run++;
                if (v == 0 && run >= 3) {
                    u32 r = run;
                    while (r >= 11) { const u32 a = r < 138 ? r : 138; L.rle[nrle++] = (u16)(18 | ((a - 11) << 8)); r -= a; }
                    if (r >= 3) { L.rle[nrle++] = (u16)(17 | ((r - 3) << 8)); r = 0; }
                    while (r) { L.rle[nrle++] = 0; r--; }
                } else {
                    L.rle[nrle++] = (u16)v;
                    u32 r = run - 1;
                    while (r >= 3) { const u32 a = r < 6 ? r : 6; L.rle[nrle++] = (u16)(16 | ((a - 3) << 8)); r -= a; }
                    while (r) { L.rle[nrle++] = (u16)v; r--; }
                }
                i += run;
            }
            for (u32 j = 0; j < 20; j++) L.cfreq[j] = 0;
            for (u32 j = 0; j < nrle; j++) L.cfreq[L.rle[j] & 31]++;
            L.ctl[1] = hlit; L.ctl[2] = hdist; L.ctl[3] = nrle;
        }
        __syncthreads();
        hlit = L.ctl[1]; hdist = L.ctl[2]; nrle = L.ctl[3];
        huff_lengths(L, L.cfreq, 19, 7, L.clcl);
        huff_codes(L.clens, 286, L.lcode);
        huff_codes(L.clens + 288, 30, L.dcode);
        huff_codes(L.clcl, 19, L.ccode);
        __syncthreads();
        if (lane == 0) {
            hclen = 19;
            while (hclen > 4 && L.clcl[d_clen_order[hclen - 1]] == 0) hclen--;
            // sizes in bits (zlib: opt_len / static_len exclude the 3 header bits)
            u64 opt = 5 + 5 + 4 + 3ull * hclen, stat = 0;
            for (u32 j = 0; j < nrle; j++) {
                const u32 sym = L.rle[j] & 31;
                opt += L.clcl[sym] + (sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0);
            }
            for (u32 s = 0; s < 286; s++) {
                const u32 f = L.lfreq[s];
                if (!f) continue;
                const u32 ex = s >= 257 ? d_len_extra[s - 257] : 0;
                opt += (u64)f * (L.clens[s] + ex);
                stat += (u64)f * ((fixed_lcode(s) >> 16) + ex);
            }
            for (u32 s = 0; s < 30; s++) {
                const u32 f = L.dfreq[s];
                if (!f) continue;
                opt += (u64)f * (L.clens[288 + s] + d_dist_extra[s]);
                stat += (u64)f * (5 + d_dist_extra[s]);
            }
            u64 optb = (opt + 3 + 7) >> 3, statb = (stat + 3 + 7) >> 3;
            if (statb <= optb) optb = statb;
            int bt;
            if ((u64)S + 4 <= optb) bt = 0;
            else if (statb == optb) bt = 1;
            else bt = 2;
            L.ctl[4] = (u32)bt;
            L.ctl[5] = hclen;
        }
        __syncthreads();
        btype = (int)L.ctl[4];
        hclen = L.ctl[5];
    }
    bp = 0;
    fw = 0;
    if (btype == 0) {  // stored block (byte aligned: the segment starts at a byte)
        if (lane == 0) {
            out[0] = final_seg ? 1 : 0;
            out[1] = (u8)S; out[2] = (u8)(S >> 8);
            out[3] = (u8)~S; out[4] = (u8)(~S >> 8);
        }
        for (u32 q = lane; q < S; q += 64) out[5 + q] = norm_byte(src[swap_pos(s0 + q, t)], t);
        if (lane == 0) { const u32 len = 5 + S; slot[0] = (u8)len; slot[1] = (u8)(len >> 8); slot[2] = (u8)(len >> 16); slot[3] = (u8)(len >> 24); }
        return;
    }
    if (btype == 1) {  // fixed codes
        for (u32 s = lane; s < 288; s += 64) L.lcode[s] = fixed_lcode(s);
        if (lane < 32) L.dcode[lane] = (5u << 16) | rev_bits(lane, 5);
    }
    __syncthreads();
    if (lane == 0) {
        u32 b = 0;
        ring_put(L, b, (final_seg ? 1u : 0u) | ((u32)btype << 1), 3); b += 3;
        if (btype == 2) {
            ring_put(L, b, hlit - 257, 5); b += 5;
            ring_put(L, b, hdist - 1, 5); b += 5;
            ring_put(L, b, hclen - 4, 4); b += 4;
            for (u32 j = 0; j < hclen; j++) { ring_put(L, b, L.clcl[d_clen_order[j]], 3); b += 3; }
            for (u32 j = 0; j < nrle; j++) {
                const u32 sym = L.rle[j] & 31, ex = L.rle[j] >> 8;
                const u32 cw = L.ccode[sym];
                ring_put(L, b, cw & 0xFFFF, cw >> 16); b += cw >> 16;
                const u32 eb = sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0;
                ring_put(L, b, ex, eb); b += eb;
            }
        }
        L.ctl[0] = b;
    }
    __syncthreads();
    bp = L.ctl[0];
    // the header may exceed a flush unit only in theory (< 400 bytes); flush if needed
    if ((bp >> 5) >= fw + DF_FLUSH) ring_flush(L, out, &fw, bp >> 5);
    if (lane == 0) L.ctl[CTL_ERR] = 0;
    __syncthreads();
    const ParseCfg cfg{level >= 4, level >= 4};
    parse_pass<true>(L, hist, wend, cfg, &bp, &fw, out, match + (u64)cl * D + w0, src, w0, t);
    if (lane == 0) {
        u32 b = bp;
        const u32 cw = L.lcode[256];
        ring_put(L, b, cw & 0xFFFF, cw >> 16); b += cw >> 16;  // end of block
        if (!final_seg) { b += 3; b = (b + 7) & ~7u; b += 32; }  // empty stored block (sync)
        L.ctl[0] = b;
    }
    __syncthreads();
    bp = L.ctl[0];
    const u32 nbytes = (bp + 7) >> 3;
    // empty stored block after a non-final segment: LEN = 0 (zero bits), NLEN = 0xFFFF
    if (!final_seg && lane == 0) ring_put(L, bp - 16, 0xFFFFu, 16);
    __syncthreads();
    ring_flush(L, out, &fw, (bp + 31) >> 5);
    if (L.ctl[CTL_ERR]) {  // inconsistent or oversized: store the segment instead
        if (lane == 0) {
            out[0] = final_seg ? 1 : 0;
            out[1] = (u8)S; out[2] = (u8)(S >> 8);
            out[3] = (u8)~S; out[4] = (u8)(~S >> 8);
        }
        for (u32 q = lane; q < S; q += 64) out[5 + q] = norm_byte(src[swap_pos(s0 + q, t)], t);
        if (lane == 0) { const u32 len = 5 + S; slot[0] = (u8)len; slot[1] = (u8)(len >> 8); slot[2] = (u8)(len >> 16); slot[3] = (u8)(len >> 24); }
        return;
    }
    if (lane == 0) { slot[0] = (u8)nbytes; slot[1] = (u8)(nbytes >> 8); slot[2] = (u8)(nbytes >> 16); slot[3] = (u8)(nbytes >> 24); }
}

__global__ __launch_bounds__(256) void deflate_finalize(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                        u32 nseg, u64 bound, u32 xfl,
                                                        u64* __restrict__ out_len, i32* __restrict__ status) {
    const u32 c = blockIdx.x, tid = threadIdx.x;
    if (c >= n) return;
    const zcg_chunk ch = chunks[c];
    if (ch.src_len < D) { if (tid == 0) { status[c] = ZCG_ERR_INVALID_DATA; out_len[c] = 0; } return; }
    if (ch.dst_cap < bound) { if (tid == 0) { status[c] = ZCG_ERR_OUTPUT_TOO_SMALL; out_len[c] = 0; } return; }
    u8* dst = (u8*)ch.dst;
    if (tid == 0) {
        const u8 h[10] = {0x1F, 0x8B, 8, 0, 0, 0, 0, 0, (u8)xfl, 255};
        for (u32 i = 0; i < 10; i++) dst[i] = h[i];
    }
    __shared__ u32 s_sz;
    u64 pos = DF_HDR;
    if (nseg == 0) {  // empty input: one final fixed block holding only end-of-block
        if (tid == 0) { dst[pos] = 0x03; dst[pos + 1] = 0x00; }
        pos += 2;
    }
    for (u32 k = 0; k < nseg; k++) {
        const u64 tmp = DF_HDR + (u64)k * DF_SLOT;
        __syncthreads();
        if (tid == 0) s_sz = ld32(dst + tmp);
        __syncthreads();
        const u64 total = s_sz;
        const u64 from = tmp + 4;
        for (u64 q = 0; q < total; q += 256 * 16) {  // dst <= src: all reads of a tile before its writes
            const u64 i = q + (u64)tid * 16;
            u32x4 v = {0u, 0u, 0u, 0u};
            u32 nb = 0;
            if (i < total) {
                nb = (total - i) < 16 ? (u32)(total - i) : 16u;
                if (nb == 16) v = ld16(dst + from + i);
                else for (u32 j = 0; j < nb; j++) ((u8*)&v)[j] = dst[from + i + j];
            }
            __syncthreads();
            if (nb == 16) st16(dst + pos + i, v);
            else for (u32 j = 0; j < nb; j++) dst[pos + i + j] = ((u8*)&v)[j];
            __syncthreads();
        }
        pos += total;
    }
    if (tid == 0) {
        out_len[c] = pos + 8;  // + CRC32 + ISIZE (kernel 3)
        status[c] = ZCG_OK;
    }
}

// GF(2) operator (32 columns) applied to a CRC: M * v.
__device__ __forceinline__ u32 gf2_times(const u32* M, u32 v) {
    u32 s = 0;
    for (u32 i = 0; v; i++, v >>= 1)
        if (v & 1) s ^= M[i];
    return s;
}

struct CrcShift { u32 m[32]; };

// 64 lanes per chunk: lane l CRCs slice l (the remainder goes to slice 0), then
// lane 0 folds them with the operator that advances a register over Lsl bytes.
// With crc_out set, only the CRC of each chunk's input is stored there (for
// the trailer dz_final writes; status and out_len are not read).
__global__ __launch_bounds__(64) void gzip_crc32(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                 u64 Lsl, CrcShift op, const u64* __restrict__ out_len,
                                                 const i32* __restrict__ status, DType t, u32* __restrict__ crc_out) {
    const u32 c = blockIdx.x, lane = threadIdx.x;
    if (c >= n) return;
    if (crc_out ? chunks[c].src_len < D : status[c] != ZCG_OK) return;
    const u8* src = (const u8*)chunks[c].src;
    const u64 rem = D - 64 * Lsl;  // slice 0 length = Lsl + rem
    const u64 a = lane == 0 ? 0 : rem + lane * Lsl;
    const u64 b = rem + (lane + 1) * Lsl;
    // raw CRC registers: slice 0 starts from 0xFFFFFFFF, the others from 0, so
    // R(A||B) = shift_len(B)(R(A)) ^ R0(B) folds them (zlib crc32_combine)
    u32 crc = lane == 0 ? 0xFFFFFFFFu : 0u;
    u64 p = a;
    for (; p < b && (p & 15); p++) crc = g_crc32_table[(crc ^ norm_byte(src[swap_pos(p, t)], t)) & 0xFF] ^ (crc >> 8);
    for (; p + 16 <= b; p += 16) {
        const u32x4 v = transform16(ld16(src + p), t);
        const u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (u32 j = 0; j < 4; j++) {
            u32 x = w[j];
#pragma unroll
            for (u32 q = 0; q < 4; q++) { crc = g_crc32_table[(crc ^ x) & 0xFF] ^ (crc >> 8); x >>= 8; }
        }
    }
    for (; p < b; p++) crc = g_crc32_table[(crc ^ norm_byte(src[swap_pos(p, t)], t)) & 0xFF] ^ (crc >> 8);
    __shared__ u32 s_crc[64];
    s_crc[lane] = crc;
    __syncthreads();
    if (lane != 0) return;
    u32 r = s_crc[0];
    for (u32 l = 1; l < 64; l++) r = gf2_times(op.m, r) ^ s_crc[l];
    r ^= 0xFFFFFFFFu;
    if (crc_out) {
        crc_out[c] = r;
        return;
    }
    u8* o = (u8*)chunks[c].dst + out_len[c] - 8;
    o[0] = (u8)r; o[1] = (u8)(r >> 8); o[2] = (u8)(r >> 16); o[3] = (u8)(r >> 24);
    const u32 isz = (u32)D;
    o[4] = (u8)isz; o[5] = (u8)(isz >> 8); o[6] = (u8)(isz >> 16); o[7] = (u8)(isz >> 24);
}

// Host: operator that advances a raw CRC register over `len` zero bytes
// (zlib crc32_combine's gf2 matrix powers).
static void gf2_square(u32* sq, const u32* m) {
    for (int i = 0; i < 32; i++) {
        u32 v = m[i], s = 0;
        for (int j = 0; v; j++, v >>= 1)
            if (v & 1) s ^= m[j];
        sq[i] = s;
    }
}
static void crc_shift_op(u64 len, u32* out) {
    u32 odd[32], even[32], res[32];
    odd[0] = 0xEDB88320u;  // one zero bit
    for (int i = 1; i < 32; i++) odd[i] = 1u << (i - 1);
    gf2_square(even, odd);  // 2 bits
    gf2_square(odd, even);  // 4 bits
    for (int i = 0; i < 32; i++) res[i] = 1u << i;  // identity
    // res = op^(8*len): square up through bits of len (each step: 8 bits * 2^k)
    u32 cur[32];
    gf2_square(cur, odd);  // 8 bits = one byte
    while (len) {
        if (len & 1) {
            u32 t[32];
            for (int i = 0; i < 32; i++) {
                u32 v = res[i], s = 0;
                for (int j = 0; v; j++, v >>= 1)
                    if (v & 1) s ^= cur[j];
                t[i] = s;
            }
            for (int i = 0; i < 32; i++) res[i] = t[i];
        }
        len >>= 1;
        if (len) {
            u32 t[32];
            gf2_square(t, cur);
            for (int i = 0; i < 32; i++) cur[i] = t[i];
        }
    }
    for (int i = 0; i < 32; i++) out[i] = res[i];
}

namespace {

constexpr u64 DF_SUB_BYTES = 128ull << 20;  // input bytes per match-finder sub-batch
constexpr u64 DF_SUPER_BYTES = 1ull << 30;  // input bytes per segment launch

struct DfLayout {
    u32 m, sm;
    u64 tot, cub_bytes;
    u64 off_ka, off_kb, off_va, off_vb, off_prev, off_match, off_cub, total;
};

DfLayout df_layout(u64 D, u32 n) {
    DfLayout y{};
    u64 m = D ? DF_SUB_BYTES / D : n;
    if (m < 1) m = 1;
    if (m > n) m = n;
    if (m > 256) m = 256;  // chunk id + 24 key bits fit 32
    y.m = (u32)m;
    y.tot = m * D;
    u64 sm = D ? DF_SUPER_BYTES / D : n;
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
    y.off_match = take(4 * (u64)y.sm * D);
    y.off_cub = take(y.cub_bytes);
    y.total = p;
    return y;
}

__device__ __forceinline__ u32 df_ser1(const u8* src, u64 x, const DType& t) {
    return norm_byte(((const gu8*)src)[swap_pos(x, t)], t);
}
typedef __attribute__((address_space(1))) u32 df_gu32_ua __attribute__((aligned(1)));
__device__ __forceinline__ u32 df_ser4(const u8* src, u64 x, const DType& t) {  // bytes x..x+3, LE
    if (!t.swap && !t.isbool) return *(const df_gu32_ua*)((const gu8*)src + x);  // (global, not flat)
    return df_ser1(src, x, t) | (df_ser1(src, x + 1, t) << 8) | (df_ser1(src, x + 2, t) << 16) |
           (df_ser1(src, x + 3, t) << 24);
}

__global__ void df_keys(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, u64 tot, DType t,
                        u32* __restrict__ keys, u32* __restrict__ vals) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tot) return;
    const u32 cl = (u32)(g / D);
    const u64 p = g - (u64)cl * D;
    const zcg_chunk ch = chunks[c0 + cl];
    const u8* src = (const u8*)ch.src;
    u32 v = 0;
    if (p + 3 <= D && ch.src_len >= D) v = df_ser1(src, p, t) | (df_ser1(src, p + 1, t) << 8) | (df_ser1(src, p + 2, t) << 16);
    keys[g] = (cl << 24) | v;
    vals[g] = (u32)g;
}

__global__ void df_chain(u64 tot, const u32* __restrict__ keys, const u32* __restrict__ vals,
                         u32* __restrict__ prev) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= tot) return;
    prev[vals[j]] = (j > 0 && keys[j] == keys[j - 1]) ? vals[j - 1] : 0xFFFFFFFFu;
}

// match[g] = len | (dist - 1) << 16 of the longest match at g (len 0: none)
__global__ void df_best(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, u64 tot, DType t, u32 depth,
                        u32 nice, const u32* __restrict__ prev, u32* __restrict__ match) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tot) return;
    const u32 cl = (u32)(g / D);
    const u64 p = g - (u64)cl * D;
    u32 best = 0, bd = 0;
    if (p + 3 <= D && chunks[c0 + cl].src_len >= D) {  // a short src is INVALID_DATA (deflate_finalize)
        const u8* src = (const u8*)chunks[c0 + cl].src;
        const u64 cbase = (u64)cl * D;
        const u32 mx = (D - p) < 258 ? (u32)(D - p) : 258u;
        // bytes p+3..p+6 are compared with every candidate: load them once;
        // the next chain link is loaded before this candidate's compare
        const u32 pw = mx >= 7 ? df_ser4(src, p + 3, t) : 0u;
        u32 q = prev[g];
        for (u32 dep = 0; dep < depth && q != 0xFFFFFFFFu; dep++) {
            const u64 qp = q - cbase;
            if (p - qp > DF_HIST) break;
            const u32 qn = prev[q];
            u32 k = 3;  // the 3 key bytes are equal
            bool diff = false;
            if (mx >= 7) {
                const u32 x = pw ^ df_ser4(src, qp + 3, t);
                if (x) { k += (u32)__builtin_ctz(x) >> 3; diff = true; }
                else k = 7;
            }
            while (!diff && k + 4 <= mx) {
                const u32 x = df_ser4(src, p + k, t) ^ df_ser4(src, qp + k, t);
                if (x) { k += (u32)__builtin_ctz(x) >> 3; diff = true; break; }
                k += 4;
            }
            if (!diff)
                while (k < mx && df_ser1(src, p + k, t) == df_ser1(src, qp + k, t)) k++;
            if (k > best && !(k == 3 && p - qp > 4096)) { best = k; bd = (u32)(p - qp); }
            if (best >= nice) break;
            q = qn;
        }
    }
    match[g] = best ? (best | ((bd - 1) << 16)) : 0u;
}

}  // namespace

// ===================== zlib-exact deflate (levels 4-9) ==========================
// gzip.rs:54-56 writes flate2's GzEncoder, i.e. zlib deflate_slow at levels
// 4-9.  zcg_zlib_core.h restates it as (1) a per-position match search,
// (2) a short sequential lazy parse and (3) per-block trees; the kernels
// below run (1) over every position (data-parallel), (2) one wave per chunk
// (wave-uniform, scalar), (3) one wave per block, then place the blocks'
// bits at their prefix-summed offsets.  Output bytes are identical to zlib's
// (tests/test_hostcore.py pins the core on the CPU, tests/test_gpu_encode.py
// the kernels).
namespace {

constexpr u64 DZ_SUPER_BYTES = 512ull << 20;  // input bytes per super-batch (match results kept for all)
#ifndef ZDZ_SUB_MIB
#define ZDZ_SUB_MIB 128  // (256: 125.7 vs 125.6-126.0 ms per C5 call; 512: 130.4)
#endif
constexpr u64 DZ_SUB_BYTES = (u64)ZDZ_SUB_MIB << 20;  // input bytes per match-search sub-batch (zlib-exact coder)
constexpr u32 DZ_TAILCAP = 2048;               // symbols a segment's parse may run past its end before syncing
constexpr u32 DZ_HDRW = 96;                 // header bit-string words per block (<= 14 + 57 + 316 * 14 bits)

struct DzBlock {     // one flushed block (zz::BlockRec) + its plan
    u32 s0, s1, b0, b1;
    u32 in_win, last, type, hbits;
    u32 dbits, pad;
    u64 bitoff;      // bit offset in the chunk's deflate stream
    u32 lcode[zz::L_CODES];  // code | len << 16 (dynamic)
    u32 dcode[zz::D_CODES];
    u32 hdr[DZ_HDRW];        // the block-type bits and (dynamic) send_all_trees, LSB first
};

struct DzChunk {
    u32 nblocks, status;
    u64 bytes;       // deflate stream bytes
    u64 fsym, fpos;  // the final symbol stream and its positions (u32 offsets from the workspace base)
    u32 nsym, nloop;
};

struct DzLayout {
    u32 m, sb, nbmax;
    u64 tot, cub_bytes, outcap;
    u64 off_ka, off_kb, off_va, off_vb, off_cub, off_m2, off_sym, off_pos, off_bm, off_tail, off_ch, off_blk,
        off_out, off_crc, total;
};

DzLayout dz_layout(u64 D, u32 n) {
    DzLayout y{};
    u64 m = D ? DZ_SUB_BYTES / D : n;
    if (m < 1) m = 1;
    if (m > n) m = n;
    if (m > 65536) m = 65536;  // chunk id + 16 key bits fit 32
    y.m = (u32)m;
    y.tot = m * D;
    u64 sb = D ? DZ_SUPER_BYTES / D : n;
    sb = sb / m * m;
    if (sb < m) sb = m;
    if (sb > n) sb = n;
    y.sb = (u32)sb;
    y.nbmax = (u32)((D + zz::BLOCK_SYMS - 1) / zz::BLOCK_SYMS + 1);
    y.outcap = (D + D / 8 + 4096 + 255) & ~255ull;
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
    y.off_cub = take(y.cub_bytes);
    y.off_m2 = take(8 * (u64)y.sb * D + 4096);   // match results; then the final symbols + positions
    y.off_sym = take(4 * (u64)y.sb * D + 4096);  // per-segment symbols (pass 1)
    y.off_pos = take(4 * (u64)y.sb * D + 4096);  // their positions
    y.off_bm = take(4 * (u64)y.sb * (D / 32 + 2));
    y.off_tail = take(8ull * 64 * DZ_TAILCAP * y.sb);
    y.off_ch = take(sizeof(DzChunk) * (u64)y.sb);
    y.off_blk = take(sizeof(DzBlock) * (u64)y.sb * y.nbmax);
    y.off_out = take(y.outcap * y.sb);
    y.off_crc = take(4ull * y.sb);  // the super-batch's input CRC32s (dz_final writes the trailers)
    y.total = p;
    return y;
}

// keys: chunk id << 16 | zlib's 15-bit hash of the serialised bytes p..p+2
// (positions past D-3 are never inserted: a group of their own).  (Hash-only
// keys sort in two radix passes instead of three and a stable sort still
// leaves each (hash, chunk) chain contiguous, but the chunks' runs then
// interleave: dz_best lost locality, 24.4 vs 23.2 ms per 128 C5 chunks, more
// than the pass saved.)
__global__ void dz_keys(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, u64 tot, DType t,
                        u32* __restrict__ keys, u32* __restrict__ vals) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tot) return;
    const u32 cl = (u32)(g / D);
    const u64 p = g - (u64)cl * D;
    const zcg_chunk ch = chunks[c0 + cl];
    u32 h = 0x8000u;
    if (p + 3 <= D && ch.src_len >= D) {
        const u8* src = (const u8*)ch.src;
        h = zz::hash3(df_ser1(src, p, t), df_ser1(src, p + 1, t), df_ser1(src, p + 2, t));
    }
    keys[g] = (cl << 16) | h;
    vals[g] = (u32)g;
}

// zz::search (zcg_zlib_core.h, the host reference) for native-order bytes and
// p + 32 <= D, over the sorted run: the chain of p = entry j is entries j-1,
// j-2, ... while the key is kj.  p's first 32 bytes stay in registers; the
// candidates come 4 at a time (their keys and positions by two 16-byte loads,
// then their first 16 bytes by four loads in flight together), and are then
// compared in chain order, so a thread waits two memory latencies per four
// candidates instead of one or two per candidate.  Same candidates, order,
// ties (the first candidate reaching a longer match), NIL and window rules,
// nice cut and reduced-budget snapshot as zz::search; its scan_end test only
// skips candidates that cannot beat `best`, so leaving it out changes no result.
__device__ zz::Match2 dz_search_run(u32 p, u32 D, const zz::Config& cfg, const u8* src, const u32* __restrict__ keys,
                                    const u32* __restrict__ vals, u64 j, u32 kj, u32 cbase) {
    zz::Match2 r{0u, 0u};
    const gu8* g = (const gu8*)src;
    typedef __attribute__((address_space(1))) u32x4 gu32x4_a4 __attribute__((aligned(4)));
    auto b4 = [&](u32 i) -> u32 { return *(const df_gu32_ua*)(g + i); };
    auto pre16 = [](u32x4 A, u32x4 B) -> u32 {
        const u32 x0 = A.x ^ B.x, x1 = A.y ^ B.y, x2 = A.z ^ B.z, x3 = A.w ^ B.w;
        if (x0) return (u32)__builtin_ctz(x0) >> 3;
        if (x1) return 4 + ((u32)__builtin_ctz(x1) >> 3);
        if (x2) return 8 + ((u32)__builtin_ctz(x2) >> 3);
        if (x3) return 12 + ((u32)__builtin_ctz(x3) >> 3);
        return 16u;
    };
    const u32 look = D - p;
    const u32 mx = look < zz::MAX_MATCH ? look : zz::MAX_MATCH;  // >= 32
    const u32 nice = cfg.nice < look ? cfg.nice : look;
    const u32 lim = p > zz::MAX_DIST ? p - zz::MAX_DIST : 0u;
    const u32 nred = cfg.chain >> 2;
    const u32x4 P0 = *(const gu32x4_ua*)(g + p), P1 = *(const gu32x4_ua*)(g + p + 16);
    u32 best = 0, bstart = 0, k = 0;
    bool red_done = false;
    // entries jj-4 .. jj-1 per block (jj >= 4 here: a shorter rest reads the
    // entries before the array start from index 0 and marks them invalid)
    for (u64 jj = j; k < cfg.chain; jj -= 4) {
        const u64 b = jj >= 4 ? jj - 4 : 0;
        const u32x4 K = *(const gu32x4_a4*)(keys + b), V = *(const gu32x4_a4*)(vals + b);
        // candidate i (chain order) = entry jj-1-i = component 3-i of the block (when jj >= 4)
        u32 cc[4];
        bool ok[4];
#pragma unroll
        for (u32 i = 0; i < 4; i++) {
            const u64 e = jj - 1 - i;  // (wraps when jj <= i: invalid)
            const u32 lane4 = (u32)(e - b);
            const u32 kv = lane4 == 0 ? K.x : lane4 == 1 ? K.y : lane4 == 2 ? K.z : K.w;
            const u32 vv = lane4 == 0 ? V.x : lane4 == 1 ? V.y : lane4 == 2 ? V.z : V.w;
            ok[i] = jj > i && kv == kj;
            cc[i] = vv - cbase;
        }
        u32x4 C[4];
#pragma unroll
        for (u32 i = 0; i < 4; i++) C[i] = *(const gu32x4_ua*)(g + (ok[i] && cc[i] < p ? cc[i] : p));
        bool stop = false;
#pragma unroll
        for (u32 i = 0; i < 4; i++) {
            const u32 c = cc[i];
            if (k == 0) {
                // hash_head != NIL && strstart - hash_head <= MAX_DIST; the
                // window-relative head at the slid window's base reads as NIL
                if (!ok[i] || c == zz::slides_at(p, D) * zz::WSIZE || p - c > zz::MAX_DIST) return r;
            } else if (!ok[i] || c <= lim) {
                stop = true;
                break;
            }
            u32 len = pre16(P0, C[i]);
            if (len == 16) {
                const u32x4 C1 = *(const gu32x4_ua*)(g + c + 16);
                len += pre16(P1, C1);
                if (len == 32) {
                    while (len + 4 <= mx) {
                        const u32 x = b4(p + len) ^ b4(c + len);
                        if (x) {
                            len += (u32)__builtin_ctz(x) >> 3;
                            goto done;
                        }
                        len += 4;
                    }
                    while (len < mx && g[p + len] == g[c + len]) len++;
                }
            }
        done:
            if (len > best) {
                best = len;
                bstart = c;
                if (best >= nice) {
                    stop = true;
                    break;
                }
            }
            if (k + 1 == nred) {
                r.red = best ? (best | ((p - bstart) << 9)) : 0u;
                red_done = true;
            }
            if (++k == cfg.chain) {
                stop = true;
                break;
            }
        }
        if (stop) break;
    }
    r.full = best ? (best | ((p - bstart) << 9)) : 0u;
    if (!red_done) r.red = r.full;
    return r;
}

// zz::search at every position of the sub-batch: m2[g] = {full, red}, one
// thread per position in the ORDER OF THE SORTED KEYS.  The stable sort of
// (chunk, hash) with ascending positions lays every hash chain out
// contiguously: position vals[j]'s chain is vals[j-1], vals[j-2], ... while
// the key stays the same -- exactly zlib's prev[] walk -- so a candidate is a
// coalesced load at a known index instead of a dependent load of prev[c] at
// a random address, and neighbouring threads walk overlapping candidate
// lists (their byte loads hit the same lines).  The result is scattered back
// to m2[vals[j]].
// (An LDS-staged variant of the prev[] walk -- each workgroup's 40 KB search
// window of bytes and u16 chain links in LDS -- measured slower: 48.9 vs
// 45.2 ms per 128 C5 chunks.)
__global__ void dz_best(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, u64 tot, DType t, zz::Config cfg,
                        const u32* __restrict__ keys, const u32* __restrict__ vals, uint2* __restrict__ m2) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= tot) return;
    const u32 kj = keys[j];
    const u32 g = vals[j];
    const u32 cl = (u32)(g / D);
    const u32 p = (u32)(g - (u64)cl * D);
    zz::Match2 r{0u, 0u};
    const zcg_chunk ch = chunks[c0 + cl];
    if (ch.src_len >= D && (kj & 0x8000u) == 0) {
        const u8* src = (const u8*)ch.src;
        const u32 cbase = (u32)((u64)cl * D);
        auto b1 = [&](u32 i) -> u32 { return df_ser1(src, i, t); };
        auto b4 = [&](u32 i) -> u32 { return df_ser4(src, i, t); };
        // zz::search asks for the chain in order (the head p, then each
        // candidate once): the next entry of the sorted run, NONE past it
        u64 jj = j;
        auto pv = [&](u32) -> u32 {
            if (jj == 0 || keys[jj - 1] != kj) {
                jj = 0;
                return zz::NONE;
            }
            jj--;
            return vals[jj] - cbase;
        };
        if (!t.swap && !t.isbool && (u64)p + 32 <= D) r = dz_search_run(p, (u32)D, cfg, src, keys, vals, j, kj, cbase);
        else r = zz::search(p, (u32)D, cfg, b4, b1, pv);
    }
    m2[g] = make_uint2(r.full, r.red);
}

// The lazy parse of one chunk, SEGMENT-PARALLEL: lane k parses positions
// [k seg, (k+1) seg) from a canonical state (zz::PState: prev_len 2, not
// pending -- the state after any match), marking the positions of its
// canonical loop tops in a bitmap (pass 1).  Then each lane continues its
// parse past its segment until it reaches a canonical loop top that a later
// segment's parse also reached (pass 2): from there the two agree, so the
// true parse is lane 0's path, its tail, the next segment's path from the
// sync symbol, and so on (stitched into one stream).  A tail that does not
// sync within DZ_TAILCAP symbols sends the chunk to a serial parse.  The
// stitched stream and block records equal deflate_slow's
// (tests/hostcore/zlib_ref.cpp zz_host_deflate_seg restates this exactly).
// The match results come from dz_best (every position searched first:
// searching on demand at the loop tops the parses visit, ~40 % of the
// positions, measured 5 347 vs 217 ms per C5 call -- each lane's searches
// are a serial chain of dependent loads).
__global__ __launch_bounds__(64) void dz_parse(const zcg_chunk* __restrict__ chunks, u32 c0, u32 nc, u64 D, DType t,
                                              zz::Config cfg, u32* __restrict__ wbase, u64 off_m2, u64 off_sym,
                                              u64 off_pos, u64 off_bm, u64 off_tail, DzChunk* __restrict__ cst,
                                              DzBlock* __restrict__ blks, u32 nbmax, u32 cb) {
    const u32 cl = blockIdx.x;  // chunk of this launch (chunks[c0 + cl]; its records at cb + cl)
    if (cl >= nc) return;
    const u32 c = cb + cl;
    const u32 lane = threadIdx.x;
    const zcg_chunk ch = chunks[c0 + cl];
    DzChunk* cs = cst + c;
    if (ch.src_len < D) {
        if (lane == 0) { cs->nblocks = 0; cs->status = ZCG_ERR_INVALID_DATA; }
        return;
    }
    const u8* src = (const u8*)ch.src;
    const u32 D32 = (u32)D;
    const uint2* mc = (const uint2*)(wbase + off_m2) + (u64)c * D;  // match results (8 B / position)
    u32* fsy = wbase + off_m2 + (u64)c * 2 * D;                      // final stream (reuses them)
    u32* fps = fsy + D;
    u32* psy = wbase + off_sym + (u64)c * D;                         // pass-1 symbols / positions
    u32* pps = wbase + off_pos + (u64)c * D;
    u32* bm = wbase + off_bm + (u64)c * (D / 32 + 2);
    u32* tsy = wbase + off_tail + (u64)c * 2 * 64 * DZ_TAILCAP + (u64)lane * 2 * DZ_TAILCAP;
    u32* tps = tsy + DZ_TAILCAP;
    const u32 seg = D32 ? (((D32 + 63) / 64 + 31) & ~31u) : 32u;
    const u32 nseg = D32 ? (D32 + seg - 1) / seg : 1u;
    const bool act = lane < nseg;
    const u32 S0 = lane * seg, S1 = (lane + 1 == nseg) ? D32 : (lane + 1) * seg;
    auto b4 = [&](u32 i) -> u32 { return df_ser4(src, i, t); };
    auto byte = [&](u32 i) -> u32 { return df_ser1(src, i, t); };
    auto get = [&](u32 p) -> zz::Match2 {
        const uint2 v = mc[p];
        return zz::Match2{v.x, v.y};
    };
    // ---- pass 1 ----
    zz::PState st = zz::fresh_state(S0);
    u32 n1 = 0, fin1 = 0;
    if (act) {
        for (u32 w = S0 / 32; w < (S1 + 31) / 32; w++) bm[w] = 0;
        u32 cwi = S0 / 32, cwv = 0;
        auto em = [&](u32 sym, u32 at) {
            psy[S0 + n1] = sym;
            pps[S0 + n1] = at;
            n1++;
        };
        while (st.p < S1) {
            if (zz::canonical(st)) {
                const u32 wi = st.p >> 5;
                if (wi != cwi) {
                    if (cwv) bm[cwi] = cwv;
                    cwi = wi;
                    cwv = 0;
                }
                cwv |= 1u << (st.p & 31);
            }
            zz::step(st, D32, cfg, get, byte, em);
        }
        if (cwv) bm[cwi] = cwv;
        if (lane + 1 == nseg && st.avail) {  // Z_FINISH: the pending literal
            em(byte(st.p - 1), st.p - 1);
            st.avail = 0;
            fin1 = 1;
        }
    }
    __syncthreads();  // every segment's bitmap is in place
    // ---- pass 2 ----
    u32 nt = 0, syncq = 0xFFFFFFFFu, tfin = 0, ovf = 0;
    if (act && lane + 1 < nseg) {
        auto em = [&](u32 sym, u32 at) {
            tsy[nt] = sym;
            tps[nt] = at;
            nt++;
        };
        while (true) {
            if (st.p >= D32) {
                if (st.avail) {
                    em(byte(st.p - 1), st.p - 1);
                    tfin = 1;
                }
                break;
            }
            if (st.p >= S1 && zz::canonical(st) && ((bm[st.p >> 5] >> (st.p & 31)) & 1u)) {
                syncq = st.p;
                break;
            }
            if (nt + 1 >= DZ_TAILCAP) {
                ovf = 1;
                break;
            }
            zz::step(st, D32, cfg, get, byte, em);
        }
    }
    __syncthreads();  // tails written
    const bool any_ovf = __ballot(ovf != 0) != 0;
    u32 nsym = 0, finlit = 0;
    u64 fsel_sy = (u64)(fsy - wbase), fsel_ps = (u64)(fps - wbase);
    if (!any_ovf) {
        // ---- stitch (wave-uniform chain walk, cooperative copies) ----
        // (8 pieces per lane in flight: a copy waits one load latency per 512 symbols)
        auto copy = [&](const u32* ssy, const u32* sps, u32 n) {
            u32 i = lane;
            for (; i + 7 * 64 < n; i += 8 * 64) {
                u32 a[8], b[8];
#pragma unroll
                for (u32 k = 0; k < 8; k++) {
                    a[k] = ssy[i + 64 * k];
                    b[k] = sps[i + 64 * k];
                }
#pragma unroll
                for (u32 k = 0; k < 8; k++) {
                    fsy[nsym + i + 64 * k] = a[k];
                    fps[nsym + i + 64 * k] = b[k];
                }
            }
            for (; i < n; i += 64) {
                fsy[nsym + i] = ssy[i];
                fps[nsym + i] = sps[i];
            }
            nsym += n;
        };
        u32 cur = 0, idx = 0;
        while (true) {
            const u32 cS0 = cur * seg;
            const u32 cn1 = (u32)__builtin_amdgcn_readlane((int)n1, (int)cur);
            copy(psy + cS0 + idx, pps + cS0 + idx, cn1 - idx);
            if (cur + 1 == nseg) {
                finlit = (u32)__builtin_amdgcn_readlane((int)fin1, (int)cur);
                break;
            }
            const u32 cnt = (u32)__builtin_amdgcn_readlane((int)nt, (int)cur);
            const u32* csy = wbase + off_tail + (u64)c * 2 * 64 * DZ_TAILCAP + (u64)cur * 2 * DZ_TAILCAP;
            copy(csy, csy + DZ_TAILCAP, cnt);
            const u32 q = (u32)__builtin_amdgcn_readlane((int)syncq, (int)cur);
            if (q == 0xFFFFFFFFu) {
                finlit = (u32)__builtin_amdgcn_readlane((int)tfin, (int)cur);
                break;
            }
            const u32 nx = q / seg;
            const u32 xS0 = nx * seg;
            const u32 xn1 = (u32)__builtin_amdgcn_readlane((int)n1, (int)nx);
            // the first symbol of segment nx at or after q (there is one: q is
            // one of its canonical loop tops)
            u32 j = 0;
            for (u32 j0 = 0; j0 < xn1; j0 += 64) {
                const u32 jj = j0 + lane;
                const u64 m = __ballot(jj < xn1 && pps[xS0 + jj] >= q);
                if (m) {
                    j = j0 + (u32)__builtin_ctzll(m);
                    break;
                }
                j = xn1;
            }
            cur = nx;
            idx = j;
        }
    } else {
        // ---- a tail did not sync: the serial parse into the pass-1 arrays ----
        __syncthreads();
        fsel_sy = (u64)(psy - wbase);
        fsel_ps = (u64)(pps - wbase);
        zz::PState s2 = zz::fresh_state(0);
        u32 k = 0;
        auto em = [&](u32 sym, u32 at) {
            if (lane == 0) {
                psy[k] = sym;
                pps[k] = at;
            }
            k++;
        };
        auto gu = [&](u32 p) -> zz::Match2 {
            const zz::Match2 v = get(p);
            return zz::Match2{(u32)__builtin_amdgcn_readfirstlane(v.full), (u32)__builtin_amdgcn_readfirstlane(v.red)};
        };
        auto bu = [&](u32 i) -> u32 { return (u32)__builtin_amdgcn_readfirstlane(df_ser1(src, i, t)); };
        while (s2.p < D32) zz::step(s2, D32, cfg, gu, bu, em);
        if (s2.avail) {
            em(bu(s2.p - 1), s2.p - 1);
            finlit = 1;
        }
        nsym = k;
    }
    __syncthreads();  // the final stream is in place
    const u32* Fs = wbase + fsel_sy;
    const u32* Fp = wbase + fsel_ps;
    const u32 nloop = nsym - finlit;
    const u32 nb = zz::num_blocks(nloop);
    auto P = [&](u32 i) -> u32 { return Fp[i]; };
    auto Y = [&](u32 i) -> u32 { return Fs[i]; };
    for (u32 k = lane; k < nb && k < nbmax; k += 64) {
        const zz::BlockRec r = zz::block_rec(k, nsym, nloop, D32, P, Y);
        DzBlock* o = blks + (u64)c * nbmax + k;
        o->s0 = r.s0; o->s1 = r.s1; o->b0 = r.b0; o->b1 = r.b1; o->in_win = r.in_win; o->last = r.last;
    }
    if (lane == 0) {
        cs->fsym = fsel_sy;
        cs->fpos = fsel_ps;
        cs->nsym = nsym;
        cs->nloop = nloop;
        cs->nblocks = nb <= nbmax ? nb : 0u;
        cs->status = nb <= nbmax ? ZCG_OK : ZCG_ERR_INVALID_DATA;
    }
}

// deflate_fast (levels 1-3): zlib's greedy parse builds its hash chains as
// it goes (positions inside a match longer than max_insert_length are never
// inserted), so the parse is serial per chunk: one wave per chunk runs
// zz::parse_fast's rules with zlib's head[] / prev[] as window-relative u16
// Pos in LDS (64 KiB each, slid like slide_hash), the next 512 input bytes
// in two registers per lane, and each chain candidate's match length from
// one 4-byte compare per lane (a ballot finds the first difference).
// Symbols leave 64 at a time in the same final-stream layout as dz_parse;
// block records come from zz::block_rec(..., fast = true), so the plan /
// emit kernels are shared.  tests/hostcore/zlib_ref.cpp (zz::parse_fast on
// the CPU) and the GPU output are compared with zlib byte for byte.
constexpr u32 DZF_LDS = 2 * 32768 * 2;  // head[] + prev[], u16 each
// RING: the last 32 KiB of input (positions (p + 262 - 32768, p + 262],
// which covers every candidate within MAX_DIST and its 258 bytes) also live
// in LDS, so a chain candidate's compare is two LDS reads per side instead
// of a global-memory round trip; 160 KiB, the whole CU's LDS
constexpr u32 DZF_RING = 32768;
constexpr u32 DZF_LDS_RING = DZF_LDS + DZF_RING;
__device__ __forceinline__ u32 dzf_ld4(const u8* src, u32 x, u32 D, const DType& t) {  // bytes past D read 0
    if (x + 4 <= D) return df_ser4(src, x, t);
    u32 v = 0;
    for (u32 k = 0; k < 4; k++)
        if (x + k < D) v |= df_ser1(src, x + k, t) << (8 * k);
    return v;
}
__global__ __launch_bounds__(64) void dz_parse_fast(const zcg_chunk* __restrict__ chunks, u32 c0, u32 nc, u64 D,
                                                   DType t, zz::Config cfg, u32* __restrict__ wbase, u64 off_m2,
                                                   DzChunk* __restrict__ cst, DzBlock* __restrict__ blks, u32 nbmax) {
    extern __shared__ __attribute__((aligned(16))) u8 smem_raw[];
    u16* hd = (u16*)smem_raw;
    u16* pv = hd + 32768;
    u8* ring = smem_raw + DZF_LDS;  // byte q at ring[q & (DZF_RING - 1)]
    const u32 c = blockIdx.x;
    if (c >= nc) return;
    const u32 lane = threadIdx.x;
    const zcg_chunk ch = chunks[c0 + c];
    DzChunk* cs = cst + c;
    if (ch.src_len < D) {
        if (lane == 0) { cs->nblocks = 0; cs->status = ZCG_ERR_INVALID_DATA; }
        return;
    }
    const u8* src = (const u8*)ch.src;
    const u32 D32 = (u32)D;
    u32* fsy = wbase + off_m2 + (u64)c * 2 * D;  // final stream: symbols, then positions
    u32* fps = fsy + D;
    for (u32 i = lane; i < 32768; i += 64) ((u32*)smem_raw)[i] = 0u;  // both tables NIL
    __syncthreads();
    auto rd = [&](const u16* a, u32 i) -> u32 { return (u32)__builtin_amdgcn_readfirstlane((u32)a[i]); };
    // input window: lane l holds bytes [wb + 4 l, +4) (w0) and [wb + 256 + 4 l, +4) (w1)
    u32 wb = 0;
    u32 w0 = dzf_ld4(src, 4 * lane, D32, t), w1 = dzf_ld4(src, 256 + 4 * lane, D32, t);
    auto wbyte = [&](u32 q) -> u32 {  // q in [wb, wb + 512)
        const u32 o = q - wb, wi = o >> 2;
        const u32 v = (u32)__builtin_amdgcn_readlane((int)(wi < 64 ? w0 : w1), (int)(wi & 63));
        return (v >> (8 * (o & 3))) & 0xFFu;
    };
    u32 base = 0, nsym = 0, rs = 0, rp = 0;
    auto emit = [&](u32 sym, u32 at) {
        const u32 k = nsym & 63;
        if (lane == k) { rs = sym; rp = at; }
        nsym++;
        if (k == 63) {
            fsy[nsym - 64 + lane] = rs;
            fps[nsym - 64 + lane] = rp;
        }
    };
    auto insert = [&](u32 q) -> u32 {  // INSERT_STRING: the previous head (relative, 0 = NIL)
        const u32 h = zz::hash3(wbyte(q), wbyte(q + 1), wbyte(q + 2));
        const u32 hh = rd(hd, h);
        if (lane == 0) {
            pv[(q - base) & zz::WMASK] = (u16)hh;
            hd[h] = (u16)(q - base);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        return hh;
    };
    // bytes [rf, F) into the ring from the register window, 64 per round
    u32 rf = 0;
    auto ring_fill = [&](u32 F) {
        for (u32 q0 = rf; q0 < F; q0 += 64) {
            const u32 q = q0 + lane;
            const u32 o = q - wb, wi = o >> 2;
            const u32 a0 = __shfl(w0, (int)(wi & 63)), a1 = __shfl(w1, (int)(wi & 63));
            const u32 v = ((wi < 64 ? a0 : a1) >> (8 * (o & 3))) & 0xFFu;
            if (q < F) ring[q & (DZF_RING - 1)] = (u8)v;
        }
        rf = F;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto ring4 = [&](u32 x) -> u32 {  // ring bytes x..x+3 (LE)
        const u32 a = x & ~3u, sh = 8 * (x & 3);
        const u32 lo = *(const u32*)(ring + (a & (DZF_RING - 1)));
        const u32 hi = *(const u32*)(ring + ((a + 4) & (DZF_RING - 1)));
        return sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
    };
    u32 p = 0;
    while (p < D32) {
        if (p - wb >= 250) {  // keep [p, p + 262) in the window (wb <= p always)
            wb = p & ~3u;
            w0 = dzf_ld4(src, wb + 4 * lane, D32, t);
            w1 = dzf_ld4(src, wb + 256 + 4 * lane, D32, t);
        }
        {
            const u32 F = p + 262 < D32 ? p + 262 : D32;
            if (F > rf) ring_fill(F);
        }
        {  // fill_window at the loop top: one slide when due
            const u32 wend = (D32 - base) > 2 * zz::WSIZE ? base + 2 * zz::WSIZE : D32;
            if (wend - p < zz::MIN_LOOKAHEAD && p - base >= zz::WSIZE + zz::MAX_DIST) {
                for (u32 i = lane; i < 32768; i += 64) {
                    const u32 x = ((u32*)smem_raw)[i];
                    const u32 lo = x & 0xFFFFu, hi = x >> 16;
                    ((u32*)smem_raw)[i] = (lo >= zz::WSIZE ? lo - zz::WSIZE : 0u) |
                                          ((hi >= zz::WSIZE ? hi - zz::WSIZE : 0u) << 16);
                }
                __syncthreads();
                base += zz::WSIZE;
            }
        }
        u32 ml = 0, md = 0;
        if (D32 - p >= zz::MIN_MATCH) {
            const u32 hh = insert(p);
            if (hh != 0 && (p - base) - hh <= zz::MAX_DIST) {
                // longest_match (zz::search's rules) over the chain from hh
                const u32 look = D32 - p;
                const u32 mx = look < zz::MAX_MATCH ? look : zz::MAX_MATCH;
                const u32 nice = cfg.nice < look ? cfg.nice : look;
                const u32 lim = p > zz::MAX_DIST ? p - zz::MAX_DIST : 0u;
                // my 4 bytes of p.. (lane l: p + 4 l ..) from the window
                const u32 pw = ring4(p + 4 * lane);
                u32 best = 0, bstart = 0, cand = hh + base;
                for (u32 k = 0; k < cfg.chain; k++) {
                    if (k > 0) {
                        const u32 r = rd(pv, (cand - base) & zz::WMASK);
                        if (r == 0) break;
                        cand = r + base;
                        if (cand <= lim) break;
                    }
                    const u32 cw = 4 * lane < mx ? ring4(cand + 4 * lane) : pw;
                    const u64 m = __ballot(pw != cw);
                    u32 len;
                    if (m) {
                        const u32 j = (u32)__builtin_ctzll(m);
                        const u32 x = (u32)__builtin_amdgcn_readlane((int)(pw ^ cw), (int)j);
                        len = 4 * j + ((u32)__builtin_ctz(x) >> 3);
                    } else {
                        len = 256;
                        while (len < mx && wbyte(p + len) == (u32)__builtin_amdgcn_readfirstlane((u32)ring[(cand + len) & (DZF_RING - 1)]))
                            len++;
                    }
                    if (len > mx) len = mx;
                    if (len > best) {
                        best = len;
                        bstart = cand;
                        if (best >= nice) break;
                    }
                }
                if (best >= zz::MIN_MATCH) {
                    ml = best;
                    md = p - bstart;
                }
            }
        }
        if (ml) {
            emit(0x80000000u | ((ml - zz::MIN_MATCH) << 16) | (md - 1), p);
            if (ml <= cfg.lazy && D32 - (p + ml) >= zz::MIN_MATCH)
                for (u32 q = p + 1; q < p + ml; q++) insert(q);
            p += ml;
        } else {
            emit(wbyte(p), p);
            p++;
        }
    }
    if (nsym & 63) {
        const u32 b0 = nsym & ~63u;
        if (lane < (nsym & 63)) {
            fsy[b0 + lane] = rs;
            fps[b0 + lane] = rp;
        }
    }
    __syncthreads();  // the final stream is in place
    const u32 nb = zz::num_blocks(nsym);
    auto P = [&](u32 i) -> u32 { return fps[i]; };
    auto Y = [&](u32 i) -> u32 { return fsy[i]; };
    for (u32 k = lane; k < nb && k < nbmax; k += 64) {
        const zz::BlockRec r = zz::block_rec(k, nsym, nsym, D32, P, Y, true);
        DzBlock* o = blks + (u64)c * nbmax + k;
        o->s0 = r.s0; o->s1 = r.s1; o->b0 = r.b0; o->b1 = r.b1; o->in_win = r.in_win; o->last = r.last;
    }
    if (lane == 0) {
        cs->fsym = (u64)(fsy - wbase);
        cs->fpos = (u64)(fps - wbase);
        cs->nsym = nsym;
        cs->nloop = nsym;
        cs->nblocks = nb <= nbmax ? nb : 0u;
        cs->status = nb <= nbmax ? ZCG_OK : ZCG_ERR_INVALID_DATA;
    }
}

struct DzPlanLds {
    zz::BlockWork bw;
    u32 lf[zz::L_CODES], df[zz::D_CODES];
    u32 hbits;
};

// One wave per block: histogram, zlib's trees and block-type decision, the
// header bit-string and the block's exact bit count.
__global__ __launch_bounds__(64) void dz_plan(u32 nc, DzChunk* __restrict__ cst, DzBlock* __restrict__ blks,
                                             u32 nbmax, const u32* __restrict__ wbase, u64 D) {
    __shared__ DzPlanLds L;
    const u32 c = blockIdx.x / nbmax, k = blockIdx.x % nbmax;
    if (c >= nc) return;
    const DzChunk cs = cst[c];
    if (cs.status != ZCG_OK || k >= cs.nblocks) return;
    DzBlock* B = blks + (u64)c * nbmax + k;
    const u32* sy = wbase + cs.fsym;
    const u32 lane = threadIdx.x;
    const u32 s0 = B->s0, s1 = B->s1;
    for (u32 i = lane; i < (u32)zz::L_CODES; i += 64) L.lf[i] = 0;
    if (lane < (u32)zz::D_CODES) L.df[lane] = 0;
    __syncthreads();
    for (u32 i = s0 + lane; i < s1; i += 64) {
        const u32 s = sy[i];
        if (!(s & 0x80000000u)) {
            atomicAdd(&L.lf[s & 0xFF], 1u);
        } else {
            atomicAdd(&L.lf[zz::len_code(((s >> 16) & 0xFF) + 3) + zz::LITERALS + 1], 1u);
            atomicAdd(&L.df[zz::dist_code((s & 0xFFFF) + 1)], 1u);
        }
    }
    __syncthreads();
    if (lane == 0) L.lf[zz::END_BLOCK] = 1;
    __syncthreads();
    for (u32 i = lane; i < (u32)zz::HEAP_SIZE; i += 64) L.bw.lt.freq[i] = i < (u32)zz::L_CODES ? L.lf[i] : 0u;
    for (u32 i = lane; i < (u32)(2 * zz::D_CODES + 1); i += 64) L.bw.dt.freq[i] = i < (u32)zz::D_CODES ? L.df[i] : 0u;
    for (u32 i = lane; i < DZ_HDRW; i += 64) B->hdr[i] = 0;
    __syncthreads();
    if (lane == 0) {
        const zz::BlockPlan pl = zz::plan_block(L.bw, B->b1 - B->b0, B->in_win != 0);
        u32 hb = 0;
        u32 acc = 0;  // header bit-string, LSB first, flushed word by word
        auto put = [&](u32 v, u32 n) {
            if (!n) return;
            v &= n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1);
            const u32 sh = hb & 31;
            acc |= v << sh;
            if (sh + n >= 32) {
                B->hdr[hb >> 5] = acc;
                acc = sh ? (v >> (32 - sh)) : 0u;
            }
            hb += n;
        };
        zz::send_header(L.bw, pl, B->last != 0, put);
        if (hb & 31) B->hdr[hb >> 5] = acc;
        B->type = pl.type;
        B->hbits = hb;
        L.hbits = hb;
        u64 db = 0;
        if (pl.type == zz::BT_DYN) {
            for (int i = 0; i < zz::L_CODES; i++) {
                const u32 x = i > zz::END_BLOCK ? zz::extra_lbits(i - 257) : 0u;
                db += (u64)L.lf[i] * (L.bw.lt.len[i] + x);
            }
            for (int i = 0; i < zz::D_CODES; i++) db += (u64)L.df[i] * (L.bw.dt.len[i] + zz::extra_dbits(i));
        } else if (pl.type == zz::BT_STATIC) {
            for (int i = 0; i < zz::L_CODES; i++) {
                const u32 x = i > zz::END_BLOCK ? zz::extra_lbits(i - 257) : 0u;
                db += (u64)L.lf[i] * (zz::static_llen(i) + x);
            }
            for (int i = 0; i < zz::D_CODES; i++) db += (u64)L.df[i] * (5 + zz::extra_dbits(i));
        }
        B->dbits = (u32)db;
    }
    __syncthreads();
    for (u32 i = lane; i < (u32)zz::L_CODES; i += 64) B->lcode[i] = L.bw.lt.code[i] | ((u32)L.bw.lt.len[i] << 16);
    if (lane < (u32)zz::D_CODES) B->dcode[lane] = L.bw.dt.code[lane] | ((u32)L.bw.dt.len[lane] << 16);
}

// Per chunk: block bit offsets (a stored block pads to a byte after its 3
// header bits), the stream length, and the boundary words cleared (blocks
// OR their first and last words in; every other word has one writer).
__global__ void dz_offsets(u32 nc, DzChunk* __restrict__ cst, DzBlock* __restrict__ blks, u32 nbmax, u8* out,
                           u64 outcap) {
    const u32 c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc) return;
    DzChunk* cs = cst + c;
    if (cs->status != ZCG_OK) return;
    u32* ow = (u32*)(out + (u64)c * outcap);
    u64 acc = 0;
    for (u32 k = 0; k < cs->nblocks; k++) {
        DzBlock* B = blks + (u64)c * nbmax + k;
        B->bitoff = acc;
        ow[acc >> 5] = 0;
        if (B->type == zz::BT_STORED) {
            acc += 3;
            acc = (acc + 7) & ~7ull;
            acc += 32 + 8ull * (B->b1 - B->b0);
        } else {
            acc += (u64)B->hbits + B->dbits;
        }
        if (acc) ow[(acc - 1) >> 5] = 0;
    }
    ow[acc >> 5] = 0;
    cs->bytes = (acc + 7) >> 3;
    if (cs->bytes + 64 > outcap) cs->status = ZCG_ERR_OUTPUT_TOO_SMALL;
}

// One wave per block: its bits at its offset.  Symbols 64 at a time: each
// lane its symbol's bit count, a wave scan places them, and the bits are
// OR-ed into an LDS ring of words flushed in order (the block's first and
// last words with global atomics, the rest with plain stores).
struct DzEmitLds {
    u32 lc[zz::L_CODES], dc[zz::D_CODES];
    u32 ring[1024];
};

__global__ __launch_bounds__(64) void dz_emit(const zcg_chunk* __restrict__ chunks, u32 c0, u32 nc, u64 D, DType t,
                                             const DzChunk* __restrict__ cst, const DzBlock* __restrict__ blks,
                                             u32 nbmax, const u32* __restrict__ wbase, u8* out, u64 outcap) {
    __shared__ DzEmitLds L;
    const u32 c = blockIdx.x / nbmax, k = blockIdx.x % nbmax;
    if (c >= nc) return;
    const DzChunk cs = cst[c];
    if (cs.status != ZCG_OK || k >= cs.nblocks) return;
    const DzBlock* B = blks + (u64)c * nbmax + k;
    const u32 lane = threadIdx.x;
    const u32* sy = wbase + cs.fsym;
    u32* ow = (u32*)(out + (u64)c * outcap);
    const u64 b0 = B->bitoff;
    const u32 type = B->type;
    const bool stat = type == zz::BT_STATIC;
    for (u32 i = lane; i < (u32)zz::L_CODES; i += 64) L.lc[i] = B->lcode[i];
    if (lane < (u32)zz::D_CODES) L.dc[lane] = B->dcode[lane];
    for (u32 i = lane; i < 1024; i += 64) L.ring[i] = 0;
    __syncthreads();
    // bit position relative to the aligned word holding bit b0
    const u64 w0 = b0 >> 5;
    u32 pos = (u32)(b0 & 31);  // next bit, relative to 32 * w0
    u32 fw = 0;                // ring words flushed (relative to w0)
    u64 bend = 0;              // the block's end bit, relative to 32 * w0
    {
        u64 len = (u64)B->hbits + B->dbits;
        if (type == zz::BT_STORED) len = 0;  // (computed below)
        bend = pos + len;
    }
    auto put_lane = [&](u32 at, u32 v, u32 n) {  // at: relative bit; n <= 32
        if (!n) return;
        v &= n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1);
        const u32 w = at >> 5, sh = at & 31;
        atomicOr(&L.ring[w & 1023], v << sh);
        if (sh + n > 32) atomicOr(&L.ring[(w + 1) & 1023], v >> (32 - sh));
    };
    auto flush_to = [&](u32 upto, bool fin) {  // words [fw, upto) are complete (fin: and the partial last one)
        __syncthreads();
        const u32 lastw = fin ? (u32)((bend + 31) >> 5) : upto;
        for (u32 w = fw + lane; w < lastw; w += 64) {
            const u32 v = L.ring[w & 1023];
            const bool edge = (w == 0) || (fin && w == lastw - 1);
            if (edge) atomicOr(&ow[w0 + w], v);
            else ow[w0 + w] = v;
            L.ring[w & 1023] = 0;
        }
        fw = lastw;
        __syncthreads();
    };
    // header bit-string
    {
        const u32 hb = B->hbits;
        for (u32 i = lane; i < (hb + 31) / 32; i += 64) {
            const u32 n = (i + 1) * 32 <= hb ? 32u : hb - i * 32;
            put_lane(pos + i * 32, B->hdr[i], n);
        }
        pos += hb;
    }
    if (type == zz::BT_STORED) {
        pos = (pos + 7) & ~7u;
        const u32 len = B->b1 - B->b0;
        if (lane == 0) {
            put_lane(pos, len & 0xFFFF, 16);
            put_lane(pos + 16, ~len & 0xFFFF, 16);
        }
        pos += 32;
        bend = pos + 8ull * len;
        const u8* src = (const u8*)chunks[c0 + c].src;
        for (u32 i0 = 0; i0 < len; i0 += 256) {
            __syncthreads();
            for (u32 i = i0 + lane; i < i0 + 256 && i < len; i += 64)
                put_lane(pos + 8 * i, df_ser1(src, (u64)B->b0 + i, t), 8);
            flush_to((pos + 8 * (i0 + 256 < len ? i0 + 256 : len)) >> 5, false);
        }
        flush_to(0, true);
        return;
    }
    const u32 s0 = B->s0, s1 = B->s1;
    for (u32 i0 = s0; i0 < s1; i0 += 64) {
        const u32 i = i0 + lane;
        zz::SymBits sb{{0, 0, 0, 0}, {0, 0, 0, 0}};
        if (i < s1) {
            const u32 s = sy[i];
            if (stat) {
                sb = zz::sym_bits(s, true, nullptr, nullptr, nullptr, nullptr);
            } else if (!(s & 0x80000000u)) {
                const u32 e = L.lc[s & 0xFF];
                sb.v[0] = e & 0xFFFF;
                sb.n[0] = e >> 16;
            } else {
                const u32 lc = (s >> 16) & 0xFF, dist = (s & 0xFFFF) + 1;
                const int code = (int)zz::len_code(lc + 3);
                const u32 e = L.lc[code + zz::LITERALS + 1];
                sb.v[0] = e & 0xFFFF;
                sb.n[0] = e >> 16;
                sb.n[1] = zz::extra_lbits(code);
                sb.v[1] = lc - zz::base_length(code);
                const int dcd = (int)zz::dist_code(dist);
                const u32 f = L.dc[dcd];
                sb.v[2] = f & 0xFFFF;
                sb.n[2] = f >> 16;
                sb.n[3] = zz::extra_dbits(dcd);
                sb.v[3] = (dist - 1) - zz::base_dist(dcd);
            }
        }
        const u32 nbits = sb.n[0] + sb.n[1] + sb.n[2] + sb.n[3];
        u32 x = nbits;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u32 y = __shfl_up(x, d, 64);
            if ((int)lane >= d) x += y;
        }
        u32 at = pos + x - nbits;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            // a part is <= 15 bits, so two parts always fit one 32-bit put
            put_lane(at, sb.v[j], sb.n[j]);
            at += sb.n[j];
        }
        pos += __shfl(x, 63, 64);
        if (((pos >> 5) - fw) >= 512) flush_to(pos >> 5, false);
    }
    if (lane == 0) {
        const u32 e = stat ? (zz::static_lcode(zz::END_BLOCK) | (7u << 16)) : L.lc[zz::END_BLOCK];
        put_lane(pos, e & 0xFFFF, e >> 16);
    }
    flush_to(0, true);
}

// Per chunk: gzip header, the stream, CRC32/ISIZE (the CRC from gzip_crc32 crc_out mode, run before).
__global__ __launch_bounds__(256) void dz_final(const zcg_chunk* __restrict__ chunks, u32 c0, u32 nc, u64 D,
                                               u64 bound, u32 xfl, const DzChunk* __restrict__ cst, const u8* out,
                                               u64 outcap, u64* __restrict__ out_len, i32* __restrict__ status,
                                               const u32* __restrict__ crc) {
    const u32 c = blockIdx.x, tid = threadIdx.x;
    if (c >= nc) return;
    const zcg_chunk ch = chunks[c0 + c];
    const DzChunk cs = cst[c];
    if (ch.src_len < D) { if (tid == 0) { status[c0 + c] = ZCG_ERR_INVALID_DATA; out_len[c0 + c] = 0; } return; }
    if (cs.status != ZCG_OK) { if (tid == 0) { status[c0 + c] = (i32)cs.status; out_len[c0 + c] = 0; } return; }
    if (ch.dst_cap < bound || ch.dst_cap < DF_HDR + cs.bytes + 8) {
        if (tid == 0) { status[c0 + c] = ZCG_ERR_OUTPUT_TOO_SMALL; out_len[c0 + c] = 0; }
        return;
    }
    u8* dst = (u8*)ch.dst;
    const u8* o = out + (u64)c * outcap;
    if (tid == 0) {
        const u8 h[10] = {0x1F, 0x8B, 8, 0, 0, 0, 0, 0, (u8)xfl, 255};
        for (u32 i = 0; i < 10; i++) dst[i] = h[i];
    }
    const u64 n = cs.bytes;
    for (u64 i = (u64)tid * 16; i < n; i += 256 * 16) {
        if (i + 16 <= n) st16(dst + DF_HDR + i, *(const u32x4*)(o + i));
        else for (u64 j = i; j < n; j++) dst[DF_HDR + j] = o[j];
    }
    if (tid == 0) {
        const u32 r = crc[c], isz = (u32)D;
        u8* tr = dst + DF_HDR + n;
        const u8 t8[8] = {(u8)r, (u8)(r >> 8), (u8)(r >> 16), (u8)(r >> 24),
                          (u8)isz, (u8)(isz >> 8), (u8)(isz >> 16), (u8)(isz >> 24)};
        for (u32 i = 0; i < 8; i++) tr[i] = t8[i];
        out_len[c0 + c] = DF_HDR + n + 8;
        status[c0 + c] = ZCG_OK;
    }
}

}  // namespace

uint64_t deflate_exact_ws_bytes(const zcg_array* a, uint32_t n) {
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    if (n == 0 || D >= (1ull << 31)) return 0;  // (chunks of >= 2 GiB: per-chunk UNSUPPORTED)
    return dz_layout(D, n).total;
}

static hipError_t launch_deflate_exact(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n, u32 level,
                                       uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                                       hipStream_t s, hipStream_t side, hipEvent_t fork, hipEvent_t join) {
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const u32 xfl = level >= 9 ? 2u : (level <= 1 ? 4u : 0u);
    const u64 bound = zcg_encode_bound(&a->compression, D);
    if (D >= (1ull << 31)) {  // u32 positions: every chunk UNSUPPORTED, the launch itself succeeds
        if (hipError_t e = hipMemsetD32Async((hipDeviceptr_t)d_status, ZCG_ERR_UNSUPPORTED, n, s); e != hipSuccess)
            return e;
        return hipMemsetAsync(d_out_len, 0, sizeof(uint64_t) * (size_t)n, s);
    }
    const DzLayout y = dz_layout(D, n);
    if (ws_bytes < y.total || y.tot >= (1ull << 31)) return hipErrorInvalidValue;
    const zz::Config cfg = zz::level_config((int)level);
    u8* w = (u8*)ws;
    uint2* m2 = (uint2*)(w + y.off_m2);
    DzChunk* cst = (DzChunk*)(w + y.off_ch);
    DzBlock* blks = (DzBlock*)(w + y.off_blk);
    u8* out = w + y.off_out;
    const bool fast = level <= 3;
    // deflate_fast takes the whole CU's 160 KiB of LDS (head/prev + the input ring)
    if (fast) {
        if (hipError_t e = lds_attr_once((const void*)dz_parse_fast, (int)DZF_LDS_RING); e != hipSuccess) return e;
    }
    const bool two = side && fork && join && !fast;  // the parse of each sub-batch on the side stream
    const u64 Lsl = D / 64;
    CrcShift op;
    crc_shift_op(Lsl, op.m);
    u32* crcb = (u32*)(w + y.off_crc);
    // blocks (trees, header bits), their bit offsets, the bits, the container
    // with its CRC32 trailer: for the chunks [s0 + cb, s0 + cb + cnt) of the
    // super-batch at s0
    auto tail = [&](u32 s0, u32 cb, u32 cnt, hipStream_t ts) -> hipError_t {
        const u64 nbk = (u64)cnt * y.nbmax;
        DzChunk* cs = cst + cb;
        DzBlock* bk = blks + (u64)cb * y.nbmax;
        u8* ot = out + (u64)cb * y.outcap;
        hipLaunchKernelGGL(dz_plan, dim3((u32)nbk), dim3(64), 0, ts, cnt, cs, bk, y.nbmax, (const u32*)w, D);
        hipLaunchKernelGGL(dz_offsets, dim3((cnt + 63) / 64), dim3(64), 0, ts, cnt, cs, bk, y.nbmax, ot, y.outcap);
        hipLaunchKernelGGL(dz_emit, dim3((u32)nbk), dim3(64), 0, ts, d_chunks, s0 + cb, cnt, D, t, (const DzChunk*)cs,
                           (const DzBlock*)bk, y.nbmax, (const u32*)w, ot, y.outcap);
        hipLaunchKernelGGL(dz_final, dim3(cnt), dim3(256), 0, ts, d_chunks, s0 + cb, cnt, D, bound, xfl,
                           (const DzChunk*)cs, (const u8*)ot, y.outcap, (u64*)d_out_len, (i32*)d_status,
                           (const u32*)crcb + cb);
        return hipGetLastError();
    };
    for (u32 s0 = 0; s0 < n; s0 += y.sb) {
        const u32 scnt = (n - s0) < y.sb ? (n - s0) : y.sb;
        // a parse that does not run leaves every chunk failed, so the kernels
        // after it never read an unset record
        if (hipError_t e = hipMemsetAsync(cst, 0xFF, sizeof(DzChunk) * (size_t)scnt, s); e != hipSuccess) return e;
        // the inputs' CRC32s: on the side stream (idle until the first parse)
        // beside the first match search, else in line.  (Sorting sub-batch
        // i + 1 on the side stream beside match search i measured slower,
        // 133.7 vs 126.0 ms per C5 call: the search takes the CUs, the sort
        // beside it ran 20 instead of 3 ms and held back the parses.)
        {
            hipStream_t cs = s;
            if (two && D > 0) {
                if (hipError_t e = hipEventRecord(fork, s); e != hipSuccess) return e;
                if (hipError_t e = hipStreamWaitEvent(side, fork, 0); e != hipSuccess) return e;
                cs = side;
            }
            hipLaunchKernelGGL(gzip_crc32, dim3(scnt), dim3(64), 0, cs, d_chunks + s0, scnt, D, Lsl, op,
                               (const u64*)nullptr, (const i32*)nullptr, t, crcb);
            if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        }
        for (u32 c0 = s0; c0 < s0 + scnt && D > 0 && !fast; c0 += y.m) {
            const u32 cnt = (s0 + scnt - c0) < y.m ? (s0 + scnt - c0) : y.m;
            const u64 tot = (u64)cnt * D;
            u32 *ka = (u32*)(w + y.off_ka), *kb = (u32*)(w + y.off_kb);
            u32 *va = (u32*)(w + y.off_va), *vb = (u32*)(w + y.off_vb);
            const u32 G = (u32)((tot + 255) / 256);
            u32 cbits = 0;
            while ((1u << cbits) < cnt) cbits++;
            hipLaunchKernelGGL(dz_keys, dim3(G), dim3(256), 0, s, d_chunks, c0, D, tot, t, ka, va);
            hipcub::DoubleBuffer<u32> dk(ka, kb), dv(va, vb);
            size_t cb = y.cub_bytes;
            hipError_t e = hipcub::DeviceRadixSort::SortPairs(w + y.off_cub, cb, dk, dv, (int)tot, 0,
                                                              (int)(16 + cbits), s);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(dz_best, dim3(G), dim3(256), 0, s, d_chunks, c0, D, tot, t, cfg,
                               (const u32*)dk.Current(), (const u32*)dv.Current(), m2 + (u64)(c0 - s0) * D);
            // the sub-batch's lazy parse (one wave per chunk: a few waves per
            // CU) runs beside the next sub-batch's sort and match search
            hipStream_t ps = s;
            if (two) {
                if ((e = hipEventRecord(fork, s)) != hipSuccess) return e;
                if ((e = hipStreamWaitEvent(side, fork, 0)) != hipSuccess) return e;
                ps = side;
            }
            hipLaunchKernelGGL(dz_parse, dim3(cnt), dim3(64), 0, ps, d_chunks, c0, cnt, D, t, cfg, (u32*)w,
                               y.off_m2 / 4, y.off_sym / 4, y.off_pos / 4, y.off_bm / 4, y.off_tail / 4, cst, blks,
                               y.nbmax, c0 - s0);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            // and the rest of the sub-batch's encode right behind it
            if (two && (e = tail(s0, c0 - s0, cnt, side)) != hipSuccess) return e;
        }
        if (two) {
            if (hipError_t e = hipEventRecord(join, side); e != hipSuccess) return e;
            if (hipError_t e = hipStreamWaitEvent(s, join, 0); e != hipSuccess) return e;
        }
        if (fast) {
            hipLaunchKernelGGL(dz_parse_fast, dim3(scnt), dim3(64), DZF_LDS_RING, s, d_chunks, s0, scnt, D, t, cfg,
                               (u32*)w, y.off_m2 / 4, cst, blks, y.nbmax);
            if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        }
        if (!fast && D == 0) {  // (empty chunks: the parse writes their empty streams)
            hipLaunchKernelGGL(dz_parse, dim3(scnt), dim3(64), 0, s, d_chunks, s0, scnt, D, t, cfg, (u32*)w,
                               y.off_m2 / 4, y.off_sym / 4, y.off_pos / 4, y.off_bm / 4, y.off_tail / 4, cst, blks,
                               y.nbmax, 0u);
            if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        }
        if (!two || D == 0) {
            if (hipError_t e = tail(s0, 0, scnt, s); e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

// levels 1-9 reproduce zlib's bytes (1-3 deflate_fast, 4-9 deflate_slow);
// level 0 (stored) and ZCG_FLAG_GZIP_SEGMENTED take the segmented coder
static bool deflate_exact_level(const zcg_array* a) {
    const int level = zcg_effective_gzip_level(a->compression.gzip_level);
    return level >= 1 && (a->compression.flags & ZCG_FLAG_GZIP_SEGMENTED) == 0;
}

uint64_t deflate_ws_bytes(const zcg_array* a, uint32_t n) {
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    if (n == 0) return 0;
    if (deflate_exact_level(a)) return deflate_exact_ws_bytes(a, n);
    return df_layout(D, n).total;
}

#ifndef ZCG_DF_CHAIN6
#define ZCG_DF_CHAIN6 32
#endif
const char* cfg_deflate() { return "deflate:CHAIN6=" ZCG_STR(ZCG_DF_CHAIN6) ",SUB=" ZCG_STR(ZDZ_SUB_MIB); }

hipError_t launch_deflate(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                          uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                          hipStream_t s, hipStream_t side, hipEvent_t fork, hipEvent_t join) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const u32 level = (u32)zcg_effective_gzip_level(a->compression.gzip_level);
    if (deflate_exact_level(a))
        return launch_deflate_exact(a, d_chunks, n, level, d_out_len, d_status, ws, ws_bytes, s, side, fork, join);
    const u32 xfl = level >= 9 ? 2u : (level <= 1 ? 4u : 0u);
    const u32 nseg = (u32)((D + DF_SEG - 1) / DF_SEG);
    const u64 bound = zcg_encode_bound(&a->compression, D);
    const DfLayout y = df_layout(D, n);
    if (nseg && (ws_bytes < y.total || y.tot >= (1ull << 31))) return hipErrorInvalidValue;
    // zlib's configuration_table: max_chain (capped for the GPU) and nice_length
    static const u32 chain[10] = {0, 4, 8, 32, 16, 32, ZCG_DF_CHAIN6, 64, 64, 64};
    static const u32 nice[10] = {0, 8, 16, 32, 16, 32, 128, 128, 258, 258};
    u8* w = (u8*)ws;
    if (nseg) {
        if (hipError_t e = lds_attr_once((const void*)deflate_segment, (int)sizeof(DefLds)); e != hipSuccess)
            return e;
        for (u32 s0 = 0; s0 < n; s0 += y.sm) {
            const u32 scnt = (n - s0) < y.sm ? (n - s0) : y.sm;
            if (level > 0) {
                for (u32 c0 = s0; c0 < s0 + scnt; c0 += y.m) {
                    const u32 cnt = (s0 + scnt - c0) < y.m ? (s0 + scnt - c0) : y.m;
                    const u64 tot = (u64)cnt * D;
                    u32 *ka = (u32*)(w + y.off_ka), *kb = (u32*)(w + y.off_kb);
                    u32 *va = (u32*)(w + y.off_va), *vb = (u32*)(w + y.off_vb);
                    const u32 G = (u32)((tot + 255) / 256);
                    u32 cbits = 0;
                    while ((1u << cbits) < cnt) cbits++;
                    hipLaunchKernelGGL(df_keys, dim3(G), dim3(256), 0, s, d_chunks, c0, D, tot, t, ka, va);
                    hipcub::DoubleBuffer<u32> dk(ka, kb), dv(va, vb);
                    size_t cb = y.cub_bytes;
                    hipError_t e = hipcub::DeviceRadixSort::SortPairs(w + y.off_cub, cb, dk, dv, (int)tot, 0,
                                                                      (int)(24 + cbits), s);
                    if (e != hipSuccess) return e;
                    hipLaunchKernelGGL(df_chain, dim3(G), dim3(256), 0, s, tot, dk.Current(), dv.Current(),
                                       (u32*)(w + y.off_prev));
                    hipLaunchKernelGGL(df_best, dim3(G), dim3(256), 0, s, d_chunks, c0, D, tot, t, chain[level],
                                       nice[level], (const u32*)(w + y.off_prev),
                                       (u32*)(w + y.off_match) + (u64)(c0 - s0) * D);
                }
            }
            const u64 nb = (u64)scnt * nseg;
            if (nb > 0x7FFFFFFFull) return hipErrorInvalidValue;
            hipLaunchKernelGGL(deflate_segment, dim3((u32)nb), dim3(64), sizeof(DefLds), s, d_chunks, s0, scnt, D,
                               nseg, bound, t, level, (const u32*)(w + y.off_match));
        }
    }
    hipLaunchKernelGGL(deflate_finalize, dim3(n), dim3(256), 0, s, d_chunks, n, D, nseg, bound, xfl,
                       (u64*)d_out_len, d_status);
    const u64 Lsl = D / 64;
    CrcShift op;
    crc_shift_op(Lsl, op.m);
    hipLaunchKernelGGL(gzip_crc32, dim3(n), dim3(64), 0, s, d_chunks, n, D, Lsl, op,
                       (const u64*)d_out_len, (const i32*)d_status, t, (u32*)nullptr);
    return hipGetLastError();
}

}  // namespace zcg
