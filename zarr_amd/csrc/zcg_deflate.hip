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
//   1. deflate_segment: one wave per 16 KiB input segment.  The segment and
//      the 32 KiB before it (deflate's window) are staged in LDS with the
//      dtype transform applied (write_data's byte order, chunk.rs:118-140).
//      The history is pre-inserted in a 4096-entry hash table; 64 lanes look
//      up 64 consecutive positions, the first verified candidate is the next
//      match (one-step lazy evaluation at level >= 4; positions inside matches
//      are inserted at level >= 4).  Pass A runs the parse for symbol
//      frequencies; the wave builds length-limited Huffman codes (zlib's
//      bl_count overflow rule) and picks stored/fixed/dynamic; pass B re-runs
//      the same deterministic parse and emits the bits through an LDS ring
//      (wave prefix sums place 64 literal codes at once).  A non-final
//      segment ends with an empty stored block so it is byte aligned.
//      Segment k is written at its upper-bound slot of dst.
//   2. deflate_finalize: per chunk, the gzip header and segment compaction.
//   3. gzip_crc32: per chunk, 64 lanes CRC their slices, lane 0 combines them
//      with a precomputed GF(2) shift operator; CRC32 + ISIZE trailer.
#include "zcg_common.h"

namespace zcg {

constexpr u32 DF_SEG = 16384;               // input bytes per segment (one deflate block)
constexpr u32 DF_HIST = 32768;              // deflate window
constexpr u32 DF_WIN = DF_SEG + DF_HIST;
constexpr u32 DF_SLOT = DF_SEG + 128;       // output slot per segment (stored worst case + sync)
constexpr u32 DF_HBITS = 12;
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

__device__ __forceinline__ u32 len_code(u32 len) {  // 3..258 -> 0..28
    u32 c = 0;
#pragma unroll
    for (u32 i = 1; i < 29; i++) c += (len >= d_len_base[i]) ? 1u : 0u;
    return c;
}
__device__ __forceinline__ u32 dist_code(u32 d) {  // 1..32768 -> 0..29
    u32 c = 0;
#pragma unroll
    for (u32 i = 1; i < 30; i++) c += (d >= d_dist_base[i]) ? 1u : 0u;
    return c;
}
__device__ __forceinline__ u32 rev_bits(u32 v, u32 n) { return n ? __builtin_bitreverse32(v) >> (32 - n) : 0u; }

struct DefLds {
    u8 win[DF_WIN + 64];
    u16 t0[1u << DF_HBITS];    // per 3-byte hash: latest position + 1 (0 = empty)
    u16 t1[1u << DF_HBITS];    // ... and the one before it
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
__device__ __forceinline__ u32 hash3(u32 v) { return ((v & 0xFFFFFFu) * 2654435761u) >> (32 - DF_HBITS); }

// Insert position p (hash h) at the head of its 2-slot bucket.  Lanes of one
// instruction that share a bucket resolve in hardware order; every candidate
// is verified before use, and pass B checks that it only emits coded symbols
// (else the segment is stored), so the stream never depends on that order.
__device__ __forceinline__ void ins2(DefLds& L, u32 h, u32 p) {
    const u16 old = L.t0[h];
    L.t1[h] = old;
    L.t0[h] = (u16)(p + 1);
}

// One pass of the segment parse over window positions [h0, wend).
// EMIT=false: symbol frequencies.  EMIT=true: bits into the ring (bp, fw).
template <bool EMIT>
__device__ void parse_pass(DefLds& L, u32 h0, u32 wend, ParseCfg cfg, u32* bp, u32* fw, u8* out) {
    const u32 lane = lane_id();
    auto rd32 = [&](u32 p) -> u32 {
        const u32* w = (const u32*)L.win;
        return __builtin_amdgcn_alignbit(w[(p >> 2) + 1], w[p >> 2], (p & 3) * 8);
    };
    // fresh buckets; insert the history positions (no matching)
    for (u32 q = lane; q < (1u << DF_HBITS) / 2; q += 64) { ((u32*)L.t0)[q] = 0; ((u32*)L.t1)[q] = 0; }
    __syncthreads();
    for (u32 g = 0; g < h0; g += 64) {
        const u32 p = g + lane;
        const bool on = p < h0 && p + 3 <= wend;
        const u32 h = on ? hash3(rd32(p)) : 0u;
        if (on) ins2(L, h, p);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    u32 ip = h0;
    // literal emission for positions [a, b) (b - a <= 64)
    auto literals = [&](u32 a, u32 b) {
        const u32 p = a + lane;
        const bool on = p < b;
        const u32 byte = on ? L.win[p] : 0u;
        if (!EMIT) {
            if (on) atomicAdd(&L.lfreq[byte], 1u);
            return;
        }
        const u32 cw = on ? L.lcode[byte] : 0u;
        const u32 nb = cw >> 16;
        if (on && nb == 0) L.ctl[CTL_ERR] = 1;
        u32 x = nb;  // wave exclusive scan of code lengths
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u32 y = __shfl_up(x, d, 64);
            if ((int)lane >= d) x += y;
        }
        const u32 tot = __shfl(x, 63, 64);
        if (on) ring_put(L, *bp + x - nb, cw & 0xFFFF, nb);
        *bp += tot;
    };
    auto match_len = [&](u32 p, u32 r) -> u32 {  // 3 bytes verified; extend to <= 258, < wend
        u32 e = p + 3;
        const u32 lim = (p + 258 < wend) ? p + 258 : wend;
        for (;;) {
            const u32 x = e + lane;
            const bool ok = x < lim && L.win[x] == L.win[x - (p - r)];
            const unsigned long long bm = __ballot(!ok);
            const u32 run = bm ? (u32)__builtin_ctzll(bm) : 64u;
            e += run;
            if (run < 64) break;
        }
        return e - p;
    };
    // best (length, ref) of lane `l`'s two candidates (wave-uniform call)
    auto best_of = [&](u32 l, u32 r0, u32 r1, u32 ok0, u32 ok1, u32* blen, u32* bref) {
        const u32 p = ip + l;
        const u32 a0 = (u32)__shfl((int)r0, (int)l, 64), a1 = (u32)__shfl((int)r1, (int)l, 64);
        const u32 k0 = (u32)__shfl((int)ok0, (int)l, 64), k1 = (u32)__shfl((int)ok1, (int)l, 64);
        u32 bl = 0, br = 0;
        if (k0) { const u32 ln = match_len(p, a0); bl = ln; br = a0; }
        if (k1) {
            const u32 ln = match_len(p, a1);
            if (ln > bl) { bl = ln; br = a1; }
        }
        if (bl == 3 && p - br > 4096) bl = 0;  // zlib TOO_FAR: a far 3-byte match does not pay
        *blen = bl;
        *bref = br;
    };
    constexpr u32 LCAP = 32;  // per-lane match measurement cap
    // lane-local match length from 3 verified bytes, capped at min(LCAP, wend - p)
    auto ext = [&](u32 p, u32 r) -> u32 {
        const u32 lim = (wend - p) < LCAP ? (wend - p) : LCAP;
        u32 k = 3;
        while (k < lim) {
            const u32 x = rd32(p + k) ^ rd32(r + k);
            if (x) { k += (u32)__builtin_ctz(x) >> 3; break; }
            k += 4;
        }
        return k < lim ? k : lim;
    };
    while (ip < wend) {
        // keep the ring from wrapping: a group adds < 2 Kbit
        if (EMIT && (*bp >> 5) >= *fw + DF_FLUSH) ring_flush(L, out, fw, *bp >> 5);
        const u32 gend = (wend - ip) < 64 ? (wend - ip) : 64u;  // positions of this group
        const u32 p = ip + lane;
        const bool valid = lane < gend && p + 3 <= wend;
        const u32 v = valid ? rd32(p) : 0u;
        const u32 h = hash3(v);
        const u32 e0 = valid ? (u32)L.t0[h] : 0u, e1 = valid ? (u32)L.t1[h] : 0u;
        const u32 r0 = e0 - 1, r1 = e1 - 1;
        auto cand_len = [&](u32 e, u32 r) -> u32 {
            if (!valid || e == 0 || r >= p || p - r > DF_HIST) return 0u;
            if (((rd32(r) ^ v) & 0xFFFFFFu) != 0) return 0u;
            const u32 ln = ext(p, r);
            return (ln == 3 && p - r > 4096) ? 0u : ln;  // zlib TOO_FAR
        };
        const u32 l0 = cand_len(e0, r0), l1 = cand_len(e1, r1);
        u32 bl = l1 > l0 ? l1 : l0;                  // ties: the nearer (t0)
        u32 br = l1 > l0 ? r1 : r0;
        // positions of this group are not in the buckets yet: try the nearest
        // of a few short distances inside the group (periodic element data)
        {
            u32 dn = 0;
#pragma unroll
            for (u32 dd = 1; dd <= 32; dd <<= 1) {
                const u32 vd = (u32)__shfl_up((int)v, dd, 64);
                if (!dn && lane >= dd && ((vd ^ v) & 0xFFFFFFu) == 0) dn = dd;
            }
            if (valid && dn) {
                const u32 ln = ext(p, p - dn);
                if (ln > bl) { bl = ln; br = p - dn; }
            }
        }
        const unsigned long long mask = __ballot(bl >= 3);
        if (valid) ins2(L, h, p);  // all lookups of the group are done
        __builtin_amdgcn_wave_barrier();
        // walk the group: successive greedy (lazy) matches from the lane lengths
        u32 pos = 0;
        while (pos < gend) {
            const unsigned long long mm = mask & (~0ull << pos);
            if (!mm) { literals(ip + pos, ip + gend); pos = gend; break; }
            u32 f = (u32)__builtin_ctzll(mm);
            u32 mlen = (u32)__shfl((int)bl, (int)f, 64), mref = (u32)__shfl((int)br, (int)f, 64);
            if (cfg.lazy && mlen < 32 && f + 1 < gend && ((mask >> (f + 1)) & 1ull)) {
                const u32 l2 = (u32)__shfl((int)bl, (int)(f + 1), 64);
                if (l2 > mlen) { f = f + 1; mlen = l2; mref = (u32)__shfl((int)br, (int)f, 64); }
            }
            const u32 mpos = ip + f;
            if (mlen == LCAP) {  // measured to the cap: extend wave-parallel up to 258
                u32 e = mpos + LCAP;
                const u32 lim = (mpos + 258 < wend) ? mpos + 258 : wend;
                const u32 d = mpos - mref;
                for (;;) {
                    const u32 x = e + lane;
                    const bool okb = x < lim && L.win[x] == L.win[x - d];
                    const unsigned long long bm = __ballot(!okb);
                    const u32 run = bm ? (u32)__builtin_ctzll(bm) : 64u;
                    e += run;
                    if (run < 64) break;
                }
                mlen = e - mpos;
            }
            if (f > pos) literals(ip + pos, ip + f);
            const u32 d = mpos - mref;
            const u32 lc = len_code(mlen), dc = dist_code(d);
            if (!EMIT) {
                if (lane == 0) { atomicAdd(&L.lfreq[257 + lc], 1u); atomicAdd(&L.dfreq[dc], 1u); }
            } else {
                const u32 lcw = L.lcode[257 + lc], dcw = L.dcode[dc];  // uniform reads
                const u32 nl = lcw >> 16, nd = dcw >> 16;
                const u32 el = d_len_extra[lc], ed = d_dist_extra[dc];
                if (lane == 0) {
                    if (nl == 0 || nd == 0) L.ctl[CTL_ERR] = 1;
                    u32 b = *bp;
                    ring_put(L, b, lcw & 0xFFFF, nl); b += nl;
                    ring_put(L, b, mlen - d_len_base[lc], el); b += el;
                    ring_put(L, b, dcw & 0xFFFF, nd); b += nd;
                    ring_put(L, b, d - d_dist_base[dc], ed);
                }
                *bp += nl + el + nd + ed;
            }
            pos = f + mlen;
            if (pos > gend) {  // the match runs past the group: insert its last two positions
                const u32 endp = ip + pos;
                if (lane < 2) {
                    const u32 q = endp - 2 + lane;
                    if (q + 3 <= wend && q >= ip + gend) ins2(L, hash3(rd32(q)), q);
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        ip += pos;
    }
    if (EMIT && (*bp >> 5) >= *fw + DF_FLUSH) ring_flush(L, out, fw, *bp >> 5);
}

__global__ __launch_bounds__(64) void deflate_segment(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                      u32 nseg, u64 bound, DType t, u32 level) {
    extern __shared__ __attribute__((aligned(16))) u8 smem_raw[];
    DefLds& L = *(DefLds*)smem_raw;
    const u32 lane = threadIdx.x;
    const u32 c = blockIdx.x / nseg, k = blockIdx.x % nseg;
    if (c >= n) return;
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
    // ---- stage [w0, s0 + S) transformed ----------------------------------------
    for (u32 q = lane * 16; q < wend; q += 64 * 16) {
        if (q + 16 <= wend) {
            *(u32x4*)(L.win + q) = transform16(ld16(src + w0 + q), t);
        } else {
            for (u32 i = q; i < wend; i++) L.win[i] = norm_byte(src[swap_pos(w0 + i, t)], t);
        }
    }
    for (u32 q = wend + lane; q < wend + 64; q += 64) L.win[q] = 0;
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
        parse_pass<false>(L, hist, wend, cfg, &bp, &fw, out);
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
        for (u32 q = lane; q < S; q += 64) out[5 + q] = L.win[hist + q];
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
    parse_pass<true>(L, hist, wend, cfg, &bp, &fw, out);
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
        for (u32 q = lane; q < S; q += 64) out[5 + q] = L.win[hist + q];
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
__global__ __launch_bounds__(64) void gzip_crc32(const zcg_chunk* __restrict__ chunks, u32 n, u64 D,
                                                 u64 Lsl, CrcShift op, const u64* __restrict__ out_len,
                                                 const i32* __restrict__ status, DType t) {
    const u32 c = blockIdx.x, lane = threadIdx.x;
    if (c >= n || status[c] != ZCG_OK) return;
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

hipError_t launch_deflate(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                          uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                          hipStream_t s) {
    (void)ws; (void)ws_bytes;
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const u32 level = (u32)zcg_effective_gzip_level(a->compression.gzip_level);
    const u32 xfl = level >= 9 ? 2u : (level <= 1 ? 4u : 0u);
    const u32 nseg = (u32)((D + DF_SEG - 1) / DF_SEG);
    const u64 bound = zcg_encode_bound(&a->compression, D);
    if (nseg) {
        static bool attr = false;
        if (!attr) {
            hipError_t e = hipFuncSetAttribute((const void*)deflate_segment,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)sizeof(DefLds));
            if (e != hipSuccess) return e;
            attr = true;
        }
        const u64 nb = (u64)n * nseg;
        if (nb > 0x7FFFFFFFull) return hipErrorInvalidValue;
        hipLaunchKernelGGL(deflate_segment, dim3((u32)nb), dim3(64), sizeof(DefLds), s, d_chunks, n, D,
                           nseg, bound, t, level);
    }
    hipLaunchKernelGGL(deflate_finalize, dim3(n), dim3(256), 0, s, d_chunks, n, D, nseg, bound, xfl,
                       (u64*)d_out_len, d_status);
    const u64 Lsl = D / 64;
    CrcShift op;
    crc_shift_op(Lsl, op.m);
    hipLaunchKernelGGL(gzip_crc32, dim3(n), dim3(64), 0, s, d_chunks, n, D, Lsl, op,
                       (const u64*)d_out_len, (const i32*)d_status, t);
    return hipGetLastError();
}

}  // namespace zcg
