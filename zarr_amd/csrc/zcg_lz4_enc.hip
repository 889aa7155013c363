// zcg_lz4_enc.hip — LZ4 frame encoder (write_chunk for CompressionType::Lz4).
//
// Reference: lz.rs:81-92 builds lz4-rs's encoder with the effective block size
// (lz.rs:55-65), BlockMode::Independent, level 0, content checksum on, no
// content size, no block checksum; LZ4F then writes
//   magic 04 22 4D 18 | FLG 0x64 | BD (id << 4) | HC = XXH32(FLG,BD) >> 8
//   blocks: u32 LE size (bit 31 = stored) + data; an end mark 0; XXH32(content).
// A block is stored uncompressed when its compressed form is not smaller
// (LZ4F_makeBlock).  The compressed bytes themselves are not pinned by the
// reference; any valid LZ4 block that LZ4_decompress_safe accepts
// is a correct encoding, checked by round trips through the oracle.
//
// Kernels (stream-ordered):
//   0. match finding, data-parallel over every position of a sub-batch
//      (<= 128 MiB): keys (block, 20-bit hash of 4 serialised bytes) sorted
//      with the positions as values (hipCUB radix sort, stable), lz_chain links
//      each position to its predecessor with the same key, lz_best walks up to
//      LZ_DEPTH candidates with offsets <= 65535 and keeps the longest match
//      that ends before the block's last 5 literals (LZ4's end-of-block rules).
//   1. lz4_block_compress: one wave per block, greedy like LZ4's fast
//      encoder: the 64 lanes hold 64 consecutive positions' precomputed
//      matches and the first one starts the next sequence; literals are read
//      from HBM with the dtype transform (write_data's byte order,
//      chunk.rs:118-140), so the kernel uses no LDS.
//      Block k is written at its upper-bound slot 7 + k*(B+4) of dst.
//   2. lz4_frame_finalize: one workgroup per chunk writes the frame header,
//      compacts the blocks to their final offsets (tile copies, dst <= src),
//      writes the end mark and the output length.
//   3. lz4_content_xxh32: 4 lanes per chunk (one XXH32 accumulator each)
//      hash the serialised content and write the content checksum.
#include <hipcub/hipcub.hpp>

#include "zcg_common.h"

namespace zcg {

constexpr u32 LE_WIN = 65536;       // LDS window (matches stay inside it)
constexpr u32 LE_HBITS = 12;        // hash table entries = 4096
constexpr u32 LE_MFLIMIT = 12;      // last match starts >= 12 bytes before block end
constexpr u32 LE_LASTLIT = 5;       // last 5 bytes are literals
constexpr u32 LE_MINLEN = 13;       // shorter blocks are literals only
constexpr u32 LE_HDR = 7;           // frame header bytes
constexpr u32 LE_MCAP = 32;         // match bytes measured by lz_best (longer ones are extended here)

// Logical (serialised) byte x of the chunk: the stream holds elements in the
// array's byte order; bool as 0/1.
__device__ __forceinline__ u8 src_byte(const u8* src, u64 x, const DType& t) {
    return norm_byte(src[swap_pos(x, t)], t);
}

// Write `n` literal bytes of the chunk starting at logical position `x` to
// out[o..).  Bytes inside the staged window come from LDS, others from src.
__device__ void put_literals(u8* out, u64 o, const u8* src, u64 x, u32 n, const u8* win, u64 wbase,
                             u32 wlen, const DType& t) {
    const u32 lane = lane_id();
    for (u32 k = lane; k < n; k += 64) {
        const u64 p = x + k;
        u8 v;
        if (p >= wbase && p < wbase + wlen) v = win[p - wbase];
        else v = src_byte(src, p, t);
        out[o + k] = v;
    }
}

// Bytes of a length field (token nibble already counts 15).
__device__ __forceinline__ u32 len_bytes(u32 v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

__device__ void put_len(u8* out, u64 o, u32 v) {  // v >= 15; writes len_bytes(v) bytes
    const u32 lane = lane_id();
    const u32 nb = len_bytes(v);
    for (u32 k = lane; k + 1 < nb; k += 64) out[o + k] = 255;
    if (lane == 0) out[o + nb - 1] = (u8)((v - 15) % 255);
}

__global__ __launch_bounds__(64) void lz4_block_compress(const zcg_chunk* __restrict__ chunks, u32 c0, u32 n,
                                                         u64 D, u32 B, u32 nbpc, u64 bound, DType t,
                                                         const u32* __restrict__ match) {
    const u32 lane = threadIdx.x;
    const u32 cl = blockIdx.x / nbpc, k = blockIdx.x % nbpc;
    if (cl >= n) return;
    const u32 c = c0 + cl;
    const zcg_chunk ch = chunks[c];
    if (ch.dst_cap < bound || ch.src_len < D) return;  // finalize reports the status
    const u8* src = (const u8*)ch.src;
    u8* dst = (u8*)ch.dst;
    const u64 b0 = (u64)k * B;                          // logical start of the block
    const u32 S = (u32)((D - b0) < B ? (D - b0) : B);   // block bytes
    const u32* mt = match + (u64)cl * D + b0;           // precomputed matches of the block
    u8* hdr = dst + LE_HDR + (u64)k * (B + 4);
    u8* out = hdr + 4;
    u64 op = 0;          // output bytes of this block
    bool stored = S < LE_MINLEN;
    u64 anchor = 0;      // block-relative start of the pending literal run
    if (!stored) {
        // match starts < S - MFLIMIT, match ends <= S - LASTLIT (lz_best clips)
        const u32 mflim = S - LE_MFLIMIT;
        u32 ip = 0;
        u32 wbase = 0xFFFFFFFFu, wm = 0;  // 64 positions' matches, one per lane
        while (ip < mflim) {
            if (ip < wbase || ip >= wbase + 64) {
                wbase = ip;
                const u32 p = ip + lane;
                wm = p < mflim ? mt[p] : 0u;
            }
            const u32 sh = ip - wbase;
            const unsigned long long m = __ballot((wm & 0xFFFF) >= 4) & (~0ull << sh);
            if (!m) { ip = wbase + 64; continue; }
            const u32 f = (u32)__builtin_ctzll(m);
            const u32 mv = __shfl(wm, (int)f, 64);
            const u32 mpos = wbase + f;
            u32 mlen = mv & 0xFFFF;
            const u32 d = mv >> 16;
            if (mlen == LE_MCAP) {  // measured to the cap: extend 64 bytes per step
                const u32 lim = S - LE_LASTLIT;  // block-relative match end limit
                u32 e2 = mpos + mlen;
                for (;;) {
                    const u32 x = e2 + lane;
                    const bool ok = x < lim && src_byte(src, b0 + x, t) == src_byte(src, b0 + x - d, t);
                    const unsigned long long bm = __ballot(!ok);
                    const u32 run = bm ? (u32)__builtin_ctzll(bm) : 64u;
                    e2 += run;
                    if (run < 64) break;
                }
                mlen = e2 - mpos;
            }
            // ---- emit the sequence: literals [anchor, mpos), match (d, mlen) ----
            const u32 lit = (u32)(mpos - anchor);
            const u64 sz = 1 + len_bytes(lit) + lit + 2 + len_bytes(mlen - 4);
            if (op + sz + 1 + LE_LASTLIT >= S) { stored = true; break; }
            if (lane == 0) out[op] = (u8)(((lit < 15 ? lit : 15) << 4) | ((mlen - 4) < 15 ? (mlen - 4) : 15));
            u64 o = op + 1;
            if (lit >= 15) { put_len(out, o, lit); o += len_bytes(lit); }
            put_literals(out, o, src, b0 + anchor, lit, nullptr, 0, 0, t);
            o += lit;
            if (lane == 0) { out[o] = (u8)(d & 0xFF); out[o + 1] = (u8)(d >> 8); }
            o += 2;
            if (mlen - 4 >= 15) { put_len(out, o, mlen - 4); o += len_bytes(mlen - 4); }
            op = o;
            anchor = mpos + mlen;
            ip = mpos + mlen;
        }
    }
    if (!stored) {  // last literals
        const u32 lit = (u32)(S - anchor);
        const u64 sz = 1 + len_bytes(lit) + lit;
        if (op + sz >= S) {
            stored = true;
        } else {
            if (lane == 0) out[op] = (u8)((lit < 15 ? lit : 15) << 4);
            u64 o = op + 1;
            if (lit >= 15) { put_len(out, o, lit); o += len_bytes(lit); }
            put_literals(out, o, src, b0 + anchor, lit, nullptr, 0, 0, t);
            op = o + lit;
        }
    }
    if (stored) {  // uncompressed block (LZ4F_makeBlock)
        for (u32 q = lane; q < S; q += 64) out[q] = src_byte(src, b0 + q, t);
        op = S;
    }
    if (lane == 0) {
        const u32 w = (u32)op | (stored ? 0x80000000u : 0u);
        hdr[0] = (u8)w; hdr[1] = (u8)(w >> 8); hdr[2] = (u8)(w >> 16); hdr[3] = (u8)(w >> 24);
    }
}

// BD byte for the effective block size (lz.rs:55-65 -> LZ4F blockSizeID 4..7)
__host__ __device__ inline u32 lz4_bd(u32 B) {
    return B <= 65536 ? 0x40u : B <= 262144 ? 0x50u : B <= 1048576 ? 0x60u : 0x70u;
}

__global__ __launch_bounds__(256) void lz4_frame_finalize(const zcg_chunk* __restrict__ chunks, u32 n,
                                                          u64 D, u32 B, u32 nbpc, u64 bound,
                                                          u64* __restrict__ out_len,
                                                          i32* __restrict__ status) {
    const u32 c = blockIdx.x, tid = threadIdx.x;
    if (c >= n) return;
    const zcg_chunk ch = chunks[c];
    if (ch.src_len < D) { if (tid == 0) { status[c] = ZCG_ERR_INVALID_DATA; out_len[c] = 0; } return; }
    if (ch.dst_cap < bound) { if (tid == 0) { status[c] = ZCG_ERR_OUTPUT_TOO_SMALL; out_len[c] = 0; } return; }
    u8* dst = (u8*)ch.dst;
    if (tid == 0) {
        dst[0] = 0x04; dst[1] = 0x22; dst[2] = 0x4D; dst[3] = 0x18;
        dst[4] = 0x64;  // version 01, independent blocks, content checksum
        dst[5] = (u8)lz4_bd(B);
        dst[6] = (u8)((xxh32(dst + 4, 2, 0) >> 8) & 0xFF);
    }
    __shared__ u32 s_sz;
    u64 pos = LE_HDR;
    for (u32 k = 0; k < nbpc; k++) {
        const u64 tmp = LE_HDR + (u64)k * (B + 4);
        __syncthreads();
        if (tid == 0) s_sz = ld32(dst + tmp);
        __syncthreads();
        const u64 total = 4 + (s_sz & 0x7FFFFFFFu);
        if (tmp != pos) {
            // dst < src: copy in 4 KiB tiles, all reads of a tile before its writes
            for (u64 q = 0; q < total; q += 256 * 16) {
                const u64 i = q + (u64)tid * 16;
                u32x4 v = {0u, 0u, 0u, 0u};
                u32 nb = 0;
                if (i < total) {
                    nb = (total - i) < 16 ? (u32)(total - i) : 16u;
                    if (nb == 16) v = ld16(dst + tmp + i);
                    else {
                        u8 b[16];
                        for (u32 j = 0; j < nb; j++) b[j] = dst[tmp + i + j];
                        for (u32 j = 0; j < nb; j++) ((u8*)&v)[j] = b[j];
                    }
                }
                __syncthreads();
                if (nb == 16) st16(dst + pos + i, v);
                else for (u32 j = 0; j < nb; j++) dst[pos + i + j] = ((u8*)&v)[j];
                __syncthreads();
            }
        }
        pos += total;
    }
    if (tid < 4) dst[pos + tid] = 0;  // end mark
    if (tid == 0) {
        out_len[c] = pos + 8;  // + end mark + content checksum (kernel 3)
        status[c] = ZCG_OK;
    }
}

// Content checksum: 16 chunks per wave, lanes 4g..4g+3 hold accumulators v1..v4
// of chunk g (XXH32 stripes of 16 serialised bytes).
__global__ __launch_bounds__(64) void lz4_content_xxh32(const zcg_chunk* __restrict__ chunks, u32 n,
                                                        u64 D, const u64* __restrict__ out_len,
                                                        const i32* __restrict__ status, DType t) {
    const u32 lane = threadIdx.x;
    const u32 g = lane >> 2, j = lane & 3;
    const u32 c = blockIdx.x * 16 + g;
    const bool act = c < n && status[c] == ZCG_OK;
    const u8* src = act ? (const u8*)chunks[c].src : nullptr;
    const u32 P1 = XXH_P1, P2 = XXH_P2;
    u32 v = (j == 0) ? P1 + P2 : (j == 1) ? P2 : (j == 2) ? 0u : 0u - P1;
    const u64 nstripe = D >= 16 ? D / 16 : 0;
    if (act) {
        u64 s = 0;
        for (; s + 8 <= nstripe; s += 8) {
            u32 w[8];
#pragma unroll
            for (u32 u = 0; u < 8; u++) {
                const u32x4 x = transform16(ld16(src + (s + u) * 16), t);
                w[u] = j == 0 ? x.x : j == 1 ? x.y : j == 2 ? x.z : x.w;
            }
#pragma unroll
            for (u32 u = 0; u < 8; u++) v = rotl32(v + w[u] * P2, 13) * P1;
        }
        for (; s < nstripe; s++) {
            const u32x4 x = transform16(ld16(src + s * 16), t);
            const u32 w = j == 0 ? x.x : j == 1 ? x.y : j == 2 ? x.z : x.w;
            v = rotl32(v + w * P2, 13) * P1;
        }
    }
    const u32 v1 = __shfl(v, (int)(lane & ~3u) + 0, 64), v2 = __shfl(v, (int)(lane & ~3u) + 1, 64);
    const u32 v3 = __shfl(v, (int)(lane & ~3u) + 2, 64), v4 = __shfl(v, (int)(lane & ~3u) + 3, 64);
    if (!act || j != 0) return;
    u32 h = D >= 16 ? rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18) : XXH_P5;
    h += (u32)D;
    u64 p = nstripe * 16;
    for (; p + 4 <= D; p += 4) {
        const u32 w = (u32)src_byte(src, p, t) | ((u32)src_byte(src, p + 1, t) << 8) |
                      ((u32)src_byte(src, p + 2, t) << 16) | ((u32)src_byte(src, p + 3, t) << 24);
        h += w * XXH_P3;
        h = rotl32(h, 17) * XXH_P4;
    }
    for (; p < D; p++) {
        h += (u32)src_byte(src, p, t) * XXH_P5;
        h = rotl32(h, 11) * XXH_P1;
    }
    h ^= h >> 15; h *= XXH_P2; h ^= h >> 13; h *= XXH_P3; h ^= h >> 16;
    u8* o = (u8*)chunks[c].dst + out_len[c] - 4;
    o[0] = (u8)h; o[1] = (u8)(h >> 8); o[2] = (u8)(h >> 16); o[3] = (u8)(h >> 24);
}

namespace {

constexpr u32 LZ_DEPTH = 4;                 // chain candidates per position
constexpr u32 LZ_CAP = LE_MCAP;             // bytes measured per candidate
constexpr u32 LZ_KEYBITS = 20;
constexpr u64 LZ_SUB_BYTES = 128ull << 20;  // input bytes per match-finder sub-batch
constexpr u64 LZ_SUPER_BYTES = 1ull << 30;  // input bytes per block-compress launch

struct LzLayout {
    u32 m, sm;
    u64 tot, cub_bytes;
    u64 off_ka, off_kb, off_va, off_vb, off_prev, off_match, off_cub, total;
};

LzLayout lz_layout(u64 D, u32 nbpc, u32 n) {
    LzLayout y{};
    u64 m = D ? LZ_SUB_BYTES / D : n;
    if (m < 1) m = 1;
    if (m > n) m = n;
    while (m > 1 && m * nbpc > 4096) m--;  // block id + 20 hash bits fit 32
    y.m = (u32)m;
    y.tot = m * D;
    u64 sm = D ? LZ_SUPER_BYTES / D : n;
    sm = sm / m * m;
    if (sm < m) sm = m;
    if (sm > n) sm = n;
    y.sm = (u32)sm;
    size_t cb = 0;
    hipcub::DoubleBuffer<u32> kk(nullptr, nullptr), v(nullptr, nullptr);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, cb, kk, v, (int)(y.tot ? y.tot : 1), 0, 32);
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

typedef __attribute__((address_space(1))) u32 le_gu32_ua __attribute__((aligned(1)));
__device__ __forceinline__ u32 lz_ser4(const u8* src, u64 x, const DType& t) {  // bytes x..x+3, LE
    if (!t.swap && !t.isbool) return *(const le_gu32_ua*)((const __attribute__((address_space(1))) u8*)src + x);  // (global, not flat)
    return (u32)src_byte(src, x, t) | ((u32)src_byte(src, x + 1, t) << 8) | ((u32)src_byte(src, x + 2, t) << 16) |
           ((u32)src_byte(src, x + 3, t) << 24);
}

__global__ void lz_keys(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, u32 B, u32 nbpc, u64 tot, DType t,
                        u32* __restrict__ keys, u32* __restrict__ vals) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tot) return;
    const u32 cl = (u32)(g / D);
    const u64 p = g - (u64)cl * D;
    const u32 blk = (u32)(p / B);
    const u64 bend = ((u64)blk + 1) * B < D ? ((u64)blk + 1) * B : D;
    u32 h = 0;
    if (p + 4 <= bend && chunks[c0 + cl].src_len >= D) h = (lz_ser4((const u8*)chunks[c0 + cl].src, p, t) * 2654435761u) >> (32 - LZ_KEYBITS);
    keys[g] = ((cl * nbpc + blk) << LZ_KEYBITS) | h;
    vals[g] = (u32)g;
}

__global__ void lz_chain(u64 tot, const u32* __restrict__ keys, const u32* __restrict__ vals,
                         u32* __restrict__ prev) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= tot) return;
    prev[vals[j]] = (j > 0 && keys[j] == keys[j - 1]) ? vals[j - 1] : 0xFFFFFFFFu;
}

// match[g] = len | offset << 16 (len 0: none); the match starts before the
// block's MFLIMIT and ends at or before its last LASTLIT bytes
__global__ void lz_best(const zcg_chunk* __restrict__ chunks, u32 c0, u64 D, u32 B, u64 tot, DType t,
                        const u32* __restrict__ prev, u32* __restrict__ match) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tot) return;
    const u32 cl = (u32)(g / D);
    const u64 p = g - (u64)cl * D;
    const u64 bs = p / B * B;
    const u64 bend = bs + B < D ? bs + B : D;
    u32 best = 0, bd = 0;
    if (p + LE_MFLIMIT < bend && chunks[c0 + cl].src_len >= D) {  // short src: INVALID_DATA in finalize
        const u8* src = (const u8*)chunks[c0 + cl].src;
        const u64 cbase = (u64)cl * D;
        u32 mx = (u32)(bend - LE_LASTLIT - p);  // bytes the match may cover
        if (mx > LZ_CAP) mx = LZ_CAP;           // longer matches are extended by lz4_block_compress
        const u32 v0 = lz_ser4(src, p, t);
        u32 q = prev[g];
        for (u32 dep = 0; dep < LZ_DEPTH && q != 0xFFFFFFFFu; dep++) {
            const u64 qp = q - cbase;
            if (p - qp > 65535) break;
            const u32 qn = prev[q];  // the next link, in flight during this candidate's compare
            if (lz_ser4(src, qp, t) == v0) {
                u32 k = 4;
                bool diff = false;
                while (k + 4 <= mx) {
                    const u32 x = lz_ser4(src, p + k, t) ^ lz_ser4(src, qp + k, t);
                    if (x) { k += (u32)__builtin_ctz(x) >> 3; diff = true; break; }
                    k += 4;
                }
                if (!diff)
                    while (k < mx && src_byte(src, p + k, t) == src_byte(src, qp + k, t)) k++;
                if (k > mx) k = mx;
                if (k > best) { best = k; bd = (u32)(p - qp); }
            }
            q = qn;
        }
    }
    match[g] = best >= 4 ? (best | (bd << 16)) : 0u;
}

}  // namespace

uint64_t lz4_encode_ws_bytes(const zcg_array* a, uint32_t n) {
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const u32 B = (u32)zcg_effective_lz4_block_size(a->compression.lz4_block_size);
    const u32 nbpc = (u32)((D + B - 1) / B);
    if (n == 0 || nbpc == 0) return 0;
    return lz_layout(D, nbpc, n).total;
}

hipError_t launch_lz4_encode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                             uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const u32 B = (u32)zcg_effective_lz4_block_size(a->compression.lz4_block_size);
    const u32 nbpc = (u32)((D + B - 1) / B);
    const u64 bound = zcg_encode_bound(&a->compression, D);
    if (nbpc) {
        if (nbpc > 4096) return hipErrorInvalidValue;
        const LzLayout y = lz_layout(D, nbpc, n);
        if (ws_bytes < y.total || y.tot >= (1ull << 31)) return hipErrorInvalidValue;
        u8* w = (u8*)ws;
        for (u32 s0 = 0; s0 < n; s0 += y.sm) {
            const u32 scnt = (n - s0) < y.sm ? (n - s0) : y.sm;
            for (u32 c0 = s0; c0 < s0 + scnt; c0 += y.m) {
                const u32 cnt = (s0 + scnt - c0) < y.m ? (s0 + scnt - c0) : y.m;
                const u64 tot = (u64)cnt * D;
                u32 *ka = (u32*)(w + y.off_ka), *kb = (u32*)(w + y.off_kb);
                u32 *va = (u32*)(w + y.off_va), *vb = (u32*)(w + y.off_vb);
                const u32 G = (u32)((tot + 255) / 256);
                u32 bbits = 0;
                while ((1u << bbits) < cnt * nbpc) bbits++;
                hipLaunchKernelGGL(lz_keys, dim3(G), dim3(256), 0, s, d_chunks, c0, D, B, nbpc, tot, t, ka, va);
                hipcub::DoubleBuffer<u32> dk(ka, kb), dv(va, vb);
                size_t cb = y.cub_bytes;
                hipError_t e = hipcub::DeviceRadixSort::SortPairs(w + y.off_cub, cb, dk, dv, (int)tot, 0,
                                                                  (int)(LZ_KEYBITS + bbits), s);
                if (e != hipSuccess) return e;
                hipLaunchKernelGGL(lz_chain, dim3(G), dim3(256), 0, s, tot, dk.Current(), dv.Current(),
                                   (u32*)(w + y.off_prev));
                hipLaunchKernelGGL(lz_best, dim3(G), dim3(256), 0, s, d_chunks, c0, D, B, tot, t,
                                   (const u32*)(w + y.off_prev), (u32*)(w + y.off_match) + (u64)(c0 - s0) * D);
            }
            const u64 nb = (u64)scnt * nbpc;
            if (nb > 0x7FFFFFFFull) return hipErrorInvalidValue;
            hipLaunchKernelGGL(lz4_block_compress, dim3((u32)nb), dim3(64), 0, s, d_chunks, s0, scnt, D, B, nbpc,
                               bound, t, (const u32*)(w + y.off_match));
        }
    }
    hipLaunchKernelGGL(lz4_frame_finalize, dim3(n), dim3(256), 0, s, d_chunks, n, D, B, nbpc, bound,
                       (u64*)d_out_len, d_status);
    hipLaunchKernelGGL(lz4_content_xxh32, dim3((n + 15) / 16), dim3(64), 0, s, d_chunks, n, D,
                       (const u64*)d_out_len, (const i32*)d_status, t);
    return hipGetLastError();
}

}  // namespace zcg
