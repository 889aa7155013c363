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
//   1. lz4_block_compress: one wave per block.  The block is parsed in 64 KiB
//      windows staged in LDS (dtype transform applied: the stream holds the
//      array's serialised bytes, chunk.rs:118-140).  The 64 lanes hash 64
//      consecutive positions at once; the first lane whose hash candidate
//      verifies is the next greedy match; matches extend 64 bytes per step.
//      Block k is written at its upper-bound slot 7 + k*(B+4) of dst.
//   2. lz4_frame_finalize: one workgroup per chunk writes the frame header,
//      compacts the blocks to their final offsets (tile copies, dst <= src),
//      writes the end mark and the output length.
//   3. lz4_content_xxh32: 4 lanes per chunk (one XXH32 accumulator each)
//      hash the serialised content and write the content checksum.
#include "zcg_common.h"

namespace zcg {

constexpr u32 LE_WIN = 65536;       // LDS window (matches stay inside it)
constexpr u32 LE_HBITS = 12;        // hash table entries = 4096
constexpr u32 LE_MFLIMIT = 12;      // last match starts >= 12 bytes before block end
constexpr u32 LE_LASTLIT = 5;       // last 5 bytes are literals
constexpr u32 LE_MINLEN = 13;       // shorter blocks are literals only
constexpr u32 LE_HDR = 7;           // frame header bytes

struct LzEncLds {
    u8 win[LE_WIN + 64];            // window bytes (+ slack for 4-byte reads)
    u16 tab[1u << LE_HBITS];        // position + 1 of the latest position per hash, 0 = empty
                                    // (match starts are < 65536 - 12, so p + 1 fits)
};

// 4 bytes at LDS window offset p (any alignment).
__device__ __forceinline__ u32 win_rd32(const u8* win, u32 p) {
    const u32* w = (const u32*)win;
    const u32 a = w[p >> 2], b = w[(p >> 2) + 1];
    return __builtin_amdgcn_alignbit(b, a, (p & 3) * 8);
}

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

__global__ __launch_bounds__(64) void lz4_block_compress(const zcg_chunk* __restrict__ chunks, u32 n,
                                                         u64 D, u32 B, u32 nbpc, u64 bound, DType t) {
    extern __shared__ __attribute__((aligned(16))) u8 smem_raw[];
    LzEncLds& L = *(LzEncLds*)smem_raw;
    const u32 lane = threadIdx.x;
    const u32 c = blockIdx.x / nbpc, k = blockIdx.x % nbpc;
    if (c >= n) return;
    const zcg_chunk ch = chunks[c];
    if (ch.dst_cap < bound || ch.src_len < D) return;  // finalize reports the status
    const u8* src = (const u8*)ch.src;
    u8* dst = (u8*)ch.dst;
    const u64 b0 = (u64)k * B;                          // logical start of the block
    const u32 S = (u32)((D - b0) < B ? (D - b0) : B);   // block bytes
    u8* hdr = dst + LE_HDR + (u64)k * (B + 4);
    u8* out = hdr + 4;
    u64 op = 0;          // output bytes of this block
    bool stored = S < LE_MINLEN;
    u64 anchor = 0;      // block-relative start of the pending literal run
    for (u32 wb = 0; wb < S && !stored; wb += LE_WIN) {
        const u32 wl = (S - wb) < LE_WIN ? (S - wb) : LE_WIN;
        // ---- stage the window (transformed), clear the hash table ----------
        const u64 g0 = b0 + wb;
        for (u32 q = lane * 16; q < wl; q += 64 * 16) {
            if (q + 16 <= wl) {
                const u32x4 v = transform16(ld16(src + g0 + q), t);
                *(u32x4*)(L.win + q) = v;
            } else {
                for (u32 i = q; i < wl; i++) L.win[i] = src_byte(src, g0 + i, t);
            }
        }
        for (u32 q = wl + lane; q < wl + 64; q += 64) L.win[q] = 0;
        for (u32 q = lane; q < (1u << LE_HBITS) / 2; q += 64) ((u32*)L.tab)[q] = 0;
        __syncthreads();
        // match starts < S - MFLIMIT (block-relative), match ends <= S - LASTLIT
        const u32 mfl = (S - LE_MFLIMIT > wb) ? (S - LE_MFLIMIT - wb) : 0;
        const u32 mflim = mfl < wl ? mfl : wl;
        const u32 mlim_b = S - LE_LASTLIT;
        const u32 mlim = (mlim_b > wb) ? ((mlim_b - wb) < wl ? (mlim_b - wb) : wl) : 0;
        u32 ip = (anchor > wb) ? (u32)(anchor - wb) : 0;
        while (ip < mflim) {
            const u32 p = ip + lane;
            const bool valid = p < mflim && p + 4 <= wl;
            const u32 v = valid ? win_rd32(L.win, p) : 0u;
            const u32 h = (v * 2654435761u) >> (32 - LE_HBITS);
            const u32 e = valid ? (u32)L.tab[h] : 0u;
            const u32 ref = e - 1;
            const bool cand = valid && e != 0 && ref < p && win_rd32(L.win, ref) == v;
            const unsigned long long m = __ballot(cand);
            // insert the positions scanned up to (and including) the chosen
            // match start, like LZ4's sequential loop; positions after it are
            // scanned again after the match and must not find themselves.
            // Same-hash lanes: the store of the highest lane lands; any entry
            // is only a candidate (verified above), so the stream stays valid.
            const u32 f = m ? (u32)__builtin_ctzll(m) : 63u;
            if (valid && lane <= f) L.tab[h] = (u16)(p + 1);
            if (!m) { ip += 64; continue; }
            u32 mpos = ip + f;
            u32 mref = (u32)__shfl((int)ref, (int)f, 64);
            // backward extension (bounded by the pending literals and the window)
            {
                const u32 lo = (anchor > wb) ? (u32)(anchor - wb) : 0u;
                for (;;) {
                    const u32 room = mpos - lo < mref ? mpos - lo : mref;
                    const bool ok = lane < room && L.win[mpos - 1 - lane] == L.win[mref - 1 - lane];
                    const unsigned long long bm = __ballot(!ok);
                    const u32 run = bm ? (u32)__builtin_ctzll(bm) : 64u;
                    mpos -= run;
                    mref -= run;
                    if (run < 64) break;
                }
            }
            // forward extension from the verified 4 bytes
            const u32 orig = ip + f;
            u32 e2 = orig + 4;
            const u32 d = orig - (u32)__shfl((int)ref, (int)f, 64);  // offset (unchanged by back-ext)
            for (;;) {
                const u32 x = e2 + lane;
                const bool ok = x < mlim && L.win[x] == L.win[x - d];
                const unsigned long long bm = __ballot(!ok);
                const u32 run = bm ? (u32)__builtin_ctzll(bm) : 64u;
                e2 += run;
                if (run < 64) break;
            }
            if (e2 < orig + 4) e2 = orig + 4;  // (cannot happen: the 4 bytes verified, mlim >= orig+4)
            const u32 mlen = e2 - mpos;
            // ---- emit the sequence: literals [anchor, wb+mpos), match (d, mlen) ----
            const u32 lit = (u32)(wb + mpos - anchor);
            const u64 sz = 1 + len_bytes(lit) + lit + 2 + len_bytes(mlen - 4);
            if (op + sz + 1 + LE_LASTLIT >= S) { stored = true; break; }
            if (lane == 0) out[op] = (u8)(((lit < 15 ? lit : 15) << 4) | ((mlen - 4) < 15 ? (mlen - 4) : 15));
            u64 o = op + 1;
            if (lit >= 15) { put_len(out, o, lit); o += len_bytes(lit); }
            put_literals(out, o, src, b0 + anchor, lit, L.win, g0, wl, t);
            o += lit;
            if (lane == 0) { out[o] = (u8)(d & 0xFF); out[o + 1] = (u8)(d >> 8); }
            o += 2;
            if (mlen - 4 >= 15) { put_len(out, o, mlen - 4); o += len_bytes(mlen - 4); }
            op = o;
            anchor = wb + e2;
            ip = e2;
        }
        __syncthreads();  // the window is restaged next
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
            const u32 wl_last = (S - (S - 1) / LE_WIN * LE_WIN);
            put_literals(out, o, src, b0 + anchor, lit, L.win, b0 + (S - 1) / LE_WIN * LE_WIN, wl_last, t);
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

hipError_t launch_lz4_encode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                             uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                             hipStream_t s) {
    (void)ws; (void)ws_bytes;
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const u32 B = (u32)zcg_effective_lz4_block_size(a->compression.lz4_block_size);
    const u32 nbpc = (u32)((D + B - 1) / B);
    const u64 bound = zcg_encode_bound(&a->compression, D);
    if (nbpc) {
        static bool attr = false;
        if (!attr) {
            hipError_t e = hipFuncSetAttribute((const void*)lz4_block_compress,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)sizeof(LzEncLds));
            if (e != hipSuccess) return e;
            attr = true;
        }
        const u64 nb = (u64)n * nbpc;
        if (nb > 0x7FFFFFFFull) return hipErrorInvalidValue;
        hipLaunchKernelGGL(lz4_block_compress, dim3((u32)nb), dim3(64), sizeof(LzEncLds), s, d_chunks,
                           n, D, B, nbpc, bound, t);
    }
    hipLaunchKernelGGL(lz4_frame_finalize, dim3(n), dim3(256), 0, s, d_chunks, n, D, B, nbpc, bound,
                       (u64*)d_out_len, d_status);
    hipLaunchKernelGGL(lz4_content_xxh32, dim3((n + 15) / 16), dim3(64), 0, s, d_chunks, n, D,
                       (const u64*)d_out_len, (const i32*)d_status, t);
    return hipGetLastError();
}

}  // namespace zcg
