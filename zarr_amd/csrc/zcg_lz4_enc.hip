// zcg_lz4_enc.hip — LZ4 frame encoder (write_chunk for CompressionType::Lz4),
// byte-identical to the reference's.
//
// Reference: lz.rs:81-92 builds lz4-rs's encoder with the effective block size
// (lz.rs:55-65), BlockMode::Independent, level 0, content checksum on, no
// content size, no block checksum; LZ4F (liblz4 1.9.3, lz4-sys) then writes
//   magic 04 22 4D 18 | FLG 0x64 | BD (id << 4) | HC = XXH32(FLG,BD) >> 8
//   blocks: u32 LE size (bit 31 = stored) + data; an end mark 0; XXH32(content).
// Each block is LZ4F_makeBlock -> LZ4F_compressBlock ->
// LZ4_compress_fast_extState_fastReset(acceleration 1) on a cleared table with
// dstCapacity = srcSize - 1, and is stored raw when that returns 0.  The
// block compressor is a deterministic serial algorithm; tests/hostcore/
// lz4_fast_ref.c restates it serially (pinned byte for byte to liblz4's
// LZ4_compress_fast by tests/test_hostcore.py) and this file restates the
// same steps with a wave-parallel search, so the GPU frames equal lz4-rs's
// frames byte for byte (tests/test_gpu_encode.py compares them with the
// oracle's liblz4 LZ4F frames).
//
// Kernels (stream-ordered):
//   1. lz4_block_exact: one wave per block, the hash table (16 KiB) in LDS.
//      The match search of LZ4_compress_generic visits positions with
//      data-independent steps (1 for the first 65 attempts, then growing by
//      the skip trigger) and, per attempt, reads the table at the position's
//      hash, writes the position there and compares 4 bytes.  The wave runs 64
//      attempts at once: lane j takes attempt k0 + j (its position from a
//      prefix sum of the steps), reads its candidate from the table, and the
//      first lane whose candidate matches ends the search.  A lane's candidate
//      is the table's value only if no earlier lane of the batch writes the
//      same hash; the lanes tag their table entries with their lane id and
//      read them back, so the batch is cut at the first lane that shares a
//      hash with an earlier lane (it starts the next batch).  The table is
//      then left exactly as the serial attempts leave it.  Catch-up, match
//      length (LZ4_count), the output-budget checks, the table fill at ip-2
//      and the next-position test are the serial code's, run wave-uniform.
//      Literals are read with the dtype transform (write_data's byte order,
//      chunk.rs:118-140).  Block k is written at its upper-bound slot
//      7 + k*(B+4) of dst.
//   2. lz4_frame_finalize: one workgroup per chunk writes the frame header,
//      compacts the blocks to their final offsets (tile copies, dst <= src),
//      writes the end mark and the output length.
//   3. lz4_content_xxh32: 4 lanes per chunk (one XXH32 accumulator each)
//      hash the serialised content and write the content checksum.
#include "zcg_common.h"

namespace zcg {

constexpr u32 LE_MFLIMIT = 12;      // MFLIMIT
constexpr u32 LE_LASTLIT = 5;       // LASTLITERALS
constexpr u32 LE_MINLEN = 13;       // LZ4_minLength: shorter blocks are literals only (-> stored)
constexpr u32 LE_HDR = 7;           // frame header bytes
constexpr u32 LE_64KLIMIT = 65536 + LE_MFLIMIT - 1;  // LZ4_64Klimit: byU16 table below it

// Logical (serialised) byte x of the chunk: the stream holds elements in the
// array's byte order; bool as 0/1.
__device__ __forceinline__ u8 src_byte(const u8* src, u64 x, const DType& t) {
    return norm_byte(src[swap_pos(x, t)], t);
}

typedef __attribute__((address_space(1))) u32 le_gu32_ua __attribute__((aligned(1)));

// The serialised chunk as the block compressor reads it (plain loads for
// little-endian non-bool types, the transform byte by byte otherwise).
struct LeSrc {
    const u8* src;
    DType t;
    bool plain;
    __device__ __forceinline__ u8 b1(u64 x) const {
        return plain ? ((const gu8*)src)[x] : src_byte(src, x, t);
    }
    __device__ __forceinline__ u32 b4(u64 x) const {
        if (plain) return *(const le_gu32_ua*)((const gu8*)src + x);
        return (u32)b1(x) | ((u32)b1(x + 1) << 8) | ((u32)b1(x + 2) << 16) | ((u32)b1(x + 3) << 24);
    }
};

__device__ __forceinline__ void le_wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ u32 le_incl_scan(u32 v) {
    const u32 lane = (u32)lane_id();
#pragma unroll
    for (u32 d = 1; d < 64; d <<= 1) {
        const u32 x = (u32)__shfl_up((int)v, d, 64);
        v += lane >= d ? x : 0u;
    }
    return v;
}

__device__ __forceinline__ u32 le_wave_min(u32 v) {
#pragma unroll
    for (u32 d = 1; d < 64; d <<= 1) {
        const u32 x = (u32)__shfl_xor((int)v, d, 64);
        v = x < v ? x : v;
    }
    return v;
}

// LZ4_hashPosition: byU16 (block < LZ4_64Klimit): hash4, 13 bits;
// byU32: hash5 of the 5 bytes at p, 12 bits (LZ4_hash5 on a 64-bit LE host)
template <bool U32>
__device__ __forceinline__ u32 le_hash(const LeSrc& v, u64 p) {
    if (!U32) return (v.b4(p) * 2654435761u) >> 19;
    const u64 q = (u64)v.b4(p) | ((u64)v.b1(p + 4) << 32);
    return (u32)(((q << 24) * 889523592379ull) >> 52);
}

// One block of S bytes starting at logical b0, compressed into out[0, cap)
// as LZ4_compress_generic (limitedOutput, noDict, acceleration 1); returns the
// compressed size, or 0 when it does not fit (the caller stores the block).
// T: the wave's 16 KiB table (u16 entries for byU16, u32 for byU32).
template <bool U32>
__device__ u32 le_block(const LeSrc& v, u64 b0, u32 S, u8* out, u32 cap, lu32* T32) {
    const u32 lane = (u32)lane_id();
    __attribute__((address_space(3))) u16* T16 = (__attribute__((address_space(3))) u16*)T32;
    auto tget = [&](u32 h) -> u32 { return U32 ? T32[h] : (u32)T16[h]; };
    auto tput = [&](u32 h, u32 x) { if (U32) T32[h] = x; else T16[h] = (u16)x; };
    auto hp = [&](u32 p) -> u32 { return le_hash<U32>(v, b0 + p); };
    auto r4 = [&](u32 p) -> u32 { return v.b4(b0 + p); };
    // write n literal bytes [a, a + n) at out[o..)
    auto put_lits = [&](u32 o, u32 a, u32 n) {
        for (u32 i = lane; i < n; i += 64) out[o + i] = v.b1(b0 + a + i);
    };
    // a length field's extra bytes (value >= 15): (x-15)/255 bytes of 255, then (x-15)%255
    auto put_len = [&](u32 o, u32 x) -> u32 {
        const u32 r = x - 15, nb = r / 255;
        for (u32 i = lane; i < nb; i += 64) out[o + i] = 255;
        if (lane == 0) out[o + nb] = (u8)(r % 255);
        return nb + 1;
    };
    u32 op = 0, anchor = 0;
    if (S >= LE_MINLEN) {
        const u32 mfl1 = S - LE_MFLIMIT + 1;  // mflimitPlusOne
        const u32 mlim = S - LE_LASTLIT;      // matchlimit
        // the table is clear (index 0 everywhere): putPosition(0) changes nothing
        u32 ip = 1;
        for (;;) {
            // ---- match search from ip: 64 attempts per step ------------------
            u32 s0 = ip, k0 = 0, mpos = 0, mref = 0;
            bool found = false;
            for (;;) {
                const u32 k = k0 + lane;
                const u32 st = k == 0 ? 1u : (63u + k) >> 6;  // the step after attempt k
                const u32 inc = le_incl_scan(st);
                const u32 pos = s0 + inc - st, nxt = s0 + inc;
                const bool valid = nxt <= mfl1;  // (a prefix of the lanes)
                const u64 vm = __ballot(valid);
                if (!vm) break;
                const u32 V = (u32)__popcll(vm);
                u32 h = 0, old = 0;
                if (valid) { h = hp(pos); old = tget(h); }
                le_wsync();
                if (valid) tput(h, lane);  // tag: who writes this hash last in the batch
                le_wsync();
                const u32 rd = valid ? tget(h) : lane;
                const bool dup = valid && rd != lane;
                // smallest lane of any hash shared inside the batch
                const u32 g = le_wave_min(dup ? (rd < lane ? rd : lane) : 64u);
                const u32 P = g + 1 < V ? g + 1 : V;  // lanes [0, P) see the serial candidates
                bool ok = false;
                if (lane < P && (!U32 || old + 65535u >= pos)) ok = r4(old) == r4(pos);
                const u64 om = __ballot(ok);
                const u32 w = om ? (u32)__builtin_ctzll(om) : 64u;
                const u32 m = w < 64 ? w : P - 1;  // last attempt taken
                // leave the table as attempts 0..m leave it (lanes <= m hash apart)
                le_wsync();
                if (valid && lane > m) tput(h, old);
                le_wsync();
                if (valid && lane <= m) tput(h, pos);
                le_wsync();
                if (w < 64) {
                    mpos = (u32)__builtin_amdgcn_readlane((int)pos, (int)w);
                    mref = (u32)__builtin_amdgcn_readlane((int)old, (int)w);
                    found = true;
                    break;
                }
                if (P == V && V < 64) break;  // attempt V ends the search: last literals
                s0 = (u32)__builtin_amdgcn_readlane((int)nxt, (int)(P - 1));
                k0 += P;
            }
            if (!found) break;
            // ---- catch up --------------------------------------------------------
            u32 mip = mpos, mm = mref;
            for (;;) {
                const u32 lim = (mip - anchor) < mm ? (mip - anchor) : mm;
                const bool eq = lane < lim && v.b1(b0 + mip - 1 - lane) == v.b1(b0 + mm - 1 - lane);
                const u64 ne = __ballot(!eq);
                const u32 c = ne ? (u32)__builtin_ctzll(ne) : 64u;
                mip -= c;
                mm -= c;
                if (c < 64) break;
            }
            // ---- literals --------------------------------------------------------
            const u32 lit = mip - anchor;
            u32 tpos = op;
            op++;
            if ((u64)op + lit + (2 + 1 + LE_LASTLIT) + lit / 255 > cap) return 0;
            if (lit >= 15) op += put_len(op, lit);
            put_lits(op, anchor, lit);
            op += lit;
            u32 tok = (lit < 15 ? lit : 15u) << 4;
            for (;;) {  // _next_match
                const u32 off = mip - mm;
                if (lane == 0) { out[op] = (u8)off; out[op + 1] = (u8)(off >> 8); }
                op += 2;
                // LZ4_count(ip + 4, match + 4, matchlimit), 256 bytes per step
                u32 mc = 0;
                for (;;) {
                    const u32 a = mip + 4 + mc + 4 * lane, bq = mm + 4 + mc + 4 * lane;
                    u32 x;
                    if (a + 4 <= mlim) {
                        x = r4(a) ^ r4(bq);
                    } else {
                        x = 0;
                        for (u32 j = 0; j < 4; j++) {
                            const bool d = a + j >= mlim || v.b1(b0 + a + j) != v.b1(b0 + bq + j);
                            x |= d ? (0xFFu << (8 * j)) : 0u;
                        }
                    }
                    const u64 dm = __ballot(x != 0);
                    if (!dm) { mc += 256; continue; }
                    const u32 f = (u32)__builtin_ctzll(dm);
                    const u32 xf = (u32)__builtin_amdgcn_readlane((int)x, (int)f);
                    mc += 4 * f + ((u32)__builtin_ctz(xf) >> 3);
                    break;
                }
                mip += mc + 4;
                if ((u64)op + (1 + LE_LASTLIT) + (mc + 240) / 255 > cap) return 0;
                if (mc >= 15) {
                    tok |= 15;
                    op += put_len(op, mc);
                } else {
                    tok |= mc;
                }
                if (lane == 0) out[tpos] = (u8)tok;
                anchor = mip;
                if (mip >= mfl1) break;
                // fill table at ip - 2, then test the next position
                const u32 h2 = hp(mip - 2);
                le_wsync();
                tput(h2, mip - 2);
                le_wsync();
                const u32 h = hp(mip);
                const u32 cand = tget(h);
                le_wsync();
                tput(h, mip);
                le_wsync();
                if ((!U32 || cand + 65535u >= mip) && r4(cand) == r4(mip)) {
                    tpos = op;
                    op++;
                    tok = 0;
                    mm = cand;
                    continue;
                }
                break;
            }
            if (anchor >= mfl1) break;
            ip = mip + 1;
        }
    }
    // ---- last literals -----------------------------------------------------------
    const u32 last = S - anchor;
    if ((u64)op + last + 1 + (last + 240) / 255 > cap) return 0;
    if (lane == 0) out[op] = (u8)((last < 15 ? last : 15u) << 4);
    op++;
    if (last >= 15) op += put_len(op, last);
    put_lits(op, anchor, last);
    return op + last;
}

__global__ __launch_bounds__(64) void lz4_block_exact(const zcg_chunk* __restrict__ chunks, u32 n, u64 D, u32 B,
                                                      u32 nbpc, u64 bound, DType t) {
    __shared__ __attribute__((aligned(16))) u32 T[4096];  // 16 KiB: 8192 u16 or 4096 u32 entries
    const u32 lane = threadIdx.x;
    const u32 c = blockIdx.x / nbpc, k = blockIdx.x % nbpc;
    if (c >= n) return;
    const zcg_chunk ch = chunks[c];
    if (ch.dst_cap < bound || ch.src_len < D) return;  // finalize reports the status
    const u64 b0 = (u64)k * B;
    const u32 S = (u32)((D - b0) < B ? (D - b0) : B);
    u8* hdr = (u8*)ch.dst + LE_HDR + (u64)k * (B + 4);
    u8* out = hdr + 4;
    const LeSrc v{(const u8*)ch.src, t, !t.swap && !t.isbool};
    for (u32 i = lane; i < 1024; i += 64) ((__attribute__((address_space(3))) u32x4*)T)[i] = u32x4{0u, 0u, 0u, 0u};
    le_wsync();
    const u32 cap = S - 1;
    const u32 cs = S >= LE_64KLIMIT ? le_block<true>(v, b0, S, out, cap, (lu32*)T)
                                    : le_block<false>(v, b0, S, out, cap, (lu32*)T);
    const bool stored = cs == 0;
    if (stored)  // LZ4F_makeBlock: the block raw
        for (u32 q = lane; q < S; q += 64) out[q] = v.b1(b0 + q);
    if (lane == 0) {
        const u32 w = stored ? (S | 0x80000000u) : cs;
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

uint64_t lz4_encode_ws_bytes(const zcg_array* a, uint32_t n) {
    (void)a;
    (void)n;
    return 0;  // the block compressor's table lives in LDS
}

hipError_t launch_lz4_encode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                             uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                             hipStream_t s) {
    (void)ws;
    (void)ws_bytes;
    if (n == 0) return hipSuccess;
    const DType t = make_dtype(a->dtype);
    const u64 D = a->chunk_num_elements * (u64)t.es;
    const u32 B = (u32)zcg_effective_lz4_block_size(a->compression.lz4_block_size);
    const u32 nbpc = (u32)((D + B - 1) / B);
    const u64 bound = zcg_encode_bound(&a->compression, D);
    if (nbpc) {
        if (nbpc > 4096) return hipErrorInvalidValue;
        const u64 nb = (u64)n * nbpc;
        if (nb > 0x7FFFFFFFull) return hipErrorInvalidValue;
        hipLaunchKernelGGL(lz4_block_exact, dim3((u32)nb), dim3(64), 0, s, d_chunks, n, D, B, nbpc, bound, t);
    }
    hipLaunchKernelGGL(lz4_frame_finalize, dim3(n), dim3(256), 0, s, d_chunks, n, D, B, nbpc, bound,
                       (u64*)d_out_len, d_status);
    hipLaunchKernelGGL(lz4_content_xxh32, dim3((n + 15) / 16), dim3(64), 0, s, d_chunks, n, D,
                       (const u64*)d_out_len, (const i32*)d_status, t);
    return hipGetLastError();
}

}  // namespace zcg
