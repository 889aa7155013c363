// zcg_raw.hip — RawCompression (src/compression/raw.rs:13-24) on gfx950.
//
// Decode = read_exact of N*size bytes (chunk.rs:112-113) + the element
// transform of read_data (byte reversal for '>' types, bool != 0).
// Encode = write_data's serialisation (chunk.rs:118-140): the same map.
//
// Pure HBM copy: each 256-thread workgroup moves one 4 KiB tile of one
// chunk, one 16-B load and one 16-B store per lane (a grid past the launch
// limit strides over the tiles), so the kernel is bound by the HBM copy
// roofline.  Algorithmic bytes
// per chunk: 2*N*size (read once, write once).
#include "zcg_common.h"

namespace zcg {

constexpr int RAW_THREADS = 256;
// one 16-byte vector per thread (4 KiB tiles): measured 2 650 / 2 685 / 2 865
// GiB/s at 4 / 2 / 1 vectors per thread (1 GiB batch); 128/512-thread
// workgroups and non-temporal stores are within noise of this
#ifndef ZCG_RAW_VPT
#define ZCG_RAW_VPT 1
#endif
constexpr int RAW_VEC_PER_THREAD = ZCG_RAW_VPT;
constexpr u64 RAW_TILE = (u64)RAW_THREADS * RAW_VEC_PER_THREAD * 16;  // 4 KiB

__device__ __forceinline__ void raw_tile(const zcg_chunk* __restrict__ chunks, u32 n, u64 nbytes,
                                         u64 tiles_per_chunk, DType t, int encode,
                                         i32* __restrict__ status, u64* __restrict__ out_len, u64 gtile) {
    const u32 c = (u32)(gtile / tiles_per_chunk);
    const u64 tile = gtile - (u64)c * tiles_per_chunk;
    if (c >= n) return;
    const zcg_chunk ch = chunks[c];
    // The chunk's verdict depends only on its descriptor: every tile computes
    // it, tile 0 publishes it.
    int st = ZCG_OK;
    if (!encode) {
        if (ch.src_len < nbytes) st = ZCG_ERR_UNEXPECTED_EOF;  // read_exact short
    } else {
        if (ch.src_len < nbytes) st = ZCG_ERR_INVALID_DATA;  // element count (chunk.rs:309-318)
        else if (ch.dst_cap < nbytes) st = ZCG_ERR_OUTPUT_TOO_SMALL;
    }
    if (tile == 0 && threadIdx.x == 0) {
        status[c] = st;
        if (out_len) out_len[c] = st == ZCG_OK ? nbytes : 0;
    }
    if (st != ZCG_OK) return;

    const u8* __restrict__ src = (const u8*)ch.src;
    u8* __restrict__ dst = (u8*)ch.dst;
    const u64 base = tile * RAW_TILE;
    const u64 end = (base + RAW_TILE < nbytes) ? base + RAW_TILE : nbytes;
    const bool aligned = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0;
    if (aligned && end - base == RAW_TILE) {
        u32x4 v[RAW_VEC_PER_THREAD];
#pragma unroll
        for (int k = 0; k < RAW_VEC_PER_THREAD; k++)
            v[k] = *(const u32x4*)(src + base + ((u64)k * RAW_THREADS + threadIdx.x) * 16);
#pragma unroll
        for (int k = 0; k < RAW_VEC_PER_THREAD; k++)
            *(u32x4*)(dst + base + ((u64)k * RAW_THREADS + threadIdx.x) * 16) = transform16(v[k], t);
        return;
    }
    // Edge tile or unaligned pointers: 16-byte pieces where they fit (they
    // start at multiples of 16 from the chunk start, hence element-aligned),
    // then single bytes.
    for (u64 p = base + (u64)threadIdx.x * 16; p < end; p += (u64)RAW_THREADS * 16) {
        if (p + 16 <= end) {
            st16(dst + p, transform16(ld16(src + p), t));
        } else {
            for (u64 q = p; q < end; q++) dst[swap_pos(q, t)] = norm_byte(src[q], t);
        }
    }
}

// one tile per workgroup; a grid larger than the launch limit strides
__global__ __launch_bounds__(RAW_THREADS) void raw_kernel(const zcg_chunk* __restrict__ chunks,
                                                          u32 n, u64 nbytes, u64 tiles_per_chunk,
                                                          DType t, int encode,
                                                          i32* __restrict__ status,
                                                          u64* __restrict__ out_len, u64 ntiles) {
    for (u64 g = blockIdx.x; g < ntiles; g += gridDim.x)
        raw_tile(chunks, n, nbytes, tiles_per_chunk, t, encode, status, out_len, g);
}

hipError_t launch_raw(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n, int32_t* d_status,
                      uint64_t* d_out_len, int encode, hipStream_t s) {
    const DType t = make_dtype(a->dtype);
    const u64 nbytes = a->chunk_num_elements * (u64)t.es;
    const u64 tiles = nbytes ? (nbytes + RAW_TILE - 1) / RAW_TILE : 1;
    const u64 grid = tiles * n;
    if (grid == 0) return hipSuccess;
    const u32 blocks = (u32)(grid < (1ull << 30) ? grid : (1ull << 30));
    hipLaunchKernelGGL(raw_kernel, dim3(blocks), dim3(RAW_THREADS), 0, s, d_chunks, n,
                       nbytes, tiles, t, encode, d_status, d_out_len, grid);
    return hipGetLastError();
}

const char* cfg_raw() { return "raw:VPT=" ZCG_STR(ZCG_RAW_VPT); }

}  // namespace zcg
