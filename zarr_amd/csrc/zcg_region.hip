// zcg_region.hip — region assembly on the device:
// ZarrNdarrayReader::read_ndarray / read_ndarray_into_with_buffer
// (src/ndarray.rs:153-268) for chunks that the batch decoders already left in
// HBM.
//
// Reference semantics kept: the chunks visited are bounded_coord_iter's grid
// range (ndarray.rs:410-432); each visited chunk covers its full nominal
// bounds, overhang included (get_chunk_bounds, ndarray.rs:434-446), so an
// element at global position g comes from chunk g / chunk_shape, at the
// chunk-local position g % chunk_shape in the chunk's memory order
// (as_ndarray, ndarray.rs:453-476: ColumnMajor = dim 0 fastest); elements no
// visited chunk covers keep Array::from_elem's fill value in read_ndarray
// (ndarray.rs:164-171) and are left untouched by read_ndarray_into.
//
// The kernel is HBM-bound byte movement (2 bytes of traffic per output byte):
// the box is walked in the chunks' memory order, 16 bytes per thread, so
// reads from a chunk row and writes to an output row with unit stride are
// both coalesced 16-byte accesses; a 16-byte piece that crosses a row or a
// chunk boundary is copied in per-element runs.  Tile starts are decomposed
// once per workgroup (scalar), threads add their offset with carries.
#include <hip/hip_runtime.h>

#include "zcg_common.h"

namespace zcg {


namespace {

constexpr u32 RG_T = 256;

struct Pos {
    u32 x[ZCG_MAX_DIMS];
};

// where element x is read from (nullptr: no visited chunk), and how many
// elements from it stay in one chunk row and one box row
__device__ __forceinline__ const u8* region_src(const RegionArgs& a, const Pos& p,
                                                const u8* const* __restrict__ table, u32* run) {
    u64 ti = 0, wi = 0;
    bool ok = true;
    u32 w0 = 0;
    for (u32 k = 0; k < a.nd; k++) {
        const u32 r = a.orr[k] + p.x[k];
        const u32 q = r / a.cs[k];
        const u32 w = r - q * a.cs[k];
        if (k == 0) w0 = w;
        ok &= (u64)q < a.gn[k];
        ti += (u64)q * a.tstr[k];
        wi += (u64)w * a.cstr[k];
    }
    const u32 r1 = a.bs[0] - p.x[0], r2 = a.cs[0] - w0;
    *run = r1 < r2 ? r1 : r2;
    if (!ok) return nullptr;
    const u8* base = table[ti];
    return base ? base + wi * a.es : nullptr;
}

__device__ __forceinline__ i64 region_dst(const RegionArgs& a, const Pos& p) {
    i64 o = 0;
    for (u32 k = 0; k < a.nd; k++) o += (i64)p.x[k] * a.ostr[k];
    return o;
}

// advance p by d elements along the fast-first order (carries)
__device__ __forceinline__ void region_advance(const RegionArgs& a, Pos& p, u32 d) {
    u32 c = d;
    for (u32 k = 0; k < a.nd && c; k++) {
        const u64 v = (u64)p.x[k] + c;
        if (v < a.bs[k]) { p.x[k] = (u32)v; c = 0; break; }
        const u64 q = v / a.bs[k];
        p.x[k] = (u32)(v - q * a.bs[k]);
        c = (u32)q;
    }
}

__device__ __forceinline__ void copy_elem(u8* dst, const u8* src, u32 es) {
    switch (es) {
    case 1: *dst = *src; break;
    case 2: *(u16*)dst = *(const u16*)src; break;
    case 4: *(u32*)dst = *(const u32*)src; break;
    default: *(u64*)dst = *(const u64*)src; break;
    }
}
__device__ __forceinline__ void fill_elem(u8* dst, u64 v, u32 es) {
    switch (es) {
    case 1: *dst = (u8)v; break;
    case 2: *(u16*)dst = (u16)v; break;
    case 4: *(u32*)dst = (u32)v; break;
    default: *(u64*)dst = v; break;
    }
}

__global__ __launch_bounds__(RG_T) void region_kernel(RegionArgs a, const u8* const* __restrict__ table,
                                                      u8* __restrict__ out) {
    const u64 tile_elems = (u64)RG_T * a.V;
    const u64 ntiles = (a.total + tile_elems - 1) / tile_elems;
    u64 fv = a.fillv;
    if (a.es == 1) fv = (fv & 0xFF) * 0x0101010101010101ull;
    else if (a.es == 2) fv = (fv & 0xFFFF) * 0x0001000100010001ull;
    else if (a.es == 4) fv = (fv & 0xFFFFFFFFull) * 0x0000000100000001ull;
    const u32x4 fill16 = {(u32)fv, (u32)(fv >> 32), (u32)fv, (u32)(fv >> 32)};
    for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        // decompose the tile start (wave-uniform, scalar)
        Pos p;
        u64 e = tile * tile_elems;
        for (u32 k = 0; k < ZCG_MAX_DIMS; k++) {
            if (k < a.nd) {
                const u64 q = e / a.bs[k];
                p.x[k] = (u32)(e - q * a.bs[k]);
                e = q;
            } else {
                p.x[k] = 0;
            }
        }
        const u64 e0 = tile * tile_elems + (u64)threadIdx.x * a.V;
        if (e0 >= a.total) continue;
        region_advance(a, p, threadIdx.x * a.V);
        u32 rem = (u32)((a.total - e0) < a.V ? (a.total - e0) : a.V);
        u32 run;
        const u8* src = region_src(a, p, table, &run);
        if (rem == a.V && run >= a.V && a.ostr[0] == 1) {  // one 16-byte piece, both sides contiguous
            u8* d = out + region_dst(a, p) * (i64)a.es;
            if (src) st16(d, ld16(src));
            else if (a.fill) st16(d, fill16);
            continue;
        }
        while (rem) {  // runs inside one chunk row and one box row
            const u32 k = run < rem ? run : rem;
            u8* d = out + region_dst(a, p) * (i64)a.es;
            const i64 ds = a.ostr[0] * (i64)a.es;
            for (u32 j = 0; j < k; j++) {
                if (src) copy_elem(d + j * ds, src + (u64)j * a.es, a.es);
                else if (a.fill) fill_elem(d + j * ds, fv, a.es);
            }
            rem -= k;
            if (!rem) break;
            region_advance(a, p, k);
            src = region_src(a, p, table, &run);
        }
    }
}

}  // namespace

hipError_t launch_region(const RegionArgs& a, const void* const* d_table, void* d_out, hipStream_t s) {
    if (a.total == 0) return hipSuccess;
    const u64 tiles = (a.total + (u64)RG_T * a.V - 1) / ((u64)RG_T * a.V);
    const u32 grid = (u32)(tiles < 262144 ? tiles : 262144);
    hipLaunchKernelGGL(region_kernel, dim3(grid), dim3(RG_T), 0, s, a, (const u8* const*)d_table, (u8*)d_out);
    return hipGetLastError();
}

}  // namespace zcg
