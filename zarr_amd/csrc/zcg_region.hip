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
// pieces per lane in flight per work unit (A/B: 1 / 2 / 4 / 8 / 16 -> 1 753 /
// 2 249 / 2 385 / 1 852 / 1 254 GiB/s of box on the bench leg)
#ifndef ZCG_RG_U
#define ZCG_RG_U 4
#endif

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
            if (a.dir) { if (src) st16((u8*)src, ld16(d)); }
            else if (src) st16(d, ld16(src));
            else if (a.fill) st16(d, fill16);
            continue;
        }
        while (rem) {  // runs inside one chunk row and one box row
            const u32 k = run < rem ? run : rem;
            u8* d = out + region_dst(a, p) * (i64)a.es;
            const i64 ds = a.ostr[0] * (i64)a.es;
            for (u32 j = 0; j < k; j++) {
                if (a.dir) { if (src) copy_elem((u8*)src + (u64)j * a.es, d + j * ds, a.es); }
                else if (src) copy_elem(d + j * ds, src + (u64)j * a.es, a.es);
                else if (a.fill) fill_elem(d + j * ds, fv, a.es);
            }
            rem -= k;
            if (!rem) break;
            region_advance(a, p, k);
            src = region_src(a, p, table, &run);
        }
    }
}

// Long box rows (the common case: the fast dimension spans many 16-byte
// pieces): one wave per box row.  The row's coordinates, chunk-table and
// chunk-offset contributions of the slow dimensions are scalar, computed once
// per row; lanes stream the row 16 bytes each.
__global__ __launch_bounds__(RG_T) void region_rows_kernel(RegionArgs a, u64 nrows,
                                                           const u8* const* __restrict__ table,
                                                           u8* __restrict__ out) {
    const u32 lane = threadIdx.x & 63;
    const u64 wid = ((u64)blockIdx.x * RG_T + threadIdx.x) >> 6;
    const u64 nwaves = ((u64)gridDim.x * RG_T) >> 6;
    u64 fv = a.fillv;
    if (a.es == 1) fv = (fv & 0xFF) * 0x0101010101010101ull;
    else if (a.es == 2) fv = (fv & 0xFFFF) * 0x0001000100010001ull;
    else if (a.es == 4) fv = (fv & 0xFFFFFFFFull) * 0x0000000100000001ull;
    const u32x4 fill16 = {(u32)fv, (u32)(fv >> 32), (u32)fv, (u32)(fv >> 32)};
    const u32 V = a.V, bs0 = a.bs[0], cs0 = a.cs[0], orr0 = a.orr[0];
    const i64 es = a.es;
    // work unit = (row, piece of U*64*V elements of it): many short units
    // keep more loads in flight per CU than one long walk per row
    constexpr u32 U = ZCG_RG_U;
    const u32 span = U * 64 * V;
    const u32 ppr = (bs0 + span - 1) / span;
    const u64 nunits = nrows * ppr;
    for (u64 unit = ru64(wid); unit < nunits; unit += nwaves) {
        const u64 row = unit / ppr;
        const u32 piece = (u32)(unit - row * ppr);
        // slow-dimension coordinates of this row (scalar)
        u64 e = row, ti = 0, wi = 0;
        i64 drow = 0;
        bool ok = true;
        for (u32 k = 1; k < ZCG_MAX_DIMS; k++) {
            if (k >= a.nd) break;
            const u64 qd = e / a.bs[k];
            const u32 x = (u32)(e - qd * a.bs[k]);
            e = qd;
            const u32 r = a.orr[k] + x;
            const u32 q = r / a.cs[k];
            ok &= (u64)q < a.gn[k];
            ti += (u64)q * a.tstr[k];
            wi += (u64)(r - q * a.cs[k]) * a.cstr[k];
            drow += (i64)x * a.ostr[k];
        }
        u8* drow_p = out + drow * es;
        // U pieces per lane in flight: loads first, then stores
        const u32 xend = (piece + 1) * span;
        for (u32 xb = piece * span + lane * V; xb < bs0 && xb < xend; xb += span) {
            u32x4 v[U];
            u8* dp[U];
            u32 mode[U];  // 0 skip, 1 load+store, 2 fill, 3 element runs
#pragma unroll
            for (u32 u = 0; u < U; u++) {
                const u32 x0 = xb + u * 64 * V;
                mode[u] = 0;
                dp[u] = drow_p + (i64)x0 * a.ostr[0] * es;
                if (x0 >= bs0) continue;
                const u32 r = orr0 + x0;
                const u32 q = r / cs0;
                const u32 w0 = r - q * cs0;
                const bool here = ok && (u64)q < a.gn[0];
                const u8* base = here ? table[ti + (u64)q * a.tstr[0]] : nullptr;
                if (!(bs0 - x0 >= V && w0 + V <= cs0 && a.ostr[0] == 1)) { mode[u] = 3; continue; }
                if (a.dir) {  // write_ndarray: box -> chunk
                    if (base) { v[u] = ld16(dp[u]); dp[u] = (u8*)base + (wi + w0) * (u64)es; mode[u] = 1; }
                } else if (base) { v[u] = ld16(base + (wi + w0) * (u64)es); mode[u] = 1; }
                else if (a.fill) { v[u] = fill16; mode[u] = 2; }
            }
#pragma unroll
            for (u32 u = 0; u < U; u++)
                if (mode[u] == 1 || mode[u] == 2) st16(dp[u], v[u]);
#pragma unroll
            for (u32 u = 0; u < U; u++) {
                if (mode[u] != 3) continue;
                const u32 x0 = xb + u * 64 * V;
                const u32 rem = bs0 - x0 < V ? bs0 - x0 : V;
                // the piece crosses a chunk boundary or ends the row: per element
                for (u32 j = 0; j < rem; j++) {
                    const u32 rj = orr0 + x0 + j;
                    const u32 qj = rj / cs0;
                    const bool hj = ok && (u64)qj < a.gn[0];
                    const u8* bj = hj ? table[ti + (u64)qj * a.tstr[0]] : nullptr;
                    u8* dj = drow_p + (i64)(x0 + j) * a.ostr[0] * es;
                    if (a.dir) { if (bj) copy_elem((u8*)bj + (wi + (rj - qj * cs0)) * (u64)es, dj, a.es); }
                    else if (bj) copy_elem(dj, bj + (wi + (rj - qj * cs0)) * (u64)es, a.es);
                    else if (a.fill) fill_elem(dj, fv, a.es);
                }
            }
        }
    }
}

}  // namespace

hipError_t launch_region(const RegionArgs& a, const void* const* d_table, void* d_out, hipStream_t s) {
    if (a.total == 0) return hipSuccess;
    if (a.bs[0] >= 32u * a.V) {  // long rows: a wave per row
        const u64 nrows = a.total / a.bs[0];
        const u64 span = (u64)ZCG_RG_U * 64 * a.V;
        const u64 units = nrows * ((a.bs[0] + span - 1) / span);
        const u64 wgs = (units + 3) / 4;
        const u32 grid = (u32)(wgs < (1u << 20) ? wgs : (1u << 20));
        hipLaunchKernelGGL(region_rows_kernel, dim3(grid), dim3(RG_T), 0, s, a, nrows, (const u8* const*)d_table,
                           (u8*)d_out);
        return hipGetLastError();
    }
    const u64 tiles = (a.total + (u64)RG_T * a.V - 1) / ((u64)RG_T * a.V);
    const u32 grid = (u32)(tiles < 262144 ? tiles : 262144);
    hipLaunchKernelGGL(region_kernel, dim3(grid), dim3(RG_T), 0, s, a, (const u8* const*)d_table, (u8*)d_out);
    return hipGetLastError();
}

const char* cfg_region() { return "region:U=" ZCG_STR(ZCG_RG_U); }

}  // namespace zcg
