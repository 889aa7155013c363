// Calibration of the rocprofv3 traffic counters (FETCH_SIZE, WRITE_SIZE and
// the TCC_EA0 request counters) on gfx950 for the access patterns the bench
// legs actually issue, against KNOWN byte counts.  Test infrastructure only:
// tools/pmc_calib.sh profiles it, tools/pmc_calib.py reduces the passes to
// profiles/r05_pmc_calibration.json, and tools/pmc_traffic.py applies the
// measured factors per kernel.
//
// Every pattern touches each unit of a buffer exactly once, in a scattered
// order (unit u = (t * ODD) mod units, a bijection), so the footprint is
// known and, at 1 GiB (4x the 256 MiB Infinity Cache, 32x the summed L2),
// no unit is re-read from cache.  Before each measured kernel a 512 MiB
// streaming write evicts the previous pattern's lines.  Each pattern is its
// own kernel instantiation (calib_k<M>) so a pass maps dispatches to
// patterns by name.
//
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/pmc_calib tools/probe/pmc_calib.hip
//   run:   pmc_calib [log2 buffer bytes, default 30]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;

// pattern table: kind 0 gather read, 1 streaming read, 2 scattered write,
// 3 streaming write
struct Pat {
    const char* name;
    int kind;
    u32 unit;    // bytes per unit (one access per unit)
    u32 width;   // bytes read / written per access
    u32 off;     // offset of the access in its unit
    u32 group;   // lanes sharing one unit (write: 4 lanes x 16 B = 64 B)
    const char* what;
};
static const Pat PATS[] = {
    {"stream16_read", 1, 16, 16, 0, 1, "coalesced 16 B/lane streaming read (control: the guide's x2 case)"},
    {"gather1_line128", 0, 128, 1, 0, 1, "1-byte read, one per 128 B line, scattered"},
    {"gather1_sector64", 0, 64, 1, 0, 1, "1-byte read, one per 64 B sector, scattered"},
    {"gather1_sector32", 0, 32, 1, 0, 1, "1-byte read, one per 32 B sector, scattered"},
    {"gather4_line128", 0, 128, 4, 0, 1, "4-byte read, one per 128 B line, scattered"},
    {"gather4_all", 0, 4, 4, 0, 1, "4-byte read of every dword once, scattered (bzip2 list-ranking gathers)"},
    {"gather16_line128", 0, 128, 16, 0, 1, "16-byte aligned read, one per 128 B line, scattered"},
    {"gather16_cross128", 0, 128, 16, 120, 1, "16-byte read straddling two 128 B lines (8 B each), scattered (LZ4/inflate far sources)"},
    {"gather16_all", 0, 16, 16, 0, 1, "16-byte read of every 16 B piece once, scattered"},
    {"gather1_all", 0, 1, 1, 0, 1, "1-byte read of every byte once, scattered"},
    {"stream16_write", 3, 16, 16, 0, 1, "coalesced 16 B/lane streaming write (control: the guide's exact case)"},
    {"scatter16_write", 2, 16, 16, 0, 1, "16-byte write of every 16 B piece once, scattered"},
    {"flush16x4_write", 2, 64, 16, 0, 4, "4 lanes x 16 B = one 64 B piece per unit, pieces scattered (inflate/LZ4 flush)"},
    {"flush16x4_half128", 2, 128, 16, 0, 4, "one 64 B piece per 128 B line (half-line writes), scattered"},
    {"write4_all", 2, 4, 4, 0, 1, "4-byte write of every dword once, scattered (bzip2 scatter)"},
};
static constexpr int NPAT = sizeof(PATS) / sizeof(PATS[0]);
static constexpr int KINDS[] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 3, 2, 2, 2, 2};
static_assert(sizeof(KINDS) / sizeof(KINDS[0]) == NPAT, "KINDS follows PATS");
static constexpr u64 ODD = 0x9E3779B97F4A7C15ull | 1ull;

template <int W>
__device__ inline u32 ld(const u8* p) {
    if constexpr (W == 1) return *p;
    else if constexpr (W == 4) return *(const u32*)p;
    else {
        // unaligned 16-byte read (the far-source form)
        typedef u32 u32x4 __attribute__((ext_vector_type(4), aligned(1)));
        const u32x4 v = *(const u32x4*)p;
        return v.x ^ v.y ^ v.z ^ v.w;
    }
}

template <int M, int KIND, int W>
__global__ void __launch_bounds__(256) calib_k(u8* buf, u64 units, u32 unit, u32 off, u32 group, u32* sink) {
    const u64 nthreads = (u64)gridDim.x * blockDim.x;
    const u64 gid = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    u32 acc = 0;
    if constexpr (KIND == 1) {
        typedef u32 u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* p = (const u32x4*)buf;
        for (u64 i = gid; i < units; i += nthreads) {
            const u32x4 v = p[i];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    } else if constexpr (KIND == 0) {
        const u64 mask = units - 1;  // units is a power of two
        for (u64 t = gid; t < units; t += nthreads) {
            const u64 u = (t * ODD) & mask;
            acc += ld<W>(buf + u * unit + off);
        }
    } else if constexpr (KIND == 3) {
        typedef u32 u32x4 __attribute__((ext_vector_type(4)));
        u32x4* p = (u32x4*)buf;
        for (u64 i = gid; i < units; i += nthreads) p[i] = u32x4{(u32)i, 1u, 2u, 3u};
    } else {
        const u64 mask = units - 1;
        const u64 lanes = units * group;
        for (u64 t = gid; t < lanes; t += nthreads) {
            const u64 g = t / group, j = t % group;
            u8* p = buf + ((g * ODD) & mask) * unit + off + j * W;
            if constexpr (W == 16) {
                typedef u32 u32x4 __attribute__((ext_vector_type(4)));
                *(u32x4*)p = u32x4{(u32)t, (u32)g, (u32)j, 7u};
            } else {
                *(u32*)p = (u32)t;
            }
        }
    }
    if (acc == 0x5EED5EEDu) sink[0] = acc;  // keeps the loads live
}

__global__ void __launch_bounds__(256) calib_evict(u32* p, u64 n) {
    const u64 nthreads = (u64)gridDim.x * blockDim.x;
    typedef u32 u32x4 __attribute__((ext_vector_type(4)));
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthreads) ((u32x4*)p)[i] = u32x4{1u, 2u, 3u, (u32)i};
}

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <int M>
static void launch(const Pat& p, u8* buf, u64 bytes, u32* sink, hipStream_t s) {
    constexpr int KIND = KINDS[M];
    const u64 units = bytes / p.unit;
    const int blocks = 8192;
    if (p.width == 1) hipLaunchKernelGGL((calib_k<M, KIND, 1>), dim3(blocks), dim3(256), 0, s, buf, units, p.unit, p.off, p.group, sink);
    else if (p.width == 4) hipLaunchKernelGGL((calib_k<M, KIND, 4>), dim3(blocks), dim3(256), 0, s, buf, units, p.unit, p.off, p.group, sink);
    else hipLaunchKernelGGL((calib_k<M, KIND, 16>), dim3(blocks), dim3(256), 0, s, buf, units, p.unit, p.off, p.group, sink);
}

template <int M>
static void run_all(u8* buf, u64 bytes, u32* sink, u32* ev, u64 evn, hipStream_t s) {
    if constexpr (M < NPAT) {
        const Pat& p = PATS[M];
        hipLaunchKernelGGL(calib_evict, dim3(8192), dim3(256), 0, s, ev, evn);
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a, s));
        launch<M>(p, buf, bytes, sink, s);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const u64 units = bytes / p.unit;
        // known bytes: reads = units * width (accessed), lines = distinct 128 B lines touched;
        // writes = units * group * width
        const u64 accessed = p.kind >= 2 ? units * p.group * p.width : units * p.width;
        const u64 line_span = (p.off % 128 + p.width + 127) / 128;  // lines one access touches
        const u64 lines = p.unit >= 128 ? units * line_span : bytes / 128;
        printf("{\"pattern\": \"%s\", \"kernel\": \"calib_k<%d\", \"kind\": \"%s\", \"buffer_bytes\": %llu, "
               "\"units\": %llu, \"unit_bytes\": %u, \"width\": %u, \"accessed_bytes\": %llu, \"lines128\": %llu, "
               "\"ms\": %.4f, \"what\": \"%s\"}\n",
               p.name, M, p.kind >= 2 ? "write" : "read", (unsigned long long)bytes, (unsigned long long)units, p.unit,
               p.width, (unsigned long long)accessed, (unsigned long long)lines, ms, p.what);
        CK(hipEventDestroy(a));
        CK(hipEventDestroy(b));
        run_all<M + 1>(buf, bytes, sink, ev, evn, s);
    }
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    if (lg < 20 || lg > 33) {
        fprintf(stderr, "log2 bytes out of range\n");
        return 2;
    }
    const u64 bytes = 1ull << lg, evb = 512ull << 20;
    u8* buf;
    u32 *sink, *ev;
    CK(hipMalloc(&buf, bytes + 256));
    CK(hipMalloc(&ev, evb));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0x5A, bytes + 256));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    run_all<0>(buf, bytes, sink, ev, evb / 16, s);
    CK(hipStreamSynchronize(s));
    CK(hipStreamDestroy(s));
    CK(hipFree(buf));
    CK(hipFree(ev));
    CK(hipFree(sink));
    return 0;
}
