// Probe: cost of byte-unaligned LDS vector accesses on gfx950 (the inflate
// wave kernel's far/near copies store and load 8 stage entries at 2-byte
// alignment).  One wave per SIMD (4 per CU, every CU), each lane at its own
// 16-byte slot plus an offset OFF bytes (OFF = 0 aligned, 2, 4, 8); per op
// kind the loop runs ITERS x 8 accesses, either as a dependent chain (each
// address depends on the last load: latency) or 8 independent accesses per
// wait (issue cost).  Prints one JSON object: cycles per access (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a1 __attribute__((aligned(1)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 u32x2_a1 __attribute__((aligned(1)));

constexpr int ITERS = 2048;

// MODE 0: dependent b128 reads; 1: independent b128 reads; 2: b128 writes;
// 3: dependent b64 reads; 4: b64 writes; 5: dependent b32 reads (aligned
// dword only, the reference point); 6 / 7: u16 reads / writes; 8: u8 reads
template <int MODE>
__global__ __launch_bounds__(64) void probe(unsigned long long* cyc, uint32_t off, uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[64 * 32 + 64];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < (64 * 32 + 64) / 4; i += 64) ((uint32_t*)buf)[i] = 0;
    __syncthreads();
    uint32_t a = lane * 32 + off, acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; it++) {
        if constexpr (MODE == 0) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const u32x4 v = *(const u32x4_a1*)(buf + a);
                a = lane * 32 + off + (v.x & 1u);  // (always + 0: the buffer is zero) dependent address
                acc += v.y;
            }
        } else if constexpr (MODE == 1) {
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) v[k] = *(const u32x4_a1*)(buf + ((a + 2 * k) & ~1u));
#pragma unroll
            for (int k = 0; k < 8; k++) acc += v[k].x ^ v[k].w;
            a = lane * 32 + off + (acc & 0u);
        } else if constexpr (MODE == 2) {
#pragma unroll
            for (int k = 0; k < 8; k++) *(u32x4_a1*)(buf + a) = u32x4{acc, acc + 1, acc + 2, (uint32_t)k};
            acc += 1;
        } else if constexpr (MODE == 3) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const u32x2 v = *(const u32x2_a1*)(buf + a);
                a = lane * 32 + off + (v.x & 1u);
                acc += v.y;
            }
        } else if constexpr (MODE == 4) {
#pragma unroll
            for (int k = 0; k < 8; k++) *(u32x2_a1*)(buf + a) = u32x2{acc, (uint32_t)k};
            acc += 1;
        } else if constexpr (MODE == 6) {  // dependent u16 reads at the offset (2-byte aligned)
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t v = *(const uint16_t*)(buf + (a & ~1u));
                a = lane * 32 + off + (v & 1u);
                acc += v;
            }
        } else if constexpr (MODE == 7) {  // u16 writes at the offset
#pragma unroll
            for (int k = 0; k < 8; k++) *(uint16_t*)(buf + (a & ~1u) + 32 * 0) = (uint16_t)(acc + k);
            acc += 1;
        } else if constexpr (MODE == 8) {  // dependent u8 reads at the offset + 1
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t v = buf[a + 1];
                a = lane * 32 + off + (v & 1u);
                acc += v;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t v = *(const uint32_t*)(buf + (a & ~3u));
                a = lane * 32 + off + (v & 1u);
                acc += v;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the writes of the iteration done
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    if (acc == 0x12345678u) sink[lane] = acc;
}

template <int MODE>
static double run(int cus, uint32_t off, unsigned long long* d, uint32_t* sink) {
    const int nblk = cus * 4;
    hipLaunchKernelGGL(probe<MODE>, dim3(nblk), dim3(64), 0, 0, d, off, sink);
    std::vector<unsigned long long> h(nblk);
    if (hipMemcpy(h.data(), d, sizeof(unsigned long long) * nblk, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    std::sort(h.begin(), h.end());
    return (double)h[nblk / 2] / (ITERS * 8.0);
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 2;
    const int cus = p.multiProcessorCount;
    unsigned long long* d;
    uint32_t* sink;
    if (hipMalloc(&d, sizeof(unsigned long long) * cus * 4) != hipSuccess) return 3;
    if (hipMalloc(&sink, 256) != hipSuccess) return 3;
    const char* names[] = {"b128_read_dependent", "b128_read_independent", "b128_write", "b64_read_dependent",
                           "b64_write", "b32_read_dependent_aligned", "u16_read_dependent", "u16_write",
                           "u8_read_dependent_off+1"};
    printf("{\"results\": [\n");
    bool first = true;
    for (uint32_t off : {0u, 2u, 4u, 8u}) {
        double c[9];
        c[0] = run<0>(cus, off, d, sink);
        c[1] = run<1>(cus, off, d, sink);
        c[2] = run<2>(cus, off, d, sink);
        c[3] = run<3>(cus, off, d, sink);
        c[4] = run<4>(cus, off, d, sink);
        c[5] = run<5>(cus, off, d, sink);
        c[6] = run<6>(cus, off, d, sink);
        c[7] = run<7>(cus, off, d, sink);
        c[8] = run<8>(cus, off, d, sink);
        for (int m = 0; m < 9; m++) {
            printf("%s {\"op\": \"%s\", \"offset\": %u, \"cycles_per_access\": %.2f}", first ? "" : ",\n", names[m], off, c[m]);
            first = false;
        }
    }
    printf("\n]}\n");
    return 0;
}
