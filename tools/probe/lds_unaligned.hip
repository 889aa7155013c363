// Probe: does gfx950 LDS honour byte-unaligned ds_write_b128 / ds_read_b128 /
// ds_read_b64 addresses (SH_MEM_CONFIG alignment_mode)?  Prints per-offset
// pass/fail; no global side effects beyond its own buffer.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[64 * 64];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 64 * 64; i += 64) buf[i] = 0xEE;
    __syncthreads();
    const uint32_t off = lane & 15;  // misalignment under test
    const uint32_t base = lane * 64 + off;
    uint32_t a = (uint32_t)(uintptr_t)(buf + base);
    uint32_t v0 = 0x03020100u + 0x04040404u * off, v1 = v0 + 0x10101010u, v2 = v1 + 0x10101010u, v3 = v2 + 0x10101010u;
    asm volatile("ds_write_b128 %0, %1\n s_waitcnt lgkmcnt(0)" ::"v"(a), "v"(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, (uint4){v0, v1, v2, v3})) : "memory");
    __syncthreads();
    // check bytes written
    uint32_t ok_w = 1;
    const uint8_t* pb = (const uint8_t*)&v0;
    uint32_t want[4] = {v0, v1, v2, v3};
    for (uint32_t k = 0; k < 16; k++) {
        const uint8_t w = (uint8_t)(want[k >> 2] >> (8 * (k & 3)));
        if (buf[base + k] != w) ok_w = 0;
    }
    if (buf[base - 1 + (off == 0 ? 1 : 0) * 0] != 0xEE && off != 0) ok_w = 0;
    if (buf[base + 16] != 0xEE) ok_w = 0;
    // unaligned ds_read_b128 of the same bytes
    __attribute__((ext_vector_type(4))) uint32_t r;
    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
    const uint32_t ok_r = (r.x == v0 && r.y == v1 && r.z == v2 && r.w == v3) ? 1u : 0u;
    __attribute__((ext_vector_type(2))) uint32_t r2;
    asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r2) : "v"(a + 4) : "memory");
    const uint32_t ok_r64 = (r2.x == v1 && r2.y == v2) ? 1u : 0u;
    out[lane] = ok_w | (ok_r << 1) | (ok_r64 << 2);
    (void)pb;
}

int main() {
    uint32_t* d;
    if (hipMalloc(&d, 64 * 4) != hipSuccess) return 2;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    uint32_t h[64];
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    int allok = 1;
    for (int off = 0; off < 16; off++) {
        printf("off %2d: write %s read_b128 %s read_b64 %s\n", off, (h[off] & 1) ? "ok" : "BAD",
               (h[off] & 2) ? "ok" : "BAD", (h[off] & 4) ? "ok" : "BAD");
        if ((h[off] & 7) != 7) allok = 0;
    }
    printf("unaligned LDS b64/b128: %s\n", allok ? "SUPPORTED" : "NOT SUPPORTED");
    return 0;
}
