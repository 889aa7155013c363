// Probe: VALU issue cost of the inflate wave kernel's integer instruction mix
// on gfx950, at 1 / 2 / 4 / 8 waves per SIMD.
//
// Every CU gets W waves per SIMD (grid = 256 CUs x 4 SIMDs x W one-wave
// workgroups; LDS is sized so that no more than 4W waves fit a CU).  Each wave
// runs ITERS x 32 instructions of one opcode over 8 independent registers
// (no dependency inside an 8-instruction window, so latency is covered by the
// window and only issue is measured), timed by s_memtime around the loop.
// Reported: cycles per wave64 instruction per SIMD = the wave's loop cycles /
// (W x instructions per wave) — the SIMD's issue cost once W waves share it —
// and the single-wave cost (W = 1).  Output: one JSON object.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>

#define REP8(x) x x x x x x x x
#define BODY8(OP)                                                                               \
    asm volatile(REP8(OP) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                 "+v"(a7), "+v"(b0), "+v"(b1) ::);

constexpr int ITERS = 4096;

// the 8 registers are used round-robin through the 8 copies via %0..%7
#define OPS_ADD "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
#define OPS_PERM "v_perm_b32 %0, %0, %8, %9\n v_perm_b32 %1, %1, %8, %9\n v_perm_b32 %2, %2, %8, %9\n v_perm_b32 %3, %3, %8, %9\n v_perm_b32 %4, %4, %8, %9\n v_perm_b32 %5, %5, %8, %9\n v_perm_b32 %6, %6, %8, %9\n v_perm_b32 %7, %7, %8, %9\n"
#define OPS_ALIGN "v_alignbit_b32 %0, %0, %8, %9\n v_alignbit_b32 %1, %1, %8, %9\n v_alignbit_b32 %2, %2, %8, %9\n v_alignbit_b32 %3, %3, %8, %9\n v_alignbit_b32 %4, %4, %8, %9\n v_alignbit_b32 %5, %5, %8, %9\n v_alignbit_b32 %6, %6, %8, %9\n v_alignbit_b32 %7, %7, %8, %9\n"
#define OPS_CND "v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n"
#define OPS_BFE "v_bfe_u32 %0, %0, %8, 7\n v_bfe_u32 %1, %1, %8, 7\n v_bfe_u32 %2, %2, %8, 7\n v_bfe_u32 %3, %3, %8, 7\n v_bfe_u32 %4, %4, %8, 7\n v_bfe_u32 %5, %5, %8, 7\n v_bfe_u32 %6, %6, %8, 7\n v_bfe_u32 %7, %7, %8, 7\n"
#define OPS_MUL24 "v_mul_u32_u24 %0, %0, %8\n v_mul_u32_u24 %1, %1, %8\n v_mul_u32_u24 %2, %2, %8\n v_mul_u32_u24 %3, %3, %8\n v_mul_u32_u24 %4, %4, %8\n v_mul_u32_u24 %5, %5, %8\n v_mul_u32_u24 %6, %6, %8\n v_mul_u32_u24 %7, %7, %8\n"
#define OPS_MULLO "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"
#define OPS_DPP "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %2, %2, %2 row_shr:1 row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %3, %3, %3 row_shr:1 row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %4, %4, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %5, %5, %5 row_shr:1 row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %6, %6, %6 row_shr:1 row_mask:0xf bank_mask:0xf\n v_add_u32_dpp %7, %7, %7 row_shr:1 row_mask:0xf bank_mask:0xf\n"
#define OPS_READLANE "v_readlane_b32 s0, %0, 5\n v_readlane_b32 s1, %1, 6\n v_readlane_b32 s2, %2, 7\n v_readlane_b32 s3, %3, 8\n v_readlane_b32 s4, %4, 9\n v_readlane_b32 s5, %5, 10\n v_readlane_b32 s6, %6, 11\n v_readlane_b32 s7, %7, 12\n"
// the kernel's mix: one of each common op per 8-instruction window
#define OPS_MIX "v_add_u32 %0, %0, %8\n v_perm_b32 %1, %1, %8, %9\n v_alignbit_b32 %2, %2, %8, %9\n v_cndmask_b32 %3, %3, %8, vcc\n v_bfe_u32 %4, %4, %8, 7\n v_mul_u32_u24 %5, %5, %8\n v_and_b32 %6, %6, %8\n v_lshlrev_b32 %7, %8, %7\n"

// the compiler's select forms: v_cndmask on a VCC / SGPR-pair mask that a
// VALU compare wrote (in the prologue, or right before it, as compiled code does)
#define OPS_CND64 "v_cndmask_b32_e64 %0, %0, %8, s[10:11]\n v_cndmask_b32_e64 %1, %1, %8, s[10:11]\n v_cndmask_b32_e64 %2, %2, %8, s[10:11]\n v_cndmask_b32_e64 %3, %3, %8, s[10:11]\n v_cndmask_b32_e64 %4, %4, %8, s[10:11]\n v_cndmask_b32_e64 %5, %5, %8, s[10:11]\n v_cndmask_b32_e64 %6, %6, %8, s[10:11]\n v_cndmask_b32_e64 %7, %7, %8, s[10:11]\n"
#define OPS_CMPCND "v_cmp_gt_u32_e64 s[10:11], %0, %8\n v_cndmask_b32_e64 %1, %1, %8, s[10:11]\n v_cmp_gt_u32_e64 s[12:13], %2, %8\n v_cndmask_b32_e64 %3, %3, %8, s[12:13]\n v_cmp_gt_u32_e64 s[10:11], %4, %8\n v_cndmask_b32_e64 %5, %5, %8, s[10:11]\n v_cmp_gt_u32_e64 s[12:13], %6, %8\n v_cndmask_b32_e64 %7, %7, %8, s[12:13]\n"
#define OPS_CMPVCC "v_cmp_gt_u32_e32 vcc, %0, %8\n v_cndmask_b32_e32 %1, %1, %8, vcc\n v_cmp_gt_u32_e32 vcc, %2, %8\n v_cndmask_b32_e32 %3, %3, %8, vcc\n v_cmp_gt_u32_e32 vcc, %4, %8\n v_cndmask_b32_e32 %5, %5, %8, vcc\n v_cmp_gt_u32_e32 vcc, %6, %8\n v_cndmask_b32_e32 %7, %7, %8, vcc\n"
#define OPS_ADD3 "v_add3_u32 %0, %0, %8, %9\n v_add3_u32 %1, %1, %8, %9\n v_add3_u32 %2, %2, %8, %9\n v_add3_u32 %3, %3, %8, %9\n v_add3_u32 %4, %4, %8, %9\n v_add3_u32 %5, %5, %8, %9\n v_add3_u32 %6, %6, %8, %9\n v_add3_u32 %7, %7, %8, %9\n"
#define OPS_AND "v_and_b32 %0, %0, %8\n v_and_b32 %1, %1, %8\n v_and_b32 %2, %2, %8\n v_and_b32 %3, %3, %8\n v_and_b32 %4, %4, %8\n v_and_b32 %5, %5, %8\n v_and_b32 %6, %6, %8\n v_and_b32 %7, %7, %8\n"
#define OPS_ADDE64 "v_add_u32_e64 %0, %0, %8\n v_add_u32_e64 %1, %1, %8\n v_add_u32_e64 %2, %2, %8\n v_add_u32_e64 %3, %3, %8\n v_add_u32_e64 %4, %4, %8\n v_add_u32_e64 %5, %5, %8\n v_add_u32_e64 %6, %6, %8\n v_add_u32_e64 %7, %7, %8\n"

template <int K>
__global__ __launch_bounds__(64) void probe(unsigned long long* cyc, uint32_t seed) {
    extern __shared__ uint32_t lds_pad[];
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, b0 = seed | 1, b1 = 0x05040100u;
    unsigned long long c0 = a0, c1 = a1, c2 = a2, c3 = a3, c4 = a4, c5 = a5, c6 = a6, c7 = a7;
    asm volatile("s_mov_b64 vcc, exec\n v_cmp_ne_u32_e64 s[10:11], %0, 0\n s_nop 4" :: "v"(b1) : "vcc", "s10", "s11");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; it++) {
        if constexpr (K == 0) { BODY8(OPS_ADD) }
        if constexpr (K == 1) { BODY8(OPS_PERM) }
        if constexpr (K == 2) { BODY8(OPS_ALIGN) }
        if constexpr (K == 3) { BODY8(OPS_CND) }
        if constexpr (K == 4) { BODY8(OPS_BFE) }
        if constexpr (K == 5) { BODY8(OPS_MUL24) }
        if constexpr (K == 6) { BODY8(OPS_MULLO) }
        if constexpr (K == 7) {
            asm volatile(REP8("v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 3, %1\n v_lshlrev_b64 %2, 3, %2\n v_lshlrev_b64 %3, 3, %3\n"
                              "v_lshlrev_b64 %4, 3, %4\n v_lshlrev_b64 %5, 3, %5\n v_lshlrev_b64 %6, 3, %6\n v_lshlrev_b64 %7, 3, %7\n")
                         : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)::);
        }
        if constexpr (K == 8) { BODY8(OPS_DPP) }
        if constexpr (K == 9) {
            asm volatile(REP8(OPS_READLANE) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),
                         "+v"(a7), "+v"(b0), "+v"(b1)::"s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7");
        }
        if constexpr (K == 10) { BODY8(OPS_MIX) }
        if constexpr (K == 11) { BODY8(OPS_CND64) }
        if constexpr (K == 12) {
            asm volatile(REP8(OPS_CMPCND) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),
                         "+v"(a7), "+v"(b0), "+v"(b1)::"s10", "s11", "s12", "s13");
        }
        if constexpr (K == 13) {
            asm volatile(REP8(OPS_CMPVCC) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),
                         "+v"(a7), "+v"(b0), "+v"(b1)::"vcc");
        }
        if constexpr (K == 14) { BODY8(OPS_ADD3) }
        if constexpr (K == 15) { BODY8(OPS_AND) }
        if constexpr (K == 16) { BODY8(OPS_ADDE64) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7)) == 0x7FFFFFFFu)
        lds_pad[threadIdx.x] = a0;  // keep results live
}

static const char* kNames[] = {"v_add_u32", "v_perm_b32", "v_alignbit_b32", "v_cndmask_b32", "v_bfe_u32",
                               "v_mul_u32_u24", "v_mul_lo_u32", "v_lshlrev_b64", "v_add_u32_dpp",
                               "v_readlane_b32", "mix8", "v_cndmask_b32_e64(sgpr)", "v_cmp_e64+v_cndmask_e64",
                               "v_cmp_e32+v_cndmask_e32(vcc)", "v_add3_u32", "v_and_b32", "v_add_u32_e64"};

static double g_max = 0;
template <int K>
static double run(int cus, int w, unsigned long long* d, std::vector<unsigned long long>& h, double* wall_ms) {
    const int nblk = cus * 4 * w;
    // LDS per workgroup so that at most 4*w one-wave workgroups fit a CU (160 KiB)
    const size_t lds = (size_t)(160 * 1024 / (4 * w)) & ~(size_t)255;
    hipFuncSetAttribute((const void*)probe<K>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(probe<K>, dim3(nblk), dim3(64), lds, 0, d, 7u);  // warm
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(probe<K>, dim3(nblk), dim3(64), lds, 0, d, 9u);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    *wall_ms = ms;
    hipMemcpy(h.data(), d, sizeof(unsigned long long) * nblk, hipMemcpyDeviceToHost);
    std::vector<unsigned long long> v(h.begin(), h.begin() + nblk);
    std::sort(v.begin(), v.end());
    const double med = (double)v[v.size() / 2];  // s_memtime = shader-clock cycles of the wave's loop
    *wall_ms = ms;
    g_max = (double)v.back();
    return med;
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 2;
    const int cus = p.multiProcessorCount;
    unsigned long long* d;
    if (hipMalloc(&d, sizeof(unsigned long long) * cus * 4 * 8) != hipSuccess) return 3;
    std::vector<unsigned long long> h(cus * 4 * 8);
    const double insts = (double)ITERS * 64;  // wave instructions per wave (8 x 8 per iteration)
    printf("{\"cus\": %d, \"clock_khz\": %d, \"insts_per_wave\": %.0f, \"results\": [\n", cus, p.clockRate, insts);
    bool first = true;
    auto one = [&](auto kc, const char* name) {
        constexpr int K = decltype(kc)::value;
        for (int w : {1, 2, 4, 8}) {
            double wall = 0;
            const double ticks = run<K>(cus, w, d, h, &wall);
            printf("%s {\"op\": \"%s\", \"waves_per_simd\": %d, \"wall_ms\": %.4f, \"loop_cycles_med\": %.0f, "
                   "\"cycles_per_inst_per_wave\": %.3f, \"cycles_per_inst_per_simd\": %.3f, \"max_loop_cycles\": %.0f, "
                   "\"cycles_per_inst_per_simd_maxwave\": %.3f}",
                   first ? "" : ",\n", name, w, wall, ticks, ticks / insts, ticks / (insts * w), g_max, g_max / (insts * w));
            first = false;
        }
    };
    one(std::integral_constant<int, 0>{}, kNames[0]);
    one(std::integral_constant<int, 1>{}, kNames[1]);
    one(std::integral_constant<int, 2>{}, kNames[2]);
    one(std::integral_constant<int, 3>{}, kNames[3]);
    one(std::integral_constant<int, 4>{}, kNames[4]);
    one(std::integral_constant<int, 5>{}, kNames[5]);
    one(std::integral_constant<int, 6>{}, kNames[6]);
    one(std::integral_constant<int, 7>{}, kNames[7]);
    one(std::integral_constant<int, 8>{}, kNames[8]);
    one(std::integral_constant<int, 9>{}, kNames[9]);
    one(std::integral_constant<int, 10>{}, kNames[10]);
    one(std::integral_constant<int, 11>{}, kNames[11]);
    one(std::integral_constant<int, 12>{}, kNames[12]);
    one(std::integral_constant<int, 13>{}, kNames[13]);
    one(std::integral_constant<int, 14>{}, kNames[14]);
    one(std::integral_constant<int, 15>{}, kNames[15]);
    one(std::integral_constant<int, 16>{}, kNames[16]);
    printf("\n]}\n");
    hipFree(d);
    return 0;
}
