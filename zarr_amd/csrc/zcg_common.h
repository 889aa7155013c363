// zcg_common.h — shared device/host definitions of the MI355X chunk-codec
// library (kernels in zcg_*.hip, C ABI in zcg_api.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zchunk_gpu.h"

namespace zcg {

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int32_t i32;
typedef int64_t i64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// byte-aligned views: gfx950 global memory accepts unaligned dword accesses
// (hipcc lowers these to global_load/store_dwordx{2,4}).
typedef u32x4 __attribute__((aligned(1))) u32x4_ua;
typedef u32x2 __attribute__((aligned(1))) u32x2_ua;
typedef uint32_t __attribute__((aligned(1))) u32_ua;
typedef uint16_t __attribute__((aligned(1))) u16_ua;

// Element transform that read_data applies after the codec (chunk.rs:103-116,
// 175-190): per-element byte reversal for Big-endian multi-byte types, and
// bool = byte != 0.  Encode (write_data, chunk.rs:118-140) is the same map.
struct DType {
    u32 es;     // element size
    u32 swap;   // 1 -> reverse bytes of each element
    u32 isbool; // 1 -> normalise bytes to 0/1
};

__host__ __device__ inline DType make_dtype(const zcg_dtype& d) {
    DType t;
    t.es = d.elem_size ? d.elem_size : 1;
    t.swap = (d.big_endian && t.es > 1 && !d.is_bool) ? 1u : 0u;
    t.isbool = d.is_bool ? 1u : 0u;
    return t;
}

__device__ __forceinline__ u32 bool_norm32(u32 x) {
    x |= (x >> 4) & 0x0f0f0f0fu;
    x |= (x >> 2) & 0x03030303u;
    x |= (x >> 1) & 0x01010101u;
    return x & 0x01010101u;
}

__device__ __forceinline__ u32 bswap16x2(u32 x) {
    return ((x & 0x00ff00ffu) << 8) | ((x >> 8) & 0x00ff00ffu);
}

// Transform 16 bytes that start at an element-aligned logical offset.
__device__ __forceinline__ u32x4 transform16(u32x4 v, const DType& t) {
    if (t.isbool) {
        v.x = bool_norm32(v.x); v.y = bool_norm32(v.y);
        v.z = bool_norm32(v.z); v.w = bool_norm32(v.w);
    } else if (t.swap) {
        if (t.es == 2) {
            v.x = bswap16x2(v.x); v.y = bswap16x2(v.y);
            v.z = bswap16x2(v.z); v.w = bswap16x2(v.w);
        } else if (t.es == 4) {
            v.x = __builtin_bswap32(v.x); v.y = __builtin_bswap32(v.y);
            v.z = __builtin_bswap32(v.z); v.w = __builtin_bswap32(v.w);
        } else {  // es == 8
            u32 a = __builtin_bswap32(v.x), b = __builtin_bswap32(v.y);
            u32 c = __builtin_bswap32(v.z), d = __builtin_bswap32(v.w);
            v.x = b; v.y = a; v.z = d; v.w = c;
        }
    }
    return v;
}

// Physical byte position of logical decoded byte p (element-local reversal).
__device__ __forceinline__ u64 swap_pos(u64 p, const DType& t) {
    if (!t.swap) return p;
    u64 m = t.es - 1;
    return (p & ~m) | (m - (p & m));
}

__device__ __forceinline__ u8 norm_byte(u8 b, const DType& t) {
    return t.isbool ? (u8)(b != 0) : b;
}

// Per-lane 16-byte piece copy with unaligned addresses.
__device__ __forceinline__ u32x4 ld16(const u8* p) { return *(const u32x4_ua*)p; }
__device__ __forceinline__ void st16(u8* p, u32x4 v) { *(u32x4_ua*)p = v; }
__device__ __forceinline__ u32x2 ld8(const u8* p) { return *(const u32x2_ua*)p; }
__device__ __forceinline__ void st8(u8* p, u32x2 v) { *(u32x2_ua*)p = v; }
__device__ __forceinline__ u32 ld32(const u8* p) { return *(const u32_ua*)p; }
__device__ __forceinline__ u32 ld16le(const u8* p) { return *(const u16_ua*)p; }

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Address-space-qualified views: global (HBM) and LDS accesses without flat
// instructions, for code whose pointers travel through structs.
typedef __attribute__((address_space(1))) u8 gu8;
typedef __attribute__((address_space(1))) u32 gu32;
typedef __attribute__((address_space(3))) u8 lu8;
typedef __attribute__((address_space(3))) u16 lu16;
typedef __attribute__((address_space(3))) u32 lu32;
typedef __attribute__((address_space(1))) u32x4 gu32x4_ua __attribute__((aligned(1)));
typedef __attribute__((address_space(1))) u32x2 gu32x2_ua __attribute__((aligned(1)));
__device__ __forceinline__ u64 ru64(u64 x) {  // wave-uniform 64-bit value -> SGPRs
    return ((u64)__builtin_amdgcn_readfirstlane((u32)(x >> 32)) << 32) |
           (u32)__builtin_amdgcn_readfirstlane((u32)x);
}

// In-place element transform of a decoded chunk by the whole wave.
__device__ inline void wave_transform(u8* dst, u64 D, const DType& t) {
    const int lane = lane_id();
    const bool al = (((uintptr_t)dst) & 15) == 0;
    for (u64 p = (u64)lane * 16; p < D; p += 64 * 16) {
        if (p + 16 <= D) {
            u32x4 v = al ? *(u32x4*)(dst + p) : ld16(dst + p);
            v = transform16(v, t);
            if (al) *(u32x4*)(dst + p) = v; else st16(dst + p, v);
        } else {
            // tail shorter than 16 bytes: whole elements only (D % es == 0)
            u8 tmp[16];
            for (u64 q = p; q < D; q++) tmp[q - p] = dst[q];
            for (u64 q = p; q < D; q++) dst[swap_pos(q, t)] = norm_byte(tmp[q - p], t);
        }
    }
}

// ---- XXH32 (LZ4 frame header / block / content checksums) --------------
constexpr u32 XXH_P1 = 2654435761u;
constexpr u32 XXH_P2 = 2246822519u;
constexpr u32 XXH_P3 = 3266489917u;
constexpr u32 XXH_P4 = 668265263u;
constexpr u32 XXH_P5 = 374761393u;

__host__ __device__ inline u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }

// Serial XXH32 over global memory (one lane).
__device__ inline u32 xxh32(const u8* p, u64 len, u32 seed) {
    const u8* end = p + len;
    u32 h;
    if (len >= 16) {
        const u8* limit = end - 16;
        u32 v1 = seed + XXH_P1 + XXH_P2, v2 = seed + XXH_P2, v3 = seed, v4 = seed - XXH_P1;
        do {
            u32x4 w = ld16(p);
            v1 = rotl32(v1 + w.x * XXH_P2, 13) * XXH_P1;
            v2 = rotl32(v2 + w.y * XXH_P2, 13) * XXH_P1;
            v3 = rotl32(v3 + w.z * XXH_P2, 13) * XXH_P1;
            v4 = rotl32(v4 + w.w * XXH_P2, 13) * XXH_P1;
            p += 16;
        } while (p <= limit);
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + XXH_P5;
    }
    h += (u32)len;
    while (p + 4 <= end) {
        h += ld32(p) * XXH_P3;
        h = rotl32(h, 17) * XXH_P4;
        p += 4;
    }
    while (p < end) {
        h += (*p) * XXH_P5;
        h = rotl32(h, 11) * XXH_P1;
        p++;
    }
    h ^= h >> 15; h *= XXH_P2; h ^= h >> 13; h *= XXH_P3; h ^= h >> 16;
    return h;
}

// ---- CRC32 (gzip header CRC / trailer), table in constant memory --------
static __constant__ u32 g_crc32_table[256] = {
    0x00000000u, 0x77073096u, 0xee0e612cu, 0x990951bau, 0x076dc419u, 0x706af48fu,
    0xe963a535u, 0x9e6495a3u, 0x0edb8832u, 0x79dcb8a4u, 0xe0d5e91eu, 0x97d2d988u,
    0x09b64c2bu, 0x7eb17cbdu, 0xe7b82d07u, 0x90bf1d91u, 0x1db71064u, 0x6ab020f2u,
    0xf3b97148u, 0x84be41deu, 0x1adad47du, 0x6ddde4ebu, 0xf4d4b551u, 0x83d385c7u,
    0x136c9856u, 0x646ba8c0u, 0xfd62f97au, 0x8a65c9ecu, 0x14015c4fu, 0x63066cd9u,
    0xfa0f3d63u, 0x8d080df5u, 0x3b6e20c8u, 0x4c69105eu, 0xd56041e4u, 0xa2677172u,
    0x3c03e4d1u, 0x4b04d447u, 0xd20d85fdu, 0xa50ab56bu, 0x35b5a8fau, 0x42b2986cu,
    0xdbbbc9d6u, 0xacbcf940u, 0x32d86ce3u, 0x45df5c75u, 0xdcd60dcfu, 0xabd13d59u,
    0x26d930acu, 0x51de003au, 0xc8d75180u, 0xbfd06116u, 0x21b4f4b5u, 0x56b3c423u,
    0xcfba9599u, 0xb8bda50fu, 0x2802b89eu, 0x5f058808u, 0xc60cd9b2u, 0xb10be924u,
    0x2f6f7c87u, 0x58684c11u, 0xc1611dabu, 0xb6662d3du, 0x76dc4190u, 0x01db7106u,
    0x98d220bcu, 0xefd5102au, 0x71b18589u, 0x06b6b51fu, 0x9fbfe4a5u, 0xe8b8d433u,
    0x7807c9a2u, 0x0f00f934u, 0x9609a88eu, 0xe10e9818u, 0x7f6a0dbbu, 0x086d3d2du,
    0x91646c97u, 0xe6635c01u, 0x6b6b51f4u, 0x1c6c6162u, 0x856530d8u, 0xf262004eu,
    0x6c0695edu, 0x1b01a57bu, 0x8208f4c1u, 0xf50fc457u, 0x65b0d9c6u, 0x12b7e950u,
    0x8bbeb8eau, 0xfcb9887cu, 0x62dd1ddfu, 0x15da2d49u, 0x8cd37cf3u, 0xfbd44c65u,
    0x4db26158u, 0x3ab551ceu, 0xa3bc0074u, 0xd4bb30e2u, 0x4adfa541u, 0x3dd895d7u,
    0xa4d1c46du, 0xd3d6f4fbu, 0x4369e96au, 0x346ed9fcu, 0xad678846u, 0xda60b8d0u,
    0x44042d73u, 0x33031de5u, 0xaa0a4c5fu, 0xdd0d7cc9u, 0x5005713cu, 0x270241aau,
    0xbe0b1010u, 0xc90c2086u, 0x5768b525u, 0x206f85b3u, 0xb966d409u, 0xce61e49fu,
    0x5edef90eu, 0x29d9c998u, 0xb0d09822u, 0xc7d7a8b4u, 0x59b33d17u, 0x2eb40d81u,
    0xb7bd5c3bu, 0xc0ba6cadu, 0xedb88320u, 0x9abfb3b6u, 0x03b6e20cu, 0x74b1d29au,
    0xead54739u, 0x9dd277afu, 0x04db2615u, 0x73dc1683u, 0xe3630b12u, 0x94643b84u,
    0x0d6d6a3eu, 0x7a6a5aa8u, 0xe40ecf0bu, 0x9309ff9du, 0x0a00ae27u, 0x7d079eb1u,
    0xf00f9344u, 0x8708a3d2u, 0x1e01f268u, 0x6906c2feu, 0xf762575du, 0x806567cbu,
    0x196c3671u, 0x6e6b06e7u, 0xfed41b76u, 0x89d32be0u, 0x10da7a5au, 0x67dd4accu,
    0xf9b9df6fu, 0x8ebeeff9u, 0x17b7be43u, 0x60b08ed5u, 0xd6d6a3e8u, 0xa1d1937eu,
    0x38d8c2c4u, 0x4fdff252u, 0xd1bb67f1u, 0xa6bc5767u, 0x3fb506ddu, 0x48b2364bu,
    0xd80d2bdau, 0xaf0a1b4cu, 0x36034af6u, 0x41047a60u, 0xdf60efc3u, 0xa867df55u,
    0x316e8eefu, 0x4669be79u, 0xcb61b38cu, 0xbc66831au, 0x256fd2a0u, 0x5268e236u,
    0xcc0c7795u, 0xbb0b4703u, 0x220216b9u, 0x5505262fu, 0xc5ba3bbeu, 0xb2bd0b28u,
    0x2bb45a92u, 0x5cb36a04u, 0xc2d7ffa7u, 0xb5d0cf31u, 0x2cd99e8bu, 0x5bdeae1du,
    0x9b64c2b0u, 0xec63f226u, 0x756aa39cu, 0x026d930au, 0x9c0906a9u, 0xeb0e363fu,
    0x72076785u, 0x05005713u, 0x95bf4a82u, 0xe2b87a14u, 0x7bb12baeu, 0x0cb61b38u,
    0x92d28e9bu, 0xe5d5be0du, 0x7cdcefb7u, 0x0bdbdf21u, 0x86d3d2d4u, 0xf1d4e242u,
    0x68ddb3f8u, 0x1fda836eu, 0x81be16cdu, 0xf6b9265bu, 0x6fb077e1u, 0x18b74777u,
    0x88085ae6u, 0xff0f6a70u, 0x66063bcau, 0x11010b5cu, 0x8f659effu, 0xf862ae69u,
    0x616bffd3u, 0x166ccf45u, 0xa00ae278u, 0xd70dd2eeu, 0x4e048354u, 0x3903b3c2u,
    0xa7672661u, 0xd06016f7u, 0x4969474du, 0x3e6e77dbu, 0xaed16a4au, 0xd9d65adcu,
    0x40df0b66u, 0x37d83bf0u, 0xa9bcae53u, 0xdebb9ec5u, 0x47b2cf7fu, 0x30b5ffe9u,
    0xbdbdf21cu, 0xcabac28au, 0x53b39330u, 0x24b4a3a6u, 0xbad03605u, 0xcdd70693u,
    0x54de5729u, 0x23d967bfu, 0xb3667a2eu, 0xc4614ab8u, 0x5d681b02u, 0x2a6f2b94u,
    0xb40bbe37u, 0xc30c8ea1u, 0x5a05df1bu, 0x2d02ef8du};

// Region assembly arguments (zcg_region.hip), built by zcg_read_region.
struct RegionArgs {
    u32 nd, es, fill, V;       // dims, element bytes, fill flag, elements per thread (16/es)
    u32 dir, pad;              // 0: chunks -> box (read_ndarray), 1: box -> chunks (write_ndarray)
    u64 total;                 // elements in the box
    u64 fillv;                 // fill element, replicated to 16 bytes below
    // per dim, fast-first order (the chunks' memory order)
    u32 bs[ZCG_MAX_DIMS];      // box extent
    u32 orr[ZCG_MAX_DIMS];     // box offset mod chunk extent
    u32 cs[ZCG_MAX_DIMS];      // chunk extent
    u64 ob[ZCG_MAX_DIMS];      // box offset / chunk extent  (= grid_lo)
    u64 gn[ZCG_MAX_DIMS];      // visited chunks along the dim
    u64 tstr[ZCG_MAX_DIMS];    // chunk-table stride
    u64 cstr[ZCG_MAX_DIMS];    // element stride inside a chunk
    i64 ostr[ZCG_MAX_DIMS];    // element stride of the output view
};

}  // namespace zcg

// Internal launchers (zcg_*.hip) used by zcg_api.cpp.
namespace zcg {
struct Workspace;  // defined in zcg_api.cpp
// Tuning constants of a kernel source, as "name:K=V,K=V" (stringified macros):
// zcg_build_config() reports them, and tests/test_abi.py checks that the
// shipped library was built with the defaults.
#define ZCG_STR2(x) #x
#define ZCG_STR(x) ZCG_STR2(x)
const char* cfg_inflate_wave();
const char* cfg_inflate_par();
const char* cfg_deflate();
const char* cfg_raw();
const char* cfg_region();
const char* cfg_lz4_dec();
const char* cfg_xz_opt();
const char* cfg_bz2();
// Per-device facts and settings, made once per device under a lock (the
// zcg_multi_* calls launch from one host thread per device): the current
// device's CU count, and a kernel's dynamic-LDS limit raised to `bytes`.
uint32_t device_cu_count();
hipError_t lds_attr_once(const void* kernel, int bytes);
// a second stream of the current device (created once; nullptr if that failed):
// kernels of one call that may run side by side are forked onto it
hipError_t launch_raw(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n, int32_t* d_status,
                      uint64_t* d_out_len, int encode, hipStream_t s);
// side / fork / join: the caller's side stream and events for the
// side-by-side lane+wave run (nullptr side: single stream)
hipError_t launch_lz4_decode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                             int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s,
                             hipStream_t side, hipEvent_t fork, hipEvent_t join);
uint64_t lz4_decode_ws_bytes(const zcg_array* a, uint32_t n);
hipError_t launch_lz4_encode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                             uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                             hipStream_t s);
uint64_t lz4_encode_ws_bytes(const zcg_array* a, uint32_t n);
hipError_t launch_inflate(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                          int32_t* d_status, hipStream_t s);
hipError_t launch_inflate_par(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                              int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s);
uint64_t inflate_par_ws_bytes(const zcg_array* a, uint32_t n);
hipError_t launch_inflate_wave(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                               int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s);
uint64_t inflate_wave_ws_bytes(const zcg_array* a, uint32_t n);
// side/fork/join (optional, nullptr: one stream): the lazy parse of each
// sub-batch runs on the side stream while the next sub-batch's match search
// runs on s (the workspace's side stream, as the LZ4 decoder uses it)
hipError_t launch_deflate(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                          uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                          hipStream_t s, hipStream_t side = nullptr, hipEvent_t fork = nullptr,
                          hipEvent_t join = nullptr);
uint64_t deflate_ws_bytes(const zcg_array* a, uint32_t n);
hipError_t launch_bzip2_decode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                               int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s);
uint64_t bzip2_decode_ws_bytes(const zcg_array* a, uint32_t n);
hipError_t launch_bzip2_encode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                               uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                               hipStream_t s);
uint64_t bzip2_encode_ws_bytes(const zcg_array* a, uint32_t n);
hipError_t launch_xz_decode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                            int32_t* d_status, void* ws, uint64_t ws_bytes, hipStream_t s);
uint64_t xz_decode_ws_bytes(const zcg_array* a, uint32_t n);
struct RegionArgs;
hipError_t launch_region(const RegionArgs& a, const void* const* d_table, void* d_out, hipStream_t s);
hipError_t launch_xz_encode(const zcg_array* a, const zcg_chunk* d_chunks, uint32_t n,
                            uint64_t* d_out_len, int32_t* d_status, void* ws, uint64_t ws_bytes,
                            hipStream_t s);
uint64_t xz_encode_ws_bytes(const zcg_array* a, uint32_t n);
}  // namespace zcg
