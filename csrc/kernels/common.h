// Shared device helpers for the gfx950 (CDNA4) kernels of the decode engine.
//
// Conventions used by every kernel in this directory:
//   * wave = 64 lanes; lane l is split as r = l & 15 (column / row inside a 16-wide MFMA tile)
//     and g = l >> 4 (lane group 0..3), matching the operand maps of
//     v_mfma_f32_16x16x32_bf16:  A[row r][k = 8g + j], B[k = 8g + j][col r],
//     C/D[row 4g + i][col r] (i = 0..3).
//   * bf16 tensors are raw __bf16; 16-byte vectors are bf16x8 (one MFMA operand fragment).
//   * Every kernel takes an explicit hipStream_t from the caller (torch's current stream),
//     so the whole decode step can be captured into one hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define DEV __device__ __forceinline__

namespace dsse {

constexpr int kWave = 64;

DEV float bf2f(bf16 x) { return (float)x; }
DEV bf16 f2bf(float x) { return (bf16)x; }

DEV f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

DEV bf16x8 ld_bf16x8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

DEV bf16x8 zero_bf16x8() {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (bf16)0.0f;
  return z;
}

// Buffer descriptor over [base, base + bytes) (wave-uniform inputs): raw buffer loads past `bytes` return zeros
// without touching memory, so a prefetch ring can run past the end of its range for free.
constexpr int kAuxNT = 2;  // buffer-load cache policy bits: non-temporal (streamed-once data)
DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <int AUX>
DEV bf16x8 ld_buf_bf16x8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}


// Non-temporal 16-byte load for once-read streams (weights, KV pages).
DEV bf16x8 ld_nt_bf16x8(const bf16* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p));
}

template <typename T>
DEV T wave_max(T v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
template <typename T>
DEV T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// 16-byte chunk swizzle inside each 256-byte window of an LDS row: conflict-free ds_read_b128 for the
// MFMA operand pattern "lane l reads row l & 15, chunk 4 (l >> 4) + s" (X tiles of the decode GEMMs,
// K tiles of the flash prefill).  Apply as chunk ^ swz(row & 15) on both the write and the read.
DEV int swz(int row) { return row ^ ((((row >> 2) ^ (row >> 3)) & 1) << 2); }

// Max / sum over the four 16-lane rows of a wave (lanes r, r+16, r+32, r+48: the xor-16 and xor-32 partners)
// with the gfx950 row swaps v_permlane16_swap / v_permlane32_swap -- VALU, no ds_bpermute round trip.
DEV float rows4_max(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  float a = __uint_as_float(p[0]), b = __uint_as_float(p[1]);
  v = a > b ? a : b;
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(q[0]);
  b = __uint_as_float(q[1]);
  return a > b ? a : b;
}
DEV float rows4_sum(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

DEV float silu(float x) { return x / (1.0f + __expf(-x)); }

// Philox4x32-10 counter-based RNG (one 32-bit output used per call site).
DEV uint4 philox4x32(uint4 ctr, uint2 key) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += 0x9E3779B9u;
    key.y += 0xBB67AE85u;
  }
  return ctr;
}
// Uniform in (0, 1]: never exactly 0 so -log(-log(u)) is finite.
DEV float u01(uint32_t x) { return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f); }

// ---- checked build (DSSE_KERNEL_CHECKS=1, `_build.py kernels-checked`) -----------------------------
// Data-dependent indices the host cannot validate without a sync (block-table entries, KV slots, token
// ids, RoPE positions, sampled ids) go through DSSE_IDX(v, bound, fallback).  In the checked build an
// out-of-range value is recorded in this translation unit's g_check word (first violation: line, value,
// bound; plus a count) and replaced by `fallback`, so the kernel never touches memory it does not own
// and the GPU never faults; the host reads the words back with torch.ops.dsse.kernel_checks().  In the
// default build DSSE_IDX is the identity and costs nothing.
#if DSSE_KERNEL_CHECKS
static __device__ int g_check[4];
DEV int check_index(int v, int bound, int line, int fallback) {
  if ((unsigned)v < (unsigned)bound) return v;
  if (atomicCAS(&g_check[0], 0, line) == 0) {
    g_check[1] = v;
    g_check[2] = bound;
  }
  atomicAdd(&g_check[3], 1);
  return fallback;
}
#define DSSE_IDX(v, bound, fallback) ::dsse::check_index((v), (bound), __LINE__, (fallback))
#define DSSE_CHECK_READER(fn)                                                              \
  extern "C" hipError_t fn(int* out, int clear) {                                          \
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(::dsse::g_check), 4 * sizeof(int)); \
    if (e == hipSuccess && clear) {                                                        \
      const int z[4] = {0, 0, 0, 0};                                                       \
      e = hipMemcpyToSymbol(HIP_SYMBOL(::dsse::g_check), z, sizeof z);                     \
    }                                                                                      \
    return e;                                                                              \
  }
#else
#define DSSE_IDX(v, bound, fallback) (v)
#define DSSE_CHECK_READER(fn)                         \
  extern "C" hipError_t fn(int* out, int) {           \
    for (int i = 0; i < 4; ++i) out[i] = 0;           \
    return hipSuccess;                                \
  }
#endif

// ---- Step anatomy stamps (diagnostic `stamps` build only, DSSE_PIPE_STAMPS; tools/step_stamps.py).  Per-wave
// records of s_memrealtime (100 MHz, one clock for every CU): [tag, grid x | grid y << 32, block x | block y << 32,
// t0 entry, t1 first operands landed, t2 main loop done, t3 stores drained, wave] appended to a per-translation-unit
// device buffer that the host binds (torch.ops.dsse.step_stamps_*).  The buffer is kStampSubs sub-buffers, chosen
// by the workgroup's linear index, each with its own counter on its own 64-byte line: one shared counter for every
// wave of the chip serialised the waves' exits and stretched the kernels it measured.  Word 0 is the capacity per
// sub-buffer.  In the default build every call below compiles to nothing.
#ifndef DSSE_PIPE_STAMPS
#define DSSE_PIPE_STAMPS 0
#endif
namespace stamps {
enum Tag { kRing = 1, kNorm = 2, kAttn = 3, kPipe = 4 };
constexpr int kSubs = 256;
constexpr int kHeader = 8 + 8 * kSubs;  // u64 words before the first sub-buffer
DEV unsigned long long now() {
#if DSSE_PIPE_STAMPS
  return __builtin_amdgcn_s_memrealtime();
#else
  return 0ull;
#endif
}
#if DSSE_PIPE_STAMPS
static __device__ unsigned long long* g_rec;
#endif
// t3 is taken here, after this wave's stores drained (vmcnt(0)); call from every wave, after its last store
DEV void record(int tag, unsigned long long t0, unsigned long long t1, unsigned long long t2) {
#if DSSE_PIPE_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t3 = now();
  unsigned long long* rec = g_rec;
  if ((threadIdx.x & 63) == 0 && rec) {
    const unsigned sub = (blockIdx.x + blockIdx.y * gridDim.x) % kSubs;
    const unsigned long long cap = rec[0];
    const unsigned long long n = atomicAdd(rec + 8 + 8 * sub, 1ull);
    if (n < cap) {
      unsigned long long* r = rec + kHeader + (sub * cap + n) * 8;
      r[0] = (unsigned long long)tag;
      r[1] = gridDim.x | ((unsigned long long)gridDim.y << 32);
      r[2] = blockIdx.x | ((unsigned long long)blockIdx.y << 32);
      r[3] = t0;
      r[4] = t1;
      r[5] = t2;
      r[6] = t3;
      r[7] = threadIdx.x >> 6;
    }
  }
#endif
}
}  // namespace stamps
#if DSSE_PIPE_STAMPS
#define DSSE_STAMPS_BINDER(fn)                                                                  \
  extern "C" hipError_t fn(void* p) {                                                            \
    return hipMemcpyToSymbol(HIP_SYMBOL(::dsse::stamps::g_rec), &p, sizeof(p));                 \
  }
#else
#define DSSE_STAMPS_BINDER(fn) \
  extern "C" hipError_t fn(void*) { return hipSuccess; }
#endif

}  // namespace dsse
