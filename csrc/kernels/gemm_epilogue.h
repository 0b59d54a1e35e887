// Fused epilogues shared by the engine GEMMs (gemm_stream.hip, gemm_wide.hip, gemm_tiled.hip) and their
// split-K reduction.  Output element (m, n = 16·tile + r) with `partner` = the value of column
// n ^ 8 of the same row (the gate/up or rotary partner under the engine's row permutations).
#pragma once
#include "api.h"

namespace dsse {

constexpr int kPartial = 5;  // internal mode: write fp32 split-K partial slabs part[ks, m, n]

DEV int vperm_tok(int off) { return ((off & 15) >> 2) * 8 + ((off >> 4) & 1) * 4 + (off & 3); }

template <int MODE>
DEV void epilogue(const GemmEpi& ep, float* part, int M, int N, int m, int tile, int r, float v, float partner) {
  if (m >= M) return;
  const int n = tile * 16 + r;
  if constexpr (MODE == kStoreBf16) {
    reinterpret_cast<bf16*>(ep.out)[(size_t)m * ep.ldo + n] = f2bf(v);
  } else if constexpr (MODE == kStoreF32) {
    reinterpret_cast<float*>(ep.out)[(size_t)m * ep.ldo + n] = v;
  } else if constexpr (MODE == kResidAdd) {
    ep.resid[(size_t)m * ep.ldr + n] += v;
  } else if constexpr (MODE == kSiluMul) {
    if (r < 8) reinterpret_cast<bf16*>(ep.out)[(size_t)m * ep.ldo + tile * 8 + r] = f2bf(silu(v) * partner);
  } else if constexpr (MODE == kQkvRope) {
    const int unit = tile >> 3, j = tile & 7;
    const int d = (r < 8) ? (8 * j + r) : (64 + 8 * j + (r - 8));
    if (unit < ep.nh + ep.nkv) {
      const float2 cs = ep.rope[(size_t)DSSE_IDX(ep.positions[m], ep.rope_len, 0) * 64 + 8 * j + (r & 7)];
      const float rot = (r < 8) ? (v * cs.x - partner * cs.y) : (v * cs.x + partner * cs.y);
      if (unit < ep.nh) {
        ep.q_out[(size_t)m * ep.nh * 128 + unit * 128 + d] = f2bf(rot);
      } else {
        const int s = ep.slots[m] < 0 ? -1 : DSSE_IDX(ep.slots[m], ep.num_slots, -1);
        if (s >= 0) {
          const int h = unit - ep.nh, blk = s / kBS, off = s % kBS;
          ep.k_cache[(((size_t)blk * ep.nkv + h) * kBS + off) * 128 + d] = f2bf(rot);
        }
      }
    } else {
      const int s = ep.slots[m] < 0 ? -1 : DSSE_IDX(ep.slots[m], ep.num_slots, -1);
      if (s >= 0) {
        const int h = unit - ep.nh - ep.nkv, blk = s / kBS, off = s % kBS;
        ep.v_cache[(((size_t)blk * ep.nkv + h) * 128 + d) * kBS + vperm_tok(off)] = f2bf(v);
      }
    }
  } else {  // kPartial
    part[(size_t)m * N + n] = v;
  }
}

// SiLU·mul epilogue of one 16x16 accumulator (rows m0 + i, i = 0..3, column 16·tile + r) for the 16x16x32 MFMA
// layout: lanes r < 8 hold gate columns, lanes r >= 8 the matching up columns (partner = lane ^ 8).  After the
// exchange both lanes of a pair hold the four (gate, up) pairs; the low lane finishes rows 0-1 and the high lane
// rows 2-3, so every lane does useful SiLU work (the per-element form ran it on half the lanes).
DEV void silu_epilogue4(const GemmEpi& ep, int M, int m0, int tile, int r, const f32x4& v) {
  float p[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) p[i] = __shfl_xor(v[i], 8);
  const bool lo = r < 8;
  bf16* out = reinterpret_cast<bf16*>(ep.out) + tile * 8 + (r & 7);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float gate = lo ? v[k] : p[2 + k], up = lo ? p[k] : v[2 + k];
    const int m = m0 + (lo ? k : 2 + k);
    if (m < M) out[(size_t)m * ep.ldo] = f2bf(silu(gate) * up);
  }
}

// Sum the S partial slabs and apply the epilogue.  One thread per (row, 16-column tile, j < 8):
// it owns columns tile*16 + j and tile*16 + 8 + j (the epilogue partners).
template <int MODE>
__global__ void __launch_bounds__(256)
splitk_reduce_kernel(const float* __restrict__ part, int S, int M, int N, GemmEpi ep) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int tiles = N / 16;
  if (idx >= M * tiles * 8) return;
  const int j = idx & 7, tile = (idx >> 3) % tiles, m = (idx >> 3) / tiles;
  const size_t base = (size_t)m * N + tile * 16 + j;
  float a = 0.f, b = 0.f;
  for (int s = 0; s < S; ++s) {
    a += part[(size_t)s * M * N + base];
    b += part[(size_t)s * M * N + base + 8];
  }
  epilogue<MODE>(ep, nullptr, M, N, m, tile, j, a, b);
  epilogue<MODE>(ep, nullptr, M, N, m, tile, j + 8, b, a);
}

// Launch the reduction of S slabs for `mode` (shared by both split-K GEMM launchers).
inline hipError_t launch_splitk_reduce(int mode, const float* part, int S, int M, int N, const GemmEpi& ep,
                                       hipStream_t st) {
  const int threads = M * (N / 16) * 8;
  const dim3 grid((threads + 255) / 256), block(256);
  switch (mode) {
    case kStoreBf16: hipLaunchKernelGGL(splitk_reduce_kernel<kStoreBf16>, grid, block, 0, st, part, S, M, N, ep); break;
    case kStoreF32: hipLaunchKernelGGL(splitk_reduce_kernel<kStoreF32>, grid, block, 0, st, part, S, M, N, ep); break;
    case kResidAdd: hipLaunchKernelGGL(splitk_reduce_kernel<kResidAdd>, grid, block, 0, st, part, S, M, N, ep); break;
    case kSiluMul: hipLaunchKernelGGL(splitk_reduce_kernel<kSiluMul>, grid, block, 0, st, part, S, M, N, ep); break;
    case kQkvRope: hipLaunchKernelGGL(splitk_reduce_kernel<kQkvRope>, grid, block, 0, st, part, S, M, N, ep); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dsse
