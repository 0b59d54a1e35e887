// Decode GEMM with the activations resident in LDS:  Y[M, N] = X[M, K] · W[N, K]ᵀ, M <= 64.
//
// Why (measured, tools/tune_gemm.py, profiles/gemm_sweep_r1.md): the register-streaming kernel in
// gemm_skinny.hip reaches ~6 TB/s at M = 1 but falls to 1.6 TB/s at M = 64, because every 16-column
// workgroup re-reads the whole X (64 x K) from L2 — 4 bytes of X per byte of weights.  Here a
// workgroup stages a K-slice of X ONCE into LDS and its waves then stream many 16-column weight
// tiles past it, so X costs LDS bandwidth (which has ~20x headroom) instead of L2/TA bandwidth.
//
//   grid.y = S K-slices of Ks columns (Ks = 128 KiB of LDS / (16·MT rows · 2 B) by default),
//   grid.x = groups of `tg_per_wg` tile-groups (NT tiles of 16 columns each) per workgroup,
//   wave w of a workgroup owns tile-groups w, w + NW, ... of its range over the whole K-slice —
//   no cross-wave reduction.  Weights stream HBM -> VGPRs through a 4-deep register ring
//   (4 x 64 B per lane per K-chunk of 128 in flight); X fragments come from LDS with
//   ds_read_b128 through a bank-conflict-free XOR swizzle of 16-byte chunks.
//   S == 1: the fused epilogue of gemm_skinny.hip (bf16 / fp32 / residual add / SiLU·mul /
//   RoPE + paged KV write) runs in the workgroup; S > 1: fp32 partials [S, M, N] are reduced by
//   splitk_reduce_kernel, which applies the same epilogue.
#include "api.h"

namespace dsse {

constexpr int kPartial = 5;  // internal mode: write fp32 split-K partial slabs

DEV int vperm2(int off) { return ((off & 15) >> 2) * 8 + ((off >> 4) & 1) * 4 + (off & 3); }

// 16-byte chunk swizzle inside each 256-byte window of an LDS row: conflict-free ds_read_b128 for
// the MFMA A-operand pattern (lane l reads row l & 15, chunk 4(l >> 4) + s).
DEV int swz(int row) { return row ^ ((((row >> 2) ^ (row >> 3)) & 1) << 2); }

// One output element with its epilogue.  `partner` = the value 8 lanes away (same row, paired column).
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
      const float2 cs = ep.rope[(size_t)ep.positions[m] * 64 + 8 * j + (r & 7)];
      const float rot = (r < 8) ? (v * cs.x - partner * cs.y) : (v * cs.x + partner * cs.y);
      if (unit < ep.nh) {
        ep.q_out[(size_t)m * ep.nh * 128 + unit * 128 + d] = f2bf(rot);
      } else {
        const int s = ep.slots[m];
        if (s >= 0) {
          const int h = unit - ep.nh, blk = s / kBS, off = s % kBS;
          ep.k_cache[(((size_t)blk * ep.nkv + h) * kBS + off) * 128 + d] = f2bf(rot);
        }
      }
    } else {
      const int s = ep.slots[m];
      if (s >= 0) {
        const int h = unit - ep.nh - ep.nkv, blk = s / kBS, off = s % kBS;
        ep.v_cache[(((size_t)blk * ep.nkv + h) * 128 + d) * kBS + vperm2(off)] = f2bf(v);
      }
    }
  } else {  // kPartial: part[(ks, m, n)]
    part[(size_t)m * N + n] = v;
  }
}

template <int MT, int NT, int NW, int DEPTH, int MODE>
__global__ void __launch_bounds__(64 * NW)
gemm_xlds_kernel(const bf16* __restrict__ X, int ldx, int M, const bf16* __restrict__ W, int K, int N,
                 int Ks, int tg_per_wg, GemmEpi ep, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int MP = 16 * MT;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int ks = blockIdx.y;
  const int k0 = ks * Ks;
  const int kl = min(Ks, K - k0);  // multiple of 128
  const int row_bytes = kl * 2;

  const int TG = N / (16 * NT);
  const int g_lo = blockIdx.x * tg_per_wg;
  const int g_hi = min(TG, g_lo + tg_per_wg);
  const int my_first = g_lo + w;
  const int ntg = my_first < g_hi ? (g_hi - my_first + NW - 1) / NW : 0;
  const int cpt = kl >> 7;  // K-chunks of 128 per tile
  const int U = ntg * cpt;

  // unit u = (tile-group my_first + (u / cpt) * NW, K-chunk u % cpt); loads past the end are
  // clamped to the last unit (harmless re-reads) so every load is unconditional.
  auto load_unit = [&](int u, bf16x8 (&wf)[NT][4]) {
    const int uu = min(u, U - 1);
    const int tg = my_first + (uu / cpt) * NW, c = uu % cpt;
    const bf16* base = W + (size_t)(tg * 16 * NT + r) * K + k0 + (c << 7) + 32 * g;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) wf[t][s] = ld_bf16x8(base + (size_t)16 * t * K + 8 * s);
  };

  // Weight ring: DEPTH chunks of 4 x 16 B per lane per tile.  The first DEPTH-1 loads are issued
  // before the X staging so the HBM stream starts at once.
  bf16x8 ring[DEPTH][NT][4];
  if (U > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH - 1; ++d) load_unit(d, ring[d]);
  }

  // ---- stage X[0:MP, k0:k0+kl] into LDS (rows >= M replicate row M-1; their outputs are dropped)
  {
    const int cpr = kl >> 3;  // 16-byte chunks per row
    for (int idx = threadIdx.x; idx < MP * cpr; idx += 64 * NW) {
      const int row = idx / cpr, c = idx - row * cpr;
      const bf16x8 v = ld_bf16x8(X + (size_t)min(row, M - 1) * ldx + k0 + 8 * c);
      const int dst = row * row_bytes + ((c >> 4) << 8) + (((c & 15) ^ swz(row & 15)) << 4);
      *reinterpret_cast<bf16x8*>(smem + dst) = v;
    }
  }
  __syncthreads();
  if (U == 0) return;

  float* part_ks = part ? part + (size_t)ks * M * N : nullptr;
  f32x4 acc[MT][NT];
  auto compute = [&](int u, const bf16x8 (&wf)[NT][4]) {
    const int tg = my_first + (u / cpt) * NW, c = u % cpt;
    if (c == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const char* xb = smem + (c << 8);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ch = ((4 * g + s) ^ swz(r)) << 4;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xb + (16 * mt + r) * row_bytes + ch);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16x16x32(xf, wf[t][s], acc[mt][t]);
      }
    }
    if (c == cpt - 1) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float v = acc[mt][t][i];
            const float partner = (MODE == kSiluMul || MODE == kQkvRope) ? __shfl_xor(v, 8) : 0.f;
            epilogue<MODE>(ep, part_ks, M, N, 16 * mt + 4 * g + i, tg * NT + t, r, v, partner);
          }
    }
  };

  for (int u0 = 0; u0 < U; u0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (u0 + d >= U) break;
      load_unit(u0 + d + DEPTH - 1, ring[(d + DEPTH - 1) % DEPTH]);
      compute(u0 + d, ring[d]);
    }
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

template <int MT, int NT, int NW, int DEPTH, int MODE>
static hipError_t launch_x(const bf16* X, int ldx, int M, const bf16* W, int K, int N, int Ks, int tg,
                           const GemmEpi& ep, float* part, hipStream_t st) {
  const int S = (K + Ks - 1) / Ks;
  const int TG = N / (16 * NT);
  const size_t lds = (size_t)16 * MT * Ks * 2;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_xlds_kernel<MT, NT, NW, DEPTH, MODE>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  dim3 grid((TG + tg - 1) / tg, S), block(64 * NW);
  hipLaunchKernelGGL((gemm_xlds_kernel<MT, NT, NW, DEPTH, MODE>), grid, block, lds, st, X, ldx, M, W, K, N, Ks, tg, ep,
                     part);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_x_mode(int mt, int nt, int nw, int depth, const bf16* X, int ldx, int M, const bf16* W, int K, int N,
                                int Ks, int tg, const GemmEpi& ep, float* part, hipStream_t st) {
#define DSSE_X_CASE(MT_, NT_, NW_, D_)                                                                \
  if (mt == MT_ && nt == NT_ && nw == NW_ && depth == D_)                                               \
    return launch_x<MT_, NT_, NW_, D_, MODE>(X, ldx, M, W, K, N, Ks, tg, ep, part, st);
#define DSSE_X_MT(MT_)                                                                                  \
  DSSE_X_CASE(MT_, 1, 4, 4) DSSE_X_CASE(MT_, 1, 8, 4) DSSE_X_CASE(MT_, 2, 8, 4) DSSE_X_CASE(MT_, 1, 8, 8) \
  DSSE_X_CASE(MT_, 1, 4, 8)
  DSSE_X_MT(1) DSSE_X_MT(2) DSSE_X_MT(4)
#undef DSSE_X_MT
#undef DSSE_X_CASE
  return hipErrorInvalidValue;
}

}  // namespace dsse

// X-in-LDS decode GEMM.  part: fp32 workspace of S * M * N floats when Ks < K (S > 1), else unused.
extern "C" hipError_t dsse_gemm_xlds(int mode, int mt, int nt, int nw, int depth, int Ks, int tg, const void* X, int ldx,
                                     int M, const void* W, int K, int N, const dsse::GemmEpi* ep, float* part,
                                     hipStream_t st) {
  using namespace dsse;
  const bf16* x = reinterpret_cast<const bf16*>(X);
  const bf16* w = reinterpret_cast<const bf16*>(W);
  const int S = (K + Ks - 1) / Ks;
  if (S == 1) {
    switch (mode) {
      case kStoreBf16: return launch_x_mode<kStoreBf16>(mt, nt, nw, depth, x, ldx, M, w, K, N, Ks, tg, *ep, nullptr, st);
      case kStoreF32: return launch_x_mode<kStoreF32>(mt, nt, nw, depth, x, ldx, M, w, K, N, Ks, tg, *ep, nullptr, st);
      case kResidAdd: return launch_x_mode<kResidAdd>(mt, nt, nw, depth, x, ldx, M, w, K, N, Ks, tg, *ep, nullptr, st);
      case kSiluMul: return launch_x_mode<kSiluMul>(mt, nt, nw, depth, x, ldx, M, w, K, N, Ks, tg, *ep, nullptr, st);
      case kQkvRope: return launch_x_mode<kQkvRope>(mt, nt, nw, depth, x, ldx, M, w, K, N, Ks, tg, *ep, nullptr, st);
    }
    return hipErrorInvalidValue;
  }
  hipError_t e = launch_x_mode<kPartial>(mt, nt, nw, depth, x, ldx, M, w, K, N, Ks, tg, *ep, part, st);
  if (e != hipSuccess) return e;
  const int threads = M * (N / 16) * 8;
  const dim3 grid((threads + 255) / 256), block(256);
  switch (mode) {
    case kStoreBf16: hipLaunchKernelGGL(splitk_reduce_kernel<kStoreBf16>, grid, block, 0, st, part, S, M, N, *ep); break;
    case kStoreF32: hipLaunchKernelGGL(splitk_reduce_kernel<kStoreF32>, grid, block, 0, st, part, S, M, N, *ep); break;
    case kResidAdd: hipLaunchKernelGGL(splitk_reduce_kernel<kResidAdd>, grid, block, 0, st, part, S, M, N, *ep); break;
    case kSiluMul: hipLaunchKernelGGL(splitk_reduce_kernel<kSiluMul>, grid, block, 0, st, part, S, M, N, *ep); break;
    case kQkvRope: hipLaunchKernelGGL(splitk_reduce_kernel<kQkvRope>, grid, block, 0, st, part, S, M, N, *ep); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
