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
#include "gemm_epilogue.h"

namespace dsse {

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
    // tiled weights: the 4 KiB block of (16-row tile, K-chunk) is contiguous and each of the four
    // loads below reads one contiguous 1 KiB of it across the wave
    const bf16* base = W + ((size_t)(tg * NT) * (K >> 7) + (k0 >> 7) + c) * kTileChunk + lane * 8;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#if DSSE_W_NT
        wf[t][s] = ld_nt_bf16x8(base + (size_t)t * (K >> 7) * kTileChunk + 512 * s);
#else
        wf[t][s] = ld_bf16x8(base + (size_t)t * (K >> 7) * kTileChunk + 512 * s);
#endif
      }
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

// Split-K partial slabs only (no reduce): part[S, M, N]; the consumer (e.g. the fused
// residual-add + RMSNorm kernel) performs the reduction.
extern "C" hipError_t dsse_gemm_xlds_partial(int mt, int nt, int nw, int depth, int Ks, int tg, const void* X, int ldx,
                                             int M, const void* W, int K, int N, float* part, hipStream_t st) {
  using namespace dsse;
  GemmEpi ep{};
  return launch_x_mode<kPartial>(mt, nt, nw, depth, reinterpret_cast<const bf16*>(X), ldx, M,
                                 reinterpret_cast<const bf16*>(W), K, N, Ks, tg, ep, part, st);
}

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
  return launch_splitk_reduce(mode, part, S, M, N, *ep, st);
}

DSSE_CHECK_READER(dsse_check_gemm_xlds)
