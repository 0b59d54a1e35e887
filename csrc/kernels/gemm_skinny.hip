// Skinny decode GEMM on MFMA for gfx950:  Y[M, N] = X[M, K] · W[N, K]ᵀ, M <= 64.
//
// This is the weight-streaming hot path of the decode step (K3/K6/K7/K8/K9 of SURVEY.md §2.4):
// every decode step streams all 14.5 GB of Mistral-7B weights once, so each op here must run
// at HBM speed.  Design (MI355X-first, not a CUDA port):
//   * one workgroup owns 16·NT output columns and KW waves split the K dimension between them;
//     partial sums meet in LDS at the end (no cross-workgroup split-K, no atomics), so the
//     workgroup count is N/(16·NT): 384 (QKV), 256 (O, down), 1792 (gate_up), 2048 (LM head).
//   * weights go straight from HBM to VGPRs (guide: "GEMV / M <= 16 decode weights: load
//     straight to VGPRs"); each lane loads 64 contiguous bytes of one weight row per 128-deep
//     K-chunk and feeds four v_mfma_f32_16x16x32_bf16 from them.  The MFMA k-order is permuted
//     (lane group g owns k in [32g, 32g+32) of the chunk) identically for X and W, so every
//     load is a full 64-byte run while the reduction stays exact.
//   * the next chunk is loaded while the current one is multiplied (2-deep register pipeline).
//   * weights come from the tiled layout (api.h kTileChunk) with non-temporal loads: 1 KiB contiguous
//     per load instruction, and the once-read stream does not evict X from L2 (M = 1: 5.5 -> 6.2 TB/s
//     on gate_up, 5.9 -> 6.5 TB/s on the LM head; profiles/gemm_stream_r1.md).
//   * fused epilogues: bf16 store, fp32 store (logits), fp32 residual add (O / down
//     projections), SiLU·mul over gate/up pairs (gate_up), and RoPE + paged-KV-cache write
//     (QKV).  The paired epilogues rely on the engine's weight-row permutation: inside each
//     16-row tile, rows 0..7 and 8..15 are partners (gate/up, or rotary dims d and d+64), so
//     the partner value is one __shfl_xor(·, 8) away.
#include "api.h"

namespace dsse {



// Position of token `off` (0..31) inside a V page row; lane group g of the attention kernel
// then reads tokens {4g..4g+3, 16+4g..16+4g+3} as one 16-byte run.
DEV int vperm(int off) { return ((off & 15) >> 2) * 8 + ((off >> 4) & 1) * 4 + (off & 3); }

template <int MT, int NT>
DEV void load_chunk(bf16x8 (&wf)[NT][4], bf16x8 (&xf)[MT][4], const bf16* const (&wp)[NT],
                    const bf16* const (&xp)[MT], int c) {
  const int off = c << 7;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s) wf[t][s] = ld_nt_bf16x8(wp[t] + (size_t)c * kTileChunk + 512 * s);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int s = 0; s < 4; ++s) xf[mt][s] = ld_bf16x8(xp[mt] + off + 8 * s);
}

template <int MT, int NT>
DEV void mma_chunk(f32x4 (&acc)[MT][NT], const bf16x8 (&wf)[NT][4], const bf16x8 (&xf)[MT][4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16x16x32(xf[mt][s], wf[t][s], acc[mt][t]);
}

template <int MT, int NT, int KW, int MODE>
__global__ void __launch_bounds__(64 * KW)
skinny_gemm_kernel(const bf16* __restrict__ X, int ldx, int M, const bf16* __restrict__ W, int K,
                   int N, GemmEpi ep) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NT;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16* wp[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wp[t] = W + (size_t)((n0 >> 4) + t) * (K >> 7) * kTileChunk + lane * 8;
  const bf16* xp[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = min(16 * mt + r, M - 1);
    xp[mt] = X + (size_t)m * ldx + 32 * g;
  }

  const int nchunks = K >> 7;
  bf16x8 wa[NT][4], xa[MT][4], wb[NT][4], xb[MT][4];
  int c = w;
  if (c < nchunks) load_chunk<MT, NT>(wa, xa, wp, xp, c);
  for (; c < nchunks; c += 2 * KW) {
    if (c + KW < nchunks) load_chunk<MT, NT>(wb, xb, wp, xp, c + KW);
    mma_chunk<MT, NT>(acc, wa, xa);
    if (c + KW >= nchunks) break;
    if (c + 2 * KW < nchunks) load_chunk<MT, NT>(wa, xa, wp, xp, c + 2 * KW);
    mma_chunk<MT, NT>(acc, wb, xb);
  }

  if constexpr (KW > 1) {
    __shared__ float red[KW - 1][MT * NT * 4][64];
    if (w > 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) red[w - 1][(mt * NT + t) * 4 + i][lane] = acc[mt][t][i];
    }
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int v = 0; v < KW - 1; ++v)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[mt][t][i] += red[v][(mt * NT + t) * 4 + i][lane];
  }

  // ---- epilogue (wave 0): element (mt, t, i) is Y[16mt + 4g + i][n0 + 16t + r] ----
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int tile = (n0 >> 4) + t;
      const int n = n0 + 16 * t + r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 16 * mt + 4 * g + i;
        const float v = acc[mt][t][i];
        if constexpr (MODE == kStoreBf16) {
          if (m < M) reinterpret_cast<bf16*>(ep.out)[(size_t)m * ep.ldo + n] = f2bf(v);
        } else if constexpr (MODE == kStoreF32) {
          if (m < M) reinterpret_cast<float*>(ep.out)[(size_t)m * ep.ldo + n] = v;
        } else if constexpr (MODE == kResidAdd) {
          if (m < M) ep.resid[(size_t)m * ep.ldr + n] += v;
        } else if constexpr (MODE == kSiluMul) {
          const float partner = __shfl_xor(v, 8);
          if (r < 8 && m < M)
            reinterpret_cast<bf16*>(ep.out)[(size_t)m * ep.ldo + tile * 8 + r] =
                f2bf(silu(v) * partner);
        } else if constexpr (MODE == kQkvRope) {
          const float partner = __shfl_xor(v, 8);
          const int unit = tile >> 3, j = tile & 7;
          const int d = (r < 8) ? (8 * j + r) : (64 + 8 * j + (r - 8));
          if (m < M) {
            if (unit < ep.nh + ep.nkv) {
              const float2 cs = ep.rope[(size_t)DSSE_IDX(ep.positions[m], ep.rope_len, 0) * 64 + 8 * j + (r & 7)];
              // r < 8: v = x1, partner = x2 -> x1 cos - x2 sin ; r >= 8: v = x2 -> x2 cos + x1 sin
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
                ep.v_cache[(((size_t)blk * ep.nkv + h) * 128 + d) * kBS + vperm(off)] = f2bf(v);
              }
            }
          }
        }
      }
    }
  }
}

template <int MT, int NT, int KW, int MODE>
static hipError_t launch_t(const bf16* X, int ldx, int M, const bf16* W, int K, int N,
                           const GemmEpi& ep, hipStream_t st) {
  dim3 grid(N / (16 * NT)), block(64 * KW);
  hipLaunchKernelGGL((skinny_gemm_kernel<MT, NT, KW, MODE>), grid, block, 0, st, X, ldx, M, W, K,
                     N, ep);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_mode(int mt, int nt, int kw, const bf16* X, int ldx, int M, const bf16* W,
                              int K, int N, const GemmEpi& ep, hipStream_t st) {
#define K_GEMM_CASE(MT_, NT_, KW_) \
  if (mt == MT_ && nt == NT_ && kw == KW_) return launch_t<MT_, NT_, KW_, MODE>(X, ldx, M, W, K, N, ep, st);
#define K_GEMM_MT(MT_) \
  K_GEMM_CASE(MT_, 1, 4) K_GEMM_CASE(MT_, 1, 8) K_GEMM_CASE(MT_, 2, 4) K_GEMM_CASE(MT_, 2, 8)
  K_GEMM_MT(1) K_GEMM_MT(2)
  // MT = 4 (M <= 64): NT = 2 at KW = 8 spills past the 256-VGPR budget of 2 waves/SIMD.
  K_GEMM_CASE(4, 1, 4) K_GEMM_CASE(4, 1, 8) K_GEMM_CASE(4, 2, 4)
#undef K_GEMM_MT
#undef K_GEMM_CASE
  return hipErrorInvalidValue;
}

}  // namespace dsse

// C entry point used by the torch bindings: returns hipSuccess or an error code.  All shape
// constraints (K % 128, N % (16·nt), M <= 16·mt <= 64) are checked by the caller.
extern "C" hipError_t dsse_skinny_gemm(int mode, int mt, int nt, int kw, const void* X, int ldx,
                                       int M, const void* W, int K, int N, const dsse::GemmEpi* ep,
                                       hipStream_t st) {
  using namespace dsse;
  const bf16* x = reinterpret_cast<const bf16*>(X);
  const bf16* w = reinterpret_cast<const bf16*>(W);
  switch (mode) {
    case kStoreBf16: return launch_mode<kStoreBf16>(mt, nt, kw, x, ldx, M, w, K, N, *ep, st);
    case kStoreF32: return launch_mode<kStoreF32>(mt, nt, kw, x, ldx, M, w, K, N, *ep, st);
    case kResidAdd: return launch_mode<kResidAdd>(mt, nt, kw, x, ldx, M, w, K, N, *ep, st);
    case kSiluMul: return launch_mode<kSiluMul>(mt, nt, kw, x, ldx, M, w, K, N, *ep, st);
    case kQkvRope: return launch_mode<kQkvRope>(mt, nt, kw, x, ldx, M, w, K, N, *ep, st);
  }
  return hipErrorInvalidValue;
}

DSSE_CHECK_READER(dsse_check_gemm_skinny)
