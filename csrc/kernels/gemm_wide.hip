// Wide-batch decode GEMM on 32x32x16 MFMAs:  Y[M, N] = X[M, K] · W[N, K]ᵀ for 64 < M <= 256 rows.
//
// At 128-256 decode rows (BASELINE config 3: 256 streams per GPU) a weight byte feeds up to 256 rows and
// the 16x16x32 X-streaming kernel (gemm_stream.hip, MT = 16) becomes LDS-bound: every X fragment it reads
// from LDS feeds one 16-column MFMA.  hipBLASLt reaches 940 TFLOP/s on gate_up but only 300-470 on the
// narrow projections, where its 128x256 / 64x64 tiles leave most CUs idle (profiles/blas_shapes_r1.log).
//
// Here a wave owns a 32-column strip of the output for all 32·MB rows (MB accumulators of 32x32 f32) and
// streams its strip of the tiled weights (api.h kTileChunk) from HBM exactly once per K range; each X
// fragment read from LDS feeds a 32x32x16 MFMA (32 cycles), so a wave's LDS traffic per MFMA cycle is
// half that of the 16x16 kernel.  X flows through two LDS slices (double-buffered, one barrier per slice)
// as in gemm_stream.  Four waves per workgroup (one per SIMD, up to 512 VGPRs each) cover 128 columns;
// narrow projections split K over workgroups (grid.y = S) into fp32 slabs [S, M, N] that the consumer
// reduces (the residual RMSNorm, or splitk_reduce_kernel for the fused epilogues).
//
// Operand maps (v_mfma_f32_32x32x16_bf16): lane l = n + 32h holds A[row n][k = 8h + j] and
// B[k = 8h + j][col n]; C/D register i of lane l is [row (i & 3) + 8 (i >> 2) + 4h][col n].
// The contraction order inside a 128-deep K chunk is permuted identically for X and W: k-step q of half h
// covers elements 32g + 8s + j with g = 2 (q >> 2) + h, s = q & 3 — exactly one 16-byte piece of the tiled
// weight chunk ([s][lane = r + 16g][j]), so each weight load instruction reads 2 x 512 contiguous bytes.
#include "gemm_epilogue.h"

namespace dsse {

typedef float f32x16 __attribute__((ext_vector_type(16)));

DEV f32x16 mfma32x32x16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

constexpr int wide_cps(int mb) { return mb >= 8 ? 1 : 2; }  // K chunks per LDS slice: 2 x 64 KiB of X

template <int MB, int NW, int RD, int MODE>
__global__ void __launch_bounds__(64 * NW)
gemm_wide_kernel(const bf16* __restrict__ X, int ldx, int M, const bf16* __restrict__ W, int K, int N, int Kr,
                 GemmEpi ep, float* __restrict__ part) {
  constexpr int CPS = wide_cps(MB);
  constexpr int MP = 32 * MB;
  constexpr int ROWB = CPS * 256;   // bytes of one X row in a slice
  constexpr int BUF = MP * ROWB;    // bytes per slice buffer
  constexpr int UPR = CPS * 16;     // 16-byte units per X row in a slice
  constexpr int PPT = (MP * UPR + 64 * NW - 1) / (64 * NW);
  constexpr int DEPTH = CPS * RD;   // weight ring (chunks)
  constexpr int QG = MB >= 8 ? 1 : 4;  // k-steps whose X fragments are read from LDS at once
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n32 = lane & 31, h = lane >> 5;
  int cg = blockIdx.x, ks = blockIdx.y;
  if (gridDim.y > 1 && 8 % gridDim.y == 0 && (gridDim.x * gridDim.y) % 8 == 0) {
    // split-K: each K range on 8/S XCDs (as gemm_stream.hip), so an XCD's L2 fetches only its range of X
    const int lin = blockIdx.y * gridDim.x + blockIdx.x, xcd = lin % 8, slot = lin / 8, per = 8 / gridDim.y;
    ks = xcd / per;
    cg = slot * per + xcd % per;
  }
  const int strip = cg * NW + w;  // host guarantees N % (32 NW) == 0
  const int k0 = ks * Kr;
  const int nch = Kr >> 7;  // multiple of CPS (host-checked)
  const int nsl = nch / CPS;
  const int KC = K >> 7;

  // One range-checked descriptor over all of W: the ring's look-ahead issues past this wave's K range get an
  // out-of-range offset and return zeros without memory traffic (clamping them re-fetched the last chunk).
  const __amdgpu_buffer_rsrc_t wrs = make_rsrc(W, (uint32_t)((size_t)N * K * 2));
  const uint32_t wbase = (uint32_t)((((size_t)(2 * strip + (n32 >> 4)) * KC + (k0 >> 7)) * kTileChunk + (n32 & 15) * 8) * 2);
  auto load_w = [&](int c, bf16x8 (&wf)[8]) {
    const uint32_t p = c < nch ? wbase + (uint32_t)c * (kTileChunk * 2) : 0xFFFFF000u;
#pragma unroll
    for (int q = 0; q < 8; ++q) wf[q] = ld_buf_bf16x8<kAuxNT>(wrs, p + ((q & 3) * 64 + 16 * (2 * (q >> 2) + h)) * 16);
  };

  // X pieces: every thread loads PPT pieces unconditionally (rows past M re-read row M - 1; those LDS rows
  // only feed output rows that are never stored).  A runtime bound on each load made hipcc branch around
  // it and wait vmcnt(0), draining the weight ring every slice.
  static_assert((MP * UPR) % (64 * NW) == 0, "X slice must split evenly over the workgroup");
  bf16x8 xs[PPT];
  auto load_x = [&](int sl) {
    const bf16* src = X + k0 + sl * (CPS * 128);
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int idx = threadIdx.x + i * 64 * NW;
      xs[i] = ld_bf16x8(src + (size_t)min(idx / UPR, M - 1) * ldx + 8 * (idx % UPR));
    }
  };
  // unit u of row `row` lives at 16-byte slot u ^ (row & 15) of its 256-byte window: the A-fragment read
  // (32 lanes = 32 consecutive rows, one unit) then hits 16 distinct slots in every ds_read_b128 lane group
  auto store_x = [&](int buf) {
    char* dst = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int idx = threadIdx.x + i * 64 * NW;
      const int row = idx / UPR, c = idx % UPR;
      *reinterpret_cast<bf16x8*>(dst + row * ROWB + ((c >> 4) << 8) + (((c & 15) ^ (row & 15)) << 4)) = xs[i];
    }
  };

  bf16x8 ring[DEPTH][8];
#pragma unroll
  for (int d = 0; d < DEPTH - 1; ++d) load_w(d, ring[d]);
  load_x(0);
  store_x(0);

  f32x16 acc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[mb][i] = 0.f;

  const int sw = n32 & 15;
  for (int sl0 = 0; sl0 < nsl; sl0 += RD) {
#pragma unroll
    for (int hh = 0; hh < RD; ++hh) {
      const int sl = sl0 + hh;
      if (hh > 0 && sl >= nsl) break;
      __syncthreads();  // slice sl visible; everyone is done reading slice sl - 1's buffer
      // unconditional (the last slice re-loads itself into the idle buffer): a branch around these loads
      // made hipcc wait vmcnt(0) at the join, draining the weight ring once per slice
      load_x(min(sl + 1, nsl - 1));
      const char* xb0 = smem + (sl & 1) * BUF + n32 * ROWB;
#pragma unroll
      for (int d = 0; d < CPS; ++d) {
        const int slot = hh * CPS + d;
        load_w(sl * CPS + d + DEPTH - 1, ring[(slot + DEPTH - 1) % DEPTH]);
        const char* xb = xb0 + (d << 8);
#pragma unroll
        for (int q0 = 0; q0 < 8; q0 += QG) {
          bf16x8 xf[QG][MB];
#pragma unroll
          for (int qq = 0; qq < QG; ++qq) {
            const int q = q0 + qq;
            const int u = 4 * (2 * (q >> 2) + h) + (q & 3);
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
              xf[qq][mb] = *reinterpret_cast<const bf16x8*>(xb + mb * 32 * ROWB + ((u ^ sw) << 4));
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int qq = 0; qq < QG; ++qq)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb) acc[mb] = mfma32x32x16(xf[qq][mb], ring[slot][q0 + qq], acc[mb]);
        }
      }
      store_x((sl + 1) & 1);
    }
  }

  float* part_ks = part ? part + (size_t)ks * M * N : nullptr;
  const int tile = 2 * strip + (n32 >> 4), r = n32 & 15;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = acc[mb][i];
      const float partner = (MODE == kSiluMul || MODE == kQkvRope) ? __shfl_xor(v, 8) : 0.f;
      epilogue<MODE>(ep, part_ks, M, N, 32 * mb + (i & 3) + 8 * (i >> 2) + 4 * h, tile, r, v, partner);
    }
}

template <int MB, int RD, int MODE>
static hipError_t launch_w(const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S, const GemmEpi& ep,
                           float* part, hipStream_t st) {
  constexpr int NW = 4;
  const size_t lds = (size_t)2 * 32 * MB * wide_cps(MB) * 256;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_wide_kernel<MB, NW, RD, MODE>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  dim3 grid(N / (32 * NW), S), block(64 * NW);
  hipLaunchKernelGGL((gemm_wide_kernel<MB, NW, RD, MODE>), grid, block, lds, st, X, ldx, M, W, K, N, K / S, ep, part);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_w_mode(int mb, int rd, const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S,
                                const GemmEpi& ep, float* part, hipStream_t st) {
  if (mb == 8 && rd == 2) return launch_w<8, 2, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  if (mb == 8 && rd == 3) return launch_w<8, 3, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  if (mb == 4 && rd == 1) return launch_w<4, 1, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  if (mb == 4 && rd == 2) return launch_w<4, 2, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  return hipErrorInvalidValue;
}

}  // namespace dsse

// Shape contract (checked by the caller): M <= 32 mb (mb 4 or 8), N % 128 == 0,
// K % (128 · cps · S) == 0 with cps = 2 (mb 4) / 1 (mb 8).  rd: weight ring depth in LDS slices
// (mb 8: 2 or 3 chunks; mb 4: 1 or 2 slices of 2 chunks).  part: fp32 [S, M, N] when S > 1;
// partial_only leaves the slabs for the consumer.
extern "C" hipError_t dsse_gemm_wide(int mode, int mb, int rd, int S, int partial_only, const void* X, int ldx, int M,
                                     const void* W, int K, int N, const dsse::GemmEpi* ep, float* part,
                                     hipStream_t st) {
  using namespace dsse;
  const bf16* x = reinterpret_cast<const bf16*>(X);
  const bf16* w = reinterpret_cast<const bf16*>(W);
  if (S == 1 && !partial_only) {
    switch (mode) {
      case kStoreBf16: return launch_w_mode<kStoreBf16>(mb, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kStoreF32: return launch_w_mode<kStoreF32>(mb, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kResidAdd: return launch_w_mode<kResidAdd>(mb, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kSiluMul: return launch_w_mode<kSiluMul>(mb, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kQkvRope: return launch_w_mode<kQkvRope>(mb, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
    }
    return hipErrorInvalidValue;
  }
  hipError_t e = launch_w_mode<kPartial>(mb, rd, x, ldx, M, w, K, N, S, *ep, part, st);
  if (e != hipSuccess || partial_only) return e;
  return launch_splitk_reduce(mode, part, S, M, N, *ep, st);
}
