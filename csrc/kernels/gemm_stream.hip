// X-streaming decode GEMM:  Y[M, N] = X[M, K] · W[N, K]ᵀ, 16 < M <= 256.
//
// Successor of gemm_xlds.hip for the batched decode step.  gemm_xlds stages a whole K-slice of X
// (up to 128 KiB) into LDS before its waves start streaming weights, and splits K across
// workgroups to bound that slice: measured on MI355X (profiles/gemm_sweep_r1.md) the prologue
// (~5 µs per workgroup at ≈11 B/clk/CU) plus the fp32 split-K slabs cost 25-40 % at M = 64.
//
// Here a workgroup of NW waves owns NW tile-groups (NT tiles of 16 output columns each, one per
// wave, accumulators live for the whole K range) and X flows through two LDS slices of CPS·128
// columns: while the waves multiply slice i, every thread has already issued the global loads of
// slice i+1 into registers and writes them to the other buffer after its last MFMA — one barrier per
// slice and no prologue beyond the first (small) slice.  Weights stream HBM -> VGPRs from the tiled
// layout (api.h kTileChunk: 4 contiguous KiB per (tile, K-chunk)) through a CPS-deep register ring
// that runs across slice boundaries.  The weight loads are non-temporal: streamed once, they must not
// evict X from L2 — with default loads the kernel slows down linearly in M (X re-fetched through the
// fabric), with nt it is flat in M (tools/gemm_ab.sh, profiles/gemm_stream_r1.md).  Split-K (grid.y = S) is only used when N is too narrow to give
// ~one workgroup per CU (O / down / QKV projections); then fp32 slabs [S, M, N] go to `part`.
//
// Rows m >= M of the X slices are never written; their MFMA rows produce garbage that is never
// stored (MFMA output rows depend only on the same A row).
#include "gemm_epilogue.h"

#include <cstdlib>
#include <type_traits>

#ifndef STREAM_X_TOUCH
#define STREAM_X_TOUCH 1  // L2 warm-up loads of the next X slice (see the kernel)
#endif

#ifndef DSSE_XCD_SPLITK
#define DSSE_XCD_SPLITK 1  // XCD-grouped split-K workgroup mapping (see the kernel)
#endif

namespace dsse {

// K-chunks of 128 per LDS slice: two slices of 16·MT rows stay within 128 KiB of LDS (MT <= 4: 512 columns,
// MT = 8 (128 rows): 256, MT = 16 (256 rows): 128 — one barrier per 2048 MFMA cycles per SIMD there).
constexpr int stream_cps(int mt) { return mt <= 4 ? 4 : (mt <= 8 ? 2 : 1); }

// Row blocks (M > 64, e.g. a 256-sequence decode bucket): the grid is (tile-group workgroups x MB row
// blocks of 64) and workgroups are renumbered so that the MB row blocks of one tile group are consecutive
// on the same XCD: they stream the same weight bytes at about the same time, so HBM serves them once and
// the XCD's L2 the other MB-1 times.  That sharing needs temporal (cached) weight loads (SHARED_W).

template <int MT, int NT, int NW, int RD, int MODE, bool SHARED_W = false>
__global__ void __launch_bounds__(64 * NW)
gemm_stream_kernel(const bf16* __restrict__ X, int ldx, int M, const bf16* __restrict__ W, int K, int N,
                   int Kr, GemmEpi ep, float* __restrict__ part) {
  constexpr int CPS = stream_cps(MT);
  constexpr int MP = 16 * MT;
  constexpr int ROWB = CPS * 256;                        // bytes of one X row in a slice
  constexpr int BUF = MP * ROWB;                         // bytes per slice buffer
  constexpr int PPH = MP * CPS * 16;                     // 16-byte pieces per slice
  constexpr int PPT = (PPH + 64 * NW - 1) / (64 * NW);   // 16-byte pieces per thread
  constexpr int XG = MT * NT <= 4 ? 4 : 2;  // k-steps whose X fragments are read at once (MT * NT <= 8)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  int wg = blockIdx.x, rb = 0;
  if constexpr (SHARED_W) {
    // bijective XCD-aware renumbering (dispatch puts workgroup i on XCD i % 8)
    const int nb = gridDim.x, xcd = wg % 8, slot = wg / 8, q = nb / 8, rem = nb % 8;
    const int id = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + slot;
    const int MB = (M + MP - 1) / MP;
    wg = id / MB;
    rb = id % MB;
    X += (size_t)rb * MP * ldx;
  }
  int ks = blockIdx.y;
  if (!SHARED_W && DSSE_XCD_SPLITK && gridDim.y > 1 && 8 % gridDim.y == 0 && (gridDim.x * gridDim.y) % 8 == 0) {
    // Split-K: keep each K range on 8/S XCDs (dispatch deals workgroup i, x-fastest, to XCD i % 8), so an
    // XCD's L2 fetches only its K range of X (1/S of it) instead of all of X.  Bijective, speed only.
    const int lin = blockIdx.y * gridDim.x + blockIdx.x, xcd = lin % 8, slot = lin / 8, per = 8 / gridDim.y;
    ks = xcd / per;
    wg = slot * per + xcd % per;
  }
  const int m0 = rb * MP;     // first row of this workgroup's row block
  const int tgi = wg * NW + w;  // host guarantees N / (16 NT) % NW == 0
  const int k0 = ks * Kr;       // this workgroup's K range
  const int nch = Kr >> 7;      // multiple of CPS (host-checked)
  const int nsl = nch / CPS;
  const int npieces = min(M - m0, MP) * CPS * 16;
  const int KC = K >> 7;

  // Weight stream through one buffer descriptor per tile covering exactly this wave's K range: the ring's
  // look-ahead loads past the range (its last DEPTH-1 issues) fail the descriptor's range check and cost no
  // memory traffic.  Clamping them to the last chunk instead re-fetched up to DEPTH-1 chunks per wave: +37 %
  // bytes for a split-K O projection with 8 chunks per wave, +9 % for gate_up.
  const int tgu = __builtin_amdgcn_readfirstlane(tgi), k0u = __builtin_amdgcn_readfirstlane(k0);
  __amdgpu_buffer_rsrc_t wrs[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
    wrs[t] = make_rsrc(W + ((size_t)(tgu * NT + t) * KC + (k0u >> 7)) * kTileChunk, (uint32_t)nch * kTileChunk * 2);
  constexpr int WAUX = SHARED_W ? 0 : kAuxNT;  // row blocks share weights through L2
  auto load_w = [&](int c, bf16x8 (&wf)[NT][4]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) wf[t][s] = ld_buf_bf16x8<WAUX>(wrs[t], (uint32_t)c * (kTileChunk * 2) + 1024 * s + lane * 16);
  };

  bf16x8 xs[PPT];
  auto load_x = [&](int sl) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int pi = threadIdx.x + i * 64 * NW;
      const bf16* src = X + k0 + sl * (CPS * 128);
      if (pi < PPH && pi < npieces)
        xs[i] = ld_bf16x8(src + (size_t)(pi / (CPS * 16)) * ldx + 8 * (pi % (CPS * 16)));
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int pi = threadIdx.x + i * 64 * NW;
      char* dst = smem + buf * BUF;
      if (pi < PPH && pi < npieces) {
        const int row = pi / (CPS * 16), c = pi % (CPS * 16);
        *reinterpret_cast<bf16x8*>(dst + row * ROWB + ((c >> 4) << 8) + (((c & 15) ^ swz(row & 15)) << 4)) = xs[i];
      }
    }
  };

  // L2 warm-up of the NEXT X slice: X is usually written by the kernel just before (RMSNorm / SiLU) on other
  // XCDs, so every XCD's L2 misses on it; one dword per 128-B line, touched a slice ahead, turns the real
  // (register-staged) X loads into L2 hits.  The touched words are folded into `touch`, consumed by a store
  // that never executes (M >= 0), so the loads stay.
  // Only for the wide-N launches (7-8 waves, no split-K: gate_up, LM head): the split-K narrow projections,
  // with 2-7 slices per workgroup, measured slower with it (+140 us per 64-stream step).
  constexpr bool TOUCH = STREAM_X_TOUCH && NW >= 7;
  constexpr int LPR = CPS * 2;                 // 128-B lines per X row of a slice
  constexpr int TOUCH_PT = (MP * LPR + 64 * NW - 1) / (64 * NW);
  const int touch_last_row = min(M - m0, MP) - 1;
  uint32_t touch = 0;
  auto touch_x = [&](int sl) {
    const char* src = reinterpret_cast<const char*>(X + k0 + sl * (CPS * 128));
#pragma unroll
    for (int i = 0; i < TOUCH_PT; ++i) {
      const int li = min(threadIdx.x + i * 64 * NW, MP * LPR - 1);
      touch ^= *reinterpret_cast<const uint32_t*>(src + (size_t)min(li / LPR, touch_last_row) * ldx * 2 +
                                                  (li % LPR) * 128);
    }
  };

  constexpr int DEPTH = CPS * RD;  // weight ring: RD slices of chunks in flight
  bf16x8 ring[DEPTH][NT][4];
#pragma unroll
  for (int d = 0; d < DEPTH - 1; ++d) load_w(d, ring[d]);
  load_x(0);
  if (TOUCH) touch_x(min(1, nsl - 1));
  store_x(0);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[mt][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // RD slices per iteration so that every ring slot index is a compile-time constant
  for (int sl0 = 0; sl0 < nsl; sl0 += RD) {
#pragma unroll
    for (int h = 0; h < RD; ++h) {
      const int sl = sl0 + h;
      if (h > 0 && sl >= nsl) break;
      __syncthreads();  // slice sl visible; everyone is done reading slice sl - 1's buffer
      const bool more = sl + 1 < nsl;
      if (TOUCH) touch_x(min(sl + 2, nsl - 1));
      if (more) load_x(sl + 1);
      const char* xb0 = smem + (sl & 1) * BUF;
#pragma unroll
      for (int d = 0; d < CPS; ++d) {
        const int slot = h * CPS + d;
        load_w(sl * CPS + d + DEPTH - 1, ring[(slot + DEPTH - 1) % DEPTH]);
        const char* xb = xb0 + (d << 8);
        // All X fragments of a group of k-steps are read from LDS before its MFMAs (the sched_barrier
        // keeps the compiler from sinking each ds_read next to its MFMA behind an lgkmcnt(0): that
        // schedule paid one LDS latency per MFMA and issued the weight loads late, draining the ring).
        if constexpr (MT * NT > 8) {  // 256 rows: VGPR-bound, the compiler's interleaved schedule is faster
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int ch = ((4 * g + s) ^ swz(r)) << 4;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
              const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xb + (16 * mt + r) * ROWB + ch);
#pragma unroll
              for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16x16x32(xf, ring[slot][t][s], acc[mt][t]);
            }
          }
          continue;
        }
#pragma unroll
        for (int s0 = 0; s0 < 4; s0 += XG) {
          bf16x8 xf[XG][MT];
#pragma unroll
          for (int s = 0; s < XG; ++s) {
            const int ch = ((4 * g + s0 + s) ^ swz(r)) << 4;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
              xf[s][mt] = *reinterpret_cast<const bf16x8*>(xb + (16 * mt + r) * ROWB + ch);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int s = 0; s < XG; ++s)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
              for (int t = 0; t < NT; ++t) acc[mt][t] = mfma16x16x32(xf[s][mt], ring[slot][t][s0 + s], acc[mt][t]);
        }
      }
      if (more) store_x((sl + 1) & 1);
    }
  }

  if (TOUCH && M < 0) part[touch & 1] = (float)touch;  // never runs: keeps the warm-up loads

  float* part_ks = part ? part + (size_t)ks * M * N : nullptr;
  if constexpr (MODE == kSiluMul) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int t = 0; t < NT; ++t) silu_epilogue4(ep, M, m0 + 16 * mt + 4 * g, tgi * NT + t, r, acc[mt][t]);
    return;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[mt][t][i];
        const float partner = (MODE == kSiluMul || MODE == kQkvRope) ? __shfl_xor(v, 8) : 0.f;
        epilogue<MODE>(ep, part_ks, M, N, m0 + 16 * mt + 4 * g + i, tgi * NT + t, r, v, partner);
      }
}

// LDS bytes of a gemm_stream launch: the two X slice buffers
constexpr size_t stream_lds(int mt) { return (size_t)2 * 16 * mt * stream_cps(mt) * 256; }

template <int MT, int NT, int NW, int RD, int MODE, bool SHARED_W = false>
static hipError_t launch_s(const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S, const GemmEpi& ep,
                           float* part, hipStream_t st) {
  const int TG = N / (16 * NT);
  const int MB = SHARED_W ? (M + 16 * MT - 1) / (16 * MT) : 1;
  const size_t lds = stream_lds(MT);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_stream_kernel<MT, NT, NW, RD, MODE, SHARED_W>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  dim3 grid(TG / NW * MB, S), block(64 * NW);
  hipLaunchKernelGGL((gemm_stream_kernel<MT, NT, NW, RD, MODE, SHARED_W>), grid, block, lds, st, X, ldx, M, W, K, N,
                     K / S, ep, part);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_s_mode(int mt, int nt, int nw, int rd, const bf16* X, int ldx, int M, const bf16* W, int K, int N,
                                int S, const GemmEpi& ep, float* part, hipStream_t st) {
  if (M > 16 * mt) {  // row blocks with L2-shared weights (64-row MFMA tiles, one or eight waves)
    if (mt == 4 && nt == 1 && nw == 4) return launch_s<4, 1, 4, 1, MODE, true>(X, ldx, M, W, K, N, S, ep, part, st);
    if (mt == 4 && nt == 1 && nw == 8) return launch_s<4, 1, 8, 1, MODE, true>(X, ldx, M, W, K, N, S, ep, part, st);
    return hipErrorInvalidValue;
  }
  // 128 / 256 rows in one workgroup: the weight ring stays 4 chunks deep (rd slices of 2 / 1 chunks)
  if (mt == 8 && nt == 1 && nw == 8 && rd == 2) return launch_s<8, 1, 8, 2, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  if (mt == 8 && nt == 1 && nw == 4 && rd == 2) return launch_s<8, 1, 4, 2, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  if (mt == 16 && nt == 1 && nw == 8 && rd == 4) return launch_s<16, 1, 8, 4, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  if (mt == 16 && nt == 1 && nw == 4 && rd == 4) return launch_s<16, 1, 4, 4, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  // two column tiles per wave: every X fragment read from LDS feeds two MFMAs
  if (mt == 8 && nt == 2 && nw == 4 && rd == 2) return launch_s<8, 2, 4, 2, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  if (mt == 16 && nt == 2 && nw == 4 && rd == 2) return launch_s<16, 2, 4, 2, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
#define K_S_CASE(MT_, NT_, NW_, RD_)         \
  if (mt == MT_ && nt == NT_ && nw == NW_ && rd == RD_) \
    return launch_s<MT_, NT_, NW_, RD_, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
#define K_S_MT(MT_) \
  K_S_CASE(MT_, 1, 8, 1) K_S_CASE(MT_, 2, 8, 1) K_S_CASE(MT_, 1, 4, 1) K_S_CASE(MT_, 1, 4, 2) K_S_CASE(MT_, 1, 8, 2)
  K_S_MT(1) K_S_MT(2) K_S_MT(4)
  // odd wave counts so that N / 16 / nw x S lands on the 256 CUs (qkv 384 tile groups: nw 3 x S 2; gate_up
  // 1792: nw 7; 36 MB-class narrow layers: nw 6)
  K_S_CASE(4, 1, 3, 1) K_S_CASE(4, 1, 5, 1) K_S_CASE(4, 1, 6, 1) K_S_CASE(4, 1, 7, 1)
  K_S_CASE(4, 1, 2, 1)
#undef K_S_MT
#undef K_S_CASE
  return hipErrorInvalidValue;
}


// ---------------------------------------------------------------------------------------------------------------
// gemm_ring: the X-streaming GEMM with X AND the weights staged by LDS-DMA in one ordered stream (M <= 16 MT).
//
// gemm_stream stages X through VGPRs one slice ahead; the `s_waitcnt vmcnt` that store_x needs for those loads
// also retires every weight load issued before them (VMEM completes in order), and at its loop heads hipcc
// waits vmcnt(0) for the register ring: the weight stream drains to a few chunks per wave.  Here nothing VMEM
// has a VGPR destination: for K-chunk c (128 columns) every wave issues its share of the chunk's X rows
// (global_load_lds) and its own 4 KiB weight chunk (buffer_load ... lds, range-checked) into LDS slot c % D,
// D - 1 chunks ahead of the MFMAs.  One counted vmcnt + barrier per chunk publishes chunk c (all waves' shares
// landed) while chunks c+1 .. c+D-2 stay in flight; the slot refilled after the MFMAs of chunk c held chunk
// c - 1, which every wave finished before that barrier.  Look-ahead issues past the last chunk keep the per-wave
// load count uniform (the vmcnt literal depends on it): the weight loads fail the buffer range check (no
// traffic), the X loads re-read the last chunk into a slot nobody reads.
// Slot = [X image: 16 MT rows x 256 B, 16-B pieces XOR-swizzled by swz() on the source address -- the DMA writes
// LDS lane-linearly -- and read back with the same XOR (gemm_stream's X image)] [NW x 4 KiB weight chunks in
// MFMA B-fragment order, read back lane-linearly].
template <int MT, int NW, int D>
struct RingGeom {
  static constexpr int SLOTX = 16 * MT * 256, SLOT = SLOTX + NW * 4096;
  static constexpr size_t LDS = (size_t)D * SLOT;
};

DEV void glds16_s(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds(const_cast<void*>(src),
                                   reinterpret_cast<__attribute__((address_space(3))) void*>(
                                       reinterpret_cast<uintptr_t>(lds_base)),
                                   16, 0, 0);
}

// FIX (round 6, the gemm_pipe.hip protocol on this kernel's small tiles): split-K slices of a column group combined
// inside the launch -- ticket first, the first S - 1 slices store their MT x 16 x 16 fp32 accumulators per wave
// (NW x MT KiB per workgroup) and count themselves done, the last waits for them (they wait for nothing), adds and
// runs the epilogue.  Used for the SiLU·mul projection of TP ranks at 17-64 rows (gate_up, N = 28672 / t), whose
// split-K otherwise needs a splitk_reduce launch.
template <int MT, int NW, int D, int MODE, bool FIX = false>
__global__ void __launch_bounds__(64 * NW)
gemm_ring_kernel(const bf16* __restrict__ X, int ldx, int M, const bf16* __restrict__ W, int K, int N, int Kr,
                 GemmEpi ep, float* __restrict__ part) {
  using G = RingGeom<MT, NW, D>;
  constexpr int MP = 16 * MT;
  constexpr int XN = MP / 4;               // 1 KiB X DMA instructions per chunk (4 rows each)
  constexpr int XI = (XN + NW - 1) / NW;  // per wave; with NW not dividing XN the surplus instructions repeat the
                                          // last one (same bytes to the same LDS address: a benign duplicate)
  static_assert(D >= 3 && G::LDS <= 160 * 1024, "ring of >= 3 slots within the CU's LDS");
  constexpr int PER = XI + 4;             // VMEM instructions per wave per chunk
  constexpr int WAUX = kAuxNT;  // weights streamed once: non-temporal
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const unsigned long long st0 = stamps::now();
  unsigned long long st1 = 0;

  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  int wg = blockIdx.x, ks = blockIdx.y;
  if (DSSE_XCD_SPLITK && gridDim.y > 1 && 8 % gridDim.y == 0 && (gridDim.x * gridDim.y) % 8 == 0) {
    const int lin = blockIdx.y * gridDim.x + blockIdx.x, xcd = lin % 8, slot = lin / 8, per = 8 / gridDim.y;
    ks = xcd / per;
    wg = slot * per + xcd % per;
  }
  const int tgi = wg * NW + w;  // this wave's 16-column tile
  const int k0 = ks * Kr;
  const int nch = Kr >> 7;
  const int KC = K >> 7;

  const int tgu = __builtin_amdgcn_readfirstlane(tgi), k0u = __builtin_amdgcn_readfirstlane(k0);
  const __amdgpu_buffer_rsrc_t wrs =
      make_rsrc(W + ((size_t)tgu * KC + (k0u >> 7)) * kTileChunk, (uint32_t)nch * kTileChunk * 2);

  // this lane's X source per DMA instruction: row 4 (w XI + i) + g, logical piece r ^ swz(row & 15)
  const bf16* xsrc[XI];
  int xdst[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    xdst[i] = __builtin_amdgcn_readfirstlane(min(w * XI + i, XN - 1));
    const int row = 4 * xdst[i] + g;
    xsrc[i] = X + (size_t)min(row, M - 1) * ldx + k0 + 8 * (r ^ swz(row & 15));
  }
  auto issue = [&](int c, int slot) {
    const int cc = min(c, nch - 1);
    char* base = smem + slot * G::SLOT;
#pragma unroll
    for (int i = 0; i < XI; ++i) glds16_s(xsrc[i] + cc * 128, base + xdst[i] * 1024);
    char* wb = base + G::SLOTX + w * 4096;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wrs, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(wb + 1024 * s)),
          16, (uint32_t)c * (kTileChunk * 2) + 1024 * s + lane * 16, 0, 0, WAUX);
  };

#pragma unroll
  for (int d = 0; d < D - 1; ++d) issue(d, d);

  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = 0; c0 < nch; c0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      if (u > 0 && c0 + u >= nch) break;
      // chunk c0 + u landed for every wave, chunks up to c0 + u + D - 2 still in flight
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((D - 2) * PER) : "memory");
      if (DSSE_PIPE_STAMPS && c0 + u == 0) st1 = stamps::now();
      const char* xb = smem + u * G::SLOT;
      const char* wb = xb + G::SLOTX + w * 4096 + lane * 16;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 xf[MT];
        const int ch = ((4 * g + s) ^ swz(r)) << 4;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xf[mt] = *reinterpret_cast<const bf16x8*>(xb + (16 * mt + r) * 256 + ch);
        const bf16x8 wf = *reinterpret_cast<const bf16x8*>(wb + 1024 * s);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma16x16x32(xf[mt], wf, acc[mt]);
      }
      // refill the slot of chunk c - 1 (every wave finished it before the barrier above); the LDS reads of this
      // chunk must be done before the slot is reused D - 1 chunks later: the next barriers order that
      issue(c0 + u + D - 1, (u + D - 1) % D);
    }
  }
  // no LDS-DMA may still be landing when the workgroup's LDS is handed to the next workgroup
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long st2 = stamps::now();

  if constexpr (FIX) {
    const int S = gridDim.y;
    if (S > 1) {
      typedef __attribute__((address_space(1))) int gint;  // shared words: global agent-scope accesses
      gint* cnt = (gint*)(ep.fix_cnt) + 4;                 // tickets [wg], done [kFixTiles + wg]; timeouts at [0]
      constexpr int kSlotF4 = NW * MT * 64;                // [wave][mt][lane]
      __syncthreads();  // every wave past its last LDS read: word 0 of the LDS carries the ticket
      int* sflag = reinterpret_cast<int*>(smem);
      if (threadIdx.x == 0) sflag[0] = __hip_atomic_fetch_add(cnt + wg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int ticket = __builtin_amdgcn_readfirstlane(sflag[0]);
      f32x4* slots = reinterpret_cast<f32x4*>(part) + (size_t)wg * (S - 1) * kSlotF4;
      const int off = w * MT * 64 + lane;
      if (ticket < S - 1) {
        f32x4* dst = slots + (size_t)ticket * kSlotF4 + off;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) dst[mt * 64] = acc[mt];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_fetch_add(cnt + kFixTiles + wg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        stamps::record(stamps::kRing | MODE << 8 | FIX << 12, st0, st1, st2);
        return;
      }
      if (threadIdx.x == 0) {
        unsigned spins = 0;
        while (__hip_atomic_load(cnt + kFixTiles + wg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S - 1) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > (1u << 22)) {
            __hip_atomic_fetch_add(cnt - 4, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(cnt + wg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cnt + kFixTiles + wg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int sl = 0; sl < S - 1; ++sl) {
        const f32x4* src = slots + (size_t)sl * kSlotF4 + off;
        f32x4 t[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) t[mt] = src[mt * 64];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] += t[mt];
      }
    }
  }

  float* part_ks = part ? part + (size_t)ks * M * N : nullptr;
  if constexpr (MODE == kSiluMul) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) silu_epilogue4(ep, M, 16 * mt + 4 * g, tgi, r, acc[mt]);
    stamps::record(stamps::kRing | MODE << 8 | FIX << 12, st0, st1, st2);
    return;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = acc[mt][i];
      const float partner = MODE == kQkvRope ? __shfl_xor(v, 8) : 0.f;
      epilogue<MODE>(ep, part_ks, M, N, 16 * mt + 4 * g + i, tgi, r, v, partner);
    }
  stamps::record(stamps::kRing | MODE << 8 | FIX << 12, st0, st1, st2);
}

template <int MT, int NW, int D, int MODE, bool FIX = false>
static hipError_t launch_r(const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S, const GemmEpi& ep,
                           float* part, hipStream_t st) {
  const size_t lds = RingGeom<MT, NW, D>::LDS;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_ring_kernel<MT, NW, D, MODE, FIX>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  dim3 grid(N / 16 / NW, S), block(64 * NW);
  hipLaunchKernelGGL((gemm_ring_kernel<MT, NW, D, MODE, FIX>), grid, block, lds, st, X, ldx, M, W, K, N, K / S, ep,
                     part);
  return hipGetLastError();
}



// Ring depth per (rows, waves): as many 128-column chunks as the LDS holds (slot = 16 MT rows x 256 B of X +
// NW x 4 KiB of weights, <= 160 KiB in all).
constexpr int ring_depth(int mt, int nw) {
  return mt == 8 ? 3 : (mt == 4 ? (nw == 3 ? 5 : (nw <= 6 ? 4 : 3)) : (nw == 4 ? 6 : 4));
}

template <int MODE>
static hipError_t launch_r_mode(int nw, const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S,
                                const GemmEpi& ep, float* part, hipStream_t st) {
#define K_R_CASE(MT_, NW_) \
  if (mt == MT_ && nw == NW_)  \
    return launch_r<MT_, NW_, ring_depth(MT_, NW_), MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  const int mt = M <= 32 ? 2 : (M <= 64 ? 4 : 8);
  K_R_CASE(8, 4)
  // (4, 5) is served by gemm_ring2 only: this kernel's 5-wave form wrote one wave's columns wrong (round 3)
  K_R_CASE(4, 3) K_R_CASE(4, 4) K_R_CASE(4, 6) K_R_CASE(4, 7) K_R_CASE(4, 8)
  K_R_CASE(2, 4) K_R_CASE(2, 7) K_R_CASE(2, 8)
#undef K_R_CASE
  return hipErrorInvalidValue;
}

// The in-launch fix-up form (SiLU·mul only; 17-64 rows, 4 / 7 / 8 waves).
static hipError_t launch_r_fix(int nw, const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S,
                               const GemmEpi& ep, float* part, hipStream_t st) {
  const int mt = M <= 32 ? 2 : 4;
  if (M > 64 || N / 16 / nw > kFixTiles) return hipErrorInvalidValue;
#define K_RF_CASE(MT_, NW_) \
  if (mt == MT_ && nw == NW_) return launch_r<MT_, NW_, ring_depth(MT_, NW_), kSiluMul, true>(X, ldx, M, W, K, N, S, ep, part, st);
  K_RF_CASE(4, 4) K_RF_CASE(4, 7) K_RF_CASE(4, 8) K_RF_CASE(2, 4) K_RF_CASE(2, 7) K_RF_CASE(2, 8)
#undef K_RF_CASE
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------------------------
// gemm_ring2: the ring GEMM with the weight look-ahead decoupled from X (round 3, profiles/r3/fillbench.md).
//
// An HBM weight stream is latency-bound (~2.3 us loaded): a CU moves weight bytes in flight / 2.3 us, up to
// ~28 GB/s (7.2 TB/s chip-wide) at 32-64 KiB in flight.  gemm_ring_kernel stages X and W through ONE ring (one
// slot = X chunk + every wave's W chunk, one vmcnt for both), so X's 16 KiB per slot limits W to 1-3 chunks in
// flight (12-28 KiB at 64 rows: 3.6-4.4 TB/s on qkv / o / down).  Here:
//   * NW compute waves, each with its OWN ring of DW weight slots (4 KiB: its 16-column tile x 128-deep chunk)
//     in LDS, filled by its own buffer_load ... lds DW - 1 chunks ahead and waited for by its own counted vmcnt
//     (its own loads only: no barrier needed for W, the wave both fills and reads its slots);
//   * XL loader waves that only stage X (16 MT rows x 128 columns per chunk, L2-resident: 86 GB/s per CU) into
//     a short ring of DX slots, DX - 1 chunks ahead;
//   * one s_barrier per chunk: the loaders' vmcnt retired X(c) before it, and every compute wave finished chunk
//     c - 1 before it, so X(c + DX - 1) may overwrite X(c - 1)'s slot right after it.
// W-slot reuse needs no barrier: a compute wave refills the slot of chunk c - 1 after its MFMAs of chunk c,
// which consumed chunk c - 1's fragments (their ds_reads completed) one iteration earlier.  Look-ahead past the
// last chunk: weights fail the buffer range check (no traffic; zeros land in a slot nobody reads), X re-reads
// the last chunk into a slot nobody reads, so every wave's per-chunk load count -- the vmcnt literals -- is
// uniform.  Same epilogues and split-K contract as gemm_ring_kernel.
template <int MT, int NW, int XL, int DX, int DW>
struct Ring2Geom {
  static constexpr int SLOTX = 16 * MT * 256;       // X chunk image (16 MT rows x 256 B)
  static constexpr int XOFF = 0, WOFF = DX * SLOTX;  // X ring, then NW x DW weight slots of 4 KiB
  static constexpr size_t LDS = (size_t)DX * SLOTX + (size_t)NW * DW * 4096;
};

template <int MT, int NW, int XL, int DX, int DW, int MODE>
__global__ void __launch_bounds__(64 * (NW + XL))
gemm_ring2_kernel(const bf16* __restrict__ X, int ldx, int M, const bf16* __restrict__ W, int K, int N, int Kr,
                  GemmEpi ep, float* __restrict__ part) {
  using G = Ring2Geom<MT, NW, XL, DX, DW>;
  constexpr int MP = 16 * MT;
  constexpr int XN = MP / 4;              // 1 KiB X DMA instructions per chunk (4 rows each)
  static_assert(XN % XL == 0, "X instructions split evenly over the loader waves");
  constexpr int XI = XN / XL;             // per loader wave per chunk
  static_assert(DX >= 3 && DW >= 3 && G::LDS <= 160 * 1024, "rings of >= 3 slots within the CU's LDS");
  constexpr int WAUX = kAuxNT;  // weights streamed once: non-temporal
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  int wg = blockIdx.x, ks = blockIdx.y;
  if (DSSE_XCD_SPLITK && gridDim.y > 1 && 8 % gridDim.y == 0 && (gridDim.x * gridDim.y) % 8 == 0) {
    const int lin = blockIdx.y * gridDim.x + blockIdx.x, xcd = lin % 8, slot = lin / 8, per = 8 / gridDim.y;
    ks = xcd / per;
    wg = slot * per + xcd % per;
  }
  const int k0 = ks * Kr;
  const int nch = Kr >> 7;
  const int KC = K >> 7;

  if (w >= NW) {  // ---------------- X loader wave
    const int lw = w - NW;
    const bf16* xsrc[XI];
    int xdst[XI];
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      xdst[i] = lw * XI + i;  // instruction index within the chunk: rows 4 xdst .. 4 xdst + 3
      const int row = 4 * xdst[i] + g;
      xsrc[i] = X + (size_t)min(row, M - 1) * ldx + k0 + 8 * (r ^ swz(row & 15));
    }
    auto issue_x = [&](int c, int slot) {
      const int cc = min(c, nch - 1);
      char* base = smem + G::XOFF + slot * G::SLOTX;
#pragma unroll
      for (int i = 0; i < XI; ++i) glds16_s(xsrc[i] + cc * 128, base + xdst[i] * 1024);
    };
#pragma unroll
    for (int d = 0; d < DX - 1; ++d) issue_x(d, d);
    for (int c0 = 0; c0 < nch; c0 += DX) {
#pragma unroll
      for (int u = 0; u < DX; ++u) {
        if (u > 0 && c0 + u >= nch) break;
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((DX - 2) * XI) : "memory");
        issue_x(c0 + u + DX - 1, (u + DX - 1) % DX);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  // ---------------- compute wave: its own 16-column tile and weight ring
  const int tgi = wg * NW + w;
  const int tgu = __builtin_amdgcn_readfirstlane(tgi), k0u = __builtin_amdgcn_readfirstlane(k0);
  const __amdgpu_buffer_rsrc_t wrs =
      make_rsrc(W + ((size_t)tgu * KC + (k0u >> 7)) * kTileChunk, (uint32_t)nch * kTileChunk * 2);
  char* wring = smem + G::WOFF + w * (DW * 4096);
  auto issue_w = [&](int c, int slot) {
    char* wb = wring + slot * 4096;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          wrs, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(wb + 1024 * s)),
          16, (uint32_t)c * (kTileChunk * 2) + 1024 * s + lane * 16, 0, 0, WAUX);
  };
#pragma unroll
  for (int d = 0; d < DW - 1; ++d) issue_w(d, d);

  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // DX and DW chunks per unrolled group: slot indices are compile-time constants in both rings
  constexpr int UN = DX * DW;
  for (int c0 = 0; c0 < nch; c0 += UN) {
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      if (u > 0 && c0 + u >= nch) break;
      // own W(c) landed (W(c+1) .. W(c+DW-2) may stay in flight), then X(c) published by the loaders
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((DW - 2) * 4) : "memory");
      const char* xb = smem + G::XOFF + (u % DX) * G::SLOTX;
      const char* wb = wring + (u % DW) * 4096 + lane * 16;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 xf[MT];
        const int ch = ((4 * g + s) ^ swz(r)) << 4;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xf[mt] = *reinterpret_cast<const bf16x8*>(xb + (16 * mt + r) * 256 + ch);
        const bf16x8 wf = *reinterpret_cast<const bf16x8*>(wb + 1024 * s);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma16x16x32(xf[mt], wf, acc[mt]);
      }
      issue_w(c0 + u + DW - 1, (u + DW - 1) % DW);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  float* part_ks = part ? part + (size_t)ks * M * N : nullptr;
  if constexpr (MODE == kSiluMul) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) silu_epilogue4(ep, M, 16 * mt + 4 * g, tgi, r, acc[mt]);
    return;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = acc[mt][i];
      const float partner = MODE == kQkvRope ? __shfl_xor(v, 8) : 0.f;
      epilogue<MODE>(ep, part_ks, M, N, 16 * mt + 4 * g + i, tgi, r, v, partner);
    }
}

template <int MT, int NW, int XL, int DX, int DW, int MODE>
static hipError_t launch_r2(const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S, const GemmEpi& ep,
                            float* part, hipStream_t st) {
  const size_t lds = Ring2Geom<MT, NW, XL, DX, DW>::LDS;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_ring2_kernel<MT, NW, XL, DX, DW, MODE>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  dim3 grid(N / 16 / NW, S), block(64 * (NW + XL));
  hipLaunchKernelGGL((gemm_ring2_kernel<MT, NW, XL, DX, DW, MODE>), grid, block, lds, st, X, ldx, M, W, K, N, K / S,
                     ep, part);
  return hipGetLastError();
}

// (rows tile MT, compute waves NW) -> loader waves, X slots, W slots per wave (LDS <= 160 KiB)
template <int MODE>
static hipError_t launch_r2_mode(int nw, const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S,
                                 const GemmEpi& ep, float* part, hipStream_t st) {
  const int mt = M <= 32 ? 2 : (M <= 64 ? 4 : 8);
#define K_R2_CASE(MT_, NW_, XL_, DX_, DW_) \
  if (mt == MT_ && nw == NW_) return launch_r2<MT_, NW_, XL_, DX_, DW_, MODE>(X, ldx, M, W, K, N, S, ep, part, st);
  // 33-64 rows: X slot 16 KiB x 3
  K_R2_CASE(4, 3, 1, 3, 8) K_R2_CASE(4, 4, 1, 3, 7) K_R2_CASE(4, 5, 1, 3, 5) K_R2_CASE(4, 6, 1, 3, 4)
  K_R2_CASE(4, 7, 1, 3, 4) K_R2_CASE(4, 8, 1, 3, 3)
  // 17-32 rows: X slot 8 KiB x 3
  K_R2_CASE(2, 3, 1, 3, 10) K_R2_CASE(2, 4, 1, 3, 8) K_R2_CASE(2, 7, 1, 3, 4) K_R2_CASE(2, 8, 1, 3, 4)
  // 65-128 rows: X slot 32 KiB x 3, two loader waves
  K_R2_CASE(8, 4, 2, 3, 4)
#undef K_R2_CASE
  return hipErrorInvalidValue;
}

}  // namespace dsse

// rd: weight-ring depth in LDS slices (mt <= 4: 1 = 4 chunks = 16 KiB per wave in flight, 2 = 8 chunks;
// mt = 8: 2, mt = 16: 4, i.e. 4 chunks).
// Shape contract (checked by the caller): K % (128 stream_cps(mt) S) == 0, (N / (16 nt)) % nw == 0,
// M <= 16 mt with mt in {1, 2, 4, 8, 16}, or M > 64 with mt = 4, nt = 1, rd = 1 (row blocks of 64).
// part: fp32 [S, M, N] workspace when S > 1.  partial_only: leave the slabs for the consumer (the fused
// residual + RMSNorm kernel) instead of reducing them here.
extern "C" hipError_t dsse_gemm_stream(int mode, int mt, int nt, int nw, int rd, int S, int partial_only, const void* X,
                                       int ldx, int M, const void* W, int K, int N, const dsse::GemmEpi* ep,
                                       float* part, hipStream_t st) {
  using namespace dsse;
  const bf16* x = reinterpret_cast<const bf16*>(X);
  const bf16* w = reinterpret_cast<const bf16*>(W);
  if (S == 1 && !partial_only) {
    switch (mode) {
      case kStoreBf16: return launch_s_mode<kStoreBf16>(mt, nt, nw, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kStoreF32: return launch_s_mode<kStoreF32>(mt, nt, nw, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kResidAdd: return launch_s_mode<kResidAdd>(mt, nt, nw, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kSiluMul: return launch_s_mode<kSiluMul>(mt, nt, nw, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kQkvRope: return launch_s_mode<kQkvRope>(mt, nt, nw, rd, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
    }
    return hipErrorInvalidValue;
  }
  hipError_t e = launch_s_mode<kPartial>(mt, nt, nw, rd, x, ldx, M, w, K, N, S, *ep, part, st);
  if (e != hipSuccess || partial_only) return e;
  return launch_splitk_reduce(mode, part, S, M, N, *ep, st);
}

// Ring variant (gemm_ring_kernel): 17 <= M <= 64 rows (16 MT-row MFMA tiles, MT = 2 / 4 by M), nw in {3, 4, 7, 8};
// 65-128 rows (MT 8) with nw = 4;
// K % (128 S) == 0, (N / 16) % nw == 0.
extern "C" hipError_t dsse_gemm_ring(int mode, int nw, int S, int partial_only, int ring2, const void* X, int ldx,
                                     int M, const void* W, int K, int N, const dsse::GemmEpi* ep, float* part,
                                     hipStream_t st) {
  using namespace dsse;
  const bf16* x = reinterpret_cast<const bf16*>(X);
  const bf16* w = reinterpret_cast<const bf16*>(W);
  if (M > 128 || M < 17 || (M > 64 && nw != 4) || K % (128 * S) != 0 || (N / 16) % nw != 0) return hipErrorInvalidValue;
  if (partial_only == 2) {  // split-K combined in the launch (SiLU·mul; `part` = dsse_gemm_ring_fix_floats)
    if (mode != kSiluMul || S < 2 || ep->fix_cnt == nullptr) return hipErrorInvalidValue;
    return launch_r_fix(nw, x, ldx, M, w, K, N, S, *ep, part, st);
  }
  // ring2: the decoupled-weight-look-ahead kernel (the single-ring kernel is the fallback for shapes it is not
  // instantiated for); chosen by the caller (bindings.cpp ring2_for)
  const bool r2 = ring2 != 0;
  auto run = [&](auto mode_tag, int s_, const GemmEpi* e_, float* p_) -> hipError_t {
    constexpr int MODE = decltype(mode_tag)::value;
    // the preferred kernel, else the other one (a shape only one of them is instantiated for)
    hipError_t e = r2 ? launch_r2_mode<MODE>(nw, x, ldx, M, w, K, N, s_, *e_, p_, st)
                      : launch_r_mode<MODE>(nw, x, ldx, M, w, K, N, s_, *e_, p_, st);
    if (e != hipErrorInvalidValue) return e;
    (void)hipGetLastError();
    return r2 ? launch_r_mode<MODE>(nw, x, ldx, M, w, K, N, s_, *e_, p_, st)
              : launch_r2_mode<MODE>(nw, x, ldx, M, w, K, N, s_, *e_, p_, st);
  };
  if (S == 1 && !partial_only) {
    switch (mode) {
      case kStoreBf16: return run(std::integral_constant<int, kStoreBf16>{}, 1, ep, nullptr);
      case kStoreF32: return run(std::integral_constant<int, kStoreF32>{}, 1, ep, nullptr);
      case kResidAdd: return run(std::integral_constant<int, kResidAdd>{}, 1, ep, nullptr);
      case kSiluMul: return run(std::integral_constant<int, kSiluMul>{}, 1, ep, nullptr);
      case kQkvRope: return run(std::integral_constant<int, kQkvRope>{}, 1, ep, nullptr);
    }
    return hipErrorInvalidValue;
  }
  hipError_t e = run(std::integral_constant<int, kPartial>{}, S, ep, part);
  if (e != hipSuccess || partial_only) return e;
  return launch_splitk_reduce(mode, part, S, M, N, *ep, st);
}

// Workspace floats of the ring kernel's in-launch fix-up: S - 1 register-order slots per column group.
extern "C" size_t dsse_gemm_ring_fix_floats(int nw, int S, int M, int N) {
  const int mt = M <= 32 ? 2 : 4;
  return (size_t)(N / 16 / nw) * (S - 1) * nw * mt * 64 * 4;
}

DSSE_CHECK_READER(dsse_check_gemm_stream)
DSSE_STAMPS_BINDER(dsse_stamps_bind_gemm_stream)
