// Prefill / wide GEMM, 256 (or 192 / 128) x 256 tile, deep LDS-DMA pipeline:  Y[M, N] = X[M, K] · W[N, K]ᵀ on the
// engine's tiled weight layout (api.h kTileChunk), M >= 128 (few tiles: split K, grid.z-style slices in the tile
// index).
//
// Why a new schedule (profiles/r4/pmc_gemm_r4.md): gemm_phased (gemm_tiled.hip cfg 4) issued the last A half of step
// t+1 one phase before the counted wait that needed it, so every K step waited ~a full L2/HBM round trip -- 44 %
// MFMA-busy, 42 % of wave time waiting on a dependency at 8192 rows.  Here every half-tile is in flight for five
// phases (~2,500 cycles) before any wave waits for it:
//
//   * 8 waves = 2 wave rows (128 rows each) x 4 wave columns (64 columns each); a wave's 128 x 64 tile is four
//     64 x 32 quadrants; a K step of 64 runs as four phases, one quadrant (16 MFMAs 16x16x32) per phase:
//         phase 0  quadrant (0, 0)   reads A rows q0 + B cols q0   issue  B-half 1 of step t+1
//         phase 1  quadrant (0, 1)   reads B cols q1                issue  A-half 1 of step t+1
//         phase 2  quadrant (1, 1)   reads A rows q1                issue  A-half 0 of step t+2
//         phase 3  quadrant (1, 0)   (operands in registers)        issue  B-half 0 of step t+2
//     one half-tile per phase (round 5: +1-5 % at 8192 rows, +2-10 % at 2048 over the round-5 first form that issued
//     0 / 1 / 2 / 1 half-tiles in phases 1 / 0 / 2 / 3, profiles/r5/pipe_even_ab_r5.log),
//     each phase = [fragment reads, DMA issue, counted vmcnt] s_barrier lgkmcnt(0) [16 MFMAs, prio 1] s_barrier,
//     with the two wave rows one barrier apart, so on every SIMD one wave's MFMA cluster overlaps the other's LDS
//     reads (the 8-phase template of the CDNA HIP guide, §5; the half-tile order is this kernel's own);
//   * a "half-tile" is what one phase's quadrant reads across the workgroup: A-half q = the 64-row quadrant q of
//     BOTH wave rows (128 rows x 128 B = 16 KiB), B-half q = the 32-column quadrant q of all four wave columns
//     (8 column tiles x 2 KiB); each is 16 one-KiB LDS-DMA instructions, two per wave;
//   * WAR: a half is re-staged >= 2 phases after its last read (A0 / B0 of buffer t & 1 read in phase 0 of t,
//     re-staged for t+2 in phases 2 / 3; B1 of buffer (t+1) & 1 last read in phase 1 of t-1, re-staged in phase 0 of
//     t; A1 read in phase 2 of t-1, re-staged in phase 1 of t) -- the lagging wave row is then still >= 1 barrier
//     past its lgkmcnt(0);
//   * RAW: counted waits, 8 in each of phases 0, 1 and 3 (four half-tiles of 2 instructions each younger than the
//     one retired): phase 0 retires B-half 1 of step t, phase 1 A-half 1 of t, phase 3 A0 / B0 of t+1 -- each in the
//     phase before its first read, so the lagging row has passed it one barrier before the leading row reads (never
//     vmcnt(0) in the steady loop);
//   * buffer-load LDS-DMA: one SGPR offset per K step, per-lane offsets fixed for the whole loop (no per-step VALU
//     address arithmetic); rows past M read as zeros (out-of-range offsets, no memory traffic); the last two steps
//     issue nothing past the end and count their waits exactly;
//   * XCD-aware tile order (bijective remap, groups of 8 row blocks swept by column) as gemm_tiled.hip;
//   * epilogues: bf16 store staged through LDS (16-byte row stores), SiLU·mul, fp32 / residual / QKV+RoPE /
//     split-K partial slabs through gemm_epilogue.h.
#include "gemm_epilogue.h"

#ifndef DSSE_PIPE_STAMPS
#define DSSE_PIPE_STAMPS 0
#endif

namespace dsse {
namespace gp {

// Diagnostic build only (_build.py variant "stamps"): workgroup-level s_memrealtime stamps (100 MHz, one clock for
// every CU) of the FIX path's phases after the fix-up counters: [wg][8] u64 (tools/pipe_stamps.py)
DEV void stamp(const GemmEpi& ep, int k, unsigned long long v) {
  if constexpr (DSSE_PIPE_STAMPS) {
    if (threadIdx.x == 0 && ep.fix_cnt)
      reinterpret_cast<unsigned long long*>(ep.fix_cnt + kStampOff)[(size_t)blockIdx.x * 8 + k] = v;
  }
}
DEV unsigned long long now() { return DSSE_PIPE_STAMPS ? __builtin_amdgcn_s_memrealtime() : 0ull; }

constexpr int kA = 256 * 128;     // A image of one K step: 256 rows x 64 bf16, swizzled 16-byte pieces
constexpr int kB = 16 * 2048;     // B image: 16 column tiles x two 1 KiB k-step blocks
constexpr int kBuf = kA + kB;     // 64 KiB per K step
constexpr size_t kLDS = 2 * (size_t)kBuf;
constexpr uint32_t kOOB = 0x80000000u;  // buffer offset past every range: the load returns zeros, no traffic

typedef __attribute__((address_space(3))) void* lds_t;

DEV void dma(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t)(reinterpret_cast<uintptr_t>(lds)), 16, voff, soff, 0, 0);
}

// A-image swizzle (as gemm_tiled.hip a_swz): piece q of LDS row `row` holds piece q ^ swz(row) of the X row;
// conflict-free ds_read_b128 for the A-fragment pattern (lane (r, g) reads row r, piece 2g + s).
DEV int a_swz(int row) { return (row >> 1) & 5; }

}  // namespace gp

// BM: rows per workgroup tile, 256, 192 or 128.  192 / 128 keep the 256-row LDS image and schedule and fill 48 / 32
// of every 64-row quadrant (the other slot rows load as zeros, no traffic, and no MFMA reads them): 12 / 8 MFMAs per
// phase instead of 16, for row counts that leave a 256-row block partly empty (the mixed prefill + decode steps'
// 320-384 rows: 192; the 161-256-row decode buckets' qkv / down: 192 / 128).  Slot row s of quadrant q, wave row wr
// holds X row m0 + wr * BM / 2 + q * BM / 4 + s.
// FIX (round 6): split-K with the slices of a tile combined inside the launch, no reduce kernel and no slabs for the
// consumer.  Ticket first: after its K loop every workgroup takes a ticket on the tile's arrival counter; the
// first S - 1 store their fp32 accumulators (16-byte stores in the MFMA register order, 1 KiB per wave instruction,
// read back by the same lanes) into slot `ticket` of the tile's workspace, drain, release, and count themselves
// done (a tile's slices are adjacent in the remapped order, so they share an XCD and its L2); the workgroup that draws ticket S - 1 waits (bounded) until the others are done -- they are
// running already and wait for nothing, so this cannot deadlock whatever the residency -- adds their slots into
// its registers and runs the normal epilogue.  The slab round trip costs (S - 1) x the tile's fp32 bytes once, on
// the tile's last arriver (profiles/r6/gemm_fix_r6.md).
template <int MODE, int BM, bool FIX = false>
__global__ void __launch_bounds__(512)
gemm_pipe_kernel(const bf16* __restrict__ X, int ldx, int M, const bf16* __restrict__ W, int K, int N, int Kr,
                 GemmEpi ep, float* __restrict__ part) {
  using namespace gp;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int wm = w >> 2, wn = w & 3;
  if constexpr (FIX) stamp(ep, 0, now());

  // ---- tile order: bijective XCD remap, then groups of 8 row blocks swept column by column (L2 panel reuse)
  constexpr int QR = BM / 4, QI = QR / 16;  // X rows per quadrant, MFMA row tiles per quadrant
  static_assert(BM == 256 || BM == 192 || BM == 128, "row tile");
  const int nbm = (M + BM - 1) / BM, nbn = N / 256, ntile = nbm * nbn;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x, xcd = bid % 8, q8 = nwg / 8, rem = nwg % 8;
  const int lid = (xcd < rem ? xcd * (q8 + 1) : rem * (q8 + 1) + (xcd - rem) * q8) + bid / 8;
  // split slices: FIX keeps a tile's S slices adjacent in the remapped order, so they run on one XCD and the last
  // arriver reads the other slices' plain-stored slots from its own L2; the slab form (consumer-reduced) keeps
  // them ntile apart
  const int S_ = nwg / ntile;
  const int ks = FIX ? lid % S_ : lid / ntile, tl = FIX ? lid / S_ : lid % ntile;
  constexpr int GM = 8;
  const int grp = tl / (GM * nbn), first = grp * GM, gsz = min(GM, nbm - first);
  const int bm = first + (tl % (GM * nbn)) % gsz, bn = (tl % (GM * nbn)) / gsz;
  const int m0 = bm * BM, n0 = bn * 256;
  const int k0 = ks * Kr, nk = Kr >> 6;
  const int KC = K >> 7;

  const __amdgpu_buffer_rsrc_t xr = make_rsrc(X, (uint32_t)(((size_t)(M - 1) * ldx + K) * 2));
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(W, (uint32_t)((size_t)N * K * 2));

  // ---- per-lane DMA offsets (bytes), fixed for the whole K loop: [half q][instruction i] of this wave
  uint32_t a_vo[2][2], b_vo[2][2];
  int a_lo[2][2], b_lo[2][2];  // LDS byte offsets inside a buffer
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = 2 * w + i;                                     // instruction j of the 16 of this half
      const int rb = (j >> 3) * 128 + q * 64 + (j & 7) * 8;        // first of its 8 rows
      const int row = rb + (lane >> 3), sr = (j & 7) * 8 + (lane >> 3);  // LDS slot row, slot row in the quadrant
      const int xrow = m0 + (j >> 3) * (BM / 2) + q * QR + sr;          // the X row it holds
      const int pc = (lane & 7) ^ a_swz(row);
      a_lo[q][i] = rb * 128;
      a_vo[q][i] = sr < QR && xrow < M ? (uint32_t)(((size_t)xrow * ldx + 32 * (pc >> 1) + 8 * (pc & 1)) * 2) : kOOB;
      const int tb = (j >> 2) * 4 + q * 2 + ((j >> 1) & 1), sub = j & 1;  // column tile of the block, k sub-step
      b_lo[q][i] = kA + tb * 2048 + sub * 1024;
      b_vo[q][i] = (uint32_t)((((size_t)(n0 / 16 + tb) * KC) * kTileChunk + sub * 512 + lane * 8) * 2);
    }
  // K step t: X columns 128c + 16h + (piece offsets), W chunk c, k sub-steps 2h, 2h+1
  auto a_so = [&](int t) {
    const int kk = k0 + 64 * t;
    return (uint32_t)(((kk >> 7) * 128 + 16 * ((kk >> 6) & 1)) * 2);
  };
  auto b_so = [&](int t) {
    const int kk = k0 + 64 * t;
    return (uint32_t)(((kk >> 7) * kTileChunk + ((kk >> 6) & 1) * 1024) * 2);
  };
  auto issue_a = [&](int q, int t) {
    char* base = smem + (t & 1) * kBuf;
    const uint32_t so = __builtin_amdgcn_readfirstlane(a_so(t));
#pragma unroll
    for (int i = 0; i < 2; ++i) dma(xr, base + a_lo[q][i], a_vo[q][i], so);
  };
  auto issue_b = [&](int q, int t) {
    char* base = smem + (t & 1) * kBuf;
    const uint32_t so = __builtin_amdgcn_readfirstlane(b_so(t));
#pragma unroll
    for (int i = 0; i < 2; ++i) dma(wr, base + b_lo[q][i], b_vo[q][i], so);
  };

  // ---- fragment reads: A rows wm*128 + 64 qm + 16 i + r (the swizzle is the same for every i), B column tiles
  // wn*4 + 2 qn + i, k sub-step sp of the step
  int a_rd[2];
#pragma unroll
  for (int sp = 0; sp < 2; ++sp) {
    const int row = wm * 128 + r;
    a_rd[sp] = row * 128 + (((2 * g + sp) ^ a_swz(row)) << 4);
  }
  f32x4 acc[8][4];
#pragma unroll
  for (int mt = 0; mt < 8; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4][2], b[4][2];
  auto read_a = [&](const char* buf, int qm) {
#pragma unroll
    for (int i = 0; i < QI; ++i)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
        a[i][sp] = *reinterpret_cast<const bf16x8*>(buf + a_rd[sp] + (64 * qm + 16 * i) * 128);
  };
  auto read_b = [&](const char* buf, int qn) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
        b[2 * qn + i][sp] =
            *reinterpret_cast<const bf16x8*>(buf + kA + (wn * 4 + 2 * qn + i) * 2048 + sp * 1024 + lane * 16);
  };
  auto mma = [&](int qm, int qn) {
    asm volatile("s_barrier\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int sp = 0; sp < 2; ++sp)
#pragma unroll
      for (int i = 0; i < QI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * qm + i][2 * qn + j] = mfma16x16x32(a[i][sp], b[2 * qn + j][sp], acc[4 * qm + i][2 * qn + j]);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_barrier" ::: "memory");
  };

  {
    // prologue: step 0 whole, then A0 / B0 of step 1 (its B1 / A1 go out in phases 0 / 1 of step 0)
    issue_a(0, 0);
    issue_b(0, 0);
    issue_b(1, 0);
    issue_a(1, 0);
    issue_a(0, 1);
    issue_b(0, 1);
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");  // A0 / B0 of step 0 landed everywhere
    if (wm == 1) asm volatile("s_barrier" ::: "memory");  // wave row 1 runs one barrier behind row 0
    // TAIL 0 = steady, 1 = step t+1 exists but t+2 does not, 2 = last step.  RAW: B1(t) waited in phase 0 and read
    // in phase 1, A1(t) waited in 1 and read in 2, A0 / B0(t+1) waited in 3 and read in phase 0 of t+1 (the
    // barrier that opens the reading phase follows every wave's wait).  WAR: B1 of buffer (t+1)&1 was last read in
    // phase 1 of t-1, A1 in phase 2 of t-1, A0 / B0 of buffer t&1 in phase 0 of t -- each restaged >= 2 phases later.
    auto step_even = [&](int t, auto tail_tag) {
      constexpr int TAIL = decltype(tail_tag)::value;
      const char* buf = smem + (t & 1) * kBuf;
      read_a(buf, 0);
      read_b(buf, 0);
      if constexpr (TAIL < 2) {
        issue_b(1, t + 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // B-half 1 of step t
      } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      mma(0, 0);
      read_b(buf, 1);
      if constexpr (TAIL < 2) {
        issue_a(1, t + 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A-half 1 of step t
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      mma(0, 1);
      read_a(buf, 1);
      if constexpr (TAIL == 0) issue_a(0, t + 2);
      mma(1, 1);
      if constexpr (TAIL == 0) {
        issue_b(0, t + 2);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A0 / B0 of step t+1
      } else if constexpr (TAIL == 1) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      }
      mma(1, 0);
    };
    int t = 0;
    for (; t < nk - 2; ++t) step_even(t, std::integral_constant<int, 0>{});
    step_even(t++, std::integral_constant<int, 1>{});  // nk >= 2 (host contract)
    step_even(t, std::integral_constant<int, 2>{});
  }
  // balance the barrier count of the two rows
  if (wm == 0) asm volatile("s_barrier" ::: "memory");

  if constexpr (FIX) {
    const int S = S_;
    if (S > 1) {
      constexpr int kSlotF4 = 8 * 8 * QI * 64;  // f32x4 per slot: [wave][qm][i < QI][nt][lane]
      typedef __attribute__((address_space(1))) int gint;  // shared words: global agent-scope accesses, never flat
      gint* cnt = (gint*)(ep.fix_cnt) + 4;   // tickets [tl], done [kFixTiles + tl]; timeouts at [0]
      __syncthreads();  // every wave past its last LDS read: word 0 of the LDS carries the ticket
      stamp(ep, 1, now());
      int* sflag = reinterpret_cast<int*>(smem);
      if (threadIdx.x == 0) sflag[0] = __hip_atomic_fetch_add(cnt + tl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int ticket = __builtin_amdgcn_readfirstlane(sflag[0]);  // wave-uniform: no waterfall around the rsrc
      stamp(ep, 2, now());
      if constexpr (DSSE_PIPE_STAMPS) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        stamp(ep, 6, ((unsigned long long)ticket << 32) | (xcc & 0xF));
      }
      f32x4* slots = reinterpret_cast<f32x4*>(part) + (size_t)tl * (S - 1) * kSlotF4;
      const int lane_off = w * (8 * QI * 64) + lane;
      if (ticket < S - 1) {
        // plain stores (they stay in this XCD's L2 for the same-XCD reader), every wave drained, then ONE agent-scope
        // release and the done count (the CDNA guide's split-K recipe: fence before the count, wait after the fence)
        f32x4* dst = slots + (size_t)ticket * kSlotF4 + lane_off;
#pragma unroll
        for (int qm = 0; qm < 2; ++qm)
#pragma unroll
          for (int i = 0; i < QI; ++i)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) dst[((qm * QI + i) * 4 + nt) * 64] = acc[4 * qm + i][nt];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        stamp(ep, 3, now());
        if (threadIdx.x == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_fetch_add(cnt + kFixTiles + tl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        stamp(ep, 4, now());
        return;
      }
      if (threadIdx.x == 0) {
        unsigned spins = 0;
        while (__hip_atomic_load(cnt + kFixTiles + tl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S - 1) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > (1u << 22)) {  // ~0.1 s: a writer never counted itself (cannot happen); flag, do not hang
            __hip_atomic_fetch_add(cnt - 4, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        // every other slice already took its ticket and counted itself: nothing touches this pair again in
        // this launch, so the last arriver leaves it zero for the next one
        __hip_atomic_store(cnt + tl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cnt + kFixTiles + tl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      stamp(ep, 3, now());
      for (int s = 0; s < S - 1; ++s) {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(slots + (size_t)s * kSlotF4, kSlotF4 * 16);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          // 2 QI accumulators in flight at once (quadrant row h / 2, column pair h % 2), then the adds
          const int qm = h >> 1, n0 = 2 * (h & 1);
          f32x4 t[QI][2];
#pragma unroll
          for (int i = 0; i < QI; ++i)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
              t[i][nt] = __builtin_bit_cast(
                  f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                             rs, (uint32_t)((lane_off + ((qm * QI + i) * 4 + n0 + nt) * 64) * 16), 0, 0));
#pragma unroll
          for (int i = 0; i < QI; ++i)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) acc[4 * qm + i][n0 + nt] += t[i][nt];
        }
      }
      if constexpr (DSSE_PIPE_STAMPS) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        stamp(ep, 4, now());
      }
    }
  }

  // acc[4 qm + i] holds X rows row0 + QR qm + 16 i (i < QI)
  const int row0 = m0 + wm * (BM / 2), tile0 = n0 / 16 + wn * 4;
  auto mrow = [&](int mt) { return row0 + QR * (mt >> 2) + 16 * (mt & 3); };
  if constexpr (MODE == kStoreBf16) {
    // stage the wave's 128 x 64 bf16 tile in LDS (all DMA retired, everyone past its last fragment read), then
    // 16-byte row stores: 8 lanes per 128-byte row, 8 rows per instruction
    __syncthreads();
    bf16* st = reinterpret_cast<bf16*>(smem + w * (128 * 64 * 2));
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = 16 * mt + 4 * g + i, cc = 16 * nt + r;
          // 16-byte chunk (cc >> 3) of row rr at chunk slot (cc >> 3) ^ (rr & 7): conflict-spread writes and reads
          st[rr * 64 + ((((cc >> 3) ^ (rr & 7)) << 3) | (cc & 7))] = f2bf(acc[mt][nt][i]);
        }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's own LDS image is complete
    bf16* out = reinterpret_cast<bf16*>(ep.out);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int rr = 8 * it + (lane >> 3), ch = lane & 7;
      if ((rr & 63) >= QR) continue;  // BM 192: slot rows 48-63 of a quadrant hold no X row
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(st + rr * 64 + ((ch ^ (rr & 7)) << 3));
      const int m = row0 + QR * (rr >> 6) + (rr & 63);
      if (m < M) *reinterpret_cast<bf16x8*>(out + (size_t)m * ep.ldo + n0 + wn * 64 + ch * 8) = v;
    }
    if constexpr (FIX) stamp(ep, 5, now());
    return;
  }
  if constexpr (MODE == kSiluMul) {
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        if ((mt & 3) < QI) silu_epilogue4(ep, M, mrow(mt) + 4 * g, tile0 + nt, r, acc[mt][nt]);
    if constexpr (FIX) stamp(ep, 5, now());
    return;
  }
  float* part_ks = part ? part + (size_t)ks * M * N : nullptr;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    if ((mt & 3) >= QI) continue;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[mt][nt][i];
        const float partner = (MODE == kQkvRope) ? __shfl_xor(v, 8) : 0.f;
        epilogue<MODE>(ep, part_ks, M, N, mrow(mt) + 4 * g + i, tile0 + nt, r, v, partner);
      }
  }
}

template <int MODE, int BM, bool FIX>
static hipError_t launch_pipe_bm(const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S, const GemmEpi& ep,
                                 float* part, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pipe_kernel<MODE, BM, FIX>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)gp::kLDS);
    attr_set = true;
  }
  const int nbm = (M + BM - 1) / BM, nbn = N / 256;
  hipLaunchKernelGGL((gemm_pipe_kernel<MODE, BM, FIX>), dim3(nbm * nbn * S), dim3(512), gp::kLDS, st, X, ldx, M, W, K,
                     N, K / S, ep, part);
  return hipGetLastError();
}
template <int MODE, bool FIX = false>
static hipError_t launch_pipe(int bm, const bf16* X, int ldx, int M, const bf16* W, int K, int N, int S,
                              const GemmEpi& ep, float* part, hipStream_t st) {
  if (bm == 128) return launch_pipe_bm<MODE, 128, FIX>(X, ldx, M, W, K, N, S, ep, part, st);
  return bm == 192 ? launch_pipe_bm<MODE, 192, FIX>(X, ldx, M, W, K, N, S, ep, part, st)
                   : launch_pipe_bm<MODE, 256, FIX>(X, ldx, M, W, K, N, S, ep, part, st);
}

}  // namespace dsse

// Shape contract (checked here): N % 256 == 0, K % (128 S) == 0 (>= 2 K steps of 64 per slice), the tiled weight
// layout (api.h), X rows of ldx >= K elements.  S > 1: partial_only 0 = fp32 slabs [S, M, N] into `part` reduced by
// launch_splitk_reduce, 1 = the slabs only (the consumer reduces them), 2 = in-launch fix-up (FIX above): `part`
// holds dsse_gemm_pipe_fix_floats() floats and ep->fix_cnt the counters (api.h), tiles <= kFixTiles.
extern "C" hipError_t dsse_gemm_pipe(int mode, int bm, int S, int partial_only, const void* X, int ldx, int M,
                                     const void* W, int K, int N, const dsse::GemmEpi* ep, float* part, hipStream_t st) {
  using namespace dsse;
  if (M < 1 || N % 256 != 0 || S < 1 || K % (128 * S) != 0 || ldx < K || (bm != 256 && bm != 192 && bm != 128))
    return hipErrorInvalidValue;
  const bf16* x = reinterpret_cast<const bf16*>(X);
  const bf16* w = reinterpret_cast<const bf16*>(W);
  if (S == 1 && !partial_only) {
    switch (mode) {
      case kStoreBf16: return launch_pipe<kStoreBf16>(bm, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kStoreF32: return launch_pipe<kStoreF32>(bm, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kResidAdd: return launch_pipe<kResidAdd>(bm, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kSiluMul: return launch_pipe<kSiluMul>(bm, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
      case kQkvRope: return launch_pipe<kQkvRope>(bm, x, ldx, M, w, K, N, 1, *ep, nullptr, st);
    }
    return hipErrorInvalidValue;
  }
  if (partial_only == 2) {
    if (ep->fix_cnt == nullptr || (size_t)((M + bm - 1) / bm) * (N / 256) > (size_t)kFixTiles) return hipErrorInvalidValue;
    switch (mode) {
      case kStoreBf16: return launch_pipe<kStoreBf16, true>(bm, x, ldx, M, w, K, N, S, *ep, part, st);
      case kStoreF32: return launch_pipe<kStoreF32, true>(bm, x, ldx, M, w, K, N, S, *ep, part, st);
      case kResidAdd: return launch_pipe<kResidAdd, true>(bm, x, ldx, M, w, K, N, S, *ep, part, st);
      case kSiluMul: return launch_pipe<kSiluMul, true>(bm, x, ldx, M, w, K, N, S, *ep, part, st);
      case kQkvRope: return launch_pipe<kQkvRope, true>(bm, x, ldx, M, w, K, N, S, *ep, part, st);
    }
    return hipErrorInvalidValue;
  }
  hipError_t e = launch_pipe<kPartial>(bm, x, ldx, M, w, K, N, S, *ep, part, st);
  if (e != hipSuccess || partial_only) return e;
  return launch_splitk_reduce(mode, part, S, M, N, *ep, st);
}

// Workspace floats of the in-launch fix-up (partial_only = 2): S - 1 register-order slots per tile.
extern "C" size_t dsse_gemm_pipe_fix_floats(int bm, int S, int M, int N) {
  const int nbm = (M + bm - 1) / bm, qi = bm / 64;
  return (size_t)nbm * (N / 256) * (S - 1) * (8 * 8 * qi * 64) * 4;
}
