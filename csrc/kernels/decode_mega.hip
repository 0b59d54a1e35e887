// Persistent decode MLP block ("mega" kernel, round 4 v2): one launch per layer runs
//
//     O projection (split-K slabs) -> residual + RMSNorm -> gate_up + SiLU·mul -> down (split-K slabs)
//     -> residual + RMSNorm with the next layer's weight -> the next layer's QKV projection (split-K slabs)
//
// for <= 64 decode rows, so a layer is two launches: the folded decode attention (attention.hip mode 3: QKV slab sum,
// RoPE, K/V write, paged attention) and this block.  Replaces six launches of the launch-per-op step (o, rmsnorm<3>,
// gate_up, down, rmsnorm<3>, next qkv; profiles/r3/decode_step_64_r3.md, VERDICT round 3 "next 1").
//
// What a persistent block can win is the time the weight stream stands still at the seams (O -> norm -> gate_up and
// down -> norm -> QKV: ~7.5 us each, profiles/r4/mega_r4.md phase stamps): the seams are chains of round trips
// (slab stores, a flag, slab loads, norm stores, a flag, the activation load), not bandwidth.  v1 kept each compute
// wave's weight stream in a 3-slot LDS ring (2 steps in flight, all the LDS there was) and matched the separate
// kernels phase for phase (1.05x slower overall).  v2 moves the weight stream into REGISTERS:
//
//   * waves 0-7 compute: each owns one 16-column weight tile of the current item; its weight blocks (tiled layout:
//     one 1 KiB sub-block = one lane-ordered MFMA B fragment per lane) go straight from HBM into a 6-step register
//     ring (4 x 16 B per lane per step, nt loads), so 5 steps (20 KiB per wave, 160 KiB per CU) stay in flight and
//     stream THROUGH a seam: when the activation arrives, the next item's first steps are already in registers.
//     The compute waves issue no other memory operation: their vmcnt waits are the compiler's, and nothing younger
//     than the weight loads ever has to be drained (item results go to LDS, not to memory);
//   * wave 8 is the loader / publisher: it polls the dependency counters, streams the activation X through a 3-slot
//     LDS ring by LDS-DMA (16 KiB per step, one s_barrier per step publishes it), and after each item stores the
//     item's result tile from LDS (write-through), drains its own stores and signals the item's counter;
//   * the RMSNorms are distributed and folded into the consumers: after the O item of column group cg completes on
//     its 8 split-K workgroups (group counter, 8 arrivals), each of them reduces its own 16-column strip for all rows
//     (8 slabs + the residual, by LDS-DMA), writes the new residual strip, y = bf16(resid · w_norm) for the strip, and
//     the strip's per-row sum of squares; gate_up consumes y unnormalised and scales its accumulators by the row's
//     1 / rms (summed from the 256 strip partials by the loader during the item), and so does the QKV projection.
//     One 64-workgroup norm phase and one flag hop per seam disappear.  Without a next layer (the last one) the
//     loader normalises its strip at the end (x = the final-norm input of the LM head).
//
// Work split (every workgroup b, cg = b >> 3, ks = b & 7):
//     O    columns 128 cg .. +128 (8 tiles), K chunks 4 ks .. +4                    -> fp32 slab ks
//     N1   strip 128 cg + 16 ks .. +16: resid += sum of 8 O slabs; xm = bf16(resid · w_ffn); ssq1[b][row]
//     GU   gate/up tiles 7b .. 7b + 6 (waves 0-6), all 32 K chunks of xm             -> h (SiLU(g·inv)·(u·inv))
//     D    columns 128 cg .. +128, K chunks 14 ks .. +14 (h columns)                 -> fp32 slab ks
//     N2   strip as N1 with the down slabs and w_next; x = bf16(resid · w_next); ssq2[b][row]
//     Q    (not on the last layer) next QKV: 6 tiles 6 (b >> 2) .. (waves 0-5), K chunks 8 (b & 3) .. +8 of x
//          -> fp32 slab (b & 3) of qkv_slabs, times inv2[row] (the folded attention sums the 4 slabs)
// Dependencies: N1 strip <- the 8 O items of its group; GU <- all 256 N1 strips; D (ks) <- the 32 GU items that
// produce h columns 1792 ks .. +1792; N2 strip <- the 8 D items of its group; Q <- all 256 N2 strips.
//
// Hand-offs (cdna_hip_programming.md Guideline 16; the "sc1 payload + agent atomic" form of MI355X_MICROARCH.md):
// every handed-off byte is stored write-through (sc1) by the loader wave, which drains its stores (vmcnt(0): it has
// nothing else in flight at that point) before one lane adds 1 to the counter (agent scope, relaxed, sharded by
// b & 7 on 128-B lines where 256 workgroups arrive).  Consumers poll relaxed (one lane per shard, s_sleep, bounded)
// and take one agent acquire before their LDS-DMA of the handed-off bytes.  Counters are monotonic (never zeroed):
// each workgroup reads the ones it polls at its start, and every counter's completion needs this workgroup's own
// O item (directly or through N1), so none can be complete then; target = base + expected, base = v0 - v0 % expected
// (powers of two: the uint32 wrap keeps the multiples).
//
// Deadlock freedom needs all 256 workgroups resident at once (one per CU), i.e. an exclusive GPU -- the engine enables
// this path only then (engine/model_runner.py).  Every spin is bounded: a timeout sets the health word p.err (read
// after each drained step) and the kernel completes with wrong values instead of hanging the GPU.
#include "gemm_epilogue.h"

namespace dsse {

namespace mega {
constexpr int kH = 4096, kF = 14336;             // Mistral-7B hidden / FFN (host-checked)
constexpr int kKCH = kH / 128, kKCF = kF / 128;  // K chunks: 32 / 112
constexpr int kWGs = 256;                        // one workgroup per CU
constexpr int kCW = 8;                           // compute waves
constexpr int kThreads = 64 * (kCW + 1);         // + the loader wave
constexpr int kRows = 64;                        // MT = 4 row tiles
constexpr int kXSlot = kRows * 256;              // 64 rows x 128 columns bf16, 16 KiB
constexpr int kXD = 3;                           // X ring slots: X(gs + 1) in flight while X(gs) is read
constexpr int kWD = 6;                           // register weight ring depth (steps)
constexpr int kLdsE = kXD * kXSlot;              // item result tile (<= 64 x 128 fp32 = 32 KiB)
constexpr int kLdsS = kLdsE + 32768;             // loader scratch: strip slabs (36 KiB) / ssq partials (64 KiB)
constexpr int kLdsInv = kLdsS + 65536;           // inv rms [2][64] fp32
constexpr int kLds = kLdsInv + 512;              // 147,968 B
static_assert(kLds <= 160 * 1024, "LDS budget");
// GEMM steps of one workgroup: O [0, 4), gate_up [4, 36), down [36, 50), next layer's QKV [50, 58)
constexpr int kOSteps = 4, kGUSteps = kKCH, kDSteps = kKCF / 8, kQSteps = 8;
constexpr int kGU0 = kOSteps, kD0 = kGU0 + kGUSteps, kQ0 = kD0 + kDSteps, kQEnd = kQ0 + kQSteps;
constexpr int kQN = 6144, kQTiles = 6;
// counters: k = index, 8 shard words each on its own 128-B line; group counters use (k0 + grp / 8, grp % 8)
enum { kCntOG = 0 /* 32 groups: 0..3 */, kCntN1 = 4, kCntGU = 5 /* 8 groups: 5..12 */, kCntDG = 13 /* 13..16 */,
       kCntN2 = 17, kSyncCounters = 18 };
constexpr int kSyncWords = kSyncCounters * 8 * 32;
constexpr int kSsqWords = 2 * kWGs * kRows;  // ssq1, ssq2: [256 strips][64 rows] fp32 after the counters
constexpr int kSpinLimit = 1 << 21;
constexpr int kAuxSc1 = 16;  // buffer cache policy: sc1 (write-through / L1-bypassing)
__host__ __device__ constexpr int sync_word(int k, int s) { return (8 * k + s) * 32; }
}  // namespace mega

namespace {

using namespace mega;

// 16 B per lane from a buffer (32-bit offsets: voffset per lane, soffset uniform) into LDS, lane-linear at lds_base
DEV void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, char* lds_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rs, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(lds_base)), 16, voff,
      soff, 0, 0);
}

DEV __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, uint32_t bytes) {
  const unsigned long long u = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return make_rsrc(reinterpret_cast<const void*>(((unsigned long long)hi << 32) | lo), bytes);
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Counter poll by one wave: lanes < nshards read one shard each (relaxed, agent scope), the sum is compared with
// the target (wrapping).  Bounded: on timeout sets the error word and returns.
DEV void wait_counter(unsigned* sync, unsigned* err, int k, int s0, int nshards, unsigned base, unsigned expected,
                      int lane) {
  unsigned* cnt = sync + sync_word(k, s0);
  for (int spins = 0;; ++spins) {
    unsigned v = lane < nshards ? __hip_atomic_load(cnt + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) v += __shfl_xor(v, o);
    v = __builtin_amdgcn_readfirstlane(v);
    if (v - base >= expected) return;
    if (spins >= kSpinLimit) {
      if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

DEV void signal_counter(unsigned* sync, int k, int shard) {
  __hip_atomic_fetch_add(sync + sync_word(k, shard), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Counter value summed over its 8 shards (lanes 0-7), wave-uniform.
DEV unsigned read_counter8(unsigned* sync, int k, int lane) {
  unsigned v = lane < 8 ? __hip_atomic_load(sync + sync_word(k, lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) v += __shfl_xor(v, o);
  return __builtin_amdgcn_readfirstlane(v);
}

DEV unsigned read_counter1(unsigned* sync, int k, int s) {
  return __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(sync + sync_word(k, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

}  // namespace

__global__ void __launch_bounds__(mega::kThreads) mega_mlp_kernel(MegaMlpParams p) {
  using namespace mega;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int M = p.M;
  const int ks = b & 7, cg = b >> 3;
  const bool has_q = p.wqkv != nullptr;
  const int nsteps = has_q ? kQEnd : kQ0;
  float* inv_lds = reinterpret_cast<float*>(smem + kLdsInv);  // [0..63] inv rms of N1, [64..127] of N2

  // optional phase stamps (bench_mega.py --stamps): the loader wave's lane 0, 100 MHz wall clock, slot i of 16
  auto stamp = [&](int i) {
    if (p.stamps != nullptr && w == kCW && lane == 0) p.stamps[b * 16 + i] = __builtin_amdgcn_s_memrealtime();
  };

  if (w < kCW) {
    // =============================== compute waves ===============================
    // weight block of step gs for this wave (bytes 0: the wave idles in this step's item, or gs is past the end)
    auto w_src = [&](int gs, uint32_t& bytes) -> const bf16* {
      bytes = 4096;
      if (gs < kGU0) return p.wo + ((size_t)(8 * cg + w) * kKCH + 4 * ks + gs) * kTileChunk;
      if (gs < kD0) {
        if (w >= 7) bytes = 0;  // gate_up items are 7 tiles: wave 7 idles
        return p.wgu + ((size_t)(7 * b + min(w, 6)) * kKCH + (gs - kGU0)) * kTileChunk;
      }
      if (gs < kQ0) return p.wd + ((size_t)(8 * cg + w) * kKCF + kDSteps * ks + (gs - kD0)) * kTileChunk;
      if (gs < nsteps) {
        if (w >= kQTiles) bytes = 0;
        return p.wqkv + ((size_t)(kQTiles * (b >> 2) + min(w, kQTiles - 1)) * kKCH + kQSteps * (b & 3) + (gs - kQ0)) *
                            kTileChunk;
      }
      bytes = 0;
      return p.wo;
    };
    auto load_w = [&](int gs, bf16x8 (&wr)[4]) {
      uint32_t bytes;
      const bf16* src = w_src(gs, bytes);
      // always 4 loads (an idle or past-the-end step reads through a 0-byte descriptor: zeros, no memory traffic), so
      // every path through the unrolled ring issues the same count and the compiler's vmcnt waits keep kWD - 1 steps
      // in flight (a skipped load on some path makes it wait for everything)
      const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(src, bytes);
#pragma unroll
      for (int s = 0; s < 4; ++s) wr[s] = ld_buf_bf16x8<kAuxNT>(rs, 1024 * s + lane * 16);
    };

    bf16x8 wr[kWD][4];
#pragma unroll
    for (int j = 0; j < kWD; ++j) load_w(j, wr[j]);
    f32x4 acc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float* E = reinterpret_cast<float*>(smem + kLdsE);
    bf16* Eh = reinterpret_cast<bf16*>(smem + kLdsE);

    for (int base = 0; base < nsteps; base += kWD) {
#pragma unroll
      for (int j = 0; j < kWD; ++j) {
        const int gs = base + j;
        if (gs < nsteps) {
          // items: O [0, 4) (kind 0: slab tile), gate_up [4, 36) (kind 1, 7 active waves), down [36, 50) (kind 0), QKV
          // [50, 58) (kind 2, 6 active waves)
          const int active = gs < kGU0 ? kCW : gs < kD0 ? 7 : gs < kQ0 ? kCW : kQTiles;
          // X(gs) published by the loader; every wave's reads of the slot X(gs + 2) reuses were done (lgkmcnt)
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          if (w < active) {
            const char* xb = smem + (gs % kXD) * kXSlot;
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const int ch = ((4 * g + s) ^ swz(r)) << 4;
              bf16x8 xf[4];
#pragma unroll
              for (int mt = 0; mt < 4; ++mt) xf[mt] = *reinterpret_cast<const bf16x8*>(xb + (16 * mt + r) * 256 + ch);
#pragma unroll
              for (int mt = 0; mt < 4; ++mt) acc[mt] = mfma16x16x32(xf[mt], wr[j][s], acc[mt]);
            }
            __builtin_amdgcn_s_setprio(0);
          }
        }
        load_w(gs + kWD, wr[j]);  // the ring slot just consumed takes the step kWD ahead (on every path: see load_w)
        if (gs < nsteps) {
          const int c = gs < kGU0 ? gs : gs < kD0 ? gs - kGU0 : gs < kQ0 ? gs - kD0 : gs - kQ0;
          const int nc = gs < kGU0 ? kOSteps : gs < kD0 ? kGUSteps : gs < kQ0 ? kDSteps : kQSteps;
          const int kind = gs < kGU0 ? 0 : gs < kD0 ? 1 : gs < kQ0 ? 0 : 2;
          const int active = gs < kGU0 ? kCW : gs < kD0 ? 7 : gs < kQ0 ? kCW : kQTiles;
          if (c == nc - 1) {
            // item result -> LDS tile E (the loader stores it, so nothing younger than the weight loads is drained here)
            if (w < active) {
              if (kind == 0) {  // fp32 [64][128]: column 16 w + r
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                  for (int i = 0; i < 4; ++i) E[(16 * mt + 4 * g + i) * 128 + 16 * w + r] = acc[mt][i];
              } else if (kind == 2) {  // fp32 [64][96] times inv2[row]
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                  for (int i = 0; i < 4; ++i) {
                    const int m = 16 * mt + 4 * g + i;
                    E[m * 96 + 16 * w + r] = acc[mt][i] * inv_lds[64 + m];
                  }
              } else {  // gate_up: SiLU(gate·inv)·(up·inv) -> bf16 [64][56], tile w -> h columns 8 w .. 8 w + 7
                const bool lo = r < 8;
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                  float pr[4];
#pragma unroll
                  for (int i = 0; i < 4; ++i) pr[i] = __shfl_xor(acc[mt][i], 8);
#pragma unroll
                  for (int k = 0; k < 2; ++k) {
                    const int m = 16 * mt + 4 * g + (lo ? k : 2 + k);
                    const float inv = inv_lds[m];
                    const float gate = (lo ? acc[mt][k] : pr[2 + k]) * inv, up = (lo ? pr[k] : acc[mt][2 + k]) * inv;
                    Eh[m * 56 + 8 * w + (r & 7)] = f2bf(silu(gate) * up);
                  }
                }
              }
            }
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // end of item: E complete
          }
        }
      }
    }
    return;
  }

  // =============================== loader / publisher wave ===============================
  stamp(0);
  float* ssq1 = reinterpret_cast<float*>(p.sync + kSyncWords);
  float* ssq2 = ssq1 + kWGs * kRows;
  char* S = smem + kLdsS;
  const float* E = reinterpret_cast<const float*>(smem + kLdsE);

  // ---- counters this workgroup polls: bases read before it contributes anything ----
  const unsigned v_og = read_counter1(p.sync, kCntOG + (cg >> 3), cg & 7);
  const unsigned v_n1 = read_counter8(p.sync, kCntN1, lane);
  const unsigned v_gu = read_counter1(p.sync, kCntGU + ks, 0);
  const unsigned v_dg = read_counter1(p.sync, kCntDG + (cg >> 3), cg & 7);
  const unsigned v_n2 = read_counter8(p.sync, kCntN2, lane);
  const unsigned base_og = v_og - v_og % 8u, base_n1 = v_n1 - v_n1 % 256u, base_gu = v_gu - v_gu % 32u;
  const unsigned base_dg = v_dg - v_dg % 8u, base_n2 = v_n2 - v_n2 % 256u;

  // X(gs) = 64 rows x 128 columns of the step's activation into X slot gs % 3 (16 DMA instructions)
  auto issue_x = [&](int gs) {
    const bf16* X;
    int ldx, col;
    if (gs < kGU0) { X = p.attn; ldx = kH; col = 128 * (4 * ks + gs); }
    else if (gs < kD0) { X = p.xm; ldx = kH; col = 128 * (gs - kGU0); }
    else if (gs < kQ0) { X = p.h; ldx = kF; col = 128 * (kDSteps * ks + gs - kD0); }
    else { X = p.x; ldx = kH; col = 128 * (kQSteps * (b & 3) + gs - kQ0); }
    char* base = smem + (gs % kXD) * kXSlot;
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(X, (uint32_t)M * ldx * 2);
#pragma unroll
    for (int i = 0; i < kRows / 4; ++i) {  // 4 rows x 256 B per instruction, XOR-swizzled 16-byte pieces
      const int row = 4 * i + g;
      dma16(rs, (uint32_t)(min(row, M - 1) * ldx + 8 * (r ^ swz(row & 15))) * 2, (uint32_t)col * 2, base + i * 1024);
    }
  };
  // the X stream of one item: one barrier per step (X(gs) landed, published), then the end-of-item barrier (E
  // written); `hook(c)` runs after step c's barrier
  auto x_item = [&](int gs0, int nc, auto hook) {
    issue_x(gs0);
    if (nc > 1) issue_x(gs0 + 1);
    for (int c = 0; c < nc; ++c) {
      if (c + 1 < nc) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      if (c + 2 < nc) issue_x(gs0 + c + 2);
      hook(c);
    }
    asm volatile("s_barrier" ::: "memory");
  };
  auto no_hook = [](int) {};
  auto acquire = [&]() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); };

  // E (fp32 [64][ncols]) -> dst rows (row stride ld floats), write-through; rows >= M fall outside the descriptor
  auto store_tile_f32 = [&](float* dst, int ld, int ncols) {
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(dst, (uint32_t)((M - 1) * ld + ncols) * 4);
    const int ppr = ncols / 4;  // 16-byte pieces per row
#pragma unroll 4
    for (int q = lane; q < kRows * ppr; q += 64) {
      const int row = q / ppr, pc = q % ppr;
      const u32x4 v = *reinterpret_cast<const u32x4*>(E + row * ncols + 4 * pc);
      if (row < M) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)(row * ld + 4 * pc) * 4, 0, kAuxSc1);
    }
  };
  // the 16-column strip of this workgroup: resid += sum of the 8 slabs; y = bf16(resid · wn) (y may be null);
  // ssq_out[b][row] = sum of squares over the strip.  Lane = row.  Returns the strip's new residual in v.
  const int col0 = 128 * cg + 16 * ks;
  auto strip = [&](const bf16* wn, bf16* y, float* ssq_out, float (&v)[16]) {
    // 8 slabs + the residual, 64 rows x 64 B each, by LDS-DMA into S[9][64 rows][16 floats]
    const __amdgpu_buffer_rsrc_t slr = uniform_rsrc(p.slabs, (uint32_t)8 * M * kH * 4);
    const __amdgpu_buffer_rsrc_t rr0 = uniform_rsrc(p.resid, (uint32_t)M * kH * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t vo = (uint32_t)(min(16 * i + (lane >> 2), M - 1) * kH + col0 + 4 * (lane & 3)) * 4;
#pragma unroll
      for (int s = 0; s < 8; ++s) dma16(slr, vo, (uint32_t)s * M * kH * 4, S + (s * 4 + i) * 1024);
      dma16(rr0, vo, 0, S + (32 + i) * 1024);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const float* Sf = reinterpret_cast<const float*>(S);
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = Sf[(8 * 64 + lane) * 16 + j];
#pragma unroll 1
    for (int s = 0; s < 8; ++s)  // one slab at a time (the loader's registers are the kernel's budget too)
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] += Sf[(s * 64 + lane) * 16 + j];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) ss += v[j] * v[j];
    const bool live = lane < M;
    const __amdgpu_buffer_rsrc_t rr = uniform_rsrc(p.resid, (uint32_t)M * kH * 4);
    if (live) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v[4 * q]), __float_as_uint(v[4 * q + 1]),
                                                     __float_as_uint(v[4 * q + 2]), __float_as_uint(v[4 * q + 3])},
                                               rr, (uint32_t)(lane * kH + col0 + 4 * q) * 4, 0, kAuxSc1);
      if (y != nullptr) {
        const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(y, (uint32_t)M * kH * 2);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bf16x8 wv = *reinterpret_cast<const bf16x8*>(wn + col0 + 8 * q);
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(v[8 * q + j] * bf2f(wv[j]));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), yr, (uint32_t)(lane * kH + col0 + 8 * q) * 2,
                                                 0, kAuxSc1);
        }
      }
    }
    const __amdgpu_buffer_rsrc_t sr = uniform_rsrc(ssq_out, kWGs * kRows * 4);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ss), sr, (uint32_t)(b * kRows + lane) * 4, 0, kAuxSc1);
  };
  // per-row inverse RMS from the 256 strip partials ssq[256][64] (DMA'd into S earlier): inv_lds[slot + row]
  auto issue_ssq = [&](const float* ssq) {
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(ssq, kWGs * kRows * 4);
#pragma unroll
    for (int i = 0; i < kWGs * kRows / 256; ++i) dma16(rs, lane * 16, i * 1024, S + i * 1024);
  };
  auto inv_from_ssq = [&](int slot) {
    const float* Sf = reinterpret_cast<const float*>(S);
    float t = 0.f;
#pragma unroll 16
    for (int i = 0; i < kWGs; ++i) t += Sf[i * kRows + lane];
    inv_lds[slot + lane] = rsqrtf(t / (float)kH + p.eps);
  };

  // ---- O ----
  x_item(0, kOSteps, no_hook);  // attn came from the previous launch: no dependency
  store_tile_f32(p.slabs + (size_t)ks * M * kH + 128 * cg, kH, 128);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) signal_counter(p.sync, kCntOG + (cg >> 3), cg & 7);
  stamp(1);
  // ---- N1 strip ----
  float v[16];
  wait_counter(p.sync, p.err, kCntOG + (cg >> 3), cg & 7, 1, base_og, 8u, lane);
  acquire();
  stamp(2);
  strip(p.w_ffn, p.xm, ssq1, v);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) signal_counter(p.sync, kCntN1, b & 7);
  stamp(3);
  // ---- gate_up ----
  wait_counter(p.sync, p.err, kCntN1, 0, 8, base_n1, 256u, lane);
  acquire();
  stamp(4);
  issue_ssq(ssq1);  // retired by step 0's wait (older than X)
  x_item(kGU0, kGUSteps, [&](int c) {
    if (c == 0) inv_from_ssq(0);  // published to the compute waves by step 1's barrier
  });
  stamp(5);
  {
    const __amdgpu_buffer_rsrc_t hr = uniform_rsrc(p.h, (uint32_t)M * kF * 2);
    const bf16* Eh = reinterpret_cast<const bf16*>(smem + kLdsE);
#pragma unroll
    for (int q = lane; q < kRows * 7; q += 64) {  // 7 pieces of 16 B per row
      const int row = q / 7, pc = q % 7;
      const u32x4 val = *reinterpret_cast<const u32x4*>(Eh + row * 56 + 8 * pc);
      if (row < M) __builtin_amdgcn_raw_buffer_store_b128(val, hr, (uint32_t)(row * kF + 56 * b + 8 * pc) * 2, 0, kAuxSc1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) signal_counter(p.sync, kCntGU + (b >> 5), 0);
  stamp(6);
  // ---- down ----
  wait_counter(p.sync, p.err, kCntGU + ks, 0, 1, base_gu, 32u, lane);
  acquire();
  stamp(7);
  x_item(kD0, kDSteps, no_hook);
  store_tile_f32(p.slabs + (size_t)ks * M * kH + 128 * cg, kH, 128);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) signal_counter(p.sync, kCntDG + (cg >> 3), cg & 7);
  stamp(8);
  // ---- N2 strip ----
  wait_counter(p.sync, p.err, kCntDG + (cg >> 3), cg & 7, 1, base_dg, 8u, lane);
  acquire();
  stamp(9);
  strip(p.w_next, has_q ? p.x : nullptr, ssq2, v);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) signal_counter(p.sync, kCntN2, b & 7);
  stamp(10);
  wait_counter(p.sync, p.err, kCntN2, 0, 8, base_n2, 256u, lane);
  acquire();
  stamp(11);
  issue_ssq(ssq2);
  if (has_q) {
    // ---- next layer's QKV ----
    x_item(kQ0, kQSteps, [&](int c) {
      if (c == 0) inv_from_ssq(64);
    });
    store_tile_f32(p.qkv_slabs + (size_t)(b & 3) * M * kQN + kQTiles * 16 * (b >> 2), kQN, kQTiles * 16);
  } else {
    // ---- last layer: x = the normalised strip (the LM head's input) ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const float* Sf = reinterpret_cast<const float*>(S);
    float t = 0.f;
#pragma unroll 16
    for (int i = 0; i < kWGs; ++i) t += Sf[i * kRows + lane];
    const float inv = rsqrtf(t / (float)kH + p.eps);
    if (lane < M) {
      const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(p.x, (uint32_t)M * kH * 2);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const bf16x8 wv = *reinterpret_cast<const bf16x8*>(p.w_next + col0 + 8 * q);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(v[8 * q + j] * inv * bf2f(wv[j]));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), xr, (uint32_t)(lane * kH + col0 + 8 * q) * 2,
                                               0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp(12);
}

}  // namespace dsse

using namespace dsse;

extern "C" size_t dsse_mega_sync_words() { return (size_t)mega::kSyncWords + mega::kSsqWords; }

// Shapes are the Mistral-7B ones (H 4096, F 14336) and M <= 64; the caller (bindings.cpp) validates them.
extern "C" hipError_t dsse_mega_mlp(const MegaMlpParams* p, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mega_mlp_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, mega::kLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(mega_mlp_kernel, dim3(mega::kWGs), dim3(mega::kThreads), mega::kLds, st, *p);
  return hipGetLastError();
}

DSSE_CHECK_READER(dsse_check_decode_mega)
