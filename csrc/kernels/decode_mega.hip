// Persistent decode MLP block ("mega" kernel): one launch per layer runs
//
//     O projection (split-K slabs) -> residual + RMSNorm -> gate_up + SiLU·mul -> down (split-K slabs)
//     -> residual + RMSNorm with the next layer's weight
//
// for <= 64 decode rows (MT = 4 MFMA row tiles), replacing five launches of the launch-per-op step
// (gemm_ring o, rmsnorm<3>, gemm_ring gate_up, gemm_ring down, rmsnorm<3>; profiles/r3/decode_step_64_r3.md:
// ~45 us of fixed cost per 131 us layer, 7 launches, VERDICT round 3 "next 1").
//
// Why it can be faster.  Every HBM byte a decode MLP block reads (weights: 33.5 + 235 + 117 MB) is independent of
// the activations; only the 0.5-1.8 MB activation hand-offs are on the dependency chain.  Between launches the weight
// stream stops (tail of one grid, launch boundary, first-load latency of the next: 5.5-7.5 us per GEMM launch).  Here
// each workgroup's weight ring keeps streaming ACROSS the seams: a compute wave always has its next two 4 KiB weight
// chunks in flight, and at an item boundary those are the next item's chunks, issued before the workgroup waits for
// that item's inputs (MI355X_MICROARCH.md price list, prefetch-credit; engine-vs-launches 0.87-0.89x at batch 1).
//
// Structure (256 workgroups = one per CU, 9 waves each):
//   * waves 0-7 compute: each owns one 16-column weight tile of the current work item and a private 3-slot LDS
//     ring of 4 KiB weight chunks (buffer_load ... lds, non-temporal), filled two GEMM steps ahead by itself and
//     waited for by its own counted vmcnt (gemm_ring2's weight ring, csrc/kernels/gemm_stream.hip);
//   * wave 8 loads X (the activation, 64 rows x 128 columns per step = 16 KiB, XOR-swizzled image) into a 3-slot
//     ring by global_load_lds, after waiting for the item's dependency counter and an agent-scope acquire;
//   * one s_barrier per GEMM step publishes X(step) and retires the compute waves' reads of step - 1.
//   Static work split (each workgroup: one O item, one gate_up item, one down item; rows' norms on 64 + 64
//   workgroups), in dependency order per workgroup:
//       O    item b:  columns 128 (b >> 3) .. +128 (8 tiles), K chunks 4 (b & 7) .. +4      -> slab (b & 7)
//       N1   row b (b < 64):  resid += sum of the 8 O slabs; xm = rmsnorm(resid) * w_ffn
//       GU   item b:  gate/up tiles 7b .. 7b + 6 (waves 0-6), all 32 K chunks              -> h (SiLU·mul)
//       D    item b:  columns 128 (b >> 3) .. +128, K chunks 14 (b & 7) .. +14 (h columns)   -> slab (b & 7)
//       N2   row b - 64 (64 <= b < 128): resid += sum of the 8 D slabs; x = rmsnorm(resid) * w_next
//       Q    (optional, every layer but the last) the next layer's QKV projection of x: columns 96 (b >> 2) .. +96
//            (6 tiles, waves 0-5), K chunks 8 (b & 3) .. +8 -> fp32 slab (b & 3) of qkv_slabs, summed + RoPE'd by the
//            folded decode attention kernel that runs next (attention.hip mode 3)
//   Dependencies (counters in `sync`, never reset: see below): N1 <- all 256 O items; GU <- all 64 N1 rows;
//   D item (ks) <- the 32 GU items that produce its K range (h columns 1792 ks .. +1792); N2 <- all 256 D items;
//   Q <- all 64 N2 rows.
//
// Hand-offs (cdna_hip_programming.md Guideline 16, the "sc1 payload + agent atomic" row of MI355X_MICROARCH.md's
// valid forms): every handed-off byte (slabs, h, xm, resid, x) is stored write-through (sc1) by buffer stores; each
// storing wave drains its stores (counted vmcnt, below), the workgroup meets at an s_barrier, and ONE lane adds 1 to
// the item's counter (agent scope, relaxed; the O / D / attention counters sharded by XCD label b & 7 and the norm
// counters by row & 7, each shard on its own 128-B line: 64 arrivals on one word took 3.4-4.8 us to become visible to
// the pollers, profiles/r4/mega_r4.md).
// Consumers poll relaxed (one lane per shard, s_sleep, bounded) and then either load with sc1 buffer loads to
// registers (norm rows: acquire-free) or, for the X ring's LDS-DMA, take ONE agent acquire first.
// Counters are monotonic (never zeroed): a workgroup reads every counter it will poll at its start, before it has
// contributed anything, and since every counter's completion needs ALL O items (the first item of every workgroup),
// none can be complete at that time; the target is base + expected with base = v0 - v0 % expected (expected a power
// of two, so the uint32 wrap-around keeps the multiples).
//
// Deadlock freedom needs all 256 workgroups resident at once (one per CU: 147 KiB of LDS each), i.e. an exclusive
// GPU -- the engine enables this path only then (engine/model_runner.py).  Every spin is bounded: a timeout sets
// the engine's health word p.err (read after each drained step) and the kernel completes with wrong values instead
// of hanging the GPU.
//
// W vmcnt accounting per compute wave: 4 LDS-DMA instructions per GEMM step (dummy steps load through a 0-byte
// descriptor: no memory traffic, same count), so "W(step) landed" is vmcnt(4) (W(step + 1) may stay in flight).
// Item-end stores are issued before that step's weight refill, so the same vmcnt(4) retires them.
#include "gemm_epilogue.h"

namespace dsse {

namespace mega {
constexpr int kH = 4096, kF = 14336;         // Mistral-7B hidden / FFN (host-checked)
constexpr int kKCH = kH / 128, kKCF = kF / 128;  // K chunks: 32 / 112
constexpr int kWGs = 256;                    // one workgroup per CU
constexpr int kCW = 8;                       // compute waves
constexpr int kThreads = 64 * (kCW + 1);     // + the X loader wave
constexpr int kRows = 64;                    // MT = 4 row tiles
constexpr int kXSlot = kRows * 256;          // 64 rows x 128 columns bf16, 16 KiB
constexpr int kWSlot = 4096;                 // one (16-column tile, 128-deep chunk) weight block
constexpr int kD = 3;                        // ring slots (X and W): 2 steps in flight + 1 being read
constexpr int kLdsW = kD * kXSlot;           // weight rings after the X ring
constexpr int kLdsCtl = kLdsW + kCW * kD * kWSlot;
// control area: norm partial sums [8] at +0, attention merge statistics [2][4][16] x (m, l) at +64 (1 KiB)
constexpr int kLdsFq = kLdsCtl + 2048;           // attention phase: per wave 6 x 128 bf16 (4 q heads, k, v)
constexpr int kLdsTrash = kLdsFq + kCW * 6 * 256;  // 1 KiB sink of the seam prefetch DMAs (contents never read)
constexpr int kLds = kLdsTrash + 1024;               // 162,816 B
static_assert(kLds <= 160 * 1024, "LDS budget");
// Seam prefetch: at the start of an item with a dependency, each compute wave issues kPF more steps of its weight
// stream (steps 2 .. 2 + kPF - 1 of the item; 0 and 1 are already in its ring) as default-policy loads whose data
// lands in the trash slot: they run while the workgroup waits at the seam and leave the lines in L2 / MALL, so the
// ring's own (nt) loads of those steps hit there.  p.pf_steps (<= kPF) of them are real, the rest dummies (0-byte
// descriptor: the vmcnt accounting is the same either way).
constexpr int kPF = 4;
static_assert(2 * 3 * 32 * 64 * 4 <= kD * kXSlot, "attention merge area fits the X ring");
// GEMM steps of one workgroup: O [0, 4), gate_up [4, 36), down [36, 50), next layer's QKV [50, 58)
constexpr int kOSteps = 4, kGUSteps = kKCH, kDSteps = kKCF / 8;
constexpr int kGU0 = kOSteps, kD0 = kGU0 + kGUSteps, kSteps = kD0 + kDSteps;
constexpr int kQN = 6144, kQTiles = 6, kQSplit = 4, kQSteps = kKCH / kQSplit;  // 64 x 96-col groups x 4 K splits
constexpr int kQ0 = kSteps, kSteps2 = kQ0 + kQSteps;
// sync words: counter k, shard s at word (8 k + s) * 32 (one 128-B line each)
enum { kCntO = 0, kCntN1 = 1, kCntGU = 2 /* + group 0..7 */, kCntD = 10, kCntN2 = 11, kCntA = 12, kSyncCounters = 13 };
constexpr int kSpinLimit = 1 << 21;
constexpr int kAuxSc1 = 16;   // buffer cache policy: sc1 (write-through / L1-bypassing)
__host__ __device__ constexpr int sync_word(int k, int s) { return (8 * k + s) * 32; }
}  // namespace mega


namespace {

using namespace mega;

DEV void mega_glds16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds(const_cast<void*>(src),
                                   reinterpret_cast<__attribute__((address_space(3))) void*>(
                                       reinterpret_cast<uintptr_t>(lds_base)),
                                   16, 0, 0);
}

DEV __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, uint32_t bytes) {
  const unsigned long long u = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return make_rsrc(reinterpret_cast<const void*>(((unsigned long long)hi << 32) | lo), bytes);
}

// Counter poll by one wave: lanes < nshards read one shard each (relaxed, agent scope), the sum is compared with
// the target (wrapping).  Bounded: on timeout sets the error word and returns.
DEV void wait_counter(unsigned* sync, unsigned* err, int k, int nshards, unsigned base, unsigned expected, int lane) {
  unsigned* cnt = sync + sync_word(k, 0);
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

// Raw barrier after this wave's own vmcnt wait (no __syncthreads: its fence would drain the weight DMA in flight).
template <int N>
DEV void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

}  // namespace

__global__ void __launch_bounds__(mega::kThreads) mega_mlp_kernel(MegaMlpParams p) {
  using namespace mega;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const bool loader = w == kCW;
  const int M = p.M;
  const int ks = b & 7, cg = b >> 3;   // O / D item: split and 128-column group
  float* red = reinterpret_cast<float*>(smem + kLdsCtl);

  // ---- compute-wave weight stream: GEMM step gs -> this wave's (tile, chunk) block ----
  auto w_src = [&](int gs, uint32_t& bytes) -> const bf16* {
    bytes = kWSlot;
    if (gs < kGU0) return p.wo + ((size_t)(8 * cg + w) * kKCH + 4 * ks + gs) * kTileChunk;
    if (gs < kD0) {
      if (w >= 7) bytes = 0;  // gate_up items are 7 tiles: wave 7 streams nothing (range-failed dummy loads)
      return p.wgu + ((size_t)(7 * b + min(w, 6)) * kKCH + (gs - kGU0)) * kTileChunk;
    }
    if (gs < kSteps) return p.wd + ((size_t)(8 * cg + w) * kKCF + kDSteps * ks + (gs - kD0)) * kTileChunk;
    if (gs < kSteps2 && p.wqkv != nullptr) {  // next layer's QKV: 6 tiles (waves 0-5) x 8 chunks
      if (w >= kQTiles) bytes = 0;
      return p.wqkv + ((size_t)(kQTiles * (b >> 2) + min(w, kQTiles - 1)) * kKCH + kQSteps * (b & 3) + (gs - kQ0)) *
                          kTileChunk;
    }
    bytes = 0;
    return p.wo;
  };
  auto issue_w = [&](int gs) {
    uint32_t bytes;
    const bf16* src = w_src(gs, bytes);
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(src, bytes);
    char* dst = smem + kLdsW + (w * kD + gs % kD) * kWSlot;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(dst + 1024 * s)),
          16, 1024 * s + lane * 16, 0, 0, kAuxNT);
  };

  auto issue_pf = [&](int gs, bool real) {
    uint32_t bytes;
    const bf16* src = w_src(gs, bytes);
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(src, real ? bytes : 0u);
#pragma unroll
    for (int s = 0; s < 4; ++s)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(smem + kLdsTrash)),
          16, 1024 * s + lane * 16, 0, 0, 0);
  };

  // ---- loader: X(gs) = 64 rows x 128 columns of the step's activation into X slot gs % 3 ----
  auto issue_x = [&](int gs) {
    const bf16* X;
    int ldx, col;
    if (gs < kGU0) { X = p.attn; ldx = kH; col = 128 * (4 * ks + gs); }
    else if (gs < kD0) { X = p.xm; ldx = kH; col = 128 * (gs - kGU0); }
    else if (gs < kSteps) { X = p.h; ldx = kF; col = 128 * (kDSteps * ks + gs - kD0); }
    else { X = p.x; ldx = kH; col = 128 * (kQSteps * (b & 3) + gs - kQ0); }
    char* base = smem + (gs % kD) * kXSlot;
#pragma unroll
    for (int i = 0; i < kRows / 4; ++i) {  // 16 DMA instructions of 4 rows x 256 B
      const int row = 4 * i + g;
      mega_glds16(X + (size_t)min(row, M - 1) * ldx + col + 8 * (r ^ swz(row & 15)), base + i * 1024);
    }
  };

  // ---- counters this workgroup polls: bases read before it contributes anything ----
  unsigned base_o = 0, base_n1 = 0, base_gu = 0, base_d = 0, base_n2 = 0, base_a = 0;
  if (loader) {
    auto rd = [&](int k, int s) { return __hip_atomic_load(p.sync + sync_word(k, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    unsigned vo = lane < 8 ? rd(kCntO, lane) : 0u, vd = lane < 8 ? rd(kCntD, lane) : 0u;
    unsigned va = lane < 8 ? rd(kCntA, lane) : 0u;
    unsigned vn1 = lane < 8 ? rd(kCntN1, lane) : 0u, vn2 = lane < 8 ? rd(kCntN2, lane) : 0u;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      vo += __shfl_xor(vo, o);
      vd += __shfl_xor(vd, o);
      va += __shfl_xor(va, o);
      vn1 += __shfl_xor(vn1, o);
      vn2 += __shfl_xor(vn2, o);
    }
    vo = __builtin_amdgcn_readfirstlane(vo);
    vd = __builtin_amdgcn_readfirstlane(vd);
    va = __builtin_amdgcn_readfirstlane(va);
    vn1 = __builtin_amdgcn_readfirstlane(vn1);
    vn2 = __builtin_amdgcn_readfirstlane(vn2);
    base_a = va - va % 256u;
    const unsigned vgu = __builtin_amdgcn_readfirstlane(rd(kCntGU + ks, 0));
    base_n2 = vn2 - vn2 % 64u;
    base_o = vo - vo % 256u;
    base_d = vd - vd % 256u;
    base_n1 = vn1 - vn1 % 64u;
    base_gu = vgu - vgu % 32u;
  }

  // optional phase stamps (bench_mega.py --stamps): the loader wave's lane 0, 100 MHz wall clock, slot i of 16
  auto stamp = [&](int i) {
    if (p.stamps != nullptr && loader && lane == 0) p.stamps[b * 16 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  f32x4 acc[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (!loader) {
    issue_w(0);
    issue_w(1);
  }

  // ---- one GEMM item: steps [gs0, gs0 + nc) ----
  // kind 0 = O / D (fp32 slab ks), 1 = gate_up (SiLU·mul -> h), 2 = next layer's QKV (fp32 slab b & 3 of
  // qkv_slabs).  dep: counter polled before the first X load; sig_k < 0: no completion counter.
  auto gemm_item = [&](int gs0, int nc, int kind, int active, int dep_k, int dep_shards, unsigned dep_base,
                       unsigned dep_exp, int sig_k, int sig_shard, int st) {
    if (loader) {
      if (dep_k >= 0) {
        wait_counter(p.sync, p.err, dep_k, dep_shards, dep_base, dep_exp, lane);
        if (st == 6) stamp(15);  // gate_up: dependency seen, before the acquire
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // X arrives by LDS-DMA: drop this CU's stale lines
        stamp(st);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      int issued = gs0;
      issue_x(issued++);
      if (nc > 1) issue_x(issued++);
      for (int c = 0; c < nc; ++c) {
        const int gs = gs0 + c;
        if (issued - gs - 1 >= 1) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        if (issued < gs0 + nc) issue_x(issued++);
      }
      __builtin_amdgcn_s_barrier();  // end of item
      stamp(st + 1);
      return;
    }
    const bool on = w < active;
    const bool pf = dep_k >= 0;  // seam prefetch (kPF steps, see kPF)
    if (pf) {
#pragma unroll
      for (int i = 0; i < kPF; ++i) issue_pf(gs0 + 2 + i, i < p.pf_steps && 2 + i < nc);
    }
    for (int c = 0; c < nc; ++c) {
      const int gs = gs0 + c;
      // own W(gs) landed; X(gs) published by the loader.  In the first two steps after a prefetch the kPF
      // prefetch steps (and W(gs + 1)) are younger than W(gs) and may stay in flight.
      if (pf && c < 2) vm_barrier<4 + 4 * kPF>();
      else vm_barrier<4>();
      if (on) {
        const char* xb = smem + (gs % kD) * kXSlot;
        const char* wb = smem + kLdsW + (w * kD + gs % kD) * kWSlot + lane * 16;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int ch = ((4 * g + s) ^ swz(r)) << 4;
          bf16x8 xf[4];
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) xf[mt] = *reinterpret_cast<const bf16x8*>(xb + (16 * mt + r) * 256 + ch);
          const bf16x8 wf = *reinterpret_cast<const bf16x8*>(wb + 1024 * s);
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) acc[mt] = mfma16x16x32(xf[mt], wf, acc[mt]);
        }
      }
      if (c == nc - 1 && on) {
        if (kind == 2) {
          const __amdgpu_buffer_rsrc_t rs =
              uniform_rsrc(p.qkv_slabs + (size_t)(b & 3) * M * kQN, (uint32_t)M * kQN * 4);
          const int n = 16 * (kQTiles * (b >> 2) + w) + r;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[mt][i]), rs,
                                                    (uint32_t)(((16 * mt + 4 * g + i) * kQN + n) * 4), 0, kAuxSc1);
        } else if (kind == 0) {
          // fp32 slab ks: part[ks][m][n], rows >= M dropped by the descriptor's range check
          const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(p.slabs + (size_t)ks * M * kH, (uint32_t)M * kH * 4);
          const int n = 16 * (8 * cg + w) + r;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[mt][i]), rs,
                                                    (uint32_t)(((16 * mt + 4 * g + i) * kH + n) * 4), 0, kAuxSc1);
        } else {
          // SiLU·mul (silu_epilogue4's lane pairing): tile t -> h columns 8t .. 8t + 7
          const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(p.h, (uint32_t)M * kF * 2);
          const int t = 7 * b + w;
          const bool lo = r < 8;
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            float pr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) pr[i] = __shfl_xor(acc[mt][i], 8);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              const float gate = lo ? acc[mt][k] : pr[2 + k], up = lo ? pr[k] : acc[mt][2 + k];
              const int m = 16 * mt + 4 * g + (lo ? k : 2 + k);
              const bf16 hv = f2bf(silu(gate) * up);
              __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, hv), rs,
                                                    (uint32_t)((m * kF + 8 * t + (r & 7)) * 2), 0, kAuxSc1);
            }
          }
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      issue_w(gs + kD - 1);  // after the item-end stores: the next vmcnt(4) retires them
    }
    vm_barrier<4>();  // end of item: every wave's stores retired
    if (sig_k >= 0 && w == 0 && lane == 0) signal_counter(p.sync, sig_k, sig_shard);
  };

  // ---- one norm row: resid[m] += sum of the 8 slabs; y[m] = rmsnorm(resid[m]) * wn (sc1 loads / stores) ----
  auto norm_item = [&](int m, const bf16* wn, bf16* y, int dep_k, int dep_shards, unsigned dep_base, int sig_k,
                       int st) {
    if (loader) {
      wait_counter(p.sync, p.err, dep_k, dep_shards, dep_base, 256u, lane);
      stamp(st);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_barrier();
      stamp(st + 1);
      return;
    }
    __builtin_amdgcn_s_barrier();  // the loader's poll matched: the slabs are complete (sc1 loads below)
    const bool live = m < M;
    const int c0 = 8 * (64 * w + lane);  // this thread's 8 columns
    float v[8];
    if (live) {
      const __amdgpu_buffer_rsrc_t rr = uniform_rsrc(p.resid + (size_t)m * kH, kH * 4);
      const __amdgpu_buffer_rsrc_t sr = uniform_rsrc(p.slabs + (size_t)m * kH, (uint32_t)(7 * M * kH + kH) * 4);
      typedef float f32x4v __attribute__((ext_vector_type(4)));
      f32x4v a0 = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rr, c0 * 4, 0, kAuxSc1));
      f32x4v a1 = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rr, c0 * 4 + 16, 0, kAuxSc1));
      f32x4v s0[8], s1[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const uint32_t off = (uint32_t)(s * M * kH + c0) * 4;
        s0[s] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(sr, off, 0, kAuxSc1));
        s1[s] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(sr, off + 16, 0, kAuxSc1));
      }
      f32x4v d0 = s0[0], d1 = s1[0];
#pragma unroll
      for (int s = 1; s < 8; ++s) { d0 += s0[s]; d1 += s1[s]; }
      a0 += d0;
      a1 += d1;
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] = a0[j]; v[4 + j] = a1[j]; }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
    ss = wave_sum(ss);
    if (lane == 0) red[w] = ss;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < kCW; ++i) tot += red[i];
    const float inv = rsqrtf(tot / (float)kH + p.eps);
    if (live) {
      const bf16x8 wv = *reinterpret_cast<const bf16x8*>(wn + c0);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j] * inv * bf2f(wv[j]));
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const __amdgpu_buffer_rsrc_t yr = uniform_rsrc(y + (size_t)m * kH, kH * 2);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), yr, c0 * 2, 0, kAuxSc1);
      const __amdgpu_buffer_rsrc_t rr = uniform_rsrc(p.resid + (size_t)m * kH, kH * 4);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                                   __float_as_uint(v[3])}, rr, c0 * 4, 0, kAuxSc1);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]),
                                                   __float_as_uint(v[7])}, rr, c0 * 4 + 16, 0, kAuxSc1);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (sig_k >= 0 && w == 0 && lane == 0) signal_counter(p.sync, sig_k, m & 7);  // 64 arrivals over 8 shards
  };

  // ---- attention phase (optional): units (sequence, kv head) = (u >> 3, u & 7), u = 2b + (w >> 2), four key-split
  // waves (w & 3) each; attention.hip paged_attention_kernel<1, 4, 1, 4>'s folded-QKV decode path (GQA group 4,
  // one query per sequence, one partition), merged through the X ring region (free: O's X depends on this phase) ----
  auto attn_item = [&]() {
    float* mo = reinterpret_cast<float*>(smem);                    // [2 units][3 waves][32][64]
    float* mml = reinterpret_cast<float*>(smem + kLdsCtl + 64);    // [2 units][4 waves][16] x (m, l)
    const int j = w >> 2, kw = w & 3;
    const int u = 2 * b + j, sq = u >> 3, hh = u & 7;
    f32x4 o[8];
    float m_run = -1e30f, l_run = 0.f;
    bool col_valid = false;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int qlen = (!loader && sq < M) ? p.q_len[sq] : 0;
    if (qlen > 0) {
      const int ctx = p.ctx_len[sq];
      const int qi = r >> 2;  // column r: query r / 4 (only query 0 exists in decode), head 4 hh + r % 4
      col_valid = qi < qlen;
      const int col_limit = col_valid ? ctx - qlen + qi + 1 : 0;
      const int kend = ctx;
      const int* bt = p.block_tables + (size_t)sq * p.max_blocks;
      auto page_of = [&](int kb) {
        const int i = __builtin_amdgcn_readfirstlane(DSSE_IDX(kb / 32, p.max_blocks, 0));
        const __attribute__((address_space(4))) int* cbt = (const __attribute__((address_space(4))) int*)bt;
        return DSSE_IDX(cbt[i], p.num_blocks, 0);
      };
      // folded QKV epilogue: sum the slabs of this unit's 4 q heads, k and v; RoPE; regroup through LDS
      const size_t slab = (size_t)M * kQN;
      const int kn_page = (ctx - 1) & ~31;
      const int sl = p.slots[sq];
      const bool owner = sl >= 0 && ((kn_page / 32) & 3) == kw;
      const int t = lane >> 3, jj = lane & 7;
      const float* base = p.qkv_in + (size_t)sq * kQN + 16 * t + jj;
      auto unit_col = [&](int uu) { return uu < 4 ? (4 * hh + uu) * 128 : (uu == 4 ? (32 + hh) * 128 : (40 + hh) * 128); };
      float xa[6][2];
#pragma unroll
      for (int uu = 0; uu < 6; ++uu) xa[uu][0] = xa[uu][1] = 0.f;
      for (int s = 0; s < p.qkv_in_S; ++s) {
#pragma unroll
        for (int uu = 0; uu < 6; ++uu) {
          xa[uu][0] += base[s * slab + unit_col(uu)];
          xa[uu][1] += base[s * slab + unit_col(uu) + 8];
        }
      }
      const float2 cs = p.rope[(size_t)DSSE_IDX(p.positions[sq], p.rope_len, 0) * 64 + 8 * t + jj];
      bf16* fq = reinterpret_cast<bf16*>(smem + kLdsFq + w * 1536);
      const int d = 8 * t + jj;
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        fq[uu * 128 + d] = f2bf(xa[uu][0] * cs.x - xa[uu][1] * cs.y);
        fq[uu * 128 + 64 + d] = f2bf(xa[uu][1] * cs.x + xa[uu][0] * cs.y);
      }
      if (owner) {
        fq[4 * 128 + d] = f2bf(xa[4][0] * cs.x - xa[4][1] * cs.y);
        fq[4 * 128 + 64 + d] = f2bf(xa[4][1] * cs.x + xa[4][0] * cs.y);
        fq[5 * 128 + d] = f2bf(xa[5][0]);
        fq[5 * 128 + 64 + d] = f2bf(xa[5][1]);
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's own LDS rows
      __builtin_amdgcn_wave_barrier();
      bf16x8 qf[4];
#pragma unroll
      for (int s = 0; s < 4; ++s)
        qf[s] = col_valid ? *reinterpret_cast<const bf16x8*>(&fq[(r & 3) * 128 + 32 * s + 8 * g]) : zero_bf16x8();
      float sc_new = -INFINITY;
      int key_limit = col_limit;
      if (owner) {
        key_limit = col_limit - 1;  // the newest key is attended here, not in the page loop
        bf16x8 kn[4];
        float dot = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          kn[q] = *reinterpret_cast<const bf16x8*>(&fq[4 * 128 + 32 * q + 8 * g]);
#pragma unroll
          for (int e = 0; e < 8; ++e) dot += bf2f(qf[q][e]) * bf2f(kn[q][e]);
        }
        dot += __shfl_xor(dot, 16);
        dot += __shfl_xor(dot, 32);
        sc_new = col_valid ? dot * p.scale_log2 : -INFINITY;
        const int sidx = DSSE_IDX(sl, p.num_slots, 0), blk = sidx / 32, off = sidx % 32;
        if (r == (off & 15)) {
          bf16* kdst = p.k_cache + (((size_t)blk * 8 + hh) * 32 + off) * 128 + 8 * g;
#pragma unroll
          for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16x8*>(kdst + 32 * q) = kn[q];
        }
        bf16* vdst = p.v_cache + ((size_t)blk * 8 + hh) * 128 * 32 + vperm_tok(off);
        vdst[(size_t)d * 32] = f2bf(xa[5][0]);
        vdst[(size_t)(64 + d) * 32] = f2bf(xa[5][1]);
        if (col_valid) {  // the newest key opens the online softmax: m = its score, p = 1, o = its V row
          m_run = sc_new;
          l_run = g == 0 ? 1.f : 0.f;
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) {
            const bf16x4 vq = *reinterpret_cast<const bf16x4*>(&fq[5 * 128 + 16 * dt + 4 * g]);
#pragma unroll
            for (int i = 0; i < 4; ++i) o[dt][i] = bf2f(vq[i]);
          }
        }
      }
      auto compute_page = [&](int kb, const bf16x8 (&k0)[4], const bf16x8 (&k1)[4], const bf16x8 (&vf)[8]) {
        f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          s0 = mfma16x16x32(k0[s], qf[s], s0);
          s1 = mfma16x16x32(k1[s], qf[s], s1);
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ka = kb + 4 * g + i, kb2 = kb + 16 + 4 * g + i;
          s0[i] = (ka < key_limit) ? s0[i] * p.scale_log2 : -INFINITY;
          s1[i] = (kb2 < key_limit) ? s1[i] * p.scale_log2 : -INFINITY;
          tmax = fmaxf(tmax, fmaxf(s0[i], s1[i]));
        }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
        const float m_new = fmaxf(m_run, tmax);
        const float alpha = exp2f(m_run - m_new);
        m_run = m_new;
        bf16x8 pf;
        float psum = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e0 = exp2f(s0[i] - m_new), e1 = exp2f(s1[i] - m_new);
          psum += e0 + e1;
          pf[i] = f2bf(e0);
          pf[4 + i] = f2bf(e1);
        }
        l_run = l_run * alpha + psum;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) o[dt] = mfma16x16x32(vf[dt], pf, o[dt] * alpha);
      };
      int kb = 32 * kw;
      int page = kb < kend ? page_of(kb) : 0;
      for (; kb < kend; kb += 128) {
        const bf16* kp = p.k_cache + ((size_t)page * 8 + hh) * 32 * 128;
        const bf16* vp = p.v_cache + ((size_t)page * 8 + hh) * 128 * 32;
        bf16x8 k0[4], k1[4], vf[8];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          k0[s] = ld_nt_bf16x8(kp + (size_t)r * 128 + 32 * s + 8 * g);
          k1[s] = ld_nt_bf16x8(kp + (size_t)(16 + r) * 128 + 32 * s + 8 * g);
        }
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) vf[dt] = ld_nt_bf16x8(vp + (size_t)(16 * dt + r) * 32 + 8 * g);
        page = page_of(min(kb + 128, kend - 1));
        compute_page(kb, k0, k1, vf);
      }
      l_run += __shfl_xor(l_run, 16);
      l_run += __shfl_xor(l_run, 32);
      if (kw != 0) {
        float* mw = mo + ((size_t)(j * 3 + kw - 1) * 32) * 64;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) mw[(dt * 4 + i) * 64 + lane] = o[dt][i];
      }
      if (g == 0) {
        mml[((j * 4 + kw) * 16 + r) * 2] = m_run;
        mml[((j * 4 + kw) * 16 + r) * 2 + 1] = l_run;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // partials of every key-split wave in LDS
    if (qlen > 0 && kw == 0 && col_valid) {
      float mm = m_run;
#pragma unroll
      for (int v = 1; v < 4; ++v) mm = fmaxf(mm, mml[((j * 4 + v) * 16 + r) * 2]);
      float scv[4], ll = 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float mv = v == 0 ? m_run : mml[((j * 4 + v) * 16 + r) * 2];
        const float lv = v == 0 ? l_run : mml[((j * 4 + v) * 16 + r) * 2 + 1];
        scv[v] = exp2f(mv - mm);
        ll += lv * scv[v];
      }
      const float inv = ll > 0.f ? 1.f / ll : 0.f;
      const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(p.attn + (size_t)sq * kH, kH * 2);
      const int col0 = (4 * hh + (r & 3)) * 128;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float a = o[dt][i] * scv[0];
#pragma unroll
          for (int v = 1; v < 4; ++v) a += mo[((size_t)(j * 3 + v - 1) * 32 + dt * 4 + i) * 64 + lane] * scv[v];
          __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, f2bf(a * inv)), rs,
                                                (uint32_t)((col0 + 16 * dt + 4 * g + i) * 2), 0, kAuxSc1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");  // attn rows stored (write-through)
    if (w == 0 && lane == 0) signal_counter(p.sync, kCntA, b & 7);
  };

  // ---- this workgroup's schedule ----
  const bool fused_attn = p.qkv_in != nullptr;
  // stamp slots: 0 start, 1 attention done, 2/3 O dependency met / done, 4/5 N1, 6/7 gate_up, 8/9 down, 10/11 N2,
  // 12/13 next QKV, 14 end, 15 gate_up dependency seen before its acquire fence
  if (fused_attn) attn_item();
  stamp(1);
  gemm_item(0, kOSteps, 0, 8, fused_attn ? kCntA : -1, 8, base_a, 256u, kCntO, ks, 2);
  if (b < kRows) norm_item(b, p.w_ffn, p.xm, kCntO, 8, base_o, kCntN1, 4);
  gemm_item(kGU0, kGUSteps, 1, 7, kCntN1, 8, base_n1, 64u, kCntGU + (b >> 5), 0, 6);
  gemm_item(kD0, kDSteps, 0, 8, kCntGU + ks, 1, base_gu, 32u, kCntD, ks, 8);
  if (b >= kRows && b < 2 * kRows) norm_item(b - kRows, p.w_next, p.x, kCntD, 8, base_d, kCntN2, 10);
  if (p.wqkv != nullptr) gemm_item(kQ0, kQSteps, 2, kQTiles, kCntN2, 8, base_n2, 64u, -1, 0, 12);
  // the look-ahead weight loads past the last step are range-failed dummies, but they still write the LDS: drain
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stamp(14);
}

}  // namespace dsse

using namespace dsse;

extern "C" size_t dsse_mega_sync_words() { return (size_t)mega::kSyncCounters * 8 * 32; }

// Shapes are the Mistral-7B ones (H 4096, F 14336) and M <= 64; the caller (bindings.cpp) validates them.
extern "C" hipError_t dsse_mega_mlp(const MegaMlpParams* p, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mega_mlp_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, mega::kLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  if (p->M < 1 || p->M > mega::kRows) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mega_mlp_kernel, dim3(mega::kWGs), dim3(mega::kThreads), mega::kLds, st, *p);
  return hipGetLastError();
}
