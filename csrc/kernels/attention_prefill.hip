// Flash prefill attention on MFMA for gfx950 (K12 of SURVEY.md §2.4): causal, GQA, paged KV,
// chunked prefill (queries = the last q_len positions of a ctx_len context).
//
// Measured need (profiles/ttft_r1.md): the decode-derived kernel in attention.hip (no LDS, K/V read
// straight from the paged cache by every wave) ran an 8k-token causal prefill at ~157 TFLOP/s,
// 56 % of the TTFT.  This kernel is the classic LDS-staged flash structure, laid out for CDNA4:
//
//   workgroup  = one KV head x 64 query tokens; 2G waves (G = Hq/Hkv q heads x 2 halves of 32
//                queries), so every K/V byte staged in LDS feeds 2G waves (GQA reuse in LDS);
//   key loop   = 64 keys (two 32-token pages) per block, a 4-block LDS ring (4 x 32 KiB) filled by LDS-DMA
//                three blocks ahead;
//   scores     = Sᵀ = K·Qᵀ (keys on MFMA rows, queries on lanes): a query's softmax statistics live
//                in one lane column, and the exponentiated scores are already the B operand of
//                Oᵀ = Vᵀ·Pᵀ — the V cache stores each page transposed with the token permutation
//                vperm(), so lane group g's 8 keys {4g..4g+3, 16+4g..16+4g+3} are one 16-byte run;
//   LDS images = K [64 keys][256 B] with the XOR-swizzled 16-byte chunks of gemm_xlds, Vᵀ [128 d]
//                [128 B] with chunk ^= (d >> 1) & 7: both read with conflict-free ds_read_b128;
//   softmax    = online, base 2, masked scores contribute exactly 0 (fully masked columns stay 0).
//
// Schedule (round 4): two phases per key block, QKᵀ(j) | softmax(j) + PV(j), one barrier before each, and the
// two query halves staggered by one barrier.  Waves w and w + 4 share a SIMD (G = 4: the same head, the two
// query halves), so while one runs the 32 MFMAs of its QKᵀ the other runs its softmax VALU work and then its PV
// MFMAs: the SIMD sees MFMA work from one wave under the other's exp / max / convert chain.  The round-1..3 form
// (all waves in lockstep, one barrier per two blocks) measured MFMA busy 22 %, 34 % of wave time waiting on
// dependencies (profiles/pmc_flash_prefill_r1.md): both waves of a SIMD reached their softmax at the same time.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "api.h"

namespace dsse {

namespace {
DEV void glds16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds(const_cast<void*>(src),
                                   reinterpret_cast<__attribute__((address_space(3))) void*>(
                                       reinterpret_cast<uintptr_t>(lds_base)),
                                   16, 0, 0);
}
constexpr int kD = 128;
constexpr int kBQ = 64;    // query tokens per workgroup
constexpr int kBK = 64;    // keys per block (2 pages)
constexpr int kKBytes = kBK * kD * 2;  // 16 KiB
constexpr int kStage = 2 * kKBytes;    // K + Vᵀ of one block
constexpr int kRing = 4;               // LDS blocks
constexpr float kRescaleThr = 8.f;     // deferred online-softmax rescale threshold (log2 units)

// KV block of page `pg` (clamped to the last page: pages past the context are a harmless, masked re-read).
// The index is workgroup-uniform, so this is a scalar load: waiting for it (lgkmcnt) does not drain the
// vector loads of the K/V blocks already in flight, as a per-lane block-table load's vmcnt(0) did.
// (The block table is read-only for the kernel's lifetime, so reading it through the constant address space
// is safe and lets the compiler issue s_load_dword.)
DEV int page_block(const int* bt, int pg, int npages, const AttnParams& p) {
  pg = __builtin_amdgcn_readfirstlane(min(pg, npages - 1));
  const __attribute__((address_space(4))) int* cbt = (const __attribute__((address_space(4))) int*)bt;
  return DSSE_IDX(cbt[DSSE_IDX(pg, p.max_blocks, 0)], p.num_blocks, 0);
}
}  // namespace

// G = q heads per kv head; HG = the q heads one workgroup takes (HG < G splits a kv head's q heads over G / HG
// workgroups: short prompts, where one workgroup per (tile, kv head) leaves most CUs idle -- a 512-token prompt is 64
// workgroups; each then stages its K/V itself, which the L2 serves)
// STAMP (diagnostic build, DSSE_FLASH_STAMPS): every wave of the first kStampWgs workgroups records the shader clock at
// six points of each key block (before / after the barrier in front of QKᵀ, before / after the barrier in front of
// softmax + PV, after the DMA issue, after the softmax) into 24 KiB of LDS past the ring, copied to `stamps` at the end; tools/flash_stamps.py reads them.
constexpr int kStampBlocks = 128, kStampWgs = 32, kStampsPerBlock = 6;
template <int G, int HG, bool STAMP>
__global__ void __launch_bounds__(128 * HG) flash_prefill_kernel(AttnParams p, unsigned* stamps) {
  constexpr int NW = 2 * HG;
  constexpr int NSPLIT = G / HG;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // kRing blocks of kStage

  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const int r = lane & 15, g = lane >> 4;
  const int wh = w % HG, wq = w / HG;
  // flat grid, head fastest: workgroup b runs on XCD b % 8, so with Hkv = 8 every XCD serves ONE kv head and
  // its 4 MiB of 8k-context K/V stays in that XCD's L2 for all the head's query tiles (a (tile, head) grid put
  // consecutive tiles on different XCDs and every XCD streamed all 8 heads); the work list is heaviest-first
  // globally, not per head
  const int h = blockIdx.x % p.hkv, rest = blockIdx.x / p.hkv;
  const int hs = rest % NSPLIT, item = rest / NSPLIT;
  const int b = p.work_seq[item];
  const int qlen = p.q_len[b], ctx = p.ctx_len[b];
  const int pos0 = ctx - qlen;                 // absolute position of query 0 of this chunk
  const int tile = p.work_tile[item];
  const int q0 = tile * kBQ + wq * 32;         // this wave's first query (within the chunk)
  const int wg_last_q = min(qlen, (tile + 1) * kBQ) - 1;
  if (tile * kBQ >= qlen) return;              // uniform
  const int kmax = pos0 + wg_last_q + 1;       // keys [0, kmax) are visible to some query of the WG
  const int nblk = (kmax + kBK - 1) / kBK;
  // key split (round 6): this item's key blocks [jb, je) and its partial slot (-1: the whole range, final output)
  const int jb = p.work_kb ? p.work_kb[2 * item] : 0;
  const int je = p.work_kb ? min(nblk, p.work_kb[2 * item + 1]) : nblk;
  const int pslot = p.work_slot ? p.work_slot[item] : -1;
  const int w_last_pos = pos0 + min(qlen, q0 + 32) - 1;  // last visible key of this wave
  const int w_first_pos = pos0 + q0;
  const int head = h * G + hs * HG + wh;
  const int* bt = p.block_tables + (size_t)b * p.max_blocks;
  const int npages = (kmax + kBS - 1) / kBS;

  // Q fragments (B operand of Sᵀ = K·Qᵀ): lane (r, g) holds Q[query 16qt + r][d = 32g + 8s + j]
  bf16x8 qf[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = min(q0 + 16 * qt + r, qlen - 1);
    const bf16* qp = p.q + ((size_t)(p.q_start[b] + qi) * p.hq + head) * kD + 32 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[qt][s] = ld_bf16x8(qp + 8 * s);
  }
  // retire the Q loads here, before any DMA is issued: otherwise the compiler's wait for them at the first QKᵀ
  // MFMA (behind an unknown number of loop-carried DMAs) is a vmcnt(0) inside the loop, draining the prefetch
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int s = 0; s < 4; ++s) asm volatile("" ::"v"(qf[qt][s]));

  // LDS-DMA: a block is 32 x 1 KiB DMA instructions, IPW per wave.  Instruction q < 16 fills keys 4q..4q+3
  // (lane -> key 4q + lane / 16, LDS slot lane % 16 = chunk ^ swz(key)); q >= 16 fills Vᵀ rows d = 8 (q - 16)
  // + lane / 8 (slot lane % 8 = chunk ^ ((d >> 1) & 7), chunk = page * 4 + 8-token group).  The swizzles sit
  // on the source address because the DMA writes LDS lane-linearly; the reads are unchanged.  Blocks past the
  // last are issued too (pages clamp to the context, nobody reads them): a branch around the DMA made the
  // compiler's waitcnt placement drain every load in flight.
  constexpr int IPW = 32 / NW;
  // Lane-constant parts of the DMA sources (element offsets inside a page block of this kv head) and, for the Vᵀ
  // pieces, which of the block's two pages the lane's chunk comes from: per block only the two page bases change
  // (scalar), so a piece costs a select and one 64-bit add instead of a per-lane 64-bit multiply-add.
  uint32_t loff[IPW];
  bool vhi[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int q = w * IPW + i;  // wave-uniform
    if (q < 16) {
      const int key = 4 * q + (lane >> 4), c = (lane & 15) ^ swz(key & 15);
      loff[i] = (key & 31) * kD + 8 * c;
      vhi[i] = false;
    } else {
      const int d = 8 * (q - 16) + (lane >> 3), c = (lane & 7) ^ ((d >> 1) & 7);
      loff[i] = d * kBS + 8 * (c & 3);
      vhi[i] = c >= 4;
    }
  }
  const size_t pstride = (size_t)p.hkv * kBS * kD;  // elements per page block (all kv heads)
  const bf16* kh = p.k_cache + (size_t)h * kBS * kD;
  const bf16* vh = p.v_cache + (size_t)h * kD * kBS;
  // Page-table entries are read one block ahead: the scalar load of block j + 1's pages is in flight while block j
  // is issued and retired by the next LDS wait, not by a dependent wait in front of this block's DMA.
  int pg0 = page_block(bt, 2 * jb, npages, p), pg1 = page_block(bt, 2 * jb + 1, npages, p);
  int jn = jb;  // next block to issue (blocks are issued in order)
  // (the page bases are pinned in SGPR pairs: left to itself the compiler folds the per-lane select of two bases into
  // a per-lane select of the page index followed by a per-lane 64-bit multiply)
  auto sbase = [&](const bf16* head, int blk) {
    uint64_t u = reinterpret_cast<uint64_t>(head + (size_t)blk * pstride);
    asm volatile("" : "+s"(u));
    return u;
  };
  auto issue_block = [&](int slot) {
    const int blk0 = pg0, blk1 = pg1;
    ++jn;
    pg0 = page_block(bt, 2 * jn, npages, p);
    pg1 = page_block(bt, 2 * jn + 1, npages, p);
    char* base = smem + slot * kStage;
    const bool kpiece = w * IPW < 16;  // wave-uniform: a wave's pieces are all K or all Vᵀ (IPW divides 16)
    const uint64_t b0 = sbase(kpiece ? kh : vh, blk0), b1 = sbase(kpiece ? kh : vh, blk1);
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int q = w * IPW + i;  // wave-uniform
      const uint64_t b = kpiece ? (q >= 8 ? b1 : b0) : (vhi[i] ? b1 : b0);
      glds16(reinterpret_cast<const bf16*>(b + 2ull * loff[i]), base + q * 1024);
    }
  };

  f32x4 o[8][2];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) o[dt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-1e30f, -1e30f};
  // per-lane partial row sums (packed pairs): reduced over the 4 lane groups of a query once, after the last block
  f32x2 l_part[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};
  const float sc = p.scale_log2;
  f32x4 s4[4][2];  // Sᵀ[key tile kt][query tile qt] of the current block, live across the mid-block barrier

  // Lane-constant parts of the fragment addresses: K row 16 kt + r, chunk (4g + s) ^ swz(r) = kt * 4096 + kofs[s];
  // Vᵀ row d = 16 dt + r, chunk (4t + g) ^ ((d >> 1) & 7) = (4t + g) ^ ((r >> 1) & 7) = dt * 2048 + vofs[t].  With the
  // slot a compile-time constant (the block loop is unrolled by the ring) every read is one base VGPR + an immediate.
  int kofs[4], vofs[2];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) kofs[s2] = r * 256 + (((4 * g + s2) ^ swz(r)) << 4);
#pragma unroll
  for (int t = 0; t < 2; ++t) vofs[t] = kKBytes + r * 128 + (((4 * t + g) ^ ((r >> 1) & 7)) << 4);

  unsigned* st_lds = reinterpret_cast<unsigned*>(smem + kRing * kStage) + w * kStampsPerBlock * kStampBlocks;
  auto stamp = [&](int j, int i) {
    if constexpr (STAMP) {
      if (lane == 0 && j < kStampBlocks) st_lds[kStampsPerBlock * j + i] = (unsigned)__builtin_amdgcn_s_memtime();
    }
  };
  // phase 1: Sᵀ = K·Qᵀ of the block in LDS slot `buf`; a key tile's 4 fragments are read one tile ahead
  auto qk = [&](int buf) {
    const char* kb = smem + buf * kStage;
    bf16x8 kf[2][4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) kf[0][s2] = *reinterpret_cast<const bf16x8*>(kb + kofs[s2]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      if (kt < 3) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
          kf[(kt + 1) & 1][s2] = *reinterpret_cast<const bf16x8*>(kb + (kt + 1) * 4096 + kofs[s2]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s4[kt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) s4[kt][qt] = mfma16x16x32(kf[kt & 1][s2], qf[qt][s2], s4[kt][qt]);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // phase 2: online softmax of block j and Oᵀ += Vᵀ·Pᵀ
  auto sm_pv = [&](int j, int buf) {
    const int key0 = j * kBK;
    const bool need_mask = key0 + kBK - 1 > w_first_pos;  // some key of the block is after some query
    bf16x8 pf[2][2];  // [qt][page t]
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qpos = pos0 + q0 + 16 * qt + r;
      const bool qvalid = q0 + 16 * qt + r < qlen;
      // max over the RAW scores (scale_log2 > 0 commutes with max); masked scores become -1e30
      float mx = -1e30f;
      if (need_mask) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = key0 + 16 * kt + 4 * g + i;
            const float v = (qvalid && key <= qpos) ? s4[kt][qt][i] : -1e30f;
            s4[kt][qt][i] = v;
            mx = fmaxf(mx, v);
          }
      } else {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) mx = fmaxf(mx, s4[kt][qt][i]);
      }
      mx = rows4_max(mx);
      // Deferred rescale: the running max (log2 units) only moves when a query's block max exceeds it by
      // more than kRescaleThr, so after the first blocks O and l are not rescaled at all (P <= 2^thr stays
      // well inside bf16 / fp32 range; the final O / l is unchanged).  Decided per wave (any lane).
      const float m_blk = mx * sc;
      if (__any(m_blk > m_run[qt] + kRescaleThr)) {
        const float m_new = fmaxf(m_run[qt], m_blk);
        // a column with no visible key yet keeps m = -1e30 and must produce p = 0, not exp2(0)
        const float alpha = __builtin_amdgcn_exp2f(m_run[qt] - (m_new < -1e29f ? 0.f : m_new));
        l_part[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
          o[dt][qt][0] *= alpha;
          o[dt][qt][1] *= alpha;
          o[dt][qt][2] *= alpha;
          o[dt][qt][3] *= alpha;
        }
        m_run[qt] = m_new;
      }
      const float m_use = m_run[qt] < -1e29f ? 0.f : m_run[qt];
      // raw v_exp_f32 (no denormal range reduction: arguments are <= thr and underflow to 0 is wanted); the scale
      // is folded into one packed FMA per score pair and the row sum is a packed add (VALU is this loop's bound:
      // profiles/r4/pmc_flash_prefill_r4.md)
      const f32x2 scv = {sc, sc}, mv = {-m_use, -m_use};
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          f32x2 v = {s4[kt][qt][i], s4[kt][qt][i + 1]};
          v = __builtin_elementwise_fma(v, scv, mv);
          v[0] = __builtin_amdgcn_exp2f(v[0]);
          v[1] = __builtin_amdgcn_exp2f(v[1]);
          s4[kt][qt][i] = v[0];
          s4[kt][qt][i + 1] = v[1];
          l_part[qt] += v;
        }
      // Pᵀ fragments: page t = key tiles 2t (keys 4g+i) and 2t+1 (keys 16+4g+i)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pf[qt][t][i] = f2bf(s4[2 * t][qt][i]);
          pf[qt][t][4 + i] = f2bf(s4[2 * t + 1][qt][i]);
        }
    }
    stamp(j, 5);
    // Oᵀ[d tile][query tile] += Vᵀ · Pᵀ: the 8 fragments of a page read before its 16 MFMAs
    const char* vb0 = smem + buf * kStage;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16x8 vf[8];
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) vf[dt] = *reinterpret_cast<const bf16x8*>(vb0 + dt * 2048 + vofs[t]);
      // keep the 8 reads ahead of the MFMAs (the scheduler otherwise pairs 2 reads with a full lgkmcnt wait)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) o[dt][qt] = mfma16x16x32(vf[dt], pf[qt][t], o[dt][qt]);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // Barrier accounting (absolute barriers, counted from the loop entry of the leading half; the lagging half,
  // wq = 1, passes one extra barrier first and one fewer at the end).  Leading half: QKᵀ(j) in interval 2j,
  // softmax/PV(j) in 2j + 1; lagging half one interval later.  So block j is read in intervals 2j .. 2j + 2:
  //   RAW  every wave's DMA of block j has retired (its own counted vmcnt) before barrier 2j;
  //   WAR  block j + 4 reuses j's slot; its DMA is issued at the start of softmax/PV(j + 1), i.e. in interval
  //        2j + 3 (leading) or 2j + 4 (lagging), after every read of block j (the last in interval 2j + 2).
  // Each wave issues block j + 3 at the start of its softmax/PV(j) phase, so at the barrier before QKᵀ(j) the
  // leading half has blocks up to j + 2 issued (wait: all but the 2 youngest blocks), and at the barrier before
  // softmax/PV(j), which for the lagging half is absolute barrier 2(j + 1), the lagging half needs block j + 1
  // with blocks up to j + 2 issued (wait: all but the youngest).
  const bool lag = wq == 1;
  issue_block(0);
  issue_block(1);
  issue_block(2);
  if (lag) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * IPW) : "memory");
  // unrolled by the ring size: each block's LDS slot is a compile-time offset (no per-read address arithmetic)
  for (int j0 = jb; j0 < je; j0 += kRing) {
#pragma unroll
    for (int k = 0; k < kRing; ++k) {
      const int j = j0 + k;  // LDS slot k = (j - jb) % kRing: block jb went to slot 0
      if (j < je) {
        const bool vis = j * kBK <= w_last_pos;  // this wave sees at least one key of the block
        stamp(j, 0);
        if (!lag) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * IPW) : "memory");
        else asm volatile("s_barrier" ::: "memory");
        stamp(j, 1);
        if (vis) qk(k);
        stamp(j, 2);
        if (!lag) asm volatile("s_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(IPW) : "memory");
        stamp(j, 3);
        issue_block((k + 3) % kRing);  // block j + 3
        stamp(j, 4);
        if (vis) sm_pv(j, k);
      }
    }
  }
  if (!lag) asm volatile("s_barrier" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may still write this workgroup's LDS after it exits
  if constexpr (STAMP) {
    if (blockIdx.x < kStampWgs) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's stamp writes have landed
      unsigned* dst = stamps + ((size_t)blockIdx.x * NW + w) * kStampsPerBlock * kStampBlocks;
      for (int i = lane; i < kStampsPerBlock * kStampBlocks; i += 64) dst[i] = i < kStampsPerBlock * nblk ? st_lds[i] : 0u;
    }
  }

  // ---- epilogue: lane (r, g) holds O[query 16qt + r][d = 16dt + 4g + i]
  if (pslot >= 0) {  // one key range of a split tile: unnormalised O and (max, sum) for flash_combine_kernel
    const size_t sb = ((size_t)(pslot * p.hkv + h) * G + hs * HG + wh) * kBQ;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int qrow = wq * 32 + 16 * qt + r;
      if (q0 + 16 * qt + r >= qlen) continue;
      const float l = rows4_sum(l_part[qt][0] + l_part[qt][1]);
      float* po = p.part_o + (sb + qrow) * kD + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) *reinterpret_cast<f32x4*>(po + 16 * dt) = o[dt][qt];
      if (g == 0) p.part_ml[sb + qrow] = make_float2(m_run[qt] < -1e29f ? 0.f : m_run[qt], l);
    }
    return;
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qi = q0 + 16 * qt + r;
    if (qi >= qlen) continue;
    const float l = rows4_sum(l_part[qt][0] + l_part[qt][1]);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16* op = p.out + ((size_t)(p.q_start[b] + qi) * p.hq + head) * kD + 4 * g;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      bf16x4 v;
      v[0] = f2bf(o[dt][qt][0] * inv);
      v[1] = f2bf(o[dt][qt][1] * inv);
      v[2] = f2bf(o[dt][qt][2] * inv);
      v[3] = f2bf(o[dt][qt][3] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * dt) = v;
    }
  }
}

// Merge the key ranges of split tiles (flash prefill key split): grid (ncomb, Hkv, G), 256 threads = 64 query rows x 4
// quarters of the head dimension; each thread reads its 32 dims of every slot once (the slots' O is relative to their
// own running max m, in log2 units: weight 2^(m - M)).
__global__ void __launch_bounds__(256) flash_combine_kernel(AttnParams p) {
  const int c = blockIdx.x, h = blockIdx.y, hl = blockIdx.z, G = p.group;
  const int qrow = threadIdx.x >> 2, dq = threadIdx.x & 3;
  const int b = p.comb[4 * c], tile = p.comb[4 * c + 1], s0 = p.comb[4 * c + 2], ns = p.comb[4 * c + 3];
  const int qi = tile * kBQ + qrow;
  if (qi >= p.q_len[b]) return;
  float mm = -1e30f;
  for (int k = 0; k < ns; ++k) mm = fmaxf(mm, p.part_ml[((size_t)((s0 + k) * p.hkv + h) * G + hl) * kBQ + qrow].x);
  f32x4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ll = 0.f;
  for (int k = 0; k < ns; ++k) {
    const size_t row = ((size_t)((s0 + k) * p.hkv + h) * G + hl) * kBQ + qrow;
    const float2 ml = p.part_ml[row];
    const float wgt = __builtin_amdgcn_exp2f(ml.x - mm);
    ll += ml.y * wgt;
    const f32x4* po = reinterpret_cast<const f32x4*>(p.part_o + row * kD + 32 * dq);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += po[j] * wgt;
  }
  const float inv = ll > 0.f ? 1.f / ll : 0.f;
  bf16* op = p.out + ((size_t)(p.q_start[b] + qi) * p.hq + h * G + hl) * kD + 32 * dq;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = f2bf(acc[j][i] * inv);
      v[4 + i] = f2bf(acc[j + 1][i] * inv);
    }
    *reinterpret_cast<bf16x8*>(op + 4 * j) = v;
  }
}

}  // namespace dsse

namespace {
template <int G, int HG, bool STAMP>
hipError_t launch_flash(int num_work, const dsse::AttnParams* p, hipStream_t st, unsigned* stamps) {
  using namespace dsse;
  constexpr int lds = kRing * kStage + (STAMP ? 2 * HG * kStampsPerBlock * kStampBlocks * 4 : 0);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&flash_prefill_kernel<G, HG, STAMP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((flash_prefill_kernel<G, HG, STAMP>), dim3(num_work * p->hkv * (G / HG)), dim3(128 * HG), lds, st,
                     *p, stamps);
  return hipGetLastError();
}

// DSSE_FLASH_STAMPS=<file>: the diagnostic build of the kernel; after each call the stamps of the first kStampWgs
// workgroups ([wg][wave][block][6] u32 shader-clock values) overwrite <file> (synchronises the device: never set it in
// serving)
hipError_t launch_stamped(int num_work, const dsse::AttnParams* p, hipStream_t st, const char* path) {
  using namespace dsse;
  if (p->group != 4) return hipErrorInvalidValue;
  const size_t n = (size_t)kStampWgs * 8 * kStampsPerBlock * kStampBlocks;
  static unsigned* buf = nullptr;
  if (buf == nullptr && hipMalloc(&buf, n * sizeof(unsigned)) != hipSuccess) return hipErrorOutOfMemory;
  (void)hipMemsetAsync(buf, 0, n * sizeof(unsigned), st);
  hipError_t e = launch_flash<4, 4, true>(num_work, p, st, buf);
  if (e != hipSuccess) return e;
  std::vector<unsigned> host(n);
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
  if ((e = hipMemcpy(host.data(), buf, n * sizeof(unsigned), hipMemcpyDeviceToHost)) != hipSuccess) return e;
  if (FILE* f = fopen(path, "wb")) {
    fwrite(host.data(), sizeof(unsigned), n, f);
    fclose(f);
  }
  return hipSuccess;
}
}  // namespace

// Work items: (sequence, 64-query tile) pairs; grid = num_work x Hkv workgroups, kv head fastest.  Requires
// G = Hq/Hkv in {1, 2, 4}.  (Splitting a kv head's q heads over G workgroups for short prompts -- 256 workgroups of
// 2 waves instead of 64 of 8 at 512 tokens -- measured 38.9 vs 28.8 us and was dropped; profiles/r4.)
// p->kwv (mode 2): q heads per workgroup (flash_hg in DSSE_KERNEL_CFG), 0 = the whole group.  Round 6 re-measured the
// split for a long prompt on ONE kv head (a TP = 8 rank: 4 q heads, 128 workgroups of 8 waves at 8k tokens, half the
// CUs idle): 2 q heads per workgroup 323 us, 1 q head 383 us, the whole group 264 us at T = 8192 (85 / 94 / 72 us
// at 2048; profiles/r6/flash_tp8_r6.log) -- every split stages the same K / V once more per workgroup, and the LDS
// fill, not the idle CUs, sets the time.
extern "C" hipError_t dsse_flash_prefill(int num_work, const dsse::AttnParams* p, hipStream_t st) {
  if (num_work <= 0) return hipSuccess;
  static const char* stamps = getenv("DSSE_FLASH_STAMPS");
  if (stamps != nullptr && stamps[0] != '\0') return launch_stamped(num_work, p, st, stamps);
  int hg = p->kwv;
  if (hg == 0 || p->work_kb) hg = p->group;  // the key split writes partial slots per whole group
  hipError_t e;
  switch (p->group) {
    case 1: e = launch_flash<1, 1, false>(num_work, p, st, nullptr); break;
    case 2: e = hg == 1 ? launch_flash<2, 1, false>(num_work, p, st, nullptr)
                        : launch_flash<2, 2, false>(num_work, p, st, nullptr); break;
    case 4: e = hg == 1 ? launch_flash<4, 1, false>(num_work, p, st, nullptr)
                        : hg == 2 ? launch_flash<4, 2, false>(num_work, p, st, nullptr)
                                  : launch_flash<4, 4, false>(num_work, p, st, nullptr); break;
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess || !p->work_kb || p->ncomb <= 0) return e;
  hipLaunchKernelGGL(dsse::flash_combine_kernel, dim3(p->ncomb, p->hkv, p->group), dim3(256), 0, st, *p);
  return hipGetLastError();
}

DSSE_CHECK_READER(dsse_check_attention_prefill)
