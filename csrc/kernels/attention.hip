// Paged GQA attention on MFMA for gfx950 (K5 decode and K12 prefill of SURVEY.md §2.4).
//
// KV cache layout (engine-owned, page = 32 tokens):
//   K: [blocks, Hkv, 32, 128]   one key row = 256 contiguous bytes
//   V: [blocks, Hkv, 128, 32]   transposed, tokens permuted inside the page by vperm() so the
//                               PV operand of lane group g is one 16-byte run
//
// One MFMA tile column is a (query token, q-head of the GQA group) pair: with G = Hq/Hkv heads
// per kv head, a 16-column tile holds QT = 16/G query tokens of one sequence.  Decode uses
// QT = 1 token (G columns live), prefill uses all 16 columns.  Scores are computed swapped,
// Sᵀ[key, col] = K · Qᵀ, so the softmax statistics of a column live in one lane column and
// the exponentiated scores are already the B operand of Oᵀ = Vᵀ · Pᵀ — no LDS round trip and
// no transposes inside the key loop.
//
// Work decomposition: a workgroup = QW × KWV waves.  The QW waves take consecutive query tiles
// (prefill: they share K/V lines through L1), the KWV waves split the key range and are merged
// in LDS; grid.z splits the key range into partitions of `part` keys (flash-decoding), merged
// by attn_combine_kernel.  Online softmax in base 2 with a finite initial max, so fully masked
// columns stay finite and produce zeros.
#include <cstdlib>

#include "api.h"
#include "gemm_epilogue.h"

#ifndef ATTN_DECODE_NT
#define ATTN_DECODE_NT 1
#endif

namespace dsse {

constexpr int kPage = 32;
constexpr int kD = 128;


// One-wave decode workgroups (256+ streams) are held to 4 waves per SIMD: the folded QKV epilogue (FQ) otherwise
// raises the register peak from 127 to 159 and costs a wave per SIMD; 104 VGPRs, no spills.
// PD: KV pages in flight per wave (a register ring of PD pages, each wave's next PD-1 pages issued before the
// current one is computed).  One-wave workgroups with PD > 1 are held to 2 waves per SIMD (256 VGPRs): the
// 2048-workgroup grid they serve (256 streams x 8 kv heads) puts 2 waves on each SIMD anyway.
// Keys per flash-decoding partition: p.part, or (p.part == 0, round 6) this work item's own key range split evenly
// over the nparts partitions in whole pages -- a graph captured for max_model_len then keeps every partition busy at
// the contexts actually served (one KV head per rank at TP = 8: 64 streams = 64 (sequence, head) pairs, all of whose
// work sat in the first partition of a max_model_len / nparts split).
DEV int part_keys(const AttnParams& p, int kmax) {
  if (p.part > 0) return p.part;
  const int per = (kmax + p.nparts - 1) / p.nparts;
  return max(kPage, (per + kPage - 1) / kPage * kPage);
}

template <int QW, int KWV, int PD = 1, int FQG = 0>
__global__ void __launch_bounds__(64 * QW * KWV, QW * KWV == 1 ? (PD > 1 ? 2 : 4) : 1)
paged_attention_kernel(AttnParams p) {
  constexpr bool FQ = FQG > 0;  // QKV epilogue folded in, GQA group FQG (= p.group)
  static_assert(PD == 1 || PD == 2, "1 or 2 pages in flight");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int qw = w / KWV, kw = w % KWV;
  const int item = blockIdx.x, h = blockIdx.y, pz = blockIdx.z;
  const int b = p.work_seq[item];
  const int qlen = p.q_len[b];
  const int ctx = p.ctx_len[b];
  const int G = p.group, QT = 16 / G;
  const int tile = p.work_tile[item] * QW + qw;  // this wave's query tile
  const int q0 = tile * QT;                       // first query index (within the sequence)

  // Column r of this wave: query qi = q0 + r / G, head h*G + r % G.
  const int qi = q0 + r / G;
  const bool col_valid = qi < qlen;
  const int qpos = ctx - qlen + qi;          // absolute position; keys [0, qpos] visible
  const int col_limit = col_valid ? qpos + 1 : 0;

  // Key range needed by the whole workgroup (all QW tiles): up to the last live query.
  const int last_q = min(qlen, (p.work_tile[item] + 1) * QW * QT) - 1;
  const int kmax = (qlen > 0 && last_q >= 0) ? (ctx - qlen + last_q + 1) : 0;
  const int part = part_keys(p, kmax);
  const int kbeg = pz * part;
  const int kend = min(kmax, kbeg + part);
  if (kbeg >= kend) return;  // uniform for the whole workgroup

  const int* bt = p.block_tables + (size_t)b * p.max_blocks;
  // One page (32 keys) per wave step.
  // KV page of key kb: a wave-uniform index, read through the constant address space (the block table is
  // read-only for the kernel) so it is an s_load_dword -- a per-lane block-table load made every page wait
  // vmcnt(0) behind it, draining the K/V loads in flight.
  auto page_of = [&](int kb) {
    const int i = __builtin_amdgcn_readfirstlane(DSSE_IDX(kb / kPage, p.max_blocks, 0));
    const __attribute__((address_space(4))) int* cbt = (const __attribute__((address_space(4))) int*)bt;
    return DSSE_IDX(cbt[i], p.num_blocks, 0);
  };
  // decode (QW = 1): every K/V byte is read once, by one wave -> non-temporal loads (ATTN_DECODE_NT, default on:
  // tools/kvbench.hip measured this access pattern at 6.3 TB/s nt vs 3.6 TB/s default policy); prefill tiles
  // (QW > 1) share the lines through L1
  constexpr bool NT = ATTN_DECODE_NT && QW == 1;
  auto ldkv = [&](const bf16* a) { return NT ? ld_nt_bf16x8(a) : ld_bf16x8(a); };
  auto load_k = [&](int page, bf16x8 (&k0)[4], bf16x8 (&k1)[4]) {
    const bf16* kp = p.k_cache + ((size_t)page * p.hkv + h) * kPage * kD;
    // K rows for keys kb + r and kb + 16 + r; k-step s of the 4 lane groups = 64 contiguous bytes of a row.
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      k0[s] = ldkv(kp + (size_t)r * kD + 32 * s + 8 * g);
      k1[s] = ldkv(kp + (size_t)(16 + r) * kD + 32 * s + 8 * g);
    }
  };
  auto load_v = [&](int page, bf16x8 (&vf)[8]) {
    const bf16* vp = p.v_cache + ((size_t)page * p.hkv + h) * kD * kPage;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) vf[dt] = ldkv(vp + (size_t)(16 * dt + r) * kPage + 8 * g);
  };
  auto load_page = [&](int page, bf16x8 (&k0)[4], bf16x8 (&k1)[4], bf16x8 (&vf)[8]) {
    load_k(page, k0, k1);
    load_v(page, vf);
  };
  constexpr int kStep = 32 * KWV;
  const int kb0 = kbeg + 32 * kw;  // this wave's first page: keys kb0 + i * kStep
  bf16x8 rk0[PD][4], rk1[PD][4];   // K rows of the pages in flight (FQ: slot 0 loaded under the slab sums)
  // Q fragments (B operand): lane (r, g) holds Q[col r][d = 32s + 8g + j] in k-step s — the same head-dim
  // order as the K fragments, so each K load instruction reads 64 contiguous bytes of 16 key rows.
  bf16x8 qf[4];
  // FQ: the newest key's K row / V row, computed from the slabs by the key-split wave that attends over its
  // page.  That wave starts its online softmax with this key and masks it out of the page loop (its cache slot
  // is written in this launch, by the same wave, for later steps).  Patching the page's fragments in registers
  // instead cost 50-80 VGPRs (a wave per SIMD).
  constexpr int kMaxG = FQ ? FQG : 1;  // the folded path is instantiated per GQA group (1, 2, 4)
  __shared__ __attribute__((aligned(16))) bf16 s_fq[FQ ? KWV : 1][FQ ? (kMaxG + 2) * kD : 1];  // q heads | k | v
  float sc_new = -INFINITY;  // newest key's score (log2 units) for column r
  int kb_new = -1;            // first key of the newest key's page, or -1 when this wave does not hold it
  int key_limit = col_limit;  // keys below are attended in the page loop
  if constexpr (FQ) {
    // QKV epilogue folded in (decode, one query per sequence = QKV row q_start[b]): sum the split-K slabs,
    // rotate, round to bf16 -- the arithmetic of splitk_reduce_kernel<kQkvRope>, in the same order.  Head
    // columns are in rotary-pair order: 16-column tile t of a head holds d = 8t + j (j < 8) and, 8 columns on,
    // its partner d + 64.  Lane l sums the pair (t, j) = (l / 8, l % 8) of every unit it needs -- all slab
    // loads of the wave are independent, so the slab latency is paid once -- and the rotated values are
    // regrouped into MFMA fragments through the wave's LDS rows.
    const int m = DSSE_IDX(p.q_start[b], p.qkv_M, 0);  // this sequence's QKV row
    const int N = (p.hq + 2 * p.hkv) * kD;
    const size_t slab = (size_t)p.qkv_M * N;
    const int kn_page = (ctx - 1) & ~(kPage - 1);
    const int sl = p.slots[m];
    // wave-uniform: this partition holds the newest key, and the key-split wave visiting its page is this one
    const bool owner = pz == (ctx - 1) / part && sl >= 0 && ((kn_page - kbeg) / kPage) % KWV == kw;
    const int t = lane >> 3, j = lane & 7;
    const float* base = p.qkv_part + (size_t)m * N + 16 * t + j;
    // Slabs 0 and 1 (slab 0 again when S == 1, masked below) are loaded unconditionally -- a guarded load is a
    // branch, and hipcc drains vmcnt at every branch -- then the K rows of the wave's first page are issued, so
    // their HBM latency overlaps the slab sums (K only: the V rows as well cost a wave per SIMD in registers).
    // Units: the group's kMaxG q heads, k, v.
    auto unit_col = [&](int u) {
      return u < kMaxG ? (h * kMaxG + u) * kD : (u == kMaxG ? p.hq + h : p.hq + p.hkv + h) * kD;
    };
    float xa[kMaxG + 2][2], xb[kMaxG + 2][2];
    {
      const float* s0 = base;
      const float* s1 = base + (p.qkv_S > 1 ? slab : 0);
#pragma unroll
      for (int u = 0; u < kMaxG + 2; ++u) {
        const int c0 = unit_col(u);
        xa[u][0] = s0[c0];
        xa[u][1] = s0[c0 + 8];
        xb[u][0] = s1[c0];
        xb[u][1] = s1[c0 + 8];
      }
    }
    load_k(page_of(min(kb0, kend - 1)), rk0[0], rk1[0]);
    const bool two = p.qkv_S > 1;
#pragma unroll
    for (int u = 0; u < kMaxG + 2; ++u) {
      xa[u][0] += two ? xb[u][0] : 0.f;  // x + 0 = x: the same sums as the reduce kernel's 0 + x0 + x1 + ...
      xa[u][1] += two ? xb[u][1] : 0.f;
    }
    for (int k = 2; k < p.qkv_S; ++k) {
      const float* sk = base + k * slab;
#pragma unroll
      for (int u = 0; u < kMaxG + 2; ++u) {
        const int c0 = unit_col(u);
        xa[u][0] += sk[c0];
        xa[u][1] += sk[c0 + 8];
      }
    }
    float (&qa)[kMaxG + 2][2] = xa;
    const float* ka = xa[kMaxG];
    const float* va = xa[kMaxG + 1];
    const float2 c = p.rope[(size_t)DSSE_IDX(p.positions[m], p.rope_len, 0) * 64 + 8 * t + j];
    bf16* fq = s_fq[kw];
    const int d = 8 * t + j;  // this lane's head dims: d and d + 64
#pragma unroll
    for (int u = 0; u < kMaxG; ++u) {
      fq[u * kD + d] = f2bf(qa[u][0] * c.x - qa[u][1] * c.y);
      fq[u * kD + 64 + d] = f2bf(qa[u][1] * c.x + qa[u][0] * c.y);
    }
    if (owner) {
      fq[kMaxG * kD + d] = f2bf(ka[0] * c.x - ka[1] * c.y);
      fq[kMaxG * kD + 64 + d] = f2bf(ka[1] * c.x + ka[0] * c.y);
      fq[(kMaxG + 1) * kD + d] = f2bf(va[0]);
      fq[(kMaxG + 1) * kD + 64 + d] = f2bf(va[1]);
    }
    // LDS rows written and read by this wave only: in-order LDS, no barrier; keep the compiler from hoisting
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s = 0; s < 4; ++s)
      qf[s] = col_valid ? *reinterpret_cast<const bf16x8*>(&fq[(r % G) * kD + 32 * s + 8 * g]) : zero_bf16x8();
    if (owner) {
      kb_new = kn_page;
      key_limit = col_limit - 1;  // decode: the newest key is the last visible one
      bf16x8 kn[4];
      float dot = 0.f;  // q · k over this lane's 32 head dims, then over the 4 lane groups
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        kn[q] = *reinterpret_cast<const bf16x8*>(&fq[kMaxG * kD + 32 * q + 8 * g]);
#pragma unroll
        for (int e = 0; e < 8; ++e) dot += bf2f(qf[q][e]) * bf2f(kn[q][e]);
      }
      dot += __shfl_xor(dot, 16);
      dot += __shfl_xor(dot, 32);
      sc_new = col_valid ? dot * p.scale_log2 : -INFINITY;
      // cache copies for later steps
      const int sidx = DSSE_IDX(sl, p.num_slots, 0), blk = sidx / kPage, off = sidx % kPage;
      if (r == (off & 15)) {
        bf16* kdst = p.k_out + (((size_t)blk * p.hkv + h) * kPage + off) * kD + 8 * g;
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16x8*>(kdst + 32 * q) = kn[q];
      }
      bf16* vdst = p.v_out + ((size_t)blk * p.hkv + h) * kD * kPage + vperm_tok(off);
      vdst[(size_t)d * kPage] = f2bf(va[0]);
      vdst[(size_t)(64 + d) * kPage] = f2bf(va[1]);
    }
  } else {
    const int qrow = p.q_start[b] + (col_valid ? qi : 0);
    const bf16* qp = p.q + ((size_t)qrow * p.hq + h * G + (r % G)) * kD + 8 * g;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = col_valid ? ld_bf16x8(qp + 32 * s) : zero_bf16x8();
  }

  float m_run = -1e30f, l_run = 0.f;
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (FQ) {
    // the newest key opens the online softmax: m = its score, p = 1 (exact in bf16 too), o = its V row
    if (kb_new >= 0 && col_valid) {
      m_run = sc_new;
      l_run = g == 0 ? 1.f : 0.f;  // per-lane partial: counted once per column
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        const bf16x4 vq = *reinterpret_cast<const bf16x4*>(&s_fq[kw][(kMaxG + 1) * kD + 16 * dt + 4 * g]);  // d = 16dt + 4g + i
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
    // element i: key kb + 4g + i (s0) / kb + 16 + 4g + i (s1), column r
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
    for (int dt = 0; dt < 8; ++dt) {
      f32x4 acc = o[dt] * alpha;
      o[dt] = mfma16x16x32(vf[dt], pf, acc);
    }
  };
  int kb = kb0;
  if constexpr (PD == 1) {
    // the next page's index is fetched one page ahead (scalar load under this page's compute)
    int page = kb < kend ? page_of(kb) : 0;
    if constexpr (FQ) {
      if (kb < kend) {  // the first page's K has been in flight since the slab sums
        bf16x8 vf[8];
        load_v(page, vf);
        page = page_of(min(kb + kStep, kend - 1));
        compute_page(kb, rk0[0], rk1[0], vf);
        kb += kStep;
      }
    }
    for (; kb < kend; kb += kStep) {
      bf16x8 k0[4], k1[4], vf[8];
      load_page(page, k0, k1, vf);
      page = page_of(min(kb + kStep, kend - 1));
      compute_page(kb, k0, k1, vf);
    }
  } else if (kb < kend) {
    // Register ring of PD pages: page i + PD - 1 is issued before page i is computed.  Look-ahead loads past the
    // wave's last page re-read that page (an L2 hit) instead of branching around them -- hipcc waits vmcnt(0)
    // at such a join, which would serialise the ring.  Page indices are fetched one issue ahead.
    bf16x8 rv[PD][8];
    const int n = (kend - kb + kStep - 1) / kStep;  // pages of this wave
    auto pg = [&](int i) { return page_of(kb0 + min(i, n - 1) * kStep); };
    if constexpr (FQ) load_v(pg(0), rv[0]);
    else load_page(pg(0), rk0[0], rk1[0], rv[0]);
#pragma unroll
    for (int d = 1; d < PD - 1; ++d) load_page(pg(d), rk0[d], rk1[d], rv[d]);
    int pnext = pg(PD - 1);
    for (int i = 0; i < n; i += PD) {
#pragma unroll
      for (int u = 0; u < PD; ++u) {
        const int ls = (u + PD - 1) % PD;
        load_page(pnext, rk0[ls], rk1[ls], rv[ls]);
        pnext = pg(i + u + PD);
        compute_page(kb0 + (i + u) * kStep, rk0[u], rk1[u], rv[u]);
        if (i + u + 1 >= n) break;
      }
    }
  }
  // l_run is a per-lane partial over this lane's keys: sum the 4 lane groups of the column.
  l_run += __shfl_xor(l_run, 16);
  l_run += __shfl_xor(l_run, 32);

  // ---- merge the KWV key-split waves of each query tile in LDS ----
  if constexpr (KWV > 1) {
    __shared__ float s_o[QW * KWV][8 * 4][64];
    __shared__ float s_m[QW * KWV][16], s_l[QW * KWV][16];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) s_o[w][dt * 4 + i][lane] = o[dt][i];
    if (g == 0) { s_m[w][r] = m_run; s_l[w][r] = l_run; }
    __syncthreads();
    if (kw != 0) return;
    float mm = m_run;
#pragma unroll
    for (int v = 1; v < KWV; ++v) mm = fmaxf(mm, s_m[w + v][r]);
    float sc[KWV], ll = 0.f;
#pragma unroll
    for (int v = 0; v < KWV; ++v) {
      const float mv = v == 0 ? m_run : s_m[w + v][r];
      const float lv = v == 0 ? l_run : s_l[w + v][r];
      sc[v] = exp2f(mv - mm);
      ll += lv * sc[v];
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float acc = o[dt][i] * sc[0];
#pragma unroll
        for (int v = 1; v < KWV; ++v) acc += s_o[w + v][dt * 4 + i][lane] * sc[v];
        o[dt][i] = acc;
      }
    m_run = mm;
    l_run = ll;
  }

  // ---- write: final (single partition) or partial (flash-decoding) ----
  // element (dt, i) of lane (r, g): d = 16dt + 4g + i, column r
  if (p.nparts == 1) {
    if (!col_valid) return;
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    bf16* op = p.out + ((size_t)(p.q_start[b] + qi) * p.hq + h * G + (r % G)) * kD;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) op[16 * dt + 4 * g + i] = f2bf(o[dt][i] * inv);
  } else {
    const size_t base = (((size_t)item * p.hkv + h) * p.nparts + pz) * QW + qw;
    float* po = p.part_o + base * 16 * kD + (size_t)r * kD;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) po[16 * dt + 4 * g + i] = o[dt][i];
    if (g == 0) p.part_ml[base * 16 + r] = make_float2(m_run, l_run);
    if constexpr (QW == 1) {
      // Last-arriver combine (round 6, opt-in attn_comb=1: measured slower than the combine launch on a TP = 8 rank,
      // bindings.cpp attn_last_arriver; decode, one query tile): the wave left in this workgroup publishes its partial
      // (stores drained, agent-scope release) and takes a ticket on its (item, kv head); the partition that draws
      // the last ticket -- every other non-empty partition has released before taking its own -- acquires, merges
      // them (attn_combine_kernel's arithmetic) and resets the ticket for the next launch.  Nobody waits.
      if (p.comb_cnt) {
        const int np = min(p.nparts, (kmax + part - 1) / part);  // the partitions that did not exit empty
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        int* cnt = p.comb_cnt + (size_t)item * p.hkv + h;
        int ticket = 0;
        if (lane == 0) ticket = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ticket = __builtin_amdgcn_readfirstlane(ticket);
        if (ticket != np - 1) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (lane == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const size_t base0 = ((size_t)item * p.hkv + h) * p.nparts;
        float mm = -1e30f;
        for (int z = 0; z < np; ++z) mm = fmaxf(mm, p.part_ml[(base0 + z) * 16 + r].x);
        f32x4 acc[8];
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
        float ll = 0.f;
        for (int z = 0; z < np; ++z) {
          const float2 ml = p.part_ml[(base0 + z) * 16 + r];
          const float sc = exp2f(ml.x - mm);
          ll += ml.y * sc;
          const float* pz_o = p.part_o + (base0 + z) * 16 * kD + (size_t)r * kD + 4 * g;
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) acc[dt] += *reinterpret_cast<const f32x4*>(pz_o + 16 * dt) * sc;
        }
        if (!col_valid) return;
        const float inv = ll > 0.f ? 1.f / ll : 0.f;
        bf16* op = p.out + ((size_t)(p.q_start[b] + qi) * p.hq + h * G + (r % G)) * kD;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) op[16 * dt + 4 * g + i] = f2bf(acc[dt][i] * inv);
      }
    }
  }
}

// Merge flash-decoding partitions: grid (num_work, hkv, QW), block 256 = (16 columns × 16 lanes),
// each thread owns 8 head dims of one column.
template <int QW>
__global__ void __launch_bounds__(256) attn_combine_kernel(AttnParams p) {
  const int item = blockIdx.x, h = blockIdx.y, qw = blockIdx.z;
  const int col = threadIdx.x >> 4, sub = threadIdx.x & 15;
  const int b = p.work_seq[item];
  const int qlen = p.q_len[b], ctx = p.ctx_len[b];
  const int G = p.group, QT = 16 / G;
  const int qi = (p.work_tile[item] * QW + qw) * QT + col / G;
  if (qi >= qlen) return;
  const int last_q = min(qlen, (p.work_tile[item] + 1) * QW * QT) - 1;
  const int kmax = ctx - qlen + last_q + 1;
  const int part = part_keys(p, kmax);
  const int np = min(p.nparts, (kmax + part - 1) / part);
  float mm = -1e30f;
  for (int z = 0; z < np; ++z) {
    const size_t base = (((size_t)item * p.hkv + h) * p.nparts + z) * QW + qw;
    mm = fmaxf(mm, p.part_ml[base * 16 + col].x);
  }
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float ll = 0.f;
  for (int z = 0; z < np; ++z) {
    const size_t base = (((size_t)item * p.hkv + h) * p.nparts + z) * QW + qw;
    const float2 ml = p.part_ml[base * 16 + col];
    const float sc = exp2f(ml.x - mm);
    ll += ml.y * sc;
    const float4* po = reinterpret_cast<const float4*>(p.part_o + (base * 16 + col) * kD + 8 * sub);
    const float4 a = po[0], c = po[1];
    acc[0] += a.x * sc; acc[1] += a.y * sc; acc[2] += a.z * sc; acc[3] += a.w * sc;
    acc[4] += c.x * sc; acc[5] += c.y * sc; acc[6] += c.z * sc; acc[7] += c.w * sc;
  }
  const float inv = ll > 0.f ? 1.f / ll : 0.f;
  bf16x8 ov;
#pragma unroll
  for (int j = 0; j < 8; ++j) ov[j] = f2bf(acc[j] * inv);
  bf16* op = p.out + ((size_t)(p.q_start[b] + qi) * p.hq + h * G + (col % G)) * kD + 8 * sub;
  *reinterpret_cast<bf16x8*>(op) = ov;
}

template <int G>
hipError_t launch_folded(int kwv, int pd, dim3 grid, const AttnParams& p, hipStream_t st) {
  if (kwv == 8) hipLaunchKernelGGL((paged_attention_kernel<1, 8, 1, G>), grid, dim3(512), 0, st, p);
  else if (kwv == 1 && pd == 2) hipLaunchKernelGGL((paged_attention_kernel<1, 1, 2, G>), grid, dim3(64), 0, st, p);
  else if (kwv == 1) hipLaunchKernelGGL((paged_attention_kernel<1, 1, 1, G>), grid, dim3(64), 0, st, p);
  else if (kwv == 2 && pd == 2) hipLaunchKernelGGL((paged_attention_kernel<1, 2, 2, G>), grid, dim3(128), 0, st, p);
  else if (kwv == 2) hipLaunchKernelGGL((paged_attention_kernel<1, 2, 1, G>), grid, dim3(128), 0, st, p);
  else hipLaunchKernelGGL((paged_attention_kernel<1, 4, 1, G>), grid, dim3(256), 0, st, p);
  return hipGetLastError();
}

}  // namespace dsse

// mode 0 = decode (QW = 1, KWV = 4), mode 1 = prefill (QW = 4, KWV = 1), mode 3 = decode reading q from the
// QKV GEMM's split-K slabs and writing the step's K / V (AttnParams::qkv_part).
extern "C" hipError_t dsse_paged_attention(int mode, int num_work, const dsse::AttnParams* p,
                                           hipStream_t st) {
  using namespace dsse;
  if (num_work <= 0) return hipSuccess;
  if (mode == 3) {
    // decode with the QKV epilogue folded in; GQA group 1, 2 or 4.  Every key-split wave sums its q slabs, so
    // fewer waves per workgroup than mode 0 pay off: 2 from 512 workgroups (64 streams: 4.58 vs 4.60 ms/step,
    // 8 waves 4.67-4.71; profiles/experiments_r2.md); from 2048 one wave without look-ahead beat two (9.95 vs
    // 10.20), two with a 2-page ring beat both (below)
    const dim3 grid(num_work, p->hkv, p->nparts);
    const int nwg = grid.x * grid.y * grid.z;
    // 2048+ workgroups (256 streams): one wave per (sequence, kv head), one page in flight -- with the
    // non-temporal K/V loads 9.70 / 9.71 ms/step vs 10.11 / 10.16 for 2 waves x 2 pages (the round-2 choice
    // under default-policy loads) and 10.31 for 2 waves x 1 page (profiles/r3/r3n_ab256.log); 512-2047: 2 waves
    // (128 streams 6.00-6.03 vs 6.23 with 4; 64 streams: look-ahead measured slower)
    const int kwv = p->kwv ? p->kwv : (nwg >= 2048 ? 1 : (nwg >= 512 ? 2 : 4));
    const int pd = p->pd ? p->pd : 1;
    hipError_t e;
    if (p->group == 1) e = launch_folded<1>(kwv, pd, grid, *p, st);
    else if (p->group == 2) e = launch_folded<2>(kwv, pd, grid, *p, st);
    else if (p->group == 4) e = launch_folded<4>(kwv, pd, grid, *p, st);
    else return hipErrorInvalidValue;
    if (e != hipSuccess) return e;
    if (p->nparts > 1 && !p->comb_cnt)
      hipLaunchKernelGGL((attn_combine_kernel<1>), dim3(num_work, p->hkv, 1), dim3(256), 0, st, *p);
  } else if (mode == 0) {
    // decode: p->kwv (attn_kwv in DSSE_KERNEL_CFG, read by the bindings) = waves per workgroup splitting the keys (1/2/4/8).
    // Measured (profiles/attention_decode_r1.md): 4 key-split waves are best up to ~1k workgroups (64 streams x
    // 8 kv heads: 29 us at 560 keys, 5.1 TB/s), one wave per (sequence, kv head) above (256 streams: 100 vs
    // 109 us, 5.9 TB/s).  (A next-page register prefetch variant cost 2-10 % and was removed.)
    const dim3 grid(num_work, p->hkv, p->nparts);
    const int kwv = p->kwv ? p->kwv : (grid.x * grid.y * grid.z >= 2048 ? 1 : 4);
    const int pd = p->pd == 2 && kwv <= 2 ? 2 : 1;  // attn_pd=2 (DSSE_KERNEL_CFG): 2-page register ring (1 / 2 waves)
    if (kwv == 8) hipLaunchKernelGGL((paged_attention_kernel<1, 8, 1>), grid, dim3(512), 0, st, *p);
    else if (kwv == 1 && pd == 2) hipLaunchKernelGGL((paged_attention_kernel<1, 1, 2>), grid, dim3(64), 0, st, *p);
    else if (kwv == 2 && pd == 2) hipLaunchKernelGGL((paged_attention_kernel<1, 2, 2>), grid, dim3(128), 0, st, *p);
    else if (kwv == 1) hipLaunchKernelGGL((paged_attention_kernel<1, 1, 1>), grid, dim3(64), 0, st, *p);
    else if (kwv == 2) hipLaunchKernelGGL((paged_attention_kernel<1, 2, 1>), grid, dim3(128), 0, st, *p);
    else hipLaunchKernelGGL((paged_attention_kernel<1, 4, 1>), grid, dim3(256), 0, st, *p);
    if (p->nparts > 1 && !p->comb_cnt)
      hipLaunchKernelGGL((attn_combine_kernel<1>), dim3(num_work, p->hkv, 1), dim3(256), 0, st, *p);
  } else {
    hipLaunchKernelGGL((paged_attention_kernel<4, 1>), dim3(num_work, p->hkv, p->nparts), dim3(256),
                       0, st, *p);
    if (p->nparts > 1)
      hipLaunchKernelGGL((attn_combine_kernel<4>), dim3(num_work, p->hkv, 4), dim3(256), 0, st, *p);
  }
  return hipGetLastError();
}

DSSE_CHECK_READER(dsse_check_attention)
