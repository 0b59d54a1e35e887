// Memory-bound helper kernels of the decode/prefill step (K1, K2, K4, K11 of SURVEY.md §2.4).
// All bf16 traffic is vectorised to 8-16 bytes per lane (guide Guideline 13).
#include <algorithm>
#include "api.h"

namespace dsse {

constexpr int kPageTok = 32;

DEV int vperm_tok(int off) { return ((off & 15) >> 2) * 8 + ((off >> 4) & 1) * 4 + (off & 3); }

// ---- K1 + K2: (embedding gather | residual add) + RMSNorm ------------------------------------
// MODE 0: y = rmsnorm(resid)            MODE 1: resid += delta; y = rmsnorm(resid)
// MODE 2: resid = embed[ids[m]]; y = rmsnorm(resid)
// MODE 3: resid += sum_s part[s, m, :] (fp32 split-K slabs of the O / down projection, fusing the
//         split-K reduction into the norm that consumes it); y = rmsnorm(resid)
// The residual stream is fp32 [M, H]; y is the bf16 input of the next GEMM.  One workgroup of
// min(1024, H/4) threads per row (a decode batch has only M <= 64 rows, so the row is spread over
// as many waves as possible to keep enough loads in flight); each thread owns H / (4·threads) float4s.
template <int MODE>
__global__ void __launch_bounds__(1024)
rmsnorm_kernel(float* __restrict__ resid, int H, const bf16* __restrict__ delta,
               const bf16* __restrict__ embed, const int* __restrict__ ids,
               const bf16* __restrict__ w, bf16* __restrict__ y, float eps,
               const float* __restrict__ part = nullptr, int nsplit = 0, int M = 0, int vocab = 0) {
  const int m = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const unsigned long long st0 = stamps::now();
  float* rrow = resid + (size_t)m * H;
  constexpr int kMaxIt = 2;  // H <= 8192
  float4 v[kMaxIt];
  const int nit = H / (4 * nt);
  float ss = 0.f;
  // the norm weights are loaded with the row, not after the block reduction: one dependent round trip fewer
  bf16x4 wv[kMaxIt];
#pragma unroll
  for (int it = 0; it < kMaxIt; ++it)
    if (it < nit) wv[it] = *reinterpret_cast<const bf16x4*>(w + (it * nt + tid) * 4);
#pragma unroll
  for (int it = 0; it < kMaxIt; ++it) {
    if (it < nit) {
      const int i = (it * nt + tid) * 4;
      float4 x;
      if constexpr (MODE == 2) {
        const bf16x4 e = *reinterpret_cast<const bf16x4*>(embed + (size_t)DSSE_IDX(ids[m], vocab, 0) * H + i);
        x = make_float4(bf2f(e[0]), bf2f(e[1]), bf2f(e[2]), bf2f(e[3]));
      } else {
        x = *reinterpret_cast<const float4*>(rrow + i);
        if constexpr (MODE == 1) {
          const bf16x4 d = *reinterpret_cast<const bf16x4*>(delta + (size_t)m * H + i);
          x.x += bf2f(d[0]); x.y += bf2f(d[1]); x.z += bf2f(d[2]); x.w += bf2f(d[3]);
        }
        if constexpr (MODE == 3) {
          const float* p = part + (size_t)m * H + i;
          const size_t slab = (size_t)M * H;
          int s = 0;
          for (; s + 4 <= nsplit; s += 4) {  // four independent loads in flight per step
            const float4 d0 = *reinterpret_cast<const float4*>(p + (s + 0) * slab);
            const float4 d1 = *reinterpret_cast<const float4*>(p + (s + 1) * slab);
            const float4 d2 = *reinterpret_cast<const float4*>(p + (s + 2) * slab);
            const float4 d3 = *reinterpret_cast<const float4*>(p + (s + 3) * slab);
            x.x += (d0.x + d1.x) + (d2.x + d3.x);
            x.y += (d0.y + d1.y) + (d2.y + d3.y);
            x.z += (d0.z + d1.z) + (d2.z + d3.z);
            x.w += (d0.w + d1.w) + (d2.w + d3.w);
          }
          for (; s < nsplit; ++s) {
            const float4 d = *reinterpret_cast<const float4*>(p + s * slab);
            x.x += d.x; x.y += d.y; x.z += d.z; x.w += d.w;
          }
        }
      }
      if constexpr (MODE != 0) *reinterpret_cast<float4*>(rrow + i) = x;
      v[it] = x;
      ss += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
    }
  }
  if (DSSE_PIPE_STAMPS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long st1 = stamps::now();  // the row's values (and slab sums) landed
  ss = wave_sum(ss);
  __shared__ float red[16];
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
  for (int i = 0; i < (nt >> 6); ++i) tot += red[i];
  const float inv = rsqrtf(tot / (float)H + eps);
  const unsigned long long st2 = stamps::now();
#pragma unroll
  for (int it = 0; it < kMaxIt; ++it) {
    if (it < nit) {
      const int i = (it * nt + tid) * 4;
      bf16x4 o;
      o[0] = f2bf(v[it].x * inv * bf2f(wv[it][0]));
      o[1] = f2bf(v[it].y * inv * bf2f(wv[it][1]));
      o[2] = f2bf(v[it].z * inv * bf2f(wv[it][2]));
      o[3] = f2bf(v[it].w * inv * bf2f(wv[it][3]));
      *reinterpret_cast<bf16x4*>(y + (size_t)m * H + i) = o;
    }
  }
  stamps::record(stamps::kNorm | MODE << 8, st0, st1, st2);
}

// ---- K4 (prefill side): RoPE on q/k + paged KV write from a library-GEMM QKV output ----------
// qkv: [T, (hq + 2 hkv) * 128] bf16 in the engine's permuted column order (inside each 16-column
// tile j of a head: columns 0..7 = dims 8j..8j+7, columns 8..15 = dims 64+8j..64+8j+7).
// A token's rows: each thread rotates 8 pairs of one (unit, tile j) with 16-byte loads and stores.
DEV void rope_kv_rows(const bf16* __restrict__ qkv, int hq, int hkv, const int* __restrict__ positions,
                      const int* __restrict__ slots, const float2* __restrict__ rope, bf16* __restrict__ q_out,
                      bf16* __restrict__ k_cache, int num_slots, int rope_len, int t) {
  const int ncols = (hq + 2 * hkv) * 128;
  const bf16* row = qkv + (size_t)t * ncols;
  const int pos = DSSE_IDX(positions[t], rope_len, 0);
  const int slot = slots[t] < 0 ? -1 : DSSE_IDX(slots[t], num_slots, -1);
  const int blk = slot >= 0 ? slot / kPageTok : 0, off = slot >= 0 ? slot % kPageTok : 0;
  const int nrot = (hq + hkv) * 8;  // q and k heads x 8 column tiles (V: v_page_write)
  for (int idx = threadIdx.x; idx < nrot; idx += blockDim.x) {
    const int u = idx >> 3, j = idx & 7;
    bf16* dst = u < hq ? q_out + ((size_t)t * hq + u) * 128
                       : (slot >= 0 ? k_cache + (((size_t)blk * hkv + (u - hq)) * kPageTok + off) * 128 : nullptr);
    if (dst == nullptr) continue;
    const bf16x8 x1 = ld_bf16x8(row + u * 128 + 16 * j);
    const bf16x8 x2 = ld_bf16x8(row + u * 128 + 16 * j + 8);
    const float4* cs4 = reinterpret_cast<const float4*>(rope + (size_t)pos * 64 + 8 * j);
    bf16x8 o1, o2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float4 cs = cs4[e];  // (cos, sin) of pairs 2e and 2e + 1
      const float a0 = bf2f(x1[2 * e]), b0 = bf2f(x2[2 * e]), a1 = bf2f(x1[2 * e + 1]), b1 = bf2f(x2[2 * e + 1]);
      o1[2 * e] = f2bf(a0 * cs.x - b0 * cs.y);
      o2[2 * e] = f2bf(b0 * cs.x + a0 * cs.y);
      o1[2 * e + 1] = f2bf(a1 * cs.z - b1 * cs.w);
      o2[2 * e + 1] = f2bf(b1 * cs.z + a1 * cs.w);
    }
    *reinterpret_cast<bf16x8*>(dst + 8 * j) = o1;
    *reinterpret_cast<bf16x8*>(dst + 64 + 8 * j) = o2;
  }
}

// ---- V into the transposed, token-permuted pages, a page row at a time -----------------------------------------
// A per-token form writes 2 bytes per (token, d): 128 scattered stores per head per token.  Here 128 threads take
// 32 consecutive rows x one kv head; thread d gathers its 32 values (coalesced
// over d) and, when the 32 rows fill one whole page in order (prefill of a page-aligned run), writes the page's row
// d as 4 x 16-byte stores in the vperm token order.  Other groups (page boundaries, padding, scattered slots) fall
// back to per-element stores.
// (rows t0 .. t0 + 31, kv head h, dim d = the thread's index in its 128-thread half; a wave never spans two heads)
DEV void v_page_write(const bf16* __restrict__ qkv, int T, int hq, int hkv, const int* __restrict__ slots,
                      bf16* __restrict__ v_cache, int num_slots, int t0, int h, int d) {
  const int ncols = (hq + 2 * hkv) * 128;
  const int lane = threadIdx.x & 63;
  const int tl = t0 + (lane & 31);
  const int my_slot = tl < T ? (slots[tl] < 0 ? -1 : DSSE_IDX(slots[tl], num_slots, -1)) : -1;
  const int s0 = __shfl(my_slot, 0);
  const bool whole = __all(s0 >= 0 && s0 % kPageTok == 0 && my_slot == s0 + (lane & 31));
  // qkv columns are in the engine's permuted order: inside 16-column tile j, columns 0-7 = dims 8j..8j+7 and columns
  // 8-15 = dims 64 + 8j .. 64 + 8j + 7
  const int col = d < 64 ? 16 * (d >> 3) + (d & 7) : 16 * ((d - 64) >> 3) + 8 + (d & 7);
  const bf16* src = qkv + (size_t)t0 * ncols + (hq + hkv + h) * 128 + col;
  if (whole) {
    bf16 v[kPageTok];
#pragma unroll
    for (int i = 0; i < kPageTok; ++i) v[i] = src[(size_t)i * ncols];
    bf16x8 o[4];
#pragma unroll
    for (int i = 0; i < kPageTok; ++i) o[vperm_tok(i) >> 3][vperm_tok(i) & 7] = v[i];
    bf16* dst = v_cache + (((size_t)(s0 / kPageTok) * hkv + h) * 128 + d) * kPageTok;
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16x8*>(dst + 8 * q) = o[q];
    return;
  }
  for (int i = 0; i < kPageTok && t0 + i < T; ++i) {
    const int sl = __shfl(my_slot, i);
    if (sl < 0) continue;
    v_cache[(((size_t)(sl / kPageTok) * hkv + h) * 128 + d) * kPageTok + vperm_tok(sl % kPageTok)] = src[(size_t)i * ncols];
  }
}

// One launch for both: blocks [0, T) rotate q / k of one token each (rope_kv_rows), the blocks after
// them write V page rows, two kv heads per 256-thread block.
__global__ void __launch_bounds__(256)
rope_kv_v_kernel(const bf16* __restrict__ qkv, int T, int hq, int hkv, const int* __restrict__ positions,
                 const int* __restrict__ slots, const float2* __restrict__ rope, bf16* __restrict__ q_out,
                 bf16* __restrict__ k_cache, bf16* __restrict__ v_cache, int num_slots, int rope_len) {
  if ((int)blockIdx.x < T) {
    rope_kv_rows(qkv, hq, hkv, positions, slots, rope, q_out, k_cache, num_slots, rope_len, blockIdx.x);
    return;
  }
  const int vb = blockIdx.x - T, hpairs = (hkv + 1) / 2;
  const int h = 2 * (vb % hpairs) + (threadIdx.x >> 7);
  if (h >= hkv) return;  // wave-uniform (128-thread halves)
  v_page_write(qkv, T, hq, hkv, slots, v_cache, num_slots, (vb / hpairs) * kPageTok, h, threadIdx.x & 127);
}

// ---- SiLU·mul over the interleaved gate/up output of a library GEMM (prefill) ---------------
// gu: [T, 2F] with 16-column tiles (0..7 gate[8t..8t+7], 8..15 up[8t..8t+7]) -> h: [T, F]
// Block (x, y) takes 1024 tiles of row y (grid-strided over rows past 65535): each thread loads its four tiles'
// gate and up halves (8 x 16 B in flight) before it computes -- the one-tile-per-iteration form with a 64-bit
// division per tile ran the 8k-row pass at 5.9 TB/s.
__global__ void __launch_bounds__(256)
silu_mul_kernel(const bf16* __restrict__ gu, bf16* __restrict__ h, int F, int T) {
  const int tiles = F / 8;
  for (int t = blockIdx.y; t < T; t += gridDim.y) {
    const bf16* src = gu + (size_t)t * 2 * F;
    bf16* dst = h + (size_t)t * F;
    const int tile0 = blockIdx.x * 1024 + threadIdx.x;
    bf16x8 gv[4], uv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int tile = tile0 + 256 * u;
      if (tile < tiles) {
        gv[u] = *reinterpret_cast<const bf16x8*>(src + tile * 16);
        uv[u] = *reinterpret_cast<const bf16x8*>(src + tile * 16 + 8);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int tile = tile0 + 256 * u;
      if (tile < tiles) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(silu(bf2f(gv[u][j])) * bf2f(uv[u][j]));
        *reinterpret_cast<bf16x8*>(dst + tile * 8) = o;
      }
    }
  }
}

// ---- decode-step metadata (runs first inside the captured graph) -----------------------------
// For slot b: live sequences process the token at positions[b]; dead slots write nothing.
__global__ void decode_prep_kernel(int B, const int* __restrict__ active, const int* __restrict__ positions,
                                   const int* __restrict__ block_tables, int max_blocks, int num_blocks,
                                   int* __restrict__ slots, int* __restrict__ ctx_len,
                                   int* __restrict__ q_len) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if (active[b]) {
    const int pos = positions[b];
    const int page = DSSE_IDX(block_tables[(size_t)b * max_blocks + DSSE_IDX(pos / kPageTok, max_blocks, 0)],
                              num_blocks, 0);
    slots[b] = page * kPageTok + pos % kPageTok;
    ctx_len[b] = pos + 1;
    q_len[b] = 1;
  } else {
    slots[b] = -1;
    ctx_len[b] = 0;
    q_len[b] = 0;
  }
}

// Token-ring head advance (one thread), the last node of a step.
__global__ void ring_advance_kernel(int* counter) { counter[0] += 1; }

}  // namespace dsse

using namespace dsse;

extern "C" hipError_t dsse_rmsnorm(int mode, int M, float* resid, int H, const void* delta,
                                   const void* embed, const int* ids, const void* w, void* y,
                                   float eps, const float* part, int nsplit, int vocab, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  const bf16* d = reinterpret_cast<const bf16*>(delta);
  const bf16* e = reinterpret_cast<const bf16*>(embed);
  const bf16* wp = reinterpret_cast<const bf16*>(w);
  bf16* yp = reinterpret_cast<bf16*>(y);
  // nit float4s per thread, nt threads: H == 4 nt nit exactly (H = 5120: 640 threads x 2), nt whole waves
  const int nit = (H / 4 + 1023) / 1024, nt = H / 4 / nit;
  if (nit > 2 || 4 * nt * nit != H || nt % 64 != 0) return hipErrorInvalidValue;
  switch (mode) {
    case 0: hipLaunchKernelGGL(rmsnorm_kernel<0>, dim3(M), dim3(nt), 0, st, resid, H, d, e, ids, wp, yp, eps, part, nsplit, M, vocab); break;
    case 1: hipLaunchKernelGGL(rmsnorm_kernel<1>, dim3(M), dim3(nt), 0, st, resid, H, d, e, ids, wp, yp, eps, part, nsplit, M, vocab); break;
    case 2: hipLaunchKernelGGL(rmsnorm_kernel<2>, dim3(M), dim3(nt), 0, st, resid, H, d, e, ids, wp, yp, eps, part, nsplit, M, vocab); break;
    case 3: hipLaunchKernelGGL(rmsnorm_kernel<3>, dim3(M), dim3(nt), 0, st, resid, H, d, e, ids, wp, yp, eps, part, nsplit, M, vocab); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

extern "C" hipError_t dsse_rope_kv_write(int T, const void* qkv, int hq, int hkv, const int* positions,
                                         const int* slots, const float2* rope, void* q_out,
                                         void* k_cache, void* v_cache, int num_slots, int rope_len,
                                         hipStream_t st) {
  if (T <= 0) return hipSuccess;
  const int vblocks = (T + kPageTok - 1) / kPageTok * ((hkv + 1) / 2);
  hipLaunchKernelGGL(rope_kv_v_kernel, dim3(T + vblocks), dim3(256), 0, st, reinterpret_cast<const bf16*>(qkv), T,
                     hq, hkv, positions, slots, rope, reinterpret_cast<bf16*>(q_out), reinterpret_cast<bf16*>(k_cache),
                     reinterpret_cast<bf16*>(v_cache), num_slots, rope_len);
  return hipGetLastError();
}

extern "C" hipError_t dsse_silu_mul(int T, int F, const void* gu, void* h, hipStream_t st) {
  if (T <= 0) return hipSuccess;
  const dim3 grid((F / 8 + 1023) / 1024, std::min(T, 65535));
  hipLaunchKernelGGL(silu_mul_kernel, grid, dim3(256), 0, st,
                     reinterpret_cast<const bf16*>(gu), reinterpret_cast<bf16*>(h), F, T);
  return hipGetLastError();
}

extern "C" hipError_t dsse_decode_prep(int B, const int* active, const int* positions,
                                       const int* block_tables, int max_blocks, int num_blocks, int* slots,
                                       int* ctx_len, int* q_len, hipStream_t st) {
  hipLaunchKernelGGL(decode_prep_kernel, dim3((B + 255) / 256), dim3(256), 0, st, B, active,
                     positions, block_tables, max_blocks, num_blocks, slots, ctx_len, q_len);
  return hipGetLastError();
}

extern "C" hipError_t dsse_ring_advance(int* counter, hipStream_t st) {
  hipLaunchKernelGGL(ring_advance_kernel, dim3(1), dim3(1), 0, st, counter);
  return hipGetLastError();
}

DSSE_CHECK_READER(dsse_check_elementwise)
DSSE_STAMPS_BINDER(dsse_stamps_bind_elementwise)
