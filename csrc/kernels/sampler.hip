// K10 sampler: greedy / temperature / top-k / top-p with a counter-based Philox RNG.
//
// One 1024-thread workgroup per batch row; the row (<= 32768 logits) stays in registers
// (<= 32 per thread).  Sampling is exact Gumbel-max: argmax_i (x_i / T + G_i) with
// G_i = -log(-log(U_i)), U_i = Philox(seed, counter = (global vocab index, position)).  The
// noise depends only on (seed, position, global index), so a vocab-sharded (tensor-parallel)
// run draws the same token as TP = 1: each rank reports its (score, index) candidate and the
// candidates are merged by max (sample_pick_kernel).  top-k / top-p thresholds are found by an
// MSB-first 8-bit radix select over order-preserving float keys — counts for top-k, softmax
// mass for top-p — four passes each, no sort.
#include "api.h"

namespace dsse {


DEV uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int kSThreads = 1024;   // filtered path: one workgroup per row
constexpr int kSMaxV = 32768;     // per-rank vocab limit (row staged in 128 KiB of LDS)
constexpr int kCThreads = 256;    // unfiltered path: one workgroup per (row, vocab chunk)

DEV bool row_filtered(const SampleParams& p, int b) {
  return p.temperature[b] > 0.f && ((p.top_k[b] > 0 && p.top_k[b] < p.V) || p.top_p[b] < 1.f);
}

// Score of one logit: greedy -> the logit itself; sampling -> logit/T + Gumbel(seed, pos, gidx).
DEV float score(float logit, float inv_t, bool greedy, uint2 seed, uint32_t pos, int gidx) {
  if (greedy) return logit;
  const uint4 rv = philox4x32(make_uint4((uint32_t)gidx, pos, 0x5353u, 0u), seed);
  return logit * inv_t - __logf(-__logf(u01(rv.x)));
}

DEV void better(float& best, int& bidx, float s, int i) {
  if (s > best || (s == best && i < bidx)) { best = s; bidx = i; }
}

template <int NT>
DEV void block_argmax(float& best, int& bidx, float* s_best, int* s_bidx) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) better(best, bidx, __shfl_xor(best, o), __shfl_xor(bidx, o));
  if ((threadIdx.x & 63) == 0) { s_best[threadIdx.x >> 6] = best; s_bidx[threadIdx.x >> 6] = bidx; }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int i = 1; i < NT / 64; ++i) better(best, bidx, s_best[i], s_bidx[i]);
}

// Unfiltered rows (greedy or pure temperature): Gumbel-max is separable, so each (row, chunk)
// workgroup proposes the best (score, index) of its vocab slice.
__global__ void __launch_bounds__(kCThreads) sample_chunk_kernel(SampleParams p) {
  const int c = blockIdx.x, b = blockIdx.y;
  if ((p.active && !p.active[b]) || row_filtered(p, b)) return;
  __shared__ float s_best[kCThreads / 64];
  __shared__ int s_bidx[kCThreads / 64];
  const float temp = p.temperature[b];
  const bool greedy = !(temp > 0.f);
  const float inv_t = greedy ? 1.f : 1.f / temp;
  const uint2 seed = p.seeds[b];
  const uint32_t pos = (uint32_t)p.positions[b];
  const int chunk = (p.V + p.nchunks - 1) / p.nchunks;
  const int lo = c * chunk, hi = min(p.V, lo + chunk);
  const float* row = p.logits + (size_t)b * p.ld;
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int i = lo + threadIdx.x; i < hi; i += kCThreads)
    better(best, bidx, score(row[i], inv_t, greedy, seed, pos, i + p.vocab_offset), i + p.vocab_offset);
  block_argmax<kCThreads>(best, bidx, s_best, s_bidx);
  if (threadIdx.x == 0) p.cand[(size_t)b * p.nchunks + c] = make_float2(best, __int_as_float(bidx));
}

// MSB-first radix select over LDS-resident base-2 logits.  Returns the key `thr` such that the
// elements with key >= thr form the smallest top set whose weight (count or softmax mass) reaches
// `target`; elements with key < floor_key are ignored.
template <bool MASS>
DEV uint32_t radix_select(const float* xs, int V, float xmax, uint32_t floor_key, float target, float* hist) {
  uint32_t prefix = 0, mask = 0;
  float remaining = target;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += kSThreads) hist[i] = 0.f;
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += kSThreads) {
      const uint32_t k = fkey(xs[i]);
      if (k >= floor_key && (k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255], MASS ? exp2f(xs[i] - xmax) : 1.f);
    }
    __syncthreads();
    float cum = 0.f;
    int digit = 0;
    for (int d = 255; d >= 0; --d) {  // every thread scans the 256 bins (no extra barrier round)
      const float hv = hist[d];
      if (cum + hv >= remaining) { digit = d; break; }
      cum += hv;
    }
    remaining -= cum;
    prefix |= (uint32_t)digit << shift;
    mask |= 255u << shift;
    __syncthreads();
  }
  return prefix;
}

template <typename T>
DEV T block_sum(T v, T* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  T tot = 0;
  for (int i = 0; i < kSThreads / 64; ++i) tot += sh[i];
  __syncthreads();
  return tot;
}
DEV float block_max(float v, float* sh) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float tot = -INFINITY;
  for (int i = 0; i < kSThreads / 64; ++i) tot = fmaxf(tot, sh[i]);
  __syncthreads();
  return tot;
}

// Rows with top-k / top-p: one workgroup per row, the whole (local) row staged in LDS.
__global__ void __launch_bounds__(kSThreads) sample_filtered_kernel(SampleParams p) {
  const int b = blockIdx.x;
  if ((p.active && !p.active[b]) || !row_filtered(p, b)) return;
  __shared__ float xs[kSMaxV];
  __shared__ float hist[256];
  __shared__ float sh[kSThreads / 64];
  __shared__ int shi[kSThreads / 64];
  const float inv_t = 1.f / p.temperature[b];
  const float* row = p.logits + (size_t)b * p.ld;
  float lmax = -INFINITY;
  for (int i = threadIdx.x; i < p.V; i += kSThreads) {
    const float x = row[i] * inv_t * 1.4426950408889634f;  // base-2 scaled
    xs[i] = x;
    lmax = fmaxf(lmax, x);
  }
  const float xmax = block_max(lmax, sh);
  uint32_t thr = 0;
  const int tk = p.top_k[b];
  const float tp = p.top_p[b];
  if (tk > 0 && tk < p.V) thr = radix_select<false>(xs, p.V, xmax, 0u, (float)tk, hist);
  if (tp < 1.f) {
    float z = 0.f;
    for (int i = threadIdx.x; i < p.V; i += kSThreads)
      if (fkey(xs[i]) >= thr) z += exp2f(xs[i] - xmax);
    z = block_sum(z, sh);
    thr = radix_select<true>(xs, p.V, xmax, thr, tp * z, hist);
  }
  const uint2 seed = p.seeds[b];
  const uint32_t pos = (uint32_t)p.positions[b];
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int i = threadIdx.x; i < p.V; i += kSThreads) {
    if (fkey(xs[i]) < thr) continue;
    const int gidx = i + p.vocab_offset;
    const uint4 rv = philox4x32(make_uint4((uint32_t)gidx, pos, 0x5353u, 0u), seed);
    better(best, bidx, xs[i] * 0.6931471805599453f - __logf(-__logf(u01(rv.x))), gidx);
  }
  block_argmax<kSThreads>(best, bidx, sh, shi);
  if (threadIdx.x == 0) {
    p.cand[(size_t)b * p.nchunks] = make_float2(best, __int_as_float(bidx));
    for (int c = 1; c < p.nchunks; ++c)
      p.cand[(size_t)b * p.nchunks + c] = make_float2(-INFINITY, __int_as_float(0x7fffffff));
  }
}

// Merge candidates [world, B, nchunks] (vocab chunks x tensor-parallel shards) and commit the token:
// next_ids[b], ring[head][b], positions[b] += 1.
__global__ void sample_pick_kernel(const float2* __restrict__ cand, int world, int B, SampleParams p) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if (p.active && !p.active[b]) return;
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int w = 0; w < world; ++w)
    for (int c = 0; c < p.nchunks; ++c) {
      const float2 v = cand[((size_t)w * B + b) * p.nchunks + c];
      better(best, bidx, v.x, __float_as_int(v.y));
    }
  bidx = DSSE_IDX(bidx, p.v_global, 0);  // no candidate (all logits NaN / -inf) is a bug upstream
  p.next_ids[b] = bidx;
  if (p.ring) p.ring[(size_t)(p.ring_counter[0] % p.ring_size) * p.ring_stride + b] = bidx;
  if (p.positions_inc) p.positions_inc[b] += 1;
}

// First-token sampling of the prompts a captured prefill / mixed graph finishes (round 6: inside the graph, no torch
// index kernels).  meta = [rows[NS] | slots[NS] | last_pos[NS] | n | ring_row] (uploaded with the graph's other
// metadata); slot_meta = the runner's per-slot sampling state [active | temperature | top_k | top_p | seeds x 2]
// (Bm each).  Gather: row i < n of xl = x[rows[i]] (zeros for i >= n) and the sampling parameters of slots[i] into
// smeta = [active | temperature | top_k | top_p | seeds x 2 | position] (NS each; active = i < n).
__global__ void __launch_bounds__(256)
prefill_sample_gather_kernel(const bf16* __restrict__ x, int T, int H, const int* __restrict__ meta, int NS,
                             const int* __restrict__ slot_meta, int Bm, bf16* __restrict__ xl, int* __restrict__ smeta) {
  const int i = blockIdx.x;
  const int n = meta[3 * NS];
  const bool on = i < n;
  const int row = on ? DSSE_IDX(meta[i], T, 0) : 0;
  const int H8 = H / 8;
  for (int c = threadIdx.x; c < H8; c += blockDim.x) {
    const bf16x8 v = on ? *reinterpret_cast<const bf16x8*>(x + (size_t)row * H + 8 * c) : zero_bf16x8();
    *reinterpret_cast<bf16x8*>(xl + (size_t)i * H + 8 * c) = v;
  }
  if (threadIdx.x == 0) {
    const int slot = on ? DSSE_IDX(meta[NS + i], Bm, 0) : 0;
    smeta[i] = on ? 1 : 0;
    smeta[NS + i] = slot_meta[Bm + slot];          // temperature (bits)
    smeta[2 * NS + i] = slot_meta[2 * Bm + slot];  // top_k
    smeta[3 * NS + i] = slot_meta[3 * Bm + slot];  // top_p (bits)
    smeta[4 * NS + 2 * i] = slot_meta[4 * Bm + 2 * slot];
    smeta[4 * NS + 2 * i + 1] = slot_meta[4 * Bm + 2 * slot + 1];
    smeta[6 * NS + i] = on ? meta[2 * NS + i] : 0;  // the sampled token's predecessor position (RNG counter)
  }
}

// Commit the picked first tokens: ids[slot], ring[ring_row][slot], positions[slot] = last_pos + 1.
__global__ void prefill_sample_commit_kernel(const int* __restrict__ meta, int NS, const int* __restrict__ new_ids,
                                             int* __restrict__ ids, int Bm, int* __restrict__ ring, int R,
                                             int* __restrict__ positions) {
  const int i = threadIdx.x;
  if (i >= NS || i >= meta[3 * NS]) return;
  const int slot = DSSE_IDX(meta[NS + i], Bm, -1);
  if (slot < 0) return;
  const int row = DSSE_IDX(meta[3 * NS + 1], R, 0);
  ids[slot] = new_ids[i];
  ring[(size_t)row * Bm + slot] = new_ids[i];
  positions[slot] = meta[2 * NS + i] + 1;
}

}  // namespace dsse

extern "C" hipError_t dsse_prefill_sample_gather(const void* x, int T, int H, const int* meta, int NS,
                                                 const int* slot_meta, int Bm, void* xl, int* smeta, hipStream_t st) {
  if (NS <= 0 || H % 8 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dsse::prefill_sample_gather_kernel, dim3(NS), dim3(256), 0, st,
                     reinterpret_cast<const bf16*>(x), T, H, meta, NS, slot_meta, Bm, reinterpret_cast<bf16*>(xl),
                     smeta);
  return hipGetLastError();
}

extern "C" hipError_t dsse_prefill_sample_commit(const int* meta, int NS, const int* new_ids, int* ids, int Bm,
                                                 int* ring, int R, int* positions, hipStream_t st) {
  if (NS <= 0 || NS > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dsse::prefill_sample_commit_kernel, dim3(1), dim3(64), 0, st, meta, NS, new_ids, ids, Bm, ring,
                     R, positions);
  return hipGetLastError();
}

// Per-rank candidate pass: fills p->cand[B, nchunks].
extern "C" hipError_t dsse_sample(int B, const dsse::SampleParams* p, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (p->V > dsse::kSMaxV || p->nchunks < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dsse::sample_chunk_kernel, dim3(p->nchunks, B), dim3(dsse::kCThreads), 0, st, *p);
  hipLaunchKernelGGL(dsse::sample_filtered_kernel, dim3(B), dim3(dsse::kSThreads), 0, st, *p);
  return hipGetLastError();
}

// Merge pass over cand [world, B, nchunks].
extern "C" hipError_t dsse_sample_pick(int B, int world, const void* cand, const dsse::SampleParams* p,
                                       hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(dsse::sample_pick_kernel, dim3((B + 63) / 64), dim3(64), 0, st,
                     reinterpret_cast<const float2*>(cand), world, B, *p);
  return hipGetLastError();
}

DSSE_CHECK_READER(dsse_check_sampler)
