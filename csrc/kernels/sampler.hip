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

constexpr int kSThreads = 1024;
constexpr int kSMaxPer = 32;  // V <= 32768

template <typename T>
DEV T block_reduce_sum(T v, T* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  T tot = 0;
#pragma unroll
  for (int i = 0; i < kSThreads / 64; ++i) tot += sh[i];
  __syncthreads();
  return tot;
}

DEV float block_reduce_max(float v, float* sh) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float tot = -INFINITY;
#pragma unroll
  for (int i = 0; i < kSThreads / 64; ++i) tot = fmaxf(tot, sh[i]);
  __syncthreads();
  return tot;
}

// MSB-first radix select.  Returns the key `thr` such that the elements with key >= thr are the
// smallest top set whose weight (count or mass) reaches `target`.  Elements with key < floor_key
// are ignored.
template <bool MASS>
DEV uint32_t radix_select(const float (&x)[kSMaxPer], const uint32_t (&key)[kSMaxPer], int nper,
                          int V, float xmax, uint32_t floor_key, float target, float* hist) {
  uint32_t prefix = 0, mask = 0;
  float remaining = target;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += kSThreads) hist[i] = 0.f;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kSMaxPer; ++j) {
      if (j < nper) {
        const int idx = j * kSThreads + threadIdx.x;
        if (idx < V && key[j] >= floor_key && (key[j] & mask) == prefix) {
          const float wgt = MASS ? exp2f(x[j] - xmax) : 1.f;
          atomicAdd(&hist[(key[j] >> shift) & 255], wgt);
        }
      }
    }
    __syncthreads();
    // every thread scans the 256 bins (cheap, avoids another barrier round)
    float cum = 0.f;
    int digit = 0;
    for (int d = 255; d >= 0; --d) {
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

__global__ void __launch_bounds__(kSThreads) sample_kernel(SampleParams p) {
  const int b = blockIdx.x;
  if (p.active && !p.active[b]) return;
  __shared__ float sh[kSThreads / 64];
  __shared__ float hist[256];
  __shared__ float s_best[kSThreads / 64];
  __shared__ int s_bidx[kSThreads / 64];

  const float* row = p.logits + (size_t)b * p.ld;
  const float temp = p.temperature[b];
  const bool greedy = !(temp > 0.f);
  const float inv_t = greedy ? 1.f : 1.f / temp;
  const int nper = (p.V + kSThreads - 1) / kSThreads;

  float x[kSMaxPer];
  uint32_t key[kSMaxPer];
  float lmax = -INFINITY;
#pragma unroll
  for (int j = 0; j < kSMaxPer; ++j) {
    const int idx = j * kSThreads + threadIdx.x;
    if (j < nper && idx < p.V) {
      x[j] = row[idx] * inv_t * 1.4426950408889634f;  // base-2 scaled logits
      key[j] = fkey(x[j]);
      lmax = fmaxf(lmax, x[j]);
    } else {
      x[j] = -INFINITY;
      key[j] = 0;
    }
  }

  uint32_t thr = 0;
  if (!greedy) {
    const int tk = p.top_k[b];
    const float tp = p.top_p[b];
    const float xmax = block_reduce_max(lmax, sh);
    if (tk > 0 && tk < p.V) thr = radix_select<false>(x, key, nper, p.V, xmax, 0u, (float)tk, hist);
    if (tp < 1.f) {
      float z = 0.f;
#pragma unroll
      for (int j = 0; j < kSMaxPer; ++j)
        if (j < nper && key[j] >= thr && x[j] > -INFINITY) z += exp2f(x[j] - xmax);
      z = block_reduce_sum(z, sh);
      thr = radix_select<true>(x, key, nper, p.V, xmax, thr, tp * z, hist);
    }
  }

  // Gumbel-max (or plain argmax) over kept elements; ties -> smallest index.
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  const uint2 seed = p.seeds ? p.seeds[b] : make_uint2(0, 0);
  const uint32_t pos = p.positions ? (uint32_t)p.positions[b] : 0u;
#pragma unroll
  for (int j = 0; j < kSMaxPer; ++j) {
    const int idx = j * kSThreads + threadIdx.x;
    if (j < nper && idx < p.V && key[j] >= thr) {
      float sc = x[j];
      const int gidx = idx + p.vocab_offset;
      if (!greedy) {
        const uint4 rv = philox4x32(make_uint4((uint32_t)gidx, pos, 0x5353u, 0u), seed);
        const float u = u01(rv.x);
        sc = x[j] * 0.6931471805599453f - __logf(-__logf(u));  // back to natural units + Gumbel
      }
      if (sc > best || (sc == best && gidx < bidx)) { best = sc; bidx = gidx; }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ob = __shfl_xor(best, o);
    const int oi = __shfl_xor(bidx, o);
    if (ob > best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
  }
  if ((threadIdx.x & 63) == 0) { s_best[threadIdx.x >> 6] = best; s_bidx[threadIdx.x >> 6] = bidx; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int i = 1; i < kSThreads / 64; ++i) {
    if (s_best[i] > best || (s_best[i] == best && s_bidx[i] < bidx)) { best = s_best[i]; bidx = s_bidx[i]; }
  }
  if (p.candidates_only) {
    p.cand[b] = make_float2(best, __int_as_float(bidx));
    return;
  }
  p.next_ids[b] = bidx;
  if (p.ring) p.ring[(size_t)(p.ring_counter[0] % p.ring_size) * p.ring_stride + b] = bidx;
  if (p.positions_inc) p.positions_inc[b] += 1;
}

// Merge per-rank candidates [world, B] (tensor-parallel vocab shards) and commit the token.
__global__ void sample_pick_kernel(const float2* __restrict__ cand, int world, int B, SampleParams p) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  if (p.active && !p.active[b]) return;
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int w = 0; w < world; ++w) {
    const float2 c = cand[(size_t)w * B + b];
    const int ci = __float_as_int(c.y);
    if (c.x > best || (c.x == best && ci < bidx)) { best = c.x; bidx = ci; }
  }
  p.next_ids[b] = bidx;
  if (p.ring) p.ring[(size_t)(p.ring_counter[0] % p.ring_size) * p.ring_stride + b] = bidx;
  if (p.positions_inc) p.positions_inc[b] += 1;
}

}  // namespace dsse

extern "C" hipError_t dsse_sample(int B, const dsse::SampleParams* p, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (p->V > dsse::kSThreads * dsse::kSMaxPer) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dsse::sample_kernel, dim3(B), dim3(dsse::kSThreads), 0, st, *p);
  return hipGetLastError();
}

extern "C" hipError_t dsse_sample_pick(int B, int world, const void* cand,
                                       const dsse::SampleParams* p, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(dsse::sample_pick_kernel, dim3((B + 63) / 64), dim3(64), 0, st,
                     reinterpret_cast<const float2*>(cand), world, B, *p);
  return hipGetLastError();
}
