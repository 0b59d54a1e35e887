// Per-CU fill-rate microbenchmark (round 3; round 6: 4 or 8 waves per workgroup, up to 32 KiB in flight per wave,
// X footprints of 2 MiB (one XCD's L2) and 8 MiB (spills the 4 MiB L2 into the Infinity Cache)): how many bytes
// per second one CU can bring on chip, by path.
//
// The decode GEMMs at 64-256 rows all measured ~35-39 GB/s of LDS-DMA fill per CU (gemm_ring at 64 rows,
// gemm_tiled at 256 rows and at 8192 rows alike: profiles/r3/fillbench.md), which bounds them whatever the
// MFMA work.  This program measures the paths separately and together, one 256-thread workgroup per CU:
//   mode 0  X: global_load_lds_dwordx4 (LDS-DMA) of an L2-resident 2 MiB buffer, every wave loading
//   mode 1  W: global_load_dwordx4 into VGPRs (nt) streaming a 2 GiB buffer once (HBM)
//   mode 2  W: buffer_load ... lds (LDS-DMA, nt) streaming the 2 GiB buffer (the ring GEMM's weight path)
//   mode 3  waves 0-1 as mode 0, waves 2-3 as mode 1 (the two paths at once, separate vmcnt counters)
//   mode 4  waves 0-1 as mode 0, waves 2-3 as mode 2
// with D 1-KiB pieces in flight per wave.  Prints GB/s per CU and chip-wide.
//   hipcc --offload-arch=gfx950 -O3 -o fillbench tools/fillbench.hip && ./fillbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void glds(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds(const_cast<void*>(src),
                                   reinterpret_cast<__attribute__((address_space(3))) void*>(
                                       reinterpret_cast<uintptr_t>(lds)),
                                   16, 0, 0);
}

template <int D>
__device__ __forceinline__ void wait_vm() {
  if constexpr (D >= 32) asm volatile("s_waitcnt vmcnt(31)" ::: "memory");
  else if constexpr (D >= 24) asm volatile("s_waitcnt vmcnt(23)" ::: "memory");
  else if constexpr (D >= 16) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  else if constexpr (D >= 12) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
  else if constexpr (D == 8) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if constexpr (D == 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (D == 2) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// iters: 1-KiB pieces per loading wave.  NW waves per workgroup; in the mixed modes the first half of the waves load
// X, the second half W.  XB: the X buffer's bytes (every workgroup sweeps all of it, so it stays cached).
template <int MODE, int D, int NW>
__global__ void __launch_bounds__(512) fill_kernel(const char* __restrict__ x, const char* __restrict__ w,
                                                   size_t w_per_wg, int iters, size_t xb, unsigned* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool mixed = MODE == 3 || MODE == 4;
  const bool x_role = MODE == 0 || (mixed && wave < NW / 2);
  const bool w_vgpr = MODE == 1 || (MODE == 3 && wave >= NW / 2);
  const bool w_lds = MODE == 2 || (MODE == 4 && wave >= NW / 2);
  const int nw = mixed ? NW / 2 : NW;  // waves per role
  const int rw = mixed ? (wave % (NW / 2)) : wave;
  unsigned acc = 0;
  char* ring = smem + wave * (D * 1024);
  if (x_role) {
    const size_t start = ((size_t)blockIdx.x * NW + wave) * 4096;
    for (int i = 0; i < iters; ++i) {
      const size_t off = (start + (size_t)i * 1024) % xb;  // 1-KiB aligned, inside the X buffer
      glds(x + off + lane * 16, ring + (i % D) * 1024);
      wait_vm<D>();
    }
  } else if (w_vgpr) {
    const char* base = w + (size_t)blockIdx.x * w_per_wg + (size_t)rw * 1024;
    u32x4 v[D];
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = u32x4{0, 0, 0, 0};
    for (int i = 0; i < iters; i += D) {
#pragma unroll
      for (int d = 0; d < D; ++d)
        v[d] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (size_t)(i + d) * nw * 1024 + lane * 16));
#pragma unroll
      for (int d = 0; d < D; ++d) acc ^= v[d].x ^ v[d].w;
    }
  } else if (w_lds) {
    const char* base = w + (size_t)blockIdx.x * w_per_wg + (size_t)rw * 1024;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, 0x7FFFFFFF,
                                                                       0x00020000);
    for (int i = 0; i < iters; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(ring + (i % D) * 1024)),
          16, (uint32_t)((size_t)i * nw * 1024 + lane * 16), 0, 0, 2);
      wait_vm<D>();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  acc ^= *reinterpret_cast<const unsigned*>(smem + threadIdx.x * 4);
  if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads
}

template <int MODE, int D, int NW>
double run(const char* x, const char* w, int iters, size_t xb, unsigned* sink, int reps, double* bytes_out) {
  const int grid = 256;
  const size_t lds = (size_t)NW * D * 1024;
  const int nw = (MODE == 3 || MODE == 4) ? NW / 2 : NW;
  const size_t w_per_wg = (size_t)iters * nw * 1024;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fill_kernel<MODE, D, NW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  fill_kernel<MODE, D, NW><<<grid, NW * 64, lds>>>(x, w, w_per_wg, iters, xb, sink);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) fill_kernel<MODE, D, NW><<<grid, NW * 64, lds>>>(x, w, w_per_wg, iters, xb, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  *bytes_out = (double)grid * NW * iters * 1024;  // every wave moves iters KiB
  return ms / reps;
}

template <int MODE, int D, int NW>
void report(const char* name, const char* x, const char* w, size_t xb, unsigned* sink) {
  static_assert((size_t)NW * D <= 160, "LDS");
  double bytes = 0;
  // the W modes stream 2 GiB per kernel: 256 WG x NW waves x iters KiB
  const int iters = 8192 / NW;
  const double ms = run<MODE, D, NW>(x, w, iters, xb, sink, 10, &bytes);
  const double gbs = bytes / (ms * 1e-3) / 1e9;
  printf("%-44s NW=%d D=%2d X=%zu MiB  %8.3f ms  chip %7.1f GB/s  per CU %6.1f GB/s\n", name, NW, D, xb >> 20, ms, gbs,
         gbs / 256);
  fflush(stdout);
}

int main() {
  char *x = nullptr, *w = nullptr;
  unsigned* sink = nullptr;
  const size_t wbytes = (size_t)2 << 30, xmax = (size_t)8 << 20;
  CHECK(hipMalloc(&x, xmax));
  CHECK(hipMalloc(&w, wbytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(x, 1, xmax));
  CHECK(hipMemset(w, 2, wbytes));
  const size_t x2 = 2u << 20, x8 = xmax;
  report<0, 4, 4>("X  LDS-DMA", x, w, x2, sink);
  report<0, 16, 4>("X  LDS-DMA", x, w, x2, sink);
  report<0, 8, 8>("X  LDS-DMA", x, w, x2, sink);
  report<0, 16, 8>("X  LDS-DMA", x, w, x2, sink);
  report<0, 16, 8>("X  LDS-DMA", x, w, x8, sink);
  report<2, 8, 4>("W  buffer_load lds nt, HBM", x, w, x2, sink);
  report<2, 16, 4>("W  buffer_load lds nt, HBM", x, w, x2, sink);
  report<2, 8, 8>("W  buffer_load lds nt, HBM", x, w, x2, sink);
  report<2, 16, 8>("W  buffer_load lds nt, HBM", x, w, x2, sink);
  report<1, 16, 4>("W  global_load->VGPR nt, HBM", x, w, x2, sink);
  report<4, 16, 4>("X LDS-DMA + W LDS-DMA (half the waves each)", x, w, x2, sink);
  report<4, 8, 8>("X LDS-DMA + W LDS-DMA (half the waves each)", x, w, x2, sink);
  report<4, 16, 8>("X LDS-DMA + W LDS-DMA (half the waves each)", x, w, x2, sink);
  report<4, 20, 8>("X LDS-DMA + W LDS-DMA (half the waves each)", x, w, x2, sink);
  report<4, 16, 8>("X LDS-DMA + W LDS-DMA (half the waves each)", x, w, x8, sink);
  report<3, 16, 8>("X LDS-DMA + W->VGPR (half the waves each)", x, w, x2, sink);
  return 0;
}
