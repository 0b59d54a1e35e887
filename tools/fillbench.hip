// Per-CU fill-rate microbenchmark (round 3): how many bytes per second one CU can bring on chip, by path.
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
  if constexpr (D >= 16) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  else if constexpr (D == 8) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if constexpr (D == 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (D == 2) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// iters: 1-KiB pieces per loading wave
template <int MODE, int D>
__global__ void __launch_bounds__(256) fill_kernel(const char* __restrict__ x, const char* __restrict__ w,
                                                   size_t w_per_wg, int iters, unsigned* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool x_role = MODE == 0 || ((MODE == 3 || MODE == 4) && wave < 2);
  const bool w_vgpr = MODE == 1 || (MODE == 3 && wave >= 2);
  const bool w_lds = MODE == 2 || (MODE == 4 && wave >= 2);
  const int nw = (MODE >= 3) ? 2 : 4;  // waves per role
  const int rw = (MODE >= 3) ? (wave & 1) : wave;
  unsigned acc = 0;
  char* ring = smem + wave * (D * 1024);
  if (x_role) {
    // 2 MiB source: pieces spread over it by workgroup and wave (L2-resident after the first pass)
    const size_t start = ((size_t)blockIdx.x * 4 + wave) * 4096;
    for (int i = 0; i < iters; ++i) {
      const size_t off = (start + (size_t)i * 1024) % (2u << 20);  // 1-KiB aligned, inside the 2 MiB buffer
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

template <int MODE, int D>
double run(const char* x, const char* w, int iters, unsigned* sink, int reps, double* bytes_out) {
  const int grid = 256;
  const size_t lds = 4 * D * 1024;
  const int nw = MODE >= 3 ? 2 : 4;
  const size_t w_per_wg = (size_t)iters * nw * 1024;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fill_kernel<MODE, D>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  fill_kernel<MODE, D><<<grid, 256, lds>>>(x, w, w_per_wg, iters, sink);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) fill_kernel<MODE, D><<<grid, 256, lds>>>(x, w, w_per_wg, iters, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  // bytes per kernel: every wave moves iters KiB
  *bytes_out = (double)grid * 4 * iters * 1024;
  return ms / reps;
}

template <int MODE, int D>
void report(const char* name, const char* x, const char* w, int iters, unsigned* sink) {
  double bytes = 0;
  const double ms = run<MODE, D>(x, w, iters, sink, 10, &bytes);
  const double gbs = bytes / (ms * 1e-3) / 1e9;
  printf("%-44s D=%2d  %8.3f ms  chip %7.1f GB/s  per CU %6.1f GB/s\n", name, D, ms, gbs, gbs / 256);
  fflush(stdout);
}

int main() {
  char *x = nullptr, *w = nullptr;
  unsigned* sink = nullptr;
  const size_t wbytes = (size_t)2 << 30;
  CHECK(hipMalloc(&x, 2u << 20));
  CHECK(hipMalloc(&w, wbytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(x, 1, 2u << 20));
  CHECK(hipMemset(w, 2, wbytes));
  // iters so that the W modes stream 2 GiB / (4 waves) per kernel: 256 WG x 4 waves x iters KiB = 2 GiB -> 2048
  const int iters = 2048;
  report<0, 4>("X  LDS-DMA, L2-resident", x, w, iters, sink);
  report<0, 8>("X  LDS-DMA, L2-resident", x, w, iters, sink);
  report<0, 16>("X  LDS-DMA, L2-resident", x, w, iters, sink);
  report<1, 4>("W  global_load->VGPR nt, HBM", x, w, iters, sink);
  report<1, 8>("W  global_load->VGPR nt, HBM", x, w, iters, sink);
  report<1, 16>("W  global_load->VGPR nt, HBM", x, w, iters, sink);
  report<2, 4>("W  buffer_load lds nt, HBM", x, w, iters, sink);
  report<2, 8>("W  buffer_load lds nt, HBM", x, w, iters, sink);
  report<2, 16>("W  buffer_load lds nt, HBM", x, w, iters, sink);
  report<3, 8>("X LDS-DMA (2 waves) + W->VGPR (2 waves)", x, w, iters, sink);
  report<3, 16>("X LDS-DMA (2 waves) + W->VGPR (2 waves)", x, w, iters, sink);
  report<4, 8>("X LDS-DMA (2 waves) + W LDS-DMA (2 waves)", x, w, iters, sink);
  report<4, 16>("X LDS-DMA (2 waves) + W LDS-DMA (2 waves)", x, w, iters, sink);
  return 0;
}
