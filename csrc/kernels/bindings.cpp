// torch operator registrations for the gfx950 kernels (namespace torch.ops.dsse).
//
// Every op validates device, dtype, contiguity and the shape contract the kernel's grid assumes
// BEFORE launching (a wrong shape on a hand-written kernel would fault the GPU), then launches on
// torch's current HIP stream so the ops compose with hipGraph capture (torch.cuda.CUDAGraph).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <atomic>
#include <string>
#include <tuple>
#include <unordered_map>

#include "api.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define DSSE_CHECK_HIP(expr)                                                        \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    TORCH_CHECK(_e == hipSuccess, "dsse kernel launch failed: ", hipGetErrorString(_e)); \
  } while (0)

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_dtype(const Tensor& t, at::ScalarType st, const char* name) {
  TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
}

// Kernel-configuration overrides: ONE environment variable, DSSE_KERNEL_CFG = "key=value,key=value" (diagnostics and
// the tests that force a kernel path; e.g. "gemm_impl=4,t_cfg=8,t_split=2").  Keys name the selector inputs below
// (gemm_impl, t_cfg, t_split, t_small, s_nw, s_nt, s_rd, s_split, s_ring, ring2, resid_nw, resid_split, qkv_split, w_split, w_rd,
// gemm_nt, gemm_kw, attn_kwv, attn_pd, fused_qkv_attn, trap_fpe); docs/operations.md lists them.  Parsed once per
// thread into a thread-local map: no getenv and no lock on the launch path.  refresh_env() (op dsse::refresh_env, for
// the tools that change it in-process) bumps a generation that makes every thread re-parse on its next lookup.
std::atomic<uint64_t> g_env_gen{1};
std::unordered_map<std::string, int> parse_kernel_cfg() {
  std::unordered_map<std::string, int> m;
  const char* v = std::getenv("DSSE_KERNEL_CFG");
  if (!v) return m;
  std::string s(v), item;
  for (size_t i = 0; i <= s.size(); ++i) {
    if (i == s.size() || s[i] == ',' || s[i] == ' ' || s[i] == ';') {
      const size_t eq = item.find('=');
      if (eq != std::string::npos && eq > 0) m[item.substr(0, eq)] = std::atoi(item.c_str() + eq + 1);
      item.clear();
    } else {
      item += (char)std::tolower((unsigned char)s[i]);
    }
  }
  return m;
}
int env_int(const char* key, int dflt) {
  thread_local std::unordered_map<std::string, int> cfg;
  thread_local uint64_t gen = 0;
  const uint64_t g = g_env_gen.load(std::memory_order_acquire);
  if (gen != g) {
    cfg = parse_kernel_cfg();
    gen = g;
  }
  auto it = cfg.find(key);
  return it == cfg.end() ? dflt : it->second;
}
// trap_fpe=1: print the native stack of a host SIGFPE (integer division by zero) before dying.
void fpe_handler(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "[dsse] SIGFPE, native stack:\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
const bool g_fpe_trap = [] {
  if (parse_kernel_cfg().count("trap_fpe") && parse_kernel_cfg()["trap_fpe"] == 1) signal(SIGFPE, fpe_handler);
  return true;
}();

void refresh_env() { g_env_gen.fetch_add(1, std::memory_order_acq_rel); }



// Tile selection for the skinny GEMM.  NT = output tiles per wave, KW = waves splitting K.
// Defaults come from the gfx950 sweep in tools/tune_gemm.py; DSSE_KERNEL_CFG gemm_nt / gemm_kw override.
void pick_tiles(int M, int N, int K, int mode, int& mt, int& nt, int& kw) {
  mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  nt = 1;
  const int chunks = K / 128;
  kw = chunks >= 32 ? 8 : 4;
  const int e_nt = env_int("gemm_nt", 0), e_kw = env_int("gemm_kw", 0);
  if (e_nt) nt = e_nt;
  if (e_kw) kw = e_kw;
  if (mt == 4 && nt == 2 && kw == 8) kw = 4;  // spill guard (see gemm_skinny.hip)
  if (N % (16 * nt) != 0) nt = 1;
  (void)mode;
}

// X-streaming kernel configuration (gemm_stream.hip).  DSSE_KERNEL_CFG overrides: s_nt, s_nw, s_rd, s_split.
struct SCfg {
  int mt, nt, nw, rd, S;
  bool ok;
  int ring_nw = 0;  // waves per workgroup of the LDS-DMA ring form (0 = stream_launch's default rule)
  bool ring_only = false;  // only the ring kernel's K contract holds (K % 128, not K % 512)
};
// 64 < M <= 256: one workgroup holds all rows (mt 8 / 16, X slices of 256 / 128 columns); M > 256: row
// blocks of 64 (mt 4, L2-shared weights).
SCfg pick_stream(int M, int N, int K, int mode = -1) {
  SCfg c{};
  c.mt = M <= 16 ? 1 : (M <= 32 ? 2 : (M <= 64 ? 4 : (M <= 128 ? 8 : (M <= 256 ? 16 : 4))));
  c.nt = M > 256 ? 1 : env_int("s_nt", 1);  // row blocks (M > 256) are instantiated for nt = 1
  // 8 waves per workgroup when that still gives ~one workgroup per CU without split-K (gate_up,
  // LM head), else 4 (narrow O / down / QKV: more, shorter workgroups; measured, profiles/gemm_stream_r1.md)
  c.nw = env_int("s_nw", (N / (16 * c.nt)) / 8 >= 192 ? 8 : 4);
  if (c.nt == 2 && c.mt <= 4) c.nw = 8;  // instantiated (nt, nw): (1, 8), (2, 8), (1, 4) — gemm_stream.hip
  if (c.nt == 2 && c.mt >= 8) c.nw = 4;   // mt 8 / 16: (1, 8), (1, 4), (2, 4)
  // 7 waves when that puts exactly one workgroup on each CU where 8 leaves CUs idle (gate_up at TP = 1:
  // 1792 tile groups -> 256 instead of 224 workgroups; 51.1 vs 56.0 us at M = 64, profiles/gemm_nw_r1.md)
  const int tg1 = N / 16;
  if (env_int("s_nw", 0) == 0 && c.mt == 4 && c.nt == 1 && M <= 64 && c.nw == 8 && tg1 % 8 == 0 &&
      tg1 / 8 < 256 && tg1 % 7 == 0 && tg1 / 7 <= 256)
    c.nw = 7;
  const bool odd_nw = c.mt == 4 && c.nt == 1 && M <= 64 && c.nw >= 2 && c.nw <= 7;  // (4, 1, 2..7, rd 1)
  if (c.nw != 4 && !odd_nw) c.nw = 8;
  if (N % (16 * c.nt) != 0 || (N / (16 * c.nt)) % c.nw != 0) c.nt = 1;
  if ((N / 16) % c.nw != 0) c.nw = 4;
  c.rd = env_int("s_rd", 1);
  if (c.nt == 2 || c.rd != 2 || M > 64 || (c.nw != 4 && c.nw != 8)) c.rd = 1;
  if (c.mt == 8) c.rd = 2;
  if (c.mt == 16) c.rd = c.nt == 2 ? 2 : 4;  // ring of 4 chunks (2 with two tiles per wave: VGPR budget)
  int cps = c.mt <= 4 ? 4 : (c.mt == 8 ? 2 : 1);  // gemm_stream.hip stream_cps
  c.ok = K % (128 * cps) == 0 && N % (16 * c.nt) == 0 && (N / (16 * c.nt)) % c.nw == 0;
  // 17-64 rows with K a multiple of 128 but not of 512 (a TP = 8 rank's down projection, K = 1792): the LDS-DMA ring
  // kernel (stream_launch) only needs K % (128 S) == 0 -- before round 6 these fell to a 128-row tiled tile
  if (!c.ok && M > 16 && M <= 64 && c.nt == 1 && K % 128 == 0 && (N / 16) % c.nw == 0 && env_int("s_ring", 1) > 0) {
    c.ok = true;
    c.ring_only = true;
    cps = 1;
  }
  if (!c.ok) return c;
  const int wgs = N / (16 * c.nt) / c.nw * (M > 16 * c.mt ? (M + 63) / 64 : 1), slices = K / (128 * cps);
  int S = env_int("s_split", 0);
  if (S <= 0 || slices % S != 0) {
    // smallest split that gives ~one workgroup per CU (256 CUs), never more than 1.25x that
    S = 1;
    for (int d = 1; d <= slices; ++d) {
      if (slices % d) continue;
      if (wgs * d > 320) break;
      S = d;
      if (wgs * d >= 192) break;
    }
  }
  c.S = S;
  return c;
}

// gemm_stream launch, or its LDS-DMA ring form (gemm_ring_kernel) where that applies: 33-64 rows, one 16-column
// tile per wave: 4 slots with 4 waves per workgroup, 3 slots with 7 / 8 (the 7-8-wave shapes; LDS; gate_up on 7
// waves = 256 workgroups: 64-stream step 4.38 vs 4.50 ms with 8).  s_ring=0 (DSSE_KERNEL_CFG) turns it off.  Measured on MI355X, 64-stream step: 4.51 / 4.52 ms vs 4.61 / 4.63 on gemm_stream; 5 slots at 4
// waves 4.55 / 4.66 (gate_up 45.8 -> 43.5 us, LM head 52.5 -> 48.3; profiles/r2/ring_*.log).
// Ring GEMM variant: ring2 (DSSE_KERNEL_CFG) unset = the decoupled-look-ahead kernel (gemm_ring2) for 65-128 rows only
// (128-stream step 6.19-6.22 vs 6.32-6.34 ms; at 33-64 rows 4.44 vs 4.40 ms: profiles/r3/ring2_ab.log,
// step_p64_r{0,2}.md), 1 = every shape it is instantiated for, 0 = never.
int ring2_for(int M) {
  const int v = env_int("ring2", -1);
  return v == 0 ? 0 : (v == 1 ? 1 : (M > 64 ? 1 : 0));
}

hipError_t stream_launch(int mode, const SCfg& c, int S, int partial_only, const void* X, int M, const void* W, int K,
                         int N, const dsse::GemmEpi* ep, float* part) {
  const int ring = env_int("s_ring", 1);
  // 17-64 rows (32-stream step 3.99 vs 4.04 ms; at 9-16 rows the ring measured 4.02 vs 3.99: gemm_stream kept)
  const bool ring_rows = (c.mt == 4 && M > 32 && M <= 64) || (c.mt == 2 && M > 16 && M <= 32) ||
                         (c.mt == 8 && M > 64 && M <= 128 && c.nw == 4);
  // partial_only 2 = split K combined in the launch: only the 17-64-row ring kernel has that form (else the caller
  // falls back to slabs + splitk_reduce)
  if (partial_only == 2 && !(ring > 0 && ring_rows && M <= 64 && c.nt == 1 && K % (128 * S) == 0 && S > 1))
    return hipErrorNotSupported;
  if (ring > 0 && ring_rows && c.nt == 1 && K % (128 * S) == 0) {
    int nw = c.nw >= 7 ? c.nw : 4;
    if (c.ring_nw > 0 && (N / 16) % c.ring_nw == 0 && M <= 64)
      return dsse_gemm_ring(mode, c.ring_nw, S, partial_only, ring2_for(M), X, K, M, W, K, N, ep, part, cur_stream());
    // QKV at 33-64 rows: 3 waves (384 tiles -> 128 x S 2 = 256 workgroups instead of 192; 64-stream step
    // 4.38-4.40 vs 4.41-4.42 ms, profiles/r2/qkv_ring3_ab.log)
    if (mode == dsse::kQkvRope && c.mt == 4 && (N / 16) % 3 == 0) nw = 3;
    if ((N / 16) % nw == 0)
      return dsse_gemm_ring(mode, nw, S, partial_only, ring2_for(M), X, K, M, W, K, N, ep, part, cur_stream());
  }
  return dsse_gemm_stream(mode, c.mt, c.nt, c.nw, c.rd, S, partial_only, X, K, M, W, K, N, ep, part, cur_stream());
}

// Wide-batch kernel configuration (gemm_wide.hip, 32x32x16 MFMAs, 128 columns per workgroup).  Env
// overrides (DSSE_KERNEL_CFG): w_split, w_rd.
struct WCfg {
  int mb, rd, S;
  bool ok;
};
WCfg pick_wide(int M, int N, int K) {
  WCfg c{};
  c.mb = M <= 128 ? 4 : 8;
  const int cps = c.mb == 8 ? 1 : 2;
  c.rd = env_int("w_rd", c.mb == 8 ? 2 : 1);
  if (c.mb == 8 && c.rd != 3) c.rd = 2;
  if (c.mb == 4 && c.rd != 2) c.rd = 1;
  c.ok = M <= 256 && N % 128 == 0 && K % (128 * cps) == 0;
  if (!c.ok) return c;
  const int wgs = N / 128, slices = K / (128 * cps);
  int S = env_int("w_split", 0);
  if (S <= 0 || slices % S != 0) {
    S = 1;
    for (int d = 1; d <= slices; ++d) {
      if (slices % d) continue;
      if (wgs * d > 320) break;
      S = d;
      if (wgs * d >= 192) break;
    }
  }
  c.S = S;
  return c;
}

// cfg 8 / 9 / 10 = the pipelined 256 / 192 / 128 x 256 kernel of gemm_pipe.hip; 0, 1, 5 = gemm_tiled.hip's
// configurations.  partial_only 2 (gemm_pipe only) = split-K slices combined inside the launch (run_pipe_fix).
hipError_t tiled_call(int mode, int cfg, int S, int partial_only, const void* X, int ldx, int M, const void* W, int K,
                      int N, const dsse::GemmEpi* ep, float* part) {
  if (cfg == 8 || cfg == 9 || cfg == 10)
    return dsse_gemm_pipe(mode, cfg == 10 ? 128 : cfg == 9 ? 192 : 256, S, partial_only, X, ldx, M, W, K, N, ep, part, cur_stream());
  return dsse_gemm_tiled(mode, cfg, S, partial_only, X, ldx, M, W, K, N, ep, part, cur_stream());
}

// In-launch split-K fix-up state (gemm_pipe.hip FIX): per device, 2 * kFixTiles arrival counters + a timeout word,
// zeroed once; every launch leaves the counters it used at zero (each tile's last arriver resets its pair), and
// launches on one stream never overlap.  (Launches of one process on two streams at once would share them: the
// engine issues every GEMM on its one compute stream.)
using dsse::kFixTiles;
#ifndef DSSE_PIPE_STAMPS
#define DSSE_PIPE_STAMPS 0
#endif
constexpr int kStampWgs = 8192;  // stamps build: [workgroup][8] u64 after the counters
at::Tensor& fix_state(const at::Device& dev) {
  static std::unordered_map<int, at::Tensor> per_dev;
  auto it = per_dev.find(dev.index());
  if (it == per_dev.end()) {
    const int64_t n = dsse::kStampOff + (DSSE_PIPE_STAMPS ? kStampWgs * 16 : 0);
    it = per_dev.emplace(dev.index(), at::zeros({n}, at::TensorOptions().dtype(at::kInt).device(dev))).first;
  }
  return it->second;
}
int* fix_counters(const at::Device& dev) { return fix_state(dev).data_ptr<int>(); }

constexpr int kMaxDecodeM = 512;  // gemm_stream: one workgroup per tile group up to 256 rows, row blocks above

// Tiled LDS-DMA GEMMs (gemm_tiled.hip, gemm_pipe.hip; prefill and wide batches).  DSSE_KERNEL_CFG overrides: t_cfg
// (0 = 256x128, 1 = 128x128, 5 = 128x256, 8 / 9 / 10 = the 256 / 192 / 128 x 256 gemm_pipe tile), t_split, t_fix
// (1 = split-K slices combined inside the launch, gemm_pipe only), t_model (0 = the round-5 row-range table).
struct TCfg {
  int cfg, S;
  bool ok;
  bool fix = false;    // S > 1 combined inside the launch (gemm_pipe FIX); else S > 1 = fp32 slabs
  double est_us = 0;   // the cost model's estimate (pipe_plan), 0 for the table's choices
};

// Cost model of one gemm_pipe launch (round 6, profiles/r6/gemm_model_r6.md).  A workgroup is bound by its LDS
// fill (X rows + weight rows through LDS-DMA: ~44 GB/s per CU when the L2 and HBM streams mix -- the 8-wave,
// 32 KiB-in-flight fillbench tops out there too, profiles/r6/fillbench_r6.log) or by its MFMA issue (~5.0 TFLOP/s
// per CU, the kernel's rate at 8192 rows), plus ~3.3 us of pipeline fill and epilogue; one 128 KiB workgroup per CU,
// so the grid runs in rounds of 256, a partial last round at 0.67 + 0.33 x its fill of a full one's time.  Split K
// costs the fp32 partial tiles: combined in the launch (FIX) ~7 us of store / release / wait plus the last arriver
// reading S - 1 slots at ~26 GB/s (the stamps of profiles/r6/pipe_fix_stamps_r6.log), or left as slabs for the
// next kernel (the norm or attention consumer, else splitk_reduce) that reads S x M x N x 4 bytes at ~4.5 TB/s
// after ~5.7 us.  Constants least-squares fitted to 238 measured launches at 192-1024 rows (12 % rms error).
double pipe_est_us(int M, int N, int K, int bm, int S, bool fix, int out_bytes = 0) {
  // kFixSync: the fit gave 7.06 us over isolated launches; 12 after the TP = 8 rank's prefill, where the fix-up GEMMs
  // (gate_up at 2048-row chunks, qkv at 8192 rows, model ties with slab forms) run beside the side stream's
  // collectives and lost 2 ms per 8k prompt to the slab forms (25.2 vs 23.3 ms, profiles/r6/tp8_fix_ab_r6.log); 12
  // keeps the fix-up where isolated launches measured it ahead (gate_up at 576 rows)
  constexpr double kFill = 43.76e3, kMfma = 5.006e6, kT0 = 3.35, kPartial = 0.666, kSlotRead = 26.48e3,
                   kFixSync = 12.0, kNext = 5.68, kHbm = 4.458e6, kCUs = 256;
  const int nbm = (M + bm - 1) / bm, rows = std::min(bm, M);
  const double Kr = (double)K / S;
  const long wgs = (long)nbm * (N / 256) * S;
  const long full = wgs / (long)kCUs, rem = wgs - full * (long)kCUs;
  const double t_wg = kT0 + std::max((double)(rows + 256) * Kr * 2 / kFill, 2.0 * bm * 256 * Kr / kMfma);
  double t = full * t_wg + (rem ? t_wg * (kPartial + (1 - kPartial) * rem / kCUs) : 0.0);
  if (S > 1) {
    const double slot = (double)bm * 256 * 4;
    t += fix ? kFixSync + (S - 1) * slot / kSlotRead : kNext + ((double)S * M * N * 4 + (double)M * N * out_bytes) / kHbm;
  }
  return t;
}

// Best gemm_pipe configuration by the model: tile 256 / 192 / 128 rows x split 1-16, slices combined in the launch
// (fix) or left as fp32 slabs -- for the caller's next kernel when `slab_consumer` (norm, attention), else for
// splitk_reduce (which also writes the bf16 output: counted).
TCfg pipe_plan(int M, int N, int K, bool slab_consumer) {
  TCfg best{};
  best.ok = false;
  const bool no_fix = env_int("t_fix", -1) == 0;  // t_fix=0 (DSSE_KERNEL_CFG): slabs only, for A/Bs
  for (int bm : {256, 192, 128}) {
    const long tiles = (long)((M + bm - 1) / bm) * (N / 256);
    for (int S = 1; S <= 16; S *= 2) {
      if (K % (128 * S) != 0) break;
      for (int fix = 0; fix < 2; ++fix) {
        if (S == 1 && fix) continue;
        if (fix && no_fix) continue;
        if (fix && (tiles > dsse::kFixTiles || (double)tiles * (S - 1) * bm * 256 * 4 > (1u << 30))) continue;
        const double t = pipe_est_us(M, N, K, bm, S, fix, slab_consumer ? 0 : 2);
        if (!best.ok || t < best.est_us * 0.98) {  // ties: the simpler (earlier) form
          best.ok = true;
          best.est_us = t;
          best.cfg = bm == 256 ? 8 : bm == 192 ? 9 : 10;
          best.S = S;
          best.fix = fix;
        }
      }
    }
  }
  return best;
}

constexpr int kModelMinM = 256;  // above this many rows every N % 256 == 0 projection is planned by pipe_plan

TCfg pick_tiled(int M, int N, int K, bool slab_consumer = false) {
  TCfg c{};
  int cfg = env_int("t_cfg", -1);
  const bool forced = cfg == 0 || cfg == 1 || cfg == 5 || cfg == 8 || cfg == 9 || cfg == 10;
  if (!forced && env_int("t_model", 1) && N % 256 == 0 && K % 128 == 0 && M > kModelMinM) {
    c = pipe_plan(M, N, K, slab_consumer);
    if (c.ok) return c;
  }
  if (!forced) {
    // up to kModelMinM rows (and N % 256 != 0): the decode buckets' measured table
    // round 5 (profiles/r5/gemm_pipe_r5.md): the 256x256 tile of gemm_pipe.hip (cfg 8: 8 waves, every LDS-DMA
    // half-tile five phases ahead of its wait) once it yields >= ~160 workgroups -- 1.35-1.40 PFLOP/s at 8192 rows,
    // +5-7 % over round 4's phased cfg 4; below that the 256x128 tile (3-stage ring) fills more CUs; 128x128 for tiny M
    const int big_tiles = ((M + 255) / 256) * (N / 256);
    cfg = (N % 256 == 0 && big_tiles >= 160) ? 8 : (M > 128 ? 0 : 1);
    // narrow projections of the wide decode buckets (N <= 8192, 128 < M <= 512: qkv / o / down at 192-256
    // streams): 128x128 tiles (4 waves) split 2-4 ways -- 256-stream step 9.88 vs 9.93 ms with 256x128
    // (same box, alternating; profiles/experiments_r2.md).
    // round 3 (profiles/r3/decode_bucket_gemm.md): in the 129-192-row bucket qkv (N 6144) and down (K 14336) on
    // 256x128 -- alone 27 vs 30 us and 42 vs 50 us, 192-stream step 8.30 vs 8.43 ms; at 193-256 rows the same
    // change measured 9.81 vs 9.71 ms per step (twice the split-K slabs for the consuming norm / attention),
    // so 128x128 stays there
    if (N <= 8192 && M > 128 && M <= 256) cfg = (M <= 192 && !(N <= 4096 && K <= 4096)) ? 0 : 1;
    // round 4 (profiles/r4/gemm_wide_r4.md): the 128x256 tile (cfg 5: twice the weight bytes in flight per CU)
    // for the weight-heavy 129-256-row shapes: gate_up 68.1 vs 73.9 us (256 rows) / 64.4 vs 66.2 (192), down
    // (K 14336) 42.9 vs 50.5 / 41.0 vs 42.0
    if (M > 128 && M <= 256 && (N > 8192 || K > 8192)) cfg = 5;
    // round 5 (profiles/r5/pipe128_r5.log): the pipe schedule on the 128-row tile (cfg 10) for the 256-row
    // bucket's qkv (N 6144) and down (K 14336): qkv 30.6 vs 33.1 us, down + norm 48.4 vs 52.1; 256-stream step
    // 9.45-9.47 vs 9.54-9.55 ms alternating (small_ab_r5.log).  129-192 rows keep the tiled kernels
    // (small192_ab_r5.log).  gate_up and o keep cfg 5 / cfg 1
    if (M > 192 && M <= 256 && N % 256 == 0 && N <= 8192 && (K > 8192 || N > 4096) && env_int("t_small", 1))
      cfg = 10;
    // t_model=0 (the round-5 table above 256 rows, for A/Bs): 257-512 rows cfg 8 / 9 / 0, 513-1024 narrow cfg 1
    if (N <= 8192 && M > 256 && M <= 512) cfg = (K > 8192 || N > 4096) ? 8 : 0;
    if (N <= 4096 && M > 512 && M <= 1024) cfg = 1;
    if (cfg == 8 && M > 256 && M <= 384) cfg = 9;
  }
  constexpr int min_wgs = 160;  // split K until this many workgroups (table choices, M <= 512)
  // tile shapes by cfg (gemm_tiled.hip launch_t_mode: 0, 1, 5; gemm_pipe.hip: 8, 9, 10)
  const int BM = cfg == 1 || cfg == 5 || cfg == 10 ? 128 : cfg == 9 ? 192 : 256, BN = cfg == 0 || cfg == 1 ? 128 : 256;
  c.cfg = cfg;
  c.S = 1;
  const bool pipe = cfg >= 8;
  c.ok = N % BN == 0 && K % (pipe ? 128 : 64) == 0;
  if (!c.ok) return c;
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  int S = env_int("t_split", 0);
  const int kq = pipe ? 128 : 64;  // K granule of a slice (gemm_pipe: >= 2 steps of 64)
  if (S <= 0 || K % (kq * S) != 0) {
    S = 1;  // split K only for the few-tile wide-decode shapes (slabs cost M x N x 4 B each)
    while (M <= kMaxDecodeM && tiles * S < min_wgs && K % (kq * S * 2) == 0 && K / (S * 2) >= 512) S *= 2;
  }
  c.S = S;
  // t_fix=1: combine the slices inside the launch (gemm_pipe only, and only when the tile count fits the counters)
  c.fix = pipe && S > 1 && env_int("t_fix", 0) == 1 && (long)((M + BM - 1) / BM) * (N / 256) <= dsse::kFixTiles;
  if (pipe) c.est_us = pipe_est_us(M, N, K, BM, S, c.fix);
  return c;
}

// One tiled / pipe launch for a plain epilogue (no slabs left for a consumer): S > 1 is combined in the launch (fix)
// or by launch_splitk_reduce.
void run_tiled(int mode, const TCfg& c, const Tensor& x, const Tensor& w, int M, int N, int K, dsse::GemmEpi& ep) {
  at::Tensor part;
  if (c.S > 1 && c.fix) {
    const int bm = c.cfg == 10 ? 128 : c.cfg == 9 ? 192 : 256;
    part = at::empty({(int64_t)dsse_gemm_pipe_fix_floats(bm, c.S, M, N)}, x.options().dtype(at::kFloat));
    ep.fix_cnt = fix_counters(x.device());
    DSSE_CHECK_HIP(tiled_call(mode, c.cfg, c.S, 2, x.data_ptr(), K, M, w.data_ptr(), K, N, &ep, part.data_ptr<float>()));
    return;
  }
  if (c.S > 1) part = at::empty({(int64_t)c.S * M * N}, x.options().dtype(at::kFloat));
  DSSE_CHECK_HIP(tiled_call(mode, c.cfg, c.S, 0, x.data_ptr(), K, M, w.data_ptr(), K, N, &ep,
                            c.S > 1 ? part.data_ptr<float>() : nullptr));
}

// 0 = register-streaming (gemm_skinny.hip; tiny batches, X re-reads are cheap), 2 = X streamed through LDS
// slices (gemm_stream.hip), 3 = gemm_wide.hip (32x32 MFMAs), 4 = gemm_tiled.hip (register-blocked, LDS-DMA).
// gemm_impl (DSSE_KERNEL_CFG) forces one (1, the removed whole-slice X-in-LDS kernel, maps to the fallback).
int gemm_impl(int M, int N, int K) {
  const int impl = env_int("gemm_impl", -1);
  if (M > 64) {
    // every branch returns a kernel whose shape contract holds (or -1): prefill calls arrive with any M and
    // tensor-parallel shard shapes
    // 65-128 rows, narrow N (4-wave stream shapes: qkv / o / down): the ring kernel with 8 row tiles, 3 slots;
    // 128-stream step 6.19 / 6.23 vs 6.36 / 6.37 ms on gemm_wide (profiles/r2/ring128_ab.log)
    if (impl < 0 && M <= 128) {
      const SCfg sc = pick_stream(M, N, K);
      if (sc.ok && sc.mt == 8 && sc.nt == 1 && sc.nw == 4) return 2;
    }
    const bool tiled_ok = pick_tiled(M, N, K).ok;
    if (tiled_ok && (M > kMaxDecodeM || impl == 4 || (impl < 0 && M > 128))) return 4;
    if (M > kMaxDecodeM) return -1;  // the decode kernels stop at kMaxDecodeM rows
    const bool wide_ok = pick_wide(M, N, K).ok, stream_ok = pick_stream(M, N, K).ok;
    if (impl == 3 && wide_ok) return 3;
    if (impl == 2 && stream_ok) return 2;
    if (wide_ok && M > 64) return 3;  // 3 = gemm_wide (32x32 MFMAs, M <= 256)
    if (stream_ok) return 2;
    if (wide_ok) return 3;
    return tiled_ok ? 4 : -1;
  }
  // M <= 64: 0 = register-streaming skinny kernel (tiny batches), 2 = gemm_stream; a shape outside the
  // stream kernel's contract goes to gemm_tiled, else the skinny kernel (no shape contract beyond N % 16)
  const int fallback = pick_tiled(M, N, K).ok ? 4 : 0;
  if (impl >= 0) {
    if (impl == 4) return fallback;
    if (impl == 3 && !pick_wide(M, N, K).ok) return pick_stream(M, N, K).ok ? 2 : fallback;
    if (impl == 2 && !pick_stream(M, N, K).ok) return fallback;
    return impl == 1 ? fallback : impl;
  }
  if (M <= 8) return 0;
  if (M <= 16 && N < 16384) return 0;
  return pick_stream(M, N, K).ok ? 2 : fallback;
}

void run_gemm(int mode, const Tensor& x, const Tensor& w, dsse::GemmEpi& ep) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(w, at::kBFloat16, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2, "x and w must be 2-D");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K, "K mismatch: x ", K, " vs w ", w.size(1));
  TORCH_CHECK(M >= 1, "GEMM needs M >= 1, got ", M);
  TORCH_CHECK(K % 128 == 0, "K must be a multiple of 128, got ", K);
  TORCH_CHECK(N % 16 == 0, "N must be a multiple of 16, got ", N);
  TORCH_CHECK((int64_t)N * K * 2 < (1LL << 31), "weight larger than 2 GiB: the decode GEMMs address it with 32-bit offsets");
  const int impl = gemm_impl(M, N, K);
  TORCH_CHECK(impl >= 0, "no GEMM kernel for M=", M, " N=", N, " K=", K, " (tiled path needs N % 128, K % 64)");
  if (impl == 4) {
    run_tiled(mode, pick_tiled(M, N, K), x, w, M, N, K, ep);
    return;
  }
  TORCH_CHECK(M <= 64 || impl >= 2, "M > 64 needs the X-streaming kernel shape contract (K % 512, N % 64)");
  if (impl == 3) {
    const WCfg c = pick_wide(M, N, K);
    at::Tensor part;
    if (c.S > 1) part = at::empty({(int64_t)c.S * M * N}, x.options().dtype(at::kFloat));
    DSSE_CHECK_HIP(dsse_gemm_wide(mode, c.mb, c.rd, c.S, 0, x.data_ptr(), K, M, w.data_ptr(), K, N, &ep,
                                  c.S > 1 ? part.data_ptr<float>() : nullptr, cur_stream()));
    return;
  }
  if (impl == 2) {
    const SCfg c = pick_stream(M, N, K, mode);
    // SiLU·mul split over K (a TP rank's gate_up at 17-64 rows): s_fix=1 (DSSE_KERNEL_CFG) combines the slices
    // inside the ring kernel instead of slabs + a splitk_reduce launch.  Off by default: on a TP = 8 rank's 64-stream
    // step the fix-up tail costs more than the launch it saves (gate_up 19-20 us vs 10 + 5 us; step 2.27 vs 2.08 ms,
    // profiles/r6/tp8_rank_r6.md)
    if (c.S > 1 && mode == dsse::kSiluMul && M <= 64 && env_int("s_fix", 0)) {
      at::Tensor ws = at::empty({(int64_t)dsse_gemm_ring_fix_floats(1, c.S, M, N)}, x.options().dtype(at::kFloat));
      ep.fix_cnt = fix_counters(x.device());
      const hipError_t e = stream_launch(mode, c, c.S, 2, x.data_ptr(), M, w.data_ptr(), K, N, &ep,
                                         ws.data_ptr<float>());
      if (e == hipSuccess) return;
      TORCH_CHECK(e == hipErrorNotSupported, "dsse kernel launch failed: ", hipGetErrorString(e));
      (void)hipGetLastError();
    }
    at::Tensor part;
    if (c.S > 1) part = at::empty({(int64_t)c.S * M * N}, x.options().dtype(at::kFloat));
    DSSE_CHECK_HIP(stream_launch(mode, c, c.S, 0, x.data_ptr(), M, w.data_ptr(), K, N, &ep,
                                 c.S > 1 ? part.data_ptr<float>() : nullptr));
    return;
  }
  int mt, nt, kw;
  pick_tiles(M, N, K, mode, mt, nt, kw);
  DSSE_CHECK_HIP(dsse_skinny_gemm(mode, mt, nt, kw, x.data_ptr(), K, M, w.data_ptr(), K, N, &ep,
                                  cur_stream()));
}

void gemm_out(const Tensor& x, const Tensor& w, Tensor& out) {
  check_gpu(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == x.size(0) && out.size(1) == w.size(0),
              "out must be [M, N]");
  dsse::GemmEpi ep{};
  ep.out = out.data_ptr();
  ep.ldo = (int)out.size(1);
  int mode;
  if (out.scalar_type() == at::kBFloat16) mode = dsse::kStoreBf16;
  else if (out.scalar_type() == at::kFloat) mode = dsse::kStoreF32;
  else TORCH_CHECK(false, "out must be bf16 or fp32");
  run_gemm(mode, x, w, ep);
}

void gemm_resid(const Tensor& x, const Tensor& w, Tensor& resid) {
  check_gpu(resid, "resid");
  check_dtype(resid, at::kFloat, "resid");
  TORCH_CHECK(resid.dim() == 2 && resid.size(0) == x.size(0) && resid.size(1) == w.size(0),
              "resid must be [M, N]");
  dsse::GemmEpi ep{};
  ep.resid = resid.data_ptr<float>();
  ep.ldr = (int)resid.size(1);
  run_gemm(dsse::kResidAdd, x, w, ep);
}

// Residual projection whose split-K reduction is left to the consuming RMSNorm (rmsnorm with `part`).
// Returns S > 0 when fp32 partial slabs [S, M, N] were written to `part` (resid untouched), or 0 when
// the product was already added into `resid` (single K-slice or register-streaming kernel).
int64_t gemm_resid_split(const Tensor& x, const Tensor& w, Tensor& resid, Tensor& part) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_gpu(part, "part");
  check_dtype(part, at::kFloat, "part");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  const bool shape_ok = M >= 1 && K % 128 == 0 && N % 16 == 0 && w.size(1) == K;
  const int impl = shape_ok ? gemm_impl(M, N, K) : 0;
  if (impl == 4) {
    const TCfg c = pick_tiled(M, N, K, true);
    if (c.S > 1 && !c.fix && part.numel() >= (int64_t)c.S * M * N) {
      check_dtype(x, at::kBFloat16, "x");
      check_dtype(w, at::kBFloat16, "w");
      dsse::GemmEpi ep{};
      DSSE_CHECK_HIP(tiled_call(dsse::kResidAdd, c.cfg, c.S, 1, x.data_ptr(), K, M, w.data_ptr(), K, N, &ep,
                                part.data_ptr<float>()));
      return c.S;
    }
  } else if (impl == 3) {
    const WCfg c = pick_wide(M, N, K);
    if (c.S > 1 && part.numel() >= (int64_t)c.S * M * N) {
      check_dtype(x, at::kBFloat16, "x");
      check_dtype(w, at::kBFloat16, "w");
      dsse::GemmEpi ep{};
      DSSE_CHECK_HIP(dsse_gemm_wide(dsse::kResidAdd, c.mb, c.rd, c.S, 1, x.data_ptr(), K, M, w.data_ptr(), K, N, &ep,
                                    part.data_ptr<float>(), cur_stream()));
      return c.S;
    }
  } else if (impl == 2) {
    SCfg c = pick_stream(M, N, K);
    // 17-64 rows on the ring: resid_nw / resid_split (DSSE_KERNEL_CFG) = waves per workgroup and K split of the O / down
    // projections (more K slices: fewer X bytes per workgroup, more slab bytes for the norm)
    const int rnw = env_int("resid_nw", 0), rsp = env_int("resid_split", 0);
    if (M > 32 && M <= 64 && rnw > 0 && rsp > 1 && (N / 16) % rnw == 0 && K % (128 * rsp) == 0) {
      c.ring_nw = rnw;
      c.S = rsp;
    }
    if (c.S > 1 && part.numel() >= (int64_t)c.S * M * N) {
      check_dtype(x, at::kBFloat16, "x");
      check_dtype(w, at::kBFloat16, "w");
      dsse::GemmEpi ep{};
      DSSE_CHECK_HIP(stream_launch(dsse::kResidAdd, c, c.S, 1, x.data_ptr(), M, w.data_ptr(), K, N, &ep,
                                   part.data_ptr<float>()));
      return c.S;
    }
  }
  gemm_resid(x, w, resid);
  return 0;
}

// bf16 projection whose split-K reduction is left to the consumer (the TP decode step's IPC all-reduce, ar_rmsnorm
// with `part`): returns S > 0 when fp32 slabs [S, M, N] went to `part` (out untouched), else 0 after writing out.
int64_t gemm_out_split(const Tensor& x, const Tensor& w, Tensor& out, Tensor& part) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_gpu(part, "part");
  check_dtype(part, at::kFloat, "part");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  const bool shape_ok = M >= 1 && K % 128 == 0 && N % 16 == 0 && w.size(1) == K;
  const int impl = shape_ok ? gemm_impl(M, N, K) : 0;
  dsse::GemmEpi ep{};
  if (impl == 2) {
    const SCfg c = pick_stream(M, N, K);
    if (c.S > 1 && part.numel() >= (int64_t)c.S * M * N) {
      check_dtype(x, at::kBFloat16, "x");
      check_dtype(w, at::kBFloat16, "w");
      DSSE_CHECK_HIP(stream_launch(dsse::kStoreBf16, c, c.S, 1, x.data_ptr(), M, w.data_ptr(), K, N, &ep,
                                   part.data_ptr<float>()));
      return c.S;
    }
  } else if (impl == 4) {
    const TCfg c = pick_tiled(M, N, K, true);
    if (c.S > 1 && !c.fix && part.numel() >= (int64_t)c.S * M * N) {
      check_dtype(x, at::kBFloat16, "x");
      check_dtype(w, at::kBFloat16, "w");
      DSSE_CHECK_HIP(tiled_call(dsse::kStoreBf16, c.cfg, c.S, 1, x.data_ptr(), K, M, w.data_ptr(), K, N, &ep,
                                part.data_ptr<float>()));
      return c.S;
    }
  }
  gemm_out(x, w, out);
  return 0;
}

void gemm_silu(const Tensor& x, const Tensor& w, Tensor& out) {
  check_gpu(out, "out");
  check_dtype(out, at::kBFloat16, "out");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == x.size(0) && out.size(1) * 2 == w.size(0),
              "out must be [M, N/2]");
  dsse::GemmEpi ep{};
  ep.out = out.data_ptr();
  ep.ldo = (int)out.size(1);
  run_gemm(dsse::kSiluMul, x, w, ep);
}

void gemm_qkv_rope(const Tensor& x, const Tensor& w, const Tensor& positions, const Tensor& slots,
                   const Tensor& rope, Tensor& q_out, Tensor& k_cache, Tensor& v_cache, int64_t nh,
                   int64_t nkv) {
  for (auto* t : {&positions, &slots, &rope}) check_gpu(*t, "metadata");
  check_gpu(q_out, "q_out");
  check_gpu(k_cache, "k_cache");
  check_gpu(v_cache, "v_cache");
  check_dtype(positions, at::kInt, "positions");
  check_dtype(slots, at::kInt, "slots");
  check_dtype(rope, at::kFloat, "rope");
  check_dtype(q_out, at::kBFloat16, "q_out");
  TORCH_CHECK(w.size(0) == (nh + 2 * nkv) * 128, "w rows must be (nh + 2 nkv) * 128");
  TORCH_CHECK(positions.numel() >= x.size(0) && slots.numel() >= x.size(0), "metadata too short");
  TORCH_CHECK(q_out.numel() >= x.size(0) * nh * 128, "q_out too small");
  TORCH_CHECK(rope.dim() == 3 && rope.size(1) == 64 && rope.size(2) == 2, "rope must be [P, 64, 2]");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == nkv && k_cache.size(2) == dsse::kBS &&
                  k_cache.size(3) == 128, "k_cache must be [blocks, nkv, 32, 128]");
  TORCH_CHECK(v_cache.sizes() == at::IntArrayRef({k_cache.size(0), nkv, 128, dsse::kBS}),
              "v_cache must be [blocks, nkv, 128, 32]");
  dsse::GemmEpi ep{};
  ep.positions = positions.data_ptr<int>();
  ep.slots = slots.data_ptr<int>();
  ep.rope = reinterpret_cast<const float2*>(rope.data_ptr<float>());
  ep.q_out = reinterpret_cast<bf16*>(q_out.data_ptr());
  ep.k_cache = reinterpret_cast<bf16*>(k_cache.data_ptr());
  ep.v_cache = reinterpret_cast<bf16*>(v_cache.data_ptr());
  ep.nh = (int)nh;
  ep.nkv = (int)nkv;
  ep.num_slots = (int)(k_cache.size(0) * dsse::kBS);
  ep.rope_len = (int)rope.size(0);
  run_gemm(dsse::kQkvRope, x, w, ep);
}

void rmsnorm(Tensor& resid, const Tensor& w, Tensor& y, double eps, const c10::optional<Tensor>& delta,
             const c10::optional<Tensor>& embed, const c10::optional<Tensor>& ids,
             const c10::optional<Tensor>& part, int64_t nsplit) {
  check_gpu(resid, "resid");
  check_gpu(w, "w");
  check_gpu(y, "y");
  check_dtype(resid, at::kFloat, "resid");
  check_dtype(w, at::kBFloat16, "w");
  check_dtype(y, at::kBFloat16, "y");
  const int M = (int)y.size(0), H = (int)y.size(1);
  TORCH_CHECK(H % 1024 == 0 && H <= 8192, "hidden size must be a multiple of 1024 and <= 8192");
  TORCH_CHECK(resid.size(0) >= M && resid.size(1) == H && w.numel() == H, "shape mismatch");
  int mode = 0;
  const void* dptr = nullptr;
  const void* eptr = nullptr;
  const int* iptr = nullptr;
  int vocab = 0;
  if (embed.has_value()) {
    TORCH_CHECK(ids.has_value(), "embedding mode needs ids");
    check_gpu(*embed, "embed");
    check_gpu(*ids, "ids");
    check_dtype(*ids, at::kInt, "ids");
    TORCH_CHECK(embed->size(1) == H && ids->numel() >= M, "embedding shape mismatch");
    mode = 2;
    eptr = embed->data_ptr();
    iptr = ids->data_ptr<int>();
    vocab = (int)embed->size(0);
  } else if (delta.has_value()) {
    check_gpu(*delta, "delta");
    check_dtype(*delta, at::kBFloat16, "delta");
    TORCH_CHECK(delta->size(0) >= M && delta->size(1) == H, "delta shape mismatch");
    mode = 1;
    dptr = delta->data_ptr();
  }
  const float* pptr = nullptr;
  if (part.has_value() && nsplit > 0 && mode == 0) {
    check_gpu(*part, "part");
    check_dtype(*part, at::kFloat, "part");
    TORCH_CHECK(part->numel() >= nsplit * M * H, "part too small for ", nsplit, " slabs");
    mode = 3;
    pptr = part->data_ptr<float>();
  }
  DSSE_CHECK_HIP(dsse_rmsnorm(mode, M, resid.data_ptr<float>(), H, dptr, eptr, iptr, w.data_ptr(),
                              y.data_ptr(), (float)eps, pptr, (int)nsplit, vocab, cur_stream()));
}

void rope_kv_write(const Tensor& qkv, const Tensor& positions, const Tensor& slots, const Tensor& rope,
                   Tensor& q_out, Tensor& k_cache, Tensor& v_cache, int64_t nh, int64_t nkv) {
  check_gpu(qkv, "qkv");
  check_dtype(qkv, at::kBFloat16, "qkv");
  const int T = (int)qkv.size(0);
  TORCH_CHECK(qkv.size(1) == (nh + 2 * nkv) * 128, "qkv width mismatch");
  TORCH_CHECK(positions.numel() >= T && slots.numel() >= T, "metadata too short");
  TORCH_CHECK(q_out.numel() >= (int64_t)T * nh * 128, "q_out too small");
  TORCH_CHECK(k_cache.size(1) == nkv && v_cache.size(1) == nkv, "cache head mismatch");
  DSSE_CHECK_HIP(dsse_rope_kv_write(T, qkv.data_ptr(), (int)nh, (int)nkv, positions.data_ptr<int>(),
                                    slots.data_ptr<int>(),
                                    reinterpret_cast<const float2*>(rope.data_ptr<float>()),
                                    q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                    (int)(k_cache.size(0) * dsse::kBS), (int)rope.size(0), cur_stream()));
}

void silu_mul(const Tensor& gu, Tensor& h) {
  check_gpu(gu, "gu");
  check_gpu(h, "h");
  const int T = (int)gu.size(0), F = (int)h.size(1);
  TORCH_CHECK(gu.size(1) == 2 * F && h.size(0) == T && F % 8 == 0, "silu_mul shape mismatch");
  DSSE_CHECK_HIP(dsse_silu_mul(T, F, gu.data_ptr(), h.data_ptr(), cur_stream()));
}

void decode_prep(const Tensor& active, const Tensor& positions, const Tensor& block_tables,
                 Tensor& slots, Tensor& ctx_len, Tensor& q_len, int64_t num_blocks) {
  for (const Tensor* t : {&active, &positions, &block_tables, (const Tensor*)&slots, (const Tensor*)&ctx_len, (const Tensor*)&q_len}) {
    check_gpu(*t, "decode metadata");
    check_dtype(*t, at::kInt, "decode metadata");
  }
  const int B = (int)active.numel();
  TORCH_CHECK(positions.numel() >= B && slots.numel() >= B && ctx_len.numel() >= B &&
                  q_len.numel() >= B && block_tables.size(0) >= B, "decode metadata too short");
  DSSE_CHECK_HIP(dsse_decode_prep(B, active.data_ptr<int>(), positions.data_ptr<int>(),
                                  block_tables.data_ptr<int>(), (int)block_tables.size(1),
                                  (int)std::min<int64_t>(num_blocks, INT32_MAX), slots.data_ptr<int>(), ctx_len.data_ptr<int>(), q_len.data_ptr<int>(),
                                  cur_stream()));
}

// Warm the Infinity Cache with the first `bytes` of `t` (all of it when bytes < 0) on `wgs` workgroups; `sink`:
// an int32 tensor of >= 1024 words the kernel never writes in practice (it keeps the loads alive).
void ring_advance(Tensor& counter) {
  check_gpu(counter, "counter");
  check_dtype(counter, at::kInt, "counter");
  DSSE_CHECK_HIP(dsse_ring_advance(counter.data_ptr<int>(), cur_stream()));
}

// Checks and parameter block shared by the paged-attention entry points (hq query heads, QW query tiles per
// workgroup, KWV key-split waves in the partition-size check).
dsse::AttnParams attn_params(int hq, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                             const Tensor& q_start, const Tensor& q_len, const Tensor& ctx_len, const Tensor& work_seq,
                             const Tensor& work_tile, Tensor& out, Tensor& part_o, Tensor& part_ml, int64_t part,
                             int64_t nparts, int qw, int kwv) {
  for (const Tensor* t : {&k_cache, &v_cache, (const Tensor*)&out}) {
    check_gpu(*t, "attention tensor");
    check_dtype(*t, at::kBFloat16, "attention tensor");
  }
  for (auto* t : {&block_tables, &q_start, &q_len, &ctx_len, &work_seq, &work_tile}) {
    check_gpu(*t, "attention metadata");
    check_dtype(*t, at::kInt, "attention metadata");
  }
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(2) == dsse::kBS && k_cache.size(3) == 128,
              "k_cache must be [blocks, Hkv, 32, 128]");
  const int hkv = (int)k_cache.size(1);
  TORCH_CHECK(v_cache.sizes() == at::IntArrayRef({k_cache.size(0), hkv, 128, dsse::kBS}),
              "v_cache must be [blocks, Hkv, 128, 32]");
  TORCH_CHECK(hq % hkv == 0 && 16 % (hq / hkv) == 0, "GQA group must divide 16");
  TORCH_CHECK(out.dim() == 3 && out.size(1) == hq && out.size(2) == 128, "out must be [T, Hq, 128]");
  const int num_work = (int)work_seq.numel();
  TORCH_CHECK(work_tile.numel() == num_work, "work lists differ in length");
  TORCH_CHECK((part % (32 * kwv) == 0 && part > 0) || (part == 0 && nparts > 1),
              "partition size must be a multiple of ", 32 * kwv, " (or 0: even split of each sequence's keys)");
  TORCH_CHECK(nparts >= 1, "nparts >= 1");
  if (nparts > 1) {
    check_gpu(part_o, "part_o");
    check_gpu(part_ml, "part_ml");
    TORCH_CHECK(part_o.numel() >= (int64_t)num_work * hkv * nparts * qw * 16 * 128, "part_o too small");
    TORCH_CHECK(part_ml.numel() >= (int64_t)num_work * hkv * nparts * qw * 16 * 2, "part_ml too small");
  }
  dsse::AttnParams p{};
  p.k_cache = reinterpret_cast<const bf16*>(k_cache.data_ptr());
  p.v_cache = reinterpret_cast<const bf16*>(v_cache.data_ptr());
  p.block_tables = block_tables.data_ptr<int>();
  p.max_blocks = (int)block_tables.size(1);
  p.num_blocks = (int)k_cache.size(0);
  p.q_start = q_start.data_ptr<int>();
  p.q_len = q_len.data_ptr<int>();
  p.ctx_len = ctx_len.data_ptr<int>();
  p.work_seq = work_seq.data_ptr<int>();
  p.work_tile = work_tile.data_ptr<int>();
  p.out = reinterpret_cast<bf16*>(out.data_ptr());
  p.part_o = nparts > 1 ? part_o.data_ptr<float>() : nullptr;
  p.part_ml = nparts > 1 ? reinterpret_cast<float2*>(part_ml.data_ptr<float>()) : nullptr;
  p.hq = hq;
  p.hkv = hkv;
  p.group = hq / hkv;
  p.part = (int)part;
  p.nparts = (int)nparts;
  p.scale_log2 = 1.4426950408889634f / sqrtf(128.f);
  const int env_kwv = env_int("attn_kwv", 0);
  p.kwv = (env_kwv == 1 || env_kwv == 2 || env_kwv == 4 || env_kwv == 8) ? env_kwv : 0;
  const int env_pd = env_int("attn_pd", 0);
  p.pd = (env_pd == 1 || env_pd == 2) ? env_pd : 0;
  return p;
}

// Decode partitions combined by their last arriver (attention.hip, round 6) instead of attn_combine_kernel: opt-in,
// attn_comb=1 (DSSE_KERNEL_CFG).  Measured slower on a TP = 8 rank's 64-stream step, 2.20 vs 1.975 ms
// (profiles/r6/attn_comb_ab_r6.log): each partition's agent-scope release costs more than the combine launch it
// saves -- as for the GEMM fix-ups.  Needs a ticket per (item, kv head).
void attn_last_arriver(dsse::AttnParams& p, int num_work, const at::Device& dev) {
  if (p.nparts > 1 && env_int("attn_comb", 0) && (long)num_work * p.hkv <= dsse::kFixTiles)
    p.comb_cnt = fix_counters(dev) + dsse::kAttnCntOff;
}

void paged_attention(int64_t mode, const Tensor& q, const Tensor& k_cache, const Tensor& v_cache,
                     const Tensor& block_tables, const Tensor& q_start, const Tensor& q_len,
                     const Tensor& ctx_len, const Tensor& work_seq, const Tensor& work_tile,
                     Tensor& out, Tensor& part_o, Tensor& part_ml, int64_t part, int64_t nparts) {
  check_gpu(q, "q");
  check_dtype(q, at::kBFloat16, "q");
  TORCH_CHECK(q.dim() == 3 && q.size(2) == 128, "q must be [T, Hq, 128]");
  TORCH_CHECK(out.sizes() == q.sizes(), "out must match q");
  TORCH_CHECK(mode >= 0 && mode <= 2, "mode: 0 decode, 1 prefill (16-query tiles), 2 flash prefill (64-query tiles)");
  const int hq = (int)q.size(1), hkv = (int)k_cache.size(1);
  if (mode == 2) TORCH_CHECK(hq % hkv == 0 && (hq / hkv == 1 || hq / hkv == 2 || hq / hkv == 4),
                             "flash prefill supports G in {1, 2, 4}");
  dsse::AttnParams p = attn_params(hq, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work_seq, work_tile,
                                   out, part_o, part_ml, part, nparts, mode == 0 ? 1 : 4, mode == 0 ? 4 : 1);
  p.q = reinterpret_cast<const bf16*>(q.data_ptr());
  const int num_work = (int)work_seq.numel();
  if (mode == 2) {
    // flash prefill: q heads per workgroup (flash_hg in DSSE_KERNEL_CFG; 0 = the launcher's rule)
    const int hg = env_int("flash_hg", 0);
    p.kwv = (hg == 1 || hg == 2 || hg == 4) && (hq / hkv) % hg == 0 ? hg : 0;
  }
  if (mode == 0) attn_last_arriver(p, num_work, q.device());
  if (mode == 2) DSSE_CHECK_HIP(dsse_flash_prefill(num_work, &p, cur_stream()));
  else DSSE_CHECK_HIP(dsse_paged_attention((int)mode, num_work, &p, cur_stream()));
}

// Flash prefill with the key split (round 6): `work` = [seq | tile | (kb0, kb1) pairs | slot] over nw items (int32,
// 5 nw), `comb` = [(seq, tile, first slot, slots)] over the split tiles (int32, 4 nc).  Items with slot -1 write `out`;
// the others leave partial O / (max, sum) in slots [0, nslots) of part_o / part_ml and flash_combine_kernel merges
// them (engine: ModelRunner._flash_split_plan).
void flash_prefill_split(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                         const Tensor& q_start, const Tensor& q_len, const Tensor& ctx_len, const Tensor& work,
                         const Tensor& comb, Tensor& out, Tensor& part_o, Tensor& part_ml, int64_t nslots) {
  check_gpu(q, "q");
  check_dtype(q, at::kBFloat16, "q");
  TORCH_CHECK(q.dim() == 3 && q.size(2) == 128, "q must be [T, Hq, 128]");
  TORCH_CHECK(out.sizes() == q.sizes(), "out must match q");
  const int hq = (int)q.size(1), hkv = (int)k_cache.size(1);
  TORCH_CHECK(hq % hkv == 0 && (hq / hkv == 1 || hq / hkv == 2 || hq / hkv == 4), "flash prefill supports G in {1, 2, 4}");
  for (const Tensor* t : {&work, &comb}) {
    check_gpu(*t, "split plan");
    check_dtype(*t, at::kInt, "split plan");
  }
  TORCH_CHECK(work.numel() % 5 == 0 && comb.numel() % 4 == 0, "work = 5 x nw, comb = 4 x nc int32");
  const int64_t nw = work.numel() / 5;
  check_gpu(part_o, "part_o");
  check_gpu(part_ml, "part_ml");
  check_dtype(part_o, at::kFloat, "part_o");
  check_dtype(part_ml, at::kFloat, "part_ml");
  TORCH_CHECK(nslots >= 0 && part_o.numel() >= nslots * hkv * hq / hkv * 64 * 128 &&
                  part_ml.numel() >= nslots * hkv * hq / hkv * 64 * 2, "part_o / part_ml too small for nslots");
  Tensor ws = work.narrow(0, 0, nw), wt = work.narrow(0, nw, nw);
  dsse::AttnParams p = attn_params(hq, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, ws, wt, out, part_o,
                                   part_ml, 32, 1, 4, 1);
  p.q = reinterpret_cast<const bf16*>(q.data_ptr());
  p.work_kb = work.data_ptr<int>() + 2 * nw;
  p.work_slot = work.data_ptr<int>() + 4 * nw;
  p.comb = comb.data_ptr<int>();
  p.ncomb = (int)(comb.numel() / 4);
  p.part_o = part_o.data_ptr<float>();
  p.part_ml = reinterpret_cast<float2*>(part_ml.data_ptr<float>());
  p.kwv = 0;
  DSSE_CHECK_HIP(dsse_flash_prefill((int)nw, &p, cur_stream()));
}

// Decode QKV projection + attention with the projection's epilogue folded into the attention kernel: the GEMM
// leaves fp32 split-K slabs in `slabs` and attention mode 3 sums them, applies RoPE, writes this step's K / V
// into the cache and attends -- one launch (the split-K reduce) fewer per layer.  Falls back to gemm_qkv_rope
// + decode attention when the chosen GEMM cannot leave slabs (the register-streaming kernel of tiny batches),
// for GQA groups other than 1, 2, 4 heads, when `slabs` is too small, or with fused_qkv_attn=0 (DSSE_KERNEL_CFG).  Returns the number of slabs (0 = fallback).
int64_t qkv_attention_decode(const Tensor& x, const Tensor& w, const Tensor& positions, const Tensor& slots,
                             const Tensor& rope, Tensor& q_out, Tensor& k_cache, Tensor& v_cache, int64_t nh,
                             int64_t nkv, Tensor& slabs, const Tensor& block_tables, const Tensor& q_start,
                             const Tensor& q_len, const Tensor& ctx_len, const Tensor& work_seq,
                             const Tensor& work_tile, Tensor& out, Tensor& part_o, Tensor& part_ml, int64_t part,
                             int64_t nparts) {
  check_gpu(x, "x");
  check_gpu(w, "w");
  check_gpu(slabs, "slabs");
  check_dtype(slabs, at::kFloat, "slabs");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  const bool shape_ok = x.dim() == 2 && w.dim() == 2 && M >= 1 && K % 128 == 0 && w.size(1) == K &&
                        N == (nh + 2 * nkv) * 128;
  const int impl = shape_ok ? gemm_impl(M, N, K) : 0;
  int S = 0;
  if (impl == 4) {
    const TCfg c = pick_tiled(M, N, K, true);
    S = c.fix ? 0 : c.S;  // combined in the launch: the unfused path (gemm_qkv_rope's FIX launch + attention)
  }
  else if (impl == 3) S = pick_wide(M, N, K).S;
  else if (impl == 2) {
    S = pick_stream(M, N, K, dsse::kQkvRope).S;
    // qkv_split (DSSE_KERNEL_CFG): split-K of the QKV projection alone (its slabs are read by the attention kernel)
    const int qs = env_int("qkv_split", 0);
    const int slices = K / (128 * ((M <= 64 || M > 256) ? 4 : (M <= 128 ? 2 : 1)));  // gemm_stream.hip stream_cps
    if (qs > 0 && slices % qs == 0) S = qs;
  }
  auto q3 = q_out.view({-1, nh, 128});
  auto o3 = out.view({-1, nh, 128});
  const bool group_ok = nkv > 0 && nh % nkv == 0 && (nh / nkv == 1 || nh / nkv == 2 || nh / nkv == 4);  // attention.hip
  if ((S <= 0 || !group_ok || slabs.numel() < (int64_t)S * M * N || env_int("fused_qkv_attn", 1) == 0)) {
    gemm_qkv_rope(x, w, positions, slots, rope, q_out, k_cache, v_cache, nh, nkv);
    paged_attention(0, q3, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work_seq, work_tile, o3, part_o,
                    part_ml, part, nparts);
    return 0;
  }
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(w, at::kBFloat16, "w");
  for (auto* t : {&positions, &slots}) {
    check_gpu(*t, "metadata");
    check_dtype(*t, at::kInt, "metadata");
  }
  check_gpu(rope, "rope");
  check_dtype(rope, at::kFloat, "rope");
  TORCH_CHECK(rope.dim() == 3 && rope.size(1) == 64 && rope.size(2) == 2, "rope must be [P, 64, 2]");
  TORCH_CHECK(positions.numel() >= M && slots.numel() >= M, "metadata too short");
  TORCH_CHECK(k_cache.size(1) == nkv, "k_cache heads must be nkv");
  TORCH_CHECK(o3.size(0) == M, "out must hold the M query rows");
  dsse::AttnParams p = attn_params((int)nh, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, work_seq,
                                   work_tile, o3, part_o, part_ml, part, nparts, 1, 4);
  dsse::GemmEpi ep{};
  const void* X = x.data_ptr();
  float* sl = slabs.data_ptr<float>();
  if (impl == 4) {
    const TCfg c = pick_tiled(M, N, K, true);
    DSSE_CHECK_HIP(tiled_call(dsse::kQkvRope, c.cfg, S, 1, X, K, M, w.data_ptr(), K, N, &ep, sl));
  } else if (impl == 3) {
    const WCfg c = pick_wide(M, N, K);
    DSSE_CHECK_HIP(dsse_gemm_wide(dsse::kQkvRope, c.mb, c.rd, S, 1, X, K, M, w.data_ptr(), K, N, &ep, sl, cur_stream()));
  } else {
    const SCfg c = pick_stream(M, N, K, dsse::kQkvRope);
    DSSE_CHECK_HIP(stream_launch(dsse::kQkvRope, c, S, 1, X, M, w.data_ptr(), K, N, &ep, sl));
  }
  p.qkv_part = sl;
  p.qkv_S = S;
  p.qkv_M = M;
  p.positions = positions.data_ptr<int>();
  p.slots = slots.data_ptr<int>();
  p.rope = reinterpret_cast<const float2*>(rope.data_ptr<float>());
  p.rope_len = (int)rope.size(0);
  p.num_slots = (int)(k_cache.size(0) * dsse::kBS);
  p.k_out = reinterpret_cast<bf16*>(k_cache.data_ptr());
  p.v_out = reinterpret_cast<bf16*>(v_cache.data_ptr());
  attn_last_arriver(p, (int)work_seq.numel(), x.device());
  DSSE_CHECK_HIP(dsse_paged_attention(3, (int)work_seq.numel(), &p, cur_stream()));
  return S;
}

dsse::SampleParams sample_params(const Tensor& temperature, const Tensor& top_k, const Tensor& top_p,
                                 const Tensor& seeds, const Tensor& positions,
                                 const c10::optional<Tensor>& active, int B) {
  for (const Tensor* t : {&temperature, &top_k, &top_p, &seeds, &positions}) check_gpu(*t, "sampling metadata");
  check_dtype(temperature, at::kFloat, "temperature");
  check_dtype(top_k, at::kInt, "top_k");
  check_dtype(top_p, at::kFloat, "top_p");
  check_dtype(seeds, at::kInt, "seeds");
  check_dtype(positions, at::kInt, "positions");
  TORCH_CHECK(temperature.numel() >= B && top_k.numel() >= B && top_p.numel() >= B && seeds.numel() >= 2 * B &&
                  positions.numel() >= B, "sampling metadata too short");
  dsse::SampleParams p{};
  p.temperature = temperature.data_ptr<float>();
  p.top_k = top_k.data_ptr<int>();
  p.top_p = top_p.data_ptr<float>();
  p.seeds = reinterpret_cast<const uint2*>(seeds.data_ptr<int>());
  p.positions = positions.data_ptr<int>();
  if (active.has_value()) {
    check_gpu(*active, "active");
    check_dtype(*active, at::kInt, "active");
    TORCH_CHECK(active->numel() >= B, "active too short");
    p.active = active->data_ptr<int>();
  }
  return p;
}

// Per-rank candidate pass: cand [B, nchunks, 2] fp32 (score, index bits).
void sample_candidates(const Tensor& logits, const Tensor& temperature, const Tensor& top_k, const Tensor& top_p,
                       const Tensor& seeds, const Tensor& positions, const c10::optional<Tensor>& active,
                       Tensor& cand, int64_t vocab_offset) {
  check_gpu(logits, "logits");
  check_dtype(logits, at::kFloat, "logits");
  check_gpu(cand, "cand");
  check_dtype(cand, at::kFloat, "cand");
  const int B = (int)logits.size(0), V = (int)logits.size(1);
  TORCH_CHECK(V <= 32768, "sampler supports V <= 32768 per rank");
  TORCH_CHECK(cand.dim() == 3 && cand.size(0) == B && cand.size(2) == 2, "cand must be [B, nchunks, 2]");
  dsse::SampleParams p = sample_params(temperature, top_k, top_p, seeds, positions, active, B);
  p.logits = logits.data_ptr<float>();
  p.ld = V;
  p.V = V;
  p.vocab_offset = (int)vocab_offset;
  p.cand = reinterpret_cast<float2*>(cand.data_ptr<float>());
  p.nchunks = (int)cand.size(1);
  DSSE_CHECK_HIP(dsse_sample(B, &p, cur_stream()));
}

// Merge pass over cand_all [world, B, nchunks, 2] and commit: next_ids, ring[head], positions += 1.
void sample_pick(const Tensor& cand_all, const c10::optional<Tensor>& active, Tensor& next_ids,
                 const c10::optional<Tensor>& ring, const c10::optional<Tensor>& ring_counter,
                 const c10::optional<Tensor>& positions_inc, int64_t vocab) {
  check_gpu(cand_all, "cand_all");
  check_gpu(next_ids, "next_ids");
  check_dtype(next_ids, at::kInt, "next_ids");
  TORCH_CHECK(cand_all.dim() == 4 && cand_all.size(3) == 2, "cand_all must be [world, B, nchunks, 2]");
  const int world = (int)cand_all.size(0), B = (int)cand_all.size(1);
  TORCH_CHECK(next_ids.numel() >= B, "next_ids too short");
  dsse::SampleParams p{};
  p.nchunks = (int)cand_all.size(2);
  p.v_global = (int)std::min<int64_t>(vocab, INT32_MAX);
  p.next_ids = next_ids.data_ptr<int>();
  if (active.has_value()) {
    TORCH_CHECK(active->numel() >= B, "active too short");
    p.active = active->data_ptr<int>();
  }
  if (ring.has_value()) {
    TORCH_CHECK(ring_counter.has_value(), "ring needs ring_counter");
    check_gpu(*ring, "ring");
    TORCH_CHECK(ring->dim() == 2 && ring->size(1) >= B, "ring must be [R, >= B]");
    p.ring = ring->data_ptr<int>();
    p.ring_counter = ring_counter->data_ptr<int>();
    p.ring_size = (int)ring->size(0);
    p.ring_stride = (int)ring->size(1);
  }
  if (positions_inc.has_value()) {
    TORCH_CHECK(positions_inc->numel() >= B, "positions_inc too short");
    p.positions_inc = positions_inc->data_ptr<int>();
  }
  DSSE_CHECK_HIP(dsse_sample_pick(B, world, cand_all.data_ptr(), &p, cur_stream()));
}

// First-token sampling inside the captured prefill / mixed graphs (sampler.hip prefill_sample_*): gather the
// finishing prompts' last rows + their slots' sampling parameters, then (after the LM head, candidates and pick)
// commit ids / ring / positions.  meta: int32 [3 NS + 2]; smeta: int32 [7 NS]; slot_meta: the runner's [6 Bm].
void prefill_sample_gather(const Tensor& x, const Tensor& meta, const Tensor& slot_meta, Tensor& xl, Tensor& smeta) {
  for (const Tensor* t : {&x, &meta, &slot_meta, (const Tensor*)&xl, (const Tensor*)&smeta})
    check_gpu(*t, "prefill_sample_gather operand");
  check_dtype(x, at::kBFloat16, "x");
  check_dtype(xl, at::kBFloat16, "xl");
  for (const Tensor* t : {&meta, &slot_meta, (const Tensor*)&smeta}) check_dtype(*t, at::kInt, "metadata");
  TORCH_CHECK(x.dim() == 2 && xl.dim() == 2 && xl.size(1) == x.size(1) && x.size(1) % 8 == 0, "x / xl shapes");
  const int NS = (int)xl.size(0), Bm = (int)(slot_meta.numel() / 6);
  TORCH_CHECK(meta.numel() >= 3 * NS + 2 && smeta.numel() >= 7 * NS && slot_meta.numel() == 6 * Bm, "metadata sizes");
  DSSE_CHECK_HIP(dsse_prefill_sample_gather(x.data_ptr(), (int)x.size(0), (int)x.size(1), meta.data_ptr<int>(), NS,
                                            slot_meta.data_ptr<int>(), Bm, xl.data_ptr(), smeta.data_ptr<int>(),
                                            cur_stream()));
}

void prefill_sample_commit(const Tensor& meta, const Tensor& new_ids, Tensor& ids, Tensor& ring, Tensor& positions) {
  for (const Tensor* t : {&meta, &new_ids, (const Tensor*)&ids, (const Tensor*)&ring, (const Tensor*)&positions}) {
    check_gpu(*t, "prefill_sample_commit operand");
    check_dtype(*t, at::kInt, "int32 operand");
  }
  const int NS = (int)new_ids.numel(), Bm = (int)ids.numel();
  TORCH_CHECK(NS <= 64 && meta.numel() >= 3 * NS + 2, "meta too short / NS > 64");
  TORCH_CHECK(ring.dim() == 2 && ring.size(1) == Bm && positions.numel() == Bm, "ring must be [R, Bm], positions [Bm]");
  DSSE_CHECK_HIP(dsse_prefill_sample_commit(meta.data_ptr<int>(), NS, new_ids.data_ptr<int>(), ids.data_ptr<int>(), Bm,
                                            ring.data_ptr<int>(), (int)ring.size(0), positions.data_ptr<int>(),
                                            cur_stream()));
}

// ---- TP all-reduce over IPC peer buffers (allreduce.hip) ------------------------------------------------------
// ar_alloc: this rank's zeroed buffer for `rows` decode rows of width H -> (64-byte IPC handle as uint8 [64],
// device pointer, uncached flag).  ar_open: a peer's handle -> its pointer in this process.  The buffers live
// until ar_close (process lifetime in the engine).
std::tuple<Tensor, int64_t, int64_t> ar_alloc(int64_t rows, int64_t H) {
  TORCH_CHECK(rows > 0 && H > 0 && H % 512 == 0 && H <= 8192, "ar_alloc: bad shape");
  Tensor h = at::zeros({64}, at::kByte);
  void* p = nullptr;
  int uncached = 0;
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle size");
  DSSE_CHECK_HIP(dsse_ar_alloc(dsse_ar_buffer_bytes((int)rows, (int)H), &p, h.data_ptr(), &uncached));
  return {h, (int64_t)reinterpret_cast<uintptr_t>(p), (int64_t)uncached};
}
int64_t ar_open(const Tensor& handle) {
  TORCH_CHECK(handle.numel() == 64 && handle.scalar_type() == at::kByte && !handle.is_cuda(), "ar_open: 64-byte CPU handle");
  void* p = nullptr;
  DSSE_CHECK_HIP(dsse_ar_open(handle.contiguous().data_ptr(), &p));
  return (int64_t)reinterpret_cast<uintptr_t>(p);
}
void ar_close(int64_t ptr, bool opened) { DSSE_CHECK_HIP(dsse_ar_close(reinterpret_cast<void*>(ptr), opened ? 1 : 0)); }

// resid[b] += sum over ranks of tmp[b] (every rank's partial, read from the peers' buffers), y = rmsnorm(resid) * w.
// peers: int64 device tensor [world] of buffer pointers in THIS process (own at index rank); epoch: int32 [rows],
// zero-initialised, owned by this all-reduce context; err: int32 [1] (set on a timed-out peer wait).
void ar_rmsnorm(const Tensor& tmp, Tensor& resid, const Tensor& w, Tensor& y, double eps, const Tensor& peers,
                int64_t rank, int64_t rows, Tensor& epoch, Tensor& err, const c10::optional<Tensor>& part,
                int64_t nsplit) {
  for (const Tensor* t : {&tmp, (const Tensor*)&resid, &w, (const Tensor*)&y, &peers, (const Tensor*)&epoch,
                          (const Tensor*)&err})
    check_gpu(*t, "ar_rmsnorm tensor");
  check_dtype(tmp, at::kBFloat16, "tmp");
  check_dtype(resid, at::kFloat, "resid");
  check_dtype(w, at::kBFloat16, "w");
  check_dtype(y, at::kBFloat16, "y");
  check_dtype(peers, at::kLong, "peers");
  check_dtype(epoch, at::kInt, "epoch");
  check_dtype(err, at::kInt, "err");
  const int M = (int)tmp.size(0), H = (int)tmp.size(1);
  TORCH_CHECK(tmp.dim() == 2 && resid.size(0) >= M && resid.size(1) == H && y.size(0) >= M && y.size(1) == H &&
                  w.numel() == H, "ar_rmsnorm: shape mismatch");
  TORCH_CHECK(M <= rows && epoch.numel() >= rows, "ar_rmsnorm: more rows than the buffers hold");
  const float* pp = nullptr;
  if (part.has_value() && nsplit > 0) {  // the partial row = sum of the GEMM's split-K slabs (tmp unused)
    check_gpu(*part, "part");
    check_dtype(*part, at::kFloat, "part");
    TORCH_CHECK(part->numel() >= nsplit * M * H, "part too small for ", nsplit, " slabs");
    pp = part->data_ptr<float>();
  }
  DSSE_CHECK_HIP(dsse_ar_rmsnorm(M, tmp.data_ptr(), resid.data_ptr<float>(), w.data_ptr(), y.data_ptr(), H, (float)eps,
                                 reinterpret_cast<const unsigned long long*>(peers.data_ptr<int64_t>()), (int)rank,
                                 (int)peers.numel(), (int)rows, reinterpret_cast<unsigned int*>(epoch.data_ptr<int>()),
                                 reinterpret_cast<unsigned int*>(err.data_ptr<int>()), pp, (int)(pp ? nsplit : 0),
                                 cur_stream()));
}

// C3 over the same IPC buffers: out[q] = rank q's `cand` rows (every rank's sampling candidates, [M, 16, 2] fp32 =
// 128 bytes per row); gepoch: int32 [rows], the gather's own counters.
void ar_gather(const Tensor& cand, Tensor& out, const Tensor& peers, int64_t rank, int64_t rows, int64_t H,
               Tensor& gepoch, Tensor& err) {
  for (const Tensor* t : {&cand, (const Tensor*)&out, &peers, (const Tensor*)&gepoch, (const Tensor*)&err})
    check_gpu(*t, "ar_gather tensor");
  check_dtype(cand, at::kFloat, "cand");
  check_dtype(out, at::kFloat, "out");
  check_dtype(peers, at::kLong, "peers");
  check_dtype(gepoch, at::kInt, "gepoch");
  check_dtype(err, at::kInt, "err");
  const int M = (int)cand.size(0), world = (int)peers.numel();
  TORCH_CHECK(cand.is_contiguous() && out.is_contiguous() && cand.numel() == (int64_t)M * 32,
              "ar_gather: cand must be contiguous [M, 16, 2] fp32 (128 bytes per row)");
  TORCH_CHECK(out.numel() == (int64_t)world * cand.numel(), "ar_gather: out must be [world, M, 16, 2]");
  TORCH_CHECK(M <= rows && gepoch.numel() >= rows, "ar_gather: more rows than the buffers hold");
  DSSE_CHECK_HIP(dsse_ar_gather(M, cand.data_ptr(), out.data_ptr(),
                                reinterpret_cast<const unsigned long long*>(peers.data_ptr<int64_t>()), (int)rank, world,
                                (int)rows, (int)H, reinterpret_cast<unsigned int*>(gepoch.data_ptr<int>()),
                                reinterpret_cast<unsigned int*>(err.data_ptr<int>()), cur_stream()));
}

int64_t kernels_abi_version() { return 16; }

// The dispatch's choice for an (M, N, K) projection: (impl, tiled cfg, split, fix, model estimate in us) -- impl as
// gemm_impl (4 = tiled / pipe); cfg / split / fix / estimate only for impl 4 (tools/bench_decode_gemm.py --plan).
std::tuple<int64_t, int64_t, int64_t, bool, double> gemm_plan(int64_t M, int64_t N, int64_t K, bool slab_consumer) {
  const int impl = gemm_impl((int)M, (int)N, (int)K);
  if (impl != 4) return {impl, -1, 0, false, 0.0};
  const TCfg c = pick_tiled((int)M, (int)N, (int)K, slab_consumer);
  return {impl, c.cfg, c.S, c.fix, c.est_us};
}

// Stamps build: the last fix-up launch's per-workgroup phase stamps ([kStampWgs, 8] int64; empty otherwise).
at::Tensor gemm_fix_stamps(int64_t device) {
  const at::Device dev(at::kCUDA, (c10::DeviceIndex)device);
  if (!DSSE_PIPE_STAMPS) return at::empty({0}, at::kLong);
  return fix_state(dev).narrow(0, dsse::kStampOff, kStampWgs * 16).view(at::kLong).view({kStampWgs, 8}).cpu();
}

// Timed-out waits of the in-launch split-K fix-up on `device` since load (0 unless a writer never counted itself).
int64_t gemm_fix_timeouts(int64_t device) {
  const at::Device dev(at::kCUDA, (c10::DeviceIndex)device);
  int v = 0;
  DSSE_CHECK_HIP(hipMemcpy(&v, fix_counters(dev), sizeof(int), hipMemcpyDeviceToHost));
  return v;
}

#if DSSE_KERNEL_CHECKS
bool kernels_checked() { return true; }
#else
bool kernels_checked() { return false; }
#endif

// Checked build: [7, 4] int32 (line, value, bound, count) of the first out-of-range index per kernel file,
// in the order of kCheckFiles; all zeros in the default build.  Synchronises the device.
const char* const kCheckFiles[7] = {"gemm_skinny.hip", "gemm_stream.hip", "attention.hip", "attention_prefill.hip",
                                    "elementwise.hip", "sampler.hip", "gemm_tiled.hip"};
Tensor kernel_checks(bool clear) {
  using Reader = hipError_t (*)(int*, int);
  static const Reader readers[7] = {dsse_check_gemm_skinny, dsse_check_gemm_stream, dsse_check_attention,
                                    dsse_check_attention_prefill, dsse_check_elementwise, dsse_check_sampler,
                                    dsse_check_gemm_tiled};
  Tensor out = at::zeros({7, 4}, at::kInt);
  if (!kernels_checked()) return out;
  DSSE_CHECK_HIP(hipDeviceSynchronize());
  for (int i = 0; i < 7; ++i) DSSE_CHECK_HIP(readers[i](out.data_ptr<int>() + 4 * i, clear ? 1 : 0));
  return out;
}
// Stamps build: step-anatomy records (common.h stamps::record) of the ring GEMMs and RMSNorms.  step_stamps_arm
// (re)binds an empty buffer of `cap` records per sub-buffer on `device` (cap 0 unbinds); step_stamps_read returns
// the records so far as [n, 8] int64 (tag, grid, block, t0..t3, wave), sub-buffer by sub-buffer (the tool sorts them
// by time).  Both synchronise the device; empty in the default build.
std::unordered_map<int, Tensor>& stamp_bufs() {
  static std::unordered_map<int, Tensor> m;
  return m;
}
bool step_stamps_arm(int64_t device, int64_t cap) {
  if (!DSSE_PIPE_STAMPS) return false;
  using namespace dsse::stamps;
  const at::Device dev(at::kCUDA, (c10::DeviceIndex)device);
  DSSE_CHECK_HIP(hipDeviceSynchronize());
  void* p = nullptr;
  if (cap > 0) {
    Tensor buf = at::zeros({kHeader + 8 * cap * kSubs}, at::TensorOptions().dtype(at::kLong).device(dev));
    const int64_t hdr = cap;
    DSSE_CHECK_HIP(hipMemcpy(buf.data_ptr(), &hdr, sizeof hdr, hipMemcpyHostToDevice));
    stamp_bufs()[dev.index()] = buf;
    p = buf.data_ptr();
  } else {
    stamp_bufs().erase(dev.index());
  }
  DSSE_CHECK_HIP(dsse_stamps_bind_gemm_stream(p));
  DSSE_CHECK_HIP(dsse_stamps_bind_elementwise(p));
  return true;
}
Tensor step_stamps_read(int64_t device) {
  using namespace dsse::stamps;
  auto it = stamp_bufs().find((int)device);
  if (!DSSE_PIPE_STAMPS || it == stamp_bufs().end()) return at::empty({0, 8}, at::kLong);
  DSSE_CHECK_HIP(hipDeviceSynchronize());
  Tensor h = it->second.cpu();
  const int64_t cap = h[0].item<int64_t>();
  std::vector<Tensor> parts;
  for (int s = 0; s < kSubs; ++s) {
    const int64_t n = std::min(h[8 + 8 * s].item<int64_t>(), cap);
    if (n > 0) parts.push_back(h.narrow(0, kHeader + (int64_t)s * cap * 8, 8 * n).view({n, 8}));
  }
  return parts.empty() ? at::empty({0, 8}, at::kLong) : at::cat(parts, 0);
}

std::string kernel_check_files() {
  std::string s;
  for (const char* f : kCheckFiles) s += std::string(s.empty() ? "" : ",") + f;
  return s;
}

}  // namespace

TORCH_LIBRARY(dsse, m) {
  m.def("gemm_out(Tensor x, Tensor w, Tensor(a!) out) -> ()");
  m.def("gemm_resid(Tensor x, Tensor w, Tensor(a!) resid) -> ()");
  m.def("gemm_silu(Tensor x, Tensor w, Tensor(a!) out) -> ()");
  m.def("gemm_qkv_rope(Tensor x, Tensor w, Tensor positions, Tensor slots, Tensor rope, Tensor(a!) q_out, "
        "Tensor(b!) k_cache, Tensor(c!) v_cache, int nh, int nkv) -> ()");
  m.def("rmsnorm(Tensor(a!) resid, Tensor w, Tensor(b!) y, float eps, Tensor? delta=None, Tensor? embed=None, "
        "Tensor? ids=None, Tensor? part=None, int nsplit=0) -> ()");
  m.def("gemm_resid_split(Tensor x, Tensor w, Tensor(a!) resid, Tensor(b!) part) -> int");
  m.def("gemm_out_split(Tensor x, Tensor w, Tensor(a!) out, Tensor(b!) part) -> int");
  m.def("refresh_env() -> ()", &refresh_env);
  m.def("rope_kv_write(Tensor qkv, Tensor positions, Tensor slots, Tensor rope, Tensor(a!) q_out, "
        "Tensor(b!) k_cache, Tensor(c!) v_cache, int nh, int nkv) -> ()");
  m.def("silu_mul(Tensor gu, Tensor(a!) h) -> ()");
  m.def("decode_prep(Tensor active, Tensor positions, Tensor block_tables, Tensor(a!) slots, "
        "Tensor(b!) ctx_len, Tensor(c!) q_len, int num_blocks=2147483647) -> ()");
  m.def("ring_advance(Tensor(a!) counter) -> ()");
  m.def("paged_attention(int mode, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor q_start, Tensor q_len, Tensor ctx_len, Tensor work_seq, Tensor work_tile, Tensor(a!) out, "
        "Tensor(b!) part_o, Tensor(c!) part_ml, int part, int nparts) -> ()");
  m.def("flash_prefill_split(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor q_start, "
        "Tensor q_len, Tensor ctx_len, Tensor work, Tensor comb, Tensor(a!) out, Tensor(b!) part_o, "
        "Tensor(c!) part_ml, int nslots) -> ()");
  m.def("qkv_attention_decode(Tensor x, Tensor w, Tensor positions, Tensor slots, Tensor rope, Tensor(a!) q_out, "
        "Tensor(b!) k_cache, Tensor(c!) v_cache, int nh, int nkv, Tensor(d!) slabs, Tensor block_tables, "
        "Tensor q_start, Tensor q_len, Tensor ctx_len, Tensor work_seq, Tensor work_tile, Tensor(e!) out, "
        "Tensor(f!) part_o, Tensor(g!) part_ml, int part, int nparts) -> int");
  m.def("sample_candidates(Tensor logits, Tensor temperature, Tensor top_k, Tensor top_p, Tensor seeds, "
        "Tensor positions, Tensor? active, Tensor(a!) cand, int vocab_offset=0) -> ()");
  m.def("sample_pick(Tensor cand_all, Tensor? active, Tensor(a!) next_ids, Tensor(b!)? ring=None, "
        "Tensor? ring_counter=None, Tensor(c!)? positions_inc=None, int vocab=2147483647) -> ()");
  m.def("prefill_sample_gather(Tensor x, Tensor meta, Tensor slot_meta, Tensor(a!) xl, Tensor(b!) smeta) -> ()");
  m.def("prefill_sample_commit(Tensor meta, Tensor new_ids, Tensor(a!) ids, Tensor(b!) ring, Tensor(c!) positions) -> ()");
  m.def("ar_alloc(int rows, int H) -> (Tensor, int, int)", &ar_alloc);
  m.def("ar_open(Tensor handle) -> int", &ar_open);
  m.def("ar_close(int ptr, bool opened) -> ()", &ar_close);
  m.def("ar_rmsnorm(Tensor tmp, Tensor(a!) resid, Tensor w, Tensor(b!) y, float eps, Tensor peers, int rank, int rows, "
        "Tensor(c!) epoch, Tensor(d!) err, Tensor? part=None, int nsplit=0) -> ()");
  m.def("ar_gather(Tensor cand, Tensor(a!) out, Tensor peers, int rank, int rows, int H, Tensor(b!) gepoch, "
        "Tensor(c!) err) -> ()");
  m.def("kernels_abi_version() -> int", &kernels_abi_version);
  m.def("gemm_plan(int M, int N, int K, bool slab_consumer=False) -> (int, int, int, bool, float)", &gemm_plan);
  m.def("gemm_fix_timeouts(int device=0) -> int", &gemm_fix_timeouts);
  m.def("gemm_fix_stamps(int device=0) -> Tensor", &gemm_fix_stamps);
  m.def("step_stamps_arm(int device=0, int cap=0) -> bool", &step_stamps_arm);
  m.def("step_stamps_read(int device=0) -> Tensor", &step_stamps_read);
  m.def("kernels_checked() -> bool", &kernels_checked);
  m.def("kernel_checks(bool clear=True) -> Tensor", &kernel_checks);
  m.def("kernel_check_files() -> str", &kernel_check_files);
}

TORCH_LIBRARY_IMPL(dsse, CUDA, m) {
  m.impl("gemm_out", &gemm_out);
  m.impl("gemm_resid", &gemm_resid);
  m.impl("gemm_resid_split", &gemm_resid_split);
  m.impl("gemm_out_split", &gemm_out_split);
  m.impl("gemm_silu", &gemm_silu);
  m.impl("gemm_qkv_rope", &gemm_qkv_rope);
  m.impl("rmsnorm", &rmsnorm);
  m.impl("rope_kv_write", &rope_kv_write);
  m.impl("silu_mul", &silu_mul);
  m.impl("decode_prep", &decode_prep);
  m.impl("ring_advance", &ring_advance);
  m.impl("paged_attention", &paged_attention);
  m.impl("flash_prefill_split", &flash_prefill_split);
  m.impl("qkv_attention_decode", &qkv_attention_decode);
  m.impl("sample_candidates", &sample_candidates);
  m.impl("sample_pick", &sample_pick);
  m.impl("prefill_sample_gather", &prefill_sample_gather);
  m.impl("prefill_sample_commit", &prefill_sample_commit);
  m.impl("ar_rmsnorm", &ar_rmsnorm);
  m.impl("ar_gather", &ar_gather);
}
