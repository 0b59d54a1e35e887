// Host-visible kernel API of the engine: parameter structs and the extern "C" launchers that the
// torch bindings (bindings.cpp) call with raw pointers and torch's current HIP stream.
#pragma once
#include "common.h"

namespace dsse {

constexpr int kBS = 32;  // KV-cache page size in tokens (fixed for every kernel)

enum GemmMode { kStoreBf16 = 0, kStoreF32 = 1, kResidAdd = 2, kSiluMul = 3, kQkvRope = 4 };

// Decode-GEMM weight layout ("tiled"): W[N, K] is stored as blocks of (16-row tile T, 128-column
// K-chunk c), block-major (T, c), each block [s = 0..3][lane = 0..63][j = 0..7] where lane l = r + 16g
// holds W[16T + r][128c + 32g + 8s + j] — exactly the MFMA B-operand fragment of k-step s.  A wave
// therefore loads every block as four fully contiguous 1 KiB runs (see ops/reference.py tile_weight).
constexpr int kTileChunk = 16 * 128;  // elements per (tile, chunk) block

struct GemmEpi {
  void* out;          // bf16 / f32 output (modes 0, 1, 3)
  int ldo;
  float* resid;       // mode 2
  int ldr;
  const int* positions;   // mode 4: per-row absolute position
  const int* slots;       // mode 4: per-row KV slot (-1 = do not write)
  const float2* rope;     // mode 4: [max_pos][64] (cos, sin)
  bf16* q_out;            // mode 4: [M, nh*128]
  bf16* k_cache;          // [blocks, nkv, kBS, 128]
  bf16* v_cache;          // [blocks, nkv, 128, kBS] (token-permuted inside a page)
  int nh, nkv;
  int num_slots;          // mode 4: KV slots in the cache (pages * kBS); checked build only
  int rope_len;           // mode 4: rows of the rope table; checked build only
  // split-K fix-up inside the launch (gemm_pipe.hip, partial_only = 2): [4 + 2 * kFixTiles] ints -- word 0 counts
  // timed-out waits, then the per-tile ticket and done counters (zero between launches: each tile's last arriver
  // resets its pair); null when unused
  int* fix_cnt;
};
constexpr int kFixTiles = 8192;  // tiles of one fix-up launch at most
// the per-device counter block (bindings.cpp fix_state): [4 words][2 kFixTiles GEMM fix-up counters]
// [kFixTiles decode-attention combine tickets][stamps build: per-workgroup stamps]
constexpr int kAttnCntOff = 4 + 2 * kFixTiles;
constexpr int kStampOff = 4 + 3 * kFixTiles;


struct AttnParams {
  const bf16* q;            // [T, Hq, 128]
  const bf16* k_cache;
  const bf16* v_cache;
  const int* block_tables;  // [B, max_blocks]
  int max_blocks;
  int num_blocks;           // pages in the KV cache (checked build: block-table entries must be below)
  const int* q_start;       // [B] first query row of the sequence in q / out
  const int* q_len;         // [B] number of query tokens (0 = inactive)
  const int* ctx_len;       // [B] number of keys in the cache including the queries
  const int* work_seq;      // [num_work] sequence of work item
  const int* work_tile;     // [num_work] query-tile block (in units of QW tiles)
  bf16* out;                // [T, Hq, 128]
  float* part_o;            // [num_work, Hkv, nparts, QW, 16, 128]
  float2* part_ml;          // [num_work, Hkv, nparts, QW, 16]
  int hq, hkv, group;       // group = hq / hkv; 16 % group == 0
  int part;                 // keys per partition (multiple of 32 * KWV); 0 = each item's keys split evenly over nparts
  int nparts;               // grid.z
  float scale_log2;         // log2(e) / sqrt(128)
  int kwv;                  // decode: waves per workgroup splitting the keys (0 = by grid size)
  int pd;                   // mode 3: KV pages in flight per wave (0 = by occupancy, 1 = no look-ahead)
  // mode 3 (decode with the QKV epilogue folded in): q comes from the QKV GEMM's fp32 split-K slabs instead
  // of `q`; the workgroup holding a sequence's newest key also writes that token's K / V into the cache.
  const float* qkv_part;    // [qkv_S, qkv_M, (hq + 2 hkv) * 128], columns in the engine's rotary-pair order
  int qkv_S, qkv_M;
  const int* positions;     // [qkv_M] absolute position of row m (RoPE)
  const int* slots;         // [qkv_M] KV slot of row m (-1 = do not write)
  const float2* rope;       // [rope_len, 64] (cos, sin)
  int rope_len, num_slots;
  bf16* k_out;              // = k_cache, writable
  bf16* v_out;              // = v_cache, writable
  // flash prefill key split (mode 2, round 6; nullptr = every item walks all its key blocks and writes `out`):
  // item i walks key blocks [work_kb[2i], work_kb[2i + 1]) and, when work_slot[i] >= 0, leaves its unnormalised O
  // and (max, sum) in partial slot work_slot[i] ([slot][Hkv][G][64 queries] of part_o / part_ml) for the combine:
  // comb[4c ..] = (sequence, 64-query tile, first slot, slots) of split tile c, ncomb of them
  const int* work_kb;
  const int* work_slot;
  const int* comb;
  int ncomb;
  // decode partitions (nparts > 1, one query tile per workgroup) combined by the last partition of each (item, kv
  // head) to finish instead of attn_combine_kernel (round 6): [num_work * hkv] arrival tickets, zero between
  // launches (the last arriver resets its ticket); null = the combine kernel
  int* comb_cnt;
};

struct SampleParams {
  const float* logits;  // [B, ld]
  int ld, V;            // row stride, local vocab size
  int vocab_offset;     // global index of local column 0
  const float* temperature;  // [B]; <= 0 -> greedy
  const int* top_k;          // [B]; <= 0 -> off
  const float* top_p;        // [B]; >= 1 -> off
  const uint2* seeds;        // [B]
  const int* positions;      // [B] position of the sampled token's predecessor (RNG counter)
  const int* active;         // [B] or null (all active)
  int* next_ids;             // [B] (pick pass)
  int* ring;                 // [ring_size, ring_stride] or null
  const int* ring_counter;
  int ring_size, ring_stride;
  int* positions_inc;        // [B] or null: positions[b] += 1 for active rows
  float2* cand;              // [B, nchunks] (score, index-as-bits) candidates
  int nchunks;               // vocab chunks per row (unfiltered path)
  int v_global;              // full vocabulary (all TP shards); checked build: sampled ids below it
};

}  // namespace dsse

extern "C" {
hipError_t dsse_skinny_gemm(int mode, int mt, int nt, int kw, const void* X, int ldx, int M,
                            const void* W, int K, int N, const dsse::GemmEpi* ep, hipStream_t st);
hipError_t dsse_gemm_stream(int mode, int mt, int nt, int nw, int rd, int S, int partial_only, const void* X, int ldx, int M,
                            const void* W, int K, int N, const dsse::GemmEpi* ep, float* part, hipStream_t st);
hipError_t dsse_gemm_ring(int mode, int nw, int S, int partial_only, int ring2, const void* X, int ldx, int M,
                          const void* W, int K, int N, const dsse::GemmEpi* ep, float* part, hipStream_t st);
hipError_t dsse_gemm_wide(int mode, int mb, int rd, int S, int partial_only, const void* X, int ldx, int M, const void* W,
                          int K, int N, const dsse::GemmEpi* ep, float* part, hipStream_t st);
hipError_t dsse_gemm_tiled(int mode, int cfg, int S, int partial_only, const void* X, int ldx, int M, const void* W,
                           int K, int N, const dsse::GemmEpi* ep, float* part, hipStream_t st);
hipError_t dsse_gemm_pipe(int mode, int bm, int S, int partial_only, const void* X, int ldx, int M, const void* W,
                          int K, int N, const dsse::GemmEpi* ep, float* part, hipStream_t st);
size_t dsse_gemm_pipe_fix_floats(int bm, int S, int M, int N);
size_t dsse_gemm_ring_fix_floats(int nw, int S, int M, int N);
hipError_t dsse_paged_attention(int mode, int num_work, const dsse::AttnParams* p, hipStream_t st);
hipError_t dsse_flash_prefill(int num_work, const dsse::AttnParams* p, hipStream_t st);
hipError_t dsse_sample(int B, const dsse::SampleParams* p, hipStream_t st);
hipError_t dsse_sample_pick(int B, int world, const void* cand, const dsse::SampleParams* p,
                            hipStream_t st);
hipError_t dsse_prefill_sample_gather(const void* x, int T, int H, const int* meta, int NS, const int* slot_meta, int Bm,
                                      void* xl, int* smeta, hipStream_t st);
hipError_t dsse_prefill_sample_commit(const int* meta, int NS, const int* new_ids, int* ids, int Bm, int* ring, int R,
                                      int* positions, hipStream_t st);
hipError_t dsse_rmsnorm(int mode, int M, float* resid, int H, const void* delta, const void* embed,
                        const int* ids, const void* w, void* y, float eps, const float* part, int nsplit,
                        int vocab, hipStream_t st);
hipError_t dsse_rope_kv_write(int T, const void* qkv, int hq, int hkv, const int* positions,
                              const int* slots, const float2* rope, void* q_out, void* k_cache,
                              void* v_cache, int num_slots, int rope_len, hipStream_t st);
hipError_t dsse_silu_mul(int T, int F, const void* gu, void* h, hipStream_t st);
hipError_t dsse_decode_prep(int B, const int* active, const int* positions, const int* block_tables,
                            int max_blocks, int num_blocks, int* slots, int* ctx_len, int* q_len, hipStream_t st);
hipError_t dsse_ring_advance(int* counter, hipStream_t st);
// TP all-reduce + residual + RMSNorm over IPC peer buffers (allreduce.hip)
size_t dsse_ar_buffer_bytes(int rows, int H);
hipError_t dsse_ar_alloc(size_t bytes, void** ptr, void* handle64, int* uncached);
hipError_t dsse_ar_open(const void* handle64, void** ptr);
hipError_t dsse_ar_close(void* ptr, int opened);
hipError_t dsse_ar_rmsnorm(int M, const void* tmp, float* resid, const void* w, void* y, int H, float eps,
                           const unsigned long long* peers, int rank, int world, int rows, unsigned int* epoch,
                           unsigned int* err, const float* part, int nsplit, hipStream_t st);
hipError_t dsse_ar_gather(int M, const void* in, void* out, const unsigned long long* peers, int rank, int world,
                          int rows, int H, unsigned int* gepoch, unsigned int* err, hipStream_t st);
// Checked build: first out-of-range index per kernel file (line, value, bound, count); zeros otherwise.
hipError_t dsse_check_gemm_skinny(int* out, int clear);
hipError_t dsse_check_gemm_stream(int* out, int clear);
hipError_t dsse_check_attention(int* out, int clear);
hipError_t dsse_check_attention_prefill(int* out, int clear);
hipError_t dsse_check_elementwise(int* out, int clear);
hipError_t dsse_check_sampler(int* out, int clear);
hipError_t dsse_check_gemm_tiled(int* out, int clear);
// Stamps build: bind the step-anatomy record buffer (common.h stamps::) of a kernel file; no-ops otherwise.
hipError_t dsse_stamps_bind_gemm_stream(void* rec);
hipError_t dsse_stamps_bind_elementwise(void* rec);
}
