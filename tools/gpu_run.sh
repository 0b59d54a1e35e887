#!/bin/bash
# One parameterised GPU-box session (replaces the per-experiment tools/gpu_r3*.sh scripts).
#   tools/gpu_run.sh OUTDIR STEP [STEP ...]
# Steps (each under its own time limit; a crash, fault or timeout ends the session at once):
#   model_test    tests/test_model_full_dims_gpu.py      ar_test       tests/test_custom_ar_gpu.py
#   gemm_test     tests/test_gemm_tiled_gpu.py           tp_test       tests/test_tp_gpu.py
#   bench64       bench.py (driver form, 64 streams)     ttft512       tools/bench_ttft.py --prompt-len 512
#   gpu_tests     the whole GPU suite (pytest -m gpu)    smoke         __graft_entry__.smoke()
#   bench256      bench.py --streams 256                 prof64        rocprofv3 kernel trace of bench.py
#   ttft8k        tools/bench_ttft.py --prompt-len 8192  c3stub        8 paced stub replicas x 256 streams (CPU only)
#   attn_bench    tools/bench_prefill_attn.py (8k / 512 causal, + SDPA arm)
#   gemm_bench    tools/bench_gemm_tiled.py at M = 8192 and 256 (engine dispatch vs library)
#   attn_test     tests/test_kernels_gpu.py -k prefill     pmc_attn / pmc_gemm  two rocprofv3 --pmc passes each
#   kern_test     tests/test_kernels_gpu.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" >> "$out/session.log"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> "$out/session.log"
  tail -3 "$out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
for s in "$@"; do
  case $s in
    tp_test) step tp_test 600 $PYT tests/test_tp_gpu.py ;;
    model_test) step model_test 600 $PYT tests/test_model_full_dims_gpu.py ;;
    ar_test) step ar_test 900 $PYT tests/test_custom_ar_gpu.py ;;
    gpu_tests) step gpu_tests 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench64) step bench64 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench256) step bench256 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 256 ;;
    bench192) step bench192 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 192 ;;
    bench256b) step bench256b 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 256 ;;
    prof64) step prof64 600 rocprofv3 --kernel-trace --stats -d "$out/prof64" -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 ;;
    prof256kwv4) DSSE_KERNEL_CFG=attn_kwv=4 step prof256kwv4 600 rocprofv3 --kernel-trace --stats -d "$out/prof256kwv4" -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --streams 256 ;;
    prof256) step prof256 600 rocprofv3 --kernel-trace --stats -d "$out/prof256" -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --streams 256 ;;
    ttft8k) step ttft8k 600 python3 tools/bench_ttft.py --prompt-len 8192 ;;
    ttft512) step ttft512 600 python3 tools/bench_ttft.py --prompt-len 512 ;;
    profttft8k)
      step profttft8k 600 rocprofv3 --kernel-trace -d "$out/profttft8k" -o run --output-format csv -- python3 tools/bench_ttft.py --prompt-len 8192 --decode-steps 0 --profile-marker
      python3 tools/trace_sum.py "$(ls "$out"/profttft8k/*/run_kernel_trace.csv "$out"/profttft8k/run_kernel_trace.csv 2>/dev/null | head -1)" --div 3 --after-kernel bitwise_not --title "8k-token prefill, per prompt (3 timed prompts, setup and warm-up excluded)" > "$out/profttft8k.md" 2>&1 ;;
    profttft512)
      step profttft512 600 rocprofv3 --kernel-trace -d "$out/profttft512" -o run --output-format csv -- python3 tools/bench_ttft.py --prompt-len 512 --decode-steps 0 --profile-marker
      python3 tools/trace_sum.py "$(ls "$out"/profttft512/*/run_kernel_trace.csv "$out"/profttft512/run_kernel_trace.csv 2>/dev/null | head -1)" --div 3 --after-kernel bitwise_not --title "512-token prefill, per prompt (3 timed prompts, setup and warm-up excluded)" > "$out/profttft512.md" 2>&1 ;;
    c3stub) HIP_VISIBLE_DEVICES= DSSE_DIST_BACKEND=gloo step c3stub 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 8 --streams 256 --steps 64 --warmup 8 --stub-step-ms 9.7 ;;
    serving13) step serving13 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 --prefill-budget 512 --itl-ratios 0,2 ;;
    serving13b) step serving13b 900 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 --prefill-budget 256,512 --itl-ratios 0 ;;
    overlap) step overlap 600 python3 tools/bench_overlap.py --streams 128 --ctx 512 --prompt 512 && step overlap64 600 python3 tools/bench_overlap.py --streams 64 --ctx 512 --prompt 512 ;;
    serving13_mx512) DSSE_MIXED=1 DSSE_MIXED_CHUNK=512 step serving13_mx512 900 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 --prefill-budget 512 --itl-ratios 0 ;;
    serving13_mx256) DSSE_MIXED=1 DSSE_MIXED_CHUNK=256 step serving13_mx256 900 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 --prefill-budget 512 --itl-ratios 0 ;;
    serving40_mx512) DSSE_MIXED=1 DSSE_MIXED_CHUNK=512 step serving40_mx512 900 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 --prefill-budget 512 --itl-ratios 0 ;;
    serving40_mx256) DSSE_MIXED=1 DSSE_MIXED_CHUNK=256 step serving40_mx256 900 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 --prefill-budget 512 --itl-ratios 0 ;;
    serving13_mx256_d0) DSSE_PIPELINE_DEPTH=0 DSSE_MIXED=1 DSSE_MIXED_CHUNK=256 step serving13_mx256_d0 900 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 --prefill-budget 512 --itl-ratios 0 ;;
    sdef13) step sdef13 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 ;;
    sdef40) step sdef40 600 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 ;;
    sdef13j08) DSSE_JIT_MARGIN_MS=0.8 step sdef13j08 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 ;;
    sdef40j08) DSSE_JIT_MARGIN_MS=0.8 step sdef40j08 600 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 ;;
    sdef13nojit) DSSE_JIT_MARGIN_MS=0 step sdef13nojit 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 ;;
    mixedb) step mixedb 300 python3 tools/bench_mixed.py --streams 64,128 ;;
    launch_env_ab)  # HIP runtime launch settings vs the default, 64-stream step (graph replays)
      step "le_default" 300 python3 bench.py --gpus 1 --steps 40 --warmup 5
      HIP_FORCE_DEV_KERNARG=1 step "le_devkernarg" 300 python3 bench.py --gpus 1 --steps 40 --warmup 5
      DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 step "le_nopacketcap" 300 python3 bench.py --gpus 1 --steps 40 --warmup 5
      DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 step "le_packetcap" 300 python3 bench.py --gpus 1 --steps 40 --warmup 5
      step "le_default2" 300 python3 bench.py --gpus 1 --steps 40 --warmup 5 ;;
    tp8_rank) step tp8_rank 300 python3 tools/bench_tp_rank.py --tp 8 ;;
    tp8_attn)  # decode attention partitions at TP = 8 (one kv head, 64 streams): 512 / 256 / 128 / 64 workgroups
      for wg in 256 128 64; do step "tp8_attn$wg" 300 python3 tools/bench_tp_rank.py --tp 8 --phase decode --attn-wgs $wg; done ;;
    tp8_chunks)  # TP = 8 rank prefill compute with 2 row chunks and unchunked (default 4)
      DSSE_TP_PREFILL_CHUNKS=2 step tp8_chunks2 300 python3 tools/bench_tp_rank.py --tp 8 --phase prefill
      DSSE_TP_PREFILL_CHUNKS=1 step tp8_chunks1 300 python3 tools/bench_tp_rank.py --tp 8 --phase prefill ;;
    tp8_split_ab)  # flash key split: ranges sized for one round of 256 workgroups (default) vs the plain length rule
      for i in 1 2; do
        DSSE_TP_PREFILL_CHUNKS=1 step "tp8_split_oneround$i" 300 python3 tools/bench_tp_rank.py --tp 8 --phase prefill
        DSSE_TP_PREFILL_CHUNKS=1 step "tp8_split_anyround$i" 300 python3 tools/bench_tp_rank.py --tp 8 --phase prefill --split-any-rounds
      done ;;
    tp_ranks24)  # one TP = 2 / 4 rank of Mistral-7B (per-rank compute, as tp8_rank)
      step tp2_rank 300 python3 tools/bench_tp_rank.py --tp 2
      step tp4_rank 300 python3 tools/bench_tp_rank.py --tp 4 ;;
    attn_comb_ab)  # decode partitions merged by their last arriver (default) vs attn_combine_kernel, TP = 8 rank
      for i in 1 2; do
        step "tp8_comb$i" 300 python3 tools/bench_tp_rank.py --tp 8 --phase decode
        DSSE_KERNEL_CFG=attn_comb=0 step "tp8_nocomb$i" 300 python3 tools/bench_tp_rank.py --tp 8 --phase decode
      done ;;
    attn_tests) step attn_tests 600 $PYT tests/test_kernels_gpu.py -k "paged_attention_decode or qkv_attention_decode or folded" tests/test_tp_gpu.py tests/test_tp_graph_gpu.py ;;
    tp8_fix_ab)  # TP = 8 rank prefill: the cost model with (default) and without (t_fix=0) the in-launch fix-up
      for i in 1 2; do
        step "tp8_pf_fix$i" 300 python3 tools/bench_tp_rank.py --tp 8 --phase prefill
        DSSE_KERNEL_CFG=t_fix=0 step "tp8_pf_nofix$i" 300 python3 tools/bench_tp_rank.py --tp 8 --phase prefill
      done ;;
    tp8_host) step tp8_host 300 python3 tools/bench_tp_rank.py --tp 8 --phase prefill --iters 2 --host-profile ;;
    runner_test) step runner_test 600 $PYT tests/test_model_runner.py tests/test_model_full_dims_gpu.py -m gpu ;;
    checked_r6)  # the device index-check build: the checked-kernel tool, and the round-6 attention paths under it
      DSSE_KERNELS_VARIANT=checked step check_kernels 300 python3 tools/check_kernels.py
      DSSE_KERNELS_VARIANT=checked step checked_attn 600 $PYT tests/test_kernels_gpu.py -k "key_split or even_partitions or one_kv_head or folded_even" tests/test_model_runner.py -m gpu ;;
    tp8_rank_nofix) DSSE_KERNEL_CFG=s_fix=0 step tp8_rank_nofix 300 python3 tools/bench_tp_rank.py --tp 8 ;;
    r6_tests2) step r6_tests2 900 $PYT tests/test_kernels_gpu.py -k "ring_silu or tp8_shard or ring_lds or gemm_silu or resid_split" tests/test_tp_graph_gpu.py tests/test_custom_ar_gpu.py ;;
    flash_tp8)  # a TP = 8 rank's prompt attention (4 q heads, 1 kv head): q-head split 4 (whole group) / 2 / 1
      for hg in 4 2 1; do DSSE_KERNEL_CFG=flash_hg=$hg step "flash_tp8_hg$hg" 300 python -u tools/bench_prefill_attn.py --T 8192,2048 --hq 4 --hkv 1; done ;;
    prof_tp8)  # kernel traces of one TP = 8 rank: 64-stream decode step and 8k prefill
      step prof_tp8_dec 300 rocprofv3 --kernel-trace -d "$out/prof_tp8_dec" -o run --output-format csv -- python3 tools/bench_tp_rank.py --tp 8 --phase decode --steps 20 --profile-marker
      python3 tools/trace_sum.py "$(ls "$out"/prof_tp8_dec/*/run_kernel_trace.csv "$out"/prof_tp8_dec/run_kernel_trace.csv 2>/dev/null | head -1)" --div 20 --after-kernel bitwise_not --title "TP=8 rank 0, 64-stream decode step (20 replays)" > "$out/prof_tp8_dec.md" 2>&1
      step prof_tp8_pf 300 rocprofv3 --kernel-trace -d "$out/prof_tp8_pf" -o run --output-format csv -- python3 tools/bench_tp_rank.py --tp 8 --phase prefill --iters 3 --profile-marker
      python3 tools/trace_sum.py "$(ls "$out"/prof_tp8_pf/*/run_kernel_trace.csv "$out"/prof_tp8_pf/run_kernel_trace.csv 2>/dev/null | head -1)" --div 3 --after-kernel bitwise_not --title "TP=8 rank 0, 8192-token prefill (3 prompts)" > "$out/prof_tp8_pf.md" 2>&1 ;;
    stamps64)  # step anatomy from in-kernel stamps (stamps build) + the same runner's counters (eager steps)
      DSSE_KERNELS_VARIANT=stamps step stamps64 300 python3 tools/step_stamps.py --streams 64 --steps 2 --out "$out/stamps64.json.gz" ;;
    pmc64)
      step pmc64_a 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES -d "$out/pmc64_a" -o run --output-format csv -- python3 tools/step_stamps.py --pmc-pass --steps 3 --warmup 1
      step pmc64_b 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum -d "$out/pmc64_b" -o run --output-format csv -- python3 tools/step_stamps.py --pmc-pass --steps 3 --warmup 1
      step pmc64_c 180 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc64_c" -o run --output-format csv -- python3 tools/step_stamps.py --pmc-pass --steps 3 --warmup 1
      python3 tools/pmc_sum.py "$out/pmc64_a" "$out/pmc64_b" "$out/pmc64_c" --kernel "gemm_ring|rmsnorm_kernel<3>|paged_attention" --title "64-stream decode step kernels (eager steps)" > "$out/pmc64.md" 2>&1 ;;
    r6_tests3) step r6_tests3 900 $PYT tests/test_kernels_gpu.py -k "one_kv_head or ring_silu or paged_attention_prefill" ;;
    r6_tests) step r6_tests 900 $PYT tests/test_kernels_gpu.py -k "tp8_shard or even_partitions or paged_attention_decode or folded" tests/test_custom_ar_gpu.py tests/test_gemm_tiled_gpu.py tests/test_model_full_dims_gpu.py tests/test_tp_graph_gpu.py ;;
    soak) step soak 900 python3 tools/bench_serving.py --rates 40 --requests 2000 --max-tokens 200 ;;
    serving40) step serving40 600 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 --prefill-budget 256,512 --itl-ratios 0,2 ;;
    gemm_test) step gemm_test 600 $PYT tests/test_gemm_tiled_gpu.py ;;
    kern_test) step kern_test 900 $PYT tests/test_kernels_gpu.py ;;
    attn_test) step attn_test 300 $PYT tests/test_kernels_gpu.py -k "prefill or rope_kv" ;;
    folded_test) step folded_test 300 $PYT tests/test_kernels_gpu.py -k "folded" ;;
    flash_stamps) DSSE_FLASH_STAMPS="$out/fs.bin" step flash_stamps 300 python -u tools/bench_prefill_attn.py --T 8192
      python3 tools/flash_stamps.py "$out/fs.bin" > "$out/flash_stamps.md" 2>&1 ;;
    attn_bench) step attn_bench 300 python -u tools/bench_prefill_attn.py --T 8192,2048,512 --sdpa ;;
    gemm_bench) step gemm_bench 300 python -u tools/bench_gemm_tiled.py --M 8192,256 --cfg auto ;;
    gemm_mid) step gemm_mid 300 python -u tools/bench_gemm_tiled.py --M 1024,512 --cfg auto ;;
    gemm_wide) step gemm_wide 300 python -u tools/bench_gemm_tiled.py --M 256,192 --cfg auto,0,1,5 --no-library ;;
    pmc_attn)
      step pmc_attn_a 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES -d "$out/pmc_attn_a" -o run --output-format csv -- python3 tools/bench_prefill_attn.py --T 8192 --rounds 1 --iters 3
      step pmc_attn_b 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum -d "$out/pmc_attn_b" -o run --output-format csv -- python3 tools/bench_prefill_attn.py --T 8192 --rounds 1 --iters 3
      python3 tools/pmc_sum.py "$out/pmc_attn_a" "$out/pmc_attn_b" --kernel flash_prefill --title "flash prefill, 8k causal, 32/8 heads" > "$out/pmc_attn.md" 2>&1 ;;
    pmc_gemm8k_ta)  # the 8192-row gate_up pipe GEMM: texture-address / LDS-DMA load path (2 TA counters per pass)
      step pmc_g8k_ta 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY -d "$out/pmc_g8k_ta" -o run --output-format csv -- python3 tools/bench_gemm_tiled.py --M 8192 --shapes gate_up --cfg auto --no-library --rounds 1 --iters 3
      python3 tools/pmc_sum.py "$out/pmc_g8k_ta" --kernel gemm_pipe --title "gate_up GEMM at M = 8192: load path" > "$out/pmc_g8k_ta.md" 2>&1 ;;
    pmc_gemm)
      step pmc_gemm_a 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES -d "$out/pmc_gemm_a" -o run --output-format csv -- python3 tools/bench_gemm_tiled.py --M 8192,256 --shapes gate_up --cfg auto --no-library --rounds 1 --iters 3
      step pmc_gemm_b 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum -d "$out/pmc_gemm_b" -o run --output-format csv -- python3 tools/bench_gemm_tiled.py --M 8192,256 --shapes gate_up --cfg auto --no-library --rounds 1 --iters 3
      python3 tools/pmc_sum.py "$out/pmc_gemm_a" "$out/pmc_gemm_b" --kernel gemm --title "gate_up GEMM (N 28672, K 4096) at M = 8192 and 256" > "$out/pmc_gemm.md" 2>&1 ;;
    tiled_ab)  # gemm_tiled stage-issue order: spread (default build) vs one burst (kernels-burst build)
      for v in "" burst; do
        DSSE_KERNELS_VARIANT=$v step "tiled_ab_qkv_$v" 300 python -u tools/bench_decode_gemm.py --shape qkv --M 160,256,384,512 --variants out &&
        DSSE_KERNELS_VARIANT=$v step "tiled_ab_o_$v" 300 python -u tools/bench_decode_gemm.py --shape o,down --M 160,256,384,512 --variants split_norm &&
        DSSE_KERNELS_VARIANT=$v step "tiled_ab_gu_$v" 300 python -u tools/bench_decode_gemm.py --shape gate_up --M 160,256,384,512 --variants silu
      done ;;
    mall)  # decode GEMMs with weights cycling through HBM (1.2 GB of copies) vs two copies resident in the MALL
      step mall_cold 300 python -u tools/bench_decode_gemm.py --shape qkv,o,down --M 64,128,256 --variants out,split_norm &&
      step mall_hot 300 python -u tools/bench_decode_gemm.py --shape qkv,o,down --M 64,128,256 --variants out,split_norm --bytes 1 ;;
    pipe192)  # gemm_pipe on the 192-row tile (cfg 9) vs the default pick at 129-384 rows
      step pipe192_qkv 300 python -u tools/bench_decode_gemm.py --shape qkv --M 160,192,320,384 --variants out,out:t_cfg=9,out:t_cfg=8 &&
      step pipe192_gu 300 python -u tools/bench_decode_gemm.py --shape gate_up --M 160,192,320,384 --variants silu,silu:t_cfg=9,silu:t_cfg=8 &&
      step pipe192_od 300 python -u tools/bench_decode_gemm.py --shape o,down --M 160,192,320,384 --variants split_norm,split_norm:t_cfg=9,split_norm:t_cfg=8 ;;
    pipe128)  # gemm_pipe on a 128-row tile (cfg 10) vs the default pick and cfg 9 at 129-256 rows
      step pipe128_qkv 300 python -u tools/bench_decode_gemm.py --shape qkv --M 128,192,256 --variants out,out:t_cfg=10,out:t_cfg=9 &&
      step pipe128_gu 300 python -u tools/bench_decode_gemm.py --shape gate_up --M 128,192,256 --variants silu,silu:t_cfg=10,silu:t_cfg=9 &&
      step pipe128_od 300 python -u tools/bench_decode_gemm.py --shape o,down --M 128,192,256 --variants split_norm,split_norm:t_cfg=10,split_norm:t_cfg=9 &&
      DSSE_KERNEL_CFG=t_cfg=10 step pipe128_test 300 $PYT tests/test_gemm_tiled_gpu.py -k "silu or resid or qkv" ;;
    small_ab)  # 256-stream step: cfg 9 / 10 picks for the decode buckets' qkv / down (default) vs t_small=0, alternating
      for i in 1 2; do
        step "small_on_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 256 &&
        DSSE_KERNEL_CFG=t_small=0 step "small_off_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 256
      done ;;
    pd_ab)  # 256-stream step: one-wave decode attention with a 2-page register ring (attn_pd=2) vs one page, alternating
      for i in 1 2; do
        step "pd1_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 256 &&
        DSSE_KERNEL_CFG=attn_pd=2 step "pd2_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 256
      done ;;
    split_sweep)  # split-K / tile sweep for the narrow projections at the mixed steps' and the 256 bucket's rows
      step sweep_qkv 300 python -u tools/bench_decode_gemm.py --shape qkv --M 256,384 --variants "out,out:t_cfg=9;t_split=2,out:t_cfg=9;t_split=8,out:t_cfg=10;t_split=2,out:t_cfg=10;t_split=8" &&
      step sweep_o 300 python -u tools/bench_decode_gemm.py --shape o --M 256,384 --variants "split_norm,split_norm:t_cfg=9;t_split=4,split_norm:t_cfg=9;t_split=8,split_norm:t_cfg=10;t_split=4,split_norm:t_cfg=10;t_split=8,split_norm:t_cfg=0;t_split=2,split_norm:t_cfg=1;t_split=2" &&
      step sweep_down 300 python -u tools/bench_decode_gemm.py --shape down --M 256,384 --variants "split_norm,split_norm:t_cfg=9;t_split=4,split_norm:t_cfg=10;t_split=4,split_norm:t_cfg=10;t_split=16" ;;
    jit_ab)  # 13 req/s serving: JIT margin 1.5 ms (default) vs 1.1 ms, alternating
      for i in 1 2; do
        step "jit15_$i" 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 &&
        DSSE_JIT_MARGIN_MS=1.1 step "jit11_$i" 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000
      done ;;
    ratio_ab)  # mixed-step ITL ratio 2.0 vs the default 1.85, at 40 and 13 req/s
      step r20_40 600 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 --itl-ratios 2.0 &&
      step r185_40 600 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 &&
      step r20_13 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 --itl-ratios 2.0 ;;
    attn_decode)  # decode attention alone (mode 0) at 64 / 256 sequences: key-split waves and pages in flight
      step attn_decode 300 python -u tools/bench_attn.py --B 64,256 --ctx 560 --configs "KWV=1;KWV=1,PD=2;KWV=2;KWV=2,PD=2;KWV=4" ;;
    kwv_ab)  # 256-stream step: decode attention key-split waves (folded QKV epilogue or not), alternating
      for i in 1 2; do
        step "kwv_def_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 256 &&
        DSSE_KERNEL_CFG=attn_kwv=4 step "kwv_4_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 256 &&
        DSSE_KERNEL_CFG=attn_kwv=2 step "kwv_2_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 256
      done ;;
    kwv64_ab)  # 64-stream step: decode attention key-split waves 2 (default) vs 4, alternating
      for i in 1 2; do
        step "kwv64_def_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 &&
        DSSE_KERNEL_CFG=attn_kwv=4 step "kwv64_4_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
      done ;;
    qboost_ab)  # serving at 40 / 13 req/s: largest mixed chunk when prompts queue (default) vs ratio-sized chunks
      step qb40_on 600 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 &&
      step qb40_off 600 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 --no-queue-boost &&
      step qb13_on 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 &&
      step qb40_on2 600 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 &&
      step qb40_off2 600 python3 tools/bench_serving.py --rates 40 --requests 600 --max-tokens 200 --no-queue-boost ;;
    qboost13_ab)  # serving at 13 req/s: queue boost on (default) vs off, alternating
      for i in 1 2; do
        step "qb13_on_$i" 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 &&
        step "qb13_off_$i" 600 python3 tools/bench_serving.py --rates 13 --requests 600 --max-tokens 1000 --no-queue-boost
      done ;;
    o512)  # o projection (+ norm) at 448-512 rows: default (256x128 split) vs the pipe tiles
      step o512 300 python -u tools/bench_decode_gemm.py --shape o --M 448,512 --variants "split_norm,split_norm:t_cfg=10;t_split=4,split_norm:t_cfg=10;t_split=2,split_norm:t_cfg=8;t_split=4,split_norm:t_cfg=8;t_split=8,split_norm:t_cfg=1;t_split=2" ;;
    small192_ab)  # 192-stream step: cfg 9 / 10 picks for qkv / down (default) vs t_small=0, alternating
      for i in 1 2; do
        step "s192_on_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 192 &&
        DSSE_KERNEL_CFG=t_small=0 step "s192_off_$i" 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 192
      done ;;
    m128)  # the 65-128-row bucket: default kernels (ring2 / gemm_wide) vs the tiled / pipe kernels forced
      step m128_gu 300 python -u tools/bench_decode_gemm.py --shape gate_up --M 96,128 --variants "silu,silu:gemm_impl=4;t_cfg=5,silu:gemm_impl=4;t_cfg=10,silu:gemm_impl=4;t_cfg=8" &&
      step m128_qkv 300 python -u tools/bench_decode_gemm.py --shape qkv,down --M 128 --variants "split_norm,split_norm:gemm_impl=4;t_cfg=10,split_norm:gemm_impl=4;t_cfg=5,split_norm:gemm_impl=4;t_cfg=1" ;;
    m256bm)  # 256 rows: 256-row tiles (X re-read less) for o / qkv / down vs the defaults
      step m256bm 300 python -u tools/bench_decode_gemm.py --shape o,qkv,down --M 256 --variants "split_norm,split_norm:t_cfg=0;t_split=4,split_norm:t_cfg=0;t_split=8,split_norm:t_cfg=8;t_split=8,split_norm:t_cfg=8;t_split=16" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done"
