#!/bin/bash
# Round-3 step A on MI355X: row-split RMSNorm numerics + whole-model numerics, A/B at 64 / 256 streams, profile.
set -o pipefail
out=gpurun_out/${1:-r3a}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "rmsnorm or resid_split" tests/test_model_full_dims_gpu.py \
  -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
bash tools/ab_env.sh r3a_norm64.log 64 "DSSE_NORM_SPLIT=0" "DSSE_NORM_SPLIT=1" 2 &&
bash tools/ab_env.sh r3a_norm256.log 256 "DSSE_NORM_SPLIT=0" "DSSE_NORM_SPLIT=1" 1 &&
mv gpurun_out/r3a_norm64.log gpurun_out/r3a_norm256.log $out/ &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof64 -o run -- python3 bench.py --steps 12 --warmup 3 > $out/prof64.log 2>&1
