#!/bin/bash
# Round-3 step M: non-temporal K/V loads in decode attention -- numerics, isolated attention, step A/B.
set -o pipefail
out=gpurun_out/${1:-r3m}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread \
  > $out/pytest.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/bench_attn.py --B 64,256 --ctx 560 --configs "KWV=2;KWV=4;KWV=1,PD=2;KWV=2,PD=2" > $out/attn_nt.log 2>&1 &&
DSSE_KERNELS_VARIANT=attdef timeout -k 10 200 python3 tools/bench_attn.py --B 64,256 --ctx 560 --configs "KWV=2;KWV=1,PD=2" > $out/attn_def.log 2>&1 || exit 1
bash tools/ab_multi.sh r3m_ab64.log 64 2 "-" "DSSE_KERNELS_VARIANT=attdef" || exit 1
bash tools/ab_multi.sh r3m_ab256.log 256 1 "-" "DSSE_KERNELS_VARIANT=attdef" "DSSE_ATTN_KWV=1" "DSSE_ATTN_KWV=4" || exit 1
mv gpurun_out/r3m_ab64.log gpurun_out/r3m_ab256.log $out/
