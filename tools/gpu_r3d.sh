#!/bin/bash
# Round-3 step D: per-CU fill-rate microbenchmark, config 5 with the subscription-aware load generator.
out=gpurun_out/${1:-r3d}
mkdir -p $out
timeout -k 10 120 ./tools/fillbench > $out/fillbench.log 2>&1
echo "fillbench rc=$?" >> $out/fillbench.log
bash tools/config5_box.sh r3d/config5
