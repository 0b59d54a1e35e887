set -o pipefail
mkdir -p gpurun_out/v4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v4/pytest.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/v4/bench64.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --streams 256 > gpurun_out/v4/bench256.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v4/prof64 -o run -- python3 bench.py --steps 12 --warmup 3 > gpurun_out/v4/prof64.log 2>&1
