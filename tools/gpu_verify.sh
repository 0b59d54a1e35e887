set -o pipefail
out=gpurun_out/${1:-v5}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $out/bench64.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $out/bench64b.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --streams 256 > $out/bench256.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof64 -o run -- python3 bench.py --steps 12 --warmup 3 > $out/prof64.log 2>&1
