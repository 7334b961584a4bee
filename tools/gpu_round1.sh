#!/bin/bash
# First GPU pass: smoke, parity tests, bench, kernel-trace profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log | tail -2
echo "== pytest gpu" && timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== rocprofv3 kernel trace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_metric" -o bench -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err" || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_bench.err"; exit 1; }
cat "$R/gpurun_out/prof_bench.json"
find "$R/gpurun_out/prof_metric" -name "*stats*" | head
