#!/bin/bash
# Parity suite on the working tree, then A/B of the working-tree library
# against the last commit's kernels (make prev) in one process.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
NO_SMOKE=1 NO_BENCH=1 bash tools/gpu_test.sh || exit $?
timeout -k 10 600 python tools/ab_variants.py --config ${AB_CONFIGS:-metric,c2,c3,c4} --variants ${AB_VARIANTS:-prev cur} \
  --rounds ${AB_ROUNDS:-6} --iters 5 --out gpurun_out/ab_prev.json > gpurun_out/ab_prev.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab_prev.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${LAT:-}" ]; then
  timeout -k 10 300 python tools/latency.py > gpurun_out/latency.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/latency.log; [ $rc -eq 0 ] || exit $rc
fi
for c in ${BENCH_CONFIGS:-}; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  cat gpurun_out/bench_$c.json
done
