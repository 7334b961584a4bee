#!/bin/bash
# Round-4 final pass at HEAD: the whole -m gpu suite, smoke(), the driver's
# N=1 command, every bench config, the torchrun 1-rank RCCL line, a rocprofv3
# kernel trace of the driver's command (its timed-dispatch mean) and of the
# changed CRC-64 paths, and the PMC traffic passes of the kernels that changed
# this round.  First failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out/r04
O="$R/gpurun_out/r04"
if [ -z "$SKIP_TESTS" ]; then
  PART="tests" bash tools/gpu_r04.sh || exit 1
  echo "== smoke $(date +%T)"
  timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
PART=driver bash tools/gpu_r04.sh || exit 1
PART=bench CONFIGS="${CONFIGS:-c2 c3 c4 c5 seg msgs xdr}" bash tools/gpu_r04.sh || exit 1
PART=nccl CONFIGS="c5 metric" BENCH_ARGS="--steps 20 --warmup 10" bash tools/gpu_r04.sh || exit 1
PART=trace CONFIGS=metric BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_r04.sh || exit 1
python3 tools/trace_steady.py $O/prof_metric/bench_kernel_trace.csv crc32c_batch_kernel 5 20 $O/prof_bench_metric.json > $O/metric_kernel_steady.json && cat $O/metric_kernel_steady.json
if [ -n "$PMC" ]; then
  PART=pmc CONFIGS="$PMC" bash tools/gpu_r04.sh || exit 1
fi
