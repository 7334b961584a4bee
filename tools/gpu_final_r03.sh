#!/bin/bash
# Round-3 final pass at HEAD: the whole -m gpu suite, smoke(), the driver's
# N=1 command, every bench config, and a rocprofv3 kernel trace of the
# driver's command (its timed-dispatch mean).  First failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out/r03
O="$R/gpurun_out/r03"
PART="tests driver" bash tools/gpu_r03.sh || exit 1
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
PART=bench CONFIGS="${CONFIGS:-c2 c3 c4 c5 seg msgs xdr}" bash tools/gpu_r03.sh || exit 1
PART=trace CONFIGS=metric BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu_r03.sh || exit 1
python3 tools/trace_steady.py $O/prof_metric/bench_kernel_trace.csv crc32c_batch_kernel 5 20 $O/prof_bench_metric.json > $O/metric_kernel_steady.json && cat $O/metric_kernel_steady.json
