#!/bin/bash
# bench.py per config under rocprofv3 --kernel-trace --stats (one run each),
# then trace_steady.py: the rocprof mean of the timed dispatches next to
# bench.py's roofline.kernel_ms.  CONFIGS, OUT (under gpurun_out/), STEPS/WARMUP.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O="$R/gpurun_out/${OUT:-trace}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-metric c2 c3 c4}; do
  echo "== $c $(date +%T)"
  case $c in metric|c2|c4|c5|msgs) k=crc32c_batch;; c3) k=crc64_batch;; seg) k="seg_kernel<64, 1>";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o bench -- \
    python3 $R/bench.py --config $c --steps ${STEPS:-50} --warmup ${WARMUP:-40} > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
  cat $O/bench_$c.json
  python3 $R/tools/trace_steady.py $O/prof_$c/bench_kernel_trace.csv "$k" ${WARMUP:-40} ${STEPS:-50} $O/bench_$c.json > $O/${c}_kernel_steady.json || exit 1
  cat $O/${c}_kernel_steady.json
done
