#!/bin/bash
# Round-2 measurement pass: bench.py per config, rocprofv3 kernel-trace
# summaries, PMC HBM traffic per config (FETCH_SIZE / WRITE_SIZE passes of
# tools/kernel_run.py), end-to-end host->device rate.  PART selects a subset.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out/r02
O="$R/gpurun_out/r02"
step() { echo "== $1 $(date +%T)"; }
if [ "${PART:-bench}" = bench ]; then
  for c in ${CONFIGS:-metric c2 c3 c4 c5 seg msgs}; do
    step "bench $c"
    timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
    cat $O/bench_$c.json
  done
  step "bench driver-style"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
  cat $O/bench_driver.json
fi
if [ "${PART:-bench}" = trace ]; then
  cd /tmp && export TMPDIR=/tmp
  for c in ${CONFIGS:-metric c3 c4}; do
    step "kernel trace $c"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o bench -- python3 $R/bench.py --config $c > $O/prof_bench_$c.json 2> $O/prof_bench_$c.err || { tail $O/prof_bench_$c.err; exit 1; }
    cat $O/prof_bench_$c.json
  done
fi
if [ "${PART:-bench}" = pmc ]; then
  cd /tmp && export TMPDIR=/tmp
  for c in ${CONFIGS:-metric c2 c3 c4 c5 msgs}; do
    k=batch_kernel
    step "pmc $c"
    timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tr_${c}_f -o p -- python3 $R/tools/kernel_run.py --config $c --iters 4 > $O/tr_${c}_f.log 2>&1 || { tail $O/tr_${c}_f.log; exit 1; }
    timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/tr_${c}_w -o p -- python3 $R/tools/kernel_run.py --config $c --iters 4 > $O/tr_${c}_w.log 2>&1 || { tail $O/tr_${c}_w.log; exit 1; }
    python3 $R/tools/pmc_traffic.py $O/tr_${c}_f $O/tr_${c}_w $k $O/pmc_traffic_$c.json $(python3 $R/tools/alg_bytes.py $c) 1 4 || exit 1
  done
fi
if [ "${PART:-bench}" = e2e ]; then
  step "e2e"
  timeout -k 10 300 python tools/e2e_h2d.py --reps 7 --out $O/e2e_h2d.json > $O/e2e.log 2>&1 || { tail $O/e2e.log; exit 1; }
  cat $O/e2e_h2d.json
fi
