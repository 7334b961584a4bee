#!/bin/bash
# Full GPU pass: parity tests, bench per config, kernel-trace stats, PMC traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
O="$R/gpurun_out"
step() { echo "== $1"; }
step pytest
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-metric c2 c3 c4 seg}; do
  step "bench $c"
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  cat $O/bench_$c.json
done
for c in metric c4; do
  step "torchrun 2 ranks $c (gloo rehearsal on one GPU)"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --config $c --gpus 2 --backend gloo --steps 5 --warmup 2 > $O/bench_2rank_gloo_$c.json 2> $O/bench_2rank_gloo_$c.err || { tail -20 $O/bench_2rank_gloo_$c.err; exit 1; }
  cat $O/bench_2rank_gloo_$c.json
done
cd /tmp && export TMPDIR=/tmp
step "kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_metric -o bench -- python3 $R/bench.py > $O/prof_bench.json 2> $O/prof_bench.err || { tail $O/prof_bench.err; exit 1; }
python3 $R/tools/trace_steady.py $O/prof_metric/bench_kernel_trace.csv crc32c_batch_kernel 40 50 $O/prof_bench.json > $O/metric_kernel_steady.json && cat $O/metric_kernel_steady.json
for c in ${PMC_CONFIGS:-metric c2 c3 c4 seg}; do
  k=crc32c_batch_kernel; n=1; [ $c = c3 ] && k=crc64_batch_kernel; [ $c = seg ] && { k=seg_; n=5; }
  step "pmc fetch/write $c"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$c -o pmc -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch_$c.json 2> $O/pmc_fetch_$c.err || { tail $O/pmc_fetch_$c.err; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$c -o pmc -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write_$c.json 2> $O/pmc_write_$c.err || { tail $O/pmc_write_$c.err; exit 1; }
  python3 $R/tools/pmc_traffic.py $O/pmc_fetch_$c $O/pmc_write_$c $k $O/pmc_traffic_$c.json $(python3 $R/tools/alg_bytes.py $c) $n
done
