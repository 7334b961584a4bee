#!/bin/bash
# Round-5 pass at HEAD: the whole -m gpu suite, smoke(), the driver's N=1
# command (with its c5_strong sub-record), the torchrun 1-rank RCCL line, and
# a rocprofv3 kernel trace of the driver's command.  First failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out/r05
O="$R/gpurun_out/r05/${TAG:-final}"; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_TESTS" ]; then
  step "full suite"
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  tail -3 $O/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|^E " $O/pytest_gpu.log | head -60; exit $rc; }
  step "smoke"
  timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
step "driver command"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
cat $O/bench_driver.json
if [ -n "$BENCH_DEFAULT" ]; then
  step "bench defaults"
  timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
  cat $O/bench_default.json
fi
for c in ${CONFIGS:-}; do
  step "bench $c"
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  cat $O/bench_$c.json
done
if [ -z "$SKIP_NCCL" ]; then
  step "torchrun 1 rank nccl"
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 1 --steps 20 --warmup 10 > $O/bench_nccl_1rank.json 2> $O/bench_nccl_1rank.err || { tail -30 $O/bench_nccl_1rank.err; exit 1; }
  cat $O/bench_nccl_1rank.json
fi
for c in ${TRACE_CONFIGS:-}; do
  step "kernel trace $c (bench defaults)"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o bench -- python3 $R/bench.py --config $c --no-cpu-baseline > $O/prof_bench_$c.json 2> $O/prof_bench_$c.err || { tail $O/prof_bench_$c.err; exit 1; }
  cd "$R"
  k=crc64_batch_kernel; [ "$c" = seg ] && k=seg_kernel
  python3 tools/trace_steady.py $O/prof_$c/bench_kernel_trace.csv $k 40 50 $O/prof_bench_$c.json > $O/${c}_kernel_steady.json && cat $O/${c}_kernel_steady.json
done
if [ -z "$SKIP_TRACE" ]; then
  step "kernel trace of the driver command"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o bench -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_bench_driver.json 2> $O/prof_bench_driver.err || { tail $O/prof_bench_driver.err; exit 1; }
  cd "$R"
  python3 tools/trace_steady.py $O/prof_driver/bench_kernel_trace.csv crc32c_batch_kernel 5 20 $O/prof_bench_driver.json > $O/metric_kernel_steady.json && cat $O/metric_kernel_steady.json
fi
