#!/bin/bash
# Full GPU pass: parity tests, bench per config, kernel-trace stats, PMC traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
O="$R/gpurun_out"
step() { echo "== $1"; }
step pytest
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1; rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-metric c2 c3 c4}; do
  step "bench $c"
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  cat $O/bench_$c.json
done
step "torchrun 2 ranks (gloo rehearsal on one GPU)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err || { tail -20 $O/bench_2rank_gloo.err; exit 1; }
cat $O/bench_2rank_gloo.json
cd /tmp && export TMPDIR=/tmp
step "kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_metric -o bench -- python3 $R/bench.py > $O/prof_bench.json 2> $O/prof_bench.err || { tail $O/prof_bench.err; exit 1; }
step "pmc fetch"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { tail $O/pmc_fetch.err; exit 1; }
step "pmc write"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write.json 2> $O/pmc_write.err || { tail $O/pmc_write.err; exit 1; }
python3 $R/tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write crc32c_batch_kernel $O/pmc_traffic_metric.json 4295229440
