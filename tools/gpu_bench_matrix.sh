#!/bin/bash
# bench.py lines: the driver's N=1 command, the self-launching 2-rank gloo
# rehearsal on one GPU (default N>1 config = C5 split; C4 global split).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
cat $O/bench_driver.json
for c in ${CONFIGS2:-c5 c4}; do
  timeout -k 10 300 python bench.py --gpus 2 --backend gloo --config $c --steps 5 --warmup 2 > $O/bench_2rank_$c.json 2> $O/bench_2rank_$c.err || { tail -20 $O/bench_2rank_$c.err; exit 1; }
  cat $O/bench_2rank_$c.json
done
