#!/bin/bash
# tools/overlap_probe.py with 1, 2 and 4 pool streams, each under a kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05/overlap; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for s in ${STREAMS:-1 2 4 1 2}; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t_${i}_$s -o k -- python3 $R/tools/overlap_probe.py --streams $s > $O/run_${i}_$s.json 2> $O/run_${i}_$s.err || { tail $O/run_${i}_$s.err; exit 1; }
  cat $O/run_${i}_$s.json
  python3 $R/tools/overlap_probe.py --analyze $O/t_${i}_$s/k_kernel_trace.csv | tr -d '\n'; echo
done
