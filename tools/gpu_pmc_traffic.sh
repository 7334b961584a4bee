#!/bin/bash
# HBM traffic per launch for one config: FETCH_SIZE and WRITE_SIZE passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${CONFIGS:-c4}; do
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tr_${c}_f -o p -- python3 $R/tools/kernel_run.py --config $c --iters 4 > $O/tr_${c}_f.log 2>&1 || { tail $O/tr_${c}_f.log; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/tr_${c}_w -o p -- python3 $R/tools/kernel_run.py --config $c --iters 4 > $O/tr_${c}_w.log 2>&1 || { tail $O/tr_${c}_w.log; exit 1; }
  python3 $R/tools/pmc_traffic.py $O/tr_${c}_f $O/tr_${c}_w batch_kernel $O/pmc_traffic_$c.json
done
