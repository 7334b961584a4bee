#!/bin/bash
# CRC-64 PMC passes: HBM traffic of c3 (kernel_run) and seg (bench.py's
# segments layout, 5 dispatches per call), then the SQ/LDS counters of c3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
[ -n "${SKIP_C3:-}" ] || CONFIGS=c3 bash $R/tools/gpu_pmc_traffic.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tr_seg_f -o p -- python3 $R/bench.py --config seg --steps 4 --warmup 1 --no-cpu-baseline > $O/tr_seg_f.log 2>&1 || { tail $O/tr_seg_f.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/tr_seg_w -o p -- python3 $R/bench.py --config seg --steps 4 --warmup 1 --no-cpu-baseline > $O/tr_seg_w.log 2>&1 || { tail $O/tr_seg_w.log; exit 1; }
python3 $R/tools/pmc_traffic.py $O/tr_seg_f $O/tr_seg_w seg_ $O/pmc_traffic_seg.json 8590589960 5 || exit 1
CONFIGS=c3 bash $R/tools/gpu_pmc.sh > $O/sq_c3.txt 2>&1 || { tail $O/sq_c3.txt; exit 1; }
cat $O/sq_c3.txt; cat $O/pmc_traffic_c3.json $O/pmc_traffic_seg.json
