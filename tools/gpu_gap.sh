#!/bin/bash
# Launch gaps of the headline on one stream: slot launches (hipExtLaunchKernel
# stop event) vs plain launches (MCHECKSUM_GPU_QUEUE_SLOTS=1: the one slot is
# busy, so the launches behind it take the static split without an event).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r05/gap; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in slots plain slots plain; do
  i=$((i+1))
  if [ $v = plain ]; then export MCHECKSUM_GPU_QUEUE_SLOTS=1; else unset MCHECKSUM_GPU_QUEUE_SLOTS; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t_${i}_$v -o k -- python3 $R/tools/overlap_probe.py --streams 1 > $O/run_${i}_$v.json 2> $O/run_${i}_$v.err || { tail $O/run_${i}_$v.err; exit 1; }
  echo "$v $(cat $O/run_${i}_$v.json)"
  python3 $R/tools/overlap_probe.py --analyze $O/t_${i}_$v/k_kernel_trace.csv | tr -d '\n'; echo
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t_probe -o k -- $R/build/gap_probe > $O/gap_probe.log 2>&1 || { tail $O/gap_probe.log; exit 1; }
grep rep $O/gap_probe.log
python3 $R/tools/overlap_probe.py --analyze $O/t_probe/k_kernel_trace.csv --kernel read_nt --group 30
