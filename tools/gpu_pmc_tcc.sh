#!/bin/bash
# L2 memory-side request counters by request size, to attribute the
# FETCH_SIZE excess of byte-packed batches (C4, msgs) against aligned ones
# (metric).  Lists the gfx950 counters first (rocprofv3 -L), then runs one
# pass per pair of TCC counters that exist (each pass its own rocprofv3 run
# under a time limit), for CONFIGS x NT settings.  Summaries with
# tools/pmc_summary.py into gpurun_out/r03/tcc_<config>_nt<NT>.txt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || { tail $O/rocprof_counters.txt; exit 1; }
grep -oE "TCC_EA0?_[A-Z0-9_]+|TCC_[A-Z_]*REQ[A-Z0-9_]*" $O/rocprof_counters.txt | sort -u > $O/tcc_names.txt
want="TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM TCC_EA0_RDREQ_LEVEL TCC_REQ TCC_MISS TCC_HIT TCC_STREAMING_REQ TCC_NC_REQ TCC_EA_RDREQ TCC_EA_RDREQ_32B"
have=""
for c in $want; do grep -qx "$c" $O/tcc_names.txt && have="$have $c"; done
echo "counters: $have"
set -- $have
passes=()
while [ $# -gt 0 ]; do
  if [ $# -ge 2 ]; then passes+=("${1}_sum ${2}_sum"); shift 2; else passes+=("${1}_sum"); shift; fi
done
for c in ${CONFIGS:-c4 metric}; do
  for nt in ${NTS:-1 0}; do
    i=0; dirs=""
    for set in "${passes[@]}"; do
      i=$((i+1))
      d=$O/tcc_${c}_nt${nt}_$i
      MCHECKSUM_GPU_NT=$nt timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $d -o p -- python3 $R/tools/kernel_run.py --config $c --iters 4 > $d.log 2>&1 || { echo "pass $c nt$nt $set failed"; tail -5 $d.log; exit 1; }
      dirs="$dirs $d"
    done
    python3 $R/tools/pmc_summary.py $dirs > $O/tcc_${c}_nt${nt}.txt || exit 1
    echo "== $c NT=$nt"; cat $O/tcc_${c}_nt${nt}.txt
  done
done
