#!/bin/bash
# bench.py for metric and c4 with 1, 2 and 3 streams (independent batches round-robin).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
for c in metric c4; do for s in 1 2 1 2 3; do
  timeout -k 10 200 python bench.py --config $c --streams $s --no-cpu-baseline > gpurun_out/st_${c}_$s.json 2> gpurun_out/st.err || { tail -20 gpurun_out/st.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/st_${c}_$s.json'));print('$c', $s, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity'])"
done; done
