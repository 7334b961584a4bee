#!/bin/bash
# bench.py (the driver's step counts) with 1 and 2 streams, interleaved, per config.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; O=gpurun_out/r05/streams2; mkdir -p $O
for c in ${CONFIGS:-metric c4}; do for s in 1 2 1 2; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --config $c --streams $s --steps 20 --warmup 5 --no-c5-strong --no-cpu-baseline > $O/${c}_${i}_$s.json 2> $O/st.err || { tail -20 $O/st.err; exit 1; }
  python -c "import json,sys;d=json.load(open('$O/${c}_${i}_$s.json'));print('$c', $s, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done; done
