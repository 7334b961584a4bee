#!/bin/bash
# The default line's sub-record order against the headline (profiles/r06/order/):
# R rounds of the driver's command with the line's current order (new_*) and
# with --no-e2e (c5_strong straight before the headline; noe2e_*), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O="$R/gpurun_out/${TAG:-r06/order}"
mkdir -p "$O"
for i in $(seq 1 ${ROUNDS:-3}); do
  timeout -k 10 300 python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/${NAME:-new}_$i.json" 2>/dev/null || exit 1
  timeout -k 10 300 python "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-e2e > "$O/noe2e_$i.json" 2>/dev/null || exit 1
done
for f in "$O"/*.json; do python3 -c "
import json; b=json.load(open('$f')); print('$(basename $f)', b['value'], b['roofline']['frac'], b['c5_strong']['roofline_frac'])"; done
