#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_variants.py --config metric,c2,c3 --rounds 5 --iters 5 --out gpurun_out/ab1.json > gpurun_out/ab1.log 2>&1; rc=$?
cat gpurun_out/ab1.log | grep -v amdgpu.ids
exit $rc
