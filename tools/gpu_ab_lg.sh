#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 500 python tools/ab_variants.py --config c2,metric,c3 --rounds 5 --iters 8 --variants base \
  --env lg2=MCHECKSUM_GPU_LOG2G=2 lg3=MCHECKSUM_GPU_LOG2G=3 lg4=MCHECKSUM_GPU_LOG2G=4 lg5=MCHECKSUM_GPU_LOG2G=5 lg6=MCHECKSUM_GPU_LOG2G=6 \
  > gpurun_out/ab_lg.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/ab_lg.log; exit $rc
