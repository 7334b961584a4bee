#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python tools/latency.py > gpurun_out/latency.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/latency.log; exit $rc
