#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
echo "== latency"; timeout -k 10 300 python tools/latency.py > gpurun_out/latency.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/latency.log; exit $rc
