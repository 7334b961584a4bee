#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 Error gpurun_out/pytest_gpu.log | head -60; exit $rc; }
echo "== ab"; timeout -k 10 600 python tools/ab_variants.py --config c4,c4_64 --rounds 6 --iters 8 --variants base prev ring6 ring8 --out gpurun_out/ab2.json > gpurun_out/ab2.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab2.log; exit $rc
