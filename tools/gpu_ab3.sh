#!/bin/bash
# CRC-64 kernel A/B: parity first, then C3 / C4-layout CRC-64 across variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 Error gpurun_out/pytest_gpu.log | head -60; exit $rc; }
echo "== ab"; timeout -k 10 600 python tools/ab_variants.py --config c3,c4_64,metric --rounds 6 --iters 8 --variants base prev sdwa0 split1 ring6 --out gpurun_out/ab10.json > gpurun_out/ab10.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab10.log; exit $rc
