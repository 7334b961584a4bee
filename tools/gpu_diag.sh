#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
echo "== sustained"; timeout -k 10 300 python tools/sustained.py 30 > gpurun_out/sustained.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/sustained.log; [ $rc -eq 0 ] || exit $rc
echo "== e2e"; timeout -k 10 300 python tools/e2e_h2d.py > gpurun_out/e2e.json 2> gpurun_out/e2e.err; rc=$?; cat gpurun_out/e2e.json; [ $rc -eq 0 ] || { tail gpurun_out/e2e.err; exit $rc; }
