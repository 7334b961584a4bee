#!/bin/bash
# GPU parity suite + smoke + headline bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|^E " gpurun_out/pytest_gpu.log | head -60; exit $rc; }
[ -n "${NO_SMOKE:-}" ] || timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
[ -n "${NO_BENCH:-}" ] || { timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }; cat gpurun_out/bench.json; }
