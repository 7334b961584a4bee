#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python tools/probe_sweep.py > gpurun_out/probe_sweep.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/probe_sweep.log; exit $rc
