#!/bin/bash
# One-state 8-byte-lane CRC-64 loop at two workgroups per CU (MCK_CRC64_L8):
# the CRC-64 parity suites, then prev (HEAD) vs cur vs ring 4 in one process.
set -o pipefail
cd $GRAFT_REPO_ROOT
PART=newtests TAG=l8 TESTS="tests/test_gpu_split64.py tests/test_gpu_full_shapes.py tests/test_gpu_parity.py tests/test_gpu_golden.py" PT=300 bash tools/gpu_r05.sh && \
PART=ab AB_CONFIGS=c3,m1,g64k AB_VARIANTS="prev cur l8r4" AB_TAG=l8_series AB_ROUNDS=6 AB_ITERS=20 AB_ENV="--series" bash tools/gpu_r05.sh
