#!/bin/bash
# Split CRC-64 plan with finer tail pieces (SplitPlan, MCK_SPLIT_TAIL): the
# CRC-64 parity suites, then prev (HEAD) vs cur vs the other refinements in one process.
set -o pipefail
cd $GRAFT_REPO_ROOT
PART=newtests TAG=tail TESTS="tests/test_gpu_split64.py tests/test_gpu_full_shapes.py" PT=300 bash tools/gpu_r05.sh && \
PART=ab AB_CONFIGS=c3 AB_VARIANTS="prev cur quarter notail" AB_TAG=tail_series2 AB_ROUNDS=10 AB_ITERS=20 AB_ENV="--series" bash tools/gpu_r05.sh
