#!/bin/bash
# Segment scan with fewer segments per scan block (MCK_SCAN_PER): the segment
# suites on the per1 build's library are not needed (the scan is the same
# code); A/B of seg / seg32 series and small-list latency.
set -o pipefail
cd $GRAFT_REPO_ROOT
PART=ab AB_CONFIGS=seg,seg32 AB_VARIANTS="prev per1 per2" AB_TAG=scan_per AB_ROUNDS=8 AB_ITERS=20 AB_ENV="--series" bash tools/gpu_r05.sh
