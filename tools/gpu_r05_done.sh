#!/bin/bash
# Slot completion words (MCK_SLOT_DONE): the slot / queue / thread / fail-closed
# suites, then prev (stop events) vs cur in one process with bench.py's series
# timing, then the driver's command.
set -o pipefail
cd $GRAFT_REPO_ROOT
PART=newtests TAG=done TESTS="tests/test_gpu_slots.py tests/test_gpu_queue.py tests/test_gpu_threads.py tests/test_gpu_fail_closed.py tests/test_gpu_split64.py tests/test_gpu_ext.py" PT=300 bash tools/gpu_r05.sh && \
PART=ab AB_CONFIGS=metric,c4,c3,seg AB_VARIANTS="prev cur" AB_TAG=done_series AB_ROUNDS=6 AB_ITERS=20 AB_ENV="--series" bash tools/gpu_r05.sh && \
PART=driver bash tools/gpu_r05.sh
