#!/bin/bash
# Round 5: CRC-64 address-formation A/B (prev = HEAD, cheap = MCK_CHEAP64 only,
# cur = + the wide-row fold), then the CRC-64 parity suites on cur.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
PART=ab AB_CONFIGS=${AB_CONFIGS:-c3,seg,c4_64,g64k} AB_VARIANTS="prev cheap cur" AB_TAG=${AB_TAG:-fold12w} AB_ROUNDS=6 bash tools/gpu_r05.sh && \
PART=newtests TAG=${AB_TAG:-fold12w} TESTS="tests/test_gpu_split64.py tests/test_gpu_parity.py tests/test_gpu_full_shapes.py tests/test_gpu_golden.py" PT=300 bash tools/gpu_r05.sh
