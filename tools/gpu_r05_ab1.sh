set -o pipefail
cd $GRAFT_REPO_ROOT
PART=ab AB_CONFIGS=c3,g64k,g16k,g4k AB_VARIANTS="prev cur" AB_TAG=fold11 AB_ROUNDS=6 bash tools/gpu_r05.sh && \
PART=newtests TAG=fold11 TESTS="tests/test_gpu_split64.py tests/test_gpu_parity.py tests/test_gpu_full_shapes.py" PT=300 bash tools/gpu_r05.sh
