# Round 3: library A/B (ab/lib_$AB_LIBS.so vs the working tree, after the Winograd tests), then an optional env A/B ($AB)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
CHECK_TESTS="tests/test_hifigan_gpu.py -k wino" AB_LIBS=${AB_LIBS:?set AB_LIBS} bash scripts/gpu_r03_ab.sh || exit 1
if [ -n "$AB" ]; then bash scripts/ab_env.sh; fi
