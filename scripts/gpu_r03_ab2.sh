# Round 3: Winograd transform-spread A/B (library) and the ConvTranspose XCD order A/B (env), one box session
set -o pipefail
cd "$GRAFT_REPO_ROOT"
CHECK_TESTS="tests/test_hifigan_gpu.py -k wino" AB_LIBS=nospread bash scripts/gpu_r03_ab.sh || exit 1
AB="r0:TTS_MI355X_XCD_REMAP=0 r2:TTS_MI355X_XCD_REMAP=2" AB_FILTER=ups bash scripts/ab_env.sh
