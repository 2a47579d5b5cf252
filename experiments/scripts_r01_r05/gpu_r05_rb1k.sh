# Kernel-7 / 11 ResBlock1 whole blocks: the new test, then an interleaved A/B on the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TTS_ERRLOG=gpurun_out/parity_errors.jsonl
timeout -k 10 300 python -u -m pytest tests/test_hifigan_gpu.py -k "whole_block" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rb1k.log 2>&1 || { tail -30 gpurun_out/pytest_rb1k.log; exit 1; }
tail -1 gpurun_out/pytest_rb1k.log
AB_NOTEST=1 AB="main:main k7:main|TTS_MI355X_RB1_WHOLE_K=7 k711:main|TTS_MI355X_RB1_WHOLE_K=7,11" AB_FILTER="c32|c64" bash scripts/ab_lib_env.sh || exit 1
