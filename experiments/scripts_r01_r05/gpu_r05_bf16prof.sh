# bf16 evidence: the rocprofv3 family / traffic / MFMA-busy tables of the HiFiGAN
# forward in TTS_MATH_BF16 at config 2's shape, and a kernel-trace of the VITS waveform side line (both
# arms: bf16 and f16x3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
# serial one-stream schedule (as scripts/gpu_r05_profiles.sh): one launch per family and forward
TTS_MI355X_SUBBATCH=1 TTS_MI355X_MRF_STREAMS=1 PROF_MODE=bf16 ROUND=r05_bf16 bash scripts/profile_round.sh > gpurun_out/profile_bf16.log 2>&1 || { tail -20 gpurun_out/profile_bf16.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vits -o vits --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits-tts --math-mode bf16 > gpurun_out/prof_vits.log 2>&1 || { tail -20 gpurun_out/prof_vits.log; exit 1; }
find gpurun_out/prof gpurun_out/prof_vits -name "*stats*.csv" | head
