# Whole-block k3 c128 excess fetch: A/B of the activation-load cache policy (nt window loads: nt,
# nt window + residual re-read: ntx, nt residual re-read only: xnt) and L2 hit / miss + FETCH counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/l2
AB_NOTEST=1 AB="main:main nt:abx/lib_nt.so ntx:abx/lib_ntx.so xnt:abx/lib_xnt.so" AB_FILTER="block|pair_k7_c32" bash scripts/ab_lib_env.sh || exit 1
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2"
export TTS_FORWARD_NAMES=gpurun_out/l2/forward_names.json
for v in main nt; do
  lib=tts-3_amd/tts_amd/_lib/libtts_mi355x.so; [ $v = nt ] && lib=abx/lib_nt.so
  TTS_MI355X_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/l2/fetch_$v -o f --output-format csv -- python3 $BENCH > gpurun_out/l2/fetch_$v.log 2>&1 || exit 1
  TTS_MI355X_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/l2/hit_$v -o h --output-format csv -- python3 $BENCH > gpurun_out/l2/hit_$v.log 2>&1 || exit 1
  echo "== $v FETCH_SIZE (KiB)"; python3 scripts/pmc_family_counters.py gpurun_out/l2/fetch_$v gpurun_out/l2/forward_names.json FETCH_SIZE | grep -E "block|wino_k11_c128|pair_k7_c32|conv_k3"
  echo "== $v TCC"; python3 scripts/pmc_family_counters.py gpurun_out/l2/hit_$v gpurun_out/l2/forward_names.json TCC_HIT_sum TCC_MISS_sum | grep -E "block|wino_k11_c128|pair_k7_c32|conv_k3"
done
