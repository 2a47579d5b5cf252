# Shader clock (GRBM_GUI_ACTIVE / 8 / duration) and MFMA busy per family, product library vs the
# activation-traffic ablation (ACT_ABLATE=1): does the ablation's gain come from DVFS (zero data)?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export TTS_MI355X_SUBBATCH=1 TTS_MI355X_MRF_STREAMS=1  # serial one-stream schedule: dispatches in executor order
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt --no-glow --no-e2e --no-xtts --no-vits --no-vits-tts --no-rb2"
for mode in f16x3 bf16; do
for v in main act; do
  OUT=gpurun_out/clk_${mode}_$v
  mkdir -p $OUT
  lib=$GRAFT_REPO_ROOT/tts-3_amd/tts_amd/_lib/libtts_mi355x.so; [ $v = act ] && lib=$GRAFT_REPO_ROOT/abx/lib_act.so
  export TTS_MI355X_LIB=$lib TTS_FORWARD_NAMES=$OUT/forward_names.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $BENCH --math-mode $mode > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o sq --output-format csv -- python3 $BENCH --math-mode $mode > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
  python3 scripts/mfma_from_pmc.py $OUT $mode $OUT/mfma_busy.json > $OUT/mfma.txt || exit 1
  echo "== $mode $v"; grep -E "wino_k11_c128|wino_k7_c128|pair_k11_c64|block_k3_c128|pair_k7_c32|forward" $OUT/mfma.txt | head -8
done
done
