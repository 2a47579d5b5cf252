# Round 4 kernel iteration: A/B of variant libraries (scripts/gpu_r04_ab.sh), then Winograd phase
# stamps of the stamp builds (scripts/wino_stamps.py) for the listed (C K dil) shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_SKIP_TESTS=1 NO_PMC=${NO_PMC:-} bash scripts/gpu_r04_ab.sh || exit 1
for lib in ${STAMP_LIBS:-}; do
  for shape in ${STAMP_SHAPES:-128_11_1}; do  # C_K_dil
    echo "== stamps $lib $shape"
    TTS_MI355X_LIB=ab/lib_$lib.so timeout -k 10 120 python scripts/wino_stamps.py ${shape//_/ } > gpurun_out/stamps_${lib}_$shape.txt 2>&1 || { tail -5 gpurun_out/stamps_${lib}_$shape.txt; exit 1; }
    cat gpurun_out/stamps_${lib}_$shape.txt
  done
done
