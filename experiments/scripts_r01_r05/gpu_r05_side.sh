# Side lines under the schedule switches: default (2 lanes, 1 stream), 1 lane x 3 streams, 4 lanes,
# and the bf16 Winograd switched off (direct convs in bf16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  for v in "def" "s3b1 TTS_MI355X_SUBBATCH=1" "b4 TTS_MI355X_SUBBATCH=4" "nowb TTS_MI355X_WINO_BF16=0"; do
    set -- $v
    name=$1; shift
    env "$@" timeout -k 10 400 python scripts/side_ab.py > gpurun_out/side_${name}_$r.json 2> gpurun_out/side_${name}_$r.err || { tail -20 gpurun_out/side_${name}_$r.err; exit 1; }
    echo "$name round $r: $(cat gpurun_out/side_${name}_$r.json)"
  done
done
