# A/B session: fused conv_post on/off (f16x3 headline), then the bf16 knobs (tile table, Winograd job
# group, bf16 Winograd on/off) on the bf16 headline workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
AB="post:main nopost:main|TTS_MI355X_POST_FUSION=0" AB_FILTER="pair_post|pair_k11_c32|conv_post" bash scripts/ab_lib_env.sh || exit 1
AB_NOTEST=1 AB_BENCH_ARGS="--math-mode bf16" AB_FILTER="wino|conv_k3|ups|block" AB="b1:main b1h3t:main|TTS_MI355X_B1_TILES=h3 b1tg1:abx/lib_tg1.so b1nowino:main|TTS_MI355X_WINO_BF16=0" bash scripts/ab_lib_env.sh || exit 1
