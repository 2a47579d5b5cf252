# A/B (one box session, environment knobs): kernel-3 c256 convs on the Winograd kernel
# (TTS_MI355X_WINO_K3=1) and conv_post as its own launch (TTS_MI355X_POST_FUSION=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB_NOTEST=1 AB="main:main k3w:main|TTS_MI355X_WINO_K3=1 nopost:main|TTS_MI355X_POST_FUSION=0 both:main|TTS_MI355X_WINO_K3=1,TTS_MI355X_POST_FUSION=0" AB_FILTER="k3_c256|post|pair_k11_c32" bash scripts/ab_lib_env.sh || exit 1
for v in main k3w; do python -c "import json;d=json.load(open('gpurun_out/ab_${v}_2.json'));print('$v', d['accuracy_vs_fp64_oracle'])"; done
