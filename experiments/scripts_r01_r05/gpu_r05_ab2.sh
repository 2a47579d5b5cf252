# A/B: cache policy of the activation stores (TTS_ST_POL: 0 default, 16 sc1, 2 nt) on the f16x3 headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
AB_NOTEST=1 AB="main:main st16:abx/lib_st16.so st2:abx/lib_st2.so" AB_FILTER="block|wino_k11_c128|pair_k11_c64|ups" bash scripts/ab_lib_env.sh || exit 1
