// Winograd F(4,4) conv1d instances (wino_kernel.hpp, wino8_kernel.hpp); the host weight transform
// pack_conv1d_wino is in pack.cpp.
#include <cmath>
#include <cstdlib>
#include <vector>

#include "wino8_kernel.hpp"

namespace tts {

// f16x3 (fp32-faithful), and bf16 (configs 3 / 5: one bf16 product per transformed point, the
// transforms in fp32; rel-RMS against fp64 in tests/test_configs_gpu.py's bf16 gate).  bf16 is the
// default there unless TTS_MI355X_WINO_BF16=0.
bool wino_supported(int mode, int Cout, int Cin, int K, int dil) {
  bool m = mode == MATH_FP32_F16X3;
  if (mode == MATH_BF16) {
    const char* e = std::getenv("TTS_MI355X_WINO_BF16");
    m = !(e && e[0] == '0');
  }
  return m && Cout % 128 == 0 && Cin % 16 == 0 && (K == 3 || K == 7 || K == 11) && (dil == 1 || dil == 3 || dil == 5);
}

// TTS_MI355X_WINO=0 keeps the direct split kernel for every conv (A/B runs, accuracy comparisons)
// (read at every generator create, so tests can compare both forms in one process)
bool wino_enabled() {
  const char* e = std::getenv("TTS_MI355X_WINO");
  return !(e && e[0] == '0');
}


void launch_wino(int mode, const Conv1dArgs& a, int B, int K, hipStream_t s) {
  TTS_REQUIRE(wino_supported(mode, a.Cout, a.Cin, K, a.dil), 3, "conv1d(winograd): unsupported configuration");
  TTS_REQUIRE((int64_t)a.Cin * a.Tin * 4 < (int64_t(1) << 31) && (int64_t)a.Cout * a.Tout * 4 < (int64_t(1) << 31), 3,
              "conv1d: a batch item's channel plane exceeds 2 GiB");
  // the 8-wave form needs 16-byte aligned input rows (every HiFiGAN MRF conv at >= 128 channels:
  // T = 8 * (T_mel + 2 pad) and more); other lengths take the 4-wave form
  // bf16 activation planes (Conv1dArgs::planes): the 8-wave form only, its DMA needs T % 8 == 0
  TTS_REQUIRE(a.planes == 0 || (mode == MATH_BF16 && a.Tin % 8 == 0), 3,
              "conv1d(winograd): bf16 planes need the bf16 scheme and T % 8 == 0");
  if (mode == MATH_BF16) {
    if (a.Tin % 4 == 0) wino8_detail::launch_s<SchemeB1>(a, B, K, s);
    else wino_detail::launch_wino_s<SchemeB1>(a, B, K, s);
  } else {
    if (a.Tin % 4 == 0) wino8_detail::launch_s<SchemeH3>(a, B, K, s);
    else wino_detail::launch_wino_s<SchemeH3>(a, B, K, s);
  }
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
