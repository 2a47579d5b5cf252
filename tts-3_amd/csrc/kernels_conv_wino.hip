// Winograd F(4,4) conv1d instances (wino_kernel.hpp) and the weight transform (host).
#include <cmath>
#include <cstdlib>
#include <vector>

#include "wino8_kernel.hpp"

namespace tts {

bool wino_supported(int mode, int Cout, int Cin, int K, int dil) {
  return mode == MATH_FP32_F16X3 && Cout % 128 == 0 && Cin % 16 == 0 && (K == 3 || K == 7 || K == 11) &&
         (dil == 1 || dil == 3 || dil == 5);
}

// TTS_MI355X_WINO=0 keeps the direct split kernel for every conv (A/B runs, accuracy comparisons)
// (read at every generator create, so tests can compare both forms in one process)
bool wino_enabled() {
  const char* e = std::getenv("TTS_MI355X_WINO");
  return !(e && e[0] == '0');
}


// U_c[p][co][ci] = gc[p] * sum_k ga[p]^k w[co][ci][4c + k]  (fp64, taps >= K are zero), laid out as
// the 7*NCH "taps" s = c*7 + p of an ordinary split-mode conv weight, then packed by
// pack_conv1d_split (one power-of-two scale for all points: see split_device.hpp / DESIGN.md).
int pack_conv1d_wino(int mode, const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out) {
  const int nch = wino_chunks(K);
  const int KS = kWinoPoints * nch;
  std::vector<float> wt((size_t)Cout * Cin * KS);
  for (int64_t oc = 0; oc < (int64_t)Cout * Cin; ++oc) {
    const float* src = w + oc * K;
    float* dst = wt.data() + oc * KS;
    for (int c = 0; c < nch; ++c)
      for (int p = 0; p < kWinoPoints; ++p) {
        double acc = 0.0;
        for (int k = 0; k < 4; ++k) {
          const int tap = 4 * c + k;
          if (tap >= K) continue;
          const double g = p == 6 ? (k == 3 ? 1.0 : 0.0) : (p == 0 ? (k == 0 ? 1.0 : 0.0) : std::pow(kWinoGa[p], k));
          acc += g * (double)src[tap];
        }
        dst[c * kWinoPoints + p] = (float)(kWinoGc[p] * acc);
      }
  }
  return pack_conv1d_split(mode, wt.data(), Cout, Cin, KS, t, out);
}

void launch_wino(int mode, const Conv1dArgs& a, int B, int K, hipStream_t s) {
  TTS_REQUIRE(wino_supported(mode, a.Cout, a.Cin, K, a.dil), 3, "conv1d(winograd): unsupported configuration");
  TTS_REQUIRE((int64_t)a.Cin * a.Tin * 4 < (int64_t(1) << 31) && (int64_t)a.Cout * a.Tout * 4 < (int64_t(1) << 31), 3,
              "conv1d: a batch item's channel plane exceeds 2 GiB");
  // the 8-wave form needs 16-byte aligned input rows (every HiFiGAN MRF conv at >= 128 channels:
  // T = 8 * (T_mel + 2 pad) and more); TTS_MI355X_WINO8=0 keeps the 4-wave form (A/B runs)
  static const bool w8 = [] {
    const char* e = std::getenv("TTS_MI355X_WINO8");
    return !(e && e[0] == '0');
  }();
  if (w8 && a.Tin % 4 == 0) wino8_detail::launch_s<SchemeH3>(a, B, K, s);
  else wino_detail::launch_wino_s<SchemeH3>(a, B, K, s);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
