// Host-side packing of PyTorch conv weights into the chunked layouts the MFMA kernels
// stage into LDS with contiguous 16-byte loads.
#include <cstring>

#include "common.hpp"

namespace tts {

int64_t packed_conv1d_numel(int Cout, int Cin, int K, const ConvTile& t) {
  const int64_t mtiles = ceil_div(Cout, t.BM);
  const int64_t chunks = ceil_div(Cin, t.CK);
  return mtiles * chunks * K * t.CK * t.BM;
}

// torch Conv1d weight w[Cout][Cin][K] -> out[mt][c][k][ci_l][co_l]
void pack_conv1d(const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out) {
  const int mtiles = ceil_div(Cout, t.BM);
  const int chunks = ceil_div(Cin, t.CK);
  int64_t o = 0;
  for (int mt = 0; mt < mtiles; ++mt)
    for (int c = 0; c < chunks; ++c)
      for (int k = 0; k < K; ++k)
        for (int cl = 0; cl < t.CK; ++cl)
          for (int ml = 0; ml < t.BM; ++ml) {
            const int co = mt * t.BM + ml;
            const int ci = c * t.CK + cl;
            out[o++] = (co < Cout && ci < Cin) ? w[((int64_t)co * Cin + ci) * K + k] : 0.f;
          }
}

int64_t packed_convT_numel(int Cin, int Cout, int U, const ConvTile& t) {
  const int64_t mtiles = ceil_div(Cout, t.BM);
  const int64_t chunks = ceil_div(Cin, t.CK);
  return mtiles * chunks * 2 * U * t.CK * t.BM;
}

// torch ConvTranspose1d weight w[Cin][Cout][2U] -> out[mt][c][tap][ci_l][co_l]
void pack_convT(const float* w, int Cin, int Cout, int U, const ConvTile& t, float* out) {
  const int K = 2 * U;
  const int mtiles = ceil_div(Cout, t.BM);
  const int chunks = ceil_div(Cin, t.CK);
  int64_t o = 0;
  for (int mt = 0; mt < mtiles; ++mt)
    for (int c = 0; c < chunks; ++c)
      for (int k = 0; k < K; ++k)
        for (int cl = 0; cl < t.CK; ++cl)
          for (int ml = 0; ml < t.BM; ++ml) {
            const int co = mt * t.BM + ml;
            const int ci = c * t.CK + cl;
            out[o++] = (co < Cout && ci < Cin) ? w[((int64_t)ci * Cout + co) * K + k] : 0.f;
          }
}

}  // namespace tts
