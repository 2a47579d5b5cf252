// Host-side packing of PyTorch conv weights into the chunked layouts the MFMA kernels
// stage into LDS with contiguous 16-byte loads.
#include <cstring>

#include "common.hpp"

namespace tts {

// MFMA-fragment layout of the conv1d A operand (see conv1d_mfma_kernel):
//   out[mb][c8][k][lane][j] = w[mb*32 + (lane&31)][c8*8 + 4*(lane>>5) + j][k]
// mb over ceil(Cout/BM)*BM/32 blocks, c8 over n_chunks*CK/8 groups (zero padded), plus one
// trailing fragments of slack for the kernel's prefetch (up to 2 steps ahead).
int64_t packed_conv1d_numel(int Cout, int Cin, int K, const ConvTile& t) {
  const int64_t mblocks = (int64_t)ceil_div(Cout, t.BM) * (t.BM / 32);
  const int64_t groups = (int64_t)ceil_div(Cin, t.CK) * (t.CK / 8);
  return mblocks * groups * K * 256 + 512;
}

void pack_conv1d(const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out) {
  const int mblocks = ceil_div(Cout, t.BM) * (t.BM / 32);
  const int groups = ceil_div(Cin, t.CK) * (t.CK / 8);
  int64_t o = 0;
  for (int mb = 0; mb < mblocks; ++mb)
    for (int c8 = 0; c8 < groups; ++c8)
      for (int k = 0; k < K; ++k)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 4; ++j) {
            const int co = mb * 32 + (lane & 31);
            const int ci = c8 * 8 + 4 * (lane >> 5) + j;
            out[o++] = (co < Cout && ci < Cin) ? w[((int64_t)co * Cin + ci) * K + k] : 0.f;
          }
  for (int i = 0; i < 512; ++i) out[o++] = 0.f;
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
