// Host-side packing of PyTorch conv weights into the chunked layouts the MFMA kernels
// stage into LDS with contiguous 16-byte loads.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "wino_consts.hpp"

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

// bf16x6 split of an fp32 value: x = p0 + p1 + p2 exactly, round-to-nearest-even per piece
// (same rounding as the device's v_cvt_pk_bf16_f32).
static inline uint16_t f2bf_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static inline float bf2f(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
void split3_host(float x, uint16_t& p0, uint16_t& p1, uint16_t& p2) {
  p0 = f2bf_rne(x);
  const float r1 = x - bf2f(p0);
  p1 = f2bf_rne(r1);
  const float r2 = r1 - bf2f(p1);
  p2 = f2bf_rne(r2);
}

// fp16 hi/lo split of a value already scaled into [0, 2^14] magnitude: x ~ hi + lo
// (round-to-nearest-even, as the device's v_cvt_f16_f32; see kernels_conv_split.hip).
static inline void split_h3_host(float x, uint16_t& hi, uint16_t& lo) {
  const _Float16 h = (_Float16)x;
  hi = __builtin_bit_cast(uint16_t, h);
  lo = __builtin_bit_cast(uint16_t, (_Float16)(x - (float)h));
}

static int split_pieces(int mode) { return mode == MATH_FP32_F16X3 ? 2 : (mode == MATH_BF16 ? 1 : 3); }

// Split-mode A-operand fragments (conv1d_split_kernel), in floats (2 x 16-bit per float):
//   out[mb][c16][k][piece][lane][j] = piece_p(w'[mb*32 + (lane&31)][c16*16 + 8*(lane>>5) + j][k])
// plus 4 steps of slack for the prefetch (up to 4 steps ahead).  w' = w for bf16x6, w * 2^-e for fp16 hi/lo with e
// chosen so max|w'| lies in [2^13, 2^14) (exact; undone in the kernel epilogue).
int64_t packed_conv1d_split_numel(int mode, int Cout, int Cin, int K, const ConvTile& t) {
  const int64_t mblocks = (int64_t)ceil_div(Cout, t.BM) * (t.BM / 32);
  const int64_t groups = (int64_t)ceil_div(Cin, t.CK) * (t.CK / 16);
  return (mblocks * groups * K + 4) * split_pieces(mode) * 64 * 4;
}

int pack_conv1d_split(int mode, const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out_f,
                      bool quad_perm) {
  const int NP = split_pieces(mode);
  int e = 0;
  if (mode == MATH_FP32_F16X3) {
    float m = 0.f;
    bool finite = true;  // std::max(m, NaN) keeps m: test every element, not the running max
    for (int64_t i = 0; i < (int64_t)Cout * Cin * K; ++i) {
      finite = finite && std::isfinite(w[i]);
      m = std::max(m, std::fabs(w[i]));
    }
    TTS_REQUIRE(finite, 1, "conv weights contain inf/NaN");
    if (m > 0.f) {
      int E;
      (void)std::frexp(m, &E);
      e = E - 14;
    }
  }
  uint16_t* out = reinterpret_cast<uint16_t*>(out_f);
  const int mblocks = ceil_div(Cout, t.BM) * (t.BM / 32);
  const int groups = ceil_div(Cin, t.CK) * (t.CK / 16);
  int64_t o = 0;
  for (int mb = 0; mb < mblocks; ++mb)
    for (int c16 = 0; c16 < groups; ++c16)
      for (int k = 0; k < K; ++k) {
        uint16_t pc[3][64][8];
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int co = mb * 32 + (lane & 31);
            const int pos = 8 * (lane >> 5) + j;  // MFMA k index = 16-bit position in the LDS row
            const int ci = c16 * 16 + (quad_perm ? 4 * quad_pos(pos >> 2) + (pos & 3) : pos);
            const float v = (co < Cout && ci < Cin) ? w[((int64_t)co * Cin + ci) * K + k] : 0.f;
            if (NP == 3) split3_host(v, pc[0][lane][j], pc[1][lane][j], pc[2][lane][j]);
            else if (NP == 2) split_h3_host(std::ldexp(v, -e), pc[0][lane][j], pc[1][lane][j]);
            else pc[0][lane][j] = f2bf_rne(v);
          }
        for (int p = 0; p < NP; ++p)
          for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; ++j) out[o++] = pc[p][lane][j];
      }
  for (int i = 0; i < 4 * NP * 64 * 8; ++i) out[o++] = 0;
  return e;
}

int pack_convT_split(int mode, const float* w, int Cin, int Cout, int U, const ConvTile& t, float* out) {
  // y[co][U*m + s - U/2] = sum_ci W[ci][co][s] x[ci][m] + W[ci][co][s+U] x[ci][m-1]
  // -> conv weight w'[co*U + s][ci][tap]: tap 0 reads x[m-1], tap 1 reads x[m]
  const int K = 2 * U;
  std::vector<float> wc((size_t)U * Cout * Cin * 2);
  for (int co = 0; co < Cout; ++co)
    for (int s = 0; s < U; ++s)
      for (int ci = 0; ci < Cin; ++ci) {
        const float* src = w + ((int64_t)ci * Cout + co) * K;
        float* dst = wc.data() + (((size_t)co * U + s) * Cin + ci) * 2;
        dst[0] = src[s + U];
        dst[1] = src[s];
      }
  return pack_conv1d_split(mode, wc.data(), U * Cout, Cin, 2, t, out);
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
  // channel order within each 16-channel group: the transform jobs store channels 4q + 2jp + e
  // (quad q, pair jp, e = 0, 1) at 16-bit position 2 (q + 4 jp) + e of the staged row, so that a
  // 32-lane store covers all banks; the MFMA k index runs over those positions
  TTS_REQUIRE(Cin % 16 == 0, 1, "winograd packing: Cin must be a multiple of 16");
  std::vector<float> wp(wt.size());
  for (int64_t o = 0; o < Cout; ++o)
    for (int g = 0; g < Cin / 16; ++g)
      for (int kk = 0; kk < 16; ++kk) {
        const int jp = kk >> 3, q = (kk >> 1) & 3, e = kk & 1;
        const int ch = 4 * q + 2 * jp + e;
        std::copy_n(wt.data() + ((size_t)o * Cin + g * 16 + ch) * KS, KS, wp.data() + ((size_t)o * Cin + g * 16 + kk) * KS);
      }
  return pack_conv1d_split(mode, wp.data(), Cout, Cin, KS, t, out, /*quad_perm=*/false);
}

}  // namespace tts
