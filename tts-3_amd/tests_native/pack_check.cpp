// Host-side check of the weight packers (csrc/pack.cpp), built with AddressSanitizer and
// UndefinedBehaviorSanitizer by `make -C tts-3_amd asan-check` (sanitizers on the
// host code).  Every output buffer is allocated at exactly the size the matching packed_*_numel
// returns, so a packer that writes past it is an ASan heap-buffer-overflow.  The layouts are
// decoded back and compared with the torch weights:
//   pack_conv1d          out[mb][c8][k][lane][j]          = w[mb*32 + (lane&31)][c8*8 + 4*(lane>>5) + j][k]
//   pack_conv1d_split    out[mb][c16][k][piece][lane][j] = piece_p(w'[mb*32 + (lane&31)][c16*16 + 8*(lane>>5) + j][k])
//   pack_convT           out[mt][c][tap][ci_l][co_l]      = w[ci][co][tap]
//   pack_convT_split     pack_conv1d_split of w'[co*U + s][ci][tap] = w[ci][co][s + U (tap 0) | s (tap 1)]
//   pack_conv1d_wino     pack_conv1d_split of U_c[p] = gc[p] * sum_k ga[p]^k w[4c + k]
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "common.hpp"
#include "wino_consts.hpp"
#include <algorithm>

using namespace tts;

static int failures = 0;
#define CHECK(cond, ...)                       \
  do {                                         \
    if (!(cond)) {                             \
      std::fprintf(stderr, "FAIL: " __VA_ARGS__); \
      std::fprintf(stderr, "\n");              \
      ++failures;                              \
    }                                          \
  } while (0)

static float h2f(uint16_t h) {
  _Float16 v;
  std::memcpy(&v, &h, 2);
  return (float)v;
}
static float bf2f(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

static std::vector<float> randw(size_t n, unsigned seed, float scale = 0.1f) {
  std::mt19937 g(seed);
  std::normal_distribution<float> d(0.f, scale);
  std::vector<float> w(n);
  for (auto& v : w) v = d(g);
  return w;
}

static ConvTile tile(int BM, int CK) {
  ConvTile t{};
  t.BM = BM; t.BN = 128; t.TM = 1; t.TN = 1; t.CK = CK; t.PD = 2;
  return t;
}

static void check_conv1d(int Cout, int Cin, int K, const ConvTile& t) {
  const auto w = randw((size_t)Cout * Cin * K, Cout * 31 + Cin * 7 + K);
  std::vector<float> out(packed_conv1d_numel(Cout, Cin, K, t));
  pack_conv1d(w.data(), Cout, Cin, K, t, out.data());
  const int mblocks = ceil_div(Cout, t.BM) * (t.BM / 32), groups = ceil_div(Cin, t.CK) * (t.CK / 8);
  size_t o = 0;
  for (int mb = 0; mb < mblocks; ++mb)
    for (int c8 = 0; c8 < groups; ++c8)
      for (int k = 0; k < K; ++k)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 4; ++j, ++o) {
            const int co = mb * 32 + (lane & 31), ci = c8 * 8 + 4 * (lane >> 5) + j;
            const float want = (co < Cout && ci < Cin) ? w[((size_t)co * Cin + ci) * K + k] : 0.f;
            CHECK(out[o] == want, "pack_conv1d %dx%dx%d at %zu", Cout, Cin, K, o);
          }
}

// decode pack_conv1d_split's element (co, ci, k) back to fp32 (w' = w * 2^-e for f16x3)
// quad_perm: position pos of a 16-channel group holds channel 4 quad_pos(pos / 4) + pos % 4 (the
// split kernels' order, common.hpp); false for the Winograd packer (its own order, decoded by caller)
static void check_split(int mode, const std::vector<float>& w, int Cout, int Cin, int K, const ConvTile& t,
                        const std::vector<float>& packed, int e, const char* what, bool quad_perm = true) {
  const int NP = mode == MATH_FP32_F16X3 ? 2 : (mode == MATH_BF16 ? 1 : 3);
  const uint16_t* p = reinterpret_cast<const uint16_t*>(packed.data());
  const int mblocks = ceil_div(Cout, t.BM) * (t.BM / 32), groups = ceil_div(Cin, t.CK) * (t.CK / 16);
  size_t step = 0;
  for (int mb = 0; mb < mblocks; ++mb)
    for (int c16 = 0; c16 < groups; ++c16)
      for (int k = 0; k < K; ++k, ++step)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int pos = 8 * (lane >> 5) + j;
            const int co = mb * 32 + (lane & 31), ci = c16 * 16 + (quad_perm ? 4 * quad_pos(pos >> 2) + (pos & 3) : pos);
            const float want = (co < Cout && ci < Cin) ? w[((size_t)co * Cin + ci) * K + k] : 0.f;
            auto piece = [&](int q) { return p[((step * NP + q) * 64 + lane) * 8 + j]; };
            double got;
            if (mode == MATH_FP32_F16X3) got = std::ldexp((double)h2f(piece(0)) + (double)h2f(piece(1)), e);
            else if (mode == MATH_BF16) got = bf2f(piece(0));
            else got = (double)bf2f(piece(0)) + (double)bf2f(piece(1)) + (double)bf2f(piece(2));
            // x6: exact; f16x3: 22 significant bits of the scaled value; bf16: one rounding
            const double tol = mode == MATH_FP32_X6 ? 0.0
                             : mode == MATH_FP32_F16X3 ? std::ldexp(1.0, e + 14 - 22)
                                                       : std::fabs(want) * std::ldexp(1.0, -8);
            if (!(std::fabs(got - want) <= tol)) {
              CHECK(false, "%s mode %d (%d,%d,%d): got %.9g want %.9g", what, mode, co, ci, k, got, (double)want);
              return;
            }
          }
  // the prefetch slack after the last step is zero
  const size_t used = step * NP * 64 * 8, total = packed.size() * 2;
  for (size_t i = used; i < total; ++i)
    if (p[i] != 0) { CHECK(false, "%s: slack not zero at %zu", what, i); return; }
}

static void check_conv1d_split(int mode, int Cout, int Cin, int K, const ConvTile& t) {
  const auto w = randw((size_t)Cout * Cin * K, Cout * 17 + Cin + K * 3 + mode);
  std::vector<float> out(packed_conv1d_split_numel(mode, Cout, Cin, K, t));
  const int e = pack_conv1d_split(mode, w.data(), Cout, Cin, K, t, out.data());
  check_split(mode, w, Cout, Cin, K, t, out, e, "pack_conv1d_split");
}

static void check_convT(int Cin, int Cout, int U, const ConvTile& t) {
  const int K = 2 * U;
  const auto w = randw((size_t)Cin * Cout * K, Cin + Cout * 5 + U);
  std::vector<float> out(packed_convT_numel(Cin, Cout, U, t));
  pack_convT(w.data(), Cin, Cout, U, t, out.data());
  size_t o = 0;
  for (int mt = 0; mt < ceil_div(Cout, t.BM); ++mt)
    for (int c = 0; c < ceil_div(Cin, t.CK); ++c)
      for (int k = 0; k < K; ++k)
        for (int cl = 0; cl < t.CK; ++cl)
          for (int ml = 0; ml < t.BM; ++ml, ++o) {
            const int co = mt * t.BM + ml, ci = c * t.CK + cl;
            const float want = (co < Cout && ci < Cin) ? w[((size_t)ci * Cout + co) * K + k] : 0.f;
            CHECK(out[o] == want, "pack_convT %d %d %d", Cin, Cout, U);
          }
}

static void check_convT_split(int mode, int Cin, int Cout, int U, const ConvTile& t) {
  const int K = 2 * U;
  const auto w = randw((size_t)Cin * Cout * K, Cin * 3 + Cout + U + mode);
  std::vector<float> out(packed_conv1d_split_numel(mode, U * Cout, Cin, 2, t));
  const int e = pack_convT_split(mode, w.data(), Cin, Cout, U, t, out.data());
  std::vector<float> wc((size_t)U * Cout * Cin * 2);
  for (int co = 0; co < Cout; ++co)
    for (int s = 0; s < U; ++s)
      for (int ci = 0; ci < Cin; ++ci) {
        wc[(((size_t)co * U + s) * Cin + ci) * 2 + 0] = w[((size_t)ci * Cout + co) * K + s + U];
        wc[(((size_t)co * U + s) * Cin + ci) * 2 + 1] = w[((size_t)ci * Cout + co) * K + s];
      }
  check_split(mode, wc, U * Cout, Cin, 2, t, out, e, "pack_convT_split");
}

static void check_wino(int Cout, int Cin, int K, const ConvTile& t) {
  const int nch = wino_chunks(K), KS = kWinoPoints * nch;
  const auto w = randw((size_t)Cout * Cin * K, Cout + Cin + K);
  std::vector<float> out(packed_conv1d_split_numel(MATH_FP32_F16X3, Cout, Cin, KS, t));
  const int e = pack_conv1d_wino(MATH_FP32_F16X3, w.data(), Cout, Cin, K, t, out.data());
  std::vector<float> u((size_t)Cout * Cin * KS);
  for (size_t oc = 0; oc < (size_t)Cout * Cin; ++oc)
    for (int c = 0; c < nch; ++c)
      for (int p = 0; p < kWinoPoints; ++p) {
        double acc = 0.0;
        for (int k = 0; k < 4; ++k) {
          if (4 * c + k >= K) continue;
          const double g = p == 6 ? (k == 3) : (p == 0 ? (k == 0) : std::pow(kWinoGa[p], k));
          acc += g * w[oc * K + 4 * c + k];
        }
        u[oc * KS + c * kWinoPoints + p] = (float)(kWinoGc[p] * acc);
      }
  // the packed k position kk of a 16-channel group holds channel 4q + 2jp + e (kk = 8jp + 2q + e)
  std::vector<float> up(u.size());
  for (int o = 0; o < Cout; ++o)
    for (int ci = 0; ci < Cin; ++ci) {
      const int kk = ci & 15, ch = (ci & ~15) + 4 * ((kk >> 1) & 3) + 2 * (kk >> 3) + (kk & 1);
      std::copy_n(u.data() + ((size_t)o * Cin + ch) * KS, KS, up.data() + ((size_t)o * Cin + ci) * KS);
    }
  check_split(MATH_FP32_F16X3, up, Cout, Cin, KS, t, out, e, "pack_conv1d_wino", /*quad_perm=*/false);
}

int main() {
  const int modes[] = {MATH_FP32_X6, MATH_FP32_F16X3, MATH_BF16};
  const int shapes[][3] = {{128, 128, 11}, {256, 512, 7}, {32, 32, 3}, {64, 64, 5}, {100, 80, 7}, {1, 7, 1},
                           {33, 17, 3}, {512, 80, 7}};
  const ConvTile tiles[] = {tile(128, 32), tile(64, 16), tile(32, 16), tile(128, 16)};
  for (const auto& s : shapes)
    for (const auto& t : tiles) {
      check_conv1d(s[0], s[1], s[2], tile(t.BM, t.CK < 8 ? 8 : t.CK));
      for (int m : modes) check_conv1d_split(m, s[0], s[1], s[2], t);
    }
  for (int U : {2, 4, 8})
    for (const auto& t : tiles) {
      check_convT(64 * U / 2, 32 * U / 2 + 3, U, t);
      for (int m : modes) check_convT_split(m, 64, 32, U, t);
    }
  for (int K : {3, 7, 11})
    for (const auto& t : tiles) check_wino(128, 144, K, t);
  // all-zero and non-finite weights: scale exponent 0 / a clean error (no UB in frexp/ldexp)
  {
    std::vector<float> z(32 * 16 * 3, 0.f), out(packed_conv1d_split_numel(MATH_FP32_F16X3, 32, 16, 3, tile(32, 16)));
    CHECK(pack_conv1d_split(MATH_FP32_F16X3, z.data(), 32, 16, 3, tile(32, 16), out.data()) == 0, "zero weights");
    z[5] = NAN;
    bool threw = false;
    try {
      pack_conv1d_split(MATH_FP32_F16X3, z.data(), 32, 16, 3, tile(32, 16), out.data());
    } catch (const Error& e) {
      threw = e.code == 1;
    }
    CHECK(threw, "NaN weights must raise TTS_ERR_INVALID");
  }
  if (failures) {
    std::fprintf(stderr, "%d pack check(s) failed\n", failures);
    return 1;
  }
  std::printf("pack_check: all packers OK\n");
  return 0;
}
