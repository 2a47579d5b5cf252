// Shared definitions for the MI355X (gfx950) mel->waveform kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace tts {

// Error type thrown inside the library and converted to a status code at the C-ABI.
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define TTS_HIP_CHECK(expr)                                                               \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      throw ::tts::Error(2, std::string(#expr) + " failed: " + hipGetErrorString(_e));    \
  } while (0)

#define TTS_REQUIRE(cond, code, msg)                    \
  do {                                                  \
    if (!(cond)) throw ::tts::Error((code), (msg));     \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float lrelu(float x, float slope) { return x > 0.f ? x : x * slope; }

// ---------------------------------------------------------------------------------------
// Conv1d ("same", stride 1) as an implicit GEMM on v_mfma_f32_32x32x2_f32.
//   rows  (MFMA i) = output channel co
//   cols  (MFMA j) = output time t
//   depth (MFMA k) = input channel ci, looped over the K taps
// ---------------------------------------------------------------------------------------
struct Conv1dArgs {
  const float* x;     // [B][Cin][Tin]
  const float* w;     // packed: [Cout_pad/BM][n_chunks][K][CK][BM]
  const float* bias;  // [Cout_pad]
  const float* res;   // [B][Cout][Tout] residual added in the epilogue, or nullptr
  float* y;           // [B][Cout][Tout] (zmode 0)
  float* z;           // [B][Cout][Tout] MRF accumulator (zmode 1..3)
  const float* cvec;  // [B][Cout] per-(batch, channel) add (cond_layer(g)), or nullptr
  const float* mask;  // [B][Tout] multiplied into the output after the bias, or nullptr
  int64_t x_bstride;  // floats between batch items of x (0 = Cin*Tin)
  int Cin, Cout, Tin, Tout;
  int dil, pad, rep_pad;
  int n_chunks;
  float in_slope, out_slope;
  int zmode;
  float zdiv;
};

// Tile shape of one conv kernel instance (PD: A-operand prefetch distance in steps).
struct ConvTile {
  int BM, BN, TM, TN, CK;
  int PD = 1;
};

// Polyphase ConvTranspose1d, K == 2*U, padding U/2: every output phase s is a dense
// [Cout x 2*Cin] GEMM over the input frames m and m-1.
struct ConvTArgs {
  const float* x;     // [B][Cin][Tin]
  const float* w;     // packed: [Cout_pad/BM][n_chunks][2U][CK][BM]
  const float* bias;  // [Cout_pad]
  float* y;           // [B][Cout][U*Tin]
  int Cin, Cout, Tin;
  int n_chunks;
  float in_slope;
};

struct PostArgs {
  const float* z;  // [B][Cin][T]
  const float* w;  // [Cin][7]
  float bias;
  float* y;        // [B][1][T]
  int Cin, T;
  float in_slope;
};

// Host-side launchers (kernels_conv.hip).
int conv1d_tile_for(int Cout, int K, int Cin, int dil, bool res);  // index into the tile table
ConvTile conv1d_tile(int idx);
int conv1d_num_tiles();
void launch_conv1d(const Conv1dArgs& a, int B, int K, int tile_idx, hipStream_t s);
int convT_tile_for(int Cout, int U);
ConvTile convT_tile(int idx, int U);
void launch_convT(const ConvTArgs& a, int B, int U, int tile_idx, hipStream_t s);
void launch_conv_post(const PostArgs& a, int B, hipStream_t s);
// cvec[b][co] = bc[co] + sum_i Wc[co][i] * g[b][i]   (cond_layer, hifigan_generator.py:228)
void launch_cond_vec(const float* g, const float* Wc, const float* bc, float* cvec, int B, int Cc,
                     int C0, hipStream_t s);

// bf16x6 split-precision conv1d (kernels_conv_x6.hip)
ConvTile conv1d_x6_tile(int idx);
int conv1d_x6_num_tiles();
int conv1d_x6_tile_for(int Cout, int K, int Cin, int dil, bool res);
void launch_conv1d_x6(const Conv1dArgs& a, int B, int K, int tile_idx, hipStream_t s);

// Math modes (TTS_MATH_* in tts_mi355x.h)
constexpr int MATH_FP32 = 0;     // v_mfma_f32_32x32x2_f32
constexpr int MATH_FP32_X6 = 1;  // bf16x6 split on v_mfma_f32_32x32x16_bf16

// Mode-dispatching helpers used by the executors and the op entry points.
inline ConvTile conv_tile(int mode, int idx) { return mode == MATH_FP32_X6 ? conv1d_x6_tile(idx) : conv1d_tile(idx); }
inline int conv_tile_for(int mode, int Cout, int K, int Cin, int dil, bool res) {
  return mode == MATH_FP32_X6 ? conv1d_x6_tile_for(Cout, K, Cin, dil, res) : conv1d_tile_for(Cout, K, Cin, dil, res);
}
inline void launch_conv(int mode, const Conv1dArgs& a, int B, int K, int tile, hipStream_t s) {
  if (mode == MATH_FP32_X6) launch_conv1d_x6(a, B, K, tile, s);
  else launch_conv1d(a, B, K, tile, s);
}

// Host-side weight packing (pack.cpp).
// Conv1d torch weight [Cout][Cin][K] -> MFMA fragments [mblock32][cgroup8][K][64][4] (+slack).
void pack_conv1d(const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out);
int64_t packed_conv1d_numel(int Cout, int Cin, int K, const ConvTile& t);
// ConvTranspose1d torch weight [Cin][Cout][2U] -> [Cout_pad/BM][n_chunks][2U][CK][BM].
void pack_convT(const float* w, int Cin, int Cout, int U, const ConvTile& t, float* out);
int64_t packed_convT_numel(int Cin, int Cout, int U, const ConvTile& t);
void pack_conv1d_x6(const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out);
int64_t packed_conv1d_x6_numel(int Cout, int Cin, int K, const ConvTile& t);
inline int64_t packed_conv_numel(int mode, int Cout, int Cin, int K, const ConvTile& t) {
  return mode == MATH_FP32_X6 ? packed_conv1d_x6_numel(Cout, Cin, K, t) : packed_conv1d_numel(Cout, Cin, K, t);
}
inline void pack_conv(int mode, const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out) {
  if (mode == MATH_FP32_X6) pack_conv1d_x6(w, Cout, Cin, K, t, out);
  else pack_conv1d(w, Cout, Cin, K, t, out);
}

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace tts
