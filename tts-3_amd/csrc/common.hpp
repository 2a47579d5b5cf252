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
constexpr int kPlaneXB16 = 1;  // Conv1dArgs::planes bit: the input x is a bf16 plane
constexpr int kPlaneYB16 = 2;  //                          y / z / res are bf16 planes

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
  // MATH_FP32_F16X3 scaling (see kernels_conv_split.hip); ignored by the other modes
  const unsigned* amax_in;  // [B][64] slots (fp32 bits) whose max bounds |x[b]|, or nullptr (scale 1)
  unsigned* amax_out;       // [B][64] slots receiving max |stored output[b]|, or nullptr
  int w_exp;                // packed weights hold w * 2^-w_exp
  // ups = U > 0 (split kernels, K = 2): polyphase ConvTranspose1d(kernel 2U, stride U, padding
  // U/2).  Rows are rho = co*U + s (Cout = U * channels), columns are frames m in [0, Tin]
  // (Tout = Tin + 1, pad = 1: taps x[m-1], x[m]); row rho, column m is stored at time
  // U*m + s - U/2 of y[b][co][0 .. U*Tin).  zmode 0, no res / mask; cvec [B][channels] is
  // added after the bias (channel co = rho / U).
  int ups;
  int64_t o_bstride;     // floats between batch items of res / y / z (0 = Cout*Tout)
  int64_t cvec_bstride;  // floats between batch items of cvec (0 = Cout)
  int mask_res;          // multiply by mask again after the residual add: (res + v) * mask
  // wn_rows = H > 0 (split modes, K = 1, H % 32 == 0): the WaveNet res_skip layer's update fused
  // into the epilogue (wavenet.py:109-113, not the last layer): rows [0, H) update h in place,
  // y[b][r][t] = (y + v) * mask (y = h, res unused), rows [H, 2H) accumulate the skip sum,
  // z[b][r - H][t] = v (zmode 1, the first layer) or z + v (zmode 2); amax_out covers h only.
  int wn_rows;
  // split tile kSplitGateTile only: the WaveNet gate fused into the epilogue (wavenet.py:6-13).
  // gate = H: the packed rows interleave 64-row blocks of the tanh half (rows [0, H)) and the
  // sigmoid half (rows [H, 2H)) (gate_row_order); y receives acts [B][H][Tout] =
  // tanh(x_in[c]) * sigmoid(x_in[H + c]); bias is in packed row order, cvec in the original one.
  int gate;
  // MATH_BF16 only (the HiFiGAN executor's bf16 activation planes, conv_device.hpp PlaneT): bit 0
  // (kPlaneXB16) x is bf16, bit 1 (kPlaneYB16) y / z / res are bf16; the pointers keep their float
  // type and address 2-byte elements.  0: fp32 everywhere.  mask / cvec / bias stay fp32.
  int planes;
};

constexpr int kSplitGateTile = 20;  // = tile 13 (128 x 128, G = 2, PD = 2) with the gate epilogue
constexpr int kSplitWinoTile = 21;  // Winograd F(4,4), 128 rows x 64 tile columns (wino_kernel.hpp)
// Winograd F(4,4) conv (kernels_conv_wino.hip): f16x3, Cout % 128 == 0, Cin % 16 == 0, K in {7, 11},
// dilation 1/3/5, no mask / replicate padding / gate / ConvTranspose form
bool wino_supported(int mode, int Cout, int Cin, int K, int dil);
bool wino_enabled();
void launch_wino(int mode, const Conv1dArgs& a, int B, int K, hipStream_t s);
// packed row rho of a gated in_layer -> original row: block j = rho / 128 holds tanh rows
// [64j, 64j + 64) then sigmoid rows [H + 64j, H + 64j + 64) (H % 64 == 0)
inline int gate_row_order(int rho, int H) {
  const int j = rho / 128, r = rho % 128;
  return r < 64 ? 64 * j + r : H + 64 * j + (r - 64);
}

// One fused ResBlock1 iteration (kernels_resblock.hip): c1 = convs1[m] (x, weights, dilation,
// lrelu slopes, f16x3 input statistics), c2 = convs2[m] (weights, res = the iteration's input x,
// output y or the MRF z, statistics of the output).  x and c2's output must not alias.
struct ResPairArgs {
  Conv1dArgs c1;
  Conv1dArgs c2;
  // post_w != nullptr (the generator's last MRF writer, c2.zmode 3): conv_post fused into the
  // epilogue (hifigan_generator.py:262-264): wav[b][t] = tanh(post_bias + sum_c,k post_w[c][k] *
  // lrelu(z[c][t - 3 + k], post_slope)) with z the final MRF sum, which is not stored.  Tiles then
  // overlap by 6 columns (3 of conv_post's halo on each side).
  const float* post_w;  // [C][7]
  float post_bias;
  float post_slope;
  float* wav;           // [B][1][T]
};
bool resblock_pair_supported(int mode, int C, int K, int dil);
bool resblock_pair_preferred(int mode, int C, int K, int dil);  // supported and measured faster
bool resblock_pair128(int mode, int C, int K);  // bf16: 128-channel k7 / k11 iterations as pairs
void launch_resblock_pair(int mode, const ResPairArgs& a, int B, int K, int C, hipStream_t s);

// A whole kernel-3 ResBlock1 (three iterations, six convs) in one kernel (kernels_resblock.hip):
// x stays in registers between iterations (residual), lrelu(x) and xt pass through LDS.
struct ResBlock3Args {
  const float* x;           // [B][C][T] block input (the upsampled o)
  const unsigned* amax_in;  // [B][64] producer statistics of x (f16x3), or nullptr
  const float* w[6];        // packed conv weights: convs1[0], convs2[0], convs1[1], convs2[1], ...
  const float* bias[6];
  int w_exp[6];
  int dil[3];               // convs1 dilations
  float* z;                 // MRF accumulator [B][C][T]
  int zmode;                // 1: z = v, 2: z += v, 3: z = (z + v) / zdiv
  float zdiv;
  unsigned* amax_out;       // [B][64] statistics of the stored value, or nullptr
  int T;
  int planes;               // 0, or kPlaneXB16 | kPlaneYB16: x and z are bf16 planes (MATH_BF16)
};
bool resblock3_supported(int mode, int C, int K, const int* dil);
void launch_resblock3(int mode, const ResBlock3Args& a, int B, int C, int K, hipStream_t s);
// A whole ResBlock2 (hifigan_generator.py:150-155: two convs of kernel K, dilations dil[0..1],
// each x = conv(lrelu(x)) + x) in one kernel; ResBlock3Args with w / bias / w_exp[0..1].
// geo64 = 1: 192-column tiles at C = 64 (default 128)
bool resblock2_supported(int mode, int C, int K, const int* dil);
bool resblock2_preferred(int mode, int C, int K, const int* dil);  // supported and measured faster
int resblock2_geo64(int mode);  // 64-channel tile geometry (TTS_MI355X_RB2_GEO64 overrides)
void launch_resblock2(int mode, const ResBlock3Args& a, int B, int C, int K, int geo64, hipStream_t s);

// Tile shape of one conv kernel instance (PD: A-operand prefetch distance in steps).
struct ConvTile {
  int BM, BN, TM, TN, CK;
  int PD = 1;
  int WINO = 0;  // Winograd F(4,4) kernel (wino_kernel.hpp): weights packed as 7*ceil(K/4) steps
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
  unsigned* amax_out;  // [B][64] slots receiving max |y[b]| (fp32 bits), or nullptr
  const float* cvec;   // [B][Cout] added after the bias (XTTS conds[i](g)), or nullptr
};

struct PostArgs {
  const float* z;  // [B][Cin][T]
  const float* w;  // [Cin][7]
  float bias;
  float* y;        // [B][1][T]
  int Cin, T;
  float in_slope;
  int z_b16;       // z is a bf16 plane (MATH_BF16 activation planes); y stays fp32
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
// out[b][c][t] = mel[b][c][clamp(w0 + t - pad, 0, T - 1)], t < W: one time window of the
// replicate-padded mel (hifigan_generator.py:281) for the windowed long-utterance forward
void launch_mel_window(const float* mel, int B, int C, int T, int pad, int64_t w0, int W, float* out, hipStream_t s);
// cvec[b][co] = bc[co] + sum_i Wc[co][i] * g[b][i]   (cond_layer, hifigan_generator.py:228)
void launch_cond_vec(const float* g, const float* Wc, const float* bc, float* cvec, int B, int Cc,
                     int C0, hipStream_t s);

// Math modes (TTS_MATH_* in tts_mi355x.h)
constexpr int MATH_FP32 = 0;        // v_mfma_f32_32x32x2_f32
constexpr int MATH_FP32_X6 = 1;     // bf16x6 split on v_mfma_f32_32x32x16_bf16
constexpr int MATH_FP32_F16X3 = 2;  // scaled fp16 hi/lo split on v_mfma_f32_32x32x16_f16
constexpr int MATH_BF16 = 3;        // bf16 operands, fp32 accumulation, fp32 activations in HBM
constexpr int MATH_LAST = MATH_BF16;

// Split-precision conv1d (kernels_conv_split.hip), mode MATH_FP32_X6 or MATH_FP32_F16X3.
ConvTile conv1d_split_tile(int mode, int idx);
int conv1d_split_num_tiles(int mode);
int conv1d_split_tile_for(int mode, int Cout, int K, int Cin, int dil, bool res);
void launch_conv1d_split(int mode, const Conv1dArgs& a, int B, int K, int tile_idx, hipStream_t s);
// window-resident form of the x8 ConvTranspose layers (kernels_convT_res.hip)
bool convT_res_supported(int mode, const Conv1dArgs& a);
void launch_convT_res(int mode, const Conv1dArgs& a, int B, hipStream_t s);
// slots[b][0..63] = max |x[b]| over n floats per item (fp32 bits, atomicMax; zero them first)
// stride: floats between batch items (0 = n, contiguous items)
void launch_amax(const float* x, int64_t n, int B, unsigned* slots, hipStream_t s, int64_t stride = 0);

// Mode-dispatching helpers used by the executors and the op entry points.
inline bool is_split_mode(int mode) { return mode == MATH_FP32_X6 || mode == MATH_FP32_F16X3 || mode == MATH_BF16; }
inline ConvTile conv_tile(int mode, int idx) {
  return is_split_mode(mode) ? conv1d_split_tile(mode, idx) : conv1d_tile(idx);
}
inline int conv_tile_for(int mode, int Cout, int K, int Cin, int dil, bool res) {
  return is_split_mode(mode) ? conv1d_split_tile_for(mode, Cout, K, Cin, dil, res)
                             : conv1d_tile_for(Cout, K, Cin, dil, res);
}
inline int conv_num_tiles(int mode) { return is_split_mode(mode) ? conv1d_split_num_tiles(mode) : conv1d_num_tiles(); }
inline void launch_conv(int mode, const Conv1dArgs& a, int B, int K, int tile, hipStream_t s) {
  if (is_split_mode(mode)) launch_conv1d_split(mode, a, B, K, tile, s);
  else launch_conv1d(a, B, K, tile, s);
}

// Host-side weight packing (pack.cpp).
// Conv1d torch weight [Cout][Cin][K] -> MFMA fragments [mblock32][cgroup8][K][64][4] (+slack).
void pack_conv1d(const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out);
int64_t packed_conv1d_numel(int Cout, int Cin, int K, const ConvTile& t);
// ConvTranspose1d torch weight [Cin][Cout][2U] -> [Cout_pad/BM][n_chunks][2U][CK][BM].
void pack_convT(const float* w, int Cin, int Cout, int U, const ConvTile& t, float* out);
int64_t packed_convT_numel(int Cin, int Cout, int U, const ConvTile& t);
// Split modes: [mblock32][cgroup16][K][piece][64][8 x 16-bit] (+4 steps of slack).  Returns the
// exponent e with which the weights were pre-scaled by 2^-e (0 for bf16x6).
// Channel order of the split kernels' 16-channel LDS rows and packed weights: the 16-bit position
// of channel quad q is 4 quad_pos(q) (quads 1 and 2 swapped).  A wave's accumulator layout then
// holds, per lane and 16-channel group, the 8 channels of 8 consecutive positions (8 half .. +7:
// channels (r & 3) + 8 ((r >> 2) & 1) + 4 half), so an output tile handed to the next conv through
// LDS is one 16-byte store per piece (conflict-free) instead of eight 32-bit ones (4-way).
__host__ __device__ constexpr int quad_pos(int q) { return q == 1 ? 2 : (q == 2 ? 1 : q); }
// quad_perm = false: position = channel (the Winograd packer applies its own order)
int pack_conv1d_split(int mode, const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out,
                      bool quad_perm = true);
int64_t packed_conv1d_split_numel(int mode, int Cout, int Cin, int K, const ConvTile& t);
// ConvTranspose1d torch weight [Cin][Cout][2U] as the K=2 conv of Conv1dArgs::ups (U*Cout rows);
// returns w_exp.  Its bias is the conv's bias repeated per phase: bias'[co*U + s] = bias[co].
int pack_convT_split(int mode, const float* w, int Cin, int Cout, int U, const ConvTile& t, float* out);
int pack_conv1d_wino(int mode, const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out);
inline int64_t packed_conv_numel(int mode, int Cout, int Cin, int K, const ConvTile& t) {
  if (t.WINO) return packed_conv1d_split_numel(mode, Cout, Cin, 7 * ((K + 3) / 4), t);
  return is_split_mode(mode) ? packed_conv1d_split_numel(mode, Cout, Cin, K, t) : packed_conv1d_numel(Cout, Cin, K, t);
}
// returns the weight scale exponent (Conv1dArgs::w_exp)
inline int pack_conv(int mode, const float* w, int Cout, int Cin, int K, const ConvTile& t, float* out) {
  if (t.WINO) return pack_conv1d_wino(mode, w, Cout, Cin, K, t, out);
  if (is_split_mode(mode)) return pack_conv1d_split(mode, w, Cout, Cin, K, t, out);
  pack_conv1d(w, Cout, Cin, K, t, out);
  return 0;
}

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace tts
