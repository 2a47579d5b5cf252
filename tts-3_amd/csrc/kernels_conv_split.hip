// conv1d on 16-bit matrix cores with fp32-faithful split precision (gfx950), two schemes:
//
// bf16x6 (MATH_FP32_X6): every fp32 operand is split exactly into three bf16 pieces,
//   x = x0 + x1 + x2 (8+8+8 significant bits, round-to-nearest-even each; the residuals are
//   exact in fp32).  Of the nine cross products the six with i + j <= 2 are accumulated in fp32
//   by v_mfma_f32_32x32x16_bf16 (bf16 x bf16 products are exact in fp32); the three dropped
//   ones are below 2^-26 |a*b|.  6 MFMAs per emulated 32x32x16 block: 2.5 PF / 6 = 417 TFLOP/s.
//
// fp16 hi/lo (MATH_FP32_F16X3; after Ootomo & Yokota's error-corrected half-precision GEMM):
//   both operands are first scaled by exact powers of two so that their max-abs lies in
//   [2^13, 2^14) (weights on the host, the input from the max-abs its producer recorded, see
//   amax_exp), then split into hi = fp16(x) and lo = fp16(x - hi): 22 significant bits.  Because
//   of the scaling, a lo piece only turns subnormal for elements below 2^-17 of the tensor's
//   max, where its absolute error (<= 2^-25) is below 2^-39 of that max, so lo needs no 2^11
//   pre-scale and hi*hi, hi*lo and lo*hi share one fp32 accumulator (lo*lo, ~2^-22 relative,
//   is dropped; MFMA accumulation rounds like fp32, as the x6 scheme shows).  The epilogue
//   multiplies by 2^(e_x + e_w), exactly.  3 MFMAs per block: 833 TFLOP/s.
//
// Structure (shared): A (weights, pre-split on the host) streams from L2 straight into VGPRs as
// fragments [mblock32][cgroup16][tap][piece][lane][8 x 16-bit], one 1 KiB dwordx4 per piece
// per wave.  B (input window) is split while staging and stored in LDS as rows of
// [piece][16 ch] 16-bit values padded by 16 B (112 B / 80 B rows: the per-lane ds_read_b128 of
// one piece is conflict-free at any tap shift).  leaky_relu before the conv is applied before
// the split.  One step = (16 input channels, one tap): NP*TM A loads, NP*TN LDS reads,
// NPROD*TM*TN MFMAs.
#include <cstdlib>
#include <string>
#include <algorithm>
#include <cstdlib>

#include "split_device.hpp"

namespace tts {

// slots[b][blockIdx.x & 63] = max |x[b]| (grid-stride per item), for inputs without producer
// statistics
__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, int64_t n, int64_t stride,
                                                   unsigned* slots) {
  const float* xb = x + (size_t)blockIdx.z * stride;
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    m = fmaxf(m, fabsf(xb[i]));
  publish_amax_block(slots, blockIdx.z, m);
}

void launch_amax(const float* x, int64_t n, int B, unsigned* slots, hipStream_t s, int64_t stride) {
  const int64_t blocks = std::min<int64_t>(128, std::max<int64_t>(1, (n + 255) / 256));
  hipLaunchKernelGGL(amax_kernel, dim3((unsigned)blocks, 1, B), dim3(256), 0, s, x, n, stride > 0 ? stride : n,
                     slots);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
namespace {
// {BM, BN, TM, TN, CK = 16*G, PD}; the same table for both schemes (indices are per scheme in
// the tuning logs).
constexpr ConvTile kSplitTiles[] = {
    {128, 128, 2, 2, 16, 1},  // 0  wide halo, Cout > 64
    {64, 256, 2, 2, 16, 1},   // 1  wide halo, 32 < Cout <= 64
    {32, 512, 1, 4, 16, 1},   // 2  wide halo, Cout <= 32
    {128, 128, 2, 2, 32, 1},  // 3
    {64, 128, 2, 1, 32, 1},   // 4
    {32, 256, 1, 2, 32, 1},   // 5
    {64, 256, 2, 2, 32, 1},   // 6
    {128, 128, 2, 2, 16, 2},  // 7
    {64, 128, 2, 1, 32, 2},   // 8
    {64, 256, 2, 2, 32, 2},   // 9
    {64, 256, 2, 2, 16, 2},   // 10
    {32, 256, 1, 2, 32, 2},   // 11
    {64, 128, 2, 1, 32, 3},   // 12
    {128, 128, 2, 2, 32, 2},  // 13
    {32, 256, 1, 2, 16, 1},   // 14 small-LDS tiles for C <= 64 (2-3 workgroups per CU)
    {32, 256, 1, 2, 16, 2},   // 15
    {32, 128, 1, 1, 16, 2},   // 16
    {64, 128, 2, 1, 16, 1},   // 17
    {64, 128, 2, 1, 16, 2},   // 18
    {32, 512, 1, 4, 16, 2},   // 19
    {128, 128, 2, 2, 32, 2},  // 20 = kSplitGateTile: 13 with the WaveNet gate epilogue
    {128, 64, 1, 2, 16, 2, 1},  // 21 = kSplitWinoTile: Winograd F(4,4), BN = tile columns
};
static_assert(kSplitGateTile == 20 && kSplitWinoTile == 21, "tile table");
constexpr int kNumSplitTiles = sizeof(kSplitTiles) / sizeof(kSplitTiles[0]);

}  // namespace

// per-scheme launchers (kernels_conv_split_{x6,h3,b1}.hip)
void launch_split_x6(const Conv1dArgs& a, int B, int K, int tile, hipStream_t s);
void launch_split_h3(const Conv1dArgs& a, int B, int K, int tile, hipStream_t s);
void launch_split_b1(const Conv1dArgs& a, int B, int K, int tile, hipStream_t s);

ConvTile conv1d_split_tile(int mode, int idx) {
  (void)mode;
  TTS_REQUIRE(idx >= 0 && idx < kNumSplitTiles, 3, "conv1d(split): bad tile index");
  return kSplitTiles[idx];
}

int conv1d_split_num_tiles(int mode) {
  (void)mode;
  return kNumSplitTiles;
}

// Tile choice per conv shape from the round-1 MI355X sweeps (profiles/r01_tune_conv_*.log).
// Any tile is correct for any Cin: channels past Cin read 0.
int conv1d_split_tile_for(int mode, int Cout, int K, int Cin, int dil, bool res) {
  (void)res;
  if ((K - 1) * dil > (K - 1) * 5) return Cout > 64 ? 0 : (Cout > 32 ? 1 : 2);  // wide-halo tiles
  static const bool b1_h3_tiles = [] {  // A/B switch: the bf16 scheme on the f16x3 tile choice
    const char* e = std::getenv("TTS_MI355X_B1_TILES");
    return e && std::string(e) == "h3";
  }();
  if (mode == MATH_FP32_F16X3 || (mode == MATH_BF16 && b1_h3_tiles)) {
    // ConvTranspose (K == 2) layers included: round-2 re-sweep, DESIGN.md section 4
    if (Cout > 64) return 13;
    if (Cout > 32) return 10;
    return 14;  // one 16-channel group, 42 KB of LDS: 3 workgroups per CU
  }
  if (Cout > 64) return (K >= 11 || Cin % 32 != 0) ? 7 : 3;
  if (Cout > 32) return K <= 3 ? 10 : 1;
  return 2;
}

void launch_conv1d_split(int mode, const Conv1dArgs& a, int B, int K, int tile, hipStream_t s) {
  if (tile == kSplitWinoTile) {
    launch_wino(mode, a, B, K, s);
    return;
  }
  TTS_REQUIRE((K == 2) == (a.ups > 0), 1, "conv1d(split): K == 2 is the ConvTranspose1d form (ups > 0)");
  TTS_REQUIRE(a.ups == 0 || ((a.ups & (a.ups - 1)) == 0 && a.Cout % a.ups == 0 && a.zmode == 0 && !a.res &&
                             !a.mask && a.Tout == a.Tin + 1 && a.pad == 1),
              1, "conv1d(split): bad ConvTranspose1d arguments");
  // every addressed plane must stay below 2 GiB (32-bit buffer offsets, OOB marker bit 31)
  TTS_REQUIRE((int64_t)a.Cin * a.Tin * 4 < (int64_t(1) << 31) && (int64_t)a.Cout * a.Tout * 4 < (int64_t(1) << 31), 3,
              "conv1d: a batch item's channel plane exceeds 2 GiB");
  if (a.ups > 0 && convT_res_supported(mode, a)) {
    launch_convT_res(mode, a, B, s);
    return;
  }
  if (mode == MATH_FP32_F16X3) launch_split_h3(a, B, K, tile, s);
  else if (mode == MATH_BF16) launch_split_b1(a, B, K, tile, s);
  else launch_split_x6(a, B, K, tile, s);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
