// conv1d on bf16 matrix cores with fp32-faithful "x6" split precision (gfx950).
//
// Every fp32 operand is split exactly into three bf16 pieces, x = x0 + x1 + x2 (8+8+8
// significant bits, round-to-nearest-even each; the residuals are exact in fp32).  Of the nine
// cross products the six with i + j <= 2 are accumulated in fp32 by v_mfma_f32_32x32x16_bf16
// (bf16 x bf16 products are exact in fp32); the three dropped ones are below 2^-26 |a*b|, and
// the pieces reproduce the operands exactly, so the result carries fp32 rounding only from the
// fp32 accumulation -- the same error model as the exact-f32 MFMA path.  Cost per emulated
// 32x32x16 block: 6 x 32 = 192 MFMA cycles vs 8 x 64 = 512 for v_mfma_f32_32x32x2_f32, i.e.
// a 2.67x higher ceiling (2.5 PF bf16 dense / 6 = 417 TFLOP/s fp32-equivalent).
//
// Structure mirrors conv1d_mfma_kernel (kernels_conv.hip):
//   A (weights, pre-split on the host) streams from L2 straight into VGPRs as fragments
//     [mblock32][cgroup16][tap][piece][lane][8 bf16], one 1 KiB dwordx4 per piece per wave.
//   B (input window) is split while staging and stored in LDS as rows of
//     [piece 3][16 ch] bf16 (96 B) padded to 112 B: the per-lane ds_read_b128 of one piece is
//     conflict-free at any tap shift.  leaky_relu before the conv is applied before the split.
//   One step = (16 input channels, one tap): 3*TM A loads, 3*TN LDS reads, 6*TM*TN MFMAs.
#include "conv_device.hpp"

namespace tts {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

constexpr int X6_ROWB = 112;  // bytes per staged row: 3 pieces x 16 ch x 2 B + 16 B pad

template <int K, int BM, int BN, int TM, int TN, int G, int HMAX, int PD>
struct X6Cfg {
  static constexpr int WM = BM / (32 * TM);
  static constexpr int WN = BN / (32 * TN);
  static constexpr int CK = 16 * G;
  static constexpr int XROWS = BN + HMAX;
  static constexpr int XSZB = G * XROWS * X6_ROWB;  // bytes per LDS buffer
  static constexpr int UNITS = G * XROWS * 4;       // staging units (group, row, channel quad)
  static constexpr int UPT = (UNITS + 255) / 256;
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(XSZB % 16 == 0, "");
};

__device__ __forceinline__ unsigned short bf16_bits(__bf16 h) { return __builtin_bit_cast(unsigned short, h); }

// x = p0 + p1 + p2 exactly (round-to-nearest-even at every piece)
__device__ __forceinline__ void split3(float x, unsigned short& p0, unsigned short& p1, unsigned short& p2) {
  const __bf16 a0 = (__bf16)x;
  const float r1 = x - (float)a0;
  const __bf16 a1 = (__bf16)r1;
  const float r2 = r1 - (float)a1;
  const __bf16 a2 = (__bf16)r2;
  p0 = bf16_bits(a0);
  p1 = bf16_bits(a1);
  p2 = bf16_bits(a2);
}

template <int K, int BM, int BN, int TM, int TN, int G, int HMAX, int PD>
__global__ __launch_bounds__(256) void conv1d_x6_kernel(Conv1dArgs a) {
  using C = X6Cfg<K, BM, BN, TM, TN, G, HMAX, PD>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * C::XSZB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / C::WN;
  const int wn = wave % C::WN;
  const int half = lane >> 5;
  const int l32 = lane & 31;

  const int t0 = blockIdx.x * BN;
  const int mt = blockIdx.y;
  const int b = blockIdx.z;
  const int d = a.dil;
  const int XW = BN + (K - 1) * d;
  const int Tin = a.Tin;
  const int Tout = a.Tout;
  const int Cin = a.Cin;
  const int nc = a.n_chunks;

  // x of batch item b; one buffer descriptor per chunk (scalar ops), every range-checked
  // offset in the per-lane voffset: zero rows and channels >= Cin read 0 through the hardware
  // range check instead of per-element selects
  const float* xb = a.x + (size_t)b * (a.x_bstride ? a.x_bstride : (int64_t)Cin * Tin);
  const unsigned chb = (unsigned)Tin * 4u;  // bytes per channel row

  // staging units (chunk invariant): unit u -> channel quad q, row r, group g
  unsigned uvoff[C::UPT];  // byte offset of channel (16g+4q) at the clamped source time, or OOB
  int ulds[C::UPT];        // LDS offset of the row's quad
#pragma unroll
  for (int i = 0; i < C::UPT; ++i) {
    const int u = tid + i * 256;
    const int q = u & 3;
    const int rr = u >> 2;
    const int g = rr / XW;
    const int r = rr - g * XW;
    const int ts = t0 - a.pad + r;
    const bool ok = (g < G) && ts >= 0 && ts < Tout;
    int src = ts - a.rep_pad;
    src = src < 0 ? 0 : (src >= Tin ? Tin - 1 : src);
    uvoff[i] = ok ? (unsigned)(16 * g + 4 * q) * chb + (unsigned)src * 4u : OOB_OFF;
    ulds[i] = (g < G) ? (g * C::XROWS + r) * X6_ROWB + 8 * q : -1;
  }

  f32x4 xreg[C::UPT];
  auto load_x = [&](int c) {
    const int c0 = c * C::CK;
    const rsrc_t rx = make_rsrc(xb + (size_t)c0 * Tin, (unsigned)(Cin - c0) * chb);
#pragma unroll
    for (int i = 0; i < C::UPT; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) xreg[i][j] = bload(rx, uvoff[i] + (unsigned)j * chb, 0u);
    }
  };
  auto store_x = [&](int buf) {
    unsigned char* xl = smem + buf * C::XSZB;
    const float slope = a.in_slope;
#pragma unroll
    for (int i = 0; i < C::UPT; ++i) {
      if (ulds[i] >= 0) {
        u16x4 p0, p1, p2;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned short h0, h1, h2;
          split3(lrelu2(xreg[i][j], slope), h0, h1, h2);
          p0[j] = h0;
          p1[j] = h1;
          p2[j] = h2;
        }
        *reinterpret_cast<u16x4*>(xl + ulds[i]) = p0;
        *reinterpret_cast<u16x4*>(xl + ulds[i] + 32) = p1;
        *reinterpret_cast<u16x4*>(xl + ulds[i] + 64) = p2;
      }
    }
  };

  // A streams: f32x4 units, fragment (mb, step s, piece p) at ((mb*S + s)*3 + p)*64 + lane
  // (descriptor per m-block from wave-uniform values, step/piece offsets in the scalar soffset)
  rsrc_t ra[TM];
  const int wmu = __builtin_amdgcn_readfirstlane(wm);
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    const int mb = mt * (BM / 32) + wmu * TM + m;
    ra[m] = make_rsrc(a.w + ((size_t)mb * nc * G * K) * 768, 0xFFFFFFFFu);
  }
  const unsigned avoff = (unsigned)lane * 16u;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n) acc[m][n] = f32x16{};

  const int xrow0 = wn * TN * 32 + l32;

  f32x4 ar[PD + 1][TM][3], bcur[TN][3], bnext[TN][3];
#pragma unroll
  for (int p = 0; p < PD; ++p)
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int q = 0; q < 3; ++q) ar[p][m][q] = bload4(ra[m], avoff, (unsigned)(p * 3 + q) * 1024u);

  auto read_b = [&](const unsigned char* xl, int g, int k, f32x4 (*dst)[3]) {
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int r = xrow0 + n * 32 + k * d;
      const unsigned char* p = xl + (g * C::XROWS + r) * X6_ROWB + 16 * half;
#pragma unroll
      for (int q = 0; q < 3; ++q) dst[n][q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
    }
  };

  load_x(0);
  store_x(0);
  __syncthreads();

  for (int c = 0; c < nc; ++c) {
    const int buf = c & 1;
    const unsigned char* xl = smem + buf * C::XSZB;
    const bool more = c + 1 < nc;
    if (more) load_x(c + 1);
    read_b(xl, 0, 0, bcur);
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int s = (c * G + g) * K + k;
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int q = 0; q < 3; ++q) ar[PD][m][q] = bload4(ra[m], avoff, (unsigned)((s + PD) * 3 + q) * 1024u);
        const bool bnext_here = (k + 1 < K) || (g + 1 < G);
        if (bnext_here) read_b(xl, (k + 1 < K) ? g : g + 1, (k + 1 < K) ? k + 1 : 0, bnext);
        __builtin_amdgcn_sched_barrier(0);
        // smallest products first: a2b0, a1b1, a0b2, a1b0, a0b1, a0b0
        constexpr int PA[6] = {2, 1, 0, 1, 0, 0};
        constexpr int PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int e = 0; e < 6; ++e)
#pragma unroll
          for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int n = 0; n < TN; ++n)
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                  __builtin_bit_cast(bf16x8, ar[0][m][PA[e]]), __builtin_bit_cast(bf16x8, bcur[n][PB[e]]),
                  acc[m][n], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < PD; ++p)
#pragma unroll
          for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int q = 0; q < 3; ++q) ar[p][m][q] = ar[p + 1][m][q];
        if (bnext_here) {
#pragma unroll
          for (int n = 0; n < TN; ++n)
#pragma unroll
            for (int q = 0; q < 3; ++q) bcur[n][q] = bnext[n][q];
        }
      }
    }
    if (more) store_x(buf ^ 1);
    __syncthreads();
  }

  conv_epilogue<TM, TN>(a, acc, b, t0 + wn * TN * 32, mt * BM + wm * TM * 32, lane);
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
namespace {
// {BM, BN, TM, TN, CK = 16*G, PD}
constexpr ConvTile kX6Tiles[] = {
    {128, 128, 2, 2, 16, 1},  // 0  Cout > 64
    {64, 256, 2, 2, 16, 1},   // 1  32 < Cout <= 64
    {32, 512, 1, 4, 16, 1},   // 2  Cout <= 32
    {128, 128, 2, 2, 32, 1},  // 3
    {64, 128, 2, 1, 32, 1},   // 4
    {32, 256, 1, 2, 32, 1},   // 5
    {64, 256, 2, 2, 32, 1},   // 6
    {128, 128, 2, 2, 16, 2},  // 7
    {64, 128, 2, 1, 32, 2},   // 8  tile 4, A prefetched 2 steps ahead
    {64, 256, 2, 2, 32, 2},   // 9  4 waves along t, 2 column blocks each
    {64, 256, 2, 2, 16, 2},   // 10
    {32, 256, 1, 2, 32, 2},   // 11 tile 5, prefetch 2
    {64, 128, 2, 1, 32, 3},   // 12 prefetch 3
};
constexpr int kNumX6Tiles = sizeof(kX6Tiles) / sizeof(kX6Tiles[0]);

template <int K, int BM, int BN, int TM, int TN, int G, int PD, bool WIDE>
void launch_x6_t(const Conv1dArgs& a, int B, hipStream_t s) {
  dim3 grid(ceil_div(a.Tout, BN), ceil_div(a.Cout, BM), B);
  const int halo = (K - 1) * a.dil;
  if (halo <= (K - 1) * 5) {
    hipLaunchKernelGGL((conv1d_x6_kernel<K, BM, BN, TM, TN, G, (K - 1) * 5, PD>), grid, dim3(256), 0, s, a);
  } else if (WIDE && halo <= 96) {
    hipLaunchKernelGGL((conv1d_x6_kernel<K, BM, BN, TM, TN, G, WIDE ? 96 : 0, PD>), grid, dim3(256), 0, s, a);
  } else {
    throw Error(3, "conv1d(x6): (kernel_size-1)*dilation = " + std::to_string(halo) + " too large for this tile");
  }
}

template <int K>
void launch_x6_k(const Conv1dArgs& a, int B, int tile, hipStream_t s) {
  switch (tile) {
    case 0: launch_x6_t<K, 128, 128, 2, 2, 1, 1, true>(a, B, s); break;
    case 1: launch_x6_t<K, 64, 256, 2, 2, 1, 1, true>(a, B, s); break;
    case 2: launch_x6_t<K, 32, 512, 1, 4, 1, 1, true>(a, B, s); break;
    case 3: launch_x6_t<K, 128, 128, 2, 2, 2, 1, false>(a, B, s); break;
    case 4: launch_x6_t<K, 64, 128, 2, 1, 2, 1, false>(a, B, s); break;
    case 5: launch_x6_t<K, 32, 256, 1, 2, 2, 1, false>(a, B, s); break;
    case 6: launch_x6_t<K, 64, 256, 2, 2, 2, 1, false>(a, B, s); break;
    case 7: launch_x6_t<K, 128, 128, 2, 2, 1, 2, false>(a, B, s); break;
    case 8: launch_x6_t<K, 64, 128, 2, 1, 2, 2, false>(a, B, s); break;
    case 9: launch_x6_t<K, 64, 256, 2, 2, 2, 2, false>(a, B, s); break;
    case 10: launch_x6_t<K, 64, 256, 2, 2, 1, 2, false>(a, B, s); break;
    case 11: launch_x6_t<K, 32, 256, 1, 2, 2, 2, false>(a, B, s); break;
    case 12: launch_x6_t<K, 64, 128, 2, 1, 2, 3, false>(a, B, s); break;
    default: throw Error(3, "conv1d(x6): bad tile index " + std::to_string(tile));
  }
}
}  // namespace

ConvTile conv1d_x6_tile(int idx) {
  TTS_REQUIRE(idx >= 0 && idx < kNumX6Tiles, 3, "conv1d(x6): bad tile index");
  return kX6Tiles[idx];
}

int conv1d_x6_num_tiles() { return kNumX6Tiles; }

// Tile choice per conv shape from the round-1 MI355X sweep (profiles/r01_tune_conv_fp32x6.log,
// buffer-addressed kernels).  Any tile is correct for any Cin: channels past Cin read 0.
int conv1d_x6_tile_for(int Cout, int K, int Cin, int dil, bool res) {
  (void)res;
  if ((K - 1) * dil > (K - 1) * 5) return Cout > 64 ? 0 : (Cout > 32 ? 1 : 2);  // wide-halo tiles
  if (Cout > 64) return (K >= 11 || Cin % 32 != 0) ? 7 : 3;
  if (Cout > 32) return K <= 3 ? 10 : 1;
  return 2;
}

void launch_conv1d_x6(const Conv1dArgs& a, int B, int K, int tile, hipStream_t s) {
  switch (K) {
    case 1: launch_x6_k<1>(a, B, tile, s); break;
    case 3: launch_x6_k<3>(a, B, tile, s); break;
    case 5: launch_x6_k<5>(a, B, tile, s); break;
    case 7: launch_x6_k<7>(a, B, tile, s); break;
    case 11: launch_x6_k<11>(a, B, tile, s); break;
    default: throw Error(3, "conv1d(x6): kernel size " + std::to_string(K) + " not supported (1,3,5,7,11)");
  }
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
