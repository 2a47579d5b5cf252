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
#include <algorithm>

#include "conv_device.hpp"

namespace tts {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned short bf16_bits(__bf16 h) { return __builtin_bit_cast(unsigned short, h); }
__device__ __forceinline__ unsigned short f16_bits(_Float16 h) { return __builtin_bit_cast(unsigned short, h); }

struct SchemeX6 {
  static constexpr int NP = 3;        // pieces per operand
  static constexpr int ROWB = 112;    // LDS bytes per staged row (3 x 32 B + 16 B pad)
  static constexpr int NACC = 1;      // accumulators per output block
  static constexpr int NPROD = 6;     // products per step, smallest first
  static constexpr int PA[6] = {2, 1, 0, 1, 0, 0};
  static constexpr int PB[6] = {0, 1, 2, 0, 1, 0};
  static constexpr int PACC[6] = {0, 0, 0, 0, 0, 0};
  static constexpr bool SCALED = false;
  // x = p0 + p1 + p2 exactly (round-to-nearest-even at every piece)
  __device__ static __forceinline__ void split(float x, unsigned short (&p)[3]) {
    const __bf16 a0 = (__bf16)x;
    const float r1 = x - (float)a0;
    const __bf16 a1 = (__bf16)r1;
    const float r2 = r1 - (float)a1;
    p[0] = bf16_bits(a0);
    p[1] = bf16_bits(a1);
    p[2] = bf16_bits((__bf16)r2);
  }
  __device__ static __forceinline__ f32x16 mfma(f32x4 a, f32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};

struct SchemeH3 {
  static constexpr int NP = 2;
  static constexpr int ROWB = 80;     // 2 x 32 B + 16 B pad
  static constexpr int NACC = 1;
  static constexpr int NPROD = 3;     // lo*hi, hi*lo, hi*hi
  static constexpr int PA[3] = {1, 0, 0};
  static constexpr int PB[3] = {0, 1, 0};
  static constexpr int PACC[3] = {0, 0, 0};
  static constexpr bool SCALED = true;
  // x (already scaled into [0, 2^14]) = hi + lo to 22 bits
  __device__ static __forceinline__ void split(float x, unsigned short (&p)[2]) {
    const _Float16 h = (_Float16)x;
    p[0] = f16_bits(h);
    p[1] = f16_bits((_Float16)(x - (float)h));
  }
  __device__ static __forceinline__ f32x16 mfma(f32x4 a, f32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

// Plain bf16 (MATH_BF16): one bf16 piece per operand, one product, fp32 accumulation.
struct SchemeB1 {
  static constexpr int NP = 1;
  static constexpr int ROWB = 48;     // 32 B + 16 B pad (conflict-free like the other pitches)
  static constexpr int NACC = 1;
  static constexpr int NPROD = 1;
  static constexpr int PA[1] = {0};
  static constexpr int PB[1] = {0};
  static constexpr int PACC[1] = {0};
  static constexpr bool SCALED = false;
  __device__ static __forceinline__ void split(float x, unsigned short (&p)[1]) { p[0] = bf16_bits((__bf16)x); }
  __device__ static __forceinline__ f32x16 mfma(f32x4 a, f32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};

// Exponent e such that max|x| * 2^-e lies in [2^13, 2^14): read the 64 max-abs slots the
// producer published (one per lane), wave max, frexp.  No statistics, zero or non-finite max:
// e = 0 (an overflowing input then yields inf, as fp16 would; NaN propagates).
__device__ __forceinline__ int amax_exp(const unsigned* slots, int b) {
  if (!slots) return 0;
  float m = __uint_as_float(slots[(size_t)b * 64 + (threadIdx.x & 63)]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  int e = 0;
  if (m > 0.f && m < INFINITY) {
    int E;
    (void)frexpf(m, &E);
    e = E - 14;
  }
  return __builtin_amdgcn_readfirstlane(e);
}

template <class S, int K, int BM, int BN, int TM, int TN, int G, int HMAX, int PD>
struct SplitCfg {
  static constexpr int WM = BM / (32 * TM);
  static constexpr int WN = BN / (32 * TN);
  static constexpr int CK = 16 * G;
  static constexpr int XROWS = BN + HMAX;
  static constexpr int XSZB = G * XROWS * S::ROWB;  // bytes per LDS buffer
  static constexpr int UNITS = G * XROWS * 4;       // staging units (group, row, channel quad)
  static constexpr int UPT = (UNITS + 255) / 256;
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(XSZB % 16 == 0, "");
};

#ifndef X6_ABLATE
#define X6_ABLATE 0
#endif

template <class S, int K, int BM, int BN, int TM, int TN, int G, int HMAX, int PD>
__global__ __launch_bounds__(256) void conv1d_split_kernel(Conv1dArgs a) {
  using C = SplitCfg<S, K, BM, BN, TM, TN, G, HMAX, PD>;
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
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
  const int ex = H3 ? amax_exp(a.amax_in, b) : 0;
  const float xscale = H3 ? ldexpf(1.f, -ex) : 1.f;  // exact power of two

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
    // source frame ts - rep_pad, clamped (replicate) when rep_pad > 0, else zero outside [0, Tin)
    const bool ok = (g < G) && ts >= 0 && ts < (a.rep_pad ? Tout : Tin);
    int src = ts - a.rep_pad;
    src = src < 0 ? 0 : (src >= Tin ? Tin - 1 : src);
    uvoff[i] = ok ? (unsigned)(16 * g + 4 * q) * chb + (unsigned)src * 4u : OOB_OFF;
    ulds[i] = (g < G) ? (g * C::XROWS + r) * S::ROWB + 8 * q : -1;
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
        u16x4 pv[NP];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned short h[NP];
          float v = lrelu2(xreg[i][j], slope);
          if (H3) v *= xscale;
          S::split(v, h);
#pragma unroll
          for (int p = 0; p < NP; ++p) pv[p][j] = h[p];
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) *reinterpret_cast<u16x4*>(xl + ulds[i] + 32 * p) = pv[p];
      }
    }
  };

  // A streams: f32x4 units, fragment (mb, step s, piece p) at ((mb*S + s)*NP + p)*64 + lane
  // (descriptor per m-block from wave-uniform values, step/piece offsets in the scalar soffset)
  rsrc_t ra[TM];
  const int wmu = __builtin_amdgcn_readfirstlane(wm);
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    const int mb = mt * (BM / 32) + wmu * TM + m;
    ra[m] = make_rsrc(a.w + ((size_t)mb * nc * G * K) * (NP * 256), 0xFFFFFFFFu);
  }
  const unsigned avoff = (unsigned)lane * 16u;

  f32x16 acc[S::NACC][TM][TN];
#pragma unroll
  for (int h = 0; h < S::NACC; ++h)
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n) acc[h][m][n] = f32x16{};

  const int xrow0 = wn * TN * 32 + l32;

  f32x4 ar[PD + 1][TM][NP], bcur[TN][NP], bnext[TN][NP];
#pragma unroll
  for (int p = 0; p < PD; ++p)
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int q = 0; q < NP; ++q) ar[p][m][q] = bload4(ra[m], avoff, (unsigned)(p * NP + q) * 1024u);

  auto read_b = [&](const unsigned char* xl, int g, int k, f32x4 (*dst)[NP]) {
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int r = xrow0 + n * 32 + k * d;
      const unsigned char* p = xl + (g * C::XROWS + r) * S::ROWB + 16 * half;
#pragma unroll
      for (int q = 0; q < NP; ++q) dst[n][q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
    }
  };

  load_x(0);
  store_x(0);
  __syncthreads();

  for (int c = 0; c < nc; ++c) {
    const int buf = c & 1;
    const unsigned char* xl = smem + buf * C::XSZB;
    const bool more = c + 1 < nc;
    if ((X6_ABLATE & 1) == 0 && more) load_x(c + 1);
    read_b(xl, 0, 0, bcur);
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int s = (c * G + g) * K + k;
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int q = 0; q < NP; ++q)
            ar[PD][m][q] = (X6_ABLATE & 2) ? ar[0][m][q] : bload4(ra[m], avoff, (unsigned)((s + PD) * NP + q) * 1024u);
        const bool bnext_here = (k + 1 < K) || (g + 1 < G);
        if (bnext_here) read_b(xl, (k + 1 < K) ? g : g + 1, (k + 1 < K) ? k + 1 : 0, bnext);
        // keep the prefetches ahead of this step's MFMAs (the scheduler otherwise sinks them
        // to their use and exposes the L2 / LDS latency every step)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < S::NPROD; ++e)
#pragma unroll
          for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int n = 0; n < TN; ++n)
              acc[S::PACC[e]][m][n] = S::mfma(ar[0][m][S::PA[e]], bcur[n][S::PB[e]], acc[S::PACC[e]][m][n]);
#pragma unroll
        for (int p = 0; p < PD; ++p)
#pragma unroll
          for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int q = 0; q < NP; ++q) ar[p][m][q] = ar[p + 1][m][q];
        if (bnext_here) {
#pragma unroll
          for (int n = 0; n < TN; ++n)
#pragma unroll
            for (int q = 0; q < NP; ++q) bcur[n][q] = bnext[n][q];
        }
      }
    }
    if ((X6_ABLATE & 1) == 0 && more) store_x(buf ^ 1);
    __syncthreads();
  }

  if constexpr (H3) {
    const float sc = ldexpf(1.f, ex + a.w_exp);  // undo both scalings (exact)
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n) acc[0][m][n] *= sc;
  }
  if constexpr (K == 2) {
    convT_epilogue<TM, TN, H3>(a, acc[0], b, t0 + wn * TN * 32, mt * BM + wm * TM * 32, lane);
  } else {
    conv_epilogue<TM, TN, H3>(a, acc[0], b, t0 + wn * TN * 32, mt * BM + wm * TM * 32, lane);
  }
}

// slots[b][blockIdx.x & 63] = max |x[b]| (grid-stride per item), for inputs without producer
// statistics
__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, int64_t n, unsigned* slots) {
  const float* xb = x + (size_t)blockIdx.z * n;
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    m = fmaxf(m, fabsf(xb[i]));
  publish_amax(slots, blockIdx.z, m);
}

void launch_amax(const float* x, int64_t n, int B, unsigned* slots, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>(512, std::max<int64_t>(1, (n + 255) / 256));
  hipLaunchKernelGGL(amax_kernel, dim3((unsigned)blocks, 1, B), dim3(256), 0, s, x, n, slots);
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
};
constexpr int kNumSplitTiles = sizeof(kSplitTiles) / sizeof(kSplitTiles[0]);

template <class S, int K, int BM, int BN, int TM, int TN, int G, int PD, bool WIDE>
void launch_split_t(const Conv1dArgs& a, int B, hipStream_t s) {
  dim3 grid(ceil_div(a.Tout, BN), ceil_div(a.Cout, BM), B);
  const int halo = (K - 1) * a.dil;
  if (halo <= (K - 1) * 5) {
    hipLaunchKernelGGL((conv1d_split_kernel<S, K, BM, BN, TM, TN, G, (K - 1) * 5, PD>), grid, dim3(256), 0, s, a);
  } else if (WIDE && halo <= 96) {
    hipLaunchKernelGGL((conv1d_split_kernel<S, K, BM, BN, TM, TN, G, WIDE ? 96 : 0, PD>), grid, dim3(256), 0, s, a);
  } else {
    throw Error(3, "conv1d(split): (kernel_size-1)*dilation = " + std::to_string(halo) + " too large for this tile");
  }
}

template <class S, int K>
void launch_split_k(const Conv1dArgs& a, int B, int tile, hipStream_t s) {
  switch (tile) {
    case 0: launch_split_t<S, K, 128, 128, 2, 2, 1, 1, true>(a, B, s); break;
    case 1: launch_split_t<S, K, 64, 256, 2, 2, 1, 1, true>(a, B, s); break;
    case 2: launch_split_t<S, K, 32, 512, 1, 4, 1, 1, true>(a, B, s); break;
    case 3: launch_split_t<S, K, 128, 128, 2, 2, 2, 1, false>(a, B, s); break;
    case 4: launch_split_t<S, K, 64, 128, 2, 1, 2, 1, false>(a, B, s); break;
    case 5: launch_split_t<S, K, 32, 256, 1, 2, 2, 1, false>(a, B, s); break;
    case 6: launch_split_t<S, K, 64, 256, 2, 2, 2, 1, false>(a, B, s); break;
    case 7: launch_split_t<S, K, 128, 128, 2, 2, 1, 2, false>(a, B, s); break;
    case 8: launch_split_t<S, K, 64, 128, 2, 1, 2, 2, false>(a, B, s); break;
    case 9: launch_split_t<S, K, 64, 256, 2, 2, 2, 2, false>(a, B, s); break;
    case 10: launch_split_t<S, K, 64, 256, 2, 2, 1, 2, false>(a, B, s); break;
    case 11: launch_split_t<S, K, 32, 256, 1, 2, 2, 2, false>(a, B, s); break;
    case 12: launch_split_t<S, K, 64, 128, 2, 1, 2, 3, false>(a, B, s); break;
    case 13: launch_split_t<S, K, 128, 128, 2, 2, 2, 2, false>(a, B, s); break;
    case 14: launch_split_t<S, K, 32, 256, 1, 2, 1, 1, false>(a, B, s); break;
    case 15: launch_split_t<S, K, 32, 256, 1, 2, 1, 2, false>(a, B, s); break;
    case 16: launch_split_t<S, K, 32, 128, 1, 1, 1, 2, false>(a, B, s); break;
    case 17: launch_split_t<S, K, 64, 128, 2, 1, 1, 1, false>(a, B, s); break;
    case 18: launch_split_t<S, K, 64, 128, 2, 1, 1, 2, false>(a, B, s); break;
    case 19: launch_split_t<S, K, 32, 512, 1, 4, 1, 2, false>(a, B, s); break;
    default: throw Error(3, "conv1d(split): bad tile index " + std::to_string(tile));
  }
}

template <class S>
void launch_split_s(const Conv1dArgs& a, int B, int K, int tile, hipStream_t s) {
  switch (K) {
    case 1: launch_split_k<S, 1>(a, B, tile, s); break;
    case 2: launch_split_k<S, 2>(a, B, tile, s); break;  // ConvTranspose1d (Conv1dArgs::ups)
    case 3: launch_split_k<S, 3>(a, B, tile, s); break;
    case 5: launch_split_k<S, 5>(a, B, tile, s); break;
    case 7: launch_split_k<S, 7>(a, B, tile, s); break;
    case 11: launch_split_k<S, 11>(a, B, tile, s); break;
    default: throw Error(3, "conv1d(split): kernel size " + std::to_string(K) + " not supported (1,3,5,7,11)");
  }
}
}  // namespace

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
  if (mode == MATH_FP32_F16X3) {
    if (Cout > 64) return 13;
    if (Cout > 32) return 10;
    return 14;  // one 16-channel group, 42 KB of LDS: 3 workgroups per CU
  }
  if (Cout > 64) return (K >= 11 || Cin % 32 != 0) ? 7 : 3;
  if (Cout > 32) return K <= 3 ? 10 : 1;
  return 2;
}

void launch_conv1d_split(int mode, const Conv1dArgs& a, int B, int K, int tile, hipStream_t s) {
  TTS_REQUIRE((K == 2) == (a.ups > 0), 1, "conv1d(split): K == 2 is the ConvTranspose1d form (ups > 0)");
  TTS_REQUIRE(a.ups == 0 || ((a.ups & (a.ups - 1)) == 0 && a.Cout % a.ups == 0 && a.zmode == 0 && !a.res &&
                             !a.mask && !a.cvec && a.Tout == a.Tin + 1 && a.pad == 1),
              1, "conv1d(split): bad ConvTranspose1d arguments");
  // every addressed plane must stay below 2 GiB (32-bit buffer offsets, OOB marker bit 31)
  TTS_REQUIRE((int64_t)a.Cin * a.Tin * 4 < (int64_t(1) << 31) && (int64_t)a.Cout * a.Tout * 4 < (int64_t(1) << 31), 3,
              "conv1d: a batch item's channel plane exceeds 2 GiB");
  if (mode == MATH_FP32_F16X3) launch_split_s<SchemeH3>(a, B, K, tile, s);
  else if (mode == MATH_BF16) launch_split_s<SchemeB1>(a, B, K, tile, s);
  else launch_split_s<SchemeX6>(a, B, K, tile, s);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
