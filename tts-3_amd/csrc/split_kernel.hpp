// The split-precision conv1d kernel template and its launch dispatch over (K, tile), shared by
// the per-scheme translation units kernels_conv_split_{x6,h3,b1}.hip (compiled in parallel).
// See kernels_conv_split.hip for the algorithm, the tile table and the selection.
#pragma once

#include <type_traits>

#include "split_device.hpp"

namespace tts {

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

#ifndef SPLIT_STAGE_8R
#define SPLIT_STAGE_8R 1  // staging lane map (see conv1d_split_kernel); 0: 4 rows x 4 quads per 16 lanes
#endif

#ifndef X6_ABLATE
#define X6_ABLATE 0  // ablation builds (scripts/gpu_ablate.sh): 1 no staging refill, 2 no A stream
#endif

// WaveNet gate epilogue (Conv1dArgs::gate, 128 x 128 tiles with 2 x 2 waves): the wm = 1 waves
// hold the sigmoid rows matching the wm = 0 waves' tanh rows, column for column; they pass
// sigmoid(v) through LDS (the staging buffers, free after the last chunk) and the wm = 0 waves
// store tanh(v) * sigmoid and publish its max-abs.  Same fp32 operations, in the same order, as
// the plain epilogue followed by glow_gate_kernel, so the result is bitwise that of the unfused pair.
constexpr int C_WN_MAX = 2;  // column-group waves of the gate tile (2 x 2 waves)

template <int TM, int TN, bool H3>
__device__ __forceinline__ void gate_epilogue(const Conv1dArgs& args, const f32x16 (&acc)[TM][TN], int b, int tbase,
                                              int mt, int wm, int wn, int lane, float* xch) {
  static_assert(TM * 32 == 64, "a wave row block must be one 64-row half");
  const Conv1dArgs a = args;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int H = a.gate;
  const int T = a.Tout;
  const rsrc_t rbias = make_rsrc(a.bias, (unsigned)(2 * H) * 4u);
  const rsrc_t rcv = make_rsrc(a.cvec ? a.cvec + (size_t)b * (a.cvec_bstride ? a.cvec_bstride : (int64_t)2 * H) : a.bias,
                               a.cvec ? (unsigned)(2 * H) * 4u : 0u);
  const int orow0 = (wm ? H : 0) + 64 * mt;  // original row of this wave's local row 0
  const int prow0 = mt * 128 + wm * 64;      // packed row
  float v[TM][TN][16];
#pragma unroll
  for (int m = 0; m < TM; ++m) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
      const float bv = bload(rbias, (unsigned)(prow0 + rr) * 4u, 0u) + bload(rcv, (unsigned)(orow0 + rr) * 4u, 0u);
#pragma unroll
      for (int n = 0; n < TN; ++n) v[m][n][r] = lrelu2((acc[m][n][r] + bv) * 1.f, 1.f);
    }
  }
  static_assert(TN == 2, "the two row-block waves split the output columns n = 0 / 1");
  // both waves of a column group evaluate their own half (wm = 0: tanh, wm = 1: sigmoid), hand the
  // half of the partner's columns over through LDS, and finish one column block each
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) v[m][n][r] = wm ? 1.f / (1.f + expf(-v[m][n][r])) : tanhf(v[m][n][r]);
  const int give = 1 - wm;  // the column block the partner finishes
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) xch[(((wm * C_WN_MAX + wn) * TM + m) * 16 + r) * 64 + lane] = give ? v[m][1][r] : v[m][0][r];
  __syncthreads();
  const int nk = wm;  // the column block this wave finishes
  const unsigned rowb = (unsigned)T * 4u;
  const rsrc_t rout = make_rsrc(a.y + (size_t)b * H * T, (unsigned)H * rowb);
  const int t = tbase + nk * 32 + l32;
  const unsigned voff0 = t < T ? (unsigned)t * 4u : OOB_OFF;
  float vm = 0.f;
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    const unsigned voff = t < T ? voff0 + (unsigned)(64 * mt + m * 32 + 4 * half) * rowb : OOB_OFF;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float mine = nk ? v[m][1][r] : v[m][0][r];
      const float other = xch[((((1 - wm) * C_WN_MAX + wn) * TM + m) * 16 + r) * 64 + lane];
      const float o = (wm ? other : mine) * (wm ? mine : other);  // tanh * sigmoid, as glow_gate_kernel
      if (H3) vm = t < T ? fmaxf(vm, fabsf(o)) : vm;
      bstore(rout, o, voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb, 0u);
    }
  }
  if (H3 && a.amax_out) publish_amax(a.amax_out, b, vm);
}

// PL: Conv1dArgs::planes as a template parameter (kPlaneXB16: bf16 input, kPlaneYB16: bf16
// outputs / residual / MRF sum); only the MATH_BF16 scheme instantiates PL != 0
#ifndef SPLIT_W_B1
#define SPLIT_W_B1 3  // waves per SIMD asked of the bf16 scheme's split conv kernels (0: no request; 3: k3 c256 1.23 -> 1.05 ms, ups x2 -13%; 4 spills)
#endif
template <class S, int K, int BM, int BN, int TM, int TN, int G, int HMAX, int PD, bool GATE = false, int PL = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(S::NP == 1 && SPLIT_W_B1 > 0 && !(TN == 4 && HMAX == 96)
                                                                          ? SPLIT_W_B1 : 1)))
void conv1d_split_kernel(Conv1dArgs a) {
  using C = SplitCfg<S, K, BM, BN, TM, TN, G, HMAX, PD>;
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
  constexpr bool XB = (PL & kPlaneXB16) != 0, YB = (PL & kPlaneYB16) != 0;
  using PX = PlaneT<XB>;
  static_assert(PL == 0 || (!GATE && !H3), "bf16 planes: plain epilogues of the bf16 scheme only");
  // the gate epilogue reuses the staging buffers for its sigmoid exchange (32 KiB)
  constexpr int XCHB = GATE ? 4 * C::WN * TM * TN * 16 * 64 : 0;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * C::XSZB > XCHB ? 2 * C::XSZB : XCHB];
  // bias (+ cvec) of this tile's BM rows, staged with the first input chunk: the epilogue then
  // reads LDS instead of paying an L2 latency after the last MFMA (conv: the sum bias + cvec,
  // as the epilogue's two range-checked loads give it; ConvTranspose: both, added in order)
  // (only where the 0.5-1 KB does not cost a workgroup per CU: 160 KB of LDS per CU)
  constexpr int LDS_MAIN = 2 * C::XSZB > XCHB ? 2 * C::XSZB : XCHB;
  constexpr bool SB = !GATE && 163840 / LDS_MAIN == 163840 / (LDS_MAIN + BM * 4 * (K == 2 ? 2 : 1) + 64);
  __shared__ float sbias[SB ? BM : 1], scvec[SB && K == 2 ? BM : 1];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / C::WN;
  const int wn = wave % C::WN;
  const int half = lane >> 5;
  const int l32 = lane & 31;

  const int bx = blockIdx.x, mt = blockIdx.y, b = blockIdx.z;
  const int t0 = bx * BN;
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
  const char* xb = static_cast<const char*>(plane_at<XB>(a.x, (size_t)b * (a.x_bstride ? a.x_bstride : (int64_t)Cin * Tin)));
  const unsigned chb = (unsigned)Tin * PX::ES;  // bytes per channel row

  // staging units (chunk invariant): unit u -> channel quad q, row r, group g.  SPLIT_STAGE_8R: a
  // 16-lane store group writes 8 consecutive rows x 2 quad positions; the row pitches (80 / 112 /
  // 48 B) put 8 consecutive rows on 8 distinct 16-B slots of the 128-B bank row, so the group's
  // 8-byte ds_write_b64 hit 32 distinct banks (4 rows x 4 quads: 2-way on half the groups), and a
  // load instruction reads 32 contiguous bytes per channel instead of 16
  unsigned uvoff[C::UPT];  // byte offset of channel (16g+4q) at the clamped source time, or OOB
  int ulds[C::UPT];        // LDS offset of the row's quad
#pragma unroll
  for (int i = 0; i < C::UPT; ++i) {
    const int u = tid + i * 256;
    const int q = SPLIT_STAGE_8R ? quad_pos((u >> 3) & 3) : (u & 3);
    const int rr = SPLIT_STAGE_8R ? (u >> 5) * 8 + (u & 7) : (u >> 2);
    const int g = rr / XW;
    const int r = rr - g * XW;
    const int ts = t0 - a.pad + r;
    // source frame ts - rep_pad, clamped (replicate) when rep_pad > 0, else zero outside [0, Tin)
    const bool ok = (g < G) && ts >= 0 && ts < (a.rep_pad ? Tout : Tin);
    int src = ts - a.rep_pad;
    src = src < 0 ? 0 : (src >= Tin ? Tin - 1 : src);
    uvoff[i] = ok ? (unsigned)(16 * g + 4 * q) * chb + (unsigned)src * PX::ES : OOB_OFF;
    ulds[i] = (g < G) ? (g * C::XROWS + r) * S::ROWB + 8 * quad_pos(q) : -1;
  }

  f32x4 xreg[C::UPT];
  auto load_x = [&](int c) {
    const int c0 = c * C::CK;
    const rsrc_t rx = make_rsrc(xb + (size_t)c0 * chb, (unsigned)(Cin - c0) * chb);
#pragma unroll
    for (int i = 0; i < C::UPT; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) xreg[i][j] = PX::ld(rx, uvoff[i] + (unsigned)j * chb, 0u);
    }
  };
  auto store_x = [&](int buf) {
    unsigned char* xl = smem + buf * C::XSZB;
    const float slope = a.in_slope;
#pragma unroll
    for (int i = 0; i < C::UPT; ++i) {
      if (ulds[i] >= 0) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = lrelu2(xreg[i][j], slope);
          if (H3) v[j] *= xscale;
        }
        split_store4<S>(xl + ulds[i], v[0], v[1], v[2], v[3]);
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

  float bpre = 0.f, cpre = 0.f;
  if (SB && tid < BM) {
    const int row = mt * BM + tid;
    if (row < a.Cout) {
      bpre = a.bias[row];
      if (K == 2) {
        const int co = row / a.ups;
        cpre = a.cvec ? a.cvec[(size_t)b * (a.Cout / a.ups) + co] : 0.f;
      } else {
        cpre = a.cvec ? a.cvec[(size_t)b * (a.cvec_bstride ? a.cvec_bstride : (int64_t)a.Cout) + row] : 0.f;
      }
    }
  }
  load_x(0);
  store_x(0);
  if (SB && tid < BM) {
    if (K == 2) {
      sbias[tid] = bpre;
      scvec[K == 2 ? tid : 0] = cpre;
    } else {
      sbias[tid] = bpre + cpre;
    }
  }
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
  if constexpr (GATE) {
    static_assert(BM == 128 && C::WM == 2, "gate epilogue");
    gate_epilogue<TM, TN, H3>(a, acc[0], b, t0 + wn * TN * 32, mt, wm, wn, lane, reinterpret_cast<float*>(smem));
  } else if constexpr (K == 2) {
    convT_epilogue<TM, TN, H3, YB>(a, acc[0], b, t0 + wn * TN * 32, mt * BM + wm * TM * 32, lane, SB ? sbias : nullptr, SB ? scvec : nullptr, mt * BM);
  } else {
    if constexpr (K == 1) {
      if (!YB && a.wn_rows) {
        conv_epilogue_wn<TM, TN, H3>(a, acc[0], b, t0 + wn * TN * 32, mt * BM + wm * TM * 32, lane, SB ? sbias : nullptr,
                                     mt * BM);
        return;
      }
    }
    conv_epilogue<TM, TN, H3, YB>(a, acc[0], b, t0 + wn * TN * 32, mt * BM + wm * TM * 32, lane, 0x7fffffff, SB ? sbias : nullptr, mt * BM);
  }
}

namespace split_detail {
// PLV: this tile has bf16-plane instances (the MATH_BF16 tile choices, conv1d_split_tile_for)
template <class S, int K, int BM, int BN, int TM, int TN, int G, int PD, bool WIDE, bool GATE = false, bool PLV = false>
void launch_split_t(const Conv1dArgs& a, int B, hipStream_t s) {
  dim3 grid(ceil_div(a.Tout, BN), ceil_div(a.Cout, BM), B);
  const int halo = (K - 1) * a.dil;
  if constexpr (GATE) {
    TTS_REQUIRE(a.gate > 0 && a.gate % 64 == 0 && a.Cout == 2 * a.gate && a.zmode == 0 && !a.res && !a.mask &&
                    a.ups == 0 && halo <= (K - 1) * 5,
                1, "conv1d(split): bad gated in_layer arguments");
    hipLaunchKernelGGL((conv1d_split_kernel<S, K, BM, BN, TM, TN, G, (K - 1) * 5, PD, true>), grid, dim3(256), 0, s,
                       a);
    return;
  }
  TTS_REQUIRE(a.gate == 0, 1, "conv1d(split): the gate epilogue needs tile kSplitGateTile");
  TTS_REQUIRE(a.wn_rows == 0 || (K == 1 && a.wn_rows % 32 == 0 && a.Cout == 2 * a.wn_rows && a.mask && a.z &&
                                 a.y && (a.zmode == 1 || a.zmode == 2) && a.ups == 0),
              1, "conv1d(split): bad WaveNet update-epilogue arguments");
  if (a.planes != 0) {
    // bf16 activation planes: the bf16 scheme's HiFiGAN tiles; x fp32 -> y bf16 only for conv_pre (K 7)
    constexpr bool OK = std::is_same<S, SchemeB1>::value && PLV && K != 1;
    TTS_REQUIRE(OK && a.wn_rows == 0 && !a.mask && (a.planes == (kPlaneXB16 | kPlaneYB16) || (a.planes == kPlaneYB16 && K == 7)),
                3, "conv1d(split): bf16 planes are not built for this tile / kernel size");
    if constexpr (OK) {
      auto go = [&](auto pl_tag) {
        constexpr int PLc = decltype(pl_tag)::value;
        if (halo <= (K - 1) * 5) {
          hipLaunchKernelGGL((conv1d_split_kernel<S, K, BM, BN, TM, TN, G, (K - 1) * 5, PD, false, PLc>), grid, dim3(256), 0, s, a);
        } else if (WIDE && halo <= 96) {
          hipLaunchKernelGGL((conv1d_split_kernel<S, K, BM, BN, TM, TN, G, WIDE ? 96 : 0, PD, false, PLc>), grid, dim3(256), 0, s, a);
        } else {
          throw Error(3, "conv1d(split): (kernel_size-1)*dilation = " + std::to_string(halo) + " too large for this tile");
        }
      };
      if (a.planes == kPlaneYB16) {
        if constexpr (K == 7) go(std::integral_constant<int, kPlaneYB16>{});
      } else {
        go(std::integral_constant<int, kPlaneXB16 | kPlaneYB16>{});
      }
    }
    return;
  }
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
    case 0: launch_split_t<S, K, 128, 128, 2, 2, 1, 1, true, false, true>(a, B, s); break;
    case 1: launch_split_t<S, K, 64, 256, 2, 2, 1, 1, true, false, true>(a, B, s); break;
    case 2: launch_split_t<S, K, 32, 512, 1, 4, 1, 1, true, false, true>(a, B, s); break;
    case 3: launch_split_t<S, K, 128, 128, 2, 2, 2, 1, false, false, true>(a, B, s); break;
    case 4: launch_split_t<S, K, 64, 128, 2, 1, 2, 1, false>(a, B, s); break;
    case 5: launch_split_t<S, K, 32, 256, 1, 2, 2, 1, false>(a, B, s); break;
    case 6: launch_split_t<S, K, 64, 256, 2, 2, 2, 1, false>(a, B, s); break;
    case 7: launch_split_t<S, K, 128, 128, 2, 2, 1, 2, false, false, true>(a, B, s); break;
    case 8: launch_split_t<S, K, 64, 128, 2, 1, 2, 2, false>(a, B, s); break;
    case 9: launch_split_t<S, K, 64, 256, 2, 2, 2, 2, false>(a, B, s); break;
    case 10: launch_split_t<S, K, 64, 256, 2, 2, 1, 2, false, false, true>(a, B, s); break;
    case 11: launch_split_t<S, K, 32, 256, 1, 2, 2, 2, false>(a, B, s); break;
    case 12: launch_split_t<S, K, 64, 128, 2, 1, 2, 3, false>(a, B, s); break;
    case 13: launch_split_t<S, K, 128, 128, 2, 2, 2, 2, false, false, true>(a, B, s); break;
    case 14: launch_split_t<S, K, 32, 256, 1, 2, 1, 1, false, false, true>(a, B, s); break;
    case 15: launch_split_t<S, K, 32, 256, 1, 2, 1, 2, false>(a, B, s); break;
    case 16: launch_split_t<S, K, 32, 128, 1, 1, 1, 2, false>(a, B, s); break;
    case 17: launch_split_t<S, K, 64, 128, 2, 1, 1, 1, false>(a, B, s); break;
    case 18: launch_split_t<S, K, 64, 128, 2, 1, 1, 2, false>(a, B, s); break;
    case 19: launch_split_t<S, K, 32, 512, 1, 4, 1, 2, false>(a, B, s); break;
    case kSplitGateTile:
      if constexpr (K == 3 || K == 5 || K == 7) launch_split_t<S, K, 128, 128, 2, 2, 2, 2, false, true>(a, B, s);
      else throw Error(3, "conv1d(split): the gated in_layer takes kernel size 3, 5 or 7");
      break;
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
}  // namespace split_detail

}  // namespace tts
