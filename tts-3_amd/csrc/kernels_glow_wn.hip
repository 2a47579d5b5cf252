// One WaveNet layer per launch (GlowWnLayerArgs, glow.hpp) for the Glow-TTS decoder and the VITS
// flows: TTS/tts/layers/generic/wavenet.py:101-115 (in_layers[l] -> + g_l ->
// fused_add_tanh_sigmoid_multiply (:6-13) -> res_skip_layers[l] -> residual / skip update).
//
// A workgroup owns 32 output columns of one utterance and the whole hidden width H (4 waves):
//   stage   h[:, t0 - pad, t0 + 32 + pad) -> LDS as split pieces (the split conv kernel's staging)
//   phase 1 the in_layer GEMM [2H] x [H*K], wave w on 32-row blocks w, w + 4, ...; + bias + cond
//           -> the fp32 xin tile in LDS (over the h window)
//   gate    tanh(xin[c]) * sigmoid(xin[H + c]) -> acts in LDS as the next GEMM's B operand
//   phase 2 the res_skip GEMM [2H or H] x [H], then the update epilogue (h_out = (h_in + rs) * mask,
//           skip (+)= rs[H:]; last layer skip = (skip + rs) * mask) and the next consumer's max-abs
// xin, acts and rs never reach HBM (the unfused layer writes and re-reads 5H floats per column)
// and the layer's four dependent launches become one.  Accumulation order, bias / cond sums,
// the gate's and the update's fp32 operations are those of conv1d_split_kernel (tile 13) +
// glow_gate_kernel + conv1d_split_kernel + glow_wn_update_kernel, so bf16 results are bitwise
// those of the unfused layer; in f16x3 the acts operand takes the fixed exponent of |acts| < 1
// instead of its per-utterance max-abs exponent (the same whenever max |acts| >= 0.5, and bitwise
// on the test inputs); bf16x6 differs in the last bit of ~10% of the outputs (not isolated).
#include <cstdlib>

#include "glow.hpp"
#include "split_device.hpp"

namespace tts {
namespace {

constexpr int WN_COLS = 32;                   // output columns per workgroup
constexpr int WN_HALO_MAX = 16;               // (K - 1) * dil
constexpr int WN_XR = WN_COLS + WN_HALO_MAX;  // staged h rows, at most
constexpr int WN_XP = WN_COLS + 1;            // fp32 pitch of the xin tile rows
#ifndef WN_PD
#define WN_PD 2  // A-operand prefetch distance (steps)
#endif
// tuning switches (A/B builds): WN_STAGE_BATCH issues every h-window load of a thread before its
// first LDS store (one HBM latency instead of one per staging round); WN_EARLY_A issues each GEMM's
// first WN_PD weight steps before the work that precedes it (the staging, the gate); WN_EPI_EARLY
// loads the update epilogue's h / skip / bias operands before the res_skip GEMM
#ifndef WN_STAGE_BATCH
#define WN_STAGE_BATCH 1
#endif
#ifndef WN_EARLY_A
#define WN_EARLY_A 1
#endif
#ifndef WN_ABLATE
#define WN_ABLATE 0  // timing ablations only (wrong results): 1 no MFMAs, 2 no A loads in the loops,
                     // 4 no gate transcendentals, 8 no h-window loads, 16 no res_skip GEMM
#endif
#ifndef WN_EPI_EARLY
#define WN_EPI_EARLY 0  // measured neutral to slightly slower (profiles/ab_r05_wn_tune.txt)
#endif
constexpr int WN_ACTS_EXP = -14;              // f16x3 exponent of acts: |acts| < 1 -> [0, 2^14)

template <class S, int H_>
struct WnCfg {
  static constexpr int H = H_;
  static constexpr int NG = H / 16;  // 16-channel groups of h and acts
  static constexpr int HWIN = NG * WN_XR * S::ROWB;
  static constexpr int XIN = 2 * H * WN_XP * 4;
  static constexpr int U1 = HWIN > XIN ? HWIN : XIN;
  static constexpr int ACTS = NG * WN_COLS * S::ROWB;
  static constexpr int LDS = U1 + ACTS;
  static_assert(LDS <= 160 * 1024, "LDS");
};

// acc[m] += W[block m] * B over NSTEP steps: A fragments streamed from the split packing (wave
// block m at ra[m], step s piece q at soffset (s * NP + q) KiB), B fragments of group g, tap k read
// from LDS by bsrc(g, k, dst); the same product order per accumulator as conv1d_split_kernel.
// Every block is computed (phase 2 of the last layer points its surplus blocks at a valid one and
// drops them in the epilogue): no branches around the MFMAs
// The first WN_PD steps' A fragments (the GEMM's prologue; wn_gemm expects them in ar[0 .. PD-1])
template <class S, int TMW>
__device__ __forceinline__ void wn_prefetch(f32x4 (&ar)[WN_PD + 1][TMW][S::NP], const rsrc_t (&ra)[TMW], unsigned avoff) {
#pragma unroll
  for (int p = 0; p < WN_PD; ++p)
#pragma unroll
    for (int m = 0; m < TMW; ++m)
#pragma unroll
      for (int q = 0; q < S::NP; ++q) ar[p][m][q] = bload4(ra[m], avoff, (unsigned)(p * S::NP + q) * 1024u);
}

// fully unrolled (NGR groups x KS taps): the prefetch ring and the B double buffer are renamed
// registers, with no moves, loop counters or branches between the MFMAs
template <class S, int TMW, int KS, int NGR, class BSrc>
__device__ __forceinline__ void wn_gemm(f32x16 (&acc)[TMW], f32x4 (&ar)[WN_PD + 1][TMW][S::NP], const rsrc_t (&ra)[TMW],
                                        unsigned avoff, BSrc bsrc) {
  constexpr int NP = S::NP;
  constexpr int ngroups = NGR;
  f32x4 bcur[NP], bnext[NP];
  bsrc(0, 0, bcur);
#pragma unroll
  for (int g = 0; g < ngroups; ++g) {
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int s = g * KS + k;
#pragma unroll
      for (int m = 0; m < TMW; ++m)
#pragma unroll
        for (int q = 0; q < NP; ++q)
          ar[WN_PD][m][q] = (WN_ABLATE & 2) ? ar[0][m][q] : bload4(ra[m], avoff, (unsigned)((s + WN_PD) * NP + q) * 1024u);
      const bool nx = (k + 1 < KS) || (g + 1 < ngroups);
      if (nx) bsrc((k + 1 < KS) ? g : g + 1, (k + 1 < KS) ? k + 1 : 0, bnext);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < S::NPROD; ++e)
#pragma unroll
        for (int m = 0; m < TMW; ++m)
          if (!(WN_ABLATE & 1)) acc[m] = S::mfma(ar[0][m][S::PA[e]], bcur[S::PB[e]], acc[m]);
#pragma unroll
      for (int p = 0; p < WN_PD; ++p)
#pragma unroll
        for (int m = 0; m < TMW; ++m)
#pragma unroll
          for (int q = 0; q < NP; ++q) ar[p][m][q] = ar[p + 1][m][q];
      if (nx) {
#pragma unroll
        for (int q = 0; q < NP; ++q) bcur[q] = bnext[q];
      }
    }
  }
}

// wn_gemm with a runtime group count (the fused start conv: C2/2 input channels), 1x1 only
template <class S, int TMW, class BSrc>
__device__ __forceinline__ void wn_gemm_rt(f32x16 (&acc)[TMW], f32x4 (&ar)[WN_PD + 1][TMW][S::NP], const rsrc_t (&ra)[TMW],
                                           int ngroups, unsigned avoff, BSrc bsrc) {
  constexpr int NP = S::NP;
  f32x4 bcur[NP];
  for (int g = 0; g < ngroups; ++g) {
    bsrc(g, 0, bcur);
#pragma unroll
    for (int m = 0; m < TMW; ++m)
#pragma unroll
      for (int q = 0; q < NP; ++q) ar[WN_PD][m][q] = bload4(ra[m], avoff, (unsigned)((g + WN_PD) * NP + q) * 1024u);
#pragma unroll
    for (int e = 0; e < S::NPROD; ++e)
#pragma unroll
      for (int m = 0; m < TMW; ++m) acc[m] = S::mfma(ar[0][m][S::PA[e]], bcur[S::PB[e]], acc[m]);
#pragma unroll
    for (int p = 0; p < WN_PD; ++p)
#pragma unroll
      for (int m = 0; m < TMW; ++m)
#pragma unroll
        for (int q = 0; q < NP; ++q) ar[p][m][q] = ar[p + 1][m][q];
  }
}

// NW waves per workgroup: 4 (one per SIMD, TMW = H / 64 row blocks each), or more with the same MFMA
// work per SIMD: 12 for H = 192 (three per SIMD, one row block each), 8 for H = 128 (one block) and
// H = 256 (two), so a SIMD's waves hide each other's load, LDS and barrier latency and the staging,
// gate and tail loops spread over more threads.  A wave whose block is past a GEMM's row count
// skips that GEMM (TMW = 1), instead of computing a dropped block
template <class S, int K, int H_, int NW>
__global__ __launch_bounds__(64 * NW) void glow_wn_layer_kernel(GlowWnLayerArgs args) {
  constexpr int TMW = 2 * H_ / 32 / NW;  // row blocks per wave (phase 1: 2H rows)
  constexpr int NT = 64 * NW;            // threads
  static_assert(TMW * NW * 32 == 2 * H_, "row blocks per wave");
  using C = WnCfg<S, H_>;
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
  constexpr int H = C::H;
  constexpr int NG = C::NG;
  __shared__ __attribute__((aligned(16))) unsigned char smem[C::LDS];
  __shared__ float red[NW];  // the end conv's per-tile max-abs
  unsigned char* hwin = smem;                   // stage / phase 1: the h window (split pieces)
  float* xin = reinterpret_cast<float*>(smem);  // after phase 1: xin tile [2H][WN_XP] fp32
  unsigned char* acts = smem + C::U1;           // phase 2's B operand (split pieces)

  const GlowWnLayerArgs a = args;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * WN_COLS;
  const int Th = a.Th;
  const int d = a.dil;
  const int XR = WN_COLS + (K - 1) * d;
  const int pad = d * (K - 1) / 2;
  const size_t item = (size_t)b * H * Th;
  const unsigned rowb = (unsigned)Th * 4u;
  const unsigned plane = (unsigned)H * rowb;
  const unsigned avoff = (unsigned)lane * 16u;

  // ---- stage the h window: unit u = (group g, channel quad q, row r), 4 channels of one frame
  const int ex = H3 ? amax_exp(a.amax_h, b) : 0;
  const float xscale = H3 ? ldexpf(1.f, -ex) : 1.f;  // exact power of two
  // phase 1's weights: wave w on 32-row blocks w + 4 m (4 TMW = 2H / 32 blocks)
  f32x16 acc[TMW];
  bool on[TMW];
  rsrc_t ra[TMW];
  f32x4 ar[WN_PD + 1][TMW][NP];
#pragma unroll
  for (int m = 0; m < TMW; ++m) {
    acc[m] = f32x16{};
    ra[m] = make_rsrc(a.w_in + (size_t)(w + NW * m) * a.steps_in * (NP * 256), 0xFFFFFFFFu);
  }
  if (WN_EARLY_A) wn_prefetch<S, TMW>(ar, ra, avoff);
  {
    const rsrc_t rh = make_rsrc(a.h_in + item, plane);
    const int units = NG * 4 * XR;
    auto unit_off = [&](int u, int& lds) -> unsigned {
      const int r = u % XR;
      const int gq = u / XR;
      const int q = gq & 3, g = gq >> 2;
      const int ts = t0 - pad + r;
      lds = (g * XR + r) * S::ROWB + 8 * quad_pos(q);
      return (u < units && ts >= 0 && ts < Th) ? (unsigned)(16 * g + 4 * q) * rowb + (unsigned)ts * 4u : OOB_OFF;
    };
    if (WN_STAGE_BATCH) {
      constexpr int UPT = (NG * 4 * WN_XR + NT - 1) / NT;
      float v[UPT][4];
      int lds[UPT];
#pragma unroll
      for (int i = 0; i < UPT; ++i) {
        const unsigned off = unit_off(tid + NT * i, lds[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] = (WN_ABLATE & 8) ? 0.f : bload(rh, off + (unsigned)j * rowb, 0u);
      }
#pragma unroll
      for (int i = 0; i < UPT; ++i) {
        if (tid + NT * i < units) {
          if (H3) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[i][j] *= xscale;
          }
          split_store4<S>(hwin + lds[i], v[i][0], v[i][1], v[i][2], v[i][3]);
        }
      }
    } else {
      for (int u = tid; u < units; u += NT) {
        int lds;
        const unsigned off = unit_off(u, lds);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = bload(rh, off + (unsigned)j * rowb, 0u);
          if (H3) v[j] *= xscale;
        }
        split_store4<S>(hwin + lds, v[0], v[1], v[2], v[3]);
      }
    }
  }
  __syncthreads();

  // ---- phase 1: in_layer
  if (!WN_EARLY_A) wn_prefetch<S, TMW>(ar, ra, avoff);
  wn_gemm<S, TMW, K, NG>(acc, ar, ra, avoff, [&](int g, int k, f32x4* dst) {
    const unsigned char* p = hwin + (g * XR + l32 + k * d) * S::ROWB + 16 * half;
#pragma unroll
    for (int q = 0; q < NP; ++q) dst[q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
  });
  if constexpr (H3) {
    const float sc = ldexpf(1.f, ex + a.w_exp_in);  // undo both scalings (exact)
#pragma unroll
    for (int m = 0; m < TMW; ++m) acc[m] *= sc;
  }
  __syncthreads();  // every wave is done with the h window: the xin tile overwrites it
  {
    const rsrc_t rbias = make_rsrc(a.b_in, (unsigned)(2 * H) * 4u);
    // an absent cond reads 0 through a 0-byte descriptor: bias + 0, as the split kernel stages it
    const rsrc_t rcv = make_rsrc(a.cvec ? a.cvec + (size_t)b * a.cvec_bstride : a.b_in, a.cvec ? (unsigned)(2 * H) * 4u : 0u);
#pragma unroll
    for (int m = 0; m < TMW; ++m) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * (w + NW * m) + (r & 3) + 8 * (r >> 2) + 4 * half;
        const float bv = bload(rbias, (unsigned)row * 4u, 0u) + bload(rcv, (unsigned)row * 4u, 0u);
        xin[row * WN_XP + l32] = acc[m][r] + bv;
      }
    }
  }
  // phase 2's weights (res_skip, 2H rows, the last layer H): wave w on blocks w + 4 m
  const int nmb = (a.last ? H : 2 * H) / 32;
#pragma unroll
  for (int m = 0; m < TMW; ++m) {
    const int mb = w + NW * m;
    acc[m] = f32x16{};
    on[m] = mb < nmb;
    ra[m] = make_rsrc(a.w_rs + (size_t)(mb < a.rs_blocks ? mb : 0) * a.steps_rs * (NP * 256), 0xFFFFFFFFu);
  }
  const bool run2 = TMW > 1 || on[0];  // wave-uniform: this wave has a res_skip block
  if (WN_EARLY_A && run2) wn_prefetch<S, TMW>(ar, ra, avoff);
  __syncthreads();

  // ---- gate: acts = tanh(xin[c]) * sigmoid(xin[H + c]) (glow_gate_kernel), 4 channels per unit
  {
    const float ascale = H3 ? ldexpf(1.f, -WN_ACTS_EXP) : 1.f;
    for (int u = tid; u < (H / 4) * WN_COLS; u += NT) {
      const int col = u & (WN_COLS - 1);
      const int cq = u / WN_COLS;
      float av[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = 4 * cq + j;
        const float x = xin[c * WN_XP + col];
        const float gg = xin[(H + c) * WN_XP + col];
        const float sg = (WN_ABLATE & 4) ? gg : 1.f / (1.f + expf(-gg));
        av[j] = ((WN_ABLATE & 4) ? x : tanhf(x)) * sg;
        if (H3) av[j] *= ascale;
      }
      split_store4<S>(acts + ((cq >> 2) * WN_COLS + col) * S::ROWB + 8 * quad_pos(cq & 3), av[0], av[1], av[2], av[3]);
    }
  }
  __syncthreads();

  // ---- update epilogue operands (glow_wn_update_kernel's on v = rs): h_in / skip / bias per block
  const int t = t0 + l32;
  const bool tok = t < Th;
  const rsrc_t rbias = make_rsrc(a.b_rs, (unsigned)nmb * 128u);
  const rsrc_t rmask = make_rsrc(a.mask + (size_t)b * Th, rowb);
  const rsrc_t rhi = make_rsrc(a.h_in + item, plane);
  const rsrc_t rho = make_rsrc(a.last ? a.h_in + item : a.h_out + item, a.last ? 0u : plane);
  const rsrc_t rsk = make_rsrc(a.skip + item, plane);
  const bool first = a.first != 0, last = a.last != 0;
  float ov[TMW][16], bv[TMW][16];
  float mv = 0.f;
  auto epi_loads = [&]() {
    mv = bload(rmask, tok ? (unsigned)t * 4u : OOB_OFF, 0u);
#pragma unroll
    for (int m = 0; m < TMW; ++m) {
      const int mb = w + NW * m;
      const bool hrow = !last && mb < H / 32;  // wave-uniform: a 32-row block is one side
      const int prow0 = (hrow || last ? 32 * mb : 32 * mb - H) + 4 * half;
      const unsigned voff = (tok && on[m]) ? ((unsigned)prow0 * (unsigned)Th + (unsigned)t) * 4u : OOB_OFF;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const unsigned ro = voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb;
        ov[m][r] = hrow ? bload(rhi, ro, 0u) : (first ? 0.f : bload(rsk, ro, 0u));
        bv[m][r] = bload(rbias, (unsigned)(32 * mb + (r & 3) + 8 * (r >> 2) + 4 * half) * 4u, 0u);
      }
    }
  };
  if (WN_EPI_EARLY) epi_loads();

  // ---- phase 2: res_skip
  if (!WN_EARLY_A && run2) wn_prefetch<S, TMW>(ar, ra, avoff);
  if (!(WN_ABLATE & 16) && run2) wn_gemm<S, TMW, 1, NG>(acc, ar, ra, avoff, [&](int g, int, f32x4* dst) {
    const unsigned char* p = acts + (g * WN_COLS + l32) * S::ROWB + 16 * half;
#pragma unroll
    for (int q = 0; q < NP; ++q) dst[q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
  });
  if constexpr (H3) {
    const float sc = ldexpf(1.f, WN_ACTS_EXP + a.w_exp_rs);
#pragma unroll
    for (int m = 0; m < TMW; ++m) acc[m] *= sc;
  }

  // ---- update epilogue (glow_wn_update_kernel's operations on v = rs)
  if (!WN_EPI_EARLY) epi_loads();
  const bool fuse_end = last && a.w_end != nullptr;  // uniform
  float so[TMW][16];  // fuse_end: this wave's final skip values (the end conv's B operand)
  float vmax = 0.f;
#pragma unroll
  for (int m = 0; m < TMW; ++m) {
    const int mb = w + NW * m;
    if (!on[m]) continue;
    const bool hrow = !last && mb < H / 32;
    const int prow0 = (hrow || last ? 32 * mb : 32 * mb - H) + 4 * half;
    const unsigned voff = tok ? ((unsigned)prow0 * (unsigned)Th + (unsigned)t) * 4u : OOB_OFF;
    float vm = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned ro = voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb;
      const float v = acc[m][r] + bv[m][r];
      if (hrow) {
        const float o = (ov[m][r] + v) * mv;
        vm = fmaxf(vm, fabsf(o));
        bstore(rho, o, ro, 0u);
      } else if (last) {
        const float o = (first ? v : ov[m][r] + v) * mv;
        vm = fmaxf(vm, fabsf(o));
        so[m][r] = o;
        if (!fuse_end) bstore(rsk, o, ro, 0u);
      } else {
        bstore(rsk, first ? v : ov[m][r] + v, ro, 0u);
      }
    }
    if (tok) vmax = fmaxf(vmax, vm);
  }
  if (!fuse_end) {
    if (H3 && a.amax_out) publish_amax(a.amax_out, b, vmax);
    return;
  }

  // ---- phase 3 (last layer): end_out = w_end * skip + b_end (conv1d_split_kernel's operations;
  // f16x3: the operand exponent of this tile's max |skip| instead of the utterance's)
  int et = 0;
  if (H3) {
    const float m = wave_max(vmax);
    if (lane == 0) red[w] = m;
  }
  __syncthreads();  // the max, and every wave is done reading acts
  if (H3) {
    float m = red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) m = fmaxf(m, red[i]);
    if (m > 0.f && m < INFINITY) {
      int E;
      (void)frexpf(m, &E);
      et = E - 14;
    }
  }
  const float sin_ = H3 ? ldexpf(1.f, -et) : 1.f;
#pragma unroll
  for (int m = 0; m < TMW; ++m) {
    if (!on[m]) continue;
    const int mb = w + NW * m;  // skip rows 32 mb .. + 31: channel groups 2 mb, 2 mb + 1
#pragma unroll
    for (int gs = 0; gs < 2; ++gs)
      store_xt8<S>(acts + ((2 * mb + gs) * WN_COLS + l32) * S::ROWB + 16 * half, so[m], 8 * gs, sin_);
  }
  const int nmb3 = a.end_rows / 32;
#pragma unroll
  for (int m = 0; m < TMW; ++m) {
    const int mb = w + NW * m;
    acc[m] = f32x16{};
    on[m] = mb < nmb3;
    ra[m] = make_rsrc(a.w_end + (size_t)(mb < a.end_blocks ? mb : 0) * a.end_steps * (NP * 256), 0xFFFFFFFFu);
  }
  const bool run3 = TMW > 1 || on[0];
  if (run3) wn_prefetch<S, TMW>(ar, ra, avoff);
  __syncthreads();
  if (run3) wn_gemm<S, TMW, 1, NG>(acc, ar, ra, avoff, [&](int g, int, f32x4* dst) {
    const unsigned char* p = acts + (g * WN_COLS + l32) * S::ROWB + 16 * half;
#pragma unroll
    for (int q = 0; q < NP; ++q) dst[q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
  });
  if constexpr (H3) {
    const float sc = ldexpf(1.f, et + a.w_exp_end);
#pragma unroll
    for (int m = 0; m < TMW; ++m) acc[m] *= sc;
  }
  const rsrc_t rbe = make_rsrc(a.b_end, (unsigned)a.end_rows * 4u);
  if (a.tail_x == nullptr) {
    const rsrc_t reo = make_rsrc(a.end_out + (size_t)b * a.end_rows * Th, (unsigned)a.end_rows * rowb);
#pragma unroll
    for (int m = 0; m < TMW; ++m) {
      if (!on[m]) continue;
      const int row0 = 32 * (w + NW * m) + 4 * half;
      const unsigned voff = tok ? ((unsigned)row0 * (unsigned)Th + (unsigned)t) * 4u : OOB_OFF;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2);
        const float bvv = bload(rbe, (unsigned)(row0 + rr) * 4u, 0u);
        bstore(reo, (acc[m][r] + bvv) * 1.f, voff + (unsigned)rr * rowb, 0u);
      }
    }
    return;
  }

  // ---- reverse flows: this flow's inverse tail on the tile's end output (glow_tail_kernel's
  // operations; num_splits 4), then the next flow's start conv (conv1d_split_kernel's operations,
  // f16x3 operand exponent of the tile's max |x0|)
  const int C2 = a.end_rows, hf = C2 / 2;
  float* eo = xin;                  // [C2][WN_XP] end output (the xin tile is free since the gate)
  float* x0t = xin + C2 * WN_XP;    // [C2/2][WN_XP] the updated x0 half
#pragma unroll
  for (int m = 0; m < TMW; ++m) {
    if (!on[m]) continue;
    const int row0 = 32 * (w + NW * m) + 4 * half;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2);
      const float bvv = bload(rbe, (unsigned)(row0 + rr) * 4u, 0u);
      eo[(row0 + rr) * WN_XP + l32] = (acc[m][r] + bvv) * 1.f;
    }
  }
  __syncthreads();
  {
    constexpr int SP = 4;
    float Wm[SP][SP];
#pragma unroll
    for (int o = 0; o < SP; ++o)
#pragma unroll
      for (int g = 0; g < SP; ++g) Wm[o][g] = a.winv[o * SP + g];
    const int G = C2 / SP;
    float vx = 0.f;
    for (int u = tid; u < G * WN_COLS; u += NT) {
      const int col = u & (WN_COLS - 1);
      const int i = u / WN_COLS;
      const int tc = t0 + col;
      const bool ok = tc < Th;
      const float m = ok ? a.mask[(size_t)b * Th + tc] : 0.f;
      float z[SP];
      int chs[SP];
#pragma unroll
      for (int g = 0; g < SP; ++g) {
        const int aa = g / (SP / 2), j = g % (SP / 2);
        const int ch = aa * hf + i * (SP / 2) + j;
        chs[g] = ch;
        const float xv = ok ? a.tail_x[((size_t)b * C2 + ch) * Th + tc] : 0.f;
        if (ch < hf) {
          z[g] = xv;  // z_0 = x_0
        } else {
          const float tt = eo[(ch - hf) * WN_XP + col];
          float sv = eo[ch * WN_XP + col];
          if (a.sigmoid_scale) sv = logf(1e-6f + 1.f / (1.f + expf(-(sv + 2.f))));
          z[g] = (xv - tt) * expf(-sv) * m;  // z_1 = (x_1 - t) * exp(-s) * mask
        }
      }
#pragma unroll
      for (int o = 0; o < SP; ++o) {
        float v = 0.f;
#pragma unroll
        for (int g = 0; g < SP; ++g) v = fmaf(Wm[o][g], z[g], v);
        v *= m;                                                  // InvConvNear: * x_mask
        const int ch = chs[o];
        v = (v - a.abias[ch]) * expf(-a.logs[ch]) * m;           // ActNorm reverse
        if (ok) a.tail_x[((size_t)b * C2 + ch) * Th + tc] = v;
        if (ch < hf) {
          x0t[ch * WN_XP + col] = v;
          vx = fmaxf(vx, fabsf(v));
        }
      }
    }
    if (H3) {
      const float mm = wave_max(vx);
      if (lane == 0) red[w] = mm;
    }
  }
  __syncthreads();
  int e2 = 0;
  if (H3) {
    float mm = red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) mm = fmaxf(mm, red[i]);
    if (mm > 0.f && mm < INFINITY) {
      int E;
      (void)frexpf(mm, &E);
      e2 = E - 14;
    }
  }
  {
    const float s2 = H3 ? ldexpf(1.f, -e2) : 1.f;
    for (int u = tid; u < (hf / 4) * WN_COLS; u += NT) {
      const int col = u & (WN_COLS - 1);
      const int cq = u / WN_COLS;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = x0t[(4 * cq + j) * WN_XP + col];
        if (H3) v[j] *= s2;
      }
      split_store4<S>(acts + ((cq >> 2) * WN_COLS + col) * S::ROWB + 8 * quad_pos(cq & 3), v[0], v[1], v[2], v[3]);
    }
  }
  const int nmbs = H / 32;
#pragma unroll
  for (int m = 0; m < TMW; ++m) {
    const int mb = w + NW * m;
    acc[m] = f32x16{};
    on[m] = mb < nmbs;
    ra[m] = make_rsrc(a.w_start + (size_t)(mb < a.start_blocks ? mb : 0) * a.start_steps * (NP * 256), 0xFFFFFFFFu);
  }
  const bool run4 = TMW > 1 || on[0];
  if (run4) wn_prefetch<S, TMW>(ar, ra, avoff);
  __syncthreads();
  if (run4) wn_gemm_rt<S, TMW>(acc, ar, ra, hf / 16, avoff, [&](int g, int, f32x4* dst) {
    const unsigned char* p = acts + (g * WN_COLS + l32) * S::ROWB + 16 * half;
#pragma unroll
    for (int q = 0; q < NP; ++q) dst[q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
  });
  if constexpr (H3) {
    const float sc = ldexpf(1.f, e2 + a.w_exp_start);
#pragma unroll
    for (int m = 0; m < TMW; ++m) acc[m] *= sc;
  }
  // h_next = (start(x0) + bias) * mask (the start conv's epilogue, glow.py:212)
  const rsrc_t rbs = make_rsrc(a.b_start, (unsigned)H * 4u);
  const rsrc_t rhn = make_rsrc(a.h_next + item, plane);
  float hmax = 0.f;
#pragma unroll
  for (int m = 0; m < TMW; ++m) {
    if (!on[m]) continue;
    const int row0 = 32 * (w + NW * m) + 4 * half;
    const unsigned voff = tok ? ((unsigned)row0 * (unsigned)Th + (unsigned)t) * 4u : OOB_OFF;
    float vm = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2);
      const float bsv = bload(rbs, (unsigned)(row0 + rr) * 4u, 0u);
      const float hv = (acc[m][r] + bsv) * mv;
      vm = fmaxf(vm, fabsf(hv));
      bstore(rhn, hv, voff + (unsigned)rr * rowb, 0u);
    }
    if (tok) hmax = fmaxf(hmax, vm);
  }
  if (H3 && a.amax_hnext) publish_amax(a.amax_hnext, b, hmax);
}

template <class S, int H, int NW>
void launch_wn_s(const GlowWnLayerArgs& a, int B, hipStream_t s) {
  const dim3 grid(ceil_div(a.Th, WN_COLS), B);
  if (a.K == 3) hipLaunchKernelGGL((glow_wn_layer_kernel<S, 3, H, NW>), grid, dim3(64 * NW), 0, s, a);
  else hipLaunchKernelGGL((glow_wn_layer_kernel<S, 5, H, NW>), grid, dim3(64 * NW), 0, s, a);
}

// more than one wave per SIMD (round 6): H = 192 (Glow-TTS LJSpeech, the VITS flows and posterior
// encoder) 12 waves, H = 128 and 256 eight; TTS_MI355X_WN_WAVES=4 keeps the round-5 four-wave form
// (Glow decoder [16, 80, 768], MI355X A/B: f16x3 1.75 -> 1.52 ms, bf16 1.28 -> 1.01 ms,
// profiles/ab_r06_wn_waves.txt)
bool wn_four_waves() {
  static const bool four = [] {
    const char* e = std::getenv("TTS_MI355X_WN_WAVES");
    return e && std::atoi(e) == 4;
  }();
  return four;
}

template <class S>
void launch_wn_h(const GlowWnLayerArgs& a, int B, hipStream_t s) {
  const bool four = wn_four_waves();
  switch (a.H) {
    case 128:
      if (four) launch_wn_s<S, 128, 4>(a, B, s);
      else launch_wn_s<S, 128, 8>(a, B, s);
      break;
    case 192:
      if (four) launch_wn_s<S, 192, 4>(a, B, s);
      else launch_wn_s<S, 192, 12>(a, B, s);
      break;
    default:
      if (four) launch_wn_s<S, 256, 4>(a, B, s);
      else launch_wn_s<S, 256, 8>(a, B, s);
      break;
  }
}

}  // namespace

bool glow_wn_layer_supported(int mode, int H, int K, int dil) {
  return is_split_mode(mode) && (H == 128 || H == 192 || H == 256) && (K == 3 || K == 5) && dil >= 1 &&
         (K - 1) * dil <= WN_HALO_MAX;
}

void launch_glow_wn_layer(int mode, const GlowWnLayerArgs& a, int B, hipStream_t s) {
  TTS_REQUIRE(glow_wn_layer_supported(mode, a.H, a.K, a.dil), 3, "glow_wn_layer: unsupported configuration");
  TTS_REQUIRE(a.h_in && a.skip && a.mask && a.w_in && a.b_in && a.w_rs && a.b_rs && (a.last || a.h_out), 1,
              "glow_wn_layer: NULL pointer");
  TTS_REQUIRE(a.last || a.h_out != a.h_in, 1, "glow_wn_layer: h_out must not alias h_in");
  TTS_REQUIRE(a.steps_in == (a.H / 16) * a.K && a.steps_rs == a.H / 16 &&
                  a.rs_blocks >= (a.last ? a.H : 2 * a.H) / 32,
              1, "glow_wn_layer: weight packing does not match");
  TTS_REQUIRE(B >= 1 && a.Th >= 1 && (int64_t)a.H * a.Th * 4 < (int64_t(1) << 31), 3,
              "glow_wn_layer: a batch item's channel plane exceeds 2 GiB");
  TTS_REQUIRE(!a.w_end || (a.last && a.b_end && a.end_out && a.end_rows % 32 == 0 && a.end_rows >= 32 &&
                           a.end_rows <= 2 * a.H && a.end_steps == a.H / 16 && a.end_blocks >= a.end_rows / 32 &&
                           (int64_t)a.end_rows * a.Th * 4 < (int64_t(1) << 31)),
              1, "glow_wn_layer: bad fused end conv arguments");
  TTS_REQUIRE(!a.tail_x || (a.w_end && a.winv && a.logs && a.abias && a.w_start && a.b_start && a.h_next &&
                            a.h_next != a.h_in && a.end_rows % 32 == 0 && 3 * a.end_rows <= 4 * a.H &&
                            a.start_steps * 16 >= a.end_rows / 2 && a.start_blocks >= a.H / 32),
              1, "glow_wn_layer: bad fused tail / start arguments");
  if (mode == MATH_FP32_F16X3) launch_wn_h<SchemeH3>(a, B, s);
  else if (mode == MATH_BF16) launch_wn_h<SchemeB1>(a, B, s);
  else launch_wn_h<SchemeX6>(a, B, s);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
