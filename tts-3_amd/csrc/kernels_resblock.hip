// Fused ResBlock1 iteration (TTS/vocoder/models/hifigan_generator.py:93-98) for C in {32, 64}:
//   xt = convs1[m](lrelu(x, 0.1)); xt = lrelu(xt, 0.1); x' = convs2[m](xt) + x   [MRF z, :255-261]
// in one kernel, so the intermediate xt never reaches HBM (per iteration the unfused path moves
// five C-channel planes, this one three: x read twice, x' written once).
//
// A workgroup (4 waves) owns RP_BN = RP_W - (K - 1) output columns.  Phase 1 computes convs1 on
// RP_W = 256 (or 192) columns (the RP_BN plus conv2's halo of (K - 1) / 2 on each side), exactly
// like conv1d_split_kernel (X staged per 16-channel chunk in LDS, weights streamed from L2).
// Its epilogue applies the bias and the lrelu, zeroes columns outside [0, T) (conv2's zero
// padding), splits the values into the scheme's pieces and stores them as conv2's B operand in
// the LDS the X staging used.  Phase 2 runs convs2 over the same RP_W columns from that buffer
// (the last K - 1 are discarded) and finishes in conv_epilogue (bias, residual, MRF sum, statistics).
// f16x3: xt's scale is the workgroup's own power of two (block max-abs): every conv2 output sums
// products of one workgroup's xt only, so the per-tile scale is exact and batch-invariant.
// The residual x is re-read from global memory, so x and x' must not alias (ping-pong buffers).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "resblock_block.hpp"
#include "split_device.hpp"

namespace tts {



// Workgroup geometry (GEO): 4 waves as WM (row blocks) x WN (column groups), each wave TM x TN
// 32x32 blocks; RP_W = convs1 columns, RP_BN = RP_W - 2 * LEAD output columns.
//   GEO 0: RP_W = 256, every wave all C rows x 64 columns (C = 32: 1 x 2 blocks, C = 64: 2 x 2)
//   GEO 1 (C = 64): RP_W = 192, waves 2 x 2, each 32 rows x 96 columns: the xt buffer shrinks
//   from 4 x 288 to 4 x 224 rows, so two workgroups fit a CU in the f16x3 scheme (LDS 72 KB
//   instead of 92 KB); the halo costs (K - 1) / 192 of the columns instead of (K - 1) / 256.
//   GEO 4 (bf16 C = 128, A/B TTS_MI355X_PAIR128_GEO=4): RP_W = 256, waves 2 x 2 of 64 x 128: a
//   weight fragment feeds 4 MFMAs instead of GEO 0's 2 (GEO 0 at C = 128 streams 64 B/clk of
//   weights per CU at full MFMA rate, the L2 port's width).
//   GEO 2 (C = 64, round 6 A/B, TTS_MI355X_PAIR_GEO64=2): RP_W = 128, waves 2 x 2 of 32 x 64,
//   double-buffered staging: 51 KB of LDS and <= 168 VGPRs, three workgroups (three waves per
//   SIMD) per CU.
//   GEO 5 / 6 (bf16 C = 128 / 256): 8 waves, two per SIMD, each 64 rows x 64 columns; 2 x 4 waves
//   on 256 columns (C = 128) or 4 x 2 on 128 (C = 256).  The xt buffer keeps the workgroup alone
//   on its CU, so the second wave per SIMD is what hides one wave's staging, hand-off and epilogue
//   latencies.  GEO 7 / 8 (the bf16 defaults): the same with waves of 32 rows x 128 columns (4 x 2
//   on 256 columns, 8 x 1 on 128), so a weight fragment feeds 4 MFMAs.

constexpr int kPostK = 7;     // conv_post kernel (hifigan_generator.py:229-230)
constexpr int kPostHalo = 3;  // its zero-padding halo per side

template <class S, int K, int C, int PD, int GEO, bool ALLX = false, bool POST = false>
struct PairCfg {
  static constexpr int RP_W = (GEO == 0 || GEO == 4 || GEO == 5 || GEO == 7) ? 256 : (GEO == 1 ? 192 : 128);
  static constexpr int LEAD = (K - 1) / 2;        // xt row 0 holds time t0 - LEAD (conv2's halo)
  static constexpr int RP_BN = RP_W - 2 * LEAD;
  static constexpr int NW = GEO >= 5 ? 8 : 4;     // waves per workgroup
  static constexpr int NT = 64 * NW;
  // GEO 4: 256 columns as 2 x 2 waves (bf16 C = 128); GEO 5 / 6: 8 waves, 2 x 4 / 4 x 2; GEO 7 / 8
  // (A/B): 8 waves of 32 rows x 128 columns, 4 x 2 / 8 x 1 (a weight fragment feeds 4 MFMAs)
  static constexpr int WN = (GEO == 0 || GEO == 5) ? 4 : (GEO == 8 ? 1 : 2);
  static constexpr int WM = NW / WN;
  static constexpr int TM = C / 32 / WM;
  static constexpr int TN = RP_W / 32 / WN;
  static constexpr int NC = C / 16;               // 16-channel groups
  static constexpr int HMAX = (K - 1) * 5;        // dilation <= 5
  static constexpr int XROWS = RP_W + HMAX;
  static constexpr int XSZB = XROWS * S::ROWB;    // one X staging buffer (16 channels)
  static constexpr int TROWS = RP_W + 32;         // + zero rows read by the discarded columns
  static constexpr int TSZB = NC * TROWS * S::ROWB;
  // ALLX: every 16-channel group of the input window is staged at once (one HBM latency for the
  // whole of phase 1, no per-chunk barriers); otherwise double-buffered per group
  static constexpr int XBUFS = ALLX ? NC : 2;
  static constexpr int LDSB0 = (XBUFS * XSZB > TSZB ? XBUFS * XSZB : TSZB);
  // POST: the final z tile (fp32 [C][RP_BN]) for the fused conv_post, after phase 2
  static constexpr int ZTB = POST ? C * RP_BN * 4 : 0;
  static constexpr int LDSB = LDSB0 > ZTB ? LDSB0 : ZTB;
  // POST: output tiles overlap by conv_post's halo on both sides
  static constexpr int STRIDE = POST ? RP_BN - 2 * kPostHalo : RP_BN;
  static constexpr int UPT = (XROWS * 4 + NT - 1) / NT;
  static_assert(TM >= 1 && TM * WM * 32 == C && TN * WN * 32 == RP_W, "geometry");
};

// C = 32 (16-bit-pair schemes): ask for 3 waves per SIMD (<= 168 VGPRs + AGPRs): the LDS already
// allows three workgroups per CU, the unconstrained allocation (173) allowed two
// PL: the planes of x, x' / z (bf16 in the bf16 scheme's activation-plane form, Conv1dArgs::planes)
#ifndef PAIR_W_B1
#define PAIR_W_B1 3  // waves per SIMD asked of the bf16 scheme's pair kernels (0: as the others; 3 measured -1% per bf16 step, profiles/ab_r06_bf16_occupancy.txt)
#endif
template <class S, int K, int C, int PD, int GEO, bool ALLX, bool POST = false, int PL = 0>
__global__ __launch_bounds__((PairCfg<S, K, C, PD, GEO, ALLX, POST>::NT)) __attribute__((amdgpu_waves_per_eu(
    C > 64 ? (GEO >= 5 ? 2 : 1) : (S::NP == 1 && PAIR_W_B1 > 0 ? PAIR_W_B1 : ((C == 32 || GEO == 2) && S::ROWB <= 80 ? 3 : 1)))))
void resblock_pair_kernel(ResPairArgs pa) {
  constexpr bool XB = (PL & kPlaneXB16) != 0, YB = (PL & kPlaneYB16) != 0;
  using PX = PlaneT<XB>;
  using PY = PlaneT<YB>;
  using P = PairCfg<S, K, C, PD, GEO, ALLX, POST>;
  constexpr int RP_W = P::RP_W, RP_BN = P::RP_BN;
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
  constexpr int TM = P::TM, TN = P::TN, NC = P::NC;
  __shared__ __attribute__((aligned(16))) unsigned char smem[P::LDSB];
  __shared__ float red[P::NW];
  constexpr int NT = P::NT;
  __shared__ float bsm[2 * C];  // convs1 and convs2 biases (epilogue reads from LDS, not L2)
  __shared__ float pws[POST ? C * kPostK : 1];  // POST: conv_post's weights (broadcast reads)

  const Conv1dArgs& a1 = pa.c1;
  const int tid = threadIdx.x;
  const float bias1 = tid < C ? a1.bias[tid] : 0.f;
  const float bias2 = tid < C ? pa.c2.bias[tid] : 0.f;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int wm = __builtin_amdgcn_readfirstlane(wave / P::WN);
  const int wn = wave % P::WN;
  const int mrow0 = wm * TM * 32;  // first output channel of this wave
  const int t0 = (int)blockIdx.x * P::STRIDE - (POST ? kPostHalo : 0);
  const int b = blockIdx.z;
  const int d = a1.dil;
  const int T = a1.Tout;
  const int XW = RP_W + (K - 1) * d;
  const int tx0 = t0 - P::LEAD;  // time of convs1 column 0
  const unsigned avoff = (unsigned)lane * 16u;

  // POST: the final MRF sum of this tile, v = (z + convs2(xt) + bias + x) / zdiv exactly as
  // conv_epilogue_impl<RES, ZM = 3> forms it, into LDS (zero outside [0, T): conv_post's zero
  // padding); then conv_post on the inner columns [3, RP_BN - 3), one column per thread, with
  // conv_post4_kernel's FMA order (bias, then channel by channel, tap by tap), and tanh
  auto post_epilogue = [&](const ResPairArgs& q, const f32x16 (&ac)[TM][TN], int bb, int tt0, int row0w, int wnn,
                           int ln) {
    const Conv1dArgs a2 = q.c2;
    const int hf = ln >> 5, lo = ln & 31;
    const size_t item = (size_t)bb * C * T;
    const unsigned plane = (unsigned)C * (unsigned)T * PY::ES;
    const rsrc_t rres = make_rsrc(plane_at<YB>(a2.res, item), plane);
    const rsrc_t rz = make_rsrc(plane_at<YB>(a2.z, item), plane);
    const unsigned rowb = (unsigned)T * PY::ES;
    float* zt = reinterpret_cast<float*>(smem);
    __syncthreads();  // every wave is past its last phase-2 read of xt
#pragma unroll
    for (int m = 0; m < TM; ++m) {
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        const int col = wnn * TN * 32 + n * 32 + lo;
        const int t = tt0 + col;
        const bool tok = t >= 0 && t < T && col < RP_BN;
        const int rw0 = row0w + m * 32 + 4 * hf;
        const unsigned voff = tok ? ((unsigned)rw0 * (unsigned)T + (unsigned)t) * PY::ES : OOB_OFF;
        float rv[16], zv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const unsigned vo = voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb;
          rv[r] = PY::ld(rres, vo, 0u);
          zv[r] = PY::ld(rz, vo, 0u);
        }
        if (col < RP_BN) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rw0 + (r & 3) + 8 * (r >> 2);
            float v = (ac[m][n][r] + bsm[C + row]) * 1.f;
            v = lrelu2(v, a2.out_slope);
            v = (v + rv[r]) * 1.f;
            v = (zv[r] + v) / a2.zdiv;
            // conv_post reads lrelu(z): applied once here instead of once per tap (bf16 planes:
            // on the value the stored plane would hold, so the separate conv_post gives the same)
            zt[row * RP_BN + col] = tok ? lrelu(PY::rt(v), q.post_slope) : 0.f;
          }
        }
      }
    }
    __syncthreads();
    const int col = kPostHalo + tid;
    const int t = tt0 + col;
    if (col < RP_BN - kPostHalo && t >= 0 && t < T) {
      float o = q.post_bias;
#pragma unroll 4
      for (int ci = 0; ci < C; ++ci) {
        const float* zr = zt + ci * RP_BN + col - kPostHalo;
#pragma unroll
        for (int k = 0; k < kPostK; ++k) o = fmaf(pws[ci * kPostK + k], zr[k], o);
      }
      q.wav[(size_t)bb * T + t] = tanhf(o);
    }
  };

  // ------------------------------------------------------------------ phase 1: convs1
  const int ex = H3 ? amax_exp(a1.amax_in, b) : 0;
  const float xscale = H3 ? ldexpf(1.f, -ex) : 1.f;
  const char* xb = static_cast<const char*>(plane_at<XB>(a1.x, (size_t)b * C * T));
  const unsigned chb = (unsigned)T * PX::ES;
  unsigned uvoff[P::UPT];
  int ulds[P::UPT];
#pragma unroll
  for (int i = 0; i < P::UPT; ++i) {
    const int u = tid + i * NT;
    // RES_STAGE_8R: 8 rows x 2 quad positions per 16-lane store group (see conv1d_split_kernel)
    const int q = RES_STAGE_8R ? quad_pos((u >> 3) & 3) : (u & 3);
    const int r = RES_STAGE_8R ? (u >> 5) * 8 + (u & 7) : (u >> 2);
    const int ts = tx0 - a1.pad + r;
    const bool ok = r < XW && ts >= 0 && ts < T;
    uvoff[i] = ok ? (unsigned)(4 * q) * chb + (unsigned)ts * PX::ES : OOB_OFF;
    ulds[i] = r < XW ? r * S::ROWB + 8 * quad_pos(q) : -1;
  }
  f32x4 xall[ALLX ? NC : 1][P::UPT];
  auto load_x = [&](int c) {
    f32x4 (&xreg)[P::UPT] = xall[ALLX ? c : 0];
    const rsrc_t rx = make_rsrc(xb + (size_t)c * 16 * chb, (unsigned)(C - c * 16) * chb);
#pragma unroll
    for (int i = 0; i < P::UPT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) xreg[i][j] = PX::ld(rx, uvoff[i] + (unsigned)j * chb, 0u);
  };
  auto store_x = [&](int buf, int c) {
    const f32x4 (&xreg)[P::UPT] = xall[ALLX ? c : 0];
    unsigned char* xl = smem + buf * P::XSZB;
#pragma unroll
    for (int i = 0; i < P::UPT; ++i) {
      if (ulds[i] >= 0) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = lrelu2(xreg[i][j], a1.in_slope);
          if (H3) v[j] *= xscale;
        }
        split_store4<S>(xl + ulds[i], v[0], v[1], v[2], v[3]);
      }
    }
  };

  rsrc_t ra[TM];
#pragma unroll
  for (int m = 0; m < TM; ++m) ra[m] = make_rsrc(a1.w + ((size_t)(wm * TM + m) * NC * K) * (NP * 256), 0xFFFFFFFFu);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n) acc[m][n] = f32x16{};

  f32x4 ar[PD + 1][TM][NP], bcur[TN][NP], bnext[TN][NP];
#pragma unroll
  for (int p = 0; p < PD; ++p)
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int q = 0; q < NP; ++q) ar[p][m][q] = bload4(ra[m], avoff, (unsigned)(p * NP + q) * 1024u);

  auto mfma_step = [&]() {
#pragma unroll
    for (int e = 0; e < S::NPROD; ++e)
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int n = 0; n < TN; ++n)
          acc[m][n] = S::mfma(ar[0][m][S::PA[e]], bcur[n][S::PB[e]], acc[m][n]);
#pragma unroll
    for (int p = 0; p < PD; ++p)
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int q = 0; q < NP; ++q) ar[p][m][q] = ar[p + 1][m][q];
  };

  const int xrow0 = wn * TN * 32 + l32;
  auto read_x = [&](const unsigned char* xl, int k, f32x4 (*dst)[NP]) {
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const unsigned char* p = xl + (xrow0 + n * 32 + k * d) * S::ROWB + 16 * half;
#pragma unroll
      for (int q = 0; q < NP; ++q) dst[n][q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
    }
  };

  if constexpr (ALLX) {
#pragma unroll
    for (int c = 0; c < NC; ++c) load_x(c);
#pragma unroll
    for (int c = 0; c < NC; ++c) store_x(c, c);
  } else {
    load_x(0);
    store_x(0, 0);
  }
  if (tid < C) {
    bsm[tid] = bias1;
    bsm[C + tid] = bias2;
  }
  if constexpr (POST)
    for (int e = tid; e < C * kPostK; e += NT) pws[e] = pa.post_w[e];
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const unsigned char* xl = smem + (ALLX ? c : (c & 1)) * P::XSZB;
    if (!ALLX && c + 1 < NC) load_x(c + 1);
    read_x(xl, 0, bcur);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int s = c * K + k;
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int q = 0; q < NP; ++q) ar[PD][m][q] = bload4(ra[m], avoff, (unsigned)((s + PD) * NP + q) * 1024u);
      if (k + 1 < K) read_x(xl, k + 1, bnext);
      __builtin_amdgcn_sched_barrier(0);
      mfma_step();
      if (k + 1 < K) {
#pragma unroll
        for (int n = 0; n < TN; ++n)
#pragma unroll
          for (int q = 0; q < NP; ++q) bcur[n][q] = bnext[n][q];
      }
    }
    if (!ALLX && c + 1 < NC) store_x((c + 1) & 1, c + 1);
    if (!ALLX || c + 1 == NC) __syncthreads();  // ALLX: only before xt overwrites the window
  }

  // ------------------------------------------------------------------ convs1 epilogue -> xt (LDS)
  {
    const float sc1 = H3 ? ldexpf(1.f, ex + a1.w_exp) : 1.f;
    float tmax = 0.f;
#pragma unroll
    for (int m = 0; m < TM; ++m) {
      float bv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) bv[r] = bsm[mrow0 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half];
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        const int t = tx0 + xrow0 + n * 32;
        const bool inside = t >= 0 && t < T;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = lrelu2(acc[m][n][r] * sc1 + bv[r], a1.out_slope);
          v = inside ? v : 0.f;
          acc[m][n][r] = v;
          tmax = fmaxf(tmax, fabsf(v));
        }
      }
    }
    float tscale = 1.f;
    int et = 0;
    if (H3) {
      tmax = wave_max(tmax);
      if (lane == 0) red[wave] = tmax;
      __syncthreads();
      float mx = red[0];
#pragma unroll
      for (int w = 1; w < P::NW; ++w) mx = fmaxf(mx, red[w]);
      if (mx > 0.f && mx < INFINITY) {
        int E;
        (void)frexpf(mx, &E);
        et = E - 14;
      }
      tscale = ldexpf(1.f, -et);
    }
    // xt pieces: row = convs1 column; registers 8 gl .. 8 gl + 7 are positions 8 half .. + 7 of
    // group (m row block, gl) (quad_pos order): one 16-byte store per piece
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n)
#pragma unroll
        for (int gl = 0; gl < 2; ++gl)
          store_xt8<S>(smem + (((mrow0 + m * 32) / 16 + gl) * P::TROWS + xrow0 + n * 32) * S::ROWB + 16 * half,
                       acc[m][n], 8 * gl, tscale);
    // zero rows RP_W .. TROWS-1 of every group (read only by the discarded columns)
    constexpr int ZB = (P::TROWS - RP_W) * S::ROWB;  // bytes per group
    for (int e = tid * 16; e < NC * ZB; e += NT * 16) {
      const int g = e / ZB;
      *reinterpret_cast<f32x4*>(smem + (g * P::TROWS + RP_W) * S::ROWB + (e - g * ZB)) = f32x4{};
    }
    __syncthreads();
    // ---------------------------------------------------------------- phase 2: convs2 from LDS
    const Conv1dArgs& a2 = pa.c2;
#pragma unroll
    for (int m = 0; m < TM; ++m) ra[m] = make_rsrc(a2.w + ((size_t)(wm * TM + m) * NC * K) * (NP * 256), 0xFFFFFFFFu);
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n) acc[m][n] = f32x16{};
#pragma unroll
    for (int p = 0; p < PD; ++p)
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int q = 0; q < NP; ++q) ar[p][m][q] = bload4(ra[m], avoff, (unsigned)(p * NP + q) * 1024u);
    const int trow0 = xrow0;  // + LEAD - (K - 1) / 2
    auto read_t = [&](int g, int k, f32x4 (*dst)[NP]) {
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        const unsigned char* p = smem + (g * P::TROWS + trow0 + n * 32 + k) * S::ROWB + 16 * half;
#pragma unroll
        for (int q = 0; q < NP; ++q) dst[n][q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
      }
    };
    read_t(0, 0, bcur);
#pragma unroll
    for (int g = 0; g < NC; ++g) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int s = g * K + k;
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int q = 0; q < NP; ++q) ar[PD][m][q] = bload4(ra[m], avoff, (unsigned)((s + PD) * NP + q) * 1024u);
        const bool more = (k + 1 < K) || (g + 1 < NC);
        if (more) read_t((k + 1 < K) ? g : g + 1, (k + 1 < K) ? k + 1 : 0, bnext);
        __builtin_amdgcn_sched_barrier(0);
        mfma_step();
        if (more) {
#pragma unroll
          for (int n = 0; n < TN; ++n)
#pragma unroll
            for (int q = 0; q < NP; ++q) bcur[n][q] = bnext[n][q];
        }
      }
    }
    if (H3) {
      const float sc2 = ldexpf(1.f, et + a2.w_exp);
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int n = 0; n < TN; ++n) acc[m][n] *= sc2;
    }
    if constexpr (POST) {
      post_epilogue(pa, acc, b, t0, mrow0, wn, lane);
    } else {
      conv_epilogue<TM, TN, H3, YB>(a2, acc, b, t0 + wn * TN * 32, mrow0, lane, t0 + RP_BN, bsm + C);
    }
  }
}

namespace {
template <class S, int K, int C, int GEO>
void launch_pair_t(const ResPairArgs& a, int B, hipStream_t s) {
  // all-at-once staging measured faster at 64 channels (-7% on k3), not at 32; GEO 2 double-buffers
  // (the LDS of three workgroups per CU)
  constexpr bool AX = C == 64 && GEO != 2;
  constexpr int PD = S::NP == 1 ? RES_PD_B1 : 2;
  auto go = [&](auto pl_tag) {
    constexpr int PL = decltype(pl_tag)::value;
    if (a.post_w) {
      using P = PairCfg<S, K, C, PD, GEO, AX, true>;
      static_assert(P::RP_BN - 2 * kPostHalo <= 256, "one conv_post column per thread");
      dim3 grid(ceil_div(a.c1.Tout, P::STRIDE), 1, B);
      hipLaunchKernelGGL((resblock_pair_kernel<S, K, C, PD, GEO, AX, true, PL>), grid, dim3(P::NT), 0, s, a);
      return;
    }
    using P = PairCfg<S, K, C, PD, GEO, AX>;
    dim3 grid(ceil_div(a.c1.Tout, P::RP_BN), 1, B);
    hipLaunchKernelGGL((resblock_pair_kernel<S, K, C, PD, GEO, AX, false, PL>), grid, dim3(P::NT), 0, s, a);
  };
  if (a.c1.planes != 0) {
    // bf16 activation planes: x, x' and z all bf16 (the bf16 scheme)
    constexpr bool OK = std::is_same<S, SchemeB1>::value;
    TTS_REQUIRE(OK && a.c1.planes == (kPlaneXB16 | kPlaneYB16) && a.c2.planes == a.c1.planes, 3,
                "resblock pair: bf16 planes need the bf16 scheme");
    if constexpr (OK) go(std::integral_constant<int, kPlaneXB16 | kPlaneYB16>{});
    return;
  }
  go(std::integral_constant<int, 0>{});
}

int pair_geo64() {
  static const int g = [] {
    const char* e = std::getenv("TTS_MI355X_PAIR_GEO64");
    return e && std::atoi(e) == 2 ? 2 : (e && std::atoi(e) == 4 ? 4 : 1);
  }();
  return g;
}

template <class S, int K>
void launch_pair_k(const ResPairArgs& a, int B, int C, hipStream_t s) {
  if constexpr (S::NP == 1) {
    // bf16 only: 128 channels on 256 columns, one wave per SIMD (4 x 32 rows x 64 columns of
    // accumulators per wave), the xt buffer 8 groups x 288 rows x 48 B = 111 KB (the 16-bit-pair
    // schemes' 80-byte rows would need 184 KB)
    if (C == 128) {
      // default GEO 7 (256 columns, 8 waves of 32 x 128, two per SIMD, a weight fragment feeding 4
      // MFMAs: step -0.2 ms against GEO 5, profiles/ab_r06_bf16_pair78.txt); TTS_MI355X_PAIR128_GEO=5
      // (8 waves of 64 x 64: k7 3.79 -> 3.59 ms, k11 4.89 -> 4.80 per forward against GEO 4,
      // profiles/ab_r06_bf16_pair8w.txt), 4 (2 x 2
      // waves of 64 x 128, one per SIMD: step 26.41 -> 26.2 ms against GEO 0,
      // profiles/ab_r06_bf16_pair128_geo.txt), 0 (4 waves of 128 x 64) or 2 (128 columns, 2 x 2 waves
      // of 64 x 64, 78 KB: two per CU) for A/B
      static const int geo = [] {
        const char* e = std::getenv("TTS_MI355X_PAIR128_GEO");
        return e && e[0] == '2' ? 2 : (e && e[0] == '0' ? 0 : (e && e[0] == '4' ? 4 : (e && e[0] == '5' ? 5 : 7)));
      }();
      if (geo == 2) launch_pair_t<S, K, 128, 2>(a, B, s);
      else if (geo == 7) launch_pair_t<S, K, 128, 7>(a, B, s);
      else if (geo == 5) launch_pair_t<S, K, 128, 5>(a, B, s);
      else if (geo == 4) launch_pair_t<S, K, 128, 4>(a, B, s);
      else launch_pair_t<S, K, 128, 0>(a, B, s);
      return;
    }
    // 256 channels on 128 columns: xt 16 groups x 160 rows x 48 B = 123 KB
    if (C == 256) {
      // default GEO 8: 8 waves of 32 rows x 128 columns, two per SIMD (k3 0.91 -> 0.86 ms per forward
      // against GEO 6, profiles/ab_r06_bf16_pair78.txt); TTS_MI355X_PAIR256_GEO=6 (8 waves of 64 x 64:
      // k7 1.80 -> 1.63 ms, k3 0.99 -> 0.91 against GEO 2, profiles/ab_r06_bf16_pair8w.txt) or 2
      // (2 x 2 waves of 128 x 64, one per SIMD)
      static const int geo = [] {
        const char* e = std::getenv("TTS_MI355X_PAIR256_GEO");
        return e && e[0] == '2' ? 2 : (e && e[0] == '6' ? 6 : 8);
      }();
      if (geo == 6) launch_pair_t<S, K, 256, 6>(a, B, s);
      else if (geo == 8) launch_pair_t<S, K, 256, 8>(a, B, s);
      else launch_pair_t<S, K, 256, 2>(a, B, s);
      return;
    }
  }
  if (C == 32) launch_pair_t<S, K, 32, 0>(a, B, s);
  else if (C == 64 && pair_geo64() == 2 && S::ROWB <= 80) launch_pair_t<S, K, 64, 2>(a, B, s);
  else if (C == 64 && pair_geo64() == 4 && S::NP == 1) launch_pair_t<S, K, 64, 4>(a, B, s);
  else if (C == 64) launch_pair_t<S, K, 64, 1>(a, B, s);
  else throw Error(3, "resblock pair: channels must be 32 or 64");
}

template <class S>
void launch_pair_s(const ResPairArgs& a, int B, int K, int C, hipStream_t s) {
  switch (K) {
    case 3: launch_pair_k<S, 3>(a, B, C, s); break;
    case 7: launch_pair_k<S, 7>(a, B, C, s); break;
    case 11: launch_pair_k<S, 11>(a, B, C, s); break;
    default: throw Error(3, "resblock pair: kernel size must be 3, 7 or 11");
  }
}
}  // namespace

bool resblock_pair_supported(int mode, int C, int K, int dil) {
  return is_split_mode(mode) && (C == 32 || C == 64 || ((C == 128 || C == 256) && mode == MATH_BF16)) &&
         (K == 3 || K == 7 || K == 11) && dil >= 1 && dil <= 5;
}

// the bf16 scheme's wide ResBlock1 iterations as pairs (direct convs, xt in LDS): 128 channels at
// kernels 7 / 11 (instead of two Winograd launches each; TTS_MI355X_PAIR128=0 keeps those) and 256
// channels at kernels 3 / 7 (TTS_MI355X_PAIR256=0 keeps the per-conv launches).  Measured per bf16
// forward (profiles/ab_r06_bf16_pair128.txt, ab_r06_bf16_pair256.txt): c128 k11 5.44 -> 4.98 ms,
// k7 4.95 -> 3.93; c256 k7 2.04 -> 1.69, k3 1.05 -> 0.99, k11 2.43 -> 2.63 (stays Winograd)
bool resblock_pair128(int mode, int C, int K) {
  if (mode != MATH_BF16) return false;
  const char* e128 = std::getenv("TTS_MI355X_PAIR128");
  const char* e256 = std::getenv("TTS_MI355X_PAIR256");
  if (C == 128) return (K == 7 || K == 11) && !(e128 && e128[0] == '0');
  if (C == 256) {
    // kernel 11 at 256 channels: Winograd unless TTS_MI355X_PAIR256_K11=1 (A/B)
    const char* e11 = std::getenv("TTS_MI355X_PAIR256_K11");
    return (K == 3 || K == 7 || (K == 11 && e11 && e11[0] == '1')) && !(e256 && e256[0] == '0');
  }
  return false;
}

// Where the fused form is the faster one (MI355X A/B, f16x3): every 32-channel iteration
// (-21..-37%, scripts/ab_fusion.sh) and, with the 192-column geometry (two workgroups per CU),
// every 64-channel one (k3 -20%, k7 -11%, k11 -1%; scripts/ab_pair_geo.sh).
bool resblock_pair_preferred(int mode, int C, int K, int dil) {
  return resblock_pair_supported(mode, C, K, dil);
}

void launch_resblock_pair(int mode, const ResPairArgs& a, int B, int K, int C, hipStream_t s) {
  TTS_REQUIRE(resblock_pair_supported(mode, C, K, a.c1.dil), 3, "resblock pair: unsupported configuration");
  TTS_REQUIRE(a.c1.Cin == C && a.c1.Cout == C && a.c2.Cin == C && a.c2.Cout == C && a.c1.Tin == a.c1.Tout &&
                  a.c2.Tout == a.c1.Tout && a.c1.rep_pad == 0 && a.c2.dil == 1,
              1, "resblock pair: bad arguments");
  TTS_REQUIRE(a.c2.res != a.c2.y || a.c2.zmode != 0, 1, "resblock pair: x and x' must not alias");
  TTS_REQUIRE(a.c1.cvec == nullptr && a.c2.cvec == nullptr && a.c1.bias && a.c2.bias, 1,
              "resblock pair: biases required, no cond vector (both are staged in LDS)");
  TTS_REQUIRE((int64_t)C * a.c1.Tout * 4 < (int64_t(1) << 31), 3, "resblock pair: plane exceeds 2 GiB");
  TTS_REQUIRE(!a.post_w || (a.c2.zmode == 3 && a.c2.res && a.c2.z && a.wav && !a.c2.mask), 1,
              "resblock pair: the fused conv_post needs the final MRF sum (zmode 3) with a residual");
  if (mode == MATH_FP32_F16X3) launch_pair_s<SchemeH3>(a, B, K, C, s);
  else if (mode == MATH_BF16) launch_pair_s<SchemeB1>(a, B, K, C, s);
  else launch_pair_s<SchemeX6>(a, B, K, C, s);
  TTS_HIP_CHECK(hipGetLastError());
}


namespace {
template <class S, int C, int GEO, int K>
void launch_res3_t(const ResBlock3Args& a, int B, hipStream_t s) {
  using P = Res3Cfg<S, C, GEO, K, 6, r3_xoff(K), r3_lead(K)>;
  dim3 grid(ceil_div(a.T, P::RP_BN), 1, B);
  launch_block_pl<S, C, GEO, K, 6, r3_xoff(K), r3_lead(K)>(a, grid, P::NT, s);
}
template <class S>
void launch_res3_s(const ResBlock3Args& a, int B, int C, int K, hipStream_t s) {
  // C = 64: 128 columns (2 waves/SIMD, a quarter of the columns are halo; 192 columns at one
  // wave per SIMD measured slower).  C = 128: 128 columns as 8 waves of 32 rows x 64 columns (two
  // per SIMD; 2 x 2 waves of 64 x 64 measured slower); LDS 8 x 138 rows.  Kernels 7 / 11 (32 and
  // 64 channels): the 256-column tile keeps 184 / 136 columns
  if (K == 7) {
    if (C == 32) launch_res3_t<S, 32, 0, 7>(a, B, s);
    else launch_res3_t<S, 64, 0, 7>(a, B, s);
    return;
  }
  if (K == 11) {
    if (C == 32) launch_res3_t<S, 32, 0, 11>(a, B, s);
    else launch_res3_t<S, 64, 0, 11>(a, B, s);
    return;
  }
  if (C == 32) launch_res3_t<S, 32, 0, 3>(a, B, s);
  else if (C == 128) {
    if constexpr (S::ROWB <= 80) launch_res3_t<S, 128, 3, 3>(a, B, s);
    else throw Error(3, "resblock3: 128 channels need a split scheme of at most 80-byte rows");
  } else launch_res3_t<S, 64, 2, 3>(a, B, s);
}
}  // namespace

bool resblock3_supported(int mode, int C, int K, const int* dil) {
  // C = 128 stages 8 groups x 138 rows: 88 KB of LDS for f16x3 / 53 KB for bf16 (x6 is not built);
  // kernels 7 / 11 at 32 / 64 channels (256-column tiles)
  if (!is_split_mode(mode)) return false;
  if (K == 3) {
    if (!(C == 32 || C == 64 || (C == 128 && mode != MATH_FP32_X6))) return false;
  } else if (K == 7 || K == 11) {
    if (!(C == 32 || C == 64)) return false;
  } else {
    return false;
  }
  // the kernel's valid-range walk: kept columns [LEAD, RP_W - LEAD) must stay inside it
  const int hk = (K - 1) / 2;
  int lo = -r3_xoff(K);
  for (int m = 0; m < 3; ++m) {
    if (dil[m] < 1 || hk * dil[m] > r3_xoff(K)) return false;
    lo = std::max(lo + hk * dil[m], 0) + hk;
  }
  return lo <= r3_lead(K);
}

void launch_resblock3(int mode, const ResBlock3Args& a, int B, int C, int K, hipStream_t s) {
  TTS_REQUIRE(resblock3_supported(mode, C, K, a.dil), 3, "resblock3: unsupported configuration");
  TTS_REQUIRE(a.zmode >= 1 && a.zmode <= 3 && a.z && a.x && a.x != a.z, 1, "resblock3: bad arguments");
  TTS_REQUIRE((int64_t)C * a.T * 4 < (int64_t(1) << 31), 3, "resblock3: plane exceeds 2 GiB");
  if (mode == MATH_FP32_F16X3) launch_res3_s<SchemeH3>(a, B, C, K, s);
  else if (mode == MATH_BF16) launch_res3_s<SchemeB1>(a, B, C, K, s);
  else launch_res3_s<SchemeX6>(a, B, C, K, s);
  TTS_HIP_CHECK(hipGetLastError());
}

bool resblock2_supported(int mode, int C, int K, const int* dil) {
  if (!is_split_mode(mode) || !(K == 3 || K == 5 || K == 7 || K == 11)) return false;
  if (!(C == 32 || C == 64 || (C == 128 && mode != MATH_FP32_X6 && (K == 3 || K == 5)))) return false;
  // the valid-range walk: both convs read inside the staged XO columns, the kept columns
  // [LEAD, RP_W - LEAD) stay inside the valid range
  const int H = rb2_halo(K), hk = (K - 1) / 2;
  int lo = -H;
  for (int m = 0; m < 2; ++m) {
    if (dil[m] < 1 || hk * dil[m] > H) return false;
    lo = std::max(lo + hk * dil[m], 0);
  }
  return lo <= H;
}

// Where one launch beats the two per-conv launches (MI355X, YourTTS decoder at 8 x 1024 frames,
// per forward, whole block vs per conv): f16x3 k3 c64 0.24 vs 0.36 ms, k7 c64 0.42 vs 0.49, k7 c32
// 0.29 vs 0.42, k11 c32 0.39 vs 0.45, k3 c128 0.41 vs 0.42; bf16 every shape (k11 c64 0.35 vs 0.44).
// f16x3 k11 c64 is slower fused (0.68 vs 0.59 ms: 30 of 128 columns are halo), and so is its
// 192-column form (0.75): it stays per conv in the 16-bit-pair split schemes.
bool resblock2_preferred(int mode, int C, int K, const int* dil) {
  if (!resblock2_supported(mode, C, K, dil)) return false;
  const char* e = std::getenv("TTS_MI355X_RB2_ALL");  // tests: every supported block fused
  if (e && e[0] == '1') return true;
  return mode == MATH_BF16 || !(C == 64 && K == 11);
}

// 192-column tiles at 64 channels: bf16 (k11 0.345 vs 0.352 ms, k7 0.272 vs 0.291, k3 0.184 vs
// 0.195); the split schemes keep 128 (f16x3 k7 0.52 vs 0.42 ms)
int resblock2_geo64(int mode) {
  const char* e = std::getenv("TTS_MI355X_RB2_GEO64");
  if (e && (e[0] == '0' || e[0] == '1')) return e[0] - '0';
  return mode == MATH_BF16 ? 1 : 0;
}

void launch_resblock2(int mode, const ResBlock3Args& a, int B, int C, int K, int geo64, hipStream_t s) {
  TTS_REQUIRE(resblock2_supported(mode, C, K, a.dil), 3, "resblock2: unsupported configuration");
  TTS_REQUIRE(a.zmode >= 1 && a.zmode <= 3 && a.z && a.x && a.x != a.z, 1, "resblock2: bad arguments");
  TTS_REQUIRE((int64_t)C * a.T * 4 < (int64_t(1) << 31), 3, "resblock2: plane exceeds 2 GiB");
  if (mode == MATH_FP32_F16X3) launch_resblock2_h3(a, B, C, K, geo64, s);
  else if (mode == MATH_BF16) launch_resblock2_b1(a, B, C, K, geo64, s);
  else launch_resblock2_x6(a, B, C, K, geo64, s);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
