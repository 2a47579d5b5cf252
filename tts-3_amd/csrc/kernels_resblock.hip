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

#include "split_device.hpp"

namespace tts {



// Workgroup geometry (GEO): 4 waves as WM (row blocks) x WN (column groups), each wave TM x TN
// 32x32 blocks; RP_W = convs1 columns, RP_BN = RP_W - 2 * LEAD output columns.
//   GEO 0: RP_W = 256, every wave all C rows x 64 columns (C = 32: 1 x 2 blocks, C = 64: 2 x 2)
//   GEO 1 (C = 64): RP_W = 192, waves 2 x 2, each 32 rows x 96 columns: the xt buffer shrinks
//   from 4 x 288 to 4 x 224 rows, so two workgroups fit a CU in the f16x3 scheme (LDS 72 KB
//   instead of 92 KB); the halo costs (K - 1) / 192 of the columns instead of (K - 1) / 256.
#ifndef RES_STAGE_8R
#define RES_STAGE_8R 1  // x staging lane map of the pair / whole-block kernels (0: 4 rows x 4 quads)
#endif

constexpr int kPostK = 7;     // conv_post kernel (hifigan_generator.py:229-230)
constexpr int kPostHalo = 3;  // its zero-padding halo per side

template <class S, int K, int C, int PD, int GEO, bool ALLX = false, bool POST = false>
struct PairCfg {
  static constexpr int RP_W = GEO == 0 ? 256 : 192;
  static constexpr int LEAD = (K - 1) / 2;        // xt row 0 holds time t0 - LEAD (conv2's halo)
  static constexpr int RP_BN = RP_W - 2 * LEAD;
  static constexpr int WN = GEO == 0 ? 4 : 2;
  static constexpr int WM = 4 / WN;
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
  static constexpr int UPT = (XROWS * 4 + 255) / 256;
  static_assert(TM >= 1 && TM * WM * 32 == C && TN * WN * 32 == RP_W, "geometry");
};

// C = 32 (16-bit-pair schemes): ask for 3 waves per SIMD (<= 168 VGPRs + AGPRs): the LDS already
// allows three workgroups per CU, the unconstrained allocation (173) allowed two
template <class S, int K, int C, int PD, int GEO, bool ALLX, bool POST = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(C == 32 && S::ROWB <= 80 ? 3 : 1)))
void resblock_pair_kernel(ResPairArgs pa) {
  using P = PairCfg<S, K, C, PD, GEO, ALLX, POST>;
  constexpr int RP_W = P::RP_W, RP_BN = P::RP_BN;
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
  constexpr int TM = P::TM, TN = P::TN, NC = P::NC;
  __shared__ __attribute__((aligned(16))) unsigned char smem[P::LDSB];
  __shared__ float red[4];
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
    const unsigned plane = (unsigned)C * (unsigned)T * 4u;
    const rsrc_t rres = make_rsrc(a2.res + item, plane);
    const rsrc_t rz = make_rsrc(a2.z + item, plane);
    const unsigned rowb = (unsigned)T * 4u;
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
        const unsigned voff = tok ? ((unsigned)rw0 * (unsigned)T + (unsigned)t) * 4u : OOB_OFF;
        float rv[16], zv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const unsigned vo = voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb;
          rv[r] = bload(rres, vo, 0u);
          zv[r] = bload(rz, vo, 0u);
        }
        if (col < RP_BN) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rw0 + (r & 3) + 8 * (r >> 2);
            float v = (ac[m][n][r] + bsm[C + row]) * 1.f;
            v = lrelu2(v, a2.out_slope);
            v = (v + rv[r]) * 1.f;
            v = (zv[r] + v) / a2.zdiv;
            // conv_post reads lrelu(z): applied once here instead of once per tap
            zt[row * RP_BN + col] = tok ? lrelu(v, q.post_slope) : 0.f;
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
  const float* xb = a1.x + (size_t)b * C * T;
  const unsigned chb = (unsigned)T * 4u;
  unsigned uvoff[P::UPT];
  int ulds[P::UPT];
#pragma unroll
  for (int i = 0; i < P::UPT; ++i) {
    const int u = tid + i * 256;
    // RES_STAGE_8R: 8 rows x 2 quad positions per 16-lane store group (see conv1d_split_kernel)
    const int q = RES_STAGE_8R ? quad_pos((u >> 3) & 3) : (u & 3);
    const int r = RES_STAGE_8R ? (u >> 5) * 8 + (u & 7) : (u >> 2);
    const int ts = tx0 - a1.pad + r;
    const bool ok = r < XW && ts >= 0 && ts < T;
    uvoff[i] = ok ? (unsigned)(4 * q) * chb + (unsigned)ts * 4u : OOB_OFF;
    ulds[i] = r < XW ? r * S::ROWB + 8 * quad_pos(q) : -1;
  }
  f32x4 xall[ALLX ? NC : 1][P::UPT];
  auto load_x = [&](int c) {
    f32x4 (&xreg)[P::UPT] = xall[ALLX ? c : 0];
    const rsrc_t rx = make_rsrc(xb + (size_t)c * 16 * T, (unsigned)(C - c * 16) * chb);
#pragma unroll
    for (int i = 0; i < P::UPT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) xreg[i][j] = bload(rx, uvoff[i] + (unsigned)j * chb, 0u);
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
    for (int e = tid; e < C * kPostK; e += 256) pws[e] = pa.post_w[e];
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
      const float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
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
    for (int e = tid * 16; e < NC * ZB; e += 256 * 16) {
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
      conv_epilogue<TM, TN, H3>(a2, acc, b, t0 + wn * TN * 32, mrow0, lane, t0 + RP_BN, bsm + C);
    }
  }
}

namespace {
template <class S, int K, int C, int GEO>
void launch_pair_t(const ResPairArgs& a, int B, hipStream_t s) {
  constexpr bool AX = C == 64;  // all-at-once staging measured faster at 64 channels (-7% on k3), not at 32
  if (a.post_w) {
    using P = PairCfg<S, K, C, 2, GEO, AX, true>;
    static_assert(P::RP_BN - 2 * kPostHalo <= 256, "one conv_post column per thread");
    dim3 grid(ceil_div(a.c1.Tout, P::STRIDE), 1, B);
    hipLaunchKernelGGL((resblock_pair_kernel<S, K, C, 2, GEO, AX, true>), grid, dim3(256), 0, s, a);
    return;
  }
  dim3 grid(ceil_div(a.c1.Tout, PairCfg<S, K, C, 2, GEO>::RP_BN), 1, B);
  hipLaunchKernelGGL((resblock_pair_kernel<S, K, C, 2, GEO, AX>), grid, dim3(256), 0, s, a);
}

template <class S, int K>
void launch_pair_k(const ResPairArgs& a, int B, int C, hipStream_t s) {
  if (C == 32) launch_pair_t<S, K, 32, 0>(a, B, s);
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
  return is_split_mode(mode) && (C == 32 || C == 64) && (K == 3 || K == 7 || K == 11) && dil >= 1 && dil <= 5;
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

// ---------------------------------------------------------------------------------------
// Whole kernel-3 ResBlock1 (hifigan_generator.py:84-99, K = 3, dilations d0..d2) in one kernel:
//   for m in 0..2:  xt = lrelu(convs1[m](lrelu(x)));  x = convs2[m](xt) + x;   z (+)= x
// All three iterations run on the same RP_W-column grid (column c <-> time t0 - R3_LEAD + c): each
// conv loses its halo at the grid edges, so the valid columns shrink by d_m + 1 per side per
// iteration (11 for dilations 1, 3, 5: the first conv reads 5 staged extra columns, the rest only
// the grid) while the kept ones, [R3_LEAD, RP_W - R3_LEAD), stay exact.  x lives in the
// accumulator layout in registers (the residual of every iteration), lrelu(x) and xt alternate
// in one LDS region as split B operands (X rows: column + 5, xt rows: column + 1).  Columns
// outside the valid range or outside [0, T) are staged as zeros; in the f16x3 scheme the scale of
// x1, x2 and of every xt is the workgroup's own power of two over its valid columns (exact and
// batch-invariant), x0 uses its producer's statistics.  One launch replaces three pair launches:
// x is read once and z written once instead of five C-planes per iteration.
// ---------------------------------------------------------------------------------------
constexpr int R3_XOFF = 5;  // X rows hold column + 5 (convs1 halo up to dilation 5)
// kept columns [R3_LEAD, RP_W - R3_LEAD): only the first conv sees the R3_XOFF staged extra
// columns, every later one loses d_m (+ 1) columns at the grid edge, 11 for dilations 1, 3, 5
constexpr int R3_LEAD = 12;

// GEO 0: 256 columns, 4 waves side by side; GEO 1 / 2: 192 / 128 columns, 2 x 2 waves;
// GEO 3: 128 columns, 8 waves (4 row blocks x 2 column halves at C = 128, two waves per SIMD).
// Measured (f16x3, per batch): C = 128 GEO 3 5.0 ms vs GEO 2 5.5 ms; 8-wave forms at C = 64
// (256 columns) and C = 32 (512 columns) were slower than GEO 2 / GEO 0 (+0.2 / +0.3 ms).
template <class S, int C, int GEO>
struct Res3Cfg {
  static constexpr int RP_W = GEO == 0 ? 256 : (GEO == 1 ? 192 : 128);
  static constexpr int RP_BN = RP_W - 2 * R3_LEAD;
  static constexpr int NW = GEO == 3 ? 8 : 4;     // waves per workgroup
  static constexpr int NT = 64 * NW;
  static constexpr int WN = GEO == 0 ? 4 : 2;
  static constexpr int WM = NW / WN;
  static constexpr int TM = C / 32 / WM;
  static constexpr int TN = RP_W / 32 / WN;
  static constexpr int NC = C / 16;
  static constexpr int PR = RP_W + 2 * R3_XOFF;  // rows per group (X: RP_W + 10, xt: RP_W + 2)
  static constexpr int LDSB = NC * PR * S::ROWB;
  static_assert(TM >= 1 && TM * WM * 32 == C && TN * WN * 32 == RP_W, "geometry");
};

template <class S, int C, int GEO>
__global__ __launch_bounds__((Res3Cfg<S, C, GEO>::NT))
__attribute__((amdgpu_waves_per_eu(C == 32 || (C == 64 && GEO == 2) || GEO == 3 ? 2 : 1)))
void resblock3_kernel(ResBlock3Args a) {
  using P = Res3Cfg<S, C, GEO>;
  constexpr int K = 3;
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
  constexpr int TM = P::TM, TN = P::TN, NC = P::NC, PR = P::PR, RP_W = P::RP_W;
  constexpr int PD = 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[P::LDSB];
  constexpr int NT = P::NT;
  __shared__ float red[2][P::NW];  // double-buffered: consecutive tile_exp calls use different halves
  __shared__ float bsm[6 * C];  // the six conv biases (read by every epilogue: LDS, not L2, latency)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int wm = __builtin_amdgcn_readfirstlane(wave / P::WN);
  const int wn = wave % P::WN;
  const int mrow0 = wm * TM * 32;
  const int t0 = blockIdx.x * P::RP_BN;
  const int b = blockIdx.z;
  const int T = a.T;
  const int tx0 = t0 - R3_LEAD;  // time of column 0
  const int xcol0 = wn * TN * 32 + l32;
  const unsigned avoff = (unsigned)lane * 16u;
  const unsigned chb = (unsigned)T * 4u;
  const float* xb = a.x + (size_t)b * C * T;
  const rsrc_t rx = make_rsrc(xb, (unsigned)C * chb);

  // ---- prologue: lrelu(x0) pieces for columns [-5, RP_W + 5) of every 16-channel group, and x0
  // itself in the acc layout.  Every load is issued before the first store (one HBM latency for
  // the whole window instead of one per group: at C = 128 that is 8 groups, 64 VGPRs of window)
  int ex = H3 ? amax_exp(a.amax_in, b) : 0;
  f32x16 xr[TM][TN];  // the running residual x (fp32), accumulator layout
  {
    const float xs = H3 ? ldexpf(1.f, -ex) : 1.f;
    constexpr int UG = (PR * 4 + NT - 1) / NT;  // units (row, quad) per group per thread
    constexpr int BPT = (C + NT - 1) / NT;
    float bl[6][BPT];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < BPT; ++j) {
        const int e = tid + j * NT;
        bl[i][j] = e < C ? a.bias[i][e] : 0.f;
      }
    f32x4 xv[NC][UG];
#pragma unroll
    for (int g = 0; g < NC; ++g)
#pragma unroll
      for (int i = 0; i < UG; ++i) {
        const int u = tid + i * NT;
        const int q = RES_STAGE_8R ? quad_pos((u >> 3) & 3) : (u & 3);
        const int r = RES_STAGE_8R ? (u >> 5) * 8 + (u & 7) : (u >> 2);
        const int ts = tx0 - R3_XOFF + r;
        const bool ok = r < PR && ts >= 0 && ts < T;
        const unsigned vo = (unsigned)(16 * g + 4 * q) * chb + (unsigned)ts * 4u;
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[g][i][j] = bload(rx, ok ? vo + (unsigned)j * chb : OOB_OFF, 0u);
      }
    // x0 in the acc layout (the residual): the same bytes as the window, so read once the window
    // has landed (L2 hits; issued together, both missed L2: 2.4x the x plane in FETCH_SIZE).  It is
    // first needed in conv 1's epilogue, so its latency hides behind conv 1's MFMAs.
    auto load_xr = [&] {
#pragma unroll
      for (int m = 0; m < TM; ++m)
#pragma unroll
        for (int n = 0; n < TN; ++n) {
          const int t = tx0 + xcol0 + n * 32;
          const bool tok = t >= 0 && t < T;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = mrow0 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
            xr[m][n][r] = bload(rx, tok ? (unsigned)co * chb + (unsigned)t * 4u : OOB_OFF, 0u);
          }
        }
    };
#pragma unroll
    for (int g = 0; g < NC; ++g)
#pragma unroll
      for (int i = 0; i < UG; ++i) {
        const int u = tid + i * NT;
        const int q = RES_STAGE_8R ? quad_pos((u >> 3) & 3) : (u & 3);
        const int r = RES_STAGE_8R ? (u >> 5) * 8 + (u & 7) : (u >> 2);
        if (r < PR) {
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = lrelu2(xv[g][i][j], 0.1f);
            if (H3) v[j] *= xs;
          }
          split_store4<S>(smem + (g * PR + r) * S::ROWB + 8 * quad_pos(q), v[0], v[1], v[2], v[3]);
        }
      }
    __builtin_amdgcn_sched_barrier(0);  // keep the loads below the window's use
    load_xr();
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < BPT; ++j) {
        const int e = tid + j * NT;
        if (e < C) bsm[i * C + e] = bl[i][j];
      }
  }
  __syncthreads();

  f32x16 acc[TM][TN];
  f32x4 ar[PD + 1][TM][NP], bcur[TN][NP], bnext[TN][NP];
  rsrc_t ra[TM];
  auto conv = [&](int wi, int roff, int kstep) {
#pragma unroll
    for (int m = 0; m < TM; ++m) ra[m] = make_rsrc(a.w[wi] + ((size_t)(wm * TM + m) * NC * K) * (NP * 256), 0xFFFFFFFFu);
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
    auto read_b = [&](int g, int k, f32x4 (*dst)[NP]) {
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        const unsigned char* pp = smem + (g * PR + xcol0 + n * 32 + roff + k * kstep) * S::ROWB + 16 * half;
#pragma unroll
        for (int q = 0; q < NP; ++q) dst[n][q] = *reinterpret_cast<const f32x4*>(pp + 32 * q);
      }
    };
    read_b(0, 0, bcur);
#pragma unroll
    for (int g = 0; g < NC; ++g) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int st = g * K + k;
#pragma unroll
        for (int m = 0; m < TM; ++m)
#pragma unroll
          for (int q = 0; q < NP; ++q)
            ar[PD][m][q] = bload4(ra[m], avoff, (unsigned)((st + PD) * NP + q) * 1024u);
        const bool more = (k + 1 < K) || (g + 1 < NC);
        if (more) read_b((k + 1 < K) ? g : g + 1, (k + 1 < K) ? k + 1 : 0, bnext);
        __builtin_amdgcn_sched_barrier(0);
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
        if (more) {
#pragma unroll
          for (int n = 0; n < TN; ++n)
#pragma unroll
            for (int q = 0; q < NP; ++q) bcur[n][q] = bnext[n][q];
        }
      }
    }
  };
  // block max of |v| over this workgroup (f16x3 scale exponent); every wave must call it.  The
  // red halves alternate per call, and the store_pieces barrier between two calls separates a
  // half's reads from its next writes, so one barrier per call suffices
  int red_half = 0;
  auto tile_exp = [&](float vmax) -> int {
    if (!H3) return 0;
    vmax = wave_max(vmax);
    if (lane == 0) red[red_half][wave] = vmax;
    __syncthreads();  // also: every wave is done reading the LDS region
    float mx = red[red_half][0];
#pragma unroll
    for (int w = 1; w < P::NW; ++w) mx = fmaxf(mx, red[red_half][w]);
    red_half ^= 1;
    int e = 0;
    if (mx > 0.f && mx < INFINITY) {
      int E;
      (void)frexpf(mx, &E);
      e = E - 14;
    }
    return e;
  };

  // acc-layout values (already zeroed where invalid) -> split pieces at LDS row column + roff;
  // rows of the region outside [roff, roff + RP_W) are zeroed
  auto store_pieces = [&](int roff, float scale) {
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n)
#pragma unroll
        for (int gl = 0; gl < 2; ++gl)
          store_xt8<S>(smem + (((mrow0 + m * 32) / 16 + gl) * PR + xcol0 + n * 32 + roff) * S::ROWB + 16 * half,
                       acc[m][n], 8 * gl, scale);
    // edge rows: [0, roff) and [roff + RP_W, PR) of every group
    constexpr int EB = 2 * R3_XOFF * S::ROWB;  // upper bound of edge bytes per group
    for (int e = tid * 16; e < NC * EB; e += NT * 16) {
      const int g = e / EB;
      const int o = e - g * EB;  // byte in the edge area: first roff rows, then the tail
      const int lead_b = roff * S::ROWB;
      const int tail_b = (PR - roff - RP_W) * S::ROWB;
      if (o < lead_b) *reinterpret_cast<f32x4*>(smem + g * PR * S::ROWB + o) = f32x4{};
      else if (o - lead_b < tail_b)
        *reinterpret_cast<f32x4*>(smem + (g * PR + roff + RP_W) * S::ROWB + (o - lead_b)) = f32x4{};
    }
  };

  int lo = -R3_XOFF, hi = RP_W + R3_XOFF;  // valid columns of the staged operand
#pragma unroll 1
  for (int it = 0; it < 3; ++it) {
    const int d = a.dil[it];
    // ---- convs1[it] on lrelu(x) (X rows = column + 5): taps at column + (k - 1) * d
    conv(2 * it, R3_XOFF - d, d);
    lo = max(lo + d, 0);  // outputs exist on the grid [0, RP_W) only
    hi = min(hi - d, RP_W);
    {
      const float sc = H3 ? ldexpf(1.f, ex + a.w_exp[2 * it]) : 1.f;
      const float* bs = bsm + (2 * it) * C;
      float vmax = 0.f;
#pragma unroll
      for (int m = 0; m < TM; ++m) {
        float bv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[r] = bs[mrow0 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half];
#pragma unroll
        for (int n = 0; n < TN; ++n) {
          const int col = xcol0 + n * 32;
          const int t = tx0 + col;
          const bool ok = col >= lo && col < hi && t >= 0 && t < T;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float v = lrelu2(acc[m][n][r] * sc + bv[r], 0.1f);
            v = ok ? v : 0.f;
            acc[m][n][r] = v;
            vmax = fmaxf(vmax, fabsf(v));
          }
        }
      }
      const int et = tile_exp(vmax);
      if (!H3) __syncthreads();  // every wave done reading X
      store_pieces(1, H3 ? ldexpf(1.f, -et) : 1.f);  // xt rows = column + 1
      __syncthreads();
      ex = et;
    }
    // ---- convs2[it] on xt: taps at column + k - 1 = xt rows column + k
    conv(2 * it + 1, 0, 1);
    lo += 1;
    hi -= 1;
    const float sc = H3 ? ldexpf(1.f, ex + a.w_exp[2 * it + 1]) : 1.f;
    const float* bs = bsm + (2 * it + 1) * C;
    if (it < 2) {
      float vmax = 0.f;
#pragma unroll
      for (int m = 0; m < TM; ++m) {
        float bv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[r] = bs[mrow0 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half];
#pragma unroll
        for (int n = 0; n < TN; ++n) {
          const int col = xcol0 + n * 32;
          const int t = tx0 + col;
          const bool ok = col >= lo && col < hi && t >= 0 && t < T;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float x1 = (acc[m][n][r] * sc + bv[r]) + xr[m][n][r];  // x = convs2(xt) + x
            xr[m][n][r] = x1;
            const float v = ok ? lrelu2(x1, 0.1f) : 0.f;  // the next convs1's operand
            acc[m][n][r] = v;
            vmax = fmaxf(vmax, fabsf(v));
          }
        }
      }
      const int e2 = tile_exp(vmax);
      if (!H3) __syncthreads();  // every wave done reading xt
      store_pieces(R3_XOFF, H3 ? ldexpf(1.f, -e2) : 1.f);
      __syncthreads();
      ex = e2;
    } else {
      // ---- final: x3 = convs2[2](xt) + x2 -> MRF z (kept columns [16, 16 + RP_BN) only)
      const rsrc_t rz = make_rsrc(a.z + (size_t)b * C * T, (unsigned)C * chb);
      float vmax = 0.f;
#pragma unroll
      for (int m = 0; m < TM; ++m) {
        float bv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[r] = bs[mrow0 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half];
#pragma unroll
        for (int n = 0; n < TN; ++n) {
          const int col = xcol0 + n * 32;
          const int t = tx0 + col;
          const bool keep = col >= R3_LEAD && col < R3_LEAD + P::RP_BN && t >= 0 && t < T;
          unsigned vo[16];
          float zv[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = mrow0 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
            vo[r] = keep ? (unsigned)co * chb + (unsigned)t * 4u : OOB_OFF;
            zv[r] = a.zmode >= 2 ? bload(rz, vo[r], 0u) : 0.f;
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float v = (acc[m][n][r] * sc + bv[r]) + xr[m][n][r];
            if (a.zmode == 2) v = zv[r] + v;
            else if (a.zmode == 3) v = (zv[r] + v) / a.zdiv;
            if (keep) vmax = fmaxf(vmax, fabsf(v));
            bstore(rz, v, vo[r], 0u);
          }
        }
      }
      if (H3 && a.amax_out) publish_amax(a.amax_out, b, vmax);
    }
  }
}

namespace {
template <class S, int C, int GEO>
void launch_res3_t(const ResBlock3Args& a, int B, hipStream_t s) {
  dim3 grid(ceil_div(a.T, Res3Cfg<S, C, GEO>::RP_BN), 1, B);
  hipLaunchKernelGGL((resblock3_kernel<S, C, GEO>), grid, dim3(Res3Cfg<S, C, GEO>::NT), 0, s, a);
}
template <class S>
void launch_res3_s(const ResBlock3Args& a, int B, int C, hipStream_t s) {
  // C = 64: 128 columns (2 waves/SIMD, a quarter of the columns are halo; 192 columns at one
  // wave per SIMD measured slower).  C = 128: 128 columns as 8 waves of 32 rows x 64 columns (two
  // per SIMD; 2 x 2 waves of 64 x 64 measured slower); LDS 8 x 138 rows
  if (C == 32) launch_res3_t<S, 32, 0>(a, B, s);
  else if (C == 128) {
    if constexpr (S::ROWB <= 80) launch_res3_t<S, 128, 3>(a, B, s);
    else throw Error(3, "resblock3: 128 channels need a split scheme of at most 80-byte rows");
  } else launch_res3_t<S, 64, 2>(a, B, s);
}
}  // namespace

bool resblock3_supported(int mode, int C, int K, const int* dil) {
  // C = 128 stages 8 groups x 138 rows: 88 KB of LDS for f16x3 / 53 KB for bf16 (x6 is not built)
  if (!is_split_mode(mode) || !(C == 32 || C == 64 || (C == 128 && mode != MATH_FP32_X6)) || K != 3) return false;
  // the kernel's valid-range walk: kept columns [R3_LEAD, RP_W - R3_LEAD) must stay inside it
  int lo = -R3_XOFF;
  for (int m = 0; m < 3; ++m) {
    if (dil[m] < 1 || dil[m] > R3_XOFF) return false;
    lo = std::max(lo + dil[m], 0) + 1;
  }
  return lo <= R3_LEAD;
}

void launch_resblock3(int mode, const ResBlock3Args& a, int B, int C, hipStream_t s) {
  TTS_REQUIRE(resblock3_supported(mode, C, 3, a.dil), 3, "resblock3: unsupported configuration");
  TTS_REQUIRE(a.zmode >= 1 && a.zmode <= 3 && a.z && a.x && a.x != a.z, 1, "resblock3: bad arguments");
  TTS_REQUIRE((int64_t)C * a.T * 4 < (int64_t(1) << 31), 3, "resblock3: plane exceeds 2 GiB");
  if (mode == MATH_FP32_F16X3) launch_res3_s<SchemeH3>(a, B, C, s);
  else if (mode == MATH_BF16) launch_res3_s<SchemeB1>(a, B, C, s);
  else launch_res3_s<SchemeX6>(a, B, C, s);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
