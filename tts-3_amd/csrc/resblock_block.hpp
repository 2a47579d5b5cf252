// ---------------------------------------------------------------------------------------
// Whole-ResBlock kernels (hifigan_generator.py:84-99 ResBlock1, :150-155 ResBlock2) in one launch.
// ResBlock1, kernel 3 (NCV = 6 convs, dilations d0..d2):
//   for m in 0..2:  xt = lrelu(convs1[m](lrelu(x)));  x = convs2[m](xt) + x;   z (+)= x
// ResBlock2, any kernel K in {3, 5, 7, 11} (NCV = 2 convs, dilations d0, d1):
//   for m in 0..1:  x = convs[m](lrelu(x)) + x;                                   z (+)= x
// Every conv runs on the same RP_W-column grid (column c <-> time t0 - LEAD + c): each conv loses
// its halo (K - 1) / 2 * d at the grid edges, so the valid columns shrink per conv (ResBlock1 k3
// with dilations 1, 3, 5: 11 per side; the first conv reads XO staged extra columns, the rest only
// the grid) while the kept ones, [LEAD, RP_W - LEAD), stay exact.  x lives in the accumulator
// layout in registers (the residual of every iteration), lrelu(x) and xt alternate in one LDS
// region as split B operands (X rows: column + XO, xt rows: column + (K - 1) / 2).  Columns
// outside the valid range or outside [0, T) are staged as zeros; in the f16x3 scheme the scale of
// every staged operand after the first is the workgroup's own power of two over its valid columns
// (exact and batch-invariant), x0 uses its producer's statistics.  One launch replaces three pair
// launches (ResBlock1) or two conv launches (ResBlock2): x is read once and z written once.
// ---------------------------------------------------------------------------------------
#pragma once
#include <type_traits>

#include "split_device.hpp"

#ifndef RES_PD_B1
#define RES_PD_B1 2  // weight prefetch depth of the whole-block and pair kernels in the bf16 scheme
#endif
#ifndef RES_STAGE_8R
#define RES_STAGE_8R 1  // x staging lane map of the pair / whole-block kernels (0: 4 rows x 4 quads)
#endif

namespace tts {

// ResBlock1 k3: X rows hold column + 5 (convs1 halo up to dilation 5); kept columns
// [R3_LEAD, RP_W - R3_LEAD): only the first conv sees the R3_XOFF staged extra columns, every
// later one loses d_m (+ 1) columns at the grid edge, 11 for dilations 1, 3, 5
#ifndef R3_XR_POL
#define R3_XR_POL 0  // cache policy of the residual re-read (A/B)
#endif
constexpr int R3_XOFF = 5;
constexpr int R3_LEAD = 12;
// ResBlock1 of kernel K (round 5: 7 and 11 at 32 / 64 channels): every conv's halo scales by
// (K - 1) / 2, so X rows hold column + 5 (K - 1) / 2 and the kept columns lose 12 (K - 1) / 2
// (K 7: 15 / 36, K 11: 25 / 60)
constexpr int r3_xoff(int K) { return R3_XOFF * ((K - 1) / 2); }
constexpr int r3_lead(int K) { return R3_LEAD * ((K - 1) / 2); }
// ResBlock2 kernel K: XO = LEAD = (K - 1) / 2 * the largest dilation it takes (K 3: 4, K 5: 6,
// K 7 / 11: 3; HiFiGAN-v3 [[1, 2], [2, 6], [3, 12]] up to kernel 5, YourTTS (1, 3) for 3, 7, 11)
constexpr int rb2_halo(int K) { return K == 3 ? 4 : (K == 5 ? 12 : (K == 7 ? 9 : 15)); }

// GEO 0: 256 columns, 4 waves side by side; GEO 1 / 2: 192 / 128 columns, 2 x 2 waves;
// GEO 3: 128 columns, 8 waves (4 row blocks x 2 column halves at C = 128, two waves per SIMD).
// Measured (f16x3, per batch): C = 128 GEO 3 5.0 ms vs GEO 2 5.5 ms; 8-wave forms at C = 64
// (256 columns) and C = 32 (512 columns) were slower than GEO 2 / GEO 0 (+0.2 / +0.3 ms).
template <class S, int C, int GEO, int K = 3, int NCV = 6, int XO = R3_XOFF, int LEAD = R3_LEAD>
struct Res3Cfg {
  static constexpr int RP_W = GEO == 0 ? 256 : (GEO == 1 ? 192 : 128);
  static constexpr int RP_BN = RP_W - 2 * LEAD;
  static constexpr int NW = GEO == 3 ? 8 : 4;     // waves per workgroup
  static constexpr int NT = 64 * NW;
  static constexpr int WN = GEO == 0 ? 4 : 2;
  static constexpr int WM = NW / WN;
  static constexpr int TM = C / 32 / WM;
  static constexpr int TN = RP_W / 32 / WN;
  static constexpr int NC = C / 16;
  static constexpr int PR = RP_W + 2 * XO;  // rows per group (X: RP_W + 2 XO, xt: RP_W + K - 1)
  static constexpr int LDSB = NC * PR * S::ROWB;
  static_assert(TM >= 1 && TM * WM * 32 == C && TN * WN * 32 == RP_W, "geometry");
};

#ifndef RB3_W_B1
#define RB3_W_B1 0  // A/B: waves per SIMD asked of the bf16 scheme's whole-block kernels (0: as the others)
#endif
#ifndef RB3_W64
#define RB3_W64 2  // A/B build option: waves per SIMD requested for the 64-channel 128-column block
#endif
// PL: ResBlock3Args::planes (the bf16 scheme: 0, or bf16 x and z planes; x stays fp32 in registers)
template <class S, int C, int GEO, int K, int NCV, int XO, int LEAD, int PL = 0>
__global__ __launch_bounds__((Res3Cfg<S, C, GEO, K, NCV, XO, LEAD>::NT))
__attribute__((amdgpu_waves_per_eu(S::NP == 1 && RB3_W_B1 > 0 ? RB3_W_B1
                                                                : (C == 64 && GEO == 2 ? RB3_W64 : (C == 32 || GEO == 3 ? 2 : 1)))))
void resblock3_kernel(ResBlock3Args a) {
  constexpr bool XB = (PL & kPlaneXB16) != 0, YB = (PL & kPlaneYB16) != 0;
  using PX = PlaneT<XB>;
  using PY = PlaneT<YB>;
  using P = Res3Cfg<S, C, GEO, K, NCV, XO, LEAD>;
  static_assert(NCV == 6 || NCV == 2, "ResBlock1 (6 convs) or ResBlock2 (2 convs)");
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
  constexpr int TM = P::TM, TN = P::TN, NC = P::NC, PR = P::PR, RP_W = P::RP_W;
  constexpr int PD = S::NP == 1 ? RES_PD_B1 : 2;  // weight prefetch steps (bf16: its own, A/B)
  __shared__ __attribute__((aligned(16))) unsigned char smem[P::LDSB];
  constexpr int NT = P::NT;
  __shared__ float red[2][P::NW];  // double-buffered: consecutive tile_exp calls use different halves
  __shared__ float bsm[NCV * C];  // the conv biases (read by every epilogue: LDS, not L2, latency)

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
  const int tx0 = t0 - LEAD;  // time of column 0
  const int xcol0 = wn * TN * 32 + l32;
  const unsigned avoff = (unsigned)lane * 16u;
  const unsigned chb = (unsigned)T * PX::ES;
  const rsrc_t rx = make_rsrc(plane_at<XB>(a.x, (size_t)b * C * T), (unsigned)C * chb);
  auto ldx = [&](unsigned off, auto pol_tag) -> float {
    if constexpr (XB) return PX::ld(rx, off, 0u);
    else return bload_x<decltype(pol_tag)::value>(rx, off, 0u);
  };

  // ---- prologue: lrelu(x0) pieces for columns [-XO, RP_W + XO) of every 16-channel group, and x0
  // itself in the acc layout.  Every load is issued before the first store (one HBM latency for
  // the whole window instead of one per group: at C = 128 that is 8 groups, 64 VGPRs of window)
  int ex = H3 ? amax_exp(a.amax_in, b) : 0;
  f32x16 xr[TM][TN];  // the running residual x (fp32), accumulator layout
  {
    const float xs = H3 ? ldexpf(1.f, -ex) : 1.f;
    constexpr int UG = (PR * 4 + NT - 1) / NT;  // units (row, quad) per group per thread
    constexpr int BPT = (C + NT - 1) / NT;
    float bl[NCV][BPT];
#pragma unroll
    for (int i = 0; i < NCV; ++i)
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
        const int ts = tx0 - XO + r;
        const bool ok = r < PR && ts >= 0 && ts < T;
        const unsigned vo = (unsigned)(16 * g + 4 * q) * chb + (unsigned)ts * PX::ES;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          xv[g][i][j] = ldx(ok ? vo + (unsigned)j * chb : OOB_OFF, std::integral_constant<int, TTS_LDX_POL>{});
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
            xr[m][n][r] = ldx(tok ? (unsigned)co * chb + (unsigned)t * PX::ES : OOB_OFF,
                              std::integral_constant<int, R3_XR_POL>{});
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
    for (int i = 0; i < NCV; ++i)
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
    constexpr int EB = 2 * XO * S::ROWB;  // upper bound of edge bytes per group
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

  constexpr int HK = (K - 1) / 2;
  int lo = -XO, hi = RP_W + XO;  // valid columns of the staged operand
  // conv ci adds the residual: x = conv(.) + x; the next conv's operand lrelu(x) goes to the X
  // rows (column + XO)
  auto residual_to_lds = [&](int ci) {
    const float sc = H3 ? ldexpf(1.f, ex + a.w_exp[ci]) : 1.f;
    const float* bs = bsm + ci * C;
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
          const float x1 = (acc[m][n][r] * sc + bv[r]) + xr[m][n][r];  // x = conv(.) + x
          xr[m][n][r] = x1;
          const float v = ok ? lrelu2(x1, 0.1f) : 0.f;  // the next conv's operand
          acc[m][n][r] = v;
          vmax = fmaxf(vmax, fabsf(v));
        }
      }
    }
    const int e2 = tile_exp(vmax);
    if (!H3) __syncthreads();  // every wave done reading the region
    store_pieces(XO, H3 ? ldexpf(1.f, -e2) : 1.f);
    __syncthreads();
    ex = e2;
  };
  // the block's last conv: x_out = conv(.) + x -> MRF z (kept columns [LEAD, LEAD + RP_BN) only)
  auto final_to_z = [&](int ci) {
    const float sc = H3 ? ldexpf(1.f, ex + a.w_exp[ci]) : 1.f;
    const float* bs = bsm + ci * C;
    const unsigned chbz = (unsigned)T * PY::ES;
    const rsrc_t rz = make_rsrc(plane_at<YB>(a.z, (size_t)b * C * T), (unsigned)C * chbz);
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
        const bool keep = col >= LEAD && col < LEAD + P::RP_BN && t >= 0 && t < T;
        unsigned vo[16];
        float zv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = mrow0 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
          vo[r] = keep ? (unsigned)co * chbz + (unsigned)t * PY::ES : OOB_OFF;
          zv[r] = a.zmode >= 2 ? PY::ld(rz, vo[r], 0u) : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = (acc[m][n][r] * sc + bv[r]) + xr[m][n][r];
          if (a.zmode == 2) v = zv[r] + v;
          else if (a.zmode == 3) v = (zv[r] + v) / a.zdiv;
          if (keep) vmax = fmaxf(vmax, fabsf(v));
          PY::st(rz, v, vo[r], 0u);
        }
      }
    }
    if (H3 && a.amax_out) publish_amax(a.amax_out, b, vmax);
  };

  if constexpr (NCV == 6) {
#pragma unroll 1
    for (int it = 0; it < 3; ++it) {
      const int d = a.dil[it];
      // ---- convs1[it] on lrelu(x) (X rows = column + XO): taps at column + (k - HK) * d
      conv(2 * it, XO - HK * d, d);
      lo = max(lo + HK * d, 0);  // outputs exist on the grid [0, RP_W) only
      hi = min(hi - HK * d, RP_W);
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
        store_pieces(HK, H3 ? ldexpf(1.f, -et) : 1.f);  // xt rows = column + HK
        __syncthreads();
        ex = et;
      }
      // ---- convs2[it] on xt: taps at column + k - HK = xt rows column + k
      conv(2 * it + 1, 0, 1);
      lo += HK;
      hi -= HK;
      if (it < 2) residual_to_lds(2 * it + 1);
      else final_to_z(2 * it + 1);
    }
  } else {
#pragma unroll 1
    for (int it = 0; it < 2; ++it) {
      const int d = a.dil[it];
      // ---- convs[it] on lrelu(x) (X rows = column + XO): taps at column + (k - HK) * d
      conv(it, XO - HK * d, d);
      lo = max(lo + HK * d, 0);
      hi = min(hi - HK * d, RP_W);
      if (it == 0) residual_to_lds(0);
      else final_to_z(1);
    }
  }
}

}  // namespace tts

namespace tts {
// ResBlock2 launchers (one translation unit per split scheme: kernels_resblock2_{h3,b1,x6}.hip).
// Geometry: C = 32 256 columns, C = 64 128 columns (geo64 = 1: 192), C = 128 128 columns as 8
// waves (kernels 3 and 5 only: 7 and 11 take Winograd F(4,4) per conv at >= 128 channels).
// the launch of one whole-block instance, with its bf16-plane form when ResBlock3Args::planes asks
template <class S, int C, int GEO, int K, int NCV, int XO, int LEAD>
void launch_block_pl(const ResBlock3Args& a, dim3 grid, int nt, hipStream_t s) {
  if (a.planes != 0) {
    constexpr bool OK = std::is_same<S, SchemeB1>::value;
    TTS_REQUIRE(OK && a.planes == (kPlaneXB16 | kPlaneYB16), 3, "resblock block: bf16 planes need the bf16 scheme");
    if constexpr (OK)
      hipLaunchKernelGGL((resblock3_kernel<S, C, GEO, K, NCV, XO, LEAD, kPlaneXB16 | kPlaneYB16>), grid, dim3(nt), 0, s, a);
    return;
  }
  hipLaunchKernelGGL((resblock3_kernel<S, C, GEO, K, NCV, XO, LEAD>), grid, dim3(nt), 0, s, a);
}
template <class S, int C, int GEO, int K>
void launch_rb2_t(const ResBlock3Args& a, int B, hipStream_t s) {
  constexpr int H = rb2_halo(K);
  using P = Res3Cfg<S, C, GEO, K, 2, H, H>;
  dim3 grid(ceil_div(a.T, P::RP_BN), 1, B);
  launch_block_pl<S, C, GEO, K, 2, H, H>(a, grid, P::NT, s);
}
template <class S, int C, int GEO>
void launch_rb2_k(const ResBlock3Args& a, int B, int K, hipStream_t s) {
  if (K == 3) launch_rb2_t<S, C, GEO, 3>(a, B, s);
  else if (K == 5) launch_rb2_t<S, C, GEO, 5>(a, B, s);
  else if (K == 7) launch_rb2_t<S, C, GEO, 7>(a, B, s);
  else launch_rb2_t<S, C, GEO, 11>(a, B, s);
}
template <class S>
void launch_rb2_s(const ResBlock3Args& a, int B, int C, int K, int geo64, hipStream_t s) {
  if (C == 32) launch_rb2_k<S, 32, 0>(a, B, K, s);
  else if (C == 64) {
    if (geo64 == 1) launch_rb2_k<S, 64, 1>(a, B, K, s);
    else launch_rb2_k<S, 64, 2>(a, B, K, s);
  } else {
    if constexpr (S::ROWB <= 80) {
      if (K == 3) launch_rb2_t<S, 128, 3, 3>(a, B, s);
      else launch_rb2_t<S, 128, 3, 5>(a, B, s);
    } else {
      throw Error(3, "resblock2: 128 channels need a split scheme of at most 80-byte rows");
    }
  }
}
void launch_resblock2_h3(const ResBlock3Args& a, int B, int C, int K, int geo64, hipStream_t s);
void launch_resblock2_b1(const ResBlock3Args& a, int B, int C, int K, int geo64, hipStream_t s);
void launch_resblock2_x6(const ResBlock3Args& a, int B, int C, int K, int geo64, hipStream_t s);
}  // namespace tts
