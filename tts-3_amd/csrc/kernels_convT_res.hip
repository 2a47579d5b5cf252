// Polyphase ConvTranspose1d (TTS/vocoder/models/hifigan_generator.py:206-218, applied at
// :253-254 after leaky_relu) for the x8 upsamplers, window-resident form (gfx950).
//
// As in conv1d_split_kernel's K = 2 form (Conv1dArgs::ups), output row rho = co * U + s and
// column m (input frame) take the taps x[m - 1], x[m]: a [U * Cout] x [2 * Cin] GEMM over the
// frames.  conv1d_split_kernel gives every 128-row block its own workgroup, so an x8 layer with
// 1024 rows stages each input window 8 times (PMC: 2.85 GB fetched for a 0.27 GB input at
// HiFiGAN-v1 stage 2) and each workgroup runs only 32 short MFMA steps between a staged window
// and its epilogue.  Here one workgroup of 8 waves stages the window of BN frames (all Cin
// channels, split into the scheme's pieces) once and then walks every (32 WR)-row pass over it:
// the waves form WR row blocks x WC column blocks of 32 x (32 TN), with no barrier after the
// staging (the LDS window is read-only), so the two waves of a SIMD drift apart and one's
// epilogue stores overlap the other's MFMAs.  The next pass's first weight steps are requested
// before the epilogue.  The x8 layer with 512 input channels (135 KB per 64-frame window, one
// workgroup per CU) splits each window's passes over RS workgroups.
// Measured (MI355X, f16x3, per batch): 512 channels 0.43 ms (RS = 2 or 4; RS = 8 0.48) against the
// split kernel's 0.52; 128-frame windows at 256 channels (TN = 4) 0.88 ms, as TN = 2.  The x2
// layers stay on conv1d_split_kernel: this form (WR = rows / 32, the other waves on further
// columns) took 1.13 / 0.95 ms (TN = 1) and 0.89 / 0.73 ms (TN = 2) against 0.77 / 0.67 ms.
// Arithmetic per output is conv1d_split_kernel's (same steps in the same order: 16-channel groups,
// tap 0 then tap 1, the scheme's products; f16x3 input scale from the producer's statistics).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "split_device.hpp"

namespace tts {

// LDS image of the window: f16x3 rows are the bare 64 B (2 pieces x 32 B) with the 16-B chunk
// c = 2 piece + half stored at c ^ ((row >> 2) & 3): the 16 lanes of a ds_read_b128 group read 16
// rows of distinct residue mod 16 (any tap shift), whose chunks then fall on 16 distinct 16-B bank
// groups, conflict-free like the split kernel's 80-B pitch, in 0.8 of its bytes (a 128-frame
// window of 256 channels, or a 64-frame window of 512, fits the 160 KB of a CU).  bf16 keeps the
// padded pitch.
template <class S>
struct ConvTResRow {
  static constexpr bool SWZ = S::NP == 2;
  static constexpr int RB = SWZ ? 32 * S::NP : S::ROWB;
  // byte offset of (row, 16-B chunk c = 2 piece + half) inside a group's image
  __device__ static __forceinline__ int at(int r, int c) { return r * RB + 16 * (SWZ ? (c ^ ((r >> 2) & 3)) : c); }
};

template <class S, int NG, int WR, int TN_>
struct ConvTResCfg {
  static constexpr int WC = 8 / WR;            // column-block waves
  static constexpr int TN = TN_;
  static constexpr int BN = WC * TN * 32;      // frames per workgroup
  static constexpr int XROWS = BN + 2;         // frames t0 - 1 .. t0 + BN (the last one pads)
  static constexpr int LDSB = NG * XROWS * ConvTResRow<S>::RB;
  static constexpr int UNITS = NG * XROWS * 4;  // staging units (group, row, channel quad)
  static constexpr int UPT = (UNITS + 511) / 512;
  static constexpr int NS = NG * 2;            // MFMA steps (group, tap)
  static constexpr int PD = 3;                 // weight prefetch distance (2, 3, 5 measured equal)
  static_assert(WR * WC == 8 && LDSB <= 160 * 1024, "8 waves, LDS window");
};

// RS: workgroups per window, each taking 1 / RS of the passes (restages the window RS times; the
// 512-channel layer's 544 windows would fill the 256 CUs only 2.1 times over)
// PL: Conv1dArgs::planes (the bf16 scheme: 0, or bf16 input and output planes)
template <class S, int NG, int WR, int TN_, int RS, int PL = 0>
__global__ __launch_bounds__(512) void convT_res_kernel(Conv1dArgs a) {
  constexpr bool XB = (PL & kPlaneXB16) != 0, YB = (PL & kPlaneYB16) != 0;
  using PX = PlaneT<XB>;
  using P = ConvTResCfg<S, NG, WR, TN_>;
  using R = ConvTResRow<S>;
  constexpr int RB = R::RB;
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
  constexpr int TN = P::TN, NS = P::NS, PD = P::PD;
  __shared__ __attribute__((aligned(16))) unsigned char smem[P::LDSB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave % WR, wc = wave / WR;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  // grid (tiles, B, RS): the pass share varies slowest, so the workgroups resident at one time
  // mostly read one share's weights (2 MB at 512 channels, inside an XCD's 4 MB L2; the whole 8.4 MB
  // set would not be)
  const int rs = RS > 1 ? (int)blockIdx.z : 0;
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * P::BN;  // first frame (column) of the tile
  const int Tin = a.Tin;
  const int Cin = a.Cin;
  const int rows = a.Cout;  // U * channels
  const int ex = H3 ? amax_exp(a.amax_in, b) : 0;
  const float xscale = H3 ? ldexpf(1.f, -ex) : 1.f;

  // ---- stage frames t0 - 1 .. t0 + BN of every channel (zero outside [0, Tin)) ----
  {
    const void* xb = plane_at<XB>(a.x, (size_t)b * (a.x_bstride ? a.x_bstride : (int64_t)Cin * Tin));
    const unsigned chb = (unsigned)Tin * PX::ES;
    const rsrc_t rx = make_rsrc(xb, (unsigned)Cin * chb);
    f32x4 xr[P::UPT];
#pragma unroll
    for (int i = 0; i < P::UPT; ++i) {
      const int u = tid + i * 512;
      const int q = u & 3;
      const int rr = u >> 2;
      const int g = rr / P::XROWS, r = rr - (rr / P::XROWS) * P::XROWS;
      const int ts = t0 - 1 + r;
      const bool ok = g < NG && ts >= 0 && ts < Tin;
      // OOB_OFF + 3 * chb stays out of range (planes < 2 GiB)
      const unsigned vo = ok ? (unsigned)(16 * g + 4 * q) * chb + (unsigned)ts * PX::ES : OOB_OFF;
#pragma unroll
      for (int j = 0; j < 4; ++j) xr[i][j] = PX::ld(rx, vo + (unsigned)j * chb, 0u);
    }
#pragma unroll
    for (int i = 0; i < P::UPT; ++i) {
      const int u = tid + i * 512;
      const int q = u & 3;
      const int rr = u >> 2;
      if (rr < NG * P::XROWS) {
        const int g = rr / P::XROWS, r = rr - (rr / P::XROWS) * P::XROWS;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = lrelu2(xr[i][j], a.in_slope);
          if (H3) v[j] *= xscale;
        }
        // quad q sits at position quad_pos(q) of each piece (the packed weights' channel order)
        const int qp = quad_pos(q);
        unsigned w0[NP], w1[NP];
        S::split2(v[0], v[1], w0);
        S::split2(v[2], v[3], w1);
        unsigned char* row = smem + g * P::XROWS * RB;
#pragma unroll
        for (int pc = 0; pc < NP; ++pc)
          *reinterpret_cast<u32x2*>(row + R::at(r, 2 * pc + (qp >> 1)) + 8 * (qp & 1)) = u32x2{w0[pc], w1[pc]};
      }
    }
  }

  // ---- weight stream of 32-row block (pass, wr): steps s = 2 * group + tap ----
  const int npt = rows / (32 * WR);                  // passes over the window
  const int pass0 = RS > 1 ? rs * npt / RS : 0;       // this workgroup's share
  const int npass = RS > 1 ? (rs + 1) * npt / RS : npt;
  const unsigned avoff = (unsigned)lane * 16u;
  auto wsrc = [&](int pass) {
    const int mb = pass * WR + wr;
    return make_rsrc(a.w + ((size_t)mb * NS) * (NP * 256), 0xFFFFFFFFu);
  };
  f32x4 ar[PD + 1][NP], bcur[TN][NP], bnext[TN][NP];
  rsrc_t ra = wsrc(pass0);
#pragma unroll
  for (int s = 0; s < PD; ++s)
#pragma unroll
    for (int q = 0; q < NP; ++q) ar[s][q] = bload4(ra, avoff, (unsigned)(s * NP + q) * 1024u);
  __syncthreads();

  // the lane's (tap, piece) chunk offsets at row l32 of this wave's first column block (32-row
  // steps keep the swizzle: it depends on row bits 2-3)
  int roff[2][NP];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int q = 0; q < NP; ++q) roff[k][q] = R::at(wc * TN * 32 + l32 + k, 2 * q + half);
  auto read_b = [&](int s, f32x4 (*dst)[NP]) {
    const int g = s >> 1, k = s & 1;
#pragma unroll
    for (int n = 0; n < TN; ++n)
#pragma unroll
      for (int q = 0; q < NP; ++q)
        dst[n][q] = *reinterpret_cast<const f32x4*>(smem + roff[k][q] + (g * P::XROWS + n * 32) * RB);
  };
  const float sc = H3 ? ldexpf(1.f, ex + a.w_exp) : 1.f;
  for (int pass = pass0; pass < npass; ++pass) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int q = 0; q < NP; ++q) asm volatile("" : "+v"(roff[k][q]));  // keep the step addresses in the pass loop
    f32x16 acc[1][TN];
#pragma unroll
    for (int n = 0; n < TN; ++n) acc[0][n] = f32x16{};
    read_b(0, bcur);
    const bool more = pass + 1 < npass;
    const rsrc_t rn = wsrc(more ? pass + 1 : pass);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      // weights of step s + PD; past the end: the next pass's first steps (same offsets)
#pragma unroll
      for (int q = 0; q < NP; ++q)
        ar[PD][q] = s + PD < NS ? bload4(ra, avoff, (unsigned)(((s + PD) * NP + q) * 1024u))
                                : bload4(rn, avoff, (unsigned)(((s + PD - NS) * NP + q) * 1024u));
      if (s + 1 < NS) read_b(s + 1, bnext);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < S::NPROD; ++e)
#pragma unroll
        for (int n = 0; n < TN; ++n) acc[0][n] = S::mfma(ar[0][S::PA[e]], bcur[n][S::PB[e]], acc[0][n]);
#pragma unroll
      for (int pp = 0; pp < PD; ++pp)
#pragma unroll
        for (int q = 0; q < NP; ++q) ar[pp][q] = ar[pp + 1][q];
      if (s + 1 < NS) {
#pragma unroll
        for (int n = 0; n < TN; ++n)
#pragma unroll
          for (int q = 0; q < NP; ++q) bcur[n][q] = bnext[n][q];
      }
    }
    ra = rn;
    if (H3) {
#pragma unroll
      for (int n = 0; n < TN; ++n) acc[0][n] *= sc;
    }
    convT_epilogue<1, TN, H3, YB>(a, acc, b, t0 + wc * TN * 32, (pass * WR + wr) * 32, lane);
  }
}

namespace {
template <class S, int NG, int WR, int TN, int RS = 1>
void launch_res_t(const Conv1dArgs& a, int B, hipStream_t s) {
  TTS_REQUIRE(a.Cin == 16 * NG && a.Cout % (32 * WR) == 0 && a.Cout / (32 * WR) >= RS, 1,
              "convT_res: bad shape for this instance");
  const dim3 grid(ceil_div(a.Tout, ConvTResCfg<S, NG, WR, TN>::BN), B, RS);
  if (a.planes != 0) {
    constexpr bool OK = std::is_same<S, SchemeB1>::value;
    TTS_REQUIRE(OK && a.planes == (kPlaneXB16 | kPlaneYB16), 3, "convT_res: bf16 planes need the bf16 scheme");
    if constexpr (OK)
      hipLaunchKernelGGL((convT_res_kernel<S, NG, WR, TN, RS, kPlaneXB16 | kPlaneYB16>), grid, dim3(512), 0, s, a);
    return;
  }
  hipLaunchKernelGGL((convT_res_kernel<S, NG, WR, TN, RS>), grid, dim3(512), 0, s, a);
}
// 256-row passes (8 row-block waves, 64-frame windows)
template <class S>
void launch_res_s(const Conv1dArgs& a, int B, hipStream_t s) {
  if (a.Cin == 512) launch_res_t<S, 32, 8, 2, 4>(a, B, s);
  else if (a.Cin == 256) launch_res_t<S, 16, 8, 2>(a, B, s);
  else launch_res_t<S, 8, 8, 2>(a, B, s);
}
}  // namespace

// The x8 ConvTranspose layers with 128, 256 or 512 input channels and a multiple of 256 rows
// (1024 or more at 512 channels), f16x3 / bf16 (the others take conv1d_split_kernel)
bool convT_res_supported(int mode, const Conv1dArgs& a) {
  const bool shape = a.ups == 8 && a.Cout % 256 == 0 && (a.Cin == 128 || a.Cin == 256 || (a.Cin == 512 && a.Cout >= 1024));
  return (mode == MATH_FP32_F16X3 || mode == MATH_BF16) && shape && a.Tout == a.Tin + 1 && a.pad == 1 &&
         a.dil == 1 && a.zmode == 0 && !a.res && !a.mask;
}

void launch_convT_res(int mode, const Conv1dArgs& a, int B, hipStream_t s) {
  if (mode == MATH_FP32_F16X3) launch_res_s<SchemeH3>(a, B, s);
  else launch_res_s<SchemeB1>(a, B, s);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
