// Polyphase ConvTranspose1d (TTS/vocoder/models/hifigan_generator.py:206-218, applied at
// :253-254 after leaky_relu) for the x8 upsamplers with Cin <= 256, window-resident form (gfx950).
//
// As in conv1d_split_kernel's K = 2 form (Conv1dArgs::ups), output row rho = co * U + s and
// column m (input frame) take the taps x[m - 1], x[m]: a [U * Cout] x [2 * Cin] GEMM over the
// frames.  conv1d_split_kernel gives every 128-row block its own workgroup, so an x8 layer with
// 1024 rows stages each input window 8 times (PMC: 2.85 GB fetched for a 0.27 GB input at
// HiFiGAN-v1 stage 2) and each workgroup runs only 32 short MFMA steps between a staged window
// and its epilogue.  Here one workgroup of 8 waves stages the window of 64 frames (all Cin
// channels, split into the scheme's pieces) once and then walks every 256-row pass over it:
// wave w owns rows 32 w .. 32 w + 31 of each pass, with no barrier after the staging (the LDS
// window is read-only), so the two waves of a SIMD drift apart and one's epilogue stores overlap
// the other's MFMAs.  The next pass's first weight steps are requested before the epilogue.
// Arithmetic per output is conv1d_split_kernel's (same steps in the same order: 16-channel groups,
// tap 0 then tap 1, the scheme's products; f16x3 input scale from the producer's statistics).
#include <algorithm>
#include <cstdlib>

#include "split_device.hpp"

namespace tts {


template <class S, int NG>
struct ConvTResCfg {
  static constexpr int BN = 64;                // frames per workgroup (2 column blocks per wave)
  static constexpr int TN = 2;
  static constexpr int XROWS = BN + 2;         // frames t0 - 1 .. t0 + 64 (the last one pads)
  static constexpr int LDSB = NG * XROWS * S::ROWB;
  static constexpr int UNITS = NG * XROWS * 4;  // staging units (group, row, channel quad)
  static constexpr int UPT = (UNITS + 511) / 512;
  static constexpr int NS = NG * 2;            // MFMA steps (group, tap)
  static constexpr int PD = 3;                 // weight prefetch distance (2, 3, 5 measured equal)
  static_assert(LDSB <= 96 * 1024, "LDS window");
};

template <class S, int NG>
__global__ __launch_bounds__(512) void convT_res_kernel(Conv1dArgs a) {
  using P = ConvTResCfg<S, NG>;
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
  constexpr int TN = P::TN, NS = P::NS, PD = P::PD;
  __shared__ __attribute__((aligned(16))) unsigned char smem[P::LDSB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * P::BN;  // first frame (column) of the tile
  const int Tin = a.Tin;
  const int Cin = a.Cin;
  const int rows = a.Cout;  // U * channels
  const int ex = H3 ? amax_exp(a.amax_in, b) : 0;
  const float xscale = H3 ? ldexpf(1.f, -ex) : 1.f;

  // ---- stage frames t0 - 1 .. t0 + 64 of every channel (zero outside [0, Tin)) ----
  {
    const float* xb = a.x + (size_t)b * (a.x_bstride ? a.x_bstride : (int64_t)Cin * Tin);
    const unsigned chb = (unsigned)Tin * 4u;
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
      const unsigned vo = ok ? (unsigned)(16 * g + 4 * q) * chb + (unsigned)ts * 4u : OOB_OFF;
#pragma unroll
      for (int j = 0; j < 4; ++j) xr[i][j] = bload(rx, vo + (unsigned)j * chb, 0u);
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
        split_store4<S>(smem + (g * P::XROWS + r) * S::ROWB + 8 * q, v[0], v[1], v[2], v[3]);
      }
    }
  }

  // ---- weight stream of 32-row block (pass, wave): steps s = 2 * group + tap ----
  const int npass = rows / 256;
  const unsigned avoff = (unsigned)lane * 16u;
  auto wsrc = [&](int pass) {
    const int mb = pass * 8 + wave;
    return make_rsrc(a.w + ((size_t)mb * NS) * (NP * 256), 0xFFFFFFFFu);
  };
  f32x4 ar[PD + 1][NP], bcur[TN][NP], bnext[TN][NP];
  rsrc_t ra = wsrc(0);
#pragma unroll
  for (int s = 0; s < PD; ++s)
#pragma unroll
    for (int q = 0; q < NP; ++q) ar[s][q] = bload4(ra, avoff, (unsigned)(s * NP + q) * 1024u);
  __syncthreads();

  int lane_off = l32 * S::ROWB + 16 * half;  // row l32 of column block 0, this lane's half
  auto read_b = [&](int s, f32x4 (*dst)[NP]) {
    const int g = s >> 1, k = s & 1;
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const unsigned char* p = smem + lane_off + (g * P::XROWS + n * 32 + k) * S::ROWB;
#pragma unroll
      for (int q = 0; q < NP; ++q) dst[n][q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
    }
  };
  const float sc = H3 ? ldexpf(1.f, ex + a.w_exp) : 1.f;
  for (int pass = 0; pass < npass; ++pass) {
    asm volatile("" : "+v"(lane_off));  // keep the step addresses inside the pass loop
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
    convT_epilogue<1, TN, H3>(a, acc, b, t0, pass * 256 + wave * 32, lane);
  }
}

namespace {
template <class S, int NG>
void launch_res_t(const Conv1dArgs& a, int B, hipStream_t s) {
  const dim3 grid(ceil_div(a.Tout, ConvTResCfg<S, NG>::BN), B);
  hipLaunchKernelGGL((convT_res_kernel<S, NG>), grid, dim3(512), 0, s, a);
}
template <class S>
void launch_res_s(const Conv1dArgs& a, int B, hipStream_t s) {
  if (a.Cin == 256) launch_res_t<S, 16>(a, B, s);
  else launch_res_t<S, 8>(a, B, s);
}
}  // namespace

// The x8 ConvTranspose layers with 128 or 256 input channels and a multiple of 256 rows, f16x3 /
// bf16 (the others take conv1d_split_kernel)
bool convT_res_supported(int mode, const Conv1dArgs& a) {
  return (mode == MATH_FP32_F16X3 || mode == MATH_BF16) && a.ups == 8 && (a.Cin == 128 || a.Cin == 256) &&
         a.Cout % 256 == 0 && a.Tout == a.Tin + 1 && a.pad == 1 && a.dil == 1 && a.zmode == 0 && !a.res && !a.mask;
}

void launch_convT_res(int mode, const Conv1dArgs& a, int B, hipStream_t s) {
  if (mode == MATH_FP32_F16X3) launch_res_s<SchemeH3>(a, B, s);
  else launch_res_s<SchemeB1>(a, B, s);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
