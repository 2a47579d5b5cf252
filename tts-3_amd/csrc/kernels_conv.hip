// HiFiGAN hot-path kernels for gfx950 (CDNA4), fp32 in / fp32 accumulate.
//
// conv1d_mfma   : "same" dilated Conv1d as an implicit GEMM on v_mfma_f32_32x32x2_f32.
//                 Reference ops: conv_pre (hifigan_generator.py:203,249), the 72 MRF convs of
//                 ResBlock1.forward (:93-98) / ResBlock2.forward (:151-154), with the
//                 leaky_relu before each conv fused into the LDS staging, the leaky_relu after
//                 convs1 fused into the epilogue, the residual add (:98) and the MRF sum
//                 z_sum += ...; o = z_sum / num_kernels (:255-261) fused into the epilogue.
// convT_mfma    : polyphase ConvTranspose1d (ups[i], :206-218, :253-254), K == 2*stride.
//                 All U phases of a 32-frame column block live in registers, so the epilogue
//                 writes U contiguous output samples per lane.
// conv_post     : leaky_relu(0.01) -> conv_post (Cout 1, k7) -> tanh (:262-264).
//
// Data layout: NCW fp32 in HBM, exactly the reference tensors.  Each workgroup owns a
// [BM output channels] x [BN output samples] tile of one batch item and loops over input
// channels in chunks of CK: the chunk's packed weights [K][CK][BM] and its input window
// [CK][BN + (K-1)*dil] are staged in LDS once and reused by every tap and every wave.
// Double-buffered: the next chunk is fetched to registers while the MFMAs run on the
// current one; one barrier per chunk.
#include <cstdint>
#include <cstdlib>

#include "conv_device.hpp"

namespace tts {

// Halo ((K-1)*dilation) the staged input window is sized for: the narrow variant covers
// dilation <= 5 (HiFiGAN v1/v2, Glow WN), the wide one HiFiGAN-v3's dilation 6 / 12.
constexpr int DMAX = 5;
constexpr int HALO_WIDE = 96;

// conv1d_mfma v2
//   A operand (weights) is streamed from L2 straight into VGPRs: the host packs W into
//   MFMA fragments [mblock32][cgroup8][tap][lane 64][4], so one coalesced 1 KiB dwordx4 per
//   wave brings 4 k-substeps (8 input channels: lane half h holds channels 4h..4h+3) of one
//   32-row block; prefetched one step ahead.
//   B operand (input window) is staged once per chunk in LDS as [group][t][8 ch + 4 pad]:
//   48-byte rows make the per-lane ds_read_b128 (4 k-substeps of one column) conflict-free
//   at any tap shift k*dil.  The leaky_relu before the conv is applied while staging.
//   One step = (channel group, tap): TM A-loads, TN b128 LDS reads, 4*TM*TN MFMAs.
template <int K, int BM, int BN, int TM, int TN, int G, int HMAX, int PD>
struct ConvCfg {
  static constexpr int WM = BM / (32 * TM);
  static constexpr int WN = BN / (32 * TN);
  static constexpr int CK = 8 * G;               // input channels per LDS chunk
  static constexpr int XROWS = BN + HMAX;        // t rows reserved per group
  static constexpr int XSZ = G * XROWS * 8;      // floats per LDS buffer (32-byte rows)
  static constexpr int UNITS = G * XROWS * 2;    // staging units (group, row, channel quad)
  static constexpr int UPT = (UNITS + 255) / 256;
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(PD == 1 || PD == 2, "A prefetch distance");
};

template <int K, int BM, int BN, int TM, int TN, int G, int HMAX, int PD>
__global__ __launch_bounds__(256) void conv1d_mfma_kernel(Conv1dArgs a) {
  using C = ConvCfg<K, BM, BN, TM, TN, G, HMAX, PD>;
  __shared__ __attribute__((aligned(16))) float smem[2 * C::XSZ];

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
  const int XW = BN + (K - 1) * d;  // rows actually used per group
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
  unsigned uvoff[C::UPT];  // byte offset of channel (8g+4q) at the clamped source time, or OOB
  int ulds[C::UPT];        // LDS offset of the row's quad
#pragma unroll
  for (int i = 0; i < C::UPT; ++i) {
    const int u = tid + i * 256;
    const int q = u & 1;
    const int rr = u >> 1;
    const int g = rr / XW;
    const int r = rr - g * XW;
    const int ts = t0 - a.pad + r;
    const bool ok = (g < G) && ts >= 0 && ts < Tout;
    int src = ts - a.rep_pad;
    src = src < 0 ? 0 : (src >= Tin ? Tin - 1 : src);
    uvoff[i] = ok ? (unsigned)(8 * g + 4 * q) * chb + (unsigned)src * 4u : OOB_OFF;
    ulds[i] = (g < G) ? xlds_off(g, r, q, C::XROWS) : -1;
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
    float* xl = smem + buf * C::XSZ;
    const float slope = a.in_slope;
#pragma unroll
    for (int i = 0; i < C::UPT; ++i) {
      if (ulds[i] >= 0) {
        f32x4 v = xreg[i];
        v[0] = lrelu2(v[0], slope); v[1] = lrelu2(v[1], slope);
        v[2] = lrelu2(v[2], slope); v[3] = lrelu2(v[3], slope);
        *reinterpret_cast<f32x4*>(xl + ulds[i]) = v;
      }
    }
  };

  // ---- A fragment streams: one per m-block of this wave, step index = c8 * K + k
  // (descriptor per m-block from wave-uniform values; step offsets go in the scalar soffset,
  // the stream is padded so no range check is needed)
  rsrc_t ra[TM];
  const int wmu = __builtin_amdgcn_readfirstlane(wm);
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    const int mb = mt * (BM / 32) + wmu * TM + m;
    ra[m] = make_rsrc(a.w + ((size_t)mb * nc * G * K) * 256, 0xFFFFFFFFu);
  }
  const unsigned avoff = (unsigned)lane * 16u;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int m = 0; m < TM; ++m)
#pragma unroll
    for (int n = 0; n < TN; ++n) acc[m][n] = f32x16{};

  const int xrow0 = wn * TN * 32 + l32;  // B: this lane's output column within the tile

  // A ring: ar[0] = current step, ar[1..PD] = in flight
  f32x4 ar[PD + 1][TM], bcur[TN], bnext[TN];
#pragma unroll
  for (int p = 0; p < PD; ++p)
#pragma unroll
    for (int m = 0; m < TM; ++m) ar[p][m] = bload4(ra[m], avoff, (unsigned)p * 1024u);

  // B read of (group g, tap k) for this lane's TN columns; quad = lane half
  auto read_b = [&](const float* xl, int g, int k, f32x4* dst) {
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int r = xrow0 + n * 32 + k * d;
      dst[n] = *reinterpret_cast<const f32x4*>(xl + xlds_off(g, r, half, C::XROWS));
    }
  };

  load_x(0);
  store_x(0);
  __syncthreads();

  for (int c = 0; c < nc; ++c) {
    const int buf = c & 1;
    const float* xl = smem + buf * C::XSZ;
    const bool more = c + 1 < nc;
    if (more) load_x(c + 1);
    read_b(xl, 0, 0, bcur);
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int s = (c * G + g) * K + k;  // global step of this (group, tap)
        // prefetch: A for step s+PD from L2 (the stream is padded), B for step s+1 from LDS
#pragma unroll
        for (int m = 0; m < TM; ++m) ar[PD][m] = bload4(ra[m], avoff, (unsigned)(s + PD) * 1024u);
        const bool bnext_here = (k + 1 < K) || (g + 1 < G);
        if (bnext_here) read_b(xl, (k + 1 < K) ? g : g + 1, (k + 1 < K) ? k + 1 : 0, bnext);
        // keep the prefetches ahead of this step's MFMAs (the scheduler otherwise sinks them
        // to their use and exposes the L2 / LDS latency every step)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int m = 0; m < TM; ++m)
#pragma unroll
            for (int n = 0; n < TN; ++n)
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[0][m][j], bcur[n][j], acc[m][n], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < PD; ++p)
#pragma unroll
          for (int m = 0; m < TM; ++m) ar[p][m] = ar[p + 1][m];
        if (bnext_here) {
#pragma unroll
          for (int n = 0; n < TN; ++n) bcur[n] = bnext[n];
        }
      }
    }
    if (more) store_x(buf ^ 1);
    __syncthreads();
  }

  conv_epilogue<TM, TN>(a, acc, b, t0 + wn * TN * 32, mt * BM + wm * TM * 32, lane);
}

// ---------------------------------------------------------------------------------------
// Polyphase ConvTranspose1d.  Output sample t = U*m + s - P (P = U/2, s = phase) is
//   y[co][t] = b[co] + sum_ci W[ci][co][s] * x[ci][m] + W[ci][co][s+U] * x[ci][m-1]
// (torch: t = i*U - P + k, k in [0, 2U)).  Frames m cover [0, Tin].
// ---------------------------------------------------------------------------------------
template <int U, int BM, int BN, int TM, int TN, int CK>
struct ConvTCfg {
  static constexpr int WM = BM / (32 * TM);
  static constexpr int WN = BN / (32 * TN);
  static constexpr int WSZ = 2 * U * CK * BM;
  static constexpr int W4 = WSZ / 4;
  static constexpr int WPT = (W4 + 255) / 256;
  static constexpr int XW = BN + 1;
  static constexpr int XSZ = CK * XW;
  static constexpr int XPT = (XSZ + 255) / 256;
  static constexpr int BUF = WSZ + ((XSZ + 3) / 4) * 4;
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(CK % 2 == 0, "");
};

template <int U, int BM, int BN, int TM, int TN, int CK>
__global__ __launch_bounds__(256) void convT_mfma_kernel(ConvTArgs a) {
  using C = ConvTCfg<U, BM, BN, TM, TN, CK>;
  __shared__ __attribute__((aligned(16))) float smem[2 * C::BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / C::WN;
  const int wn = wave % C::WN;
  const int half = lane >> 5;
  const int l32 = lane & 31;

  const int m0 = blockIdx.x * BN;
  const int mt = blockIdx.y;
  const int b = blockIdx.z;
  const int Tin = a.Tin;
  const int Tout = U * Tin;

  const float* __restrict__ xb = a.x + (size_t)b * a.Cin * Tin;
  const f32x4* __restrict__ wg = reinterpret_cast<const f32x4*>(a.w) + (size_t)mt * a.n_chunks * C::W4;

  int xoff[C::XPT];
  int xrow[C::XPT];
#pragma unroll
  for (int i = 0; i < C::XPT; ++i) {
    const int e = tid + i * 256;
    const int r = e / C::XW;
    const int col = e - r * C::XW;
    const int ms = m0 - 1 + col;  // source frame
    const bool ok = (e < C::XSZ) && ms >= 0 && ms < Tin;
    xoff[i] = r * Tin + (ok ? ms : 0);
    xrow[i] = ok ? r : 0x40000000;
  }

  f32x4 wreg[C::WPT];
  float xreg[C::XPT];

  auto load_chunk = [&](int c) {
    const f32x4* wc = wg + (size_t)c * C::W4;
#pragma unroll
    for (int i = 0; i < C::WPT; ++i) {
      const int idx = tid + i * 256;
      if ((C::W4 % 256) == 0 || idx < C::W4) wreg[i] = wc[idx];
    }
    const int rows_left = a.Cin - c * CK;
    const float* xc = xb + (size_t)c * CK * Tin;
#pragma unroll
    for (int i = 0; i < C::XPT; ++i) xreg[i] = (xrow[i] < rows_left) ? xc[xoff[i]] : 0.f;
  };

  auto store_chunk = [&](int buf) {
    f32x4* wl = reinterpret_cast<f32x4*>(smem + buf * C::BUF);
#pragma unroll
    for (int i = 0; i < C::WPT; ++i) {
      const int idx = tid + i * 256;
      if ((C::W4 % 256) == 0 || idx < C::W4) wl[idx] = wreg[i];
    }
    float* xl = smem + buf * C::BUF + C::WSZ;
    const float slope = a.in_slope;
#pragma unroll
    for (int i = 0; i < C::XPT; ++i) {
      const int e = tid + i * 256;
      if (e < C::XSZ) xl[e] = lrelu(xreg[i], slope);
    }
  };

  f32x16 acc[U][TM][TN];
#pragma unroll
  for (int s = 0; s < U; ++s)
#pragma unroll
    for (int m = 0; m < TM; ++m)
#pragma unroll
      for (int n = 0; n < TN; ++n) acc[s][m][n] = f32x16{};

  const int wcol = wm * TM * 32 + l32;
  const int xcol = wn * TN * 32 + l32;

  auto compute = [&](int buf) {
    const float* wl = smem + buf * C::BUF;
    const float* xl = wl + C::WSZ;
#pragma unroll
    for (int cp = 0; cp < CK / 2; ++cp) {
      const int ci = 2 * cp + half;
      float b0[TN], b1[TN];
#pragma unroll
      for (int n = 0; n < TN; ++n) {
        b0[n] = xl[ci * C::XW + xcol + n * 32 + 1];  // x[m]
        b1[n] = xl[ci * C::XW + xcol + n * 32];      // x[m-1]
      }
#pragma unroll
      for (int s = 0; s < U; ++s) {
#pragma unroll
        for (int m = 0; m < TM; ++m) {
          const float a0 = wl[(s * CK + ci) * BM + wcol + m * 32];
          const float a1 = wl[((s + U) * CK + ci) * BM + wcol + m * 32];
#pragma unroll
          for (int n = 0; n < TN; ++n) {
            acc[s][m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0[n], acc[s][m][n], 0, 0, 0);
            acc[s][m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1[n], acc[s][m][n], 0, 0, 0);
          }
        }
      }
    }
  };

  const int nc = a.n_chunks;
  load_chunk(0);
  store_chunk(0);
  __syncthreads();
  for (int c = 0; c < nc; ++c) {
    const int buf = c & 1;
    if (c + 1 < nc) load_chunk(c + 1);
    compute(buf);
    if (c + 1 < nc) store_chunk(buf ^ 1);
    __syncthreads();
  }

  const int Cout = a.Cout;
  constexpr int P = U / 2;
  float vmax = 0.f;  // max |stored value| for the fp16 hi/lo consumers (amax_out)
#pragma unroll
  for (int m = 0; m < TM; ++m) {
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int mm = m0 + wn * TN * 32 + n * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = mt * BM + wm * TM * 32 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (co >= Cout || mm > Tin) continue;
        const float bb = a.bias[co];
        const float cc = a.cvec ? a.cvec[(size_t)b * Cout + co] : 0.f;  // XTTS conds[i](g)
        float* yrow = a.y + ((size_t)b * Cout + co) * Tout;
        if constexpr (U == 8) {
          // phases 0..3 -> t = 8mm-4 .. 8mm-1 ; phases 4..7 -> t = 8mm .. 8mm+3
          if (mm >= 1) {
            f32x4 v = {acc[0][m][n][r] + bb + cc, acc[1][m][n][r] + bb + cc, acc[2][m][n][r] + bb + cc,
                       acc[3][m][n][r] + bb + cc};
            vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
            *reinterpret_cast<f32x4*>(yrow + 8 * mm - 4) = v;
          }
          if (mm < Tin) {
            f32x4 v = {acc[4][m][n][r] + bb + cc, acc[5][m][n][r] + bb + cc, acc[6][m][n][r] + bb + cc,
                       acc[7][m][n][r] + bb + cc};
            vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
            *reinterpret_cast<f32x4*>(yrow + 8 * mm) = v;
          }
        } else {
#pragma unroll
          for (int s = 0; s < U; ++s) {
            const int t = U * mm + s - P;
            if (t >= 0 && t < Tout) {
              const float v = acc[s][m][n][r] + bb + cc;
              vmax = fmaxf(vmax, fabsf(v));
              yrow[t] = v;
            }
          }
        }
      }
    }
  }
  if (a.amax_out) publish_amax(a.amax_out, b, vmax);
}

// ---------------------------------------------------------------------------------------
// Tail: y = tanh(b + sum_ci sum_k w[ci][k] * lrelu(z[ci][t+k-3], slope)).
// One workgroup = 1024 samples, 4 consecutive per thread.  The input window streams through LDS
// in chunks of 8 channels, double-buffered: the next chunk's loads are in flight while the
// current one is consumed (the kernel is an HBM read of the Cin-channel plane; one output per
// thread with the whole window staged first left it latency-bound at 1.5 TB/s).
// LDS row j <-> time t0 - 4 + j, so the interior lands 16-B aligned at j = 4 + 4*tid.
// ---------------------------------------------------------------------------------------
constexpr int POST_T = 1024;
constexpr int POST_K = 7;
constexpr int POST_C = 8;
constexpr int POST_W = POST_T + 8;
constexpr int POST_MAXC = 64;

// ZB: z is a bf16 plane (PostArgs::z_b16, the bf16 scheme's activation planes)
template <bool ZB = false>
__global__ __launch_bounds__(256) void conv_post_kernel(PostArgs a) {
  using PZ = PlaneT<ZB>;
  __shared__ __attribute__((aligned(16))) float zs[2][POST_C][POST_W];
  __shared__ float ws[POST_MAXC * POST_K];
  const int Cin = a.Cin;
  const int T = a.T;
  const int tid = threadIdx.x;
  const int t0 = blockIdx.x * POST_T;
  const int b = blockIdx.y;
  const rsrc_t rz = make_rsrc(plane_at<ZB>(a.z, (size_t)b * Cin * T), (unsigned)Cin * (unsigned)T * PZ::ES);
  const float slope = a.in_slope;
  for (int e = tid; e < Cin * POST_K; e += 256) ws[e] = a.w[e];
  // per thread: 4 interior samples t0 + 4*tid + j, and for tid < 6 one halo sample
  const int ti = t0 + 4 * tid;
  const int th = tid < 3 ? t0 - 3 + tid : t0 + POST_T + (tid - 3);  // halo times (tid < 6)
  const int jh = tid < 3 ? 1 + tid : POST_T + 4 + (tid - 3);
  const bool hok = tid < 6 && th >= 0 && th < T;
  const int nch = (Cin + POST_C - 1) / POST_C;
  float xi[POST_C][4], xh[POST_C];
  auto load = [&](int ch) {
#pragma unroll
    for (int c = 0; c < POST_C; ++c) {
      const int ci = ch * POST_C + c;
      const unsigned row = (unsigned)ci * (unsigned)T;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        xi[c][j] = PZ::ld(rz, (ci < Cin && ti + j < T) ? (row + (unsigned)(ti + j)) * PZ::ES : OOB_OFF, 0u);
      xh[c] = PZ::ld(rz, (ci < Cin && hok) ? (row + (unsigned)th) * PZ::ES : OOB_OFF, 0u);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int c = 0; c < POST_C; ++c) {
      f32x4 v = {lrelu(xi[c][0], slope), lrelu(xi[c][1], slope), lrelu(xi[c][2], slope), lrelu(xi[c][3], slope)};
      *reinterpret_cast<f32x4*>(&zs[buf][c][4 + 4 * tid]) = v;
      if (tid < 6) zs[buf][c][jh] = lrelu(xh[c], slope);
    }
  };
  float acc[4] = {a.bias, a.bias, a.bias, a.bias};
  load(0);
  store(0);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nch) load(ch + 1);
#pragma unroll
    for (int c = 0; c < POST_C; ++c) {
      const int ci = ch * POST_C + c;
      if (ci >= Cin) break;
      // outputs t0 + 4*tid + o use rows 1 + 4*tid + o + k, k < 7: rows 4*tid .. 4*tid + 11
      const f32x4 r0 = *reinterpret_cast<const f32x4*>(&zs[buf][c][4 * tid]);
      const f32x4 r1 = *reinterpret_cast<const f32x4*>(&zs[buf][c][4 * tid + 4]);
      const f32x4 r2 = *reinterpret_cast<const f32x4*>(&zs[buf][c][4 * tid + 8]);
      const float row[12] = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3], r2[0], r2[1], r2[2], r2[3]};
#pragma unroll
      for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int k = 0; k < POST_K; ++k) acc[o] = fmaf(ws[ci * POST_K + k], row[1 + o + k], acc[o]);
    }
    if (ch + 1 < nch) store(buf ^ 1);
    __syncthreads();
  }
  const rsrc_t ry = make_rsrc(a.y + (size_t)b * T, (unsigned)T * 4u);
#pragma unroll
  for (int o = 0; o < 4; ++o) bstore(ry, tanhf(acc[o]), ti + o < T ? (unsigned)(ti + o) * 4u : OOB_OFF, 0u);
}

// T % 4 == 0 form (the generator's T = 256 * T'): no LDS window and no barrier in the channel
// loop.  Each lane owns 4 consecutive samples and loads them per channel as one dwordx4; the 3
// samples on either side come from the neighbour lanes (ds_bpermute), lanes 0 and 63 load the
// vector beyond their wave's edge themselves (out-of-range vectors read as the zero padding).
// 8 channels of loads are in flight ahead of the math.  Same FMA order as conv_post_kernel.
constexpr int POST4_C = 8;
template <bool ZB = false>
__global__ __launch_bounds__(256) void conv_post4_kernel(PostArgs a) {
  using PZ = PlaneT<ZB>;
  __shared__ float ws[POST_MAXC * POST_K];
  const int Cin = a.Cin;
  const int T = a.T;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int b = blockIdx.y;
  const int ti = blockIdx.x * POST_T + 4 * tid;
  const rsrc_t rz = make_rsrc(plane_at<ZB>(a.z, (size_t)b * Cin * T), (unsigned)Cin * (unsigned)T * PZ::ES);
  const float slope = a.in_slope;
  for (int e = tid; e < Cin * POST_K; e += 256) ws[e] = a.w[e];
  const bool inb = ti < T;
  const int te = lane == 0 ? ti - 4 : ti + 4;  // wave-edge vector (lanes 0 and 63 only)
  const bool eok = (lane == 0 || lane == 63) && te >= 0 && te < T;
  const int nb = (Cin + POST4_C - 1) / POST4_C;
  f32x4 cm[POST4_C], ce[POST4_C], nm[POST4_C], ne[POST4_C];
  auto load = [&](f32x4 (&m)[POST4_C], f32x4 (&e)[POST4_C], int cb) {
#pragma unroll
    for (int c = 0; c < POST4_C; ++c) {
      const int ci = cb * POST4_C + c;
      const unsigned row = (unsigned)ci * (unsigned)T;
      m[c] = pload4<ZB>(rz, (ci < Cin && inb) ? (row + (unsigned)ti) * PZ::ES : OOB_OFF, 0u);
      e[c] = pload4<ZB>(rz, (ci < Cin && eok) ? (row + (unsigned)te) * PZ::ES : OOB_OFF, 0u);
    }
  };
  load(cm, ce, 0);
  __syncthreads();  // ws
  float acc[4] = {a.bias, a.bias, a.bias, a.bias};
  for (int cb = 0; cb < nb; ++cb) {
    if (cb + 1 < nb) load(nm, ne, cb + 1);
#pragma unroll
    for (int c = 0; c < POST4_C; ++c) {
      const int ci = cb * POST4_C + c;
      if (ci >= Cin) break;
      float m[4], e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        m[j] = lrelu(cm[c][j], slope);
        e[j] = lrelu(ce[c][j], slope);
      }
      float row[12];  // times ti - 4 .. ti + 7 (row[0] and row[11] unused)
      row[0] = row[11] = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float l = __shfl(m[1 + j], lane - 1);
        const float r = __shfl(m[j], lane + 1);
        row[1 + j] = lane == 0 ? e[1 + j] : l;
        row[8 + j] = lane == 63 ? e[j] : r;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) row[4 + j] = m[j];
#pragma unroll
      for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int k = 0; k < POST_K; ++k) acc[o] = fmaf(ws[ci * POST_K + k], row[1 + o + k], acc[o]);
    }
#pragma unroll
    for (int c = 0; c < POST4_C; ++c) {
      cm[c] = nm[c];
      ce[c] = ne[c];
    }
  }
  const rsrc_t ry = make_rsrc(a.y + (size_t)b * T, (unsigned)T * 4u);
  const f32x4 yv = {tanhf(acc[0]), tanhf(acc[1]), tanhf(acc[2]), tanhf(acc[3])};
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, yv), ry, inb ? (int)((unsigned)ti * 4u) : (int)OOB_OFF, 0, 0);
}

// cvec[b][co] = bc[co] + sum_k Wc[co][k] * g[b][k] (the cond_layer GEMVs, hifigan_generator.py:228,
// wavenet.py:98-99): one wave per output row, its lanes across k (coalesced row reads, the row
// held in registers for every batch item), a butterfly sum per item.  A tile-through-LDS form
// (32 dependent load rounds per 32 columns) took 150 us per call at 1536 x 256.
__global__ __launch_bounds__(256) void cond_vec_kernel(const float* g, const float* Wc, const float* bc,
                                                     float* cvec, int B, int Cc, int C0) {
  const int lane = threadIdx.x & 63;
  const int co = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (co >= C0) return;  // wave-uniform
  const float* w = Wc + (size_t)co * Cc;
  constexpr int KR = 8;  // up to 512 input channels in registers, the rest streamed
  float wr[KR];
#pragma unroll
  for (int i = 0; i < KR; ++i) {
    const int k = lane + 64 * i;
    wr[i] = k < Cc ? w[k] : 0.f;
  }
  const float bias = bc[co];
  for (int b = 0; b < B; ++b) {
    const float* gb = g + (size_t)b * Cc;
    float p = 0.f;
#pragma unroll
    for (int i = 0; i < KR; ++i) {
      const int k = lane + 64 * i;
      if (k < Cc) p = fmaf(wr[i], gb[k], p);
    }
    for (int k = 64 * KR + lane; k < Cc; k += 64) p = fmaf(w[k], gb[k], p);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
    if (lane == 0) cvec[(size_t)b * C0 + co] = p + bias;
  }
}

// ---------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------
namespace {
// {BM, BN, TM, TN, CK = 8*G, PD}.  Tiles 0-2 are the defaults picked by conv1d_tile_for;
// the rest are tuning candidates (scripts/tune_conv.py), narrow halo only.
constexpr ConvTile kConvTiles[] = {
    {128, 128, 2, 2, 16, 1},  // 0  Cout > 64
    {64, 256, 2, 2, 16, 1},   // 1  32 < Cout <= 64
    {32, 512, 1, 4, 8, 1},    // 2  Cout <= 32
    {128, 128, 2, 2, 32, 1},  // 3
    {128, 128, 2, 2, 16, 2},  // 4
    {128, 256, 2, 4, 16, 1},  // 5
    {64, 256, 2, 2, 32, 1},   // 6
    {64, 512, 2, 4, 16, 1},   // 7
    {32, 256, 1, 2, 16, 1},   // 8
    {32, 512, 1, 4, 16, 1},   // 9
    {64, 128, 2, 1, 16, 1},   // 10
    {128, 128, 2, 2, 32, 2},  // 11
    {64, 256, 2, 2, 16, 2},   // 12
    {32, 256, 1, 2, 32, 1},   // 13
};
constexpr int kNumConvTiles = sizeof(kConvTiles) / sizeof(kConvTiles[0]);

template <int K, int BM, int BN, int TM, int TN, int G, int PD, bool WIDE>
void launch_conv1d_t(const Conv1dArgs& a, int B, hipStream_t s) {
  dim3 grid(ceil_div(a.Tout, BN), ceil_div(a.Cout, BM), B);
  const int halo = (K - 1) * a.dil;
  if (halo <= (K - 1) * DMAX) {
    hipLaunchKernelGGL((conv1d_mfma_kernel<K, BM, BN, TM, TN, G, (K - 1) * DMAX, PD>), grid, dim3(256), 0, s, a);
  } else if (WIDE && halo <= HALO_WIDE) {
    hipLaunchKernelGGL((conv1d_mfma_kernel<K, BM, BN, TM, TN, G, WIDE ? HALO_WIDE : 0, PD>), grid, dim3(256), 0, s,
                       a);
  } else {
    throw Error(3, "conv1d: (kernel_size-1)*dilation = " + std::to_string(halo) + " exceeds " +
                       std::to_string(WIDE ? HALO_WIDE : (K - 1) * DMAX) + " for this tile");
  }
}

template <int K>
void launch_conv1d_k(const Conv1dArgs& a, int B, int tile, hipStream_t s) {
  switch (tile) {
    case 0: launch_conv1d_t<K, 128, 128, 2, 2, 2, 1, true>(a, B, s); break;
    case 1: launch_conv1d_t<K, 64, 256, 2, 2, 2, 1, true>(a, B, s); break;
    case 2: launch_conv1d_t<K, 32, 512, 1, 4, 1, 1, true>(a, B, s); break;
    case 3: launch_conv1d_t<K, 128, 128, 2, 2, 4, 1, false>(a, B, s); break;
    case 4: launch_conv1d_t<K, 128, 128, 2, 2, 2, 2, false>(a, B, s); break;
    case 8: launch_conv1d_t<K, 32, 256, 1, 2, 2, 1, false>(a, B, s); break;
    case 10: launch_conv1d_t<K, 64, 128, 2, 1, 2, 1, false>(a, B, s); break;
    case 11: launch_conv1d_t<K, 128, 128, 2, 2, 4, 2, false>(a, B, s); break;
#ifdef TTS_TUNING_TILES  // candidates that never won the round-1 sweep (scripts/tune_conv.py)
    case 5: launch_conv1d_t<K, 128, 256, 2, 4, 2, 1, false>(a, B, s); break;
    case 6: launch_conv1d_t<K, 64, 256, 2, 2, 4, 1, false>(a, B, s); break;
    case 7: launch_conv1d_t<K, 64, 512, 2, 4, 2, 1, false>(a, B, s); break;
    case 9: launch_conv1d_t<K, 32, 512, 1, 4, 2, 1, false>(a, B, s); break;
    case 12: launch_conv1d_t<K, 64, 256, 2, 2, 2, 2, false>(a, B, s); break;
    case 13: launch_conv1d_t<K, 32, 256, 1, 2, 4, 1, false>(a, B, s); break;
#endif
    default: throw Error(3, "conv1d: bad tile index " + std::to_string(tile));
  }
}

// convT tiles: index by (U, Cout class)
template <int U>
struct ConvTTiles;
template <>
struct ConvTTiles<8> {
  static constexpr ConvTile t[] = {{64, 64, 1, 1, 8}, {32, 128, 1, 1, 8}};
};
template <>
struct ConvTTiles<4> {
  static constexpr ConvTile t[] = {{64, 128, 1, 2, 8}, {32, 256, 1, 2, 8}};
};
template <>
struct ConvTTiles<2> {
  static constexpr ConvTile t[] = {{64, 256, 2, 2, 8}, {32, 512, 1, 4, 8}};
};

template <int U, int BM, int BN, int TM, int TN, int CK>
void launch_convT_t(const ConvTArgs& a, int B, hipStream_t s) {
  dim3 grid(ceil_div(a.Tin + 1, BN), ceil_div(a.Cout, BM), B);
  hipLaunchKernelGGL((convT_mfma_kernel<U, BM, BN, TM, TN, CK>), grid, dim3(256), 0, s, a);
}
}  // namespace

// Tile choice per conv shape, from the round-1 sweep on MI355X (profiles/r01_tune_conv.log,
// HiFiGAN-v1 shapes at B=32 x 1034 frames).  `res`: the epilogue adds a residual.
int conv1d_tile_for(int Cout, int K, int Cin, int dil, bool res) {
  (void)res;
  if ((K - 1) * dil > (K - 1) * DMAX) return Cout > 64 ? 0 : (Cout > 32 ? 1 : 2);  // wide-halo tiles
  if (Cout > 64) {
    if (Cin % 32 != 0) return K <= 3 ? 4 : 0;  // conv_pre (Cin 80), Glow start
    return (K >= 11 && Cout <= 128) ? 3 : 11;
  }
  if (Cout > 32) return 10;
  return K >= 11 ? 2 : 8;
}

ConvTile conv1d_tile(int idx) {
  TTS_REQUIRE(idx >= 0 && idx < kNumConvTiles, 3, "conv1d: bad tile index");
  return kConvTiles[idx];
}

int conv1d_num_tiles() { return kNumConvTiles; }

void launch_conv1d(const Conv1dArgs& a, int B, int K, int tile, hipStream_t s) {
  // every addressed plane must stay below 2 GiB (32-bit buffer offsets, OOB marker bit 31)
  TTS_REQUIRE((int64_t)a.Cin * a.Tin * 4 < (int64_t(1) << 31) && (int64_t)a.Cout * a.Tout * 4 < (int64_t(1) << 31), 3,
              "conv1d: a batch item's channel plane exceeds 2 GiB");
  switch (K) {
    case 1: launch_conv1d_k<1>(a, B, tile, s); break;
    case 3: launch_conv1d_k<3>(a, B, tile, s); break;
    case 5: launch_conv1d_k<5>(a, B, tile, s); break;
    case 7: launch_conv1d_k<7>(a, B, tile, s); break;
    case 11: launch_conv1d_k<11>(a, B, tile, s); break;
    default: throw Error(3, "conv1d: kernel size " + std::to_string(K) + " not supported (1,3,5,7,11)");
  }
  TTS_HIP_CHECK(hipGetLastError());
}

int convT_tile_for(int Cout, int /*U*/) { return Cout > 32 ? 0 : 1; }

ConvTile convT_tile(int idx, int U) {
  TTS_REQUIRE(idx == 0 || idx == 1, 3, "convT: bad tile index");
  switch (U) {
    case 8: return ConvTTiles<8>::t[idx];
    case 4: return ConvTTiles<4>::t[idx];
    case 2: return ConvTTiles<2>::t[idx];
    default: throw Error(3, "ConvTranspose1d stride " + std::to_string(U) + " not supported (2,4,8)");
  }
}

void launch_convT(const ConvTArgs& a, int B, int U, int tile, hipStream_t s) {
  switch (U) {
    case 8:
      if (tile == 0) launch_convT_t<8, 64, 64, 1, 1, 8>(a, B, s);
      else launch_convT_t<8, 32, 128, 1, 1, 8>(a, B, s);
      break;
    case 4:
      if (tile == 0) launch_convT_t<4, 64, 128, 1, 2, 8>(a, B, s);
      else launch_convT_t<4, 32, 256, 1, 2, 8>(a, B, s);
      break;
    case 2:
      if (tile == 0) launch_convT_t<2, 64, 256, 2, 2, 8>(a, B, s);
      else launch_convT_t<2, 32, 512, 1, 4, 8>(a, B, s);
      break;
    default: throw Error(3, "ConvTranspose1d stride " + std::to_string(U) + " not supported (2,4,8)");
  }
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_conv_post(const PostArgs& a, int B, hipStream_t s) {
  TTS_REQUIRE(a.Cin >= 1 && a.Cin <= POST_MAXC, 3, "conv_post: more than 64 input channels");
  TTS_REQUIRE((int64_t)a.Cin * a.T * 4 < (int64_t(1) << 31), 3, "conv_post: channel plane exceeds 2 GiB");
  dim3 grid(ceil_div(a.T, POST_T), B);
  // the vector form needs 16-byte aligned rows (T % 4 == 0) and plane bases
  const bool vec = a.T % 4 == 0 && ((uintptr_t)a.z & 15) == 0 && ((uintptr_t)a.y & 15) == 0;
  if (a.z_b16) {
    if (vec) hipLaunchKernelGGL(conv_post4_kernel<true>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(conv_post_kernel<true>, grid, dim3(256), 0, s, a);
  } else {
    if (vec) hipLaunchKernelGGL(conv_post4_kernel<false>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(conv_post_kernel<false>, grid, dim3(256), 0, s, a);
  }
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_cond_vec(const float* g, const float* Wc, const float* bc, float* cvec, int B, int Cc,
                     int C0, hipStream_t s) {
  hipLaunchKernelGGL(cond_vec_kernel, dim3(ceil_div(C0, 4)), dim3(256), 0, s, g, Wc, bc, cvec, B, Cc, C0);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
