// VITS text side: the StochasticDurationPredictor's elementwise / normalisation kernels (its 1x1
// convs run on the conv kernels).  Reference: TTS/tts/layers/vits/stochastic_duration_predictor.py
// (DilatedDepthSeparableConv :11-63, ElementwiseAffine :66-83, ConvFlow :86-148, reverse chain
// :273-282) and TTS/tts/layers/vits/transforms.py (the rational-quadratic spline, :12-198).
//
// The SDP state z is [B][2][T]; flips (torch.flip(z, [1]), :279) are not materialised: the host
// tracks the parity p (logical channel c lives in physical channel c ^ p).
#include <cmath>

#include "text.hpp"

namespace tts {

namespace {
constexpr int kColTile = 64;  // columns per workgroup of the channel-normalising kernels

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
}  // namespace

// ---------------------------------------------------------------------------------------
// v = DW ? sep_conv(x * mask) (depthwise, k taps, dilation d, zero padding d(k-1)/2) : a;
// u = gelu(LayerNorm2_C(v) * gamma + beta)           (stochastic_duration_predictor.py:55-60)
// DW: out = u;  else: x += u (the residual x = x + y, :62)
// One workgroup = 64 columns of one utterance, all C channels (staged in LDS for the statistics).
// ---------------------------------------------------------------------------------------
template <bool DW>
__global__ void __launch_bounds__(256) dds_ln_gelu_kernel(const float* __restrict__ a, float* x,
                                                          const float* __restrict__ mask,
                                                          const float* __restrict__ wdw,
                                                          const float* __restrict__ bdw,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* out, int C, int T,
                                                          int k, int d) {
  extern __shared__ float v[];  // [C][64]
  __shared__ float red[4][kColTile];
  const int col = threadIdx.x & 63, cg = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int t = blockIdx.x * kColTile + col;
  const bool ok = t < T;
  const float* mb = mask + (size_t)b * T;
  float s = 0.f;
  for (int c = cg; c < C; c += 4) {
    float val = 0.f;
    if (ok) {
      if constexpr (DW) {
        const float* xr = x + ((size_t)b * C + c) * T;
        const int h = d * (k - 1) / 2;
        float acc = bdw[c];
        for (int j = 0; j < k; ++j) {
          const int tt = t - h + j * d;
          if (tt >= 0 && tt < T) acc = fmaf(wdw[c * k + j], xr[tt] * mb[tt], acc);
        }
        val = acc;
      } else {
        val = a[((size_t)b * C + c) * T + t];
      }
    }
    v[c * kColTile + col] = val;
    s += val;
  }
  red[cg][col] = s;
  __syncthreads();
  const float mean = (red[0][col] + red[1][col] + red[2][col] + red[3][col]) / (float)C;
  __syncthreads();
  float q = 0.f;
  for (int c = cg; c < C; c += 4) {
    const float dv = v[c * kColTile + col] - mean;
    q = fmaf(dv, dv, q);
  }
  red[cg][col] = q;
  __syncthreads();
  const float var = (red[0][col] + red[1][col] + red[2][col] + red[3][col]) / (float)C;
  const float rstd = 1.f / sqrtf(var + 1e-5f);
  if (!ok) return;
  for (int c = cg; c < C; c += 4) {
    const float u = gelu_erf((v[c * kColTile + col] - mean) * rstd * gamma[c] + beta[c]);
    const size_t o = ((size_t)b * C + c) * T + t;
    if constexpr (DW) out[o] = u;
    else x[o] += u;
  }
}

void launch_dds_sep_ln_gelu(const float* x, const float* mask, const float* w, const float* bias, const float* gamma,
                            const float* beta, float* out, int B, int C, int T, int k, int d, hipStream_t s) {
  TTS_REQUIRE(C >= 1 && C <= 512 && B >= 1 && B <= 65535 && T >= 1, 1, "dds: bad shape");
  dim3 grid(ceil_div(T, kColTile), B);
  hipLaunchKernelGGL(dds_ln_gelu_kernel<true>, grid, dim3(256), sizeof(float) * C * kColTile, s, nullptr,
                     const_cast<float*>(x), mask, w, bias, gamma, beta, out, C, T, k, d);
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_dds_ln_gelu_add(const float* a, float* x, const float* gamma, const float* beta, int B, int C, int T,
                            hipStream_t s) {
  TTS_REQUIRE(C >= 1 && C <= 512 && B >= 1 && B <= 65535 && T >= 1, 1, "dds: bad shape");
  dim3 grid(ceil_div(T, kColTile), B);
  hipLaunchKernelGGL(dds_ln_gelu_kernel<false>, grid, dim3(256), sizeof(float) * C * kColTile, s, a, x, nullptr,
                     nullptr, nullptr, gamma, beta, nullptr, C, T, 0, 0);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// z = noise * noise_scale (:277), or the ElementwiseAffine reverse (:81-83) on both logical
// channels c: z[c ^ p] = (z[c ^ p] - t[c]) * exp(-log_scale[c]) * mask; logw (if not NULL) =
// the result's logical channel 0 (:281-282).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) sdp_init_kernel(const float* __restrict__ noise, float* __restrict__ z, float ns,
                                                       int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) z[i] = noise ? noise[i] * ns : 0.f;
}

__global__ void __launch_bounds__(256) sdp_affine_kernel(float* __restrict__ z, const float* __restrict__ tr,
                                                         const float* __restrict__ ls, const float* __restrict__ mask,
                                                         float* __restrict__ logw, int T, int p) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (t >= T) return;
  const float m = mask[(size_t)b * T + t];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    float* zp = z + ((size_t)b * 2 + (c ^ p)) * T + t;
    const float r = (*zp - tr[c]) * expf(-ls[c]) * m;
    *zp = r;
    if (c == 0 && logw) logw[(size_t)b * T + t] = r;
  }
}

void launch_sdp_init(const float* noise, float* z, float noise_scale, int B, int T, hipStream_t s) {
  const int n = B * 2 * T;
  hipLaunchKernelGGL(sdp_init_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, noise, z, noise_scale, n);
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_sdp_affine(float* z, const float* tr, const float* ls, const float* mask, float* logw, int B, int T, int p,
                       hipStream_t s) {
  hipLaunchKernelGGL(sdp_affine_kernel, dim3(ceil_div(T, 256), B), dim3(256), 0, s, z, tr, ls, mask, logw, T, p);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// ConvFlow tail, reverse (:135-148): h [B][3nb-1][T] (proj(h) * mask); per position the
// unconstrained rational-quadratic spline, inverse, tails "linear" (transforms.py:50-94, :97-160)
// on x1 = logical channel 1; then z = cat(x0, x1) * mask.  One thread per position, fp32.
// ---------------------------------------------------------------------------------------
constexpr int kSplineMaxBins = 16;

__global__ void __launch_bounds__(256) sdp_spline_kernel(const float* __restrict__ h, float* __restrict__ z,
                                                         const float* __restrict__ mask, int T, int p, int nb,
                                                         float tail, float hscale) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (t >= T) return;
  constexpr float kMinW = 1e-3f, kMinH = 1e-3f, kMinD = 1e-3f;  // transforms.py:7-9
  const int nh = 3 * nb - 1;
  const float* hb = h + (size_t)b * nh * T + t;
  float* z0 = z + ((size_t)b * 2 + p) * T + t;
  float* z1 = z + ((size_t)b * 2 + (1 ^ p)) * T + t;
  const float m = mask[(size_t)b * T + t];
  float x = *z1;
  if (x >= -tail && x <= tail) {
    const float left = -tail, right = tail;
    float cw[kSplineMaxBins + 1], ch[kSplineMaxBins + 1], dv[kSplineMaxBins + 1];
    // widths / heights: softmax over the bins (max-subtracted), min width, cumsum, pinned ends
    auto edges = [&](int off, float minv, float* cum) {
      float mx = -INFINITY;
      for (int i = 0; i < nb; ++i) mx = fmaxf(mx, hb[(size_t)(off + i) * T] * hscale);
      float e[kSplineMaxBins], sum = 0.f;
      for (int i = 0; i < nb; ++i) {
        e[i] = expf(hb[(size_t)(off + i) * T] * hscale - mx);
        sum += e[i];
      }
      float run = 0.f;
      cum[0] = left;
      for (int i = 0; i < nb; ++i) {
        run += minv + (1.f - minv * nb) * (e[i] / sum);
        cum[i + 1] = (right - left) * run + left;
      }
      cum[nb] = right;
    };
    edges(0, kMinW, cw);
    edges(nb, kMinH, ch);
    // derivatives: the linear-tail constant at both ends, softplus inside (F.softplus threshold 20)
    const float cst = logf(expf(1.f - kMinD) - 1.f);
    for (int i = 0; i <= nb; ++i) {
      const float u = (i == 0 || i == nb) ? cst : hb[(size_t)(2 * nb + i - 1) * T];
      dv[i] = kMinD + (u > 20.f ? u : log1pf(expf(u)));
    }
    // bin: searchsorted on the cumulative heights with eps on the last edge (transforms.py:45-47)
    int idx = -1;
    for (int i = 0; i <= nb; ++i) idx += (x >= (i == nb ? ch[i] + 1e-6f : ch[i])) ? 1 : 0;
    const float icw = cw[idx], ibw = cw[idx + 1] - cw[idx];
    const float ich = ch[idx], ih = ch[idx + 1] - ch[idx];
    const float idl = ih / ibw;
    const float d0 = dv[idx], d1 = dv[idx + 1];
    const float dx = x - ich;
    const float s = d0 + d1 - 2.f * idl;
    const float qa = dx * s + ih * (idl - d0);
    const float qb = ih * d0 - dx * s;
    const float qc = -idl * dx;
    const float disc = qb * qb - 4.f * qa * qc;
    const float root = (2.f * qc) / (-qb - sqrtf(disc));
    x = root * ibw + icw;
  }
  *z1 = x * m;
  *z0 = *z0 * m;
}

void launch_sdp_spline(const float* h, float* z, const float* mask, int B, int T, int p, int nb, float tail,
                       float hscale, hipStream_t s) {
  TTS_REQUIRE(nb >= 1 && nb <= kSplineMaxBins, 3, "spline: num_bins must be 1..16");
  hipLaunchKernelGGL(sdp_spline_kernel, dim3(ceil_div(T, 256), B), dim3(256), 0, s, h, z, mask, T, p, nb, tail,
                     hscale);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
