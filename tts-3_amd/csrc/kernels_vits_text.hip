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

// the [C][64] LDS staging passes the 64 KiB default dynamic-LDS limit above 255 channels: raise the
// function's limit once (to the 512-channel maximum vits_sdp_validate accepts, 128 KiB + 1 KiB static)
template <bool DW>
void dds_lds_limit(int C) {
  if (sizeof(float) * C * kColTile <= 64 * 1024) return;
  static const bool raised = [] {
    TTS_HIP_CHECK(hipFuncSetAttribute((const void*)dds_ln_gelu_kernel<DW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)(sizeof(float) * 512 * kColTile)));
    return true;
  }();
  (void)raised;
}

void launch_dds_sep_ln_gelu(const float* x, const float* mask, const float* w, const float* bias, const float* gamma,
                            const float* beta, float* out, int B, int C, int T, int k, int d, hipStream_t s) {
  TTS_REQUIRE(C >= 1 && C <= 512 && B >= 1 && B <= 65535 && T >= 1, 1, "dds: bad shape");
  dds_lds_limit<true>(C);
  dim3 grid(ceil_div(T, kColTile), B);
  hipLaunchKernelGGL(dds_ln_gelu_kernel<true>, grid, dim3(256), sizeof(float) * C * kColTile, s, nullptr,
                     const_cast<float*>(x), mask, w, bias, gamma, beta, out, C, T, k, d);
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_dds_ln_gelu_add(const float* a, float* x, const float* gamma, const float* beta, int B, int C, int T,
                            hipStream_t s) {
  TTS_REQUIRE(C >= 1 && C <= 512 && B >= 1 && B <= 65535 && T >= 1, 1, "dds: bad shape");
  dds_lds_limit<false>(C);
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

// ---------------------------------------------------------------------------------------
// Vits.inference glue (vits.py:1119-1161) that ran on ATen before round 6
// ---------------------------------------------------------------------------------------
// w = durations.unsqueeze(0); w_ceil = ceil(w); y_lengths = clamp_min(sum(w_ceil), 1) (:1141-1146):
// dur [T] shared by every utterance (dur_bstride 0) or [B][T]; no x_mask, no length_scale
__global__ void __launch_bounds__(256) given_durations_kernel(const float* __restrict__ dur, int64_t dur_bstride,
                                                              float* __restrict__ w_ceil, int64_t* __restrict__ y_len,
                                                              int T) {
  __shared__ float part[4];
  const int b = blockIdx.x;
  float s = 0.f;
  for (int t = threadIdx.x; t < T; t += 256) {
    const float wc = ceilf(dur[(size_t)b * dur_bstride + t]);
    w_ceil[(size_t)b * T + t] = wc;
    s += wc;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) y_len[b] = (int64_t)fmaxf((part[0] + part[1]) + (part[2] + part[3]), 1.f);
}

void launch_given_durations(const float* dur, int64_t dur_bstride, float* w_ceil, int64_t* y_len, int B, int T,
                            hipStream_t s) {
  hipLaunchKernelGGL(given_durations_kernel, dim3(B), dim3(256), 0, s, dur, dur_bstride, w_ceil, y_len, T);
  TTS_HIP_CHECK(hipGetLastError());
}

// out[b][c][t] = z[b][c][t] * y_mask[b][t] for t < T_out <= T: (z * y_mask)[:, :, :max_inference_len]
// (:1161); z may carry a batch stride other than C * T
__global__ void __launch_bounds__(256) mask_slice_kernel(const float* __restrict__ z, const float* __restrict__ m,
                                                         float* __restrict__ out, int C, int T, int T_out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y, b = blockIdx.z;
  if (t >= T_out) return;
  out[((size_t)b * C + c) * T_out + t] = z[((size_t)b * C + c) * T + t] * m[(size_t)b * T + t];
}

void launch_mask_slice(const float* z, const float* m, float* out, int B, int C, int T, int T_out, hipStream_t s) {
  TTS_REQUIRE(B >= 1 && B <= 65535 && C >= 1 && C <= 65535 && T_out >= 1 && T_out <= T, 1, "mask_slice: bad shape");
  hipLaunchKernelGGL(mask_slice_kernel, dim3(ceil_div(T_out, 256), C, B), dim3(256), 0, s, z, m, out, C, T, T_out);
  TTS_HIP_CHECK(hipGetLastError());
}

// upsampling_z (vits.py:944-959): z2 = F.interpolate(z, scale_factor=[f], mode="linear") (align_corners
// False, output length floor(T f)); y_mask2 = sequence_mask(y_lengths * f) with the float lengths
// (fp32, as the long * python-float product is).  The source coordinate follows ATen's
// upsample_linear1d: src = max(inv * (dst + 0.5) - 0.5, 0) with inv = (float)(1.0 / f), i0 = min(floor(src), T - 1),
// i1 = i0 + (i0 < T - 1), l1 = src - i0, l0 = 1 - l1, z2 = l0 z[i0] + l1 z[i1]
__global__ void __launch_bounds__(256) upsample_z_kernel(const float* __restrict__ z, const int64_t* __restrict__ ylen,
                                                         float* __restrict__ z2, float* __restrict__ m2, int C, int T,
                                                         int T2, float inv, float f) {
  const int t2 = blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y, b = blockIdx.z;
  if (t2 >= T2) return;
  float src = __fadd_rn(__fmul_rn(inv, (float)t2 + 0.5f), -0.5f);  // two roundings, as ATen (no fma)
  src = src < 0.f ? 0.f : src;
  const int i0 = min((int)floorf(src), T - 1);
  const int i1 = i0 + (i0 < T - 1 ? 1 : 0);
  const float l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  const float l0 = 1.f - l1;
  const float* zr = z + ((size_t)b * C + c) * T;
  z2[((size_t)b * C + c) * T2 + t2] = l0 * zr[i0] + l1 * zr[i1];
  if (c == 0 && m2) m2[(size_t)b * T2 + t2] = (float)t2 < (float)ylen[b] * f ? 1.f : 0.f;
}

void launch_upsample_z(const float* z, const int64_t* y_len, float* z2, float* m2, int B, int C, int T, int T2,
                       double factor, hipStream_t s) {
  TTS_REQUIRE(B >= 1 && B <= 65535 && C >= 1 && C <= 65535 && T >= 1 && T2 >= 1 && factor > 0.0, 1,
              "upsample_z: bad shape");
  const float inv = (float)(1.0 / factor);
  hipLaunchKernelGGL(upsample_z_kernel, dim3(ceil_div(T2, 256), C, B), dim3(256), 0, s, z, y_len, z2, m2, C, T, T2,
                     inv, (float)factor);
  TTS_HIP_CHECK(hipGetLastError());
}

// out[b][:] = table[clamp(ids[b], 0, num - 1)][:] (nn.Embedding rows: emb_g(sid), emb_l(lid), vits.py:1117,
// :1124; the reference raises IndexError on an out-of-range id, a device kernel cannot, so it clamps)
__global__ void __launch_bounds__(256) embedding_rows_kernel(const float* __restrict__ table,
                                                             const int64_t* __restrict__ ids, float* __restrict__ out,
                                                             int dim, int num, int64_t id_stride) {
  const int b = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= dim) return;
  int64_t id = ids[(size_t)b * id_stride];
  id = id < 0 ? 0 : (id >= num ? num - 1 : id);
  out[(size_t)b * dim + c] = table[(size_t)id * dim + c];
}

void launch_embedding_rows(const float* table, const int64_t* ids, int64_t id_stride, float* out, int B, int dim,
                           int num, hipStream_t s) {
  TTS_REQUIRE(B >= 1 && B <= 65535 && dim >= 1 && num >= 1, 1, "embedding_rows: bad shape");
  hipLaunchKernelGGL(embedding_rows_kernel, dim3(ceil_div(dim, 256), B), dim3(256), 0, s, table, ids, out, dim, num,
                     id_stride);
  TTS_HIP_CHECK(hipGetLastError());
}

// out[b] = d[b] / max(||d[b]||_2, 1e-12) (F.normalize, the d-vector path of _set_cond_input, :884-886):
// one workgroup per row, the squares summed in fp32
__global__ void __launch_bounds__(256) l2_normalize_kernel(const float* __restrict__ d, float* __restrict__ out, int C) {
  __shared__ float part[4];
  const int b = blockIdx.x;
  const float* r = d + (size_t)b * C;
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) s = fmaf(r[c], r[c], s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  const float nrm = fmaxf(sqrtf((part[0] + part[1]) + (part[2] + part[3])), 1e-12f);
  for (int c = threadIdx.x; c < C; c += 256) out[(size_t)b * C + c] = r[c] / nrm;
}

void launch_l2_normalize(const float* d, float* out, int B, int C, hipStream_t s) {
  TTS_REQUIRE(B >= 1 && C >= 1, 1, "l2_normalize: bad shape");
  hipLaunchKernelGGL(l2_normalize_kernel, dim3(B), dim3(256), 0, s, d, out, C);
  TTS_HIP_CHECK(hipGetLastError());
}

// y[b][c][t] = ((x[b][c][t] + v1[b][c]) + v2[b][c]) * mask[b][t] (v1 / v2 may be NULL): the
// deterministic duration predictor's input, x + cond(g) + cond_lang(lang_emb), masked by conv_1's
// x * x_mask (glow_tts/duration_predictor.py:56-64)
__global__ void __launch_bounds__(256) add_vec_mask_kernel(const float* __restrict__ x, const float* __restrict__ v1,
                                                           const float* __restrict__ v2, const float* __restrict__ m,
                                                           float* __restrict__ y, int C, int T) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y, b = blockIdx.z;
  if (t >= T) return;
  float v = x[((size_t)b * C + c) * T + t];
  if (v1) v = v + v1[(size_t)b * C + c];
  if (v2) v = v + v2[(size_t)b * C + c];
  y[((size_t)b * C + c) * T + t] = v * m[(size_t)b * T + t];
}

void launch_add_vec_mask(const float* x, const float* v1, const float* v2, const float* m, float* y, int B, int C,
                         int T, hipStream_t s) {
  TTS_REQUIRE(B >= 1 && B <= 65535 && C >= 1 && C <= 65535 && T >= 1, 1, "add_vec_mask: bad shape");
  hipLaunchKernelGGL(add_vec_mask_kernel, dim3(ceil_div(T, 256), C, B), dim3(256), 0, s, x, v1, v2, m, y, C, T);
  TTS_HIP_CHECK(hipGetLastError());
}

// out = a + b elementwise (n floats): the SDP's cond(g) + cond_lang(lang_emb) per-utterance vector
__global__ void __launch_bounds__(256) vec_add_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                      float* __restrict__ out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

void launch_vec_add(const float* a, const float* b, float* out, int n, hipStream_t s) {
  hipLaunchKernelGGL(vec_add_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, a, b, out, n);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
