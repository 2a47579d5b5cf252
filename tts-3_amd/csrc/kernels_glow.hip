// Elementwise kernels of the reverse Glow-TTS decoder flow (gfx950).
//   squeeze / unsqueeze      decoder.py:8-47
//   gate                     wavenet.py:6-13 (fused_add_tanh_sigmoid_multiply, g = 0)
//   wn_update                wavenet.py:109-115 (residual/skip split of res_skip_layers)
//   tail                     glow.py:222-224 (coupling affine inverse) -> glow.py:102-137
//                            (InvConvNear inverse) -> normalization.py:96-98 (ActNorm inverse),
//                            fused: one thread owns the S channels InvConvNear mixes.
//   forward direction (reverse=False, decoder.py:119-133): head = ActNorm -> InvConvNear of one
//   flow block (normalization.py:99-100, glow.py:126-135); couple_fwd = the coupling affine
//   (glow.py:225-227) fused with the next block's head; the logdet terms sum per utterance in
//   fixed order (partials per workgroup, then glow_logdet_kernel).
#include "glow.hpp"
#include "conv_device.hpp"

namespace tts {

// xs[b][s*C + c][t'] = x[b][c][nsq*t' + s] * msq[t'],  msq[t'] = mask[b][nsq*t' + nsq - 1]
__global__ __launch_bounds__(256) void glow_squeeze_kernel(const float* x, const float* mask, float* xs,
                                                           float* msq, int C, int T, int nsq) {
  const int Th = T / nsq;
  const int b = blockIdx.y;
  const int64_t n = (int64_t)C * nsq * Th;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int tq = (int)(i % Th);
    const int ch = (int)(i / Th);
    const int sidx = ch / C, c = ch - sidx * C;
    const float m = mask[(size_t)b * T + (size_t)nsq * tq + nsq - 1];
    xs[(size_t)b * n + i] = x[((size_t)b * C + c) * T + (size_t)nsq * tq + sidx] * m;
    if (ch == 0) msq[(size_t)b * Th + tq] = m;
  }
}

// y[b][c][nsq*t' + s] = xs[b][s*C + c][t'] * msq[t']
__global__ __launch_bounds__(256) void glow_unsqueeze_kernel(const float* xs, const float* msq, float* y,
                                                             int C, int Th, int nsq) {
  const int b = blockIdx.y;
  const int T = Th * nsq;
  const int64_t n = (int64_t)C * T;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int t = (int)(i % T);
    const int c = (int)(i / T);
    const int tq = t / nsq, sidx = t - tq * nsq;
    y[(size_t)b * n + i] = xs[((size_t)b * C * nsq + (size_t)sidx * C + c) * Th + tq] * msq[(size_t)b * Th + tq];
  }
}

// acts[b][c][t] = tanh(xin[b][c][t]) * sigmoid(xin[b][c+H][t])
// amax_* ([B][64] slots, or nullptr): max |output| per utterance for the f16x3 consumers
__global__ __launch_bounds__(256) void glow_gate_kernel(const float* xin, float* acts, int H, int Th,
                                                        unsigned* amax) {
  const int b = blockIdx.y;
  const int64_t n = (int64_t)H * Th;
  float vm = 0.f;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float a = xin[(size_t)b * 2 * n + i];
    const float g = xin[(size_t)b * 2 * n + n + i];
    const float sg = 1.f / (1.f + expf(-g));
    const float v = tanhf(a) * sg;
    acts[(size_t)b * n + i] = v;
    vm = fmaxf(vm, fabsf(v));
  }
  if (amax) publish_amax_block(amax, b, vm);
}

// not last: h = (h + rs[:H]) * mask ; skip (+)= rs[H:]       last: skip = (skip + rs) * mask
__global__ __launch_bounds__(256) void glow_wn_update_kernel(float* h, float* skip, const float* rs,
                                                             const float* mask, int H, int Th, int first,
                                                             int last, unsigned* amax) {
  const int b = blockIdx.y;
  const int64_t n = (int64_t)H * Th;
  float vm = 0.f;  // max |h| (not last: the next in_layer's input) or |skip| (last: the end conv's)
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int t = (int)(i % Th);
    const float m = mask[(size_t)b * Th + t];
    if (!last) {
      const float r0 = rs[(size_t)b * 2 * n + i];
      const float r1 = rs[(size_t)b * 2 * n + n + i];
      const float hv = (h[(size_t)b * n + i] + r0) * m;
      h[(size_t)b * n + i] = hv;
      skip[(size_t)b * n + i] = first ? r1 : skip[(size_t)b * n + i] + r1;
      vm = fmaxf(vm, fabsf(hv));
    } else {
      const float r = rs[(size_t)b * n + i];
      const float sk = (first ? r : skip[(size_t)b * n + i] + r) * m;
      skip[(size_t)b * n + i] = sk;
      vm = fmaxf(vm, fabsf(sk));
    }
  }
  if (amax) publish_amax_block(amax, b, vm);
}

// One thread per (b, group i, t).  Group i of InvConvNear (glow.py:116-117) holds channels
// ch(a, j) = a*C2/2 + i*S/2 + j for a in {0,1}, j < S/2; its weight row index is a*S/2 + j.
template <int S>
__global__ __launch_bounds__(256) void glow_tail_kernel(GlowTailArgs a) {
  const int b = blockIdx.y;
  const int C2 = a.C2, Th = a.Th;
  const int half = C2 / 2;
  const int G = C2 / S;
  const int64_t n = (int64_t)G * Th;
  float W[S][S];
#pragma unroll
  for (int o = 0; o < S; ++o)
#pragma unroll
    for (int g = 0; g < S; ++g) W[o][g] = a.winv[o * S + g];
  float vm = 0.f;  // max |x_0| of the updated x (the next flow's statistics)
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e % Th);
    const int i = (int)(e / Th);
    const float m = a.mask[(size_t)b * Th + t];
    float z[S];
    int chs[S];
#pragma unroll
    for (int g = 0; g < S; ++g) {
      const int aa = g / (S / 2), j = g % (S / 2);
      const int ch = aa * half + i * (S / 2) + j;
      chs[g] = ch;
      const float xv = a.x[((size_t)b * C2 + ch) * Th + t];
      if (ch < half) {
        z[g] = xv;  // z_0 = x_0
      } else {
        const float tt = a.out[((size_t)b * C2 + (ch - half)) * Th + t];
        float sv = a.out[((size_t)b * C2 + ch) * Th + t];
        if (a.sigmoid_scale) sv = logf(1e-6f + 1.f / (1.f + expf(-(sv + 2.f))));
        z[g] = (xv - tt) * expf(-sv) * m;  // z_1 = (x_1 - t) * exp(-s) * mask
      }
    }
#pragma unroll
    for (int o = 0; o < S; ++o) {
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < S; ++g) v = fmaf(W[o][g], z[g], v);
      v *= m;                                                         // InvConvNear: * x_mask
      const int ch = chs[o];
      v = (v - a.bias[ch]) * expf(-a.logs[ch]) * m;                   // ActNorm reverse
      a.x[((size_t)b * C2 + ch) * Th + t] = v;
      if (ch < half) vm = fmaxf(vm, fabsf(v));
    }
  }
  if (a.amax_x0) publish_amax_block(a.amax_x0, b, vm);
}

// ActNorm forward then InvConvNear forward of one flow block on the S channels of group i, in
// registers: v = (bias + exp(logs) * x) * mask; z = W . v * mask.  Returns |z_0| max contribution.
template <int S>
__device__ __forceinline__ float glow_head_group(float (&z)[S], const int (&chs)[S], const float (&W)[S][S],
                                                 const float* logs, const float* bias, float m, int half) {
  float v[S];
#pragma unroll
  for (int g = 0; g < S; ++g) v[g] = (bias[chs[g]] + expf(logs[chs[g]]) * z[g]) * m;  // ActNorm (:99)
  float vm = 0.f;
#pragma unroll
  for (int o = 0; o < S; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int g = 0; g < S; ++g) acc = fmaf(W[o][g], v[g], acc);
    z[o] = acc * m;  // InvConvNear: conv2d, then * x_mask (glow.py:132-135)
    if (chs[o] < half) vm = fmaxf(vm, fabsf(z[o]));
  }
  return vm;
}

// Block sum (256 threads) of a double, fixed order; thread 0 returns it
__device__ __forceinline__ double block_sum_d(double v) {
  __shared__ double red[256];
  red[threadIdx.x] = v;
  __syncthreads();
#pragma unroll
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  return red[0];
}

// Flow block 0's head (the later heads run inside glow_couple_fwd_kernel)
template <int S>
__global__ __launch_bounds__(256) void glow_head_kernel(GlowHeadArgs a) {
  const int b = blockIdx.y;
  const int C2 = a.C2, Th = a.Th, half = C2 / 2;
  const int64_t n = (int64_t)(C2 / S) * Th;
  float W[S][S];
#pragma unroll
  for (int o = 0; o < S; ++o)
#pragma unroll
    for (int g = 0; g < S; ++g) W[o][g] = a.w[o * S + g];
  float vm = 0.f;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e % Th), i = (int)(e / Th);
    const float m = a.mask[(size_t)b * Th + t];
    float z[S];
    int chs[S];
#pragma unroll
    for (int g = 0; g < S; ++g) {
      chs[g] = (g / (S / 2)) * half + i * (S / 2) + g % (S / 2);
      z[g] = a.x[((size_t)b * C2 + chs[g]) * Th + t];
    }
    vm = fmaxf(vm, glow_head_group<S>(z, chs, W, a.logs, a.bias, m, half));
#pragma unroll
    for (int g = 0; g < S; ++g) a.x[((size_t)b * C2 + chs[g]) * Th + t] = z[g];
  }
  if (a.amax_x0) publish_amax_block(a.amax_x0, b, vm);
}

// Coupling forward (glow.py:216-227): z_1 = (t + exp(s) * x_1) * mask, logdet partial sum(s * mask);
// then, when a.w != nullptr, the next flow block's head on the same S channels
template <int S>
__global__ __launch_bounds__(256) void glow_couple_fwd_kernel(GlowCoupleArgs a) {
  const int b = blockIdx.y;
  const int C2 = a.C2, Th = a.Th, half = C2 / 2;
  const int64_t n = (int64_t)(C2 / S) * Th;
  const bool head = a.w != nullptr;
  float W[S][S];
#pragma unroll
  for (int o = 0; o < S; ++o)
#pragma unroll
    for (int g = 0; g < S; ++g) W[o][g] = head ? a.w[o * S + g] : 0.f;
  float vm = 0.f;
  double ld = 0.0;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e % Th), i = (int)(e / Th);
    const float m = a.mask[(size_t)b * Th + t];
    float z[S];
    int chs[S];
#pragma unroll
    for (int g = 0; g < S; ++g) {
      const int ch = (g / (S / 2)) * half + i * (S / 2) + g % (S / 2);
      chs[g] = ch;
      const float xv = a.x[((size_t)b * C2 + ch) * Th + t];
      if (ch < half) {
        z[g] = xv;  // z_0 = x_0
      } else {
        const float tt = a.out[((size_t)b * C2 + (ch - half)) * Th + t];
        float sv = a.out[((size_t)b * C2 + ch) * Th + t];
        if (a.sigmoid_scale) sv = logf(1e-6f + 1.f / (1.f + expf(-(sv + 2.f))));
        z[g] = (tt + expf(sv) * xv) * m;  // z_1 = (t + exp(s) * x_1) * x_mask
        ld += (double)(sv * m);           // torch.sum(s * x_mask, [1, 2])
      }
    }
    if (head) vm = fmaxf(vm, glow_head_group<S>(z, chs, W, a.logs, a.bias, m, half));
#pragma unroll
    for (int g = 0; g < S; ++g) a.x[((size_t)b * C2 + chs[g]) * Th + t] = z[g];
  }
  if (a.ld_part) {
    const double tot = block_sum_d(ld);
    if (threadIdx.x == 0) a.ld_part[(size_t)b * gridDim.x + blockIdx.x] = tot;
  }
  if (head && a.amax_x0) publish_amax_block(a.amax_x0, b, vm);
}

// logdet[b] = per_len * x_len[b] + sum of the coupling partials [nparts][B][npb] (fixed order, fp64);
// x_len = sum_t mask[b][t] (normalization.py:91, glow.py:122); per_len = sum over flow blocks of
// sum(logs) + logdet(W) * C2 / S (the ActNorm and InvConvNear terms)
__global__ __launch_bounds__(256) void glow_logdet_kernel(const double* parts, int nparts, int npb, const float* mask,
                                                          int Th, double per_len, float* logdet, int B) {
  const int b = blockIdx.x;
  double xl = 0.0, ps = 0.0;
  for (int t = threadIdx.x; t < Th; t += 256) xl += (double)mask[(size_t)b * Th + t];
  for (int k = threadIdx.x; k < nparts * npb; k += 256) {
    const int f = k / npb, j = k - f * npb;
    ps += parts[((size_t)f * B + b) * npb + j];
  }
  xl = block_sum_d(xl);
  __syncthreads();
  ps = block_sum_d(ps);
  if (threadIdx.x == 0) logdet[b] = (float)(per_len * xl + ps);
}

namespace {
dim3 ew_grid(int64_t n, int B, int64_t cap = 4096) {
  int64_t g = (n + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return dim3((unsigned)g, B);
}
}  // namespace

void launch_glow_squeeze(const float* x, const float* mask, float* xs, float* msq, int B, int C, int T,
                         int nsq, hipStream_t s) {
  const int Th = T / nsq;
  hipLaunchKernelGGL(glow_squeeze_kernel, ew_grid((int64_t)C * nsq * Th, B), dim3(256), 0, s, x, mask, xs,
                     msq, C, T, nsq);
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_glow_unsqueeze(const float* xs, const float* msq, float* y, int B, int C, int Th, int nsq,
                           hipStream_t s) {
  hipLaunchKernelGGL(glow_unsqueeze_kernel, ew_grid((int64_t)C * Th * nsq, B), dim3(256), 0, s, xs, msq, y,
                     C, Th, nsq);
  TTS_HIP_CHECK(hipGetLastError());
}

// y[b][c][t] = x[b][C-1-c][t]  (torch.flip(x, [1]))
__global__ __launch_bounds__(256) void channel_flip_kernel(const float* x, float* y, int C, int T) {
  const int b = blockIdx.y;
  const int64_t n = (int64_t)C * T;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i / T);
    const int t = (int)(i - (int64_t)c * T);
    y[(size_t)b * n + i] = x[(size_t)b * n + (int64_t)(C - 1 - c) * T + t];
  }
}

void launch_channel_flip(const float* x, float* y, int B, int C, int T, hipStream_t s) {
  hipLaunchKernelGGL(channel_flip_kernel, ew_grid((int64_t)C * T, B), dim3(256), 0, s, x, y, C, T);
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_glow_gate(const float* xin, float* acts, int B, int H, int Th, hipStream_t s, unsigned* amax) {
  // with statistics: at most 128 workgroups per item (a few elements per thread, 128 atomics)
  hipLaunchKernelGGL(glow_gate_kernel, ew_grid((int64_t)H * Th, B, amax ? 128 : 4096), dim3(256), 0, s, xin, acts,
                     H, Th, amax);
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_glow_wn_update(float* h, float* skip, const float* rs, const float* mask, int B, int H, int Th,
                           int first, int last, hipStream_t s, unsigned* amax) {
  hipLaunchKernelGGL(glow_wn_update_kernel, ew_grid((int64_t)H * Th, B, amax ? 128 : 4096), dim3(256), 0, s, h,
                     skip, rs, mask, H, Th, first, last, amax);
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_glow_head(const GlowHeadArgs& a, int B, hipStream_t s) {
  const int64_t n = (int64_t)(a.C2 / a.S) * a.Th;
  const int64_t cap = a.amax_x0 ? 128 : 4096;
  switch (a.S) {
    case 2: hipLaunchKernelGGL(glow_head_kernel<2>, ew_grid(n, B, cap), dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL(glow_head_kernel<4>, ew_grid(n, B, cap), dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL(glow_head_kernel<8>, ew_grid(n, B, cap), dim3(256), 0, s, a); break;
    default: throw Error(3, "InvConvNear num_splits must be 2, 4 or 8");
  }
  TTS_HIP_CHECK(hipGetLastError());
}

int glow_couple_parts(int C2, int S, int Th) {
  return (int)ew_grid((int64_t)(C2 / S) * Th, 1, kGlowLogdetParts).x;
}

void launch_glow_couple_fwd(const GlowCoupleArgs& a, int B, hipStream_t s) {
  const int64_t n = (int64_t)(a.C2 / a.S) * a.Th;
  const dim3 grid = ew_grid(n, B, kGlowLogdetParts);  // fixed per shape: the logdet sums are deterministic
  switch (a.S) {
    case 2: hipLaunchKernelGGL(glow_couple_fwd_kernel<2>, grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL(glow_couple_fwd_kernel<4>, grid, dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL(glow_couple_fwd_kernel<8>, grid, dim3(256), 0, s, a); break;
    default: throw Error(3, "InvConvNear num_splits must be 2, 4 or 8");
  }
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_glow_logdet(const double* parts, int nparts, int npb, const float* mask, int Th, double per_len,
                        float* logdet, int B, hipStream_t s) {
  hipLaunchKernelGGL(glow_logdet_kernel, dim3(B), dim3(256), 0, s, parts, nparts, npb, mask, Th, per_len, logdet, B);
  TTS_HIP_CHECK(hipGetLastError());
}

void launch_glow_tail(const GlowTailArgs& a, int B, hipStream_t s) {
  const int64_t n = (int64_t)(a.C2 / a.S) * a.Th;
  const int64_t cap = a.amax_x0 ? 128 : 4096;  // with statistics: one atomic per workgroup, <= 128 per item
  switch (a.S) {
    case 2: hipLaunchKernelGGL(glow_tail_kernel<2>, ew_grid(n, B, cap), dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL(glow_tail_kernel<4>, ew_grid(n, B, cap), dim3(256), 0, s, a); break;
    case 8: hipLaunchKernelGGL(glow_tail_kernel<8>, ew_grid(n, B, cap), dim3(256), 0, s, a); break;
    default: throw Error(3, "InvConvNear num_splits must be 2, 4 or 8");
  }
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts

// ---------------------------------------------------------------------------------------------
// VITS PosteriorEncoder sample (networks.py:286-287): m, logs = split(stats); z = (m + eps *
// exp(logs)) * mask.  stats = proj(x) * mask is already masked.
#include "vits.hpp"

namespace tts {

__global__ __launch_bounds__(256) void posterior_sample_kernel(const float* stats, const float* eps,
                                                               const float* mask, float* z, float* m, float* logs,
                                                               int Co, int T) {
  const int b = blockIdx.y;
  const int64_t n = (int64_t)Co * T;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int t = (int)(i % T);
    const float mv = stats[(size_t)b * 2 * n + i];
    const float lv = stats[(size_t)b * 2 * n + n + i];
    const float e = eps ? eps[(size_t)b * n + i] : 0.f;
    z[(size_t)b * n + i] = (mv + e * expf(lv)) * mask[(size_t)b * T + t];
    if (m) m[(size_t)b * n + i] = mv;
    if (logs) logs[(size_t)b * n + i] = lv;
  }
}

void launch_posterior_sample(const float* stats, const float* eps, const float* mask, float* z, float* m,
                             float* logs, int B, int Co, int T, hipStream_t s) {
  int64_t g = ((int64_t)Co * T + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(posterior_sample_kernel, dim3((unsigned)g, B), dim3(256), 0, s, stats, eps, mask, z, m, logs,
                     Co, T);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
