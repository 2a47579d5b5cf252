// Elementwise kernels of the reverse Glow-TTS decoder flow (gfx950).
//   squeeze / unsqueeze      decoder.py:8-47
//   gate                     wavenet.py:6-13 (fused_add_tanh_sigmoid_multiply, g = 0)
//   wn_update                wavenet.py:109-115 (residual/skip split of res_skip_layers)
//   tail                     glow.py:222-224 (coupling affine inverse) -> glow.py:102-137
//                            (InvConvNear inverse) -> normalization.py:96-98 (ActNorm inverse),
//                            fused: one thread owns the S channels InvConvNear mixes.
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
