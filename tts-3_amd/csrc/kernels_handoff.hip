// TTS -> vocoder hand-off and the int16 wav writer on gfx950 (elementwise / one reduction,
// HBM-bound; every access coalesced along time).
//
// Reference (Coqui TTS 0.22.0):
//   TTS/utils/synthesizer.py:412-428  mel = tts_ap.denormalize(model_outputs.T); x =
//       vocoder_ap.normalize(mel); optional interpolate_vocoder_input (sample-rate mismatch)
//   TTS/utils/audio/processor.py:259-336  normalize / denormalize (range or mean-var)
//   TTS/tts/utils/helpers.py:14-39        StandardScaler (mel_scaler)
//   TTS/vocoder/utils/generic_utils.py:11-29  F.interpolate(bilinear, align_corners=False,
//       recompute_scale_factor=True) with scale [1, sr_vocoder / sr_tts]
//   TTS/utils/audio/numpy_transforms.py:430-447 / processor.py:605-625  save_wav int16 scaling
//
// Arithmetic follows the reference's numpy dtypes: the range (de)normalisation is fp32 with the
// Python scalars rounded to fp32 (numpy 2 weak scalars), evaluated in the reference's order;
// the mean-var path runs in fp64 because the stats are fp64 arrays (numpy upcasts, then the
// in-place result is rounded back to fp32).
#include "handoff.hpp"

// numpy evaluates every operation with its own rounding: no a*b+c contraction into FMAs here
#pragma clang fp contract(off)

namespace tts {

__device__ __forceinline__ float denorm_range(float s, const AudioNormDev& n) {
  if (n.symmetric_norm) {
    if (n.clip_norm) s = fminf(fmaxf(s, -n.max_norm), n.max_norm);
    s = ((s + n.max_norm) * n.neg_min_level_db / n.two_max_norm) + n.min_level_db;
  } else {
    if (n.clip_norm) s = fminf(fmaxf(s, 0.f), n.max_norm);
    s = (s * n.neg_min_level_db / n.max_norm) + n.min_level_db;
  }
  return s + n.ref_level_db;
}

__device__ __forceinline__ float norm_range(float s, const AudioNormDev& n) {
  s = s - n.ref_level_db;
  float sn = (s - n.min_level_db) / n.neg_min_level_db;
  if (n.symmetric_norm) {
    sn = (n.two_max_norm * sn) - n.max_norm;
    if (n.clip_norm) sn = fminf(fmaxf(sn, -n.max_norm), n.max_norm);
  } else {
    sn = n.max_norm * sn;
    if (n.clip_norm) sn = fminf(fmaxf(sn, 0.f), n.max_norm);
  }
  return sn;
}

__device__ __forceinline__ float renorm(float x, int c, const AudioNormDev& de, const AudioNormDev& no) {
  if (de.signal_norm) {
    if (de.mean) x = (float)((double)(float)((double)x * de.scale[c]) + de.mean[c]);  // X *= scale_; X += mean_
    else x = denorm_range(x, de);
  }
  if (no.signal_norm) {
    if (no.mean) x = (float)((double)(float)((double)x - no.mean[c]) / no.scale[c]);  // X -= mean_; X /= scale_
    else x = norm_range(x, no);
  }
  return x;
}

// out[b][c][j] for j < T_out: renorm of in[b][t][c] (time-major, model_outputs) or in[b][c][t];
// with T_out != T the time axis is resampled linearly (align_corners=False, scale T/T_out).
__global__ void __launch_bounds__(256) handoff_kernel(HandoffArgs a) {
  const int b = blockIdx.z;
  const int c = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= a.T_out) return;
  const int T = a.T, C = a.C;
  auto load = [&](int t) {
    const float v = a.time_major ? a.in[((size_t)b * T + t) * C + c] : a.in[((size_t)b * C + c) * T + t];
    return renorm(v, c, a.de, a.no);
  };
  float y;
  if (a.T_out == T) {
    y = load(j);
  } else {
    // PyTorch upsample_linear: src = scale * (j + 0.5) - 0.5, clamped at 0; scale = T / T_out
    // (recompute_scale_factor=True) or 1 / scale_factor as given (a.src_scale > 0)
    const float scale = a.src_scale > 0.f ? a.src_scale : (float)T / (float)a.T_out;
    float src = scale * ((float)j + 0.5f) - 0.5f;
    src = src < 0.f ? 0.f : src;
    const int i0 = (int)src;
    const int i1 = i0 + (i0 < T - 1 ? 1 : 0);
    const float l1 = src - (float)i0, l0 = 1.f - l1;
    y = l0 * load(i0) + l1 * load(i1);
  }
  a.out[((size_t)b * C + c) * a.T_out + j] = y;
}

void launch_handoff(const HandoffArgs& a, int B, hipStream_t s) {
  dim3 grid(ceil_div(a.T_out, 256), a.C, B);
  hipLaunchKernelGGL(handoff_kernel, grid, dim3(256), 0, s, a);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// save_wav scaling: wav_norm = wav * (32767 / max(0.01, max|wav|)); astype(int16) (truncation).
// Pass 1: per-utterance max|wav| (atomicMax on the fp32 bits, non-negative); pass 2: scale +
// truncate.  len[b] (or n when len is NULL) bounds each utterance's samples.
// Non-finite contract (numpy on x86, numpy_transforms.py:436-438, pinned by
// tests/test_oracle_golden.py::test_wav_int16_nonfinite_contract):
//  * np.max propagates NaN and Python's max(0.01, nan) returns 0.01, so one NaN sample makes the
//    scale 32767 / 0.01: the max runs on the fp32 bits as unsigned integers (|NaN| sorts above inf);
//  * astype(int16) converts through int32 (cvttss2si: NaN, +-inf and |v| >= 2^31 give INT_MIN)
//    and keeps the low 16 bits, so those samples become 0 and other out-of-range ones wrap.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) wav_amax_kernel(const float* __restrict__ wav, int64_t n,
                                                       const int64_t* __restrict__ len, unsigned* __restrict__ amax) {
  const int b = blockIdx.y;
  const int64_t L = len ? (len[b] < n ? len[b] : n) : n;
  const float* w = wav + (size_t)b * n;
  unsigned m = 0u;  // fp32 bits of |w|: unsigned order = float order, NaN above inf
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < L; i += (int64_t)gridDim.x * 256)
    m = max(m, __float_as_uint(w[i]) & 0x7FFFFFFFu);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(amax + b, m);
}

__global__ void __launch_bounds__(256) wav_int16_kernel(const float* __restrict__ wav, int64_t n,
                                                        const int64_t* __restrict__ len,
                                                        const unsigned* __restrict__ amax, int16_t* __restrict__ out) {
  const int b = blockIdx.y;
  const int64_t L = len ? (len[b] < n ? len[b] : n) : n;
  const float mx = fmaxf(0.01f, __uint_as_float(amax[b]));  // fmaxf(0.01, NaN) = 0.01, as max(0.01, nan)
  const float scale = 32767.f / mx;
  const float* w = wav + (size_t)b * n;
  int16_t* o = out + (size_t)b * n;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = w[i] * scale;
    // truncation toward zero like astype; NaN / inf / |v| >= 2^31 -> INT_MIN (x86 cvttss2si) -> 0
    const int iv = (v >= -2147483648.f && v < 2147483648.f) ? (int)v : (int)0x80000000;
    o[i] = i < L ? (int16_t)iv : (int16_t)0;
  }
}

void launch_wav_int16(const float* wav, int B, int64_t n, const int64_t* len, unsigned* amax, int16_t* out,
                      hipStream_t s) {
  TTS_HIP_CHECK(hipMemsetAsync(amax, 0, sizeof(unsigned) * B, s));
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1024);
  dim3 grid(blocks, B);
  hipLaunchKernelGGL(wav_amax_kernel, grid, dim3(256), 0, s, wav, n, len, amax);
  TTS_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(wav_int16_kernel, grid, dim3(256), 0, s, wav, n, len, amax, out);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// One time window of the replicate-padded mel (windowed HiFiGAN forward, hifigan.cpp)
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) mel_window_kernel(const float* __restrict__ mel, int T, int pad, int64_t w0,
                                                         int W, float* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= W) return;
  const size_t row = (size_t)blockIdx.z * gridDim.y + blockIdx.y;  // b * C + c
  int64_t src = w0 + t - pad;
  src = src < 0 ? 0 : (src >= T ? T - 1 : src);
  out[row * W + t] = mel[row * (size_t)T + src];
}

void launch_mel_window(const float* mel, int B, int C, int T, int pad, int64_t w0, int W, float* out, hipStream_t s) {
  TTS_REQUIRE(B >= 1 && C >= 1 && C <= 65535 && B <= 65535 && T >= 1 && W >= 1, 1, "mel_window: bad shape");
  hipLaunchKernelGGL(mel_window_kernel, dim3((W + 255) / 256, C, B), dim3(256), 0, s, mel, T, pad, w0, W, out);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
