// Glow-TTS text side on gfx950: token embedding, channel LayerNorm, relative-position
// multi-head self-attention, and the duration / alignment glue of GlowTTS.inference.
//
// Reference (Coqui TTS 0.22.0):
//   TTS/tts/layers/glow_tts/encoder.py:162-165    emb(x) * sqrt(H), transpose, sequence_mask
//   TTS/tts/layers/generic/normalization.py:23-28 LayerNorm over channels, eps 1e-4
//   TTS/tts/layers/glow_tts/transformer.py:142-180 attention (+ relative keys / values)
//   TTS/tts/models/glow_tts.py:349-361            durations, y_mask, generate_path, y_mean, z
//   TTS/tts/utils/helpers.py:154-169              generate_path
//
// All activations are [B][C][T] fp32 (the reference's NCW).  These kernels are latency-bound
// (a 16 x 128-token batch is ~2k positions): they are written to keep every access coalesced
// along T and to do each reduction in one workgroup, not for MFMA (the matmuls of the encoder
// run on the conv kernels as 1x1 / k3 / k5 convolutions).
#include "text.hpp"

namespace tts {

// ---------------------------------------------------------------------------------------
// x[b][c][t] = emb[tok[b][t]][c] * scale * mask[b][t];  mask[b][t] = t < len[b]
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) embed_kernel(const int64_t* __restrict__ tok, const int64_t* __restrict__ len,
                                                    const float* __restrict__ emb, const float* __restrict__ lang,
                                                    float* __restrict__ x, float* __restrict__ mask, int He, int H,
                                                    int T, int num_chars, float scale) {
  const int b = blockIdx.y;
  const int t = blockIdx.x * 64 + (threadIdx.x & 63);
  const int cq = threadIdx.x >> 6;  // 4 waves split the channels
  if (t >= T) return;
  const int64_t L = len[b];
  const float m = (int64_t)t < L ? 1.f : 0.f;
  int64_t id = tok[(size_t)b * T + t];
  // the reference raises IndexError on an out-of-range id; padded positions carry any id
  // (they are masked), so clamp instead of reading out of bounds
  id = id < 0 ? 0 : (id >= num_chars ? num_chars - 1 : id);
  const float* e = emb + (size_t)id * He;
  float* xo = x + (size_t)b * H * T + t;
  for (int c = cq; c < He; c += 4) xo[(size_t)c * T] = e[c] * scale * m;
  // channels He .. H: the utterance's language embedding, cat((emb * sqrt(He), lang_emb.expand(T)))
  // (vits/networks.py:90-91), masked with the rest (:96)
  for (int c = He + cq; c < H; c += 4) xo[(size_t)c * T] = lang[(size_t)b * (H - He) + (c - He)] * m;
  if (cq == 0 && mask) mask[(size_t)b * T + t] = m;
}

void launch_embed(const int64_t* tok, const int64_t* len, const float* emb, float* x, float* mask, int B, int H,
                  int T, int num_chars, float scale, hipStream_t s, const float* lang, int He) {
  if (He <= 0) He = H;
  TTS_REQUIRE(He <= H && (He == H || lang != nullptr), 1, "embed: the language embedding channels need lang_emb");
  dim3 grid(ceil_div(T, 64), B);
  hipLaunchKernelGGL(embed_kernel, grid, dim3(256), 0, s, tok, len, emb, lang, x, mask, He, H, T, num_chars, scale);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// y = LayerNorm_C(a [+ r]) * gamma + beta, then optional relu, then * mask.
// One workgroup = 16 time columns x 16 channel slices (a 16-lane group reads 64 contiguous bytes
// of one channel row); the partial sums meet in LDS.  Two-pass mean / variance exactly as the
// reference formula.  A 16 x 128-token batch is 128 workgroups (latency-bound: each thread holds
// at most C/16 values in registers between the passes).  y may alias a or r.
// ---------------------------------------------------------------------------------------
constexpr int LN_T = 16;
constexpr int LN_S = 16;
constexpr int LN_MAXV = 48;  // C <= 768

__global__ void __launch_bounds__(256) layernorm_kernel(const float* a, const float* r, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, const float* __restrict__ mask,
                                                        float* y, int C, int T, float eps, int relu) {
  __shared__ float part[LN_S][LN_T];
  const int b = blockIdx.y;
  const int col = threadIdx.x & (LN_T - 1);
  const int sl = threadIdx.x / LN_T;
  const int t = blockIdx.x * LN_T + col;
  const bool ok = t < T;
  const size_t base = (size_t)b * C * T + (ok ? t : 0);
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = sl + i * LN_S;
    v[i] = 0.f;
    if (c < C) {
      v[i] = a[base + (size_t)c * T];
      if (r) v[i] += r[base + (size_t)c * T];
      s += v[i];
    }
  }
  part[sl][col] = s;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int i = 0; i < LN_S; ++i) tot += part[i][col];
  const float mean = tot / (float)C;
  __syncthreads();
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = sl + i * LN_S;
    if (c < C) {
      const float d = v[i] - mean;
      q += d * d;
    }
  }
  part[sl][col] = q;
  __syncthreads();
  float qt = 0.f;
#pragma unroll
  for (int i = 0; i < LN_S; ++i) qt += part[i][col];
  const float var = qt / (float)C;
  const float rs = 1.f / sqrtf(var + eps);
  const float m = mask ? mask[(size_t)b * T + (ok ? t : 0)] : 1.f;
  if (!ok) return;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = sl + i * LN_S;
    if (c < C) {
      float o = (v[i] - mean) * rs * gamma[c] + beta[c];
      if (relu) o = fmaxf(o, 0.f);
      y[base + (size_t)c * T] = o * m;
    }
  }
}

void launch_layernorm(const float* a, const float* r, const float* gamma, const float* beta, const float* mask,
                      float* y, int B, int C, int T, float eps, bool relu, hipStream_t s) {
  TTS_REQUIRE(C <= LN_S * LN_MAXV, 3, "LayerNorm: more than 768 channels");
  dim3 grid(ceil_div(T, LN_T), B);
  hipLaunchKernelGGL(layernorm_kernel, grid, dim3(256), 0, s, a, r, gamma, beta, mask, y, C, T, eps, relu ? 1 : 0);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// gated_conv layer tail (gated_conv.py:30-36): LayerNorm over the conv's 2H channels, GLU over
// the channel halves, residual add; the layer's next conv reads o * x_mask, so the output is
// masked here.  Same slicing as layernorm_kernel: channels c and c + C/2 sit in one thread when
// C/2 is a multiple of LN_S.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) layernorm_glu_kernel(const float* a, const float* res,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ mask, float* y, int C, int T,
                                                            float eps) {
  __shared__ float part[LN_S][LN_T];
  const int b = blockIdx.y;
  const int col = threadIdx.x & (LN_T - 1);
  const int sl = threadIdx.x / LN_T;
  const int t = blockIdx.x * LN_T + col;
  const bool ok = t < T;
  const int Ch = C / 2;
  const size_t base = (size_t)b * C * T + (ok ? t : 0);
  const size_t hbase = (size_t)b * Ch * T + (ok ? t : 0);
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = sl + i * LN_S;
    v[i] = 0.f;
    if (c < C) {
      v[i] = a[base + (size_t)c * T];
      s += v[i];
    }
  }
  part[sl][col] = s;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int i = 0; i < LN_S; ++i) tot += part[i][col];
  const float mean = tot / (float)C;
  __syncthreads();
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = sl + i * LN_S;
    if (c < C) {
      const float d = v[i] - mean;
      q += d * d;
    }
  }
  part[sl][col] = q;
  __syncthreads();
  float qt = 0.f;
#pragma unroll
  for (int i = 0; i < LN_S; ++i) qt += part[i][col];
  const float var = qt / (float)C;
  const float rs = 1.f / sqrtf(var + eps);
  const float m = mask ? mask[(size_t)b * T + (ok ? t : 0)] : 1.f;
  if (!ok) return;
  const int ih = Ch / LN_S;  // slice offset of channel c + C/2
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = sl + i * LN_S;
    if (c < Ch && i + ih < LN_MAXV) {
      const int c2 = c + Ch;
      const float o1 = (v[i] - mean) * rs * gamma[c] + beta[c];
      const float o2 = (v[i + ih] - mean) * rs * gamma[c2] + beta[c2];
      const float g = o1 * (1.f / (1.f + expf(-o2)));
      y[hbase + (size_t)c * T] = (res[hbase + (size_t)c * T] + g) * m;
    }
  }
}

void launch_layernorm_glu(const float* a, const float* res, const float* gamma, const float* beta, const float* mask,
                          float* y, int B, int C, int T, float eps, hipStream_t s) {
  TTS_REQUIRE(C <= LN_S * LN_MAXV && C % (2 * LN_S) == 0, 3,
              "gated_conv LayerNorm: 2 x hidden channels must be a multiple of 32 and at most 768");
  dim3 grid(ceil_div(T, LN_T), B);
  hipLaunchKernelGGL(layernorm_glu_kernel, grid, dim3(256), 0, s, a, res, gamma, beta, mask, y, C, T, eps);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// Conv1dBN tail (res_conv_bn.py:39-44) and the residual block's add + mask (:124-127)
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) bn_act_kernel(const float* a, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, const float* res,
                                                     const float* __restrict__ mask, float* y, int C, int T, int lo,
                                                     int hi) {
  const int b = blockIdx.z, c = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  const size_t i = ((size_t)b * C + c) * T + t;
  const float v = (t >= lo && t < hi) ? fmaxf(a[i], 0.f) : 0.f;
  float o = v * scale[c] + shift[c];
  if (res) o = (o + res[i]) * mask[(size_t)b * T + t];
  y[i] = o;
}

void launch_bn_act(const float* a, const float* scale, const float* shift, const float* res, const float* mask,
                   float* y, int B, int C, int T, int lo, int hi, hipStream_t s) {
  TTS_REQUIRE(!res || mask, 1, "bn_act: the residual form needs the mask");
  dim3 grid(ceil_div(T, 256), C, B);
  hipLaunchKernelGGL(bn_act_kernel, grid, dim3(256), 0, s, a, scale, shift, res, mask, y, C, T, lo, hi);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// TimeDepthSeparableConv middle (time_depth_sep_conv.py:50-54): GLU, depthwise conv (norm2
// folded), swish.  One thread per output; the GLU of each tap's input is recomputed (k <= 11).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) glu_dw_swish_kernel(const float* __restrict__ a, const float* __restrict__ w,
                                                           const float* __restrict__ bias, float* __restrict__ y,
                                                           int C, int T, int k) {
  const int b = blockIdx.z, c = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  const float* a1 = a + ((size_t)b * 2 * C + c) * T;
  const float* a2 = a1 + (size_t)C * T;
  const int p = (k - 1) / 2;
  float v = 0.f;
  for (int j = 0; j < k; ++j) {
    const int ts = t - p + j;
    if (ts >= 0 && ts < T) v = fmaf(w[c * k + j], a1[ts] * (1.f / (1.f + expf(-a2[ts]))), v);
  }
  v += bias[c];
  y[((size_t)b * C + c) * T + t] = v * (1.f / (1.f + expf(-v)));
}

void launch_glu_dw_swish(const float* a, const float* w, const float* bias, float* y, int B, int C, int T, int k,
                         hipStream_t s) {
  TTS_REQUIRE(k >= 1 && k <= 31 && k % 2 == 1, 3, "time_depth_separable: kernel_size must be odd and <= 31");
  dim3 grid(ceil_div(T, 256), C, B);
  hipLaunchKernelGGL(glu_dw_swish_kernel, grid, dim3(256), 0, s, a, w, bias, y, C, T, k);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// Relative-position multi-head self-attention (transformer.py:142-180), one workgroup per
// (8 queries, head, utterance):
//   s[i][j] = (q_i . k_j) / sqrt(dk) + [|j-i| <= W] (q_i . ek[j-i+W]) / sqrt(dk)
//   s = mask_i * mask_j [* |j-i| <= input_length] ? s : -1e4;  p = softmax_j(s)
//   o_i = sum_j p[i][j] v_j + sum_{|j-i| <= W} p[i][j] ev[j-i+W]
// qkv: [B][3H][T] (rows q | k | v, head h = channels h*dk .. h*dk+dk-1), out: [B][H][T].
// LDS: Q [8][dk], a K / V chunk [dk][64+1] (pad: conflict-free column reads), the 8 score
// rows [8][T] (the whole row, so the softmax is the reference's exact two-pass form).
// ---------------------------------------------------------------------------------------
constexpr int ATT_QB = 8;
constexpr int ATT_KC = 64;
constexpr int ATT_MAX_DK = 128;

__global__ void __launch_bounds__(256) attention_kernel(const float* __restrict__ qkv, const float* __restrict__ mask,
                                                        const float* __restrict__ ek, const float* __restrict__ ev,
                                                        float* __restrict__ out, int H, int dk, int T, int W,
                                                        int band) {
  extern __shared__ float lds[];
  float* Qs = lds;                             // [ATT_QB][dk]
  float* Kc = Qs + ATT_QB * ATT_MAX_DK;        // [dk][ATT_KC + 1]
  float* S = Kc + ATT_MAX_DK * (ATT_KC + 1);   // [ATT_QB][T]
  const int i0 = blockIdx.x * ATT_QB;
  const int h = blockIdx.y;
  const int b = blockIdx.z;
  const int tid = threadIdx.x;
  const size_t plane = (size_t)T;
  const float* q = qkv + ((size_t)b * 3 * H + (size_t)h * dk) * plane;
  const float* k = q + (size_t)H * plane;
  const float* v = k + (size_t)H * plane;
  const float* mb = mask + (size_t)b * T;
  const float rsd = sqrtf((float)dk);

  for (int e = tid; e < ATT_QB * dk; e += 256) {
    const int d = e / ATT_QB, qi = e % ATT_QB;
    const int i = i0 + qi;
    Qs[qi * dk + d] = i < T ? q[(size_t)d * plane + i] : 0.f;
  }
  // scores: thread = (query qi = tid / 32, keys jj = tid % 32 and jj + 32 of the chunk)
  const int qi = tid >> 5;
  const int jj = tid & 31;
  for (int j0 = 0; j0 < T; j0 += ATT_KC) {
    __syncthreads();  // Qs ready / previous chunk consumed
    for (int e = tid; e < dk * ATT_KC; e += 256) {
      const int d = e / ATT_KC, c = e % ATT_KC;
      const int j = j0 + c;
      Kc[d * (ATT_KC + 1) + c] = j < T ? k[(size_t)d * plane + j] : 0.f;
    }
    __syncthreads();
    float s0 = 0.f, s1 = 0.f;
    for (int d = 0; d < dk; ++d) {
      const float qv = Qs[qi * dk + d];
      s0 += qv * Kc[d * (ATT_KC + 1) + jj];
      s1 += qv * Kc[d * (ATT_KC + 1) + jj + 32];
    }
    if (j0 + jj < T) S[qi * T + j0 + jj] = s0 / rsd;
    if (j0 + jj + 32 < T) S[qi * T + j0 + jj + 32] = s1 / rsd;
  }
  __syncthreads();
  // relative keys: (query, offset) pairs; each (query, key) receives at most one term
  if (W > 0) {
    const int R = 2 * W + 1;
    for (int e = tid; e < ATT_QB * R; e += 256) {
      const int qq = e / R, rr = e % R;
      const int i = i0 + qq, j = i + rr - W;
      if (i < T && j >= 0 && j < T) {
        float acc = 0.f;
        for (int d = 0; d < dk; ++d) acc += Qs[qq * dk + d] * ek[rr * dk + d];
        S[qq * T + j] += acc / rsd;
      }
    }
    __syncthreads();
  }
  // mask + softmax: wave w owns rows 2w, 2w+1
  const int lane = tid & 63;
  const int wv = tid >> 6;
  for (int rr = 0; rr < 2; ++rr) {
    const int row = 2 * wv + rr;
    const int i = i0 + row;
    const float mi = i < T ? mb[i] : 0.f;
    float* Sr = S + row * T;
    float mx = -INFINITY;
    for (int j = lane; j < T; j += 64) {
      // band >= 0: input_length's block mask (transformer.py:148-150), -1e4 outside |j - i| <= band
      const bool in_band = band < 0 || (j - i <= band && i - j <= band);
      const float sv = (mi != 0.f && mb[j] != 0.f && in_band) ? Sr[j] : -1e4f;
      Sr[j] = sv;
      mx = fmaxf(mx, sv);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
    for (int j = lane; j < T; j += 64) {
      const float e = expf(Sr[j] - mx);
      Sr[j] = e;
      sum += e;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    for (int j = lane; j < T; j += 64) Sr[j] = Sr[j] / sum;
  }
  // output: thread = (query tid / 32, channels d = tid % 32 + 32 m)
  float acc[ATT_MAX_DK / 32];
#pragma unroll
  for (int m = 0; m < ATT_MAX_DK / 32; ++m) acc[m] = 0.f;
  for (int j0 = 0; j0 < T; j0 += ATT_KC) {
    __syncthreads();
    for (int e = tid; e < dk * ATT_KC; e += 256) {
      const int d = e / ATT_KC, c = e % ATT_KC;
      const int j = j0 + c;
      Kc[d * (ATT_KC + 1) + c] = j < T ? v[(size_t)d * plane + j] : 0.f;
    }
    __syncthreads();
    const int n = min(ATT_KC, T - j0);
    for (int c = 0; c < n; ++c) {
      const float p = S[qi * T + j0 + c];
#pragma unroll
      for (int m = 0; m < ATT_MAX_DK / 32; ++m) {
        const int d = jj + 32 * m;
        if (d < dk) acc[m] += p * Kc[d * (ATT_KC + 1) + c];
      }
    }
  }
  const int i = i0 + qi;
  if (i >= T) return;
  if (W > 0) {
    for (int rr = 0; rr <= 2 * W; ++rr) {
      const int j = i + rr - W;
      if (j < 0 || j >= T) continue;
      const float p = S[qi * T + j];
#pragma unroll
      for (int m = 0; m < ATT_MAX_DK / 32; ++m) {
        const int d = jj + 32 * m;
        if (d < dk) acc[m] += p * ev[rr * dk + d];
      }
    }
  }
  float* o = out + ((size_t)b * H + (size_t)h * dk) * plane + i;
#pragma unroll
  for (int m = 0; m < ATT_MAX_DK / 32; ++m) {
    const int d = jj + 32 * m;
    if (d < dk) o[(size_t)d * plane] = acc[m];
  }
}

size_t attention_lds_bytes(int T) {
  return sizeof(float) * ((size_t)ATT_QB * ATT_MAX_DK + (size_t)ATT_MAX_DK * (ATT_KC + 1) + (size_t)ATT_QB * T);
}

void launch_attention(const float* qkv, const float* mask, const float* ek, const float* ev, float* out, int B,
                      int H, int heads, int T, int W, hipStream_t s, int band) {
  const int dk = H / heads;
  TTS_REQUIRE(dk >= 1 && dk <= ATT_MAX_DK && dk * heads == H, 3, "attention: head size must be <= 128");
  TTS_REQUIRE(T <= ATTN_MAX_T, 3, "attention: more than " + std::to_string(ATTN_MAX_T) + " tokens");
  const size_t lds = attention_lds_bytes(T);
  if (lds > 64 * 1024) {
    static bool raised = false;  // one attribute call per process (the limit is per function)
    if (!raised) {
      TTS_HIP_CHECK(hipFuncSetAttribute((const void*)attention_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)attention_lds_bytes(ATTN_MAX_T)));
      raised = true;
    }
  }
  dim3 grid(ceil_div(T, ATT_QB), heads, B);
  hipLaunchKernelGGL(attention_kernel, grid, dim3(256), lds, s, qkv, mask, W > 0 ? ek : nullptr,
                     W > 0 ? ev : nullptr, out, H, dk, T, W, band);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// Durations (glow_tts.py:350-352, :147): one workgroup per utterance.
//   w = (exp(logw) - 1) * x_mask * length_scale;  w_ceil = max(ceil(w), 1)
//   y_len = max(sum(w_ceil), 1);  o_attn_dur = log(1 + w_ceil * x_mask) * x_mask
// (the sum over frames of token i's alignment row is w_ceil[i] for every unmasked token, since
// y_len >= the cumulative duration of every token).  Sums of integers < 2^24 are exact in fp32.
// ---------------------------------------------------------------------------------------
// vits = 1 (vits.py:1145-1148): w = exp(logw) * x_mask * length_scale, w_ceil = ceil(w) (a token may
// get 0 frames), no o_attn_dur.
__global__ void __launch_bounds__(256) durations_kernel(const float* __restrict__ logw, const float* __restrict__ xm,
                                                        float* __restrict__ w_ceil, int64_t* __restrict__ y_len,
                                                        float* __restrict__ dur, int T, float length_scale, int vits) {
  __shared__ float part[4];
  const int b = blockIdx.x;
  float s = 0.f;
  for (int t = threadIdx.x; t < T; t += 256) {
    const float m = xm[(size_t)b * T + t];
    const float e = expf(logw[(size_t)b * T + t]);
    const float w = (vits ? e : e - 1.f) * m * length_scale;
    const float wc = vits ? ceilf(w) : fmaxf(ceilf(w), 1.f);
    w_ceil[(size_t)b * T + t] = wc;
    if (dur) dur[(size_t)b * T + t] = logf(1.f + wc * m) * m;
    s += wc;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = part[0] + part[1] + part[2] + part[3];
    y_len[b] = (int64_t)fmaxf(tot, 1.f);
  }
}

void launch_durations(const float* logw, const float* xm, float* w_ceil, int64_t* y_len, float* dur, int B, int T,
                      float length_scale, hipStream_t s, int vits) {
  hipLaunchKernelGGL(durations_kernel, dim3(B), dim3(256), 0, s, logw, xm, w_ceil, y_len, dur, T, length_scale, vits);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// Alignment expansion (glow_tts.py:353-361, helpers.py:154-169, compute_outputs :138-148; VITS:
// vits.py:1147-1154).
// Token i covers frames [cum[i-1], cum[i]) with cum the inclusive cumsum of w_ceil; attn[i][j]
// = that indicator * x_mask[i] * y_mask[j], and since each frame is covered by exactly one
// token, y_mean[:, j] = attn^T o_mean is a gather of that token's column (exact: one product
// by 1.0 plus zeros).  One workgroup = 256 frames of one utterance; it rebuilds cum in LDS.
//   z = (y_mean + exp(y_log_scale) * noise * noise_scale) * y_mask
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) expand_kernel(ExpandArgs a) {
  extern __shared__ float cum[];  // [T_x]
  __shared__ float part[256];
  const int b = blockIdx.y;
  const int Tx = a.T_x;
  const float* wc = a.w_ceil + (size_t)b * Tx;
  // inclusive scan: each thread sums a contiguous segment, then a scan over the 256 partials
  const int seg = (Tx + 255) / 256;
  const int lo = threadIdx.x * seg, hi = min(Tx, lo + seg);
  float s = 0.f;
  for (int t = lo; t < hi; ++t) s += wc[t];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const float add = threadIdx.x >= off ? part[threadIdx.x - off] : 0.f;
    __syncthreads();
    part[threadIdx.x] += add;
    __syncthreads();
  }
  float run = threadIdx.x > 0 ? part[threadIdx.x - 1] : 0.f;
  for (int t = lo; t < hi; ++t) {
    run += wc[t];
    cum[t] = run;
  }
  __syncthreads();
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= a.T_y) return;
  const int64_t yl = a.y_len[b];
  const float ym = (int64_t)j < yl ? 1.f : 0.f;
  const float fj = (float)j;
  // first token with cum > j (Glow: cum strictly increases, every w_ceil >= 1; VITS: a token with
  // w_ceil = 0 repeats its predecessor's cum, and the first token past j is the one covering it)
  int l = 0, r = Tx;
  while (l < r) {
    const int mid = (l + r) >> 1;
    if (cum[mid] > fj) r = mid; else l = mid + 1;
  }
  const int i = l;  // == Tx: no token covers frame j
  const float att = (i < Tx) ? a.x_mask[(size_t)b * Tx + i] * ym : 0.f;
  const size_t C = a.C, Ty = a.T_y;
  for (size_t c = 0; c < C; ++c) {
    const float mu = att != 0.f ? a.o_mean[((size_t)b * C + c) * Tx + i] : 0.f;
    const float ls = (att != 0.f && a.o_log_scale) ? a.o_log_scale[((size_t)b * C + c) * Tx + i] : 0.f;
    const size_t o = ((size_t)b * C + c) * Ty + j;
    const float nz = a.noise ? a.noise[o] : 0.f;
    // Glow (glow_tts.py:361): (y_mean + exp(y_log_scale) * noise * noise_scale) * y_mask; VITS
    // (vits.py:1154): m_p + noise * exp(logs_p) * noise_scale, unmasked
    a.z[o] = a.vits ? mu + nz * expf(ls) * a.noise_scale : (mu + expf(ls) * nz * a.noise_scale) * ym;
    if (a.y_mean) a.y_mean[o] = mu;
    if (a.y_log_scale) a.y_log_scale[o] = ls;
  }
  a.y_mask[(size_t)b * Ty + j] = ym;
  if (a.attn) {
    float* at = a.attn + (size_t)b * Tx * Ty + j;
    for (int t = 0; t < Tx; ++t) at[(size_t)t * Ty] = (t == i) ? att : 0.f;
  }
}

void launch_expand(const ExpandArgs& a, int B, hipStream_t s) {
  TTS_REQUIRE(a.T_x <= EXPAND_MAX_TX, 3, "expand: more than " + std::to_string(EXPAND_MAX_TX) + " tokens");
  dim3 grid(ceil_div(a.T_y, 256), B);
  hipLaunchKernelGGL(expand_kernel, grid, dim3(256), sizeof(float) * (size_t)a.T_x, s, a);
  TTS_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// Speaker-conditioned duration predictor input (encoder.py:166-168)
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) dp_input_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                       const float* __restrict__ mask, float* __restrict__ xdp, int H,
                                                       int Cg, int T) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  const int b = blockIdx.z;
  if (t >= T) return;
  const int C = H + Cg;
  const float m = mask[(size_t)b * T + t];
  // x_dp * x_mask with x_dp = cat(x, g.expand(T)); m is 0 or 1, so the product is exact
  const float v = c < H ? x[((size_t)b * H + c) * T + t] : g[(size_t)b * Cg + (c - H)];
  xdp[((size_t)b * C + c) * T + t] = v * m;
}

void launch_dp_input(const float* x, const float* g, const float* mask, float* xdp, int B, int H, int Cg, int T,
                     hipStream_t s) {
  TTS_REQUIRE(B >= 1 && B <= 65535 && H + Cg <= 65535 && T >= 1, 1, "dp_input: bad shape");
  hipLaunchKernelGGL(dp_input_kernel, dim3((T + 255) / 256, H + Cg, B), dim3(256), 0, s, x, g, mask, xdp, H, Cg, T);
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
