// Glow-TTS text side: encoder executor (glow_encoder.cpp) and its kernels (kernels_text.hip).
// Reference: TTS/tts/layers/glow_tts/encoder.py:83-179, transformer.py, duration_predictor.py,
// glow.py:11-67 (prenet), TTS/tts/models/glow_tts.py:342-363 (inference glue).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "common.hpp"
#include "hifigan.hpp"
#include "tts_mi355x.h"

namespace tts {

constexpr int ATTN_MAX_T = 3072;     // tokens per utterance (score rows live in LDS)
constexpr int EXPAND_MAX_TX = 16384;  // tokens per utterance of the alignment expansion (LDS cumsum)

// x [B][H][T] = cat(emb[tok] * scale (He channels), lang [B][H - He] broadcast over T) * mask
// (He = 0: H, no language embedding)
void launch_embed(const int64_t* tok, const int64_t* len, const float* emb, float* x, float* mask, int B, int H,
                  int T, int num_chars, float scale, hipStream_t s, const float* lang = nullptr, int He = 0);
// y = LN_C(a [+ r]) * gamma + beta [relu] * mask (mask may be NULL); y may alias a or r
void launch_layernorm(const float* a, const float* r, const float* gamma, const float* beta, const float* mask,
                      float* y, int B, int C, int T, float eps, bool relu, hipStream_t s);
// gated_conv layer tail: y[c] = (res[c] + LN(a)[c] * sigmoid(LN(a)[c + C/2])) * mask for c < C/2,
// LN over the C channels of a (gamma, beta [C]); y may alias res
void launch_layernorm_glu(const float* a, const float* res, const float* gamma, const float* beta, const float* mask,
                          float* y, int B, int C, int T, float eps, hipStream_t s);
// Conv1dBN tail (res_conv_bn.py:39-44): v = t in [lo, hi) ? relu(a) : 0 (the zero-padded border of
// the unpadded conv); y = v * scale[c] + shift[c] (BatchNorm, eval); then, with res: y = (y + res)
// * mask (the residual block's add and mask, :124-127).  y may alias a.
void launch_bn_act(const float* a, const float* scale, const float* shift, const float* res, const float* mask,
                   float* y, int B, int C, int T, int lo, int hi, hipStream_t s);
// TimeDepthSeparableConv middle (time_depth_sep_conv.py:50-54): u = glu(a) over a's 2C channels,
// v = depthwise conv k (weights [C][k] and bias with norm2 folded in, zero padding (k-1)/2),
// y = v * sigmoid(v)
void launch_glu_dw_swish(const float* a, const float* w, const float* bias, float* y, int B, int C, int T, int k,
                         hipStream_t s);
// out[B][H][T] = multi-head attention of qkv [B][3H][T] (W = 0: no relative embeddings)
// band >= 0: scores with |j - i| > band are -1e4 (input_length, transformer.py:148-150); -1: none
void launch_attention(const float* qkv, const float* mask, const float* ek, const float* ev, float* out, int B,
                      int H, int heads, int T, int W, hipStream_t s, int band = -1);
// xdp[b][c][t] = (c < H ? x[b][c][t] : g[b][c - H]) * mask[b][t]: the speaker-conditioned duration
// predictor's input cat(x, g.expand(T)) (encoder.py:166-168, masked at duration_predictor.py:66)
void launch_dp_input(const float* x, const float* g, const float* mask, float* xdp, int B, int H, int Cg, int T,
                     hipStream_t s);
// vits = 1: the VITS rule (vits.py:1145-1148), w_ceil = ceil(exp(logw) * x_mask * length_scale)
void launch_durations(const float* logw, const float* xm, float* w_ceil, int64_t* y_len, float* dur, int B, int T,
                      float length_scale, hipStream_t s, int vits = 0);

struct ExpandArgs {
  const float* w_ceil;       // [B][T_x]
  const float* x_mask;       // [B][T_x]
  const int64_t* y_len;      // [B]
  const float* o_mean;       // [B][C][T_x]
  const float* o_log_scale;  // [B][C][T_x] or NULL (zeros: mean_only)
  const float* noise;        // [B][C][T_y] or NULL (zeros)
  float noise_scale;
  int C, T_x, T_y;
  float* z;                  // [B][C][T_y]
  float* y_mask;             // [B][T_y]
  float* y_mean;             // [B][C][T_y] or NULL
  float* y_log_scale;        // [B][C][T_y] or NULL
  float* attn;               // [B][T_x][T_y] or NULL
  int vits;                  // 1: z = m_p + noise * exp(logs_p) * noise_scale, unmasked (vits.py:1154)
};
void launch_expand(const ExpandArgs& a, int B, hipStream_t s);

// VITS StochasticDurationPredictor pieces (kernels_vits_text.hip)
// out = gelu(LayerNorm2(sep_conv(x * mask))) (depthwise [C][k], dilation d, zero padding d(k-1)/2)
void launch_dds_sep_ln_gelu(const float* x, const float* mask, const float* w, const float* bias, const float* gamma,
                            const float* beta, float* out, int B, int C, int T, int k, int d, hipStream_t s);
// x += gelu(LayerNorm2(a))
void launch_dds_ln_gelu_add(const float* a, float* x, const float* gamma, const float* beta, int B, int C, int T,
                            hipStream_t s);
void launch_sdp_init(const float* noise, float* z, float noise_scale, int B, int T, hipStream_t s);
void launch_sdp_affine(float* z, const float* tr, const float* ls, const float* mask, float* logw, int B, int T, int p,
                       hipStream_t s);
void launch_sdp_spline(const float* h, float* z, const float* mask, int B, int T, int p, int nb, float tail,
                       float hscale, hipStream_t s);
// Vits.inference glue (kernels_vits_text.hip)
void launch_given_durations(const float* dur, int64_t dur_bstride, float* w_ceil, int64_t* y_len, int B, int T,
                            hipStream_t s);
void launch_mask_slice(const float* z, const float* m, float* out, int B, int C, int T, int T_out, hipStream_t s);
void launch_upsample_z(const float* z, const int64_t* y_len, float* z2, float* m2, int B, int C, int T, int T2,
                       double factor, hipStream_t s);
void launch_embedding_rows(const float* table, const int64_t* ids, int64_t id_stride, float* out, int B, int dim,
                           int num, hipStream_t s);
void launch_l2_normalize(const float* d, float* out, int B, int C, hipStream_t s);
void launch_add_vec_mask(const float* x, const float* v1, const float* v2, const float* m, float* y, int B, int C,
                         int T, hipStream_t s);
void launch_vec_add(const float* a, const float* b, float* out, int n, hipStream_t s);

// emb_channels: width of emb.weight (0 = hidden_channels); less than hidden_channels for the VITS
// TextEncoder with a language embedding, whose transformer runs at hidden + language_emb_dim
std::vector<int64_t> glow_encoder_weight_shapes(const TtsGlowEncoderCfg& c, bool with_dp = true, int emb_channels = 0);
void glow_encoder_validate(const TtsGlowEncoderCfg& c);

class GlowEncoder {
 public:
  // with_dp = false: no duration predictor (its weights are absent from host_weights), the VITS
  // TextEncoder's use of the same RelativePositionTransformer (vits/networks.py:29-100)
  // emb_channels: see glow_encoder_weight_shapes (the embedding is scaled by sqrt(emb_channels))
  GlowEncoder(const TtsGlowEncoderCfg& cfg, const float* const* host_weights, int device, bool with_dp = true,
              int emb_channels = 0);
  ~GlowEncoder();
  GlowEncoder(const GlowEncoder&) = delete;
  GlowEncoder& operator=(const GlowEncoder&) = delete;
  // g: [B][c_in_channels] speaker vector (the reference's g [B][c_in][1]), NULL when c_in_channels == 0
  // x_out [B][H][T] (may be NULL): the encoder state before the heads (x * x_mask); logw may be NULL
  // without a duration predictor
  // lang [B][hidden - emb_channels]: the language embedding appended to every token's embedding
  void forward(const int64_t* tok, const int64_t* len, const float* g, int B, int T, float* x_m, float* x_logs,
               float* logw, float* x_mask, hipStream_t s, Profiler* prof = nullptr, float* x_out = nullptr,
               const float* lang = nullptr);
  int device() const { return device_; }

 private:
  struct Conv {
    int Cin = 0, Cout = 0, K = 1, tile = 0, n_chunks = 0, dil = 1, pad = 0;
    float* w = nullptr;
    float* b = nullptr;
  };
  struct Affine {  // BatchNorm (eval) as y = x * scale + shift
    float* scale = nullptr;
    float* shift = nullptr;
  };
  struct ConvBN {  // residual_conv_bn: conv (k padded to an odd size) -> border zero -> relu -> BN
    Conv conv;
    Affine bn;
    int lo = 0, hi = 0;  // valid output window offsets: [lo, T - hi)
  };
  struct TdsLayer {  // time_depth_separable (BatchNorms folded into the convs)
    Conv time_conv, time_conv2;
    float* dw_w = nullptr;
    float* dw_b = nullptr;
  };
  struct Norm {
    float* gamma = nullptr;
    float* beta = nullptr;
  };
  struct Layer {
    Conv qkv, o, ffn1, ffn2;
    float* ek = nullptr;
    float* ev = nullptr;
    Norm n1, n2;
  };
  void reserve(int B, int T);

  TtsGlowEncoderCfg cfg_;
  int device_;
  bool with_dp_ = true;
  int emb_ch_ = 0;
  float* emb_ = nullptr;
  Conv pre_conv_[3], pre_proj_;
  Norm pre_norm_[3];
  std::vector<Layer> layers_;
  std::vector<Conv> gconv_;        // gated_conv layers
  std::vector<Norm> gnorm_;
  std::vector<ConvBN> rcbn_;       // residual_conv_bn: num_res_blocks x num_conv_blocks
  Conv post_;                      // residual_conv_bn postnet (BatchNorm folded)
  std::vector<TdsLayer> tds_;
  Conv proj_m_, proj_s_, dp1_, dp2_, dp_proj_;
  Norm dpn1_, dpn2_;
  float* arena_ = nullptr;
  float* ws_ = nullptr;
  size_t ws_bytes_ = 0;
};

// ---------------------------------------------------------------------------------------
// VITS text side (vits_text.cpp): TextEncoder on the Glow encoder's transformer, and the
// StochasticDurationPredictor in the reverse (inference) direction.
// ---------------------------------------------------------------------------------------
std::vector<int64_t> vits_text_encoder_weight_shapes(const TtsVitsTextEncoderCfg& c);
void vits_text_encoder_validate(const TtsVitsTextEncoderCfg& c);
TtsGlowEncoderCfg vits_text_encoder_glow_cfg(const TtsVitsTextEncoderCfg& c);

class VitsTextEncoder {
 public:
  VitsTextEncoder(const TtsVitsTextEncoderCfg& cfg, const float* const* host_weights, int device);
  // lang [B][language_emb_dim] (NULL without a language embedding); x [B][hidden + language_emb_dim][T]
  void forward(const int64_t* tok, const int64_t* len, const float* lang, int B, int T, float* x, float* m,
               float* logs, float* x_mask, hipStream_t s, Profiler* prof = nullptr);
  int device() const { return enc_->device(); }

 private:
  TtsVitsTextEncoderCfg cfg_;
  std::unique_ptr<GlowEncoder> enc_;
};

std::vector<int64_t> vits_sdp_weight_shapes(const TtsVitsSdpCfg& c);
void vits_sdp_validate(const TtsVitsSdpCfg& c);

class VitsSdp {
 public:
  VitsSdp(const TtsVitsSdpCfg& cfg, const float* const* host_weights, int device);
  ~VitsSdp();
  VitsSdp(const VitsSdp&) = delete;
  VitsSdp& operator=(const VitsSdp&) = delete;
  // logw [B][1][T] = StochasticDurationPredictor(x, x_mask, g, reverse=True, noise_scale) with the
  // standard normal draw noise [B][2][T] given (stochastic_duration_predictor.py:256-282)
  // lang [B][language_emb_dim] or NULL (cond_lang, :253-254)
  void reverse(const float* x, const float* x_mask, const float* g, const float* lang, const float* noise,
               float noise_scale, int B, int T, float* logw, hipStream_t s, Profiler* prof = nullptr);
  int device() const { return device_; }

 private:
  struct Conv {
    int Cin = 0, Cout = 0, tile = 0, n_chunks = 0;
    float* w = nullptr;
    float* b = nullptr;
  };
  struct Dds {  // DilatedDepthSeparableConv, 3 layers
    float* sep_w[3] = {};
    float* sep_b[3] = {};
    Conv c1x1[3];
    float* n1g[3] = {};
    float* n1b[3] = {};
    float* n2g[3] = {};
    float* n2b[3] = {};
  };
  struct ConvFlow {
    Conv pre, proj;
    Dds dds;
  };
  void reserve(int B, int T);

  TtsVitsSdpCfg cfg_;
  int device_;
  Conv pre_, proj_;
  Dds dds_;
  float* ea_tr_ = nullptr;  // flows.0 (ElementwiseAffine) translation [2], log_scale [2]
  float* ea_ls_ = nullptr;
  std::vector<ConvFlow> flows_;  // flows.1 .. flows.num_flows
  float* cond_w_ = nullptr;      // cond [H][gin], bias [H] (fp32, launch_cond_vec)
  float* cond_b_ = nullptr;
  float* lang_w_ = nullptr;      // cond_lang [H][L], bias [H]
  float* lang_b_ = nullptr;
  float* arena_ = nullptr;
  float* ws_ = nullptr;
  size_t ws_bytes_ = 0;
};

// The deterministic DurationPredictor of VITS with use_sdp=False (vits.py:694-702,
// glow_tts/duration_predictor.py): x = x + cond(g) + cond_lang(lang); [2 x (conv k -> relu -> LayerNorm
// (eps 1e-4))] -> proj (1x1) -> * mask
std::vector<int64_t> vits_dp_weight_shapes(const TtsVitsDpCfg& c);
void vits_dp_validate(const TtsVitsDpCfg& c);

class VitsDp {
 public:
  VitsDp(const TtsVitsDpCfg& cfg, const float* const* host_weights, int device);
  ~VitsDp();
  VitsDp(const VitsDp&) = delete;
  VitsDp& operator=(const VitsDp&) = delete;
  void forward(const float* x, const float* x_mask, const float* g, const float* lang, int B, int T, float* logw,
               hipStream_t s, Profiler* prof = nullptr);
  int device() const { return device_; }

 private:
  struct Conv {
    int Cin = 0, Cout = 0, K = 1, tile = 0, n_chunks = 0;
    float* w = nullptr;
    float* b = nullptr;
  };
  void reserve(int B, int T);

  TtsVitsDpCfg cfg_;
  int device_;
  Conv c1_, c2_, proj_;
  float *n1g_ = nullptr, *n1b_ = nullptr, *n2g_ = nullptr, *n2b_ = nullptr;
  float *cond_w_ = nullptr, *cond_b_ = nullptr, *lang_w_ = nullptr, *lang_b_ = nullptr;
  float* arena_ = nullptr;
  float* ws_ = nullptr;
  size_t ws_bytes_ = 0;
};

}  // namespace tts
