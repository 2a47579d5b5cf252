/*
 * tts_mi355x.h — C-ABI of the MI355X-native mel→waveform path.
 *
 * This library replaces, for inference on gfx950, the PyTorch-ATen compute under two
 * reference modules of Coqui TTS 0.22.0 (paths relative to the reference repo root):
 *
 *   HiFiGAN generator  TTS/vocoder/models/hifigan_generator.py
 *       HifiganGenerator.__init__        :163-234   -> tts_hifigan_create
 *       HifiganGenerator.forward         :236-265   -> tts_hifigan_forward (pad = 0)
 *       HifiganGenerator.inference       :267-282   -> tts_hifigan_forward (pad = inference_padding)
 *       HifiganGenerator.remove_weight_norm :284-291 (weights arrive already folded)
 *   Glow-TTS decoder   TTS/tts/layers/glow_tts/decoder.py
 *       Decoder.__init__                 :68-111    -> tts_glow_decoder_create
 *       Decoder.forward(reverse=True/False) :113-137 -> tts_glow_decoder_forward
 *       Decoder.store_inverse            :139-141   (W^-1 arrives precomputed)
 *   Glow-TTS encoder   TTS/tts/layers/glow_tts/encoder.py (rel_pos_transformer)
 *       Encoder.__init__                 :83-141    -> tts_glow_encoder_create
 *       Encoder.forward                  :143-179   -> tts_glow_encoder_forward
 *   TTS -> vocoder hand-off  TTS/utils/synthesizer.py:412-428 -> tts_mel_handoff
 *   save_wav int16 scaling   TTS/utils/audio/numpy_transforms.py:430-447 -> tts_wav_to_int16
 *   Glow-TTS inference glue  TTS/tts/models/glow_tts.py
 *       GlowTTS.inference durations      :349-351   -> tts_glow_durations
 *       generate_path + compute_outputs + z :352-361 -> tts_glow_expand
 *
 * The reference has no native FFI for this path (it is pure Python over ATen); the Python
 * binding a maintainer adds is the ctypes stub in INTEGRATION.md.
 *
 * Conventions
 *   - All tensors are fp32, contiguous NCW ([batch][channel][time]) device pointers of the
 *     device the handle was created on.  Weights are passed as HOST pointers in the
 *     reference's PyTorch layouts (Conv1d [Cout][Cin][K], ConvTranspose1d [Cin][Cout][K]),
 *     already weight-norm-folded; the library packs them into kernel layouts once.
 *   - Every entry point returns TTS_OK (0) or a TTS_ERR_* code; no C++ exception crosses
 *     the ABI.  tts_last_error() returns the calling thread's last message.
 *   - forward calls are stream-ordered on the given hipStream_t (NULL = default stream),
 *     never synchronise (except *_profiled), never allocate after the first call for a given
 *     (B, T) or smaller (the per-handle workspace grows only).
 *   - A handle may be used from one host thread at a time; distinct handles are independent.
 */
#ifndef TTS_MI355X_H
#define TTS_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TTS_OK 0
#define TTS_ERR_INVALID 1     /* bad argument / shape (reference: ValueError / assert)      */
#define TTS_ERR_HIP 2         /* HIP runtime error                                           */
#define TTS_ERR_UNSUPPORTED 3 /* configuration outside the implemented path                 */
#define TTS_ERR_OOM 4         /* device allocation failed                                   */

/* Arithmetic of the conv contractions (both produce fp32 results from fp32 inputs):
 *   TTS_MATH_FP32     v_mfma_f32_32x32x2_f32, exact fp32 products, fp32 accumulation
 *   TTS_MATH_FP32_X6  each fp32 operand split exactly into 3 bf16 pieces, the 6 significant
 *                     cross products accumulated in fp32 on v_mfma_f32_32x32x16_bf16
 *                     (dropped terms < 2^-26 relative; 2.67x the fp32-MFMA ceiling)
 *   TTS_MATH_FP32_F16X3  each operand, scaled by an exact power of two so its max-abs lies in
 *                     [2^13, 2^14), split into hi = fp16(x) and lo = fp16(x - hi); hi*hi, hi*lo
 *                     and lo*hi accumulated in fp32 on v_mfma_f32_32x32x16_f16 (22 significant
 *                     bits per operand, dropped term ~2^-22 relative; 5.3x the fp32-MFMA
 *                     ceiling).  The
 *                     scales come from max-abs statistics each producing kernel records; the
 *                     HiFiGAN executor runs conv_pre (user input, no statistics) in FP32_X6.
 *                     HiFiGAN, the Glow decoder and the VITS flow; the Glow encoder rejects it
 *                     (TTS_ERR_UNSUPPORTED).
 *   TTS_MATH_BF16     bf16 operands on v_mfma_f32_32x32x16_bf16 with fp32 accumulation (the bf16
 *                     arithmetic of configs 3 / 5; not fp32-faithful: ~2^-9 relative per product).
 *                     The HiFiGAN executor keeps its internal activation planes in HBM as bf16 (one
 *                     rounding per stored plane, as a bf16 PyTorch forward has; the environment
 *                     variable TTS_MI355X_BF16_PLANES=0 at create time keeps them fp32); every tensor
 *                     crossing this ABI stays fp32. */
#define TTS_MATH_FP32 0
#define TTS_MATH_FP32_X6 1
#define TTS_MATH_FP32_F16X3 2
#define TTS_MATH_BF16 3

#define TTS_MAX_UPSAMPLES 8
#define TTS_MAX_KERNELS 4
#define TTS_MAX_DILATIONS 4

/* ------------------------------------------------------------------------------------ */
/* Library                                                                               */
/* ------------------------------------------------------------------------------------ */

/* Last error message of the calling thread ("" if none). */
const char* tts_last_error(void);
/* ABI version (major*100 + minor). */
int tts_abi_version(void);
/* Target the device code was built for ("gfx950"). */
const char* tts_build_target(void);
/* Provenance: "target=gfx950 src=<16 hex>", the first 16 hex digits of the sha256 of the
 * library's sources (tts-3_amd/Makefile HASHED: sorted paths, contents concatenated) at build time. */
const char* tts_build_info(void);

/* ------------------------------------------------------------------------------------ */
/* HiFiGAN generator                                                                     */
/* ------------------------------------------------------------------------------------ */

/* Mirrors HifiganGenerator.__init__ arguments (hifigan_generator.py:163-178). */
typedef struct TtsHifiganCfg {
  int in_channels;                      /* num_mels (setup_generator, vocoder/models/__init__.py:41) */
  int out_channels;                     /* 1 */
  int resblock_type;                    /* 1 = ResBlock1 (:18-105), 2 = ResBlock2 (:108-159) */
  int num_kernels;                      /* len(resblock_kernel_sizes) */
  int resblock_kernel_sizes[TTS_MAX_KERNELS];
  int num_dilations;                    /* len(resblock_dilation_sizes[j]); 3 (type 1) or 2 (type 2) */
  int resblock_dilation_sizes[TTS_MAX_KERNELS][TTS_MAX_DILATIONS];
  int num_upsamples;                    /* len(upsample_factors) */
  int upsample_factors[TTS_MAX_UPSAMPLES];
  int upsample_kernel_sizes[TTS_MAX_UPSAMPLES];
  int upsample_initial_channel;
  int inference_padding;                /* default 5 (:173) */
  int cond_channels;                    /* 0 = no cond_layer (:227-228) */
  int conv_post_bias;                   /* default 1 (:177) */
  int math_mode;                        /* TTS_MATH_FP32 (default), _X6, _F16X3 or TTS_MATH_BF16 */
  int cond_in_each_up_layer;            /* XTTS generator (TTS/tts/layers/xtts/hifigan_decoder.py:199, :276-279):
                                           o = ups[i](o) + conds[i](g) after every upsampling; needs cond_channels */
} TtsHifiganCfg;

/* Number of host weight tensors create() expects, and the element count of tensor idx.
 * Order (state_dict order of the reference module after remove_weight_norm):
 *   conv_pre.weight [C0][in][7], conv_pre.bias [C0]
 *   for i < num_upsamples:  ups.i.weight [C_i][C_i/2][k_i], ups.i.bias [C_i/2]
 *   for r < num_upsamples*num_kernels (resblocks.r):
 *       type 1: convs1.m.weight/bias for m < 3, then convs2.m.weight/bias for m < 3
 *       type 2: convs.m.weight/bias for m < num_dilations
 *   conv_post.weight [out][C_last][7], conv_post.bias [out] (only if conv_post_bias)
 *   cond_layer.weight [C0][cond][1], cond_layer.bias [C0]  (only if cond_channels > 0)
 *   conds.i.weight [C_{i+1}][cond][1], conds.i.bias [C_{i+1}] for i < num_upsamples
 *                                                          (only if cond_in_each_up_layer)
 * with C0 = upsample_initial_channel, C_i = C0 >> i. */
int tts_hifigan_num_weights(const TtsHifiganCfg* cfg);
int64_t tts_hifigan_weight_numel(const TtsHifiganCfg* cfg, int idx);

/* Build a generator on HIP device `device`: validates cfg, packs + uploads weights. */
int tts_hifigan_create(const TtsHifiganCfg* cfg, const float* const* host_weights, int device,
                       void** handle);
int tts_hifigan_destroy(void* handle);

/* Output samples per batch item: prod(upsample_factors) * (T + 2*pad). */
int64_t tts_hifigan_output_length(const void* handle, int T, int pad);
/* Workspace the handle needs for (B, T, pad), and an explicit pre-allocation. */
int64_t tts_hifigan_workspace_bytes(const void* handle, int B, int T, int pad);
int tts_hifigan_reserve(void* handle, int B, int T, int pad);

/* wav[B][out][hop*(T+2*pad)] = G(replicate_pad(mel[B][C][T], pad)).  pad = 0 is
 * HifiganGenerator.forward, pad = inference_padding is .inference (hifigan_generator.py:281).
 * d_g ([B][cond_channels], may be NULL when cond_channels == 0) is the global conditioning
 * vector (the reference's g[B][cond][1], :250-251).
 * Streams: the call is ordered on hip_stream; internally it forks onto the handle's own lane /
 * branch streams and joins back before returning.  Those streams, their events and the handle's
 * workspace are per handle, so one handle must be driven from one caller stream at a time (a
 * second stream must wait for the first call's completion); use one handle per concurrent stream.
 * Non-finite mel values are outside the contract: the kernels build without NaN semantics, so a
 * NaN or inf input yields an unspecified waveform for that utterance (the other utterances of the
 * batch are unaffected: every statistic is per utterance). */
int tts_hifigan_forward(void* handle, const float* d_mel, int B, int C, int T, int pad,
                        const float* d_g, float* d_wav, void* hip_stream);

/* Same computation, with a hipEvent pair around every kernel launch.  Synchronises the
 * stream before returning.  records[i] describes launch i in issue order. */
typedef struct TtsLaunchRecord {
  char name[48];    /* kernel family, e.g. "mrf_conv_k11_c128" */
  double flops;     /* algorithmic FLOPs of this launch (2*MACs, no padding waste) */
  double bytes;     /* compulsory HBM bytes of this launch (inputs + weights + outputs) */
  float ms;         /* measured duration */
} TtsLaunchRecord;
int tts_hifigan_forward_profiled(void* handle, const float* d_mel, int B, int C, int T, int pad,
                                 const float* d_g, float* d_wav, void* hip_stream,
                                 TtsLaunchRecord* records, int max_records, int* n_records);

/* ------------------------------------------------------------------------------------ */
/* Glow-TTS decoder flow (reverse)                                                        */
/* ------------------------------------------------------------------------------------ */

/* Mirrors Decoder.__init__ (decoder.py:68-81). */
typedef struct TtsGlowDecoderCfg {
  int in_channels;         /* 80 (out_channels of GlowTTS) */
  int hidden_channels;     /* 192 (hidden_channels_dec) */
  int kernel_size;         /* 5 */
  int dilation_rate;       /* 1 */
  int num_flow_blocks;     /* 12 */
  int num_coupling_layers; /* 4 */
  int num_splits;          /* 4 */
  int num_squeeze;         /* 2 */
  int sigmoid_scale;       /* 0 */
  int c_in_channels;       /* 0 = unconditioned; > 0: speaker vector size, every WN gets a cond_layer
                              (wavenet.py:64-66, :98-107) */
  int math_mode;           /* TTS_MATH_FP32 (default), _X6, _F16X3 or TTS_MATH_BF16 */
} TtsGlowDecoderCfg;

/* Host weight order, per flow block b < num_flow_blocks (flows 3b, 3b+1, 3b+2):
 *   actnorm.logs [C2], actnorm.bias [C2]                          (C2 = in*num_squeeze)
 *   invconv.weight_inv [S][S]  (torch.inverse(weight), glow.py:139-141)
 *   invconv.weight [S][S]      (the forward direction, glow.py:126-130; since ABI 112)
 *   coupling.start.weight [H][C2/2] (weight-norm folded), coupling.start.bias [H]
 *   if c_in_channels: wn.cond_layer.weight [2*H*L][c_in] (weight-norm folded), bias [2*H*L]
 *   for l < L: wn.in_layers.l.weight [2H][H][k], wn.in_layers.l.bias [2H]
 *              wn.res_skip_layers.l.weight [l<L-1 ? 2H : H][H], bias
 *   coupling.end.weight [C2][H], coupling.end.bias [C2] */
int tts_glow_decoder_num_weights(const TtsGlowDecoderCfg* cfg);
int64_t tts_glow_decoder_weight_numel(const TtsGlowDecoderCfg* cfg, int idx);
int tts_glow_decoder_create(const TtsGlowDecoderCfg* cfg, const float* const* host_weights,
                            int device, void** handle);
int tts_glow_decoder_destroy(void* handle);
/* (y, logdet) = Decoder.forward(x, x_mask, g, reverse=reverse) (decoder.py:113-137): y[B][C][T'] with
 * T' = T rounded down to a multiple of num_squeeze (decoder.py:19); d_mask is [B][1][T] (0/1); d_g is
 * the speaker vector [B][c_in_channels] (the reference's g [B][c_in][1]), NULL when c_in_channels == 0.
 * reverse = 1: the inference direction (glow_tts.py:363), d_logdet unused (the reference returns None).
 * reverse = 0: the flows in order (GlowTTS.decoder_inference, glow_tts.py:333); d_logdet [B] fp32
 * receives logdet_tot (ActNorm + InvConvNear + coupling terms, summed per utterance in fp64 in a fixed
 * order), or is NULL to skip it.  Since ABI 112 (d_logdet added). */
int tts_glow_decoder_forward(void* handle, const float* d_x, const float* d_mask, const float* d_g, int B,
                             int C, int T, int reverse, float* d_y, float* d_logdet, void* hip_stream);
/* Same with a hipEvent pair around every launch (synchronises; see tts_hifigan_forward_profiled). */
int tts_glow_decoder_forward_profiled(void* handle, const float* d_x, const float* d_mask, const float* d_g,
                                      int B, int C, int T, int reverse, float* d_y, float* d_logdet,
                                      void* hip_stream, TtsLaunchRecord* records, int max_records,
                                      int* n_records);

/* ------------------------------------------------------------------------------------ */
/* Glow-TTS encoder (rel_pos_transformer) and the GlowTTS.inference glue                   */
/* ------------------------------------------------------------------------------------ */

/* Mirrors Encoder.__init__ (encoder.py:83-141) for encoder_type "rel_pos_transformer", with the
 * transformer's encoder_params flattened (transformer.py:345-357; GlowTTS passes
 * in = out = hidden = hidden_channels_enc). */
typedef struct TtsGlowEncoderCfg {
  int num_chars;            /* embedding rows */
  int out_channels;         /* 80 (mel channels) */
  int hidden_channels;      /* 192 (hidden_channels_enc) */
  int hidden_channels_dp;   /* 256 */
  int hidden_channels_ffn;  /* 768 (encoder_params) */
  int num_heads;            /* 2 */
  int num_layers;           /* 6 */
  int kernel_size;          /* 3: FFN conv kernel (encoder_params) */
  int rel_attn_window_size; /* 0 = None (Glow-TTS default); 4 in the VITS-style encoders */
  int mean_only;            /* 1 (GlowTTSConfig default): x_logs = zeros */
  int use_prenet;           /* 1: ResidualConv1dLayerNormBlock(k5, 3 layers) before the transformer */
  int c_in_channels;        /* 0 = unconditioned; > 0: speaker vector size, the duration predictor reads
                               cat(x, g.expand(T)) (encoder.py:166-168; GlowTTS c_in_channels) */
  int math_mode;            /* TTS_MATH_FP32 (default), TTS_MATH_FP32_X6 or TTS_MATH_BF16 */
  /* since ABI 113: the other encoder types of encoder.py:97-123 (0 = rel_pos_transformer) */
  int encoder_type;         /* TTS_ENC_REL_POS_TRANSFORMER / _GATED_CONV / _RESIDUAL_CONV_BN / _TIME_DEPTH_SEPARABLE */
  int num_conv_blocks;      /* residual_conv_bn: convs per residual block (2) */
  int num_res_blocks;       /* residual_conv_bn: residual blocks (13) = entries of dilations */
  int dilations[32];        /* residual_conv_bn: dilation of each residual block */
  int layer_norm_type;      /* rel_pos_transformer: 1 (LayerNorm, eps 1e-4; 0 = 1) or 2 (LayerNorm2, eps 1e-5) */
  int has_input_length;     /* rel_pos_transformer: 1 when input_length is set (transformer.py:148-150): */
  int input_length;         /*   scores with |i - j| > input_length are -1e4 (block-limited attention) */
} TtsGlowEncoderCfg;

#define TTS_ENC_REL_POS_TRANSFORMER 0
#define TTS_ENC_GATED_CONV 1          /* GatedConvBlock(H, kernel_size, dropout, num_layers), no prenet */
#define TTS_ENC_RESIDUAL_CONV_BN 2    /* ResidualConv1dBNBlock + postnet conv1x1 -> BatchNorm */
#define TTS_ENC_TIME_DEPTH_SEPARABLE 3 /* TimeDepthSeparableConvBlock (prenet as rel_pos) */

/* Host weight order (R = 2*rel_attn_window_size + 1, dk = hidden/num_heads, H = hidden, k =
 * kernel_size; a BatchNorm "BN(C)" is weight [C], bias [C], running_mean [C], running_var [C]):
 *   emb.weight [num_chars][H]
 *   if use_prenet (rel_pos_transformer, time_depth_separable):
 *                  for l < 3: prenet.conv_layers.l.weight [H][H][5], bias [H],
 *                             prenet.norm_layers.l.gamma [H], beta [H]
 *                  prenet.proj.weight [H][H][1], bias [H]
 *   gated_conv, for l < num_layers: encoder.conv_layers.l.weight [2H][H][k], bias [2H],
 *                                   encoder.norm_layers.l.gamma [2H], beta [2H]
 *   residual_conv_bn, for i < num_res_blocks, j < num_conv_blocks:
 *       encoder.res_blocks.i.conv_bn_blocks.j.conv1d.weight [H][H][k], bias [H], .norm BN(H)
 *     then postnet.0.weight [H][H][1], bias [H], postnet.1 BN(H)
 *   time_depth_separable, for l < num_layers: encoder.layers.l.time_conv.weight [2H][H][1], bias [2H],
 *       norm1 BN(2H), depth_conv.weight [H][1][k], bias [H], norm2 BN(H),
 *       time_conv2.weight [H][H][1], bias [H], norm3 BN(H)
 *   rel_pos_transformer, for l < num_layers (encoder.*):
 *       attn_layers.l.conv_q.weight [H][H][1], bias, conv_k.*, conv_v.*, conv_o.*
 *       if rel_attn_window_size: attn_layers.l.emb_rel_k [1][R][dk], emb_rel_v [1][R][dk]
 *       norm_layers_1.l.gamma [H], beta [H]
 *       ffn_layers.l.conv_1.weight [ffn][H][k], bias [ffn], conv_2.weight [H][ffn][k], bias [H]
 *       norm_layers_2.l.gamma [H], beta [H]
 *   proj_m.weight [out][H][1], bias [out];  if !mean_only: proj_s.weight, bias
 *   duration_predictor.conv_1.weight [dp][H + c_in_channels][3], bias, norm_1.gamma, beta,
 *                      conv_2.weight [dp][dp][3], bias, norm_2.gamma, beta,
 *                      proj.weight [1][dp][1], proj.bias [1] */
int tts_glow_encoder_num_weights(const TtsGlowEncoderCfg* cfg);
int64_t tts_glow_encoder_weight_numel(const TtsGlowEncoderCfg* cfg, int idx);
int tts_glow_encoder_create(const TtsGlowEncoderCfg* cfg, const float* const* host_weights, int device,
                            void** handle);
int tts_glow_encoder_destroy(void* handle);
/* (x_m, x_logs, logw, x_mask) = Encoder.forward(tokens, lengths, g): tokens [B][T] int64 (ids in
 * [0, num_chars); padded positions may hold any id), lengths [B] int64, d_g the speaker vector
 * [B][c_in_channels] (the reference's g [B][c_in][1]; NULL when c_in_channels == 0); outputs x_m,
 * x_logs [B][out][T], logw [B][1][T], x_mask [B][1][T].  x_logs may be NULL when mean_only.
 * T <= 3072. */
int tts_glow_encoder_forward(void* handle, const int64_t* d_tokens, const int64_t* d_lengths, const float* d_g,
                             int B, int T, float* d_x_m, float* d_x_logs, float* d_logw, float* d_x_mask,
                             void* hip_stream);
int tts_glow_encoder_forward_profiled(void* handle, const int64_t* d_tokens, const int64_t* d_lengths,
                                      const float* d_g, int B, int T, float* d_x_m, float* d_x_logs, float* d_logw,
                                      float* d_x_mask,
                                      void* hip_stream, TtsLaunchRecord* records, int max_records,
                                      int* n_records);

/* glow_tts.py:350-352 and :147: w_ceil[B][1][T_x] = max(ceil((exp(logw) - 1) * x_mask *
 * length_scale), 1); y_lengths[B] (int64) = max(sum(w_ceil), 1); o_attn_dur [B][1][T_x] =
 * log(1 + sum_j attn[i][j]) * x_mask (may be NULL).  The caller reads y_lengths back to size
 * T_y = max(y_lengths) (the reference's sequence_mask(y_lengths, None), glow_tts.py:353). */
int tts_glow_durations(const float* d_logw, const float* d_x_mask, int B, int T_x, float length_scale,
                       float* d_w_ceil, int64_t* d_y_lengths, float* d_o_attn_dur, void* hip_stream);
/* glow_tts.py:353-361: y_mask [B][1][T_y]; attn = generate_path(w_ceil, x_mask*y_mask)
 * (helpers.py:154-169); y_mean = attn^T o_mean, y_log_scale = attn^T o_log_scale (compute_outputs
 * :138-145); z = (y_mean + exp(y_log_scale) * noise * noise_scale) * y_mask.
 * o_log_scale NULL = zeros (mean_only); noise [B][C][T_y] (torch.randn_like drawn by the caller)
 * NULL = zeros.  y_mean, y_log_scale [B][C][T_y] and attn [B][T_x][T_y] may be NULL.
 * T_y must be >= max(y_lengths).  T_x <= 16384. */
int tts_glow_expand(const float* d_w_ceil, const float* d_x_mask, const int64_t* d_y_lengths,
                    const float* d_o_mean, const float* d_o_log_scale, const float* d_noise, float noise_scale,
                    int B, int C, int T_x, int T_y, float* d_z, float* d_y_mask, float* d_y_mean,
                    float* d_y_log_scale, float* d_attn, void* hip_stream);

/* ------------------------------------------------------------------------------------ */
/* TTS -> vocoder hand-off and the int16 wav writer                                       */
/* ------------------------------------------------------------------------------------ */

/* AudioProcessor normalisation fields (processor.py:259-336; BaseAudioConfig defaults
 * shared_configs.py:126-154), as the Python values (they are rounded to fp32 where numpy
 * would).  d_mel_mean / d_mel_scale: device fp64 [C] mel_scaler statistics (mean-var
 * normalisation, processor.py:275-277 / :316-318), or NULL for range normalisation. */
typedef struct TtsAudioNormCfg {
  int signal_norm;     /* 0: identity */
  int symmetric_norm;
  int clip_norm;
  double max_norm;
  double min_level_db;
  double ref_level_db;
  const double* d_mel_mean;
  const double* d_mel_scale;
} TtsAudioNormCfg;

/* Synthesizer hand-off (synthesizer.py:412-428), batched: out[B][C][T_out] =
 * interpolate(vocoder_ap.normalize(tts_ap.denormalize(in))).  in: model_outputs [B][T][C]
 * (time_major = 1) or [B][C][T].  T_out == T: no resampling; otherwise the time axis is resampled
 * like interpolate_vocoder_input (vocoder/utils/generic_utils.py:11-29: bilinear,
 * align_corners=False, recompute_scale_factor=True; pass T_out = floor(T * sr_voc / sr_tts) and
 * src_scale = 0, which maps with T / T_out).  src_scale > 0 maps output j to source
 * src_scale * (j + 0.5) - 0.5 instead: F.interpolate(mode="linear", scale_factor=s) without
 * recompute_scale_factor passes src_scale = 1/s (the XTTS latent upsampling,
 * xtts/hifigan_decoder.py:688-698).  denorm / norm may be NULL (identity). */
int tts_mel_handoff(const float* d_in, int B, int T, int C, int time_major, const TtsAudioNormCfg* denorm,
                    const TtsAudioNormCfg* norm, int T_out, float src_scale, float* d_out, void* hip_stream);
/* save_wav scaling (numpy_transforms.py:436-438): out = int16(wav * (32767 / max(0.01, max|wav|)))
 * per utterance.  wav [B][n] fp32; d_lengths [B] (int64, NULL = n) limits each utterance (samples
 * beyond it are written as 0); d_scratch: B x uint32 of device memory. */
int tts_wav_to_int16(const float* d_wav, int B, int64_t n, const int64_t* d_lengths, unsigned* d_scratch,
                     int16_t* d_out, void* hip_stream);

/* ------------------------------------------------------------------------------------ */
/* VITS flow: ResidualCouplingBlocks, reverse (TTS/tts/layers/vits/networks.py:169-232)     */
/* ------------------------------------------------------------------------------------ */

/* Mirrors ResidualCouplingBlocks.__init__ (networks.py:169-202; VITS builds it at
 * vits.py:675-682 with mean-only blocks). */
typedef struct TtsVitsFlowCfg {
  int channels;        /* 192 (hidden_channels) */
  int hidden_channels; /* 192 */
  int kernel_size;     /* 5 (kernel_size_flow) */
  int dilation_rate;   /* 1 (dilation_rate_flow) */
  int num_layers;      /* 4 (num_layers_flow) */
  int num_flows;       /* 4 */
  int cond_channels;   /* speaker embedding size, 0 = none (embedded_speaker_dim) */
  int math_mode;       /* TTS_MATH_FP32 (default), _X6, _F16X3 or TTS_MATH_BF16 */
} TtsVitsFlowCfg;

/* Host weight order, per flow f < num_flows (weight norm folded: w = g * v / ||v||):
 *   pre.weight [H][C/2], pre.bias [H]
 *   for l < L: enc.in_layers.l.weight [2H][H][k], enc.in_layers.l.bias [2H]
 *   for l < L: enc.res_skip_layers.l.weight [l<L-1 ? 2H : H][H], bias
 *   if cond_channels: enc.cond_layer.weight [2*H*L][cond_channels], enc.cond_layer.bias [2*H*L]
 *   post.weight [C/2][H], post.bias [C/2] */
int tts_vits_flow_num_weights(const TtsVitsFlowCfg* cfg);
int64_t tts_vits_flow_weight_numel(const TtsVitsFlowCfg* cfg, int index);
int tts_vits_flow_create(const TtsVitsFlowCfg* cfg, const float* const* host_weights, int device,
                         void** handle);
int tts_vits_flow_destroy(void* handle);
/* y[B][C][T] = ResidualCouplingBlocks(x, mask, g, reverse=reverse) (networks.py:217-232).  x, y:
 * [B][C][T] fp32 (y may equal x: in place), mask: [B][T], g: [B][cond_channels] (NULL when
 * cond_channels == 0).  reverse = 1: the inference direction (vits.py:1155); reverse = 0: the
 * posterior side of voice conversion, z_p = flow(z, y_mask, g) (vits.py:1226; since ABI 112). */
int tts_vits_flow_forward(void* handle, const float* d_x, const float* d_mask, const float* d_g, int B,
                          int C, int T, int reverse, float* d_y, void* hip_stream);
int tts_vits_flow_forward_profiled(void* handle, const float* d_x, const float* d_mask, const float* d_g,
                                   int B, int C, int T, int reverse, float* d_y, void* hip_stream,
                                   TtsLaunchRecord* records, int max_records, int* n_records);

/* ------------------------------------------------------------------------------------ */
/* VITS posterior encoder (TTS/tts/layers/vits/networks.py:235-288), since ABI 112        */
/* ------------------------------------------------------------------------------------ */

/* Mirrors PosteriorEncoder.__init__ (networks.py:236-273); VITS builds it from the linear
 * spectrogram (vits.py:594-602: in = fft_size/2 + 1 = 513, out = hidden = 192, k5, d1, 16 layers). */
typedef struct TtsVitsPosteriorCfg {
  int in_channels;     /* 513 */
  int out_channels;    /* 192 */
  int hidden_channels; /* 192 */
  int kernel_size;     /* 5 */
  int dilation_rate;   /* 1 */
  int num_layers;      /* 16 */
  int cond_channels;   /* speaker embedding size, 0 = none */
  int math_mode;       /* TTS_MATH_* (f16x3 / fp32x6 / fp32 / bf16) */
} TtsVitsPosteriorCfg;

/* Host weight order (weight norm folded):
 *   pre.weight [H][in], pre.bias [H]
 *   for l < L: enc.in_layers.l.weight [2H][H][k], bias [2H]
 *   for l < L: enc.res_skip_layers.l.weight [l<L-1 ? 2H : H][H], bias
 *   if cond_channels: enc.cond_layer.weight [2*H*L][cond_channels], bias [2*H*L]
 *   proj.weight [2*out][H], proj.bias [2*out] */
int tts_vits_posterior_num_weights(const TtsVitsPosteriorCfg* cfg);
int64_t tts_vits_posterior_weight_numel(const TtsVitsPosteriorCfg* cfg, int index);
int tts_vits_posterior_create(const TtsVitsPosteriorCfg* cfg, const float* const* host_weights, int device,
                              void** handle);
int tts_vits_posterior_destroy(void* handle);
/* (z, m, logs) = PosteriorEncoder.forward(x, x_lengths, g)[:3] (networks.py:275-288): x [B][in][T],
 * mask [B][T] (sequence_mask(x_lengths)), g [B][cond_channels] or NULL, eps [B][out][T] the standard
 * normal sample the reference draws with torch.randn_like (NULL: zero noise, z = m); z, m, logs
 * [B][out][T] fp32 (m or logs may be NULL when not wanted). */
int tts_vits_posterior_forward(void* handle, const float* d_x, const float* d_mask, const float* d_g,
                               const float* d_eps, int B, int C, int T, float* d_z, float* d_m, float* d_logs,
                               void* hip_stream);
int tts_vits_posterior_forward_profiled(void* handle, const float* d_x, const float* d_mask, const float* d_g,
                                        const float* d_eps, int B, int C, int T, float* d_z, float* d_m,
                                        float* d_logs, void* hip_stream, TtsLaunchRecord* records,
                                        int max_records, int* n_records);

/* ------------------------------------------------------------------------------------ */
/* VITS text side of Vits.inference (TTS/tts/models/vits.py:1121-1155), since ABI 114       */
/* ------------------------------------------------------------------------------------ */

/* Mirrors TextEncoder.__init__ (TTS/tts/layers/vits/networks.py:29-81; VITS builds it at
 * vits.py:653-663 with out = hidden = hidden_channels).  The transformer is the Glow encoder's
 * RelativePositionTransformer with layer_norm_type "2" and rel_attn_window_size 4. */
typedef struct TtsVitsTextEncoderCfg {
  int n_vocab;             /* num_chars */
  int out_channels;        /* 192 */
  int hidden_channels;     /* 192 */
  int hidden_channels_ffn; /* 768 */
  int num_heads;           /* 2 */
  int num_layers;          /* 6 */
  int kernel_size;         /* 3 (FFN) */
  int language_emb_dim;    /* 0, or L > 0 (YourTTS): the transformer runs at H + L channels (since ABI 115) */
  int math_mode;           /* TTS_MATH_FP32, _X6 or TTS_MATH_BF16 */
} TtsVitsTextEncoderCfg;

/* Host weight order, with E = H + language_emb_dim (networks.py:63-64): emb.weight [n_vocab][H]; per
 * layer l: encoder.attn_layers.l.conv_q/k/v/o (weight [E][E][1], bias [E]), emb_rel_k [1][9][dk],
 * emb_rel_v [1][9][dk] (dk = E / num_heads), encoder.norm_layers_1.l gamma [E], beta [E],
 * encoder.ffn_layers.l.conv_1 (weight [ffn][E][k], bias), conv_2 (weight [E][ffn][k], bias),
 * encoder.norm_layers_2.l gamma, beta; proj.weight [2 out][E][1], proj.bias [2 out]. */
int tts_vits_text_encoder_num_weights(const TtsVitsTextEncoderCfg* cfg);
int64_t tts_vits_text_encoder_weight_numel(const TtsVitsTextEncoderCfg* cfg, int index);
int tts_vits_text_encoder_create(const TtsVitsTextEncoderCfg* cfg, const float* const* host_weights, int device,
                                 void** handle);
int tts_vits_text_encoder_destroy(void* handle);
/* (x, m, logs, x_mask) = TextEncoder.forward(tokens, lengths, lang_emb) (networks.py:83-100): tokens
 * [B][T] int64, lengths [B] int64, lang_emb [B][language_emb_dim] (NULL when language_emb_dim = 0;
 * the reference's [B][L][1]); x [B][E][T], m and logs [B][out][T], x_mask [B][1][T].  T <= 3072. */
int tts_vits_text_encoder_forward(void* handle, const int64_t* d_tokens, const int64_t* d_lengths,
                                  const float* d_lang_emb, int B, int T, float* d_x, float* d_m, float* d_logs,
                                  float* d_x_mask, void* hip_stream);
int tts_vits_text_encoder_forward_profiled(void* handle, const int64_t* d_tokens, const int64_t* d_lengths,
                                           const float* d_lang_emb, int B, int T, float* d_x, float* d_m,
                                           float* d_logs, float* d_x_mask, void* hip_stream,
                                           TtsLaunchRecord* records, int max_records, int* n_records);

/* Mirrors StochasticDurationPredictor.__init__ (TTS/tts/layers/vits/stochastic_duration_predictor.py:
 * 185-227; VITS: in = hidden_channels, hidden 192, kernel 3, 4 flows, cond = embedded_speaker_dim when
 * condition_dp_on_speaker, vits.py:684-692).  ConvFlows use 10 bins, tail bound 5 (:96-104). */
typedef struct TtsVitsSdpCfg {
  int in_channels;      /* 192 (+ language_emb_dim: the text encoder's x width, :191-192) */
  int hidden_channels;  /* 192 (<= 512) */
  int kernel_size;      /* 3 */
  int num_flows;        /* 4 */
  int cond_channels;    /* 0 = no cond layer */
  int language_emb_dim; /* 0 = no cond_lang layer (since ABI 115) */
  int math_mode;        /* TTS_MATH_FP32, _X6 or TTS_MATH_BF16 (its 1x1 convs) */
} TtsVitsSdpCfg;

/* Host weight order (the inference-side tensors in state_dict order; post_* are training-only):
 *   pre.weight [H][in][1], pre.bias [H]
 *   DDS(convs): convs_sep.i.weight [H][1][k], bias [H] (i < 3); convs_1x1.i.weight [H][H][1], bias [H];
 *               norms_1.i.gamma [H], beta [H]; norms_2.i.gamma [H], beta [H]
 *   proj.weight [H][H][1], proj.bias [H]
 *   flows.0.translation [2][1], flows.0.log_scale [2][1]
 *   for f = 1 .. num_flows: flows.f.pre.weight [H][1][1], bias [H]; DDS(flows.f.convs);
 *                           flows.f.proj.weight [29][H][1], bias [29]
 *   if cond_channels: cond.weight [H][cond][1], cond.bias [H]
 *   if language_emb_dim: cond_lang.weight [H][L][1], cond_lang.bias [H] */
int tts_vits_sdp_num_weights(const TtsVitsSdpCfg* cfg);
int64_t tts_vits_sdp_weight_numel(const TtsVitsSdpCfg* cfg, int index);
int tts_vits_sdp_create(const TtsVitsSdpCfg* cfg, const float* const* host_weights, int device, void** handle);
int tts_vits_sdp_destroy(void* handle);
/* logw [B][1][T] = StochasticDurationPredictor.forward(x, x_mask, g=g, lang_emb=lang, reverse=True,
 * noise_scale) (:242-282): x [B][in][T], x_mask [B][1][T], g [B][cond_channels] or NULL, lang
 * [B][language_emb_dim] or NULL (x = pre(x) + cond(g) + cond_lang(lang), :249-254), noise [B][2][T]
 * the standard normal draw of :277 (torch.randn(B, 2, T); NULL = zeros). */
int tts_vits_sdp_reverse(void* handle, const float* d_x, const float* d_x_mask, const float* d_g,
                         const float* d_lang_emb, const float* d_noise, float noise_scale, int B, int T,
                         float* d_logw, void* hip_stream);
int tts_vits_sdp_reverse_profiled(void* handle, const float* d_x, const float* d_x_mask, const float* d_g,
                                  const float* d_lang_emb, const float* d_noise, float noise_scale, int B, int T,
                                  float* d_logw, void* hip_stream, TtsLaunchRecord* records, int max_records,
                                  int* n_records);

/* Mirrors the deterministic DurationPredictor VITS builds with use_sdp=False (vits.py:694-702:
 * TTS/tts/layers/glow_tts/duration_predictor.py:6-44 with in = hidden_channels, filter 256, kernel 3,
 * cond = embedded_speaker_dim, language_emb_dim), since ABI 115. */
typedef struct TtsVitsDpCfg {
  int in_channels;      /* hidden_channels (192); the module adds language_emb_dim itself (:28-29) */
  int hidden_channels;  /* filter channels, 256 */
  int kernel_size;      /* 3 (odd, <= 11) */
  int cond_channels;    /* 0 = no cond layer */
  int language_emb_dim; /* 0 = no cond_lang layer */
  int math_mode;        /* TTS_MATH_FP32, _X6 or TTS_MATH_BF16 */
} TtsVitsDpCfg;

/* Host weight order (state_dict order), I = in_channels + language_emb_dim, F = hidden_channels:
 *   conv_1.weight [F][I][k], conv_1.bias [F]; norm_1.gamma [F], norm_1.beta [F];
 *   conv_2.weight [F][F][k], conv_2.bias [F]; norm_2.gamma [F], norm_2.beta [F];
 *   proj.weight [1][F][1], proj.bias [1];
 *   if cond_channels: cond.weight [I][cond][1], cond.bias [I];
 *   if language_emb_dim: cond_lang.weight [I][L][1], cond_lang.bias [I] */
int tts_vits_dp_num_weights(const TtsVitsDpCfg* cfg);
int64_t tts_vits_dp_weight_numel(const TtsVitsDpCfg* cfg, int index);
int tts_vits_dp_create(const TtsVitsDpCfg* cfg, const float* const* host_weights, int device, void** handle);
int tts_vits_dp_destroy(void* handle);
/* logw [B][1][T] = DurationPredictor.forward(x, x_mask, g, lang_emb) (duration_predictor.py:49-68):
 * x [B][I][T], x_mask [B][1][T], g [B][cond_channels] or NULL, lang [B][language_emb_dim] or NULL. */
int tts_vits_dp_forward(void* handle, const float* d_x, const float* d_x_mask, const float* d_g,
                        const float* d_lang_emb, int B, int T, float* d_logw, void* hip_stream);
int tts_vits_dp_forward_profiled(void* handle, const float* d_x, const float* d_x_mask, const float* d_g,
                                 const float* d_lang_emb, int B, int T, float* d_logw, void* hip_stream,
                                 TtsLaunchRecord* records, int max_records, int* n_records);

/* vits.py:1145-1148: w_ceil [B][1][T_x] = ceil(exp(logw) * x_mask * length_scale); y_lengths [B]
 * (int64) = max(sum(w_ceil), 1).  The caller reads y_lengths back for T_y = max(y_lengths). */
int tts_vits_durations(const float* d_logw, const float* d_x_mask, int B, int T_x, float length_scale,
                       float* d_w_ceil, int64_t* d_y_lengths, void* hip_stream);
/* vits.py:1147-1154: y_mask [B][1][T_y]; attn = generate_path(w_ceil, x_mask * y_mask) [B][T_x][T_y]
 * (may be NULL); m_p' = attn^T m_p, logs_p' = attn^T logs_p ([B][C][T_y], may be NULL);
 * z_p = m_p' + noise * exp(logs_p') * noise_scale (not masked; noise [B][C][T_y] NULL = zeros).
 * T_y >= max(y_lengths), T_x <= 16384. */
int tts_vits_expand(const float* d_w_ceil, const float* d_x_mask, const int64_t* d_y_lengths, const float* d_m_p,
                    const float* d_logs_p, const float* d_noise, float noise_scale, int B, int C, int T_x, int T_y,
                    float* d_z_p, float* d_y_mask, float* d_m_p_out, float* d_logs_p_out, float* d_attn,
                    void* hip_stream);

/* The rest of Vits.inference's glue on the device (since ABI 115).
 * Given durations (vits.py:1141-1146): w = durations.unsqueeze(0); w_ceil [B][1][T_x] = ceil(w) (no
 * mask, no length_scale), y_lengths [B] = max(sum(w_ceil), 1); durations [T_x] shared by every
 * utterance (dur_bstride 0) or [B][T_x] (dur_bstride T_x). */
int tts_vits_durations_given(const float* d_durations, int64_t dur_bstride, int B, int T_x, float* d_w_ceil,
                             int64_t* d_y_lengths, void* hip_stream);
/* (z * y_mask)[:, :, :T_out] (vits.py:1161): z [B][C][T] (batch stride C * T), y_mask [B][1][T],
 * out [B][C][T_out], 1 <= T_out <= T. */
int tts_vits_mask_slice(const float* d_z, const float* d_y_mask, int B, int C, int T, int T_out, float* d_out,
                        void* hip_stream);
/* upsampling_z (vits.py:944-959, encoder_sample_rate with interpolate_z): z2 [B][C][T2] =
 * F.interpolate(z [B][C][T], scale_factor=[factor], mode="linear"), T2 = floor(T * factor);
 * y_mask2 [B][1][T2] = sequence_mask(y_lengths * factor) (may be NULL).  The reference's product
 * z2 * y_mask2 needs ceil(max(y_lengths) * factor) == T2; the caller checks it. */
int tts_vits_upsample_z(const float* d_z, const int64_t* d_y_lengths, int B, int C, int T, double factor, int T2,
                        float* d_z2, float* d_y_mask2, void* hip_stream);
/* out [B][dim] = table[ids[b * id_stride]] (nn.Embedding rows: emb_g(sid), emb_l(lid)); ids are
 * clamped to [0, num) (the reference raises IndexError; a device kernel cannot). */
int tts_embedding_rows(const float* d_table, int num, int dim, const int64_t* d_ids, int64_t id_stride, int B,
                       float* d_out, void* hip_stream);
/* out [B][C] = d / max(||d||_2, 1e-12) per row (F.normalize(d_vectors), vits.py:884-886). */
int tts_l2_normalize_rows(const float* d_in, int B, int C, float* d_out, void* hip_stream);

/* ------------------------------------------------------------------------------------ */
/* Single-op entry points (test / tuning surface).  These pack the host weights into a     */
/* temporary device buffer on every call and synchronise; they are not the hot path.        */
/* ------------------------------------------------------------------------------------ */

/* y = epilogue(conv1d(act_in(x_padded), w) + b), "same" conv: pad = dil*(K-1)/2.
 * x_padded[t] = x[clamp(t - rep_pad, 0, Tin-1)] for t in [0, Tin + 2*rep_pad).
 * act_in / act_out = leaky_relu with the given slope (1.0 = identity).
 * Epilogue: v = act_out(acc + b) + (res ? res : 0);
 *   zmode 0: y = v;  1: z = v;  2: z = z + v;  3: z = (z + v) / zdiv. */
typedef struct TtsConv1dDesc {
  int B, Cin, Cout, Tin, K, dil, rep_pad;
  float in_slope, out_slope;
  int zmode;
  float zdiv;
  int math_mode; /* TTS_MATH_FP32 / TTS_MATH_FP32_X6 / TTS_MATH_FP32_F16X3 */
} TtsConv1dDesc;
int tts_op_conv1d(const TtsConv1dDesc* d, const float* d_x, const float* h_w, const float* h_b,
                  const float* d_res, float* d_y, float* d_z, void* hip_stream);

/* Tuning: same computation with an explicit tile configuration (tile < 0: automatic), launched
 * `reps` times; *ms receives the mean kernel time (hipEvents on hip_stream). */
int tts_op_conv1d_bench(const TtsConv1dDesc* d, const float* d_x, const float* h_w, const float* h_b,
                        const float* d_res, float* d_y, float* d_z, int tile, int reps, float* ms,
                        void* hip_stream);
/* Number of conv1d tile configurations compiled into the library for a math mode. */
int tts_op_conv1d_num_tiles(int math_mode);

/* y = conv_transpose1d(act_in(x), w[Cin][Cout][K], b, stride, padding=(K-stride)/2);
 * requires K == 2*stride (every HiFiGAN config) with stride 2, 4 or 8; math_mode TTS_MATH_*
 * (the split modes run the polyphase K=2 conv form of the executor). */
int tts_op_conv_transpose1d(const float* d_x, int B, int Cin, int Tin, const float* h_w,
                            const float* h_b, int Cout, int K, int stride, float in_slope,
                            int math_mode, float* d_y, void* hip_stream);

/* y[B][1][T] = tanh(conv1d(leaky_relu(z, in_slope), w[1][Cin][7], b, pad 3)). */
int tts_op_conv_post(const float* d_z, int B, int Cin, int T, const float* h_w, const float* h_b,
                     float in_slope, float* d_y, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* TTS_MI355X_H */
