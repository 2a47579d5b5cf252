// Glow-TTS Encoder executor: every matmul of the reference runs on the conv kernels (1x1 q|k|v
// as one 3H-row conv, conv_o with the residual fused, FFN k3 with the relu and the mask fused,
// prenet k5, duration predictor k3), the rest on kernels_text.hip.
// Reference: TTS/tts/layers/glow_tts/encoder.py:97-179, glow.py:55-67 (prenet),
// transformer.py:117-201 (attention), :319-341 (FFN), :415-432 (layer loop),
// duration_predictor.py:47-73, normalization.py:23-28; the other encoder types:
// generic/gated_conv.py:15-36, generic/res_conv_bn.py:19-127, generic/time_depth_sep_conv.py:5-84.
// BatchNorms (eval) that directly follow a conv are folded into it on the host; the one after a
// relu (Conv1dBN, res_conv_bn.py:43-44) runs as a per-channel affine.
//
// Masking: the reference masks conv INPUTS (x * x_mask); here every producer masks its output
// instead (conv epilogue mask, LayerNorm * mask).  Padded positions never reach a valid one
// (convs read masked planes, attention fills masked keys with -1e4) and every output the
// encoder returns is multiplied by x_mask, so the returned tensors are the same.
#include <cmath>
#include <cstring>

#include "text.hpp"

namespace tts {

namespace {
int heads_dk(const TtsGlowEncoderCfg& c) { return c.hidden_channels / c.num_heads; }
constexpr double kBnEps = 1e-5;  // nn.BatchNorm1d default
// residual_conv_bn convs run with an odd kernel: an even reference kernel gets a zero tap appended
int odd_k(int k) { return k % 2 ? k : k + 1; }
}  // namespace

std::vector<int64_t> glow_encoder_weight_shapes(const TtsGlowEncoderCfg& c, bool with_dp, int emb_channels) {
  std::vector<int64_t> n;
  const int64_t H = c.hidden_channels, F = c.hidden_channels_ffn, K = c.kernel_size, D = c.hidden_channels_dp;
  const int et = c.encoder_type;
  n.push_back((int64_t)c.num_chars * (emb_channels > 0 ? emb_channels : H));  // emb.weight
  auto bn = [&](int64_t C) { for (int i = 0; i < 4; ++i) n.push_back(C); };
  if (c.use_prenet && (et == TTS_ENC_REL_POS_TRANSFORMER || et == TTS_ENC_TIME_DEPTH_SEPARABLE)) {
    for (int l = 0; l < 3; ++l) {
      n.push_back(H * H * 5); n.push_back(H);  // prenet.conv_layers.l
      n.push_back(H); n.push_back(H);          // prenet.norm_layers.l gamma, beta
    }
    n.push_back(H * H); n.push_back(H);        // prenet.proj
  }
  if (et == TTS_ENC_GATED_CONV) {
    for (int l = 0; l < c.num_layers; ++l) {
      n.push_back(2 * H * H * K); n.push_back(2 * H);  // encoder.conv_layers.l
      n.push_back(2 * H); n.push_back(2 * H);          // encoder.norm_layers.l
    }
  } else if (et == TTS_ENC_RESIDUAL_CONV_BN) {
    for (int i = 0; i < c.num_res_blocks; ++i)
      for (int j = 0; j < c.num_conv_blocks; ++j) {
        n.push_back(H * H * K); n.push_back(H);  // res_blocks.i.conv_bn_blocks.j.conv1d
        bn(H);                                   // .norm
      }
    n.push_back(H * H); n.push_back(H); bn(H);   // postnet.0 (conv1x1), postnet.1 (BatchNorm)
  } else if (et == TTS_ENC_TIME_DEPTH_SEPARABLE) {
    for (int l = 0; l < c.num_layers; ++l) {
      n.push_back(2 * H * H); n.push_back(2 * H); bn(2 * H);  // time_conv, norm1
      n.push_back(H * K); n.push_back(H); bn(H);              // depth_conv, norm2
      n.push_back(H * H); n.push_back(H); bn(H);              // time_conv2, norm3
    }
  }
  for (int l = 0; et == TTS_ENC_REL_POS_TRANSFORMER && l < c.num_layers; ++l) {
    for (int j = 0; j < 4; ++j) { n.push_back(H * H); n.push_back(H); }  // conv_q, conv_k, conv_v, conv_o
    if (c.rel_attn_window_size > 0) {
      const int64_t R = 2 * c.rel_attn_window_size + 1;
      n.push_back(R * heads_dk(c)); n.push_back(R * heads_dk(c));  // emb_rel_k, emb_rel_v
    }
    n.push_back(H); n.push_back(H);                          // norm_layers_1.l
    n.push_back(F * H * K); n.push_back(F);                  // ffn_layers.l.conv_1
    n.push_back(H * F * K); n.push_back(H);                  // ffn_layers.l.conv_2
    n.push_back(H); n.push_back(H);                          // norm_layers_2.l
  }
  n.push_back((int64_t)c.out_channels * H); n.push_back(c.out_channels);  // proj_m
  if (!c.mean_only) { n.push_back((int64_t)c.out_channels * H); n.push_back(c.out_channels); }  // proj_s
  if (!with_dp) return n;
  // dp conv_1 reads cat(x, g) when speaker-conditioned (encoder.py:166-168: H + c_in channels)
  n.push_back(D * (H + c.c_in_channels) * 3); n.push_back(D); n.push_back(D); n.push_back(D);  // dp conv_1, norm_1
  n.push_back(D * D * 3); n.push_back(D); n.push_back(D); n.push_back(D);  // dp conv_2, norm_2
  n.push_back(D); n.push_back(1);                                           // dp proj
  return n;
}

void glow_encoder_validate(const TtsGlowEncoderCfg& c) {
  const int et = c.encoder_type;
  TTS_REQUIRE(et >= TTS_ENC_REL_POS_TRANSFORMER && et <= TTS_ENC_TIME_DEPTH_SEPARABLE, 1, "unknown encoder_type");
  TTS_REQUIRE(c.num_chars >= 1 && c.out_channels >= 1 && c.hidden_channels >= 1 && c.hidden_channels_dp >= 1, 1,
              "bad Glow encoder configuration");
  const auto kset = [](int k) { return k == 1 || k == 3 || k == 5 || k == 7 || k == 11; };
  if (et == TTS_ENC_GATED_CONV) {
    TTS_REQUIRE(c.num_layers >= 1, 1, "gated_conv: num_layers must be >= 1");
    TTS_REQUIRE(kset(c.kernel_size), 3, "gated_conv: kernel_size must be 1, 3, 5, 7 or 11");
    TTS_REQUIRE(c.hidden_channels % 16 == 0 && 2 * c.hidden_channels <= 768, 3,
                "gated_conv: hidden_channels must be a multiple of 16 and at most 384");
  } else if (et == TTS_ENC_RESIDUAL_CONV_BN) {
    TTS_REQUIRE(c.num_res_blocks >= 1 && c.num_res_blocks <= 32 && c.num_conv_blocks >= 1, 1,
                "residual_conv_bn: 1..32 residual blocks (one dilation each) of >= 1 convs");
    TTS_REQUIRE(kset(odd_k(c.kernel_size)), 3, "residual_conv_bn: kernel_size must be 1-7, 10 or 11");
    for (int i = 0; i < c.num_res_blocks; ++i)
      TTS_REQUIRE(c.dilations[i] >= 1 && (odd_k(c.kernel_size) - 1) * c.dilations[i] <= (odd_k(c.kernel_size) - 1) * 5, 3,
                  "residual_conv_bn: dilations must be 1..5");
    TTS_REQUIRE(!c.use_prenet, 1,
                "residual_conv_bn with use_prenet: the reference calls its nn.Sequential prenet with (x, x_mask) "
                "and raises TypeError (encoder.py:158)");
  } else if (et == TTS_ENC_TIME_DEPTH_SEPARABLE) {
    TTS_REQUIRE(c.num_layers >= 2, 1, "time_depth_separable: num_layers must be > 1 (time_depth_sep_conv.py:64)");
    TTS_REQUIRE(c.kernel_size % 2 == 1 && c.kernel_size <= 31, 3,
                "time_depth_separable: kernel_size must be odd (time_depth_sep_conv.py:63) and <= 31");
  } else {
    TTS_REQUIRE(c.hidden_channels_ffn >= 1 && c.num_layers >= 1, 1, "bad Glow encoder configuration");
    TTS_REQUIRE(c.num_heads >= 1 && c.hidden_channels % c.num_heads == 0, 1,
                "channels should be divisible by num_heads (transformer.py:75)");
    TTS_REQUIRE(heads_dk(c) <= 128, 3, "attention head size above 128 is not implemented");
    TTS_REQUIRE(kset(c.kernel_size), 3, "FFN kernel_size must be 1, 3, 5, 7 or 11");
  }
  TTS_REQUIRE(c.rel_attn_window_size >= 0, 1, "rel_attn_window_size must be >= 0 (0 = None)");
  TTS_REQUIRE(c.layer_norm_type >= 0 && c.layer_norm_type <= 2, 1, " [!] Unknown layer norm type");
  TTS_REQUIRE(!c.has_input_length || c.input_length >= 0, 1, "input_length must be >= 0");
  TTS_REQUIRE(c.c_in_channels >= 0, 1, "c_in_channels must be >= 0");
  TTS_REQUIRE(c.math_mode >= MATH_FP32 && c.math_mode <= MATH_LAST, 1, "unknown math_mode");
  TTS_REQUIRE(c.math_mode != MATH_FP32_F16X3, 3,
              "Glow encoder: math_mode FP32_F16X3 is not implemented (use FP32, FP32_X6 or BF16)");
}

GlowEncoder::GlowEncoder(const TtsGlowEncoderCfg& cfg, const float* const* hw, int device, bool with_dp,
                         int emb_channels)
    : cfg_(cfg), device_(device), with_dp_(with_dp),
      emb_ch_(emb_channels > 0 ? emb_channels : cfg.hidden_channels) {
  glow_encoder_validate(cfg_);
  TTS_REQUIRE(emb_ch_ <= cfg_.hidden_channels && (emb_ch_ == cfg_.hidden_channels ||
                                                  cfg_.encoder_type == TTS_ENC_REL_POS_TRANSFORMER),
              1, "Glow encoder: embedding narrower than the encoder only for the relative-position transformer");
  DeviceGuard g(device_);
  const auto shapes = glow_encoder_weight_shapes(cfg_, with_dp_, emb_ch_);
  for (size_t i = 0; i < shapes.size(); ++i)
    TTS_REQUIRE(hw[i] != nullptr, 1, "weight pointer " + std::to_string(i) + " is NULL");
  const int H = cfg_.hidden_channels, F = cfg_.hidden_channels_ffn, K = cfg_.kernel_size;
  const int D = cfg_.hidden_channels_dp;
  const int mode = cfg_.math_mode;

  std::vector<float> host;
  std::vector<std::pair<size_t, float**>> fix;
  auto align = [](size_t n) { return (n + 63) & ~size_t(63); };
  auto put = [&](const float* src, size_t n, float** dst) {
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    std::memcpy(host.data() + off, src, n * sizeof(float));
    fix.push_back({off, dst});
  };
  // conv from one or more row blocks of torch weights [rows][Cin][K] stacked along Cout
  // conv from one or more row blocks of torch weights [rows][Cin][k] stacked along Cout; kc > k
  // appends zero taps (an even reference kernel on the odd-kernel conv); bn (weight, bias, mean,
  // var) folds a following BatchNorm into the weights and bias
  auto put_conv = [&](Conv& cv, std::vector<std::pair<const float*, const float*>> parts, int rows_each, int Cin,
                      int k, int dil = 1, int pad = -1, int kc = 0, const float* const* bn = nullptr) {
    const int Cout = rows_each * (int)parts.size();
    kc = kc ? kc : k;
    cv.Cin = Cin; cv.Cout = Cout; cv.K = kc; cv.dil = dil;
    cv.pad = pad >= 0 ? pad : dil * (k - 1) / 2;
    // text batches are short (a 16 x 128-token batch is 2,048 columns): the split modes take the
    // 32x128 tile (4 waves side by side) so a conv launches Cout/32 x B workgroups, not Cout/128 x B
    cv.tile = is_split_mode(mode) ? 16 : conv_tile_for(mode, Cout, kc, Cin, dil, false);
    const ConvTile t = conv_tile(mode, cv.tile);
    cv.n_chunks = ceil_div(Cin, t.CK);
    std::vector<float> w((size_t)Cout * Cin * kc, 0.f), b(Cout);
    for (size_t p = 0; p < parts.size(); ++p) {
      for (int r = 0; r < rows_each; ++r)
        for (int ci = 0; ci < Cin; ++ci)
          std::memcpy(w.data() + (((size_t)p * rows_each + r) * Cin + ci) * kc,
                      parts[p].first + ((size_t)r * Cin + ci) * k, sizeof(float) * k);
      std::memcpy(b.data() + p * rows_each, parts[p].second, sizeof(float) * rows_each);
    }
    if (bn) {  // y = (conv - mean) / sqrt(var + eps) * gamma + beta, in double
      for (int co = 0; co < Cout; ++co) {
        const double sc = (double)bn[0][co] / std::sqrt((double)bn[3][co] + kBnEps);
        for (size_t i = 0; i < (size_t)Cin * kc; ++i) w[(size_t)co * Cin * kc + i] = (float)(w[(size_t)co * Cin * kc + i] * sc);
        b[co] = (float)(((double)b[co] - bn[2][co]) * sc + bn[1][co]);
      }
    }
    const size_t n = packed_conv_numel(mode, Cout, Cin, kc, t);
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    const int w_exp = pack_conv(mode, w.data(), Cout, Cin, kc, t, host.data() + off);
    TTS_REQUIRE(w_exp == 0, 3, "Glow encoder: scaled weight packing is not supported");
    fix.push_back({off, &cv.w});
    const size_t nb = (size_t)ceil_div(Cout, t.BM) * t.BM;
    const size_t offb = host.size();
    host.resize(offb + align(nb), 0.f);
    std::memcpy(host.data() + offb, b.data(), Cout * sizeof(float));
    fix.push_back({offb, &cv.b});
  };
  auto put_norm = [&](Norm& n, const float* gm, const float* bt, int C) {
    put(gm, C, &n.gamma);
    put(bt, C, &n.beta);
  };

  // BatchNorm (weight, bias, running_mean, running_var) -> device scale / shift
  auto put_affine = [&](Affine& af, const float* const* bn, int C) {
    std::vector<float> sc(C), sh(C);
    for (int c = 0; c < C; ++c) {
      const double s = (double)bn[0][c] / std::sqrt((double)bn[3][c] + kBnEps);
      sc[c] = (float)s;
      sh[c] = (float)((double)bn[1][c] - (double)bn[2][c] * s);
    }
    put(sc.data(), C, &af.scale);
    put(sh.data(), C, &af.shift);
  };
  const int et = cfg_.encoder_type;

  size_t wi = 0;
  put(hw[wi++], (size_t)cfg_.num_chars * emb_ch_, &emb_);
  if (cfg_.use_prenet && (et == TTS_ENC_REL_POS_TRANSFORMER || et == TTS_ENC_TIME_DEPTH_SEPARABLE)) {
    for (int l = 0; l < 3; ++l) {
      put_conv(pre_conv_[l], {{hw[wi], hw[wi + 1]}}, H, H, 5);
      put_norm(pre_norm_[l], hw[wi + 2], hw[wi + 3], H);
      wi += 4;
    }
    put_conv(pre_proj_, {{hw[wi], hw[wi + 1]}}, H, H, 1);
    wi += 2;
  }
  if (et == TTS_ENC_GATED_CONV) {
    gconv_.resize(cfg_.num_layers);
    gnorm_.resize(cfg_.num_layers);
    for (int l = 0; l < cfg_.num_layers; ++l) {
      put_conv(gconv_[l], {{hw[wi], hw[wi + 1]}}, 2 * H, H, K);
      put_norm(gnorm_[l], hw[wi + 2], hw[wi + 3], 2 * H);
      wi += 4;
    }
  } else if (et == TTS_ENC_RESIDUAL_CONV_BN) {
    const int k = cfg_.kernel_size;
    rcbn_.resize((size_t)cfg_.num_res_blocks * cfg_.num_conv_blocks);
    for (int i = 0; i < cfg_.num_res_blocks; ++i) {
      const int d = cfg_.dilations[i];
      const int ptot = d * (k - 1), ps = ptot / 2;  // ZeroPad (pad_s, pad_e) of the conv's output
      for (int j = 0; j < cfg_.num_conv_blocks; ++j) {
        ConvBN& cb = rcbn_[(size_t)i * cfg_.num_conv_blocks + j];
        put_conv(cb.conv, {{hw[wi], hw[wi + 1]}}, H, H, k, d, ps, odd_k(k));
        put_affine(cb.bn, hw + wi + 2, H);
        cb.lo = ps;
        cb.hi = ptot - ps;
        wi += 6;
      }
    }
    put_conv(post_, {{hw[wi], hw[wi + 1]}}, H, H, 1, 1, 0, 0, hw + wi + 2);
    wi += 6;
  } else if (et == TTS_ENC_TIME_DEPTH_SEPARABLE) {
    const int k = cfg_.kernel_size;
    tds_.resize(cfg_.num_layers);
    for (int l = 0; l < cfg_.num_layers; ++l) {
      TdsLayer& L = tds_[l];
      put_conv(L.time_conv, {{hw[wi], hw[wi + 1]}}, 2 * H, H, 1, 1, 0, 0, hw + wi + 2);
      wi += 6;
      std::vector<float> dw((size_t)H * k), db(H);  // depth_conv with norm2 folded
      for (int c = 0; c < H; ++c) {
        const double sc = (double)hw[wi + 2][c] / std::sqrt((double)hw[wi + 5][c] + kBnEps);
        for (int j = 0; j < k; ++j) dw[(size_t)c * k + j] = (float)(hw[wi][(size_t)c * k + j] * sc);
        db[c] = (float)(((double)hw[wi + 1][c] - hw[wi + 4][c]) * sc + hw[wi + 3][c]);
      }
      put(dw.data(), dw.size(), &L.dw_w);
      put(db.data(), db.size(), &L.dw_b);
      wi += 6;
      put_conv(L.time_conv2, {{hw[wi], hw[wi + 1]}}, H, H, 1, 1, 0, 0, hw + wi + 2);
      wi += 6;
    }
  }
  layers_.resize(et == TTS_ENC_REL_POS_TRANSFORMER ? cfg_.num_layers : 0);
  for (int l = 0; l < (int)layers_.size(); ++l) {
    Layer& L = layers_[l];
    put_conv(L.qkv, {{hw[wi], hw[wi + 1]}, {hw[wi + 2], hw[wi + 3]}, {hw[wi + 4], hw[wi + 5]}}, H, H, 1);
    put_conv(L.o, {{hw[wi + 6], hw[wi + 7]}}, H, H, 1);
    wi += 8;
    if (cfg_.rel_attn_window_size > 0) {
      const size_t R = 2 * cfg_.rel_attn_window_size + 1;
      put(hw[wi], R * heads_dk(cfg_), &L.ek);
      put(hw[wi + 1], R * heads_dk(cfg_), &L.ev);
      wi += 2;
    }
    put_norm(L.n1, hw[wi], hw[wi + 1], H);
    put_conv(L.ffn1, {{hw[wi + 2], hw[wi + 3]}}, F, H, K);
    put_conv(L.ffn2, {{hw[wi + 4], hw[wi + 5]}}, H, F, K);
    put_norm(L.n2, hw[wi + 6], hw[wi + 7], H);
    wi += 8;
  }
  put_conv(proj_m_, {{hw[wi], hw[wi + 1]}}, cfg_.out_channels, H, 1);
  wi += 2;
  if (!cfg_.mean_only) {
    put_conv(proj_s_, {{hw[wi], hw[wi + 1]}}, cfg_.out_channels, H, 1);
    wi += 2;
  }
  if (with_dp_) {
    put_conv(dp1_, {{hw[wi], hw[wi + 1]}}, D, H + cfg_.c_in_channels, 3);
    put_norm(dpn1_, hw[wi + 2], hw[wi + 3], D);
    put_conv(dp2_, {{hw[wi + 4], hw[wi + 5]}}, D, D, 3);
    put_norm(dpn2_, hw[wi + 6], hw[wi + 7], D);
    put_conv(dp_proj_, {{hw[wi + 8], hw[wi + 9]}}, 1, D, 1);
    wi += 10;
  }
  TTS_REQUIRE(wi == shapes.size(), 2, "internal: Glow encoder weight count mismatch");

  if (hipMalloc(&arena_, host.size() * sizeof(float)) != hipSuccess) throw Error(4, "hipMalloc(weights) failed");
  TTS_HIP_CHECK(hipMemcpy(arena_, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
  for (auto& p : fix) *p.second = arena_ + p.first;
}

GlowEncoder::~GlowEncoder() {
  DeviceGuard g(device_);
  if (arena_) (void)hipFree(arena_);
  if (ws_) (void)hipFree(ws_);
}

void GlowEncoder::reserve(int B, int T) {
  const int H = cfg_.hidden_channels, F = cfg_.hidden_channels_ffn, D = cfg_.hidden_channels_dp;
  const size_t plane = (size_t)B * T;
  const size_t big = std::max({(size_t)3 * H, (size_t)F, (size_t)D});
  const size_t dpin = cfg_.c_in_channels > 0 ? plane * (H + cfg_.c_in_channels) + 64 : 0;  // cat(x, g) * mask
  const size_t need = (plane * (3 * (size_t)H + big + std::max((size_t)H, (size_t)D)) + dpin) * sizeof(float) + 4096;
  if (need <= ws_bytes_) return;
  if (ws_) { TTS_HIP_CHECK(hipFree(ws_)); ws_ = nullptr; ws_bytes_ = 0; }
  if (hipMalloc(&ws_, need) != hipSuccess) throw Error(4, "hipMalloc(workspace) failed");
  ws_bytes_ = need;
}

void GlowEncoder::forward(const int64_t* tok, const int64_t* len, const float* g, int B, int T, float* x_m,
                          float* x_logs, float* logw, float* x_mask, hipStream_t s, Profiler* prof, float* x_out,
                          const float* lang) {
  TTS_REQUIRE(tok && len && x_m && x_mask && (logw || !with_dp_), 1, "NULL input/output pointer");
  TTS_REQUIRE(emb_ch_ == cfg_.hidden_channels || lang != nullptr, 1,
              "this encoder appends a language embedding (language_emb_dim > 0): pass lang_emb");
  TTS_REQUIRE(cfg_.c_in_channels == 0 || g != nullptr, 1, "c_in_channels > 0 requires g");
  TTS_REQUIRE(B >= 1 && T >= 1, 1, "batch and token count must be >= 1");
  // the attention kernel keeps whole score rows in LDS; the convolutional encoder types have no such bound
  TTS_REQUIRE(cfg_.encoder_type != TTS_ENC_REL_POS_TRANSFORMER || T <= ATTN_MAX_T, 3,
              "more than " + std::to_string(ATTN_MAX_T) + " tokens per utterance (rel_pos_transformer)");
  DeviceGuard dg(device_);
  reserve(B, T);
  const int H = cfg_.hidden_channels, F = cfg_.hidden_channels_ffn, D = cfg_.hidden_channels_dp;
  const int mode = cfg_.math_mode;
  const size_t plane = (size_t)B * T;
  const double P = (double)plane;
  auto al = [](size_t n) { return (n + 63) & ~size_t(63); };
  float* p = ws_;
  float* X0 = p; p += al(plane * H);   // layer state ping
  float* X1 = p; p += al(plane * H);   // layer state pong
  float* A = p; p += al(plane * H);    // attention output
  const size_t big = std::max({(size_t)3 * H, (size_t)F, (size_t)D});
  float* Wd = p; p += al(plane * big);  // qkv / FFN hidden / dp hidden
  float* Nb = p; p += al(plane * std::max((size_t)H, (size_t)D));  // LayerNorm output of prenet / dp
  float* Xdp = cfg_.c_in_channels > 0 ? p : nullptr;                // dp input cat(x, g) * mask
  const float* mask = x_mask;
  constexpr float kEps = 1e-4f;  // normalization.py:6

  auto conv = [&](const char* name, const Conv& cv, const float* in, float* out, const float* res, const float* m,
                  float out_slope, bool mask_res) {
    Conv1dArgs a{};
    a.x = in; a.w = cv.w; a.bias = cv.b; a.y = out; a.res = res; a.mask = m;
    a.Cin = cv.Cin; a.Cout = cv.Cout; a.Tin = T; a.Tout = T;
    a.dil = cv.dil; a.pad = cv.pad; a.rep_pad = 0; a.n_chunks = cv.n_chunks;  // same padding (transformer.py:335)
    a.in_slope = 1.f; a.out_slope = out_slope; a.zmode = 0; a.zdiv = 1.f;
    a.mask_res = mask_res ? 1 : 0;
    run(prof, s, name, 2.0 * P * cv.Cout * cv.Cin * cv.K, 4.0 * P * (cv.Cin + cv.Cout + (res ? cv.Cout : 0)),
        [&] { launch_conv(mode, a, B, cv.K, cv.tile, s); });
  };
  auto norm = [&](const char* name, const Norm& n, const float* a, const float* r, float* y, int C, bool relu,
                  float eps = kEps) {
    run(prof, s, name, 0.0, 4.0 * P * C * (r ? 3 : 2),
        [&] { launch_layernorm(a, r, n.gamma, n.beta, mask, y, B, C, T, eps, relu, s); });
  };
  // the transformer's own LayerNorms: LayerNorm2 (layer_norm_type "2") is F.layer_norm, eps 1e-5
  // (normalization.py:42-53), the same normalisation with another eps
  const float eps_tf = cfg_.layer_norm_type == 2 ? 1e-5f : kEps;

  // emb(x) * sqrt(H), transpose, x_mask (encoder.py:162-164); VITS with a language embedding:
  // cat(emb(x) * sqrt(H), lang_emb.expand) with H the embedding width (vits/networks.py:86-96)
  const float scale = (float)std::sqrt((double)emb_ch_);
  run(prof, s, "enc_embed", 0.0, 4.0 * P * H + 16.0 * P,
      [&] { launch_embed(tok, len, emb_, X0, x_mask, B, H, T, cfg_.num_chars, scale, s, lang, emb_ch_); });
  float* x = X0;
  const int et = cfg_.encoder_type;
  if (cfg_.use_prenet && (et == TTS_ENC_REL_POS_TRANSFORMER || et == TTS_ENC_TIME_DEPTH_SEPARABLE)) {  // glow.py:61-67
    const float* in = X0;
    for (int l = 0; l < 3; ++l) {
      conv("enc_prenet_conv", pre_conv_[l], in, Wd, nullptr, mask, 1.f, false);
      norm("enc_layernorm", pre_norm_[l], Wd, nullptr, Nb, H, true);  // LN(x*mask) -> relu
      in = Nb;
    }
    conv("enc_prenet_proj", pre_proj_, Nb, X1, X0, mask, 1.f, true);  // (x_res + proj(x)) * mask
    x = X1;
  }
  if (et == TTS_ENC_GATED_CONV) {
    // gated_conv.py:30-36: o = o + glu(LN(conv(o * mask))); x is masked on entry and every layer
    // output is masked (the reference's o differs only at padded positions, which the next conv
    // and every returned tensor multiply by x_mask)
    for (int l = 0; l < cfg_.num_layers; ++l) {
      conv("enc_gated_conv", gconv_[l], x, Wd, nullptr, nullptr, 1.f, false);
      run(prof, s, "enc_layernorm_glu", 0.0, 4.0 * P * 3 * H,
          [&] { launch_layernorm_glu(Wd, x, gnorm_[l].gamma, gnorm_[l].beta, mask, x, B, 2 * H, T, kEps, s); });
    }
  } else if (et == TTS_ENC_RESIDUAL_CONV_BN) {
    // res_conv_bn.py:119-127: o = x * mask; per block: o = (convbn^n(o) + o) * mask.  Inside a
    // block nothing is masked (the reference's second conv reads the first one's BatchNorm output
    // at padded positions too)
    float* o = x;
    float* t1 = (x == X0) ? X1 : X0;
    const int nb = cfg_.num_conv_blocks;
    for (int i = 0; i < cfg_.num_res_blocks; ++i) {
      const float* in = o;
      for (int j = 0; j < nb; ++j) {
        const ConvBN& cb = rcbn_[(size_t)i * nb + j];
        const bool last = j + 1 == nb;
        float* dst = last ? t1 : (j % 2 ? A : Wd);
        TTS_REQUIRE(T > cb.lo + cb.hi, 3,
                    "residual_conv_bn: fewer tokens than the dilated kernel spans (the reference's conv raises)");
        conv("enc_res_conv", cb.conv, in, dst, nullptr, nullptr, 1.f, false);
        run(prof, s, "enc_bn_act", 0.0, 4.0 * P * H * (last ? 4 : 2), [&] {
          launch_bn_act(dst, cb.bn.scale, cb.bn.shift, last ? o : nullptr, last ? mask : nullptr, dst, B, H, T, cb.lo,
                        T - cb.hi, s);
        });
        in = dst;
      }
      std::swap(o, t1);
    }
    // postnet: conv1x1 -> BatchNorm (folded), * x_mask (encoder.py:161-162)
    float* px = (o == X0) ? X1 : X0;
    conv("enc_postnet", post_, o, px, nullptr, mask, 1.f, false);
    x = px;
  } else if (et == TTS_ENC_TIME_DEPTH_SEPARABLE) {
    // time_depth_sep_conv.py:44-56, :82-84: x = layer(x * mask) = x*mask + tc2(swish(dw(glu(tc(x*mask)))));
    // inputs are masked by their producer; the glu / depthwise stage is not masked (the
    // reference's depthwise conv reads it at padded positions)
    for (int l = 0; l < cfg_.num_layers; ++l) {
      const TdsLayer& L = tds_[l];
      float* other = (x == X0) ? X1 : X0;
      conv("enc_tds_time_conv", L.time_conv, x, Wd, nullptr, nullptr, 1.f, false);
      run(prof, s, "enc_tds_glu_dw_swish", 2.0 * P * H * cfg_.kernel_size, 4.0 * P * 3 * H,
          [&] { launch_glu_dw_swish(Wd, L.dw_w, L.dw_b, A, B, H, T, cfg_.kernel_size, s); });
      conv("enc_tds_time_conv2", L.time_conv2, A, other, x, mask, 1.f, true);  // (x + tc2(.)) * mask
      x = other;
    }
  }
  // transformer layers (transformer.py:420-431); x is masked on entry
  for (int l = 0; l < (int)layers_.size(); ++l) {
    const Layer& L = layers_[l];
    float* other = (x == X0) ? X1 : X0;
    conv("enc_qkv", L.qkv, x, Wd, nullptr, nullptr, 1.f, false);
    run(prof, s, "enc_attention", 4.0 * (double)B * T * T * H, 4.0 * P * 4 * H, [&] {
      launch_attention(Wd, mask, L.ek, L.ev, A, B, H, cfg_.num_heads, T, cfg_.rel_attn_window_size, s,
                       cfg_.has_input_length ? cfg_.input_length : -1);
    });
    conv("enc_attn_o", L.o, A, other, x, nullptr, 1.f, false);          // x + conv_o(attn)
    norm("enc_layernorm", L.n1, other, nullptr, other, H, false, eps_tf);  // norm_layers_1, * mask
    conv("enc_ffn1", L.ffn1, other, Wd, nullptr, mask, 0.f, false);      // relu(conv_1(x*mask)) * mask
    conv("enc_ffn2", L.ffn2, Wd, x, other, mask, 1.f, false);            // x + conv_2(h*mask)*mask
    norm("enc_layernorm", L.n2, x, nullptr, x, H, false, eps_tf);          // norm_layers_2, * mask
  }
  if (x_out) TTS_HIP_CHECK(hipMemcpyAsync(x_out, x, plane * H * sizeof(float), hipMemcpyDeviceToDevice, s));
  // heads (encoder.py:171-178)
  conv("enc_proj_m", proj_m_, x, x_m, nullptr, mask, 1.f, false);
  if (!cfg_.mean_only) {
    TTS_REQUIRE(x_logs != nullptr, 1, "x_logs is NULL (mean_only = 0)");
    conv("enc_proj_s", proj_s_, x, x_logs, nullptr, mask, 1.f, false);
  } else if (x_logs) {
    TTS_HIP_CHECK(hipMemsetAsync(x_logs, 0, plane * cfg_.out_channels * sizeof(float), s));
  }
  if (!with_dp_) return;
  // duration predictor (duration_predictor.py:63-73) on x (detached: same values), or on
  // cat(x, g.expand(T)) for a speaker-conditioned model (encoder.py:166-168; the predictor masks
  // its whole input, :66, and x is already masked)
  const float* xdp = x;
  if (Xdp) {
    const int Cc = cfg_.c_in_channels;
    run(prof, s, "enc_dp_input", 0.0, 4.0 * P * (2 * H + Cc + 1),
        [&] { launch_dp_input(x, g, mask, Xdp, B, H, Cc, T, s); });
    xdp = Xdp;
  }
  conv("enc_dp_conv", dp1_, xdp, Wd, nullptr, mask, 0.f, false);
  norm("enc_layernorm", dpn1_, Wd, nullptr, Nb, D, false);
  conv("enc_dp_conv", dp2_, Nb, Wd, nullptr, mask, 0.f, false);
  norm("enc_layernorm", dpn2_, Wd, nullptr, Nb, D, false);
  conv("enc_dp_proj", dp_proj_, Nb, logw, nullptr, mask, 1.f, false);
  (void)F;
}

}  // namespace tts
