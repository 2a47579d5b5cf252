// VITS text side of Vits.inference (TTS/tts/models/vits.py:1121-1152):
// * TextEncoder (TTS/tts/layers/vits/networks.py:29-100): the Glow encoder's RelativePositionTransformer
//   (LayerNorm2, window 4, no prenet, no duration predictor) with proj (H -> 2 out) split into the
//   m / logs heads;
// * StochasticDurationPredictor(reverse=True) (TTS/tts/layers/vits/stochastic_duration_predictor.py):
//   its 1x1 convs on the conv kernels, the depthwise conv + LayerNorm2 + gelu stages, the spline and
//   the affine flow on kernels_vits_text.hip.
#include <cmath>
#include <cstring>

#include "text.hpp"

namespace tts {

// ---------------------------------------------------------------------------------------
// TextEncoder
// ---------------------------------------------------------------------------------------
void vits_text_encoder_validate(const TtsVitsTextEncoderCfg& c) {
  TTS_REQUIRE(c.n_vocab >= 1 && c.out_channels >= 1 && c.hidden_channels >= 1 && c.hidden_channels_ffn >= 1 &&
                  c.num_layers >= 1 && c.num_heads >= 1,
              1, "bad VITS TextEncoder configuration");
  TTS_REQUIRE(c.language_emb_dim >= 0, 1, "language_emb_dim must be >= 0");
  glow_encoder_validate(vits_text_encoder_glow_cfg(c));
}

// networks.py:66-77: RelativePositionTransformer(in = out = hidden, layer_norm_type "2",
// rel_attn_window_size 4); proj is carried as the Glow encoder's proj_m / proj_s pair.  With a
// language embedding the transformer and proj run at E = hidden + language_emb_dim (:63-64) while
// the token embedding keeps hidden channels (GlowEncoder's emb_channels)
TtsGlowEncoderCfg vits_text_encoder_glow_cfg(const TtsVitsTextEncoderCfg& c) {
  TtsGlowEncoderCfg g{};
  g.num_chars = c.n_vocab;
  g.out_channels = c.out_channels;
  g.hidden_channels = c.hidden_channels + c.language_emb_dim;
  g.hidden_channels_dp = g.hidden_channels;  // no duration predictor (with_dp = false)
  g.hidden_channels_ffn = c.hidden_channels_ffn;
  g.num_heads = c.num_heads;
  g.num_layers = c.num_layers;
  g.kernel_size = c.kernel_size;
  g.rel_attn_window_size = 4;
  g.mean_only = 0;
  g.use_prenet = 0;
  g.c_in_channels = 0;
  g.math_mode = c.math_mode;
  g.encoder_type = TTS_ENC_REL_POS_TRANSFORMER;
  g.layer_norm_type = 2;
  return g;
}

std::vector<int64_t> vits_text_encoder_weight_shapes(const TtsVitsTextEncoderCfg& c) {
  const TtsGlowEncoderCfg g = vits_text_encoder_glow_cfg(c);
  std::vector<int64_t> n = glow_encoder_weight_shapes(g, false, c.hidden_channels);
  // the last four are proj_m / proj_s (weight, bias): the reference has one proj [2 out][E][1]
  n.resize(n.size() - 4);
  n.push_back((int64_t)2 * c.out_channels * g.hidden_channels);
  n.push_back((int64_t)2 * c.out_channels);
  return n;
}

VitsTextEncoder::VitsTextEncoder(const TtsVitsTextEncoderCfg& cfg, const float* const* hw, int device) : cfg_(cfg) {
  vits_text_encoder_validate(cfg_);
  const auto shapes = vits_text_encoder_weight_shapes(cfg_);
  for (size_t i = 0; i < shapes.size(); ++i)
    TTS_REQUIRE(hw[i] != nullptr, 1, "weight pointer " + std::to_string(i) + " is NULL");
  const size_t np = shapes.size() - 2;  // proj.weight, proj.bias
  const size_t wsz = (size_t)cfg_.out_channels * (cfg_.hidden_channels + cfg_.language_emb_dim);
  std::vector<const float*> ptrs(hw, hw + np);
  // m, logs = torch.split(proj(x) * mask, out, dim=1) (networks.py:98-99): rows [0, out) and [out, 2 out)
  ptrs.push_back(hw[np]);
  ptrs.push_back(hw[np + 1]);
  ptrs.push_back(hw[np] + wsz);
  ptrs.push_back(hw[np + 1] + cfg_.out_channels);
  enc_ = std::make_unique<GlowEncoder>(vits_text_encoder_glow_cfg(cfg_), ptrs.data(), device, false,
                                       cfg_.hidden_channels);
}

void VitsTextEncoder::forward(const int64_t* tok, const int64_t* len, const float* lang, int B, int T, float* x,
                              float* m, float* logs, float* x_mask, hipStream_t s, Profiler* prof) {
  TTS_REQUIRE(x && m && logs, 1, "NULL output pointer");
  TTS_REQUIRE(cfg_.language_emb_dim == 0 || lang != nullptr, 1,
              "this TextEncoder has language_emb_dim > 0: pass lang_emb [B][language_emb_dim]");
  enc_->forward(tok, len, nullptr, B, T, m, logs, nullptr, x_mask, s, prof, x,
                cfg_.language_emb_dim > 0 ? lang : nullptr);
}

// ---------------------------------------------------------------------------------------
// StochasticDurationPredictor
// ---------------------------------------------------------------------------------------
namespace {
constexpr int kSdpBins = 10;          // ConvFlow num_bins (stochastic_duration_predictor.py:102)
constexpr float kSdpTailBound = 5.f;  // ConvFlow tail_bound (:103)
constexpr int kDdsLayers = 3;         // DilatedDepthSeparableConv(num_layers=3) everywhere in the SDP

void dds_shapes(std::vector<int64_t>& n, int64_t H, int64_t k) {
  for (int i = 0; i < kDdsLayers; ++i) { n.push_back(H * k); n.push_back(H); }  // convs_sep.i
  for (int i = 0; i < kDdsLayers; ++i) { n.push_back(H * H); n.push_back(H); }  // convs_1x1.i
  for (int i = 0; i < 2 * kDdsLayers; ++i) { n.push_back(H); n.push_back(H); }  // norms_1.i, norms_2.i
}
}  // namespace

void vits_sdp_validate(const TtsVitsSdpCfg& c) {
  TTS_REQUIRE(c.in_channels >= 1 && c.hidden_channels >= 1 && c.hidden_channels <= 512 && c.num_flows >= 1, 1,
              "bad StochasticDurationPredictor configuration");
  TTS_REQUIRE(c.kernel_size >= 1 && c.kernel_size % 2 == 1 && c.kernel_size <= 9, 3,
              "StochasticDurationPredictor: odd kernel_size <= 9");
  TTS_REQUIRE(c.cond_channels >= 0, 1, "cond_channels must be >= 0");
  TTS_REQUIRE(c.language_emb_dim >= 0, 1, "language_emb_dim must be >= 0");
  TTS_REQUIRE(c.math_mode >= MATH_FP32 && c.math_mode <= MATH_LAST && c.math_mode != MATH_FP32_F16X3, 3,
              "StochasticDurationPredictor: math_mode FP32, FP32_X6 or BF16");
}

// Host weight order: state_dict order of the inference-side modules (see tts_mi355x.h)
std::vector<int64_t> vits_sdp_weight_shapes(const TtsVitsSdpCfg& c) {
  std::vector<int64_t> n;
  const int64_t H = c.hidden_channels, k = c.kernel_size, nh = 3 * kSdpBins - 1;
  n.push_back(H * c.in_channels); n.push_back(H);  // pre
  dds_shapes(n, H, k);                              // convs
  n.push_back(H * H); n.push_back(H);               // proj
  n.push_back(2); n.push_back(2);                   // flows.0 translation, log_scale
  for (int f = 0; f < c.num_flows; ++f) {           // flows.1 .. flows.num_flows (ConvFlow, half = 1)
    n.push_back(H); n.push_back(H);                 // pre [H][1][1]
    dds_shapes(n, H, k);
    n.push_back(nh * H); n.push_back(nh);           // proj [29][H][1]
  }
  if (c.cond_channels > 0) { n.push_back(H * c.cond_channels); n.push_back(H); }           // cond
  if (c.language_emb_dim > 0) { n.push_back(H * c.language_emb_dim); n.push_back(H); }     // cond_lang
  return n;
}

VitsSdp::VitsSdp(const TtsVitsSdpCfg& cfg, const float* const* hw, int device) : cfg_(cfg), device_(device) {
  vits_sdp_validate(cfg_);
  DeviceGuard g(device_);
  const auto shapes = vits_sdp_weight_shapes(cfg_);
  for (size_t i = 0; i < shapes.size(); ++i)
    TTS_REQUIRE(hw[i] != nullptr, 1, "weight pointer " + std::to_string(i) + " is NULL");
  const int H = cfg_.hidden_channels, k = cfg_.kernel_size, mode = cfg_.math_mode;
  std::vector<float> host;
  std::vector<std::pair<size_t, float**>> fix;
  auto align = [](size_t n) { return (n + 63) & ~size_t(63); };
  auto put = [&](const float* src, size_t n, float** dst) {
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    std::memcpy(host.data() + off, src, n * sizeof(float));
    fix.push_back({off, dst});
  };
  auto put_conv = [&](Conv& cv, const float* w, const float* b, int Cout, int Cin) {
    cv.Cin = Cin; cv.Cout = Cout;
    // short text batches: the split modes take the 32x128 tile, as the Glow encoder does
    cv.tile = is_split_mode(mode) ? 16 : conv_tile_for(mode, Cout, 1, Cin, 1, false);
    const ConvTile t = conv_tile(mode, cv.tile);
    cv.n_chunks = ceil_div(Cin, t.CK);
    const size_t n = packed_conv_numel(mode, Cout, Cin, 1, t);
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    TTS_REQUIRE(pack_conv(mode, w, Cout, Cin, 1, t, host.data() + off) == 0, 3, "SDP: scaled packing unsupported");
    fix.push_back({off, &cv.w});
    const size_t nb = (size_t)ceil_div(Cout, t.BM) * t.BM;
    const size_t offb = host.size();
    host.resize(offb + align(nb), 0.f);
    std::memcpy(host.data() + offb, b, Cout * sizeof(float));
    fix.push_back({offb, &cv.b});
  };
  size_t wi = 0;
  auto put_dds = [&](Dds& d) {
    for (int i = 0; i < kDdsLayers; ++i) {
      put(hw[wi], (size_t)H * k, &d.sep_w[i]);
      put(hw[wi + 1], H, &d.sep_b[i]);
      wi += 2;
    }
    for (int i = 0; i < kDdsLayers; ++i) { put_conv(d.c1x1[i], hw[wi], hw[wi + 1], H, H); wi += 2; }
    for (int i = 0; i < kDdsLayers; ++i) { put(hw[wi], H, &d.n1g[i]); put(hw[wi + 1], H, &d.n1b[i]); wi += 2; }
    for (int i = 0; i < kDdsLayers; ++i) { put(hw[wi], H, &d.n2g[i]); put(hw[wi + 1], H, &d.n2b[i]); wi += 2; }
  };
  put_conv(pre_, hw[wi], hw[wi + 1], H, cfg_.in_channels); wi += 2;
  put_dds(dds_);
  put_conv(proj_, hw[wi], hw[wi + 1], H, H); wi += 2;
  put(hw[wi], 2, &ea_tr_); put(hw[wi + 1], 2, &ea_ls_); wi += 2;
  flows_.resize(cfg_.num_flows);
  for (auto& F : flows_) {
    put_conv(F.pre, hw[wi], hw[wi + 1], H, 1); wi += 2;
    put_dds(F.dds);
    put_conv(F.proj, hw[wi], hw[wi + 1], 3 * kSdpBins - 1, H); wi += 2;
  }
  if (cfg_.cond_channels > 0) {
    put(hw[wi], (size_t)H * cfg_.cond_channels, &cond_w_);
    put(hw[wi + 1], H, &cond_b_);
    wi += 2;
  }
  if (cfg_.language_emb_dim > 0) {
    put(hw[wi], (size_t)H * cfg_.language_emb_dim, &lang_w_);
    put(hw[wi + 1], H, &lang_b_);
    wi += 2;
  }
  TTS_REQUIRE(wi == shapes.size(), 2, "internal: SDP weight count mismatch");
  if (hipMalloc(&arena_, host.size() * sizeof(float)) != hipSuccess) throw Error(4, "hipMalloc(weights) failed");
  TTS_HIP_CHECK(hipMemcpy(arena_, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
  for (auto& p : fix) *p.second = arena_ + p.first;
}

VitsSdp::~VitsSdp() {
  DeviceGuard g(device_);
  if (arena_) (void)hipFree(arena_);
  if (ws_) (void)hipFree(ws_);
}

void VitsSdp::reserve(int B, int T) {
  const size_t plane = (size_t)B * T;
  const int H = cfg_.hidden_channels;
  // xs, h, a, u [H]; hp [29]; z [2]; cond vectors [2][B][H]
  const size_t need = (plane * (4 * (size_t)H + 3 * kSdpBins - 1 + 2) + 2 * (size_t)B * H + 8 * 64) * sizeof(float);
  if (need <= ws_bytes_) return;
  if (ws_) { TTS_HIP_CHECK(hipFree(ws_)); ws_ = nullptr; ws_bytes_ = 0; }
  if (hipMalloc(&ws_, need) != hipSuccess) throw Error(4, "hipMalloc(workspace) failed");
  ws_bytes_ = need;
}

void VitsSdp::reverse(const float* x, const float* x_mask, const float* g, const float* lang, const float* noise,
                      float noise_scale, int B, int T, float* logw, hipStream_t s, Profiler* prof) {
  TTS_REQUIRE(x && x_mask && logw, 1, "NULL input/output pointer");
  TTS_REQUIRE(cfg_.cond_channels == 0 || g != nullptr, 1, "cond_channels > 0 requires g");
  TTS_REQUIRE(cfg_.language_emb_dim == 0 || lang != nullptr, 1, "language_emb_dim > 0 requires lang_emb");
  TTS_REQUIRE(B >= 1 && T >= 1, 1, "batch and token count must be >= 1");
  DeviceGuard dg(device_);
  reserve(B, T);
  const int H = cfg_.hidden_channels, k = cfg_.kernel_size, mode = cfg_.math_mode;
  const int NH = 3 * kSdpBins - 1;
  const size_t plane = (size_t)B * T;
  const double P = (double)plane;
  auto al = [](size_t n) { return (n + 63) & ~size_t(63); };
  float* p = ws_;
  float* xs = p; p += al(plane * H);   // the SDP's conditioning x (proj(DDS(pre(x) + cond(g))) * mask)
  float* h = p; p += al(plane * H);    // a DDS state
  float* a = p; p += al(plane * H);    // depthwise-conv stage output
  float* u = p; p += al(plane * H);    // 1x1 conv output
  float* hp = p; p += al(plane * NH);  // ConvFlow proj output
  float* z = p; p += al(plane * 2);    // flow state [B][2][T]
  float* cvec = p; p += al((size_t)B * H);  // cond(g) [+ cond_lang(lang)] [B][H]
  float* cvec2 = p;                         // cond_lang(lang) [B][H] when both are present

  auto conv = [&](const char* name, const Conv& cv, const float* in, int64_t in_bstride, float* out, const float* res,
                  const float* m, const float* cv_vec) {
    Conv1dArgs c{};
    c.x = in; c.w = cv.w; c.bias = cv.b; c.y = out; c.res = res; c.mask = m; c.cvec = cv_vec;
    c.x_bstride = in_bstride;
    c.Cin = cv.Cin; c.Cout = cv.Cout; c.Tin = T; c.Tout = T;
    c.dil = 1; c.pad = 0; c.rep_pad = 0; c.n_chunks = cv.n_chunks;
    c.in_slope = 1.f; c.out_slope = 1.f; c.zmode = 0; c.zdiv = 1.f;
    run(prof, s, name, 2.0 * P * cv.Cout * cv.Cin, 4.0 * P * (cv.Cin + cv.Cout + (res ? cv.Cout : 0)),
        [&] { launch_conv(mode, c, B, 1, cv.tile, s); });
  };
  // DilatedDepthSeparableConv (:46-63) on st in place (g already added); the final * mask is left
  // to the consumer (a 1x1 proj whose output is masked: proj(x * m) * m = proj(x) * m for m in {0, 1})
  auto dds = [&](const Dds& d, float* st) {
    int dil = 1;
    for (int i = 0; i < kDdsLayers; ++i) {
      run(prof, s, "sdp_dds_sep", 2.0 * P * H * k, 4.0 * P * 2 * H, [&] {
        launch_dds_sep_ln_gelu(st, x_mask, d.sep_w[i], d.sep_b[i], d.n1g[i], d.n1b[i], a, B, H, T, k, dil, s);
      });
      conv("sdp_dds_1x1", d.c1x1[i], a, 0, u, nullptr, nullptr, nullptr);
      run(prof, s, "sdp_dds_ln_add", 0.0, 4.0 * P * 3 * H,
          [&] { launch_dds_ln_gelu_add(u, st, d.n2g[i], d.n2b[i], B, H, T, s); });
      dil *= k;
    }
  };

  // x = pre(x) [+ cond(g)] [+ cond_lang(lang)] (:249-254); x = proj(DDS(x, mask)) * mask (:257-258).
  // The per-utterance vectors enter the pre conv's epilogue as one sum (fp32 rounding of the order)
  const float* cv = nullptr;
  if (cond_w_) {
    run(prof, s, "sdp_cond", 2.0 * B * H * cfg_.cond_channels, 4.0 * B * (H + cfg_.cond_channels),
        [&] { launch_cond_vec(g, cond_w_, cond_b_, cvec, B, cfg_.cond_channels, H, s); });
    cv = cvec;
  }
  if (lang_w_) {
    const int L = cfg_.language_emb_dim;
    float* dst = cond_w_ ? cvec2 : cvec;
    run(prof, s, "sdp_cond_lang", 2.0 * B * H * L, 4.0 * B * (H + L),
        [&] { launch_cond_vec(lang, lang_w_, lang_b_, dst, B, L, H, s); });
    if (cond_w_) run(prof, s, "sdp_cond_add", 0.0, 12.0 * B * H, [&] { launch_vec_add(cvec, cvec2, cvec, B * H, s); });
    cv = cvec;
  }
  conv("sdp_pre", pre_, x, 0, h, nullptr, nullptr, cv);
  dds(dds_, h);
  conv("sdp_proj", proj_, h, 0, xs, nullptr, x_mask, nullptr);

  // flows = reversed(flows)[:-2] + [flows[0]] (:275-276): ConvFlow num_flows .. 2, then the affine
  run(prof, s, "sdp_noise", 0.0, 8.0 * P * 2, [&] { launch_sdp_init(noise, z, noise_scale, B, T, s); });
  int par = 0;  // physical channel of logical channel 0
  const float hscale = 1.f / std::sqrt((float)H);
  for (int f = cfg_.num_flows; f >= 2; --f) {
    const ConvFlow& F = flows_[f - 1];
    par ^= 1;  // z = torch.flip(z, [1]) (:279)
    // h = pre(x0) + g, g = the SDP's x (ConvFlow.forward :127-129; DDS adds g first, :52-53)
    conv("sdp_flow_pre", F.pre, z + (size_t)par * T, (int64_t)2 * T, h, xs, nullptr, nullptr);
    dds(F.dds, h);
    conv("sdp_flow_proj", F.proj, h, 0, hp, nullptr, x_mask, nullptr);
    run(prof, s, "sdp_spline", 0.0, 4.0 * P * (NH + 5),
        [&] { launch_sdp_spline(hp, z, x_mask, B, T, par, kSdpBins, kSdpTailBound, hscale, s); });
  }
  par ^= 1;
  run(prof, s, "sdp_affine", 0.0, 4.0 * P * 5,
      [&] { launch_sdp_affine(z, ea_tr_, ea_ls_, x_mask, logw, B, T, par, s); });
}

// ---------------------------------------------------------------------------------------
// DurationPredictor (use_sdp = False; vits.py:694-702, glow_tts/duration_predictor.py:21-68)
// ---------------------------------------------------------------------------------------
void vits_dp_validate(const TtsVitsDpCfg& c) {
  TTS_REQUIRE(c.in_channels >= 1 && c.hidden_channels >= 1 && c.hidden_channels <= 768, 1,
              "bad DurationPredictor configuration (hidden_channels 1..768)");
  TTS_REQUIRE(c.kernel_size >= 1 && c.kernel_size % 2 == 1 && c.kernel_size <= 11, 3,
              "DurationPredictor: odd kernel_size <= 11");
  TTS_REQUIRE(c.cond_channels >= 0 && c.language_emb_dim >= 0, 1, "cond_channels / language_emb_dim must be >= 0");
  TTS_REQUIRE(c.math_mode >= MATH_FP32 && c.math_mode <= MATH_LAST && c.math_mode != MATH_FP32_F16X3, 3,
              "DurationPredictor: math_mode FP32, FP32_X6 or BF16");
}

std::vector<int64_t> vits_dp_weight_shapes(const TtsVitsDpCfg& c) {
  const int64_t I = (int64_t)c.in_channels + c.language_emb_dim, F = c.hidden_channels, k = c.kernel_size;
  std::vector<int64_t> n = {F * I * k, F, F, F, F * F * k, F, F, F, F, 1};  // conv_1, norm_1, conv_2, norm_2, proj
  if (c.cond_channels > 0) { n.push_back(I * c.cond_channels); n.push_back(I); }     // cond
  if (c.language_emb_dim > 0) { n.push_back(I * c.language_emb_dim); n.push_back(I); }  // cond_lang
  return n;
}

VitsDp::VitsDp(const TtsVitsDpCfg& cfg, const float* const* hw, int device) : cfg_(cfg), device_(device) {
  vits_dp_validate(cfg_);
  DeviceGuard g(device_);
  const auto shapes = vits_dp_weight_shapes(cfg_);
  for (size_t i = 0; i < shapes.size(); ++i)
    TTS_REQUIRE(hw[i] != nullptr, 1, "weight pointer " + std::to_string(i) + " is NULL");
  const int I = cfg_.in_channels + cfg_.language_emb_dim, F = cfg_.hidden_channels, k = cfg_.kernel_size;
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
  auto put_conv = [&](Conv& cv, const float* w, const float* b, int Cout, int Cin, int K) {
    cv.Cin = Cin; cv.Cout = Cout; cv.K = K;
    // text batches are short: the split modes take the 32x128 tile, as the Glow encoder does
    cv.tile = is_split_mode(mode) ? 16 : conv_tile_for(mode, Cout, K, Cin, 1, false);
    const ConvTile t = conv_tile(mode, cv.tile);
    cv.n_chunks = ceil_div(Cin, t.CK);
    const size_t n = packed_conv_numel(mode, Cout, Cin, K, t);
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    TTS_REQUIRE(pack_conv(mode, w, Cout, Cin, K, t, host.data() + off) == 0, 3, "DP: scaled packing unsupported");
    fix.push_back({off, &cv.w});
    const size_t nb = (size_t)ceil_div(Cout, t.BM) * t.BM;
    const size_t offb = host.size();
    host.resize(offb + align(nb), 0.f);
    std::memcpy(host.data() + offb, b, Cout * sizeof(float));
    fix.push_back({offb, &cv.b});
  };
  put_conv(c1_, hw[0], hw[1], F, I, k);
  put(hw[2], F, &n1g_); put(hw[3], F, &n1b_);
  put_conv(c2_, hw[4], hw[5], F, F, k);
  put(hw[6], F, &n2g_); put(hw[7], F, &n2b_);
  put_conv(proj_, hw[8], hw[9], 1, F, 1);
  size_t wi = 10;
  if (cfg_.cond_channels > 0) {
    put(hw[wi], (size_t)I * cfg_.cond_channels, &cond_w_); put(hw[wi + 1], I, &cond_b_);
    wi += 2;
  }
  if (cfg_.language_emb_dim > 0) {
    put(hw[wi], (size_t)I * cfg_.language_emb_dim, &lang_w_); put(hw[wi + 1], I, &lang_b_);
    wi += 2;
  }
  TTS_REQUIRE(wi == shapes.size(), 2, "internal: DP weight count mismatch");
  if (hipMalloc(&arena_, host.size() * sizeof(float)) != hipSuccess) throw Error(4, "hipMalloc(weights) failed");
  TTS_HIP_CHECK(hipMemcpy(arena_, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
  for (auto& p : fix) *p.second = arena_ + p.first;
}

VitsDp::~VitsDp() {
  DeviceGuard g(device_);
  if (arena_) (void)hipFree(arena_);
  if (ws_) (void)hipFree(ws_);
}

void VitsDp::reserve(int B, int T) {
  const size_t plane = (size_t)B * T;
  const size_t I = (size_t)cfg_.in_channels + cfg_.language_emb_dim, F = cfg_.hidden_channels;
  // xin [I]; h, n [F]; cond vectors [2][B][I]
  const size_t need = (plane * (I + 2 * F) + 2 * (size_t)B * I + 5 * 64) * sizeof(float);
  if (need <= ws_bytes_) return;
  if (ws_) { TTS_HIP_CHECK(hipFree(ws_)); ws_ = nullptr; ws_bytes_ = 0; }
  if (hipMalloc(&ws_, need) != hipSuccess) throw Error(4, "hipMalloc(workspace) failed");
  ws_bytes_ = need;
}

void VitsDp::forward(const float* x, const float* x_mask, const float* g, const float* lang, int B, int T,
                     float* logw, hipStream_t s, Profiler* prof) {
  TTS_REQUIRE(x && x_mask && logw, 1, "NULL input/output pointer");
  TTS_REQUIRE(B >= 1 && T >= 1, 1, "batch and token count must be >= 1");
  TTS_REQUIRE(!g || cfg_.cond_channels > 0, 1, "g given to a DurationPredictor without a cond layer");
  TTS_REQUIRE(!lang || cfg_.language_emb_dim > 0, 1, "lang_emb given to a DurationPredictor without cond_lang");
  DeviceGuard dg(device_);
  reserve(B, T);
  const int I = cfg_.in_channels + cfg_.language_emb_dim, F = cfg_.hidden_channels, k = cfg_.kernel_size;
  const int mode = cfg_.math_mode;
  const size_t plane = (size_t)B * T;
  const double P = (double)plane;
  auto al = [](size_t n) { return (n + 63) & ~size_t(63); };
  float* p = ws_;
  float* xin = p; p += al(plane * I);
  float* h = p; p += al(plane * F);
  float* nb = p; p += al(plane * F);
  float* v1 = p; p += al((size_t)B * I);
  float* v2 = p;
  constexpr float kEps = 1e-4f;  // generic LayerNorm (normalization.py:6)

  auto conv = [&](const char* name, const Conv& cv, const float* in, float* out, float out_slope) {
    Conv1dArgs c{};
    c.x = in; c.w = cv.w; c.bias = cv.b; c.y = out; c.mask = x_mask;
    c.Cin = cv.Cin; c.Cout = cv.Cout; c.Tin = T; c.Tout = T;
    c.dil = 1; c.pad = (cv.K - 1) / 2; c.rep_pad = 0; c.n_chunks = cv.n_chunks;  // padding = kernel_size // 2
    c.in_slope = 1.f; c.out_slope = out_slope; c.zmode = 0; c.zdiv = 1.f;
    run(prof, s, name, 2.0 * P * cv.Cout * cv.Cin * cv.K, 4.0 * P * (cv.Cin + cv.Cout),
        [&] { launch_conv(mode, c, B, cv.K, cv.tile, s); });
  };
  // x = x + cond(g); x = x + cond_lang(lang) (:56-60); conv_1 reads x * x_mask (:62)
  const float* a1 = nullptr;
  const float* a2 = nullptr;
  if (g) {
    run(prof, s, "dp_cond", 2.0 * B * I * cfg_.cond_channels, 4.0 * B * (I + cfg_.cond_channels),
        [&] { launch_cond_vec(g, cond_w_, cond_b_, v1, B, cfg_.cond_channels, I, s); });
    a1 = v1;
  }
  if (lang) {
    const int L = cfg_.language_emb_dim;
    run(prof, s, "dp_cond_lang", 2.0 * B * I * L, 4.0 * B * (I + L),
        [&] { launch_cond_vec(lang, lang_w_, lang_b_, v2, B, L, I, s); });
    a2 = v2;
  }
  run(prof, s, "dp_input", 0.0, 4.0 * P * (2 * I + 1), [&] { launch_add_vec_mask(x, a1, a2, x_mask, xin, B, I, T, s); });
  // conv_1 -> relu -> norm_1 -> conv_2(x * mask) -> relu -> norm_2 -> proj(x * mask) * mask (:62-68);
  // the conv epilogues mask their output (the padded columns feed only the next masked read) and
  // the LayerNorm multiplies by the mask
  conv("dp_conv", c1_, xin, h, 0.f);
  run(prof, s, "dp_layernorm", 0.0, 8.0 * P * F,
      [&] { launch_layernorm(h, nullptr, n1g_, n1b_, x_mask, nb, B, F, T, kEps, false, s); });
  conv("dp_conv", c2_, nb, h, 0.f);
  run(prof, s, "dp_layernorm", 0.0, 8.0 * P * F,
      [&] { launch_layernorm(h, nullptr, n2g_, n2b_, x_mask, nb, B, F, T, kEps, false, s); });
  conv("dp_proj", proj_, nb, logw, 1.f);
  (void)k;
}

}  // namespace tts
