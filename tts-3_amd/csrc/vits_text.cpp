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
  TTS_REQUIRE(c.language_emb_dim == 0, 3,
              "VITS TextEncoder: language embeddings (language_emb_dim > 0, networks.py:63-64) are not implemented");
  glow_encoder_validate(vits_text_encoder_glow_cfg(c));
}

// networks.py:66-77: RelativePositionTransformer(in = out = hidden, layer_norm_type "2",
// rel_attn_window_size 4); proj is carried as the Glow encoder's proj_m / proj_s pair
TtsGlowEncoderCfg vits_text_encoder_glow_cfg(const TtsVitsTextEncoderCfg& c) {
  TtsGlowEncoderCfg g{};
  g.num_chars = c.n_vocab;
  g.out_channels = c.out_channels;
  g.hidden_channels = c.hidden_channels;
  g.hidden_channels_dp = c.hidden_channels;  // no duration predictor (with_dp = false)
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
  std::vector<int64_t> n = glow_encoder_weight_shapes(g, false);
  // the last four are proj_m / proj_s (weight, bias): the reference has one proj [2 out][H][1]
  n.resize(n.size() - 4);
  n.push_back((int64_t)2 * c.out_channels * c.hidden_channels);
  n.push_back((int64_t)2 * c.out_channels);
  return n;
}

VitsTextEncoder::VitsTextEncoder(const TtsVitsTextEncoderCfg& cfg, const float* const* hw, int device) : cfg_(cfg) {
  vits_text_encoder_validate(cfg_);
  const auto shapes = vits_text_encoder_weight_shapes(cfg_);
  for (size_t i = 0; i < shapes.size(); ++i)
    TTS_REQUIRE(hw[i] != nullptr, 1, "weight pointer " + std::to_string(i) + " is NULL");
  const size_t np = shapes.size() - 2;  // proj.weight, proj.bias
  const size_t wsz = (size_t)cfg_.out_channels * cfg_.hidden_channels;
  std::vector<const float*> ptrs(hw, hw + np);
  // m, logs = torch.split(proj(x) * mask, out, dim=1) (networks.py:98-99): rows [0, out) and [out, 2 out)
  ptrs.push_back(hw[np]);
  ptrs.push_back(hw[np + 1]);
  ptrs.push_back(hw[np] + wsz);
  ptrs.push_back(hw[np + 1] + cfg_.out_channels);
  enc_ = std::make_unique<GlowEncoder>(vits_text_encoder_glow_cfg(cfg_), ptrs.data(), device, false);
}

void VitsTextEncoder::forward(const int64_t* tok, const int64_t* len, int B, int T, float* x, float* m, float* logs,
                              float* x_mask, hipStream_t s, Profiler* prof) {
  TTS_REQUIRE(x && m && logs, 1, "NULL output pointer");
  enc_->forward(tok, len, nullptr, B, T, m, logs, nullptr, x_mask, s, prof, x);
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
  TTS_REQUIRE(c.language_emb_dim == 0, 3,
              "StochasticDurationPredictor: language embeddings (cond_lang) are not implemented");
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
  if (c.cond_channels > 0) { n.push_back(H * c.cond_channels); n.push_back(H); }  // cond
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
  // xs, h, a, u [H]; hp [29]; z [2]; cond vector [B][H]
  const size_t need = (plane * (4 * (size_t)H + 3 * kSdpBins - 1 + 2) + (size_t)B * H + 7 * 64) * sizeof(float);
  if (need <= ws_bytes_) return;
  if (ws_) { TTS_HIP_CHECK(hipFree(ws_)); ws_ = nullptr; ws_bytes_ = 0; }
  if (hipMalloc(&ws_, need) != hipSuccess) throw Error(4, "hipMalloc(workspace) failed");
  ws_bytes_ = need;
}

void VitsSdp::reverse(const float* x, const float* x_mask, const float* g, const float* noise, float noise_scale,
                      int B, int T, float* logw, hipStream_t s, Profiler* prof) {
  TTS_REQUIRE(x && x_mask && logw, 1, "NULL input/output pointer");
  TTS_REQUIRE(cfg_.cond_channels == 0 || g != nullptr, 1, "cond_channels > 0 requires g");
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
  float* cvec = p;                     // cond(g) [B][H]

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

  // x = pre(x) [+ cond(g)] (:249-252); x = proj(DDS(x, mask)) * mask (:257-258)
  const float* cv = nullptr;
  if (cond_w_) {
    run(prof, s, "sdp_cond", 2.0 * B * H * cfg_.cond_channels, 4.0 * B * (H + cfg_.cond_channels),
        [&] { launch_cond_vec(g, cond_w_, cond_b_, cvec, B, cfg_.cond_channels, H, s); });
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

}  // namespace tts
