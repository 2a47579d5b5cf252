// VITS flow (ResidualCouplingBlocks) in the reverse (inference) direction:
//   for flow in reversed(flows): x = flip(x, channels); x = flow(x, mask, g, reverse=True)
// (TTS/tts/layers/vits/networks.py:217-232) with the mean-only ResidualCouplingBlock (:144-166):
//   h = pre(x0) * mask; h = WN(h, mask, g); m = post(h) * mask; x1 = (x1 - m) * mask.
//
// No data is flipped between flows: the flips only permute channels, so the flow at flip parity p
// (p = number of flips applied before it, mod 2) reads its x0 half and updates its x1 half of
// the UNflipped tensor, with pre's input columns and post's output rows reversed on the host when
// p is odd; an odd number of flows leaves one net flip, applied once at the end.  The coupling
// update runs in post's epilogue: with post negated on the host, (acc - b) * mask + x1 then
// * mask again (Conv1dArgs::mask_res) is exactly (x1 - m) * mask.
// WN (wavenet.py:94-115) reuses the Glow kernels; its speaker conditioning cond_layer(g)
// (:98-99, :103-107) is a per-(utterance, channel) vector added in the in-layer epilogue.
#include "vits.hpp"

#include <cstring>

#include "glow.hpp"

namespace tts {

std::vector<int64_t> vits_flow_weight_shapes(const TtsVitsFlowCfg& c) {
  std::vector<int64_t> n;
  const int half = c.channels / 2;
  const int H = c.hidden_channels;
  const int L = c.num_layers;
  for (int f = 0; f < c.num_flows; ++f) {
    n.push_back((int64_t)H * half);  // pre.weight [H][half][1]
    n.push_back(H);                  // pre.bias
    for (int l = 0; l < L; ++l) {
      n.push_back((int64_t)2 * H * H * c.kernel_size);  // enc.in_layers.l.weight (folded)
      n.push_back(2 * H);
    }
    for (int l = 0; l < L; ++l) {
      const int rsc = (l < L - 1) ? 2 * H : H;
      n.push_back((int64_t)rsc * H);  // enc.res_skip_layers.l.weight (folded)
      n.push_back(rsc);
    }
    if (c.cond_channels > 0) {
      n.push_back((int64_t)2 * H * L * c.cond_channels);  // enc.cond_layer.weight (folded)
      n.push_back((int64_t)2 * H * L);
    }
    n.push_back((int64_t)half * H);  // post.weight [half][H][1]
    n.push_back(half);               // post.bias
  }
  return n;
}

void vits_flow_validate(const TtsVitsFlowCfg& c) {
  TTS_REQUIRE(c.channels >= 2 && c.channels % 2 == 0, 1, "channels must be even (networks.py:114)");
  TTS_REQUIRE(c.hidden_channels >= 2 && c.hidden_channels % 2 == 0, 1, "hidden_channels must be even (wavenet.py:50)");
  TTS_REQUIRE(c.num_layers >= 1 && c.num_flows >= 1, 1, "bad VITS flow configuration");
  TTS_REQUIRE(c.kernel_size == 1 || c.kernel_size == 3 || c.kernel_size == 5 || c.kernel_size == 7 ||
                  c.kernel_size == 11,
              3, "kernel_size must be 1, 3, 5, 7 or 11");
  TTS_REQUIRE(c.dilation_rate >= 1, 1, "dilation_rate must be >= 1");
  int d = 1;
  for (int l = 0; l < c.num_layers; ++l) {
    TTS_REQUIRE((c.kernel_size - 1) * d <= 96, 3, "(kernel_size-1)*dilation above 96 is not implemented");
    d *= c.dilation_rate;
  }
  TTS_REQUIRE(c.cond_channels >= 0, 1, "cond_channels must be >= 0");
  TTS_REQUIRE(c.math_mode >= MATH_FP32 && c.math_mode <= MATH_LAST, 1, "unknown math_mode");
}

VitsFlow::VitsFlow(const TtsVitsFlowCfg& cfg, const float* const* hw, int device) : cfg_(cfg), device_(device) {
  vits_flow_validate(cfg_);
  amax_prepass_ = flow_amax_prepass();
  wn_fused_ = flow_wn_fused(cfg_.math_mode, cfg_.hidden_channels);
  wn_layer_ = flow_wn_layer(cfg_.math_mode, cfg_.hidden_channels, cfg_.kernel_size, cfg_.dilation_rate,
                            cfg_.num_layers);
  DeviceGuard g(device_);
  const auto shapes = vits_flow_weight_shapes(cfg_);
  for (size_t i = 0; i < shapes.size(); ++i)
    TTS_REQUIRE(hw[i] != nullptr, 1, "weight pointer " + std::to_string(i) + " is NULL");
  const int half = cfg_.channels / 2;
  const int H = cfg_.hidden_channels;
  const int L = cfg_.num_layers;
  const int F = cfg_.num_flows;
  const int mode = cfg_.math_mode;

  std::vector<float> host;
  auto align = [](size_t n) { return (n + 63) & ~size_t(63); };
  std::vector<std::pair<size_t, float**>> fix;
  auto put_raw = [&](const float* src, size_t n, float** dst) {
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    std::memcpy(host.data() + off, src, n * sizeof(float));
    fix.push_back({off, dst});
  };
  std::vector<float> wperm, bperm;
  auto put_conv = [&](Conv& cv, const float* w, const float* b, int Cin, int Cout, int K, int dil,
                      bool gate = false) {
    cv.Cin = Cin; cv.Cout = Cout; cv.K = K; cv.dil = dil;
    cv.tile = flow_conv_tile(mode, Cout, K, Cin, dil);
    cv.gated = gate && flow_gate_fused(mode, Cout / 2, K, dil);
    if (cv.gated) {
      gate_permute_rows(w, b, Cout / 2, Cin, K, wperm, bperm);
      w = wperm.data();
      b = bperm.data();
      cv.tile = kSplitGateTile;
    }
    const ConvTile t = conv_tile(mode, cv.tile);
    cv.n_chunks = ceil_div(Cin, t.CK);
    const size_t n = packed_conv_numel(mode, Cout, Cin, K, t);
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    cv.w_exp = pack_conv(mode, w, Cout, Cin, K, t, host.data() + off);
    fix.push_back({off, &cv.w});
    const size_t nb = (size_t)ceil_div(Cout, t.BM) * t.BM;
    const size_t offb = host.size();
    host.resize(offb + align(nb), 0.f);
    std::memcpy(host.data() + offb, b, Cout * sizeof(float));
    fix.push_back({offb, &cv.b});
  };

  flows_.resize(F);
  size_t wi = 0;
  for (int f = 0; f < F; ++f) {
    Flow& Fl = flows_[f];
    // flow f runs after F - f flips (networks.py:230-231)
    const bool flipped = ((F - f) & 1) != 0;
    Fl.in_off = flipped ? (int64_t)half : 0;
    Fl.out_off = flipped ? 0 : (int64_t)half;
    {  // pre: logical x0[c] = x[C-1-c] when flipped -> reads x[half + j] with column half-1-j
      std::vector<float> w((size_t)H * half);
      for (int h = 0; h < H; ++h)
        for (int j = 0; j < half; ++j) w[(size_t)h * half + j] = hw[wi][(size_t)h * half + (flipped ? half - 1 - j : j)];
      put_conv(Fl.pre, w.data(), hw[wi + 1], half, H, 1, 1);
      wi += 2;
    }
    Fl.in_layers.resize(L);
    Fl.res_skip.resize(L);
    int d = 1;
    for (int l = 0; l < L; ++l) {
      put_conv(Fl.in_layers[l], hw[wi], hw[wi + 1], H, 2 * H, cfg_.kernel_size, d, true);
      wi += 2;
      d *= cfg_.dilation_rate;
    }
    for (int l = 0; l < L; ++l) {
      put_conv(Fl.res_skip[l], hw[wi], hw[wi + 1], H, (l < L - 1) ? 2 * H : H, 1, 1);
      wi += 2;
    }
    if (cfg_.cond_channels > 0) {
      put_raw(hw[wi], (size_t)2 * H * L * cfg_.cond_channels, &Fl.cond_w);
      put_raw(hw[wi + 1], (size_t)2 * H * L, &Fl.cond_b);
      wi += 2;
    }
    {  // post, negated (reverse) and as is (forward); row s of the updated half is logical
       // x1[half-1-s] when flipped
      std::vector<float> w((size_t)half * H), b(half);
      for (int sign = -1; sign <= 1; sign += 2) {
        for (int s = 0; s < half; ++s) {
          const int src = flipped ? half - 1 - s : s;
          for (int h = 0; h < H; ++h) w[(size_t)s * H + h] = sign * hw[wi][(size_t)src * H + h];
          b[s] = sign * hw[wi + 1][src];
        }
        put_conv(sign < 0 ? Fl.post : Fl.post_fwd, w.data(), b.data(), H, half, 1, 1);
      }
      wi += 2;
    }
  }
  if (hipMalloc(&arena_, host.size() * sizeof(float)) != hipSuccess) throw Error(4, "hipMalloc(weights) failed");
  TTS_HIP_CHECK(hipMemcpy(arena_, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
  for (auto& p : fix) *p.second = arena_ + p.first;
}

VitsFlow::~VitsFlow() {
  DeviceGuard g(device_);
  if (arena_) (void)hipFree(arena_);
  if (ws_) (void)hipFree(ws_);
}

// f16x3 statistics: per flow (execution order) 2L + 2 groups of [B][64] slots: pre's input half,
// h before each in_layer, acts before each res_skip layer, the final skip (post's input)
size_t VitsFlow::amax_floats(int B) const {
  if (cfg_.math_mode != MATH_FP32_F16X3) return 0;
  return (size_t)cfg_.num_flows * (2 * cfg_.num_layers + 2) * B * 64;
}

void VitsFlow::reserve(int B, int T) {
  const int H = cfg_.hidden_channels;
  const size_t plane = (size_t)B * T;
  // h H, xin 2H, acts H, rs 2H, skip H; cond vectors [B][2*H*L]; odd num_flows: a C-channel copy
  const size_t odd = (cfg_.num_flows & 1) ? plane * cfg_.channels + 64 : 0;
  const size_t need =
      (plane * 7 * H + (size_t)B * 2 * H * cfg_.num_layers + 64 * 8 + odd + amax_floats(B) + 64) * sizeof(float);
  if (need <= ws_bytes_) return;
  if (ws_) { TTS_HIP_CHECK(hipFree(ws_)); ws_ = nullptr; ws_bytes_ = 0; }
  if (hipMalloc(&ws_, need) != hipSuccess) throw Error(4, "hipMalloc(workspace) failed");
  ws_bytes_ = need;
}

void VitsFlow::reverse(const float* x, const float* mask, const float* g, int B, int C, int T, float* y,
                       hipStream_t s, Profiler* prof) {
  run_flows(true, x, mask, g, B, C, T, y, s, prof);
}

// Forward: flow f sees x after f flips (networks.py:225-228); the weights were permuted for
// parity (F - f) mod 2 (the reverse direction's), which agrees when F is even.  With F odd the
// tensor is flipped once up front: flow f then sees f + 1 flips of the stored tensor, the same
// parity as F - f, and after the F flows and F flips the stored tensor is the output as is.
void VitsFlow::forward(const float* x, const float* mask, const float* g, int B, int C, int T, float* y,
                       hipStream_t s, Profiler* prof) {
  run_flows(false, x, mask, g, B, C, T, y, s, prof);
}

void VitsFlow::run_flows(bool rev, const float* x, const float* mask, const float* g, int B, int C, int T,
                         float* y, hipStream_t s, Profiler* prof) {
  TTS_REQUIRE(x && mask && y, 1, "NULL input/output pointer");
  TTS_REQUIRE(B >= 1 && T >= 1, 1, "batch and length must be >= 1");
  TTS_REQUIRE(C == cfg_.channels, 1, "channel count does not match the flow");
  TTS_REQUIRE(cfg_.cond_channels == 0 || g != nullptr, 1, "cond_channels > 0 requires g");
  DeviceGuard dg(device_);
  reserve(B, T);
  const int H = cfg_.hidden_channels;
  const int L = cfg_.num_layers;
  const size_t plane = (size_t)B * T;
  auto al = [](size_t n) { return (n + 63) & ~size_t(63); };
  float* p = ws_;
  float* hb = p; p += al(plane * H);
  float* xin = p; p += al(plane * 2 * H);
  float* acts = p; p += al(plane * H);
  float* rs = p; p += al(plane * 2 * H);
  float* skip = p; p += al(plane * H);
  float* cvec = p; p += al((size_t)B * 2 * H * L);
  const bool h3 = cfg_.math_mode == MATH_FP32_F16X3;
  unsigned* amax = h3 ? reinterpret_cast<unsigned*>(p) : nullptr;
  p += al(amax_floats(B));
  const int ng = 2 * L + 2;
  auto slots = [&](int fi, int kind) -> unsigned* { return h3 ? amax + ((size_t)fi * ng + kind) * B * 64 : nullptr; };
  if (h3) TTS_HIP_CHECK(hipMemsetAsync(amax, 0, amax_floats(B) * sizeof(unsigned), s));
  const bool odd = (cfg_.num_flows & 1) != 0;
  const double P = (double)B * T;
  float* out = y;  // reverse: the flow updates `work` in place; an odd count flips it into y at the end
  float* work = (odd && rev) ? p : y;
  y = work;
  if (!rev && odd) {  // forward, odd count: the one up-front flip (x may alias y: flip through p)
    const float* src = x;
    if (x == work) {
      TTS_HIP_CHECK(hipMemcpyAsync(p, x, plane * C * sizeof(float), hipMemcpyDeviceToDevice, s));
      src = p;
    }
    run(prof, s, "vits_flip", 0.0, 8.0 * P * C, [&] { launch_channel_flip(src, work, B, C, T, s); });
  } else if (work != x) {
    TTS_HIP_CHECK(hipMemcpyAsync(work, x, plane * C * sizeof(float), hipMemcpyDeviceToDevice, s));
  }
  const int64_t xbs = (int64_t)C * T;  // batch stride of x / y

  auto conv = [&](const char* name, const Conv& cv, const float* in, int64_t in_bstride, float* o, const float* m,
                  const float* res, int64_t o_bstride, const float* cv_vec, int64_t cv_bstride, bool mask_res,
                  const unsigned* amax_in = nullptr, unsigned* amax_out = nullptr) {
    Conv1dArgs a{};
    a.gate = cv.gated ? cv.Cout / 2 : 0;
    a.amax_in = amax_in; a.amax_out = amax_out; a.w_exp = cv.w_exp;
    a.x = in; a.w = cv.w; a.bias = cv.b; a.y = o; a.mask = m; a.x_bstride = in_bstride; a.res = res;
    a.o_bstride = o_bstride; a.cvec = cv_vec; a.cvec_bstride = cv_bstride; a.mask_res = mask_res ? 1 : 0;
    a.Cin = cv.Cin; a.Cout = cv.Cout; a.Tin = T; a.Tout = T;
    a.dil = cv.dil; a.pad = cv.dil * (cv.K - 1) / 2; a.rep_pad = 0; a.n_chunks = cv.n_chunks;
    a.in_slope = 1.f; a.out_slope = 1.f; a.zmode = 0; a.zdiv = 1.f;
    run(prof, s, name, 2.0 * P * cv.Cout * cv.Cin * cv.K, 4.0 * P * (cv.Cin + cv.Cout + (res ? cv.Cout : 0)),
        [&] { launch_conv(cfg_.math_mode, a, B, cv.K, cv.tile, s); });
  };

  const int NF = cfg_.num_flows;
  for (int k = 0; k < NF; ++k) {
    const int f = rev ? NF - 1 - k : k;  // flow index; k is the execution index
    const Flow& Fl = flows_[f];
    if (cfg_.cond_channels > 0) {  // g = cond_layer(g)  (wavenet.py:98-99): [B][2*H*L]
      run(prof, s, "vits_cond", 2.0 * B * 2 * H * L * cfg_.cond_channels, 4.0 * B * 2 * H * L,
          [&] { launch_cond_vec(g, Fl.cond_w, Fl.cond_b, cvec, B, cfg_.cond_channels, 2 * H * L, s); });
    }
    const int fi = k;
    const int half = C / 2;
    if (h3 && (fi == 0 || amax_prepass_))  // statistics of x0 (pre's input half); later flows: the previous post conv
      run(prof, s, "vits_amax_x0", 0.0, 2.0 * P * half,
          [&] { launch_amax(y + Fl.in_off * T, (int64_t)half * T, B, slots(fi, 0), s, xbs); });
    // h = pre(x0) * mask  (networks.py:157)
    conv("vits_pre", Fl.pre, y + Fl.in_off * T, xbs, hb, mask, nullptr, 0, nullptr, 0, false, slots(fi, 0),
         slots(fi, 1));
    float* hcur = hb;
    float* hnext = xin;  // the one-launch layers' second h buffer
    for (int l = 0; l < L; ++l) {
      // x_in = in_layers[l](h) (+ g_l)   (wavenet.py:101-107)
      const float* gl = cfg_.cond_channels > 0 ? cvec + (size_t)l * 2 * H : nullptr;
      if (wn_layer_) {  // wavenet.py:101-115 in one launch
        GlowWnLayerArgs w = wn_layer_weights(cfg_.math_mode, Fl.in_layers[l], Fl.res_skip[l], H, T, l, L);
        w.h_in = hcur; w.h_out = hnext; w.skip = skip; w.mask = mask;
        w.cvec = gl; w.cvec_bstride = (int64_t)2 * H * L;
        w.amax_h = slots(fi, 1 + l);
        w.amax_out = l < L - 1 ? slots(fi, 2 + l) : slots(fi, 2 * L + 1);
        run(prof, s, "vits_wn_layer", 2.0 * P * H * (2.0 * H * Fl.in_layers[l].K + Fl.res_skip[l].Cout),
            4.0 * P * H * 4, [&] { launch_glow_wn_layer(cfg_.math_mode, w, B, s); });
        std::swap(hcur, hnext);
        continue;
      }
      if (Fl.in_layers[l].gated) {  // in_layer + g_l + gate (:108) in one launch
        conv("vits_wn_in_gate", Fl.in_layers[l], hb, 0, acts, nullptr, nullptr, 0, gl, (int64_t)2 * H * L, false,
             slots(fi, 1 + l), slots(fi, 1 + L + l));
      } else {
        conv("vits_wn_in", Fl.in_layers[l], hb, 0, xin, nullptr, nullptr, 0, gl, (int64_t)2 * H * L, false,
             slots(fi, 1 + l));
        run(prof, s, "vits_gate", 0.0, 12.0 * P * H,
            [&] { launch_glow_gate(xin, acts, B, H, T, s, slots(fi, 1 + L + l)); });  // :108
      }
      if (l < L - 1 && wn_fused_) {  // :109-113 in one launch (Conv1dArgs::wn_rows)
        const Conv& cv = Fl.res_skip[l];
        Conv1dArgs a{};
        a.x = acts; a.w = cv.w; a.bias = cv.b; a.y = hb; a.z = skip; a.mask = mask; a.wn_rows = H;
        a.amax_in = slots(fi, 1 + L + l); a.amax_out = slots(fi, 2 + l); a.w_exp = cv.w_exp;
        a.Cin = cv.Cin; a.Cout = cv.Cout; a.Tin = T; a.Tout = T; a.dil = 1; a.pad = 0; a.n_chunks = cv.n_chunks;
        a.in_slope = 1.f; a.out_slope = 1.f; a.zmode = l == 0 ? 1 : 2; a.zdiv = 1.f;
        run(prof, s, "vits_wn_res_skip_update", 2.0 * P * cv.Cout * cv.Cin, 4.0 * P * (cv.Cin + 2 * cv.Cout),
            [&] { launch_conv(cfg_.math_mode, a, B, 1, cv.tile, s); });
      } else {
        conv("vits_wn_res_skip", Fl.res_skip[l], acts, 0, rs, nullptr, nullptr, 0, nullptr, 0, false,
             slots(fi, 1 + L + l));  // :109
        run(prof, s, "vits_wn_update", 0.0, 24.0 * P * H, [&] {
          launch_glow_wn_update(hb, skip, rs, mask, B, H, T, l == 0, l == L - 1, s,
                                l < L - 1 ? slots(fi, 2 + l) : slots(fi, 2 * L + 1));
        });  // :110-115
      }
    }
    // reverse: x1 = (x1 - post(h) * mask) * mask; forward: x1 = post(h) * mask + x1 * mask; in
    // place on y (networks.py:159-165)
    float* x1 = y + Fl.out_off * T;
    // the half it writes is the next flow's x0 (the flip alternates the halves): its statistics
    conv("vits_post", rev ? Fl.post : Fl.post_fwd, skip, 0, x1, mask, x1, xbs, nullptr, 0, true,
         slots(fi, 2 * L + 1), k + 1 < NF && !amax_prepass_ ? slots(fi + 1, 0) : nullptr);
  }
  if (odd && rev) run(prof, s, "vits_flip", 0.0, 8.0 * P * C, [&] { launch_channel_flip(work, out, B, C, T, s); });
}

}  // namespace tts

namespace tts {

// ---------------------------------------------------------------------------------------
// PosteriorEncoder (networks.py:235-288)
// ---------------------------------------------------------------------------------------
std::vector<int64_t> vits_posterior_weight_shapes(const TtsVitsPosteriorCfg& c) {
  std::vector<int64_t> n;
  const int H = c.hidden_channels;
  const int L = c.num_layers;
  n.push_back((int64_t)H * c.in_channels);  // pre.weight [H][in][1]
  n.push_back(H);
  for (int l = 0; l < L; ++l) {
    n.push_back((int64_t)2 * H * H * c.kernel_size);  // enc.in_layers.l.weight (folded)
    n.push_back(2 * H);
  }
  for (int l = 0; l < L; ++l) {
    const int rsc = (l < L - 1) ? 2 * H : H;
    n.push_back((int64_t)rsc * H);  // enc.res_skip_layers.l.weight (folded)
    n.push_back(rsc);
  }
  if (c.cond_channels > 0) {
    n.push_back((int64_t)2 * H * L * c.cond_channels);  // enc.cond_layer.weight (folded)
    n.push_back((int64_t)2 * H * L);
  }
  n.push_back((int64_t)2 * c.out_channels * H);  // proj.weight [2 out][H][1]
  n.push_back(2 * c.out_channels);
  return n;
}

void vits_posterior_validate(const TtsVitsPosteriorCfg& c) {
  TTS_REQUIRE(c.in_channels >= 1 && c.out_channels >= 1, 1, "bad posterior encoder channels");
  TTS_REQUIRE(c.hidden_channels >= 2 && c.hidden_channels % 2 == 0, 1, "hidden_channels must be even (wavenet.py:50)");
  TTS_REQUIRE(c.num_layers >= 1, 1, "num_layers must be >= 1");
  TTS_REQUIRE(c.kernel_size == 1 || c.kernel_size == 3 || c.kernel_size == 5 || c.kernel_size == 7 ||
                  c.kernel_size == 11,
              3, "kernel_size must be 1, 3, 5, 7 or 11");
  TTS_REQUIRE(c.dilation_rate >= 1, 1, "dilation_rate must be >= 1");
  int d = 1;
  for (int l = 0; l < c.num_layers; ++l) {
    TTS_REQUIRE((c.kernel_size - 1) * d <= 96, 3, "(kernel_size-1)*dilation above 96 is not implemented");
    d *= c.dilation_rate;
  }
  TTS_REQUIRE(c.cond_channels >= 0, 1, "cond_channels must be >= 0");
  TTS_REQUIRE(c.math_mode >= MATH_FP32 && c.math_mode <= MATH_LAST, 1, "unknown math_mode");
}

VitsPosterior::VitsPosterior(const TtsVitsPosteriorCfg& cfg, const float* const* hw, int device)
    : cfg_(cfg), device_(device) {
  vits_posterior_validate(cfg_);
  wn_layer_ = flow_wn_layer(cfg_.math_mode, cfg_.hidden_channels, cfg_.kernel_size, cfg_.dilation_rate,
                            cfg_.num_layers);
  DeviceGuard g(device_);
  const auto shapes = vits_posterior_weight_shapes(cfg_);
  for (size_t i = 0; i < shapes.size(); ++i)
    TTS_REQUIRE(hw[i] != nullptr, 1, "weight pointer " + std::to_string(i) + " is NULL");
  const int H = cfg_.hidden_channels;
  const int L = cfg_.num_layers;
  const int mode = cfg_.math_mode;
  std::vector<float> host;
  auto align = [](size_t n) { return (n + 63) & ~size_t(63); };
  std::vector<std::pair<size_t, float**>> fix;
  auto put_raw = [&](const float* src, size_t n, float** dst) {
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    std::memcpy(host.data() + off, src, n * sizeof(float));
    fix.push_back({off, dst});
  };
  std::vector<float> wperm, bperm;
  auto put_conv = [&](Conv& cv, const float* w, const float* b, int Cin, int Cout, int K, int dil, bool gate = false) {
    cv.Cin = Cin; cv.Cout = Cout; cv.K = K; cv.dil = dil;
    cv.tile = flow_conv_tile(mode, Cout, K, Cin, dil);
    cv.gated = gate && flow_gate_fused(mode, Cout / 2, K, dil);
    if (cv.gated) {
      gate_permute_rows(w, b, Cout / 2, Cin, K, wperm, bperm);
      w = wperm.data();
      b = bperm.data();
      cv.tile = kSplitGateTile;
    }
    const ConvTile t = conv_tile(mode, cv.tile);
    cv.n_chunks = ceil_div(Cin, t.CK);
    const size_t n = packed_conv_numel(mode, Cout, Cin, K, t);
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    cv.w_exp = pack_conv(mode, w, Cout, Cin, K, t, host.data() + off);
    fix.push_back({off, &cv.w});
    const size_t nb = (size_t)ceil_div(Cout, t.BM) * t.BM;
    const size_t offb = host.size();
    host.resize(offb + align(nb), 0.f);
    std::memcpy(host.data() + offb, b, Cout * sizeof(float));
    fix.push_back({offb, &cv.b});
  };
  size_t wi = 0;
  put_conv(pre_, hw[0], hw[1], cfg_.in_channels, H, 1, 1);
  wi = 2;
  in_layers_.resize(L);
  res_skip_.resize(L);
  int d = 1;
  for (int l = 0; l < L; ++l, wi += 2) {
    put_conv(in_layers_[l], hw[wi], hw[wi + 1], H, 2 * H, cfg_.kernel_size, d, true);
    d *= cfg_.dilation_rate;
  }
  for (int l = 0; l < L; ++l, wi += 2) put_conv(res_skip_[l], hw[wi], hw[wi + 1], H, (l < L - 1) ? 2 * H : H, 1, 1);
  if (cfg_.cond_channels > 0) {
    put_raw(hw[wi], (size_t)2 * H * L * cfg_.cond_channels, &cond_w_);
    put_raw(hw[wi + 1], (size_t)2 * H * L, &cond_b_);
    wi += 2;
  }
  put_conv(proj_, hw[wi], hw[wi + 1], H, 2 * cfg_.out_channels, 1, 1);
  if (hipMalloc(&arena_, host.size() * sizeof(float)) != hipSuccess) throw Error(4, "hipMalloc(weights) failed");
  TTS_HIP_CHECK(hipMemcpy(arena_, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
  for (auto& p : fix) *p.second = arena_ + p.first;
}

VitsPosterior::~VitsPosterior() {
  DeviceGuard g(device_);
  if (arena_) (void)hipFree(arena_);
  if (ws_) (void)hipFree(ws_);
}

// f16x3 statistics: the input spectrogram, h before each in_layer, acts before each res_skip,
// the final skip (proj's input): 2L + 2 groups of [B][64] slots
size_t VitsPosterior::amax_floats(int B) const {
  if (cfg_.math_mode != MATH_FP32_F16X3) return 0;
  return (size_t)(2 * cfg_.num_layers + 2) * B * 64;
}

void VitsPosterior::reserve(int B, int T) {
  const int H = cfg_.hidden_channels;
  const size_t plane = (size_t)B * T;
  // h H, xin 2H, acts H, rs 2H, skip H, stats 2 out; cond vectors [B][2HL]
  const size_t need = (plane * (7 * H + 2 * cfg_.out_channels) + (size_t)B * 2 * H * cfg_.num_layers + 64 * 8 +
                       amax_floats(B) + 64) * sizeof(float);
  if (need <= ws_bytes_) return;
  if (ws_) { TTS_HIP_CHECK(hipFree(ws_)); ws_ = nullptr; ws_bytes_ = 0; }
  if (hipMalloc(&ws_, need) != hipSuccess) throw Error(4, "hipMalloc(workspace) failed");
  ws_bytes_ = need;
}

void VitsPosterior::forward(const float* x, const float* mask, const float* g, const float* eps, int B, int C, int T,
                            float* z, float* m, float* logs, hipStream_t s, Profiler* prof) {
  TTS_REQUIRE(x && mask && z, 1, "NULL input/output pointer");
  TTS_REQUIRE(B >= 1 && T >= 1, 1, "batch and length must be >= 1");
  TTS_REQUIRE(C == cfg_.in_channels, 1, "channel count does not match the posterior encoder");
  TTS_REQUIRE(cfg_.cond_channels == 0 || g != nullptr, 1, "cond_channels > 0 requires g");
  TTS_REQUIRE((int64_t)C * T * 4 < (int64_t(1) << 31), 3, "posterior encoder: input plane exceeds 2 GiB");
  DeviceGuard dg(device_);
  reserve(B, T);
  const int H = cfg_.hidden_channels;
  const int L = cfg_.num_layers;
  const int Co = cfg_.out_channels;
  const size_t plane = (size_t)B * T;
  auto al = [](size_t n) { return (n + 63) & ~size_t(63); };
  float* p = ws_;
  float* hb = p; p += al(plane * H);
  float* xin = p; p += al(plane * 2 * H);
  float* acts = p; p += al(plane * H);
  float* rs = p; p += al(plane * 2 * H);
  float* skip = p; p += al(plane * H);
  float* stats = p; p += al(plane * 2 * Co);
  float* cvec = p; p += al((size_t)B * 2 * H * L);
  const bool h3 = cfg_.math_mode == MATH_FP32_F16X3;
  unsigned* amax = h3 ? reinterpret_cast<unsigned*>(p) : nullptr;
  auto slots = [&](int kind) -> unsigned* { return h3 ? amax + (size_t)kind * B * 64 : nullptr; };
  if (h3) TTS_HIP_CHECK(hipMemsetAsync(amax, 0, amax_floats(B) * sizeof(unsigned), s));
  const double P = (double)B * T;
  auto conv = [&](const char* name, const Conv& cv, const float* in, float* o, const float* msk, const float* cv_vec,
                  const unsigned* amax_in, unsigned* amax_out) {
    Conv1dArgs a{};
    a.gate = cv.gated ? cv.Cout / 2 : 0;
    a.amax_in = amax_in; a.amax_out = amax_out; a.w_exp = cv.w_exp;
    a.x = in; a.w = cv.w; a.bias = cv.b; a.y = o; a.mask = msk;
    a.cvec = cv_vec; a.cvec_bstride = cv_vec ? (int64_t)2 * H * L : 0;
    a.Cin = cv.Cin; a.Cout = cv.Cout; a.Tin = T; a.Tout = T;
    a.dil = cv.dil; a.pad = cv.dil * (cv.K - 1) / 2; a.rep_pad = 0; a.n_chunks = cv.n_chunks;
    a.in_slope = 1.f; a.out_slope = 1.f; a.zmode = 0; a.zdiv = 1.f;
    run(prof, s, name, 2.0 * P * cv.Cout * cv.Cin * cv.K, 4.0 * P * (cv.Cin + cv.Cout),
        [&] { launch_conv(cfg_.math_mode, a, B, cv.K, cv.tile, s); });
  };
  if (cfg_.cond_channels > 0)  // g = cond_layer(g) (wavenet.py:98-99)
    run(prof, s, "vits_post_cond", 2.0 * B * 2 * H * L * cfg_.cond_channels, 4.0 * B * 2 * H * L,
        [&] { launch_cond_vec(g, cond_w_, cond_b_, cvec, B, cfg_.cond_channels, 2 * H * L, s); });
  if (h3)  // statistics of the spectrogram (pre's input)
    run(prof, s, "vits_post_amax", 0.0, 4.0 * P * C, [&] { launch_amax(x, (int64_t)C * T, B, slots(0), s); });
  // h = pre(x) * mask (networks.py:283)
  conv("vits_post_pre", pre_, x, hb, mask, nullptr, slots(0), slots(1));
  float* hcur = hb;
  float* hnext = xin;  // the one-launch layers' second h buffer
  for (int l = 0; l < L; ++l) {  // WN (wavenet.py:94-115)
    const float* gl = cfg_.cond_channels > 0 ? cvec + (size_t)l * 2 * H : nullptr;
    if (wn_layer_) {  // wavenet.py:101-115 in one launch
      GlowWnLayerArgs w = wn_layer_weights(cfg_.math_mode, in_layers_[l], res_skip_[l], H, T, l, L);
      w.h_in = hcur; w.h_out = hnext; w.skip = skip; w.mask = mask;
      w.cvec = gl; w.cvec_bstride = (int64_t)2 * H * L;
      w.amax_h = slots(1 + l);
      w.amax_out = l < L - 1 ? slots(2 + l) : slots(2 * L + 1);
      run(prof, s, "vits_post_wn_layer", 2.0 * P * H * (2.0 * H * in_layers_[l].K + res_skip_[l].Cout),
          4.0 * P * H * 4, [&] { launch_glow_wn_layer(cfg_.math_mode, w, B, s); });
      std::swap(hcur, hnext);
      continue;
    }
    if (in_layers_[l].gated) {
      conv("vits_post_wn_in_gate", in_layers_[l], hb, acts, nullptr, gl, slots(1 + l), slots(1 + L + l));
    } else {
      conv("vits_post_wn_in", in_layers_[l], hb, xin, nullptr, gl, slots(1 + l), nullptr);
      run(prof, s, "vits_post_gate", 0.0, 12.0 * P * H,
          [&] { launch_glow_gate(xin, acts, B, H, T, s, slots(1 + L + l)); });
    }
    if (l < L - 1 && flow_wn_fused(cfg_.math_mode, H)) {  // :109-113 in one launch (Conv1dArgs::wn_rows)
      const Conv& cv = res_skip_[l];
      Conv1dArgs a{};
      a.x = acts; a.w = cv.w; a.bias = cv.b; a.y = hb; a.z = skip; a.mask = mask; a.wn_rows = H;
      a.amax_in = slots(1 + L + l); a.amax_out = slots(2 + l); a.w_exp = cv.w_exp;
      a.Cin = cv.Cin; a.Cout = cv.Cout; a.Tin = T; a.Tout = T; a.dil = 1; a.pad = 0; a.n_chunks = cv.n_chunks;
      a.in_slope = 1.f; a.out_slope = 1.f; a.zmode = l == 0 ? 1 : 2; a.zdiv = 1.f;
      run(prof, s, "vits_post_wn_res_skip_update", 2.0 * P * cv.Cout * cv.Cin, 4.0 * P * (cv.Cin + 2 * cv.Cout),
          [&] { launch_conv(cfg_.math_mode, a, B, 1, cv.tile, s); });
    } else {
      conv("vits_post_wn_res_skip", res_skip_[l], acts, rs, nullptr, nullptr, slots(1 + L + l), nullptr);
      run(prof, s, "vits_post_wn_update", 0.0, 24.0 * P * H, [&] {
        launch_glow_wn_update(hb, skip, rs, mask, B, H, T, l == 0, l == L - 1, s,
                              l < L - 1 ? slots(2 + l) : slots(2 * L + 1));
      });
    }
  }
  // stats = proj(h) * mask (networks.py:285), then split and sample (:286-287)
  conv("vits_post_proj", proj_, skip, stats, mask, nullptr, slots(2 * L + 1), nullptr);
  run(prof, s, "vits_post_sample", 0.0, 4.0 * P * Co * 6,
      [&] { launch_posterior_sample(stats, eps, mask, z, m, logs, B, Co, T, s); });
}

}  // namespace tts
