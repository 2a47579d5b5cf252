// Glow-TTS decoder flow, reverse direction, on the MFMA conv kernel + fused elementwise tails.
// Reference: TTS/tts/layers/glow_tts/decoder.py:113-137, glow.py:102-137 and :201-230,
// wavenet.py:94-115, normalization.py:88-103.
#include "glow.hpp"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>

namespace tts {

// log(det(W)) of an S x S matrix in fp64 (partial-pivot LU).  The InvConvNear weight is born with
// det > 0 (glow.py:94-95); otherwise this returns what torch.logdet gives (glow.py:128): -inf for a
// singular matrix, NaN for a negative determinant.  Only the forward direction's logdet reads it, so a
// checkpoint with such a weight still loads and runs reverse (the reference's inference path)
double logdet_fp64(const float* w, int S) {
  std::vector<double> a((size_t)S * S);
  for (int i = 0; i < S * S; ++i) a[i] = w[i];
  double ld = 0.0;
  int sign = 1;
  for (int k = 0; k < S; ++k) {
    int p = k;
    for (int r = k + 1; r < S; ++r)
      if (std::fabs(a[(size_t)r * S + k]) > std::fabs(a[(size_t)p * S + k])) p = r;
    if (a[(size_t)p * S + k] == 0.0) return -std::numeric_limits<double>::infinity();
    if (p != k) {
      for (int c = 0; c < S; ++c) std::swap(a[(size_t)p * S + c], a[(size_t)k * S + c]);
      sign = -sign;
    }
    const double piv = a[(size_t)k * S + k];
    if (piv < 0) sign = -sign;
    ld += std::log(std::fabs(piv));
    for (int r = k + 1; r < S; ++r) {
      const double f = a[(size_t)r * S + k] / piv;
      for (int c = k; c < S; ++c) a[(size_t)r * S + c] -= f * a[(size_t)k * S + c];
    }
  }
  return sign > 0 ? ld : std::numeric_limits<double>::quiet_NaN();
}

int flow_conv_tile(int mode, int Cout, int K, int Cin, int dil) {
  // A/B switches for the flow convs' tile (split modes, plain tiles 0-19): TTS_MI355X_FLOW_TILE_K
  // for the in_layers (K > 1), TTS_MI355X_FLOW_TILE_1X1 for start / res_skip / end
  if (is_split_mode(mode)) {
    const char* e = std::getenv(K > 1 ? "TTS_MI355X_FLOW_TILE_K" : "TTS_MI355X_FLOW_TILE_1X1");
    if (e && *e) {
      const int t = std::atoi(e);
      TTS_REQUIRE(t >= 0 && t < kSplitGateTile, 1, "flow tile override out of range");
      return t;
    }
  }
  return conv_tile_for(mode, Cout, K, Cin, dil, false);
}

bool flow_gate_fused(int mode, int H, int K, int dil) {
  // opt-in: at config 3 (144 workgroups per in_layer launch) the fused launch measured 1.63 ms
  // against 1.27 + 0.39 ms for the pair, but the decoder's wall time 2.95 ms against 2.84 ms
  const char* e = std::getenv("TTS_MI355X_FLOW_GATE");
  if (!(e && e[0] == '1')) return false;
  return is_split_mode(mode) && H % 64 == 0 && (K == 3 || K == 5 || K == 7) && (K - 1) * dil <= (K - 1) * 5;
}

bool flow_wn_fused(int mode, int H) {
  // opt-in (TTS_MI355X_WN_FUSION=1): the res_skip conv's epilogue updates h and the skip sum itself
  // (Conv1dArgs::wn_rows) for every WN layer but the last.  Measured at config 3 ([16,80,768]):
  // 22.7 us per fused launch against 14.3 + 8.3 us for the pair, decoder 2.67 vs 2.61 ms: the
  // epilogue's h / skip gathers after the last MFMA cost what the update kernel did
  const char* e = std::getenv("TTS_MI355X_WN_FUSION");
  return (e && e[0] == '1') && is_split_mode(mode) && H % 32 == 0;
}

bool flow_wn_layer(int mode, int H, int K, int dilation_rate, int L) {
  const char* e = std::getenv("TTS_MI355X_WN_LAYER");
  if (e && e[0] == '0') return false;
  if (flow_wn_fused(mode, H)) return false;  // the opt-in arms keep their own launches
  int d = 1;
  for (int l = 0; l < L; ++l) {
    if (!glow_wn_layer_supported(mode, H, K, d) || flow_gate_fused(mode, H, K, d)) return false;
    d *= dilation_rate;
  }
  return true;
}

bool flow_amax_prepass() {
  const char* e = std::getenv("TTS_MI355X_FLOW_AMAX_PREPASS");
  return e && e[0] == '1';
}

void gate_permute_rows(const float* w, const float* b, int H, int Cin, int K, std::vector<float>& wp,
                       std::vector<float>& bp) {
  const size_t row = (size_t)Cin * K;
  wp.resize((size_t)2 * H * row);
  bp.resize((size_t)2 * H);
  for (int rho = 0; rho < 2 * H; ++rho) {
    const int o = gate_row_order(rho, H);
    std::memcpy(wp.data() + rho * row, w + o * row, row * sizeof(float));
    bp[rho] = b[o];
  }
}

std::vector<int64_t> glow_weight_shapes(const TtsGlowDecoderCfg& c) {
  std::vector<int64_t> n;
  const int C2 = c.in_channels * c.num_squeeze;
  const int H = c.hidden_channels;
  const int S = c.num_splits;
  for (int f = 0; f < c.num_flow_blocks; ++f) {
    n.push_back(C2);                      // actnorm.logs
    n.push_back(C2);                      // actnorm.bias
    n.push_back((int64_t)S * S);          // invconv.weight_inv
    n.push_back((int64_t)S * S);          // invconv.weight (the forward direction)
    n.push_back((int64_t)H * (C2 / 2));   // start.weight
    n.push_back(H);                       // start.bias
    if (c.c_in_channels > 0) {            // wn.cond_layer (weight norm folded), wavenet.py:64-66
      n.push_back((int64_t)2 * H * c.num_coupling_layers * c.c_in_channels);
      n.push_back((int64_t)2 * H * c.num_coupling_layers);
    }
    for (int l = 0; l < c.num_coupling_layers; ++l) {
      n.push_back((int64_t)2 * H * H * c.kernel_size);
      n.push_back(2 * H);
      const int rsc = (l < c.num_coupling_layers - 1) ? 2 * H : H;
      n.push_back((int64_t)rsc * H);
      n.push_back(rsc);
    }
    n.push_back((int64_t)C2 * H);  // end.weight
    n.push_back(C2);               // end.bias
  }
  return n;
}

void glow_validate(const TtsGlowDecoderCfg& c) {
  TTS_REQUIRE(c.in_channels >= 1 && c.hidden_channels >= 2 && c.num_flow_blocks >= 1 &&
                  c.num_coupling_layers >= 1,
              1, "bad Glow decoder configuration");
  TTS_REQUIRE(c.num_squeeze >= 1, 1, "num_squeeze must be >= 1");
  TTS_REQUIRE(c.num_splits == 2 || c.num_splits == 4 || c.num_splits == 8, 3, "num_splits must be 2, 4 or 8");
  TTS_REQUIRE((c.in_channels * c.num_squeeze) % c.num_splits == 0, 1,
              "channels*num_squeeze must be divisible by num_splits (glow.py:109)");
  TTS_REQUIRE((c.in_channels * c.num_squeeze) % 2 == 0, 1, "coupling needs an even channel count");
  TTS_REQUIRE(c.kernel_size % 2 == 1, 1, "kernel_size must be odd (wavenet.py:49)");
  TTS_REQUIRE(c.kernel_size == 1 || c.kernel_size == 3 || c.kernel_size == 5 || c.kernel_size == 7 ||
                  c.kernel_size == 11,
              3, "kernel_size must be 1, 3, 5, 7 or 11");
  int d = 1;
  for (int l = 0; l < c.num_coupling_layers; ++l) {
    TTS_REQUIRE((c.kernel_size - 1) * d <= 96, 3, "(kernel_size-1)*dilation above 96 is not implemented");
    d *= c.dilation_rate;
  }
  TTS_REQUIRE(c.c_in_channels >= 0, 1, "c_in_channels must be >= 0");
  TTS_REQUIRE(c.math_mode >= MATH_FP32 && c.math_mode <= MATH_LAST, 1, "unknown math_mode");
}

GlowDecoder::GlowDecoder(const TtsGlowDecoderCfg& cfg, const float* const* hw, int device)
    : cfg_(cfg), device_(device) {
  glow_validate(cfg_);
  amax_prepass_ = flow_amax_prepass();
  wn_fused_ = flow_wn_fused(cfg_.math_mode, cfg_.hidden_channels);
  wn_layer_ = flow_wn_layer(cfg_.math_mode, cfg_.hidden_channels, cfg_.kernel_size, cfg_.dilation_rate,
                            cfg_.num_coupling_layers);
  {
    const char* e = std::getenv("TTS_MI355X_WN_END");
    const int C2 = cfg_.in_channels * cfg_.num_squeeze;
    wn_end_ = wn_layer_ && !(e && e[0] == '0') && C2 % 32 == 0 && C2 <= 2 * cfg_.hidden_channels;
    const char* et = std::getenv("TTS_MI355X_WN_TAIL");
    wn_tail_ = wn_end_ && !(et && et[0] == '0') && cfg_.num_splits == 4 && 3 * C2 <= 4 * cfg_.hidden_channels;
  }
  DeviceGuard g(device_);
  const auto shapes = glow_weight_shapes(cfg_);
  for (size_t i = 0; i < shapes.size(); ++i)
    TTS_REQUIRE(hw[i] != nullptr, 1, "weight pointer " + std::to_string(i) + " is NULL");
  const int C2 = cfg_.in_channels * cfg_.num_squeeze;
  const int H = cfg_.hidden_channels;
  const int S = cfg_.num_splits;
  const int L = cfg_.num_coupling_layers;

  std::vector<float> host;
  auto align = [](size_t n) { return (n + 63) & ~size_t(63); };
  struct Pending { size_t off; float** dst; };
  std::vector<std::pair<size_t, float**>> fix;  // (offset, pointer to patch)
  auto put = [&](const float* src, size_t n, float** dst) {
    const size_t off = host.size();
    host.resize(off + align(n), 0.f);
    std::memcpy(host.data() + off, src, n * sizeof(float));
    fix.push_back({off, dst});
  };
  std::vector<float> wperm, bperm;
  auto put_conv = [&](Conv& cv, const float* w, const float* b, int Cin, int Cout, int K, int dil,
                      bool gate = false) {
    cv.Cin = Cin; cv.Cout = Cout; cv.K = K; cv.dil = dil;
    const int mode = cfg_.math_mode;
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

  flows_.resize(cfg_.num_flow_blocks);
  size_t wi = 0;
  for (int f = 0; f < cfg_.num_flow_blocks; ++f) {
    Flow& F = flows_[f];
    put(hw[wi], C2, &F.logs); put(hw[wi + 1], C2, &F.bias); put(hw[wi + 2], (size_t)S * S, &F.winv);
    put(hw[wi + 3], (size_t)S * S, &F.w);
    {  // forward logdet per unmasked frame: torch.sum(logs) (normalization.py:100) and
       // torch.logdet(weight) * (C2 / S) (glow.py:128), here in fp64 from the fp32 parameters
      double sl = 0.0;
      for (int c = 0; c < C2; ++c) sl += (double)hw[wi][c];
      F.per_len = sl + logdet_fp64(hw[wi + 3], S) * ((double)C2 / S);
    }
    wi += 4;
    put_conv(F.start, hw[wi], hw[wi + 1], C2 / 2, H, 1, 1); wi += 2;
    if (cfg_.c_in_channels > 0) {  // cond_layer stays fp32 [2HL][c_in] (launch_cond_vec)
      put(hw[wi], (size_t)2 * H * L * cfg_.c_in_channels, &F.cond_w);
      put(hw[wi + 1], (size_t)2 * H * L, &F.cond_b);
      wi += 2;
    }
    F.in_layers.resize(L); F.res_skip.resize(L);
    int d = 1;
    for (int l = 0; l < L; ++l) {
      put_conv(F.in_layers[l], hw[wi], hw[wi + 1], H, 2 * H, cfg_.kernel_size, d, true); wi += 2;
      const int rsc = (l < L - 1) ? 2 * H : H;
      put_conv(F.res_skip[l], hw[wi], hw[wi + 1], H, rsc, 1, 1); wi += 2;
      d *= cfg_.dilation_rate;
    }
    put_conv(F.end, hw[wi], hw[wi + 1], H, C2, 1, 1); wi += 2;
  }
  if (hipMalloc(&arena_, host.size() * sizeof(float)) != hipSuccess) throw Error(4, "hipMalloc(weights) failed");
  TTS_HIP_CHECK(hipMemcpy(arena_, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
  for (auto& p : fix) *p.second = arena_ + p.first;
}

GlowDecoder::~GlowDecoder() {
  DeviceGuard g(device_);
  if (arena_) (void)hipFree(arena_);
  if (ws_) (void)hipFree(ws_);
}

// f16x3 statistics: per flow (in execution order) 2L + 2 groups of [B][64] slots: the start conv's
// input x0, h before each in_layer, acts before each res_skip layer, and the final skip
size_t GlowDecoder::amax_floats(int B) const {
  if (cfg_.math_mode != MATH_FP32_F16X3) return 0;
  return (size_t)cfg_.num_flow_blocks * (2 * cfg_.num_coupling_layers + 2) * B * 64;
}

void GlowDecoder::reserve(int B, int Th) {
  const int C2 = cfg_.in_channels * cfg_.num_squeeze;
  const int H = cfg_.hidden_channels;
  const size_t plane = (size_t)B * Th;
  // xs C2, h H, xin 2H, acts H, rs 2H, skip H, out C2, msq 1; cond vectors [B][2HL]; f16x3: max-abs
  // slot groups
  const size_t cond = cfg_.c_in_channels > 0 ? (size_t)B * 2 * H * cfg_.num_coupling_layers + 64 : 0;
  // forward direction: logdet partials [flows][B][kGlowLogdetParts] fp64
  const size_t ldp = (size_t)cfg_.num_flow_blocks * B * kGlowLogdetParts * 2 + 64;
  const size_t need = plane * (2 * C2 + 7 * H + 1) * sizeof(float) + 64 * 10 * sizeof(float) +
                      (cond + amax_floats(B) + ldp) * sizeof(float);
  if (need <= ws_bytes_) return;
  if (ws_) { TTS_HIP_CHECK(hipFree(ws_)); ws_ = nullptr; ws_bytes_ = 0; }
  if (hipMalloc(&ws_, need) != hipSuccess) throw Error(4, "hipMalloc(workspace) failed");
  ws_bytes_ = need;
}

void GlowDecoder::reverse(const float* x, const float* mask, const float* g, int B, int C, int T, float* y,
                          hipStream_t s, Profiler* prof) {
  run_flows(true, x, mask, g, B, C, T, y, nullptr, s, prof);
}

void GlowDecoder::forward(const float* x, const float* mask, const float* g, int B, int C, int T, float* y,
                          float* logdet, hipStream_t s, Profiler* prof) {
  run_flows(false, x, mask, g, B, C, T, y, logdet, s, prof);
}

void GlowDecoder::run_flows(bool rev, const float* x, const float* mask, const float* g, int B, int C, int T,
                            float* y, float* logdet, hipStream_t s, Profiler* prof) {
  TTS_REQUIRE(x && mask && y, 1, "NULL input/output pointer");
  TTS_REQUIRE(cfg_.c_in_channels == 0 || g != nullptr, 1, "c_in_channels > 0 requires g");
  TTS_REQUIRE(B >= 1, 1, "batch must be >= 1");
  TTS_REQUIRE(C == cfg_.in_channels, 1, "channel count does not match the decoder");
  const int nsq = cfg_.num_squeeze;
  const int Th = T / nsq;
  TTS_REQUIRE(Th >= 1, 1, "T too short for num_squeeze");
  DeviceGuard dg(device_);
  reserve(B, Th);
  const int C2 = C * nsq;
  const int H = cfg_.hidden_channels;
  const int L = cfg_.num_coupling_layers;
  const int NF = cfg_.num_flow_blocks;
  const size_t plane = (size_t)B * Th;
  auto al = [](size_t n) { return (n + 63) & ~size_t(63); };
  float* p = ws_;
  float* xs = p; p += al(plane * C2);
  float* hb = p; p += al(plane * H);
  float* xin = p; p += al(plane * 2 * H);
  float* acts = p; p += al(plane * H);
  float* rs = p; p += al(plane * 2 * H);
  float* skip = p; p += al(plane * H);
  float* out = p; p += al(plane * C2);
  float* msq = p; p += al(plane);
  float* cvec = nullptr;  // cond_layer(g) of the current flow, [B][2HL] (wavenet.py:98-99)
  if (cfg_.c_in_channels > 0) { cvec = p; p += al((size_t)B * 2 * H * L); }
  const bool h3 = cfg_.math_mode == MATH_FP32_F16X3;
  unsigned* amax = h3 ? reinterpret_cast<unsigned*>(p) : nullptr;
  p += al(amax_floats(B));
  double* ldp = reinterpret_cast<double*>(p);  // forward: logdet partials [NF][B][npb]
  const int ng = 2 * L + 2;
  // slot group: flow fi (execution order), kind 0 = x0, 1 + l = h_l, 1 + L + l = acts_l, 2L + 1 = skip
  auto slots = [&](int fi, int kind) -> unsigned* { return h3 ? amax + ((size_t)fi * ng + kind) * B * 64 : nullptr; };
  if (h3) TTS_HIP_CHECK(hipMemsetAsync(amax, 0, amax_floats(B) * sizeof(unsigned), s));

  // squeeze (decoder.py:128, :8-28); without squeeze the mask is used as is
  const double P = (double)B * Th;  // squeezed positions
  if (nsq > 1) {
    run(prof, s, "glow_squeeze", 0.0, 8.0 * P * C2 + 8.0 * P,
        [&] { launch_glow_squeeze(x, mask, xs, msq, B, C, T, nsq, s); });
  } else {
    TTS_HIP_CHECK(hipMemcpyAsync(xs, x, plane * C2 * sizeof(float), hipMemcpyDeviceToDevice, s));
    TTS_HIP_CHECK(hipMemcpyAsync(msq, mask, plane * sizeof(float), hipMemcpyDeviceToDevice, s));
  }

  auto conv = [&](const char* name, const Conv& cv, const float* in, int64_t in_bstride, float* o, const float* m,
                  const unsigned* amax_in = nullptr, unsigned* amax_out = nullptr, const float* cv_vec = nullptr) {
    Conv1dArgs a{};
    a.gate = cv.gated ? cv.Cout / 2 : 0;
    a.x = in; a.w = cv.w; a.bias = cv.b; a.y = o; a.mask = m; a.x_bstride = in_bstride;
    a.cvec = cv_vec; a.cvec_bstride = cv_vec ? (int64_t)2 * H * L : 0;
    a.amax_in = amax_in; a.amax_out = amax_out; a.w_exp = cv.w_exp;
    a.Cin = cv.Cin; a.Cout = cv.Cout; a.Tin = Th; a.Tout = Th;
    a.dil = cv.dil; a.pad = cv.dil * (cv.K - 1) / 2; a.rep_pad = 0; a.n_chunks = cv.n_chunks;
    a.in_slope = 1.f; a.out_slope = 1.f; a.zmode = 0; a.zdiv = 1.f;
    run(prof, s, name, 2.0 * P * cv.Cout * cv.Cin * cv.K, 4.0 * P * (cv.Cin + cv.Cout),
        [&] { launch_conv(cfg_.math_mode, a, B, cv.K, cv.tile, s); });
  };

  // out = end(WN(start(x_0) * mask, mask, g)) of flow block f (glow.py:212-214); fi = execution index
  // x0 statistics: the max-abs slots of flow fi's start-conv input come from the previous
  // elementwise kernel (the tail / head / coupling kernels) except for the first reverse flow, or
  // from a strided pre-pass for every flow (TTS_MI355X_FLOW_AMAX_PREPASS=1)
  // reverse flows with the one-launch layers: the last layer of flow fi may also run the flow's
  // inverse tail and the next flow's start conv (wn_tail_), leaving the next flow's h in pending_h
  float* pending_h = nullptr;
  auto coupling_net = [&](const Flow& F, int fi, const Flow* next_start = nullptr) -> bool {
    bool tail_fused = false;
    if (cvec)  // g = cond_layer(g) (wavenet.py:98-99); every flow has its own cond_layer
      run(prof, s, "glow_cond", 2.0 * B * 2 * H * L * cfg_.c_in_channels, 4.0 * B * 2 * H * L,
          [&] { launch_cond_vec(g, F.cond_w, F.cond_b, cvec, B, cfg_.c_in_channels, 2 * H * L, s); });
    if (h3 && ((rev && fi == 0) || amax_prepass_))
      run(prof, s, "glow_amax_x0", 0.0, 2.0 * P * C2,
          [&] { launch_amax(xs, (int64_t)(C2 / 2) * Th, B, slots(fi, 0), s, (int64_t)C2 * Th); });
    // h = start(x_0) * mask  (glow.py:212; x_0 = first C2/2 channels of xs)
    float* hcur = hb;
    float* hnext = xin;  // the one-launch layers' second h buffer (they have no xin plane)
    if (pending_h) {  // computed by the previous flow's last layer
      hcur = pending_h;
      hnext = pending_h == hb ? xin : hb;
      pending_h = nullptr;
    } else {
      conv("glow_start", F.start, xs, (int64_t)C2 * Th, hb, msq, slots(fi, 0), slots(fi, 1));
    }
    for (int l = 0; l < L; ++l) {
      // x_in = in_layers[l](h) + g_l  (wavenet.py:101-107; g_l = cond rows [2Hl, 2H(l+1)))
      const float* gl = cvec ? cvec + (size_t)l * 2 * H : nullptr;
      if (wn_layer_) {  // wavenet.py:101-115 in one launch
        const Conv& ci = F.in_layers[l];
        const Conv& cr = F.res_skip[l];
        GlowWnLayerArgs w = wn_layer_weights(cfg_.math_mode, ci, cr, H, Th, l, L);
        w.h_in = hcur; w.h_out = hnext; w.skip = skip; w.mask = msq;
        w.cvec = gl; w.cvec_bstride = (int64_t)2 * H * L;
        w.amax_h = slots(fi, 1 + l);
        w.amax_out = l < L - 1 ? slots(fi, 2 + l) : slots(fi, 2 * L + 1);
        if (wn_end_ && l == L - 1) {  // glow.py:214 in the same launch
          const ConvTile te = conv_tile(cfg_.math_mode, F.end.tile);
          w.w_end = F.end.w; w.b_end = F.end.b; w.end_out = out; w.end_rows = F.end.Cout;
          w.end_steps = F.end.n_chunks * (te.CK / 16);
          w.end_blocks = ceil_div(F.end.Cout, te.BM) * te.BM / 32;
          w.w_exp_end = F.end.w_exp;
          w.amax_out = nullptr;  // skip is not written: nothing reads its statistics
          if (next_start) {  // glow.py:222-224 -> :102-137 -> normalization.py:96-98, then the next :212
            const Conv& cs = next_start->start;
            const ConvTile ts = conv_tile(cfg_.math_mode, cs.tile);
            w.tail_x = xs; w.winv = F.winv; w.logs = F.logs; w.abias = F.bias;
            w.sigmoid_scale = cfg_.sigmoid_scale;
            w.w_start = cs.w; w.b_start = cs.b; w.h_next = hnext; w.amax_hnext = slots(fi + 1, 1);
            w.start_steps = cs.n_chunks * (ts.CK / 16);
            w.start_blocks = ceil_div(cs.Cout, ts.BM) * ts.BM / 32;
            w.w_exp_start = cs.w_exp;
            pending_h = hnext;
            tail_fused = true;
          }
        }
        run(prof, s, "glow_wn_layer", 2.0 * P * H * (2.0 * H * ci.K + cr.Cout), 4.0 * P * H * 4,
            [&] { launch_glow_wn_layer(cfg_.math_mode, w, B, s); });
        std::swap(hcur, hnext);
        continue;
      }
      if (F.in_layers[l].gated) {  // wavenet.py:101 + :108 in one launch, acts straight from the epilogue
        conv("glow_wn_in_gate", F.in_layers[l], hb, 0, acts, nullptr, slots(fi, 1 + l), slots(fi, 1 + L + l), gl);
      } else {
        conv("glow_wn_in", F.in_layers[l], hb, 0, xin, nullptr, slots(fi, 1 + l), nullptr, gl);  // wavenet.py:101
        run(prof, s, "glow_gate", 0.0, 12.0 * P * H,
            [&] { launch_glow_gate(xin, acts, B, H, Th, s, slots(fi, 1 + L + l)); });  // :108
      }
      if (l < L - 1 && wn_fused_) {  // :109-113 in one launch (Conv1dArgs::wn_rows)
        const Conv& cv = F.res_skip[l];
        Conv1dArgs a{};
        a.x = acts; a.w = cv.w; a.bias = cv.b; a.y = hb; a.z = skip; a.mask = msq; a.wn_rows = H;
        a.amax_in = slots(fi, 1 + L + l); a.amax_out = slots(fi, 2 + l); a.w_exp = cv.w_exp;
        a.Cin = cv.Cin; a.Cout = cv.Cout; a.Tin = Th; a.Tout = Th; a.dil = 1; a.pad = 0; a.n_chunks = cv.n_chunks;
        a.in_slope = 1.f; a.out_slope = 1.f; a.zmode = l == 0 ? 1 : 2; a.zdiv = 1.f;
        run(prof, s, "glow_wn_res_skip_update", 2.0 * P * cv.Cout * cv.Cin, 4.0 * P * (cv.Cin + 2 * cv.Cout),
            [&] { launch_conv(cfg_.math_mode, a, B, 1, cv.tile, s); });
      } else {
        conv("glow_wn_res_skip", F.res_skip[l], acts, 0, rs, nullptr, slots(fi, 1 + L + l));  // :109
        run(prof, s, "glow_wn_update", 0.0, 24.0 * P * H, [&] {
          launch_glow_wn_update(hb, skip, rs, msq, B, H, Th, l == 0, l == L - 1, s,
                                l < L - 1 ? slots(fi, 2 + l) : slots(fi, 2 * L + 1));
        });  // :110-115
      }
    }
    if (!(wn_layer_ && wn_end_))
      conv("glow_end", F.end, skip, 0, out, nullptr, slots(fi, 2 * L + 1));  // glow.py:214
    return tail_fused;
  };

  if (rev) {
    // flows in reverse: for each block (last first): CouplingBlock^-1, InvConvNear^-1, ActNorm^-1
    for (int f = NF - 1; f >= 0; --f) {
      const Flow& F = flows_[f];
      const int fi = NF - 1 - f;
      if (coupling_net(F, fi, (wn_tail_ && f > 0) ? &flows_[f - 1] : nullptr)) continue;
      GlowTailArgs ta{};
      ta.x = xs; ta.out = out; ta.mask = msq; ta.winv = F.winv; ta.logs = F.logs; ta.bias = F.bias;
      ta.C2 = C2; ta.Th = Th; ta.S = cfg_.num_splits; ta.sigmoid_scale = cfg_.sigmoid_scale;
      ta.amax_x0 = (h3 && f > 0 && !amax_prepass_) ? slots(fi + 1, 0) : nullptr;
      run(prof, s, "glow_tail", 0.0, 16.0 * P * C2, [&] { launch_glow_tail(ta, B, s); });
    }
  } else {
    // flows in order (decoder.py:119-133): ActNorm, InvConvNear, CouplingBlock per block; the head of
    // block 0 runs alone, every later head inside the previous block's coupling kernel
    GlowHeadArgs ha{};
    ha.x = xs; ha.mask = msq; ha.w = flows_[0].w; ha.logs = flows_[0].logs; ha.bias = flows_[0].bias;
    ha.C2 = C2; ha.Th = Th; ha.S = cfg_.num_splits;
    ha.amax_x0 = (h3 && !amax_prepass_) ? slots(0, 0) : nullptr;
    run(prof, s, "glow_head", 0.0, 8.0 * P * C2, [&] { launch_glow_head(ha, B, s); });
    const int npb = glow_couple_parts(C2, cfg_.num_splits, Th);
    double per_len = 0.0;
    for (int f = 0; f < NF; ++f) {
      const Flow& F = flows_[f];
      per_len += F.per_len;
      coupling_net(F, f);
      GlowCoupleArgs ca{};
      ca.x = xs; ca.out = out; ca.mask = msq; ca.C2 = C2; ca.Th = Th; ca.S = cfg_.num_splits;
      ca.sigmoid_scale = cfg_.sigmoid_scale;
      ca.ld_part = logdet ? ldp + (size_t)f * B * npb : nullptr;
      if (f + 1 < NF) {
        ca.w = flows_[f + 1].w; ca.logs = flows_[f + 1].logs; ca.bias = flows_[f + 1].bias;
        ca.amax_x0 = (h3 && !amax_prepass_) ? slots(f + 1, 0) : nullptr;
      }
      run(prof, s, f + 1 < NF ? "glow_couple_head" : "glow_couple", 0.0, 16.0 * P * C2,
          [&] { launch_glow_couple_fwd(ca, B, s); });
    }
    if (logdet)
      run(prof, s, "glow_logdet", 0.0, 8.0 * B * NF * npb + 4.0 * P,
          [&] { launch_glow_logdet(ldp, NF, npb, msq, Th, per_len, logdet, B, s); });
  }
  if (nsq > 1) {
    run(prof, s, "glow_unsqueeze", 0.0, 8.0 * P * C2 + 4.0 * P,
        [&] { launch_glow_unsqueeze(xs, msq, y, B, C, Th, nsq, s); });
  } else {
    TTS_HIP_CHECK(hipMemcpyAsync(y, xs, plane * C2 * sizeof(float), hipMemcpyDeviceToDevice, s));
  }
}

}  // namespace tts
