// HiFiGAN generator executor: builds the launch plan of HifiganGenerator.forward
// (TTS/vocoder/models/hifigan_generator.py:236-265) from the constructor arguments,
// owns the packed weights and the activation workspace in HBM, and enqueues the kernels
// on the caller's stream.
#include "hifigan.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace tts {

namespace {
bool valid_conv_k(int k) { return k == 1 || k == 3 || k == 5 || k == 7 || k == 11; }
}  // namespace

// ---------------------------------------------------------------------------------------
// Weight inventory (order documented in tts_mi355x.h)
// ---------------------------------------------------------------------------------------
std::vector<int64_t> hifigan_weight_shapes(const TtsHifiganCfg& c) {
  std::vector<int64_t> n;
  const int C0 = c.upsample_initial_channel;
  n.push_back((int64_t)C0 * c.in_channels * 7);
  n.push_back(C0);
  for (int i = 0; i < c.num_upsamples; ++i) {
    const int ci = C0 >> i, co = C0 >> (i + 1);
    n.push_back((int64_t)ci * co * c.upsample_kernel_sizes[i]);
    n.push_back(co);
  }
  for (int i = 0; i < c.num_upsamples; ++i) {
    const int ch = C0 >> (i + 1);
    for (int j = 0; j < c.num_kernels; ++j) {
      const int k = c.resblock_kernel_sizes[j];
      const int nconv = (c.resblock_type == 1) ? 6 : 2;
      for (int m = 0; m < nconv; ++m) {
        n.push_back((int64_t)ch * ch * k);
        n.push_back(ch);
      }
    }
  }
  const int cl = C0 >> c.num_upsamples;
  n.push_back((int64_t)c.out_channels * cl * 7);
  if (c.conv_post_bias) n.push_back(c.out_channels);
  if (c.cond_channels > 0) {
    n.push_back((int64_t)C0 * c.cond_channels);
    n.push_back(C0);
  }
  if (c.cond_in_each_up_layer) {
    for (int i = 0; i < c.num_upsamples; ++i) {
      n.push_back((int64_t)(C0 >> (i + 1)) * c.cond_channels);
      n.push_back(C0 >> (i + 1));
    }
  }
  return n;
}

void hifigan_validate(const TtsHifiganCfg& c) {
  TTS_REQUIRE(c.in_channels >= 1, 1, "in_channels must be >= 1");
  TTS_REQUIRE(c.out_channels == 1, 3, "only out_channels == 1 is implemented");
  TTS_REQUIRE(c.resblock_type == 1 || c.resblock_type == 2, 1, "resblock_type must be '1' or '2'");
  TTS_REQUIRE(c.num_kernels >= 1 && c.num_kernels <= TTS_MAX_KERNELS, 1, "bad num_kernels");
  TTS_REQUIRE(c.num_upsamples >= 1 && c.num_upsamples <= TTS_MAX_UPSAMPLES, 1, "bad num_upsamples");
  const int need_d = c.resblock_type == 1 ? 3 : 2;
  TTS_REQUIRE(c.num_dilations >= need_d && c.num_dilations <= TTS_MAX_DILATIONS, 1,
              "resblock_dilation_sizes too short for the resblock type");
  for (int j = 0; j < c.num_kernels; ++j) {
    TTS_REQUIRE(valid_conv_k(c.resblock_kernel_sizes[j]), 3,
                "resblock kernel size " + std::to_string(c.resblock_kernel_sizes[j]) +
                    " not implemented (1,3,5,7,11)");
    for (int m = 0; m < need_d; ++m) {
      const int d = c.resblock_dilation_sizes[j][m];
      TTS_REQUIRE(d >= 1 && (c.resblock_kernel_sizes[j] - 1) * d <= 96, 3,
                  "resblock (kernel_size-1)*dilation must be <= 96");
    }
  }
  int C = c.upsample_initial_channel;
  for (int i = 0; i < c.num_upsamples; ++i) {
    const int u = c.upsample_factors[i];
    TTS_REQUIRE(u == 2 || u == 4 || u == 8, 3, "upsample factor must be 2, 4 or 8");
    TTS_REQUIRE(c.upsample_kernel_sizes[i] == 2 * u, 3,
                "upsample kernel size must equal 2*factor (polyphase kernel)");
    C >>= 1;
    TTS_REQUIRE(C >= 1, 1, "upsample_initial_channel too small for the number of upsamples");
  }
  TTS_REQUIRE(c.inference_padding >= 0, 1, "inference_padding must be >= 0");
  TTS_REQUIRE(c.cond_channels >= 0, 1, "cond_channels must be >= 0");
  TTS_REQUIRE(!c.cond_in_each_up_layer || c.cond_channels > 0, 1, "cond_in_each_up_layer needs cond_channels > 0");
  TTS_REQUIRE(c.math_mode >= MATH_FP32 && c.math_mode <= MATH_LAST, 1, "unknown math_mode");
}

// ---------------------------------------------------------------------------------------
Hifigan::Hifigan(const TtsHifiganCfg& cfg, const float* const* hw, int device)
    : cfg_(cfg), device_(device) {
  hifigan_validate(cfg_);
  DeviceGuard g(device_);
  const auto shapes = hifigan_weight_shapes(cfg_);
  for (size_t i = 0; i < shapes.size(); ++i)
    TTS_REQUIRE(hw[i] != nullptr, 1, "weight pointer " + std::to_string(i) + " is NULL");

  // 1) describe layers, 2) size the arena, 3) pack on host, 4) one upload.
  const int C0 = cfg_.upsample_initial_channel;
  const int mode = cfg_.math_mode;
  // TTS_MI355X_NO_PAIR_FUSION=1 keeps every resblock conv a separate launch (the tests' reference arm)
  const char* nf = std::getenv("TTS_MI355X_NO_PAIR_FUSION");
  const bool pair_fusion = !(nf && nf[0] == '1');
  const char* pf = std::getenv("TTS_MI355X_POST_FUSION");
  post_fusion_ = !(pf && pf[0] == '0');
  const char* ms = std::getenv("TTS_MI355X_MRF_STREAMS");
  nbs_ = ms ? std::max(1, std::min(std::atoi(ms), cfg.num_kernels)) : cfg.num_kernels;
  nbs_env_ = ms != nullptr;
  const char* sb = std::getenv("TTS_MI355X_SUBBATCH");
  n_lanes_ = sb ? std::max(1, std::min(std::atoi(sb), 8)) : 2;
  rb2_geo64_ = resblock2_geo64(mode);
  // bf16 planes: every MRF stage length is then a multiple of 8 (the Winograd DMA's 16-byte rows)
  const char* bp = std::getenv("TTS_MI355X_BF16_PLANES");
  planes16_ = mode == MATH_BF16 && !(bp && bp[0] == '0') && cfg_.num_upsamples >= 1 &&
              cfg_.upsample_factors[0] % 8 == 0;
  size_t wi = 0;
  std::vector<std::pair<const float*, const float*>> src;  // (w, b) per packed layer
  auto add_conv = [&](int Cin, int Cout, int K, int dil, const char* fam, bool res, int lmode, bool pair128 = false) {
    ConvLayer L;
    L.Cin = Cin; L.Cout = Cout; L.K = K; L.dil = dil; L.pad = dil * (K - 1) / 2;
    L.mode = lmode;
    L.tile = conv_tile_for(lmode, Cout, K, Cin, dil, res);
    if (pair128) {
      // a bf16 128-channel pair (resblock_pair128): the direct packing with 16-channel chunks
      // (tile 7: 128 x 128, one 16-channel group per chunk) instead of the Winograd packing
      L.tile = 7;
      const ConvTile t = conv_tile(lmode, L.tile);
      L.n_chunks = ceil_div(Cin, t.CK);
      L.w_numel = packed_conv_numel(lmode, Cout, Cin, K, t);
      L.b_numel = (int64_t)ceil_div(Cout, t.BM) * t.BM;
      L.name = std::string(fam) + "_k" + std::to_string(K) + "_c" + std::to_string(Cout);
      return L;
    }
    // the MRF convs at >= 128 channels, kernels 7 and 11: Winograd F(4,4) (wino8_kernel.hpp;
    // MI355X, B=32: k11 c128 2.20 -> 1.73 ms, k7 c128 1.56 -> 1.43, k11 c256 1.16 -> 0.80, k7 c256
    // 0.82 -> 0.60 per launch; TTS_MI355X_WINO=0 keeps the direct kernel).  Kernel 3 is supported
    // but measured within 2-4% of the direct kernel (1.05 vs 1.07 ms at c128), not worth the
    // Winograd rounding, so it stays direct.
    // TTS_MI355X_WINO_K3=1 (A/B): kernel 3 at >= 256 channels (stage 1's per-conv k3 path; the
    // 128-channel k3 block stays a whole-block launch) on the Winograd kernel as well
    const bool wino_k3 = [] {
      const char* e = std::getenv("TTS_MI355X_WINO_K3");
      return e && e[0] == '1';
    }();
    const bool k_ok = K >= 7 || (K == 3 && Cout >= 256 && wino_k3);
    if (std::string(fam) == "mrf_conv" && k_ok && wino_enabled() && wino_supported(lmode, Cout, Cin, K, dil)) {
      L.tile = kSplitWinoTile;
      fam = "mrf_wino";
    }
    const ConvTile t = conv_tile(lmode, L.tile);
    L.n_chunks = ceil_div(Cin, t.CK);
    L.w_numel = packed_conv_numel(lmode, Cout, Cin, K, t);
    L.b_numel = (int64_t)ceil_div(Cout, t.BM) * t.BM;
    L.name = std::string(fam) + "_k" + std::to_string(K) + "_c" + std::to_string(Cout);
    return L;
  };

  pre_ = add_conv(cfg_.in_channels, C0, 7, 1, "conv_pre", false, mode);
  src.push_back({hw[wi], hw[wi + 1]}); wi += 2;
  for (int i = 0; i < cfg_.num_upsamples; ++i) {
    ConvTLayer L;
    L.Cin = C0 >> i; L.Cout = C0 >> (i + 1); L.U = cfg_.upsample_factors[i];
    L.mode = mode;
    if (is_split_mode(mode)) {
      // split modes: the K=2 polyphase conv form (Conv1dArgs::ups), U*Cout rows
      L.tile = conv_tile_for(mode, L.U * L.Cout, 2, L.Cin, 1, false);
      const ConvTile t = conv_tile(mode, L.tile);
      L.n_chunks = ceil_div(L.Cin, t.CK);
      L.w_numel = packed_conv_numel(mode, L.U * L.Cout, L.Cin, 2, t);
      L.b_numel = (int64_t)ceil_div(L.U * L.Cout, t.BM) * t.BM;
    } else {
      L.tile = convT_tile_for(L.Cout, L.U);
      const ConvTile t = convT_tile(L.tile, L.U);
      L.n_chunks = ceil_div(L.Cin, t.CK);
      L.w_numel = packed_convT_numel(L.Cin, L.Cout, L.U, t);
      L.b_numel = (int64_t)ceil_div(L.Cout, t.BM) * t.BM;
    }
    L.name = "ups_u" + std::to_string(L.U) + "_c" + std::to_string(L.Cout);
    ups_.push_back(L);
  }
  std::vector<std::pair<const float*, const float*>> usrc;
  for (int i = 0; i < cfg_.num_upsamples; ++i) { usrc.push_back({hw[wi], hw[wi + 1]}); wi += 2; }

  for (int i = 0; i < cfg_.num_upsamples; ++i) {
    const int ch = C0 >> (i + 1);
    for (int j = 0; j < cfg_.num_kernels; ++j) {
      const int k = cfg_.resblock_kernel_sizes[j];
      ResBlock rb;
      if (cfg_.resblock_type == 1) {
        // state_dict order: convs1.0..2 then convs2.0..2
        const float* w1[3]; const float* b1[3]; const float* w2[3]; const float* b2[3];
        for (int m = 0; m < 3; ++m) { w1[m] = hw[wi]; b1[m] = hw[wi + 1]; wi += 2; }
        for (int m = 0; m < 3; ++m) { w2[m] = hw[wi]; b2[m] = hw[wi + 1]; wi += 2; }
        // fused convs1 -> convs2 iterations (kernels_resblock.hip) where supported; they reuse the
        // conv packing, which needs 32-row blocks covering the channels and 16-channel groups
        rb.fused = pair_fusion;
        const bool p128 = pair_fusion && resblock_pair128(mode, ch, k);
        // the whole-block kernel reads the packing as [32-row block][16-channel group][tap]: the
        // conv tile must cover the channels without padding
        bool tiles_ok = true;
        for (int m = 0; m < 3; ++m) {
          rb.convs.push_back(add_conv(ch, ch, k, cfg_.resblock_dilation_sizes[j][m], "mrf_conv", false, mode, p128));
          src.push_back({w1[m], b1[m]});
          rb.convs.push_back(add_conv(ch, ch, k, 1, "mrf_conv", true, mode, p128));
          src.push_back({w2[m], b2[m]});
          for (int c = 0; c < 2; ++c) {
            const ConvTile t = conv_tile(mode, rb.convs[2 * m + c].tile);
            const int dil = rb.convs[2 * m].dil;
            // the fused kernels read the direct split packing: a Winograd-packed conv (7 *
            // ceil(K/4) steps) must take the per-conv path
            tiles_ok = tiles_ok && !t.WINO && t.CK % 16 == 0 && ch % t.CK == 0 && ch % t.BM == 0;
            rb.fused = rb.fused && !t.WINO && t.CK == 16 && ceil_div(ch, t.BM) * t.BM == ch &&
                       resblock_pair_preferred(mode, ch, k, dil);
          }
        }
        rb.fused3 = pair_fusion && tiles_ok;
      } else {
        bool tiles_ok = true;
        for (int m = 0; m < 2; ++m) {
          rb.convs.push_back(add_conv(ch, ch, k, cfg_.resblock_dilation_sizes[j][m], "mrf_conv", true, mode));
          src.push_back({hw[wi], hw[wi + 1]}); wi += 2;
          // the whole-block kernel reads the direct split packing (not Winograd) as [32-row
          // block][16-channel group][tap]
          const ConvTile t = conv_tile(mode, rb.convs[m].tile);
          tiles_ok = tiles_ok && !t.WINO && t.CK % 16 == 0 && ch % t.CK == 0 && ch % t.BM == 0;
        }
        rb.fused2 = pair_fusion && tiles_ok;
      }
      if (rb.fused2 || (cfg_.resblock_type == 1 && rb.fused3)) {
        // whole-block fusion (kernels_resblock.hip resblock3_kernel): TTS_MI355X_RESBLOCK3 =
        // "0" off, "<C>" blocks of at most C channels, "all" every supported block (default; MI355X
        // A/B scripts/ab_res3.sh: c32 k3 2.52 -> 1.87 ms, c64 k3 3.18 -> 2.93 ms per batch)
        const int policy = [] {  // read at create time (the tests switch it per generator)
          const char* e = std::getenv("TTS_MI355X_RESBLOCK3");
          if (!e) return 1 << 30;
          if (std::string(e) == "all") return 1 << 30;
          return std::atoi(e);
        }();
        // kernels 7 / 11 as whole blocks (TTS_MI355X_RB1_WHOLE_K lists them, e.g. "7" or "7,11"; A/B)
        const std::string wk = [] {
          const char* e = std::getenv("TTS_MI355X_RB1_WHOLE_K");
          return std::string(e ? e : "");
        }();
        const bool k_ok = k == 3 || wk.find(std::to_string(k)) != std::string::npos;
        if (cfg_.resblock_type == 1)
          rb.fused3 = ch <= policy && k_ok && resblock3_supported(mode, ch, k, cfg_.resblock_dilation_sizes[j]);
        else
          rb.fused2 = ch <= policy && resblock2_preferred(mode, ch, k, cfg_.resblock_dilation_sizes[j]);
      }
      res_.push_back(rb);
    }
  }
  post_w_ = hw[wi]; wi += 1;
  post_bias_ = cfg_.conv_post_bias ? hw[wi][0] : 0.f;
  if (cfg_.conv_post_bias) wi += 1;
  const float* cond_w = nullptr; const float* cond_b = nullptr;
  if (cfg_.cond_channels > 0) { cond_w = hw[wi]; cond_b = hw[wi + 1]; wi += 2; }
  std::vector<std::pair<const float*, const float*>> upcond;  // conds.i (XTTS)
  if (cfg_.cond_in_each_up_layer)
    for (int i = 0; i < cfg_.num_upsamples; ++i) { upcond.push_back({hw[wi], hw[wi + 1]}); wi += 2; }

  // arena layout
  std::vector<ConvLayer*> convs;
  convs.push_back(&pre_);
  for (auto& rb : res_) for (auto& c : rb.convs) convs.push_back(&c);
  int64_t total = 0;
  auto align = [](int64_t n) { return (n + 63) & ~int64_t(63); };
  for (auto* c : convs) total += align(c->w_numel) + align(c->b_numel);
  for (auto& u : ups_) total += align(u.w_numel) + align(u.b_numel);
  const int Cl = C0 >> cfg_.num_upsamples;
  total += align((int64_t)Cl * 7);
  if (cfg_.cond_channels > 0) total += align((int64_t)C0 * cfg_.cond_channels) + align(C0);
  for (size_t i = 0; i < upcond.size(); ++i)
    total += align((int64_t)(C0 >> (i + 1)) * cfg_.cond_channels) + align(C0 >> (i + 1));

  std::vector<float> host(total, 0.f);
  int64_t off = 0;
  std::vector<int64_t> offs;
  // conv1d layers: src[] is in the same order as convs[] (pre, then resblock convs)
  // resblock convs were pushed in execution order (c1_0, c2_0, c1_1, ...), matching src.
  {
    // src[0] is conv_pre; src[1..] resblocks
    size_t si = 0;
    for (auto* c : convs) {
      const ConvTile t = conv_tile(c->mode, c->tile);
      c->w_exp = pack_conv(c->mode, src[si].first, c->Cout, c->Cin, c->K, t, host.data() + off);
      offs.push_back(off); off += align(c->w_numel);
      std::memcpy(host.data() + off, src[si].second, sizeof(float) * c->Cout);
      offs.push_back(off); off += align(c->b_numel);
      ++si;
    }
  }
  for (size_t i = 0; i < ups_.size(); ++i) {
    auto& u = ups_[i];
    if (is_split_mode(u.mode)) {
      const ConvTile t = conv_tile(u.mode, u.tile);
      u.w_exp = pack_convT_split(u.mode, usrc[i].first, u.Cin, u.Cout, u.U, t, host.data() + off);
      offs.push_back(off); off += align(u.w_numel);
      for (int co = 0; co < u.Cout; ++co)
        for (int ph = 0; ph < u.U; ++ph) host[off + (int64_t)co * u.U + ph] = usrc[i].second[co];
    } else {
      const ConvTile t = convT_tile(u.tile, u.U);
      pack_convT(usrc[i].first, u.Cin, u.Cout, u.U, t, host.data() + off);
      offs.push_back(off); off += align(u.w_numel);
      std::memcpy(host.data() + off, usrc[i].second, sizeof(float) * u.Cout);
    }
    offs.push_back(off); off += align(u.b_numel);
  }
  std::memcpy(host.data() + off, post_w_, sizeof(float) * Cl * 7);
  const int64_t post_off = off; off += align((int64_t)Cl * 7);
  int64_t cond_w_off = -1, cond_b_off = -1;
  if (cfg_.cond_channels > 0) {
    std::memcpy(host.data() + off, cond_w, sizeof(float) * C0 * cfg_.cond_channels);
    cond_w_off = off; off += align((int64_t)C0 * cfg_.cond_channels);
    std::memcpy(host.data() + off, cond_b, sizeof(float) * C0);
    cond_b_off = off; off += align(C0);
  }
  std::vector<std::pair<int64_t, int64_t>> upcond_off;
  for (size_t i = 0; i < upcond.size(); ++i) {
    const int64_t ci = C0 >> (i + 1);
    std::memcpy(host.data() + off, upcond[i].first, sizeof(float) * ci * cfg_.cond_channels);
    const int64_t wo = off; off += align(ci * cfg_.cond_channels);
    std::memcpy(host.data() + off, upcond[i].second, sizeof(float) * ci);
    upcond_off.push_back({wo, off}); off += align(ci);
  }

  weights_bytes_ = (size_t)total * sizeof(float);
  if (hipMalloc(&arena_, weights_bytes_) != hipSuccess) throw Error(4, "hipMalloc(weights) failed");
  TTS_HIP_CHECK(hipMemcpy(arena_, host.data(), weights_bytes_, hipMemcpyHostToDevice));
  size_t oi = 0;
  for (auto* c : convs) { c->w = arena_ + offs[oi++]; c->b = arena_ + offs[oi++]; }
  for (auto& u : ups_) { u.w = arena_ + offs[oi++]; u.b = arena_ + offs[oi++]; }
  post_wd_ = arena_ + post_off;
  if (cfg_.cond_channels > 0) { cond_wd_ = arena_ + cond_w_off; cond_bd_ = arena_ + cond_b_off; }
  for (auto& o : upcond_off) up_cond_.push_back({arena_ + o.first, arena_ + o.second});
  hop_ = 1;
  for (int i = 0; i < cfg_.num_upsamples; ++i) hop_ *= cfg_.upsample_factors[i];
}

Hifigan::~Hifigan() {
  DeviceGuard g(device_);
  for (Lane& ln : lanes_) {
    for (hipStream_t st : ln.branch) (void)hipStreamDestroy(st);
    if (ln.own) (void)hipStreamDestroy(ln.own);
    for (hipEvent_t e : ln.ev_z) (void)hipEventDestroy(e);
    if (ln.ev_ups) (void)hipEventDestroy(ln.ev_ups);
    if (ln.ev_done) (void)hipEventDestroy(ln.ev_done);
  }
  if (ev_start_) (void)hipEventDestroy(ev_start_);
  if (arena_) (void)hipFree(arena_);
  if (ws_) (void)hipFree(ws_);
  if (win_) (void)hipFree(win_);
}

int64_t Hifigan::out_len(int T, int pad) const { return (int64_t)hop_ * (T + 2 * pad); }

int64_t Hifigan::plane_floats(int B, int T, int pad) const {
  // largest C_i * len_i over the stages (conv_pre output included)
  const int64_t L = T + 2 * pad;
  int64_t best = (int64_t)cfg_.upsample_initial_channel * L;
  int64_t len = L;
  for (int i = 0; i < cfg_.num_upsamples; ++i) {
    len *= cfg_.upsample_factors[i];
    const int64_t c = (int64_t)(cfg_.upsample_initial_channel >> (i + 1)) * len;
    if (c > best) best = c;
  }
  return ((best * B + 63) / 64) * 64;
}

// max-abs slot groups (fp16 hi/lo mode), [B][64] each: 0 the mel, 1 conv_pre's output, then per
// stage i from stage_group(i): the upsampled input o, per resblock conv its output
// (convs1 -> t, convs2 -> x), and the stage's MRF output z/num_kernels
int Hifigan::n_planes(int nbs) const { return 2 + 2 * nbs; }

// branch streams of each lane when the batch splits over lanes: one, unless TTS_MI355X_MRF_STREAMS
// asks for more (forward(); ADVICE r5: a split lane's region is sized for the planes it uses)
int Hifigan::split_nbs() const { return nbs_env_ ? nbs_ : 1; }

void Hifigan::ensure_lanes() {
  if (!lanes_.empty()) return;
  auto stream = [] {
    // non-blocking: no implicit ordering with the legacy null stream; every dependency is an event
    hipStream_t st;
    TTS_HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    return st;
  };
  auto event = [] {
    hipEvent_t e;
    TTS_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  };
  lanes_.resize(n_lanes_);
  for (int i = 0; i < n_lanes_; ++i) {
    Lane& ln = lanes_[i];
    if (i > 0) ln.own = stream();
    for (int j = 1; j < nbs_; ++j) ln.branch.push_back(stream());
    ln.ev_ups = event();
    ln.ev_done = event();
    for (int j = 0; j < cfg_.num_kernels; ++j) ln.ev_z.push_back(event());
  }
  ev_start_ = event();
}

int64_t Hifigan::lane_bytes(int B, int64_t L, int nbs) const {
  const int64_t cond = cond_floats(B);
  const int64_t amax = cfg_.math_mode == MATH_FP32_F16X3 ? (int64_t)amax_groups() * B * 64 : 0;
  return ((n_planes(nbs) * plane_floats(B, (int)L, 0) + cond + amax + 63) / 64 * 64) * (int64_t)sizeof(float);
}

int Hifigan::amax_groups() const { return 2 + cfg_.num_upsamples * (2 + cfg_.num_kernels * 6); }
int Hifigan::stage_group(int i) const { return 2 + i * (2 + cfg_.num_kernels * 6); }

int64_t Hifigan::cond_floats(int B) const {
  // cond_layer(g) [B][C0], then (XTTS) conds[i](g) [B][C_{i+1}] per stage
  if (cfg_.cond_channels <= 0) return 0;
  int64_t n = (((int64_t)B * cfg_.upsample_initial_channel + 63) / 64) * 64;
  if (cfg_.cond_in_each_up_layer)
    for (int i = 0; i < cfg_.num_upsamples; ++i)
      n += (((int64_t)B * (cfg_.upsample_initial_channel >> (i + 1)) + 63) / 64) * 64;
  return n;
}

// ---------------------------------------------------------------------------------------
// Time windows for long utterances
// ---------------------------------------------------------------------------------------
int Hifigan::window_halo() const {
  // receptive-field radius of one output sample, in mel frames: conv_pre (k7), then per stage the
  // polyphase ConvTranspose (output n reads x[m-1] and x[m], m = floor((n + U/2) / U): up to 1.5
  // input samples from n / U) and the widest MRF branch (ResBlock1: sum_m (k-1)/2 * (d_m + 1);
  // ResBlock2: sum_m (k-1)/2 * d_m samples at the stage's rate), then conv_post (k7) at the
  // output rate.  The +2 frames are slack (tests/test_hifigan_gpu.py probes the radius)
  double r = 3.0, rate = 1.0;
  for (int i = 0; i < cfg_.num_upsamples; ++i) {
    r += 1.5 / rate;
    rate *= cfg_.upsample_factors[i];
    int widest = 0;
    for (int j = 0; j < cfg_.num_kernels; ++j) {
      const int h = (cfg_.resblock_kernel_sizes[j] - 1) / 2;
      int w = 0;
      for (int m = 0; m < (cfg_.resblock_type == 1 ? 3 : 2); ++m)
        w += h * cfg_.resblock_dilation_sizes[j][m] + (cfg_.resblock_type == 1 ? h : 0);
      widest = std::max(widest, w);
    }
    r += widest / rate;
  }
  r += 3.0 / rate;
  return (int)std::ceil(r) + 2;
}

int64_t Hifigan::max_window_frames() const {
  // the kernels address one batch item's channel plane with 32-bit byte offsets: C * len < 2^29
  int64_t cr = cfg_.upsample_initial_channel, rate = 1;
  for (int i = 0; i < cfg_.num_upsamples; ++i) {
    rate *= cfg_.upsample_factors[i];
    cr = std::max(cr, (int64_t)(cfg_.upsample_initial_channel >> (i + 1)) * rate);
  }
  return ((int64_t(1) << 29) - 1) / cr;
}

int64_t Hifigan::window_payload() const {
  // TTS_MI355X_WINDOW_FRAMES=<n> forces n-frame payloads (tests: windows at ordinary lengths)
  const char* e = std::getenv("TTS_MI355X_WINDOW_FRAMES");
  const int64_t cap = max_window_frames() - 2 * window_halo();
  if (e && std::atoll(e) > 0) return std::min<int64_t>(std::atoll(e), cap);
  return cap;
}

bool Hifigan::windowed(int64_t L) const {
  const char* e = std::getenv("TTS_MI355X_WINDOW_FRAMES");
  return L > max_window_frames() || (e && std::atoll(e) > 0 && L > std::atoll(e));
}

int64_t Hifigan::plain_workspace_bytes(int B, int64_t L, bool window) const {
  // the schedules forward() runs on this region: the whole batch as one lane with nbs_ branch
  // streams (a window, B = 1 or one lane), one stream when profiled, or one region per lane of a
  // split batch with split_nbs() streams each
  const int nl = std::min(n_lanes_, B);
  if (window || nl == 1) return lane_bytes(B, L, nbs_);
  int64_t lanes = 0;
  for (int i = 0; i < nl; ++i) lanes += lane_bytes(lane_batch(B, i), L, split_nbs());
  return std::max(lane_bytes(B, L, 1), lanes);
}

int64_t Hifigan::window_buffer_bytes(int B, int64_t W) const {
  return ((((int64_t)B * cfg_.in_channels * W + 63) / 64) * 64 + (int64_t)B * hop_ * W) * (int64_t)sizeof(float);
}

int64_t Hifigan::workspace_bytes(int B, int T, int pad) const {
  const int64_t L = (int64_t)T + 2 * pad;
  if (!windowed(L)) return plain_workspace_bytes(B, L, false);
  const int64_t W = std::min<int64_t>(L, window_payload() + 2 * window_halo());
  return plain_workspace_bytes(B, W, true) + window_buffer_bytes(B, W);
}

void Hifigan::reserve_plain(int B, int64_t L, bool window) {
  const int64_t need = plain_workspace_bytes(B, L, window);
  if ((size_t)need <= ws_bytes_) return;
  DeviceGuard g(device_);
  if (ws_) { TTS_HIP_CHECK(hipFree(ws_)); ws_ = nullptr; ws_bytes_ = 0; }
  if (hipMalloc(&ws_, need) != hipSuccess) throw Error(4, "hipMalloc(workspace) failed");
  ws_bytes_ = need;
}

void Hifigan::reserve(int B, int T, int pad) {
  const int64_t L = (int64_t)T + 2 * pad;
  if (!windowed(L)) {
    reserve_plain(B, L);
    return;
  }
  const int64_t W = std::min<int64_t>(L, window_payload() + 2 * window_halo());
  reserve_plain(B, W, true);
  const int64_t need = window_buffer_bytes(B, W);
  if ((size_t)need <= win_bytes_) return;
  DeviceGuard g(device_);
  if (win_) { TTS_HIP_CHECK(hipFree(win_)); win_ = nullptr; win_bytes_ = 0; }
  if (hipMalloc(&win_, need) != hipSuccess) throw Error(4, "hipMalloc(window buffers) failed");
  win_bytes_ = need;
}

void Hifigan::forward(const float* mel, int B, int C, int T, int pad, const float* gvec, float* wav,
                      hipStream_t s, Profiler* prof) {
  TTS_REQUIRE(mel && wav, 1, "NULL input/output pointer");
  TTS_REQUIRE(B >= 1, 1, "batch must be >= 1");
  TTS_REQUIRE(C == cfg_.in_channels, 1,
              "mel has " + std::to_string(C) + " channels, generator expects " + std::to_string(cfg_.in_channels));
  TTS_REQUIRE(T >= 1, 1, "T must be >= 1");
  TTS_REQUIRE(pad >= 0, 1, "pad must be >= 0");
  TTS_REQUIRE(cfg_.cond_channels == 0 || gvec != nullptr, 1, "cond_channels > 0 requires g");
  const int64_t L = (int64_t)T + 2 * pad;
  if (!windowed(L)) {
    DeviceGuard dg(device_);
    reserve_plain(B, L);
    // a profiled forward stays on one stream (its per-launch timings are serial)
    if (prof) {
      forward_plain(mel, B, C, T, pad, gvec, wav, s, prof, ws_, nullptr);
      return;
    }
    ensure_lanes();
    const int nl = std::min(n_lanes_, B);
    // split batches run one stream per lane unless TTS_MI355X_MRF_STREAMS says otherwise
    for (Lane& ln : lanes_) ln.nbs = nl > 1 ? split_nbs() : nbs_;
    if (nl == 1) {
      forward_plain(mel, B, C, T, pad, gvec, wav, s, nullptr, ws_, &lanes_[0]);
      return;
    }
    // sub-batches on concurrent lanes: lane 0 on the caller's stream, lane i > 0 on its own stream
    // after everything enqueued on s so far; s waits for every lane at the end
    TTS_HIP_CHECK(hipEventRecord(ev_start_, s));
    float* ws = ws_;
    int b0 = 0;
    for (int i = 0; i < nl; ++i) {
      const int Bi = lane_batch(B, i);
      Lane& ln = lanes_[i];
      const hipStream_t si = i == 0 ? s : ln.own;
      if (i > 0) TTS_HIP_CHECK(hipStreamWaitEvent(si, ev_start_, 0));
      forward_plain(mel + (int64_t)b0 * C * T, Bi, C, T, pad,
                    gvec ? gvec + (int64_t)b0 * cfg_.cond_channels : nullptr, wav + (int64_t)b0 * out_len(T, pad), si,
                    nullptr, ws, &ln);
      if (i > 0) {
        TTS_HIP_CHECK(hipEventRecord(ln.ev_done, si));
        TTS_HIP_CHECK(hipStreamWaitEvent(s, ln.ev_done, 0));
      }
      ws += lane_bytes(Bi, L, ln.nbs) / (int64_t)sizeof(float);
      b0 += Bi;
    }
    return;
  }
  DeviceGuard dg(device_);
  reserve(B, T, pad);
  const int h = window_halo();
  const int64_t P = window_payload();
  TTS_REQUIRE(P >= 1, 3, "window payload must be >= 1 frame");
  const int64_t Wmax = std::min<int64_t>(L, P + 2 * h);
  float* melw = win_;
  float* outw = win_ + (((int64_t)B * C * Wmax + 63) / 64) * 64;
  for (int64_t s0 = 0; s0 < L; s0 += P) {
    const int64_t s1 = std::min(L, s0 + P);
    const int64_t w0 = std::max<int64_t>(0, s0 - h), w1 = std::min(L, s1 + h);
    const int W = (int)(w1 - w0);
    // melw[b][c][t] = replicate_pad(mel)[b][c][w0 + t]  (hifigan_generator.py:281)
    run(prof, s, "mel_window", 0.0, 8.0 * B * C * (double)W,
        [&] { launch_mel_window(mel, B, C, T, pad, w0, W, melw, s); });
    if (!prof) {
      ensure_lanes();
      lanes_[0].nbs = nbs_;
    }
    forward_plain(melw, B, C, W, 0, gvec, outw, s, prof, ws_, prof ? nullptr : &lanes_[0]);
    // the payload's samples: outw[b][hop*(s0-w0) ...) -> wav[b][hop*s0 ...)
    TTS_HIP_CHECK(hipMemcpy2DAsync(wav + hop_ * s0, sizeof(float) * hop_ * L, outw + hop_ * (s0 - w0),
                                   sizeof(float) * hop_ * W, sizeof(float) * hop_ * (s1 - s0), B,
                                   hipMemcpyDeviceToDevice, s));
  }
}

void Hifigan::forward_plain(const float* mel, int B, int C, int T, int pad, const float* gvec, float* wav,
                            hipStream_t s, Profiler* prof, float* ws, Lane* lane) {
  DeviceGuard g(device_);

  const int64_t plane = plane_floats(B, T, pad);
  float* bufZ = ws;               // conv_pre output, then the MRF sum of each stage
  float* bufO = ws + plane;       // upsampled stage input o
  const int np = n_planes(lane ? lane->nbs : 1);  // the planes this schedule uses (lane_bytes)
  float* cvec = cfg_.cond_channels > 0 ? ws + np * plane : nullptr;
  const bool h3 = cfg_.math_mode == MATH_FP32_F16X3;
  unsigned* amax = h3 ? reinterpret_cast<unsigned*>(ws + np * plane + cond_floats(B)) : nullptr;
  // concurrent MRF branches (a lane with more than one stream; never in a profiled forward)
  const int nbs = lane ? lane->nbs : 1;
  const bool conc = nbs > 1;
  const int K = cfg_.num_kernels;
  auto bstream = [&](int j) { return std::max(0, j - (K - nbs)); };  // branch j -> stream index
  auto slots = [&](int grp) -> unsigned* { return amax ? amax + (size_t)grp * B * 64 : nullptr; };  // [B][64]
  if (h3) TTS_HIP_CHECK(hipMemsetAsync(amax, 0, (size_t)amax_groups() * B * 64 * sizeof(unsigned), s));

  const int L = T + 2 * pad;
  const int C0 = cfg_.upsample_initial_channel;
  bool post_done = false;  // conv_post ran inside the last MRF launch (ResPairArgs::post_w)
  if (cvec) {
    run(prof, s, "cond_layer", 2.0 * B * C0 * cfg_.cond_channels, 4.0 * (B * cfg_.cond_channels + C0 * cfg_.cond_channels + B * C0),
        [&] { launch_cond_vec(gvec, cond_wd_, cond_bd_, cvec, B, cfg_.cond_channels, C0, s); });
  }

  auto conv = [&](const ConvLayer& Ld, const float* x, int Tin, int Tout, int rep, float in_slope,
                  float out_slope, const float* res, float* y, int zmode, const float* cv,
                  const unsigned* amax_in = nullptr, unsigned* amax_out = nullptr, hipStream_t st = nullptr) {
    if (!st) st = s;
    Conv1dArgs a{};
    a.amax_in = amax_in; a.amax_out = amax_out; a.w_exp = Ld.w_exp;
    a.x = x; a.w = Ld.w; a.bias = Ld.b; a.res = res; a.y = y; a.z = bufZ; a.cvec = cv;
    a.Cin = Ld.Cin; a.Cout = Ld.Cout; a.Tin = Tin; a.Tout = Tout;
    a.dil = Ld.dil; a.pad = Ld.pad; a.rep_pad = rep; a.n_chunks = Ld.n_chunks;
    a.in_slope = in_slope; a.out_slope = out_slope; a.zmode = zmode; a.zdiv = (float)cfg_.num_kernels;
    a.planes = planes16_ ? (x == mel ? kPlaneYB16 : kPlaneXB16 | kPlaneYB16) : 0;
    const double ex = (planes16_ && x != mel) ? 2.0 : 4.0, ey = planes16_ ? 2.0 : 4.0;  // bytes per element
    const double flops = 2.0 * B * Ld.Cout * (double)Ld.Cin * Ld.K * Tout;
    double bytes = ex * B * Ld.Cin * Tin + 4.0 * Ld.Cout * Ld.Cin * Ld.K + ey * B * Ld.Cout * Tout;
    if (res) bytes += ey * B * Ld.Cout * (double)Tout;
    if (zmode >= 2) bytes += ey * B * Ld.Cout * (double)Tout;
    run(prof, st, Ld.name.c_str(), flops, bytes, [&] { launch_conv(Ld.mode, a, B, Ld.K, Ld.tile, st); });
  };

  // conv_pre on the replicate-padded mel (hifigan_generator.py:281, :249) [+ cond_layer(g), :250-251]
  if (h3)
    run(prof, s, "amax_mel", 0.0, 4.0 * B * C * (double)T,
        [&] { launch_amax(mel, (int64_t)C * T, B, slots(0), s); });
  conv(pre_, mel, T, L, pad, 1.f, 1.f, nullptr, bufZ, 0, cvec, slots(0), slots(1));

  int len = L;
  const float* cur = bufZ;
  float* upvec = cvec ? cvec + (((int64_t)B * C0 + 63) / 64) * 64 : nullptr;  // conds[i](g), XTTS
  for (int i = 0; i < cfg_.num_upsamples; ++i) {
    const ConvTLayer& U = ups_[i];
    const int g0 = stage_group(i);
    const float* ucv = nullptr;  // o = ups[i](o) + conds[i](g) (xtts/hifigan_decoder.py:276-279)
    if (cfg_.cond_in_each_up_layer) {
      const int ci = U.Cout;
      run(prof, s, "cond_up", 2.0 * B * ci * cfg_.cond_channels, 4.0 * (B * cfg_.cond_channels + ci * cfg_.cond_channels + B * ci),
          [&] { launch_cond_vec(gvec, up_cond_[i].first, up_cond_[i].second, upvec, B, cfg_.cond_channels, ci, s); });
      ucv = upvec;
      upvec += (((int64_t)B * ci + 63) / 64) * 64;
    }  // this stage's slot groups: o, per conv, z
    const unsigned* z_amax = slots(i == 0 ? 1 : stage_group(i - 1) + 1 + cfg_.num_kernels * 6);
    const int lout = len * U.U;
    const double uflops = 2.0 * B * U.Cout * (double)U.Cin * 2 * lout;
    const double es = planes16_ ? 2.0 : 4.0;
    const double ubytes = es * ((double)B * U.Cin * len + (double)B * U.Cout * lout) + 4.0 * U.Cin * U.Cout * 2 * U.U;
    if (is_split_mode(U.mode)) {
      Conv1dArgs a{};
      a.planes = planes16_ ? kPlaneXB16 | kPlaneYB16 : 0;
      a.x = cur; a.w = U.w; a.bias = U.b; a.y = bufO;
      a.Cin = U.Cin; a.Cout = U.U * U.Cout; a.Tin = len; a.Tout = len + 1;
      a.dil = 1; a.pad = 1; a.n_chunks = U.n_chunks;
      a.in_slope = 0.1f; a.out_slope = 1.f; a.zdiv = 1.f;
      a.amax_in = z_amax; a.amax_out = slots(g0); a.w_exp = U.w_exp; a.ups = U.U;
      a.cvec = ucv;
      run(prof, s, U.name.c_str(), uflops, ubytes, [&] { launch_conv(U.mode, a, B, 2, U.tile, s); });
    } else {
      ConvTArgs ta{};
      ta.x = cur; ta.w = U.w; ta.bias = U.b; ta.y = bufO;
      ta.Cin = U.Cin; ta.Cout = U.Cout; ta.Tin = len; ta.n_chunks = U.n_chunks; ta.in_slope = 0.1f;
      ta.cvec = ucv;
      run(prof, s, U.name.c_str(), uflops, ubytes, [&] { launch_convT(ta, B, U.U, U.tile, s); });
    }
    len = lout;
    if (conc) TTS_HIP_CHECK(hipEventRecord(lane->ev_ups, s));  // o is ready for every branch
    // MRF: z = sum_j resblock_j(o); o = z / num_kernels (:255-261)
    for (int j = 0; j < K; ++j) {
      const ResBlock& rb = res_[i * K + j];
      // branch j: its stream and that stream's X / T planes
      const int bj = conc ? bstream(j) : 0;
      const hipStream_t sj = bj > 0 ? lane->branch[bj - 1] : s;
      float* bufX = ws + (2 + 2 * bj) * plane;  // resblock running residual x
      float* bufT = bufX + plane;               // convs1 output (already leaky-relu'd)
      if (bj > 0) TTS_HIP_CHECK(hipStreamWaitEvent(sj, lane->ev_ups, 0));
      // the MRF-sum writer of branch j reads the z branch j - 1 wrote: keep that order
      auto zorder = [&] {
        if (bj > 0 && bstream(j - 1) != bj) TTS_HIP_CHECK(hipStreamWaitEvent(sj, lane->ev_z[j - 1], 0));
      };
      auto zdone = [&] {
        if (conc) TTS_HIP_CHECK(hipEventRecord(lane->ev_z[j], sj));
      };
      const int zlast = (cfg_.num_kernels == 1 || j == 0) ? 1 : (j == cfg_.num_kernels - 1 ? 3 : 2);
      const int gj = g0 + 1 + j * 6;  // slot group of conv c of this resblock: gj + c
      const int gz = g0 + 1 + cfg_.num_kernels * 6;  // the stage's z / num_kernels
      if (cfg_.resblock_type == 1 && rb.fused3) {
        // the three iterations in one launch: o -> MRF z
        ResBlock3Args ra{};
        ra.x = bufO; ra.amax_in = slots(g0);
        ra.planes = planes16_ ? kPlaneXB16 | kPlaneYB16 : 0;
        for (int c = 0; c < 6; ++c) { ra.w[c] = rb.convs[c].w; ra.bias[c] = rb.convs[c].b; ra.w_exp[c] = rb.convs[c].w_exp; }
        for (int m = 0; m < 3; ++m) ra.dil[m] = rb.convs[2 * m].dil;
        ra.z = bufZ; ra.zmode = zlast; ra.zdiv = (float)cfg_.num_kernels;
        ra.amax_out = j == cfg_.num_kernels - 1 ? slots(gz) : nullptr;
        ra.T = len;
        const ConvLayer& L1 = rb.convs[0];
        const double flops = 12.0 * B * L1.Cout * (double)L1.Cin * L1.K * len;
        const double bytes = (planes16_ ? 2.0 : 4.0) * B * L1.Cout * len * (zlast >= 2 ? 3 : 2) +
                             4.0 * 6.0 * L1.Cout * L1.Cin * L1.K;
        const std::string nm = "mrf_block_k" + std::to_string(L1.K) + "_c" + std::to_string(L1.Cout);
        zorder();
        run(prof, sj, nm.c_str(), flops, bytes, [&] { launch_resblock3(L1.mode, ra, B, L1.Cout, L1.K, sj); });
        zdone();
      } else if (cfg_.resblock_type == 1 && rb.fused) {
        // x_{m+1} = convs2[m](lrelu(convs1[m](lrelu(x_m)))) + x_m in one launch per m; the
        // iterates ping-pong between X and T (o -> X -> T -> X / the MRF z)
        for (int m = 0; m < 3; ++m) {
          const ConvLayer& L1 = rb.convs[2 * m];
          const ConvLayer& L2 = rb.convs[2 * m + 1];
          const float* xin = (m == 0) ? bufO : (m == 1 ? bufX : bufT);
          float* xout = (m == 1) ? bufT : bufX;
          const bool last = (m == 2);
          ResPairArgs pa{};
          Conv1dArgs& c1 = pa.c1;
          c1.x = xin; c1.w = L1.w; c1.bias = L1.b; c1.Cin = L1.Cin; c1.Cout = L1.Cout; c1.Tin = len; c1.Tout = len;
          c1.dil = L1.dil; c1.pad = L1.pad; c1.n_chunks = L1.n_chunks; c1.in_slope = 0.1f; c1.out_slope = 0.1f;
          c1.zdiv = 1.f; c1.w_exp = L1.w_exp;
          c1.planes = planes16_ ? kPlaneXB16 | kPlaneYB16 : 0;
          c1.amax_in = (m == 0) ? slots(g0) : slots(gj + 2 * m - 1);
          Conv1dArgs& c2 = pa.c2;
          c2.x = nullptr; c2.w = L2.w; c2.bias = L2.b; c2.res = xin; c2.y = xout; c2.z = bufZ;
          c2.Cin = L2.Cin; c2.Cout = L2.Cout; c2.Tin = len; c2.Tout = len; c2.dil = 1; c2.pad = L2.pad;
          c2.n_chunks = L2.n_chunks; c2.in_slope = 1.f; c2.out_slope = 1.f; c2.zmode = last ? zlast : 0;
          c2.zdiv = (float)cfg_.num_kernels; c2.w_exp = L2.w_exp;
          c2.planes = c1.planes;
          c2.amax_out = last ? (j == cfg_.num_kernels - 1 ? slots(gz) : nullptr) : slots(gj + 2 * m + 1);
          // the generator's last MRF writer: conv_post runs in its epilogue (the final z never
          // reaches HBM); TTS_MI355X_POST_FUSION=0 keeps the separate conv_post launch
          const bool post = last && zlast == 3 && i == cfg_.num_upsamples - 1 && post_fusion_ &&
                            cfg_.out_channels == 1;
          if (post) {
            pa.post_w = post_wd_; pa.post_bias = post_bias_; pa.post_slope = 0.01f; pa.wav = wav;
            c2.amax_out = nullptr;  // nothing reads the final z's statistics
            post_done = true;
          }
          double flops = 4.0 * B * L1.Cout * (double)L1.Cin * L1.K * len;
          const double es = planes16_ ? 2.0 : 4.0;
          double bytes = es * B * L1.Cout * len * (last ? (zlast >= 2 ? 4 : 3) : 3) + 4.0 * 2.0 * L1.Cout * L1.Cin * L1.K;
          if (post) {
            flops += 2.0 * B * len * (double)L1.Cout * 7;
            bytes += 4.0 * B * len - es * B * L1.Cout * len;  // + wav, - the z store
          }
          const std::string nm = std::string(post ? "mrf_pair_post_k" : "mrf_pair_k") + std::to_string(L1.K) +
                                 "_c" + std::to_string(L1.Cout);
          if (last) zorder();
          run(prof, sj, nm.c_str(), flops, bytes, [&] { launch_resblock_pair(L1.mode, pa, B, L1.K, L1.Cout, sj); });
          if (last) zdone();
        }
      } else if (cfg_.resblock_type == 1) {
        for (int m = 0; m < 3; ++m) {
          const float* xin = (m == 0) ? bufO : bufX;
          const unsigned* xin_amax = (m == 0) ? slots(g0) : slots(gj + 2 * m - 1);
          const bool last = (m == 2);
          // xt = convs1[m](lrelu(x)); xt = lrelu(xt)       (ResBlock1.forward :94-96)
          conv(rb.convs[2 * m], xin, len, len, 0, 0.1f, 0.1f, nullptr, bufT, 0, nullptr, xin_amax, slots(gj + 2 * m),
               sj);
          // x = convs2[m](xt) + x                          (:97-98)
          if (last) zorder();
          conv(rb.convs[2 * m + 1], bufT, len, len, 0, 1.f, 1.f, xin, bufX, last ? zlast : 0, nullptr,
               slots(gj + 2 * m), last ? (j == cfg_.num_kernels - 1 ? slots(gz) : nullptr) : slots(gj + 2 * m + 1), sj);
          if (last) zdone();
        }
      } else if (rb.fused2) {
        // both convs in one launch: o -> MRF z
        ResBlock3Args ra{};
        ra.x = bufO; ra.amax_in = slots(g0);
        ra.planes = planes16_ ? kPlaneXB16 | kPlaneYB16 : 0;
        for (int c = 0; c < 2; ++c) {
          ra.w[c] = rb.convs[c].w; ra.bias[c] = rb.convs[c].b; ra.w_exp[c] = rb.convs[c].w_exp;
          ra.dil[c] = rb.convs[c].dil;
        }
        ra.z = bufZ; ra.zmode = zlast; ra.zdiv = (float)cfg_.num_kernels;
        ra.amax_out = j == cfg_.num_kernels - 1 ? slots(gz) : nullptr;
        ra.T = len;
        const ConvLayer& L1 = rb.convs[0];
        const double flops = 4.0 * B * L1.Cout * (double)L1.Cin * L1.K * len;
        const double bytes = (planes16_ ? 2.0 : 4.0) * B * L1.Cout * len * (zlast >= 2 ? 3 : 2) +
                             4.0 * 2.0 * L1.Cout * L1.Cin * L1.K;
        const std::string nm = "mrf_block2_k" + std::to_string(L1.K) + "_c" + std::to_string(L1.Cout);
        zorder();
        run(prof, sj, nm.c_str(), flops, bytes,
            [&] { launch_resblock2(L1.mode, ra, B, L1.Cout, L1.K, rb2_geo64_, sj); });
        zdone();
      } else {
        for (int m = 0; m < 2; ++m) {
          const float* xin = (m == 0) ? bufO : bufX;
          const unsigned* xin_amax = (m == 0) ? slots(g0) : slots(gj + m - 1);
          const bool last = (m == 1);
          // x = convs[m](lrelu(x)) + x                     (ResBlock2.forward :151-154)
          if (last) zorder();
          conv(rb.convs[m], xin, len, len, 0, 0.1f, 1.f, xin, bufX, last ? zlast : 0, nullptr, xin_amax,
               last ? (j == cfg_.num_kernels - 1 ? slots(gz) : nullptr) : slots(gj + m), sj);
          if (last) zdone();
        }
      }
    }
    // the stage's z (and every branch before it) is complete before the next stage's ups
    if (conc && bstream(K - 1) > 0) TTS_HIP_CHECK(hipStreamWaitEvent(s, lane->ev_z[K - 1], 0));
    cur = bufZ;
  }
  // leaky_relu (default slope 0.01!) -> conv_post -> tanh (:262-264)
  if (post_done) return;
  PostArgs pa{};
  pa.z = bufZ; pa.w = post_wd_; pa.bias = post_bias_; pa.y = wav;
  pa.Cin = C0 >> cfg_.num_upsamples; pa.T = len; pa.in_slope = 0.01f;
  pa.z_b16 = planes16_ ? 1 : 0;
  run(prof, s, "conv_post", 2.0 * B * len * (double)pa.Cin * 7,
      (planes16_ ? 2.0 : 4.0) * B * pa.Cin * len + 4.0 * B * len, [&] { launch_conv_post(pa, B, s); });
}

}  // namespace tts
