// VITS flow (ResidualCouplingBlocks) executor, reverse direction
// (TTS/tts/layers/vits/networks.py:169-232, mean-only ResidualCouplingBlock :103-166).
#pragma once

#include <vector>

#include "common.hpp"
#include "hifigan.hpp"
#include "tts_mi355x.h"

namespace tts {

std::vector<int64_t> vits_flow_weight_shapes(const TtsVitsFlowCfg& c);
void vits_flow_validate(const TtsVitsFlowCfg& c);

class VitsFlow {
 public:
  VitsFlow(const TtsVitsFlowCfg& cfg, const float* const* host_weights, int device);
  ~VitsFlow();
  VitsFlow(const VitsFlow&) = delete;
  VitsFlow& operator=(const VitsFlow&) = delete;
  void reverse(const float* x, const float* mask, const float* g, int B, int C, int T, float* y, hipStream_t s,
               Profiler* prof = nullptr);
  // reverse=False (networks.py:225-228): for flow in flows: x = flow(x); x = flip(x)
  void forward(const float* x, const float* mask, const float* g, int B, int C, int T, float* y, hipStream_t s,
               Profiler* prof = nullptr);
  int device() const { return device_; }

 private:
  struct Conv {
    int Cin = 0, Cout = 0, K = 1, dil = 1, tile = 0, n_chunks = 0, w_exp = 0;
    bool gated = false;  // in_layer with the WN gate fused (kSplitGateTile)
    float* w = nullptr;
    float* b = nullptr;
  };
  struct Flow {
    Conv pre, post;  // pre/post already permuted for the flip parity this flow runs at; post negated
    Conv post_fwd;   // the same rows, not negated (forward direction: x1 = m + x1 * mask)
    std::vector<Conv> in_layers, res_skip;
    float* cond_w = nullptr;  // [2*H*L][cond_channels] fp32, or nullptr
    float* cond_b = nullptr;  // [2*H*L]
    int64_t in_off = 0;       // channel offset (x T) of the half pre reads
    int64_t out_off = 0;      // channel offset (x T) of the half the coupling updates
  };
  void run_flows(bool rev, const float* x, const float* mask, const float* g, int B, int C, int T, float* y,
                 hipStream_t s, Profiler* prof);
  void reserve(int B, int T);
  size_t amax_floats(int B) const;

  TtsVitsFlowCfg cfg_;
  int device_;
  std::vector<Flow> flows_;
  float* arena_ = nullptr;
  float* ws_ = nullptr;
  size_t ws_bytes_ = 0;
  bool amax_prepass_ = false;
  bool wn_fused_ = false;  // res_skip conv + WN update in one launch (flow_wn_fused)
  bool wn_layer_ = false;  // every WN layer in one launch (launch_glow_wn_layer, flow_wn_layer)
};

std::vector<int64_t> vits_posterior_weight_shapes(const TtsVitsPosteriorCfg& c);
void vits_posterior_validate(const TtsVitsPosteriorCfg& c);
// z = (m + eps * exp(logs)) * mask from stats [B][2*out][T] = proj(x) * mask (networks.py:285-287)
void launch_posterior_sample(const float* stats, const float* eps, const float* mask, float* z, float* m,
                             float* logs, int B, int Co, int T, hipStream_t s);

// PosteriorEncoder (networks.py:235-288): pre (1x1) -> WN -> proj (1x1) -> split -> sample
class VitsPosterior {
 public:
  VitsPosterior(const TtsVitsPosteriorCfg& cfg, const float* const* host_weights, int device);
  ~VitsPosterior();
  VitsPosterior(const VitsPosterior&) = delete;
  VitsPosterior& operator=(const VitsPosterior&) = delete;
  void forward(const float* x, const float* mask, const float* g, const float* eps, int B, int C, int T, float* z,
               float* m, float* logs, hipStream_t s, Profiler* prof = nullptr);
  int device() const { return device_; }

 private:
  struct Conv {
    int Cin = 0, Cout = 0, K = 1, dil = 1, tile = 0, n_chunks = 0, w_exp = 0;
    bool gated = false;
    float* w = nullptr;
    float* b = nullptr;
  };
  void reserve(int B, int T);
  size_t amax_floats(int B) const;

  TtsVitsPosteriorCfg cfg_;
  int device_;
  Conv pre_, proj_;
  std::vector<Conv> in_layers_, res_skip_;
  bool wn_layer_ = false;  // every WN layer in one launch (launch_glow_wn_layer, flow_wn_layer)
  float* cond_w_ = nullptr;
  float* cond_b_ = nullptr;
  float* arena_ = nullptr;
  float* ws_ = nullptr;
  size_t ws_bytes_ = 0;
};

}  // namespace tts
