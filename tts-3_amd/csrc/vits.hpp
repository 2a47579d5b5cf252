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
    std::vector<Conv> in_layers, res_skip;
    float* cond_w = nullptr;  // [2*H*L][cond_channels] fp32, or nullptr
    float* cond_b = nullptr;  // [2*H*L]
    int64_t in_off = 0;       // channel offset (x T) of the half pre reads
    int64_t out_off = 0;      // channel offset (x T) of the half the coupling updates
  };
  void reserve(int B, int T);
  size_t amax_floats(int B) const;

  TtsVitsFlowCfg cfg_;
  int device_;
  std::vector<Flow> flows_;
  float* arena_ = nullptr;
  float* ws_ = nullptr;
  size_t ws_bytes_ = 0;
  bool amax_prepass_ = false;
};

}  // namespace tts
