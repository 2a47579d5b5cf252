// HiFiGAN generator executor (see hifigan.cpp) and the small host utilities it shares
// with the Glow decoder executor.
#pragma once

#include <string>
#include <vector>

#include "common.hpp"
#include "tts_mi355x.h"

namespace tts {

// Restores the caller's current HIP device on scope exit (torch keeps its own notion).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    TTS_HIP_CHECK(hipGetDevice(&prev));
    if (prev != dev) TTS_HIP_CHECK(hipSetDevice(dev));
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

// Per-launch hipEvent timing for *_profiled entry points.
struct Profiler {
  struct Rec {
    std::string name;
    double flops, bytes;
    hipEvent_t a, b;
  };
  std::vector<Rec> recs;
  ~Profiler() {
    for (auto& r : recs) {
      (void)hipEventDestroy(r.a);
      (void)hipEventDestroy(r.b);
    }
  }
};

template <class F>
void run(Profiler* p, hipStream_t s, const char* name, double flops, double bytes, F&& launch) {
  if (!p) {
    launch();
    return;
  }
  Profiler::Rec r{name, flops, bytes, nullptr, nullptr};
  TTS_HIP_CHECK(hipEventCreate(&r.a));
  TTS_HIP_CHECK(hipEventCreate(&r.b));
  TTS_HIP_CHECK(hipEventRecord(r.a, s));
  launch();
  TTS_HIP_CHECK(hipEventRecord(r.b, s));
  p->recs.push_back(r);
}

std::vector<int64_t> hifigan_weight_shapes(const TtsHifiganCfg& c);
void hifigan_validate(const TtsHifiganCfg& c);

class Hifigan {
 public:
  Hifigan(const TtsHifiganCfg& cfg, const float* const* host_weights, int device);
  ~Hifigan();
  Hifigan(const Hifigan&) = delete;
  Hifigan& operator=(const Hifigan&) = delete;

  int64_t out_len(int T, int pad) const;
  int64_t workspace_bytes(int B, int T, int pad) const;
  void reserve(int B, int T, int pad);
  // Utterances whose padded length L = T + 2 pad exceeds one window (a channel plane of a batch
  // item would pass 2 GiB, the kernels' 32-bit buffer range, or TTS_MI355X_WINDOW_FRAMES is set)
  // run as overlapping time windows: payload [s0, s1) with window_halo() frames of context on
  // each side (>= the generator's receptive-field radius), each window through the plain
  // forward on a gathered copy of the replicate-padded mel, the payload's samples copied out.
  void forward(const float* mel, int B, int C, int T, int pad, const float* g, float* wav,
               hipStream_t s, Profiler* prof);
  int device() const { return device_; }
  int window_halo() const;        // receptive-field radius in mel frames, rounded up, + 2
  int64_t max_window_frames() const;  // largest window whose every channel plane stays < 2 GiB
  int64_t window_payload() const;     // payload frames per window

 private:
  struct ConvLayer {
    int Cin = 0, Cout = 0, K = 0, dil = 1, pad = 0, tile = 0, n_chunks = 0;
    int mode = 0;   // math mode of this layer (TTS_MATH_*)
    int w_exp = 0;  // packed weights hold w * 2^-w_exp (fp16 hi/lo mode)
    int64_t w_numel = 0, b_numel = 0;
    float* w = nullptr;
    float* b = nullptr;
    std::string name;
  };
  struct ConvTLayer {
    int Cin = 0, Cout = 0, U = 0, tile = 0, n_chunks = 0;
    int mode = 0;   // split modes run the K=2 polyphase conv form (Conv1dArgs::ups)
    int w_exp = 0;
    int64_t w_numel = 0, b_numel = 0;
    float* w = nullptr;
    float* b = nullptr;
    std::string name;
  };
  struct ResBlock {
    std::vector<ConvLayer> convs;  // type 1: c1_0, c2_0, c1_1, c2_1, c1_2, c2_2; type 2: c_0, c_1
    bool fused = false;            // type 1 iterations run as fused convs1 -> convs2 launches
    bool fused3 = false;           // type 1, kernel 3: the whole block in one launch (resblock3)
    bool fused2 = false;           // type 2: the whole block in one launch (resblock2)
  };

  // Execution lanes: the batch may split into n_lanes_ sub-batches (TTS_MI355X_SUBBATCH), each a
  // complete forward on its own workspace region and streams (utterances are independent and every
  // kernel is batch-invariant, so the output is bitwise the same); within a lane the MRF branches
  // spread over nbs_ streams (TTS_MI355X_MRF_STREAMS, default one per branch): branch j runs on
  // stream max(0, j - (num_kernels - nbs_)), each stream with its own X / T planes; the branches'
  // MRF-sum launches stay in order j = 0, 1, ... through events, so z = ((r0 + r1) + r2) / 3
  struct Lane {
    hipStream_t own = nullptr;         // lanes > 0: their main stream (lane 0 uses the caller's)
    std::vector<hipStream_t> branch;   // nbs_ - 1 branch streams
    hipEvent_t ev_ups = nullptr, ev_done = nullptr;
    std::vector<hipEvent_t> ev_z;      // per MRF branch
    int nbs = 1;                       // branch streams this forward uses (<= nbs_)
  };
  void forward_plain(const float* mel, int B, int C, int T, int pad, const float* g, float* wav, hipStream_t s,
                     Profiler* prof, float* ws, Lane* lane);
  void ensure_lanes();
  int64_t lane_bytes(int B, int64_t L, int nbs) const;
  int lane_batch(int B, int i) const { return B / n_lanes_ + (i < B % n_lanes_ ? 1 : 0); }
  bool windowed(int64_t L) const;
  int64_t plain_workspace_bytes(int B, int64_t L, bool window) const;
  int64_t window_buffer_bytes(int B, int64_t W) const;
  void reserve_plain(int B, int64_t L, bool window = false);
  int64_t plane_floats(int B, int T, int pad) const;
  int64_t cond_floats(int B) const;
  int amax_groups() const;
  int stage_group(int i) const;
  int n_planes(int nbs) const;  // activation planes of a lane's workspace (Z, O, then X / T per branch stream)
  int split_nbs() const;

  TtsHifiganCfg cfg_;
  int device_;
  int hop_ = 1;
  int rb2_geo64_ = 0;         // ResBlock2 at 64 channels: 1 = 192-column tiles (resblock2_geo64)
  bool post_fusion_ = true;  // conv_post inside the last MRF launch (TTS_MI355X_POST_FUSION=0: off)
  // MATH_BF16: the Z / O / X / T activation planes hold bf16 (conv_device.hpp PlaneT), halving the
  // bytes every kernel stages, gathers and stores; TTS_MI355X_BF16_PLANES=0 keeps fp32 planes
  bool planes16_ = false;
  // defaults (A/B on MI355X, config 2): two sub-batch lanes with one stream each when B >= 2
  // (51.5 ms per batch), else one lane with a stream per MRF branch (51.8 ms at B = 32; 3 x 2
  // streams: 52.5 ms)
  int nbs_ = 1;      // MRF branch streams per lane (workspace planes are sized for it)
  int n_lanes_ = 2;  // sub-batches
  bool nbs_env_ = false;
  std::vector<Lane> lanes_;
  hipEvent_t ev_start_ = nullptr;
  ConvLayer pre_;
  std::vector<ConvTLayer> ups_;
  std::vector<ResBlock> res_;
  const float* post_w_ = nullptr;  // host pointer, only valid during construction
  float post_bias_ = 0.f;
  float* post_wd_ = nullptr;
  float* cond_wd_ = nullptr;
  float* cond_bd_ = nullptr;
  std::vector<std::pair<float*, float*>> up_cond_;  // conds.i (w [C_i][cond], b [C_i]), XTTS
  float* arena_ = nullptr;
  size_t weights_bytes_ = 0;
  float* ws_ = nullptr;
  size_t ws_bytes_ = 0;
  float* win_ = nullptr;  // windowed forward: gathered mel window [B][C][W] + window output [B][hop*W]
  size_t win_bytes_ = 0;
};

}  // namespace tts
