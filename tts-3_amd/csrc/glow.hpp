// Glow-TTS decoder flow executor, reverse direction
// (TTS/tts/layers/glow_tts/decoder.py:113-137 with reverse=True).
#pragma once

#include <string>
#include <vector>

#include "common.hpp"
#include "hifigan.hpp"
#include "tts_mi355x.h"

namespace tts {

std::vector<int64_t> glow_weight_shapes(const TtsGlowDecoderCfg& c);
void glow_validate(const TtsGlowDecoderCfg& c);

// Elementwise kernels of the flow (kernels_glow.hip).
struct GlowTailArgs {
  float* x;            // [B][C2][Th], updated in place
  const float* out;    // [B][C2][Th] = end(WN(...)): rows [0,C2/2) = t, [C2/2,C2) = s
  const float* mask;   // [B][Th]
  const float* winv;   // [S][S] device
  const float* logs;   // [C2]
  const float* bias;   // [C2]
  int C2, Th, S;
  int sigmoid_scale;
  unsigned* amax_x0;   // [B][64] slots receiving max |x[:, :C2/2]| after the update (the next flow's
                       // start-conv input, f16x3), or nullptr
};
void launch_glow_squeeze(const float* x, const float* mask, float* xs, float* msq, int B, int C, int T,
                         int nsq, hipStream_t s);
void launch_glow_unsqueeze(const float* xs, const float* msq, float* y, int B, int C, int Th, int nsq,
                           hipStream_t s);
// amax: [B][64] max-abs slots of the output (f16x3 statistics of the next conv's input), or nullptr
// Conv tile of the Glow / VITS flow convs (glow.cpp): the plain per-shape table (smaller tiles for
// the flows' short column counts measured slower).
int flow_conv_tile(int mode, int Cout, int K, int Cin, int dil);
// Whether a WN in_layer (H -> 2H, kernel K, dilation dil) runs with the gate fused into its conv
// epilogue (kSplitGateTile): split modes, H % 64 == 0, K in {3, 5, 7}, the tile's halo, and
// TTS_MI355X_FLOW_GATE=1 at create time (opt-in: measured slower end to end at config 3).
bool flow_gate_fused(int mode, int H, int K, int dil);
bool flow_wn_fused(int mode, int H);
// Whether the WN layers of a flow run as one launch each (launch_glow_wn_layer): split modes, the
// supported (H, K, dilations), no opt-in gate / update fusion, unless TTS_MI355X_WN_LAYER=0 at
// create time (layer l's dilation: dilation_rate^l, wavenet.py:68)
bool flow_wn_layer(int mode, int H, int K, int dilation_rate, int L);
// f16x3 statistics of each flow's x0 (the start / pre conv input): by default the previous flow's
// last writer publishes them (the Glow tail kernel, the VITS post conv epilogue) and only the first
// flow runs a strided max-abs pre-pass; TTS_MI355X_FLOW_AMAX_PREPASS=1 at create time runs the
// pre-pass for every flow instead (the reference arm of the equality tests).
bool flow_amax_prepass();
// in_layer weights [2H][H][K] and bias [2H] in gate_row_order (for kSplitGateTile)
void gate_permute_rows(const float* w, const float* b, int H, int Cin, int K, std::vector<float>& wp,
                       std::vector<float>& bp);

void launch_glow_gate(const float* xin, float* acts, int B, int H, int Th, hipStream_t s,
                      unsigned* amax = nullptr);
void launch_glow_wn_update(float* h, float* skip, const float* rs, const float* mask, int B, int H,
                           int Th, int first, int last, hipStream_t s, unsigned* amax = nullptr);
void launch_glow_tail(const GlowTailArgs& a, int B, hipStream_t s);

// One WaveNet layer in one launch (wavenet.py:101-115): in_layer (H -> 2H, kernel K, dilation) +
// bias + cond -> fused_add_tanh_sigmoid_multiply -> res_skip (1x1) -> the h / skip update, per
// 32-column tile with the whole hidden width in the workgroup: xin, acts and rs never reach HBM,
// and 4 launches per layer become 1.  h is double-buffered (h_out != h_in: neighbouring tiles still
// read h_in's halo).  The fp32 operations are those of the unfused launches in the same order; in
// f16x3 the acts operand takes the fixed exponent of |acts| < 1 (the unfused res_skip's own
// per-utterance exponent whenever max |acts| >= 0.5), bf16 / bf16x6 take no scale.
// TTS_MI355X_WN_LAYER=0 at create time keeps the four launches per layer.
struct GlowWnLayerArgs {
  const float* h_in;     // [B][H][Th]
  float* h_out;          // [B][H][Th] (not the last layer)
  float* skip;           // [B][H][Th], = rs[H:] (first layer) or += (later ones)
  const float* mask;     // [B][Th]
  const float* w_in;     // in_layer, split packing (32-row blocks of steps_in steps)
  const float* b_in;     // [2H]
  const float* cvec;     // g_l rows [2H] of item b at cvec + b * cvec_bstride, or nullptr
  int64_t cvec_bstride;
  const float* w_rs;     // res_skip (1x1) split packing, rs_rows = 2H (H for the last layer)
  const float* b_rs;
  const unsigned* amax_h;  // f16x3: max-abs slots of h_in (its producer's), else nullptr
  unsigned* amax_out;      // f16x3: slots of h_out (not last) or skip (last), else nullptr
  int w_exp_in, w_exp_rs;
  int steps_in, steps_rs;  // packed steps per 32-row block
  int rs_blocks;           // 32-row blocks allocated in w_rs
  int H, Th, K, dil, first, last;
  // last layer only, optional (w_end != nullptr): the 1x1 conv that consumes skip (the Glow
  // coupling's `end`, glow.py:214) in the same launch: end_out = w_end * skip + b_end, end_rows
  // rows; skip itself is then not written.  Its f16x3 operand scale is the tile's max-abs exponent.
  const float* w_end;
  const float* b_end;
  float* end_out;        // [B][end_rows][Th]
  int end_rows, end_steps, end_blocks, w_exp_end;
  // reverse direction, with the end conv, optional (tail_x != nullptr): the flow's inverse tail
  // (glow_tail_kernel: coupling, InvConvNear, ActNorm; num_splits 4) on the tile's end output, x
  // updated in place, then the next flow's start conv into h_next (its f16x3 operand exponent:
  // the tile's max |x0|); end_out, the tail launch and the next start launch are not needed
  float* tail_x;           // [B][C2 = end_rows][Th]
  const float* winv;       // [4][4]
  const float* logs;       // [C2] ActNorm of this flow
  const float* abias;      // [C2]
  int sigmoid_scale;
  const float* w_start;    // next flow's start conv (C2/2 -> H), split packing
  const float* b_start;
  float* h_next;           // [B][H][Th], != h_in
  unsigned* amax_hnext;    // f16x3 slots of h_next, else nullptr
  int start_steps, start_blocks, w_exp_start;
};
// split modes, H in {128, 192, 256}, K in {3, 5}, (K - 1) * dil <= 16
bool glow_wn_layer_supported(int mode, int H, int K, int dil);
void launch_glow_wn_layer(int mode, const GlowWnLayerArgs& a, int B, hipStream_t s);
// The weight fields of layer l (l of L) from its in_layer / res_skip convs (any executor's Conv with
// w, b, w_exp, tile, n_chunks, Cout, K, dil); the caller fills the planes, cond and statistics
template <class Cv>
GlowWnLayerArgs wn_layer_weights(int mode, const Cv& ci, const Cv& cr, int H, int Th, int l, int L) {
  const ConvTile ti = conv_tile(mode, ci.tile), tr = conv_tile(mode, cr.tile);
  GlowWnLayerArgs w{};
  w.w_in = ci.w; w.b_in = ci.b; w.w_rs = cr.w; w.b_rs = cr.b;
  w.w_exp_in = ci.w_exp; w.w_exp_rs = cr.w_exp;
  w.steps_in = ci.n_chunks * (ti.CK / 16) * ci.K;
  w.steps_rs = cr.n_chunks * (tr.CK / 16);
  w.rs_blocks = ceil_div(cr.Cout, tr.BM) * tr.BM / 32;
  w.H = H; w.Th = Th; w.K = ci.K; w.dil = ci.dil; w.first = l == 0; w.last = l == L - 1;
  return w;
}
// forward direction (reverse=False)
struct GlowHeadArgs {  // ActNorm -> InvConvNear forward of one flow block, in place
  float* x;            // [B][C2][Th]
  const float* mask;   // [B][Th]
  const float* w;      // [S][S] InvConvNear weight (glow.py:97-100)
  const float* logs;   // [C2]
  const float* bias;   // [C2]
  int C2, Th, S;
  unsigned* amax_x0;   // f16x3 statistics of x[:, :C2/2] after the update, or nullptr
};
struct GlowCoupleArgs {  // coupling forward of one block, then (w != nullptr) the next block's head
  float* x;
  const float* out;    // end(WN(...)): rows [0,C2/2) = t, [C2/2,C2) = s
  const float* mask;
  int C2, Th, S;
  int sigmoid_scale;
  double* ld_part;     // [B][glow_couple_parts()] partial sums of s * mask, or nullptr
  const float* w;      // next block's head (nullptr: none)
  const float* logs;
  const float* bias;
  unsigned* amax_x0;
};
constexpr int kGlowLogdetParts = 128;  // at most this many workgroups (logdet partials) per utterance
void launch_glow_head(const GlowHeadArgs& a, int B, hipStream_t s);
int glow_couple_parts(int C2, int S, int Th);
void launch_glow_couple_fwd(const GlowCoupleArgs& a, int B, hipStream_t s);
void launch_glow_logdet(const double* parts, int nparts, int npb, const float* mask, int Th, double per_len,
                        float* logdet, int B, hipStream_t s);
void launch_channel_flip(const float* x, float* y, int B, int C, int T, hipStream_t s);  // torch.flip(x, [1])

class GlowDecoder {
 public:
  GlowDecoder(const TtsGlowDecoderCfg& cfg, const float* const* host_weights, int device);
  ~GlowDecoder();
  GlowDecoder(const GlowDecoder&) = delete;
  GlowDecoder& operator=(const GlowDecoder&) = delete;
  // g: [B][c_in_channels] speaker vector (the reference's g [B][c_in][1]), NULL when c_in_channels == 0
  void reverse(const float* x, const float* mask, const float* g, int B, int C, int T, float* y, hipStream_t s,
               Profiler* prof = nullptr);
  // reverse=False (decoder.py:119-133): y = the flows in order, logdet[B] (fp32, nullptr: not computed)
  void forward(const float* x, const float* mask, const float* g, int B, int C, int T, float* y, float* logdet,
               hipStream_t s, Profiler* prof = nullptr);
  int device() const { return device_; }

 private:
  struct Conv {
    int Cin = 0, Cout = 0, K = 1, dil = 1, tile = 0, n_chunks = 0, w_exp = 0;
    bool gated = false;  // in_layer with the WN gate fused (kSplitGateTile)
    float* w = nullptr;
    float* b = nullptr;
  };
  struct Flow {
    float* logs = nullptr;
    float* bias = nullptr;
    float* winv = nullptr;
    float* w = nullptr;       // InvConvNear weight (forward direction)
    double per_len = 0.0;     // sum(logs) + logdet(W) * C2 / S: the block's logdet per unmasked frame
    float* cond_w = nullptr;  // wn.cond_layer [2HL][c_in] fp32 (c_in_channels > 0)
    float* cond_b = nullptr;
    Conv start, end;
    std::vector<Conv> in_layers, res_skip;
  };
  void run_flows(bool rev, const float* x, const float* mask, const float* g, int B, int C, int T, float* y,
                 float* logdet, hipStream_t s, Profiler* prof);
  void reserve(int B, int Th);
  size_t amax_floats(int B) const;

  TtsGlowDecoderCfg cfg_;
  int device_;
  std::vector<Flow> flows_;
  float* arena_ = nullptr;
  float* ws_ = nullptr;
  size_t ws_bytes_ = 0;
  bool amax_prepass_ = false;
  bool wn_fused_ = false;  // res_skip conv + WN update in one launch (flow_wn_fused)
  bool wn_layer_ = false;  // every WN layer in one launch (glow_wn_layer_kernel, flow_wn_layer)
  bool wn_end_ = false;    // ... and the coupling's end conv inside the last one (TTS_MI355X_WN_END)
  bool wn_tail_ = false;   // ... and, reverse, the tail + the next flow's start conv (TTS_MI355X_WN_TAIL)
};

}  // namespace tts
