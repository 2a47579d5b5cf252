// extern "C" entry points of libtts_mi355x.so (declared in include/tts_mi355x.h).
// Every call converts library exceptions into a status code + thread-local message.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "glow.hpp"
#include "handoff.hpp"
#include "hifigan.hpp"
#include "text.hpp"
#include "vits.hpp"
#include "tts_mi355x.h"

namespace {
thread_local std::string g_last_error;

template <class F>
int guarded(F&& f) {
  try {
    g_last_error.clear();
    f();
    return TTS_OK;
  } catch (const tts::Error& e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "host allocation failed";
    return TTS_ERR_OOM;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return TTS_ERR_INVALID;
  } catch (...) {
    g_last_error = "unknown error";
    return TTS_ERR_INVALID;
  }
}

void export_records(const tts::Profiler& prof, TtsLaunchRecord* records, int max_records, int* n_records) {
  *n_records = (int)prof.recs.size();
  for (int i = 0; i < (int)prof.recs.size() && i < max_records && records; ++i) {
    const auto& r = prof.recs[i];
    std::memset(records[i].name, 0, sizeof(records[i].name));
    std::strncpy(records[i].name, r.name.c_str(), sizeof(records[i].name) - 1);
    records[i].flops = r.flops;
    records[i].bytes = r.bytes;
    float ms = 0.f;
    TTS_HIP_CHECK(hipEventElapsedTime(&ms, r.a, r.b));
    records[i].ms = ms;
  }
}

// RAII device buffer for the single-op entry points.
struct TmpDev {
  float* p = nullptr;
  explicit TmpDev(const float* host, size_t n) {
    if (n == 0) return;
    if (hipMalloc(&p, n * sizeof(float)) != hipSuccess) throw tts::Error(4, "hipMalloc failed");
    if (host) TTS_HIP_CHECK(hipMemcpy(p, host, n * sizeof(float), hipMemcpyHostToDevice));
  }
  ~TmpDev() {
    if (p) (void)hipFree(p);
  }
};
}  // namespace

extern "C" {

const char* tts_last_error(void) { return g_last_error.c_str(); }
int tts_abi_version(void) { return 115; }
const char* tts_build_target(void) { return "gfx950"; }

// ----------------------------------------------------------------------------- HiFiGAN
int tts_hifigan_num_weights(const TtsHifiganCfg* cfg) {
  int n = -1;
  int st = guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::hifigan_validate(*cfg);
    n = (int)tts::hifigan_weight_shapes(*cfg).size();
  });
  return st == TTS_OK ? n : -st;
}

int64_t tts_hifigan_weight_numel(const TtsHifiganCfg* cfg, int idx) {
  int64_t n = -1;
  guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::hifigan_validate(*cfg);
    auto s = tts::hifigan_weight_shapes(*cfg);
    TTS_REQUIRE(idx >= 0 && idx < (int)s.size(), 1, "weight index out of range");
    n = s[idx];
  });
  return n;
}

int tts_hifigan_create(const TtsHifiganCfg* cfg, const float* const* host_weights, int device,
                       void** handle) {
  return guarded([&] {
    TTS_REQUIRE(cfg && host_weights && handle, 1, "NULL argument");
    *handle = nullptr;
    *handle = new tts::Hifigan(*cfg, host_weights, device);
  });
}

int tts_hifigan_destroy(void* handle) {
  return guarded([&] { delete static_cast<tts::Hifigan*>(handle); });
}

int64_t tts_hifigan_output_length(const void* handle, int T, int pad) {
  if (!handle) return -1;
  return static_cast<const tts::Hifigan*>(handle)->out_len(T, pad);
}

int64_t tts_hifigan_workspace_bytes(const void* handle, int B, int T, int pad) {
  if (!handle) return -1;
  return static_cast<const tts::Hifigan*>(handle)->workspace_bytes(B, T, pad);
}

int tts_hifigan_reserve(void* handle, int B, int T, int pad) {
  return guarded([&] {
    TTS_REQUIRE(handle, 1, "NULL handle");
    TTS_REQUIRE(B >= 1 && T >= 1 && pad >= 0, 1, "bad shape");
    static_cast<tts::Hifigan*>(handle)->reserve(B, T, pad);
  });
}

int tts_hifigan_forward(void* handle, const float* d_mel, int B, int C, int T, int pad,
                        const float* d_g, float* d_wav, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(handle, 1, "NULL handle");
    static_cast<tts::Hifigan*>(handle)->forward(d_mel, B, C, T, pad, d_g, d_wav,
                                                static_cast<hipStream_t>(hip_stream), nullptr);
  });
}

int tts_hifigan_forward_profiled(void* handle, const float* d_mel, int B, int C, int T, int pad,
                                 const float* d_g, float* d_wav, void* hip_stream,
                                 TtsLaunchRecord* records, int max_records, int* n_records) {
  return guarded([&] {
    TTS_REQUIRE(handle && n_records, 1, "NULL argument");
    auto* h = static_cast<tts::Hifigan*>(handle);
    auto s = static_cast<hipStream_t>(hip_stream);
    tts::Profiler prof;
    {
      tts::DeviceGuard g(h->device());
      h->forward(d_mel, B, C, T, pad, d_g, d_wav, s, &prof);
      TTS_HIP_CHECK(hipStreamSynchronize(s));
    }
    export_records(prof, records, max_records, n_records);
  });
}

// ----------------------------------------------------------------------------- Glow encoder + glue
int tts_glow_encoder_num_weights(const TtsGlowEncoderCfg* cfg) {
  int n = -1;
  int st = guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::glow_encoder_validate(*cfg);
    n = (int)tts::glow_encoder_weight_shapes(*cfg).size();
  });
  return st == TTS_OK ? n : -st;
}

int64_t tts_glow_encoder_weight_numel(const TtsGlowEncoderCfg* cfg, int idx) {
  int64_t n = -1;
  guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::glow_encoder_validate(*cfg);
    auto s = tts::glow_encoder_weight_shapes(*cfg);
    TTS_REQUIRE(idx >= 0 && idx < (int)s.size(), 1, "weight index out of range");
    n = s[idx];
  });
  return n;
}

int tts_glow_encoder_create(const TtsGlowEncoderCfg* cfg, const float* const* host_weights, int device,
                            void** handle) {
  return guarded([&] {
    TTS_REQUIRE(cfg && host_weights && handle, 1, "NULL argument");
    *handle = nullptr;
    *handle = new tts::GlowEncoder(*cfg, host_weights, device);
  });
}

int tts_glow_encoder_destroy(void* handle) {
  return guarded([&] { delete static_cast<tts::GlowEncoder*>(handle); });
}

int tts_glow_encoder_forward(void* handle, const int64_t* d_tokens, const int64_t* d_lengths, const float* d_g,
                             int B, int T, float* d_x_m, float* d_x_logs, float* d_logw, float* d_x_mask,
                             void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(handle, 1, "NULL handle");
    static_cast<tts::GlowEncoder*>(handle)->forward(d_tokens, d_lengths, d_g, B, T, d_x_m, d_x_logs, d_logw,
                                                    d_x_mask, static_cast<hipStream_t>(hip_stream));
  });
}

int tts_glow_encoder_forward_profiled(void* handle, const int64_t* d_tokens, const int64_t* d_lengths,
                                      const float* d_g, int B, int T, float* d_x_m, float* d_x_logs, float* d_logw,
                                      float* d_x_mask,
                                      void* hip_stream, TtsLaunchRecord* records, int max_records,
                                      int* n_records) {
  return guarded([&] {
    TTS_REQUIRE(handle && n_records, 1, "NULL argument");
    auto* h = static_cast<tts::GlowEncoder*>(handle);
    auto s = static_cast<hipStream_t>(hip_stream);
    tts::Profiler prof;
    {
      tts::DeviceGuard g(h->device());
      h->forward(d_tokens, d_lengths, d_g, B, T, d_x_m, d_x_logs, d_logw, d_x_mask, s, &prof);
      TTS_HIP_CHECK(hipStreamSynchronize(s));
    }
    export_records(prof, records, max_records, n_records);
  });
}

int tts_glow_durations(const float* d_logw, const float* d_x_mask, int B, int T_x, float length_scale,
                       float* d_w_ceil, int64_t* d_y_lengths, float* d_o_attn_dur, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_logw && d_x_mask && d_w_ceil && d_y_lengths, 1, "NULL argument");
    TTS_REQUIRE(B >= 1 && T_x >= 1, 1, "batch and token count must be >= 1");
    tts::launch_durations(d_logw, d_x_mask, d_w_ceil, d_y_lengths, d_o_attn_dur, B, T_x, length_scale,
                          static_cast<hipStream_t>(hip_stream));
    TTS_HIP_CHECK(hipGetLastError());
  });
}

int tts_glow_expand(const float* d_w_ceil, const float* d_x_mask, const int64_t* d_y_lengths,
                    const float* d_o_mean, const float* d_o_log_scale, const float* d_noise, float noise_scale,
                    int B, int C, int T_x, int T_y, float* d_z, float* d_y_mask, float* d_y_mean,
                    float* d_y_log_scale, float* d_attn, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_w_ceil && d_x_mask && d_y_lengths && d_o_mean && d_z && d_y_mask, 1, "NULL argument");
    TTS_REQUIRE(B >= 1 && C >= 1 && T_x >= 1 && T_y >= 1, 1, "bad expand shape");
    tts::ExpandArgs a{};
    a.w_ceil = d_w_ceil; a.x_mask = d_x_mask; a.y_len = d_y_lengths; a.o_mean = d_o_mean;
    a.o_log_scale = d_o_log_scale; a.noise = d_noise; a.noise_scale = noise_scale;
    a.C = C; a.T_x = T_x; a.T_y = T_y;
    a.z = d_z; a.y_mask = d_y_mask; a.y_mean = d_y_mean; a.y_log_scale = d_y_log_scale; a.attn = d_attn;
    tts::launch_expand(a, B, static_cast<hipStream_t>(hip_stream));
    TTS_HIP_CHECK(hipGetLastError());
  });
}

// ----------------------------------------------------------------------------- VITS text side
int tts_vits_text_encoder_num_weights(const TtsVitsTextEncoderCfg* cfg) {
  int n = -1;
  int st = guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_text_encoder_validate(*cfg);
    n = (int)tts::vits_text_encoder_weight_shapes(*cfg).size();
  });
  return st == TTS_OK ? n : -st;
}

int64_t tts_vits_text_encoder_weight_numel(const TtsVitsTextEncoderCfg* cfg, int idx) {
  int64_t n = -1;
  guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_text_encoder_validate(*cfg);
    auto s = tts::vits_text_encoder_weight_shapes(*cfg);
    TTS_REQUIRE(idx >= 0 && idx < (int)s.size(), 1, "weight index out of range");
    n = s[idx];
  });
  return n;
}

int tts_vits_text_encoder_create(const TtsVitsTextEncoderCfg* cfg, const float* const* host_weights, int device,
                                 void** handle) {
  return guarded([&] {
    TTS_REQUIRE(cfg && host_weights && handle, 1, "NULL argument");
    *handle = nullptr;
    *handle = new tts::VitsTextEncoder(*cfg, host_weights, device);
  });
}

int tts_vits_text_encoder_destroy(void* handle) {
  return guarded([&] { delete static_cast<tts::VitsTextEncoder*>(handle); });
}

int tts_vits_text_encoder_forward(void* handle, const int64_t* d_tokens, const int64_t* d_lengths,
                                  const float* d_lang_emb, int B, int T, float* d_x, float* d_m, float* d_logs,
                                  float* d_x_mask, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(handle, 1, "NULL handle");
    static_cast<tts::VitsTextEncoder*>(handle)->forward(d_tokens, d_lengths, d_lang_emb, B, T, d_x, d_m, d_logs,
                                                        d_x_mask, static_cast<hipStream_t>(hip_stream));
  });
}

int tts_vits_text_encoder_forward_profiled(void* handle, const int64_t* d_tokens, const int64_t* d_lengths,
                                           const float* d_lang_emb, int B, int T, float* d_x, float* d_m,
                                           float* d_logs, float* d_x_mask, void* hip_stream,
                                           TtsLaunchRecord* records, int max_records, int* n_records) {
  return guarded([&] {
    TTS_REQUIRE(handle && n_records, 1, "NULL argument");
    auto* h = static_cast<tts::VitsTextEncoder*>(handle);
    auto s = static_cast<hipStream_t>(hip_stream);
    tts::Profiler prof;
    {
      tts::DeviceGuard g(h->device());
      h->forward(d_tokens, d_lengths, d_lang_emb, B, T, d_x, d_m, d_logs, d_x_mask, s, &prof);
      TTS_HIP_CHECK(hipStreamSynchronize(s));
    }
    export_records(prof, records, max_records, n_records);
  });
}

int tts_vits_sdp_num_weights(const TtsVitsSdpCfg* cfg) {
  int n = -1;
  int st = guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_sdp_validate(*cfg);
    n = (int)tts::vits_sdp_weight_shapes(*cfg).size();
  });
  return st == TTS_OK ? n : -st;
}

int64_t tts_vits_sdp_weight_numel(const TtsVitsSdpCfg* cfg, int idx) {
  int64_t n = -1;
  guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_sdp_validate(*cfg);
    auto s = tts::vits_sdp_weight_shapes(*cfg);
    TTS_REQUIRE(idx >= 0 && idx < (int)s.size(), 1, "weight index out of range");
    n = s[idx];
  });
  return n;
}

int tts_vits_sdp_create(const TtsVitsSdpCfg* cfg, const float* const* host_weights, int device, void** handle) {
  return guarded([&] {
    TTS_REQUIRE(cfg && host_weights && handle, 1, "NULL argument");
    *handle = nullptr;
    *handle = new tts::VitsSdp(*cfg, host_weights, device);
  });
}

int tts_vits_sdp_destroy(void* handle) {
  return guarded([&] { delete static_cast<tts::VitsSdp*>(handle); });
}

int tts_vits_sdp_reverse(void* handle, const float* d_x, const float* d_x_mask, const float* d_g,
                         const float* d_lang_emb, const float* d_noise, float noise_scale, int B, int T,
                         float* d_logw, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(handle, 1, "NULL handle");
    static_cast<tts::VitsSdp*>(handle)->reverse(d_x, d_x_mask, d_g, d_lang_emb, d_noise, noise_scale, B, T, d_logw,
                                                static_cast<hipStream_t>(hip_stream));
  });
}

int tts_vits_sdp_reverse_profiled(void* handle, const float* d_x, const float* d_x_mask, const float* d_g,
                                  const float* d_lang_emb, const float* d_noise, float noise_scale, int B, int T,
                                  float* d_logw, void* hip_stream, TtsLaunchRecord* records, int max_records,
                                  int* n_records) {
  return guarded([&] {
    TTS_REQUIRE(handle && n_records, 1, "NULL argument");
    auto* h = static_cast<tts::VitsSdp*>(handle);
    auto s = static_cast<hipStream_t>(hip_stream);
    tts::Profiler prof;
    {
      tts::DeviceGuard g(h->device());
      h->reverse(d_x, d_x_mask, d_g, d_lang_emb, d_noise, noise_scale, B, T, d_logw, s, &prof);
      TTS_HIP_CHECK(hipStreamSynchronize(s));
    }
    export_records(prof, records, max_records, n_records);
  });
}

int tts_vits_dp_num_weights(const TtsVitsDpCfg* cfg) {
  int n = -1;
  int st = guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_dp_validate(*cfg);
    n = (int)tts::vits_dp_weight_shapes(*cfg).size();
  });
  return st == TTS_OK ? n : -st;
}

int64_t tts_vits_dp_weight_numel(const TtsVitsDpCfg* cfg, int idx) {
  int64_t n = -1;
  guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_dp_validate(*cfg);
    auto s = tts::vits_dp_weight_shapes(*cfg);
    TTS_REQUIRE(idx >= 0 && idx < (int)s.size(), 1, "weight index out of range");
    n = s[idx];
  });
  return n;
}

int tts_vits_dp_create(const TtsVitsDpCfg* cfg, const float* const* host_weights, int device, void** handle) {
  return guarded([&] {
    TTS_REQUIRE(cfg && host_weights && handle, 1, "NULL argument");
    *handle = nullptr;
    *handle = new tts::VitsDp(*cfg, host_weights, device);
  });
}

int tts_vits_dp_destroy(void* handle) {
  return guarded([&] { delete static_cast<tts::VitsDp*>(handle); });
}

int tts_vits_dp_forward(void* handle, const float* d_x, const float* d_x_mask, const float* d_g,
                        const float* d_lang_emb, int B, int T, float* d_logw, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(handle, 1, "NULL handle");
    static_cast<tts::VitsDp*>(handle)->forward(d_x, d_x_mask, d_g, d_lang_emb, B, T, d_logw,
                                               static_cast<hipStream_t>(hip_stream));
  });
}

int tts_vits_dp_forward_profiled(void* handle, const float* d_x, const float* d_x_mask, const float* d_g,
                                 const float* d_lang_emb, int B, int T, float* d_logw, void* hip_stream,
                                 TtsLaunchRecord* records, int max_records, int* n_records) {
  return guarded([&] {
    TTS_REQUIRE(handle && n_records, 1, "NULL argument");
    auto* h = static_cast<tts::VitsDp*>(handle);
    auto s = static_cast<hipStream_t>(hip_stream);
    tts::Profiler prof;
    {
      tts::DeviceGuard g(h->device());
      h->forward(d_x, d_x_mask, d_g, d_lang_emb, B, T, d_logw, s, &prof);
      TTS_HIP_CHECK(hipStreamSynchronize(s));
    }
    export_records(prof, records, max_records, n_records);
  });
}

int tts_vits_durations(const float* d_logw, const float* d_x_mask, int B, int T_x, float length_scale,
                       float* d_w_ceil, int64_t* d_y_lengths, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_logw && d_x_mask && d_w_ceil && d_y_lengths, 1, "NULL argument");
    TTS_REQUIRE(B >= 1 && T_x >= 1, 1, "batch and token count must be >= 1");
    tts::launch_durations(d_logw, d_x_mask, d_w_ceil, d_y_lengths, nullptr, B, T_x, length_scale,
                          static_cast<hipStream_t>(hip_stream), 1);
    TTS_HIP_CHECK(hipGetLastError());
  });
}

int tts_vits_expand(const float* d_w_ceil, const float* d_x_mask, const int64_t* d_y_lengths, const float* d_m_p,
                    const float* d_logs_p, const float* d_noise, float noise_scale, int B, int C, int T_x, int T_y,
                    float* d_z_p, float* d_y_mask, float* d_m_p_out, float* d_logs_p_out, float* d_attn,
                    void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_w_ceil && d_x_mask && d_y_lengths && d_m_p && d_logs_p && d_z_p && d_y_mask, 1, "NULL argument");
    TTS_REQUIRE(B >= 1 && C >= 1 && T_x >= 1 && T_y >= 1, 1, "bad expand shape");
    tts::ExpandArgs a{};
    a.w_ceil = d_w_ceil; a.x_mask = d_x_mask; a.y_len = d_y_lengths; a.o_mean = d_m_p;
    a.o_log_scale = d_logs_p; a.noise = d_noise; a.noise_scale = noise_scale;
    a.C = C; a.T_x = T_x; a.T_y = T_y;
    a.z = d_z_p; a.y_mask = d_y_mask; a.y_mean = d_m_p_out; a.y_log_scale = d_logs_p_out; a.attn = d_attn;
    a.vits = 1;
    tts::launch_expand(a, B, static_cast<hipStream_t>(hip_stream));
    TTS_HIP_CHECK(hipGetLastError());
  });
}

int tts_vits_durations_given(const float* d_durations, int64_t dur_bstride, int B, int T_x, float* d_w_ceil,
                             int64_t* d_y_lengths, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_durations && d_w_ceil && d_y_lengths, 1, "NULL argument");
    TTS_REQUIRE(B >= 1 && T_x >= 1 && (dur_bstride == 0 || dur_bstride >= T_x), 1, "bad durations shape");
    tts::launch_given_durations(d_durations, dur_bstride, d_w_ceil, d_y_lengths, B, T_x,
                                static_cast<hipStream_t>(hip_stream));
  });
}

int tts_vits_mask_slice(const float* d_z, const float* d_y_mask, int B, int C, int T, int T_out, float* d_out,
                        void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_z && d_y_mask && d_out, 1, "NULL argument");
    tts::launch_mask_slice(d_z, d_y_mask, d_out, B, C, T, T_out, static_cast<hipStream_t>(hip_stream));
  });
}

int tts_vits_upsample_z(const float* d_z, const int64_t* d_y_lengths, int B, int C, int T, double factor, int T2,
                        float* d_z2, float* d_y_mask2, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_z && d_z2 && (d_y_lengths || !d_y_mask2), 1, "NULL argument");
    TTS_REQUIRE(factor > 0.0 && T2 == (int)std::floor((double)T * factor), 1,
                "upsample_z: T2 must be floor(T * factor) (F.interpolate's output length)");
    tts::launch_upsample_z(d_z, d_y_lengths, d_z2, d_y_mask2, B, C, T, T2, factor,
                           static_cast<hipStream_t>(hip_stream));
  });
}

int tts_embedding_rows(const float* d_table, int num, int dim, const int64_t* d_ids, int64_t id_stride, int B,
                       float* d_out, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_table && d_ids && d_out, 1, "NULL argument");
    tts::launch_embedding_rows(d_table, d_ids, id_stride, d_out, B, dim, num, static_cast<hipStream_t>(hip_stream));
  });
}

int tts_l2_normalize_rows(const float* d_in, int B, int C, float* d_out, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_in && d_out, 1, "NULL argument");
    tts::launch_l2_normalize(d_in, d_out, B, C, static_cast<hipStream_t>(hip_stream));
  });
}

// ----------------------------------------------------------------------------- hand-off / wav writer
namespace {
tts::AudioNormDev to_dev(const TtsAudioNormCfg* c) {
  tts::AudioNormDev d{};
  if (!c || !c->signal_norm) return d;  // signal_norm = 0: identity
  TTS_REQUIRE((c->d_mel_mean == nullptr) == (c->d_mel_scale == nullptr), 1,
              "mel_scaler needs both d_mel_mean and d_mel_scale");
  d.signal_norm = 1;
  d.symmetric_norm = c->symmetric_norm;
  d.clip_norm = c->clip_norm;
  d.max_norm = (float)c->max_norm;
  d.two_max_norm = (float)(2.0 * c->max_norm);       // (2 * self.max_norm) in Python
  d.min_level_db = (float)c->min_level_db;
  d.neg_min_level_db = (float)(-c->min_level_db);   // -self.min_level_db in Python
  d.ref_level_db = (float)c->ref_level_db;
  d.mean = c->d_mel_mean;
  d.scale = c->d_mel_scale;
  return d;
}
}  // namespace

int tts_mel_handoff(const float* d_in, int B, int T, int C, int time_major, const TtsAudioNormCfg* denorm,
                    const TtsAudioNormCfg* norm, int T_out, float src_scale, float* d_out, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_in && d_out, 1, "NULL argument");
    TTS_REQUIRE(B >= 1 && T >= 1 && C >= 1 && T_out >= 1, 1, "bad hand-off shape");
    TTS_REQUIRE(C <= 65535 && B <= 65535, 3, "hand-off: C and B must be <= 65535");
    tts::HandoffArgs a{};
    a.in = d_in; a.out = d_out; a.T = T; a.C = C; a.T_out = T_out; a.time_major = time_major ? 1 : 0;
    a.src_scale = src_scale;
    a.de = to_dev(denorm);
    a.no = to_dev(norm);
    tts::launch_handoff(a, B, static_cast<hipStream_t>(hip_stream));
    TTS_HIP_CHECK(hipGetLastError());
  });
}

int tts_wav_to_int16(const float* d_wav, int B, int64_t n, const int64_t* d_lengths, unsigned* d_scratch,
                     int16_t* d_out, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_wav && d_scratch && d_out, 1, "NULL argument");
    TTS_REQUIRE(B >= 1 && B <= 65535 && n >= 1, 1, "bad wav shape");
    tts::launch_wav_int16(d_wav, B, n, d_lengths, d_scratch, d_out, static_cast<hipStream_t>(hip_stream));
    TTS_HIP_CHECK(hipGetLastError());
  });
}

// ----------------------------------------------------------------------------- Glow decoder
int tts_glow_decoder_num_weights(const TtsGlowDecoderCfg* cfg) {
  int n = -1;
  int st = guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::glow_validate(*cfg);
    n = (int)tts::glow_weight_shapes(*cfg).size();
  });
  return st == TTS_OK ? n : -st;
}

int64_t tts_glow_decoder_weight_numel(const TtsGlowDecoderCfg* cfg, int idx) {
  int64_t n = -1;
  guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::glow_validate(*cfg);
    auto s = tts::glow_weight_shapes(*cfg);
    TTS_REQUIRE(idx >= 0 && idx < (int)s.size(), 1, "weight index out of range");
    n = s[idx];
  });
  return n;
}

int tts_glow_decoder_create(const TtsGlowDecoderCfg* cfg, const float* const* host_weights,
                            int device, void** handle) {
  return guarded([&] {
    TTS_REQUIRE(cfg && host_weights && handle, 1, "NULL argument");
    *handle = nullptr;
    *handle = new tts::GlowDecoder(*cfg, host_weights, device);
  });
}

int tts_glow_decoder_destroy(void* handle) {
  return guarded([&] { delete static_cast<tts::GlowDecoder*>(handle); });
}

int tts_glow_decoder_forward(void* handle, const float* d_x, const float* d_mask, const float* d_g, int B,
                             int C, int T, int reverse, float* d_y, float* d_logdet, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(handle, 1, "NULL handle");
    TTS_REQUIRE(reverse == 0 || reverse == 1, 1, "reverse must be 0 or 1");
    auto* h = static_cast<tts::GlowDecoder*>(handle);
    if (reverse) h->reverse(d_x, d_mask, d_g, B, C, T, d_y, static_cast<hipStream_t>(hip_stream));
    else h->forward(d_x, d_mask, d_g, B, C, T, d_y, d_logdet, static_cast<hipStream_t>(hip_stream));
  });
}

int tts_glow_decoder_forward_profiled(void* handle, const float* d_x, const float* d_mask, const float* d_g,
                                      int B, int C, int T, int reverse, float* d_y, float* d_logdet,
                                      void* hip_stream, TtsLaunchRecord* records, int max_records, int* n_records) {
  return guarded([&] {
    TTS_REQUIRE(handle && n_records, 1, "NULL argument");
    TTS_REQUIRE(reverse == 0 || reverse == 1, 1, "reverse must be 0 or 1");
    auto* h = static_cast<tts::GlowDecoder*>(handle);
    auto s = static_cast<hipStream_t>(hip_stream);
    tts::Profiler prof;
    {
      tts::DeviceGuard g(h->device());
      if (reverse) h->reverse(d_x, d_mask, d_g, B, C, T, d_y, s, &prof);
      else h->forward(d_x, d_mask, d_g, B, C, T, d_y, d_logdet, s, &prof);
      TTS_HIP_CHECK(hipStreamSynchronize(s));
    }
    export_records(prof, records, max_records, n_records);
  });
}

// ----------------------------------------------------------------------------- VITS flow
int tts_vits_flow_num_weights(const TtsVitsFlowCfg* cfg) {
  int n = -1;
  int st = guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_flow_validate(*cfg);
    n = (int)tts::vits_flow_weight_shapes(*cfg).size();
  });
  return st == TTS_OK ? n : -st;
}

int64_t tts_vits_flow_weight_numel(const TtsVitsFlowCfg* cfg, int idx) {
  int64_t n = -1;
  guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_flow_validate(*cfg);
    auto s = tts::vits_flow_weight_shapes(*cfg);
    TTS_REQUIRE(idx >= 0 && idx < (int)s.size(), 1, "weight index out of range");
    n = s[idx];
  });
  return n;
}

int tts_vits_flow_create(const TtsVitsFlowCfg* cfg, const float* const* host_weights, int device, void** handle) {
  return guarded([&] {
    TTS_REQUIRE(cfg && host_weights && handle, 1, "NULL argument");
    *handle = nullptr;
    *handle = new tts::VitsFlow(*cfg, host_weights, device);
  });
}

int tts_vits_flow_destroy(void* handle) {
  return guarded([&] { delete static_cast<tts::VitsFlow*>(handle); });
}

int tts_vits_flow_forward(void* handle, const float* d_x, const float* d_mask, const float* d_g, int B, int C,
                          int T, int reverse, float* d_y, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(handle, 1, "NULL handle");
    TTS_REQUIRE(reverse == 0 || reverse == 1, 1, "reverse must be 0 or 1");
    auto* h = static_cast<tts::VitsFlow*>(handle);
    if (reverse) h->reverse(d_x, d_mask, d_g, B, C, T, d_y, static_cast<hipStream_t>(hip_stream));
    else h->forward(d_x, d_mask, d_g, B, C, T, d_y, static_cast<hipStream_t>(hip_stream));
  });
}

int tts_vits_flow_forward_profiled(void* handle, const float* d_x, const float* d_mask, const float* d_g, int B,
                                   int C, int T, int reverse, float* d_y, void* hip_stream,
                                   TtsLaunchRecord* records, int max_records, int* n_records) {
  return guarded([&] {
    TTS_REQUIRE(handle && n_records, 1, "NULL argument");
    TTS_REQUIRE(reverse == 0 || reverse == 1, 1, "reverse must be 0 or 1");
    auto* h = static_cast<tts::VitsFlow*>(handle);
    auto s = static_cast<hipStream_t>(hip_stream);
    tts::Profiler prof;
    {
      tts::DeviceGuard g(h->device());
      if (reverse) h->reverse(d_x, d_mask, d_g, B, C, T, d_y, s, &prof);
      else h->forward(d_x, d_mask, d_g, B, C, T, d_y, s, &prof);
      TTS_HIP_CHECK(hipStreamSynchronize(s));
    }
    export_records(prof, records, max_records, n_records);
  });
}

// ----------------------------------------------------------------------------- VITS posterior encoder
int tts_vits_posterior_num_weights(const TtsVitsPosteriorCfg* cfg) {
  int n = -1;
  int st = guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_posterior_validate(*cfg);
    n = (int)tts::vits_posterior_weight_shapes(*cfg).size();
  });
  return st == TTS_OK ? n : -st;
}

int64_t tts_vits_posterior_weight_numel(const TtsVitsPosteriorCfg* cfg, int idx) {
  int64_t n = -1;
  guarded([&] {
    TTS_REQUIRE(cfg, 1, "NULL cfg");
    tts::vits_posterior_validate(*cfg);
    auto s = tts::vits_posterior_weight_shapes(*cfg);
    TTS_REQUIRE(idx >= 0 && idx < (int)s.size(), 1, "weight index out of range");
    n = s[idx];
  });
  return n;
}

int tts_vits_posterior_create(const TtsVitsPosteriorCfg* cfg, const float* const* host_weights, int device,
                              void** handle) {
  return guarded([&] {
    TTS_REQUIRE(cfg && host_weights && handle, 1, "NULL argument");
    *handle = nullptr;
    *handle = new tts::VitsPosterior(*cfg, host_weights, device);
  });
}

int tts_vits_posterior_destroy(void* handle) {
  return guarded([&] { delete static_cast<tts::VitsPosterior*>(handle); });
}

int tts_vits_posterior_forward(void* handle, const float* d_x, const float* d_mask, const float* d_g,
                               const float* d_eps, int B, int C, int T, float* d_z, float* d_m, float* d_logs,
                               void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(handle, 1, "NULL handle");
    static_cast<tts::VitsPosterior*>(handle)->forward(d_x, d_mask, d_g, d_eps, B, C, T, d_z, d_m, d_logs,
                                                      static_cast<hipStream_t>(hip_stream));
  });
}

int tts_vits_posterior_forward_profiled(void* handle, const float* d_x, const float* d_mask, const float* d_g,
                                        const float* d_eps, int B, int C, int T, float* d_z, float* d_m,
                                        float* d_logs, void* hip_stream, TtsLaunchRecord* records,
                                        int max_records, int* n_records) {
  return guarded([&] {
    TTS_REQUIRE(handle && n_records, 1, "NULL argument");
    auto* h = static_cast<tts::VitsPosterior*>(handle);
    auto s = static_cast<hipStream_t>(hip_stream);
    tts::Profiler prof;
    {
      tts::DeviceGuard g(h->device());
      h->forward(d_x, d_mask, d_g, d_eps, B, C, T, d_z, d_m, d_logs, s, &prof);
      TTS_HIP_CHECK(hipStreamSynchronize(s));
    }
    export_records(prof, records, max_records, n_records);
  });
}

// ----------------------------------------------------------------------------- single ops
static void op_conv1d_impl(const TtsConv1dDesc* d, const float* d_x, const float* h_w, const float* h_b,
                           const float* d_res, float* d_y, float* d_z, int tile, int reps, float* ms,
                           void* hip_stream) {
  TTS_REQUIRE(d && d_x && h_w && h_b, 1, "NULL argument");
  TTS_REQUIRE(d->B >= 1 && d->Cin >= 1 && d->Cout >= 1 && d->Tin >= 1 && d->K >= 1 && d->dil >= 1, 1,
              "bad conv1d shape");
  TTS_REQUIRE((d->K % 2) == 1, 3, "conv1d: only odd kernel sizes ('same' padding)");
  TTS_REQUIRE(d->zmode >= 0 && d->zmode <= 3, 1, "bad zmode");
  TTS_REQUIRE(d->zmode == 0 ? d_y != nullptr : d_z != nullptr, 1, "missing output pointer");
  const int mode = d->math_mode;
  TTS_REQUIRE(mode >= tts::MATH_FP32 && mode <= tts::MATH_LAST, 1, "unknown math_mode");
  if (tile < 0) tile = tts::conv_tile_for(mode, d->Cout, d->K, d->Cin, d->dil, d_res != nullptr);
  const tts::ConvTile t = tts::conv_tile(mode, tile);
  std::vector<float> packed(tts::packed_conv_numel(mode, d->Cout, d->Cin, d->K, t));
  const int w_exp = tts::pack_conv(mode, h_w, d->Cout, d->Cin, d->K, t, packed.data());
  std::vector<float> bias((size_t)tts::ceil_div(d->Cout, t.BM) * t.BM, 0.f);
  std::memcpy(bias.data(), h_b, sizeof(float) * d->Cout);
  TmpDev w(packed.data(), packed.size()), b(bias.data(), bias.size());
  tts::Conv1dArgs a{};
  a.x = d_x; a.w = w.p; a.bias = b.p; a.res = d_res; a.y = d_y; a.z = d_z; a.cvec = nullptr;
  a.Cin = d->Cin; a.Cout = d->Cout; a.Tin = d->Tin; a.Tout = d->Tin + 2 * d->rep_pad;
  a.dil = d->dil; a.pad = d->dil * (d->K - 1) / 2; a.rep_pad = d->rep_pad;
  a.n_chunks = tts::ceil_div(d->Cin, t.CK);
  a.in_slope = d->in_slope; a.out_slope = d->out_slope; a.zmode = d->zmode; a.zdiv = d->zdiv;
  a.w_exp = w_exp;
  auto s = static_cast<hipStream_t>(hip_stream);
  // fp16 hi/lo mode: the input's max-abs statistic (the executors get it from the producer)
  std::unique_ptr<TmpDev> slots;
  if (mode == tts::MATH_FP32_F16X3) {
    slots.reset(new TmpDev(nullptr, (size_t)d->B * 64));
    TTS_HIP_CHECK(hipMemsetAsync(slots->p, 0, (size_t)d->B * 64 * sizeof(float), s));
    tts::launch_amax(d_x, (int64_t)d->Cin * d->Tin, d->B, reinterpret_cast<unsigned*>(slots->p), s);
    a.amax_in = reinterpret_cast<const unsigned*>(slots->p);
  }
  if (reps <= 0) {
    tts::launch_conv(mode, a, d->B, d->K, tile, s);
  } else {
    tts::launch_conv(mode, a, d->B, d->K, tile, s);  // warm-up
    hipEvent_t e0, e1;
    TTS_HIP_CHECK(hipEventCreate(&e0));
    TTS_HIP_CHECK(hipEventCreate(&e1));
    TTS_HIP_CHECK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) tts::launch_conv(mode, a, d->B, d->K, tile, s);
    TTS_HIP_CHECK(hipEventRecord(e1, s));
    TTS_HIP_CHECK(hipEventSynchronize(e1));
    float total = 0.f;
    TTS_HIP_CHECK(hipEventElapsedTime(&total, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (ms) *ms = total / reps;
  }
  TTS_HIP_CHECK(hipStreamSynchronize(s));
}

int tts_op_conv1d(const TtsConv1dDesc* d, const float* d_x, const float* h_w, const float* h_b,
                  const float* d_res, float* d_y, float* d_z, void* hip_stream) {
  return guarded([&] { op_conv1d_impl(d, d_x, h_w, h_b, d_res, d_y, d_z, -1, 0, nullptr, hip_stream); });
}

int tts_op_conv1d_bench(const TtsConv1dDesc* d, const float* d_x, const float* h_w, const float* h_b,
                        const float* d_res, float* d_y, float* d_z, int tile, int reps, float* ms,
                        void* hip_stream) {
  return guarded([&] { op_conv1d_impl(d, d_x, h_w, h_b, d_res, d_y, d_z, tile, reps, ms, hip_stream); });
}

int tts_op_conv1d_num_tiles(int math_mode) {
  if (math_mode < tts::MATH_FP32 || math_mode > tts::MATH_LAST) {
    g_last_error = "unknown math_mode";
    return -TTS_ERR_INVALID;
  }
  return tts::conv_num_tiles(math_mode);
}

int tts_op_conv_transpose1d(const float* d_x, int B, int Cin, int Tin, const float* h_w,
                            const float* h_b, int Cout, int K, int stride, float in_slope,
                            int math_mode, float* d_y, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_x && h_w && h_b && d_y, 1, "NULL argument");
    TTS_REQUIRE(B >= 1 && Cin >= 1 && Cout >= 1 && Tin >= 1, 1, "bad conv_transpose1d shape");
    TTS_REQUIRE(K == 2 * stride, 3, "conv_transpose1d: requires kernel_size == 2*stride");
    TTS_REQUIRE(stride == 2 || stride == 4 || stride == 8, 3, "conv_transpose1d: stride must be 2, 4 or 8");
    TTS_REQUIRE(math_mode >= tts::MATH_FP32 && math_mode <= tts::MATH_LAST, 1, "unknown math_mode");
    auto s = static_cast<hipStream_t>(hip_stream);
    if (tts::is_split_mode(math_mode)) {
      const int tile = tts::conv_tile_for(math_mode, stride * Cout, 2, Cin, 1, false);
      const tts::ConvTile t = tts::conv_tile(math_mode, tile);
      std::vector<float> packed(tts::packed_conv_numel(math_mode, stride * Cout, Cin, 2, t));
      const int w_exp = tts::pack_convT_split(math_mode, h_w, Cin, Cout, stride, t, packed.data());
      std::vector<float> bias((size_t)tts::ceil_div(stride * Cout, t.BM) * t.BM, 0.f);
      for (int co = 0; co < Cout; ++co)
        for (int ph = 0; ph < stride; ++ph) bias[(size_t)co * stride + ph] = h_b[co];
      TmpDev w(packed.data(), packed.size()), b(bias.data(), bias.size());
      tts::Conv1dArgs a{};
      a.x = d_x; a.w = w.p; a.bias = b.p; a.y = d_y;
      a.Cin = Cin; a.Cout = stride * Cout; a.Tin = Tin; a.Tout = Tin + 1;
      a.dil = 1; a.pad = 1; a.n_chunks = tts::ceil_div(Cin, t.CK);
      a.in_slope = in_slope; a.out_slope = 1.f; a.zdiv = 1.f; a.w_exp = w_exp; a.ups = stride;
      std::unique_ptr<TmpDev> slots;
      if (math_mode == tts::MATH_FP32_F16X3) {
        slots.reset(new TmpDev(nullptr, (size_t)B * 64));
        TTS_HIP_CHECK(hipMemsetAsync(slots->p, 0, (size_t)B * 64 * sizeof(float), s));
        tts::launch_amax(d_x, (int64_t)Cin * Tin, B, reinterpret_cast<unsigned*>(slots->p), s);
        a.amax_in = reinterpret_cast<const unsigned*>(slots->p);
      }
      tts::launch_conv(math_mode, a, B, 2, tile, s);
      TTS_HIP_CHECK(hipStreamSynchronize(s));
      return;
    }
    const int tile = tts::convT_tile_for(Cout, stride);
    const tts::ConvTile t = tts::convT_tile(tile, stride);
    std::vector<float> packed(tts::packed_convT_numel(Cin, Cout, stride, t));
    tts::pack_convT(h_w, Cin, Cout, stride, t, packed.data());
    std::vector<float> bias((size_t)tts::ceil_div(Cout, t.BM) * t.BM, 0.f);
    std::memcpy(bias.data(), h_b, sizeof(float) * Cout);
    TmpDev w(packed.data(), packed.size()), b(bias.data(), bias.size());
    tts::ConvTArgs a{};
    a.x = d_x; a.w = w.p; a.bias = b.p; a.y = d_y;
    a.Cin = Cin; a.Cout = Cout; a.Tin = Tin; a.n_chunks = tts::ceil_div(Cin, t.CK); a.in_slope = in_slope;
    tts::launch_convT(a, B, stride, tile, s);
    TTS_HIP_CHECK(hipStreamSynchronize(s));
  });
}

int tts_op_conv_post(const float* d_z, int B, int Cin, int T, const float* h_w, const float* h_b,
                     float in_slope, float* d_y, void* hip_stream) {
  return guarded([&] {
    TTS_REQUIRE(d_z && h_w && d_y, 1, "NULL argument");
    TTS_REQUIRE(B >= 1 && Cin >= 1 && T >= 1, 1, "bad conv_post shape");
    TmpDev w(h_w, (size_t)Cin * 7);
    tts::PostArgs a{};
    a.z = d_z; a.w = w.p; a.bias = h_b ? h_b[0] : 0.f; a.y = d_y; a.Cin = Cin; a.T = T; a.in_slope = in_slope;
    auto s = static_cast<hipStream_t>(hip_stream);
    tts::launch_conv_post(a, B, s);
    TTS_HIP_CHECK(hipStreamSynchronize(s));
  });
}

}  // extern "C"
