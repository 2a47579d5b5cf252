// TTS -> vocoder hand-off (mel renormalisation + resampling) and the int16 wav writer
// (kernels_handoff.hip).  Reference: TTS/utils/synthesizer.py:412-428,
// TTS/utils/audio/processor.py:259-336, TTS/utils/audio/numpy_transforms.py:430-447.
#pragma once

#include <algorithm>

#include "common.hpp"
#include "tts_mi355x.h"

namespace tts {

// AudioProcessor normalisation parameters with the Python scalars pre-rounded to fp32.
struct AudioNormDev {
  int signal_norm, symmetric_norm, clip_norm;
  float max_norm, two_max_norm, min_level_db, neg_min_level_db, ref_level_db;
  const double* mean;   // mel_scaler.mean_ [C] (device) or NULL: range normalisation
  const double* scale;  // mel_scaler.scale_ [C]
};

struct HandoffArgs {
  const float* in;  // [B][T][C] (time_major) or [B][C][T]
  float* out;       // [B][C][T_out]
  int T, C, T_out, time_major;
  float src_scale;  // > 0: source step per output step (1 / scale_factor); else T / T_out
  AudioNormDev de, no;
};

void launch_handoff(const HandoffArgs& a, int B, hipStream_t s);
void launch_wav_int16(const float* wav, int B, int64_t n, const int64_t* len, unsigned* amax, int16_t* out,
                      hipStream_t s);

}  // namespace tts
