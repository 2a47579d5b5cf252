// conv1d_split_kernel instances of one scheme (SchemeB1); see split_kernel.hpp.
#include "split_kernel.hpp"

namespace tts {

void launch_split_b1(const Conv1dArgs& a, int B, int K, int tile, hipStream_t s) {
  split_detail::launch_split_s<SchemeB1>(a, B, K, tile, s);
}

}  // namespace tts
