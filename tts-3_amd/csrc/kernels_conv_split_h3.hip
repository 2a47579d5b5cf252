// conv1d_split_kernel instances of one scheme (SchemeH3); see split_kernel.hpp.
#include "split_kernel.hpp"

namespace tts {

void launch_split_h3(const Conv1dArgs& a, int B, int K, int tile, hipStream_t s) {
  split_detail::launch_split_s<SchemeH3>(a, B, K, tile, s);
}

}  // namespace tts
