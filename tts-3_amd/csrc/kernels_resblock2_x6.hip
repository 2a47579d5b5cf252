// Whole-ResBlock2 kernels (resblock_block.hpp) for the SchemeX6 split scheme: one compile unit per
// scheme keeps the build parallel.
#include "resblock_block.hpp"

namespace tts {
void launch_resblock2_x6(const ResBlock3Args& a, int B, int C, int K, int geo64, hipStream_t s) {
  launch_rb2_s<SchemeX6>(a, B, C, K, geo64, s);
}
}  // namespace tts
