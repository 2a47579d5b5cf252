// Winograd F(4,4) constants shared by the device kernels (wino_kernel.hpp) and the host weight
// transform (pack.cpp): plain constexprs, no device code, so the host packers build on their own
// (tts-3_amd/Makefile asan-check).
#pragma once

namespace tts {

constexpr int kWinoPoints = 7;
constexpr int wino_chunks(int K) { return (K + 3) / 4; }
// G[p][k] = gc[p] * ga[p]^k (k = 0..3); p = 6 (inf) only has k = 3.
constexpr double kWinoGc[7] = {0.25, 1.0 / 6, 1.0 / 18, 1.0 / 72, 1.0 / 120, 32.0 / 45, 0.5};
constexpr double kWinoGa[7] = {0.0, 1.0, -1.0, 2.0, -2.0, 0.5, 0.0};
constexpr int kWinoBtShift = 5;  // max row sum of |BT| = 30 < 2^5: scale the input by 2^-(e+5)

}  // namespace tts
