// Device-side pieces shared by the conv kernels (fp32 MFMA and bf16x6 split variants).
#pragma once

#include "common.hpp"

namespace tts {

// LDS float offset of channel quad q (0/1) of input row r in group g.  The quad index is
// XOR-swizzled with bit 3 of the row: every ds_read_b128 lane group (16 lanes, rows
// r0 + {0-3,12-15,20-27} or {4-11,16-19,28-31}) then hits 16 distinct 16-byte bank slots
// for ANY row shift r0 (the tap offset k*dil), with no padding.
__device__ __forceinline__ int xlds_off(int g, int r, int q, int xrows) {
  return (g * xrows + r) * 8 + 4 * (q ^ ((r >> 3) & 1));
}

// Conv1d epilogue on a TM x TN grid of 32x32 accumulators (v_mfma_f32_32x32x*):
// lane holds column (lane&31) and rows (r&3) + 8*(r>>2) + 4*(lane>>5) of each block.
//   v = act_out(acc + bias[co] [+ cvec[b][co]]) [* mask[b][t]] [+ res]
//   zmode 0: y = v;  1: z = v;  2: z += v;  3: z = (z + v) / zdiv   (HiFiGAN MRF sum, :255-261)
// `res` may alias `y` (the resblock residual is updated in place) and z is read-modify-write,
// so every value this thread reads is loaded BEFORE its first store: otherwise the compiler
// cannot hoist a load above the previous element's store and each element pays a full memory
// round trip (measured: residual convs 2x slower).
template <int TM, int TN>
__device__ __forceinline__ void conv_epilogue(const Conv1dArgs& args, const f32x16 (&acc)[TM][TN], int b,
                                              int tbase, int cobase, int lane) {
  // copy the argument block: a store through `out` could alias it in the compiler's view
  const Conv1dArgs a = args;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int Cout = a.Cout;
  const int Tout = a.Tout;
  const int zmode = a.zmode;
  const float* __restrict__ bias = a.bias;
  const float* cvec = a.cvec;
  const float* mask = a.mask;
  const float* res = a.res;
  const float* zin = (zmode >= 2) ? a.z : nullptr;
  float* out = (zmode == 0) ? a.y : a.z;

  // per-batch bases (wave-uniform) + 32-bit in-item offsets: one VGPR per gathered address
  const size_t item = (size_t)b * Cout * Tout;
  const float* rb = res ? res + item : nullptr;
  const float* zb = zin ? zin + item : nullptr;
  float* ob = out + item;
  const float* cb = cvec ? cvec + (size_t)b * Cout : nullptr;
  const float* mb = mask ? mask + (size_t)b * Tout : nullptr;
  // per 32x32 block: gather every value this thread reads, then compute and store
  // (TM*TN memory round trips per thread)
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = cobase + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
      const int cc = co < Cout ? co : 0;
      float v = bias[cc];
      if (cb) v += cb[cc];
      bv[r] = v;
    }
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int t = tbase + n * 32 + l32;
      const float mv = mb ? mb[t < Tout ? t : 0] : 1.f;
      float rv[16], zv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = cobase + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        const bool ok = co < Cout && t < Tout;
        const int off = ok ? co * Tout + t : 0;
        rv[r] = rb ? rb[off] : 0.f;
        zv[r] = zb ? zb[off] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = cobase + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (co < Cout && t < Tout) {
          float v = acc[m][n][r] + bv[r];
          if (mb) v *= mv;
          v = lrelu(v, a.out_slope);
          if (rb) v += rv[r];
          if (zmode == 2) v = zv[r] + v;
          else if (zmode == 3) v = (zv[r] + v) / a.zdiv;
          ob[co * Tout + t] = v;
        }
      }
    }
  }
}

}  // namespace tts
