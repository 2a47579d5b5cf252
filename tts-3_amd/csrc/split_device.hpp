// Split-precision operand schemes shared by the split conv kernels (kernels_conv_split.hip,
// kernels_resblock.hip): how an fp32 operand becomes 16-bit MFMA pieces, which piece products
// are accumulated, and the f16x3 input scale from a producer's max-abs statistics.
#pragma once

#include "conv_device.hpp"

namespace tts {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned short bf16_bits(__bf16 h) { return __builtin_bit_cast(unsigned short, h); }
__device__ __forceinline__ unsigned short f16_bits(_Float16 h) { return __builtin_bit_cast(unsigned short, h); }

struct SchemeX6 {
  static constexpr int NP = 3;        // pieces per operand
  static constexpr int ROWB = 112;    // LDS bytes per staged row (3 x 32 B + 16 B pad)
  static constexpr int NACC = 1;      // accumulators per output block
  static constexpr int NPROD = 6;     // products per step, smallest first
  static constexpr int PA[6] = {2, 1, 0, 1, 0, 0};
  static constexpr int PB[6] = {0, 1, 2, 0, 1, 0};
  static constexpr int PACC[6] = {0, 0, 0, 0, 0, 0};
  static constexpr bool SCALED = false;
  // x = p0 + p1 + p2 exactly (round-to-nearest-even at every piece)
  __device__ static __forceinline__ void split(float x, unsigned short (&p)[3]) {
    const __bf16 a0 = (__bf16)x;
    const float r1 = x - (float)a0;
    const __bf16 a1 = (__bf16)r1;
    const float r2 = r1 - (float)a1;
    p[0] = bf16_bits(a0);
    p[1] = bf16_bits(a1);
    p[2] = bf16_bits((__bf16)r2);
  }
  __device__ static __forceinline__ void split2(float x0, float x1, unsigned (&w)[3]) {
    unsigned short a[3], b[3];
    split(x0, a);
    split(x1, b);
#pragma unroll
    for (int p = 0; p < 3; ++p) w[p] = (unsigned)a[p] | ((unsigned)b[p] << 16);
  }
  __device__ static __forceinline__ f32x16 mfma(f32x4 a, f32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};

struct SchemeH3 {
  static constexpr int NP = 2;
  static constexpr int ROWB = 80;     // 2 x 32 B + 16 B pad
  static constexpr int NACC = 1;
  static constexpr int NPROD = 3;     // lo*hi, hi*lo, hi*hi
  static constexpr int PA[3] = {1, 0, 0};
  static constexpr int PB[3] = {0, 1, 0};
  static constexpr int PACC[3] = {0, 0, 0};
  static constexpr bool SCALED = true;
  // x (already scaled into [0, 2^14]) = hi + lo to 22 bits
  __device__ static __forceinline__ void split(float x, unsigned short (&p)[2]) {
    const _Float16 h = (_Float16)x;
    p[0] = f16_bits(h);
    p[1] = f16_bits((_Float16)(x - (float)h));
  }
  // two values -> (hi pair, lo pair) words, the same bits as split(): hi = v_cvt_pk_f16_f32 (round
  // to nearest even); the remainders x - hi are exact in fp32 and v_fma_mix_f32 forms them straight
  // from the packed fp16 halves (-hi * 1 + x, one rounding of an exact value), so a pair costs 4
  // VALU instead of 6 (two v_cvt_f32_f16 + two v_sub_f32)
  __device__ static __forceinline__ void split2(float x0, float x1, unsigned (&w)[2]) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 h = __builtin_convertvector((f2){x0, x1}, h2);
    const unsigned hb = __builtin_bit_cast(unsigned, h);
    float r0, r1;
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r0) : "v"(hb), "v"(x0));
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r1) : "v"(hb), "v"(x1));
    w[0] = hb;
    w[1] = __builtin_bit_cast(unsigned, __builtin_convertvector((f2){r0, r1}, h2));
  }
  __device__ static __forceinline__ f32x16 mfma(f32x4 a, f32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

// Plain bf16 (MATH_BF16): one bf16 piece per operand, one product, fp32 accumulation.
struct SchemeB1 {
  static constexpr int NP = 1;
  static constexpr int ROWB = 48;     // 32 B + 16 B pad (conflict-free like the other pitches)
  static constexpr int NACC = 1;
  static constexpr int NPROD = 1;
  static constexpr int PA[1] = {0};
  static constexpr int PB[1] = {0};
  static constexpr int PACC[1] = {0};
  static constexpr bool SCALED = false;
  __device__ static __forceinline__ void split(float x, unsigned short (&p)[1]) { p[0] = bf16_bits((__bf16)x); }
  __device__ static __forceinline__ void split2(float x0, float x1, unsigned (&w)[1]) {
    w[0] = (unsigned)bf16_bits((__bf16)x0) | ((unsigned)bf16_bits((__bf16)x1) << 16);
  }
  __device__ static __forceinline__ f32x16 mfma(f32x4 a, f32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};

// 4 consecutive channels of one staged row -> the pieces' 8-byte slots (dst + 32 p)
template <class S>
__device__ __forceinline__ void split_store4(unsigned char* dst, float v0, float v1, float v2, float v3) {
  unsigned w0[S::NP], w1[S::NP];
  S::split2(v0, v1, w0);
  S::split2(v2, v3, w1);
#pragma unroll
  for (int p = 0; p < S::NP; ++p) *reinterpret_cast<u32x2*>(dst + 32 * p) = u32x2{w0[p], w1[p]};
}

// Accumulator registers r0 .. r0 + 7 of one lane (8 channels of one 16-channel group, positions
// 8 half .. + 7 in quad_pos order) -> split pieces, one 16-byte store per piece at dst + 32 p
// (dst: the lane's row, + 16 half).  8 consecutive lanes' rows cover the 32 banks (row pitch
// ROWB / 4 = 4 x odd dwords): conflict-free.
template <class S, class V>
__device__ __forceinline__ void store_xt8(unsigned char* dst, const V& acc, int r0, float scale) {
  unsigned w[4][S::NP];
#pragma unroll
  for (int k = 0; k < 4; ++k) S::split2(acc[r0 + 2 * k] * scale, acc[r0 + 2 * k + 1] * scale, w[k]);
#pragma unroll
  for (int p = 0; p < S::NP; ++p)
    *reinterpret_cast<u32x4_t*>(dst + 32 * p) = u32x4_t{w[0][p], w[1][p], w[2][p], w[3][p]};
}

// Exponent e such that max|x| * 2^-e lies in [2^13, 2^14): read the 64 max-abs slots the
// producer published (one per lane), wave max, frexp.  No statistics, zero or non-finite max:
// e = 0 (an overflowing input then yields inf, as fp16 would; NaN propagates).
__device__ __forceinline__ int amax_exp(const unsigned* slots, int b) {
  if (!slots) return 0;
  float m = __uint_as_float(slots[(size_t)b * 64 + (threadIdx.x & 63)]);
  m = wave_max(m);
  int e = 0;
  if (m > 0.f && m < INFINITY) {
    int E;
    (void)frexpf(m, &E);
    e = E - 14;
  }
  return __builtin_amdgcn_readfirstlane(e);
}

}  // namespace tts
