// Device-side pieces shared by the conv kernels (fp32 MFMA and bf16x6 split variants).
#pragma once

#include "common.hpp"

namespace tts {

// ---- raw buffer access (CDNA buffer resource descriptors) -------------------------------
// A 128-bit descriptor in SGPRs + a 32-bit per-lane byte offset + a wave-uniform soffset: no
// 64-bit address arithmetic per access, and the hardware range check returns 0 for loads /
// drops stores whose offset is >= num_records.  OOB_OFF marks a lane's access invalid (callers
// keep voffset + soffset < 2^32, i.e. every addressed plane < 2 GiB; checked on the host).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned OOB_OFF = 0x80000000u;

#ifndef ACT_ABLATE
#define ACT_ABLATE 0  // timing ablation only (wrong results): every activation-plane descriptor (a range
                      // other than the weights' 0xFFFFFFFF) is cut to its first 64 KiB, so plane loads
                      // past it return 0 and stores are dropped without touching memory
#endif
__device__ __forceinline__ unsigned act_range(unsigned bytes) {
  return (ACT_ABLATE && bytes != 0xFFFFFFFFu && bytes > 65536u) ? 65536u : bytes;
}
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)act_range(bytes), 0x00020000);
}
__device__ __forceinline__ float bload(rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
}
__device__ __forceinline__ f32x4 bload4(rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}
// cache policy of the activation-plane stores (A/B knob; gfx950 buffer CPol bits: 1 sc0, 2 nt, 16
// sc1): 0 keeps the written lines in the XCD's L2 (default), sc1 / nt stream them past it
#ifndef TTS_ST_POL
#define TTS_ST_POL 0
#endif
// cache policy of activation-window loads (A/B knob, same CPol bits): 2 (nt) streams them through
// the L2 with evict-first, so they do not displace the weights every workgroup re-reads
#ifndef TTS_LDX_POL
#define TTS_LDX_POL 0
#endif
template <int POL = TTS_LDX_POL>
__device__ __forceinline__ float bload_x(rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, POL));
}
__device__ __forceinline__ void bstore(rsrc_t r, float v, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)voff, (int)soff, TTS_ST_POL);
}
// Activation planes in HBM (Conv1dArgs::planes): fp32, or bf16 in the MATH_BF16 scheme (the MFMA
// operands are bf16 there anyway; the plane then costs 2 B per element instead of 4).  ES: bytes
// per element; ld / st take byte offsets like bload / bstore.  A bf16 store rounds to nearest even
// (v_cvt_pk_bf16_f32), a load widens exactly.
__device__ __forceinline__ unsigned short f32_to_bf16_bits(float v) {
  return __builtin_bit_cast(unsigned short, (__bf16)v);
}
__device__ __forceinline__ float bf16_bits_to_f32(unsigned b) { return __builtin_bit_cast(float, b << 16); }
__device__ __forceinline__ float bf16_round(float v) { return bf16_bits_to_f32(f32_to_bf16_bits(v)); }
template <bool B16>
struct PlaneT {
  static constexpr unsigned ES = 4u;
  __device__ static __forceinline__ float ld(rsrc_t r, unsigned voff, unsigned soff) { return bload(r, voff, soff); }
  __device__ static __forceinline__ void st(rsrc_t r, float v, unsigned voff, unsigned soff) { bstore(r, v, voff, soff); }
  // the value a store followed by a load gives back
  __device__ static __forceinline__ float rt(float v) { return v; }
};
template <>
struct PlaneT<true> {
  static constexpr unsigned ES = 2u;
  __device__ static __forceinline__ float ld(rsrc_t r, unsigned voff, unsigned soff) {
    return bf16_bits_to_f32((unsigned)__builtin_amdgcn_raw_buffer_load_b16(r, (int)voff, (int)soff, 0));
  }
  __device__ static __forceinline__ void st(rsrc_t r, float v, unsigned voff, unsigned soff) {
    __builtin_amdgcn_raw_buffer_store_b16(f32_to_bf16_bits(v), r, (int)voff, (int)soff, TTS_ST_POL);
  }
  __device__ static __forceinline__ float rt(float v) { return bf16_round(v); }
};
// element e of a plane based at p (float* in the argument blocks, bf16 when B16)
template <bool B16>
__device__ __forceinline__ const void* plane_at(const float* p, size_t e) {
  return reinterpret_cast<const char*>(p) + e * PlaneT<B16>::ES;
}
// 4 consecutive elements at byte offset voff (8-byte aligned for bf16, 16 for fp32)
template <bool B16>
__device__ __forceinline__ f32x4 pload4(rsrc_t r, unsigned voff, unsigned soff) {
  if constexpr (B16) {
    const u32x2_t w = __builtin_bit_cast(u32x2_t, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0));
    return f32x4{bf16_bits_to_f32(w[0] & 0xffffu), bf16_bits_to_f32(w[0] >> 16), bf16_bits_to_f32(w[1] & 0xffffu),
                 bf16_bits_to_f32(w[1] >> 16)};
  } else {
    return bload4(r, voff, soff);
  }
}
template <bool B16>
__device__ __forceinline__ void pstore4(rsrc_t r, f32x4 v, unsigned voff, unsigned soff) {
  if constexpr (B16) {
    const u32x2_t w = {(unsigned)f32_to_bf16_bits(v[0]) | ((unsigned)f32_to_bf16_bits(v[1]) << 16),
                       (unsigned)f32_to_bf16_bits(v[2]) | ((unsigned)f32_to_bf16_bits(v[3]) << 16)};
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, w), r, (int)voff, (int)soff, TTS_ST_POL);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, (int)voff, (int)soff, TTS_ST_POL);
  }
}

// LDS-DMA of 16 bytes per lane (buffer_load_dwordx4 ... lds: lane l's bytes land at lds + 16 l),
// issued from inline asm.  With the builtin, the compiler's waitcnt pass makes every later LDS
// access of the issuing wave wait (vmcnt) until the DMA has landed, whatever buffer it touches, so
// the wave stalls for an HBM round trip right after each DMA; the callers order the DMA'd data
// themselves (explicit s_waitcnt vmcnt + barrier before any wave reads it).  Extra vector-memory
// operations the compiler does not see only make its own vmcnt waits stricter (in-order counter).
// M0 is reserved: the compiler sets it before each of its own uses, so clobbering it here is safe.
__device__ __forceinline__ void lds_dma_b128(const void* base, unsigned bytes, unsigned voff, const void* lds) {
  const unsigned long long p = reinterpret_cast<unsigned long long>(base);
  // every operand is wave-uniform; readfirstlane puts them in SGPRs (the "s" constraint alone does not)
  const u32x4_t d = {(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)p),
                     (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)(p >> 32) & 0xffffu)),
                     (unsigned)__builtin_amdgcn_readfirstlane((int)act_range(bytes)), 0x00020000u};
  const unsigned m =
      (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(unsigned long)(__attribute__((address_space(3))) const void*)lds);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(d), "s"(m)
               : "memory", "m0");
#pragma clang diagnostic pop
}

// L2 prefetch of one 4-byte element per lane through the LDS-DMA path: the line lands in L2 on
// its way to a scratch LDS area (256 bytes at lds), and no VGPR is written, so nothing has to stay
// live until the load returns.  Later vmcnt waits of the issuing wave count it (in order).
__device__ __forceinline__ void l2_touch_dma(const void* base, unsigned bytes, unsigned voff, const void* lds) {
  const unsigned long long p = reinterpret_cast<unsigned long long>(base);
  const u32x4_t d = {(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)p),
                     (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)(p >> 32) & 0xffffu)),
                     (unsigned)__builtin_amdgcn_readfirstlane((int)act_range(bytes)), 0x00020000u};
  const unsigned m =
      (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(unsigned long)(__attribute__((address_space(3))) const void*)lds);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds" ::"v"(voff), "s"(d), "s"(m)
               : "memory", "m0");
#pragma clang diagnostic pop
}

// leaky_relu for 0 < slope <= 1 (slope 1 = identity): max(x, slope*x), 2 VALU
__device__ __forceinline__ float lrelu2(float x, float slope) { return fmaxf(x, x * slope); }
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// LDS float offset of channel quad q (0/1) of input row r in group g.  The quad index is
// XOR-swizzled with bit 3 of the row: every ds_read_b128 lane group (16 lanes, rows
// r0 + {0-3,12-15,20-27} or {4-11,16-19,28-31}) then hits 16 distinct 16-byte bank slots
// for ANY row shift r0 (the tap offset k*dil), with no padding.
__device__ __forceinline__ int xlds_off(int g, int r, int q, int xrows) {
  return (g * xrows + r) * 8 + 4 * (q ^ ((r >> 3) & 1));
}

// Max over the 64 lanes of a wave, returned wave-uniform (called with every lane active): DPP
// row operations (quad swaps, half-row / row mirrors, row broadcasts 15 and 31), a few cycles each,
// instead of six dependent ds_bpermute round trips.  fmaxf drops NaN like the shuffle form did.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_max_step(float v) {
  const int o = __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v), CTRL, ROWS, 0xF, false);
  return fmaxf(v, __builtin_bit_cast(float, o));
}
__device__ __forceinline__ float wave_max(float v) {
  v = dpp_max_step<0xB1, 0xF>(v);   // quad_perm [1, 0, 3, 2]
  v = dpp_max_step<0x4E, 0xF>(v);   // quad_perm [2, 3, 0, 1]
  v = dpp_max_step<0x141, 0xF>(v);  // row_half_mirror: 8-lane halves
  v = dpp_max_step<0x140, 0xF>(v);  // row_mirror: rows of 16
  v = dpp_max_step<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
  v = dpp_max_step<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3: lane 63 holds the max
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// Conv1d epilogue on a TM x TN grid of 32x32 accumulators (v_mfma_f32_32x32x*):
// lane holds column (lane&31) and rows (r&3) + 8*(r>>2) + 4*(lane>>5) of each block.
//   v = act_out(acc + bias[co] [+ cvec[b][co]]) [* mask[b][t]] [+ res]
//   zmode 0: y = v;  1: z = v;  2: z += v;  3: z = (z + v) / zdiv   (HiFiGAN MRF sum, :255-261)
// `res` may alias `y` (the resblock residual is updated in place) and z is read-modify-write,
// so every value this thread reads is loaded BEFORE its first store: otherwise the compiler
// cannot hoist a load above the previous element's store and each element pays a full memory
// round trip (measured: residual convs 2x slower).
// Max-abs statistics for the fp16 hi/lo consumers: 64 slots per batch item (slots[b][64]); a
// wave's max goes to slot blockIdx.x & 63 of its item (fp32 bits order like unsigned integers
// for non-negative values).  Per item, so an utterance's scaling never depends on its batch.
__device__ __forceinline__ void publish_amax(unsigned* slots, int b, float v) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) atomicMax(slots + (size_t)b * 64 + (blockIdx.x & 63), __float_as_uint(v));
}

// Workgroup form for the grid-stride elementwise kernels (256 threads, called by every thread):
// one atomic per workgroup instead of one per wave; thousands of per-wave atomics on an item's
// two slot cache lines serialise in L2 and doubled the Glow gate / update kernels' time.
__device__ __forceinline__ void publish_amax_block(unsigned* slots, int b, float v) {
  __shared__ float red[4];
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(slots + (size_t)b * 64 + (blockIdx.x & 63),
              __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// sbias: bias + cvec of rows sbase.. already staged in LDS by the caller (rows >= Cout hold 0,
// the same sums the two range-checked loads give), else nullptr
template <int TM, int TN, bool RES, int ZM, bool AMAX, bool YB = false>
__device__ __forceinline__ void conv_epilogue_impl(const Conv1dArgs& a, const f32x16 (&acc)[TM][TN], int b,
                                                   int tbase, int cobase, int lane, int tend,
                                                   const float* sbias, int sbase) {
  using PY = PlaneT<YB>;  // res / z / y element type
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int Cout = a.Cout;
  const int Tout = a.Tout;
  const unsigned plane = (unsigned)Cout * (unsigned)Tout * PY::ES;  // bytes of one batch item
  const size_t item = (size_t)b * (a.o_bstride ? a.o_bstride : (int64_t)Cout * Tout);
  const rsrc_t rres = make_rsrc(RES ? plane_at<YB>(a.res, item) : a.bias, RES ? plane : 0u);
  const rsrc_t rz = make_rsrc(ZM >= 2 ? plane_at<YB>(a.z, item) : a.bias, ZM >= 2 ? plane : 0u);
  const rsrc_t rout = make_rsrc(plane_at<YB>(a.zmode == 0 ? a.y : a.z, item), plane);
  const rsrc_t rcv = make_rsrc(a.cvec ? a.cvec + (size_t)b * (a.cvec_bstride ? a.cvec_bstride : (int64_t)Cout) : a.bias,
                               a.cvec ? (unsigned)Cout * 4u : 0u);
  const rsrc_t rmask = make_rsrc(a.mask ? a.mask + (size_t)b * Tout : a.bias, a.mask ? (unsigned)Tout * 4u : 0u);
  const rsrc_t rbias = make_rsrc(a.bias, (unsigned)Cout * 4u);
  const bool has_mask = a.mask != nullptr;
  const bool mask_res = RES && a.mask_res && has_mask;
  const float oslope = a.out_slope;
  const float zdiv = a.zdiv;
  const unsigned rowb = (unsigned)Tout * PY::ES;
  float vmax = 0.f;  // AMAX: max |stored value|
  // per 32x32 block: gather every value this thread reads, then compute and store.  Every
  // range-checked offset is in the per-lane voffset (lane row cobase + m*32 + 4*half, column t;
  // register r adds row (r&3) + 8*(r>>2)); an absent cvec reads 0 through a 0-byte descriptor.
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned co = (unsigned)(cobase + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half);
      bv[r] = sbias ? sbias[(int)co - sbase] : bload(rbias, co * 4u, 0u) + bload(rcv, co * 4u, 0u);
    }
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int t = tbase + n * 32 + l32;
      const int row0 = cobase + m * 32 + 4 * half;
      // rows >= Cout land past the plane through the row term; columns >= min(Tout, tend) are
      // marked OOB
      const bool tok = t < Tout && t < tend;
      const unsigned voff = tok ? ((unsigned)row0 * (unsigned)Tout + (unsigned)t) * PY::ES : OOB_OFF;
      const float mv = has_mask ? bload(rmask, (tok ? (unsigned)t * 4u : OOB_OFF), 0u) : 1.f;
      const float mv2 = mask_res ? mv : 1.f;  // (res + v) * mask for the VITS coupling update
      unsigned vo[16];
      float rv[16], zv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        vo[r] = voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb;
        if (RES) rv[r] = PY::ld(rres, vo[r], 0u);
        if (ZM >= 2) zv[r] = PY::ld(rz, vo[r], 0u);
      }
      float vm = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = (acc[m][n][r] + bv[r]) * mv;  // mv = 1 without a mask (exact)
        v = lrelu2(v, oslope);
        if (RES) v = (v + rv[r]) * mv2;  // mv2 = 1 unless mask_res (exact)
        if (ZM == 2) v = zv[r] + v;
        if (ZM == 3) v = (zv[r] + v) / zdiv;
        if (AMAX) vm = fmaxf(vm, fabsf(v));  // rows >= Cout hold exact zeros
        PY::st(rout, v, vo[r], 0u);
      }
      if (AMAX && tok) vmax = fmaxf(vmax, vm);
    }
  }
  if (AMAX && a.amax_out) publish_amax(a.amax_out, b, vmax);
}

// WaveNet residual / skip update epilogue (Conv1dArgs::wn_rows, wavenet.py:109-113): the same fp32
// operations as glow_wn_update_kernel on the conv output v = acc + bias: h = (h + v) * mask for
// rows < H, skip = v or skip + v for rows >= H.  H % 32 == 0, so a 32-row block is one side.
template <int TM, int TN, bool AMAX>
__device__ __forceinline__ void conv_epilogue_wn(const Conv1dArgs& args, const f32x16 (&acc)[TM][TN], int b,
                                                 int tbase, int cobase, int lane, const float* sbias, int sbase) {
  const Conv1dArgs a = args;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int H = a.wn_rows;
  const int T = a.Tout;
  const size_t item = (size_t)b * H * T;
  const unsigned plane = (unsigned)H * (unsigned)T * 4u;
  const rsrc_t rh = make_rsrc(a.y + item, plane);
  const rsrc_t rsk = make_rsrc(a.z + item, plane);
  const rsrc_t rmask = make_rsrc(a.mask + (size_t)b * T, (unsigned)T * 4u);
  const rsrc_t rbias = make_rsrc(a.bias, (unsigned)(2 * H) * 4u);
  const bool first = a.zmode == 1;
  const unsigned rowb = (unsigned)T * 4u;
  float vmax = 0.f;
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    const int rb0 = cobase + m * 32;  // first row of this 32-row block (wave-uniform)
    if (rb0 >= 2 * H) continue;
    const bool hrow = rb0 < H;
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned co = (unsigned)(rb0 + (r & 3) + 8 * (r >> 2) + 4 * half);
      bv[r] = sbias ? sbias[(int)co - sbase] : bload(rbias, co * 4u, 0u);
    }
    const rsrc_t rdst = hrow ? rh : rsk;
    const int prow0 = (hrow ? rb0 : rb0 - H) + 4 * half;  // row in the destination plane
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int t = tbase + n * 32 + l32;
      const bool tok = t < T;
      const unsigned voff = tok ? ((unsigned)prow0 * (unsigned)T + (unsigned)t) * 4u : OOB_OFF;
      const float mv = bload(rmask, tok ? (unsigned)t * 4u : OOB_OFF, 0u);
      float ov[16];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ov[r] = (hrow || !first) ? bload(rdst, voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb, 0u) : 0.f;
      float vm = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[m][n][r] + bv[r];
        float o;
        if (hrow) {
          o = (ov[r] + v) * mv;
          vm = fmaxf(vm, fabsf(o));
        } else {
          o = first ? v : ov[r] + v;
        }
        bstore(rdst, o, voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb, 0u);
      }
      if (AMAX && tok) vmax = fmaxf(vmax, vm);
    }
  }
  if (AMAX && a.amax_out) publish_amax(a.amax_out, b, vmax);
}

// Polyphase ConvTranspose1d epilogue (Conv1dArgs::ups = U): row rho = co*U + s, column frame m
// -> y[b][co][U*m + s - U/2].  For U = 8 a lane's registers r = 4i..4i+3 hold the phases
// 4*half .. 4*half+3 of one channel, i.e. 4 consecutive samples.
// sb / scv: bias and cvec of rows sbase.. staged in LDS by the caller (or nullptr)
template <int TM, int TN, bool AMAX, bool YB = false>
__device__ __forceinline__ void convT_epilogue(const Conv1dArgs& a, const f32x16 (&acc)[TM][TN], int b, int tbase,
                                               int cobase, int lane, const float* sb = nullptr,
                                               const float* scv = nullptr, int sbase = 0) {
  using PY = PlaneT<YB>;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int U = a.ups;
  const int lgU = __builtin_ctz(U);
  const int Cr = a.Cout >> lgU;   // channels
  const int Tin = a.Tin;
  const int To = Tin << lgU;      // output samples
  const unsigned plane = (unsigned)Cr * (unsigned)To * PY::ES;
  const rsrc_t rout = make_rsrc(plane_at<YB>(a.y, (size_t)b * Cr * To), plane);
  const rsrc_t rbias = make_rsrc(a.bias, (unsigned)a.Cout * 4u);
  // cvec: 0 records when absent, so every read returns 0 and (acc + bias) + 0 is exact
  const rsrc_t rcv = make_rsrc(a.cvec ? a.cvec + (size_t)b * Cr : a.bias, a.cvec ? (unsigned)Cr * 4u : 0u);
  float vmax = 0.f;
#pragma unroll
  for (int m = 0; m < TM; ++m) {
    float bv[16], cv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned rho = (unsigned)(cobase + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half);
      bv[r] = sb ? sb[(int)rho - sbase] : bload(rbias, rho * 4u, 0u);
      cv[r] = sb ? scv[(int)rho - sbase] : bload(rcv, (rho >> lgU) * 4u, 0u);
    }
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const int mm = tbase + n * 32 + l32;
      if (U == 8) {
        // registers 4i..4i+3 are phases 4*half .. 4*half+3 of channel co: samples t0 .. t0+3 with
        // t0 = 8*mm + 4*half - 4 (16-B aligned, wholly inside or outside [0, To)): one dwordx4
        // store each, and a wave's 64 lanes write 1 KiB of one row contiguously
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rho = cobase + m * 32 + 8 * i + 4 * half;
          const int co = rho >> 3;
          const int t0 = (mm << 3) + 4 * half - 4;
          const unsigned off = (t0 >= 0 && t0 < To) ? ((unsigned)co * (unsigned)To + (unsigned)t0) * PY::ES : OOB_OFF;
          f32x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = (acc[m][n][4 * i + j] + bv[4 * i + j]) + cv[4 * i + j];
            if (AMAX && off != OOB_OFF && co < Cr) vmax = fmaxf(vmax, fabsf(v[j]));
          }
          pstore4<YB>(rout, v, off, 0u);
        }
        continue;
      }
      if (U == 2) {
        // registers r, r+1 (r even) are phases 0, 1 of channel co: samples 2*mm - 1, 2*mm, one
        // dwordx2 store (dword-aligned) unless the pair straddles the plane's start or end
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const int rho = cobase + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
          const int co = rho >> 1;
          const int t = 2 * mm - 1;
          const float v0 = (acc[m][n][r] + bv[r]) + cv[r];
          const float v1 = (acc[m][n][r + 1] + bv[r + 1]) + cv[r + 1];
          const unsigned rowoff = (unsigned)co * (unsigned)To;
          if (!YB && t >= 0 && t + 1 < To) {
            if (AMAX && co < Cr) vmax = fmaxf(vmax, fmaxf(fabsf(v0), fabsf(v1)));
            const f32x2 v = {v0, v1};
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), rout, (int)((rowoff + (unsigned)t) * 4u), 0, TTS_ST_POL);
          } else {
            // (bf16: the pair starts at an odd sample, 2-byte aligned: two 16-bit stores)
            const unsigned off0 = (t >= 0 && t < To) ? (rowoff + (unsigned)t) * PY::ES : OOB_OFF;
            const unsigned off1 = (t + 1 >= 0 && t + 1 < To) ? (rowoff + (unsigned)t + 1u) * PY::ES : OOB_OFF;
            if (AMAX && co < Cr) {
              if (off0 != OOB_OFF) vmax = fmaxf(vmax, fabsf(v0));
              if (off1 != OOB_OFF) vmax = fmaxf(vmax, fabsf(v1));
            }
            PY::st(rout, v0, off0, 0u);
            PY::st(rout, v1, off1, 0u);
          }
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rho = cobase + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        const int co = rho >> lgU;
        const int t = (mm << lgU) + (rho & (U - 1)) - (U >> 1);
        // rows >= Cout land past the plane (co >= Cr); samples outside [0, To) are marked OOB
        const unsigned off = (t >= 0 && t < To) ? ((unsigned)co * (unsigned)To + (unsigned)t) * PY::ES : OOB_OFF;
        const float v = (acc[m][n][r] + bv[r]) + cv[r];
        if (AMAX && off != OOB_OFF && co < Cr) vmax = fmaxf(vmax, fabsf(v));
        PY::st(rout, v, off, 0u);
      }
    }
  }
  if (AMAX && a.amax_out) publish_amax(a.amax_out, b, vmax);
}

// The per-element options are template parameters (one uniform dispatch per tile), so the
// unrolled epilogue carries no per-element branches.
template <int TM, int TN, bool AMAX = false, bool YB = false>
__device__ __forceinline__ void conv_epilogue(const Conv1dArgs& args, const f32x16 (&acc)[TM][TN], int b,
                                              int tbase, int cobase, int lane, int tend = 0x7fffffff,
                                              const float* sbias = nullptr, int sbase = 0) {
  // copy the argument block: a store through `out` could alias it in the compiler's view
  const Conv1dArgs a = args;
  const int zm = a.zmode <= 1 ? 0 : a.zmode;
#define TTS_EPI(RES, ZM) conv_epilogue_impl<TM, TN, RES, ZM, AMAX, YB>(a, acc, b, tbase, cobase, lane, tend, sbias, sbase)
  if (a.res) {
    if (zm == 0) TTS_EPI(true, 0);
    else if (zm == 2) TTS_EPI(true, 2);
    else TTS_EPI(true, 3);
  } else {
    if (zm == 0) TTS_EPI(false, 0);
    else if (zm == 2) TTS_EPI(false, 2);
    else TTS_EPI(false, 3);
  }
#undef TTS_EPI
}

}  // namespace tts
