// Winograd F(4,4) conv1d, 8-wave point-split form (gfx950).  Same arithmetic as
// conv1d_wino_kernel (wino_kernel.hpp: transforms, split, packed weights), different schedule:
//
// * 512 threads, two waves per SIMD.  Waves w and w+4 compute the same 32 output channels x 64
//   tile columns; wave w accumulates points 0-3, wave w+4 points 4-6 (128 accumulator registers
//   each instead of 224 for all seven), so the workgroup keeps two waves on every SIMD and one
//   wave's stalls (input loads, transform VALU, barriers) overlap the other's MFMAs.
// * The input window of a 16-channel chunk reaches LDS by LDS-DMA (buffer_load_dwordx4 ... lds),
//   two chunks ahead, issued by waves 4-7 only: vector-memory counters retire in order, so the
//   wave that issues an HBM load stalls at its next weight-prefetch wait until the load lands;
//   waves 0-3, which carry 4/7 of the MFMAs, never issue one and keep the matrix pipe busy.
// * The transform of chunk c+1 (raw fp32 window in LDS -> 7 split point planes) is spread evenly
//   over all eight waves (one channel quad of one tile column per lane, four channel pieces
//   placed between the MFMA steps of chunk c).
// * Barriers are bare s_barrier with an explicit lgkmcnt wait: __syncthreads' fence would also
//   drain the DMA and weight loads in flight.
// * Epilogue: the two waves of a pair swap their partial point sums through LDS (each finishes
//   one 32-column block), then store 16-byte vectors of 4 consecutive samples (dilation 1) or
//   transpose their rows through LDS first (dilation 3, 5), as wino_kernel.hpp.
#pragma once

#include <type_traits>

#include "wino_kernel.hpp"

namespace tts {

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#ifndef WINO_STAMPS
#define WINO_STAMPS 0  // diagnostic builds only: per-wave s_memtime stamps into Conv1dArgs::z (zmode 0)
#endif
// stamp slot i of this wave: z viewed as u64[workgroup][wave][32] (lane 0 stores)
#define WSTAMP(i)                                                                                            \
  do {                                                                                                       \
    if (WINO_STAMPS && (threadIdx.x & 63) == 0) {                                                            \
      const size_t wg = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z);      \
      reinterpret_cast<unsigned long long*>(a.z)[(wg * 8 + (threadIdx.x >> 6)) * 32 + (i)] =                   \
          __builtin_amdgcn_s_memtime();                                                                      \
    }                                                                                                        \
  } while (0)

// XB: the input plane is bf16 (Conv1dArgs::planes, MATH_BF16): the raw window in LDS holds 2-byte
// elements, AL = 8 per 16-byte DMA unit instead of 4
template <class S, int K, int D, bool XB = false>
struct Wino8Cfg {
  static constexpr int ES = XB ? 2 : 4;              // bytes per raw element
  static constexpr int AL = 16 / ES;                 // raw elements per 16-byte DMA unit
  static constexpr int NCH = wino_chunks(K);
  static constexpr int NS = kWinoPoints * NCH;       // packed steps per 16-channel chunk (c*7 + p)
  static constexpr int PAD = D * (K - 1) / 2;
  static constexpr int BNT = 64;                     // tile columns per workgroup (2 x 32)
  static constexpr int J = BNT / D;                  // tiles per residue class
  static constexpr int TW = 4 * D * J;               // output samples per workgroup
  static constexpr int XROWS = BNT + (NCH - 1) * D;  // transformed columns (halo of the chunk shifts)
  static constexpr int PLANE = XROWS * S::ROWB;
  static constexpr int TSZ = kWinoPoints * PLANE;    // bytes of one transformed buffer
  // raw window: times t0 - PAD - ROFF ... (16-byte aligned start; t0 is a multiple of 4, of 8 but at
  // D = 3 (TW = 252), where the bf16 form takes its offset per workgroup: roff <= 7, span for 7)
  static constexpr bool RT_ROFF = XB && TW % 8 != 0;
  static constexpr int ROFF = RT_ROFF ? 7 : (AL - PAD % AL) % AL;
  static constexpr int RSPAN = (XROWS - 1) % D + 4 * D * ((XROWS - 1) / D) + 6 * D + ROFF + 1;
  static constexpr int RSPAN4 = (RSPAN + AL - 1) / AL * AL;
  // RPITCH / AL odd: the 16-byte units of consecutive channel rows cycle through the bank row
  static constexpr int RPITCH = RSPAN4 % (2 * AL) == AL ? RSPAN4 : RSPAN4 + AL;
  static constexpr int RF4 = (16 * RPITCH / AL + 63) / 64 * 64;         // 16-byte units per raw buffer (DMA rows of 64)
  static constexpr int RSZ = RF4 * 16;
  static constexpr int NDMA = RF4 / 64;              // DMA instructions per chunk (waves 4-7)
  static constexpr int UNITS = XROWS * 4;            // (column, channel quad)
  static constexpr int UPW = (UNITS + 7) / 8;        // units per wave
  static constexpr int PITCH = 256;                  // epilogue transpose row (samples)
  static_assert(UPW <= 64 && UNITS <= 256 + 64 && 3 * NCH >= 3, "one transform round per wave; the DMA spreads over 3 steps");
  static_assert(2 * (UNITS - 256) <= 4 * 64, "spread leftover jobs: one per lane of waves 4-7");
  static_assert(TW <= PITCH, "");
  // the transformed buffers double as the epilogue's exchange (8 waves x 8 rows x 64 lanes x 16 B) and
  // transpose regions; the bf16 scheme's 48-byte rows need the floor
  static constexpr int EPI = 4 * 16 * PITCH * 4 > 8 * 8 * 4 * 64 * 4 ? 4 * 16 * PITCH * 4 : 8 * 8 * 4 * 64 * 4;
  static constexpr int TSM = 2 * TSZ > EPI ? 2 * TSZ : EPI;
};

// PL: Conv1dArgs::planes (MATH_BF16 only: 0, or bf16 input and bf16 res / z / y)
template <class S, int K, int D, bool LRELU, int PL = 0>
__global__ __launch_bounds__(512) void conv1d_wino8_kernel(Conv1dArgs a) {
  constexpr bool XB = (PL & kPlaneXB16) != 0, YB = (PL & kPlaneYB16) != 0;
  using C = Wino8Cfg<S, K, D, XB>;
  constexpr int NP = S::NP;
  constexpr int NCH = C::NCH;
  constexpr bool H3 = S::SCALED;
  static_assert(PL == 0 || !H3, "bf16 planes: the bf16 scheme only");
// weight prefetch depths (steps) of the two point groups and the transform-piece read->math gap
// (steps) per kernel size; round-4 re-tune after the conflict-free job reads (3 rounds x 3 builds,
// one box session): PD 3 / PD1 4 / GAP11 1 gave 53.5 ms per batch against 53.9 for the round-3
// values 2 / 6 / 0 (PD 3 alone or GAP11 1 alone: 53.7; PD1 8 spills; GAP7 0: 54.1)
#ifndef WINO8_PD
#define WINO8_PD 3
#endif
#ifndef WINO8_EARLY_W
#define WINO8_EARLY_W 0
#endif
#ifndef WINO8_PD1
#define WINO8_PD1 4
#endif
#ifndef WINO8_PD11
#define WINO8_PD11 WINO8_PD  // kernel 11, points 0-3 (A/B: 2 keeps the kernel below 256 VGPRs)
#endif
#ifndef WINO8_PD_B1
#define WINO8_PD_B1 3
#endif
#ifndef WINO8_PD1_B1
#define WINO8_PD1_B1 4
#endif
#ifndef WINO8_GAP7
#define WINO8_GAP7 1
#endif
#ifndef WINO8_GAP11
#define WINO8_GAP11 1
#endif
  __shared__ __attribute__((aligned(16))) unsigned char tsm[C::TSM];  // transformed planes
  __shared__ __attribute__((aligned(16))) unsigned char rsm[2 * C::RSZ];  // raw input windows
  __shared__ float wbias[128];  // bias + cvec of the 128 rows, staged in the prologue (the epilogue
                                // reads LDS instead of paying an L2 latency per pass)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3;   // 32-row block
  const int grp = wave >> 2;  // 0: points 0-3 (+ no loads), 1: points 4-6 (+ the input DMA)
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int bx = blockIdx.x, mt = blockIdx.y, b = blockIdx.z;
  const int t0 = bx * C::TW;
  const int Tin = a.Tin;
  const int Cin = a.Cin;
  const int nc = a.n_chunks;
  const int ex = H3 ? amax_exp(a.amax_in, b) + kWinoBtShift : 0;
  const float xscale = H3 ? ldexpf(1.f, -ex) : 1.f;
  const float slope = a.in_slope;
  const char* xb = static_cast<const char*>(plane_at<XB>(a.x, (size_t)b * (a.x_bstride ? a.x_bstride : (int64_t)Cin * Tin)));
  const unsigned chb = (unsigned)Tin * (unsigned)C::ES;

  // ---- input DMA (waves 4-7): raw[ch][RPITCH] elements, window start ta = t0 - PAD - roff ----
  const int roff = C::RT_ROFF ? (((t0 - C::PAD) % 8) + 8) % 8 : C::ROFF;  // ta = 0 mod AL
  const int ta = t0 - C::PAD - roff;
  // DMA instructions i = wm + 4k of raw(c) -> R[rb], for k in [k0, k1) (wave-uniform)
#ifndef WINO8_ASM_DMA
#define WINO8_ASM_DMA 1  // 0: the LDS-DMA builtin (the compiler then waits for each DMA at the next LDS access)
#endif
  auto dma = [&](int c, int rb, int k0 = 0, int k1 = 64) {
    const int c0 = c * 16;
    const rsrc_t rx = make_rsrc(xb + (size_t)c0 * chb, (unsigned)(Cin - c0) * chb);
    for (int i = wm + 4 * k0; i < C::NDMA && i < wm + 4 * k1; i += 4) {
      const int f = i * 64 + lane;
      constexpr int UPR = C::RPITCH / C::AL;  // 16-byte units per channel row
      const int ch = f / UPR, t = ta + C::AL * (f - ch * UPR);
      const unsigned vo = (ch < 16 && t >= 0 && t < Tin) ? (unsigned)ch * chb + (unsigned)t * (unsigned)C::ES : OOB_OFF;
      if (WINO8_ASM_DMA) {
        lds_dma_b128(xb + (size_t)c0 * chb, (unsigned)(Cin - c0) * chb, vo, rsm + rb * C::RSZ + i * 1024);
      } else {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rx, (__attribute__((address_space(3))) void*)(rsm + rb * C::RSZ + i * 1024), 16, (int)vo, 0, 0, 0);
      }
    }
  };

  // ---- transform jobs: unit (column row, channel quad q) ----
#ifndef WINO8_DENSE
#define WINO8_DENSE 1
#endif
#ifndef WINO8_SPREAD
#define WINO8_SPREAD 1
#endif
  // dense: waves 0-3 (which issue no HBM loads and so never wait on one) take units 0-255 with every
  // lane, all four channel pieces each; else every wave takes UPW units (balanced, but only UPW of
  // its 64 lanes active).  The units past 256 (the chunk halo: 4-40 of them): with WINO8_SPREAD
  // each lane of waves 4-7 takes one (unit, piece pair) job, dealt round-robin over the four waves,
  // so every SIMD runs the transform instructions of one full and one half pass; otherwise wave 4
  // alone takes them whole and its SIMD runs two full passes per chunk while the others run one.
#ifndef WINO8_TG_B1
#define WINO8_TG_B1 0
#endif
  // the point group whose waves take the dense units (f16x3: group 0; the DMA waves were slower);
  // bf16 carries a third of the MFMAs, so its balance is measured separately (WINO8_TG_B1)
  constexpr int TG = S::NP == 1 ? WINO8_TG_B1 : 0;
  const int e = lane * 4 + wm;  // leftover job of a lane of the other group
  const int u = WINO8_DENSE ? (grp == TG ? wm * 64 + lane
                                         : (WINO8_SPREAD ? 256 + (e >> 1) : (wm == 0 ? 256 + lane : C::UNITS)))
                            : wave * C::UPW + lane;
  const bool uok = (WINO8_DENSE || lane < C::UPW) && u < C::UNITS;
  // pieces a lane transforms: all four, or one pair (2 jp, 2 jp + 1) for a spread leftover job
  constexpr bool SPREAD = WINO8_DENSE && WINO8_SPREAD;
  const int jp = e & 1;
  float tkeep[7], jraw[7];
  // D = 1: a column's 7 inputs are raw floats 4 urow + ROFF ... + 6 of its channel row, read as NU
  // aligned float4s (ds_read_b128).  The lanes of a 16-lane group hold 4 columns x 4 channel quads:
  // float4 slots c * RPITCH / 4 + urow, RPITCH / 4 odd, cover all 16 slots of the bank row (no
  // conflict), where 7 ds_read_b32 at one sub-offset put 32 lanes on 8 banks (4-way).  bf16 input:
  // NU 8-byte groups of 4 elements (ds_read_b64), widened in job_finish
  constexpr int NU = (C::ROFF + 6) / 4 + 1;
  f32x4 jraw4[XB ? 1 : NU];
  u32x2_t jraw8[XB ? NU : 1];
  // piece j: channel 4q + j; pairs are written after channels 1 and 3.  A piece runs in two parts
  // one MFMA step apart: job_load issues its 7 LDS reads, job_finish transforms (and splits and
  // stores every second piece), so the reads' latency hides behind the step's MFMAs
  // job index j = 0..3 -> channel piece (a spread lane maps its jobs 0, 1 onto its pair; 2, 3 are empty)
  auto piece = [&](int j) { return SPREAD && grp != TG ? 2 * jp + j : j; };
  const int jrow0 = u >> 2, jq0 = u & 3;  // the lane's unit: column row, channel quad
#ifndef WINO8_REMAT
#define WINO8_REMAT 0  // A/B: 1 = kernels 3 / 7 recompute the unit as kernel 11 does
#endif
#ifndef WINO8_REMAT11
#define WINO8_REMAT11 1
#endif
  // kernel 11: the dense group recomputes its unit from the lane id at every job.  That kernel runs
  // at the 256-VGPR limit and otherwise spills these lane-derived offsets (36 B of scratch, every
  // reload a scratch load with a vmcnt wait behind the weight prefetches): k11 c128 -3%, c256 -2%.
  // Kernel 7 does not spill and runs 2.5% slower with the recomputation
  // (profiles/ab_r05_wino_remat.txt)
  constexpr bool remat = K == 11 ? WINO8_REMAT11 : WINO8_REMAT;
  auto job_unit = [&](int& jrow, int& jq) {
    if (remat && WINO8_DENSE && grp == TG) {
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      const int uu = wm * 64 + ln;
      jrow = uu >> 2;
      jq = uu & 3;
    } else {
      jrow = jrow0;
      jq = jq0;
    }
  };
  auto job_load = [&](int rb, int j) {
    if (SPREAD && grp != TG && j >= 2) return;
    if (!uok) return;
    int jrow, jq;
    job_unit(jrow, jq);
    if constexpr (D == 1 && XB) {
      const u32x2_t* raw8 =
          reinterpret_cast<const u32x2_t*>(rsm + rb * C::RSZ) + (4 * jq + piece(j)) * (C::RPITCH / 4) + jrow;
#pragma unroll
      for (int u4 = 0; u4 < NU; ++u4) jraw8[u4] = raw8[u4];
    } else if constexpr (D == 1) {
      const f32x4* raw4 =
          reinterpret_cast<const f32x4*>(rsm + rb * C::RSZ) + (4 * jq + piece(j)) * (C::RPITCH / 4) + jrow;
#pragma unroll
      for (int u4 = 0; u4 < NU; ++u4) jraw4[u4] = raw4[u4];
    } else if constexpr (XB) {
      const int jjj = jrow / D, jrho = jrow - jjj * D;
      const unsigned short* raw = reinterpret_cast<const unsigned short*>(rsm + rb * C::RSZ) +
                                  (4 * jq + piece(j)) * C::RPITCH + jrho + 4 * D * jjj + roff;
#pragma unroll
      for (int k = 0; k < 7; ++k) jraw[k] = bf16_bits_to_f32(raw[D * k]);
    } else {
      const int jjj = jrow / D, jrho = jrow - jjj * D;
      const float* raw = reinterpret_cast<const float*>(rsm + rb * C::RSZ) + (4 * jq + piece(j)) * C::RPITCH +
                         jrho + 4 * D * jjj + C::ROFF;
#pragma unroll
      for (int k = 0; k < 7; ++k) jraw[k] = raw[D * k];
    }
  };
  auto job_finish = [&](int tb, int j) {
    if (SPREAD && grp != TG && j >= 2) return;
    if (!uok) return;
    int jrow, jq;
    job_unit(jrow, jq);
    float v[7], t[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      float x;
      if constexpr (D == 1 && XB) {
        const unsigned w = jraw8[(C::ROFF + k) / 4][((C::ROFF + k) % 4) / 2];
        x = bf16_bits_to_f32((C::ROFF + k) % 2 ? w >> 16 : w & 0xffffu);
      } else {
        x = D == 1 ? jraw4[(C::ROFF + k) / 4][(C::ROFF + k) % 4] : jraw[k];
      }
      if (LRELU) x = lrelu2(x, slope);
      v[k] = H3 ? x * xscale : x;
    }
    wino_bt(v, t);
    if ((j & 1) == 0) {
#pragma unroll
      for (int k = 0; k < 7; ++k) tkeep[k] = t[k];
      return;
    }
    // word uq + 4 * pair of the row (channels 4 uq + 2 pair, +1; the weights are packed in this
    // channel order, pack_conv1d_wino): a 32-lane half (8 rows x 4 quads) covers all 32 banks
    unsigned char* base = tsm + tb * C::TSZ + jrow * S::ROWB + 4 * jq + 16 * (piece(j) >> 1);
#pragma unroll
    for (int p = 0; p < kWinoPoints; ++p) {
      unsigned w[NP];
      split_pair<S>(tkeep[p], t[p], w);
#pragma unroll
      for (int q = 0; q < NP; ++q) *reinterpret_cast<unsigned*>(base + p * C::PLANE + 32 * q) = w[q];
    }
  };

  // ---- weights: this wave's 32-row block, packed steps (chunk, c*7 + p) ----
  const int mb = mt * 4 + wm;
  const rsrc_t ra = make_rsrc(a.w + ((size_t)mb * nc * C::NS) * (NP * 256), 0xFFFFFFFFu);
  const unsigned avoff = (unsigned)lane * 16u;

#ifndef WINO8_NOXCH
#define WINO8_NOXCH 0
#endif
  // NX (A/B): each wave accumulates all 7 points of ONE 32-column block (wave w column block 0,
  // wave w + 4 block 1, the same 32 rows and weight steps): no partial-sum exchange in the
  // epilogue and equal MFMA work in both groups, for twice the weight loads per MFMA (the pair's
  // two waves load the same addresses).  The per-accumulator MFMA sequence and the output
  // transform's sums are those of the point split, so the results are bitwise the same.
  constexpr bool NX = WINO8_NOXCH != 0;
  constexpr int NA = NX ? 7 : 4, NB = NX ? 1 : 2;  // accumulators: points x column blocks
  f32x16 acc[NA][NB];
#pragma unroll
  for (int p = 0; p < NA; ++p)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[p][n] = f32x16{};
  WSTAMP(0);

  float bpre = 0.f;
  if (tid < 128) {
    const int co = mt * 128 + tid;
    if (co < a.Cout) {
      bpre = a.bias[co];
      const float cv = a.cvec ? a.cvec[(size_t)b * (a.cvec_bstride ? a.cvec_bstride : (int64_t)a.Cout) + co] : 0.f;
      bpre = bpre + cv;  // the sum the two range-checked epilogue loads gave
    }
  }
  // prologue: raw(0), raw(1) -> R0, R1; transform raw(0) -> T0.  With WINO8_EARLY_W the transform
  // runs inside run() after the first weight prefetch is issued, so those loads overlap it; WL is
  // the number of weight loads a wave has issued after its DMAs
  if (grp == 1) {
    dma(0, 0);
    if (nc > 1) dma(1, 1);
  }
  auto prologue = [&](auto wl_tag) {
    constexpr int WL = decltype(wl_tag)::value;
    if (grp == 1) {
      // raw(0) only: a wave issues at least NDMA / 4 instructions of raw(1) after it (in order)
      if (nc > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::NDMA / 4 + WL) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WL) : "memory");
    }
    WSTAMP(1);
    if (tid < 128) wbias[tid] = bpre;
    lds_sync();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      job_load(0, j);
      job_finish(0, j);
    }
    // raw(1) must have landed before the barrier: chunk 0's transform jobs read R[1] from its first
    // step on (this also waits for the prefetched weights, which overlapped the transform above)
    if (grp == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_sync();
    WSTAMP(2);
  };
  if (!WINO8_EARLY_W) prologue(std::integral_constant<int, 0>{});

  // the chunk loop of one point group (NPG points starting at P0); both groups run it with the
  // same barrier sequence
  auto run = [&](auto npg_tag, auto p0_tag, auto g1_tag) {
    constexpr int NPG = decltype(npg_tag)::value;
    constexpr int P0 = decltype(p0_tag)::value;
    constexpr bool G1 = decltype(g1_tag)::value;  // the DMA-issuing group (waves 4-7)
    constexpr int NV = NPG * NCH;  // MFMA steps per chunk for this wave
    // weight prefetch depth: the DMA-issuing waves (P0 > 0, 96 accumulator registers) prefetch
    // further ahead, so the in-order wait for their input DMA falls PDG steps after its issue
    // the bf16 scheme's steps are a third as long (one product per MAC): its own depths (A/B)
    constexpr int PD = NP == 1 ? (G1 ? WINO8_PD1_B1 : WINO8_PD_B1)
                               : (G1 ? WINO8_PD1 : (K == 11 ? WINO8_PD11 : WINO8_PD));
    // steps between a transform piece's LDS reads and its math (no later than the next piece's
    // reads); measured per kernel size
    constexpr int GAP0 = K == 11 ? WINO8_GAP11 : WINO8_GAP7;
    constexpr int GAP = GAP0 < NV / 4 ? GAP0 : NV / 4;
    auto aoff = [&](int ck, int v) {  // byte soffset of virtual step v of chunk ck (v may run past NV)
      const int ck2 = ck + v / NV, v2 = v % NV;
      // prefetches past the last chunk (never used) re-read step 0 instead of running off the array
      return ck2 < nc ? (unsigned)((ck2 * C::NS + (v2 / NPG) * 7 + P0 + v2 % NPG) * NP) * 1024u : 0u;
    };
    f32x4 ar[PD + 1][NP], bcur[NB][NP], bnext[NB][NP];
#pragma unroll
    for (int v = 0; v < PD; ++v)
#pragma unroll
      for (int q = 0; q < NP; ++q) ar[v][q] = bload4(ra, avoff, aoff(0, v) + (unsigned)q * 1024u);
    if (WINO8_EARLY_W) prologue(std::integral_constant<int, PD * NP>{});
    auto read_b = [&](const unsigned char* tl, int v, f32x4 (*dst)[NP]) {
      const int p = P0 + v % NPG, c = v / NPG;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const unsigned char* ptr = tl + p * C::PLANE + ((NX ? grp : n) * 32 + l32 + c * D) * S::ROWB + 16 * half;
#pragma unroll
        for (int q = 0; q < NP; ++q) dst[n][q] = *reinterpret_cast<const f32x4*>(ptr + 32 * q);
      }
    };
    for (int ck = 0; ck < nc; ++ck) {
      const int tb = ck & 1;
      const unsigned char* tl = tsm + tb * C::TSZ;
      const bool more = ck + 1 < nc;
      read_b(tl, 0, bcur);
      if (ck < 8) WSTAMP(3 + 2 * ck);
#pragma unroll
      for (int v = 0; v < NV; ++v) {
#pragma unroll
        for (int q = 0; q < NP; ++q)
          ar[PD][q] = (WINO_ABLATE & 4) ? ar[0][q]
                                        : bload4(ra, avoff, ((WINO_ABLATE & 64) ? 0u : aoff(ck, v + PD)) + (unsigned)q * 1024u);
        if (v + 1 < NV) read_b(tl, v + 1, bnext);
        // raw(ck+2) -> R[ck & 1] (raw(ck) is consumed), two DMA instructions per step
        if ((WINO_ABLATE & 32) == 0 && G1 && ck + 2 < nc && v < 3) dma(ck + 2, tb, 2 * v, v == 2 ? 64 : 2 * v + 2);
        __builtin_amdgcn_sched_barrier(0);
        const int p = v % NPG;
#pragma unroll
        for (int e = 0; e < S::NPROD; ++e)
#pragma unroll
          for (int n = 0; n < NB; ++n) {
            if (WINO_ABLATE & 8) acc[p][n][e] += ar[0][S::PA[e]][0] * bcur[n][S::PB[e]][0];
            else acc[p][n] = S::mfma(ar[0][S::PA[e]], bcur[n][S::PB[e]], acc[p][n]);
          }
#pragma unroll
        for (int pp = 0; pp < PD; ++pp)
#pragma unroll
          for (int q = 0; q < NP; ++q) ar[pp][q] = ar[pp + 1][q];
        if (v + 1 < NV) {
#pragma unroll
          for (int n = 0; n < NB; ++n)
#pragma unroll
            for (int q = 0; q < NP; ++q) bcur[n][q] = bnext[n][q];
        }
        // transform pieces of chunk ck+1 (raw in R[(ck+1) & 1]) between the MFMA steps: piece j
        // loads after step (j * NV) / 4 and finishes GAP steps later (0: at once)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int vj = (j * NV) / 4;
          if ((WINO_ABLATE & 2) == 0 && more) {
            if (GAP > 0 && vj + GAP < NV && v == vj + GAP) job_finish(tb ^ 1, j);
            if (v == vj) {
              job_load(tb ^ 1, j);
              if (GAP == 0 || vj + GAP >= NV) job_finish(tb ^ 1, j);
            }
          }
        }
      }
      // raw(ck+2) landed: at most the weight loads issued after the last DMA (steps 3.. of this chunk)
      // may still be in flight
      constexpr int NAFTER = (PD < NV - 3 ? PD : NV - 3) * NP;
      if (G1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NAFTER) : "memory");
      if (ck < 8) WSTAMP(4 + 2 * ck);
      lds_sync();
    }
  };
#ifndef WINO8_PRIO
#define WINO8_PRIO 0  // A/B: 1 = s_setprio 1 on the DMA waves (4-7) for the main loop, 2 = on waves 0-3
#endif
  if (WINO8_PRIO == 1 && grp == 1) __builtin_amdgcn_s_setprio(1);
  if (WINO8_PRIO == 2 && grp == 0) __builtin_amdgcn_s_setprio(1);
  if constexpr (NX) {
    if (grp == 0) run(std::integral_constant<int, 7>{}, std::integral_constant<int, 0>{}, std::false_type{});
    else run(std::integral_constant<int, 7>{}, std::integral_constant<int, 0>{}, std::true_type{});
  } else {
    if (grp == 0) run(std::integral_constant<int, 4>{}, std::integral_constant<int, 0>{}, std::false_type{});
    else run(std::integral_constant<int, 3>{}, std::integral_constant<int, 4>{}, std::true_type{});
  }

#ifndef WINO8_EPI_PF
#define WINO8_EPI_PF 0
#endif
  // L2 prefetch of the epilogue's gathers (dilation 1: the residual and the MRF sum): every
  // 128-byte line of this workgroup's 128-row x TW-sample output tile is touched once, right after
  // the wave's last weight load, so the gathers after the output transform and the partial-sum
  // exchange hit L2 instead of HBM.  The LDS-DMA writes land in the raw windows, which nothing
  // reads after the last chunk's transform (the chunk before it)
  if constexpr (WINO8_EPI_PF && D == 1) {
    if (a.res || a.zmode >= 2) {
      constexpr unsigned YES = PlaneT<YB>::ES;
      constexpr int LPR = C::TW * (int)YES / 128;  // lines per row
      const unsigned plane = (unsigned)a.Cout * (unsigned)a.Tout * YES;
      const size_t item = (size_t)b * (a.o_bstride ? a.o_bstride : (int64_t)a.Cout * a.Tout);
      const void* pres = a.res ? plane_at<YB>(a.res, item) : nullptr;
      const void* pz = a.zmode >= 2 ? plane_at<YB>(a.z, item) : nullptr;
#pragma unroll
      for (int i = 0; i < (128 * LPR + 511) / 512; ++i) {
        const int l = tid + 512 * i;
        const int co = mt * 128 + l / LPR, ln = l % LPR;
        const int t = t0 + ln * (128 / (int)YES);
        const unsigned vo = (l < 128 * LPR && co < a.Cout && t < a.Tout) ? ((unsigned)co * (unsigned)a.Tout + (unsigned)t) * YES : OOB_OFF;
        if (pres) l2_touch_dma(pres, plane, vo, rsm);
        if (pz) l2_touch_dma(pz, plane, vo, rsm + 256);
      }
    }
  }

  // ---- epilogue ----
  if (WINO_ABLATE & 16) {
    float sum = 0.f;
#pragma unroll
    for (int p = 0; p < NA; ++p)
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) sum += acc[p][n][r];
    if (sum == 1234.5f) a.y[threadIdx.x] = sum;
    return;
  }
  // the f16x3 rescale sc (an exact power of two) commutes with the output transform: applied once
  // per output in wino_apply instead of once per point here
  const float sc = H3 ? ldexpf(1.f, ex + a.w_exp) : 1.f;
  const int nk = grp;  // the column block this wave finishes
  float y[4][16];
  if constexpr (NX) {
    // all 7 points of column block nk in this wave: the point-split sums (points 0-3) + (4-6),
    // formed exactly as the exchange below forms them
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float m0 = acc[0][0][r], m1 = acc[1][0][r], m2 = acc[2][0][r], m3 = acc[3][0][r];
      const float m4 = acc[4][0][r], m5 = acc[5][0][r], m6 = acc[6][0][r];
      const float s12 = m1 + m2, d12 = m1 - m2;
      y[0][r] = ((m0 + s12) + m3) + (m4 + m5);
      y[1][r] = fmaf(2.f, m3, d12) + fmaf(-2.f, m4, 0.5f * m5);
      y[2][r] = fmaf(4.f, m3, s12) + fmaf(4.f, m4, 0.25f * m5);
      y[3][r] = fmaf(8.f, m3, d12) + (fmaf(-8.f, m4, 0.125f * m5) + m6);
    }
    WSTAMP(20);
  } else {
  // partial outputs of this wave's points: yp[n][i][r]
  float yp[2][4][16];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (grp == 0) {
        const float m0 = acc[0][n][r], m1 = acc[1][n][r], m2 = acc[2][n][r], m3 = acc[3][n][r];
        const float s12 = m1 + m2, d12 = m1 - m2;
        yp[n][0][r] = (m0 + s12) + m3;
        yp[n][1][r] = fmaf(2.f, m3, d12);
        yp[n][2][r] = fmaf(4.f, m3, s12);
        yp[n][3][r] = fmaf(8.f, m3, d12);
      } else {
        const float m4 = acc[0][n][r], m5 = acc[1][n][r], m6 = acc[2][n][r];
        yp[n][0][r] = m4 + m5;
        yp[n][1][r] = fmaf(-2.f, m4, 0.5f * m5);
        yp[n][2][r] = fmaf(4.f, m4, 0.25f * m5);
        yp[n][3][r] = fmaf(-8.f, m4, 0.125f * m5) + m6;
      }
    }
  WSTAMP(20);
  // swap halves: group 0 finishes column block 0, group 1 block 1 (two passes of 8 rows per lane)
  // [wm][grp][8 r][64 lanes] float4 (the 4 outputs i of one register r): one ds_write_b128 /
  // ds_read_b128 per r, lanes contiguous (conflict-free), 64 KiB
  f32x4* xch = reinterpret_cast<f32x4*>(tsm);
  lds_sync();  // every wave is past its last LDS read of the main loop
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = grp == 0 ? yp[1][i][8 * h + r] : yp[0][i][8 * h + r];
      xch[((wm * 2 + grp) * 8 + r) * 64 + lane] = v;
    }
    lds_sync();
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const f32x4 other = xch[((wm * 2 + (1 - grp)) * 8 + r) * 64 + lane];
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i][8 * h + r] = (grp == 0 ? yp[0][i][8 * h + r] : yp[1][i][8 * h + r]) + other[i];
    }
    lds_sync();
  }
  }

  WSTAMP(21);
  const int zm = a.zmode <= 1 ? 0 : a.zmode;
  const int cobase = mt * 128 + wm * 32;
  auto finish = [&](auto res_tag, auto zm_tag) {
    constexpr bool RES = decltype(res_tag)::value;
    constexpr int ZM = decltype(zm_tag)::value;
    const int Cout = a.Cout;
    const int Tout = a.Tout;
    constexpr unsigned YES = PlaneT<YB>::ES;
    const unsigned plane = (unsigned)Cout * (unsigned)Tout * YES;
    const size_t item = (size_t)b * (a.o_bstride ? a.o_bstride : (int64_t)Cout * Tout);
    const rsrc_t rres = make_rsrc(RES ? plane_at<YB>(a.res, item) : a.bias, RES ? plane : 0u);
    const rsrc_t rz = make_rsrc(ZM >= 2 ? plane_at<YB>(a.z, item) : a.bias, ZM >= 2 ? plane : 0u);
    const rsrc_t rout = make_rsrc(plane_at<YB>(a.zmode == 0 ? a.y : a.z, item), plane);
    const float oslope = a.out_slope;
    const float zdiv = a.zdiv;
    float vmax = 0.f;
    if constexpr (D == 1) {
      const int t = t0 + 4 * (nk * 32 + l32);
      const int nvalid = Tout - t < 4 ? (Tout - t > 0 ? Tout - t : 0) : 4;
      const bool full = nvalid == 4 && (Tout & 3) == 0;
      // gather GR vectors (residual, MRF sum) before computing and storing them: all 16 at once
      // pay one memory latency per tile instead of two (the accumulators are dead by now); with
      // both a residual and an MRF sum to read, 16 at once would spill, so two rounds of 8
      constexpr int GR = (RES && ZM >= 2) ? 8 : 16;
#pragma unroll
      for (int r0 = 0; r0 < 16; r0 += GR) {
        float bias[GR];
        unsigned voff[GR];
        WinoIn gin[GR];
#pragma unroll
        for (int k = 0; k < GR; ++k) {
          const int r = r0 + k;
          const unsigned co = (unsigned)(cobase + (r & 3) + 8 * (r >> 2) + 4 * half);
          bias[k] = wbias[co - (unsigned)(mt * 128)];
          voff[k] = nvalid > 0 ? (co * (unsigned)Tout + (unsigned)t) * YES : OOB_OFF;
          gin[k] = wino_gather<RES, ZM, YB>(rres, rz, voff[k], full, nvalid);
        }
#pragma unroll
        for (int k = 0; k < GR; ++k) {
          const int r = r0 + k;
          const f32x4 yv = {y[0][r], y[1][r], y[2][r], y[3][r]};
          const f32x4 v = wino_apply<RES, ZM, H3>(yv, bias[k], oslope, zdiv, gin[k], nvalid, vmax, sc);
          wino_store<YB>(rout, v, voff[k], full, nvalid);
        }
      }
    } else {
      // pair region [16 rows][PITCH] per pass; the pair's two waves read 8 rows each
      float* tile = reinterpret_cast<float*>(tsm) + wm * (16 * C::PITCH);
      const int nn = nk * 32 + l32;
      const int jj = nn / D, rho = nn - (nn / D) * D;
      const int tl = 4 * lane;
      const int t = t0 + tl;
      const int lim = (C::TW < Tout - t0 ? C::TW : Tout - t0) - tl;
      const int nvalid = lim < 4 ? (lim > 0 ? lim : 0) : 4;
      const bool full = nvalid == 4 && (Tout & 3) == 0;
#pragma unroll
      for (int ps = 0; ps < 2; ++ps) {
        if (jj < C::J) {
#pragma unroll
          for (int r = 8 * ps; r < 8 * ps + 8; ++r) {
            const int rl = (r & 3) + 8 * ((r >> 2) - 2 * ps) + 4 * half;
#pragma unroll
            for (int i = 0; i < 4; ++i) tile[rl * C::PITCH + rho + D * (4 * jj + i)] = y[i][r];
          }
        }
        lds_sync();
        float bias[8];
        unsigned voff[8];
        WinoIn gin[8];
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
          const int co = cobase + 16 * ps + grp * 8 + rr;
          bias[rr] = wbias[co - mt * 128];
          voff[rr] = nvalid > 0 ? ((unsigned)co * (unsigned)Tout + (unsigned)t) * YES : OOB_OFF;
          gin[rr] = wino_gather<RES, ZM, YB>(rres, rz, voff[rr], full, nvalid);
        }
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
          const f32x4 yv = *reinterpret_cast<const f32x4*>(tile + (grp * 8 + rr) * C::PITCH + tl);
          const f32x4 v = wino_apply<RES, ZM, H3>(yv, bias[rr], oslope, zdiv, gin[rr], nvalid, vmax, sc);
          wino_store<YB>(rout, v, voff[rr], full, nvalid);
        }
        lds_sync();
      }
    }
    if (H3 && a.amax_out) publish_amax(a.amax_out, b, vmax);
    WSTAMP(22);
  };
  using BT = std::true_type;
  using BF = std::false_type;
  using Z0 = std::integral_constant<int, 0>;
  using Z2 = std::integral_constant<int, 2>;
  using Z3 = std::integral_constant<int, 3>;
  if (a.res) {
    if (zm == 0) finish(BT{}, Z0{});
    else if (zm == 2) finish(BT{}, Z2{});
    else finish(BT{}, Z3{});
  } else {
    if (zm == 0) finish(BF{}, Z0{});
    else if (zm == 2) finish(BF{}, Z2{});
    else finish(BF{}, Z3{});
  }
}

namespace wino8_detail {
template <class S, int K, int D>
void launch_d(const Conv1dArgs& a, int B, hipStream_t s) {
  using C = Wino8Cfg<S, K, D>;
  const dim3 grid(ceil_div(a.Tout, C::TW), ceil_div(a.Cout, 128), B);
  if (a.planes != 0) {
    // bf16 activation planes (MATH_BF16): 16-byte aligned bf16 rows
    constexpr bool OK = std::is_same<S, SchemeB1>::value;
    TTS_REQUIRE(OK && a.planes == (kPlaneXB16 | kPlaneYB16) && a.Tin % 8 == 0, 3,
                "conv1d(winograd8): bf16 planes need the bf16 scheme and T % 8 == 0");
    if constexpr (OK) {
      constexpr int PL = kPlaneXB16 | kPlaneYB16;
      if constexpr (D == 1) {
        if (a.in_slope == 1.f) {
          hipLaunchKernelGGL((conv1d_wino8_kernel<S, K, D, false, PL>), grid, dim3(512), 0, s, a);
          return;
        }
      }
      hipLaunchKernelGGL((conv1d_wino8_kernel<S, K, D, true, PL>), grid, dim3(512), 0, s, a);
    }
    return;
  }
  if constexpr (D == 1) {
    if (a.in_slope == 1.f) {
      hipLaunchKernelGGL((conv1d_wino8_kernel<S, K, D, false>), grid, dim3(512), 0, s, a);
      return;
    }
  }
  hipLaunchKernelGGL((conv1d_wino8_kernel<S, K, D, true>), grid, dim3(512), 0, s, a);
}

template <class S, int K>
void launch_k(const Conv1dArgs& a, int B, hipStream_t s) {
  switch (a.dil) {
    case 1: launch_d<S, K, 1>(a, B, s); break;
    case 3: launch_d<S, K, 3>(a, B, s); break;
    case 5: launch_d<S, K, 5>(a, B, s); break;
    default: throw Error(3, "conv1d(winograd8): dilation must be 1, 3 or 5");
  }
}

template <class S>
void launch_s(const Conv1dArgs& a, int B, int K, hipStream_t s) {
  TTS_REQUIRE(a.mask == nullptr && a.ups == 0 && a.gate == 0 && a.rep_pad == 0 && a.Tin == a.Tout &&
                  a.pad == a.dil * (K - 1) / 2 && a.Tin % 4 == 0,
              1, "conv1d(winograd8): unsupported arguments");
  switch (K) {
    case 3: launch_k<S, 3>(a, B, s); break;
    case 7: launch_k<S, 7>(a, B, s); break;
    case 11: launch_k<S, 11>(a, B, s); break;
    default: throw Error(3, "conv1d(winograd8): kernel size must be 3, 7 or 11");
  }
}
}  // namespace wino8_detail

}  // namespace tts
