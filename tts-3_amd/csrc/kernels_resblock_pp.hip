// Fused ResBlock1 iteration (TTS/vocoder/models/hifigan_generator.py:93-98) at C in {32, 64},
// ping-pong form (gfx950):
//   xt = lrelu(convs1[m](lrelu(x, 0.1)), 0.1);   x' = convs2[m](xt) + x   [+ MRF z, :255-261]
//
// resblock_pair_kernel (kernels_resblock.hip) runs convs1 and then convs2 of one tile on the same
// four waves.  Every wave of a workgroup reaches the prologue (input window from HBM), the
// convs1 -> xt hand-off (block max, split, LDS stores, three barriers) and the epilogue
// (residual / MRF gathers from HBM) at the same time, so the matrix pipe idles through all of
// them; at 32 and 64 channels that is half of a tile's time (MFMA busy 28-45%).
//
// Here one persistent workgroup of eight waves walks a list of tiles as two groups, waves 0-3
// (group A: convs1) and waves 4-7 (group B: convs2); wave w and w + 4 share a SIMD.  The groups
// alternate between their MFMA phase and their LDS / memory phase, half a period apart, so the
// matrix pipe always has one group's MFMAs.  A period has two workgroup barriers:
//   phase 1   A: convs1(p) MFMAs (the raw window of tile p + 1 is requested PD steps before the
//                end), lrelu, bias, edge zeros, wave max -> red
//             B: epilogue of tile p - 2 (bias, residual, MRF sum, statistics, stores), then the
//                first K1 steps of convs2(p - 1)
//   --- barrier 1 ---
//   phase 2   A: block max -> xt(p) scale, split xt(p) into LDS buffer p & 1, split the window of
//                tile p + 1 into X
//             B: the other steps of convs2(p - 1) from buffer (p - 1) & 1 (its residual
//                requested PD steps before the end)
//   --- barrier 2 ---
// The HBM requests of a group are issued after its last weight load of the phase (the vector
// memory counter retires in order: a weight wait behind an HBM load would stall the step loop);
// the first weight steps of a group's next MFMA phase are requested once those have landed.
// The translation unit builds with -fno-slp-vectorize: packed fp32 VALU (v_pk_mul_f32 ...)
// issued beside the other group's MFMAs costs ~25 cycles each (MI355X_MICROARCH.md).
//
// Arithmetic per tile is the one of resblock_pair_kernel: the f16x3 scale of xt is the tile's own
// power of two (block max over its RP_W columns, exact and batch-invariant); the input scale is
// the producer's per-utterance statistic.  Tiles are RP_W = 128 (C = 64) or 256 (C = 32) columns
// with (K - 1) / 2 halo columns on each side (RP_BN = RP_W - (K - 1) outputs).
#include <algorithm>
#include <cstdlib>

#include "split_device.hpp"

namespace tts {

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#ifndef PP_ABLATE
#define PP_ABLATE 0  // diagnostic builds only: 1 = no window loads (stale X), 2 = no epilogue stores
#endif
#ifndef PP_BPD
#define PP_BPD 1  // B-operand LDS reads issued this many steps ahead (2 measured no better)
#endif
#ifndef PP_K1
#define PP_K1 0  // convs2 steps in phase 1 (0: NS / 2)
#endif
#ifndef PP_PD
#define PP_PD 4  // weight prefetch distance: each group's MFMA phase runs alone on the matrix pipe
#endif

#ifndef PP_STAMPS
#define PP_STAMPS 0  // diagnostic builds: s_memtime per phase of periods 8..23 of workgroups 0..7
#endif
#if PP_STAMPS
__device__ unsigned long long g_pp_stamps[8][16][8][8];  // [workgroup][period - 8][wave][slot]
#endif
// the C = 64, K = 11 launches without the MRF gather record (the last one wins)
#define PPST(i)                                                                                      \
  do {                                                                                               \
    if constexpr (PP_STAMPS && C == 64 && K == 11 && !ZG) {                                          \
      if (lane == 0 && blockIdx.x < 8 && p >= 8 && p < 24)                                           \
        g_pp_stamps_ref[blockIdx.x][p - 8][wave][i] = __builtin_amdgcn_s_memtime();                  \
    }                                                                                                \
  } while (0)

template <class S, int K, int C>
struct PPCfg {
  static constexpr int WM = C / 32;           // 32-row blocks per group
  static constexpr int WN = 4 / WM;           // column groups per group
  static constexpr int TN = 2;                // 32-column blocks per wave
  static constexpr int RP_W = WN * TN * 32;   // 256 (C = 32) / 128 (C = 64)
  static constexpr int LEAD = (K - 1) / 2;
  static constexpr int RP_BN = RP_W - 2 * LEAD;
  static constexpr int NC = C / 16;           // 16-channel groups
  static constexpr int HMAX = (K - 1) * 5;    // dilation <= 5
  // window rows: RP_W + HMAX (one per frame), or (V4 form) from the frame rounded down to a
  // multiple of 4, so that every lane loads 4 aligned frames of one channel with one dwordx4
  static constexpr int XROWS4 = (RP_W + HMAX + 3 + 3) / 4 * 4;
  static constexpr int NQ = XROWS4 / 4;                       // frame quads per channel (V4)
  static constexpr int UPT4 = (NC * 16 * NQ + 255) / 256;    // dwordx4 units per A lane (V4)
  static constexpr int XROWS = XROWS4;
  static constexpr int XSZB = XROWS * S::ROWB;  // X: one 16-channel group
  static constexpr int TROWS = RP_W + 16;     // xt rows (convs2 reads RP_W + K - 2 at most)
  static constexpr int TGB = TROWS * S::ROWB; // xt: one 16-channel group
  static constexpr int XB = NC * XSZB;
  static constexpr int TB = NC * TGB;
  static constexpr int LDSB = XB + 2 * TB;    // X + two xt buffers
  static constexpr int UPT = (XROWS * 4 + 255) / 256;  // window units (row, channel quad) per A lane
  static constexpr int NS = NC * K;           // MFMA steps per conv
  static constexpr int PD = PP_PD < NS ? PP_PD : NS - 1;  // weight prefetch distance (steps)
  static_assert(K - 2 < 16, "xt rows");
  static_assert(PD < NS, "prefetch distance");
  // convs2 steps group B runs in phase 1 (beside group A's convs1), the rest in phase 2; the
  // residual request (step NS - PD) must fall in phase 2
  static constexpr int K1A = PP_K1 > 0 ? PP_K1 : NS / 2;
  static constexpr int K1 = K1A < NS - PD ? K1A : NS - PD;
  static_assert(LDSB <= 160 * 1024 - 1024, "LDS");
};

template <class S, int K, int C, bool ZG, bool V4>
__global__ __launch_bounds__(512) void resblock_pp_kernel(ResPairArgs pa, int ntx, int ntiles) {
  using P = PPCfg<S, K, C>;
  constexpr int NP = S::NP;
  constexpr bool H3 = S::SCALED;
  constexpr int TN = P::TN, NC = P::NC, NS = P::NS, PD = P::PD, RP_W = P::RP_W, RP_BN = P::RP_BN;
  __shared__ __attribute__((aligned(16))) unsigned char smem[P::LDSB];
  __shared__ float red[4];
  __shared__ int etsm[2];
  __shared__ float bsm[2 * C];  // convs1 / convs2 biases

  const Conv1dArgs& a1 = pa.c1;
  const Conv1dArgs& a2 = pa.c2;
#if PP_STAMPS
  auto& g_pp_stamps_ref = g_pp_stamps;
#else
  unsigned long long (*g_pp_stamps_ref)[16][8][8] = nullptr;
#endif
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;  // 0: convs1 (A), 1: convs2 (B)
  const int gw = wave & 3;
  const int wm = gw / P::WN;
  const int wn = gw % P::WN;
  const int mrow0 = wm * 32;
  const int xrow0 = wn * TN * 32 + l32;  // this lane's column of block n = 0
  const int d = a1.dil;
  const int T = a1.Tout;
  const unsigned chb = (unsigned)T * 4u;
  const int G = gridDim.x;
  const int nloc = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / G + 1 : 0;
  const unsigned avoff = (unsigned)lane * 16u;
  int lane_off = xrow0 * S::ROWB + 16 * half;
  auto tile_id = [&](int p) { return (int)blockIdx.x + p * G; };

  if (tid < C) {
    bsm[tid] = a1.bias[tid];
    bsm[C + tid] = a2.bias[tid];
  }

  // ---- per-group weight stream (32-row block wm of convs1 / convs2) ----
  const rsrc_t ra = make_rsrc((grp == 0 ? a1.w : a2.w) + ((size_t)wm * NC * K) * (NP * 256), 0xFFFFFFFFu);
  // B operands: bq[0] = this step, bq[j] = step + j (LDS reads BPD steps ahead: a group's MFMA
  // phase runs alone on its SIMDs, so one step of MFMAs must cover an LDS read's latency)
  constexpr int BPD = PP_BPD;
  f32x4 ar[PD + 1][NP], bq[BPD + 1][TN][NP];
  f32x16 acc[TN];

  // B operand of step s (group c = s / K, tap k = s % K): rows xrow0 + n*32 + k*kstride of
  // region base + c*gstride
  // The lane's row offset is laundered once per use site group (lane_off) so that the compiler
  // cannot hoist the 2 * NS step addresses out of the period loop (they would stay live in VGPRs
  // across it); every step then adds wave-uniform and immediate offsets only.
  auto read_b = [&](const unsigned char* base, int gstride, int kstride, int s, f32x4 (*dst)[NP]) {
    const int c = s / K, k = s - (s / K) * K;
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      const unsigned char* p = base + lane_off + c * gstride + (n * 32 + k * kstride) * S::ROWB;
#pragma unroll
      for (int q = 0; q < NP; ++q) dst[n][q] = *reinterpret_cast<const f32x4*>(p + 32 * q);
    }
  };
  // one MFMA step s: weights of step s + PD (the last PD steps load none: the next period's
  // first steps are requested by prefetch_w after the period's HBM loads have landed), the next
  // B operand, the products; `hook` runs right before the weight load of step s
  auto prefetch_w = [&]() {
#pragma unroll
    for (int s = 0; s < PD; ++s)
#pragma unroll
      for (int q = 0; q < NP; ++q) ar[s][q] = bload4(ra, avoff, (unsigned)(s * NP + q) * 1024u);
  };
  auto step = [&](const unsigned char* base, int gstride, int kstride, int s, auto&& hook) {
    hook(s);
    if (s + PD < NS) {
#pragma unroll
      for (int q = 0; q < NP; ++q) ar[PD][q] = bload4(ra, avoff, (unsigned)(((s + PD) * NP + q) * 1024u));
    }
    if (s + BPD < NS) read_b(base, gstride, kstride, s + BPD, bq[BPD]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int e = 0; e < S::NPROD; ++e)
#pragma unroll
      for (int n = 0; n < TN; ++n) acc[n] = S::mfma(ar[0][S::PA[e]], bq[0][n][S::PB[e]], acc[n]);
#pragma unroll
    for (int pp = 0; pp < PD; ++pp)
#pragma unroll
      for (int q = 0; q < NP; ++q) ar[pp][q] = ar[pp + 1][q];
#pragma unroll
    for (int j = 0; j < BPD; ++j)
      if (s + 1 + j < NS) {
#pragma unroll
        for (int n = 0; n < TN; ++n)
#pragma unroll
          for (int q = 0; q < NP; ++q) bq[j][n][q] = bq[j + 1][n][q];
      }
  };

  // ---- group A: the input window of a tile (raw fp32 in registers, then split into X) ----
  // V4 (T % 4 == 0): lane unit = (16-channel group, channel, frame quad): one dwordx4 of 4 frames,
  // stored as 4 rows x 2-byte pieces; X row r holds frame fa + r with fa the window start rounded
  // down to a multiple of 4, and the MFMA reads shift by roff = start - fa.  Otherwise: unit =
  // (row, channel quad), 4 dword loads of 4 channels, one u16x4 store per piece.
  const int ta = tid & 255;
  constexpr int UPW = V4 ? P::UPT4 : NC * P::UPT;
  f32x4 xraw[UPW];
  int roff_next = 0;
  auto load_window = [&](int p) {
    const int id = tile_id(p);
    const int b = id / ntx;
    const int tx0 = (id - b * ntx) * RP_BN - P::LEAD;
    const float* xb = a1.x + (size_t)b * C * T;
    if constexpr (V4) {
      const int a0 = tx0 - a1.pad;
      const int fa = a0 - (((a0 % 4) + 4) % 4);
      roff_next = a0 - fa;
      const rsrc_t rx = make_rsrc(xb, (unsigned)C * chb);
#pragma unroll
      for (int i = 0; i < UPW; ++i) {
        const int u = ta + i * 256;
        const int c16 = u & 15, rest = u >> 4;
        const int g = rest / P::NQ, tq = rest - (rest / P::NQ) * P::NQ;
        const int ts = fa + 4 * tq;
        const bool ok = g < NC && ts >= 0 && ts < T;  // whole quads: fa and T are multiples of 4
        unsigned vo = ok ? (unsigned)(16 * g + c16) * chb + (unsigned)ts * 4u : OOB_OFF;
        asm volatile("" : "+v"(vo));
        xraw[i] = bload4(rx, vo, 0u);
      }
    } else {
      const int XW = RP_W + (K - 1) * d;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const rsrc_t rx = make_rsrc(xb + (size_t)c * 16 * T, (unsigned)(C - c * 16) * chb);
#pragma unroll
        for (int i = 0; i < P::UPT; ++i) {
          const int u = ta + i * 256;
          const int q = u & 3, r = u >> 2;
          const int ts = tx0 - a1.pad + r;
          const bool ok = r < XW && ts >= 0 && ts < T;
          // OOB_OFF + 3 * chb stays >= 2^31 (planes < 2 GiB): still out of range.  Laundered: the
          // compiler otherwise splits the loads into exec-masked branches on vo == OOB_OFF
          unsigned vo = ok ? (unsigned)(4 * q) * chb + (unsigned)ts * 4u : OOB_OFF;
          asm volatile("" : "+v"(vo));
#pragma unroll
          for (int j = 0; j < 4; ++j) xraw[c * P::UPT + i][j] = bload(rx, vo + (unsigned)j * chb, 0u);
        }
      }
    }
  };
  auto store_window = [&](int ex) {
    const float xs = H3 ? ldexpf(1.f, -ex) : 1.f;
    if constexpr (V4) {
#pragma unroll
      for (int i = 0; i < UPW; ++i) {
        const int u = ta + i * 256;
        const int c16 = u & 15, rest = u >> 4;
        const int g = rest / P::NQ, tq = rest - (rest / P::NQ) * P::NQ;
        if (g < NC) {
          unsigned char* dst = smem + g * P::XSZB + (4 * tq) * S::ROWB + 2 * c16;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            unsigned short h[NP];
            float v = lrelu2(xraw[i][j], a1.in_slope);
            if (H3) v *= xs;
            S::split(v, h);
#pragma unroll
            for (int pq = 0; pq < NP; ++pq) *reinterpret_cast<unsigned short*>(dst + j * S::ROWB + 32 * pq) = h[pq];
          }
        }
      }
    } else {
      const int XW = RP_W + (K - 1) * d;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < P::UPT; ++i) {
          const int u = ta + i * 256;
          const int q = u & 3, r = u >> 2;
          if (r < XW) {
            u16x4 pv[NP];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              unsigned short h[NP];
              float v = lrelu2(xraw[c * P::UPT + i][j], a1.in_slope);
              if (H3) v *= xs;
              S::split(v, h);
#pragma unroll
              for (int pq = 0; pq < NP; ++pq) pv[pq][j] = h[pq];
            }
#pragma unroll
            for (int pq = 0; pq < NP; ++pq)
              *reinterpret_cast<u16x4*>(smem + c * P::XSZB + r * S::ROWB + 8 * q + 32 * pq) = pv[pq];
          }
        }
    }
  };

  // ---- group B: epilogue gathers (residual x, MRF z) of tile p and the store ----
  const unsigned rowb = chb;
  float rv[TN][16], zv[TN][16];
  auto b_tile = [&](int p, int& b, int& t0) {
    const int id = tile_id(p);
    b = id / ntx;
    t0 = (id - b * ntx) * RP_BN;
  };
  auto b_voff = [&](int t0, int n) -> unsigned {
    const int t = t0 + wn * TN * 32 + n * 32 + l32;
    const bool tok = t < T && t < t0 + RP_BN;
    return tok ? ((unsigned)(mrow0 + 4 * half) * (unsigned)T + (unsigned)t) * 4u : OOB_OFF;
  };
  auto gather = [&](int p, bool res, bool zz) {
    int b, t0;
    b_tile(p, b, t0);
    const size_t item = (size_t)b * C * T;
    const unsigned plane = (unsigned)C * chb;
    const rsrc_t rres = make_rsrc(a2.res + item, plane);
    const rsrc_t rz = make_rsrc(ZG ? a2.z + item : a2.bias, ZG ? plane : 0u);
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      // OOB_OFF + 31 rows stays >= 2^31 > the plane (C >= 32, plane < 2 GiB): out of range
      unsigned voff = b_voff(t0, n);
      asm volatile("" : "+v"(voff));
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const unsigned vo = voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb;
        if (res) rv[n][r] = bload(rres, vo, 0u);
        if (ZG && zz) zv[n][r] = bload(rz, vo, 0u);
      }
    }
  };

  // ---- prologue: X(0), the first weight steps ----
  // the f16x3 input exponent of a tile's utterance: the producer's 64 slots are read at the start
  // of the period before (one lane each) and reduced after barrier 1 (amax_exp without its wait)
  auto slot_load = [&](int p) -> float {
    if (!H3 || !a1.amax_in) return 0.f;
    return __uint_as_float(a1.amax_in[(size_t)(tile_id(p) / ntx) * 64 + lane]);
  };
  auto slot_exp = [&](float m) -> int {
    if (!H3 || !a1.amax_in) return 0;
    m = wave_max(m);
    int e = 0;
    if (m > 0.f && m < INFINITY) {
      int E;
      (void)frexpf(m, &E);
      e = E - 14;
    }
    return __builtin_amdgcn_readfirstlane(e);
  };
  int roff = 0;  // X row of the window's first frame (V4)
  if (grp == 0 && nloc > 0) {
    load_window(0);
    store_window(slot_exp(slot_load(0)));
    roff = roff_next;
  }
  prefetch_w();
  __syncthreads();

  // epilogue of group B's tile p: v = acc * 2^(et + w_exp) + bias (+ x) [MRF z]; the residual was
  // requested PD steps before the end of its MFMA phase, the MRF sums are requested here
  auto b_epilogue = [&](int p) {
    gather(p, false, true);
    int b, t0;
    b_tile(p, b, t0);
    const int et = etsm[p & 1];
    const float sc2 = H3 ? ldexpf(1.f, et + a2.w_exp) : 1.f;
    const size_t item = (size_t)b * C * T;
    const unsigned plane = (unsigned)C * chb;
    const rsrc_t rout = make_rsrc((a2.zmode == 0 ? a2.y : a2.z) + item, plane);
    const float oslope = a2.out_slope;
    const float zdiv = a2.zdiv;
    const bool zdivide = a2.zmode == 3;
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) bv[r] = bsm[C + mrow0 + (r & 3) + 8 * (r >> 2) + 4 * half];
    float vmax = 0.f;
#pragma unroll
    for (int n = 0; n < TN; ++n) {
      unsigned voff = b_voff(t0, n);
      const bool tok = voff != OOB_OFF;
      asm volatile("" : "+v"(voff));
      float vm = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = acc[n][r] * sc2 + bv[r];
        v = lrelu2(v, oslope);
        v = v + rv[n][r];
        if (ZG) v = zdivide ? (zv[n][r] + v) / zdiv : zv[n][r] + v;
        vm = fmaxf(vm, fabsf(v));
        if (!(PP_ABLATE & 2)) bstore(rout, v, voff + (unsigned)((r & 3) + 8 * (r >> 2)) * rowb, 0u);
      }
      if (tok) vmax = fmaxf(vmax, vm);
    }
    if (H3 && a2.amax_out) publish_amax(a2.amax_out, b, vmax);
  };

  // nloc + 2 periods: group A's MFMA phase runs tiles 0 .. nloc-1 in periods 0 .. nloc-1, group B's
  // tiles 0 .. nloc-1 in periods 1 .. nloc, B's last epilogue is in period nloc + 1
  if (grp == 0) {
    // ================================ group A: convs1 ================================
    int ex = nloc > 0 ? slot_exp(slot_load(0)) : 0;
    for (int p = 0; p <= nloc + 1; ++p) {
      asm volatile("" : "+v"(lane_off));
      const bool cur = p < nloc, more = p + 1 < nloc;
      float slot_next = 0.f;
      int ex_next = 0;
      PPST(0);
      // ---- phase 1: convs1 of tile p (group B runs its epilogue) ----
      if (cur) {
        // unconditional loads (the last tile re-reads its own slots / window): a branch around
        // them would leave the wait-count pass two paths to merge, and it then waits for every
        // outstanding load at the next weight use
        slot_next = slot_load(more ? p + 1 : p);
        const int id = tile_id(p);
        const int b = id / ntx;
        const int tx0 = (id - b * ntx) * RP_BN - P::LEAD;
#pragma unroll
        for (int n = 0; n < TN; ++n) acc[n] = f32x16{};
#pragma unroll
        for (int j = 0; j < BPD; ++j) read_b(smem + roff * S::ROWB, P::XSZB, d, j, bq[j]);
        // the next tile's window after the period's last weight load
        auto hook = [&](int s) {
          if (!(PP_ABLATE & 1) && s == NS - PD) load_window(more ? p + 1 : p);
        };
#pragma unroll
        for (int s = 0; s < NS; ++s) step(smem + roff * S::ROWB, P::XSZB, d, s, hook);
        PPST(1);
        // lrelu(acc * 2^(ex + w_exp) + bias), zero outside [0, T) (convs2's zero padding)
        const float sc1 = H3 ? ldexpf(1.f, ex + a1.w_exp) : 1.f;
        float tmax = 0.f;
        float bv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[r] = bsm[mrow0 + (r & 3) + 8 * (r >> 2) + 4 * half];
#pragma unroll
        for (int n = 0; n < TN; ++n) {
          const int t = tx0 + xrow0 + n * 32;
          const bool inside = t >= 0 && t < T;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float v = lrelu2(acc[n][r] * sc1 + bv[r], a1.out_slope);
            v = inside ? v : 0.f;
            acc[n][r] = v;
            tmax = fmaxf(tmax, fabsf(v));
          }
        }
        tmax = wave_max(tmax);
        if (lane == 0) red[gw] = tmax;
        ex_next = slot_exp(slot_next);
      }
      PPST(2);
      lds_barrier();  // -------------------------------------------- barrier 1
      PPST(3);
      // ---- phase 2: xt(p) and the window of tile p + 1 into LDS (group B runs convs2(p - 1)) ----
      if (cur) {
        int et = 0;
        if (H3) {
          const float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
          if (mx > 0.f && mx < INFINITY) {
            int E;
            (void)frexpf(mx, &E);
            et = E - 14;
          }
        }
        const float tscale = H3 ? ldexpf(1.f, -et) : 1.f;
        unsigned char* xt = smem + P::XB + (p & 1) * P::TB;
        // xt pieces: row = column, group = co / 16; registers r, r + 1 (r even) are channels co, co + 1
#pragma unroll
        for (int n = 0; n < TN; ++n) {
          const int row = xrow0 + n * 32;
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const int co = mrow0 + (r & 3) + 8 * (r >> 2) + 4 * half;
            unsigned short h0[NP], h1[NP];
            S::split(acc[n][r] * tscale, h0);
            S::split(acc[n][r + 1] * tscale, h1);
            unsigned char* dst = xt + (co >> 4) * P::TGB + row * S::ROWB + 2 * (co & 15);
#pragma unroll
            for (int q = 0; q < NP; ++q) *reinterpret_cast<unsigned*>(dst + 32 * q) = (unsigned)h0[q] | ((unsigned)h1[q] << 16);
          }
        }
        // rows RP_W .. TROWS - 1 of every group: read only by the discarded columns
        constexpr int ZB = (P::TROWS - RP_W) * S::ROWB;
        for (int e = ta * 16; e < NC * ZB; e += 256 * 16) {
          const int g = e / ZB;
          *reinterpret_cast<f32x4*>(xt + g * P::TGB + RP_W * S::ROWB + (e - g * ZB)) = f32x4{};
        }
        if (ta == 0) etsm[p & 1] = et;
        PPST(4);
        if (more) {
          ex = ex_next;
          store_window(ex);
          roff = roff_next;
          PPST(5);
          prefetch_w();
        }
      }
      PPST(6);
      lds_barrier();  // -------------------------------------------- barrier 2
      PPST(7);
    }
  } else {
    // ================================ group B: convs2 ================================
    for (int p = 0; p <= nloc + 1; ++p) {
      asm volatile("" : "+v"(lane_off));
      const bool cur = p >= 1 && p <= nloc;
      const unsigned char* xt = smem + P::XB + ((p - 1) & 1) * P::TB;
      PPST(0);
      // ---- phase 1: epilogue of tile p - 2, then the first K1 steps of convs2(p - 1)
      //      (group A runs convs1(p)) ----
      if (p >= 2) {
        b_epilogue(p - 2);
        prefetch_w();
      }
      if (cur) {
#pragma unroll
        for (int n = 0; n < TN; ++n) acc[n] = f32x16{};
#pragma unroll
        for (int j = 0; j < BPD; ++j) read_b(xt, P::TGB, 1, j, bq[j]);
        auto nohook = [&](int) {};
#pragma unroll
        for (int s = 0; s < P::K1; ++s) step(xt, P::TGB, 1, s, nohook);
      }
      PPST(2);
      lds_barrier();  // -------------------------------------------- barrier 1
      PPST(3);
      // ---- phase 2: the rest of convs2(p - 1) from buffer (p - 1) & 1 (group A writes LDS) ----
      if (cur) {
        // the residual after the last weight load; it lands during barrier 2 / the next phase 1
        auto hook = [&](int s) {
          if (s == NS - PD) gather(p - 1, true, false);
        };
#pragma unroll
        for (int s = P::K1; s < NS; ++s) step(xt, P::TGB, 1, s, hook);
      }
      PPST(4);
      PPST(6);
      lds_barrier();  // -------------------------------------------- barrier 2
      PPST(7);
    }
  }
}

namespace {
int num_cus() {
  static int n[64] = {};
  int dev = 0;
  TTS_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) dev = 0;
  if (n[dev] == 0) {
    int v = 0;
    TTS_HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev));
    n[dev] = v > 0 ? v : 256;
  }
  return n[dev];
}

template <class S, int K, int C>
void launch_pp_t(const ResPairArgs& a, int B, hipStream_t s) {
  using P = PPCfg<S, K, C>;
  const int ntx = ceil_div(a.c1.Tout, P::RP_BN);
  const int64_t nt = (int64_t)ntx * B;
  TTS_REQUIRE(nt < (int64_t(1) << 30), 3, "resblock pair: too many tiles");
  const int ntiles = (int)nt;
  const int grid = std::min(ntiles, num_cus());
  // V4 window loads need whole frame quads: T % 4 == 0 (every HiFiGAN stage at T' % 4 == 0... and
  // the bench shapes); TTS_MI355X_PP_V4=0 keeps the dword form (A/B runs)
  static const bool v4on = [] {
    const char* e = std::getenv("TTS_MI355X_PP_V4");
    return !(e && e[0] == '0');
  }();
  const bool v4 = v4on && a.c1.Tout % 4 == 0;
  const bool zg = a.c2.zmode >= 2;
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, s, a, ntx, ntiles); };
  if (zg && v4) go(resblock_pp_kernel<S, K, C, true, true>);
  else if (zg) go(resblock_pp_kernel<S, K, C, true, false>);
  else if (v4) go(resblock_pp_kernel<S, K, C, false, true>);
  else go(resblock_pp_kernel<S, K, C, false, false>);
}

template <class S, int K>
void launch_pp_k(const ResPairArgs& a, int B, int C, hipStream_t s) {
  if (C == 32) launch_pp_t<S, K, 32>(a, B, s);
  else launch_pp_t<S, K, 64>(a, B, s);
}

template <class S>
void launch_pp_s(const ResPairArgs& a, int B, int K, int C, hipStream_t s) {
  switch (K) {
    case 3: launch_pp_k<S, 3>(a, B, C, s); break;
    case 7: launch_pp_k<S, 7>(a, B, C, s); break;
    case 11: launch_pp_k<S, 11>(a, B, C, s); break;
    default: throw Error(3, "resblock pair (ping-pong): kernel size must be 3, 7 or 11");
  }
}
}  // namespace

// f16x3 and bf16 (the bf16x6 rows, 112 B, do not fit X and two xt buffers in LDS).  Opt-in
// (TTS_MI355X_PAIR_PP=1, read at the first launch): on MI355X it measured within a few percent of
// resblock_pair_kernel at two workgroups per CU, slower at C = 64, K = 11
bool resblock_pp_enabled(int mode, int C, int K) {
  static const bool on = [] {
    const char* e = std::getenv("TTS_MI355X_PAIR_PP");
    return e && e[0] == '1';
  }();
  return on && (mode == MATH_FP32_F16X3 || mode == MATH_BF16) && (C == 32 || C == 64) &&
         (K == 3 || K == 7 || K == 11);
}

#if PP_STAMPS
extern "C" int tts_debug_pp_stamps(void* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pp_stamps), sizeof(g_pp_stamps)) == hipSuccess ? 0 : 2;
}
#endif

void launch_resblock_pp(int mode, const ResPairArgs& a, int B, int K, int C, hipStream_t s) {
  if (mode == MATH_FP32_F16X3) launch_pp_s<SchemeH3>(a, B, K, C, s);
  else if (mode == MATH_BF16) launch_pp_s<SchemeB1>(a, B, K, C, s);
  else throw Error(3, "resblock pair (ping-pong): f16x3 / bf16 only");
  TTS_HIP_CHECK(hipGetLastError());
}

}  // namespace tts
