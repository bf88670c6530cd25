// One-dimensional Winograd F(2,3) along x for the stride-1 3x3 convs of stock HardNet
// (hardnet/HardNet.py:290-291 conv3: 64 -> 64 at 16x16, :296-297 conv5: 128 -> 128 at 8x8; BN
// folded into the weights, ReLU fused).  Per output row y and column pair (2t, 2t+1), with
// d_k = x[y + ky - 1][2t - 1 + k] (zero outside the patch):
//   V0 = d0 - d2,  V1 = d1 + d2,  V2 = d2 - d1,  V3 = d1 - d3              (B^T d)
//   U_xi[ky] = sum_kx G[xi][kx] W[ky][kx],  G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]
//   m_xi = sum_{ky, ci} V_xi[y + ky][t][ci] U_xi[ky][ci][co]                 (4 GEMMs, K = 3 CIN)
//   out[y][2t] = m0 + m1 + m2,  out[y][2t+1] = m1 - m2 - m3                 (A^T m)
// 12 multiplies per output pair and input channel instead of 18: the MFMA work of the two layers
// drops by a third.  The 2-D F(2x2,3x3) form (hn_wino.hip, experiments only) needs 16 transform
// positions per 2x2 tile -- a 3.2x larger operand image than the input window and the input
// transform in the MFMA waves -- and measured slower than the direct kernels; the 1-D form's
// image is 1.8x the window and its transform runs in the producer waves, beside the loads they
// already issue.
//
// The kernel is k_conv_ws's warp-specialised loop (hn_hardnet.hip): 4 producer waves stage the
// next 32-channel chunk of a work tile while the MFMA waves run the current one; the producers
// load 4 input columns per output column pair, form V in fp32 and split it to bf16 hi / lo
// (bf16x3 products, hn_common.h mfma3).  The MFMA waves accumulate m0 into out[2t] and -m3 into
// out[2t+1] directly (U3 is packed negated) and m1 / m2 in a third accumulator folded into both
// after their K-steps.  Operand image per plane: [patch][window row wr][xi][t][32 channels bf16],
// 64 bytes per position, 16-byte chunk q at q ^ (wr & 3): a 32x32x16 operand read (one M tile =
// 32 / NTX consecutive rows x NTX column pairs) and a producer's 8-lane store group are
// bank-conflict free (tests/test_lds_banks.py).
#include <cstdlib>

#include "hn_common.h"
#include "hn_internal.h"

namespace {

// Work tile = NP whole patches (every window row above / below the patch is padding, so the image
// holds the H real rows of each patch and ONE zero row per plane that the padding reads point at).
// CST: the epilogue goes through a per-wave LDS scratch so that each store writes 8 whole 128-byte
// pixel slices (k_conv_ws's CST), one output column parity at a time.
template <int CIN, int COUT, int H, int NP, int WM, int WN, bool CST>
struct W1Cfg {
  static constexpr int TR = H;              // output rows per work tile (whole patches)
  static constexpr int NTX = H / 2;         // output column pairs per row
  static constexpr int BM = NP * TR * NTX;  // GEMM M (output row x column pair) per work tile
  static constexpr int MT = BM / WM / 32, NT = COUT / WN / 32;
  static constexpr int NTOT = COUT / 32, NCC = CIN / 32;
  static constexpr int XROW = NTX * 64;  // bytes of one (row, xi) run of positions per plane
  static constexpr int RS = 4 * XROW;    // bytes per image row per plane
  static constexpr int PS = TR * RS;     // per patch per plane
  static constexpr int ZROW = NP * PS;   // the zero row (offset within a plane)
  static constexpr int PLANE = ZROW + RS;
  static constexpr int BUF = 2 * PLANE;
  static constexpr int NWC = WM * WN, NWP = 4, NTHR = (NWC + NWP) * 64, PTHR = NWP * 64;
  static constexpr int UNITS = NP * TR * NTX * 4;  // (patch, row, column pair, 8-channel group)
  static_assert(64 % (4 * NTX) == 0 && PTHR % (4 * NTX) == 0, "a row's units share one wave");
  static constexpr int UPT = (UNITS + PTHR - 1) / PTHR;
  static constexpr bool DEEP = UPT <= 2;  // two stages of loads in flight
  static constexpr int SROW = 36;                       // CST: floats per pixel slice of the scratch
  static constexpr int SCR_OFF = 2 * BUF;
  static constexpr int SCR = CST ? 32 * SROW * 4 : 0;   // CST: one 32-pixel x 32-channel tile per MFMA wave
  static constexpr int BIAS_OFF = SCR_OFF + NWC * SCR;
  static constexpr int SMEM = BIAS_OFF + COUT * 4;
  static constexpr int NKS = 24;  // K-steps per stage: 4 xi x 3 ky x 2 halves of 16 channels
  static constexpr unsigned CHUNK_BYTES = NKS * NTOT * 2 * 64 * 16;
  static_assert(SMEM <= 160 * 1024, "LDS");
  static_assert(MT >= 1 && NT >= 1 && MT * WM * 32 == BM && NT * WN * 32 == COUT, "tiling");
  static_assert((TR * NTX) % 32 == 0 && 32 % NTX == 0, "an M tile = 32 / NTX whole rows of one patch");
  static_assert(RS % 256 == 0, "image rows on 256-byte boundaries (the bank-conflict argument)");
};

// ABL (timing-only ablation builds, HN_EXPERIMENTS library only; wrong results): bit 0 idle producers
// (barriers only), bit 1 no MFMAs (operands still loaded), bit 2 no weight loads (K-step 0's fragments
// reused), bit 3 no epilogue stores, bit 4 idle MFMA waves, bit 5 no weight loads after the prologue
template <int CIN, int COUT, int H, int NP, int WM, int WN, bool CST, int WD = 3, int ABL = 0>
__global__ __launch_bounds__((WM * WN + 4) * 64) void k_conv_w1(const float* __restrict__ in, float* __restrict__ out,
                                                                const uint4* __restrict__ wp,
                                                                const float* __restrict__ bias, int P) {
  using C = W1Cfg<CIN, COUT, H, NP, WM, WN, CST>;
  constexpr int TR = C::TR;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wave >= C::NWC;
  const int r = lane & 31, h = lane >> 5;
  const int nwg = gridDim.x, rb = xcd_remap(blockIdx.x, nwg);
  const int ntiles = (P + NP - 1) / NP;
  const int my_tiles = rb < ntiles ? (ntiles - 1 - rb) / nwg + 1 : 0;
  const int NS = my_tiles * C::NCC;
  if (NS == 0) return;
  char* const buf0 = smem;
  char* const buf1 = smem + C::BUF;
  auto tile_of = [&](int s) { return (rb + (s / C::NCC) * nwg) * NP; };  // first patch of stage s's tile

  // ---- producer side ----
  // A unit (patch, window row, column pair t, 8-channel group) loads input columns 2t - 1 and 2t (the
  // last pair also column W - 1); d2 / d3 are the next pair's loads, taken from lane + 4 (a window
  // row's units are 4 NTX consecutive lanes of one wave) -- no pixel is loaded twice
  const int ptid = tid - C::NWC * 64;
  float4 pf[C::UPT][6], pf2[C::UPT][6];
  // Loads are buffer loads over the stage's tile: a padding column, an absent third column or a patch
  // past P gets an offset beyond the resource and reads zero in hardware. No branch, so the compiler's
  // vmcnt accounting stays exact and stage s + 1's write waits only for stage s + 1's loads (with
  // if-guarded global loads it waited vmcnt(0), i.e. also for the stage s + 2 loads just issued).
  constexpr unsigned PATCH_BYTES = (unsigned)H * H * CIN * 4, OOB = 0x80000000u;
  auto produce_loads = [&](int s, float4 (&d)[C::UPT][6]) {
    // a stage past the last one (the loops below issue it unconditionally) gets an empty resource
    const bool live = s < NS;
    const int p0 = live ? tile_of(s) : 0;
    const int cc = s % C::NCC;
    const int nval = !live ? 0 : P - p0 < NP ? P - p0 : NP;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(in + (size_t)p0 * H * H * CIN, (unsigned)nval * PATCH_BYTES);
#pragma unroll
    for (int k = 0; k < C::UPT; ++k) {
      const int u = ptid + k * C::PTHR;
      const int g = u & 3, t = (u >> 2) % C::NTX, rest = (u >> 2) / C::NTX;
      const int y = rest % TR, np = rest / TR;
      const bool rowok = C::UNITS % C::PTHR == 0 || u < C::UNITS;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int x = 2 * t - 1 + j;
        const bool ok = rowok && (j < 2 || t == C::NTX - 1) && (unsigned)x < (unsigned)H;
        const unsigned vo = ok ? (unsigned)(((np * H + y) * H + x) * CIN + cc * 32 + g * 8) * 4u : OOB;
        d[k][2 * j] = __builtin_bit_cast(float4, buf_load16(rs, vo, 0));
        d[k][2 * j + 1] = __builtin_bit_cast(float4, buf_load16(rs, vo, 16));
      }
    }
  };
  auto shfl4 = [&](const float4& v) {
    return make_float4(__shfl_down(v.x, 4, 64), __shfl_down(v.y, 4, 64), __shfl_down(v.z, 4, 64),
                       __shfl_down(v.w, 4, 64));
  };
  auto produce_write = [&](char* dst, const float4 (&d)[C::UPT][6]) {
#pragma unroll
    for (int k = 0; k < C::UPT; ++k) {
      const int u = ptid + k * C::PTHR;
      const int g = u & 3, t = (u >> 2) % C::NTX, rest = (u >> 2) / C::NTX;
      const int y = rest % TR, np = rest / TR;
      const bool last = t == C::NTX - 1;
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      float4 dd[4][2];  // d0..d3, channels 0-3 / 4-7
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float4 n0 = shfl4(d[k][i]), n1 = shfl4(d[k][2 + i]);  // every lane joins the shuffles
        dd[0][i] = d[k][i];
        dd[1][i] = d[k][2 + i];
        dd[2][i] = last ? d[k][4 + i] : n0;
        dd[3][i] = last ? z : n1;
      }
      if (C::UNITS % C::PTHR == 0 || u < C::UNITS) {  // compile-time true for conv3 / conv5: no branch
        const int off = np * C::PS + y * C::RS + t * 64 + 16 * (g ^ ((y + 1) & 3));  // window row y + 1
#pragma unroll
        for (int xi = 0; xi < 4; ++xi) {
          float4 v[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const float4 d0 = dd[0][i], d1 = dd[1][i], d2 = dd[2][i], d3 = dd[3][i];
            if (xi == 0) v[i] = make_float4(d0.x - d2.x, d0.y - d2.y, d0.z - d2.z, d0.w - d2.w);
            if (xi == 1) v[i] = make_float4(d1.x + d2.x, d1.y + d2.y, d1.z + d2.z, d1.w + d2.w);
            if (xi == 2) v[i] = make_float4(d2.x - d1.x, d2.y - d1.y, d2.z - d1.z, d2.w - d1.w);
            if (xi == 3) v[i] = make_float4(d1.x - d3.x, d1.y - d3.y, d1.z - d3.z, d1.w - d3.w);
          }
          uint4 hi, lo;
          split8(v[0], v[1], hi, lo);
          *reinterpret_cast<uint4*>(dst + off + xi * C::XROW) = hi;
          *reinterpret_cast<uint4*>(dst + C::PLANE + off + xi * C::XROW) = lo;
        }
      }
    }
  };

  // the zero rows (both buffers, both planes): what every padding-row operand read returns
  for (int i = tid; i < 4 * C::RS / 16; i += C::NTHR) {
    const int q = i / (C::RS / 16), o = (i % (C::RS / 16)) * 16;
    *reinterpret_cast<uint4*>(smem + (q >> 1) * C::BUF + (q & 1) * C::PLANE + C::ZROW + o) = make_uint4(0, 0, 0, 0);
  }
  // the two roles split here and share no value: each matches the other's barriers one for one
  if constexpr ((ABL & 64) != 0) {  // A/B: the MFMA waves issue ahead of the producers
    if (!producer) __builtin_amdgcn_s_setprio(1);
  }
  if constexpr ((ABL & 128) != 0) {  // A/B: the producers issue ahead of the MFMA waves
    if (producer) __builtin_amdgcn_s_setprio(1);
  }
  if (producer) {
    if constexpr ((ABL & 1) != 0) {  // timing only: idle producers
#pragma unroll 1
      for (int s = 0; s <= NS; ++s) __syncthreads();
      return;
    }
    // Loads and writes are unconditional (a stage past NS loads zeros from an empty resource and is
    // written into the buffer nobody reads again): any branch around them makes the compiler's vmcnt
    // merge conservative, and a vmcnt(0) here also waits for the loads issued one stage ahead.
    produce_loads(0, pf);
    produce_write(buf0, pf);
    produce_loads(1, pf);
    __syncthreads();
    if constexpr (!C::DEEP) {
#pragma unroll 1
      for (int s = 0; s < NS; ++s) {
        produce_write((s & 1) ? buf0 : buf1, pf);
        produce_loads(s + 2, pf);
        __syncthreads();
      }
    } else {
      // stage s + 2's loads are issued before stage s + 1 is written: two stages of MFMA work to land
#pragma unroll 1
      for (int s = 0; s < NS; s += 2) {
        produce_loads(s + 2, pf2);
        produce_write(buf1, pf);
        __syncthreads();
        if (s + 1 >= NS) break;
        produce_loads(s + 3, pf);
        produce_write(buf0, pf2);
        __syncthreads();
      }
    }
    return;
  }

  // ---- MFMA side ----
  for (int i = tid; i < COUT; i += C::NWC * 64) reinterpret_cast<float*>(smem + C::BIAS_OFF)[i] = bias[i];
  __syncthreads();
  if constexpr ((ABL & 16) != 0) {  // timing only: idle MFMA waves (the producers alone)
#pragma unroll 1
    for (int s = 0; s < NS; ++s) __syncthreads();
    return;
  }
  const int wm = wave / WN, wn = wave % WN;
  const float* const sbias = reinterpret_cast<const float*>(smem + C::BIAS_OFF);
  // per-lane part of an operand address: M tile mt's position + its swizzled chunk for (ky, ks); the
  // K-step's xi / ky offsets and the hi / lo plane are immediates
  int ylr[C::MT], vo[C::MT][3][2];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) {
    const int m = (wm * C::MT + mt) * 32 + r;
    const int np = m / (TR * C::NTX), rem = m % (TR * C::NTX);
    ylr[mt] = rem / C::NTX;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int wr = ylr[mt] + ky;  // window row: input row wr - 1; rows -1 and TR read the zero row
      const int rowb = (wr >= 1 && wr <= TR) ? np * C::PS + (wr - 1) * C::RS : C::ZROW;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        vo[mt][ky][ks] = rowb + (rem % C::NTX) * 64 + 16 * ((2 * ks + h) ^ (wr & 3));
        asm volatile("" : "+v"(vo[mt][ky][ks]));  // one opaque register each (no re-split sums in the K-loop)
      }
    }
  }
  const __amdgpu_buffer_rsrc_t wr_ = make_rsrc(wp, C::NCC * C::CHUNK_BYTES);
  const unsigned wvoff = (wn * C::NT * 2 * 64 + lane) * 16;
  f32x16 y0a[C::MT][C::NT], y1a[C::MT][C::NT], ma[C::MT][C::NT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < C::NT; ++nt) y0a[mt][nt] = y1a[mt][nt] = ma[mt][nt] = f32x16{};

  auto load_b = [&](int cc, int kx, uint4 (&dst)[C::NT][2]) {
#pragma unroll
    for (int nt = 0; nt < C::NT; ++nt) {
      const unsigned k = cc * C::CHUNK_BYTES + (((ABL & 4) ? 0 : kx) * C::NTOT + nt) * 2 * 64 * 16;
      dst[nt][0] = buf_load16(wr_, wvoff, k);
      dst[nt][1] = buf_load16(wr_, wvoff, k + 64 * 16);
    }
  };
  // WD: weight ring depth, K-step fragments loaded WD - 1 steps ahead (a K-step is 6 MFMAs here, half
  // the direct kernel's, so the same depth covers half the L2 latency)
  static_assert(C::NKS % WD == 0, "the weight ring runs on across stages");
  uint4 bq[WD][C::NT][2];
#pragma unroll
  for (int k = 0; k + 1 < WD; ++k) load_b(0, k, bq[k]);
#pragma unroll 1
  for (int s = 0; s < NS; ++s) {
    const char* cur = (s & 1) ? buf1 : buf0;
    const int cc = s % C::NCC, ccn = (s + 1) % C::NCC;
    uint4 aq[2][C::MT][2];
    auto load_a = [&](int kx, uint4 (&dst)[C::MT][2]) {
      const int xi = kx / 6, ky = (kx % 6) >> 1, ks = kx & 1;
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        const char* pa = cur + vo[mt][ky][ks];
        dst[mt][0] = *reinterpret_cast<const uint4*>(pa + xi * C::XROW);
        dst[mt][1] = *reinterpret_cast<const uint4*>(pa + (C::PLANE + xi * C::XROW));
      }
    };
    load_a(0, aq[0]);
#pragma unroll
    for (int kx = 0; kx < C::NKS; ++kx) {
      if constexpr ((ABL & 32) != 0) {  // timing only: no weight loads after the prologue
      } else if (kx + WD - 1 < C::NKS)
        load_b(cc, kx + WD - 1, bq[(kx + WD - 1) % WD]);
      else  // the next stage's first fragments, unconditionally (valid weights even after the last
            // stage): a branch here made the compiler's vmcnt merge wait vmcnt(0) at the stage's end
        load_b(ccn, kx + WD - 1 - C::NKS, bq[(kx + WD - 1) % WD]);
      if (kx + 1 < C::NKS) load_a(kx + 1, aq[(kx + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const int xi = kx / 6;
      if (kx == 12) {  // m1 complete: out[2t] += m1, out[2t+1] += m1
#pragma unroll
        for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < C::NT; ++nt) {
            y0a[mt][nt] += ma[mt][nt];
            y1a[mt][nt] += ma[mt][nt];
          }
      }
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        const bf16x8 xh = as_bf16x8(aq[kx & 1][mt][0]), xl = as_bf16x8(aq[kx & 1][mt][1]);
#pragma unroll
        for (int nt = 0; nt < C::NT; ++nt) {
          const bf16x8 wh = as_bf16x8(bq[kx % WD][nt][0]), wl = as_bf16x8(bq[kx % WD][nt][1]);
          if constexpr ((ABL & 2) != 0)  // timing only: no MFMA, operands kept live
            y0a[mt][nt][0] += __builtin_bit_cast(float, aq[kx & 1][mt][0].x ^ aq[kx & 1][mt][1].y ^
                                                            bq[kx % WD][nt][0].z ^ bq[kx % WD][nt][1].w);
          else if (xi == 0)
            y0a[mt][nt] = mfma3(wh, wl, xh, xl, y0a[mt][nt]);
          else if (xi == 3)
            y1a[mt][nt] = mfma3(wh, wl, xh, xl, y1a[mt][nt]);
          else  // m1 (kx 6..11) / m2 (kx 12..17) start from zero
            ma[mt][nt] = mfma3(wh, wl, xh, xl, (kx % 6 == 0) ? f32x16{} : ma[mt][nt]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // m2 complete: out[2t] += m2, out[2t+1] -= m2
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < C::NT; ++nt) {
        y0a[mt][nt] += ma[mt][nt];
        y1a[mt][nt] -= ma[mt][nt];
      }
    if (cc == C::NCC - 1) {
      const int p0 = tile_of(s);
#pragma unroll
      for (int nt = 0; nt < C::NT; ++nt) {
        float4 bv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          bv[q] = *reinterpret_cast<const float4*>(sbias + (wn * C::NT + nt) * 32 + 8 * q + 4 * h);
#pragma unroll
        for (int mt = 0; mt < C::MT; ++mt) {
          const int m0 = (wm * C::MT + mt) * 32;  // the M tile: 32 / NTX whole rows of patch np
          const int np = m0 / (TR * C::NTX), yb = (m0 % (TR * C::NTX)) / C::NTX;
          if ((NP == 1 || p0 + np < P) && ((ABL & 8) == 0 || y0a[mt][nt][0] == 1234.5f)) {  // ABL 8: timing only
            // pixel (row yb + m / NTX, column 2 (m % NTX) + par) of M index m = m0 + m
            float* const ob = out + (((size_t)p0 + np) * H + yb) * H * COUT + (wn * C::NT + nt) * 32;
#pragma unroll
            for (int par = 0; par < 2; ++par) {
              const f32x16& yv = par ? y1a[mt][nt] : y0a[mt][nt];
              float4 v[4];
#pragma unroll
              for (int q = 0; q < 4; ++q)
                v[q] = make_float4(relu0(yv[4 * q + 0] + bv[q].x), relu0(yv[4 * q + 1] + bv[q].y),
                                   relu0(yv[4 * q + 2] + bv[q].z), relu0(yv[4 * q + 3] + bv[q].w));
              if constexpr (CST) {
                float* scr = reinterpret_cast<float*>(smem + C::SCR_OFF) + wave * (C::SCR / 4);
#pragma unroll
                for (int q = 0; q < 4; ++q) *reinterpret_cast<float4*>(scr + r * C::SROW + 8 * q + 4 * h) = v[q];
                __builtin_amdgcn_wave_barrier();  // same wave: its LDS accesses execute in order
                asm volatile("" ::: "memory");
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                  const int ml = 8 * k + (lane >> 3), c4 = lane & 7;
                  const int px = (ml / C::NTX) * H + 2 * (ml % C::NTX) + par;
                  *reinterpret_cast<float4*>(ob + (size_t)px * COUT + 4 * c4) =
                      *reinterpret_cast<const float4*>(scr + ml * C::SROW + 4 * c4);
                }
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
              } else {
                const int px = (r / C::NTX) * H + 2 * (r % C::NTX) + par;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                  *reinterpret_cast<float4*>(ob + (size_t)px * COUT + 8 * q + 4 * h) = v[q];
              }
            }
          }
          y0a[mt][nt] = y1a[mt][nt] = f32x16{};
        }
      }
    }
    __syncthreads();
  }
}

template <int CIN, int COUT, int H, int NP, int WM, int WN, bool CST, int WD, int ABL = 0>
hipError_t launch_w1(const float* in, float* out, const void* wp, const float* bias, int P, hipStream_t st) {
  using C = W1Cfg<CIN, COUT, H, NP, WM, WN, CST>;
  const void* fn = reinterpret_cast<const void*>(&k_conv_w1<CIN, COUT, H, NP, WM, WN, CST, WD, ABL>);
  int resident = 0;
  const hipError_t e = hn_resident_blocks(fn, C::NTHR, C::SMEM, &resident);
  if (e != hipSuccess) return e;
  const int tiles = (P + NP - 1) / NP;
  const int grid = std::min(tiles, resident);
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_conv_w1<CIN, COUT, H, NP, WM, WN, CST, WD, ABL>), dim3(grid), dim3(C::NTHR), C::SMEM, st, in, out,
                     static_cast<const uint4*>(wp), bias, P);
  return hipGetLastError();
}

#ifdef HN_EXPERIMENTS  // F(4,3) conv3 (k_conv_w4): measured slower than k_conv_w1 (11.2 vs 9.9 ms), experiments library only
// ---------------------------------------------------------------------------------------
// F(4,3) along x (k_conv_w4): per output row y and column quad (4t .. 4t+3), d_k = x[y + ky - 1][4t - 1 + k]
// (k = 0..5, zero outside the patch), Toom-Cook points 0, 1, -1, 1/2, -1/2, infinity:
//   V = B^T d:  V0 = d0/4 - 5 d2/4 + d4            V1 = -(d1 + d2)/4 + d3 + d4
//               V2 = (d1 - d2)/4 - d3 + d4          V3 = d4 - d2 - (d1 - d3)/2
//               V4 = d4 - d2 + (d1 - d3)/2          V5 = d1/4 - 5 d3/4 + d5
//   U_xi[ky] = sum_kx G[xi][kx] W[ky][kx],  G = [4 0 0; 2/3 2/3 2/3; 2/3 -2/3 2/3; -8/3 -4/3 -2/3; -8/3 4/3 -2/3; 0 0 1]
//   y0 = m0 + m1 + m2 + m3 + m4,  y1 = m1 - m2 + (m3 - m4)/2,  y2 = m1 + m2 + (m3 + m4)/4,
//   y3 = m1 - m2 + (m3 - m4)/8 + m5                                                   (A^T m)
// 18 multiplies per output quad and input channel instead of 36 (F(2,3): 24): the layer's MFMA work is
// 3/4 of the F(2,3) kernel's and so is the weight stream per patch (precision: tests/precision/
// wino1d_precision.py "1:4 3:4 5:2", 1.9e-5 from fp64 against 1.7e-5 for the F(2,3) form).
// Same producer / MFMA wave split as k_conv_w1, but the MFMAs are 16x16x32 with the weights as the A
// operand (16 output channels x 32 input channels) and the transformed positions as B: each MFMA wave
// owns 16 output channels of every position of the tile (M = 64 positions = 4 B tiles), so a weight
// fragment is used by 4 MFMAs (k_conv_w1: 2) -- the weight stream that bounds k_conv_w1 drops to half
// per MFMA -- and the result lanes hold 4 consecutive channels of one pixel (16-byte stores, no LDS
// transpose).  Operand image per plane: [patch][xi][row -1 .. H][quad][32 channels bf16], zero rows -1
// and H inside every (patch, xi) block, 256-byte rows, 16-byte chunk c of row r at c ^ 2 (r & 1):
// the B-operand reads (lane l: position l & 15, chunk l >> 4) and the producers' 8-lane store groups
// are bank-conflict free (tests/test_lds_banks.py).
// Accumulation: m0 into Y0, m5 into Y3 (xi order 0, 5, 1, 2, 3, 4), m1..m4 each into one of two
// temporaries that is folded into Y0..Y3 (A^T coefficients) over the next xi's three K-steps, so that
// no fold waits on the MFMA that produced its temporary.
template <int CIN, int COUT, int H, int NP, int WN>
struct W4Cfg {
  static constexpr int NTX = H / 4;           // column quads per row
  static constexpr int POS = NP * H * NTX;    // positions per xi and work tile
  static constexpr int MT = POS / 16;         // 16-position B tiles
  static constexpr int NCC = CIN / 32;        // 32-channel stages
  static constexpr int NT = COUT / 16 / WN;   // 16-channel output tiles per MFMA wave
  static constexpr int RB = NTX * 64;         // bytes per image row
  static constexpr int HR = H + 2;            // image rows per (patch, xi) block
  static constexpr int XB = HR * RB;          // bytes per (patch, xi) block
  static constexpr int PLANE = NP * 6 * XB;
  static constexpr int BUF = 2 * PLANE;
  static constexpr int NWC = WN, NWP = 4, NTHR = (NWC + NWP) * 64, PTHR = NWP * 64;
  static constexpr int UNITS = NP * H * NTX * 4;  // (patch, row, quad, 8-channel group)
  static constexpr int UPT = UNITS / PTHR;
  static constexpr bool DEEP = UPT <= 2;
  static constexpr int SMEM = 2 * BUF;
  static constexpr int NKS = 18;  // K-steps per stage: 6 xi x 3 ky, K = the stage's 32 channels
  static constexpr unsigned KSTEP_BYTES = (COUT / 16) * 2 * 64 * 16;  // every output tile's hi + lo fragments
  static constexpr unsigned CHUNK_BYTES = NKS * KSTEP_BYTES;
  static_assert(RB == 256, "the bank-conflict argument assumes 256-byte image rows");
  static_assert(UNITS % PTHR == 0 && UPT >= 1, "whole units per producer thread");
  static_assert(POS % 16 == 0 && NT >= 1 && NT * WN * 16 == COUT, "tiling");
  static_assert(SMEM <= 160 * 1024, "LDS");
};

// the K-step order's xi sequence (m0 and m5 straight into their outputs first)
__host__ __device__ constexpr int w4_xi(int xo) { return xo == 0 ? 0 : xo == 1 ? 5 : xo - 1; }

// ABL (timing-only builds, HN_EXPERIMENTS library, HN_W4_ABL): as k_conv_w1's bits 0 (idle producers),
// 1 (no MFMAs), 4 (idle MFMA waves), 5 (no weight loads after the prologue)
template <int CIN, int COUT, int H, int NP, int WN, int WD, int ABL = 0>
__global__ __launch_bounds__((WN + 4) * 64) void k_conv_w4(const float* __restrict__ in, float* __restrict__ out,
                                                           const uint4* __restrict__ wp,
                                                           const float* __restrict__ bias, int P) {
  using C = W4Cfg<CIN, COUT, H, NP, WN>;
  constexpr int NTX = C::NTX;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wave >= C::NWC;
  const int nwg = gridDim.x, rb = xcd_remap(blockIdx.x, nwg);
  const int ntiles = (P + NP - 1) / NP;
  const int my_tiles = rb < ntiles ? (ntiles - 1 - rb) / nwg + 1 : 0;
  const int NS = my_tiles * C::NCC;
  if (NS == 0) return;
  char* const buf0 = smem;
  char* const buf1 = smem + C::BUF;
  auto tile_of = [&](int s) { return (rb + (s / C::NCC) * nwg) * NP; };

  // the zero rows -1 and H of every (patch, xi) block, both buffers and planes
  constexpr int ZCH = C::RB / 16, NZ = 2 * 2 * NP * 6 * 2 * ZCH;
  for (int i = tid; i < NZ; i += C::NTHR) {
    const int q = i % ZCH, rest = i / ZCH;
    const int row = (rest & 1) ? C::HR - 1 : 0, blk = (rest >> 1) % (NP * 6), bp = (rest >> 1) / (NP * 6);
    *reinterpret_cast<uint4*>(smem + bp * C::PLANE + blk * C::XB + row * C::RB + q * 16) = make_uint4(0, 0, 0, 0);
  }

  if (producer) {
    if constexpr ((ABL & 1) != 0) {
#pragma unroll 1
      for (int s = 0; s <= NS; ++s) __syncthreads();
      return;
    }
    // a unit (patch, row y, quad t, 8-channel group g) loads input columns 4t - 1 .. 4t + 2 (the last quad
    // also column H - 1); d4 / d5 are the next quad's first two columns, taken from lane + 4
    const int ptid = tid - C::NWC * 64;
    float4 pf[C::UPT][10], pf2[C::UPT][10];
    constexpr unsigned PATCH_BYTES = (unsigned)H * H * CIN * 4, OOB = 0x80000000u;
    auto produce_loads = [&](int s, float4 (&d)[C::UPT][10]) {
      const bool live = s < NS;
      const int p0 = live ? tile_of(s) : 0;
      const int cc = s % C::NCC;
      const int nval = !live ? 0 : P - p0 < NP ? P - p0 : NP;
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(in + (size_t)p0 * H * H * CIN, (unsigned)nval * PATCH_BYTES);
#pragma unroll
      for (int k = 0; k < C::UPT; ++k) {
        const int u = ptid + k * C::PTHR;
        const int g = u & 3, t = (u >> 2) % NTX, rest = (u >> 2) / NTX;
        const int y = rest % H, np = rest / H;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const int x = 4 * t - 1 + j;
          const bool ok = (j < 4 || t == NTX - 1) && (unsigned)x < (unsigned)H;
          const unsigned vo = ok ? (unsigned)(((np * H + y) * H + x) * CIN + cc * 32 + g * 8) * 4u : OOB;
          d[k][2 * j] = __builtin_bit_cast(float4, buf_load16(rs, vo, 0));
          d[k][2 * j + 1] = __builtin_bit_cast(float4, buf_load16(rs, vo, 16));
        }
      }
    };
    auto shfl4 = [&](const float4& v) {
      return make_float4(__shfl_down(v.x, 4, 64), __shfl_down(v.y, 4, 64), __shfl_down(v.z, 4, 64),
                         __shfl_down(v.w, 4, 64));
    };
    auto produce_write = [&](char* dst, const float4 (&d)[C::UPT][10]) {
#pragma unroll
      for (int k = 0; k < C::UPT; ++k) {
        const int u = ptid + k * C::PTHR;
        const int g = u & 3, t = (u >> 2) % NTX, rest = (u >> 2) / NTX;
        const int y = rest % H, np = rest / H;
        const bool last = t == NTX - 1;
        float4 dd[6][2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const float4 n0 = shfl4(d[k][i]), n1 = shfl4(d[k][2 + i]);  // every lane joins the shuffles
          dd[0][i] = d[k][i];
          dd[1][i] = d[k][2 + i];
          dd[2][i] = d[k][4 + i];
          dd[3][i] = d[k][6 + i];
          dd[4][i] = last ? d[k][8 + i] : n0;
          dd[5][i] = last ? make_float4(0.f, 0.f, 0.f, 0.f) : n1;
        }
        const int off = np * 6 * C::XB + (y + 1) * C::RB + t * 64 + 16 * (g ^ (2 * (y & 1)));
#pragma unroll
        for (int xi = 0; xi < 6; ++xi) {
          float4 v[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            auto tr = [&](float d0, float d1, float d2, float d3, float d4, float d5) {
              switch (xi) {
                case 0: return fmaf(0.25f, d0, fmaf(-1.25f, d2, d4));
                case 1: return fmaf(-0.25f, d1 + d2, d3 + d4);
                case 2: return fmaf(0.25f, d1 - d2, d4 - d3);
                case 3: return fmaf(-0.5f, d1 - d3, d4 - d2);
                case 4: return fmaf(0.5f, d1 - d3, d4 - d2);
                default: return fmaf(0.25f, d1, fmaf(-1.25f, d3, d5));
              }
            };
            v[i] = make_float4(tr(dd[0][i].x, dd[1][i].x, dd[2][i].x, dd[3][i].x, dd[4][i].x, dd[5][i].x),
                               tr(dd[0][i].y, dd[1][i].y, dd[2][i].y, dd[3][i].y, dd[4][i].y, dd[5][i].y),
                               tr(dd[0][i].z, dd[1][i].z, dd[2][i].z, dd[3][i].z, dd[4][i].z, dd[5][i].z),
                               tr(dd[0][i].w, dd[1][i].w, dd[2][i].w, dd[3][i].w, dd[4][i].w, dd[5][i].w));
          }
          uint4 hi, lo;
          split8(v[0], v[1], hi, lo);
          *reinterpret_cast<uint4*>(dst + off + xi * C::XB) = hi;
          *reinterpret_cast<uint4*>(dst + C::PLANE + off + xi * C::XB) = lo;
        }
      }
    };
    produce_loads(0, pf);
    produce_write(buf0, pf);
    produce_loads(1, pf);
    __syncthreads();
    if constexpr (!C::DEEP) {
#pragma unroll 1
      for (int s = 0; s < NS; ++s) {
        produce_write((s & 1) ? buf0 : buf1, pf);
        produce_loads(s + 2, pf);
        __syncthreads();
      }
    } else {
#pragma unroll 1
      for (int s = 0; s < NS; s += 2) {
        produce_loads(s + 2, pf2);
        produce_write(buf1, pf);
        __syncthreads();
        if (s + 1 >= NS) break;
        produce_loads(s + 3, pf);
        produce_write(buf0, pf2);
        __syncthreads();
      }
    }
    return;
  }

  // ---- MFMA side ----
  __syncthreads();
  if constexpr ((ABL & 16) != 0) {
#pragma unroll 1
    for (int s = 0; s < NS; ++s) __syncthreads();
    return;
  }
  const int h4 = lane >> 4;
  // per-lane part of a B-operand (position) address for M tile mt and kernel row ky; xi is an immediate
  int vo[C::MT][3];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) {
    const int pos = mt * 16 + (lane & 15);
    const int np = pos / (H * NTX), rem = pos % (H * NTX), y = rem / NTX, t = rem % NTX;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int r = y + ky - 1;  // input row; -1 and H are the block's zero rows
      vo[mt][ky] = np * 6 * C::XB + (r + 1) * C::RB + t * 64 + 16 * (h4 ^ (2 * (r & 1)));
      asm volatile("" : "+v"(vo[mt][ky]));
    }
  }
  const __amdgpu_buffer_rsrc_t wr_ = make_rsrc(wp, C::NCC * C::CHUNK_BYTES);
  const unsigned wvoff = (wave * C::NT * 2 * 64 + lane) * 16;
  float4 bv[C::NT];
#pragma unroll
  for (int nt = 0; nt < C::NT; ++nt)
    bv[nt] = *reinterpret_cast<const float4*>(bias + (wave * C::NT + nt) * 16 + 4 * h4);
  f32x4_t Y[4][C::MT][C::NT], T[2][C::MT][C::NT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < C::NT; ++nt) {
#pragma unroll
      for (int q = 0; q < 4; ++q) Y[q][mt][nt] = f32x4_t{};
      T[0][mt][nt] = T[1][mt][nt] = f32x4_t{};
    }
  // fold piece `part` (0: Y0, 1: Y1, 2: Y2, 3: Y3) of temporary T[ti] holding m_xi
  auto fold = [&](int ti, int xi, int part) {
    constexpr float cf[5][4] = {{0, 0, 0, 0}, {1, 1, 1, 1}, {1, -1, 1, -1}, {1, 0.5f, 0.25f, 0.125f},
                                {1, -0.5f, 0.25f, -0.125f}};
    const float c = cf[xi][part];
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < C::NT; ++nt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (c == 1.f) Y[part][mt][nt][j] += T[ti][mt][nt][j];
          else if (c == -1.f) Y[part][mt][nt][j] -= T[ti][mt][nt][j];
          else Y[part][mt][nt][j] = fmaf(c, T[ti][mt][nt][j], Y[part][mt][nt][j]);
        }
  };
  auto load_b = [&](int cc, int kx, uint4 (&dst)[C::NT][2]) {
#pragma unroll
    for (int nt = 0; nt < C::NT; ++nt) {
      const unsigned k = cc * C::CHUNK_BYTES + kx * C::KSTEP_BYTES + nt * 2 * 64 * 16;
      dst[nt][0] = buf_load16(wr_, wvoff, k);
      dst[nt][1] = buf_load16(wr_, wvoff, k + 64 * 16);
    }
  };
  static_assert(C::NKS % WD == 0, "the weight ring runs on across stages");
  uint4 bq[WD][C::NT][2];
#pragma unroll
  for (int k = 0; k + 1 < WD; ++k) load_b(0, k, bq[k]);
#pragma unroll 1
  for (int s = 0; s < NS; ++s) {
    const char* cur = (s & 1) ? buf1 : buf0;
    const int cc = s % C::NCC, ccn = (s + 1) % C::NCC;
    const bool pend = cc != 0;  // xi 4's temporary (T[1]) of the previous stage still to fold
    // one B fragment pair per M tile, reloaded for the next K-step right behind its own three MFMAs
    // (12 MFMAs of cover; a second set of 32 registers went to the weight ring instead)
    uint4 aq[C::MT][2];
    auto load_a = [&](int kx, int mt) {
      const int xi = w4_xi(kx / 3), ky = kx % 3;
      const char* pa = cur + vo[mt][ky];
      aq[mt][0] = *reinterpret_cast<const uint4*>(pa + xi * C::XB);
      aq[mt][1] = *reinterpret_cast<const uint4*>(pa + (C::PLANE + xi * C::XB));
    };
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt) load_a(0, mt);
#pragma unroll
    for (int kx = 0; kx < C::NKS; ++kx) {
      if constexpr ((ABL & 32) != 0) {
      } else if (kx + WD - 1 < C::NKS)
        load_b(cc, kx + WD - 1, bq[(kx + WD - 1) % WD]);
      else
        load_b(ccn, kx + WD - 1 - C::NKS, bq[(kx + WD - 1) % WD]);
      __builtin_amdgcn_sched_barrier(0);
      const int xo = kx / 3, ky = kx % 3, xi = w4_xi(xo);
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        const uint4 xh = aq[mt][0], xl = aq[mt][1];
#pragma unroll
        for (int nt = 0; nt < C::NT; ++nt) {
          const uint4 wh = bq[kx % WD][nt][0], wl = bq[kx % WD][nt][1];
          f32x4_t& acc = xi == 0 ? Y[0][mt][nt] : xi == 5 ? Y[3][mt][nt] : T[xo & 1][mt][nt];
          f32x4_t a = (xo >= 2 && ky == 0) ? f32x4_t{} : acc;
          if constexpr ((ABL & 2) != 0) {
            acc[0] += __builtin_bit_cast(float, xh.x ^ xl.y ^ wh.z ^ wl.w);
            continue;
          }
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wh), as_bf16x8(xh), a, 0, 0, 0);
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wh), as_bf16x8(xl), a, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wl), as_bf16x8(xh), a, 0, 0, 0);
        }
        if (kx + 1 < C::NKS) load_a(kx + 1, mt);
      }
      // folds, behind this K-step's MFMAs: the previous xi's temporary over this xi's three K-steps
      if (xo >= 3) {
        const int pxi = w4_xi(xo - 1), ti = (xo - 1) & 1;
        if (ky == 0) { fold(ti, pxi, 0); fold(ti, pxi, 1); }
        if (ky == 1) fold(ti, pxi, 2);
        if (ky == 2) fold(ti, pxi, 3);
      } else if (pend && kx < 4) {  // xi 4 of the previous stage: Y1, Y2, Y3, then Y0 (after m0's MFMAs)
        fold(1, 4, kx == 3 ? 0 : kx + 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (cc == C::NCC - 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) fold(1, 4, q);
      const int p0 = tile_of(s);
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        const int pos = mt * 16 + (lane & 15);
        const int np = pos / (H * NTX), rem = pos % (H * NTX), y = rem / NTX, t = rem % NTX;
        if (NP == 1 || p0 + np < P) {
          float* const ob = out + (((size_t)p0 + np) * H + y) * H * COUT + (size_t)(4 * t) * COUT + 4 * h4;
#pragma unroll
          for (int nt = 0; nt < C::NT; ++nt)
#pragma unroll
            for (int par = 0; par < 4; ++par) {
              const f32x4_t& yv = Y[par][mt][nt];
              *reinterpret_cast<float4*>(ob + par * COUT + (wave * C::NT + nt) * 16) =
                  make_float4(relu0(yv[0] + bv[nt].x), relu0(yv[1] + bv[nt].y), relu0(yv[2] + bv[nt].z),
                              relu0(yv[3] + bv[nt].w));
            }
        }
#pragma unroll
        for (int nt = 0; nt < C::NT; ++nt)
#pragma unroll
          for (int q = 0; q < 4; ++q) Y[q][mt][nt] = f32x4_t{};
      }
    }
    __syncthreads();
  }
}

template <int CIN, int COUT, int H, int NP, int WN, int WD, int ABL = 0>
hipError_t launch_w4(const float* in, float* out, const void* wp, const float* bias, int P, hipStream_t st) {
  using C = W4Cfg<CIN, COUT, H, NP, WN>;
  const void* fn = reinterpret_cast<const void*>(&k_conv_w4<CIN, COUT, H, NP, WN, WD, ABL>);
  int resident = 0;
  const hipError_t e = hn_resident_blocks(fn, C::NTHR, C::SMEM, &resident);
  if (e != hipSuccess) return e;
  const int tiles = (P + NP - 1) / NP;
  const int grid = std::min(tiles, resident);
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_conv_w4<CIN, COUT, H, NP, WN, WD, ABL>), dim3(grid), dim3(C::NTHR), C::SMEM, st, in, out,
                     static_cast<const uint4*>(wp), bias, P);
  return hipGetLastError();
}

using W4Conv3 = W4Cfg<64, 64, 16, 1, 4>;
#endif  // HN_EXPERIMENTS

using W1Conv3 = W1Cfg<64, 64, 16, 1, 2, 2, true>;
using W1Conv5 = W1Cfg<128, 128, 8, 2, 1, 4, true>;

}  // namespace

// conv3: one patch per work tile, 2 x 2 MFMA waves of 2 M tiles; conv5: two patches, 1 x 4 waves.
// wd: the weight ring depth (HN_VARIANT digit j = 3, k = 4, l = 6, q = 8)
hipError_t hn_launch_wino1(int layer, int wd, const HardnetDev& d, const float* in, float* out, int P,
                           hipStream_t st) {
  if (P <= 0) return hipSuccess;
  if (!d.wino1[layer]) return hipErrorInvalidValue;
#ifdef HN_EXPERIMENTS  // wd = 100 + ABL: the timing-only ablations (weight ring 8)
#define HN_W1_ABL(CI, CO, HH, NPP, WMM, WNN, L)                                                              \
  if (wd == 101) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 1>(in, out, d.wino1[L], d.bias[L], P, st); \
  if (wd == 102) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 2>(in, out, d.wino1[L], d.bias[L], P, st); \
  if (wd == 104) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 4>(in, out, d.wino1[L], d.bias[L], P, st); \
  if (wd == 108) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 8>(in, out, d.wino1[L], d.bias[L], P, st); \
  if (wd == 116) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 16>(in, out, d.wino1[L], d.bias[L], P, st); \
  if (wd == 132) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 32>(in, out, d.wino1[L], d.bias[L], P, st); \
  if (wd == 134) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 34>(in, out, d.wino1[L], d.bias[L], P, st); \
  if (wd == 164) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 64>(in, out, d.wino1[L], d.bias[L], P, st); \
  if (wd == 228) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 128>(in, out, d.wino1[L], d.bias[L], P, st);
// weight rings 3 / 4 (digits j / k): measured slower than 6 / 8
#define HN_W1_SHALLOW(CI, CO, HH, NPP, WMM, WNN, L)                                                          \
  if (wd == 3) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 3>(in, out, d.wino1[L], d.bias[L], P, st); \
  if (wd == 4) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 4>(in, out, d.wino1[L], d.bias[L], P, st);
#else
#define HN_W1_ABL(CI, CO, HH, NPP, WMM, WNN, L)
#define HN_W1_SHALLOW(CI, CO, HH, NPP, WMM, WNN, L)
#endif
#define HN_W1(L, CI, CO, HH, NPP, WMM, WNN)                                                                      \
  if (layer == L) {                                                                                             \
    HN_W1_SHALLOW(CI, CO, HH, NPP, WMM, WNN, L)                                                                 \
    if (wd == 6) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 6>(in, out, d.wino1[L], d.bias[L], P, st); \
    if (wd == 8) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8>(in, out, d.wino1[L], d.bias[L], P, st); \
    HN_W1_ABL(CI, CO, HH, NPP, WMM, WNN, L)                                                                     \
  }
  HN_W1(3, 64, 64, 16, 1, 2, 2)
  HN_W1(5, 128, 128, 8, 2, 1, 4)
#undef HN_W1
#undef HN_W1_ABL
#undef HN_W1_SHALLOW
  return hipErrorInvalidValue;
}

#ifdef HN_EXPERIMENTS
// conv3 as F(4,3) (k_conv_w4); wd: the weight ring depth (HN_VARIANT digit w = 6, x = 9)
hipError_t hn_launch_wino4(int layer, int wd, const HardnetDev& d, const float* in, float* out, int P,
                           hipStream_t st) {
  if (P <= 0) return hipSuccess;
  if (layer != 3 || !d.wino4[layer]) return hipErrorInvalidValue;
#ifdef HN_EXPERIMENTS
  if (const char* e = std::getenv("HN_W4_ABL")) {
    switch (std::atoi(e)) {
      case 1: return launch_w4<64, 64, 16, 1, 4, 6, 1>(in, out, d.wino4[3], d.bias[3], P, st);
      case 2: return launch_w4<64, 64, 16, 1, 4, 6, 2>(in, out, d.wino4[3], d.bias[3], P, st);
      case 16: return launch_w4<64, 64, 16, 1, 4, 6, 16>(in, out, d.wino4[3], d.bias[3], P, st);
      case 32: return launch_w4<64, 64, 16, 1, 4, 6, 32>(in, out, d.wino4[3], d.bias[3], P, st);
      case 34: return launch_w4<64, 64, 16, 1, 4, 6, 34>(in, out, d.wino4[3], d.bias[3], P, st);
    }
  }
#endif
  if (wd == 6) return launch_w4<64, 64, 16, 1, 4, 6>(in, out, d.wino4[3], d.bias[3], P, st);
  if (wd == 9) return launch_w4<64, 64, 16, 1, 4, 9>(in, out, d.wino4[3], d.bias[3], P, st);
  return hipErrorInvalidValue;
}
#endif  // HN_EXPERIMENTS

// LDS bytes of the layer's configuration (tests / DESIGN.md)
int hn_wino1_lds_bytes(int layer) {
  switch (layer) {
    case 3: return W1Conv3::SMEM;
    case 5: return W1Conv5::SMEM;
  }
  return -1;
}
