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
// reused), bit 3 no epilogue stores, bit 4 idle MFMA waves
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
      if (kx + WD - 1 < C::NKS)
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
  if (wd == 116) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8, 16>(in, out, d.wino1[L], d.bias[L], P, st);
#else
#define HN_W1_ABL(CI, CO, HH, NPP, WMM, WNN, L)
#endif
#define HN_W1(L, CI, CO, HH, NPP, WMM, WNN)                                                                      \
  if (layer == L) {                                                                                             \
    if (wd == 3) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 3>(in, out, d.wino1[L], d.bias[L], P, st); \
    if (wd == 4) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 4>(in, out, d.wino1[L], d.bias[L], P, st); \
    if (wd == 6) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 6>(in, out, d.wino1[L], d.bias[L], P, st); \
    if (wd == 8) return launch_w1<CI, CO, HH, NPP, WMM, WNN, true, 8>(in, out, d.wino1[L], d.bias[L], P, st); \
    HN_W1_ABL(CI, CO, HH, NPP, WMM, WNN, L)                                                                     \
  }
  HN_W1(3, 64, 64, 16, 1, 2, 2)
  HN_W1(5, 128, 128, 8, 2, 1, 4)
#undef HN_W1
#undef HN_W1_ABL
  return hipErrorInvalidValue;
}

// LDS bytes of the layer's configuration (tests / DESIGN.md)
int hn_wino1_lds_bytes(int layer) {
  switch (layer) {
    case 3: return W1Conv3::SMEM;
    case 5: return W1Conv5::SMEM;
  }
  return -1;
}
