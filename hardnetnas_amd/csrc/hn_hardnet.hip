// Stock HardNet descriptor forward on gfx950 (hardnet/HardNet.py:275-315).
//
// Kernels (activations between them are NHWC fp32 in the caller's workspace):
//   k_stem      input_norm (HardNet.py:306-310) + conv0 3x3 1->32 + BN + ReLU, VALU fp32.
//               Also the NAS stem ConvBNRelu(1->32) with NORM=false.
//   k_conv3x3   conv1..conv5 (HardNet.py:284-298) as implicit GEMMs on the bf16 MFMA
//               (v_mfma_f32_32x32x16_bf16) in bf16x3 split precision, BN folded into
//               weights + bias, ReLU fused.  The input window of a tile (all rows the
//               9 taps touch, zero-padded) is staged once per 32-channel chunk into LDS
//               as bf16 hi/lo planes; the 9 taps then read shifted views of it.
//   k_head      conv6 8x8 -> 128 (HardNet.py:300-301) as a [P,8192]x[8192,128] GEMM,
//               BN folded, L2Norm (Utils.py:15-22) fused in the epilogue.
#include "hn_common.h"
#include "hn_internal.h"

#include <algorithm>
#include <cstdlib>

// ------------------------------------------------------------------------------------
// stem
// ------------------------------------------------------------------------------------
template <bool NORM>
__global__ __launch_bounds__(256) void k_stem(const float* __restrict__ in, float* __restrict__ out,
                                              const float* __restrict__ w,   // [9][32]
                                              const float* __restrict__ b,   // [32]
                                              float eps) {
  __shared__ float tile[34 * 34];
  __shared__ float red[8];
  const int t = threadIdx.x;
  const size_t p = blockIdx.x;
  const float4 v = reinterpret_cast<const float4*>(in + p * 1024)[t];
  for (int i = t; i < 34 * 34; i += 256) tile[i] = 0.f;
  float mean = 0.f, sd = 1.f;
  if (NORM) {  // (x - mean) / (std_unbiased + eps), HardNet.py:307-310
    float s = wave_sum(v.x + v.y + v.z + v.w);
    if ((t & 63) == 0) red[t >> 6] = s;
    __syncthreads();
    mean = (red[0] + red[1] + red[2] + red[3]) * (1.f / 1024.f);
    const float d0 = v.x - mean, d1 = v.y - mean, d2 = v.z - mean, d3 = v.w - mean;
    float q = wave_sum(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
    if ((t & 63) == 0) red[4 + (t >> 6)] = q;
    __syncthreads();
    sd = sqrtf((red[4] + red[5] + red[6] + red[7]) * (1.f / 1023.f)) + eps;
  }
  __syncthreads();
  {
    const int q = 4 * t, y = q >> 5, x = q & 31;
    float* d = tile + (y + 1) * 34 + x + 1;
    d[0] = (v.x - mean) / sd; d[1] = (v.y - mean) / sd;
    d[2] = (v.z - mean) / sd; d[3] = (v.w - mean) / sd;
  }
  __syncthreads();
#pragma unroll 1
  for (int k = 0; k < 4; ++k) {
    const int q = t + 256 * k, y = q >> 5, x = q & 31;
    float xin[9];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) xin[ky * 3 + kx] = tile[(y + ky) * 34 + x + kx];
    float4* o = reinterpret_cast<float4*>(out + (p * 1024 + q) * 32);
#pragma unroll
    for (int c4 = 0; c4 < 8; ++c4) {
      float r[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = 4 * c4 + j;
        float acc = 0.f;
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) acc = fmaf(xin[tp], w[tp * 32 + c], acc);
        r[j] = fmaxf(acc + b[c], 0.f);
      }
      o[c4] = make_float4(r[0], r[1], r[2], r[3]);
    }
  }
}

// ------------------------------------------------------------------------------------
// conv3x3 implicit GEMM, bf16x3 on MFMA 32x32x16
// ------------------------------------------------------------------------------------
// LDS row stride chosen so that the ds_read_b128 A-fragment reads are bank-conflict
// free: pixel stride is 80 B (64 B of 32 bf16 channels + 16 B pad -> 5 slots of 16 B,
// odd, so 16 consecutive pixels hit 16 distinct slots); when a 32-row M tile spans
// several output rows, the row stride must shift the slot pattern so that the
// ds_read_b128 lane groups {0-3,12-15,20-27},{4-11,16-19,28-31} stay distinct
// (WOUT 16: S*RS/16 = 0 mod 16; WOUT 8: S*RS/16 = 8 mod 16).  Checked exhaustively by
// tests/test_lds_banks.py.
constexpr int conv_row_stride(int ncols, int wout, int s) {
  int rs = ncols * 80;
  if (wout >= 32) return rs;
  const int want = (wout == 16) ? 0 : 8;
  while (((s * rs / 16) % 16) != want) rs += 16;
  return rs;
}

// PX: bytes per window pixel per plane.  80 = 64 data + 16 pad (conflict-free by padding); 64 =
// no pad, the 16-byte channel chunk q of window row wr stored at chunk q ^ ((wr / S) & 3), which
// keeps the 32x32x16 operand reads and the producer stores conflict-free when a 32-pixel tile is
// 4 output rows of 8 (its rows read window rows S yl + ky: distinct swizzles) -- 20 % less LDS.
template <int CIN, int COUT, int HIN, int S, int NP, int TR, int WM, int WN, int PX = 80>
struct ConvCfg {
  static constexpr int HOUT = HIN / S, WOUT = HOUT;
  static constexpr int RIN = (S == 1) ? TR + 2 : 2 * TR + 1;
  static constexpr int NCOLS = (S == 1) ? HIN + 2 : HIN + 1;
  // (64-byte layout: one spare slot between the even and odd columns, so that a producer store
  // group's odd / even pixel pair never lands 512 bytes apart)
  static constexpr int HALF = PX == 80 ? (NCOLS + 1) / 2 : (NCOLS + 1) / 2 + 1;
  static constexpr int BM = NP * TR * WOUT;
  static constexpr int RT = HOUT / TR;
  static constexpr int MT = BM / WM / 32, NT = COUT / WN / 32;
  static constexpr int NTOT = COUT / 32, NCC = CIN / 32;
  static_assert(PX == 80 || (PX == 64 && (S == 2 || HIN / S == 8)),
                "the 64-byte swizzled layout: stride 2, or 8-wide output rows");
  static constexpr int RS = PX == 80 ? conv_row_stride(NCOLS, WOUT, S)
                                     : (S == 1 ? NCOLS : HALF + NCOLS / 2) * PX;
  static constexpr int PS = RIN * RS;
  static constexpr int PLANE = NP * PS;
  static constexpr int LDS = 2 * PLANE;
  static_assert(WM * WN == 2 || WM * WN == 4 || WM * WN == 8, "2/4/8 waves");
  static_assert(MT >= 1 && NT >= 1 && MT * WM * 32 == BM && NT * WN * 32 == COUT, "tiling");
  static_assert(NP == 1 || TR == HOUT, "multi-patch tiles cover whole patches");
  static_assert((TR * WOUT) % 32 == 0, "M tiles stay inside one patch");
  static constexpr int colofs(int kx) {
    return S == 1 ? kx : ((kx & 1) ? HALF + (kx >> 1) : (kx >> 1));
  }
};

// Blocks b, b+8, b+16, ... are dispatched to the same XCD (MI355X_MICROARCH.md, XCD
// placement; a speed property only).  Give each XCD a contiguous range of tiles so the
// row tiles of one patch -- which share halo rows -- hit the same L2.  Bijective for any
// grid size (cdna_hip_programming.md T1).

// STEM = true (conv1 only): `in` is the raw [P,1,32,32] patch batch; the kernel computes
// input_norm (HardNet.py:306-310) and conv0+BN+ReLU (HardNet.py:281-283) for the window
// rows it needs (VALU fp32, weights uniform -> scalar loads) straight into the LDS window,
// so the 128 KB/patch a0 activation never touches HBM.
template <int CIN, int COUT, int HIN, int S, int NP, int TR, int WM, int WN, bool STEM>
__global__ __launch_bounds__(256) void k_conv3x3(const float* __restrict__ in, float* __restrict__ out,
                                                 const uint4* __restrict__ wp,
                                                 const float* __restrict__ bias, int P,
                                                 const float* __restrict__ stem_w,
                                                 const float* __restrict__ stem_b, float eps,
                                                 int dbg, float relu_lo) {
  using C = ConvCfg<CIN, COUT, HIN, S, NP, TR, WM, WN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int pg = tile / C::RT, rt = tile % C::RT;
  const int p0 = pg * NP, y0 = rt * TR;
  const int r = lane & 31, h = lane >> 5;

  int abase[C::MT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) {
    const int m = (wm * C::MT + mt) * 32 + r;
    const int np = m / (TR * C::WOUT), rem = m % (TR * C::WOUT);
    const int yl = rem / C::WOUT, xo = rem % C::WOUT;
    abase[mt] = np * C::PS + yl * S * C::RS + xo * 80 + h * 16;
  }
  f32x16 acc[C::MT][C::NT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < C::NT; ++nt) acc[mt][nt] = f32x16{};

#pragma unroll 1
  for (int cc = 0; cc < C::NCC; ++cc) {
    if (cc) __syncthreads();
    if constexpr (STEM) {
      static_assert(CIN == 32 && HIN == 32 && S == 1 && NP == 1, "stem fusion is conv1-only");
      float* pt = reinterpret_cast<float*>(smem + C::LDS);  // [34][34] normalised, zero ring
      float* red = pt + 34 * 34;
      const float4 v = reinterpret_cast<const float4*>(in + (size_t)p0 * 1024)[tid];
      for (int i = tid; i < 34 * 34; i += 256) pt[i] = 0.f;
      float mean = 0.f, sd = 1.f;
      if (eps >= 0.f) {
        const float s0 = wave_sum(v.x + v.y + v.z + v.w);
        if (lane == 0) red[wave] = s0;
        __syncthreads();
        mean = (red[0] + red[1] + red[2] + red[3]) * (1.f / 1024.f);
        const float d0 = v.x - mean, d1 = v.y - mean, d2 = v.z - mean, d3 = v.w - mean;
        const float q = wave_sum(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
        if (lane == 0) red[4 + wave] = q;
        __syncthreads();
        sd = sqrtf((red[4] + red[5] + red[6] + red[7]) * (1.f / 1023.f)) + eps;
      }
      __syncthreads();
      {
        const int q = 4 * tid, y = q >> 5, x = q & 31;
        float* d = pt + (y + 1) * 34 + x + 1;
        d[0] = (v.x - mean) / sd; d[1] = (v.y - mean) / sd;
        d[2] = (v.z - mean) / sd; d[3] = (v.w - mean) / sd;
      }
      __syncthreads();
      // conv0 on the MFMA: C[32 ch][32 px] = W0^T[32 ch][16 taps] x X[16 taps][32 px]
      // (taps 9..15 zero), bf16x3.  Lane (r, h) then owns 16 channels of window pixel r.
      constexpr int NPIX = C::RIN * C::NCOLS;
      constexpr int NT0 = (NPIX + 31) / 32;
      bf16x8 w0h, w0l;
      float b16[16];
      {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tap = 8 * h + j;
          const float v = tap < 9 ? stem_w[tap * 32 + r] : 0.f;
          w0h[j] = (__bf16)v;
          w0l[j] = (__bf16)(v - (float)w0h[j]);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) b16[i] = stem_b[(i & 3) + 8 * (i >> 2) + 4 * h];
      }
#pragma unroll 1
      for (int t = wave; t < NT0; t += 4) {
        const int pix = t * 32 + r;
        const int wr = pix / C::NCOLS, wc = pix % C::NCOLS;
        const int y = y0 - 1 + wr, x = wc - 1;
        const bool inside = pix < NPIX && (unsigned)y < 32u && (unsigned)x < 32u;
        const int yc = inside ? y : 0, xc = inside ? x : 0;
        bf16x8 xh, xl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int tap = 8 * h + j;
          const float v = tap < 9 ? pt[(yc + tap / 3) * 34 + xc + tap % 3] : 0.f;
          xh[j] = (__bf16)v;
          xl[j] = (__bf16)(v - (float)xh[j]);
        }
        const f32x16 c0 = mfma3(w0h, w0l, xh, xl, f32x16{});
        if (pix < NPIX) {
          char* dst = smem + wr * C::RS + wc * 80 + 8 * h;
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // channels 8q + 4h + {0..3}
            bf16x4 oh, ol;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float v = inside ? fmaxf(c0[4 * q + j] + b16[4 * q + j], 0.f) : 0.f;
              oh[j] = (__bf16)v;
              ol[j] = (__bf16)(v - (float)oh[j]);
            }
            *reinterpret_cast<uint2*>(dst + 16 * q) = __builtin_bit_cast(uint2, oh);
            *reinterpret_cast<uint2*>(dst + C::PLANE + 16 * q) = __builtin_bit_cast(uint2, ol);
          }
        }
      }
    } else {
      // unit = (window pixel, 8-channel group); thread's units are tid + 256*k.  The
      // window coordinates advance incrementally (no per-unit division); offsets are
      // 32-bit relative to the tile's first patch.
      constexpr int UNITS = NP * C::RIN * C::NCOLS * 4;
      constexpr int DPIX = 256 / 4;                        // pixels advanced per iteration
      constexpr int DWC = DPIX % C::NCOLS, DWR = DPIX / C::NCOLS;
      const float* pin = in + (size_t)p0 * HIN * HIN * CIN + cc * 32;
      const int g = tid & 3;
      int wc = (tid >> 2) % C::NCOLS, wr = (tid >> 2) / C::NCOLS, np = 0;
      while (wr >= C::RIN) { wr -= C::RIN; ++np; }
#pragma unroll 2
      for (int u = tid; u < UNITS; u += 256) {
        const int y = y0 * S - 1 + wr, x = wc - 1;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
        if ((NP == 1 || p0 + np < P) && (unsigned)y < (unsigned)HIN && (unsigned)x < (unsigned)HIN) {
          const float4* src =
              reinterpret_cast<const float4*>(pin + ((np * HIN + y) * HIN + x) * CIN + g * 8);
          a = src[0];
          b = src[1];
        }
        uint4 hi, lo;
        split8(a, b, hi, lo);
        const int pc = (S == 1) ? wc : ((wc & 1) ? C::HALF + (wc >> 1) : (wc >> 1));
        const int off = np * C::PS + wr * C::RS + pc * 80 + g * 16;
        *reinterpret_cast<uint4*>(smem + off) = hi;
        *reinterpret_cast<uint4*>(smem + C::PLANE + off) = lo;
        wc += DWC;
        wr += DWR;
        if (wc >= C::NCOLS) { wc -= C::NCOLS; ++wr; }
        while (wr >= C::RIN) { wr -= C::RIN; ++np; }
      }
    }
    __syncthreads();
    // 18 k-steps (9 taps x 2 halves of the 32-channel chunk), software-pipelined:
    // B fragments (global/L2) are loaded 2 steps ahead, A fragments (LDS) 1 step ahead.
    const uint4* wcc = wp + (size_t)cc * 9 * 2 * C::NTOT * 2 * 64;
    constexpr int NKS = 18;
    uint4 bq[3][C::NT][2];
    uint4 aq[2][C::MT][2];
    auto load_b = [&](int ksx, uint4 (&dst)[C::NT][2]) {
#pragma unroll
      for (int nt = 0; nt < C::NT; ++nt) {
        const int idx = ((ksx * C::NTOT + wn * C::NT + nt) * 2) * 64 + lane;
        dst[nt][0] = wcc[idx];
        dst[nt][1] = wcc[idx + 64];
      }
    };
    auto load_a = [&](int ksx, uint4 (&dst)[C::MT][2]) {
      const int tap = ksx >> 1, ks = ksx & 1;
      const int toff = (tap / 3) * C::RS + C::colofs(tap % 3) * 80 + ks * 32;
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        dst[mt][0] = *reinterpret_cast<const uint4*>(smem + abase[mt] + toff);
        dst[mt][1] = *reinterpret_cast<const uint4*>(smem + C::PLANE + abase[mt] + toff);
      }
    };
    load_b(0, bq[0]);
    load_b(1, bq[1]);
    load_a(0, aq[0]);
#pragma unroll
    for (int ksx = 0; ksx < NKS; ++ksx) {
      if (ksx + 2 < NKS) load_b(ksx + 2, bq[(ksx + 2) % 3]);
      if (ksx + 1 < NKS) load_a(ksx + 1, aq[(ksx + 1) & 1]);
      // pin the issue order: hipcc otherwise sinks the prefetches next to their use
      __builtin_amdgcn_sched_barrier(0);
      // weights are the MFMA A operand (rows = output channels), the activation window
      // the B operand (columns = output pixels): C[channel][pixel], so each lane ends up
      // with 4 consecutive channels of one pixel per register group (16-byte stores).
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        const bf16x8 xh = as_bf16x8(aq[ksx & 1][mt][0]), xl = as_bf16x8(aq[ksx & 1][mt][1]);
#pragma unroll
        for (int nt = 0; nt < C::NT; ++nt)
          acc[mt][nt] = mfma3(as_bf16x8(bq[ksx % 3][nt][0]), as_bf16x8(bq[ksx % 3][nt][1]), xh, xl,
                              acc[mt][nt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // epilogue: + folded-BN bias, ReLU, NHWC fp32 16-byte stores.  acc[mt][nt] is
  // C[channel][pixel]: lane (r, h) holds pixel r of the M tile and channels
  // 8q + 4h + {0..3} (q = 0..3) of the N tile.  Tiles cover whole output rows (and whole
  // patches when NP > 1), so tile pixel m is output pixel (p0*HOUT + y0)*WOUT + m.
  float* obase = out + ((size_t)(p0 * C::HOUT + y0) * C::WOUT + wm * C::MT * 32 + r) * COUT +
                 wn * C::NT * 32 + 4 * h;
#ifdef HN_EXPERIMENTS
  if (dbg & 1) {  // ablation: keep the accumulators live, one store per lane
    float sum = 0.f;
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < C::NT; ++nt)
#pragma unroll
        for (int i = 0; i < 16; ++i) sum += acc[mt][nt][i];
    obase[0] = sum;
    return;
  }
#endif
#pragma unroll
  for (int nt = 0; nt < C::NT; ++nt) {
    float4 bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      bv[q] = *reinterpret_cast<const float4*>(bias + (wn * C::NT + nt) * 32 + 8 * q + 4 * h);
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt) {
      const bool ok = NP == 1 || p0 + ((wm * C::MT + mt) * 32) / (TR * C::WOUT) < P;
      if (!ok) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 v;
        v.x = fmaxf(acc[mt][nt][4 * q + 0] + bv[q].x, relu_lo);
        v.y = fmaxf(acc[mt][nt][4 * q + 1] + bv[q].y, relu_lo);
        v.z = fmaxf(acc[mt][nt][4 * q + 2] + bv[q].z, relu_lo);
        v.w = fmaxf(acc[mt][nt][4 * q + 3] + bv[q].w, relu_lo);
        *reinterpret_cast<float4*>(obase + (size_t)mt * 32 * COUT + nt * 32 + 8 * q) = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// k_conv_pipe: persistent, double-buffered version of k_conv3x3.
//
// Each workgroup loops over its tiles (tile = rb + k*gridDim, rb XCD-remapped) and over
// the 32-channel chunks of each tile ("stages").  While the MFMA K-loop of stage s reads
// LDS buffer s&1, the global loads of stage s+1's window are issued *inside* that loop,
// one unit per K-step after the weight loads of the step (vmcnt retires in issue order,
// so a weight-fragment wait never waits on a younger window load); after the K-loop the
// prefetched registers are split to bf16 hi/lo and written into buffer (s+1)&1, and one
// barrier ends the stage.  STEM (conv1): the next tile's raw patch is prefetched the same
// way and input_norm + conv0 (MFMA) fill the next window.
// ------------------------------------------------------------------------------------
template <int CIN, int COUT, int HIN, int S, int NP, int TR, int WM, int WN, bool STEM, bool CST = false>
struct PipeCfg : ConvCfg<CIN, COUT, HIN, S, NP, TR, WM, WN> {
  using B = ConvCfg<CIN, COUT, HIN, S, NP, TR, WM, WN>;
  static constexpr int NW = WM * WN, NTHR = NW * 64;
  static constexpr int UNITS = NP * B::RIN * B::NCOLS * 4;
  static constexpr int UPT = (UNITS + NTHR - 1) / NTHR;
  static constexpr int BUF = B::LDS;
  static constexpr int PBUF = 2 * BUF;
  static constexpr int SROW = 20;             // CST: floats per pixel row (16 channels + pad)
  static constexpr int SCR = 32 * SROW * 4;   // CST: one 32-pixel x 16-channel half tile per wave
  static constexpr int SMEM = 2 * BUF + (STEM ? 34 * 34 * 4 : 0) + (CST ? NW * SCR : 0);
  static_assert(SMEM <= 160 * 1024, "LDS");
  static_assert(!(STEM && CST), "the CST epilogue scratch starts where the STEM buffers live");
  static_assert(UPT <= 18, "prefetch fits in the K-loop");
};

// ABL (ablation builds only, never shipped): bit0 no weight loads in the K-loop, bit1 no
// LDS fragment reads, bit2 no next-stage staging.
// CST: the epilogue goes through a per-wave LDS scratch, 16 channels at a time, so that each
// store instruction writes 16 pixel rows of 64 bytes instead of 32 x 32 bytes.
template <int CIN, int COUT, int HIN, int S, int NP, int TR, int WM, int WN, bool STEM, int ABL = 0,
          bool CST = false>
__global__ __launch_bounds__(WM * WN * 64, 2) void k_conv_pipe(
    const float* __restrict__ in, float* __restrict__ out, const uint4* __restrict__ wp,
    const float* __restrict__ bias, int P, const float* __restrict__ stem_w,
    const float* __restrict__ stem_b, float eps, float relu_lo) {
  using C = PipeCfg<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM, CST>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int r = lane & 31, h = lane >> 5;
  const int nwg = gridDim.x, rb = xcd_remap(blockIdx.x, nwg);
  const int ntiles = (P + NP - 1) / NP * C::RT;
  const int my_tiles = rb < ntiles ? (ntiles - 1 - rb) / nwg + 1 : 0;
  const int NS = my_tiles * C::NCC;
  if (NS == 0) return;
  // this wave's bias channels, loaded once (an epilogue global load waits behind the next stage's
  // staging loads in vmcnt)
  float4 bvr[C::NT][4];
#pragma unroll
  for (int nt = 0; nt < C::NT; ++nt)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      bvr[nt][q] = *reinterpret_cast<const float4*>(bias + (wn * C::NT + nt) * 32 + 8 * q + 4 * h);

  int abase[C::MT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) {
    const int m = (wm * C::MT + mt) * 32 + r;
    const int np = m / (TR * C::WOUT), rem = m % (TR * C::WOUT);
    const int yl = rem / C::WOUT, xo = rem % C::WOUT;
    abase[mt] = np * C::PS + yl * S * C::RS + xo * 80 + h * 16;
  }

  auto tile_of = [&](int s, int& p0, int& y0) {
    const int t = rb + (s / C::NCC) * nwg;
    p0 = (t / C::RT) * NP;
    y0 = (t % C::RT) * TR;
  };

  // ---------------- window staging (non-stem): prefetch registers -------------------
  float4 pf[C::UPT][2];
  auto prefetch_unit = [&](int s, int k) {
    const int u = tid + k * C::NTHR;
    int p0, y0;
    tile_of(s, p0, y0);
    const int cc = s % C::NCC;
    const int g = u & 3, pix = u >> 2;
    const int wc = pix % C::NCOLS, t2 = pix / C::NCOLS;
    const int wr = t2 % C::RIN, np = t2 / C::RIN;
    const int y = y0 * S - 1 + wr, x = wc - 1;
    pf[k][0] = pf[k][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (u < C::UNITS && (NP == 1 || p0 + np < P) && (unsigned)y < (unsigned)HIN &&
        (unsigned)x < (unsigned)HIN) {
      const float4* src = reinterpret_cast<const float4*>(
          in + ((((size_t)p0 + np) * HIN + y) * HIN + x) * CIN + cc * 32 + g * 8);
      pf[k][0] = src[0];
      pf[k][1] = src[1];
    }
  };
  auto write_unit = [&](char* dst, int k) {
    const int u = tid + k * C::NTHR;
    if (u < C::UNITS) {
      const int g = u & 3, pix = u >> 2;
      const int wc = pix % C::NCOLS, t2 = pix / C::NCOLS;
      const int wr = t2 % C::RIN, np = t2 / C::RIN;
      uint4 hi, lo;
      split8(pf[k][0], pf[k][1], hi, lo);
      const int pc = (S == 1) ? wc : ((wc & 1) ? C::HALF + (wc >> 1) : (wc >> 1));
      const int off = np * C::PS + wr * C::RS + pc * 80 + g * 16;
      *reinterpret_cast<uint4*>(dst + off) = hi;
      *reinterpret_cast<uint4*>(dst + C::PLANE + off) = lo;
    }
  };
  auto write_window = [&](char* dst) {
#pragma unroll
    for (int k = 0; k < C::UPT; ++k) write_unit(dst, k);
  };

  // ---------------- stem staging: raw patch -> input_norm -> conv0 (MFMA) -----------
  float4 pv[4];  // the whole 1024-float patch, per wave (lane l holds float4s l + 64k)
  float* pt = reinterpret_cast<float*>(smem + C::PBUF);
  auto patch_ptr = [&](int s) {
    int p0, y0;
    tile_of(s, p0, y0);
    return reinterpret_cast<const float4*>(in + (size_t)p0 * 1024) + lane;
  };
  if constexpr (STEM) {
    static_assert(CIN == 32 && HIN == 32 && S == 1 && NP == 1, "stem fusion is conv1-only");
    for (int i = tid; i < 34 * 34; i += C::NTHR) pt[i] = 0.f;  // zero ring, interior rewritten
    __syncthreads();
  }
  auto stem_stage = [&](int s, char* dst) {
    int p0, y0;
    tile_of(s, p0, y0);
    float mean = 0.f, sd = 1.f;
    if (eps >= 0.f) {  // HardNet.py:307-310, every wave reduces the full patch itself
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) a += (pv[k].x + pv[k].y) + (pv[k].z + pv[k].w);
      mean = wave_sum(a) * (1.f / 1024.f);
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d0 = pv[k].x - mean, d1 = pv[k].y - mean, d2 = pv[k].z - mean,
                    d3 = pv[k].w - mean;
        q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
      sd = sqrtf(wave_sum(q) * (1.f / 1023.f)) + eps;
    }
    // each wave writes its share of the normalised patch; explicit constant-index cases
    // (a pv[wave] form would be a runtime-indexed array -> scratch)
    const int wu = __builtin_amdgcn_readfirstlane(wave);
#define HN_PUT(K)                                                                          \
  {                                                                                        \
    const int q4 = 4 * (lane + 64 * K), y = q4 >> 5, x = q4 & 31;                          \
    float* d = pt + (y + 1) * 34 + x + 1;                                                  \
    d[0] = (pv[K].x - mean) / sd; d[1] = (pv[K].y - mean) / sd;                             \
    d[2] = (pv[K].z - mean) / sd; d[3] = (pv[K].w - mean) / sd;                             \
  }
    if (wu % 4 == 0 || C::NW == 1) HN_PUT(0)
    if (wu % 4 == 1 || C::NW <= 1) HN_PUT(1)
    if (wu % 4 == 2 || (C::NW <= 2 && wu % 2 == 0)) HN_PUT(2)
    if (wu % 4 == 3 || (C::NW <= 2 && wu % 2 == 1)) HN_PUT(3)
#undef HN_PUT
    __syncthreads();
    constexpr int NPIX = C::RIN * C::NCOLS;
    constexpr int NT0 = (NPIX + 31) / 32;
    bf16x8 w0h, w0l;  // conv0 weights as the A operand (rows = channels), taps 9..15 zero
    {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tap = 8 * h + j;
        const float v = tap < 9 ? stem_w[tap * 32 + r] : 0.f;
        w0h[j] = (__bf16)v;
        w0l[j] = (__bf16)(v - (float)w0h[j]);
      }
    }
#pragma unroll 1
    for (int t = wave; t < NT0; t += C::NW) {
      const int pix = t * 32 + r;
      const int wr = pix / C::NCOLS, wc = pix % C::NCOLS;
      const int y = y0 - 1 + wr, x = wc - 1;
      const bool inside = pix < NPIX && (unsigned)y < 32u && (unsigned)x < 32u;
      const int yc = inside ? y : 0, xc = inside ? x : 0;
      bf16x8 xh, xl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tap = 8 * h + j;
        const float v = tap < 9 ? pt[(yc + tap / 3) * 34 + xc + tap % 3] : 0.f;
        xh[j] = (__bf16)v;
        xl[j] = (__bf16)(v - (float)xh[j]);
      }
      const f32x16 c0 = mfma3(w0h, w0l, xh, xl, f32x16{});
      if (pix < NPIX) {
        char* o = dst + wr * C::RS + wc * 80 + 8 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bf16x4 oh, ol;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float v =
                inside ? fmaxf(c0[4 * q + j] + stem_b[8 * q + 4 * h + j], 0.f) : 0.f;
            oh[j] = (__bf16)v;
            ol[j] = (__bf16)(v - (float)oh[j]);
          }
          *reinterpret_cast<uint2*>(o + 16 * q) = __builtin_bit_cast(uint2, oh);
          *reinterpret_cast<uint2*>(o + C::PLANE + 16 * q) = __builtin_bit_cast(uint2, ol);
        }
      }
    }
  };

  // ---------------- prologue ---------------------------------------------------------
  char* const buf0 = smem;
  char* const buf1 = smem + C::BUF;
  if constexpr (STEM) {
    {
      const float4* pp = patch_ptr(0);
      pv[0] = pp[0]; pv[1] = pp[64]; pv[2] = pp[128]; pv[3] = pp[192];
    }
    stem_stage(0, buf0);
  } else {
#pragma unroll
    for (int k = 0; k < C::UPT; ++k) prefetch_unit(0, k);
    write_window(buf0);
  }
  __syncthreads();

  f32x16 acc[C::MT][C::NT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < C::NT; ++nt) acc[mt][nt] = f32x16{};

#pragma unroll 1
  for (int s = 0; s < NS; ++s) {
    const char* cur = (s & 1) ? buf1 : buf0;
    char* nxt = (s & 1) ? buf0 : buf1;
    const int cc = s % C::NCC;
    const bool more = s + 1 < NS;
    constexpr int NKS = 18;
    constexpr unsigned CHUNK_BYTES = 9 * 2 * C::NTOT * 2 * 64 * 16;
    const __amdgpu_buffer_rsrc_t wr_ = make_rsrc(wp, C::NCC * CHUNK_BYTES);
    const unsigned wvoff = (wn * C::NT * 2 * 64 + lane) * 16;
    const unsigned wsoff = cc * CHUNK_BYTES;
    uint4 bq[3][C::NT][2];
    uint4 aq[2][C::MT][2];
    auto load_b = [&](int ksx, uint4 (&dst)[C::NT][2]) {
#pragma unroll
      for (int nt = 0; nt < C::NT; ++nt) {
        const unsigned k = ((ksx * C::NTOT + nt) * 2) * 64 * 16;
        dst[nt][0] = buf_load16(wr_, wvoff, wsoff + k);
        dst[nt][1] = buf_load16(wr_, wvoff, wsoff + k + 64 * 16);
      }
    };
    auto load_a = [&](int ksx, uint4 (&dst)[C::MT][2]) {
      const int tap = ksx >> 1, ks = ksx & 1;
      const int toff = (tap / 3) * C::RS + C::colofs(tap % 3) * 80 + ks * 32;
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        dst[mt][0] = *reinterpret_cast<const uint4*>(cur + abase[mt] + toff);
        dst[mt][1] = *reinterpret_cast<const uint4*>(cur + C::PLANE + abase[mt] + toff);
      }
    };
    load_b(0, bq[0]);
    load_b(1, bq[1]);
    load_a(0, aq[0]);
#pragma unroll
    for (int ksx = 0; ksx < NKS; ++ksx) {
      if (!(ABL & 1) && ksx + 2 < NKS) load_b(ksx + 2, bq[(ksx + 2) % 3]);
      if ((ABL & 1) && ksx + 2 < NKS) {
#pragma unroll
        for (int nt = 0; nt < C::NT; ++nt) {
          bq[(ksx + 2) % 3][nt][0] = bq[ksx % 3][nt][0];
          bq[(ksx + 2) % 3][nt][1] = bq[ksx % 3][nt][1];
        }
      }
      // next stage's window: the loads of unit ksx are issued at K-step ksx and the unit
      // is split + written into the other LDS buffer two K-steps later (the double buffer
      // makes `nxt` writable for the whole stage), so the staging VALU co-issues with the
      // MFMAs of this wave
      if (!STEM && !(ABL & 4) && more && ksx >= 2 && ksx - 2 < C::UPT) write_unit(nxt, ksx - 2);
      if (!(ABL & 4) && more) {  // next stage's window loads, one unit per K-step
        if constexpr (STEM) {
          if (ksx == 0) pv[0] = patch_ptr(s + 1)[0];
          if (ksx == 1) pv[1] = patch_ptr(s + 1)[64];
          if (ksx == 2) pv[2] = patch_ptr(s + 1)[128];
          if (ksx == 3) pv[3] = patch_ptr(s + 1)[192];
        } else {
          if (ksx < C::UPT) prefetch_unit(s + 1, ksx);
        }
      }
      if (!(ABL & 2) && ksx + 1 < NKS) load_a(ksx + 1, aq[(ksx + 1) & 1]);
      if ((ABL & 2) && ksx + 1 < NKS) {
#pragma unroll
        for (int mt = 0; mt < C::MT; ++mt) {
          aq[(ksx + 1) & 1][mt][0] = aq[ksx & 1][mt][0];
          aq[(ksx + 1) & 1][mt][1] = aq[ksx & 1][mt][1];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        const bf16x8 xh = as_bf16x8(aq[ksx & 1][mt][0]), xl = as_bf16x8(aq[ksx & 1][mt][1]);
#pragma unroll
        for (int nt = 0; nt < C::NT; ++nt)
          acc[mt][nt] = mfma3(as_bf16x8(bq[ksx % 3][nt][0]), as_bf16x8(bq[ksx % 3][nt][1]), xh, xl,
                              acc[mt][nt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    if (cc == C::NCC - 1) {  // epilogue of this tile (see k_conv3x3)
      int p0, y0;
      tile_of(s, p0, y0);
      float* obase = out + ((size_t)(p0 * C::HOUT + y0) * C::WOUT + wm * C::MT * 32 + r) * COUT +
                     wn * C::NT * 32 + 4 * h;
#pragma unroll
      for (int nt = 0; nt < C::NT; ++nt) {
        const float4* bv = bvr[nt];
#pragma unroll
        for (int mt = 0; mt < C::MT; ++mt) {
          const bool ok = NP == 1 || p0 + ((wm * C::MT + mt) * 32) / (TR * C::WOUT) < P;
          if (ok) {
            float* scr = reinterpret_cast<float*>(smem + 2 * C::BUF) + wave * (C::SCR / 4);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float4 v;
              v.x = fmaxf(acc[mt][nt][4 * q + 0] + bv[q].x, relu_lo);
              v.y = fmaxf(acc[mt][nt][4 * q + 1] + bv[q].y, relu_lo);
              v.z = fmaxf(acc[mt][nt][4 * q + 2] + bv[q].z, relu_lo);
              v.w = fmaxf(acc[mt][nt][4 * q + 3] + bv[q].w, relu_lo);
              if constexpr (CST) {
                *reinterpret_cast<float4*>(scr + r * C::SROW + 8 * (q & 1) + 4 * h) = v;
                if (q & 1) {  // channels 16 (q / 2) .. + 15 of the tile: 16 rows of 64 bytes per store
                  __builtin_amdgcn_wave_barrier();
                  asm volatile("" ::: "memory");
                  float* ob = out + ((size_t)(p0 * C::HOUT + y0) * C::WOUT + (wm * C::MT + mt) * 32) * COUT +
                              (wn * C::NT + nt) * 32 + 16 * (q >> 1);
#pragma unroll
                  for (int k = 0; k < 2; ++k) {
                    const int pl = 16 * k + (lane >> 2), c4 = lane & 3;
                    *reinterpret_cast<float4*>(ob + (size_t)pl * COUT + 4 * c4) =
                        *reinterpret_cast<const float4*>(scr + pl * C::SROW + 4 * c4);
                  }
                  __builtin_amdgcn_wave_barrier();
                  asm volatile("" ::: "memory");
                }
              } else {
                *reinterpret_cast<float4*>(obase + (size_t)mt * 32 * COUT + nt * 32 + 8 * q) = v;
              }
            }
          }
          acc[mt][nt] = f32x16{};
        }
      }
    }
    if (!(ABL & 4) && more) {
      if constexpr (STEM) {
        stem_stage(s + 1, nxt);
      } else {
#pragma unroll
        for (int k = NKS - 2; k < C::UPT; ++k) write_unit(nxt, k);  // units beyond the K-loop
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------
// k_conv_ws: warp-specialised persistent conv.  NWC = WM*WN compute waves run the MFMA
// K-loop on LDS buffer s&1 (weight fragments streamed 2 K-steps ahead); 4 producer waves
// own the next stage's window: they issue ALL its global loads at once (their vmcnt is
// their own, so the compute waves' weight waits never queue behind them -- the in-order
// vmcnt problem of k_conv_pipe), then split to bf16 hi/lo into buffer (s+1)&1.  One
// barrier per stage.  For the HBM-heavy stride-2 layers this keeps ~UNITS*32 B per
// workgroup in flight instead of one unit per K-step.
// ------------------------------------------------------------------------------------
template <int CIN, int COUT, int HIN, int S, int NP, int TR, int WM, int WN, bool STEM = false, int PX = 80,
          bool CST = false, bool PST = false>
struct WsCfg : ConvCfg<CIN, COUT, HIN, S, NP, TR, WM, WN, PX> {
  using B = ConvCfg<CIN, COUT, HIN, S, NP, TR, WM, WN, PX>;
  static constexpr int NWC = WM * WN, NWP = 4, NTHR = (NWC + NWP) * 64, PTHR = NWP * 64;
  static constexpr int UNITS = NP * B::RIN * B::NCOLS * 4;
  static constexpr int UPT = STEM ? 1 : (UNITS + PTHR - 1) / PTHR;
  static constexpr int BUF = B::LDS;
  static constexpr int PBUF = 34 * 34 * 4;  // one private normalised patch per producer wave
  static constexpr int SROW = 36;                   // CST: floats per pixel row of the scratch
  static constexpr int SCR = 32 * SROW * 4;          // CST: one 32 x 32 tile per MFMA wave
  // PST: a tile's outputs are staged in the window buffer its last stage has just consumed (pixels
  // below MB) and an extra region (the rest), then stored by the producer waves as whole pixel rows
  static constexpr int OSTR = COUT * 4 + 16;    // bytes per staged output pixel (+16: conflict-free writes)
  static constexpr int OCH = B::BM * COUT / 4;  // 16-byte output chunks per tile
  static constexpr int OPT = OCH / PTHR;
  static constexpr int MB = PST ? (B::BM < BUF / OSTR ? B::BM : BUF / OSTR) : 0;
  static constexpr int XST = PST ? (B::BM - MB) * OSTR : 0;
  // the bias (read by the epilogue from LDS: a global load there queues behind the next stage's
  // weight prefetch in the in-order vmcnt) after the STEM / CST regions, then PST's extra staging
  static constexpr int BIAS_OFF = 2 * BUF + (STEM ? NWP * PBUF : 0) + (CST ? NWC * SCR : 0);
  static constexpr int SMEM = BIAS_OFF + COUT * 4 + XST;
  static constexpr bool DEEP = !STEM && UPT <= 6;  // two stages of loads in flight
  static_assert(SMEM <= 160 * 1024, "LDS");
  static_assert(!(STEM && CST), "the CST epilogue scratch starts where the STEM buffers live");
  static_assert(!PST || (!STEM && !CST && OCH % PTHR == 0), "PST");
};

// STEM (conv1 only): the producers load the raw patch, reduce mean/std per wave, write the
// normalised patch into their own LDS copy (no cross-wave hand-off) and run conv0 on the
// MFMA straight into the next window (input_norm + conv0 + BN + ReLU, HardNet.py:281-283,
// 306-310).
// CST: the epilogue transposes each 32-pixel x 32-channel tile through a per-wave LDS scratch
// so that every store instruction writes 8 whole 128-byte pixel rows (8 lanes per row) instead
// of 32 pixels x 32 bytes.
template <int CIN, int COUT, int HIN, int S, int NP, int TR, int WM, int WN, bool STEM, int ABL = 0,
          int PX = 80, bool CST = false, bool PST = false>
__global__ __launch_bounds__((WM * WN + 4) * 64) void k_conv_ws(
    const float* __restrict__ in, float* __restrict__ out, const uint4* __restrict__ wp,
    const float* __restrict__ bias, int P, const float* __restrict__ stem_w,
    const float* __restrict__ stem_b, float eps, float relu_lo) {
  using C = WsCfg<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM, PX, CST, PST>;
  static_assert(PX == 80 || !STEM, "the stem producer writes the 80-byte layout");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wave >= C::NWC;
  const int r = lane & 31, h = lane >> 5;
  const int nwg = gridDim.x, rb = xcd_remap(blockIdx.x, nwg);
  const int ntiles = (P + NP - 1) / NP * C::RT;
  // STEM: each workgroup takes a contiguous range of tiles, so consecutive stages mostly
  // share a patch and the producers normalise each patch once; otherwise strided tiles.
  const int per = (ntiles + nwg - 1) / nwg;
  const int t_begin = STEM ? rb * per : rb;
  const int my_tiles = STEM ? max(0, min(per, ntiles - t_begin))
                            : (rb < ntiles ? (ntiles - 1 - rb) / nwg + 1 : 0);
  const int NS = my_tiles * C::NCC;
  if (NS == 0) return;
  char* const buf0 = smem;
  char* const buf1 = smem + C::BUF;
  // PST staging slot of output pixel m of the tile whose last stage read buffer `b`
  auto stage_at = [&](const char* b, int m) -> char* {
    return m < C::MB ? const_cast<char*>(b) + m * C::OSTR : smem + C::BIAS_OFF + COUT * 4 + (m - C::MB) * C::OSTR;
  };

  auto tile_of = [&](int s, int& p0, int& y0) {
    const int t = STEM ? t_begin + s / C::NCC : rb + (s / C::NCC) * nwg;
    p0 = (t / C::RT) * NP;
    y0 = (t % C::RT) * TR;
  };
  // ---- producer side ----
  const int ptid = tid - C::NWC * 64;
  float4 pf[C::UPT][2], pf2[C::UPT][2];  // two stages in flight (non-STEM)
  auto produce_loads = [&](int s, float4 (&pf)[C::UPT][2]) {
    int p0, y0;
    tile_of(s, p0, y0);
    const int cc = s % C::NCC;
#pragma unroll
    for (int k = 0; k < C::UPT; ++k) {
      const int u = ptid + k * C::PTHR;
      const int g = u & 3, pix = u >> 2;
      const int wc = pix % C::NCOLS, t2 = pix / C::NCOLS;
      const int wr = t2 % C::RIN, np = t2 / C::RIN;
      const int y = y0 * S - 1 + wr, x = wc - 1;
      pf[k][0] = pf[k][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (u < C::UNITS && (NP == 1 || p0 + np < P) && (unsigned)y < (unsigned)HIN &&
          (unsigned)x < (unsigned)HIN) {
        const float4* src = reinterpret_cast<const float4*>(
            in + ((((size_t)p0 + np) * HIN + y) * HIN + x) * CIN + cc * 32 + g * 8);
        pf[k][0] = src[0];
        pf[k][1] = src[1];
      }
    }
  };
  auto produce_write = [&](char* dst, const float4 (&pf)[C::UPT][2]) {
#pragma unroll
    for (int k = 0; k < C::UPT; ++k) {
      const int u = ptid + k * C::PTHR;
      if (u < C::UNITS) {
        const int g = u & 3, pix = u >> 2;
        const int wc = pix % C::NCOLS, t2 = pix / C::NCOLS;
        const int wr = t2 % C::RIN, np = t2 / C::RIN;
        uint4 hi, lo;
        split8(pf[k][0], pf[k][1], hi, lo);
        const int pc = (S == 1) ? wc : ((wc & 1) ? C::HALF + (wc >> 1) : (wc >> 1));
        const int gs = PX == 80 ? g : g ^ ((wr / S) & 3);  // swizzled chunk (64-byte layout)
        const int off = np * C::PS + wr * C::RS + pc * PX + gs * 16;
        *reinterpret_cast<uint4*>(dst + off) = hi;
        *reinterpret_cast<uint4*>(dst + C::PLANE + off) = lo;
      }
    }
  };

  // PST: after the stage barrier that ends a tile, wait for the MFMA waves to stage the outputs in
  // that stage's buffer (B_x), read them, release the buffer (B_y: the MFMA waves pass it KY K-steps
  // into the next stage, the producers refill the buffer only after it), then store whole pixel rows
  auto pstore = [&](int s, const char* src) {
    int p0, y0;
    tile_of(s, p0, y0);
    // the tile's valid patches only (NP > 1: the batch's last tile may be half empty)
    const int vp = NP == 1 ? 1 : min(NP, P - p0);
    const __amdgpu_buffer_rsrc_t orsrc =
        make_rsrc(out + (size_t)(p0 * C::HOUT + y0) * C::WOUT * COUT, (unsigned)vp * TR * C::WOUT * COUT * 4);
    __syncthreads();  // B_x
    constexpr int G = 8;  // chunks read per batch (the next stage's loads are in flight in pf)
    static_assert(!PST || C::OPT % G == 0, "batches");
#pragma unroll
    for (int k0 = 0; k0 < C::OPT; k0 += G) {
      uint4 rv[G];
#pragma unroll
      for (int k = 0; k < G; ++k) {
        const int c = ptid + (k0 + k) * C::PTHR, m = c / (COUT / 4), j = c % (COUT / 4);
        rv[k] = *reinterpret_cast<const uint4*>(stage_at(src, m) + 16 * j);
      }
#pragma unroll
      for (int k = 0; k < G; ++k) buf_store16(orsrc, rv[k], (unsigned)(ptid * 16), (unsigned)((k0 + k) * C::PTHR * 16));
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B_y
  };

  // ---- stem producer (STEM only) ----
  const int pw_ = wave - C::NWC;
  float* pt = reinterpret_cast<float*>(smem + 2 * C::BUF + (producer ? pw_ : 0) * C::PBUF);
  float4 pv[4];
  int cur_patch = -1;
  bf16x8 w0h{}, w0l{};
  float b16[16];
  if (STEM && producer) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int tap = 8 * h + j;
      const float v = tap < 9 ? stem_w[tap * 32 + r] : 0.f;
      w0h[j] = (__bf16)v;
      w0l[j] = (__bf16)(v - (float)w0h[j]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) b16[i] = stem_b[8 * (i >> 2) + 4 * h + (i & 3)];
  }
  auto stem_loads = [&](int s) {
    int p0, y0;
    tile_of(s, p0, y0);
    if (p0 == cur_patch) return;
    const float4* pp = reinterpret_cast<const float4*>(in + (size_t)p0 * 1024) + lane;
    pv[0] = pp[0]; pv[1] = pp[64]; pv[2] = pp[128]; pv[3] = pp[192];
  };
  auto stem_write = [&](int s, char* dst) {
    int p0, y0;
    tile_of(s, p0, y0);
    if (p0 != cur_patch) {
    cur_patch = p0;
    float mean = 0.f, sd = 1.f;
    if (eps >= 0.f) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) a += (pv[k].x + pv[k].y) + (pv[k].z + pv[k].w);
      mean = wave_sum(a) * (1.f / 1024.f);
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d0 = pv[k].x - mean, d1 = pv[k].y - mean, d2 = pv[k].z - mean,
                    d3 = pv[k].w - mean;
        q += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
      }
      sd = sqrtf(wave_sum(q) * (1.f / 1023.f)) + eps;
    }
    const float inv = 1.f / sd;  // one division; (x-mean)*inv is within 1 ulp of the reference's /
#define HN_PUT(K)                                                                          \
  {                                                                                        \
    const int q4 = 4 * (lane + 64 * K), y = q4 >> 5, x = q4 & 31;                          \
    float* d = pt + (y + 1) * 34 + x + 1;                                                  \
    d[0] = (pv[K].x - mean) * inv; d[1] = (pv[K].y - mean) * inv;                           \
    d[2] = (pv[K].z - mean) * inv; d[3] = (pv[K].w - mean) * inv;                           \
  }
    HN_PUT(0) HN_PUT(1) HN_PUT(2) HN_PUT(3)
#undef HN_PUT
    }
    constexpr int NPIX = C::RIN * C::NCOLS;
    constexpr int NT0 = (NPIX + 31) / 32;
#pragma unroll 1
    for (int t = pw_; t < NT0; t += C::NWP) {
      const int pix = t * 32 + r;
      const int wr = pix / C::NCOLS, wc = pix % C::NCOLS;
      const int y = y0 - 1 + wr, x = wc - 1;
      const bool inside = pix < NPIX && (unsigned)y < 32u && (unsigned)x < 32u;
      const int yc = inside ? y : 0, xc = inside ? x : 0;
      bf16x8 xh, xl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tap = 8 * h + j;
        const float v = tap < 9 ? pt[(yc + tap / 3) * 34 + xc + tap % 3] : 0.f;
        xh[j] = (__bf16)v;
        xl[j] = (__bf16)(v - (float)xh[j]);
      }
      const f32x16 c0 = mfma3(w0h, w0l, xh, xl, f32x16{});
      if (pix < NPIX) {
        char* o = dst + wr * C::RS + wc * 80 + 8 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bf16x4 oh, ol;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float v = inside ? fmaxf(c0[4 * q + j] + b16[4 * q + j], 0.f) : 0.f;
            oh[j] = (__bf16)v;
            ol[j] = (__bf16)(v - (float)oh[j]);
          }
          *reinterpret_cast<uint2*>(o + 16 * q) = __builtin_bit_cast(uint2, oh);
          *reinterpret_cast<uint2*>(o + C::PLANE + 16 * q) = __builtin_bit_cast(uint2, ol);
        }
      }
    }
  };

  if (producer) {
    if constexpr (STEM) {
      static_assert(CIN == 32 && HIN == 32 && S == 1 && NP == 1, "stem fusion is conv1-only");
      for (int i = lane; i < 34 * 34; i += 64) pt[i] = 0.f;  // own zero ring
      stem_loads(0);
      stem_write(0, buf0);
    } else {
      produce_loads(0, pf);
      produce_write(buf0, pf);
      if (NS > 1) produce_loads(1, pf);
    }
  } else {
    for (int i = tid; i < COUT; i += C::NWC * 64) reinterpret_cast<float*>(smem + C::BIAS_OFF)[i] = bias[i];
  }
  __syncthreads();

  if (producer) {
    if constexpr ((ABL & 32) != 0) {  // timing only: no barriers at all
    } else if constexpr ((ABL & 8) != 0) {  // timing only: idle producers
#pragma unroll 1
      for (int s = 0; s < NS; ++s) __syncthreads();
    } else if constexpr (STEM) {
#pragma unroll 1
      for (int s = 0; s < NS; ++s) {
        if (s + 1 < NS) {
          stem_loads(s + 1);
          stem_write(s + 1, (s & 1) ? buf0 : buf1);
        }
        __syncthreads();
      }
    } else if constexpr (!C::DEEP) {
#pragma unroll 1
      for (int s = 0; s < NS; ++s) {
        if (s + 1 < NS) {
          produce_write((s & 1) ? buf0 : buf1, pf);
          if (s + 2 < NS) produce_loads(s + 2, pf);
        }
        __syncthreads();
        if constexpr (PST)
          if (s % C::NCC == C::NCC - 1) pstore(s, (s & 1) ? buf1 : buf0);
      }
    } else {
      // stage s + 2's loads are issued before stage s + 1 is written, so each load has two
      // stages of MFMA work to land in
#pragma unroll 1
      for (int s = 0; s < NS; s += 2) {
        if (s + 2 < NS) produce_loads(s + 2, pf2);
        if (s + 1 < NS) produce_write(buf1, pf);
        __syncthreads();
        if constexpr (PST)
          if (s % C::NCC == C::NCC - 1) pstore(s, buf0);
        if (s + 1 >= NS) break;
        if (s + 3 < NS) produce_loads(s + 3, pf);
        if (s + 2 < NS) produce_write(buf0, pf2);
        __syncthreads();
        if constexpr (PST)
          if ((s + 1) % C::NCC == C::NCC - 1) pstore(s + 1, buf1);
      }
    }
    return;
  }

  // ---- compute side ----
  const int wm = wave / WN, wn = wave % WN;
  // the bias from LDS (a global load in the epilogue would wait for the weight prefetch ahead of it
  // in vmcnt; with PST it would hold up every wave after the tile's last stage barrier)
  const float* const sbias = reinterpret_cast<const float*>(smem + C::BIAS_OFF);
  int abase[C::MT], ylr[C::MT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) {
    const int m = (wm * C::MT + mt) * 32 + r;
    const int np = m / (TR * C::WOUT), rem = m % (TR * C::WOUT);
    const int yl = rem / C::WOUT, xo = rem % C::WOUT;
    abase[mt] = np * C::PS + yl * S * C::RS + xo * PX + (PX == 80 ? h * 16 : 0);
    ylr[mt] = yl;
  }
  constexpr unsigned CHUNK_BYTES = 9 * 2 * C::NTOT * 2 * 64 * 16;
  const __amdgpu_buffer_rsrc_t wr_ = make_rsrc(wp, C::NCC * CHUNK_BYTES);
  const unsigned wvoff = (wn * C::NT * 2 * 64 + lane) * 16;
  f32x16 acc[C::MT][C::NT];
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < C::NT; ++nt) acc[mt][nt] = f32x16{};

  constexpr int NKS = 18;
  // weight fragments of K-step k of channel chunk cc; a stage's first two K-steps are
  // fetched during the previous stage's last two, i.e. before its epilogue stores, which
  // would otherwise sit in front of them in the in-order vmcnt queue
  auto load_b = [&](int cc, int ksx, uint4 (&dst)[C::NT][2]) {
#pragma unroll
    for (int nt = 0; nt < C::NT; ++nt) {
      const unsigned k = cc * CHUNK_BYTES +
                         (((ABL & 1) ? 0 : ksx) * C::NTOT + nt) * 2 * 64 * 16;  // ABL 1: timing only
      dst[nt][0] = buf_load16(wr_, wvoff, k);
      dst[nt][1] = buf_load16(wr_, wvoff, k + 64 * 16);
    }
  };
  constexpr int WD = 3;  // weight ring depth: K-step fragments loaded WD - 1 steps ahead
  static_assert(NKS % WD == 0, "the weight ring runs on across stages");
  uint4 bq[WD][C::NT][2];
#pragma unroll
  for (int k = 0; k + 1 < WD; ++k) load_b(0, k, bq[k]);
#pragma unroll 1
  for (int s = 0; s < NS; ++s) {
    const char* cur = (s & 1) ? buf1 : buf0;
    const int cc = s % C::NCC, ccn = (s + 1) % C::NCC;
    uint4 aq[2][C::MT][2];
    auto load_a = [&](int ksx, uint4 (&dst)[C::MT][2]) {
      const int tap = (ABL & 2) ? 0 : ksx >> 1, ks = (ABL & 2) ? 0 : ksx & 1;  // ABL 2: timing only
      const int toff = (tap / 3) * C::RS + C::colofs(tap % 3) * PX + (PX == 80 ? ks * 32 : 0);
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        // 64-byte layout: chunk 2 ks + h of window row 2 yl + ky sits at (2 ks + h) ^ ((yl + ky / 2) & 3)
        const int co = PX == 80 ? 0 : 16 * ((2 * ks + h) ^ ((ylr[mt] + (tap / 3) / S) & 3));
        dst[mt][0] = *reinterpret_cast<const uint4*>(cur + abase[mt] + toff + co);
        dst[mt][1] = *reinterpret_cast<const uint4*>(cur + C::PLANE + abase[mt] + toff + co);
      }
    };
    load_a(0, aq[0]);
#pragma unroll
    for (int ksx = 0; ksx < NKS; ++ksx) {
      if (ksx + WD - 1 < NKS)
        load_b(cc, ksx + WD - 1, bq[(ksx + WD - 1) % WD]);
      else  // the next stage's first fragments, unconditionally (valid weights even after the last
            // stage): a branch here made the compiler's vmcnt merge wait vmcnt(0) at the stage's end
        load_b(ccn, ksx + WD - 1 - NKS, bq[(ksx + WD - 1) % WD]);
      if (ksx + 1 < NKS) load_a(ksx + 1, aq[(ksx + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (PST) {
        // B_y of the previous tile (see pstore), at the first K-step: same-box conv4 6.93 ms there,
        // 6.95 at K-step 1, 7.02 at 2, 7.09 at 4; the producers' window writes wait for it
        if (ksx == 0 && cc == 0 && s > 0) __builtin_amdgcn_s_barrier();
      }
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        const bf16x8 xh = as_bf16x8(aq[ksx & 1][mt][0]), xl = as_bf16x8(aq[ksx & 1][mt][1]);
#pragma unroll
        for (int nt = 0; nt < C::NT; ++nt) {
          if constexpr (ABL & 16)  // timing only: no MFMA, operands kept live
            acc[mt][nt][0] += __builtin_bit_cast(float, aq[ksx & 1][mt][0].x ^ aq[ksx & 1][mt][1].y ^
                                                           bq[ksx % WD][nt][0].z ^ bq[ksx % WD][nt][1].w);
          else
            acc[mt][nt] = mfma3(as_bf16x8(bq[ksx % WD][nt][0]), as_bf16x8(bq[ksx % WD][nt][1]), xh,
                                xl, acc[mt][nt]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (PST && cc == C::NCC - 1) {
      __syncthreads();  // B_s: the stage's buffer is free
      char* stg = const_cast<char*>(cur);
#pragma unroll
      for (int nt = 0; nt < C::NT; ++nt) {
        float4 bv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          bv[q] = *reinterpret_cast<const float4*>(sbias + (wn * C::NT + nt) * 32 + 8 * q + 4 * h);
#pragma unroll
        for (int mt = 0; mt < C::MT; ++mt) {
          char* o = stage_at(stg, (wm * C::MT + mt) * 32 + r) + ((wn * C::NT + nt) * 32 + 4 * h) * 4;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float4 v;
            v.x = fmaxf(acc[mt][nt][4 * q + 0] + bv[q].x, relu_lo);
            v.y = fmaxf(acc[mt][nt][4 * q + 1] + bv[q].y, relu_lo);
            v.z = fmaxf(acc[mt][nt][4 * q + 2] + bv[q].z, relu_lo);
            v.w = fmaxf(acc[mt][nt][4 * q + 3] + bv[q].w, relu_lo);
            *reinterpret_cast<float4*>(o + 32 * q) = v;
          }
          acc[mt][nt] = f32x16{};
        }
      }
      __syncthreads();  // B_x
      continue;
    }
    if (cc == C::NCC - 1) {
      int p0, y0;
      tile_of(s, p0, y0);
      float* obase = out + ((size_t)(p0 * C::HOUT + y0) * C::WOUT + wm * C::MT * 32 + r) * COUT +
                     wn * C::NT * 32 + 4 * h;
#pragma unroll
      for (int nt = 0; nt < C::NT; ++nt) {
        float4 bv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          bv[q] = *reinterpret_cast<const float4*>(sbias + (wn * C::NT + nt) * 32 + 8 * q + 4 * h);
#pragma unroll
        for (int mt = 0; mt < C::MT; ++mt) {
          const bool ok = NP == 1 || p0 + ((wm * C::MT + mt) * 32) / (TR * C::WOUT) < P;
          if (ok) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float4 v;
              v.x = fmaxf(acc[mt][nt][4 * q + 0] + bv[q].x, relu_lo);
              v.y = fmaxf(acc[mt][nt][4 * q + 1] + bv[q].y, relu_lo);
              v.z = fmaxf(acc[mt][nt][4 * q + 2] + bv[q].z, relu_lo);
              v.w = fmaxf(acc[mt][nt][4 * q + 3] + bv[q].w, relu_lo);
              if constexpr (CST) {
                float* scr = reinterpret_cast<float*>(smem + 2 * C::BUF) + wave * (C::SCR / 4);
                *reinterpret_cast<float4*>(scr + r * C::SROW + 8 * q + 4 * h) = v;
              } else if (!(ABL & 4) || v.x == 1234.5f) {  // ABL 4: timing only, no stores
                *reinterpret_cast<float4*>(obase + (size_t)mt * 32 * COUT + nt * 32 + 8 * q) = v;
              }
            }
          }
          if (CST && ok) {  // same wave: its LDS accesses execute in order
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const float* scr = reinterpret_cast<const float*>(smem + 2 * C::BUF) + wave * (C::SCR / 4);
            float* ob = out + ((size_t)(p0 * C::HOUT + y0) * C::WOUT + (wm * C::MT + mt) * 32) * COUT +
                        (wn * C::NT + nt) * 32;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const int pl = 8 * k + (lane >> 3), c4 = lane & 7;
              *reinterpret_cast<float4*>(ob + (size_t)pl * COUT + 4 * c4) =
                  *reinterpret_cast<const float4*>(scr + pl * C::SROW + 4 * c4);
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
          }
          acc[mt][nt] = f32x16{};
        }
      }
    }
    if constexpr (!(ABL & 32)) __syncthreads();
  }
  if constexpr (PST) __builtin_amdgcn_s_barrier();  // B_y of the last tile
}

// ------------------------------------------------------------------------------------
// head: [P, K] x [K, 128] + bias, L2 normalise rows.  4 waves = 2 (M) x 2 (N);
// each wave 32 patches x 64 columns.
// ------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void k_head(const float* __restrict__ a, float* __restrict__ out,
                                              const uint4* __restrict__ wp,
                                              const float* __restrict__ bias, int P, float l2eps) {
  __shared__ float ssq[2][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  const int pbase = blockIdx.x * 64 + wm * 32;
  const int pa = min(pbase + r, P - 1);
  const float* arow = a + (size_t)pa * K + h * 8;
  f32x16 acc[2] = {f32x16{}, f32x16{}};
#pragma unroll 4
  for (int ks = 0; ks < K / 16; ++ks) {
    const float4 x0 = *reinterpret_cast<const float4*>(arow + ks * 16);
    const float4 x1 = *reinterpret_cast<const float4*>(arow + ks * 16 + 4);
    uint4 hi, lo;
    split8(x0, x1, hi, lo);
    const bf16x8 ah = as_bf16x8(hi), al = as_bf16x8(lo);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int idx = ((ks * 4 + wn * 2 + nt) * 2) * 64 + lane;
      acc[nt] = mfma3(ah, al, as_bf16x8(wp[idx]), as_bf16x8(wp[idx + 64]), acc[nt]);
    }
  }
  float b0 = bias[wn * 64 + r], b1 = bias[wn * 64 + 32 + r];
  float part[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc[0][i] += b0;
    acc[1][i] += b1;
    part[i] = half_sum(acc[0][i] * acc[0][i] + acc[1][i] * acc[1][i]);
  }
  if (r == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) ssq[wn][wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h] = part[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    const int p = pbase + row;
    const float norm = sqrtf(ssq[0][wm * 32 + row] + ssq[1][wm * 32 + row] + l2eps);
    if (p < P) {
      out[(size_t)p * 128 + wn * 64 + r] = acc[0][i] / norm;
      out[(size_t)p * 128 + wn * 64 + 32 + r] = acc[1][i] / norm;
    }
  }
}

// ------------------------------------------------------------------------------------
// k_head2: the same GEMM + bias + L2 with both operands staged through double-buffered LDS
// in K-chunks of 32: all global loads of chunk c+1 are issued before the MFMAs of chunk c
// (A rows fp32 -> bf16 hi/lo, 80-byte rows = conflict-free ds_read_b128; B fragments
// copied linearly), so the K-loop reads only LDS.  4 waves = 2 (M: 32 patches) x 2 (N: 64).
// ------------------------------------------------------------------------------------
template <int K, bool F16>
__global__ __launch_bounds__(256) void k_head2(const float* __restrict__ a, float* __restrict__ out,
                                               const uint4* __restrict__ wp,
                                               const float* __restrict__ bias, int P, float l2eps) {
  constexpr int KC = 32, NCH = K / KC;
  constexpr int AROW = 80;                    // bytes per patch row per plane (64 data + 16 pad)
  constexpr int APLANE = 64 * AROW;           // 64 patches
  constexpr int ABYTES = 2 * APLANE;          // hi + lo
  constexpr int BBYTES = 2 * 4 * 2 * 64 * 16;  // 2 k-steps x 4 ntiles x 2 planes x 1 KB
  constexpr int BUF = ABYTES + BBYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  __shared__ float ssq[2][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  const int pbase = blockIdx.x * 64;
  // staging assignment: A = 64 rows x 32 fp32 = 512 float4 (2 per thread);
  // B = 2 ks x 4 nt x 2 planes x 64 lanes = 1024 uint4 (4 per thread)
  const int arow0 = tid >> 3, acol = (tid & 7) * 4;  // rows arow0 and arow0 + 32
  const int pa0 = min(pbase + arow0, P - 1), pa1 = min(pbase + arow0 + 32, P - 1);
  float4 ra0, ra1;
  uint4 rb0, rb1, rb2, rb3;  // named registers: an indexed array here ends up in scratch
#define HN_LOAD_CHUNK(c)                                                                   \
  {                                                                                        \
    ra0 = *reinterpret_cast<const float4*>(a + (size_t)pa0 * K + (c) * KC + acol);         \
    ra1 = *reinterpret_cast<const float4*>(a + (size_t)pa1 * K + (c) * KC + acol);         \
    const uint4* wc_ = wp + (size_t)(c) * 1024 + tid;                                      \
    rb0 = wc_[0]; rb1 = wc_[256]; rb2 = wc_[512]; rb3 = wc_[768];                          \
  }
  auto put_row = [&](char* buf, int row, const float4 v) {
    uint2 hv, lv;
    if (F16) {  // fp16x3 split (hn_common.h split8_f16)
      typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
      f16x4 hi, lo;
      hi[0] = (_Float16)v.x; lo[0] = (_Float16)(v.x - (float)hi[0]);
      hi[1] = (_Float16)v.y; lo[1] = (_Float16)(v.y - (float)hi[1]);
      hi[2] = (_Float16)v.z; lo[2] = (_Float16)(v.z - (float)hi[2]);
      hi[3] = (_Float16)v.w; lo[3] = (_Float16)(v.w - (float)hi[3]);
      hv = __builtin_bit_cast(uint2, hi);
      lv = __builtin_bit_cast(uint2, lo);
    } else {
      bf16x4 hi, lo;
      hi[0] = (__bf16)v.x; lo[0] = (__bf16)(v.x - (float)hi[0]);
      hi[1] = (__bf16)v.y; lo[1] = (__bf16)(v.y - (float)hi[1]);
      hi[2] = (__bf16)v.z; lo[2] = (__bf16)(v.z - (float)hi[2]);
      hi[3] = (__bf16)v.w; lo[3] = (__bf16)(v.w - (float)hi[3]);
      hv = __builtin_bit_cast(uint2, hi);
      lv = __builtin_bit_cast(uint2, lo);
    }
    *reinterpret_cast<uint2*>(buf + row * AROW + acol * 2) = hv;
    *reinterpret_cast<uint2*>(buf + APLANE + row * AROW + acol * 2) = lv;
  };
#define HN_STORE_CHUNK(buf)                                                                \
  {                                                                                        \
    put_row(buf, arow0, ra0);                                                              \
    put_row(buf, arow0 + 32, ra1);                                                         \
    uint4* bd_ = reinterpret_cast<uint4*>(buf + ABYTES) + tid;                             \
    bd_[0] = rb0; bd_[256] = rb1; bd_[512] = rb2; bd_[768] = rb3;                          \
  }
  f32x16 acc[2] = {f32x16{}, f32x16{}};
  HN_LOAD_CHUNK(0)
  HN_STORE_CHUNK(smem)
  __syncthreads();
#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    const char* cur = smem + (c & 1) * BUF;
    if (c + 1 < NCH) HN_LOAD_CHUNK(c + 1)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int aoff = (wm * 32 + r) * AROW + ks * 32 + h * 16;
      const uint4 ah = *reinterpret_cast<const uint4*>(cur + aoff);
      const uint4 al = *reinterpret_cast<const uint4*>(cur + APLANE + aoff);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int boff = ABYTES + (((ks * 4 + wn * 2 + nt) * 2) * 64 + lane) * 16;
        const uint4 bh = *reinterpret_cast<const uint4*>(cur + boff);
        const uint4 bl = *reinterpret_cast<const uint4*>(cur + boff + 64 * 16);
        if (F16)
          acc[nt] = mfma3_f16(as_f16x8(ah), as_f16x8(al), as_f16x8(bh), as_f16x8(bl), acc[nt]);
        else
          acc[nt] = mfma3(as_bf16x8(ah), as_bf16x8(al), as_bf16x8(bh), as_bf16x8(bl), acc[nt]);
      }
    }
    if (c + 1 < NCH) HN_STORE_CHUNK(smem + ((c + 1) & 1) * BUF)
    __syncthreads();
  }
#undef HN_LOAD_CHUNK
#undef HN_STORE_CHUNK
  const float b0 = bias[wn * 64 + r], b1 = bias[wn * 64 + 32 + r];
  float part[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc[0][i] += b0;
    acc[1][i] += b1;
    part[i] = half_sum(acc[0][i] * acc[0][i] + acc[1][i] * acc[1][i]);
  }
  if (r == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) ssq[wn][wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h] = part[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    const int p = pbase + wm * 32 + row;
    const float norm = sqrtf(ssq[0][wm * 32 + row] + ssq[1][wm * 32 + row] + l2eps);
    if (p < P) {
      out[(size_t)p * 128 + wn * 64 + r] = acc[0][i] / norm;
      out[(size_t)p * 128 + wn * 64 + 32 + r] = acc[1][i] / norm;
    }
  }
}

// ------------------------------------------------------------------------------------
// k_head3: the same GEMM + bias + L2 fed by LDS-DMA (global_load_lds_dwordx4) into rings of
// K-chunks, so no register holds a staged operand: A (the activations, from HBM) in a DA-deep
// ring and B (the weights, L2 / MALL) in a DB-deep one.  128 patches per workgroup, 8 waves =
// 4 (M: 32 patches) x 2 (N: 64 columns); at the HardNet chunk of 32,768 patches one workgroup
// per CU.
//   A (fp32): 128 rows x 128 B per chunk; the 16-byte piece c of row j lands at piece
//     c ^ ((j >> 1) & 7) (the swizzle rides on the per-lane SOURCE address, the DMA image being
//     lane-linear), so each 16-lane ds_read_b128 group of a fragment read (16 consecutive rows,
//     one logical piece) hits 16 distinct bank slots; each wave splits its own fragments to
//     hi / lo at read time.
//   B: the chunk's 16 KB of pre-split fragments ([ks][4 n-tiles][hi, lo][64 lanes], the k_head2
//     packing) copied linearly.
// Iteration j issues B(j + DB - 1) and then A(j + DA - 1) (2 + 2 DMA instructions per wave; the
// prologue is iterations 1 - max(DA, DB) .. -1).  vmcnt retires in issue order, so at the top of
// iteration c the wave waits until only the instructions issued after the later of A(c) / B(c)
// are outstanding -- B first in each iteration lets a shallow B ring keep the deeper A chunks in
// flight -- then lgkmcnt(0) + s_barrier (every wave's chunk c landed; chunk c - 1's slots free
// for the refills).  The DMA is inline asm (M0 set and restored in the same statement) so hipcc
// does not track it as an LDS write.  Accumulation order = k_head2's (bit-identical results).
//
// SPLIT > 1 (small batches, hn_launch_head): workgroup (block, s) runs only K-chunks s NCH / SPLIT ..
// (s + 1) NCH / SPLIT - 1 and writes its raw accumulators to part[s][P][128]; k_head_fin sums the SPLIT
// partials in order s = 0, 1, .. and adds the bias and the L2 norm.  At the reference eval loop's 512
// patches one unsplit workgroup per 128 patches would leave 252 of 256 CUs idle while each streams all
// 8,192 K (its 4 MB of weights and 4 MB of activations through one CU's LDS-DMA path: ~0.2 ms).
// ------------------------------------------------------------------------------------
template <int N>
HN_DEV void head_wait_vm() {  // s_waitcnt vmcnt(N), lgkmcnt / expcnt untouched
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int K, bool F16, int DA, int DB, int SPLIT = 1>
__global__ __launch_bounds__(512) void k_head3(const float* __restrict__ a, float* __restrict__ out,
                                               const uint4* __restrict__ wp,
                                               const float* __restrict__ bias, int P, float l2eps,
                                               float* __restrict__ part = nullptr) {
  constexpr int KC = 32, NCH = K / KC / SPLIT, M = 128;  // NCH: this workgroup's K-chunks
  static_assert((K / KC) % SPLIT == 0, "split");
  constexpr int ABYTES = M * KC * 4;           // 16 KB per A chunk
  constexpr int BBYTES = 2 * 4 * 2 * 64 * 16;  // 16 KB per B chunk
  static_assert(ABYTES == 16 * 1024 && BBYTES == 16 * 1024, "two DMA instructions per wave each");
  static_assert(DA >= 2 && DB >= 2 && NCH >= DA && NCH >= DB && (DA + DB) * 16 <= 152, "rings");
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  __shared__ __attribute__((aligned(16))) char sa[DA * ABYTES];
  __shared__ __attribute__((aligned(16))) char sbw[DB * BBYTES];
  __shared__ float ssq[2][M];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;
  const int pbase = blockIdx.x * M;
  const int kc0 = SPLIT > 1 ? (int)blockIdx.y * NCH : 0;  // the first K-chunk of this workgroup

  // this wave's DMA instructions 2 wave + k (k = 0, 1) of each chunk; chunk c adds c * KC floats
  // (A) / c * 1024 uint4 (B) to the source
  const float* asrc[2];
  const uint4* bsrc[2];
  unsigned adst[2], bdst[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int gi = 2 * wave + k, s = gi * 64 + lane, row = s >> 3, c = (s & 7) ^ ((row >> 1) & 7);
    asrc[k] = a + (size_t)min(pbase + row, P - 1) * K + c * 4 + (size_t)kc0 * KC;
    bsrc[k] = wp + gi * 64 + lane + (size_t)kc0 * 1024;
    adst[k] = (unsigned)(uintptr_t)(lds_ptr_t)(sa + gi * 1024);
    bdst[k] = (unsigned)(uintptr_t)(lds_ptr_t)(sbw + gi * 1024);
  }
  auto dma = [](const void* src, unsigned dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  };
  auto live = [](int chunk) { return chunk >= 0 && chunk < NCH; };
  auto issue = [&](int j) {  // iteration j's DMA: B(j + DB - 1), then A(j + DA - 1)
    const int cb = j + DB - 1, ca = j + DA - 1;
    if (live(cb)) {
      const unsigned so = (unsigned)(cb % DB) * BBYTES;
      dma(bsrc[0] + (size_t)cb * 1024, bdst[0] + so);
      dma(bsrc[1] + (size_t)cb * 1024, bdst[1] + so);
    }
    if (live(ca)) {
      const unsigned so = (unsigned)(ca % DA) * ABYTES;
      dma(asrc[0] + (size_t)ca * KC, adst[0] + so);
      dma(asrc[1] + (size_t)ca * KC, adst[1] + so);
    }
  };
  // DMA instructions issued after the later of A(c) / B(c) (this wave's own; even, <= 2 (DA + DB))
  auto after = [&](int c) {
    constexpr int MN = DA < DB ? DA : DB;
    int n = 0;
    for (int i = c - MN + 2; i < c; ++i) n += 2 * live(i + DB - 1) + 2 * live(i + DA - 1);
    if (DB < DA) n += 2 * live(c - DB + 1 + DA - 1);  // the A half of B(c)'s iteration
    return n;
  };
  const int arow = 32 * wm + r, asw = (arow >> 1) & 7;
  f32x16 acc[2] = {f32x16{}, f32x16{}};
  for (int j = 1 - (DA > DB ? DA : DB); j < 0; ++j) issue(j);
#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    switch (after(c)) {
      case 0: head_wait_vm<0>(); break;
      case 2: head_wait_vm<2>(); break;
      case 4: head_wait_vm<4>(); break;
      case 6: head_wait_vm<6>(); break;
      case 8: head_wait_vm<8>(); break;
      case 10: head_wait_vm<10>(); break;
      case 12: head_wait_vm<12>(); break;
      default: head_wait_vm<14>(); break;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue(c);
    const char* ast = sa + (c % DA) * ABYTES + arow * (KC * 4);
    const char* bst = sbw + (c % DB) * BBYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int p0 = 4 * ks + 2 * h;
      const float4 x0 = *reinterpret_cast<const float4*>(ast + ((p0 ^ asw) << 4));
      const float4 x1 = *reinterpret_cast<const float4*>(ast + (((p0 + 1) ^ asw) << 4));
      uint4 ah, al;
      if (F16) split8_f16(x0, x1, ah, al);
      else split8(x0, x1, ah, al);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const char* bp = bst + ((((ks * 4 + wn * 2 + nt) * 2) * 64 + lane) << 4);
        const uint4 bh = *reinterpret_cast<const uint4*>(bp);
        const uint4 bl = *reinterpret_cast<const uint4*>(bp + 1024);
        if (F16)
          acc[nt] = mfma3_f16(as_f16x8(ah), as_f16x8(al), as_f16x8(bh), as_f16x8(bl), acc[nt]);
        else
          acc[nt] = mfma3(as_bf16x8(ah), as_bf16x8(al), as_bf16x8(bh), as_bf16x8(bl), acc[nt]);
      }
    }
  }
  if constexpr (SPLIT > 1) {  // raw partial sums of this K range (k_head_fin finishes)
    float* pp = part + (size_t)blockIdx.y * P * 128;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int p = pbase + wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
      if (p < P) {
        pp[(size_t)p * 128 + wn * 64 + r] = acc[0][i];
        pp[(size_t)p * 128 + wn * 64 + 32 + r] = acc[1][i];
      }
    }
    return;
  }
  const float b0 = bias[wn * 64 + r], b1 = bias[wn * 64 + 32 + r];
  float part_ss[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    acc[0][i] += b0;
    acc[1][i] += b1;
    part_ss[i] = half_sum(acc[0][i] * acc[0][i] + acc[1][i] * acc[1][i]);
  }
  if (r == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) ssq[wn][wm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h] = part_ss[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    const int p = pbase + wm * 32 + row;
    const float norm = sqrtf(ssq[0][wm * 32 + row] + ssq[1][wm * 32 + row] + l2eps);
    if (p < P) {
      out[(size_t)p * 128 + wn * 64 + r] = acc[0][i] / norm;
      out[(size_t)p * 128 + wn * 64 + 32 + r] = acc[1][i] / norm;
    }
  }
}

// k_head3's SPLIT partials [SPLIT][P][128] summed in split order + bias, then y / sqrt(sum y^2 + l2eps) (the
// two 64-column halves summed apart, then added, as k_head3).  32 lanes per patch, 4 columns each.
template <int SPLIT>
__global__ __launch_bounds__(256) void k_head_fin(const float* __restrict__ part, float* __restrict__ out,
                                                  const float* __restrict__ bias, int P, float l2eps) {
  const int t = threadIdx.x;
  const int p = blockIdx.x * 8 + (t >> 5);
  const int n = (t & 31) * 4;
  if (p >= P) return;  // (a whole 32-lane half-wave: the shuffles below stay inside it)
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int s = 0; s < SPLIT; ++s) {
    const float4 q = *reinterpret_cast<const float4*>(part + ((size_t)s * P + p) * 128 + n);
    v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
  }
  const float4 b = *reinterpret_cast<const float4*>(bias + n);
  v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
  float ss = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) ss += __shfl_xor(ss, o);  // each 64-column half (16 lanes)
  ss += __shfl_xor(ss, 16);                                  // the two halves
  const float norm = sqrtf(ss + l2eps);
  v.x /= norm; v.y /= norm; v.z /= norm; v.w /= norm;
  *reinterpret_cast<float4*>(out + (size_t)p * 128 + n) = v;
}

// ------------------------------------------------------------------------------------
// k_head4: k_head3 at 256 patches per workgroup.  The head is bound by what one CU can pull
// through LDS-DMA (~12 B/clk: per 128-patch k_head3 chunk 16 KB of activations + 16 KB of weights
// arrive in ~2,700 cycles against ~770 MFMA cycles per SIMD), and half of those bytes are the
// weights, re-streamed by every workgroup.  256 patches per workgroup carry the same 16 KB of
// weights per chunk for twice the activations: 48 KB per 256 patches instead of 64 KB.  Each of
// the 8 waves owns 32 patches x all 128 columns (4 accumulator tiles), so every activation
// fragment is split once (k_head3 splits each twice, once per column half).  Rings: A DA x 32 KB,
// B DB x 16 KB.  The DMA schedule, the K-chunk accumulation order and the L2 norm's summation
// order (two 64-column half sums, then + l2eps) are k_head3's: bit-identical results.
// ------------------------------------------------------------------------------------
// ABL (timing only, experiments library, HN_HEAD_ABL): bit 0 issues 3 of each wave's 4 A DMA instructions per
// chunk (24 of the 32 KB: the traffic of a 3-byte activation format), bit 1 streams the weights only into the
// ring's first DB chunks (no weight traffic after the prologue)
// PF: the fragments of chunk c + 1 are read from LDS into registers while chunk c's MFMAs run (DMA three
// chunks ahead, rings of 3): the MFMAs no longer wait for their LDS reads after each barrier
template <int K, bool F16, int DA, int DB, int ABL = 0, bool PF = false>
__global__ __launch_bounds__(512) void k_head4(const float* __restrict__ a, float* __restrict__ out,
                                               const uint4* __restrict__ wp,
                                               const float* __restrict__ bias, int P, float l2eps) {
  constexpr int KC = 32, NCH = K / KC, M = 256;
  constexpr int ABYTES = M * KC * 4;           // 32 KB per A chunk: 4 DMA instructions per wave
  constexpr int BBYTES = 2 * 4 * 2 * 64 * 16;  // 16 KB per B chunk: 2 per wave
  constexpr int NA = 4, NB = 2;
  static_assert(DA >= 2 && DB >= 2 && NCH >= DA && NCH >= DB && DA * 32 + DB * 16 <= 152, "rings");
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  __shared__ __attribute__((aligned(16))) char sa[DA * ABYTES];
  __shared__ __attribute__((aligned(16))) char sbw[DB * BBYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int pbase = blockIdx.x * M;

  const float* asrc[NA];
  const uint4* bsrc[NB];
  unsigned adst[NA], bdst[NB];
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    const int gi = NA * wave + k, s = gi * 64 + lane, row = s >> 3, c = (s & 7) ^ ((row >> 1) & 7);
    asrc[k] = a + (size_t)min(pbase + row, P - 1) * K + c * 4;
    adst[k] = (unsigned)(uintptr_t)(lds_ptr_t)(sa + gi * 1024);
  }
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int gi = NB * wave + k;
    bsrc[k] = wp + gi * 64 + lane;
    bdst[k] = (unsigned)(uintptr_t)(lds_ptr_t)(sbw + gi * 1024);
  }
  auto dma = [](const void* src, unsigned dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
  };
  auto live = [](int chunk) { return chunk >= 0 && chunk < NCH; };
  constexpr int J0 = 1 - (DA > DB ? DA : DB);  // first (prologue) iteration
  auto issue = [&](int j) {  // iteration j's DMA: B(j + DB - 1), then A(j + DA - 1)
    const int cb = j + DB - 1, ca = j + DA - 1;
    if (live(cb) && ((ABL & 2) == 0 || cb < DB)) {
      const unsigned so = (unsigned)(cb % DB) * BBYTES;
#pragma unroll
      for (int k = 0; k < NB; ++k) dma(bsrc[k] + (size_t)cb * 1024, bdst[k] + so);
    }
    if (live(ca)) {
      const unsigned so = (unsigned)(ca % DA) * ABYTES;
#pragma unroll
      for (int k = 0; k < NA - (ABL & 1); ++k) dma(asrc[k] + (size_t)ca * KC, adst[k] + so);
    }
  };
  // this wave's DMA instructions issued after the latest one of A(c) / B(c): walk the issue
  // sequence back from iteration c - 1 to the first group belonging to chunk c
  auto after = [&](int c) {
    int n = 0;
    for (int i = c - 1; i >= J0; --i) {
      if (live(i + DA - 1)) {
        if (i + DA - 1 == c) return n;
        n += NA;
      }
      if (live(i + DB - 1)) {
        if (i + DB - 1 == c) return n;
        n += NB;
      }
    }
    return 0;
  };
  const int arow = 32 * wave + r, asw = (arow >> 1) & 7;
  f32x16 acc[4] = {f32x16{}, f32x16{}, f32x16{}, f32x16{}};
  if constexpr (PF) {
    static_assert(DA == 3 && DB == 3 && NCH % 2 == 0 && NCH >= 4, "PF: chunk c + 3 refills chunk c's slots");
    constexpr int PER = NA + NB;  // DMA instructions per wave per chunk
    auto issue_chunk = [&](int ch) {
      if (ch >= NCH) return;
      const unsigned sb = (unsigned)(ch % 3) * BBYTES, sa_ = (unsigned)(ch % 3) * ABYTES;
#pragma unroll
      for (int k = 0; k < NB; ++k) dma(bsrc[k] + (size_t)ch * 1024, bdst[k] + sb);
#pragma unroll
      for (int k = 0; k < NA; ++k) dma(asrc[k] + (size_t)ch * KC, adst[k] + sa_);
    };
    float4 xa[2][2][2];
    uint4 bq[2][2][4][2];
    auto read_frags = [&](int ch, int bs) {
      const char* ast = sa + (ch % 3) * ABYTES + arow * (KC * 4);
      const char* bst = sbw + (ch % 3) * BBYTES;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int p0 = 4 * ks + 2 * h;
        xa[bs][ks][0] = *reinterpret_cast<const float4*>(ast + ((p0 ^ asw) << 4));
        xa[bs][ks][1] = *reinterpret_cast<const float4*>(ast + (((p0 + 1) ^ asw) << 4));
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const char* bp = bst + ((((ks * 4 + nt) * 2) * 64 + lane) << 4);
          bq[bs][ks][nt][0] = *reinterpret_cast<const uint4*>(bp);
          bq[bs][ks][nt][1] = *reinterpret_cast<const uint4*>(bp + 1024);
        }
      }
    };
    auto mfmas = [&](int bs) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint4 ah, al;
        if (F16) split8_f16(xa[bs][ks][0], xa[bs][ks][1], ah, al);
        else split8(xa[bs][ks][0], xa[bs][ks][1], ah, al);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const uint4 bh = bq[bs][ks][nt][0], bl = bq[bs][ks][nt][1];
          if (F16)
            acc[nt] = mfma3_f16(as_f16x8(ah), as_f16x8(al), as_f16x8(bh), as_f16x8(bl), acc[nt]);
          else
            acc[nt] = mfma3(as_bf16x8(ah), as_bf16x8(al), as_bf16x8(bh), as_bf16x8(bl), acc[nt]);
        }
      }
    };
    issue_chunk(0);
    issue_chunk(1);
    issue_chunk(2);
    head_wait_vm<2 * PER>();  // chunk 0 landed (1 and 2 in flight)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    read_frags(0, 0);
    // iteration c: chunk c + 1 landed (c + 2 may be in flight) and every wave's reads of chunk c done ->
    // barrier -> refill chunk c's slots with chunk c + 3 -> read chunk c + 1 -> chunk c's MFMAs
    auto step = [&](int c, int bs) {
      if (c + 2 < NCH) head_wait_vm<PER>();
      else head_wait_vm<0>();
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      issue_chunk(c + 3);
      if (c + 1 < NCH) read_frags(c + 1, bs ^ 1);
      mfmas(bs);
    };
#pragma unroll 1
    for (int c = 0; c < NCH; c += 2) {
      step(c, 0);
      step(c + 1, 1);
    }
  } else {
  for (int j = J0; j < 0; ++j) issue(j);
#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    switch (after(c)) {
      case 0: head_wait_vm<0>(); break;
      case 2: head_wait_vm<2>(); break;
      case 4: head_wait_vm<4>(); break;
      case 6: head_wait_vm<6>(); break;
      case 8: head_wait_vm<8>(); break;
      case 10: head_wait_vm<10>(); break;
      case 12: head_wait_vm<12>(); break;
      case 14: head_wait_vm<14>(); break;
      case 16: head_wait_vm<16>(); break;
      case 18: head_wait_vm<18>(); break;
      case 20: head_wait_vm<20>(); break;
      case 22: head_wait_vm<22>(); break;
      default: head_wait_vm<0>(); break;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue(c);
    const char* ast = sa + (c % DA) * ABYTES + arow * (KC * 4);
    const char* bst = sbw + (c % DB) * BBYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int p0 = 4 * ks + 2 * h;
      const float4 x0 = *reinterpret_cast<const float4*>(ast + ((p0 ^ asw) << 4));
      const float4 x1 = *reinterpret_cast<const float4*>(ast + (((p0 + 1) ^ asw) << 4));
      uint4 ah, al;
      if (F16) split8_f16(x0, x1, ah, al);
      else split8(x0, x1, ah, al);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const char* bp = bst + ((((ks * 4 + nt) * 2) * 64 + lane) << 4);
        const uint4 bh = *reinterpret_cast<const uint4*>(bp);
        const uint4 bl = *reinterpret_cast<const uint4*>(bp + 1024);
        if (F16)
          acc[nt] = mfma3_f16(as_f16x8(ah), as_f16x8(al), as_f16x8(bh), as_f16x8(bl), acc[nt]);
        else
          acc[nt] = mfma3(as_bf16x8(ah), as_bf16x8(al), as_bf16x8(bh), as_bf16x8(bl), acc[nt]);
      }
    }
  }
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const float b = bias[32 * nt + r];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[nt][i] += b;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    // k_head3's order: each 64-column half summed over its lanes, then the halves + l2eps
    const float s01 = half_sum(acc[0][i] * acc[0][i] + acc[1][i] * acc[1][i]);
    const float s23 = half_sum(acc[2][i] * acc[2][i] + acc[3][i] * acc[3][i]);
    const float norm = sqrtf(s01 + s23 + l2eps);
    const int p = pbase + 32 * wave + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (p < P) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) out[(size_t)p * 128 + 32 * nt + r] = acc[nt][i] / norm;
    }
  }
}

// ------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------
// stem-fused kernels carry the normalised patch (34x34 fp32) + 8 reduction floats
template <class CFG, bool STEM>
constexpr int conv_lds() { return CFG::LDS + (STEM ? (34 * 34 + 8) * 4 : 0); }

#define HN_CONV(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN)                             \
  using NAME##_cfg = ConvCfg<CIN, COUT, HIN, S, NP, TR, WM, WN>;                           \
  static hipError_t NAME##_lo(const float* in, float* out, const void* wp, const float* bias,\
                         int P, const float* sw, const float* sb, float eps,               \
                         hipStream_t st, float lo) {                                       \
    constexpr int lds = conv_lds<NAME##_cfg, STEM>();                                      \
    int resident = 0; /* sets the dynamic-LDS limit on this device */                     \
    hipError_t e = hn_resident_blocks(                                                     \
        reinterpret_cast<const void*>(&k_conv3x3<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM>), \
        256, lds, &resident);                                                              \
    if (e != hipSuccess) return e;                                                         \
    const int grid = (P + NP - 1) / NP * NAME##_cfg::RT;                                   \
    hipLaunchKernelGGL((k_conv3x3<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM>), dim3(grid),   \
                       dim3(256), lds, st, in, out, static_cast<const uint4*>(wp), bias, P, \
                       sw, sb, eps, hn_knobs().dbg, lo);                                   \
    return hipGetLastError();                                                              \
  }                                                                                        \
  static hipError_t NAME(const float* in, float* out, const void* wp, const float* bias,   \
                         int P, const float* sw, const float* sb, float eps, hipStream_t st) { \
    return NAME##_lo(in, out, wp, bias, P, sw, sb, eps, st, 0.f);                          \
  }

// variant 0 = default tiling; variant 1 = smaller LDS footprint / more workgroups per CU
HN_CONV(conv1s_launch, true, 32, 32, 32, 1, 1, 8, 4, 1)
#ifdef HN_EXPERIMENTS  // superseded tiling (experiments library only)
HN_CONV(conv1s_v1, true, 32, 32, 32, 1, 1, 4, 4, 1)
#endif
HN_CONV(conv1_launch, false, 32, 32, 32, 1, 1, 8, 4, 1)
HN_CONV(conv2_launch, false, 32, 64, 32, 2, 1, 8, 2, 2)
#ifdef HN_EXPERIMENTS  // superseded tiling (experiments library only)
HN_CONV(conv2_v1, false, 32, 64, 32, 2, 1, 4, 2, 2)
#endif
HN_CONV(conv3_launch, false, 64, 64, 16, 1, 1, 16, 2, 2)
#ifdef HN_EXPERIMENTS  // superseded tiling (experiments library only)
HN_CONV(conv3_v1, false, 64, 64, 16, 1, 1, 8, 2, 2)
#endif
HN_CONV(conv4_launch, false, 64, 128, 16, 2, 1, 8, 1, 4)
#ifdef HN_EXPERIMENTS  // superseded tiling (experiments library only)
HN_CONV(conv4_v1, false, 64, 128, 16, 2, 1, 4, 1, 4)
#endif
HN_CONV(conv5_launch, false, 128, 128, 8, 1, 2, 8, 1, 4)
#ifdef HN_EXPERIMENTS  // superseded tiling (experiments library only)
HN_CONV(conv5_v1, false, 128, 128, 8, 1, 1, 8, 1, 4)
#endif

// persistent launch: grid = min(tiles, resident workgroups) (occupancy query, cached)
#define HN_PIPE(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN) HN_PIPE_A(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, 0)
#define HN_PIPE_A(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL) HN_PIPE_C(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL, false)
#define HN_PIPE_C(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL, CST)                 \
  using NAME##_cfg = PipeCfg<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM, CST>;                \
  static hipError_t NAME##_lo(const float* in, float* out, const void* wp, const float* bias,\
                         int P, const float* sw, const float* sb, float eps,               \
                         hipStream_t st, float lo) {                                       \
    constexpr int lds = NAME##_cfg::SMEM;                                                  \
    const void* fn = reinterpret_cast<const void*>(                                        \
        &k_conv_pipe<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM, ABL, CST>);                       \
    int resident = 0;                                                                      \
    const hipError_t e = hn_resident_blocks(fn, NAME##_cfg::NTHR, lds, &resident);         \
    if (e != hipSuccess) return e;                                                         \
    const int tiles = (P + NP - 1) / NP * NAME##_cfg::RT;                                  \
    const int grid = std::min(tiles, resident);                                            \
    hipLaunchKernelGGL((k_conv_pipe<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM, ABL, CST>), dim3(grid), \
                       dim3(NAME##_cfg::NTHR), lds, st, in, out,                           \
                       static_cast<const uint4*>(wp), bias, P, sw, sb, eps, lo);               \
    return hipGetLastError();                                                              \
  }                                                                                        \
  static hipError_t NAME(const float* in, float* out, const void* wp, const float* bias,   \
                         int P, const float* sw, const float* sb, float eps, hipStream_t st) { \
    return NAME##_lo(in, out, wp, bias, P, sw, sb, eps, st, 0.f);                          \
  }

#ifdef HN_EXPERIMENTS  // superseded tiling (experiments library only)
HN_PIPE(pipe1s, true, 32, 32, 32, 1, 1, 4, 4, 1)
HN_PIPE(pipe1s_t8, true, 32, 32, 32, 1, 1, 8, 4, 1)
HN_PIPE(pipe2, false, 32, 64, 32, 2, 1, 4, 2, 2)
HN_PIPE(pipe2_t2, false, 32, 64, 32, 2, 1, 2, 1, 2)
HN_PIPE(pipe3, false, 64, 64, 16, 1, 1, 8, 2, 2)
HN_PIPE(pipe3_t16, false, 64, 64, 16, 1, 1, 16, 2, 2)
HN_PIPE(pipe4, false, 64, 128, 16, 2, 1, 4, 1, 4)
HN_PIPE(pipe4_t8, false, 64, 128, 16, 2, 1, 8, 1, 4)
HN_PIPE(pipe5, false, 128, 128, 8, 1, 1, 8, 1, 4)
HN_PIPE(pipe5_np2, false, 128, 128, 8, 1, 2, 8, 1, 4)
#endif
HN_PIPE_C(pipe5_cst, false, 128, 128, 8, 1, 2, 8, 1, 4, 0, true)  // HN_VARIANT digit g at conv5

#define HN_WS(NAME, CIN, COUT, HIN, S, NP, TR, WM, WN) HN_WS_S(NAME, false, CIN, COUT, HIN, S, NP, TR, WM, WN)
#define HN_WS_S(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN) HN_WS_A(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, 0)
#define HN_WS_A(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL) HN_WS_X(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL, 80)
#define HN_WS_X(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL, PX) HN_WS_C(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL, PX, false)
#define HN_WS_C(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL, PX, CST) \
  HN_WS_P(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL, PX, CST, false)
#define HN_WS_P(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN, ABL, PX, CST, PST)        \
  using NAME##_cfg = WsCfg<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM, PX, CST, PST>;              \
  static hipError_t NAME##_lo(const float* in, float* out, const void* wp, const float* bias,\
                         int P, const float* sw, const float* sb, float eps, hipStream_t st, \
                         float lo) {                                                       \
    constexpr int lds = NAME##_cfg::SMEM;                                                  \
    const void* fn =                                                                       \
        reinterpret_cast<const void*>(&k_conv_ws<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM, ABL, PX, CST, PST>); \
    int resident = 0;                                                                      \
    const hipError_t e = hn_resident_blocks(fn, NAME##_cfg::NTHR, lds, &resident);         \
    if (e != hipSuccess) return e;                                                         \
    const int tiles = (P + NP - 1) / NP * NAME##_cfg::RT;                                  \
    const int grid = std::min(tiles, resident);                                            \
    hipLaunchKernelGGL((k_conv_ws<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM, ABL, PX, CST, PST>), dim3(grid), \
                       dim3(NAME##_cfg::NTHR), lds, st, in, out,                           \
                       static_cast<const uint4*>(wp), bias, P, sw, sb, eps, lo);               \
    return hipGetLastError();                                                              \
  }                                                                                        \
  static hipError_t NAME(const float* in, float* out, const void* wp, const float* bias,   \
                         int P, const float* sw, const float* sb, float eps, hipStream_t st) { \
    return NAME##_lo(in, out, wp, bias, P, sw, sb, eps, st, 0.f);                          \
  }

HN_WS_S(ws1s, true, 32, 32, 32, 1, 1, 4, 4, 1)
HN_WS_S(ws1s_t8, true, 32, 32, 32, 1, 1, 8, 4, 1)
HN_WS(ws2, 32, 64, 32, 2, 1, 4, 2, 2)
HN_WS(ws2_t2, 32, 64, 32, 2, 1, 2, 1, 2)
#ifdef HN_EXPERIMENTS  // conv3..conv5's generic warp-specialised tilings, superseded by their defaults
HN_WS(ws3, 64, 64, 16, 1, 1, 8, 2, 2)
HN_WS(ws3_t16, 64, 64, 16, 1, 1, 16, 2, 2)
HN_WS(ws4, 64, 128, 16, 2, 1, 4, 1, 4)
HN_WS(ws4_t8, 64, 128, 16, 2, 1, 8, 1, 4)
HN_WS(ws5, 128, 128, 8, 1, 1, 8, 1, 4)
HN_WS(ws5_np2, 128, 128, 8, 1, 2, 8, 1, 4)
#endif
// conv4 with the 64-byte swizzled window: two patches per stage (twice the weight reuse of ws4_t8)
// -- HN_VARIANT digit d -- and the same layout at one patch (digit e)
#ifdef HN_EXPERIMENTS  // superseded tiling (experiments library only)
HN_WS_X(ws4_np2s, false, 64, 128, 16, 2, 2, 8, 1, 4, 0, 64)
HN_WS_X(ws4_s, false, 64, 128, 16, 2, 1, 8, 1, 4, 0, 64)
#endif
HN_WS_X(ws4_np2s22, false, 64, 128, 16, 2, 2, 8, 2, 2, 0, 64)  // digit f: 2 x 2 waves
// digit i: the same with the outputs stored by the producer waves (PST)
HN_WS_P(ws4_pst, false, 64, 128, 16, 2, 2, 8, 2, 2, 0, 64, false, true)
// conv3 with the epilogue transposed through LDS for whole-row stores (CST): HN_VARIANT digit g
// (the default, conv3 12.8 -> 12.1 ms).  The same on conv4's one-patch tiling (8.49 -> 8.35 ms)
// and conv5's k_conv_ws form (13.0 -> 12.6) stays behind their defaults; conv5's k_conv_pipe
// gets the half-tile form (pipe5_cst, 11.9 -> 11.5 ms, the default).
HN_WS_C(ws3_cst, false, 64, 64, 16, 1, 1, 16, 2, 2, 0, 80, true)
#ifdef HN_EXPERIMENTS
// conv3 with the outputs stored by the producer waves (PST, HN_VARIANT digit i): 12.8 vs 12.1 ms
// for the CST form (same-box A/B; the DEEP producers' two extra barriers per tile cost more than
// the MFMA waves' whole-row stores)
HN_WS_P(ws3_pst, false, 64, 64, 16, 1, 1, 16, 2, 2, 0, 80, false, true)
#endif

// wider N tiles (fewer A-fragment reads, weights shared through L1)
#ifdef HN_EXPERIMENTS  // superseded tiling (experiments library only)
HN_WS(ws3_w8, 64, 64, 16, 1, 1, 16, 4, 1)
HN_WS(ws4_w8, 64, 128, 16, 2, 1, 8, 2, 2)
HN_WS(ws5_w8, 128, 128, 8, 1, 2, 8, 2, 2)
#endif
#ifdef HN_EXPERIMENTS
// ablation builds (timing only, wrong results; the HN_EXPERIMENTS library only): weights
// fetched once per stage
HN_WS_A(ws3_a1, false, 64, 64, 16, 1, 1, 16, 2, 2, 45)
HN_WS_A(ws4_a1, false, 64, 128, 16, 2, 1, 8, 1, 4, 45)
HN_WS_A(ws5_a1, false, 128, 128, 8, 1, 2, 8, 1, 4, 45)
HN_WS_A(ws3_a2, false, 64, 64, 16, 1, 1, 16, 2, 2, 8)
HN_WS_A(ws4_a2, false, 64, 128, 16, 2, 1, 8, 1, 4, 8)
HN_WS_A(ws5_a2, false, 128, 128, 8, 1, 2, 8, 1, 4, 8)
HN_WS_A(ws3_a3, false, 64, 64, 16, 1, 1, 16, 2, 2, 40)
HN_WS_A(ws4_a3, false, 64, 128, 16, 2, 1, 8, 1, 4, 40)
HN_WS_A(ws5_a3, false, 128, 128, 8, 1, 2, 8, 1, 4, 40)
#endif

hipError_t hn_launch_stem(const float* in, float* out, const float* w, const float* b, int P,
                          bool norm, float eps, hipStream_t st) {
  if (norm)
    hipLaunchKernelGGL(k_stem<true>, dim3(P), dim3(256), 0, st, in, out, w, b, eps);
  else
    hipLaunchKernelGGL(k_stem<false>, dim3(P), dim3(256), 0, st, in, out, w, b, eps);
  return hipGetLastError();
}

// HN_VARIANT digit v is a tiling this library has for conv layer `layer` (0 = stem + conv1,
// 1 = conv1 alone, 2..5 = conv2..conv5); mirrors the dispatch below.  Digits 4 / 8 / 9 are the
// timing-only ablation builds of conv3..conv5 (HN_EXPERIMENTS library only).
bool hn_hardnet_variant_ok(int layer, int v) {
  // the product library: the defaults (digits 6 0 5 q i l) and one fallback per stage -- 0 (k_conv3x3)
  // everywhere, 5 / 6 (warp-specialised, smaller / larger tile) for the HN_NO_C12 stem+conv1 and conv2,
  // 15 (conv4 on the 64-byte swizzled window with the MFMA waves' own stores, digit f), 16 (direct conv3 /
  // conv5 with epilogue stores through LDS, digit g), 21 / 26 (1-D Winograd F(2,3), weight ring 6 / 8).
  // The measured-slower tilings (1, 2, 3, 7, 13, 14, 5 / 6 on conv3..conv5), the Winograd kernels 17 (2-D),
  // 19 / 20 (shallower rings), 32 / 33 (F(4,3) conv3) and the timing-only ablations exist only with
  // -DHN_EXPERIMENTS.
  if (layer < 0 || layer > 5) return false;
#ifdef HN_EXPERIMENTS
  if (v == 18 && layer == 3) return true;
  if (v == 4 || v == 8 || v == 9) return layer >= 3;
  if (v == 13 || v == 14) return layer == 4;
  if (v == 17) return layer == 3 || layer == 5;  // Winograd F(2x2,3x3), hn_wino.hip
  if (v == 7) return layer >= 3;
  if (v == 1 || v == 2 || v == 3) return true;
  if (v == 5 || v == 6) return true;
  if (v == 19 || v == 20) return layer == 3 || layer == 5;  // 1-D Winograd F(2,3), weight ring 3 / 4
  if (v == 32 || v == 33) return layer == 3;                 // F(4,3) (k_conv_w4), weight ring 6 / 9 (digits w / x)
  if ((v >= 22 && v <= 25) || v == 29 || v == 30 || v == 31) return layer == 3 || layer == 5;  // its timing-only ablations (ABL 1 / 2 / 4 / 8; t: 16; u: 32, v: 34)
  if (v == 34 || v == 35) return layer == 3 || layer == 5;  // wave-priority A/B (y: MFMA waves first, z: producers first)
#endif
  if (v == 15 || v == 18) return layer == 4;  // 18: outputs stored by the producer waves
  if (v == 21 || v == 26) return layer == 3 || layer == 5;  // 1-D Winograd F(2,3) (hn_wino1.hip), weight ring 6 / 8
  if (v == 16) return layer == 3 || layer == 5;
  if (v == 5 || v == 6) return layer <= 2;  // (layer 1 always runs conv1_launch)
  if (v == 0) return true;
  return false;
}

// layer 0 = fused stem (input_norm + conv0) + conv1 from the raw patches
hipError_t hn_launch_hardnet_conv(int layer, int variant, const HardnetDev& d, const float* in,
                                  float* out, int P, float eps, hipStream_t st) {
  if (!hn_hardnet_variant_ok(layer, variant)) return hipErrorInvalidValue;
#ifdef HN_EXPERIMENTS
  if (variant == 8 || variant == 9 || variant == 4) {  // ablation (timing only)
    const int a = variant == 8 ? 1 : variant == 9 ? 2 : 3;
    switch (layer) {
      case 3: return (a == 1 ? ws3_a1 : a == 2 ? ws3_a2 : ws3_a3)(in, out, d.wpack[3], d.bias[3], P, nullptr, nullptr, 0.f, st);
      case 4: return (a == 1 ? ws4_a1 : a == 2 ? ws4_a2 : ws4_a3)(in, out, d.wpack[4], d.bias[4], P, nullptr, nullptr, 0.f, st);
      case 5: return (a == 1 ? ws5_a1 : a == 2 ? ws5_a2 : ws5_a3)(in, out, d.wpack[5], d.bias[5], P, nullptr, nullptr, 0.f, st);
    }
    return hipErrorInvalidValue;
  }
#endif
  if (variant == 15 || (variant == 18 && layer == 4)) {  // conv4, 64-byte swizzled window, two patches per stage
    if (layer != 4) return hipErrorInvalidValue;
    return (variant == 18 ? ws4_pst : ws4_np2s22)(in, out, d.wpack[4], d.bias[4], P, nullptr, nullptr, 0.f, st);
  }
#ifdef HN_EXPERIMENTS
  if (variant == 18 && layer == 3) return ws3_pst(in, out, d.wpack[3], d.bias[3], P, nullptr, nullptr, 0.f, st);
#endif
#ifdef HN_EXPERIMENTS
  if (variant == 13 || variant == 14) {  // conv4, 64-byte swizzled window (2 / 1 patches per stage)
    if (layer != 4) return hipErrorInvalidValue;
    return (variant == 13 ? ws4_np2s : ws4_s)(in, out, d.wpack[4], d.bias[4], P, nullptr, nullptr, 0.f, st);
  }
  if (variant == 17) return hn_launch_wino(layer, d, in, out, P, st);
  if (variant == 7) {  // warp-specialised, NT = 2
    switch (layer) {
      case 3: return ws3_w8(in, out, d.wpack[3], d.bias[3], P, nullptr, nullptr, 0.f, st);
      case 4: return ws4_w8(in, out, d.wpack[4], d.bias[4], P, nullptr, nullptr, 0.f, st);
      case 5: return ws5_w8(in, out, d.wpack[5], d.bias[5], P, nullptr, nullptr, 0.f, st);
    }
    return hipErrorInvalidValue;
  }
#endif
  if (variant == 21) return hn_launch_wino1(layer, 6, d, in, out, P, st);
  if (variant == 26) return hn_launch_wino1(layer, 8, d, in, out, P, st);
#ifdef HN_EXPERIMENTS
  if (variant == 19 || variant == 20) return hn_launch_wino1(layer, variant == 19 ? 3 : 4, d, in, out, P, st);
  if (variant == 32 || variant == 33) return hn_launch_wino4(layer, variant == 32 ? 6 : 9, d, in, out, P, st);
  if (variant >= 22 && variant <= 25) return hn_launch_wino1(layer, 100 + (1 << (variant - 22)), d, in, out, P, st);
  if (variant == 29) return hn_launch_wino1(layer, 116, d, in, out, P, st);
  if (variant == 30 || variant == 31) return hn_launch_wino1(layer, variant == 30 ? 132 : 134, d, in, out, P, st);
  if (variant == 34 || variant == 35) return hn_launch_wino1(layer, variant == 34 ? 164 : 228, d, in, out, P, st);
#endif
  if (variant == 16) {  // coalesced epilogue stores
    switch (layer) {
      case 3: return ws3_cst(in, out, d.wpack[3], d.bias[3], P, nullptr, nullptr, 0.f, st);
      case 5: return pipe5_cst(in, out, d.wpack[5], d.bias[5], P, nullptr, nullptr, 0.f, st);
    }
    return hipErrorInvalidValue;
  }
  if (variant == 5 || variant == 6) {  // warp-specialised: 5 = smaller tile, 6 = larger
    const bool big = variant == 6;
    switch (layer) {
      case 0:
        return (big ? ws1s_t8 : ws1s)(in, out, d.wpack[1], d.bias[1], P, d.stem_w, d.stem_b, eps, st);
      case 2: return (big ? ws2_t2 : ws2)(in, out, d.wpack[2], d.bias[2], P, nullptr, nullptr, 0.f, st);
#ifdef HN_EXPERIMENTS
      case 3: return (big ? ws3_t16 : ws3)(in, out, d.wpack[3], d.bias[3], P, nullptr, nullptr, 0.f, st);
      case 4: return (big ? ws4_t8 : ws4)(in, out, d.wpack[4], d.bias[4], P, nullptr, nullptr, 0.f, st);
      case 5: return (big ? ws5_np2 : ws5)(in, out, d.wpack[5], d.bias[5], P, nullptr, nullptr, 0.f, st);
#endif
    }
    return hipErrorInvalidValue;
  }
#ifdef HN_EXPERIMENTS
  if (variant >= 2) {  // persistent pipelined kernels: 2 = smaller tile, 3 = larger tile
    const bool big = variant == 3;
    switch (layer) {
      case 0:
        return (big ? pipe1s_t8 : pipe1s)(in, out, d.wpack[1], d.bias[1], P, d.stem_w, d.stem_b, eps, st);
      case 2: return (big ? pipe2 : pipe2_t2)(in, out, d.wpack[2], d.bias[2], P, nullptr, nullptr, 0.f, st);
      case 3: return (big ? pipe3_t16 : pipe3)(in, out, d.wpack[3], d.bias[3], P, nullptr, nullptr, 0.f, st);
      case 4: return (big ? pipe4_t8 : pipe4)(in, out, d.wpack[4], d.bias[4], P, nullptr, nullptr, 0.f, st);
      case 5: return (big ? pipe5_np2 : pipe5)(in, out, d.wpack[5], d.bias[5], P, nullptr, nullptr, 0.f, st);
    }
    return hipErrorInvalidValue;
  }
#endif
#ifdef HN_EXPERIMENTS
  if (variant == 1) {
    switch (layer) {
      case 0: return conv1s_v1(in, out, d.wpack[1], d.bias[1], P, d.stem_w, d.stem_b, eps, st);
      case 2: return conv2_v1(in, out, d.wpack[2], d.bias[2], P, nullptr, nullptr, 0.f, st);
      case 3: return conv3_v1(in, out, d.wpack[3], d.bias[3], P, nullptr, nullptr, 0.f, st);
      case 4: return conv4_v1(in, out, d.wpack[4], d.bias[4], P, nullptr, nullptr, 0.f, st);
      case 5: return conv5_v1(in, out, d.wpack[5], d.bias[5], P, nullptr, nullptr, 0.f, st);
    }
  }
#endif
  switch (layer) {
    case 0: return conv1s_launch(in, out, d.wpack[1], d.bias[1], P, d.stem_w, d.stem_b, eps, st);
    case 1: return conv1_launch(in, out, d.wpack[1], d.bias[1], P, nullptr, nullptr, 0.f, st);
    case 2: return conv2_launch(in, out, d.wpack[2], d.bias[2], P, nullptr, nullptr, 0.f, st);
    case 3: return conv3_launch(in, out, d.wpack[3], d.bias[3], P, nullptr, nullptr, 0.f, st);
    case 4: return conv4_launch(in, out, d.wpack[4], d.bias[4], P, nullptr, nullptr, 0.f, st);
    case 5: return conv5_launch(in, out, d.wpack[5], d.bias[5], P, nullptr, nullptr, 0.f, st);
  }
  return hipErrorInvalidValue;
}

// Train mode (hn_train.hip): layer `layer`'s production tiling as a plain convolution over NHWC
// fp32 -- zero bias, no ReLU floor -- with bf16x3 fragments packed on the GPU (k_pack3x3).  The
// stride-1 layers also run the data gradient (weights flipped and transposed: same shapes).
hipError_t hn_launch_conv_raw(int layer, const void* wp, const float* zero_bias, const float* in, float* out,
                              int P, hipStream_t st) {
  if (P <= 0) return hipSuccess;
  const float lo = -INFINITY;
  switch (layer) {
    case 1: return conv1_launch_lo(in, out, wp, zero_bias, P, nullptr, nullptr, 0.f, st, lo);
    case 2: return ws2_lo(in, out, wp, zero_bias, P, nullptr, nullptr, 0.f, st, lo);
    case 3: return ws3_cst_lo(in, out, wp, zero_bias, P, nullptr, nullptr, 0.f, st, lo);
    case 4: return ws4_np2s22_lo(in, out, wp, zero_bias, P, nullptr, nullptr, 0.f, st, lo);
    case 5: return pipe5_cst_lo(in, out, wp, zero_bias, P, nullptr, nullptr, 0.f, st, lo);
  }
  return hipErrorInvalidValue;
}

hipError_t hn_launch_head(const float* a, float* out, const void* wp, const float* bias, int P,
                          int K, float l2eps, hipStream_t st, bool f16, float* part) {
  const int grid = (P + 63) / 64;
  // HN_HEAD: 1 k_head, 2 k_head2, 3 k_head3, 4 (default) k_head4 from 61,440 patches, the split-K k_head3 up to
  // kHeadSplitMaxP patches (when the caller passes the scratch), k_head3 in between
  const int form = hn_knobs().head;
  const uint4* w = static_cast<const uint4*>(wp);
  if (form >= 4 && part && P <= kHeadSplitMaxP && ((K == 8192 && !f16) || (K == 2048 && f16))) {
    // every batch up to kHeadSplitMaxP patches sums the same K ranges in the same order: its descriptors do
    // not depend on the batch they come in (bit for bit); the unsplit forms reassociate the K sum
    const dim3 g((P + 127) / 128, head_split(K));
    if (K == 8192)
      hipLaunchKernelGGL((k_head3<8192, false, 4, 4, head_split(8192)>), g, dim3(512), 0, st, a, out, w, bias, P,
                         l2eps, part);
    else
      hipLaunchKernelGGL((k_head3<2048, true, 4, 4, head_split(2048)>), g, dim3(512), 0, st, a, out, w, bias, P,
                         l2eps, part);
    if (const hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    if (K == 8192)
      hipLaunchKernelGGL(k_head_fin<head_split(8192)>, dim3((P + 7) / 8), dim3(256), 0, st, part, out, bias, P, l2eps);
    else
      hipLaunchKernelGGL(k_head_fin<head_split(2048)>, dim3((P + 7) / 8), dim3(256), 0, st, part, out, bias, P, l2eps);
    return hipGetLastError();
  }
#define HN_HEAD3(KK, F, DA, DB)                                                                              \
  if (K == KK && f16 == F) {                                                                                 \
    hipLaunchKernelGGL((k_head3<KK, F, DA, DB>), dim3((P + 127) / 128), dim3(512), 0, st, a, out, w, bias, P, \
                       l2eps);                                                                               \
    return hipGetLastError();                                                                                \
  }
  // both rings 4 deep (128 KB): same-box A/B of the HardNet head at A / B depths 4 / 4, 5 / 3, 5 / 4,
  // 4 / 5 = 2.11, 2.29, 2.33, 2.31 ms (k_head2 2.33)
  // k_head4 (256 patches per workgroup) when the launch still gives most CUs a workgroup
#define HN_HEAD4(KK, F, DA, DB)                                                                              \
  if (K == KK && f16 == F) {                                                                                 \
    hipLaunchKernelGGL((k_head4<KK, F, DA, DB>), dim3((P + 255) / 256), dim3(512), 0, st, a, out, w, bias, P, \
                       l2eps);                                                                               \
    return hipGetLastError();                                                                                \
  }
  if (form >= 4 && P >= 240 * 256) {
#ifdef HN_EXPERIMENTS  // (ahead of the prefetching form, which has no ablation builds)
    if (const char* e = std::getenv("HN_HEAD_ABL")) {
      const int abl = std::atoi(e);
      if (K == 8192 && !f16 && (abl == 1 || abl == 2 || abl == 3)) {
        const dim3 g((P + 255) / 256), b(512);
        if (abl == 1) hipLaunchKernelGGL((k_head4<8192, false, 3, 3, 1>), g, b, 0, st, a, out, w, bias, P, l2eps);
        if (abl == 2) hipLaunchKernelGGL((k_head4<8192, false, 3, 3, 2>), g, b, 0, st, a, out, w, bias, P, l2eps);
        if (abl == 3) hipLaunchKernelGGL((k_head4<8192, false, 3, 3, 3>), g, b, 0, st, a, out, w, bias, P, l2eps);
        return hipGetLastError();
      }
    }
#endif
    if (hn_knobs().head_pf && K == 8192 && !f16) {
      hipLaunchKernelGGL((k_head4<8192, false, 3, 3, 0, true>), dim3((P + 255) / 256), dim3(512), 0, st, a, out, w,
                         bias, P, l2eps);
      return hipGetLastError();
    }
    HN_HEAD4(8192, false, 3, 3) HN_HEAD4(2048, true, 3, 3)
  }
  if (form >= 3) {
    HN_HEAD3(8192, false, 4, 4) HN_HEAD3(2048, true, 4, 4)
  }
#undef HN_HEAD3
#undef HN_HEAD4
  if (K == 8192 && !f16 && form == 1)
    hipLaunchKernelGGL(k_head<8192>, dim3(grid), dim3(256), 0, st, a, out, w, bias, P, l2eps);
  else if (K == 8192 && !f16)
    hipLaunchKernelGGL((k_head2<8192, false>), dim3(grid), dim3(256), 0, st, a, out, w, bias, P, l2eps);
  else if (K == 2048 && f16)  // NAS head: 4x4 conv 128 -> 128 (model_supernet.py:64-68)
    hipLaunchKernelGGL((k_head2<2048, true>), dim3(grid), dim3(256), 0, st, a, out, w, bias, P, l2eps);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// LDS bytes of each conv config (exported for tests / DESIGN.md)
int hn_conv_lds_bytes(int layer) {
  switch (layer) {
    case 1: return conv1_launch_cfg::LDS;
    case 2: return conv2_launch_cfg::LDS;
    case 3: return conv3_launch_cfg::LDS;
    case 4: return conv4_launch_cfg::LDS;
    case 5: return conv5_launch_cfg::LDS;
  }
  return -1;
}
