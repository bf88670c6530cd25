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

template <int CIN, int COUT, int HIN, int S, int NP, int TR, int WM, int WN>
struct ConvCfg {
  static constexpr int HOUT = HIN / S, WOUT = HOUT;
  static constexpr int RIN = (S == 1) ? TR + 2 : 2 * TR + 1;
  static constexpr int NCOLS = (S == 1) ? HIN + 2 : HIN + 1;
  static constexpr int HALF = (NCOLS + 1) / 2;
  static constexpr int BM = NP * TR * WOUT;
  static constexpr int RT = HOUT / TR;
  static constexpr int MT = BM / WM / 32, NT = COUT / WN / 32;
  static constexpr int NTOT = COUT / 32, NCC = CIN / 32;
  static constexpr int RS = conv_row_stride(NCOLS, WOUT, S);
  static constexpr int PS = RIN * RS;
  static constexpr int PLANE = NP * PS;
  static constexpr int LDS = 2 * PLANE;
  static_assert(WM * WN == 4, "4 waves");
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
HN_DEV int xcd_remap(int bid, int nblocks) {
  const int xcd = bid & 7, idx = bid >> 3;
  const int q = nblocks >> 3, r = nblocks & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// STEM = true (conv1 only): `in` is the raw [P,1,32,32] patch batch; the kernel computes
// input_norm (HardNet.py:306-310) and conv0+BN+ReLU (HardNet.py:281-283) for the window
// rows it needs (VALU fp32, weights uniform -> scalar loads) straight into the LDS window,
// so the 128 KB/patch a0 activation never touches HBM.
template <int CIN, int COUT, int HIN, int S, int NP, int TR, int WM, int WN, bool STEM>
__global__ __launch_bounds__(256) void k_conv3x3(const float* __restrict__ in, float* __restrict__ out,
                                                 const uint4* __restrict__ wp,
                                                 const float* __restrict__ bias, int P,
                                                 const float* __restrict__ stem_w,
                                                 const float* __restrict__ stem_b, float eps) {
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
      constexpr int NPIX = C::RIN * C::NCOLS;
      for (int u = tid; u < NPIX; u += 256) {
        const int wr = u / C::NCOLS, wc = u % C::NCOLS;
        const int y = y0 - 1 + wr, x = wc - 1;
        char* dst = smem + wr * C::RS + wc * 80;
        if (y >= 0 && y < 32 && x >= 0 && x < 32) {
          float xin[9];
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) xin[ky * 3 + kx] = pt[(y + ky) * 34 + x + kx];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float a[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int c = g * 8 + j;
              float s0 = 0.f;
#pragma unroll
              for (int tp = 0; tp < 9; ++tp) s0 = fmaf(xin[tp], stem_w[tp * 32 + c], s0);
              a[j] = fmaxf(s0 + stem_b[c], 0.f);
            }
            uint4 hi, lo;
            split8(make_float4(a[0], a[1], a[2], a[3]), make_float4(a[4], a[5], a[6], a[7]), hi, lo);
            *reinterpret_cast<uint4*>(dst + g * 16) = hi;
            *reinterpret_cast<uint4*>(dst + C::PLANE + g * 16) = lo;
          }
        } else {
          const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            *reinterpret_cast<uint4*>(dst + g * 16) = z;
            *reinterpret_cast<uint4*>(dst + C::PLANE + g * 16) = z;
          }
        }
      }
    } else {
      constexpr int UNITS = NP * C::RIN * C::NCOLS * 4;
      for (int u = tid; u < UNITS; u += 256) {
        const int g = u & 3, pix = u >> 2;
        const int wc = pix % C::NCOLS, t2 = pix / C::NCOLS;
        const int wr = t2 % C::RIN, np = t2 / C::RIN;
        const int p = p0 + np, y = y0 * S - 1 + wr, x = wc - 1;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
        if (p < P && y >= 0 && y < HIN && x >= 0 && x < HIN) {
          const float4* src = reinterpret_cast<const float4*>(
              in + (((size_t)p * HIN + y) * HIN + x) * CIN + cc * 32 + g * 8);
          a = src[0];
          b = src[1];
        }
        uint4 hi, lo;
        split8(a, b, hi, lo);
        const int pc = (S == 1) ? wc : ((wc & 1) ? C::HALF + (wc >> 1) : (wc >> 1));
        const int off = np * C::PS + wr * C::RS + pc * 80 + g * 16;
        *reinterpret_cast<uint4*>(smem + off) = hi;
        *reinterpret_cast<uint4*>(smem + C::PLANE + off) = lo;
      }
    }
    __syncthreads();
    const uint4* wcc = wp + (size_t)cc * 9 * 2 * C::NTOT * 2 * 64;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ky = tap / 3, kx = tap % 3;
        const int toff = ky * C::RS + C::colofs(kx) * 80 + ks * 32;
        bf16x8 bh[C::NT], bl[C::NT];
#pragma unroll
        for (int nt = 0; nt < C::NT; ++nt) {
          const int idx = (((tap * 2 + ks) * C::NTOT + wn * C::NT + nt) * 2) * 64 + lane;
          bh[nt] = as_bf16x8(wcc[idx]);
          bl[nt] = as_bf16x8(wcc[idx + 64]);
        }
#pragma unroll
        for (int mt = 0; mt < C::MT; ++mt) {
          const bf16x8 ah = as_bf16x8(*reinterpret_cast<const uint4*>(smem + abase[mt] + toff));
          const bf16x8 al =
              as_bf16x8(*reinterpret_cast<const uint4*>(smem + C::PLANE + abase[mt] + toff));
#pragma unroll
          for (int nt = 0; nt < C::NT; ++nt) acc[mt][nt] = mfma3(ah, al, bh[nt], bl[nt], acc[mt][nt]);
        }
      }
    }
  }

  // epilogue: + folded-BN bias, ReLU, NHWC fp32 store
#pragma unroll
  for (int nt = 0; nt < C::NT; ++nt) {
    const int n = (wn * C::NT + nt) * 32 + r;
    const float bv = bias[n];
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        const int m = (wm * C::MT + mt) * 32 + row;
        const int np = m / (TR * C::WOUT), rem = m % (TR * C::WOUT);
        const int yl = rem / C::WOUT, xo = rem % C::WOUT;
        const int p = p0 + np;
        if (p < P)
          out[(((size_t)p * C::HOUT + y0 + yl) * C::WOUT + xo) * COUT + n] =
              fmaxf(acc[mt][nt][i] + bv, 0.f);
      }
    }
  }
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
// host launchers
// ------------------------------------------------------------------------------------
// stem-fused kernels carry the normalised patch (34x34 fp32) + 8 reduction floats
template <class CFG, bool STEM>
constexpr int conv_lds() { return CFG::LDS + (STEM ? (34 * 34 + 8) * 4 : 0); }

#define HN_CONV(NAME, STEM, CIN, COUT, HIN, S, NP, TR, WM, WN)                             \
  using NAME##_cfg = ConvCfg<CIN, COUT, HIN, S, NP, TR, WM, WN>;                           \
  static hipError_t NAME(const float* in, float* out, const void* wp, const float* bias,   \
                         int P, const float* sw, const float* sb, float eps,               \
                         hipStream_t st) {                                                 \
    constexpr int lds = conv_lds<NAME##_cfg, STEM>();                                      \
    static bool attr = false;                                                              \
    if (!attr) {                                                                           \
      hipError_t e = hipFuncSetAttribute(                                                  \
          reinterpret_cast<const void*>(&k_conv3x3<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM>), \
          hipFuncAttributeMaxDynamicSharedMemorySize, lds);                                \
      if (e != hipSuccess) return e;                                                       \
      attr = true;                                                                         \
    }                                                                                      \
    const int grid = (P + NP - 1) / NP * NAME##_cfg::RT;                                   \
    hipLaunchKernelGGL((k_conv3x3<CIN, COUT, HIN, S, NP, TR, WM, WN, STEM>), dim3(grid),   \
                       dim3(256), lds, st, in, out, static_cast<const uint4*>(wp), bias, P, \
                       sw, sb, eps);                                                       \
    return hipGetLastError();                                                              \
  }

// variant 0 = default tiling; variant 1 = smaller LDS footprint / more workgroups per CU
HN_CONV(conv1s_launch, true, 32, 32, 32, 1, 1, 8, 4, 1)
HN_CONV(conv1s_v1, true, 32, 32, 32, 1, 1, 4, 4, 1)
HN_CONV(conv1_launch, false, 32, 32, 32, 1, 1, 8, 4, 1)
HN_CONV(conv2_launch, false, 32, 64, 32, 2, 1, 8, 2, 2)
HN_CONV(conv2_v1, false, 32, 64, 32, 2, 1, 4, 2, 2)
HN_CONV(conv3_launch, false, 64, 64, 16, 1, 1, 16, 2, 2)
HN_CONV(conv3_v1, false, 64, 64, 16, 1, 1, 8, 2, 2)
HN_CONV(conv4_launch, false, 64, 128, 16, 2, 1, 8, 1, 4)
HN_CONV(conv4_v1, false, 64, 128, 16, 2, 1, 4, 1, 4)
HN_CONV(conv5_launch, false, 128, 128, 8, 1, 2, 8, 1, 4)
HN_CONV(conv5_v1, false, 128, 128, 8, 1, 1, 8, 1, 4)

hipError_t hn_launch_stem(const float* in, float* out, const float* w, const float* b, int P,
                          bool norm, float eps, hipStream_t st) {
  if (norm)
    hipLaunchKernelGGL(k_stem<true>, dim3(P), dim3(256), 0, st, in, out, w, b, eps);
  else
    hipLaunchKernelGGL(k_stem<false>, dim3(P), dim3(256), 0, st, in, out, w, b, eps);
  return hipGetLastError();
}

// layer 0 = fused stem (input_norm + conv0) + conv1 from the raw patches
hipError_t hn_launch_hardnet_conv(int layer, int variant, const HardnetDev& d, const float* in,
                                  float* out, int P, float eps, hipStream_t st) {
  const bool v1 = variant == 1;
  switch (layer) {
    case 0:
      return (v1 ? conv1s_v1 : conv1s_launch)(in, out, d.wpack[1], d.bias[1], P, d.stem_w,
                                               d.stem_b, eps, st);
    case 1: return conv1_launch(in, out, d.wpack[1], d.bias[1], P, nullptr, nullptr, 0.f, st);
    case 2:
      return (v1 ? conv2_v1 : conv2_launch)(in, out, d.wpack[2], d.bias[2], P, nullptr, nullptr, 0.f, st);
    case 3:
      return (v1 ? conv3_v1 : conv3_launch)(in, out, d.wpack[3], d.bias[3], P, nullptr, nullptr, 0.f, st);
    case 4:
      return (v1 ? conv4_v1 : conv4_launch)(in, out, d.wpack[4], d.bias[4], P, nullptr, nullptr, 0.f, st);
    case 5:
      return (v1 ? conv5_v1 : conv5_launch)(in, out, d.wpack[5], d.bias[5], P, nullptr, nullptr, 0.f, st);
  }
  return hipErrorInvalidValue;
}

hipError_t hn_launch_head(const float* a, float* out, const void* wp, const float* bias, int P,
                          int K, float l2eps, hipStream_t st) {
  const int grid = (P + 63) / 64;
  if (K == 8192)
    hipLaunchKernelGGL(k_head<8192>, dim3(grid), dim3(256), 0, st, a, out,
                       static_cast<const uint4*>(wp), bias, P, l2eps);
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
