// Fused NAS front: the stem ConvBNRelu(1->32, 3x3) (model_supernet.py:57-58,
// fbnet_builder.py:352-404) and the first searched layer (SEARCH_SPACE2[0] = (32, 32, s2),
// lookup_table_builder.py:22-45) in one kernel, so the two 128 KB/patch tensors of the
// 32x32 stage (stem output, pw output) never reach HBM.
//
//   MODE FRONT_IRF:     IRFBlock pw 1x1 (groups, BN, ReLU) [+ ChannelShuffle] -> dw kxk s2
//                       (BN, ReLU)  (fbnet_builder.py:455-570); writes the dw output
//                       [P,16,16,MID]; pwl/residual/SE follow as separate kernels.
//   MODE FRONT_MAXPOOL: the "skip" op at stride 2 = MaxPool2d(3, 2, 1)
//                       (fbnet_builder.py:202-228); writes [P,16,16,32].
//
// One workgroup (4 waves) owns a band of 4 output rows of one patch.  The band's
// 2*3+k pw rows (halo recomputed by the neighbouring band) are produced row by row: a wave
// computes the stem for one image row (32 pixels) on the VALU straight into the MFMA
// B-operand layout (lane = pixel, 16 channels per lane), keeps it in registers, and runs
// the 1x1 conv for each 32-channel chunk of MID as a 32x32x32 fp16x3 MFMA tile (weights =
// A operand, BN scale folded, shuffle folded into the row order, groups densified).  The
// chunk's pw rows go to LDS; the depthwise conv reads them from LDS (fp32 VALU) and
// writes float4s of 4 channels to HBM.
#include "hn_common.h"
#include "hn_internal.h"

namespace {

constexpr int FRONT_IRF = 0, FRONT_MAXPOOL = 1;
constexpr int RB = 4;   // output rows per band
constexpr int PS = 36;  // floats per pixel in the LDS pw band (32 channels + 4 pad)

template <int K, int MID, int MODE, bool NORM>
__global__ __launch_bounds__(256) void k_front(const float* __restrict__ in,
                                               float* __restrict__ out,
                                               const float* __restrict__ stem_w,  // [9][32]
                                               const float* __restrict__ stem_b,  // [32]
                                               const uint4* __restrict__ apack,
                                               const float* __restrict__ pw_b,  // [MID] (dw order)
                                               const float* __restrict__ dw_w,  // [K*K][MID]
                                               const float* __restrict__ dw_b,  // [MID]
                                               float eps) {
  constexpr int KK = MODE == FRONT_MAXPOOL ? 3 : K;
  constexpr int PAD = KK / 2;
  constexpr int IR = 2 * (RB - 1) + KK;  // pw rows of the band
  constexpr int PC = 32 + 2 * PAD;       // columns incl. zero padding
  constexpr int NT = (IR + 3) / 4;       // row tiles per wave
  constexpr int OC = MODE == FRONT_MAXPOOL ? 32 : MID;
  __shared__ float s_in[34 * 34];
  __shared__ __attribute__((aligned(16))) float s_sw[9 * 32 + 32];
  __shared__ __attribute__((aligned(16))) float s_pw[IR * PC * PS];
  __shared__ __attribute__((aligned(16))) float s_dw[KK * KK * 32 + 32];
  __shared__ float red[8];

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int px = lane & 31, h = lane >> 5;
  const long patch = blockIdx.x >> 2;
  const int r0 = (blockIdx.x & 3) * RB;
  const int row0 = 2 * r0 - PAD;

  // ---- phase 0: patch (+ input_norm) and stem weights to LDS, zero the pw band --------
  const float4 v = reinterpret_cast<const float4*>(in + patch * 1024)[t];
  for (int i = t; i < 34 * 34; i += 256) s_in[i] = 0.f;
  for (int i = t; i < IR * PC * PS / 4; i += 256)
    reinterpret_cast<float4*>(s_pw)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = t; i < 9 * 32 + 32; i += 256) s_sw[i] = i < 288 ? stem_w[i] : stem_b[i - 288];
  float mean = 0.f, sd = 1.f;
  if (NORM) {  // (x - mean) / (std_unbiased + eps), as k_stem
    const float s = wave_sum(v.x + v.y + v.z + v.w);
    if (lane == 0) red[w] = s;
    __syncthreads();
    mean = (red[0] + red[1] + red[2] + red[3]) * (1.f / 1024.f);
    const float d0 = v.x - mean, d1 = v.y - mean, d2 = v.z - mean, d3 = v.w - mean;
    const float q = wave_sum(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3);
    if (lane == 0) red[4 + w] = q;
    __syncthreads();
    sd = sqrtf((red[4] + red[5] + red[6] + red[7]) * (1.f / 1023.f)) + eps;
  }
  __syncthreads();
  {
    const int q = 4 * t, y = q >> 5, x = q & 31;
    float* d = s_in + (y + 1) * 34 + x + 1;
    if (NORM) {
      d[0] = (v.x - mean) / sd; d[1] = (v.y - mean) / sd;
      d[2] = (v.z - mean) / sd; d[3] = (v.w - mean) / sd;
    } else {
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  }
  __syncthreads();

  // ---- phase A: stem rows of the band (lane: pixel px, channels 8h..8h+7, 16+8h..+7) ----
  uint4 bh[NT][2], bl[NT][2];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int ri = w + 4 * i, y = row0 + ri;
    bh[i][0] = bh[i][1] = bl[i][0] = bl[i][1] = make_uint4(0, 0, 0, 0);
    if (ri >= IR || y < 0 || y >= 32) continue;  // wave-uniform
    float a[16];
    {
      const float4* b4 = reinterpret_cast<const float4*>(s_sw + 288);
      const float4 b0 = b4[2 * h], b1 = b4[2 * h + 1], b2 = b4[4 + 2 * h], b3 = b4[5 + 2 * h];
      a[0] = b0.x; a[1] = b0.y; a[2] = b0.z; a[3] = b0.w; a[4] = b1.x; a[5] = b1.y; a[6] = b1.z; a[7] = b1.w;
      a[8] = b2.x; a[9] = b2.y; a[10] = b2.z; a[11] = b2.w; a[12] = b3.x; a[13] = b3.y; a[14] = b3.z; a[15] = b3.w;
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const float xv = s_in[(y + tap / 3) * 34 + px + tap % 3];
      const float4* w4 = reinterpret_cast<const float4*>(s_sw + tap * 32);
      const float4 w0 = w4[2 * h], w1 = w4[2 * h + 1], w2 = w4[4 + 2 * h], w3 = w4[5 + 2 * h];
      a[0] = fmaf(w0.x, xv, a[0]); a[1] = fmaf(w0.y, xv, a[1]); a[2] = fmaf(w0.z, xv, a[2]); a[3] = fmaf(w0.w, xv, a[3]);
      a[4] = fmaf(w1.x, xv, a[4]); a[5] = fmaf(w1.y, xv, a[5]); a[6] = fmaf(w1.z, xv, a[6]); a[7] = fmaf(w1.w, xv, a[7]);
      a[8] = fmaf(w2.x, xv, a[8]); a[9] = fmaf(w2.y, xv, a[9]); a[10] = fmaf(w2.z, xv, a[10]); a[11] = fmaf(w2.w, xv, a[11]);
      a[12] = fmaf(w3.x, xv, a[12]); a[13] = fmaf(w3.y, xv, a[13]); a[14] = fmaf(w3.z, xv, a[14]); a[15] = fmaf(w3.w, xv, a[15]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = fmaxf(a[j], 0.f);
    if (MODE == FRONT_MAXPOOL) {
      float4* d = reinterpret_cast<float4*>(s_pw + (ri * PC + PAD + px) * PS);
      d[2 * h] = make_float4(a[0], a[1], a[2], a[3]);
      d[2 * h + 1] = make_float4(a[4], a[5], a[6], a[7]);
      d[4 + 2 * h] = make_float4(a[8], a[9], a[10], a[11]);
      d[5 + 2 * h] = make_float4(a[12], a[13], a[14], a[15]);
    } else {
      split8_f16(make_float4(a[0], a[1], a[2], a[3]), make_float4(a[4], a[5], a[6], a[7]), bh[i][0], bl[i][0]);
      split8_f16(make_float4(a[8], a[9], a[10], a[11]), make_float4(a[12], a[13], a[14], a[15]), bh[i][1], bl[i][1]);
    }
  }

  if (MODE == FRONT_MAXPOOL) {
    __syncthreads();
    // MaxPool2d(3, 2, 1): padding never wins since every window holds a ReLU output >= 0
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int item = t + 256 * j, q = item & 7, p = item >> 3, orr = p >> 4, ox = p & 15;
      float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const float4 a = *reinterpret_cast<const float4*>(s_pw + ((2 * orr + dy) * PC + 2 * ox + dx) * PS + 4 * q);
          m.x = fmaxf(m.x, a.x); m.y = fmaxf(m.y, a.y); m.z = fmaxf(m.z, a.z); m.w = fmaxf(m.w, a.w);
        }
      *reinterpret_cast<float4*>(out + ((patch * 16 + r0 + orr) * 16 + ox) * 32 + 4 * q) = m;
    }
    return;
  }

  // ---- phases B/C per 32-channel chunk of MID ------------------------------------------
#pragma unroll 1
  for (int m = 0; m < MID / 32; ++m) {
    // dw weights + bias of the chunk
    for (int i = t; i < KK * KK * 8 + 8; i += 256) {
      float4 wv;
      if (i < KK * KK * 8)
        wv = *reinterpret_cast<const float4*>(dw_w + (i >> 3) * MID + 32 * m + 4 * (i & 7));
      else
        wv = *reinterpret_cast<const float4*>(dw_b + 32 * m + 4 * (i - KK * KK * 8));
      reinterpret_cast<float4*>(s_dw)[i] = wv;
    }
    const uint4* ap = apack + (size_t)m * 4 * 64 + lane;
    const f16x8 ah0 = as_f16x8(ap[0]), al0 = as_f16x8(ap[64]);
    const f16x8 ah1 = as_f16x8(ap[128]), al1 = as_f16x8(ap[192]);
    float4 bias[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bias[q] = *reinterpret_cast<const float4*>(pw_b + 32 * m + 8 * q + 4 * h);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const int ri = w + 4 * i, y = row0 + ri;
      if (ri >= IR || y < 0 || y >= 32) continue;
      f32x16 acc = {};
      acc = mfma3_f16(ah0, al0, as_f16x8(bh[i][0]), as_f16x8(bl[i][0]), acc);
      acc = mfma3_f16(ah1, al1, as_f16x8(bh[i][1]), as_f16x8(bl[i][1]), acc);
      float4* d = reinterpret_cast<float4*>(s_pw + (ri * PC + PAD + px) * PS);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        d[2 * q + h] = make_float4(fmaxf(acc[4 * q] + bias[q].x, 0.f), fmaxf(acc[4 * q + 1] + bias[q].y, 0.f),
                                   fmaxf(acc[4 * q + 2] + bias[q].z, 0.f), fmaxf(acc[4 * q + 3] + bias[q].w, 0.f));
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int item = t + 256 * j, q = item & 7, p = item >> 3, orr = p >> 4, ox = p & 15;
      float4 acc = reinterpret_cast<const float4*>(s_dw + KK * KK * 32)[q];
#pragma unroll
      for (int dy = 0; dy < KK; ++dy)
#pragma unroll
        for (int dx = 0; dx < KK; ++dx) {
          const float4 wv = reinterpret_cast<const float4*>(s_dw + (dy * KK + dx) * 32)[q];
          const float4 a = *reinterpret_cast<const float4*>(s_pw + ((2 * orr + dy) * PC + 2 * ox + dx) * PS + 4 * q);
          acc.x = fmaf(wv.x, a.x, acc.x); acc.y = fmaf(wv.y, a.y, acc.y);
          acc.z = fmaf(wv.z, a.z, acc.z); acc.w = fmaf(wv.w, a.w, acc.w);
        }
      acc.x = fmaxf(acc.x, 0.f); acc.y = fmaxf(acc.y, 0.f); acc.z = fmaxf(acc.z, 0.f); acc.w = fmaxf(acc.w, 0.f);
      *reinterpret_cast<float4*>(out + ((patch * 16 + r0 + orr) * 16 + ox) * OC + 32 * m + 4 * q) = acc;
    }
    __syncthreads();
  }
}

template <int K, int MID, int MODE>
hipError_t front_launch(const HnFrontArgs& a, int P, bool norm, float eps, hipStream_t st) {
  const dim3 grid((unsigned)P * 4), block(256);
  if (norm)
    hipLaunchKernelGGL((k_front<K, MID, MODE, true>), grid, block, 0, st, a.in, a.out, a.stem_w, a.stem_b,
                       a.apack, a.pw_b, a.dw_w, a.dw_b, eps);
  else
    hipLaunchKernelGGL((k_front<K, MID, MODE, false>), grid, block, 0, st, a.in, a.out, a.stem_w, a.stem_b,
                       a.apack, a.pw_b, a.dw_w, a.dw_b, eps);
  return hipGetLastError();
}

}  // namespace

bool hn_front_supported(int k, int mid) {
  return (k == 3 || k == 5) && (mid == 32 || mid == 96 || mid == 128);
}

hipError_t hn_launch_front(const HnFrontArgs& a, int P, int k, int mid, bool maxpool, bool norm,
                           float eps, hipStream_t st) {
  if (P <= 0) return hipSuccess;
  if (maxpool) return front_launch<3, 32, FRONT_MAXPOOL>(a, P, norm, eps, st);
#define HN_FRONT(KK, MM) \
  if (k == KK && mid == MM) return front_launch<KK, MM, FRONT_IRF>(a, P, norm, eps, st);
  HN_FRONT(3, 32) HN_FRONT(3, 96) HN_FRONT(3, 128) HN_FRONT(5, 32) HN_FRONT(5, 96) HN_FRONT(5, 128)
#undef HN_FRONT
  return hipErrorInvalidValue;
}
