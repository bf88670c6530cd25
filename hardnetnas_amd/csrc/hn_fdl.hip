// FDLNet HardNetNeiMask front: the layers before the three IRFBlocks,
// 32x32 patch -> 8x8x64 NHWC, in one pass.
//
//   MODE 0, "NASNet" (FDLNet-master/latency/NASNet/model/des.py:13-24):
//     input_norm -> Conv 3x3 (bias) -> BN(affine=False) -> Conv 1x1 s2 32->32 + BN + ReLU
//     -> Conv 1x1 s2 32->64 + BN + ReLU.
//     The two stride-2 1x1 convs read only every other pixel of their input, so output pixel
//     (oy, ox) depends on the stem at the single input pixel (4 oy, 4 ox): a per-pixel MLP
//     9 taps -> 32 -> 32 -> 64.
//   MODE 1, "NASNet_0.1" (latency/NASNet_0.1/model/des.py:17-23):
//     input_norm -> Conv 3x3 (bias) -> MaxPool(3, 2, 1) -> Identity -> ConvBNRelu 1x1 s2 32->64.
//     Output pixel (oy, ox) = 1x1 conv of the max-pool at (2 oy, 2 ox), i.e. the maximum of the
//     stem over rows / columns 4 o - 1 .. 4 o + 1 (padding excluded, as -inf).
//
// k_fdl_front (HN_FDL_VALU=1, kept for A/B): one wave per patch (4 per workgroup); lane = output
// pixel (lane >> 3, lane & 7).  fp32 VALU
// throughout (3,360 / 4,640 FMA per lane): the weights are wave-uniform (scalar loads), BN is
// folded into them on the host.  input_norm as des.py:40-47: (x - mean) / (std_unbiased + eps).
#include "hn_common.h"
#include "hn_internal.h"
#include "hn_preproc.h"

#include <algorithm>
#include <cstdlib>

namespace {

template <int MODE>
__global__ __launch_bounds__(256) void k_fdl_front(const float* __restrict__ in, float* __restrict__ out,
                                                   const float* __restrict__ ws,  // [9][32] stem (BN folded in MODE 0)
                                                   const float* __restrict__ bs,  // [32]
                                                   const float* __restrict__ w1,  // [32][32] (cin, cout), MODE 0
                                                   const float* __restrict__ b1,  // [32]
                                                   const float* __restrict__ w2,  // [32][64] (cin, cout)
                                                   const float* __restrict__ b2,  // [64]
                                                   int P, float eps) {
  __shared__ float s_x[4][34 * 34];  // normalised patches with a zero border
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const long p = (long)blockIdx.x * 4 + w;
  float* xs = s_x[w];
  for (int i = lane; i < 34 * 34; i += 64) xs[i] = 0.f;
  __syncthreads();  // the zero border before the interior stores
  if (p < P) {      // wave-uniform
    const float4* src = reinterpret_cast<const float4*>(in + p * 1024);
    float v[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 q = src[lane + 64 * k];
      v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
    }
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) a += v[j];
    const float mean = wave_sum(a) * (1.f / 1024.f);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) q += (v[j] - mean) * (v[j] - mean);
    const float sd = sqrtf(wave_sum(q) * (1.f / 1023.f)) + eps;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int px = 4 * (lane + 64 * k), y = px >> 5, x = px & 31;
#pragma unroll
      for (int j = 0; j < 4; ++j) xs[(y + 1) * 34 + x + 1 + j] = (v[4 * k + j] - mean) / sd;
    }
  }
  __syncthreads();
  if (p >= P) return;

  const int oy = lane >> 3, ox = lane & 7;
  // stem (3x3, pad 1) at input pixel (y, x) into s[32]
  auto stem = [&](int y, int x, float (&s)[32]) {
    float tap[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) tap[k] = xs[(y + k / 3) * 34 + x + k % 3];
#pragma unroll
    for (int c = 0; c < 32; ++c) {
      float acc = bs[c];
#pragma unroll
      for (int k = 0; k < 9; ++k) acc = fmaf(ws[k * 32 + c], tap[k], acc);
      s[c] = acc;
    }
  };
  float h[32];
  if constexpr (MODE == 0) {
    float s[32];
    stem(4 * oy, 4 * ox, s);
#pragma unroll
    for (int co = 0; co < 32; ++co) {
      float acc = b1[co];
#pragma unroll
      for (int ci = 0; ci < 32; ++ci) acc = fmaf(w1[ci * 32 + co], s[ci], acc);
      h[co] = relu0(acc);
    }
  } else {
#pragma unroll
    for (int c = 0; c < 32; ++c) h[c] = -__builtin_huge_valf();
#pragma unroll 1
    for (int dy = -1; dy <= 1; ++dy) {
      const int y = 4 * oy + dy;
      if (y < 0) continue;  // rows 4 oy - 1 .. 4 oy + 1 stay below 32
#pragma unroll 1
      for (int dx = -1; dx <= 1; ++dx) {
        const int x = 4 * ox + dx;
        if (x < 0) continue;
        float s[32];
        stem(y, x, s);
#pragma unroll
        for (int c = 0; c < 32; ++c) h[c] = fmaxf(h[c], s[c]);
      }
    }
  }
  float* dst = out + ((p * 8 + oy) * 8 + ox) * 64;
#pragma unroll
  for (int c4 = 0; c4 < 16; ++c4) {
    float r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = 4 * c4 + j;
      float acc = b2[co];
#pragma unroll
      for (int ci = 0; ci < 32; ++ci) acc = fmaf(w2[ci * 64 + co], h[ci], acc);
      r[j] = relu0(acc);
    }
    reinterpret_cast<float4*>(dst)[c4] = make_float4(r[0], r[1], r[2], r[3]);
  }
}

// k_fdl_front_mfma: the same front on the MFMA (32x32x16 fp16x3 split products, fp32
// accumulate).  Persistent workgroups of 4 waves, one patch per wave per iteration (the next
// patch prefetched into registers); a patch's 64 output pixels are two 32-pixel tiles whose
// chains interleave.  Operand roles as k_front: A = weights (rows = output channels), B =
// pixels, so the accumulator leaves lane (px, h) with channels 8q + 4h + r (i = 4q + r) of
// pixel px -- used as-is as the next 1x1's B operand (K-step ks = accumulator entries
// 8ks .. 8ks + 7; the A operand is packed in that channel order), so the whole chain stays in
// registers and only the 8x8x64 output leaves the wave.
//   stem: K = 9 taps + the bias in K slot 9 (B = 1.0 there), BN folded on the host (MODE 0).
//   MODE 0: stem -> 1x1 32 -> 32 (+ReLU) -> 1x1 32 -> 64 (+ReLU), one stem pixel per output.
//   MODE 1: max over the 3x3 window of stem pixels (invalid positions excluded) -> 1x1 -> 64.
// U8: -1 = fp32 [P,1,32,32] input; HN_RESIZE_* = uint8 patches resized, /255'd and
// Normalize'd in the patch load (hn_preproc.h, the arithmetic of hn_preprocess), one patch ahead
template <int MODE, int U8 = -1>
__global__ __launch_bounds__(256) void k_fdl_front_mfma(const void* __restrict__ in_, float* __restrict__ out,
                                                        const float* __restrict__ ws,  // [9][32]
                                                        const float* __restrict__ bs,  // [32]
                                                        const float* __restrict__ w1,  // [32][32] (cin, cout)
                                                        const float* __restrict__ b1,  // [32]
                                                        const float* __restrict__ w2,  // [32][64] (cin, cout)
                                                        const float* __restrict__ b2,  // [64]
                                                        int P, float eps, float pmean, float pstd, int pnorm) {
  __shared__ float s_x[4][34 * 34];  // normalised patches with a zero border
  // per-wave 32-pixel x 32-channel output tile, transposed for stores of whole 128-byte rows
  __shared__ __attribute__((aligned(16))) float s_o[4][32 * 36];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r = lane & 31, h = lane >> 5;
  float* xs = s_x[w];
  float* so = s_o[w];
  for (int i = lane; i < 34 * 34; i += 64) xs[i] = 0.f;  // the border stays zero
  // ---- A operands (fp16 hi / lo), built once per wave --------------------------------------
  auto split_a = [&](const float (&v)[8], f16x8& hi, f16x8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      hi[j] = (_Float16)v[j];
      lo[j] = (_Float16)(v[j] - (float)hi[j]);
    }
  };
  f16x8 sh, sl;  // stem: row = channel r, K = taps 8h .. 8h + 7 (slot 9 = bias)
  {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int tap = 8 * h + j;
      v[j] = tap < 9 ? ws[tap * 32 + r] : (tap == 9 ? bs[r] : 0.f);
    }
    split_a(v, sh, sl);
  }
  // 1x1 weights: row = output channel, K-step ks entry j = input channel 8 (2 ks + j / 4) + 4 h + j % 4
  auto pack_pw = [&](const float* wt, int ncout, int co, int ks, f16x8& hi, f16x8& lo) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = wt[(8 * (2 * ks + (j >> 2)) + 4 * h + (j & 3)) * ncout + co];
    split_a(v, hi, lo);
  };
  f16x8 ah1[2], al1[2], ah2[2][2], al2[2][2];  // [ks] / [nt][ks]
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    if (MODE == 0) pack_pw(w1, 32, r, ks, ah1[ks], al1[ks]);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) pack_pw(w2, 64, 32 * nt + r, ks, ah2[nt][ks], al2[nt][ks]);
  }
  // bias in the accumulator order (channel 8q + 4h + r' at i = 4q + r')
  auto bias16 = [&](const float* b) {
    f32x16 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 x = *reinterpret_cast<const float4*>(b + 8 * q + 4 * h);
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
    }
    return v;
  };
  // B operand of a K-step from an accumulator (ReLU'd by the caller): entries 8ks .. 8ks + 7
  auto bfrag = [](const f32x16& c, int ks, f16x8& hi, f16x8& lo) {
    uint4 uh, ul;
    split8_f16(make_float4(c[8 * ks], c[8 * ks + 1], c[8 * ks + 2], c[8 * ks + 3]),
               make_float4(c[8 * ks + 4], c[8 * ks + 5], c[8 * ks + 6], c[8 * ks + 7]), uh, ul);
    hi = as_f16x8(uh);
    lo = as_f16x8(ul);
  };

  const long stride = (long)gridDim.x * 4;
  long p = (long)blockIdx.x * 4 + w;
  // the lane's pixels: 4 runs of 4, (y, x) = (px >> 5, px & 31), px = 4 (lane + 64 k)
  const float* in = static_cast<const float*>(in_);
  const uint8_t* in8 = static_cast<const uint8_t*>(in_);
  constexpr int INB = U8 == HN_RESIZE_NONE ? 1024 : 4096;  // bytes per uint8 patch
  float4 vn[4];
  hnpre::U8Px<U8 < 0 ? HN_RESIZE_NONE : U8, 4> rn[4];
  auto fetch = [&](long pp) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (U8 < 0) {
        vn[k] = reinterpret_cast<const float4*>(in + pp * 1024)[lane + 64 * k];
      } else {
        const int px = 4 * (lane + 64 * k);
        rn[k].load(in8 + pp * INB, px >> 5, px & 31);
      }
    }
  };
  if (p < P) fetch(p);
#pragma unroll 1
  for (; p < P; p += stride) {  // wave-uniform
    float v[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (U8 < 0) {
        v[4 * k] = vn[k].x; v[4 * k + 1] = vn[k].y; v[4 * k + 2] = vn[k].z; v[4 * k + 3] = vn[k].w;
      } else {
        const int px = 4 * (lane + 64 * k);
        int q[4];
        rn[k].resized(px >> 5, px & 31, q);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 * k + j] = hnpre::to_input(q[j], pmean, pstd, pnorm);
      }
    }
    if (p + stride < P) fetch(p + stride);
    // input_norm as des.py:40-47: (x - mean) / (std_unbiased + eps)
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) a += v[j];
    const float mean = wave_sum(a) * (1.f / 1024.f);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) q += (v[j] - mean) * (v[j] - mean);
    const float sd = sqrtf(wave_sum(q) * (1.f / 1023.f)) + eps;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int px = 4 * (lane + 64 * k), y = px >> 5, x = px & 31;
#pragma unroll
      for (int j = 0; j < 4; ++j) xs[(y + 1) * 34 + x + 1 + j] = (v[4 * k + j] - mean) / sd;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's stores before its reads
    __builtin_amdgcn_wave_barrier();

    // stem at input pixel (y, x) for this lane's pixel of tile tt: B = taps 8h .. (slot 9 = 1.0)
    auto stem = [&](int y, int x) {
      float tp[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tap = 8 * h + j;
        tp[j] = tap < 9 ? xs[(y + tap / 3) * 34 + x + tap % 3] : (tap == 9 ? 1.f : 0.f);
      }
      uint4 xh, xl;
      split8_f16(make_float4(tp[0], tp[1], tp[2], tp[3]), make_float4(tp[4], tp[5], tp[6], tp[7]), xh, xl);
      return mfma3_f16(sh, sl, as_f16x8(xh), as_f16x8(xl), f32x16{});
    };
    f32x16 hmid[2];  // the 32 channels feeding the last 1x1, per tile
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int op = 32 * tt + r, oy = op >> 3, ox = op & 7;  // this lane's output pixel
      if constexpr (MODE == 0) {
        const f32x16 s0 = stem(4 * oy, 4 * ox);  // (padded coordinates: +1 -1 cancel)
        f32x16 c = bias16(b1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          f16x8 bh, bl;
          bfrag(s0, ks, bh, bl);
          c = mfma3_f16(ah1[ks], al1[ks], bh, bl, c);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = relu0(c[i]);
        hmid[tt] = c;
      } else {
        f32x16 m;
#pragma unroll
        for (int i = 0; i < 16; ++i) m[i] = -__builtin_huge_valf();
#pragma unroll 1
        for (int d = 0; d < 9; ++d) {
          const int y = 4 * oy + d / 3 - 1, x = 4 * ox + d % 3 - 1;
          const bool ok = y >= 0 && x >= 0;  // rows / columns 4o + 1 stay below 32
          const f32x16 s0 = stem(ok ? y : 0, ok ? x : 0);
#pragma unroll
          for (int i = 0; i < 16; ++i) m[i] = ok ? fmaxf(m[i], s0[i]) : m[i];
        }
        hmid[tt] = m;
      }
    }
    // last 1x1 32 -> 64 + BN + ReLU, both tiles, both output-channel halves
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      f16x8 bh[2], bl[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bfrag(hmid[tt], ks, bh[ks], bl[ks]);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        f32x16 c = bias16(b2 + 32 * nt);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) c = mfma3_f16(ah2[nt][ks], al2[nt][ks], bh[ks], bl[ks], c);
        if constexpr (MODE == 1) {  // (the transposed form measured slower here: 1.59 -> 1.68 ms)
          float* dst = out + (p * 64 + 32 * tt + r) * 64 + 32 * nt + 4 * h;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq)
            *reinterpret_cast<float4*>(dst + 8 * qq) =
                make_float4(relu0(c[4 * qq]), relu0(c[4 * qq + 1]), relu0(c[4 * qq + 2]),
                            relu0(c[4 * qq + 3]));
          continue;
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          *reinterpret_cast<float4*>(so + r * 36 + 8 * qq + 4 * h) =
              make_float4(relu0(c[4 * qq]), relu0(c[4 * qq + 1]), relu0(c[4 * qq + 2]),
                          relu0(c[4 * qq + 3]));
        __builtin_amdgcn_wave_barrier();  // (one wave: its LDS accesses execute in order)
        asm volatile("" ::: "memory");
        float* dst = out + (p * 64 + 32 * tt) * 64 + 32 * nt;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int pl = 8 * k + (lane >> 3), c4 = lane & 7;
          *reinterpret_cast<float4*>(dst + pl * 64 + 4 * c4) = *reinterpret_cast<const float4*>(so + pl * 36 + 4 * c4);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
      }
    }
    __builtin_amdgcn_wave_barrier();  // this patch's reads of xs before the next patch's stores
  }
}

}  // namespace

hipError_t hn_launch_fdl_front(const HnFdlFrontArgs& a, int P, int mode, float eps, hipStream_t st,
                               const HnU8In* u8) {
  if (P <= 0) return hipSuccess;
  if (mode != 0 && mode != 1) return hipErrorInvalidValue;
  if (!hn_knobs().fdl_valu) {  // HN_FDL_VALU=1: the fp32 VALU form (A/B)
    const void* src = u8 ? static_cast<const void*>(u8->in) : static_cast<const void*>(a.in);
    const float pm = u8 ? u8->mean : 0.f, ps = u8 ? u8->stdv : 1.f;
    const int pn = u8 ? u8->normalize : 0;
    // persistent grid: the resident workgroups of the instantiation launched (the PIL loads hold more registers)
#define HN_FDL_GO(M, ...)                                                                                          \
  {                                                                                                                \
    int resident = 0;                                                                                              \
    const hipError_t e = hn_resident_blocks(reinterpret_cast<const void*>(&k_fdl_front_mfma<M, ##__VA_ARGS__>), 256, \
                                            0, &resident);                                                         \
    if (e != hipSuccess) return e;                                                                                 \
    hipLaunchKernelGGL((k_fdl_front_mfma<M, ##__VA_ARGS__>), dim3(std::min((P + 3) / 4, resident)), dim3(256), 0, st, \
                       src, a.out, a.stem_w, a.stem_b, a.w1, a.b1, a.w2, a.b2, P, eps, pm, ps, pn);                \
  }
#define HN_FDL_MODES(M)                                                          \
  if (!u8) HN_FDL_GO(M)                                                          \
  else if (u8->resize == HN_RESIZE_NONE) HN_FDL_GO(M, HN_RESIZE_NONE)            \
  else if (u8->resize == HN_RESIZE_CV2_LINEAR) HN_FDL_GO(M, HN_RESIZE_CV2_LINEAR) \
  else if (u8->resize == HN_RESIZE_PIL_BILINEAR) HN_FDL_GO(M, HN_RESIZE_PIL_BILINEAR) \
  else return hipErrorInvalidValue;
    if (mode == 0) {
      HN_FDL_MODES(0)
    } else {
      HN_FDL_MODES(1)
    }
#undef HN_FDL_MODES
#undef HN_FDL_GO
    return hipGetLastError();
  }
  if (u8) return hipErrorInvalidValue;  // the VALU A/B form reads fp32 patches only
  const int grid = (P + 3) / 4;
  if (mode == 0)
    hipLaunchKernelGGL(k_fdl_front<0>, dim3(grid), dim3(256), 0, st, a.in, a.out, a.stem_w, a.stem_b,
                       a.w1, a.b1, a.w2, a.b2, P, eps);
  else
    hipLaunchKernelGGL(k_fdl_front<1>, dim3(grid), dim3(256), 0, st, a.in, a.out, a.stem_w, a.stem_b,
                       a.w1, a.b1, a.w2, a.b2, P, eps);
  return hipGetLastError();
}
