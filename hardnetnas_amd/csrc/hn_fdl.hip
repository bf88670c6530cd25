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
// One wave per patch (4 per workgroup); lane = output pixel (lane >> 3, lane & 7).  fp32 VALU
// throughout (3,360 / 4,640 FMA per lane): the weights are wave-uniform (scalar loads), BN is
// folded into them on the host.  input_norm as des.py:40-47: (x - mean) / (std_unbiased + eps).
#include "hn_common.h"
#include "hn_internal.h"

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
      h[co] = fmaxf(acc, 0.f);
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
      r[j] = fmaxf(acc, 0.f);
    }
    reinterpret_cast<float4*>(dst)[c4] = make_float4(r[0], r[1], r[2], r[3]);
  }
}

}  // namespace

hipError_t hn_launch_fdl_front(const HnFdlFrontArgs& a, int P, int mode, float eps, hipStream_t st) {
  if (P <= 0) return hipSuccess;
  const int grid = (P + 3) / 4;
  if (mode == 0)
    hipLaunchKernelGGL(k_fdl_front<0>, dim3(grid), dim3(256), 0, st, a.in, a.out, a.stem_w, a.stem_b,
                       a.w1, a.b1, a.w2, a.b2, P, eps);
  else if (mode == 1)
    hipLaunchKernelGGL(k_fdl_front<1>, dim3(grid), dim3(256), 0, st, a.in, a.out, a.stem_w, a.stem_b,
                       a.w1, a.b1, a.w2, a.b2, P, eps);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
