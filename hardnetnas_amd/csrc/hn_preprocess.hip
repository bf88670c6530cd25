// Patch preprocessing on device: uint8 PhotoTour patches -> the fp32
// [B,1,32,32] network input, bit-exact with the reference loaders.
//
//   HN_RESIZE_CV2_LINEAR  hardnet/HardNet.py:345-349 + Utils.py:10-11: cv2.resize 64->32
//                         INTER_LINEAR, which OpenCV runs as its 2x area-fast path:
//                         (a + b + c + d + 2) >> 2 per 2x2 block.
//   HN_RESIZE_PIL_BILINEAR hardnet/HardNet.py:333-337: PIL Image.resize((32,32), BILINEAR):
//                         separable triangle filter (support 2 at scale 2), 22-bit fixed-point
//                         coefficients, horizontal then vertical pass, each rounding and
//                         clipping to uint8.
//   HN_RESIZE_NONE        input already 32x32 uint8 (cv2.resize to the same size = copy).
// then ToTensor (x / 255.f) and optionally Normalize ((x - mean) / std), fp32, same op order.
//
// HBM-bound byte work: 4 KiB in + 4 KiB out per 64x64 patch.  One wave per patch: the patch
// is read with 16-byte loads into LDS, filtered from LDS, and written as float4 rows.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hardnet_mi355x.h"
#include "hn_internal.h"

namespace {

// Pillow coefficients for 64 -> 32 (precompute_coeffs + normalize_coeffs_8bpc):
// interior taps at 2c-1..2c+2 = 0.125, 0.375, 0.375, 0.125; the border outputs have three
// taps 0.75/1.75, 0.75/1.75, 0.25/1.75 quantised to 22 bits.
constexpr int kPB = 22;
constexpr int kK0 = 524288, kK1 = 1572864, kE1 = 1797559, kE0 = 599186;

__device__ __forceinline__ int clip8(int ss) {
  ss >>= kPB;
  return ss < 0 ? 0 : (ss > 255 ? 255 : ss);
}

// 4 taps of one output (pos c) over a row of 64 pixels p[]; p is LDS, p[i] for i in [0,64)
__device__ __forceinline__ int pil_tap(const uint8_t* p, int c) {
  int ss = 1 << (kPB - 1);
  if (c == 0) {
    ss += p[0] * kE1 + p[1] * kE1 + p[2] * kE0;
  } else if (c == 31) {
    ss += p[61] * kE0 + p[62] * kE1 + p[63] * kE1;
  } else {
    const int x = 2 * c - 1;
    ss += p[x] * kK0 + p[x + 1] * kK1 + p[x + 2] * kK1 + p[x + 3] * kK0;
  }
  return clip8(ss);
}

__device__ __forceinline__ float to_input(int v, float mean, float stdv, int norm) {
  float f = (float)v / 255.0f;
  if (norm) f = (f - mean) / stdv;
  return f;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_preprocess(const uint8_t* __restrict__ in, int64_t n,
                                                    float* __restrict__ out, float mean,
                                                    float stdv, int norm) {
  constexpr int IN_HW = MODE == HN_RESIZE_NONE ? 32 : 64;
  constexpr int IN_BYTES = IN_HW * IN_HW;
  __shared__ __attribute__((aligned(16))) uint8_t s_in[4][IN_BYTES];
  __shared__ __attribute__((aligned(16))) uint8_t s_h[4][MODE == HN_RESIZE_PIL_BILINEAR ? 64 * 32 : 16];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t patch = (int64_t)blockIdx.x * 4 + w;
  if (patch >= n) return;  // whole wave exits together; no block barrier below
  const uint4* src = reinterpret_cast<const uint4*>(in + patch * IN_BYTES);
  uint4* dst = reinterpret_cast<uint4*>(s_in[w]);
#pragma unroll
  for (int i = 0; i < IN_BYTES / 16 / 64; ++i) dst[i * 64 + lane] = src[i * 64 + lane];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  const uint8_t* p = s_in[w];
  if (MODE == HN_RESIZE_PIL_BILINEAR) {
    // horizontal pass: 64 rows x 32 outputs
#pragma unroll 4
    for (int j = 0; j < 32; ++j) {
      const int t = j * 64 + lane, r = t >> 5, c = t & 31;
      s_h[w][t] = (uint8_t)pil_tap(p + r * 64, c);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  float4* o = reinterpret_cast<float4*>(out + patch * 1024);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = i * 256 + lane * 4, y = e >> 5, x0 = e & 31;
    int v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = x0 + k;
      if (MODE == HN_RESIZE_NONE) {
        v[k] = p[y * 32 + x];
      } else if (MODE == HN_RESIZE_CV2_LINEAR) {
        const uint8_t* q = p + (2 * y) * 64 + 2 * x;
        v[k] = (q[0] + q[1] + q[64] + q[65] + 2) >> 2;
      } else {
        const uint8_t* h = s_h[w];
        int ss = 1 << (kPB - 1);
        if (y == 0) {
          ss += h[x] * kE1 + h[32 + x] * kE1 + h[64 + x] * kE0;
        } else if (y == 31) {
          ss += h[61 * 32 + x] * kE0 + h[62 * 32 + x] * kE1 + h[63 * 32 + x] * kE1;
        } else {
          const int r = 2 * y - 1;
          ss += h[r * 32 + x] * kK0 + h[(r + 1) * 32 + x] * kK1 + h[(r + 2) * 32 + x] * kK1 +
                h[(r + 3) * 32 + x] * kK0;
        }
        v[k] = clip8(ss);
      }
    }
    o[e >> 2] = make_float4(to_input(v[0], mean, stdv, norm), to_input(v[1], mean, stdv, norm),
                            to_input(v[2], mean, stdv, norm), to_input(v[3], mean, stdv, norm));
  }
}

}  // namespace

hipError_t hn_launch_preprocess(const uint8_t* in, int64_t n, int resize, int norm, float mean,
                                float stdv, float* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 3) / 4)), block(256);
  switch (resize) {
    case HN_RESIZE_NONE:
      hipLaunchKernelGGL(k_preprocess<HN_RESIZE_NONE>, grid, block, 0, st, in, n, out, mean, stdv, norm);
      break;
    case HN_RESIZE_CV2_LINEAR:
      hipLaunchKernelGGL(k_preprocess<HN_RESIZE_CV2_LINEAR>, grid, block, 0, st, in, n, out, mean, stdv,
                         norm);
      break;
    case HN_RESIZE_PIL_BILINEAR:
      hipLaunchKernelGGL(k_preprocess<HN_RESIZE_PIL_BILINEAR>, grid, block, 0, st, in, n, out, mean,
                         stdv, norm);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
