// uint8 patch -> fp32 network input, shared by the standalone preprocessing kernel
// (hn_preprocess.hip) and the fused patch load of k_c12 (hn_c12.hip), so that both produce
// bit-identical inputs (the same integer filters, then the same fp32 ops):
//   HN_RESIZE_CV2_LINEAR   hardnet/HardNet.py:345-349 + Utils.py:10-11: cv2.resize 64->32
//                          INTER_LINEAR = OpenCV's 2x area-fast path, (a + b + c + d + 2) >> 2
//   HN_RESIZE_PIL_BILINEAR hardnet/HardNet.py:333-337: PIL resize((32, 32), BILINEAR): separable
//                          triangle filter (support 2 at scale 2), 22-bit fixed-point
//                          coefficients, horizontal then vertical pass, each rounding and
//                          clipping to uint8
//   HN_RESIZE_NONE         already 32x32 (cv2.resize to the same size is a copy)
// then ToTensor (v / 255.f) and optionally Normalize ((x - mean) / std) in fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hardnet_mi355x.h"

namespace hnpre {

// Pillow coefficients for 64 -> 32 (precompute_coeffs + normalize_coeffs_8bpc): interior taps
// at 2c-1..2c+2 = 0.125, 0.375, 0.375, 0.125; the border outputs have three taps 0.75/1.75,
// 0.75/1.75, 0.25/1.75 quantised to 22 bits.
constexpr int kPB = 22;
constexpr int kK0 = 524288, kK1 = 1572864, kE1 = 1797559, kE0 = 599186;

__device__ __forceinline__ int clip8(int ss) {
  ss >>= kPB;
  return ss < 0 ? 0 : (ss > 255 ? 255 : ss);
}

__device__ __forceinline__ float to_input(int v, float mean, float stdv, int norm) {
  float f = (float)v / 255.0f;
  if (norm) f = (f - mean) / stdv;
  return f;
}

__device__ __forceinline__ int byte_at(uint32_t w, int k) { return (int)((w >> (8 * k)) & 0xffu); }

// One thread's N consecutive output pixels (y, x .. x + N - 1) of a 32x32 patch (N = 2 or 4,
// x a multiple of N), as raw bytes fetched ahead of use (loads only; `value` does the math).
//   NONE: the N input bytes;  CV2: input rows 2y, 2y + 1, columns 2x .. 2x + 2N - 1;
//   PIL : input rows 2y - 1 .. 2y + 2 (clamped), columns 2x - 1 .. 2x + 2N (clamped at the
//         borders, where the border taps do not read them).
template <int MODE, int N>
struct U8Px {
  static_assert(N == 2 || N == 4, "2 or 4 pixels per thread");
  static constexpr int ROWS = MODE == HN_RESIZE_PIL_BILINEAR ? 4 : MODE == HN_RESIZE_CV2_LINEAR ? 2 : 1;
  static constexpr int W = MODE == HN_RESIZE_NONE ? 1 : N / 2;  // 32-bit words per row
  uint32_t mid[ROWS][W];  // NONE: N bytes in mid[0][0]; else columns 2x .. 2x + 2N - 1
  uint32_t edge[ROWS];    // PIL: byte 0 = column 2x - 1, byte 1 = column 2x + 2N

  __device__ __forceinline__ void load(const uint8_t* __restrict__ patch, int y, int x) {
    if constexpr (MODE == HN_RESIZE_NONE) {
      const uint8_t* s = patch + y * 32 + x;
      mid[0][0] = N == 4 ? *reinterpret_cast<const uint32_t*>(s)
                         : (uint32_t)*reinterpret_cast<const uint16_t*>(s);
    } else {
#pragma unroll
      for (int k = 0; k < ROWS; ++k) {
        int r = MODE == HN_RESIZE_PIL_BILINEAR ? 2 * y - 1 + k : 2 * y + k;
        r = r < 0 ? 0 : (r > 63 ? 63 : r);
        const uint8_t* s = patch + r * 64 + 2 * x;
        if constexpr (N == 4) {
          const uint2 v = *reinterpret_cast<const uint2*>(s);
          mid[k][0] = v.x;
          mid[k][1] = v.y;
        } else {
          mid[k][0] = *reinterpret_cast<const uint32_t*>(s);
        }
        if constexpr (MODE == HN_RESIZE_PIL_BILINEAR) {
          const int cl = 2 * x - 1 < 0 ? 0 : 2 * x - 1, cr = 2 * x + 2 * N > 63 ? 63 : 2 * x + 2 * N;
          edge[k] = (uint32_t)patch[r * 64 + cl] | ((uint32_t)patch[r * 64 + cr] << 8);
        }
      }
    }
  }

  // byte of row k at column 2x + j, j = -1 .. 2N
  __device__ __forceinline__ int b(int k, int j) const {
    if (j < 0) return byte_at(edge[k], 0);
    if (j >= 2 * N) return byte_at(edge[k], 1);
    return byte_at(mid[k][j >> 2], j & 3);
  }

  // the N output values (uint8 after resizing), i = 0 .. N - 1
  __device__ __forceinline__ void resized(int y, int x, int (&v)[N]) const {
    if constexpr (MODE == HN_RESIZE_NONE) {
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = byte_at(mid[0][0], i);
    } else if constexpr (MODE == HN_RESIZE_CV2_LINEAR) {
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = (b(0, 2 * i) + b(0, 2 * i + 1) + b(1, 2 * i) + b(1, 2 * i + 1) + 2) >> 2;
    } else {
      int hv[4][N];  // horizontal pass of the 4 rows, rounded and clipped to uint8
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < N; ++i) {
          const int c = x + i;
          int ss = 1 << (kPB - 1);
          if (c == 0)
            ss += b(k, 0) * kE1 + b(k, 1) * kE1 + b(k, 2) * kE0;
          else if (c == 31)
            ss += b(k, 2 * i - 1) * kE0 + b(k, 2 * i) * kE1 + b(k, 2 * i + 1) * kE1;
          else
            ss += b(k, 2 * i - 1) * kK0 + b(k, 2 * i) * kK1 + b(k, 2 * i + 1) * kK1 + b(k, 2 * i + 2) * kK0;
          hv[k][i] = clip8(ss);
        }
#pragma unroll
      for (int i = 0; i < N; ++i) {
        int ss = 1 << (kPB - 1);
        if (y == 0)
          ss += hv[1][i] * kE1 + hv[2][i] * kE1 + hv[3][i] * kE0;  // rows 0, 1, 2
        else if (y == 31)
          ss += hv[0][i] * kE0 + hv[1][i] * kE1 + hv[2][i] * kE1;  // rows 61, 62, 63
        else
          ss += hv[0][i] * kK0 + hv[1][i] * kK1 + hv[2][i] * kK1 + hv[3][i] * kK0;
        v[i] = clip8(ss);
      }
    }
  }
};

}  // namespace hnpre
