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
// reads its rows with 16-byte loads straight into registers (the PIL mode exchanges the
// horizontally filtered rows through 2 KiB of LDS) and writes float4 rows.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hardnet_mi355x.h"
#include "hn_internal.h"
#include "hn_preproc.h"

namespace {

using hnpre::clip8;
using hnpre::kE0;
using hnpre::kE1;
using hnpre::kK0;
using hnpre::kK1;
using hnpre::kPB;
using hnpre::to_input;

__device__ __forceinline__ int byte_of(const uint4& q, int k) {  // k is a compile-time constant
  const unsigned w = k < 4 ? q.x : k < 8 ? q.y : k < 12 ? q.z : q.w;
  return (int)((w >> (8 * (k & 3))) & 0xffu);
}

__device__ __forceinline__ void store4(float* o, const int* v, float mean, float stdv, int norm) {
  *reinterpret_cast<float4*>(o) =
      make_float4(to_input(v[0], mean, stdv, norm), to_input(v[1], mean, stdv, norm),
                  to_input(v[2], mean, stdv, norm), to_input(v[3], mean, stdv, norm));
}

// One wave per patch, four patches per 256-thread block; no block-level barriers, so a
// wave past the end of the batch simply exits.
template <int MODE>
__global__ __launch_bounds__(256) void k_preprocess(const uint8_t* __restrict__ in, int64_t n,
                                                    float* __restrict__ out, float mean,
                                                    float stdv, int norm) {
  __shared__ __attribute__((aligned(16))) uint8_t s_h[4][MODE == HN_RESIZE_PIL_BILINEAR ? 64 * 32 : 16];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t patch = (int64_t)blockIdx.x * 4 + w;
  if (patch >= n) return;
  float* o = out + patch * 1024;
  if (MODE == HN_RESIZE_NONE) {
    // lane owns 16 consecutive pixels
    const uint4 q = reinterpret_cast<const uint4*>(in + patch * 1024)[lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int v[4] = {byte_of(q, 4 * j), byte_of(q, 4 * j + 1), byte_of(q, 4 * j + 2), byte_of(q, 4 * j + 3)};
      store4(o + lane * 16 + 4 * j, v, mean, stdv, norm);
    }
  } else if (MODE == HN_RESIZE_CV2_LINEAR) {
    // coalesced loads: chunk i, lane l holds input row 16i + l/4, columns 16*(l&3) .. +15.
    // Rows 2y and 2y+1 sit in lanes l and l^4; each lane of the pair averages 8 of the 16
    // columns (4 outputs) with its partner's copy.
    const uint4* src = reinterpret_cast<const uint4*>(in + patch * 4096);
    const int odd = (lane >> 2) & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 q = src[i * 64 + lane];
      uint4 pq;
      pq.x = __shfl_xor(q.x, 4);
      pq.y = __shfl_xor(q.y, 4);
      pq.z = __shfl_xor(q.z, 4);
      pq.w = __shfl_xor(q.w, 4);
      // this lane's 8 columns: words (x,y) for the even-row lane, (z,w) for the odd-row lane
      const unsigned m0 = odd ? q.z : q.x, m1 = odd ? q.w : q.y;
      const unsigned p0 = odd ? pq.z : pq.x, p1 = odd ? pq.w : pq.y;
      int v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned mw = k < 2 ? m0 : m1, pw = k < 2 ? p0 : p1;
        const int sh = 16 * (k & 1);
        const int sum = (int)((mw >> sh) & 0xff) + (int)((mw >> (sh + 8)) & 0xff) +
                        (int)((pw >> sh) & 0xff) + (int)((pw >> (sh + 8)) & 0xff);
        v[k] = (sum + 2) >> 2;
      }
      const int y = i * 8 + (lane >> 3), x = 8 * (lane & 3) + 4 * odd;
      store4(o + y * 32 + x, v, mean, stdv, norm);
    }
  } else {
    // horizontal pass: lane owns input row `lane` (64 bytes, held in registers), writes its
    // 32 filtered bytes to LDS
    const uint4* src = reinterpret_cast<const uint4*>(in + patch * 4096 + lane * 64);
    const uint4 q0 = src[0], q1 = src[1], q2 = src[2], q3 = src[3];
#define PX(i) ((i) < 16 ? byte_of(q0, (i)) : (i) < 32 ? byte_of(q1, (i)-16) : (i) < 48 ? byte_of(q2, (i)-32) : byte_of(q3, (i)-48))
    unsigned packed[8];
#pragma unroll
    for (int c4 = 0; c4 < 8; ++c4) {
      unsigned wd = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = 4 * c4 + k;
        int ss = 1 << (kPB - 1);
        if (c == 0) {
          ss += PX(0) * kE1 + PX(1) * kE1 + PX(2) * kE0;
        } else if (c == 31) {
          ss += PX(61) * kE0 + PX(62) * kE1 + PX(63) * kE1;
        } else {
          ss += PX(2 * c - 1) * kK0 + PX(2 * c) * kK1 + PX(2 * c + 1) * kK1 + PX(2 * c + 2) * kK0;
        }
        wd |= (unsigned)clip8(ss) << (8 * k);
      }
      packed[c4] = wd;
    }
#undef PX
    uint4* hrow = reinterpret_cast<uint4*>(s_h[w] + lane * 32);
    hrow[0] = make_uint4(packed[0], packed[1], packed[2], packed[3]);
    hrow[1] = make_uint4(packed[4], packed[5], packed[6], packed[7]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // vertical pass: lane owns a 4x4 output block (rows 4*(lane>>3).., cols 4*(lane&7)..)
    const int x0 = 4 * (lane & 7), y0 = 4 * (lane >> 3);
    const unsigned* h = reinterpret_cast<const unsigned*>(s_h[w]);
    unsigned hr[10];  // h rows 2*y0-1 .. 2*y0+8 (clamped; unused at the borders)
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      int r = 2 * y0 - 1 + i;
      r = r < 0 ? 0 : (r > 63 ? 63 : r);
      hr[i] = h[r * 8 + (x0 >> 2)];
    }
#pragma unroll
    for (int dy = 0; dy < 4; ++dy) {
      const int y = y0 + dy;
      int v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#define HV(i) ((int)((hr[(i)] >> (8 * k)) & 0xffu))
        int ss = 1 << (kPB - 1);
        if (y == 0) {
          ss += HV(1) * kE1 + HV(2) * kE1 + HV(3) * kE0;  // h rows 0, 1, 2
        } else if (y == 31) {
          ss += HV(2 * dy) * kE0 + HV(2 * dy + 1) * kE1 + HV(2 * dy + 2) * kE1;  // rows 61..63
        } else {
          ss += HV(2 * dy) * kK0 + HV(2 * dy + 1) * kK1 + HV(2 * dy + 2) * kK1 + HV(2 * dy + 3) * kK0;
        }
#undef HV
        v[k] = clip8(ss);
      }
      store4(o + y * 32 + x0, v, mean, stdv, norm);
    }
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
