// hardnetNAS sampled-descriptor kernels (fp32, NHWC), fbnet_building_blocks/fbnet_builder.py.
//
//   k_pw       1x1 grouped conv + folded BN (+ReLU) (+residual) (ConvBNRelu pw / pwl,
//              fbnet_builder.py:352-404, 455-570); the "mid" ChannelShuffle
//              (fbnet_builder.py:332-349) is applied as a scatter on the output channel.
//   k_dw       depthwise kxk conv, stride s, pad k/2 + folded BN + ReLU (IRFBlock.dw).
//   k_maxpool  MaxPool2d(3, 2, 1) of the strided "skip" op (fbnet_builder.py:202-228).
//   k_se       SEModule (fbnet_builder.py:407-421), one workgroup per patch, in place.
//   k_nas_head Conv2d(C, 128, 4) + BN(affine=False) + y/||y|| (model_supernet.py:64-68,84).
// The whole NAS path stays in exact fp32 (it is HBM-bound).
#include "hn_common.h"
#include "hn_internal.h"

__global__ __launch_bounds__(256) void k_pw(const float* __restrict__ in, float* __restrict__ out,
                                            const float* __restrict__ wt,   // [KG][COUT]
                                            const float* __restrict__ bias, // [COUT]
                                            const float* __restrict__ res,  // [pix][COUT] or null
                                            long npix, int cin, int cout, int groups, int relu,
                                            int shuffle_g) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const int nq = cout >> 2;
  if (idx >= npix * nq) return;
  const long pix = idx / nq;
  const int n = (int)(idx % nq) * 4;
  const int kg = cin / groups, ng = cout / groups;
  const int g = n / ng;
  const float* x = in + pix * cin + g * kg;
  float4 acc = *reinterpret_cast<const float4*>(bias + n);
  for (int k = 0; k < kg; k += 4) {
    const float4 xv = *reinterpret_cast<const float4*>(x + k);
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 w = *reinterpret_cast<const float4*>(wt + (long)(k + j) * cout + n);
      acc.x = fmaf(xs[j], w.x, acc.x);
      acc.y = fmaf(xs[j], w.y, acc.y);
      acc.z = fmaf(xs[j], w.z, acc.z);
      acc.w = fmaf(xs[j], w.w, acc.w);
    }
  }
  if (relu) {
    acc.x = fmaxf(acc.x, 0.f); acc.y = fmaxf(acc.y, 0.f);
    acc.z = fmaxf(acc.z, 0.f); acc.w = fmaxf(acc.w, 0.f);
  }
  if (res) {
    const float4 rv = *reinterpret_cast<const float4*>(res + pix * cout + n);
    acc.x += rv.x; acc.y += rv.y; acc.z += rv.z; acc.w += rv.w;
  }
  float* o = out + pix * cout;
  if (shuffle_g > 1) {  // channel c = j*(C/g)+i  ->  position i*g + j
    const int cg = cout / shuffle_g;
    const float v[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = n + j;
      o[(c % cg) * shuffle_g + c / cg] = v[j];
    }
  } else {
    *reinterpret_cast<float4*>(o + n) = acc;
  }
}

template <int K>
__global__ __launch_bounds__(256) void k_dw(const float* __restrict__ in, float* __restrict__ out,
                                            const float* __restrict__ wd,  // [K*K][C]
                                            const float* __restrict__ bias, int P, int hin,
                                            int c, int s) {
  const int hout = hin / s;
  const int cq = c >> 2;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)P * hout * hout * cq) return;
  const int c4 = (int)(idx % cq) * 4;
  long t = idx / cq;
  const int xo = (int)(t % hout);
  t /= hout;
  const int yo = (int)(t % hout);
  const long p = t / hout;
  float4 acc = *reinterpret_cast<const float4*>(bias + c4);
  const float* base = in + p * hin * hin * c;
#pragma unroll
  for (int ky = 0; ky < K; ++ky) {
    const int y = yo * s - K / 2 + ky;
    if (y < 0 || y >= hin) continue;
#pragma unroll
    for (int kx = 0; kx < K; ++kx) {
      const int x = xo * s - K / 2 + kx;
      if (x < 0 || x >= hin) continue;
      const float4 v = *reinterpret_cast<const float4*>(base + ((long)y * hin + x) * c + c4);
      const float4 w = *reinterpret_cast<const float4*>(wd + (ky * K + kx) * c + c4);
      acc.x = fmaf(v.x, w.x, acc.x);
      acc.y = fmaf(v.y, w.y, acc.y);
      acc.z = fmaf(v.z, w.z, acc.z);
      acc.w = fmaf(v.w, w.w, acc.w);
    }
  }
  acc.x = fmaxf(acc.x, 0.f); acc.y = fmaxf(acc.y, 0.f);
  acc.z = fmaxf(acc.z, 0.f); acc.w = fmaxf(acc.w, 0.f);
  *reinterpret_cast<float4*>(out + (((p * hout) + yo) * (long)hout + xo) * c + c4) = acc;
}

__global__ __launch_bounds__(256) void k_maxpool(const float* __restrict__ in, float* __restrict__ out,
                                                 int P, int hin, int c) {
  const int hout = hin / 2, cq = c >> 2;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)P * hout * hout * cq) return;
  const int c4 = (int)(idx % cq) * 4;
  long t = idx / cq;
  const int xo = (int)(t % hout);
  t /= hout;
  const int yo = (int)(t % hout);
  const long p = t / hout;
  float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  const float* base = in + p * hin * hin * c;
  for (int ky = 0; ky < 3; ++ky) {
    const int y = yo * 2 - 1 + ky;
    if (y < 0 || y >= hin) continue;
    for (int kx = 0; kx < 3; ++kx) {
      const int x = xo * 2 - 1 + kx;
      if (x < 0 || x >= hin) continue;
      const float4 v = *reinterpret_cast<const float4*>(base + ((long)y * hin + x) * c + c4);
      m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y);
      m.z = fmaxf(m.z, v.z); m.w = fmaxf(m.w, v.w);
    }
  }
  *reinterpret_cast<float4*>(out + (((p * hout) + yo) * (long)hout + xo) * c + c4) = m;
}

// SE in place on y [P][hw][c]; one 256-thread workgroup per patch (c <= 256).
__global__ __launch_bounds__(256) void k_se(float* __restrict__ y, const float* __restrict__ w1,
                                            const float* __restrict__ b1,  // [mid][c], [mid]
                                            const float* __restrict__ w2,
                                            const float* __restrict__ b2,  // [c][mid], [c]
                                            int hw, int c, int mid) {
  __shared__ float avg[256], s1[256], sc[256];
  const int t = threadIdx.x;
  float* base = y + (long)blockIdx.x * hw * c;
  if (t < c) {
    float s = 0.f;
    for (int q = 0; q < hw; ++q) s += base[(long)q * c + t];
    avg[t] = s / (float)hw;
  }
  __syncthreads();
  if (t < mid) {
    float s = b1[t];
    for (int k = 0; k < c; ++k) s = fmaf(w1[t * c + k], avg[k], s);
    s1[t] = fmaxf(s, 0.f);
  }
  __syncthreads();
  if (t < c) {
    float s = b2[t];
    for (int k = 0; k < mid; ++k) s = fmaf(w2[t * mid + k], s1[k], s);
    sc[t] = 1.f / (1.f + expf(-s));
  }
  __syncthreads();
  for (long i = t; i < (long)hw * c; i += 256) base[i] *= sc[i % c];
}

// head: [P, K] x [K, 128] + bias, then y / sqrt(sum y^2 + eps).  128 threads = 4 patches.
__global__ __launch_bounds__(128) void k_nas_head(const float* __restrict__ a, float* __restrict__ out,
                                                  const float* __restrict__ wt,  // [K][128]
                                                  const float* __restrict__ bias, int P, int K,
                                                  float l2eps) {
  const int t = threadIdx.x;
  const int p = blockIdx.x * 4 + (t >> 5);
  const int n = (t & 31) * 4;
  const int pa = min(p, P - 1);
  const float* x = a + (long)pa * K;
  float4 acc = *reinterpret_cast<const float4*>(bias + n);
  for (int k = 0; k < K; k += 4) {
    const float4 xv = *reinterpret_cast<const float4*>(x + k);
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 w = *reinterpret_cast<const float4*>(wt + (long)(k + j) * 128 + n);
      acc.x = fmaf(xs[j], w.x, acc.x);
      acc.y = fmaf(xs[j], w.y, acc.y);
      acc.z = fmaf(xs[j], w.z, acc.z);
      acc.w = fmaf(xs[j], w.w, acc.w);
    }
  }
  const float ss = half_sum(acc.x * acc.x + acc.y * acc.y + acc.z * acc.z + acc.w * acc.w);
  const float norm = sqrtf(ss + l2eps);
  if (p < P) {
    float4 o = make_float4(acc.x / norm, acc.y / norm, acc.z / norm, acc.w / norm);
    *reinterpret_cast<float4*>(out + (long)p * 128 + n) = o;
  }
}

static inline unsigned blocks(long n, int per) { return (unsigned)((n + per - 1) / per); }

hipError_t hn_launch_pw(const float* in, float* out, const float* wt, const float* bias,
                        const float* res, long npix, int cin, int cout, int groups, bool relu,
                        int shuffle_g, hipStream_t st) {
  hipLaunchKernelGGL(k_pw, dim3(blocks(npix * (cout / 4), 256)), dim3(256), 0, st, in, out, wt,
                     bias, res, npix, cin, cout, groups, relu ? 1 : 0, shuffle_g);
  return hipGetLastError();
}

hipError_t hn_launch_dw(const float* in, float* out, const float* wd, const float* bias, int P,
                        int hin, int c, int k, int s, hipStream_t st) {
  const int hout = hin / s;
  const unsigned g = blocks((long)P * hout * hout * (c / 4), 256);
  if (k == 3)
    hipLaunchKernelGGL(k_dw<3>, dim3(g), dim3(256), 0, st, in, out, wd, bias, P, hin, c, s);
  else if (k == 5)
    hipLaunchKernelGGL(k_dw<5>, dim3(g), dim3(256), 0, st, in, out, wd, bias, P, hin, c, s);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t hn_launch_maxpool(const float* in, float* out, int P, int hin, int c, hipStream_t st) {
  const int hout = hin / 2;
  hipLaunchKernelGGL(k_maxpool, dim3(blocks((long)P * hout * hout * (c / 4), 256)), dim3(256), 0,
                     st, in, out, P, hin, c);
  return hipGetLastError();
}

hipError_t hn_launch_se(float* y, const float* w1, const float* b1, const float* w2,
                        const float* b2, int P, int hw, int c, int mid, hipStream_t st) {
  if (c > 256 || mid > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_se, dim3(P), dim3(256), 0, st, y, w1, b1, w2, b2, hw, c, mid);
  return hipGetLastError();
}

hipError_t hn_launch_nas_head(const float* a, float* out, const float* wt, const float* bias,
                              int P, int K, float l2eps, hipStream_t st) {
  hipLaunchKernelGGL(k_nas_head, dim3((P + 3) / 4), dim3(128), 0, st, a, out, wt, bias, P, K,
                     l2eps);
  return hipGetLastError();
}
