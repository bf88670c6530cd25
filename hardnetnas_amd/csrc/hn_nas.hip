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

#include <cstdlib>
#include <type_traits>

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
    acc.x = relu0(acc.x); acc.y = relu0(acc.y);
    acc.z = relu0(acc.z); acc.w = relu0(acc.w);
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

// LDS-tiled pointwise GEMM: one workgroup computes TM pixels x TN output channels of one
// group (K = cin/groups, chunked by 32); each thread a 4 px x 4 ch register tile, so
// TM = 4096 / TN (TN = 16/32/64 follows the group width -- no idle threads on the narrow
// grouped convs).  fp32 FMA chains, exact like the reference's fp32 conv up to summation
// order.  Also the NAS head GEMM (K = 16*C, N = 128).
constexpr int PW_TK = 32;
template <int TN>
__global__ __launch_bounds__(256) void k_pw_tiled(const float* __restrict__ in, float* __restrict__ out,
                                                  const float* __restrict__ wt,   // [KG][COUT]
                                                  const float* __restrict__ bias,
                                                  const float* __restrict__ res, long npix, int cin,
                                                  int cout, int groups, int relu, int shuffle_g) {
  constexpr int TXN = TN / 4, TM = 4096 / TN;
  __shared__ float xs[PW_TK][TM + 4];  // k-major: xs[k][pixel]
  __shared__ float ws[PW_TK][TN];
  const int t = threadIdx.x, tx = t % TXN, ty = t / TXN;
  const int kg = cin / groups, ng = cout / groups;
  const int ntn = (ng + TN - 1) / TN;
  const int g = blockIdx.y / ntn, n0 = (blockIdx.y % ntn) * TN;
  const long p0 = (long)blockIdx.x * TM;
  float acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + tx * 4 + j;
    const float bv = n < ng ? bias[g * ng + n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][j] = bv;
  }
  for (int k0 = 0; k0 < kg; k0 += PW_TK) {
    const int kc = min(PW_TK, kg - k0);
    __syncthreads();
    for (int e = t; e < TM * (PW_TK / 4); e += 256) {
      const int px = e / (PW_TK / 4), k4 = (e % (PW_TK / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p0 + px < npix && k4 < kc)
        v = *reinterpret_cast<const float4*>(in + (p0 + px) * cin + g * kg + k0 + k4);
      xs[k4 + 0][px] = v.x; xs[k4 + 1][px] = v.y; xs[k4 + 2][px] = v.z; xs[k4 + 3][px] = v.w;
    }
    for (int e = t; e < PW_TK * TXN; e += 256) {
      const int k = e / TXN, n4 = (e % TXN) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < kc && n0 + n4 < ng)
        v = *reinterpret_cast<const float4*>(wt + (long)(k0 + k) * cout + g * ng + n0 + n4);
      *reinterpret_cast<float4*>(&ws[k][n4]) = v;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < kc; ++k) {
      const float4 a = *reinterpret_cast<const float4*>(&xs[k][ty * 4]);
      const float4 b = *reinterpret_cast<const float4*>(&ws[k][tx * 4]);
      const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long px = p0 + ty * 4 + i;
    const int nl = n0 + tx * 4;
    if (px >= npix || nl >= ng) continue;
    const int n = g * ng + nl;
    float4 v = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
    if (relu) {
      v.x = relu0(v.x); v.y = relu0(v.y); v.z = relu0(v.z); v.w = relu0(v.w);
    }
    if (res) {
      const float4 rv = *reinterpret_cast<const float4*>(res + px * cout + n);
      v.x += rv.x; v.y += rv.y; v.z += rv.z; v.w += rv.w;
    }
    float* o = out + px * cout;
    if (shuffle_g > 1) {  // channel c = j*(C/g)+i  ->  position i*g + j
      const int cg = cout / shuffle_g;
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = n + j;
        o[(c % cg) * shuffle_g + c / cg] = vv[j];
      }
    } else {
      *reinterpret_cast<float4*>(o + n) = v;
    }
  }
}

// y / sqrt(sum y^2 + eps) over rows of 128 (model_supernet.py:84 has eps = 0), in place.
__global__ __launch_bounds__(256) void k_l2rows(float* __restrict__ y, int P, float l2eps) {
  const int t = threadIdx.x;
  const int p = blockIdx.x * 8 + (t >> 5);
  const int n = (t & 31) * 4;
  if (p >= P) return;
  float4 v = *reinterpret_cast<const float4*>(y + (long)p * 128 + n);
  const float ss = half_sum(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w);
  const float norm = sqrtf(ss + l2eps);
  v.x /= norm; v.y /= norm; v.z /= norm; v.w /= norm;
  *reinterpret_cast<float4*>(y + (long)p * 128 + n) = v;
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
  acc.x = relu0(acc.x); acc.y = relu0(acc.y);
  acc.z = relu0(acc.z); acc.w = relu0(acc.w);
  *reinterpret_cast<float4*>(out + (((p * hout) + yo) * (long)hout + xo) * c + c4) = acc;
}

// LDS-staged depthwise conv: one workgroup = (patch, strip of T output rows, 32-channel
// group).  The zero-padded input strip [(T-1)*S+K rows][W+K-1 cols][32 ch] fp32 and the
// tap weights are staged once; each thread then computes 4 channels of output pixels from
// LDS (ds_read_b128: for S = 1 the 16-lane groups hit 16 distinct slots).
template <int K, int S, int HIN, int T>
__global__ __launch_bounds__(256) void k_dw_lds(const float* __restrict__ in, float* __restrict__ out,
                                                const float* __restrict__ wd,  // [K*K][C]
                                                const float* __restrict__ bias, int P, int c) {
  constexpr int HOUT = HIN / S, PAD = K / 2;
  constexpr int RIN = (T - 1) * S + K, WIN = HIN + K - 1;
  constexpr int ROWB = WIN * 32;  // floats per LDS row
  __shared__ __attribute__((aligned(16))) float xs[RIN * ROWB];
  __shared__ __attribute__((aligned(16))) float ws[K * K * 32];
  const int t = threadIdx.x;
  const int ngrp = c / 32;
  const int strips = HOUT / T;
  const int bid = blockIdx.x;
  const int cg = bid % ngrp, st = (bid / ngrp) % strips;
  const long p = bid / ngrp / strips;
  const int y0 = st * T;                 // first output row
  const int iy0 = y0 * S - PAD;          // first input row of the strip
  const float* src = in + p * HIN * HIN * c + cg * 32;
  for (int e = t; e < RIN * WIN * 8; e += 256) {
    const int q = e & 7, pix = e >> 3;
    const int col = pix % WIN, row = pix / WIN;
    const int y = iy0 + row, x = col - PAD;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)y < (unsigned)HIN && (unsigned)x < (unsigned)HIN)
      v = *reinterpret_cast<const float4*>(src + ((long)y * HIN + x) * c + q * 4);
    *reinterpret_cast<float4*>(&xs[row * ROWB + col * 32 + q * 4]) = v;
  }
  for (int e = t; e < K * K * 8; e += 256) {
    const int q = e & 7, tap = e >> 3;
    *reinterpret_cast<float4*>(&ws[tap * 32 + q * 4]) =
        *reinterpret_cast<const float4*>(wd + (long)tap * c + cg * 32 + q * 4);
  }
  __syncthreads();
  const int q = t & 7;
  const float4 b = *reinterpret_cast<const float4*>(bias + cg * 32 + q * 4);
  for (int o = t >> 3; o < T * HOUT; o += 32) {
    const int yo = o / HOUT, xo = o % HOUT;
    float4 acc = b;
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const float4 v =
            *reinterpret_cast<const float4*>(&xs[(yo * S + ky) * ROWB + (xo * S + kx) * 32 + q * 4]);
        const float4 w = *reinterpret_cast<const float4*>(&ws[(ky * K + kx) * 32 + q * 4]);
        acc.x = fmaf(v.x, w.x, acc.x);
        acc.y = fmaf(v.y, w.y, acc.y);
        acc.z = fmaf(v.z, w.z, acc.z);
        acc.w = fmaf(v.w, w.w, acc.w);
      }
    acc.x = relu0(acc.x); acc.y = relu0(acc.y);
    acc.z = relu0(acc.z); acc.w = relu0(acc.w);
    *reinterpret_cast<float4*>(out + ((p * HOUT + y0 + yo) * (long)HOUT + xo) * c + cg * 32 + q * 4) = acc;
  }
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

// k_skip_s2: the "skip" op where the channel count changes (fbnet_builder.py:202-228) --
// MaxPool2d(3, 2, 1) then ConvBNRelu 1x1 CIN -> COUT -- in one pass, so the pooled tensor never
// reaches HBM.  32-pixel tiles of the flattened [P, HOUT, HOUT] output; the 4 waves of a
// workgroup cover COUT / 32 channel tiles x PT = 128 / COUT pixel tiles.  The workgroup first
// pools the PT tiles into their MFMA B fragments (K-step of 16 input channels: lane (pixel, h)
// holds channels 16 ks + 8 h .. + 7), split to fp16 hi / lo in LDS; after a barrier each wave
// runs its channel tile's 32x32x16 fp16x3 MFMA K-loop with the weights (BN folded) resident in
// registers, bias + ReLU, float4 stores.
template <int HIN, int CIN, int COUT>
__global__ __launch_bounds__(256) void k_skip_s2(const float* __restrict__ in, float* __restrict__ out,
                                                 const float* __restrict__ wt,    // [CIN][COUT]
                                                 const float* __restrict__ bias,  // [COUT]
                                                 int P) {
  constexpr int HOUT = HIN / 2, NT = COUT / 32, PT = 4 / NT, KS = CIN / 16;
  static_assert(NT * PT == 4, "4 waves");
  __shared__ uint4 s_b[PT][KS][2][64];
  // per-wave output tile, transposed for stores of 128-byte rows
  __shared__ __attribute__((aligned(16))) float s_o[4][32 * 36];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int nt = w % NT, pt = w / NT;  // this wave's MFMA work
  // A operand: row = output channel 32 nt + r, K-step ks = input channels 16 ks + 8 h + j
  f16x8 ah[KS], al[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = wt[(16 * ks + 8 * h + j) * COUT + 32 * nt + r];
      ah[ks][j] = (_Float16)v;
      al[ks][j] = (_Float16)(v - (float)ah[ks][j]);
    }
  }
  f32x16 b0;  // bias in the accumulator order (channel 8q + 4h + r' at i = 4q + r')
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 x = *reinterpret_cast<const float4*>(bias + 32 * nt + 8 * q + 4 * h);
    b0[4 * q] = x.x; b0[4 * q + 1] = x.y; b0[4 * q + 2] = x.z; b0[4 * q + 3] = x.w;
  }
  const long npix = (long)P * HOUT * HOUT;
  const long ntile = (npix + 31) / 32;
#pragma unroll 1
  for (long g = (long)blockIdx.x * PT; g < ntile; g += (long)gridDim.x * PT) {  // workgroup-uniform
    // pool the PT tiles cooperatively: item = (pixel, channel quad), consecutive threads on
    // consecutive quads of one pixel (coalesced 256-byte rows); the padding row / column -1 is
    // replaced by row / column 0, in the same window (a repeat does not change a max) -- no
    // branches, all 9 loads in flight.  The quad lands in its B-fragment slot: K-step c4 / 4,
    // lane half (c4 / 2) & 1, 8-byte half c4 & 1 of the lane's 16-byte entry.
#pragma unroll
    for (int it = t; it < 32 * PT * (CIN / 4); it += 256) {
      const int c4 = it % (CIN / 4), pxl = it / (CIN / 4), tp = pxl / 32, px = pxl % 32;
      const long op = (g + tp) * 32 + px;
      float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
      if (op < npix) {
        const long p = op / (HOUT * HOUT);
        const int rem = (int)(op % (HOUT * HOUT)), oy = rem / HOUT, ox = rem % HOUT;
        const float* base = in + p * HIN * HIN * CIN + 4 * c4;
        m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int y = max(2 * oy - 1 + ky, 0);  // (rows / columns 2 o + 1 stay inside)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int x = max(2 * ox - 1 + kx, 0);
            const float4 a = *reinterpret_cast<const float4*>(base + (y * HIN + x) * CIN);
            m.x = fmaxf(m.x, a.x); m.y = fmaxf(m.y, a.y); m.z = fmaxf(m.z, a.z); m.w = fmaxf(m.w, a.w);
          }
        }
      }
      typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
      f16x4_t hi, lo;
      hi[0] = (_Float16)m.x; lo[0] = (_Float16)(m.x - (float)hi[0]);
      hi[1] = (_Float16)m.y; lo[1] = (_Float16)(m.y - (float)hi[1]);
      hi[2] = (_Float16)m.z; lo[2] = (_Float16)(m.z - (float)hi[2]);
      hi[3] = (_Float16)m.w; lo[3] = (_Float16)(m.w - (float)hi[3]);
      const int ks = c4 >> 2, ln = ((c4 >> 1) & 1) * 32 + px, half = c4 & 1;
      reinterpret_cast<uint2*>(&s_b[tp][ks][0][ln])[half] = __builtin_bit_cast(uint2, hi);
      reinterpret_cast<uint2*>(&s_b[tp][ks][1][ln])[half] = __builtin_bit_cast(uint2, lo);
    }
    __syncthreads();
    f32x16 c = b0;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      c = mfma3_f16(ah[ks], al[ks], as_f16x8(s_b[pt][ks][0][lane]), as_f16x8(s_b[pt][ks][1][lane]), c);
    float* so = s_o[w];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(so + r * 36 + 8 * q + 4 * h) =
          make_float4(relu0(c[4 * q]), relu0(c[4 * q + 1]), relu0(c[4 * q + 2]),
                      relu0(c[4 * q + 3]));
    __builtin_amdgcn_wave_barrier();  // (one wave: its LDS accesses execute in order)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pl = 8 * k + (lane >> 3), c4 = lane & 7;
      const long op = (g + pt) * 32 + pl;
      if (op < npix)
        *reinterpret_cast<float4*>(out + op * COUT + 32 * nt + 4 * c4) =
            *reinterpret_cast<const float4*>(so + pl * 36 + 4 * c4);
    }
    __syncthreads();  // s_b is rewritten by the next tile group
  }
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
    s1[t] = relu0(s);
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
  const bool naive = hn_knobs().naive_pw;
  if (naive) {
    hipLaunchKernelGGL(k_pw, dim3(blocks(npix * (cout / 4), 256)), dim3(256), 0, st, in, out, wt,
                       bias, res, npix, cin, cout, groups, relu ? 1 : 0, shuffle_g);
  } else {
    const int ng = cout / groups;
    auto launch = [&](auto tn) {
      constexpr int TN = decltype(tn)::value, TM = 4096 / TN;
      const dim3 grid((unsigned)((npix + TM - 1) / TM), groups * ((ng + TN - 1) / TN));
      hipLaunchKernelGGL(k_pw_tiled<TN>, grid, dim3(256), 0, st, in, out, wt, bias, res, npix,
                         cin, cout, groups, relu ? 1 : 0, shuffle_g);
    };
    if (ng <= 16)
      launch(std::integral_constant<int, 16>{});
    else if (ng <= 32)
      launch(std::integral_constant<int, 32>{});
    else
      launch(std::integral_constant<int, 64>{});
  }
  return hipGetLastError();
}

template <int K, int S, int HIN, int T>
static hipError_t dw_lds(const float* in, float* out, const float* wd, const float* bias, int P,
                         int c, hipStream_t st) {
  const unsigned grid = (unsigned)P * (HIN / S / T) * (c / 32);
  hipLaunchKernelGGL((k_dw_lds<K, S, HIN, T>), dim3(grid), dim3(256), 0, st, in, out, wd, bias, P, c);
  return hipGetLastError();
}

hipError_t hn_launch_dw(const float* in, float* out, const float* wd, const float* bias, int P,
                        int hin, int c, int k, int s, hipStream_t st) {
  const int hout = hin / s;
  const bool naive = hn_knobs().naive_dw;
  if (!naive && c % 32 == 0) {
    // strips of T output rows: LDS <= ~60 KB for every SEARCH_SPACE2 shape
#define HN_DWCASE(KK, SS, HH, TT) \
  if (k == KK && s == SS && hin == HH) return dw_lds<KK, SS, HH, TT>(in, out, wd, bias, P, c, st);
    HN_DWCASE(3, 1, 32, 8) HN_DWCASE(3, 2, 32, 4) HN_DWCASE(5, 1, 32, 8) HN_DWCASE(5, 2, 32, 4)
    HN_DWCASE(3, 1, 16, 8) HN_DWCASE(3, 2, 16, 8) HN_DWCASE(5, 1, 16, 8) HN_DWCASE(5, 2, 16, 8)
    HN_DWCASE(3, 1, 8, 8) HN_DWCASE(3, 2, 8, 4) HN_DWCASE(5, 1, 8, 8) HN_DWCASE(5, 2, 8, 4)
    HN_DWCASE(3, 1, 4, 4) HN_DWCASE(5, 1, 4, 4)
#undef HN_DWCASE
  }
  const unsigned g = blocks((long)P * hout * hout * (c / 4), 256);
  if (k == 3)
    hipLaunchKernelGGL(k_dw<3>, dim3(g), dim3(256), 0, st, in, out, wd, bias, P, hin, c, s);
  else if (k == 5)
    hipLaunchKernelGGL(k_dw<5>, dim3(g), dim3(256), 0, st, in, out, wd, bias, P, hin, c, s);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <int HIN, int CIN, int COUT>
static hipError_t skip_s2_launch(const float* in, float* out, const float* wt, const float* bias, int P,
                                 hipStream_t st) {
  int resident = 0;  // persistent grid
  const hipError_t e =
      hn_resident_blocks(reinterpret_cast<const void*>(&k_skip_s2<HIN, CIN, COUT>), 256, 0, &resident);
  if (e != hipSuccess) return e;
  constexpr int PT = 4 / (COUT / 32);
  const long groups = (((long)P * (HIN / 2) * (HIN / 2) + 31) / 32 + PT - 1) / PT;
  const int grid = (int)(groups < resident ? groups : resident);
  hipLaunchKernelGGL((k_skip_s2<HIN, CIN, COUT>), dim3(grid), dim3(256), 0, st, in, out, wt, bias, P);
  return hipGetLastError();
}

bool hn_skip_s2_supported(int hin, int cin, int cout) {
  return (hin == 16 && cin == 32 && cout == 64) || (hin == 8 && cin == 64 && cout == 128);
}

hipError_t hn_launch_skip_s2(const float* in, float* out, const float* wt, const float* bias, int P, int hin,
                             int cin, int cout, hipStream_t st) {
  if (P <= 0) return hipSuccess;
  if (hin == 16 && cin == 32 && cout == 64) return skip_s2_launch<16, 32, 64>(in, out, wt, bias, P, st);
  if (hin == 8 && cin == 64 && cout == 128) return skip_s2_launch<8, 64, 128>(in, out, wt, bias, P, st);
  return hipErrorInvalidValue;
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
  // [P, K] x [K, 128] on the tiled GEMM, then the row L2 normalisation
  hipError_t e = hn_launch_pw(a, out, wt, bias, nullptr, P, K, 128, 1, false, 0, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_l2rows, dim3((P + 7) / 8), dim3(256), 0, st, out, P, l2eps);
  return hipGetLastError();
}
