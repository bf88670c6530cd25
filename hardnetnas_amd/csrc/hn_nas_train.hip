// Train-mode hardnetNAS on the GPU (second half): the forward with BatchNorm
// batch statistics (affine BN, running-statistics update) and the backward to every parameter, as
// the reference's training step runs it through autograd over
//   * the sampled descriptor (HN_KIND_NAS): model_supernet.py:53-85 with each MixedOperation
//     replaced by its arch op -- stem ConvBNRelu (fbnet_builder.py:352-404), six IRFBlock /
//     Identity layers (:455-570, :202-228; ChannelShuffle :332-349, SEModule :407-421), the 4x4
//     head conv + BatchNorm2d(affine=False) + y / ||y|| (:64-68, :84);
//   * the supernet (HN_KIND_NAS_SUPERNET): every layer runs all 17 CANDIDATE_BLOCKS on the same
//     input and outputs sum_j m_j op_j(x) (MixedOperation.forward, model_supernet.py:23-36); the
//     soft weights m (the Gumbel-softmax draw, made by the caller) come in as a device array and
//     the backward returns d loss / d m_j = <d out, op_j(x)> next to the parameter gradients.
//
// Layout and arithmetic follow hn_train.hip: activations channel-major across the batch (CNHW,
// [C][B][H][W]), so a 1x1 conv (pointwise, grouped: one GEMM per group) is one f32-MFMA GEMM over
// the whole batch (exact fp32 products; weight gradients as split-K slices summed in fp64) and a
// BatchNorm channel is one contiguous row for its statistics (fp64 partial sums).  Depthwise convs,
// max-pooling and the SE vectors are VALU kernels.  Saved between the calls: every BN's normalised
// output z and 1/sigma, and every activation a later layer or the backward reads.
#include "hn_common.h"
#include "hn_internal.h"
#include "hn_train_kernels.h"

#include <cstring>
#include <vector>

namespace {

constexpr int NOPS = 17;  // CANDIDATE_BLOCKS

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
// BatchNorm apply: y (conv output, in place) -> z = (y - mean) * rstd; a = act(gamma z + beta) [+ res].
// The channel's statistics come from k_bn_part's slice sums, combined by thread 0 of every workgroup in
// k_bn_final's order and arithmetic (so mean / rstd are k_bn_final's values); workgroup (c, 0) also
// writes rstd and the running statistics -- one launch fewer per BatchNorm than part / final / apply.
// mix (the supernet's MixedOperation, an op's last BatchNorm): also mix = (mixacc ? mix : 0) + mixc[0] a, the
// FMA k_axpy would run on the stored a, so the layer's weighted sum needs no launch of its own
HN_DEV void bna_apply_body(float* __restrict__ y, long L, const double* __restrict__ part, int NS, float eps,
                           float mom, float* __restrict__ rmean, float* __restrict__ rvar,
                           float* __restrict__ rstd_out, const float* __restrict__ gamma,
                           const float* __restrict__ beta, int relu, const float* __restrict__ res,
                           float* __restrict__ a, const float* __restrict__ mixc, float* __restrict__ mix, int mixacc,
                           int c, int by, int gy) {
  __shared__ float st[2];
  if (threadIdx.x == 0) {
    double s1 = 0.0, s2 = 0.0;
    for (int sl = 0; sl < NS; ++sl) {
      s1 += part[((long)c * NS + sl) * 2];
      s2 += part[((long)c * NS + sl) * 2 + 1];
    }
    const double mean = s1 / (double)L;
    const double var = fmax(s2 / (double)L - mean * mean, 0.0);
    st[0] = (float)mean;
    st[1] = (float)(1.0 / sqrt(var + (double)eps));
    if (by == 0) {
      rstd_out[c] = st[1];
      if (rmean) {
        rmean[c] = (1.f - mom) * rmean[c] + mom * (float)mean;
        rvar[c] = (1.f - mom) * rvar[c] + mom * (float)(L > 1 ? var * (double)L / (double)(L - 1) : var);
      }
    }
  }
  __syncthreads();
  const float mu = st[0], rs = st[1], g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  const float mc = mix ? *mixc : 0.f;
  const long base = (long)c * L, step = (long)gy * 256;
  for (long i = (long)by * 256 + threadIdx.x; i < L; i += step) {
    const float z = (y[base + i] - mu) * rs;
    y[base + i] = z;
    if (a) {
      float v = fmaf(g, z, b);
      if (relu) v = fmaxf(v, 0.f);
      if (res) v += res[base + i];
      a[base + i] = v;
      if (mix) mix[base + i] = mixacc ? fmaf(mc, v, mix[base + i]) : mc * v;
    }
  }
}
__global__ __launch_bounds__(256) void k_bna_apply(float* __restrict__ y, long L, const double* __restrict__ part,
                                                   int NS, float eps, float mom, float* __restrict__ rmean,
                                                   float* __restrict__ rvar, float* __restrict__ rstd_out,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   int relu, const float* __restrict__ res, float* __restrict__ a,
                                                   const float* __restrict__ mixc, float* __restrict__ mix,
                                                   int mixacc) {
  bna_apply_body(y, L, part, NS, eps, mom, rmean, rvar, rstd_out, gamma, beta, relu, res, a, mixc, mix, mixacc,
                 blockIdx.x, blockIdx.y, gridDim.y);
}

// The supernet's BatchNorms of one layer phase (every IRF op's pw BN, or every dw BN: one row length L) in one
// k_bn_part and one apply launch: entry q owns global channels c0 .. c0 + C - 1 and its own slice count and
// partial-sum region, and runs the single-BatchNorm bodies (bn_part_body, bna_apply_body) unchanged -- the
// same statistics and outputs bit for bit
constexpr int kBnMulti = 17;
struct BnEntry {
  float* y;
  float* a;
  float* rstd;
  const float* gamma;
  const float* beta;
  float* rm;
  float* rv;
  long p0;  // first double of its partial sums
  int C, NS, c0;
};
struct BnMulti {
  BnEntry e[kBnMulti];
  int n;
};
HN_DEV int bn_entry(const BnMulti& t, int gc) {
  int q = 0;
  while (q + 1 < t.n && t.e[q + 1].c0 <= gc) ++q;
  return q;
}
__global__ __launch_bounds__(256) void k_bn_part_multi(BnMulti t, long L, double* __restrict__ part) {
  const BnEntry& E = t.e[bn_entry(t, blockIdx.x)];
  if ((int)blockIdx.y >= E.NS) return;  // workgroup-uniform
  bn_part_body(E.y, L, E.NS, part + E.p0, (int)blockIdx.x - E.c0, blockIdx.y);
}
__global__ __launch_bounds__(256) void k_bna_apply_multi(BnMulti t, long L, const double* __restrict__ part, float eps,
                                                         float mom, int relu) {
  const BnEntry& E = t.e[bn_entry(t, blockIdx.x)];
  bna_apply_body(E.y, L, part + E.p0, E.NS, eps, mom, E.rm, E.rv, E.rstd, E.gamma, E.beta, relu, nullptr, E.a,
                 nullptr, nullptr, 0, (int)blockIdx.x - E.c0, blockIdx.y, gridDim.y);
}

// backward through [ReLU o] affine BN(train): g = da [* (gamma z + beta > 0)]; slice sums of g and g z
__global__ __launch_bounds__(256) void k_bna_bwd_part(const float* __restrict__ da, const float* __restrict__ z, long L,
                                                      int NS, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int relu,
                                                      double* __restrict__ part) {
  __shared__ double sh[8];
  const int c = blockIdx.x, sl = blockIdx.y;
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  const long per = (L + NS - 1) / NS, b = sl * per, e = min(L, b + per), base = (long)c * L;
  double s1 = 0.0, s2 = 0.0;
  for (long i = b + threadIdx.x; i < e; i += 256) {
    const float zv = z[base + i];
    float v = da[base + i];
    if (relu && fmaf(gm, zv, bt) <= 0.f) v = 0.f;
    s1 += v;
    s2 += (double)v * zv;
  }
  block_sum2(s1, s2, sh);
  if (threadIdx.x == 0) {
    part[((long)c * NS + sl) * 2] = s1;
    part[((long)c * NS + sl) * 2 + 1] = s2;
  }
}

// dy = rstd * (gamma g - m1 - z m2); dy may alias da.  m1 / m2 from k_bna_bwd_part's slice sums, combined
// by thread 0 of every workgroup in k_bna_bwd_final's order; workgroup (c, 0) writes d gamma / d beta
__global__ __launch_bounds__(256) void k_bna_bwd_apply(const float* da, const float* __restrict__ z, long L,
                                                       const double* __restrict__ part, int NS,
                                                       float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                       const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       int relu, float* dy) {
  __shared__ float st[2];
  const int c = blockIdx.x;
  if (threadIdx.x == 0) {
    double s1 = 0.0, s2 = 0.0;
    for (int sl = 0; sl < NS; ++sl) {
      s1 += part[((long)c * NS + sl) * 2];
      s2 += part[((long)c * NS + sl) * 2 + 1];
    }
    if (blockIdx.y == 0) {
      if (dgamma) dgamma[c] = (float)s2;
      if (dbeta) dbeta[c] = (float)s1;
    }
    const double g0 = gamma ? (double)gamma[c] : 1.0;
    st[0] = (float)(g0 * s1 / (double)L);
    st[1] = (float)(g0 * s2 / (double)L);
  }
  __syncthreads();
  const float m1 = st[0], m2 = st[1], rs = rstd[c];
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  const long base = (long)c * L, step = (long)gridDim.y * 256;
  for (long i = (long)blockIdx.y * 256 + threadIdx.x; i < L; i += step) {
    const float zv = z[base + i];
    float v = da[base + i];
    if (relu && fmaf(gm, zv, bt) <= 0.f) v = 0.f;
    dy[base + i] = rs * (gm * v - m1 - zv * m2);
  }
}

// depthwise KxK conv, stride S, pad K/2 (fbnet_builder.py:455-570 "dw"), over CNHW; channel c of the
// output reads input row src(c) -- the ChannelShuffle of the pw output folded in (g = pw groups; 1: none)
HN_DEV int shuffle_src(int c, int C, int g) { return g > 1 ? (c % g) * (C / g) + c / g : c; }

template <int K, int S>
__global__ __launch_bounds__(256) void k_dw_fwd(const float* __restrict__ a, int C, int g, long B, int H,
                                                const float* __restrict__ w, float* __restrict__ y) {
  constexpr int P = K / 2;
  const int HO = H / S;
  const long total = (long)C * B * HO * HO;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ox = (int)(e % HO), oy = (int)((e / HO) % HO);
    const long cb = e / ((long)HO * HO);
    const int c = (int)(cb / B);
    const long b = cb % B;
    const float* src = a + ((long)shuffle_src(c, C, g) * B + b) * H * H;
    const float* wc = w + c * K * K;
    float s = 0.f;
#pragma unroll
    for (int dy = 0; dy < K; ++dy) {
      const int iy = oy * S - P + dy;
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        const int ix = ox * S - P + dx;
        if (ix >= 0 && ix < H) s = fmaf(wc[dy * K + dx], src[iy * H + ix], s);
      }
    }
    y[e] = s;
  }
}

// k_dw_fwd of several ops of one layer with the same kernel size (blockIdx.y = op): the same per-output sum
struct DwEntry {
  const float* a;
  const float* w;
  float* y;
  int C, g;
};
struct DwMulti {
  DwEntry e[NOPS];
  int n;
};
template <int K, int S>
__global__ __launch_bounds__(256) void k_dw_fwd_multi(DwMulti t, long B, int H) {
  constexpr int P = K / 2;
  const DwEntry& E = t.e[blockIdx.y];
  const int HO = H / S;
  const long total = (long)E.C * B * HO * HO;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ox = (int)(e % HO), oy = (int)((e / HO) % HO);
    const long cb = e / ((long)HO * HO);
    const int c = (int)(cb / B);
    const long b = cb % B;
    const float* src = E.a + ((long)shuffle_src(c, E.C, E.g) * B + b) * H * H;
    const float* wc = E.w + c * K * K;
    float s = 0.f;
#pragma unroll
    for (int dy = 0; dy < K; ++dy) {
      const int iy = oy * S - P + dy;
      if (iy < 0 || iy >= H) continue;
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        const int ix = ox * S - P + dx;
        if (ix >= 0 && ix < H) s = fmaf(wc[dy * K + dx], src[iy * H + ix], s);
      }
    }
    E.y[e] = s;
  }
}

// data gradient: input pixel (iy, ix) of row src(c) collects the taps that landed on it
template <int K, int S>
__global__ __launch_bounds__(256) void k_dw_dgrad(const float* __restrict__ dy, int C, int g, long B, int H,
                                                  const float* __restrict__ w, float* __restrict__ da) {
  constexpr int P = K / 2;
  const int HO = H / S;
  const long total = (long)C * B * H * H;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ix = (int)(e % H), iy = (int)((e / H) % H);
    const long cb = e / ((long)H * H);
    const int c = (int)(cb / B);
    const long b = cb % B;
    const float* d = dy + cb * HO * HO;
    const float* wc = w + c * K * K;
    float s = 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int ty = iy + P - ky;
      if (ty < 0 || ty % S) continue;
      const int oy = ty / S;
      if (oy >= HO) continue;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int tx = ix + P - kx;
        if (tx < 0 || tx % S) continue;
        const int ox = tx / S;
        if (ox < HO) s = fmaf(wc[ky * K + kx], d[oy * HO + ox], s);
      }
    }
    da[((long)shuffle_src(c, C, g) * B + b) * H * H + iy * H + ix] = s;
  }
}

// weight gradient: dW[c][tap] = sum over (b, oy, ox) of dy . a_src(c)[tap-shifted]; grid (C, NS),
// per-thread fp32 sums over its elements of the slice, fp64 across threads and slices
template <int K, int S>
__global__ __launch_bounds__(256) void k_dw_wgrad_part(const float* __restrict__ dy, const float* __restrict__ a, int C,
                                                       int g, long B, int H, int NS, double* __restrict__ part) {
  constexpr int P = K / 2, KK = K * K;
  __shared__ double sh[4][KK];
  const int HO = H / S, c = blockIdx.x, sl = blockIdx.y;
  const long n = B * HO * HO, per = (n + NS - 1) / NS, b0 = sl * per, e0 = min(n, b0 + per);
  const float* src = a + (long)shuffle_src(c, C, g) * B * H * H;
  const float* d = dy + (long)c * n;
  float acc[KK];
#pragma unroll
  for (int t = 0; t < KK; ++t) acc[t] = 0.f;
  for (long e = b0 + threadIdx.x; e < e0; e += 256) {
    const int ox = (int)(e % HO), oy = (int)((e / HO) % HO);
    const long b = e / ((long)HO * HO);
    const float dv = d[e];
    const float* ab = src + b * H * H;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy * S - P + ky;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int ix = ox * S - P + kx;
        if (iy >= 0 && iy < H && ix >= 0 && ix < H) acc[ky * K + kx] = fmaf(dv, ab[iy * H + ix], acc[ky * K + kx]);
      }
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < KK; ++t) {
    double v = acc[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) sh[wv][t] = v;
  }
  __syncthreads();
  if (threadIdx.x < KK) {
    const int t = threadIdx.x;
    part[((long)c * NS + sl) * KK + t] = sh[0][t] + sh[1][t] + sh[2][t] + sh[3][t];
  }
}

__global__ __launch_bounds__(256) void k_dw_wgrad_final(const double* __restrict__ part, int C, int NS, int KK,
                                                        float* __restrict__ dw) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= C * KK) return;
  const int c = e / KK, t = e % KK;
  double s = 0.0;
  for (int sl = 0; sl < NS; ++sl) s += part[((long)c * NS + sl) * KK + t];
  dw[e] = (float)s;
}

// MaxPool2d(3, 2, 1) over CNHW rows of H x H ("skip" at stride 2, fbnet_builder.py:202-228); the
// backward routes each window's gradient to its first strict maximum in row-major order, as ATen's
// CPU max_pool2d (the reference) does
__global__ __launch_bounds__(256) void k_maxpool_fwd(const float* __restrict__ x, long CB, int H, float* __restrict__ y) {
  const int HO = H / 2;
  const long total = CB * HO * HO;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ox = (int)(e % HO), oy = (int)((e / HO) % HO);
    const float* r = x + (e / ((long)HO * HO)) * H * H;
    float m = -INFINITY;
    for (int dy = 0; dy < 3; ++dy) {
      const int iy = 2 * oy - 1 + dy;
      if (iy < 0 || iy >= H) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int ix = 2 * ox - 1 + dx;
        if (ix >= 0 && ix < H) m = fmaxf(m, r[iy * H + ix]);
      }
    }
    y[e] = m;
  }
}

__global__ __launch_bounds__(256) void k_maxpool_bwd(const float* __restrict__ dy, const float* __restrict__ x, long CB,
                                                     int H, float* __restrict__ dx) {
  const int HO = H / 2;
  const long total = CB * H * H;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ix = (int)(e % H), iy = (int)((e / H) % H);
    const long cb = e / ((long)H * H);
    const float* r = x + cb * H * H;
    float s = 0.f;
    for (int oy = max(0, iy / 2); oy <= min(HO - 1, (iy + 1) / 2); ++oy)
      for (int ox = max(0, ix / 2); ox <= min(HO - 1, (ix + 1) / 2); ++ox) {
        float m = -INFINITY;
        int am = -1;
        for (int ky = 0; ky < 3; ++ky) {
          const int yy = 2 * oy - 1 + ky;
          if (yy < 0 || yy >= H) continue;
          for (int kx = 0; kx < 3; ++kx) {
            const int xx = 2 * ox - 1 + kx;
            if (xx < 0 || xx >= H) continue;
            const float v = r[yy * H + xx];
            if (v > m || am < 0) {
              m = v;
              am = yy * H + xx;
            }
          }
        }
        if (am == iy * H + ix) s += dy[cb * HO * HO + oy * HO + ox];
      }
    dx[e] += s;
  }
}

// the stride-2 1x1 convs of the FDLNet fronts read every other pixel: y [R][H/2][H/2] = x[R][2i][2j]
// (CNHW rows R = C x B); the backward scatters back with zeros in between
__global__ __launch_bounds__(256) void k_sub2(const float* __restrict__ x, long R, int H, float* __restrict__ y) {
  const int HO = H / 2;
  const long total = R * HO * HO;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ox = (int)(e % HO), oy = (int)((e / HO) % HO);
    y[e] = x[(e / ((long)HO * HO)) * H * H + 2 * oy * H + 2 * ox];
  }
}
__global__ __launch_bounds__(256) void k_unsub2(const float* __restrict__ dy, long R, int H, float* __restrict__ dx) {
  const int HO = H / 2;
  const long total = R * H * H;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ix = (int)(e % H), iy = (int)((e / H) % H);
    dx[e] = ((ix | iy) & 1) ? 0.f : dy[(e / ((long)H * H)) * HO * HO + (iy / 2) * HO + ix / 2];
  }
}

// y = (acc ? y : 0) + c x, c = coef ? *coef : 1
__global__ __launch_bounds__(256) void k_axpy(long n, const float* __restrict__ coef, const float* __restrict__ x,
                                              float* __restrict__ y, int acc) {
  const float c = coef ? *coef : 1.f;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256)
    y[e] = acc ? fmaf(c, x[e], y[e]) : c * x[e];
}

// <a, b_j> over n elements for the NOPS ops j of a supernet layer (blockIdx.y = j): per-workgroup fp64
// partials, then one fixed-order sum per op
struct DotSrc {
  const float* b[NOPS];
};
__global__ __launch_bounds__(256) void k_dot_part(const float* __restrict__ a, DotSrc src, long n,
                                                  double* __restrict__ part) {
  __shared__ double sh[8];
  const float* __restrict__ b = src.b[blockIdx.y];
  double s = 0.0, z = 0.0;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) s += (double)a[e] * b[e];
  block_sum2(s, z, sh);
  if (threadIdx.x == 0) part[(long)blockIdx.y * gridDim.x + blockIdx.x] = s;
}
// one wave per op: lane l sums partials l, l + 64, ... in order, then a fixed butterfly over the 64 lanes
__global__ __launch_bounds__(64) void k_dot_final(const double* __restrict__ part, int n, float* __restrict__ out) {
  const double* p = part + (long)blockIdx.x * n;
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 64) s += p[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (threadIdx.x == 0) out[blockIdx.x] = (float)s;
}

// The supernet's 1x1 convs of one layer phase (every IRF op's pw, or every op's pwl, each group of a grouped
// conv a problem) in one launch: problem q is pw_fwd's GEMM C [M][N] = A [M][K] . B [K][N] (row strides K, N,
// N), workgroup t takes tile t - tile0[q] of problem q, and gemm_tile runs the exact k_gemm tile -- so each
// output equals the separate launch's bit for bit.  One launch per tile height (BM 32 for M <= 32, else 64,
// gemm()'s choice).
constexpr int kPwBatch = 40;
struct PwProb {
  const float* A;
  const float* B;
  float* C;
  int M, K;
};
struct PwBatch {
  PwProb p[kPwBatch];
  int tile0[kPwBatch + 1];
  int n;
  long N;
};
template <int BM>
__global__ __launch_bounds__(256) void k_gemm_pw_batch(PwBatch b) {
  const int t = (int)blockIdx.x;
  int q = 0;
  while (q + 1 < b.n && b.tile0[q + 1] <= t) ++q;
  const PwProb& pr = b.p[q];
  const long nt = (b.N + GBN - 1) / GBN, lt = t - b.tile0[q];
  const GemmArgs g{pr.A, pr.B, pr.C, pr.M, b.N, pr.K, pr.K, 1, b.N, 1, b.N, 1, 1.f, 0.f};
  gemm_tile<BM>(g, StridedB{}, (lt / nt) * BM, (lt % nt) * GBN, 0, pr.K, 0, nullptr);
}

// SEModule (fbnet_builder.py:407-421): out = x * sigmoid(W2 relu(W1 avgpool(x) + b1) + b2)
// one wave per (channel, patch) row: lanes stride the HW contiguous values (coalesced), then a butterfly
// (one thread per row walking it serially read 4-byte pieces HW floats apart across the wave)
__global__ __launch_bounds__(256) void k_se_pool(const float* __restrict__ x, long CB, int HW, float* __restrict__ pooled) {
  const int lane = threadIdx.x & 63;
  for (long cb = ((long)blockIdx.x * 256 + threadIdx.x) >> 6; cb < CB; cb += (long)gridDim.x * 4) {
    const float* r = x + cb * HW;
    float s = 0.f;
    for (int i = lane; i < HW; i += 64) s += r[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) pooled[cb] = s / (float)HW;
  }
}
// v[r][j] = act(v[r][j] + bias[r]): act 1 = ReLU, 2 = sigmoid
__global__ __launch_bounds__(256) void k_bias_act(float* __restrict__ v, int R, long N, const float* __restrict__ bias,
                                                  int act) {
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < (long)R * N; e += (long)gridDim.x * 256) {
    float t = v[e] + bias[e / N];
    if (act == 1) t = fmaxf(t, 0.f);
    if (act == 2) t = 1.f / (1.f + expf(-t));
    v[e] = t;
  }
}
__global__ __launch_bounds__(256) void k_se_scale(const float* __restrict__ x, const float* __restrict__ s, long CB,
                                                  int HW, float* __restrict__ out) {
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < CB * HW; e += (long)gridDim.x * 256) out[e] = x[e] * s[e / HW];
}
// dq[cb] = (sum_hw dO x) s (1 - s)   (the gradient at the sigmoid's input)
// (one wave per row, as k_se_pool)
__global__ __launch_bounds__(256) void k_se_bwd_ds(const float* __restrict__ dO, const float* __restrict__ x,
                                                   const float* __restrict__ s, long CB, int HW, float* __restrict__ dq) {
  const int lane = threadIdx.x & 63;
  for (long cb = ((long)blockIdx.x * 256 + threadIdx.x) >> 6; cb < CB; cb += (long)gridDim.x * 4) {
    float acc = 0.f;
    for (int i = lane; i < HW; i += 64) acc = fmaf(dO[cb * HW + i], x[cb * HW + i], acc);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) {
      const float sv = s[cb];
      dq[cb] = acc * sv * (1.f - sv);
    }
  }
}
__global__ __launch_bounds__(256) void k_relu_mask(float* __restrict__ d, const float* __restrict__ h, long n) {
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256)
    if (!(h[e] > 0.f)) d[e] = 0.f;
}
// dx = dO s + dpooled / HW
__global__ __launch_bounds__(256) void k_se_bwd_dx(const float* __restrict__ dO, const float* __restrict__ s,
                                                   const float* __restrict__ dpooled, long CB, int HW,
                                                   float* __restrict__ dx) {
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < CB * HW; e += (long)gridDim.x * 256)
    dx[e] = fmaf(dO[e], s[e / HW], dpooled[e / HW] / (float)HW);
}
// out[r] = sum_j x[r][j] (fp64), one workgroup per row
__global__ __launch_bounds__(256) void k_rowsum(const float* __restrict__ x, long N, float* __restrict__ out) {
  __shared__ double sh[8];
  const float* r = x + (long)blockIdx.x * N;
  double s = 0.0, z = 0.0;
  for (long j = threadIdx.x; j < N; j += 256) s += r[j];
  block_sum2(s, z, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = (float)s;
}

// the 4x4 head conv (model_supernet.py:64-68) as a GEMM over the CNHW [C][B][16] layer output:
// column k = c * 16 + yx of patch j
struct HeadB {  // forward: B(k, j = patch)
  const float* x;
  long B;
  HN_DEV float at(const GemmArgs&, long k, long j) const { return x[(k >> 4) * B * 16 + j * 16 + (k & 15)]; }
};
struct HeadBT {  // weight gradient: B(k = patch, j = column)
  const float* x;
  long B;
  HN_DEV float at(const GemmArgs&, long k, long j) const { return x[(j >> 4) * B * 16 + k * 16 + (j & 15)]; }
};
// dcol [K = C * 16][B] -> dX [C][B][16]
__global__ __launch_bounds__(256) void k_head_scatter(const float* __restrict__ dcol, int C, long B,
                                                      float* __restrict__ dx) {
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < (long)C * B * 16; e += (long)gridDim.x * 256) {
    const int yx = (int)(e & 15);
    const long cb = e >> 4, b = cb % B;
    const int c = (int)(cb / B);
    dx[e] = dcol[((long)c * 16 + yx) * B + b];
  }
}

// every kernel launched on grid_of(n) walks its n elements in a grid-stride loop (the grid is capped)
unsigned grid_of(long n) { return (unsigned)std::max<long>(1, std::min<long>((n + 255) / 256, 65536)); }

#define HCK(x)                        \
  do {                                \
    hipError_t e_ = (x);              \
    if (e_ != hipSuccess) return e_;  \
  } while (0)

// split-K slices gemm() uses for a weight gradient (the same rule, hn_train_kernels.h)
long gemm_slices(long M, long N, long K) {
  const int bm = M <= 32 ? 32 : 64;
  const long tiles = ((N + GBN - 1) / GBN) * ((M + bm - 1) / bm);
  long ks = hn_knobs().train_splitk;
  if (tiles < 256 && K > 64) {
    const long want = std::min<long>((256 + tiles - 1) / tiles, (K + 63) / 64);
    ks = std::min(ks, ((K + want - 1) / want + GBK - 1) / GBK * GBK);
  }
  return K > ks ? (K + ks - 1) / ks : 1;
}

// ------------------------------------------------------------------------------------------
// the network plan: every op of every layer, its tensors (indices into the caller's pointer
// array, in state_dict order) and its saved buffers (offsets into the saved region)
// ------------------------------------------------------------------------------------------
enum OpKind { IRF = 0, SKIP_ID = 1, SKIP_MP = 2, SKIP_MPCONV = 3, SKIP_CONV = 4 };

struct OpPlan {
  int op = 0, kind = IRF;
  int cin = 0, cout = 0, s = 1, hin = 0, hout = 0, mid = 0, k = 3, g = 1, se = 0, semid = 0, res = 0;
  // tensor indices (-1: none); a BN index points at its weight (bias, running_mean, running_var follow)
  int pw_w = -1, pw_bn = -1, dw_w = -1, dw_bn = -1, pwl_w = -1, pwl_bn = -1;
  int se_w1 = -1, se_b1 = -1, se_w2 = -1, se_b2 = -1, sk_w = -1, sk_bn = -1;
  // saved offsets (bytes)
  size_t z1 = 0, r1 = 0, a1 = 0, z2 = 0, r2 = 0, a2 = 0, z3 = 0, r3 = 0, o3 = 0, out = 0;
  size_t pooled = 0, hh = 0, sg = 0, mp = 0;
  bool out_is_input = false;
};

struct LayerPlan {
  int cin = 0, cout = 0, s = 1, hin = 0, hout = 0;
  std::vector<OpPlan> ops;
  size_t sum = 0;  // supernet: saved sum_j m_j out_j
};

struct Plan {
  long B = 0;
  bool super = false;
  int fdl = 0;  // FDLNet HardNetNeiMask front: 1 NASNet, 2 NASNet_0.1 (0: the NAS stem)
  float in_eps = 0.f;
  int nt = 0;  // tensors consumed
  std::vector<int> gw;  // tensor slots whose gradient the backward always writes (every conv / SE weight and bias)
  int stem_w = -1, stem_bn = -1, head_w = -1, head_rm = -1;
  size_t x0z = 0, x0r = 0, x0a = 0;    // stem (FDL: conv0 output + bias; NASNet: its BN's z, in place)
  // FDL front: input_norm; NASNet: BN(affine=False) -> 1x1 s2 32->32 BN ReLU -> 1x1 s2 32->64 BN ReLU;
  // NASNet_0.1: MaxPool(3, 2, 1) -> 1x1 s2 32->64 BN ReLU (FDLIdentity)
  int stem_b = -1, f_bn0 = -1, f_w1 = -1, f_bn1 = -1, f_w2 = -1, f_bn2 = -1;
  size_t xn = 0, xsd = 0, f_xs1 = 0, f_z1 = 0, f_r1 = 0, f_a1 = 0, f_mp = 0, f_xs2 = 0, f_z2 = 0, f_r2 = 0, f_a2 = 0;
  size_t hz = 0, hr = 0;               // head
  std::vector<LayerPlan> layers;
  size_t saved = 0;
  // scratch
  size_t maxact = 0;  // floats
  size_t g0 = 0, g1 = 0, t0 = 0, t1 = 0, t2 = 0, part = 0, bnpart = 0, dwpart = 0,
         se0 = 0, se1 = 0, se2 = 0, hcol = 0, dotpart = 0, scratch = 0;
  size_t part_floats = 0;
};

constexpr int kDotParts = 512;

Plan make_plan(const hn_arch_desc& d, long B) {
  Plan P;
  P.B = B;
  P.super = d.kind == HN_KIND_NAS_SUPERNET;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) / 256 * 256;
    return o;
  };
  auto act = [&](int c, int hw) { return (size_t)c * B * hw * hw * sizeof(float); };
  size_t maxact = (size_t)32 * B * 1024, part = 0;
  auto wg = [&](long M, long N, long K) { part = std::max(part, (size_t)(M * N * gemm_slices(M, N, K))); };
  int nt = 0;
  auto bn = [&]() { const int t = nt; nt += 4; return t; };
  auto wt = [&]() { P.gw.push_back(nt); return nt++; };  // a weight slot: its gradient pointer must be valid
  P.fdl = d.kind == HN_KIND_FDL_NASNET ? 1 : d.kind == HN_KIND_FDL_NASNET01 ? 2 : 0;
  int hw = 32;
  if (P.fdl) {
    // FDLNet fronts (des.py), in state_dict order: features.0.{weight, bias}, then
    //   NASNet    : features.1.{running_mean, running_var}, .2.weight, .3.{w, b, rm, rv}, .5.weight, .6.{...}
    //   NASNet_0.1: features.3.conv.conv.weight, features.3.conv.bn.{...}
    P.in_eps = d.input_norm_eps;
    P.xn = take((size_t)B * 1024 * sizeof(float));
    P.xsd = take((size_t)B * sizeof(float));
    P.stem_w = wt();
    P.stem_b = wt();
    P.x0z = take(act(32, 32));
    if (P.fdl == 1) {
      P.f_bn0 = nt;
      nt += 2;
      P.x0r = take(32 * sizeof(float));
      P.f_xs1 = take(act(32, 16));
      P.f_w1 = wt();
      P.f_bn1 = bn();
      P.f_z1 = take(act(32, 16));
      P.f_r1 = take(32 * sizeof(float));
      P.f_a1 = take(act(32, 16));
      wg(32, 32, B * 256);
    } else {
      P.f_mp = take(act(32, 16));
    }
    P.f_xs2 = take(act(32, 8));
    P.f_w2 = wt();
    P.f_bn2 = bn();
    P.f_z2 = take(act(64, 8));
    P.f_r2 = take(64 * sizeof(float));
    P.f_a2 = take(act(64, 8));
    wg(64, 32, B * 64);
    hw = 8;
  } else {
    // stem ConvBNRelu(1 -> 32, 3x3): conv.weight, bn.{weight, bias, running_mean, running_var}
    P.stem_w = wt();
    P.stem_bn = bn();
    P.x0z = take(act(32, 32));
    P.x0r = take(32 * sizeof(float));
    P.x0a = take(act(32, 32));
  }
  for (int i = 0; i < d.n_layers; ++i) {
    LayerPlan L;
    L.cin = d.c_in[i];
    L.cout = d.c_out[i];
    L.s = d.stride[i];
    L.hin = hw;
    L.hout = hw / L.s;
    const int nops = P.super ? NOPS : 1;
    for (int j = 0; j < nops; ++j) {
      OpPlan o;
      o.op = P.super ? j : d.op[i];
      const HnOpSpec& sp = kHnOps[o.op];
      o.cin = L.cin, o.cout = L.cout, o.s = L.s, o.hin = L.hin, o.hout = L.hout;
      const int Li = L.hin, Lo = L.hout;
      if (sp.skip) {
        if (o.cin == o.cout) {
          o.kind = o.s == 1 ? SKIP_ID : SKIP_MP;
          if (o.kind == SKIP_ID) o.out_is_input = true;
          else o.out = take(act(o.cout, Lo));
        } else {
          o.kind = o.s == 1 ? SKIP_CONV : SKIP_MPCONV;
          o.sk_w = wt();
          o.sk_bn = bn();
          if (o.kind == SKIP_MPCONV) o.mp = take(act(o.cin, Lo));
          o.z1 = take(act(o.cout, Lo));
          o.r1 = take(o.cout * sizeof(float));
          o.out = take(act(o.cout, Lo));
          wg(o.cout, o.cin, B * Lo * Lo);
          maxact = std::max(maxact, (size_t)o.cout * B * Lo * Lo);
        }
      } else {
        o.kind = IRF;
        o.k = sp.k;
        o.g = sp.g;
        o.se = sp.se;
        o.mid = o.cin * sp.e;
        o.res = o.s == 1 && o.cin == o.cout;
        o.pw_w = wt();
        o.pw_bn = bn();
        o.dw_w = wt();
        o.dw_bn = bn();
        o.pwl_w = wt();
        o.pwl_bn = bn();
        o.z1 = take(act(o.mid, Li));
        o.r1 = take(o.mid * sizeof(float));
        o.a1 = take(act(o.mid, Li));
        o.z2 = take(act(o.mid, Lo));
        o.r2 = take(o.mid * sizeof(float));
        o.a2 = take(act(o.mid, Lo));
        o.z3 = take(act(o.cout, Lo));
        o.r3 = take(o.cout * sizeof(float));
        o.o3 = take(act(o.cout, Lo));
        if (o.se) {
          o.semid = o.cout / 4 > 8 ? o.cout / 4 : 8;
          o.se_w1 = wt();
          o.se_b1 = wt();
          o.se_w2 = wt();
          o.se_b2 = wt();
          o.pooled = take((size_t)o.cout * B * sizeof(float));
          o.hh = take((size_t)o.semid * B * sizeof(float));
          o.sg = take((size_t)o.cout * B * sizeof(float));
          o.out = take(act(o.cout, Lo));
          wg(o.cout, o.semid, B);
          wg(o.semid, o.cout, B);
        } else {
          o.out = o.o3;
        }
        wg(o.mid / o.g, o.cin / o.g, B * Li * Li);
        wg(o.cout / o.g, o.mid / o.g, B * Lo * Lo);
        maxact = std::max({maxact, (size_t)o.mid * B * Li * Li, (size_t)o.cout * B * Lo * Lo});
      }
      maxact = std::max({maxact, (size_t)o.cin * B * Li * Li, (size_t)o.cout * B * Lo * Lo});
      L.ops.push_back(o);
    }
    if (P.super) L.sum = take(act(L.cout, L.hout));
    P.layers.push_back(L);
    hw = L.hout;
  }
  // head: conv_k1.weight [128][C][4][4], batchnorm.{running_mean, running_var}
  const int cl = d.c_out[d.n_layers - 1];
  P.head_w = wt();
  P.head_rm = nt;
  nt += 2;
  P.hz = take((size_t)128 * B * sizeof(float));
  P.hr = take(128 * sizeof(float));
  wg(128, (long)cl * 16, B);
  P.nt = nt;
  P.saved = off;
  // scratch
  off = 0;
  P.maxact = maxact;
  P.g0 = take(maxact * 4);
  P.g1 = take(maxact * 4);
  P.t0 = take(maxact * 4);
  P.t1 = take(maxact * 4);
  P.t2 = take(maxact * 4);
  part = std::max(part, (size_t)32 * 9 * wgrad0_slices(B));
  P.part_floats = part;
  P.part = take(part * 4);
  // (one BatchNorm of up to 512 channels, or a layer phase of the supernet's: NS <= ceil(2048 / C) per channel)
  P.bnpart = take(std::max<size_t>((size_t)512 * kBnSlices, (size_t)NOPS * (2048 + 512)) * 2 * sizeof(double));
  P.dwpart = take((size_t)512 * kBnSlices * 25 * sizeof(double));
  P.se0 = take((size_t)512 * B * sizeof(float));
  P.se1 = take((size_t)512 * B * sizeof(float));
  P.se2 = take((size_t)512 * B * sizeof(float));
  P.hcol = take((size_t)cl * 16 * B * sizeof(float));
  P.dotpart = take((size_t)NOPS * kDotParts * sizeof(double));
  P.scratch = off;
  return P;
}

// ------------------------------------------------------------------------------------------
// host building blocks
// ------------------------------------------------------------------------------------------
struct Ctx {
  const Plan& P;
  float* const* T;  // caller's tensors (state_dict order)
  float* const* G;  // gradients (nullptr entries: buffers)
  char* sv;
  char* sc;
  hipStream_t st;
  float mom;
  float* f(size_t off) const { return reinterpret_cast<float*>(sv + off); }
  float* s(size_t off) const { return reinterpret_cast<float*>(sc + off); }
};

// train-mode BN over [C][L] (y in place -> z), rstd saved; a = act(gamma z + beta) [+ res]
hipError_t bn_fwd(const Ctx& c, float* y, int C, long L, int bnt, bool affine, bool relu, const float* res, float* a,
                  float* rstd, const float* mixc = nullptr, float* mix = nullptr, bool mixacc = false) {
  const int NS = bn_slices(C, L);
  double* part = reinterpret_cast<double*>(c.sc + c.P.bnpart);
  hipLaunchKernelGGL(k_bn_part, dim3(C, NS), dim3(256), 0, c.st, y, L, NS, part);
  float* rm = c.T[affine ? bnt + 2 : bnt];
  float* rv = c.T[affine ? bnt + 3 : bnt + 1];
  hipLaunchKernelGGL(k_bna_apply, bn_row_grid(C, L), dim3(256), 0, c.st, y, L, part, NS, 1e-5f, c.mom, rm, rv, rstd,
                     affine ? c.T[bnt] : nullptr, affine ? c.T[bnt + 1] : nullptr, relu ? 1 : 0, res, a, mixc, mix,
                     mixacc ? 1 : 0);
  return hipGetLastError();
}

// train-mode affine BN + ReLU over several (y [C][L] -> z in place, a) of one row length, two launches
struct BnBatcher {
  const Ctx& c;
  long L;
  BnMulti t{};
  int channels = 0, rows = 1;
  long doubles = 0;
  void add(float* y, int C, int bnt, float* a, float* rstd) {
    BnEntry& E = t.e[t.n++];
    E = BnEntry{y, a, rstd, c.T[bnt], c.T[bnt + 1], c.T[bnt + 2], c.T[bnt + 3], doubles, C, bn_slices(C, L), channels};
    channels += C;
    doubles += (long)C * E.NS * 2;
    rows = std::max(rows, (int)bn_row_grid(C, L).y);
  }
  hipError_t run() {
    if (!t.n) return hipSuccess;
    int ns = 1;
    for (int q = 0; q < t.n; ++q) ns = std::max(ns, t.e[q].NS);
    double* part = reinterpret_cast<double*>(c.sc + c.P.bnpart);
    hipLaunchKernelGGL(k_bn_part_multi, dim3((unsigned)channels, (unsigned)ns), dim3(256), 0, c.st, t, L, part);
    hipLaunchKernelGGL(k_bna_apply_multi, dim3((unsigned)channels, (unsigned)rows), dim3(256), 0, c.st, t, L, part,
                       1e-5f, c.mom, 1);
    return hipGetLastError();
  }
};

// backward through [ReLU o] BN: da -> dy (may alias), d gamma / d beta written
hipError_t bn_bwd(const Ctx& c, const float* da, const float* z, const float* rstd, int C, long L, int bnt, bool affine,
                  bool relu, float* dy) {
  const int NS = bn_slices(C, L);
  double* part = reinterpret_cast<double*>(c.sc + c.P.bnpart);
  const float* gm = affine ? c.T[bnt] : nullptr;
  const float* bt = affine ? c.T[bnt + 1] : nullptr;
  hipLaunchKernelGGL(k_bna_bwd_part, dim3(C, NS), dim3(256), 0, c.st, da, z, L, NS, gm, bt, relu ? 1 : 0, part);
  hipLaunchKernelGGL(k_bna_bwd_apply, bn_row_grid(C, L), dim3(256), 0, c.st, da, z, L, part, NS,
                     affine ? c.G[bnt] : nullptr, affine ? c.G[bnt + 1] : nullptr, rstd, gm, bt, relu ? 1 : 0, dy);
  return hipGetLastError();
}

// 1x1 conv with `g` groups over CNHW rows of L: y [cout][L] = W [cout][cin/g] . x (per group)
hipError_t pw_fwd(const Ctx& c, const float* w, int cout, int cin, int g, const float* x, long L, float* y) {
  const int cog = cout / g, cig = cin / g;
  for (int gi = 0; gi < g; ++gi) {
    GemmArgs a{w + (long)gi * cog * cig, x + (long)gi * cig * L, y + (long)gi * cog * L, cog, L, cig, cig, 1, L, 1,
               L, 1, 1.f, 0.f};
    HCK(gemm(a, c.st));
  }
  return hipSuccess;
}
hipError_t pw_wgrad(const Ctx& c, const float* dy, const float* x, int cout, int cin, int g, long L, float* dw) {
  const int cog = cout / g, cig = cin / g;
  for (int gi = 0; gi < g; ++gi) {
    GemmArgs a{dy + (long)gi * cog * L, x + (long)gi * cig * L, dw + (long)gi * cog * cig, cog, cig, L, L, 1, 1, L,
               cig, 1, 1.f, 0.f};
    HCK(gemm(a, c.st, c.s(c.P.part)));
  }
  return hipSuccess;
}
// dx [cin][L] (+)= W^T . dy
hipError_t pw_dgrad(const Ctx& c, const float* w, const float* dy, int cout, int cin, int g, long L, float* dx,
                    bool acc) {
  const int cog = cout / g, cig = cin / g;
  for (int gi = 0; gi < g; ++gi) {
    GemmArgs a{w + (long)gi * cog * cig, dy + (long)gi * cog * L, dx + (long)gi * cig * L, cig, L, cog, 1, cig, L,
               1, L, 1, 1.f, acc ? 1.f : 0.f};
    HCK(gemm(a, c.st));
  }
  return hipSuccess;
}

// pw_fwd's per-group GEMMs of several ops gathered, then launched as k_gemm_pw_batch (<= 2 launches per flush)
struct PwBatcher {
  const Ctx& c;
  long N;
  std::vector<PwProb> small, big;  // M <= 32 / M > 32
  void add(const float* w, int cout, int cin, int g, const float* x, float* y) {
    const int cog = cout / g, cig = cin / g;
    for (int gi = 0; gi < g; ++gi) {
      const PwProb p{w + (long)gi * cog * cig, x + (long)gi * cig * N, y + (long)gi * cog * N, cog, cig};
      (cog <= 32 ? small : big).push_back(p);
    }
  }
  template <int BM>
  hipError_t launch(const std::vector<PwProb>& v) {
    for (size_t q0 = 0; q0 < v.size(); q0 += kPwBatch) {
      PwBatch b{};
      b.N = N;
      b.n = (int)std::min<size_t>(kPwBatch, v.size() - q0);
      const long nt = (N + GBN - 1) / GBN;
      int tiles = 0;
      for (int q = 0; q < b.n; ++q) {
        b.p[q] = v[q0 + q];
        b.tile0[q] = tiles;
        tiles += (int)(nt * ((b.p[q].M + BM - 1) / BM));
      }
      b.tile0[b.n] = tiles;
      hipLaunchKernelGGL((k_gemm_pw_batch<BM>), dim3((unsigned)tiles), dim3(256), 0, c.st, b);
      HCK(hipGetLastError());
    }
    return hipSuccess;
  }
  hipError_t flush() {
    HCK(launch<32>(small));
    HCK(launch<64>(big));
    small.clear();
    big.clear();
    return hipSuccess;
  }
};

hipError_t dw_fwd(const Ctx& c, const OpPlan& o, const float* a, float* y) {
  const long n = (long)o.mid * c.P.B * o.hout * o.hout;
  const float* w = c.T[o.dw_w];
#define HN_DW(KK, SS) \
  if (o.k == KK && o.s == SS) hipLaunchKernelGGL((k_dw_fwd<KK, SS>), dim3(grid_of(n)), dim3(256), 0, c.st, a, o.mid, o.g, c.P.B, o.hin, w, y);
  HN_DW(3, 1) HN_DW(3, 2) HN_DW(5, 1) HN_DW(5, 2)
#undef HN_DW
  return hipGetLastError();
}
hipError_t dw_bwd(const Ctx& c, const OpPlan& o, const float* dy, const float* a, float* da) {
  const long n = (long)o.mid * c.P.B * o.hin * o.hin, no = c.P.B * o.hout * o.hout;
  const float* w = c.T[o.dw_w];
  const int NS = bn_slices(o.mid, no), KK = o.k * o.k;
  double* part = reinterpret_cast<double*>(c.sc + c.P.dwpart);
#define HN_DW(KK_, SS)                                                                                            \
  if (o.k == KK_ && o.s == SS) {                                                                                  \
    hipLaunchKernelGGL((k_dw_dgrad<KK_, SS>), dim3(grid_of(n)), dim3(256), 0, c.st, dy, o.mid, o.g, c.P.B, o.hin, \
                       w, da);                                                                                    \
    hipLaunchKernelGGL((k_dw_wgrad_part<KK_, SS>), dim3(o.mid, NS), dim3(256), 0, c.st, dy, a, o.mid, o.g, c.P.B, \
                       o.hin, NS, part);                                                                          \
  }
  HN_DW(3, 1) HN_DW(3, 2) HN_DW(5, 1) HN_DW(5, 2)
#undef HN_DW
  hipLaunchKernelGGL(k_dw_wgrad_final, dim3((o.mid * KK + 255) / 256), dim3(256), 0, c.st, part, o.mid, NS, KK,
                     c.G[o.dw_w]);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// forward / backward of one op (x: the layer input [cin][B][hin^2])
// ------------------------------------------------------------------------------------------
// mixc / mix / mixacc (the supernet): an IRF op without SE adds mixc[0] x its output into mix inside its last
// BatchNorm and sets *mixed; the caller mixes the other ops' outputs itself
// stages (IRF ops; the supernet runs its pw / pwl GEMMs batched across ops in between): 1 the pw GEMM, 2 its
// BatchNorm + the dw + its BatchNorm, 4 the pwl GEMM, 8 the pwl BatchNorm [+ SE] (the op's output)
constexpr int kOpAll = 15;
hipError_t op_fwd(const Ctx& c, OpPlan& o, const float* x, const float** out, const float* mixc = nullptr,
                  float* mix = nullptr, bool mixacc = false, bool* mixed = nullptr, int stages = kOpAll) {
  if (mixed) *mixed = false;
  const long B = c.P.B, Li = B * o.hin * o.hin, Lo = B * o.hout * o.hout;
  switch (o.kind) {
    case SKIP_ID:
      *out = x;
      return hipSuccess;
    case SKIP_MP:
      hipLaunchKernelGGL(k_maxpool_fwd, dim3(grid_of((long)o.cin * Lo)), dim3(256), 0, c.st, x, (long)o.cin * B, o.hin,
                         c.f(o.out));
      *out = c.f(o.out);
      return hipGetLastError();
    case SKIP_MPCONV:
    case SKIP_CONV: {
      const float* in = x;
      if (o.kind == SKIP_MPCONV) {
        hipLaunchKernelGGL(k_maxpool_fwd, dim3(grid_of((long)o.cin * Lo)), dim3(256), 0, c.st, x, (long)o.cin * B,
                           o.hin, c.f(o.mp));
        in = c.f(o.mp);
      }
      HCK(pw_fwd(c, c.T[o.sk_w], o.cout, o.cin, 1, in, Lo, c.f(o.z1)));
      HCK(bn_fwd(c, c.f(o.z1), o.cout, Lo, o.sk_bn, true, true, nullptr, c.f(o.out), c.f(o.r1)));
      *out = c.f(o.out);
      return hipSuccess;
    }
  }
  // IRFBlock: pw (+BN+ReLU) -> [shuffle] -> dw (+BN+ReLU) -> pwl (+BN) [+ x] [-> SE]
  if (stages & 1) HCK(pw_fwd(c, c.T[o.pw_w], o.mid, o.cin, o.g, x, Li, c.f(o.z1)));
  if (stages & 2) {
    HCK(bn_fwd(c, c.f(o.z1), o.mid, Li, o.pw_bn, true, true, nullptr, c.f(o.a1), c.f(o.r1)));
    HCK(dw_fwd(c, o, c.f(o.a1), c.f(o.z2)));
    HCK(bn_fwd(c, c.f(o.z2), o.mid, Lo, o.dw_bn, true, true, nullptr, c.f(o.a2), c.f(o.r2)));
  }
  if (stages & 4) HCK(pw_fwd(c, c.T[o.pwl_w], o.cout, o.mid, o.g, c.f(o.a2), Lo, c.f(o.z3)));
  if (!(stages & 8)) return hipSuccess;
  const bool mx = mix && !o.se;
  HCK(bn_fwd(c, c.f(o.z3), o.cout, Lo, o.pwl_bn, true, false, o.res ? x : nullptr, c.f(o.o3), c.f(o.r3),
             mx ? mixc : nullptr, mx ? mix : nullptr, mixacc));
  if (mx) *mixed = true;
  if (o.se) {
    const long CB = (long)o.cout * B;
    const int HW = o.hout * o.hout;
    float* pooled = c.f(o.pooled);
    hipLaunchKernelGGL(k_se_pool, dim3(grid_of(CB * 64)), dim3(256), 0, c.st, c.f(o.o3), CB, HW, pooled);
    GemmArgs a1{c.T[o.se_w1], pooled, c.f(o.hh), o.semid, B, o.cout, o.cout, 1, B, 1, B, 1, 1.f, 0.f};
    HCK(gemm(a1, c.st));
    hipLaunchKernelGGL(k_bias_act, dim3(grid_of((long)o.semid * B)), dim3(256), 0, c.st, c.f(o.hh), o.semid, B,
                       c.T[o.se_b1], 1);
    GemmArgs a2{c.T[o.se_w2], c.f(o.hh), c.f(o.sg), o.cout, B, o.semid, o.semid, 1, B, 1, B, 1, 1.f, 0.f};
    HCK(gemm(a2, c.st));
    hipLaunchKernelGGL(k_bias_act, dim3(grid_of(CB)), dim3(256), 0, c.st, c.f(o.sg), o.cout, B, c.T[o.se_b2], 2);
    hipLaunchKernelGGL(k_se_scale, dim3(grid_of(CB * HW)), dim3(256), 0, c.st, c.f(o.o3), c.f(o.sg), CB, HW,
                       c.f(o.out));
  }
  *out = c.f(o.out);
  return hipGetLastError();
}

// dO: the gradient of this op's output (may be overwritten); dX accumulates the input gradient
hipError_t op_bwd(const Ctx& c, const OpPlan& o, const float* x, float* dO, float* dX) {
  const long B = c.P.B, Li = B * o.hin * o.hin, Lo = B * o.hout * o.hout;
  float* t1 = c.s(c.P.t1);
  float* t2 = c.s(c.P.t2);
  switch (o.kind) {
    case SKIP_ID:
      hipLaunchKernelGGL(k_axpy, dim3(grid_of((long)o.cin * Li)), dim3(256), 0, c.st, (long)o.cin * Li, nullptr, dO,
                         dX, 1);
      return hipGetLastError();
    case SKIP_MP:
      hipLaunchKernelGGL(k_maxpool_bwd, dim3(grid_of((long)o.cin * Li)), dim3(256), 0, c.st, dO, x, (long)o.cin * B,
                         o.hin, dX);
      return hipGetLastError();
    case SKIP_MPCONV:
    case SKIP_CONV: {
      const float* in = o.kind == SKIP_MPCONV ? c.f(o.mp) : x;
      HCK(bn_bwd(c, dO, c.f(o.z1), c.f(o.r1), o.cout, Lo, o.sk_bn, true, true, t1));
      HCK(pw_wgrad(c, t1, in, o.cout, o.cin, 1, Lo, c.G[o.sk_w]));
      if (o.kind == SKIP_CONV) return pw_dgrad(c, c.T[o.sk_w], t1, o.cout, o.cin, 1, Lo, dX, true);
      HCK(pw_dgrad(c, c.T[o.sk_w], t1, o.cout, o.cin, 1, Lo, t2, false));
      hipLaunchKernelGGL(k_maxpool_bwd, dim3(grid_of((long)o.cin * Li)), dim3(256), 0, c.st, t2, x, (long)o.cin * B,
                         o.hin, dX);
      return hipGetLastError();
    }
  }
  float* dO3 = dO;
  if (o.se) {
    const long CB = (long)o.cout * B;
    const int HW = o.hout * o.hout;
    float* dq = c.s(c.P.se0);
    float* dh = c.s(c.P.se1);
    float* dp = c.s(c.P.se2);
    float* part = c.s(c.P.part);
    hipLaunchKernelGGL(k_se_bwd_ds, dim3(grid_of(CB * 64)), dim3(256), 0, c.st, dO, c.f(o.o3), c.f(o.sg), CB, HW, dq);
    GemmArgs w2{dq, c.f(o.hh), c.G[o.se_w2], o.cout, o.semid, B, B, 1, 1, B, o.semid, 1, 1.f, 0.f};  // dW2 = dq h^T
    HCK(gemm(w2, c.st, part));
    hipLaunchKernelGGL(k_rowsum, dim3(o.cout), dim3(256), 0, c.st, dq, B, c.G[o.se_b2]);
    GemmArgs h2{c.T[o.se_w2], dq, dh, o.semid, B, o.cout, 1, o.semid, B, 1, B, 1, 1.f, 0.f};  // dh = W2^T dq
    HCK(gemm(h2, c.st));
    hipLaunchKernelGGL(k_relu_mask, dim3(grid_of((long)o.semid * B)), dim3(256), 0, c.st, dh, c.f(o.hh),
                       (long)o.semid * B);
    GemmArgs w1{dh, c.f(o.pooled), c.G[o.se_w1], o.semid, o.cout, B, B, 1, 1, B, o.cout, 1, 1.f, 0.f};
    HCK(gemm(w1, c.st, part));
    hipLaunchKernelGGL(k_rowsum, dim3(o.semid), dim3(256), 0, c.st, dh, B, c.G[o.se_b1]);
    GemmArgs p1{c.T[o.se_w1], dh, dp, o.cout, B, o.semid, 1, o.cout, B, 1, B, 1, 1.f, 0.f};  // dpooled = W1^T dh
    HCK(gemm(p1, c.st));
    hipLaunchKernelGGL(k_se_bwd_dx, dim3(grid_of(CB * HW)), dim3(256), 0, c.st, dO, c.f(o.sg), dp, CB, HW, t1);
    dO3 = t1;
  }
  // buffers: dO3 (dO, or t1 after SE) -> dy3 in t2 -> da2 in dO -> dy2 in t2 -> da1 in dO -> dy1 in t2
  if (o.res)
    hipLaunchKernelGGL(k_axpy, dim3(grid_of((long)o.cout * Lo)), dim3(256), 0, c.st, (long)o.cout * Lo, nullptr, dO3,
                       dX, 1);
  HCK(bn_bwd(c, dO3, c.f(o.z3), c.f(o.r3), o.cout, Lo, o.pwl_bn, true, false, t2));  // pwl BN (no ReLU)
  HCK(pw_wgrad(c, t2, c.f(o.a2), o.cout, o.mid, o.g, Lo, c.G[o.pwl_w]));
  HCK(pw_dgrad(c, c.T[o.pwl_w], t2, o.cout, o.mid, o.g, Lo, dO, false));
  HCK(bn_bwd(c, dO, c.f(o.z2), c.f(o.r2), o.mid, Lo, o.dw_bn, true, true, t2));  // dw BN + ReLU
  HCK(dw_bwd(c, o, t2, c.f(o.a1), dO));
  HCK(bn_bwd(c, dO, c.f(o.z1), c.f(o.r1), o.mid, Li, o.pw_bn, true, true, t2));  // pw BN + ReLU
  HCK(pw_wgrad(c, t2, x, o.mid, o.cin, o.g, Li, c.G[o.pw_w]));
  return pw_dgrad(c, c.T[o.pw_w], t2, o.mid, o.cin, o.g, Li, dX, true);
}

// ------------------------------------------------------------------------------------------
// whole network
// ------------------------------------------------------------------------------------------
// FDLNet front (des.py:8-55 / NASNet_0.1 des.py:10-55) -> the first block's input [64][B][8][8]
hipError_t fdl_front_fwd(Ctx& c, Plan& P, const float* in) {
  const long B = P.B;
  // input_norm (des.py:40-47, mean / std detached), conv0 3x3 (k_fwd0) + its bias
  hipLaunchKernelGGL(k_input_norm, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, c.st, in, B, P.in_eps, c.f(P.xn),
                     c.f(P.xsd));
  hipLaunchKernelGGL(k_fwd0, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, c.st, c.f(P.xn), c.T[P.stem_w], B,
                     c.f(P.x0z));
  hipLaunchKernelGGL(k_bias_act, dim3(grid_of(32 * B * 1024)), dim3(256), 0, c.st, c.f(P.x0z), 32, B * 1024,
                     c.T[P.stem_b], 0);
  HCK(hipGetLastError());
  const float* s2in;  // the input of the stride-2 1x1 conv to 64 channels, [32][B][16][16]
  if (P.fdl == 1) {
    // BatchNorm2d(32, affine=False), no ReLU: z in place is the next input
    HCK(bn_fwd(c, c.f(P.x0z), 32, B * 1024, P.f_bn0, false, false, nullptr, nullptr, c.f(P.x0r)));
    hipLaunchKernelGGL(k_sub2, dim3(grid_of(32 * B * 256)), dim3(256), 0, c.st, c.f(P.x0z), 32 * B, 32, c.f(P.f_xs1));
    HCK(pw_fwd(c, c.T[P.f_w1], 32, 32, 1, c.f(P.f_xs1), B * 256, c.f(P.f_z1)));
    HCK(bn_fwd(c, c.f(P.f_z1), 32, B * 256, P.f_bn1, true, true, nullptr, c.f(P.f_a1), c.f(P.f_r1)));
    s2in = c.f(P.f_a1);
  } else {
    hipLaunchKernelGGL(k_maxpool_fwd, dim3(grid_of(32 * B * 256)), dim3(256), 0, c.st, c.f(P.x0z), 32 * B, 32,
                       c.f(P.f_mp));
    s2in = c.f(P.f_mp);  // FDLIdentity(32, 32, 1): nothing
  }
  hipLaunchKernelGGL(k_sub2, dim3(grid_of(32 * B * 64)), dim3(256), 0, c.st, s2in, 32 * B, 16, c.f(P.f_xs2));
  HCK(pw_fwd(c, c.T[P.f_w2], 64, 32, 1, c.f(P.f_xs2), B * 64, c.f(P.f_z2)));
  return bn_fwd(c, c.f(P.f_z2), 64, B * 64, P.f_bn2, true, true, nullptr, c.f(P.f_a2), c.f(P.f_r2));
}

// the input of the first searched layer
const float* first_input(const Ctx& c, const Plan& P) { return P.fdl ? c.f(P.f_a2) : c.f(P.x0a); }

hipError_t nas_fwd(Ctx& c, Plan& P, const float* in, const float* soft, float* out) {
  const long B = P.B;
  if (P.fdl) {
    HCK(fdl_front_fwd(c, P, in));
  } else {
    // stem: conv (k_fwd0 on the raw 32x32 patches, taps as the MFMA's K) -> BN -> ReLU
    hipLaunchKernelGGL(k_fwd0, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, c.st, in, c.T[P.stem_w], B, c.f(P.x0z));
    HCK(hipGetLastError());
    HCK(bn_fwd(c, c.f(P.x0z), 32, B * 1024, P.stem_bn, true, true, nullptr, c.f(P.x0a), c.f(P.x0r)));
  }
  const float* x = first_input(c, P);
  for (size_t i = 0; i < P.layers.size(); ++i) {
    LayerPlan& L = P.layers[i];
    if (!P.super) {
      HCK(op_fwd(c, L.ops[0], x, &x));
      continue;
    }
    const long n = (long)L.cout * B * L.hout * L.hout;
    // every IRF op's pw GEMMs in one batched launch per tile height, then each op's BatchNorm / dw / BatchNorm,
    // then every pwl GEMM batched, then each op's output in op order with the weighted sum
    // (MixedOperation: sum_j m_j op_j(x), model_supernet.py:23-36)
    PwBatcher pw{c, B * L.hin * L.hin, {}, {}}, pwl{c, B * L.hout * L.hout, {}, {}};
    for (int j = 0; j < NOPS; ++j) {
      OpPlan& o = L.ops[j];
      if (o.kind == IRF) pw.add(c.T[o.pw_w], o.mid, o.cin, o.g, x, c.f(o.z1));
    }
    HCK(pw.flush());
    // the pw BatchNorms of every op, the dw of each, the dw BatchNorms of every op (op_fwd stage 2, batched)
    BnBatcher b1{c, B * L.hin * L.hin}, b2{c, B * L.hout * L.hout};
    for (int j = 0; j < NOPS; ++j) {
      OpPlan& o = L.ops[j];
      if (o.kind != IRF) continue;
      b1.add(c.f(o.z1), o.mid, o.pw_bn, c.f(o.a1), c.f(o.r1));
      b2.add(c.f(o.z2), o.mid, o.dw_bn, c.f(o.a2), c.f(o.r2));
      pwl.add(c.T[o.pwl_w], o.cout, o.mid, o.g, c.f(o.a2), c.f(o.z3));
    }
    HCK(b1.run());
    {  // every op's dw, one launch per kernel size
      DwMulti d3{}, d5{};
      long n3 = 0, n5 = 0;
      for (int j = 0; j < NOPS; ++j) {
        const OpPlan& o = L.ops[j];
        if (o.kind != IRF) continue;
        DwMulti& d = o.k == 3 ? d3 : d5;
        d.e[d.n++] = DwEntry{c.f(o.a1), c.T[o.dw_w], c.f(o.z2), o.mid, o.g};
        (o.k == 3 ? n3 : n5) = std::max(o.k == 3 ? n3 : n5, (long)o.mid * B * L.hout * L.hout);
      }
#define HN_DWM(KK, SS, D, N)                                                                                       \
  if (D.n && L.s == SS)                                                                                            \
    hipLaunchKernelGGL((k_dw_fwd_multi<KK, SS>), dim3(grid_of(N), (unsigned)D.n), dim3(256), 0, c.st, D, B, L.hin);
      HN_DWM(3, 1, d3, n3) HN_DWM(3, 2, d3, n3) HN_DWM(5, 1, d5, n5) HN_DWM(5, 2, d5, n5)
#undef HN_DWM
      HCK(hipGetLastError());
    }
    HCK(b2.run());
    HCK(pwl.flush());
    for (int j = 0; j < NOPS; ++j) {
      const float* oj = nullptr;
      bool mixed = false;
      HCK(op_fwd(c, L.ops[j], x, &oj, soft + i * NOPS + j, c.f(L.sum), j > 0, &mixed, L.ops[j].kind == IRF ? 8 : kOpAll));
      if (!mixed)
        hipLaunchKernelGGL(k_axpy, dim3(grid_of(n)), dim3(256), 0, c.st, n, soft + i * NOPS + j, oj, c.f(L.sum),
                           j > 0 ? 1 : 0);
    }
    x = c.f(L.sum);
  }
  // head: 4x4 conv (GEMM, K = C x 16) -> BatchNorm2d(affine=False) -> y / ||y||
  const int cl = P.layers.back().cout;
  GemmArgs h{c.T[P.head_w], nullptr, c.f(P.hz), 128, B, (long)cl * 16, (long)cl * 16, 1, 0, 0, B, 1, 1.f, 0.f};
  HCK(gemm(h, c.st, nullptr, HeadB{x, B}));
  HCK(bn_fwd(c, c.f(P.hz), 128, B, P.head_rm, false, false, nullptr, nullptr, c.f(P.hr)));
  hipLaunchKernelGGL(k_l2_fwd, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, c.st, c.f(P.hz), B, 0.f, out);
  return hipGetLastError();
}

hipError_t nas_bwd(Ctx& c, Plan& P, const float* in, const float* soft, const float* dout, float* dsoft) {
  const long B = P.B;
  float* g = c.s(P.g0);   // gradient of the current layer's output
  float* gx = c.s(P.g1);  // gradient of its input
  // head: L2 -> BN(affine=False) -> conv (dW = dY col^T; d col = W^T dY, scattered to CNHW)
  float* dz = c.s(P.se0);
  hipLaunchKernelGGL(k_l2_bwd, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, c.st, c.f(P.hz), dout, B, 0.f, dz);
  HCK(hipGetLastError());
  HCK(bn_bwd(c, dz, c.f(P.hz), c.f(P.hr), 128, B, P.head_rm, false, false, dz));
  const int cl = P.layers.back().cout;
  const long K = (long)cl * 16;
  const float* xl = P.super ? c.f(P.layers.back().sum) : nullptr;
  if (!P.super) {  // the sampled net's last layer output: its op's out (or its input, for an identity)
    const float* x = first_input(c, P);
    for (size_t i = 0; i + 1 < P.layers.size(); ++i) {
      const OpPlan& o = P.layers[i].ops[0];
      x = o.out_is_input ? x : c.f(o.out);
    }
    const OpPlan& o = P.layers.back().ops[0];
    xl = o.out_is_input ? x : c.f(o.out);
  }
  GemmArgs wh{dz, nullptr, c.G[P.head_w], 128, K, B, B, 1, 0, 1, K, 1, 1.f, 0.f};
  HCK(gemm(wh, c.st, c.s(P.part), HeadBT{xl, B}));
  GemmArgs dh{c.T[P.head_w], dz, c.s(P.hcol), K, B, 128, 1, K, B, 1, B, 1, 1.f, 0.f};
  HCK(gemm(dh, c.st));
  hipLaunchKernelGGL(k_head_scatter, dim3(grid_of(K * B)), dim3(256), 0, c.st, c.s(P.hcol), cl, B, g);
  HCK(hipGetLastError());
  // layer inputs, front to back
  std::vector<const float*> xin(P.layers.size());
  {
    const float* x = first_input(c, P);
    for (size_t i = 0; i < P.layers.size(); ++i) {
      xin[i] = x;
      if (P.super) x = c.f(P.layers[i].sum);
      else x = P.layers[i].ops[0].out_is_input ? x : c.f(P.layers[i].ops[0].out);
    }
  }
  for (int i = (int)P.layers.size() - 1; i >= 0; --i) {
    const LayerPlan& L = P.layers[i];
    const long nin = (long)L.cin * B * L.hin * L.hin, nout = (long)L.cout * B * L.hout * L.hout;
    HCK(hipMemsetAsync(gx, 0, nin * sizeof(float), c.st));
    if (!P.super) {
      HCK(op_bwd(c, L.ops[0], xin[i], g, gx));
    } else {
      float* dOj = c.s(P.t0);
      double* dp = reinterpret_cast<double*>(c.sc + P.dotpart);
      // d m_j = <d out, op_j(x)> for all 17 ops at once (g is not written by the op backwards below)
      DotSrc ds;
      for (int j = 0; j < NOPS; ++j) ds.b[j] = L.ops[j].out_is_input ? xin[i] : c.f(L.ops[j].out);
      const unsigned np = std::min<unsigned>(kDotParts, grid_of(nout));
      hipLaunchKernelGGL(k_dot_part, dim3(np, NOPS), dim3(256), 0, c.st, g, ds, nout, dp);
      hipLaunchKernelGGL(k_dot_final, dim3(NOPS), dim3(64), 0, c.st, dp, (int)np, dsoft + i * NOPS);
      for (int j = 0; j < NOPS; ++j) {
        hipLaunchKernelGGL(k_axpy, dim3(grid_of(nout)), dim3(256), 0, c.st, nout, soft + i * NOPS + j, g, dOj, 0);
        HCK(op_bwd(c, L.ops[j], xin[i], dOj, gx));
      }
    }
    std::swap(g, gx);
  }
  const float* x0 = in;  // conv0's input
  if (P.fdl) {
    // g = d front output [64][B][8][8]: ReLU o BN -> 1x1 s2 conv (weight grad; data grad scattered)
    float* t1 = c.s(P.t1);
    float* t2 = c.s(P.t2);
    HCK(bn_bwd(c, g, c.f(P.f_z2), c.f(P.f_r2), 64, B * 64, P.f_bn2, true, true, t1));
    HCK(pw_wgrad(c, t1, c.f(P.f_xs2), 64, 32, 1, B * 64, c.G[P.f_w2]));
    HCK(pw_dgrad(c, c.T[P.f_w2], t1, 64, 32, 1, B * 64, t2, false));
    hipLaunchKernelGGL(k_unsub2, dim3(grid_of(32 * B * 256)), dim3(256), 0, c.st, t2, 32 * B, 16, t1);  // [32][B][256]
    if (P.fdl == 1) {
      HCK(bn_bwd(c, t1, c.f(P.f_z1), c.f(P.f_r1), 32, B * 256, P.f_bn1, true, true, t2));
      HCK(pw_wgrad(c, t2, c.f(P.f_xs1), 32, 32, 1, B * 256, c.G[P.f_w1]));
      HCK(pw_dgrad(c, c.T[P.f_w1], t2, 32, 32, 1, B * 256, t1, false));
      hipLaunchKernelGGL(k_unsub2, dim3(grid_of(32 * B * 1024)), dim3(256), 0, c.st, t1, 32 * B, 32, g);
      HCK(bn_bwd(c, g, c.f(P.x0z), c.f(P.x0r), 32, B * 1024, P.f_bn0, false, false, gx));  // BN(affine=False)
    } else {
      HCK(hipMemsetAsync(gx, 0, (size_t)32 * B * 1024 * sizeof(float), c.st));
      hipLaunchKernelGGL(k_maxpool_bwd, dim3(grid_of(32 * B * 1024)), dim3(256), 0, c.st, t1, c.f(P.x0z), 32 * B, 32,
                         gx);
    }
    hipLaunchKernelGGL(k_rowsum, dim3(32), dim3(256), 0, c.st, gx, B * 1024, c.G[P.stem_b]);  // conv0 bias
    HCK(hipGetLastError());
    x0 = c.f(P.xn);
  } else {
    // stem: ReLU o BN -> conv weight gradient (k_wgrad0; the input gradient is not formed)
    HCK(bn_bwd(c, g, c.f(P.x0z), c.f(P.x0r), 32, B * 1024, P.stem_bn, true, true, gx));
  }
  const long ns = wgrad0_slices(B);
  hipLaunchKernelGGL(k_wgrad0, dim3((unsigned)(ns / 4)), dim3(256), 0, c.st, x0, gx, B, c.s(P.part));
  HCK(hipGetLastError());
  GemmArgs gs{nullptr, nullptr, c.G[P.stem_w], 32, 9, 0, 0, 0, 0, 0, 9, 1, 1.f, 0.f};
  hipLaunchKernelGGL(k_splitk_sum, dim3((unsigned)((32 * 9 + 63) / 64)), dim3(1024), 0, c.st, gs, (int)ns,
                     c.s(P.part));
  return hipGetLastError();
}

}  // namespace

// ------------------------------------------------------------------------------------------
// entry points (hn_api.hip validates and forwards)
// ------------------------------------------------------------------------------------------
int hn_nas_train_plan(const hn_arch_desc& d, long B, size_t* n_tensors, size_t* saved, size_t* scratch) {
  const Plan P = make_plan(d, B);
  if (n_tensors) *n_tensors = (size_t)P.nt;
  if (saved) *saved = P.saved;
  if (scratch) *scratch = P.scratch;
  return 0;
}

// the first weight slot whose gradient pointer is NULL, or -1 (frozen parameters still need a buffer:
// the weight-gradient kernels write unconditionally; only the affine BN gradients may be NULL)
int hn_nas_train_null_grad_slot(const hn_arch_desc& d, float* const* grads) {
  const Plan P = make_plan(d, 2);
  for (int i : P.gw)
    if (!grads[i]) return i;
  return -1;
}

hipError_t hn_nas_train_forward_impl(const hn_arch_desc& d, const float* in, long B, float* const* tensors,
                                     float momentum, const float* soft, float* out, char* saved, char* scratch,
                                     hipStream_t st) {
  Plan P = make_plan(d, B);
  Ctx c{P, tensors, nullptr, saved, scratch, st, momentum};
  return nas_fwd(c, P, in, soft, out);
}

hipError_t hn_nas_train_backward_impl(const hn_arch_desc& d, const float* dout, long B, const float* in,
                                      float* const* tensors, const float* soft, float* const* grads, float* dsoft,
                                      char* saved, char* scratch, hipStream_t st) {
  Plan P = make_plan(d, B);
  Ctx c{P, tensors, grads, saved, scratch, st, 0.f};
  return nas_bwd(c, P, in, soft, dout, dsoft);
}
