// Kernels shared by the train-mode paths (hn_train.hip: stock HardNet; hn_nas_train.hip: the
// hardnetNAS descriptors and supernet): the generic f32-MFMA GEMM with split-K fp64 sums and its
// B-operand loaders, BatchNorm batch-statistics passes over CNHW rows, input_norm, L2Norm, the
// counter-hash dropout mask, and conv0's 1 -> 32 3x3 forward / weight gradient on 32x32 patches.
// Included by each train translation unit inside an anonymous namespace (one private copy each).
#pragma once
#include "hn_common.h"
#include "hn_internal.h"

#include <algorithm>

namespace {

// ------------------------------------------------------------------------------------------
// generic fp32 GEMM: C(i,j) = alpha * sum_k A(i,k) B(k,j) + beta * C(i,j), element strides
// A(i,k) = A[i*sai + k*sak], B(k,j) = B[k*sbk + j*sbj], C(i,j) = C[i*sci + j*scj].  64x64
// workgroup tiles (4 waves of 32x32, v_mfma_f32_32x32x2_f32), K steps of 16 staged through LDS
// as fp32 (bounds-checked, zero-filled).
// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// counter-hash dropout mask (keep with probability 1 - p), recomputed in the backward
// ------------------------------------------------------------------------------------------
HN_DEV float drop_scale(unsigned long long seed, unsigned long long e, float p) {
  unsigned long long x = seed ^ (e * 0x9E3779B97F4A7C15ull);
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  const float u = (float)(x >> 40) * (1.0f / 16777216.0f);  // [0, 1)
  return u < p ? 0.f : 1.f / (1.f - p);
}

// the input of the next layer from a saved BN output: relu(z) [x dropout]
struct ActIn {
  const float* z;  // CNHW
  int relu;
  float drop_p;    // 0: no dropout
  unsigned long long seed;
};
HN_DEV float act_at(const ActIn& a, long idx) {
  float v = a.z[idx];
  if (a.relu) v = fmaxf(v, 0.f);
  if (a.drop_p > 0.f) v *= drop_scale(a.seed, (unsigned long long)idx, a.drop_p);
  return v;
}

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  long M, N, K;
  long sai, sak, sbk, sbj, sci, scj;
  float alpha, beta;
};

// split-K: workgroup z of gridDim.z covers K range [z * kslice, (z + 1) * kslice) and writes
// its partial tile to part[z] (M x N, row-major); k_splitk_sum adds the slices in fp64, so a
// weight gradient's reduction over all B*H*W positions never runs as one fp32 chain.
// Tiles: 64 (M) x 128 (N) per workgroup, 4 waves of 32 x 64 (two 32 x 32 f32 accumulators),
// K stages of 32 double-buffered in LDS with the next stage's global loads in registers while
// the current stage's MFMAs run (each operand is loaded along whichever index is contiguous).
constexpr int GBM = 64, GBN = 128, GBK = 32;  // (GBM: the largest M tile)

// B operand loaders: plain strided memory, or an implicit im2col of a saved BN output
// (relu(z) [x dropout]) for a 3x3 / 8x8 conv layer with compile-time geometry, so the forward
// and the weight gradient never materialise the column matrix:
//   Im2col<..., false>: B(k, j) = col(kconv = k, pos = j)   (forward, N = B Ho Wo)
//   Im2col<..., true> : B(k, j) = col(kconv = j, pos = k)   (wgrad,  K = B Ho Wo)
struct StridedB {
  HN_DEV float at(const GemmArgs& g, long k, long j) const { return g.B[k * g.sbk + j * g.sbj]; }
};
template <int C, int H, int KS, int S, int PAD, bool T>
struct Im2colB {
  static constexpr int HO = (H + 2 * PAD - KS) / S + 1, HWO = HO * HO, KK = KS * KS;
  ActIn a;
  long B;  // batch (CNHW channel stride = B * H * H)
  HN_DEV float at(const GemmArgs&, long k, long j) const {
    const long kc = T ? j : k, pos = T ? k : j;
    const int c = (int)(kc / KK), tap = (int)(kc % KK), dy = tap / KS, dx = tap % KS;
    const long p = pos / HWO;
    const int o = (int)(pos % HWO), oy = o / HO, ox = o % HO;
    const int y = oy * S - PAD + dy, x = ox * S - PAD + dx;
    return (y >= 0 && y < H && x >= 0 && x < H) ? act_at(a, ((long)c * B + p) * (H * H) + y * H + x) : 0.f;
  }
};

// dgrad as an implicit GEMM (no column matrix, no col2im): dX[c][pos_in] = sum over (co, tap) of
// Wt[c][co][tap] . dY[co][pos_out(pos_in, tap)], the entry zero where the tap does not land on a
// stride-S output; B(k = co * KS^2 + tap, j = pos_in), contiguous along j
template <int COUT, int H, int KS, int S, int PAD>
struct Col2imB {
  static constexpr int HO = (H + 2 * PAD - KS) / S + 1, HWO = HO * HO, KK = KS * KS;
  const float* dY;  // [COUT][B][HO][HO]
  long B;
  HN_DEV float at(const GemmArgs&, long k, long j) const {
    const int co = (int)(k / KK), tap = (int)(k % KK), dy = tap / KS, dx = tap % KS;
    const long p = j / (H * H);
    const int q = (int)(j % (H * H)), y = q / H, x = q % H;
    const int ty = y + PAD - dy, tx = x + PAD - dx;
    if (ty < 0 || tx < 0 || ty % S || tx % S) return 0.f;
    const int oy = ty / S, ox = tx / S;
    return (oy < HO && ox < HO) ? dY[((long)co * B + p) * HWO + oy * HO + ox] : 0.f;
  }
};

// Wt[c][co][tap] = W[co][c][tap]
__global__ __launch_bounds__(256) void k_wt(const float* __restrict__ w, int cout, int cin, int kk, float* __restrict__ wt) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)cout * cin * kk) return;
  const int tap = (int)(e % kk), c = (int)((e / kk) % cin), co = (int)(e / ((long)kk * cin));
  wt[((long)c * cout + co) * kk + tap] = w[e];
}

// BM = 64: 2 x 2 waves of 32 x 64; BM = 32 (the 32-output-channel layers): 1 x 4 waves of 32 x 32
// one workgroup's output tile: rows i0 .., columns j0 .., K range [kb, ke) (split-K slice z into part[z])
template <int BM, class BL>
HN_DEV void gemm_tile(const GemmArgs& g, const BL& bl, long i0, long j0, long kb, long ke, int z,
                      float* __restrict__ part) {
  constexpr int GBM = BM, WN = BM == 64 ? 64 : 32;  // M rows per workgroup, N columns per wave
  __shared__ float sA[2][GBK][GBM + 4];   // [k][m]
  __shared__ float sB[2][GBK][GBN + 4];   // [k][n]
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = BM == 64 ? w >> 1 : 0, wn = BM == 64 ? w & 1 : w, r = lane & 31, h = lane >> 5;
  const bool a_k = g.sak == 1, b_n = g.sbj == 1;  // contiguous index of each operand
  constexpr int AN = GBM * GBK / 256, BNN = GBK * GBN / 256;  // 8 / 16 elements per thread
  float ra[AN], rb[BNN];
  auto load = [&](long k0) {
#pragma unroll
    for (int e = 0; e < AN; ++e) {
      const int idx = t + 256 * e;
      const int mm = a_k ? idx / GBK : idx % GBM, kk = a_k ? idx % GBK : idx / GBM;
      const long gi = i0 + mm, gk = k0 + kk;
      ra[e] = (gi < g.M && gk < ke) ? g.A[gi * g.sai + gk * g.sak] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < BNN; ++e) {
      const int idx = t + 256 * e;
      const int kk = b_n ? idx / GBN : idx % GBK, nn = b_n ? idx % GBN : idx / GBK;
      const long gk = k0 + kk, gj = j0 + nn;
      rb[e] = (gk < ke && gj < g.N) ? bl.at(g, gk, gj) : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int e = 0; e < AN; ++e) {
      const int idx = t + 256 * e;
      const int mm = a_k ? idx / GBK : idx % GBM, kk = a_k ? idx % GBK : idx / GBM;
      sA[buf][kk][mm] = ra[e];
    }
#pragma unroll
    for (int e = 0; e < BNN; ++e) {
      const int idx = t + 256 * e;
      const int kk = b_n ? idx / GBN : idx % GBK, nn = b_n ? idx % GBN : idx / GBK;
      sB[buf][kk][nn] = rb[e];
    }
  };
  f32x16 acc0{}, acc1{};
  load(kb);
  store(0);
  __syncthreads();
  int buf = 0;
  for (long k0 = kb; k0 < ke; k0 += GBK) {
    const bool more = k0 + GBK < ke;
    if (more) load(k0 + GBK);
    // v_mfma_f32_32x32x2_f32: exact fp32 products (an fmaf chain per output, bitwise), so the
    // backward through train-mode BatchNorm -- whose 1/sigma amplifies rounding -- carries fp32
    // accuracy, as the reference's fp32 autograd does (bf16x3's 2^-16 products measured 3-10x
    // further from the fp64 gradients than torch-CPU fp32)
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 2) {
      const float av = sA[buf][kk + h][wm * 32 + r];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, sB[buf][kk + h][wn * WN + r], acc0, 0, 0, 0);
      if constexpr (BM == 64)
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, sB[buf][kk + h][wn * WN + 32 + r], acc1, 0, 0, 0);
    }
    if (more) {
      store(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }
  // acc[4q + e]: row 8q + 4h + e, column r of each 32 x 32 sub-tile
#pragma unroll
  for (int nt = 0; nt < (BM == 64 ? 2 : 1); ++nt) {
    const long j = j0 + wn * WN + nt * 32 + r;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long i = i0 + wm * 32 + 8 * q + 4 * h + e;
        const float v = nt ? acc1[4 * q + e] : acc0[4 * q + e];
        if (i < g.M && j < g.N) {
          if (part) {
            part[((long)z * g.M + i) * g.N + j] = v;
          } else {
            float* c = g.C + i * g.sci + j * g.scj;
            *c = g.beta == 0.f ? g.alpha * v : g.alpha * v + g.beta * *c;
          }
        }
      }
  }
}

template <int BM, class BL>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g, BL bl, long kslice, float* __restrict__ part) {
  const long kb = (long)blockIdx.z * kslice;
  gemm_tile<BM>(g, bl, (long)blockIdx.y * BM, (long)blockIdx.x * GBN, kb, min(g.K, kb + kslice), (int)blockIdx.z,
                part);
}

// 64 consecutive outputs x 16 slice groups per workgroup: lane x of group y sums slices y, y + 16,
// ... (coalesced 256-byte rows per slice), then the 16 group sums are added in a fixed order
// (deterministic; fp64 throughout)
__global__ __launch_bounds__(1024) void k_splitk_sum(GemmArgs g, int S, const float* __restrict__ part) {
  __shared__ double red[16][64];
  const int x = threadIdx.x & 63, y = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 64 + x, mn = g.M * g.N;
  double s = 0.0;
  if (e < mn)
    for (int z = y; z < S; z += 16) s += part[(long)z * mn + e];
  red[y][x] = s;
  __syncthreads();
  if (y != 0 || e >= mn) return;
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) t += red[k][x];
  const long i = e / g.N, j = e % g.N;
  float* c = g.C + i * g.sci + j * g.scj;
  *c = g.beta == 0.f ? (float)(g.alpha * t) : (float)(g.alpha * t + g.beta * (double)*c);
}

// part: scratch for the split-K partials, M x N x slices floats (nullptr: one slice).
// The B loader's contiguous index: StridedB reads g.sbj to decide; Im2colB<.., T> is
// contiguous along pos (N for the forward, K for the wgrad) -- set in g.sbj / g.sbk.
template <class BL = StridedB>
hipError_t gemm(const GemmArgs& g, hipStream_t st, float* part = nullptr, BL bl = BL{}) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  const int bm = g.M <= 32 ? 32 : 64;
  const long tiles = ((g.N + GBN - 1) / GBN) * ((g.M + bm - 1) / bm);
  long ks = hn_knobs().train_splitk;  // K per slice (HN_TRAIN_SPLITK, default 1024)
  if (part && tiles < 256 && g.K > 64) {  // a small grid: split K until every CU has a workgroup
    const long want = std::min<long>((256 + tiles - 1) / tiles, (g.K + 63) / 64);
    ks = std::min(ks, ((g.K + want - 1) / want + GBK - 1) / GBK * GBK);
  }
  const int S = part && g.K > ks ? (int)((g.K + ks - 1) / ks) : 1;
  const dim3 grid((unsigned)((g.N + GBN - 1) / GBN), (unsigned)((g.M + bm - 1) / bm), (unsigned)S);
  if (bm == 32)
    hipLaunchKernelGGL((k_gemm<32, BL>), grid, dim3(256), 0, st, g, bl, S > 1 ? ks : g.K, S > 1 ? part : nullptr);
  else
    hipLaunchKernelGGL((k_gemm<64, BL>), grid, dim3(256), 0, st, g, bl, S > 1 ? ks : g.K, S > 1 ? part : nullptr);
  if (S > 1) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_splitk_sum, dim3((unsigned)((g.M * g.N + 63) / 64)), dim3(1024), 0, st, g, S, part);
  }
  return hipGetLastError();
}

// col2im (gather) for the strided / 8x8 dgrads: d_in [C][B][H][W] patches [n0, n0 + n) = sum of the
// dcol [C*KS*KS][n*Ho*Wo] entries that read them
__global__ __launch_bounds__(256) void k_col2im(const float* __restrict__ dcol, int C, long B, int H, int W, int KS,
                                                int S, int PAD, int Ho, int Wo, long n0, long n,
                                                float* __restrict__ din) {
  const long cols = n * Ho * Wo;
  const long total = (long)C * n * H * W;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int x = (int)(e % W), y = (int)((e / W) % H);
    const long p = (e / ((long)W * H)) % n;
    const int c = (int)(e / ((long)W * H * n));
    float s = 0.f;
    for (int dy = 0; dy < KS; ++dy) {
      const int ty = y + PAD - dy;
      if (ty < 0 || ty % S) continue;
      const int oy = ty / S;
      if (oy >= Ho) continue;
      for (int dx = 0; dx < KS; ++dx) {
        const int tx = x + PAD - dx;
        if (tx < 0 || tx % S) continue;
        const int ox = tx / S;
        if (ox >= Wo) continue;
        s += dcol[((long)c * KS * KS + dy * KS + dx) * cols + p * Ho * Wo + oy * Wo + ox];
      }
    }
    din[(((long)c * B + n0 + p) * H + y) * W + x] = s;
  }
}

// ------------------------------------------------------------------------------------------
// BatchNorm2d(affine=False) in train mode over CNHW rows of L values.  Statistics in two
// stages so the whole GPU works on them: grid (C, NS) workgroups each reduce a slice of a
// channel's row in fp64 (sum y, sum y^2 -- fp64 keeps E[y^2] - E[y]^2 exact enough), then one
// thread per channel combines its NS partials in a fixed order (deterministic).
// ------------------------------------------------------------------------------------------
HN_DEV void block_sum2(double& a, double& b, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[2 * w] = a;
    sh[2 * w + 1] = b;
  }
  __syncthreads();
  a = sh[0] + sh[2] + sh[4] + sh[6];
  b = sh[1] + sh[3] + sh[5] + sh[7];
}

constexpr int kBnSlices = 64;  // partial-sum workgroups per channel (at most)
int bn_slices(long C, long L) {
  return (int)std::max<long>(1, std::min<long>(kBnSlices, std::min<long>((2048 + C - 1) / C, (L + 4095) / 4096)));
}

// forward stats: part[(c * NS + s) * 2 + {0, 1}] = sum y, sum y^2 over slice s of row c
HN_DEV void bn_part_body(const float* __restrict__ y, long L, int NS, double* __restrict__ part, int c, int sl) {
  __shared__ double sh[8];
  const float* row = y + (long)c * L;
  double s1 = 0.0, s2 = 0.0;
  if ((L & 3) == 0) {  // float4 loads: slices of a multiple of 4 elements (rows start 16-byte aligned)
    const long per = ((L + NS - 1) / NS + 3) & ~3L, b = sl * per, e = min(L, b + per);
    for (long i = b + 4 * threadIdx.x; i < e; i += 1024) {
      const float4 v = *reinterpret_cast<const float4*>(row + i);
      s1 += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
      s2 += ((double)v.x * v.x + (double)v.y * v.y) + ((double)v.z * v.z + (double)v.w * v.w);
    }
  } else {
    const long per = (L + NS - 1) / NS, b = sl * per, e = min(L, b + per);
    for (long i = b + threadIdx.x; i < e; i += 256) {
      const double v = row[i];
      s1 += v;
      s2 += v * v;
    }
  }
  block_sum2(s1, s2, sh);
  if (threadIdx.x == 0) {
    part[((long)c * NS + sl) * 2] = s1;
    part[((long)c * NS + sl) * 2 + 1] = s2;
  }
}
__global__ __launch_bounds__(256) void k_bn_part(const float* __restrict__ y, long L, int NS, double* __restrict__ part) {
  bn_part_body(y, L, NS, part, blockIdx.x, blockIdx.y);
}

// the channel's batch statistics from k_bn_part's slice sums (fixed slice order): mean, 1/sqrt(var + eps);
// with `upd`, rstd saved and the running statistics updated (var unbiased)
HN_DEV void bn_stats(const double* __restrict__ part, int c, int NS, long L, float eps, float mom, bool upd,
                     float* __restrict__ rmean, float* __restrict__ rvar, float* __restrict__ rstd_out, float& mu,
                     float& rs) {
  double s1 = 0.0, s2 = 0.0;
  for (int sl = 0; sl < NS; ++sl) {
    s1 += part[((long)c * NS + sl) * 2];
    s2 += part[((long)c * NS + sl) * 2 + 1];
  }
  const double mean = s1 / (double)L;
  const double var = fmax(s2 / (double)L - mean * mean, 0.0);
  mu = (float)mean;
  rs = (float)(1.0 / sqrt(var + (double)eps));
  if (upd) {
    rstd_out[c] = rs;
    if (rmean) {
      rmean[c] = (1.f - mom) * rmean[c] + mom * (float)mean;
      rvar[c] = (1.f - mom) * rvar[c] + mom * (float)(L > 1 ? var * (double)L / (double)(L - 1) : var);
    }
  }
}

// y (in place) -> z = (y - mean) * rstd over [C][L]; grid (C, S): workgroup (c, s) walks row c
// (no per-element channel division), float4 when rows are 16-byte aligned.  Thread 0 of every workgroup
// combines the channel's slice sums (bn_stats); workgroup (c, 0) also saves rstd and updates the running
// statistics -- no separate statistics launch between k_bn_part and this one
__global__ __launch_bounds__(256) void k_bn_apply(float* __restrict__ y, long L, const double* __restrict__ part,
                                                  int NS, float eps, float mom, float* __restrict__ rmean,
                                                  float* __restrict__ rvar, float* __restrict__ rstd_out) {
  __shared__ float st[2];
  const int c = blockIdx.x;
  if (threadIdx.x == 0) bn_stats(part, c, NS, L, eps, mom, blockIdx.y == 0, rmean, rvar, rstd_out, st[0], st[1]);
  __syncthreads();
  const float mu = st[0], rs = st[1];
  float* row = y + (long)c * L;
  const long step = (long)gridDim.y * 256;
  if ((L & 3) == 0) {
    float4* r4 = reinterpret_cast<float4*>(row);
    for (long i = (long)blockIdx.y * 256 + threadIdx.x; i < L / 4; i += step) {
      float4 v = r4[i];
      v.x = (v.x - mu) * rs;
      v.y = (v.y - mu) * rs;
      v.z = (v.z - mu) * rs;
      v.w = (v.w - mu) * rs;
      r4[i] = v;
    }
  } else {
    for (long i = (long)blockIdx.y * 256 + threadIdx.x; i < L; i += step) row[i] = (row[i] - mu) * rs;
  }
}
// row-wise grid for the BN element passes: about 4,096 workgroups in all
dim3 bn_row_grid(long C, long L) {
  const long per_row = std::max<long>(1, std::min<long>((4096 + C - 1) / C, ((L + 3) / 4 + 255) / 256));
  return dim3((unsigned)C, (unsigned)std::min<long>(per_row, 65535));
}

// backward through [dropout o] ReLU o BN(train): g = da * relu'(z) [* mask] (recomputed by
// k_bn_bwd_apply, not stored), and the slice sums of g and g z
__global__ __launch_bounds__(256) void k_bn_bwd_part(const float* __restrict__ da, const float* __restrict__ z, long L,
                                                     int NS, int relu, float drop_p, unsigned long long seed,
                                                     double* __restrict__ part) {
  __shared__ double sh[8];
  const int c = blockIdx.x, sl = blockIdx.y;
  const long per = (L + NS - 1) / NS, b = sl * per, e = min(L, b + per);
  const long base = (long)c * L;
  double s1 = 0.0, s2 = 0.0;
  auto acc = [&](float v, float zv, long i) {
    if (relu && zv <= 0.f) v = 0.f;
    if (drop_p > 0.f) v *= drop_scale(seed, (unsigned long long)(base + i), drop_p);
    s1 += v;
    s2 += (double)v * zv;
  };
  if ((L & 3) == 0) {  // float4 loads over slices of a multiple of 4 elements
    const long per4 = (per + 3) & ~3L, b4 = sl * per4, e4 = min(L, b4 + per4);
    for (long i = b4 + 4 * threadIdx.x; i < e4; i += 1024) {
      const float4 zv = *reinterpret_cast<const float4*>(z + base + i);
      const float4 v = *reinterpret_cast<const float4*>(da + base + i);
      acc(v.x, zv.x, i);
      acc(v.y, zv.y, i + 1);
      acc(v.z, zv.z, i + 2);
      acc(v.w, zv.w, i + 3);
    }
  } else {
    for (long i = b + threadIdx.x; i < e; i += 256) acc(da[base + i], z[base + i], i);
  }
  block_sum2(s1, s2, sh);
  if (threadIdx.x == 0) {
    part[((long)c * NS + sl) * 2] = s1;
    part[((long)c * NS + sl) * 2 + 1] = s2;
  }
}

// dy = rstd * (g - m1 - z m2) with g = da * relu'(z) [* mask] as in k_bn_bwd_part, in place; grid (C, S)
// as k_bn_apply; m1 = mean(g), m2 = mean(g z) combined from k_bn_bwd_part's slice sums by thread 0 of
// every workgroup (fixed slice order)
__global__ __launch_bounds__(256) void k_bn_bwd_apply(float* __restrict__ g, const float* __restrict__ z, long L,
                                                      const double* __restrict__ part, int NS,
                                                      const float* __restrict__ rstd, int relu, float drop_p,
                                                      unsigned long long seed) {
  __shared__ float st[2];
  const int c = blockIdx.x;
  if (threadIdx.x == 0) {
    double s1 = 0.0, s2 = 0.0;
    for (int sl = 0; sl < NS; ++sl) {
      s1 += part[((long)c * NS + sl) * 2];
      s2 += part[((long)c * NS + sl) * 2 + 1];
    }
    st[0] = (float)(s1 / (double)L);
    st[1] = (float)(s2 / (double)L);
  }
  __syncthreads();
  const float m1 = st[0], m2 = st[1], rs = rstd[c];
  const long base = (long)c * L, step = (long)gridDim.y * 256;
  auto one = [&](float v, float zv, long i) {
    if (relu && zv <= 0.f) v = 0.f;
    if (drop_p > 0.f) v *= drop_scale(seed, (unsigned long long)(base + i), drop_p);
    return rs * (v - m1 - zv * m2);
  };
  if ((L & 3) == 0) {
    float4* g4 = reinterpret_cast<float4*>(g + base);
    const float4* z4 = reinterpret_cast<const float4*>(z + base);
    for (long i = (long)blockIdx.y * 256 + threadIdx.x; i < L / 4; i += step) {
      const float4 zv = z4[i];
      float4 v = g4[i];
      v.x = one(v.x, zv.x, 4 * i);
      v.y = one(v.y, zv.y, 4 * i + 1);
      v.z = one(v.z, zv.z, 4 * i + 2);
      v.w = one(v.w, zv.w, 4 * i + 3);
      g4[i] = v;
    }
  } else {
    for (long i = (long)blockIdx.y * 256 + threadIdx.x; i < L; i += step) g[base + i] = one(g[base + i], z[base + i], i);
  }
}

// input_norm (HardNet.py:306-310, mean / std detached): one wave per patch; saves 1 / (std + eps)
__global__ __launch_bounds__(256) void k_input_norm(const float* __restrict__ in, long B, float eps,
                                                    float* __restrict__ xn, float* __restrict__ inv_sd) {
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= B) return;
  float v[16];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    v[j] = in[p * 1024 + j * 64 + lane];
    s += v[j];
  }
  const float mean = wave_sum(s) * (1.f / 1024.f);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) q += (v[j] - mean) * (v[j] - mean);
  const float sd = sqrtf(wave_sum(q) * (1.f / 1023.f)) + eps;
#pragma unroll
  for (int j = 0; j < 16; ++j) xn[p * 1024 + j * 64 + lane] = (v[j] - mean) / sd;
  if (lane == 0) inv_sd[p] = 1.f / sd;
}

__global__ __launch_bounds__(256) void k_scale_rows(float* __restrict__ g, long B, const float* __restrict__ s) {
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < B * 1024; e += (long)gridDim.x * 256) g[e] *= s[e >> 10];
}

// L2Norm (Utils.py:15-22) of z6 [128][B] -> out [B][128]; one wave per patch
__global__ __launch_bounds__(256) void k_l2_fwd(const float* __restrict__ z, long B, float eps, float* __restrict__ out) {
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= B) return;
  const float a = z[(long)lane * B + p], b = z[(long)(lane + 64) * B + p];
  const float n = sqrtf(wave_sum(a * a + b * b) + eps);
  out[p * 128 + lane] = a / n;
  out[p * 128 + 64 + lane] = b / n;
}

// dz6 [128][B] from dout [B][128]: y = z / n, dz = (dy - y (y . dy)) / n
__global__ __launch_bounds__(256) void k_l2_bwd(const float* __restrict__ z, const float* __restrict__ dout, long B,
                                                float eps, float* __restrict__ dz) {
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= B) return;
  const float a = z[(long)lane * B + p], b = z[(long)(lane + 64) * B + p];
  const float n = sqrtf(wave_sum(a * a + b * b) + eps);
  const float ya = a / n, yb = b / n, da = dout[p * 128 + lane], db = dout[p * 128 + 64 + lane];
  const float dot = wave_sum(ya * da + yb * db);
  dz[(long)lane * B + p] = (da - ya * dot) / n;
  dz[(long)(lane + 64) * B + p] = (db - yb * dot) / n;
}


// ------------------------------------------------------------------------------------------
// conv0 (1 -> 32, 3x3, pad 1, on the normalised patch xn [B][32][32]): the 9 taps are the MFMA's
// K (forward: 5 K-pairs, tap 9 zero) or its N (weight gradient: columns 0..8 of the 32).
// k_fwd0: one wave per patch, the patch in LDS with a zero frame; output row y = one 32-position
// tile: z[co][b][y][x] = sum_t W[co][t] . xn[y + t / 3 - 1][x + t % 3 - 1].
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fwd0(const float* __restrict__ xn, const float* __restrict__ W, long B,
                                              float* __restrict__ z) {
  __shared__ float smem[4][34 * 34 + 2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  float* s = smem[w];
  for (int i = lane; i < 34 * 34; i += 64) s[i] = 0.f;
  __builtin_amdgcn_wave_barrier();
  const long b = (long)blockIdx.x * 4 + w;
  if (b >= B) return;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int e = lane + 64 * i;
    s[(e / 32 + 1) * 34 + e % 32 + 1] = xn[b * 1024 + e];
  }
  __builtin_amdgcn_wave_barrier();
  float a[5];  // A[m = co r][k = tap 2 j + h]
#pragma unroll
  for (int j = 0; j < 5; ++j) a[j] = 2 * j + h < 9 ? W[r * 9 + 2 * j + h] : 0.f;
#pragma unroll 2
  for (int y = 0; y < 32; ++y) {
    f32x16 acc = f32x16{};
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int t = 2 * j + h;
      const float bv = t < 9 ? s[(y + t / 3) * 34 + r + t % 3] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) z[((long)(8 * q + 4 * h + e) * B + b) * 1024 + y * 32 + r] = acc[4 * q + e];
  }
}

// k_wgrad0: dW[co][t] = sum over (b, y, x) of dY[co][b][y][x] . xn[b][y + t / 3 - 1][x + t % 3 - 1]:
// A[m = co][k = position pair] from the wave's LDS dY row, B[k][n = tap] from the patch in LDS
// (taps 9..31 zero), one MFMA per position pair; NPC patches per workgroup chunk, one split-K slice
// per wave.
constexpr int kWg0Npc = 8;
__global__ __launch_bounds__(256) void k_wgrad0(const float* __restrict__ xn, const float* __restrict__ dY, long B,
                                                float* __restrict__ part) {
  __shared__ float smem[4][34 * 34 + 32 * 33 + 2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  float* sx = smem[w];
  float* sy = sx + 34 * 34;  // [32 co][33]
  for (int i = lane; i < 34 * 34; i += 64) sx[i] = 0.f;
  __builtin_amdgcn_wave_barrier();
  const int tdy = r < 9 ? r / 3 : 0, tdx = r < 9 ? r % 3 : 0;
  f32x16 acc = f32x16{};
#pragma unroll 1
  for (int pi = 0; pi < kWg0Npc / 4; ++pi) {
    const long b = (long)blockIdx.x * kWg0Npc + w + 4 * pi;
    if (b >= B) break;  // wave-uniform
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = lane + 64 * i;
      sx[(e / 32 + 1) * 34 + e % 32 + 1] = xn[b * 1024 + e];
    }
    float vy[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // dY row 0: lane -> channel (lane * 16 + i) / 32
      const int e = lane * 16 + i;
      vy[i] = dY[((long)(e / 32) * B + b) * 1024 + e % 32];
    }
#pragma unroll 1
    for (int y = 0; y < 32; ++y) {
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int e = lane * 16 + i;
        sy[(e / 32) * 33 + e % 32] = vy[i];
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (y + 1 < 32) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int e = lane * 16 + i;
          vy[i] = dY[((long)(e / 32) * B + b) * 1024 + (y + 1) * 32 + e % 32];
        }
      }
      const float* xr = sx + (y + tdy) * 34 + tdx;
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int x = 2 * m + h;
        const float bv = r < 9 ? xr[x] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(sy[r * 33 + x], bv, acc, 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
  // acc[4q + e] = dW[co = 8q + 4h + e][tap r] (r < 9)
  float* dst = part + ((long)blockIdx.x * 4 + w) * 288;
  if (r < 9)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[(8 * q + 4 * h + e) * 9 + r] = acc[4 * q + e];
}

static long wgrad0_slices(long B) { return 4 * ((B + kWg0Npc - 1) / kWg0Npc); }

}  // namespace
