// Fused distance_matrix_vector + hardest-in-batch negative (hardnet/Losses.py:5-13, 87-110)
// without materialising the B x B matrix (a 65,536-pair batch would be 17.2 GB).
//
//   dm(i,j)  = sqrt(|a_i|^2 + |p_j|^2 - 2 a_i.p_j + 1e-6) + 1e-8
//   d(i,j)   = dm(i,j) + 10*[i==j];  d += 10 where d < 0.008
//   pos[i]   = dm(i,i);   min_neg[i] = min_j d(i,j)   (min with min_i d(i,j) if anchor_swap)
//
// One workgroup owns 64 anchor rows and sweeps all positives in 64-column tiles staged
// through LDS; row minima stay in registers, column minima go to the workspace with an
// atomicMin on the (non-negative) float bit pattern.  fp32 VALU.
#include "hn_common.h"
#include "hn_internal.h"

namespace {
constexpr int TM = 64, TN = 64, D = 128, LDP = D + 4;

__global__ __launch_bounds__(256) void k_colmin_init(unsigned* cm, int B) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < B) cm[i] = 0x7f800000u;  // +inf
}

__global__ __launch_bounds__(256) void k_pairdist(const float* __restrict__ a, const float* __restrict__ p,
                                                  int B, int swap, float* __restrict__ pos,
                                                  float* __restrict__ rowmin, unsigned* __restrict__ colmin) {
  __shared__ float sa[TM][LDP];
  __shared__ float sp[TN][LDP];
  __shared__ float asq[TM], psq[TN];
  __shared__ float red[16][TN];
  const int t = threadIdx.x;
  const int ty = t >> 4, tx = t & 15;  // 16 x 16 threads, 4 x 4 outputs each
  const int i0 = blockIdx.x * TM;
  for (int e = t; e < TM * D / 4; e += 256) {
    const int r = e / (D / 4), c = (e % (D / 4)) * 4;
    const int gi = min(i0 + r, B - 1);
    *reinterpret_cast<float4*>(&sa[r][c]) = *reinterpret_cast<const float4*>(a + (size_t)gi * D + c);
  }
  __syncthreads();
  if (t < TM) {
    float s = 0.f;
    for (int c = 0; c < D; ++c) s = fmaf(sa[t][c], sa[t][c], s);
    asq[t] = s;
  }
  float rmin[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
  for (int j0 = 0; j0 < B; j0 += TN) {
    __syncthreads();
    for (int e = t; e < TN * D / 4; e += 256) {
      const int r = e / (D / 4), c = (e % (D / 4)) * 4;
      const int gj = min(j0 + r, B - 1);
      *reinterpret_cast<float4*>(&sp[r][c]) = *reinterpret_cast<const float4*>(p + (size_t)gj * D + c);
    }
    __syncthreads();
    if (t < TN) {
      float s = 0.f;
      for (int c = 0; c < D; ++c) s = fmaf(sp[t][c], sp[t][c], s);
      psq[t] = s;
    }
    float dot[4][4] = {};
    for (int c = 0; c < D; c += 4) {
      float4 av[4], pv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        av[u] = *reinterpret_cast<const float4*>(&sa[ty + 16 * u][c]);
        pv[u] = *reinterpret_cast<const float4*>(&sp[tx + 16 * u][c]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          dot[u][v] = fmaf(av[u].x, pv[v].x, dot[u][v]);
          dot[u][v] = fmaf(av[u].y, pv[v].y, dot[u][v]);
          dot[u][v] = fmaf(av[u].z, pv[v].z, dot[u][v]);
          dot[u][v] = fmaf(av[u].w, pv[v].w, dot[u][v]);
        }
    }
    __syncthreads();  // psq ready
    float cmin[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + ty + 16 * u;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int j = j0 + tx + 16 * v;
        float dm = sqrtf((asq[ty + 16 * u] + psq[tx + 16 * v]) - 2.0f * dot[u][v] + 1e-6f) + 1e-8f;
        float d = dm;
        if (i == j) {
          if (i < B) pos[i] = dm;
          d += 10.f;
        }
        if (d < 0.008f) d += 10.f;
        if (i < B && j < B) {
          rmin[u] = fminf(rmin[u], d);
          cmin[v] = fminf(cmin[v], d);
        }
      }
    }
    if (swap) {
#pragma unroll
      for (int v = 0; v < 4; ++v) red[ty][tx + 16 * v] = cmin[v];
      __syncthreads();
      if (t < TN) {
        float m = red[0][t];
        for (int k = 1; k < 16; ++k) m = fminf(m, red[k][t]);
        if (j0 + t < B) atomicMin(colmin + j0 + t, __float_as_uint(m));
      }
    }
  }
  // reduce row minima over the 16 threads sharing a row (tx), write
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) red[tx][ty + 16 * u] = rmin[u];
  __syncthreads();
  if (t < TM) {
    float m = red[0][t];
    for (int k = 1; k < 16; ++k) m = fminf(m, red[k][t]);
    if (i0 + t < B) rowmin[i0 + t] = m;
  }
}

__global__ __launch_bounds__(256) void k_combine(float* rowmin, const unsigned* colmin, int B) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < B) rowmin[i] = fminf(rowmin[i], __uint_as_float(colmin[i]));
}
}  // namespace

hipError_t hn_launch_pairdist(const float* a, const float* p, int B, int D_, int swap,
                              float* pos, float* minneg, void* ws, hipStream_t st) {
  if (D_ != D) return hipErrorInvalidValue;
  unsigned* cm = static_cast<unsigned*>(ws);
  const unsigned g = (B + 255) / 256;
  if (swap) hipLaunchKernelGGL(k_colmin_init, dim3(g), dim3(256), 0, st, cm, B);
  hipLaunchKernelGGL(k_pairdist, dim3((B + TM - 1) / TM), dim3(256), 0, st, a, p, B, swap, pos,
                     minneg, cm);
  if (swap) hipLaunchKernelGGL(k_combine, dim3(g), dim3(256), 0, st, minneg, cm, B);
  return hipGetLastError();
}
