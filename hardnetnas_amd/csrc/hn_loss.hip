// Train-mode loss_HardNet with batch_reduce 'min' (hardnet/Losses.py:87-154, the default of the
// training loop, HardNet.py:408-413) and its backward (HardNet.py:421-423), without the B x B
// distance matrix: forward and backward run on these kernels end to end.
//
// Forward (k_lmin_tiles + k_lmin_finish):
//   d_ij  = sqrt((|a_i|^2 + |p_j|^2) - 2 a_i.p_j + 1e-6) + 1e-8        (Losses.py:5-13, :93)
//   dn_ij = d_ij + 10 [i = j];  dn_ij += 10 if dn_ij < 0.008            (:95-101)
//   row_i = min_j dn_ij (argmin r_i),  col_i = min_k dn_ki (argmin c_i) (:103-108)
//   mn_i  = anchor_swap ? min(row_i, col_i) : row_i,  pos_i = d_ii
//   loss  = mean_i f(pos_i, mn_i)  (triplet_margin / softmax / contrastive, :142-153)
// The products are exact fp32 FMAs (the reference's torch.bmm is fp32); minima carry their
// argmin packed below the value bits in one u64 (dn >= 0, so the float bits order like the
// floats), so a tie keeps the first index whatever order the workgroups finish in.
//
// Backward (k_lmin_bwd_src + k_lmin_bwd_gather) -- what autograd does over the reference
// formulation: the min selects one entry per row (torch.min(dim) routes the gradient to its
// argmin), torch.minimum splits a tie between the row and the column entry in halves, and
// sqrt(u) passes g / (2 sqrt(u)) to u = |a_i|^2 + |p_j|^2 - 2 a_i.p_j + 1e-6, i.e.
// 2 a_i - 2 p_j to a_i and 2 p_j - 2 a_i to p_j.  Row i's hardest negative (i, r_i) feeds p_{r_i},
// the column minimum (c_i, i) feeds a_{c_i}: the gather kernel gives each target row the terms
// of every source that selected it, in increasing source order (deterministic: the per-target source
// lists are built by a counting pass, a scan and an unordered fill, and each target's wave orders its
// list before summing -- O(B) work for any selection pattern but a target with > 64 sources, which
// scans all sources in order).
#include "hn_common.h"
#include "hn_internal.h"

namespace {

constexpr int D = 128;   // descriptor length
constexpr int TM = 64;   // rows (anchors) per workgroup
constexpr int TN = 64;   // columns (positives) per tile

HN_DEV unsigned long long key_of(float v, int idx) {
  return ((unsigned long long)__float_as_uint(v) << 32) | (unsigned)idx;
}
HN_DEV float key_val(unsigned long long k) { return __uint_as_float((unsigned)(k >> 32)); }
HN_DEV int key_idx(unsigned long long k) { return (int)(unsigned)(k & 0xffffffffu); }
HN_DEV unsigned long long umin64(unsigned long long x, unsigned long long y) { return x < y ? x : y; }

__global__ __launch_bounds__(256) void k_lmin_init(unsigned long long* __restrict__ colbest, int B) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < B; i += gridDim.x * 256) colbest[i] = ~0ull;
}

// |v|^2 of every row (a then p), one wave per row; for w < B also the positive distance d_ii from
// |a_i - p_i|^2 directly: the expanded |a|^2 + |p|^2 - 2 a.p of the distance matrix cancels for the
// close pairs of a training batch (the reference's fp32 loss carries that error: 2e-6 on a mean of
// distances), the difference form keeps d_ii at fp32 accuracy
HN_DEV float diff_sq(const float* a, const float* p, int lane) {
  const float2 u = reinterpret_cast<const float2*>(a)[lane], v = reinterpret_cast<const float2*>(p)[lane];
  const float dx = u.x - v.x, dy = u.y - v.y;
  return wave_sum(fmaf(dx, dx, dy * dy));
}
__global__ __launch_bounds__(256) void k_lmin_sq(const float* __restrict__ a, const float* __restrict__ p, int B,
                                                 float* __restrict__ sq, float* __restrict__ pos,
                                                 float* __restrict__ posx) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= 2 * B) return;
  const float* r = (w < B ? a + (size_t)w * D : p + (size_t)(w - B) * D);
  const float2 v = reinterpret_cast<const float2*>(r)[lane];
  const float s = wave_sum(v.x * v.x + v.y * v.y);
  if (lane == 0) sq[w] = s;
  if (w < B) {
    const float x = diff_sq(a + (size_t)w * D, p + (size_t)w * D, lane);
    if (lane == 0) {
      pos[w] = sqrtf(x + 1e-6f) + 1e-8f;
      posx[w] = x;  // (kept for the backward's sqrt derivative)
    }
  }
}

// One workgroup per 64 anchors, all positives in 64-column tiles.  Thread (ty, tx) computes the
// 4 x 4 block rows 4ty..4ty+3 x columns 4tx..4tx+3 of a tile from k-major LDS copies (float4
// reads: 16 consecutive float4 across tx, broadcast across ty).
__global__ __launch_bounds__(256) void k_lmin_tiles(const float* __restrict__ a, const float* __restrict__ p,
                                                    const float* __restrict__ sq, int B, int swap,
                                                    unsigned long long* __restrict__ rowbest,
                                                    unsigned long long* __restrict__ colbest,
                                                    float* __restrict__ pos) {
  __shared__ float4 As[D][TM / 4];
  __shared__ float4 Ps[D][TN / 4];
  __shared__ unsigned long long red[16][TN];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int r0 = blockIdx.x * TM;
  // anchors -> As (k-major); rows past B are zero (their results are never stored)
  for (int e = tid; e < TM * D / 4; e += 256) {
    const int row = e % TM, k4 = e / TM;  // consecutive threads: consecutive rows (conflict-free LDS stores)
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + row < B) v = reinterpret_cast<const float4*>(a + (size_t)(r0 + row) * D)[k4];
    float* as = reinterpret_cast<float*>(&As[0][0]);
    as[(4 * k4 + 0) * TM + row] = v.x;
    as[(4 * k4 + 1) * TM + row] = v.y;
    as[(4 * k4 + 2) * TM + row] = v.z;
    as[(4 * k4 + 3) * TM + row] = v.w;
  }
  float asq[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) asq[r] = (r0 + 4 * ty + r < B) ? sq[r0 + 4 * ty + r] : 0.f;
  unsigned long long best[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  for (int c0 = 0; c0 < B; c0 += TN) {
    __syncthreads();  // previous tile's readers are done with Ps / red
    for (int e = tid; e < TN * D / 4; e += 256) {
      const int col = e % TN, k4 = e / TN;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c0 + col < B) v = reinterpret_cast<const float4*>(p + (size_t)(c0 + col) * D)[k4];
      float* ps = reinterpret_cast<float*>(&Ps[0][0]);
      ps[(4 * k4 + 0) * TN + col] = v.x;
      ps[(4 * k4 + 1) * TN + col] = v.y;
      ps[(4 * k4 + 2) * TN + col] = v.z;
      ps[(4 * k4 + 3) * TN + col] = v.w;
    }
    __syncthreads();
    float acc[4][4] = {};
#pragma unroll 4
    for (int k = 0; k < D; ++k) {
      const float4 av = As[k][ty], pv = Ps[k][tx];
      const float ar[4] = {av.x, av.y, av.z, av.w}, pc[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(ar[r], pc[c], acc[r][c]);
    }
    unsigned long long cb[4] = {~0ull, ~0ull, ~0ull, ~0ull};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int j = c0 + 4 * tx + c;
      if (j >= B) continue;
      const float psq = sq[B + j];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = r0 + 4 * ty + r;
        if (i >= B) continue;
        const float x = (asq[r] + psq) - 2.0f * acc[r][c];
        const float d = sqrtf(x + 1e-6f) + 1e-8f;
        float dn = d;
        if (i == j) dn = d + 10.0f;  // (pos[i] comes from k_lmin_sq's difference form)
        if (dn < 0.008f) dn += 10.0f;
        best[r] = umin64(best[r], key_of(dn, j));
        if (swap) cb[c] = umin64(cb[c], key_of(dn, i));
      }
    }
    if (swap) {  // column minima over the workgroup's 64 rows -> one atomic per column
#pragma unroll
      for (int c = 0; c < 4; ++c) red[ty][4 * tx + c] = cb[c];
      __syncthreads();
      if (tid < TN && c0 + tid < B) {
        unsigned long long m = red[0][tid];
#pragma unroll
        for (int t = 1; t < 16; ++t) m = umin64(m, red[t][tid]);
        atomicMin(colbest + c0 + tid, m);
      }
    }
  }
  // row minima over the 16 threads (tx) sharing a row
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) red[tx][4 * ty + r] = best[r];
  __syncthreads();
  if (tid < TM && r0 + tid < B) {
    unsigned long long m = red[0][tid];
#pragma unroll
    for (int t = 1; t < 16; ++t) m = umin64(m, red[t][tid]);
    rowbest[r0 + tid] = m;
  }
}

// per-row loss f(pos, mn) and its partials d f / d pos, d f / d mn (autograd's forms)
HN_DEV float loss_of(int type, float margin, float ps, float mn, float* dpos, float* dmn) {
  if (type == 0) {  // clamp(margin + pos - mn, min=0); clamp's backward passes at t >= 0
    const float t = margin + ps - mn;
    *dpos = t >= 0.f ? 1.f : 0.f;
    *dmn = -*dpos;
    return fmaxf(t, 0.f);
  }
  if (type == 1) {  // -log(exp_pos / (exp_pos + exp(2 - mn) + eps))
    const float ep = expf(2.0f - ps), en = expf(2.0f - mn);
    const float den = ep + en + 1e-8f;
    *dpos = (en + 1e-8f) / den;
    *dmn = -en / den;
    return -logf(ep / den);
  }
  const float t = margin - mn;  // clamp(margin - mn, min=0) + pos
  *dpos = 1.f;
  *dmn = t >= 0.f ? -1.f : 0.f;
  return fmaxf(t, 0.f) + ps;
}

// one workgroup: the mean in a fixed order (deterministic)
__global__ __launch_bounds__(1024) void k_lmin_finish(const unsigned long long* __restrict__ rowbest,
                                                      const unsigned long long* __restrict__ colbest,
                                                      const float* __restrict__ pos, int B, int swap, float margin,
                                                      int type, float* __restrict__ loss) {
  // the per-row losses in fp32 (as the reference computes them), their sum in fp64 in a fixed order,
  // so the mean carries no summation error of its own (the reference's fp32 torch.mean does)
  __shared__ double part[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < B; i += 1024) {
    const float vr = key_val(rowbest[i]);
    const float mn = swap ? fminf(vr, key_val(colbest[i])) : vr;
    float dp, dm;
    s += (double)loss_of(type, margin, pos[i], mn, &dp, &dm);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 16; ++w) t += part[w];
    loss[0] = (float)(t / (double)B);
  }
}

HN_DEV float dot128(const float* x, const float* y) {
  const float4* a = reinterpret_cast<const float4*>(x);
  const float4* b = reinterpret_cast<const float4*>(y);
  float s = 0.f;
  for (int k = 0; k < D / 4; ++k) {
    const float4 u = a[k], v = b[k];
    s = fmaf(u.x, v.x, s);
    s = fmaf(u.y, v.y, s);
    s = fmaf(u.z, v.z, s);
    s = fmaf(u.w, v.w, s);
  }
  return s;
}
// 1 / (2 sqrt(u)) for entry (i, j): sqrt's backward factor
HN_DEV float half_rsq(const float* a, const float* p, const float* sq, int B, int i, int j) {
  const float x = (sq[i] + sq[B + j]) - 2.0f * dot128(a + (size_t)i * D, p + (size_t)j * D);
  return 0.5f / sqrtf(x + 1e-6f);
}

// per source row: the coefficients of its selected entries (pos (i,i), row negative (i, r_i),
// column negative (c_i, i)) and the indices, as g / (2 sqrt(u)) of each
__global__ __launch_bounds__(256) void k_lmin_bwd_src(const float* __restrict__ a, const float* __restrict__ p,
                                                      const float* __restrict__ sq,
                                                      const unsigned long long* __restrict__ rowbest,
                                                      const unsigned long long* __restrict__ colbest,
                                                      const float* __restrict__ pos,
                                                      const float* __restrict__ posx, int B, int swap, float margin,
                                                      int type, const float* __restrict__ dloss,
                                                      float* __restrict__ coef, int* __restrict__ idx) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B) return;
  const float g = dloss[0] / (float)B;  // mean's backward
  const float vr = key_val(rowbest[i]);
  const float vc = swap ? key_val(colbest[i]) : INFINITY;
  const float mn = swap ? fminf(vr, vc) : vr;
  float dp, dm;
  loss_of(type, margin, pos[i], mn, &dp, &dm);
  // torch.minimum(row, col): the gradient to the smaller, halves on a tie
  const float fr = !swap || vr < vc ? 1.f : vr > vc ? 0.f : 0.5f;
  const int r = key_idx(rowbest[i]);
  const int c = swap ? key_idx(colbest[i]) : 0;
  const float gp = g * dp, gn = g * dm;
  // the positive entry: sqrt's backward at the forward's own |a_i - p_i|^2 (k_lmin_sq's difference form)
  const float cp = gp != 0.f ? gp * (0.5f / sqrtf(posx[i] + 1e-6f)) : 0.f;
  coef[3 * i + 0] = cp;
  coef[3 * i + 1] = gn * fr != 0.f ? gn * fr * half_rsq(a, p, sq, B, i, r) : 0.f;
  coef[3 * i + 2] = gn * (1.f - fr) != 0.f ? gn * (1.f - fr) * half_rsq(a, p, sq, B, c, i) : 0.f;
  idx[2 * i + 0] = r;
  idx[2 * i + 1] = c;
}

// Per-target source lists.  Target t < B is anchor t (sources k with a column negative c_k = t, coef
// slot 2; only with anchor_swap), t >= B positive t - B (sources with a row negative r_k = t - B, slot 1).
HN_DEV int src_target(const float* coef, const int* idx, int k, int slot, int B) {  // -1: no term
  if (coef[3 * k + 1 + slot] == 0.f) return -1;
  return slot ? idx[2 * k + 1] : B + idx[2 * k];
}
__global__ __launch_bounds__(256) void k_lmin_bwd_count(const float* __restrict__ coef, const int* __restrict__ idx,
                                                        int B, int swap, int* __restrict__ cnt) {
  for (int k = blockIdx.x * 256 + threadIdx.x; k < B; k += gridDim.x * 256)
    for (int slot = 0; slot < 1 + swap; ++slot) {
      const int tg = src_target(coef, idx, k, slot, B);
      if (tg >= 0) atomicAdd(cnt + tg, 1);
    }
}
// exclusive scan of cnt[n] -> off[n] in one workgroup (contiguous chunk per thread); fill[] := 0
__global__ __launch_bounds__(1024) void k_lmin_bwd_scan(const int* __restrict__ cnt, int n, int* __restrict__ off,
                                                        int* __restrict__ fill) {
  __shared__ int tot[1024];
  const int tid = threadIdx.x, per = (n + 1023) / 1024, b0 = min(n, tid * per), b1 = min(n, b0 + per);
  int s = 0;
  for (int i = b0; i < b1; ++i) s += cnt[i];
  tot[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan of the thread totals
    const int v = tid >= o ? tot[tid - o] : 0;
    __syncthreads();
    tot[tid] += v;
    __syncthreads();
  }
  int run = tot[tid] - s;
  for (int i = b0; i < b1; ++i) {
    off[i] = run;
    run += cnt[i];
    fill[i] = 0;
  }
}
__global__ __launch_bounds__(256) void k_lmin_bwd_fill(const float* __restrict__ coef, const int* __restrict__ idx,
                                                       int B, int swap, const int* __restrict__ off,
                                                       int* __restrict__ fill, int* __restrict__ list) {
  for (int k = blockIdx.x * 256 + threadIdx.x; k < B; k += gridDim.x * 256)
    for (int slot = 0; slot < 1 + swap; ++slot) {
      const int tg = src_target(coef, idx, k, slot, B);
      if (tg >= 0) list[off[tg] + atomicAdd(fill + tg, 1)] = k;  // unordered; the gather orders it
    }
}

// one wave per target row: t < B the anchor gradient of row t, else the positive gradient of row
// t - B; each lane holds 2 of the 128 dims.  Terms: the target's own entries, then every source
// whose selected negative lies in the target's row / column, in increasing source order.
__global__ __launch_bounds__(256) void k_lmin_bwd_gather(const float* __restrict__ a, const float* __restrict__ p,
                                                         int B, int swap, const float* __restrict__ coef,
                                                         const int* __restrict__ idx, const int* __restrict__ cnt,
                                                         const int* __restrict__ off, const int* __restrict__ list,
                                                         float* __restrict__ ga, float* __restrict__ gp) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t >= 2 * B) return;
  const bool anc = t < B;
  const int i = anc ? t : t - B;
  const float2* A2 = reinterpret_cast<const float2*>(a);
  const float2* P2 = reinterpret_cast<const float2*>(p);
  // self = the target row's own vector, other(j) = the partner row on the other side
  const float2 self = anc ? A2[(size_t)i * 64 + lane] : P2[(size_t)i * 64 + lane];
  auto other = [&](int j) { return anc ? P2[(size_t)j * 64 + lane] : A2[(size_t)j * 64 + lane]; };
  float2 acc = make_float2(0.f, 0.f);
  auto add = [&](float w, const float2& o) {  // w (2 self - 2 other)
    acc.x = fmaf(w, 2.0f * self.x - 2.0f * o.x, acc.x);
    acc.y = fmaf(w, 2.0f * self.y - 2.0f * o.y, acc.y);
  };
  const float cpos = coef[3 * i];
  if (cpos != 0.f) add(cpos, other(i));
  // anchor row i: its own row negative (i, r_i); positive row i: its own column negative (c_i, i)
  const float cown = coef[3 * i + (anc ? 1 : 2)];
  if (cown != 0.f) add(cown, other(idx[2 * i + (anc ? 0 : 1)]));
  // scattered terms: anchor i collects column negatives with c_k = i; positive j row negatives with r_k = j
  const int slot = anc ? 1 : 0;
  const int n = cnt[t];  // sources that selected an entry of this target (wave-uniform)
  if (n > 0 && n <= 64) {
    // the list in increasing source order: lane j holds source s_j, its rank = #{sources < s_j}
    const int sj = lane < n ? list[off[t] + lane] : 0x7fffffff;
    int rank = 0;
    for (int o = 0; o < n; ++o) rank += __shfl(sj, o, 64) < sj ? 1 : 0;
    for (int r = 0; r < n; ++r) {
      const unsigned long long m = __ballot(lane < n && rank == r);
      const int kk = __shfl(sj, __ffsll((unsigned long long)m) - 1, 64);
      add(coef[3 * kk + 1 + slot], other(kk));
    }
  } else if (n > 64) {  // a heavily selected target: every source, in order
    for (int k0 = 0; k0 < B; k0 += 64) {
      const int k = k0 + lane;
      const bool hit = k < B && idx[2 * k + slot] == i && coef[3 * k + 1 + slot] != 0.f;
      unsigned long long m = __ballot(hit);
      while (m) {
        const int kk = k0 + __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        add(coef[3 * kk + 1 + slot], other(kk));
      }
    }
  }
  float2* G = reinterpret_cast<float2*>(anc ? ga : gp);
  G[(size_t)i * 64 + lane] = acc;
}

}  // namespace

// saved layout (hn_loss_train_saved_bytes): sq [2B] f32 | rowbest [B] u64 | colbest [B] u64 |
// pos [B] f32 | posx [B] f32 (|a_i - p_i|^2) | coef [3B] f32 | idx [2B] i32 | cnt, off, fill, list [2B] i32
// (the backward's source lists)
size_t hn_loss_train_saved_bytes(long B) {
  auto al = [](size_t n) { return (n + 255) / 256 * 256; };
  return al(2 * B * 4) + 2 * al(B * 8) + 2 * al(B * 4) + al(3 * B * 4) + 5 * al(2 * B * 4);
}

namespace {
struct LossSaved {
  float* sq;
  unsigned long long *rowbest, *colbest;
  float* pos;
  float* posx;
  float* coef;
  int* idx;
  int *cnt, *off, *fill, *list;
};
LossSaved loss_saved(void* ws, long B) {
  auto al = [](size_t n) { return (n + 255) / 256 * 256; };
  char* c = static_cast<char*>(ws);
  LossSaved s;
  s.sq = reinterpret_cast<float*>(c);
  c += al(2 * B * 4);
  s.rowbest = reinterpret_cast<unsigned long long*>(c);
  c += al(B * 8);
  s.colbest = reinterpret_cast<unsigned long long*>(c);
  c += al(B * 8);
  s.pos = reinterpret_cast<float*>(c);
  c += al(B * 4);
  s.posx = reinterpret_cast<float*>(c);
  c += al(B * 4);
  s.coef = reinterpret_cast<float*>(c);
  c += al(3 * B * 4);
  s.idx = reinterpret_cast<int*>(c);
  c += al(2 * B * 4);
  s.cnt = reinterpret_cast<int*>(c);
  c += al(2 * B * 4);
  s.off = reinterpret_cast<int*>(c);
  c += al(2 * B * 4);
  s.fill = reinterpret_cast<int*>(c);
  c += al(2 * B * 4);
  s.list = reinterpret_cast<int*>(c);
  return s;
}
}  // namespace

hipError_t hn_launch_loss_train_fwd(const float* a, const float* p, int B, int swap, float margin, int type,
                                    float* loss, void* saved, hipStream_t st) {
  const LossSaved s = loss_saved(saved, B);
  hipLaunchKernelGGL(k_lmin_sq, dim3((2 * B + 3) / 4), dim3(256), 0, st, a, p, B, s.sq, s.pos, s.posx);
  if (swap) hipLaunchKernelGGL(k_lmin_init, dim3(std::min((B + 255) / 256, 1024)), dim3(256), 0, st, s.colbest, B);
  hipLaunchKernelGGL(k_lmin_tiles, dim3((B + TM - 1) / TM), dim3(256), 0, st, a, p, s.sq, B, swap, s.rowbest,
                     s.colbest, s.pos);
  hipLaunchKernelGGL(k_lmin_finish, dim3(1), dim3(1024), 0, st, s.rowbest, s.colbest, s.pos, B, swap, margin, type,
                     loss);
  return hipGetLastError();
}

hipError_t hn_launch_loss_train_bwd(const float* a, const float* p, int B, int swap, float margin, int type,
                                    const float* dloss, float* ga, float* gp, void* saved, hipStream_t st) {
  const LossSaved s = loss_saved(saved, B);
  hipLaunchKernelGGL(k_lmin_bwd_src, dim3((B + 255) / 256), dim3(256), 0, st, a, p, s.sq, s.rowbest, s.colbest,
                     s.pos, s.posx, B, swap, margin, type, dloss, s.coef, s.idx);
  const int g = std::min((B + 255) / 256, 2048);
  if (hipError_t e = hipMemsetAsync(s.cnt, 0, sizeof(int) * 2 * (size_t)B, st)) return e;
  hipLaunchKernelGGL(k_lmin_bwd_count, dim3(g), dim3(256), 0, st, s.coef, s.idx, B, swap, s.cnt);
  hipLaunchKernelGGL(k_lmin_bwd_scan, dim3(1), dim3(1024), 0, st, s.cnt, 2 * B, s.off, s.fill);
  hipLaunchKernelGGL(k_lmin_bwd_fill, dim3(g), dim3(256), 0, st, s.coef, s.idx, B, swap, s.off, s.fill, s.list);
  hipLaunchKernelGGL(k_lmin_bwd_gather, dim3((2 * B + 3) / 4), dim3(256), 0, st, a, p, B, swap, s.coef, s.idx, s.cnt,
                     s.off, s.list, ga, gp);
  return hipGetLastError();
}
