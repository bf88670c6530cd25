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

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace {

// min(v[l], v[l ^ 32]) with v_permlane32_swap (VALU; __shfl_xor(v, 32) is an LDS ds_bpermute round
// trip on the epilogue's critical path)
HN_DEV float half_swap_min(float v) {
  const unsigned u = __float_as_uint(v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fminf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

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
// ---------------------------------------------------------------------------------------
// MFMA version, over a block of anchor rows (the whole matrix on one GPU, or one rank's row
// shard of it when the batch is sharded -- SURVEY.md 8(e), config 5 at scale).
//
// x(i,j) = (|a_i|^2 + |p_j|^2) - 2 a_i.p_j with the dot on the bf16 MFMA in bf16x3 split
// precision.  dm = sqrt(x + 1e-6) + 1e-8 is monotone in x, so minima are tracked on x: per
// anchor row the min over unmasked entries (xu) and over the +10 entries (the diagonal and
// dm < 0.008, xm); min_neg = min(dm(xu), dm(xm) + 10) -- the reference's min over
// dm + 10*eye + 10*[dm + 10*eye < 0.008] (Losses.py:95-105).  The 0.008 test is done on x
// against the exact float threshold X* (mask_threshold_x: dm(x) < 0.008 <=> x < X* in fp32),
// so the epilogue has no sqrt; without anchor_swap it runs on y = x - |a_i|^2 (one FMA per
// entry, threshold X* - |a_i|^2 per row).  Wave-uniform "edge" tiles (the diagonal, ragged
// rows / columns) take a checked path.  Column minima (anchor_swap, Losses.py:106-108) are
// reduced over the workgroup's 4 waves in LDS, then one atomicMin per column per workgroup.
// pos (the diagonal) is recomputed in exact fp32 by k_pos.  One workgroup = 128 anchors (4
// waves x 32, A fragments resident in registers) sweeping the positives in double-buffered
// LDS tiles of 64 (rows padded to 272 B: conflict-free ds_read_b128).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float dm_of(float x) { return sqrtf(fmaxf(x + 1e-6f, 0.f)) + 1e-8f; }

__global__ __launch_bounds__(256) void k_sq(const float* __restrict__ v, int B, float* __restrict__ sq) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= B) return;
  const float a0 = v[(size_t)i * 128 + lane], a1 = v[(size_t)i * 128 + 64 + lane];
  const float s = wave_sum(a0 * a0 + a1 * a1);
  if (lane == 0) sq[i] = s;
}

// pos[i] = dm(a_i, p_{row0 + i}) for the NA local anchors
__global__ __launch_bounds__(256) void k_pos(const float* __restrict__ a, const float* __restrict__ p,
                                             const float* __restrict__ asq, const float* __restrict__ psq,
                                             int NA, int row0, float* __restrict__ pos) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= NA) return;
  const size_t pj = (size_t)(row0 + i) * 128;
  const float d = wave_sum(a[(size_t)i * 128 + lane] * p[pj + lane] +
                           a[(size_t)i * 128 + 64 + lane] * p[pj + 64 + lane]);
  if (lane == 0) pos[i] = dm_of((asq[i] + psq[row0 + i]) - 2.0f * d);
}

// NW waves per workgroup (32 anchors each): every workgroup streams all B positives through LDS,
// so the positives' L2/MALL traffic is B * 512 bytes per 32 * NW anchors -- 8 waves (one
// workgroup per CU, still two waves per SIMD) halve it against 4.
constexpr int kPdWaves = 8;
template <bool SWAP, int NW>
__global__ __launch_bounds__(NW * 64) void k_pairdist_rows(
    const float* __restrict__ a, int NA, int row0, const float* __restrict__ p, int B,
    const float* __restrict__ asq, const float* __restrict__ psq, float xthr,
    float* __restrict__ rowmin, unsigned* __restrict__ colmin) {
  constexpr int TN = 64, ROWB = 272, PLANE = TN * ROWB, BUF = 2 * PLANE + TN * 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  __shared__ float2 cred[3][NW][TN];  // per-wave squared column minima (unmasked, masked) of a tile (SWAP), tile % 3
  __shared__ __attribute__((aligned(16))) float ainit[NW][32];  // -|a_i|^2 / 2 per wave row
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int i0 = blockIdx.x * (32 * NW) + wave * 32;  // this wave's first local anchor
  const int g0 = row0 + i0;                     // ... and its global row
  // A fragments: lane (r, h) holds anchor i0+r (clamped), k = 16 ks + 8 h + j
  bf16x8 ah[8], al[8];
  {
    const int ia = min(i0 + r, NA - 1);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const float4 x0 = *reinterpret_cast<const float4*>(a + (size_t)ia * 128 + ks * 16 + h * 8);
      const float4 x1 = *reinterpret_cast<const float4*>(a + (size_t)ia * 128 + ks * 16 + h * 8 + 4);
      uint4 hi, lo;
      split8(x0, x1, hi, lo);
      ah[ks] = as_bf16x8(hi);
      al[ks] = as_bf16x8(lo);
    }
  }
  // every MFMA chain starts from -|a_i|^2 / 2 in the row of anchor i, so that
  // x = |p_j|^2 - 2 acc = |a_i|^2 + |p_j|^2 - 2 a_i.p_j is one FMA per entry and no per-row
  // value occupies registers; rows past NA start at -inf (x = +inf: they reach no minimum)
  if (lane < 32) ainit[wave][lane] = i0 + lane < NA ? -0.5f * asq[i0 + lane] : -INFINITY;
  float xu[16], xm[16];  // minima of x over unmasked / +10-masked entries
#pragma unroll
  for (int i = 0; i < 16; ++i) { xu[i] = INFINITY; xm[i] = INFINITY; }

  // P tile staging, in two halves of 32 rows (one per sub-tile, so few loads are in flight per
  // thread): thread -> row of the half, PQ consecutive float4; rows past B repeat row B - 1
  // (with its diagonal test done on the clamped column, a repeated column changes no minimum)
  constexpr int PQ = 1024 / (NW * 64);  // float4 per thread per half
  constexpr int TPR = 32 / PQ;          // threads per row
  const int srow = tid / TPR, scol = (tid % TPR) * PQ * 4;
  // the next tile's P rows in registers: with 8 waves both halves are loaded a whole tile (two
  // chains) before their store (measured 3.40 -> 3.33 ms at 65,536 pairs); the 4-wave form keeps
  // one half in flight per chain (its 8 more registers would cost the second wave per SIMD)
  constexpr bool DEEP = NW == 8;
  float4 pr[2][PQ];
  auto load_half = [&](int j0, int half) {
    const int jr = min(j0 + half * 32 + srow, B - 1);
#pragma unroll
    for (int q = 0; q < PQ; ++q) pr[half][q] = *reinterpret_cast<const float4*>(p + (size_t)jr * 128 + scol + q * 4);
  };
  auto store_half = [&](char* buf, int j0, int half) {
    const int row = half * 32 + srow;
#pragma unroll
    for (int q = 0; q < PQ; q += 2) {
      uint4 hi, lo;
      split8(pr[half][q], pr[half][q + 1], hi, lo);
      *reinterpret_cast<uint4*>(buf + row * ROWB + (scol + q * 4) * 2) = hi;
      *reinterpret_cast<uint4*>(buf + PLANE + row * ROWB + (scol + q * 4) * 2) = lo;
    }
    if (tid < 32) reinterpret_cast<float*>(buf + 2 * PLANE)[half * 32 + tid] = psq[min(j0 + half * 32 + tid, B - 1)];
  };
  // One 32-column sub-tile's MFMA chain (bf16x3, K = 128) with the epilogue of the previous
  // sub-tile woven into its gaps: two of that sub-tile's 16 accumulator entries per K-step become
  // x (pj = |p_j|^2 of this lane's column) and enter the lane's running minimum lm.  After the
  // chain, the sub-tile is "clean" unless it holds the diagonal (dsel = column - g0, -1000 when
  // it has none: accumulator row rr(i) is on it iff rr(i) == dsel) or some lane saw x < X*
  // (lm < xthr) -- both rare, and the test is wave-uniform.  A clean sub-tile has no +10 entry,
  // so its row minima are plain fmins and its column minimum is lm; otherwise the masked
  // form runs over the 16 kept x values.  B fragments are read one K-step ahead.
  float cu, cm;
  auto epi_masked = [&](const f32x16& xv, int dsel) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rr = (i & 3) + 8 * (i >> 2) + 4 * h;
      const float v = xv[i];
      const bool m = v < xthr || rr == dsel;
      const float tu = m ? INFINITY : v, tm = m ? v : INFINITY;
      xu[i] = fminf(xu[i], tu);
      xm[i] = fminf(xm[i], tm);
      if constexpr (SWAP) {
        cu = fminf(cu, tu);
        cm = fminf(cm, tm);
      }
    }
  };
  auto epi_finish = [&](const f32x16& xv, float lm, int dsel, int cslot) {
    cu = INFINITY;
    cm = INFINITY;
    if (__any(dsel != -1000 || lm < xthr)) {
      epi_masked(xv, dsel);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) xu[i] = fminf(xu[i], xv[i]);
      cu = lm;
    }
    if constexpr (SWAP) {
      cu = half_swap_min(cu);
      cm = half_swap_min(cm);
      if (h == 0) (&cred[0][0][0])[cslot + r] = make_float2(cu, cm);
    }
  };
  auto chain_epi = [&](const char* cur, int nt, f32x16 accp, float pj, int dsel, int cslot) {
    f32x16 acc;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // accumulator rows 8q + 4h + {0..3}
      const float4 v = *reinterpret_cast<const float4*>(&ainit[wave][8 * q + 4 * h]);
      acc[4 * q] = v.x;
      acc[4 * q + 1] = v.y;
      acc[4 * q + 2] = v.z;
      acc[4 * q + 3] = v.w;
    }
    float lm = INFINITY;
    const char* base = cur + (nt * 32 + r) * ROWB + h * 16;
    uint4 bh = *reinterpret_cast<const uint4*>(base);
    uint4 bl = *reinterpret_cast<const uint4*>(base + PLANE);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      uint4 nh, nl;
      if (ks + 1 < 8) {
        nh = *reinterpret_cast<const uint4*>(base + (ks + 1) * 32);
        nl = *reinterpret_cast<const uint4*>(base + PLANE + (ks + 1) * 32);
      }
      acc = mfma3(ah[ks], al[ks], as_bf16x8(bh), as_bf16x8(bl), acc);
      accp[2 * ks] = fmaf(-2.0f, accp[2 * ks], pj);
      accp[2 * ks + 1] = fmaf(-2.0f, accp[2 * ks + 1], pj);
      lm = fminf(lm, fminf(accp[2 * ks], accp[2 * ks + 1]));
      if (ks + 1 < 8) {
        bh = nh;
        bl = nl;
      }
    }
    epi_finish(accp, lm, dsel, cslot);
    return acc;
  };
  auto epilogue = [&](f32x16 accp, float pj, int dsel, int cslot) {
    float lm = INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      accp[i] = fmaf(-2.0f, accp[i], pj);
      lm = fminf(lm, accp[i]);
    }
    epi_finish(accp, lm, dsel, cslot);
  };
  auto reduce_cols = [&](int t) {  // tile t's column minima over the 4 waves: one atomic per column
    const int j = t * TN + lane;
    const float2* c = cred[t % 3][0];
    float2 ce = c[lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float2 x = c[w * TN + lane];
      ce.x = fminf(ce.x, x.x);
      ce.y = fminf(ce.y, x.y);
    }
    // dm_of is monotone: the distance of the squared minimum is the minimum distance
    const float d = fminf(dm_of(ce.x), dm_of(ce.y) + 10.f);
    if (j < B && d < INFINITY) atomicMin(colmin + j, __float_as_uint(d));
  };
  auto sub_meta = [&](const float* ps, int j0, int nt, float& pj, int& dsel, int& cslot, int t) {
    const int jb = j0 + nt * 32;
    pj = ps[nt * 32 + r];
    // overlap of the wave's rows with the sub-tile's (clamped) columns
    const int jlo = min(jb, B - 1), jhi = min(jb + 31, B - 1);
    dsel = (jlo < g0 + 32 && jhi >= g0) ? min(jb + r, B - 1) - g0 : -1000;
    cslot = ((t % 3) * NW + wave) * TN + nt * 32;
  };

  const int ntile = (B + TN - 1) / TN;
  load_half(0, 0);
  store_half(smem, 0, 0);
  load_half(0, 1);
  store_half(smem, 0, 1);
  __syncthreads();
  // software pipeline over 32-column sub-tiles: the chain of sub-tile k runs beside the epilogue
  // of sub-tile k - 1 (a harmless empty one before the first)
  f32x16 accp{};
  float pjp = INFINITY;
  int dselp = -1000, cslotp = wave * TN + 32;  // (tile 0's slot: overwritten by the real sub-tile)
#pragma unroll 1
  for (int t = 0; t < ntile; ++t) {
    const char* cur = smem + (t & 1) * BUF;
    const int j0 = t * TN;
    const bool more = t + 1 < ntile;
    char* nxt = smem + ((t + 1) & 1) * BUF;
    if (SWAP && t >= 2 && wave == (t - 2) % NW) reduce_cols(t - 2);
    const float* ps = reinterpret_cast<const float*>(cur + 2 * PLANE);
    if constexpr (DEEP) {  // both halves in flight across both chains
      if (more) {
        load_half(j0 + TN, 0);
        load_half(j0 + TN, 1);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        accp = chain_epi(cur, nt, accp, pjp, dselp, cslotp);
        sub_meta(ps, j0, nt, pjp, dselp, cslotp, t);
      }
      if (more) {
        store_half(nxt, j0 + TN, 0);
        store_half(nxt, j0 + TN, 1);
      }
    } else {  // one half in flight per chain
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        if (more) load_half(j0 + TN, nt);
        accp = chain_epi(cur, nt, accp, pjp, dselp, cslotp);
        sub_meta(ps, j0, nt, pjp, dselp, cslotp, t);
        if (more) store_half(nxt, j0 + TN, nt);
      }
    }
    __syncthreads();
  }
  epilogue(accp, pjp, dselp, cslotp);
  if (SWAP) {
    __syncthreads();
    if (ntile >= 2 && wave == (ntile - 2) % NW) reduce_cols(ntile - 2);
    if (wave == (ntile - 1) % NW) reduce_cols(ntile - 1);
  }
  // row minima: reduce over the 32 lanes of each half-wave (the columns)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float u = xu[i], m = xm[i];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      u = fminf(u, __shfl_xor(u, o, 64));
      m = fminf(m, __shfl_xor(m, o, 64));
    }
    const int row = i0 + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (r == 0 && row < NA) rowmin[row] = fminf(dm_of(u), dm_of(m) + 10.f);
  }
}

// ---------------------------------------------------------------------------------------
// The same computation with the positives pre-split ONCE (k_split_planes: bf16 hi / lo planes
// [B][128] in the workspace) and staged by LDS-DMA (global_load_lds, 16 B per lane) into a ring
// of three tile buffers: no register staging, no per-tile split, two tiles in flight while the
// waves compute on the third.  A buffer's rows are 256 B, the 16-byte chunk c of row j stored at
// chunk c ^ (j & 15) (the swizzle is applied on the per-lane SOURCE address, the LDS image being
// lane-linear), so each 16-lane ds_read_b128 group of a B-fragment read (16 consecutive rows, one
// logical chunk) hits 16 distinct chunks: conflict-free.  Each buffer is its own __shared__ object
// and the tile loop is unrolled by three, so every ds_read names its buffer at compile time and
// hipcc does not wait for the in-flight DMA into the other buffers; the waits are counted
// s_waitcnt vmcnt(N) (N = this wave's DMA instructions for the tile issued after the one to
// retire) followed by a raw s_barrier.
// ---------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* lds_ptr_t;


__global__ __launch_bounds__(256) void k_split_planes(const float* __restrict__ p, int B, uint16_t* __restrict__ ph,
                                                      uint16_t* __restrict__ pl) {
  const long e = ((long)blockIdx.x * 256 + threadIdx.x) * 8;  // 8 consecutive values per thread
  if (e >= (long)B * 128) return;
  const float4 x0 = *reinterpret_cast<const float4*>(p + e), x1 = *reinterpret_cast<const float4*>(p + e + 4);
  uint4 hi, lo;
  split8(x0, x1, hi, lo);
  *reinterpret_cast<uint4*>(ph + e) = hi;
  *reinterpret_cast<uint4*>(pl + e) = lo;
}

template <int N>
HN_DEV void wait_vm() {  // s_waitcnt vmcnt(N), lgkmcnt / expcnt untouched
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// ABL (timing only, experiments library, HN_PAIRDIST_ABL): bit 0 no epilogue (the distance / minimum VALU and
// the masked path), bit 1 no positive-tile DMA after the prologue (stale tiles), bit 2 no MFMAs
// SPREAD: the next-but-one tile's DMA issued inside the first sub-tile's MFMA chain instead of before it
template <bool SWAP, int NW, int ABL = 0, bool SPREAD = false>
__global__ __launch_bounds__(NW * 64) void k_pairdist_ring(
    const float* __restrict__ a, int NA, int row0, const uint16_t* __restrict__ ph, const uint16_t* __restrict__ pl,
    int B, const float* __restrict__ asq, const float* __restrict__ psq, float xthr, float* __restrict__ rowmin,
    unsigned* __restrict__ colmin) {
  constexpr int TN = 64, ROWB = 256, PLANE = TN * ROWB, BUF = 2 * PLANE + TN * 4;
  constexpr int G = 2 * PLANE / 1024 / NW;  // DMA instructions per wave per tile (4 at NW = 8)
  static_assert(G * NW * 1024 == 2 * PLANE, "tile split");
  __shared__ __attribute__((aligned(16))) char sb0[BUF], sb1[BUF], sb2[BUF];
  __shared__ float2 cred[3][NW][TN];
  __shared__ float xms[NW][16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int i0 = blockIdx.x * (32 * NW) + wave * 32;
  const int g0 = row0 + i0;
  bf16x8 ah[8], al[8];
  {
    const int ia = min(i0 + r, NA - 1);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const float4 x0 = *reinterpret_cast<const float4*>(a + (size_t)ia * 128 + ks * 16 + h * 8);
      const float4 x1 = *reinterpret_cast<const float4*>(a + (size_t)ia * 128 + ks * 16 + h * 8 + 4);
      uint4 hi, lo;
      split8(x0, x1, hi, lo);
      ah[ks] = as_bf16x8(hi);
      al[ks] = as_bf16x8(lo);
    }
  }
  // row minima of the unmasked entries in registers; those of the masked entries (rare: only the
  // masked sub-tiles touch them) in LDS, each lane its own 16 slots, so that the common epilogue
  // path and the masked one leave the same registers live (no per-sub-tile copies at the join)
  // -|a_i|^2 / 2 of this lane's 16 accumulator rows: every chain starts from it
  f32x16 areg;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int ia = i0 + (i & 3) + 8 * (i >> 2) + 4 * h;
    areg[i] = ia < NA ? -0.5f * asq[ia] : -INFINITY;
  }
  float xu[16];
  float* xm = &xms[wave][0][lane];
#pragma unroll
  for (int i = 0; i < 16; ++i) { xu[i] = INFINITY; xm[64 * i] = INFINITY; }

  // tile j0's rows (clamped to B - 1) into a buffer: wave instruction gi = wave * G + k covers plane
  // gi / 16, rows 4 (gi % 16) .. +3; lane L fills row 4 (gi % 16) + L / 16, chunk L % 16 with the
  // row's logical chunk (L % 16) ^ (row & 15); wave 0 adds |p_j|^2 of the 64 rows (4 B per lane)
  // The DMA goes through inline asm (the guide's glds16 recipe: M0 set and restored in the same
  // statement), so hipcc does not track it as a pending LDS write: its alias analysis would
  // otherwise wait vmcnt(0) before LDS reads of the other buffers; the waits here are explicit.
  const unsigned wv = __builtin_amdgcn_readfirstlane(wave);
  // DMA instruction k of this wave's share of tile j0 (k = G: wave 0's |p|^2 piece)
  auto issue_piece = [&](char* buf, int j0, int k) {
    if constexpr ((ABL & 2) != 0) {
      if (j0 >= 2 * TN) return;
    }
    if (k == G) {
      if (wv == 0) {
        const float* src = psq + min(j0 + lane, B - 1);
        const unsigned dst = (unsigned)(uintptr_t)(lds_ptr_t)(buf + 2 * PLANE);
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
      }
      return;
    }
    {
      const int gi = wave * G + k, plane = gi >> 4, r4 = (gi & 15) * 4;
      const int row = r4 + (lane >> 4), d = lane & 15;
      const int jr = min(j0 + row, B - 1);
      const uint16_t* src = (plane ? pl : ph) + (size_t)jr * 128 + ((d ^ (row & 15)) << 3);
      const int gu = (int)wv * G + k;
      const unsigned dst = (unsigned)(uintptr_t)(lds_ptr_t)(buf + (gu >> 4) * PLANE + (gu & 15) * 4 * ROWB);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
    }
  };
  auto issue = [&](char* buf, int j0) {
    if constexpr ((ABL & 2) != 0) {
      if (j0 >= 2 * TN) return;
    }
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int gi = wave * G + k, plane = gi >> 4, r4 = (gi & 15) * 4;
      const int row = r4 + (lane >> 4), d = lane & 15;
      const int jr = min(j0 + row, B - 1);
      const uint16_t* src = (plane ? pl : ph) + (size_t)jr * 128 + ((d ^ (row & 15)) << 3);
      const int gu = (int)wv * G + k;
      const unsigned dst = (unsigned)(uintptr_t)(lds_ptr_t)(buf + (gu >> 4) * PLANE + (gu & 15) * 4 * ROWB);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
    }
    if (wv == 0) {
      const float* src = psq + min(j0 + lane, B - 1);
      const unsigned dst = (unsigned)(uintptr_t)(lds_ptr_t)(buf + 2 * PLANE);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
    }
  };
  // this wave's share of the older tile's DMA retired, then every wave's (LDS reads of the buffer
  // about to be refilled are complete before the barrier: lgkmcnt(0))
  auto sync_tile = [&](bool more) {
    if (more) {
      if (wv == 0) wait_vm<G + 1>(); else wait_vm<G>();
    } else {
      wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  float cu, cm;
  auto epi_masked = [&](const f32x16& xv, int dsel) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rr = (i & 3) + 8 * (i >> 2) + 4 * h;
      const float v = xv[i];
      const bool m = v < xthr || rr == dsel;
      const float tu = m ? INFINITY : v, tm = m ? v : INFINITY;
      xu[i] = fminf(xu[i], tu);
      xm[64 * i] = fminf(xm[64 * i], tm);
      if constexpr (SWAP) {
        cu = fminf(cu, tu);
        cm = fminf(cm, tm);
      }
    }
  };
  auto epi_finish = [&](const f32x16& xv, float lm, int dsel, int cslot) {
    cu = INFINITY;
    cm = INFINITY;
    if (__any(dsel != -1000 || lm < xthr)) {
      epi_masked(xv, dsel);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) xu[i] = fminf(xu[i], xv[i]);
      cu = lm;
    }
    if constexpr (SWAP) {
      cu = half_swap_min(cu);
      cm = half_swap_min(cm);
      if (h == 0) (&cred[0][0][0])[cslot + r] = make_float2(cu, cm);
    }
  };
  // one 32-column sub-tile's bf16x3 chain (K = 128) with the previous sub-tile's epilogue woven in
  auto chain_epi = [&](const char* cur, int nt, f32x16 accp, float pj, int dsel, int cslot, auto hook) {
    f32x16 acc = areg;
    float lm = INFINITY;
    const int row = nt * 32 + r, sw = row & 15;
    const char* base = cur + row * ROWB;
    uint4 bh = *reinterpret_cast<const uint4*>(base + ((h ^ sw) << 4));
    uint4 bl = *reinterpret_cast<const uint4*>(base + PLANE + ((h ^ sw) << 4));
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      uint4 nh, nl;
      if (ks + 1 < 8) {
        const int off = ((2 * (ks + 1) + h) ^ sw) << 4;
        nh = *reinterpret_cast<const uint4*>(base + off);
        nl = *reinterpret_cast<const uint4*>(base + PLANE + off);
      }
      if constexpr ((ABL & 4) != 0)
        acc[ks] += __builtin_bit_cast(float, bh.x ^ bl.y);
      else
        acc = mfma3(ah[ks], al[ks], as_bf16x8(bh), as_bf16x8(bl), acc);
      hook(ks);
      if constexpr ((ABL & 1) != 0) {
        if (ks + 1 < 8) {
          bh = nh;
          bl = nl;
        }
        continue;
      }
      accp[2 * ks] = fmaf(-2.0f, accp[2 * ks], pj);
      accp[2 * ks + 1] = fmaf(-2.0f, accp[2 * ks + 1], pj);
      lm = fminf(lm, fminf(accp[2 * ks], accp[2 * ks + 1]));
      if (ks + 1 < 8) {
        bh = nh;
        bl = nl;
      }
    }
    if constexpr ((ABL & 1) == 0) epi_finish(accp, lm, dsel, cslot);
    else xu[0] = fminf(xu[0], accp[0]);
    return acc;
  };
  auto reduce_cols = [&](int t) {
    const int j = t * TN + lane;
    const float2* c = cred[t % 3][0];
    float2 ce = c[lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float2 x = c[w * TN + lane];
      ce.x = fminf(ce.x, x.x);
      ce.y = fminf(ce.y, x.y);
    }
    // dm_of is monotone: the distance of the squared minimum is the minimum distance
    const float d = fminf(dm_of(ce.x), dm_of(ce.y) + 10.f);
    if (j < B && d < INFINITY) atomicMin(colmin + j, __float_as_uint(d));
  };
  auto sub_meta = [&](const float* ps, int j0, int nt, float& pj, int& dsel, int& cslot, int t) {
    const int jb = j0 + nt * 32;
    pj = ps[nt * 32 + r];
    const int jlo = min(jb, B - 1), jhi = min(jb + 31, B - 1);
    dsel = (jlo < g0 + 32 && jhi >= g0) ? min(jb + r, B - 1) - g0 : -1000;
    cslot = ((t % 3) * NW + wave) * TN + nt * 32;
  };

  const int ntile = (B + TN - 1) / TN;
  f32x16 accp{};
  float pjp = INFINITY;
  int dselp = -1000, cslotp = wave * TN + 32;
  // prologue: tiles 0 and 1 in flight, wait for tile 0
  issue(sb0, 0);
  if (ntile > 1) issue(sb1, TN);
  sync_tile(ntile > 1);
  // tile t on buffer t % 3 (compile-time within the unrolled step): tile t + 2's DMA goes into the
  // buffer tile t - 1 was read from (every wave passed the barrier after reading it)
  auto step = [&](const char* cur, char* nxt2, int t) {
    const int j0 = t * TN;
    if (SWAP && t >= 2 && wave == (t - 2) % NW) reduce_cols(t - 2);
    const bool more2 = t + 2 < ntile;
    const float* ps = reinterpret_cast<const float*>(cur + 2 * PLANE);
    if constexpr (SPREAD) {
      // tile t + 2's DMA spread over the first sub-tile's MFMA chain (the G pieces evenly behind its 8
      // mfma3, |p|^2 last), so the issue stalls of the two waves of a SIMD do not meet after the barrier
      accp = chain_epi(cur, 0, accp, pjp, dselp, cslotp, [&](int ks) {
#pragma unroll
        for (int k = 0; k < G; ++k)
          if (more2 && (k * 8) / G == ks) issue_piece(nxt2, j0 + 2 * TN, k);
      });
      if (more2) issue_piece(nxt2, j0 + 2 * TN, G);
      sub_meta(ps, j0, 0, pjp, dselp, cslotp, t);
      accp = chain_epi(cur, 1, accp, pjp, dselp, cslotp, [](int) {});
      sub_meta(ps, j0, 1, pjp, dselp, cslotp, t);
    } else {
      if (more2) issue(nxt2, j0 + 2 * TN);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        accp = chain_epi(cur, nt, accp, pjp, dselp, cslotp, [](int) {});
        sub_meta(ps, j0, nt, pjp, dselp, cslotp, t);
      }
    }
    sync_tile(more2);  // retire tile t + 1's DMA, leaving tile t + 2's in flight
  };
#pragma unroll 1
  for (int t = 0; t < ntile; t += 3) {
    step(sb0, sb2, t);
    if (t + 1 < ntile) step(sb1, sb0, t + 1);
    if (t + 2 < ntile) step(sb2, sb1, t + 2);
  }
  {  // the last sub-tile's epilogue
    float lm = INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      accp[i] = fmaf(-2.0f, accp[i], pjp);
      lm = fminf(lm, accp[i]);
    }
    epi_finish(accp, lm, dselp, cslotp);
  }
  if (SWAP) {
    __syncthreads();
    if (ntile >= 2 && wave == (ntile - 2) % NW) reduce_cols(ntile - 2);
    if (wave == (ntile - 1) % NW) reduce_cols(ntile - 1);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float u = xu[i], m = xm[64 * i];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      u = fminf(u, __shfl_xor(u, o, 64));
      m = fminf(m, __shfl_xor(m, o, 64));
    }
    const int row = i0 + (i & 3) + 8 * (i >> 2) + 4 * h;
    if (r == 0 && row < NA) rowmin[row] = fminf(dm_of(u), dm_of(m) + 10.f);
  }
}

// The margin losses of loss_HardNet (Losses.py:142-153) over the 'min' reduce, one workgroup
// (fixed summation order: deterministic); min_neg = min(row_min, col_min) when col_min is given.
__global__ __launch_bounds__(1024) void k_loss(const float* __restrict__ pos, const float* __restrict__ rmin,
                                               const float* __restrict__ cmin, int n, float margin,
                                               int type, float scale, float* __restrict__ min_neg,
                                               float* __restrict__ loss) {
  __shared__ float part[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const float mn = cmin ? fminf(rmin[i], cmin[i]) : rmin[i];
    if (min_neg) min_neg[i] = mn;
    const float ps = pos[i];
    float l;
    if (type == 0) {
      l = fmaxf(margin + ps - mn, 0.f);
    } else if (type == 1) {
      const float ep = expf(2.0f - ps);
      l = -logf(ep / (ep + expf(2.0f - mn) + 1e-8f));
    } else {
      l = fmaxf(margin - mn, 0.f) + ps;
    }
    s += l;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += part[w];
    loss[0] = t * scale;
  }
}

// X*: the smallest fp32 x with sqrt(x + 1e-6) + 1e-8 >= 0.008 in fp32, so that the
// reference's mask test (dm < 0.008, Losses.py:101) is exactly x < X* (dm is monotone in x).
float mask_threshold_x() {
  auto masked = [](float x) {
    const float u = x + 1e-6f;
    return !(u >= 0.f) || std::sqrt(u) + 1e-8f < 0.008f;
  };
  uint32_t lo = 0, hi = 0x3f800000u;  // x = 0 is masked, x = 1 is not
  while (hi - lo > 1) {
    const uint32_t mid = lo + (hi - lo) / 2;
    float x;
    std::memcpy(&x, &mid, 4);
    (masked(x) ? lo : hi) = mid;
  }
  float x;
  std::memcpy(&x, &hi, 4);
  return x;
}

}  // namespace

// workspace: |a|^2 [NA] | |p|^2 [B] | (ring form) bf16 hi / lo planes of the positives [B][128] each
size_t hn_pairdist_rows_ws_bytes(long NA, long B) {
  return (size_t)((NA + 63) / 64 * 64 + (B + 63) / 64 * 64) * sizeof(float) + (size_t)B * 128 * 2 * sizeof(uint16_t);
}

hipError_t hn_launch_pairdist_rows(const float* a, int NA, int row0, const float* p, int B, float* pos,
                                   float* rowmin, float* colmin, void* ws, hipStream_t st) {
  float* asq = static_cast<float*>(ws);
  float* psq = asq + ((NA + 63) / 64) * 64;
  uint16_t* ph = reinterpret_cast<uint16_t*>(psq + ((B + 63) / 64) * 64);
  uint16_t* pl = ph + (size_t)B * 128;
  static const float xthr = mask_threshold_x();
  if (colmin) hipLaunchKernelGGL(k_colmin_init, dim3((B + 255) / 256), dim3(256), 0, st,
                                 reinterpret_cast<unsigned*>(colmin), B);
  hipLaunchKernelGGL(k_sq, dim3((NA + 3) / 4), dim3(256), 0, st, a, NA, asq);
  hipLaunchKernelGGL(k_sq, dim3((B + 3) / 4), dim3(256), 0, st, p, B, psq);
  hipLaunchKernelGGL(k_pos, dim3((NA + 3) / 4), dim3(256), 0, st, a, p, asq, psq, NA, row0, pos);
  const bool ring = !hn_knobs().pairdist_reg;  // HN_PAIRDIST_REG=1: the register-staged form
  if (ring)
    hipLaunchKernelGGL(k_split_planes, dim3((unsigned)(((long)B * 16 + 255) / 256)), dim3(256), 0, st, p, B, ph, pl);
  // 8-wave workgroups when they still give every CU one (NA >= 65,536 anchors), else 4-wave
  // ones (twice the workgroups: a row shard of a sharded batch)
  auto go = [&](auto nw) {
    constexpr int NW = decltype(nw)::value;
    const dim3 grid((NA + 32 * NW - 1) / (32 * NW)), block(64 * NW);
    unsigned* cm = reinterpret_cast<unsigned*>(colmin);
    const bool spread = hn_knobs().pairdist_spread;
#ifdef HN_EXPERIMENTS
    const char* abl_e = std::getenv("HN_PAIRDIST_ABL");
    const int abl = abl_e ? std::atoi(abl_e) : 0;
    if (ring && colmin && abl > 0) {
      switch (abl) {
        case 1: hipLaunchKernelGGL((k_pairdist_ring<true, NW, 1>), grid, block, 0, st, a, NA, row0, ph, pl, B, asq, psq, xthr, rowmin, cm); break;
        case 2: hipLaunchKernelGGL((k_pairdist_ring<true, NW, 2>), grid, block, 0, st, a, NA, row0, ph, pl, B, asq, psq, xthr, rowmin, cm); break;
        case 3: hipLaunchKernelGGL((k_pairdist_ring<true, NW, 3>), grid, block, 0, st, a, NA, row0, ph, pl, B, asq, psq, xthr, rowmin, cm); break;
        case 4: hipLaunchKernelGGL((k_pairdist_ring<true, NW, 4>), grid, block, 0, st, a, NA, row0, ph, pl, B, asq, psq, xthr, rowmin, cm); break;
        case 6: hipLaunchKernelGGL((k_pairdist_ring<true, NW, 6>), grid, block, 0, st, a, NA, row0, ph, pl, B, asq, psq, xthr, rowmin, cm); break;
      }
    } else
#endif
    if (ring && colmin && spread)
      hipLaunchKernelGGL((k_pairdist_ring<true, NW, 0, true>), grid, block, 0, st, a, NA, row0, ph, pl, B, asq, psq,
                         xthr, rowmin, cm);
    else if (ring && spread)
      hipLaunchKernelGGL((k_pairdist_ring<false, NW, 0, true>), grid, block, 0, st, a, NA, row0, ph, pl, B, asq, psq,
                         xthr, rowmin, nullptr);
    else if (ring && colmin)
      hipLaunchKernelGGL((k_pairdist_ring<true, NW>), grid, block, 0, st, a, NA, row0, ph, pl, B, asq, psq, xthr,
                         rowmin, cm);
    else if (ring)
      hipLaunchKernelGGL((k_pairdist_ring<false, NW>), grid, block, 0, st, a, NA, row0, ph, pl, B, asq, psq, xthr,
                         rowmin, nullptr);
    else if (colmin)
      hipLaunchKernelGGL((k_pairdist_rows<true, NW>), grid, block, 0, st, a, NA, row0, p, B, asq, psq, xthr,
                         rowmin, cm);
    else
      hipLaunchKernelGGL((k_pairdist_rows<false, NW>), grid, block, 0, st, a, NA, row0, p, B, asq, psq, xthr,
                         rowmin, nullptr);
  };
  if (NA >= 256 * 32 * kPdWaves)
    go(std::integral_constant<int, kPdWaves>{});
  else
    go(std::integral_constant<int, 4>{});
  return hipGetLastError();
}

hipError_t hn_launch_pairdist(const float* a, const float* p, int B, int D_, int swap,
                              float* pos, float* minneg, void* ws, hipStream_t st) {
  if (D_ != D) return hipErrorInvalidValue;
  unsigned* cm = static_cast<unsigned*>(ws);
  const unsigned g = (B + 255) / 256;
  const bool valu = hn_knobs().pairdist_valu;  // HN_PAIRDIST_VALU (A/B), read once per process
  if (!valu) {
    float* colmin = swap ? reinterpret_cast<float*>(cm) : nullptr;
    hipError_t e = hn_launch_pairdist_rows(a, B, 0, p, B, pos, minneg, colmin, cm + ((B + 63) / 64) * 64, st);  // (ws: hn_pairdist_rows_ws_bytes)
    if (e != hipSuccess) return e;
    if (swap) hipLaunchKernelGGL(k_combine, dim3(g), dim3(256), 0, st, minneg, cm, B);
    return hipGetLastError();
  }
  if (swap) hipLaunchKernelGGL(k_colmin_init, dim3(g), dim3(256), 0, st, cm, B);
  hipLaunchKernelGGL(k_pairdist, dim3((B + TM - 1) / TM), dim3(256), 0, st, a, p, B, swap, pos,
                     minneg, cm);
  if (swap) hipLaunchKernelGGL(k_combine, dim3(g), dim3(256), 0, st, minneg, cm, B);
  return hipGetLastError();
}

hipError_t hn_launch_loss(const float* pos, const float* rmin, const float* cmin, int n, float margin,
                          int type, float scale, float* min_neg, float* loss, hipStream_t st) {
  hipLaunchKernelGGL(k_loss, dim3(1), dim3(1024), 0, st, pos, rmin, cmin, n, margin, type, scale, min_neg,
                     loss);
  return hipGetLastError();
}
