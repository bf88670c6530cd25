// C ABI of the MI355X descriptor forward (include/hardnet_mi355x.h).
//
// Host-side responsibilities: validate the architecture and the flat parameter blob,
// fold eval-mode BatchNorm into conv weight + bias (in double), pack weights into the
// device layouts the kernels consume, and sequence the kernel launches of one forward
// on the caller's stream over fixed-size patch chunks.
#include "hardnet_mi355x.h"
#include "hn_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

static thread_local std::string g_err;

// ---------------------------------------------------------------------------------------
// launcher knobs and the per-device occupancy cache (hn_internal.h)
// ---------------------------------------------------------------------------------------
static int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

void hn_read_knobs(HnKnobs* k) {
  *k = HnKnobs{};
  k->c12_cfg = env_int("HN_C12_CFG", 15);
  k->head = std::getenv("HN_HEAD_V1") ? 1 : env_int("HN_HEAD", 4);
  k->head_pf = env_int("HN_HEAD_PF", 1) != 0;
  k->fdl_valu = std::getenv("HN_FDL_VALU") != nullptr;
  k->naive_pw = std::getenv("HN_NAIVE_PW") != nullptr;
  k->naive_dw = std::getenv("HN_NAIVE_DW") != nullptr;
  k->no_skipfuse = std::getenv("HN_NO_SKIPFUSE") != nullptr;
  k->no_irfskip = std::getenv("HN_NO_IRFSKIP") != nullptr;
  k->pairdist_valu = std::getenv("HN_PAIRDIST_VALU") != nullptr;
  k->pairdist_reg = env_int("HN_PAIRDIST_REG", 0) != 0;
  k->pairdist_spread = env_int("HN_PAIRDIST_SPREAD", 1) != 0;
  k->front_fold = env_int("HN_FRONT_FOLD", 0) != 0;
  k->u8_apart = env_int("HN_U8_APART", 0) != 0;
  k->front_xch3 = env_int("HN_FRONT_XCH3", 0) != 0;
  k->no_mpfront = env_int("HN_NO_MPFRONT", 0) != 0;
  k->pipeline = env_int("HN_PIPELINE", 0) != 0;

  k->train_splitk = std::max(32, env_int("HN_TRAIN_SPLITK", 1024)) / 32 * 32;
  k->train_f32 = env_int("HN_TRAIN_F32", 17) & 255;
#ifdef HN_EXPERIMENTS
  k->c12_abl = env_int("HN_C12_ABL", 0) & 4095;  // (65: k_c12s stamps with P1 on the A-waves)
  k->c12w_pd = env_int("HN_C12W_PD", 11);
  k->dbg = env_int("HN_DEBUG", 0);
  k->irf3 = env_int("HN_IRF3", 0) != 0;
#endif
}

static thread_local const HnKnobs* tl_knobs = nullptr;

const HnKnobs& hn_knobs() {
  if (tl_knobs) return *tl_knobs;
  static std::once_flag once;
  static HnKnobs process;
  std::call_once(once, [] { hn_read_knobs(&process); });
  return process;
}

namespace {
struct KnobScope {  // makes a model's knobs current on this thread for one API call
  const HnKnobs* prev;
  explicit KnobScope(const HnKnobs* k) : prev(tl_knobs) { tl_knobs = k; }
  ~KnobScope() { tl_knobs = prev; }
};
}  // namespace

hipError_t hn_resident_blocks(const void* fn, int nthreads, int lds, int* resident) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find({fn, dev});
  if (it != cache.end()) {
    *resident = it->second;
    return hipSuccess;
  }
  if (lds > 0 && (e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds)) != hipSuccess)
    return e;
  int per_cu = 0, cus = 0;
  if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, nthreads, lds)) != hipSuccess) return e;
  if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
  const int r = std::max(1, per_cu) * std::max(1, cus);
  cache[{fn, dev}] = r;
  *resident = r;
  return hipSuccess;
}

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess)                                                                  \
      return fail(HN_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_));             \
  } while (0)

// candidate op table, restating hardnetNAS/fbnet_building_blocks/fbnet_builder.py:36-191
// for CANDIDATE_BLOCKS (lookup_table_builder.py:18-20), in that index order.
const HnOpSpec kHnOps[17] = {
    {"skip", 1, 0, 0, 0, 0},        {"ir_k3_e1", 0, 1, 3, 1, 0},    {"ir_k3_e3", 0, 3, 3, 1, 0},
    {"ir_k3_s4", 0, 4, 3, 4, 0},    {"ir_k5_e1", 0, 1, 5, 1, 0},    {"ir_k5_e3", 0, 3, 5, 1, 0},
    {"ir_k5_s4", 0, 4, 5, 4, 0},    {"ir_k3_e1_se", 0, 1, 3, 1, 1}, {"ir_k3_e3_se", 0, 3, 3, 1, 1},
    {"ir_k3_s4_se", 0, 4, 3, 4, 1}, {"ir_k5_e1_se", 0, 1, 5, 1, 1}, {"ir_k5_e3_se", 0, 3, 5, 1, 1},
    {"ir_k5_s4_se", 0, 4, 5, 4, 1}, {"ir_k3_s2", 0, 1, 3, 2, 0},    {"ir_k5_s2", 0, 1, 5, 2, 0},
    {"ir_k3_s2_se", 0, 1, 3, 2, 1}, {"ir_k5_s2_se", 0, 1, 5, 2, 1},
};

namespace {

using OpSpec = HnOpSpec;
const OpSpec* const kOps = kHnOps;

struct NasLayer {
  int op = 0, cin = 0, cout = 0, stride = 1, hin = 0, hout = 0;
  int skip = 0, e = 1, k = 3, g = 1, se = 0, mid = 0, semid = 0;
  int skip_conv = 0;  // skip op with a 1x1 ConvBNRelu (C changes)
  float *pw_w = nullptr, *pw_b = nullptr, *dw_w = nullptr, *dw_b = nullptr;
  float *pwl_w = nullptr, *pwl_b = nullptr;
  float *se_w1 = nullptr, *se_b1 = nullptr, *se_w2 = nullptr, *se_b2 = nullptr;
  uint16_t* front_a = nullptr;  // fused front (layer 0): pw as MFMA A operand, dw channel order
  uint16_t* front_pwl16 = nullptr;  // fused front: pwl as 16x16x32 A operands
  float* front_b = nullptr;
  uint16_t *irf_pw_a = nullptr, *irf_pwl_a = nullptr;  // fused IRF block (layers >= 1)
  uint16_t* skip_a = nullptr;  // the 64 -> 128 skip's 1x1 weights as 32x32x16 fp16 hi / lo A fragments (k_irf_skip)
  float* irf_pw_b = nullptr;
};

struct Cursor {
  const float* p;
  size_t n, i = 0;
  bool ok = true;
  const float* take(size_t k) {
    if (i + k > n) {
      ok = false;
      return nullptr;
    }
    const float* r = p + i;
    i += k;
    return r;
  }
};

uint16_t f2bf(float x) {  // round-to-nearest-even, as v_cvt_pk_bf16_f32
  uint32_t u;
  std::memcpy(&u, &x, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// eval BatchNorm folded into the preceding bias-free conv:
//   y = (conv(x) - mean) * gamma / sqrt(var + eps) + beta
struct Folded {
  std::vector<float> w, b;
};
Folded fold(const float* w, size_t per_out, int cout, const float* gamma, const float* beta,
            const float* mean, const float* var, float eps) {
  Folded f;
  f.w.resize((size_t)cout * per_out);
  f.b.resize(cout);
  for (int n = 0; n < cout; ++n) {
    const double sc = (gamma ? (double)gamma[n] : 1.0) / std::sqrt((double)var[n] + (double)eps);
    for (size_t j = 0; j < per_out; ++j)
      f.w[(size_t)n * per_out + j] = (float)((double)w[(size_t)n * per_out + j] * sc);
    f.b[n] = (float)((beta ? (double)beta[n] : 0.0) - (double)mean[n] * sc);
  }
  return f;
}

struct Prof {
  bool on = false;
  struct Pend {
    int stage;
    hipEvent_t a, b;
  };
  std::vector<hipEvent_t> pool;
  std::vector<Pend> pend;
  std::vector<std::string> names;
  std::vector<double> ms;
  std::vector<int64_t> cnt;
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
  int stage_id(const char* name) {
    for (size_t i = 0; i < names.size(); ++i)
      if (names[i] == name) return (int)i;
    names.emplace_back(name);
    ms.push_back(0.0);
    cnt.push_back(0);
    return (int)names.size() - 1;
  }
  ~Prof() {
    for (auto& p : pend) {
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

}  // namespace

struct hn_model {
  Prof prof;
  HnKnobs knobs;  // launcher A/B switches, read once at hn_create
  hn_arch_desc desc{};
  int device = 0;
  std::vector<void*> allocs;
  HardnetDev hd;
  float *stem_w = nullptr, *stem_b = nullptr;  // NAS stem
  float *fdl_w1 = nullptr, *fdl_b1 = nullptr, *fdl_w2 = nullptr, *fdl_b2 = nullptr;  // FDL front 1x1s
  std::vector<NasLayer> layers;
  float *head_w = nullptr, *head_b = nullptr;  // NAS head
  uint16_t* head_pack = nullptr;               // NAS head as fp16x3 MFMA B operand (K = 2048)
  int head_k = 0;
  int chunk = 32768;
  bool unfused_stem = false;  // HN_UNFUSED_STEM=1: separate stem kernel (A/B, debugging)
  bool c12 = true;            // fused stem+conv1+conv2 (k_c12); HN_NO_C12=1 -> separate kernels
  int subchunk = 65536;       // HardNet conv3..conv5 patches per launch (HN_SUBCHUNK)
  int c12group = 65536;       // HardNet k_c12 patches per launch (HN_C12_GROUP; >= the sub-chunk)
  int c4sub = 0;              // HardNet conv4 patches per launch inside a sub-chunk (HN_C4_SUB; 0: the sub-chunk)
  uint16_t* front_spack = nullptr;  // fused front: stem as MFMA A operand
  int front = 0;  // NAS: 1 = stem + layer-0 IRF pw/dw fused, 2 = stem + layer-0 maxpool fused
  bool no_front = false;  // HN_NO_FRONT=1: unfused NAS stem/layer 0 (A/B, debugging)
  bool no_irf = false;    // HN_NO_IRF=1: layer-by-layer pw/dw/pwl kernels (A/B, debugging)
  bool no_irf2 = false;   // HN_NO_IRF2=1: one k_irf launch per block (no two-block fusion)
  // conv tiling per layer (index 0 = stem+conv1, 2..5 = conv2..5); defaults are the best
  // measured on MI355X (tools/tune_variants.py); HN_VARIANT="003303" style override
  // 19 / 20 / 21 / 26 = 1-D Winograd F(2,3) (hn_wino1.hip; conv3 / conv5) with a weight ring of depth
  // 3 / 4 / 6 / 8 (same-box HardNet 5.25 Mpatches/s at 3 / 3, 5.40 at 6 / 6; conv3 at 8: 10.2 -> 9.9 ms,
  // conv5 flat past 6); conv4: 18 = two patches per stage on the 64-byte swizzled window (15) with the
  // outputs stored by the producer waves; 16 = the direct conv3 / conv5 with epilogue stores through LDS
  // (the forms before 19)
  int variant[6] = {6, 0, 5, 26, 18, 21};
  size_t ws_floats_per_patch = 0;  // per buffer
  int n_bufs = 0;
  // the chunk pipeline's second stream and events (created on first use; the mutex keeps one call's
  // record / wait sequence whole when several host threads share the model)
  hipStream_t st2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_ready[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr};
  std::mutex pipe_mu;

  template <class T>
  int upload(const std::vector<T>& v, T** out) {
    void* d = nullptr;
    if (hipMalloc(&d, v.size() * sizeof(T)) != hipSuccess)
      return fail(HN_ERR_NOMEM, "hipMalloc of parameters failed");
    allocs.push_back(d);
    HIPCHK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = static_cast<T*>(d);
    return HN_OK;
  }
  ~hn_model() {
    for (void* p : allocs) (void)hipFree(p);
    for (hipEvent_t e : {ev_fork, ev_ready[0], ev_ready[1], ev_free[0], ev_free[1]})
      if (e) (void)hipEventDestroy(e);
    if (st2) (void)hipStreamDestroy(st2);
  }
};

// ---------------------------------------------------------------------------------------
// parameter accounting
// ---------------------------------------------------------------------------------------
static int check_desc(const hn_arch_desc* d) {
  if (!d) return fail(HN_ERR_ARG, "desc is NULL");
  if (d->kind == HN_KIND_HARDNET) return HN_OK;
  const bool fdl = d->kind == HN_KIND_FDL_NASNET || d->kind == HN_KIND_FDL_NASNET01;
  if (d->kind != HN_KIND_NAS && !fdl) return fail(HN_ERR_ARG, "unknown desc->kind");
  if (d->n_layers < 1 || d->n_layers > HN_MAX_LAYERS)
    return fail(HN_ERR_ARG, "n_layers out of range");
  int hw = fdl ? 8 : 32, c = fdl ? 64 : 32;  // FDL: the fixed front leaves 8x8x64
  for (int i = 0; i < d->n_layers; ++i) {
    if (d->op[i] < 0 || d->op[i] >= 17) return fail(HN_ERR_ARG, "op index out of range");
    if (d->c_in[i] != c) return fail(HN_ERR_ARG, "c_in does not chain");
    if (d->stride[i] != 1 && d->stride[i] != 2) return fail(HN_ERR_ARG, "stride must be 1/2");
    if (d->c_out[i] % 4 || d->c_in[i] % 4 || d->c_out[i] > 256)
      return fail(HN_ERR_ARG, "channel counts must be multiples of 4 and <= 256");
    hw /= d->stride[i];
    c = d->c_out[i];
  }
  if (hw != 4) return fail(HN_ERR_ARG, "NAS head expects a 4x4 final map (SEARCH_SPACE2)");
  if (fdl && c != 128) return fail(HN_ERR_ARG, "FDL head expects 128 channels (des.py)");
  return HN_OK;
}

static size_t nas_layer_params(const hn_arch_desc* d, int i) {
  const OpSpec& s = kOps[d->op[i]];
  const size_t ci = d->c_in[i], co = d->c_out[i];
  if (s.skip) return ci == co ? 0 : ci * co + 4 * co;
  const size_t mid = ci * s.e;
  size_t n = mid * (ci / s.g) + 4 * mid;  // pw
  n += mid * s.k * s.k + 4 * mid;         // dw
  n += co * (mid / s.g) + 4 * co;         // pwl
  if (s.se) {
    const size_t m = co / 4 > 8 ? co / 4 : 8;
    n += m * co + m + co * m + co;
  }
  return n;
}

extern "C" int hn_param_count(const hn_arch_desc* desc, size_t* n_out) {
  int rc = check_desc(desc);
  if (rc) return rc;
  if (!n_out) return fail(HN_ERR_ARG, "n_out is NULL");
  if (desc->kind == HN_KIND_HARDNET) {
    // 7 convs: weights + running_mean + running_var (BN affine=False), HardNet.py:280-302
    *n_out = 1334560 + 2 * (32 + 32 + 64 + 64 + 128 + 128 + 128);
    return HN_OK;
  }
  size_t n = 32 * 9 + 4 * 32;  // first: ConvBNRelu(1, 32, 3)
  if (desc->kind == HN_KIND_FDL_NASNET)  // des.py:14-24: stem (+bias) + BN stats, 1x1 32 + BN, 1x1 64 + BN
    n = 32 * 9 + 32 + 2 * 32 + 32 * 32 + 4 * 32 + 64 * 32 + 4 * 64;
  else if (desc->kind == HN_KIND_FDL_NASNET01)  // stem (+bias), Identity(32, 64, 2) ConvBNRelu
    n = 32 * 9 + 32 + 64 * 32 + 4 * 64;
  for (int i = 0; i < desc->n_layers; ++i) n += nas_layer_params(desc, i);
  n += (size_t)128 * desc->c_out[desc->n_layers - 1] * 16 + 2 * 128;  // head conv + BN stats
  *n_out = n;
  return HN_OK;
}

// ---------------------------------------------------------------------------------------
// packing
// ---------------------------------------------------------------------------------------
// conv1..5 of HardNet as bf16x3 MFMA fragments: [cc][tap][ks][nt][plane][lane][8]
static std::vector<uint16_t> pack_conv3x3(const std::vector<float>& w, int cin, int cout) {
  const int ncc = cin / 32, ntot = cout / 32;
  std::vector<uint16_t> out((size_t)ncc * 9 * 2 * ntot * 2 * 64 * 8);
  size_t o = 0;
  for (int cc = 0; cc < ncc; ++cc)
    for (int tap = 0; tap < 9; ++tap)
      for (int ks = 0; ks < 2; ++ks)
        for (int nt = 0; nt < ntot; ++nt) {
          uint16_t* hi = &out[o];
          uint16_t* lo = &out[o + 64 * 8];
          for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; ++j) {
              const int n = nt * 32 + (lane & 31);
              const int c = cc * 32 + ks * 16 + (lane >> 5) * 8 + j;
              const float v = w[((size_t)n * cin + c) * 9 + tap];
              const uint16_t h = f2bf(v);
              hi[lane * 8 + j] = h;
              lo[lane * 8 + j] = f2bf(v - bf2f(h));
            }
          o += 2 * 64 * 8;
        }
  return out;
}

// head conv (kernel kk x kk over an NHWC map): GEMM k = (y*kk + x)*cin + c,
// fragments [ks][nt][plane][lane][8]
// folded weights whose fp16 hi half is not finite (|w| >= 65520 or NaN): counted while a model is
// packed (per calling thread), hn_create then fails instead of packing an infinite fragment
static thread_local long tl_f16_out_of_range = 0;
static void put_f16_split(float v, uint16_t* hi, uint16_t* lo) {  // hn_common.h split8_f16
  const _Float16 hv = (_Float16)v;
  if (!std::isfinite((float)hv)) ++tl_f16_out_of_range;
  const _Float16 lv = (_Float16)(v - (float)hv);
  std::memcpy(hi, &hv, 2);
  std::memcpy(lo, &lv, 2);
}

static std::vector<uint16_t> pack_head(const std::vector<float>& w, int cin, int kk, bool f16 = false) {
  const int K = cin * kk * kk;
  std::vector<uint16_t> out((size_t)(K / 16) * 4 * 2 * 64 * 8);
  size_t o = 0;
  for (int ks = 0; ks < K / 16; ++ks)
    for (int nt = 0; nt < 4; ++nt) {
      uint16_t* hi = &out[o];
      uint16_t* lo = &out[o + 64 * 8];
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int n = nt * 32 + (lane & 31);
          const int k = ks * 16 + (lane >> 5) * 8 + j;
          const int c = k % cin, yx = k / cin;
          const float v = w[((size_t)n * cin + c) * kk * kk + yx];
          if (f16) {
            put_f16_split(v, &hi[lane * 8 + j], &lo[lane * 8 + j]);
          } else {
            const uint16_t h = f2bf(v);
            hi[lane * 8 + j] = h;
            lo[lane * 8 + j] = f2bf(v - bf2f(h));
          }
        }
      o += 2 * 64 * 8;
    }
  return out;
}

// [cout][kg] -> [kg][cout]
static std::vector<float> transpose_pw(const std::vector<float>& w, int cout, int kg) {
  std::vector<float> t((size_t)kg * cout);
  for (int n = 0; n < cout; ++n)
    for (int k = 0; k < kg; ++k) t[(size_t)k * cout + n] = w[(size_t)n * kg + k];
  return t;
}


// Fused-front stem weights as the MFMA A operand: [plane hi/lo][lane][8] fp16, lane
// (r = l & 31 = output channel, h = l >> 5) holding taps 8h..8h+7 (taps >= 9 are zero).
// The fused front's stem as 32x32x16 A operands [op][plane hi/lo][lane][8] fp16, lane (channel
// r = l & 31, K slots 8 (l >> 5) ..): op 0 = the 9 taps in K slots 0..8 (one image row per MFMA);
// op 1 = the same taps shifted to K slots 3..11, so that one B operand holding the 4 x 3 input
// window of two adjacent rows (slot 3 dy + dx, dy = 0..3) feeds row y (op 0) and row y + 1 (op 1).
static std::vector<uint16_t> pack_front_stem(const Folded& f) {
  std::vector<uint16_t> a(2 * 2 * 64 * 8, 0);
  for (int op = 0; op < 2; ++op)
    for (int lane = 0; lane < 64; ++lane)
      for (int j = 0; j < 8; ++j) {
        const int r = lane & 31, tap = 8 * (lane >> 5) + j - 3 * op;
        uint16_t* d = &a[(size_t)op * 2 * 64 * 8];
        put_f16_split(tap >= 0 && tap < 9 ? f.w[(size_t)r * 9 + tap] : 0.f, &d[lane * 8 + j], &d[64 * 8 + lane * 8 + j]);
      }
  return a;
}

// Fused-front pw weights (fp16 hi/lo) as the MFMA A operand (rows = output channels in dw
// order, i.e. after ChannelShuffle(g); grouped conv densified with zeros):
// [MID/32][kstep][plane hi/lo][lane][8] fp16, lane (r = l & 31, h = l >> 5), element j
// multiplying stem channel kappa(16*kstep + 8h + j) -- the order in which the stem MFMA
// leaves its outputs in the lanes (C row (i & 3) + 8 (i >> 2) + 4h for i = 8*kstep + j).
static void pack_front(const Folded& f, int mid, int g, std::vector<uint16_t>* a,
                       std::vector<float>* bias) {
  const int cin = 32, kg = cin / g, cg = mid / g;
  auto src = [&](int d) { return g > 1 ? (d % g) * cg + d / g : d; };  // fbnet_builder.py:332-349
  a->assign((size_t)mid / 32 * 2 * 2 * 64 * 8, 0);
  bias->resize(mid);
  for (int d = 0; d < mid; ++d) (*bias)[d] = f.b[src(d)];
  for (int mc = 0; mc < mid / 32; ++mc)
    for (int ks = 0; ks < 2; ++ks)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int d = 32 * mc + (lane & 31), h = lane >> 5;
          const int k = (j & 3) + 8 * (2 * ks + (j >> 2)) + 4 * h;  // stem channel
          const int c = src(d), grp = c / (mid / g);
          const float v = (k >= grp * kg && k < (grp + 1) * kg) ? f.w[(size_t)c * kg + (k - grp * kg)] : 0.f;
          const size_t o = ((((size_t)mc * 2 + ks) * 2) * 64 + lane) * 8 + j;
          put_f16_split(v, &(*a)[o], &(*a)[o + 64 * 8]);
        }
}

// 1x1 conv [cout][cin/g] (groups densified with zeros, output rows permuted by row_src) as
// the fp16x3 MFMA A operand: [cout/32][cin/16][plane][lane][8], lane (r = l & 31, h = l >> 5)
// holding W[row_src(32t + r)][16s + 8h + j].
template <class RowSrc>
static std::vector<uint16_t> pack_1x1_a(const std::vector<float>& w, int cout, int cin, int g,
                                        RowSrc row_src) {
  const int kg = cin / g;
  std::vector<uint16_t> a((size_t)cout / 32 * (cin / 16) * 2 * 64 * 8, 0);
  for (int tt = 0; tt < cout / 32; ++tt)
    for (int ks = 0; ks < cin / 16; ++ks)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int c = row_src(32 * tt + (lane & 31)), k = 16 * ks + 8 * (lane >> 5) + j;
          const int grp = c / (cout / g);
          const float v = (k >= grp * kg && k < (grp + 1) * kg) ? w[(size_t)c * kg + (k - grp * kg)] : 0.f;
          const size_t o = ((((size_t)tt * (cin / 16) + ks) * 2) * 64 + lane) * 8 + j;
          put_f16_split(v, &a[o], &a[o + 64 * 8]);
        }
  return a;
}

// 1x1 conv (cout = 32, groups densified) as 16x16x32 fp16 hi/lo A operands: [cin/32][out tile 2][plane]
// [lane 64][8], lane (row = l & 15 -> output channel 16 tile + row, k-group l >> 4 -> input
// channels 32 chunk + 8 (l >> 4) + j) -- the NAS front's pwl (hn_front.hip, no-fold form)
static std::vector<uint16_t> pack_1x1_a16(const std::vector<float>& w, int cout, int cin, int g) {
  const int kg = cin / g;
  std::vector<uint16_t> a((size_t)cin / 32 * (cout / 16) * 2 * 64 * 8, 0);
  for (int ch = 0; ch < cin / 32; ++ch)
    for (int tt = 0; tt < cout / 16; ++tt)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int c = 16 * tt + (lane & 15), k = 32 * ch + 8 * (lane >> 4) + j;
          const int grp = c / (cout / g);
          const float v = (k >= grp * kg && k < (grp + 1) * kg) ? w[(size_t)c * kg + (k - grp * kg)] : 0.f;
          const size_t o = ((((size_t)ch * (cout / 16) + tt) * 2) * 64 + lane) * 8 + j;
          put_f16_split(v, &a[o], &a[o + 64 * 8]);
        }
  return a;
}

// 3x3 conv (cin = 32, BN folded) as 16x16x32 bf16 hi/lo A operands for k_c12:
// [tap 9][group of 16 output channels][plane][lane 64][8], lane (row = l & 15 -> output
// channel 16 g + row, k-group l >> 4 -> input channels 8 (l >> 4) + j).
static std::vector<uint16_t> pack_c12(const std::vector<float>& w, int cout) {
  const int cin = 32, ng = cout / 16;
  std::vector<uint16_t> a((size_t)9 * ng * 2 * 64 * 8);
  for (int tap = 0; tap < 9; ++tap)
    for (int g = 0; g < ng; ++g)
      for (int lane = 0; lane < 64; ++lane)
        for (int j = 0; j < 8; ++j) {
          const int oc = 16 * g + (lane & 15), ic = 8 * (lane >> 4) + j;
          const float v = w[((size_t)oc * cin + ic) * 9 + tap];
          const uint16_t hv = f2bf(v);
          const size_t o = (((size_t)tap * ng + g) * 2 * 64 + lane) * 8 + j;
          a[o] = hv;
          a[o + 64 * 8] = f2bf(v - bf2f(hv));
        }
  return a;
}

// conv1 (cin = cout = 32, BN folded) as 1-D Winograd F(4,3) along x for k_c12w (hn_c12w.hip):
// Toom-Cook points 0, 1, -1, 1/2, -1/2, inf; U_xi[ky] = sum_kx G[xi][kx] W[ky][kx] in fp64, bf16
// hi / lo 16x16x32 A fragments [xi 6][ky 3][group 2][plane][lane 64][8], lane (row = l & 15 ->
// output channel 16 g + row, k-group l >> 4 -> input channels 8 (l >> 4) + j)
static std::vector<uint16_t> pack_c12w(const std::vector<float>& w) {
  static const double G[6][3] = {{4, 0, 0},           {2.0 / 3, 2.0 / 3, 2.0 / 3},   {2.0 / 3, -2.0 / 3, 2.0 / 3},
                                 {-8.0 / 3, -4.0 / 3, -2.0 / 3}, {-8.0 / 3, 4.0 / 3, -2.0 / 3}, {0, 0, 1}};
  std::vector<uint16_t> a((size_t)6 * 3 * 2 * 2 * 64 * 8);
  for (int xi = 0; xi < 6; ++xi)
    for (int ky = 0; ky < 3; ++ky)
      for (int g = 0; g < 2; ++g)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int oc = 16 * g + (lane & 15), ic = 8 * (lane >> 4) + j;
            double u = 0;
            for (int kx = 0; kx < 3; ++kx) u += G[xi][kx] * (double)w[((size_t)oc * 32 + ic) * 9 + ky * 3 + kx];
            const float v = (float)u;
            const uint16_t hv = f2bf(v);
            const size_t o = ((((size_t)(xi * 3 + ky) * 2 + g) * 2) * 64 + lane) * 8 + j;
            a[o] = hv;
            a[o + 64 * 8] = f2bf(v - bf2f(hv));
          }
  return a;
}

// stride-1 3x3 conv (BN folded) as 1-D Winograd F(2,3) along x (hn_wino1.hip): U_xi[ky] =
// sum_kx G[xi][kx] W[ky][kx] in fp64 (U3 negated: it accumulates into the odd output column with a
// minus sign), bf16 hi / lo A fragments [cin/32][xi][ky][ks][cout/32][plane][lane][8] in the
// kernel's K-step order kx = 6 xi + 2 ky + ks
static std::vector<uint16_t> pack_wino1(const std::vector<float>& w, int cin, int cout) {
  static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
  const int ncc = cin / 32, ntot = cout / 32;
  std::vector<uint16_t> out((size_t)ncc * 24 * ntot * 2 * 64 * 8);
  size_t o = 0;
  for (int cc = 0; cc < ncc; ++cc)
    for (int kx = 0; kx < 24; ++kx)
      for (int nt = 0; nt < ntot; ++nt) {
        const int xi = kx / 6, ky = (kx % 6) / 2, ks = kx % 2;
        uint16_t* hi = &out[o];
        uint16_t* lo = &out[o + 64 * 8];
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int n = nt * 32 + (lane & 31);
            const int c = cc * 32 + ks * 16 + (lane >> 5) * 8 + j;
            double u = 0;
            for (int t = 0; t < 3; ++t) u += G[xi][t] * (double)w[((size_t)n * cin + c) * 9 + ky * 3 + t];
            const float v = (float)(xi == 3 ? -u : u);
            const uint16_t hv = f2bf(v);
            hi[lane * 8 + j] = hv;
            lo[lane * 8 + j] = f2bf(v - bf2f(hv));
          }
        o += 2 * 64 * 8;
      }
  return out;
}

// stride-1 3x3 conv (BN folded) as 1-D Winograd F(4,3) along x (hn_wino1.hip k_conv_w4): U_xi[ky] =
// sum_kx G[xi][kx] W[ky][kx] in fp64, bf16 hi / lo A fragments of the 16x16x32 MFMA
// [cin/32][kx 18][cout/16][plane][lane][8] in the kernel's K-step order kx = 3 xo + ky, xi = w4_xi(xo)
// (lane: output channel 16 nt + (lane & 15), input channels 32 cc + 8 (lane >> 4) + j)
static std::vector<uint16_t> pack_wino4(const std::vector<float>& w, int cin, int cout) {
  static const double G[6][3] = {{4, 0, 0},
                                 {2.0 / 3, 2.0 / 3, 2.0 / 3},
                                 {2.0 / 3, -2.0 / 3, 2.0 / 3},
                                 {-8.0 / 3, -4.0 / 3, -2.0 / 3},
                                 {-8.0 / 3, 4.0 / 3, -2.0 / 3},
                                 {0, 0, 1}};
  static const int XO[6] = {0, 5, 1, 2, 3, 4};
  const int ncc = cin / 32, ntot = cout / 16;
  std::vector<uint16_t> out((size_t)ncc * 18 * ntot * 2 * 64 * 8);
  size_t o = 0;
  for (int cc = 0; cc < ncc; ++cc)
    for (int kx = 0; kx < 18; ++kx)
      for (int nt = 0; nt < ntot; ++nt) {
        const int xi = XO[kx / 3], ky = kx % 3;
        uint16_t* hi = &out[o];
        uint16_t* lo = &out[o + 64 * 8];
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int n = nt * 16 + (lane & 15);
            const int c = cc * 32 + (lane >> 4) * 8 + j;
            double u = 0;
            for (int t = 0; t < 3; ++t) u += G[xi][t] * (double)w[((size_t)n * cin + c) * 9 + ky * 3 + t];
            const float v = (float)u;
            const uint16_t hv = f2bf(v);
            hi[lane * 8 + j] = hv;
            lo[lane * 8 + j] = f2bf(v - bf2f(hv));
          }
        o += 2 * 64 * 8;
      }
  return out;
}

#ifdef HN_EXPERIMENTS
// stride-1 3x3 conv (BN folded) as Winograd F(2x2,3x3) U = G g G^T (fp64, then bf16 hi/lo),
// packed as the B operand of hn_wino.hip's 32x32x16 MFMAs: [cout/32][cin/16][xi 16][plane][lane
// 64][8], lane (column l & 31 -> output channel, k-group l >> 5 -> input channels 8 (l >> 5) + j)
static std::vector<uint16_t> pack_wino(const std::vector<float>& w, int cin, int cout) {
  static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
  const int ncb = cout / 32, nks = cin / 16;
  std::vector<uint16_t> a((size_t)ncb * nks * 16 * 2 * 64 * 8);
  for (int cb = 0; cb < ncb; ++cb)
    for (int ks = 0; ks < nks; ++ks)
      for (int xi = 0; xi < 16; ++xi)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int co = 32 * cb + (lane & 31), ci = 16 * ks + 8 * (lane >> 5) + j;
            const float* g = &w[((size_t)co * cin + ci) * 9];
            const int i0 = xi >> 2, j0 = xi & 3;
            double u = 0;
            for (int r = 0; r < 3; ++r)
              for (int c = 0; c < 3; ++c) u += G[i0][r] * (double)g[r * 3 + c] * G[j0][c];
            const float v = (float)u;
            const uint16_t hv = f2bf(v);
            const size_t o = ((((size_t)(cb * nks + ks) * 16 + xi) * 2) * 64 + lane) * 8 + j;
            a[o] = hv;
            a[o + 64 * 8] = f2bf(v - bf2f(hv));
          }
  return a;
}
#endif

static int build_hardnet(hn_model* m, Cursor& cur) {
  static const int cin[7] = {1, 32, 32, 64, 64, 128, 128};
  static const int cout[7] = {32, 32, 64, 64, 128, 128, 128};
  static const int ks[7] = {3, 3, 3, 3, 3, 3, 8};
  const float eps = m->desc.bn_eps;
  for (int l = 0; l < 7; ++l) {
    const size_t per = (size_t)cin[l] * ks[l] * ks[l];
    const float* w = cur.take(per * cout[l]);
    const float* mean = cur.take(cout[l]);
    const float* var = cur.take(cout[l]);
    if (!cur.ok) return fail(HN_ERR_ARG, "host_params too short");
    Folded f = fold(w, per, cout[l], nullptr, nullptr, mean, var, eps);
    int rc;
    if (l == 0) {
      std::vector<float> sw(9 * 32);
      for (int n = 0; n < 32; ++n)
        for (int t = 0; t < 9; ++t) sw[t * 32 + n] = f.w[n * 9 + t];
      if ((rc = m->upload(sw, &m->hd.stem_w))) return rc;
      if ((rc = m->upload(f.b, &m->hd.stem_b))) return rc;
      continue;
    }
    std::vector<uint16_t> pk = (l < 6) ? pack_conv3x3(f.w, cin[l], cout[l]) : pack_head(f.w, 128, 8);
    uint16_t* d = nullptr;
    if ((rc = m->upload(pk, &d))) return rc;
    m->hd.wpack[l] = d;
    if ((rc = m->upload(f.b, &m->hd.bias[l]))) return rc;
    if (l == 3 || l == 5) {  // 1-D Winograd F(2,3) U fragments (hn_wino1.hip)
      uint16_t* c = nullptr;
      if ((rc = m->upload(pack_wino1(f.w, cin[l], cout[l]), &c))) return rc;
      m->hd.wino1[l] = c;
    }
#ifdef HN_EXPERIMENTS
    if (l == 3) {  // 1-D Winograd F(4,3) U fragments (hn_wino1.hip k_conv_w4, experiments library only)
      uint16_t* c = nullptr;
      if ((rc = m->upload(pack_wino4(f.w, cin[l], cout[l]), &c))) return rc;
      m->hd.wino4[l] = c;
    }
    if (l == 3 || l == 5) {  // Winograd U fragments (experiments library only)
      uint16_t* c = nullptr;
      if ((rc = m->upload(pack_wino(f.w, cin[l], cout[l]), &c))) return rc;
      m->hd.wino[l] = c;
    }
#endif
    if (l == 1 || l == 2) {
      uint16_t* c = nullptr;
      if ((rc = m->upload(pack_c12(f.w, cout[l]), &c))) return rc;
      (l == 1 ? m->hd.c12_w1 : m->hd.c12_w2) = c;
    }
    if (l == 1) {
      uint16_t* c = nullptr;
      if ((rc = m->upload(pack_c12w(f.w), &c))) return rc;
      m->hd.c12_w1w = c;
    }
  }
  m->ws_floats_per_patch = 32 * 32 * 32;
  m->n_bufs = 3;
  return HN_OK;
}

static int take_cbr(hn_model* m, Cursor& cur, int cout, size_t per_out, Folded* f) {
  const float* w = cur.take((size_t)cout * per_out);
  const float* g = cur.take(cout);
  const float* b = cur.take(cout);
  const float* mu = cur.take(cout);
  const float* var = cur.take(cout);
  if (!cur.ok) return fail(HN_ERR_ARG, "host_params too short");
  *f = fold(w, per_out, cout, g, b, mu, var, m->desc.bn_eps);
  return HN_OK;
}

static int build_nas_layers(hn_model* m, Cursor& cur, int hw, size_t maxf);

// stem [32][9] -> [tap][32] for the VALU stem / front kernels
static std::vector<float> stem_taps(const std::vector<float>& w) {
  std::vector<float> sw(9 * 32);
  for (int n = 0; n < 32; ++n)
    for (int t = 0; t < 9; ++t) sw[t * 32 + n] = w[n * 9 + t];
  return sw;
}

static int build_nas(hn_model* m, Cursor& cur) {
  int rc;
  Folded f;
  if ((rc = take_cbr(m, cur, 32, 9, &f))) return rc;
  if ((rc = m->upload(stem_taps(f.w), &m->stem_w))) return rc;
  if ((rc = m->upload(f.b, &m->stem_b))) return rc;
  if (!m->no_front && (rc = m->upload(pack_front_stem(f), &m->front_spack))) return rc;
  return build_nas_layers(m, cur, 32, 32 * 32 * 32);
}

// FDLNet HardNetNeiMask (des.py): the front's parameters in state_dict order, BN folded
// (in double) into the conv before it; the stem keeps its conv bias.
static int build_fdl(hn_model* m, Cursor& cur) {
  const bool v0 = m->desc.kind == HN_KIND_FDL_NASNET;
  const float* w0 = cur.take(32 * 9);
  const float* b0 = cur.take(32);
  if (!cur.ok) return fail(HN_ERR_ARG, "host_params too short");
  Folded s;
  if (v0) {  // features.1: BatchNorm2d(32, affine=False) on conv + bias
    const float* mu = cur.take(32);
    const float* var = cur.take(32);
    if (!cur.ok) return fail(HN_ERR_ARG, "host_params too short");
    s = fold(w0, 9, 32, nullptr, nullptr, mu, var, m->desc.bn_eps);
    for (int c = 0; c < 32; ++c)  // bias: (b - mu) * sc, in double
      s.b[c] = (float)(((double)b0[c] - (double)mu[c]) / std::sqrt((double)var[c] + (double)m->desc.bn_eps));
  } else {
    s.w.assign(w0, w0 + 32 * 9);
    s.b.assign(b0, b0 + 32);
  }
  int rc;
  if ((rc = m->upload(stem_taps(s.w), &m->stem_w))) return rc;
  if ((rc = m->upload(s.b, &m->stem_b))) return rc;
  Folded f;
  if (v0) {
    // features.2 (Conv 1x1 s2 32 -> 32) + features.3 (BN): weight, then gamma, beta, mean, var
    const float* w = cur.take(32 * 32);
    const float* g = cur.take(32);
    const float* be = cur.take(32);
    const float* mu = cur.take(32);
    const float* var = cur.take(32);
    if (!cur.ok) return fail(HN_ERR_ARG, "host_params too short");
    f = fold(w, 32, 32, g, be, mu, var, m->desc.bn_eps);
    if ((rc = m->upload(transpose_pw(f.w, 32, 32), &m->fdl_w1))) return rc;
    if ((rc = m->upload(f.b, &m->fdl_b1))) return rc;
  }
  // NASNet: features.5 + features.6; NASNet_0.1: features.3.conv.{conv,bn} -- same order
  if ((rc = take_cbr(m, cur, 64, 32, &f))) return rc;
  if ((rc = m->upload(transpose_pw(f.w, 64, 32), &m->fdl_w2))) return rc;
  if ((rc = m->upload(f.b, &m->fdl_b2))) return rc;
  return build_nas_layers(m, cur, 8, 8 * 8 * 64);
}

static int build_nas_layers(hn_model* m, Cursor& cur, int hw, size_t maxf) {
  const hn_arch_desc& d = m->desc;
  const bool fdl = d.kind != HN_KIND_NAS;
  int rc;
  Folded f;
  for (int i = 0; i < d.n_layers; ++i) {
    NasLayer L;
    const OpSpec& s = kOps[d.op[i]];
    L.op = d.op[i];
    L.cin = d.c_in[i];
    L.cout = d.c_out[i];
    L.stride = d.stride[i];
    L.hin = hw;
    L.hout = hw / L.stride;
    L.skip = s.skip;
    if (s.skip) {
      L.skip_conv = L.cin != L.cout;
      if (i == 0 && !m->no_front && L.cin == 32 && L.cout == 32 && L.hin == 32 && L.stride == 2)
        m->front = 2;
      if (L.skip_conv) {
        if ((rc = take_cbr(m, cur, L.cout, L.cin, &f))) return rc;
        if ((rc = m->upload(transpose_pw(f.w, L.cout, L.cin), &L.pw_w))) return rc;
        if ((rc = m->upload(f.b, &L.pw_b))) return rc;
        if (L.cin == 64 && L.cout == 128 &&
            (rc = m->upload(pack_1x1_a(f.w, L.cout, L.cin, 1, [](int c) { return c; }), &L.skip_a)))
          return rc;
      }
      maxf = std::max(maxf, (size_t)L.cin * L.hout * L.hout);
      maxf = std::max(maxf, (size_t)L.cout * L.hout * L.hout);
    } else {
      L.e = s.e;
      L.k = s.k;
      L.g = s.g;
      L.se = s.se;
      L.mid = L.cin * L.e;
      if ((rc = take_cbr(m, cur, L.mid, L.cin / L.g, &f))) return rc;
      if ((rc = m->upload(transpose_pw(f.w, L.mid, L.cin / L.g), &L.pw_w))) return rc;
      if ((rc = m->upload(f.b, &L.pw_b))) return rc;
      if (i == 0 && !m->no_front && L.cin == 32 && L.hin == 32 && L.stride == 2 &&
          hn_front_supported(L.k, L.mid)) {
        std::vector<uint16_t> a;
        std::vector<float> b;
        pack_front(f, L.mid, L.g, &a, &b);
        if ((rc = m->upload(a, &L.front_a))) return rc;
        if ((rc = m->upload(b, &L.front_b))) return rc;
        m->front = 1;
      }
      const bool irf = (i > 0 || fdl) && !m->no_irf &&
                       hn_irf_supported(L.cin, L.cout, L.hin, L.stride, L.k, L.mid);
      if (irf) {
        const int g = L.g, cg = L.mid / g;
        auto src = [&](int d) { return g > 1 ? (d % g) * cg + d / g : d; };  // ChannelShuffle
        if ((rc = m->upload(pack_1x1_a(f.w, L.mid, L.cin, g, src), &L.irf_pw_a))) return rc;
        std::vector<float> b(L.mid);
        for (int d = 0; d < L.mid; ++d) b[d] = f.b[src(d)];
        if ((rc = m->upload(b, &L.irf_pw_b))) return rc;
      }
      if ((rc = take_cbr(m, cur, L.mid, (size_t)L.k * L.k, &f))) return rc;
      {
        std::vector<float> wd((size_t)L.k * L.k * L.mid);
        for (int c = 0; c < L.mid; ++c)
          for (int t = 0; t < L.k * L.k; ++t) wd[(size_t)t * L.mid + c] = f.w[(size_t)c * L.k * L.k + t];
        if ((rc = m->upload(wd, &L.dw_w))) return rc;
        if ((rc = m->upload(f.b, &L.dw_b))) return rc;
      }
      if ((rc = take_cbr(m, cur, L.cout, L.mid / L.g, &f))) return rc;
      if ((rc = m->upload(transpose_pw(f.w, L.cout, L.mid / L.g), &L.pwl_w))) return rc;
      if ((rc = m->upload(f.b, &L.pwl_b))) return rc;
      if ((L.irf_pw_a || (i == 0 && L.front_a)) &&
          (rc = m->upload(pack_1x1_a(f.w, L.cout, L.mid, L.g, [](int c) { return c; }), &L.irf_pwl_a)))
        return rc;
      if (i == 0 && L.front_a && (rc = m->upload(pack_1x1_a16(f.w, L.cout, L.mid, L.g), &L.front_pwl16)))
        return rc;
      if (L.se) {
        L.semid = L.cout / 4 > 8 ? L.cout / 4 : 8;
        const size_t n1 = (size_t)L.semid * L.cout;
        const float* w1 = cur.take(n1);
        const float* b1 = cur.take(L.semid);
        const float* w2 = cur.take(n1);
        const float* b2 = cur.take(L.cout);
        if (!cur.ok) return fail(HN_ERR_ARG, "host_params too short");
        if ((rc = m->upload(std::vector<float>(w1, w1 + n1), &L.se_w1))) return rc;
        if ((rc = m->upload(std::vector<float>(b1, b1 + L.semid), &L.se_b1))) return rc;
        if ((rc = m->upload(std::vector<float>(w2, w2 + n1), &L.se_w2))) return rc;
        if ((rc = m->upload(std::vector<float>(b2, b2 + L.cout), &L.se_b2))) return rc;
      }
      maxf = std::max(maxf, (size_t)L.mid * L.hin * L.hin);
      maxf = std::max(maxf, (size_t)L.mid * L.hout * L.hout);
      maxf = std::max(maxf, (size_t)L.cout * L.hout * L.hout);
    }
    m->layers.push_back(L);
    hw = L.hout;
  }
  const int cl = d.c_out[d.n_layers - 1];
  const float* w = cur.take((size_t)128 * cl * 16);
  const float* mu = cur.take(128);
  const float* var = cur.take(128);
  if (!cur.ok) return fail(HN_ERR_ARG, "host_params too short");
  f = fold(w, (size_t)cl * 16, 128, nullptr, nullptr, mu, var, d.bn_eps);
  {
    const int K = cl * 16;
    std::vector<float> wt((size_t)K * 128);
    for (int n = 0; n < 128; ++n)
      for (int c = 0; c < cl; ++c)
        for (int yx = 0; yx < 16; ++yx)
          wt[((size_t)yx * cl + c) * 128 + n] = f.w[((size_t)n * cl + c) * 16 + yx];
    if ((rc = m->upload(wt, &m->head_w))) return rc;
    if ((rc = m->upload(f.b, &m->head_b))) return rc;
    m->head_k = K;
    if (K == 2048 && (rc = m->upload(pack_head(f.w, cl, 4, true), &m->head_pack))) return rc;
  }
  m->ws_floats_per_patch = maxf;
  m->n_bufs = 4;
  return HN_OK;
}

extern "C" int hn_create(const hn_arch_desc* desc, const float* host_params, size_t n_params,
                         hn_model** out) {
  int rc = check_desc(desc);
  if (rc) return rc;
  if (!out || !host_params) return fail(HN_ERR_ARG, "NULL argument");
  size_t want = 0;
  if ((rc = hn_param_count(desc, &want))) return rc;
  if (want != n_params)
    return fail(HN_ERR_ARG, "host_params has " + std::to_string(n_params) + " floats, expected " +
                                std::to_string(want));
  hn_model* m = new hn_model();
  m->desc = *desc;
  if (const char* e = std::getenv("HN_CHUNK")) m->chunk = std::max(64, std::atoi(e));
  if (const char* e = std::getenv("HN_UNFUSED_STEM")) m->unfused_stem = std::atoi(e) != 0;
  if (const char* e = std::getenv("HN_NO_FRONT")) m->no_front = std::atoi(e) != 0;
  if (const char* e = std::getenv("HN_NO_C12")) m->c12 = std::atoi(e) == 0;
  if (const char* e = std::getenv("HN_SUBCHUNK")) m->subchunk = std::max(64, std::atoi(e));
  if (const char* e = std::getenv("HN_C12_GROUP")) m->c12group = std::max(64, std::atoi(e));
  if (const char* e = std::getenv("HN_C4_SUB")) m->c4sub = std::max(0, std::atoi(e));
  if (const char* e = std::getenv("HN_NO_IRF")) m->no_irf = std::atoi(e) != 0;
  if (const char* e = std::getenv("HN_NO_IRF2")) m->no_irf2 = std::atoi(e) != 0;
  if (const char* e = std::getenv("HN_VARIANT")) {
    int i = 0;
    for (const char* c = e; *c && i < 6; ++c)
      if (*c >= '0' && *c <= '9') m->variant[i++] = *c - '0';
      else if (*c >= 'a' && *c <= 'z') m->variant[i++] = 10 + (*c - 'a');
  }
  hn_read_knobs(&m->knobs);
  // k_head4 takes 256 patches per workgroup: chunks of 65,536 keep every CU busy in the head
  if (m->knobs.head == 4 && !std::getenv("HN_CHUNK")) m->chunk = 65536;
  for (int l = 0; l < 6; ++l)
    if (!hn_hardnet_variant_ok(l, m->variant[l])) {
      const std::string msg = "HN_VARIANT: tiling " + std::to_string(m->variant[l]) +
                              " is not available for layer " + std::to_string(l);
      delete m;
      return fail(HN_ERR_ARG, msg);
    }
  if (!hn_c12_cfg_ok(m->knobs.c12_cfg, m->knobs.c12_abl)) {
    delete m;
    return fail(HN_ERR_ARG, "HN_C12_CFG / HN_C12_ABL: no such k_c12 build in this library");
  }
  if (m->knobs.head < 1 || m->knobs.head > 4) {
    delete m;
    return fail(HN_ERR_ARG, "HN_HEAD: head GEMM form must be 1, 2, 3 or 4");
  }
  (void)hipGetDevice(&m->device);
  Cursor cur{host_params, n_params};
  tl_f16_out_of_range = 0;
  rc = desc->kind == HN_KIND_HARDNET ? build_hardnet(m, cur)
       : desc->kind == HN_KIND_NAS    ? build_nas(m, cur)
                                      : build_fdl(m, cur);
  if (!rc && cur.i != n_params) rc = fail(HN_ERR_ARG, "host_params not fully consumed");
  if (!rc && tl_f16_out_of_range)
    rc = fail(HN_ERR_ARG, std::to_string(tl_f16_out_of_range) +
                              " BN-folded weights are outside the fp16 range of the fp16x3 kernels (|w| >= 65520 "
                              "or not finite)");
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return HN_OK;
}

// HardNet on k_c12: k_c12 runs per group (HN_C12_GROUP patches, its output a2 spanning the group) and
// conv3..conv5 per sub-chunk of it, so a3 spans one sub-chunk and the head's input (a5, 32 KiB per
// patch) the chunk
static bool hardnet_subchunked(const hn_model* m) {
  return m->desc.kind == HN_KIND_HARDNET && m->c12 && !m->unfused_stem;
}
static int64_t hardnet_sub(const hn_model* m, int64_t p) { return std::max<int64_t>(1, std::min<int64_t>(p, m->subchunk)); }
static int64_t hardnet_group(const hn_model* m, int64_t p) {
  return std::max(hardnet_sub(m, p), std::min<int64_t>(p, m->c12group));
}

// the chunk pipeline (forward_hardnet_pipe): a HardNet batch of more than one chunk, one k_c12 group per chunk
static bool hardnet_pipelined(const hn_model* m, int64_t batch) {
  return m->knobs.pipeline && hardnet_subchunked(m) && batch > m->chunk && hardnet_group(m, m->chunk) >= m->chunk;
}

extern "C" int hn_workspace_bytes(const hn_model* m, int64_t batch, size_t* bytes_out) {
  if (!m || !bytes_out || batch < 0) return fail(HN_ERR_ARG, "bad argument");
  const int64_t p = batch < m->chunk ? batch : m->chunk;
  if (hardnet_subchunked(m)) {
    *bytes_out = ((size_t)(hardnet_sub(m, p) + hardnet_group(m, p)) * 16384 + (size_t)p * 8192) * sizeof(float);
    // the pipeline's second k_c12 output buffer (64 KiB per patch of a chunk)
    if (hardnet_pipelined(m, batch)) *bytes_out += (size_t)p * 16384 * sizeof(float);
  } else {
    *bytes_out = (size_t)p * m->ws_floats_per_patch * m->n_bufs * sizeof(float);
  }
  return HN_OK;
}

// Launch one stage; with profiling on, bracket it by a hipEvent pair on the same stream.
#define STAGE_ON(SS, NAME, CALL)                                                           \
  do {                                                                                     \
    hipEvent_t a_ = nullptr;                                                               \
    if (m->prof.on) {                                                                      \
      a_ = m->prof.get();                                                                  \
      HIPCHK(hipEventRecord(a_, SS));                                                      \
    }                                                                                      \
    HIPCHK(CALL);                                                                          \
    if (m->prof.on) {                                                                      \
      hipEvent_t b_ = m->prof.get();                                                       \
      HIPCHK(hipEventRecord(b_, SS));                                                      \
      m->prof.pend.push_back({m->prof.stage_id(NAME), a_, b_});                            \
    }                                                                                      \
  } while (0)
#define STAGE(NAME, CALL) STAGE_ON(st, NAME, CALL)

// conv3 .. conv5 of a k_c12 group's n patches (its output a2 [n][16,384 floats]) in sub-chunks of `sub`: conv3 into
// a0, conv4 back over the sub-chunk's a2 slots (consumed by conv3; in HN_C4_SUB pieces), conv5 into a5 rows
// a5 + [patch][8,192 floats]
static int hardnet_convs(hn_model* m, float* a2, int n, int sub, float* a0, float* a5, hipStream_t st) {
  for (int s0 = 0; s0 < n; s0 += sub) {
    const int ns = std::min(sub, n - s0);
    float* const a2s = a2 + (size_t)s0 * 16384;
    STAGE("conv3", hn_launch_hardnet_conv(3, m->variant[3], m->hd, a2s, a0, ns, 0.f, st));
    const int c4 = m->c4sub > 0 ? m->c4sub : ns;
    for (int q = 0; q < ns; q += c4)  // (a3 is 16,384 floats per patch, a4 8,192)
      STAGE("conv4", hn_launch_hardnet_conv(4, m->variant[4], m->hd, a0 + (size_t)q * 16384, a2s + (size_t)q * 8192,
                                            std::min(c4, ns - q), 0.f, st));
    STAGE("conv5", hn_launch_hardnet_conv(5, m->variant[5], m->hd, a2s, a5 + (size_t)s0 * 8192, ns, 0.f, st));
  }
  return HN_OK;
}

// pmax: the largest chunk of this call; the buffers keep the same offsets for every chunk
static int forward_hardnet(hn_model* m, const float* in, int P, int pmax, float* out, float* ws,
                           hipStream_t st, const HnU8In* u8 = nullptr) {
  const size_t per = m->ws_floats_per_patch * (size_t)pmax;
  float* a0 = ws;
  float* a1 = ws + per;
  float* a2 = ws + 2 * per;
  const float ineps = m->desc.input_norm_eps;
  if (hardnet_subchunked(m)) {
    // k_c12 over groups (HN_C12_GROUP) and the conv stages over sub-chunks of a group (HN_SUBCHUNK);
    // both default to 65,536 patches, one launch of each per chunk (same box: 5.46 against 5.24
    // Mpatches/s for 16,384-patch launches; k_c12s 20.9 -> 18.5 ms per 262,144-patch step, conv4 7.3 ->
    // 8.2; a 65,536 group over 16,384 sub-chunks measured 5.26-5.29).  The head GEMM runs
    // once per chunk over the a5 of all sub-chunks.  conv4 writes its output over the sub-chunk's a2 slots,
    // which conv3 has consumed.  Workspace (hn_workspace_bytes): [a3: sub x 64 KiB] [a2 / a4: group x 64 KiB]
    // [a5: pmax x 32 KiB]
    const int sub = (int)hardnet_sub(m, P), grp = (int)hardnet_group(m, P);
    a0 = ws;
    a2 = ws + (size_t)16384 * hardnet_sub(m, pmax);
    a1 = a2 + (size_t)16384 * hardnet_group(m, pmax);
    for (int g0 = 0; g0 < P; g0 += grp) {
      const int ng = std::min(grp, P - g0);
      if (u8) {
        HnU8In gin = *u8;
        gin.in += (size_t)g0 * (u8->resize == HN_RESIZE_NONE ? 1024 : 4096);
        STAGE("stem+conv1+conv2", hn_launch_c12(nullptr, a2, m->hd, ng, ineps, st, &gin));
      } else {
        STAGE("stem+conv1+conv2", hn_launch_c12(in + (size_t)g0 * 1024, a2, m->hd, ng, ineps, st));
      }
      if (int rc = hardnet_convs(m, a2, ng, sub, a0, a1 + (size_t)g0 * 8192, st)) return rc;
    }
    // a0 -- conv3's output, consumed -- holds the small-batch head's split-K partials (8,192 floats per patch
    // against its 16,384 per sub-chunk patch)
    float* const hs = (size_t)16384 * hardnet_sub(m, pmax) >= (size_t)8192 * P ? a0 : nullptr;
    STAGE("head", hn_launch_head(a1, out, m->hd.wpack[6], m->hd.bias[6], P, 8192, m->desc.l2_eps, st, false, hs));
    return HN_OK;
  } else {
    if (m->unfused_stem) {
      STAGE("stem", hn_launch_stem(in, a0, m->hd.stem_w, m->hd.stem_b, P, ineps >= 0.f, ineps, st));
      STAGE("conv1", hn_launch_hardnet_conv(1, 0, m->hd, a0, a1, P, 0.f, st));
    } else {
      STAGE("stem+conv1", hn_launch_hardnet_conv(0, m->variant[0], m->hd, in, a1, P, ineps, st));
    }
    STAGE("conv2", hn_launch_hardnet_conv(2, m->variant[2], m->hd, a1, a2, P, 0.f, st));
  }
  STAGE("conv3", hn_launch_hardnet_conv(3, m->variant[3], m->hd, a2, a1, P, 0.f, st));
  STAGE("conv4", hn_launch_hardnet_conv(4, m->variant[4], m->hd, a1, a2, P, 0.f, st));
  STAGE("conv5", hn_launch_hardnet_conv(5, m->variant[5], m->hd, a2, a1, P, 0.f, st));
  STAGE("head", hn_launch_head(a1, out, m->hd.wpack[6], m->hd.bias[6], P, 8192, m->desc.l2_eps, st, false, a2));
  return HN_OK;
}

// A HardNet batch of n > 1 chunks (hn_forward): chunk k + 1's k_c12s runs on a second stream into the other of
// two k_c12 output buffers while chunk k's conv3 .. head run on the caller's stream, so the kernels' ramps and
// tails overlap.  Opt-in (HN_PIPELINE=1): at 262,144 patches it measured 5.46 / 5.59 -> 5.55 / 5.55 Mpatches/s on one
// box (within that box's noise), and k_c12s's launches, sharing the GPU, then time at 6.0 instead of 4.6-4.7 ms.
// Order: c12(k + 1) waits until conv5(k - 1) has finished with its buffer (ev_free), conv3(k) waits for c12(k)
// (ev_ready); conv3 .. head of consecutive chunks stay in order on the caller's stream, which waits for every
// chunk's k_c12s -- the second stream is forked from and joined back into it (graph capture included).
// Workspace: [a3: sub x 64 KiB] [a2 x 2: chunk x 64 KiB each] [a5: chunk x 32 KiB].
static int forward_hardnet_pipe(hn_model* m, const float* in, int64_t batch, float* out, float* ws, hipStream_t st) {
  std::lock_guard<std::mutex> lock(m->pipe_mu);
  if (!m->st2) {
    HIPCHK(hipStreamCreateWithFlags(&m->st2, hipStreamNonBlocking));
    for (hipEvent_t* e : {&m->ev_fork, &m->ev_ready[0], &m->ev_ready[1], &m->ev_free[0], &m->ev_free[1]})
      HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  const int C = m->chunk, sub = (int)hardnet_sub(m, C);
  const int n = (int)((batch + C - 1) / C);
  const float ineps = m->desc.input_norm_eps;
  float* const a0 = ws;
  float* const a2b[2] = {ws + (size_t)16384 * sub, ws + (size_t)16384 * sub + (size_t)16384 * C};
  float* const a1 = a2b[1] + (size_t)16384 * C;
  auto rows = [&](int k) { return (int)std::min<int64_t>(C, batch - (int64_t)k * C); };
  auto c12 = [&](int k, hipStream_t s) -> int {
    STAGE_ON(s, "stem+conv1+conv2", hn_launch_c12(in + (size_t)k * C * 1024, a2b[k & 1], m->hd, rows(k), ineps, s));
    return HN_OK;
  };
  HIPCHK(hipEventRecord(m->ev_fork, st));
  HIPCHK(hipStreamWaitEvent(m->st2, m->ev_fork, 0));
  if (int rc = c12(0, st)) return rc;
  for (int k = 0; k < n; ++k) {
    const int P = rows(k);
    if (k + 1 < n) {
      if (k >= 1) HIPCHK(hipStreamWaitEvent(m->st2, m->ev_free[(k + 1) & 1], 0));
      if (int rc = c12(k + 1, m->st2)) return rc;
      HIPCHK(hipEventRecord(m->ev_ready[(k + 1) & 1], m->st2));
    }
    if (k >= 1) HIPCHK(hipStreamWaitEvent(st, m->ev_ready[k & 1], 0));
    float* const a2 = a2b[k & 1];
    if (int rc = hardnet_convs(m, a2, P, sub, a0, a1, st)) return rc;
    if (k + 2 < n) HIPCHK(hipEventRecord(m->ev_free[k & 1], st));  // a2b[k & 1] free for c12(k + 2)
    float* const hs = (size_t)16384 * sub >= (size_t)8192 * P ? a0 : nullptr;
    STAGE("head", hn_launch_head(a1, out + (size_t)k * C * 128, m->hd.wpack[6], m->hd.bias[6], P, 8192,
                                 m->desc.l2_eps, st, false, hs));
  }
  return HN_OK;
}

static int forward_nas(hn_model* m, const float* in, int P, int pmax, float* out, float* ws,
                       hipStream_t st, const HnU8In* u8 = nullptr) {
  const size_t per = m->ws_floats_per_patch * (size_t)pmax;
  float* x = ws;
  float* t1 = ws + per;
  float* t2 = ws + 2 * per;
  float* y = ws + 3 * per;
  const float ineps = m->desc.input_norm_eps;
  size_t first = 0;
  if (m->desc.kind != HN_KIND_NAS) {  // FDLNet front (des.py) -> 8x8x64
    const HnFdlFrontArgs fa{in, x, m->stem_w, m->stem_b, m->fdl_w1, m->fdl_b1, m->fdl_w2, m->fdl_b2};
    STAGE("front", hn_launch_fdl_front(fa, P, m->desc.kind == HN_KIND_FDL_NASNET ? 0 : 1, ineps, st, u8));
  } else if (m->front == 2 && !u8 && ineps < 0.f && !m->knobs.no_mpfront && m->layers.size() > 2 &&
             m->layers[1].skip && !m->layers[1].skip_conv && m->layers[1].stride == 1 && m->layers[2].irf_pwl_a &&
             !m->layers[2].se &&
             hn_mpfront_irf_supported(m->layers[2].cin, m->layers[2].cout, m->layers[2].hin, m->layers[2].stride,
                                      m->layers[2].k, m->layers[2].mid)) {
    // the max-pool front, the identity layer 1 and the 16x16 stride-2 layer-2 block in one kernel
    // (k_mpfront_irf): the 16x16x32 front output never reaches HBM
    const NasLayer& L = m->layers[2];
    const HnIrfArgs ia{nullptr, x, reinterpret_cast<const uint4*>(L.irf_pw_a), L.irf_pw_b, L.dw_w, L.dw_b,
                       reinterpret_cast<const uint4*>(L.irf_pwl_a), L.pwl_b};
    STAGE("front+irf", hn_launch_mpfront_irf(in, reinterpret_cast<const uint4*>(m->front_spack), m->stem_b, ia, P, L.k,
                                             L.mid, false, ineps, st));
    first = 3;
  } else if (m->front) {
    const NasLayer& L = m->layers[0];
    const bool mp = m->front == 2;
    const HnFrontArgs fa{in, x, reinterpret_cast<const uint4*>(m->front_spack), m->stem_b,
                         reinterpret_cast<const uint4*>(L.front_a), L.front_b, L.dw_w, L.dw_b,
                         reinterpret_cast<const uint4*>(L.irf_pwl_a), L.pwl_b,
                         reinterpret_cast<const uint4*>(L.front_pwl16)};
    STAGE("front", hn_launch_front(fa, P, L.k, L.mid, mp, ineps >= 0.f, ineps, st, u8));
    if (!mp && L.se)
      STAGE("se", hn_launch_se(x, L.se_w1, L.se_b1, L.se_w2, L.se_b2, P, L.hout * L.hout, L.cout,
                               L.semid, st));
    first = 1;
  } else {
    STAGE("stem", hn_launch_stem(in, x, m->stem_w, m->stem_b, P, ineps >= 0.f, ineps, st));
  }
  for (size_t li = first; li < m->layers.size(); ++li) {
    const NasLayer& L = m->layers[li];
    const long npix_out = (long)P * L.hout * L.hout;
    if (L.skip) {
      const float* src = x;
      const bool nofuse = m->knobs.no_skipfuse;  // (A/B, layerwise tests)
      if (L.stride == 2 && L.skip_conv && !nofuse && hn_skip_s2_supported(L.hin, L.cin, L.cout)) {
        STAGE("skip", hn_launch_skip_s2(x, y, L.pw_w, L.pw_b, P, L.hin, L.cin, L.cout, st));
        std::swap(x, y);
        continue;
      }
      if (L.stride == 2) {
        STAGE("maxpool", hn_launch_maxpool(x, t1, P, L.hin, L.cin, st));
        src = t1;
      }
      if (L.skip_conv) {
        STAGE("pw", hn_launch_pw(src, y, L.pw_w, L.pw_b, nullptr, npix_out, L.cin, L.cout, 1, true, 0, st));
        std::swap(x, y);
      } else if (L.stride == 2) {
        std::swap(x, t1);
      }
      continue;
    }
    if (L.irf_pwl_a && li + 1 < m->layers.size() && !m->no_irf2) {
      // this block and the next in one kernel (k_irf2) when this one is stride 1 without SE and
      // the next is a stride-2 block at the same resolution: the activation between them stays in LDS
      const NasLayer& N = m->layers[li + 1];
      if (!L.se && N.irf_pwl_a && L.stride == 1 && L.cin == L.cout && N.stride == 2 && N.cin == L.cout &&
          N.hin == L.hin && hn_irf2_supported(L.cin, L.hin, L.k, L.mid, N.cout, N.k, N.mid)) {
        const HnIrfArgs ia{x, nullptr, reinterpret_cast<const uint4*>(L.irf_pw_a), L.irf_pw_b, L.dw_w, L.dw_b,
                           reinterpret_cast<const uint4*>(L.irf_pwl_a), L.pwl_b};
        const HnIrfArgs ib{nullptr, y, reinterpret_cast<const uint4*>(N.irf_pw_a), N.irf_pw_b, N.dw_w, N.dw_b,
                           reinterpret_cast<const uint4*>(N.irf_pwl_a), N.pwl_b};
#ifdef HN_EXPERIMENTS
        if (li + 2 < m->layers.size() && !N.se && m->knobs.irf3) {
          // and the 4x4 128 -> 128 stride-1 block after the pair (k_irf3): B's output tile stays in LDS for it
          const NasLayer& C = m->layers[li + 2];
          if (C.irf_pwl_a && !C.se && C.stride == 1 && C.cin == N.cout && C.cout == N.cout && C.hin == N.hout &&
              N.cout == 128 && L.cin == 64 && L.hin == 8 && hn_irf3_supported(L.k, L.mid, N.k, N.mid, C.k, C.mid)) {
            const HnIrfArgs ic{nullptr, y, reinterpret_cast<const uint4*>(C.irf_pw_a), C.irf_pw_b, C.dw_w, C.dw_b,
                               reinterpret_cast<const uint4*>(C.irf_pwl_a), C.pwl_b};
            STAGE("irf3", hn_launch_irf3(ia, ib, ic, P, L.k, N.k, C.k, st));
            std::swap(x, y);
            li += 2;
            continue;
          }
        }
#endif
        STAGE("irf2", hn_launch_irf2(ia, ib, P, L.cin, L.hin, L.k, L.mid, N.cout, N.k, N.mid, st));
        if (N.se)
          STAGE("se", hn_launch_se(y, N.se_w1, N.se_b1, N.se_w2, N.se_b2, P, N.hout * N.hout, N.cout, N.semid, st));
        std::swap(x, y);
        ++li;
        continue;
      }
    }
    if (L.irf_pwl_a && !L.se && !m->knobs.no_skipfuse && !m->knobs.no_irfskip &&
        hn_irf_skip_supported(L.cin, L.cout, L.hin, L.stride, L.k, L.mid)) {
      // the 8x8 stride-2 skip after this block (past identity skips) in the same kernel (k_irf_skip)
      size_t ni = li + 1;
      while (ni < m->layers.size() && m->layers[ni].skip && !m->layers[ni].skip_conv && m->layers[ni].stride == 1) ++ni;
      if (ni < m->layers.size()) {
        const NasLayer& N = m->layers[ni];
        if (N.skip && N.skip_conv && N.stride == 2 && N.hin == L.hout && N.cin == L.cout && N.cout == 128 && N.skip_a) {
          const HnIrfArgs ia{x, y, reinterpret_cast<const uint4*>(L.irf_pw_a), L.irf_pw_b, L.dw_w, L.dw_b,
                             reinterpret_cast<const uint4*>(L.irf_pwl_a), L.pwl_b};
          STAGE("irf+skip", hn_launch_irf_skip(ia, reinterpret_cast<const uint4*>(N.skip_a), N.pw_b, P, L.k, L.mid, st));
          std::swap(x, y);
          li = ni;
          continue;
        }
      }
    }
    if (L.irf_pwl_a) {
      const HnIrfArgs ia{x, y, reinterpret_cast<const uint4*>(L.irf_pw_a), L.irf_pw_b, L.dw_w, L.dw_b,
                         reinterpret_cast<const uint4*>(L.irf_pwl_a), L.pwl_b};
      STAGE("irf", hn_launch_irf(ia, P, L.cin, L.cout, L.hin, L.stride, L.k, L.mid, st));
      if (L.se)
        STAGE("se", hn_launch_se(y, L.se_w1, L.se_b1, L.se_w2, L.se_b2, P, L.hout * L.hout, L.cout,
                                 L.semid, st));
      std::swap(x, y);
      continue;
    }
    const long npix_in = (long)P * L.hin * L.hin;
    STAGE("pw", hn_launch_pw(x, t1, L.pw_w, L.pw_b, nullptr, npix_in, L.cin, L.mid, L.g, true,
                             L.g > 1 ? L.g : 0, st));
    STAGE("dw", hn_launch_dw(t1, t2, L.dw_w, L.dw_b, P, L.hin, L.mid, L.k, L.stride, st));
    const bool res = L.stride == 1 && L.cin == L.cout;
    STAGE("pwl", hn_launch_pw(t2, y, L.pwl_w, L.pwl_b, res ? x : nullptr, npix_out, L.mid, L.cout,
                              L.g, false, 0, st));
    if (L.se)
      STAGE("se", hn_launch_se(y, L.se_w1, L.se_b1, L.se_w2, L.se_b2, P, L.hout * L.hout, L.cout,
                               L.semid, st));
    std::swap(x, y);
  }
  if (m->head_pack) {
    // (any of the four buffers but the head's input holds the small-batch split-K partials)
    float* const hs = m->ws_floats_per_patch >= (size_t)head_split(m->head_k) * 128 ? (x == ws ? ws + per : ws) : nullptr;
    STAGE("head", hn_launch_head(x, out, m->head_pack, m->head_b, P, m->head_k, m->desc.l2_eps, st, true, hs));
  } else
    STAGE("head", hn_launch_nas_head(x, out, m->head_w, m->head_b, P, m->head_k, m->desc.l2_eps, st));
  return HN_OK;
}

extern "C" int hn_forward(hn_model* m, const float* d_in, int64_t batch, float* d_out,
                          void* d_workspace, size_t workspace_bytes, void* hip_stream) {
  if (!m) return fail(HN_ERR_ARG, "model is NULL");
  if (batch < 0) return fail(HN_ERR_ARG, "negative batch");
  if (batch == 0) return HN_OK;
  if (!d_in || !d_out || !d_workspace) return fail(HN_ERR_ARG, "NULL device pointer");
  if ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_out) |
       reinterpret_cast<uintptr_t>(d_workspace)) & 15)
    return fail(HN_ERR_ARG, "device pointers must be 16-byte aligned");
  size_t need = 0;
  hn_workspace_bytes(m, batch, &need);
  if (workspace_bytes < need)
    return fail(HN_ERR_WORKSPACE, "workspace too small: need " + std::to_string(need) + " bytes");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  KnobScope knobs(&m->knobs);
  if (hardnet_pipelined(m, batch)) return forward_hardnet_pipe(m, d_in, batch, d_out, static_cast<float*>(d_workspace), st);
  for (int64_t off = 0; off < batch; off += m->chunk) {
    const int P = (int)std::min<int64_t>(m->chunk, batch - off);
    const float* in = d_in + off * 1024;
    float* out = d_out + off * 128;
    float* ws = static_cast<float*>(d_workspace);
    const int pmax = (int)std::min<int64_t>(m->chunk, batch);
    const int rc = m->desc.kind == HN_KIND_HARDNET ? forward_hardnet(m, in, P, pmax, out, ws, st)
                                                   : forward_nas(m, in, P, pmax, out, ws, st);
    if (rc) return rc;
  }
  return HN_OK;
}

// uint8 input: the stock HardNet's fused k_c12, FDLNet's MFMA front and the NAS
// models' fused front preprocess in their patch loads in every resize mode; every other model /
// configuration (HN_NO_FRONT, HN_FRONT_FOLD, HN_FDL_VALU, the A/B configurations) runs hn_preprocess
// into the workspace tail first.
static bool u8_fused(const hn_model* m, int resize) {
  if (m->knobs.u8_apart) return false;
  if (m->desc.kind == HN_KIND_FDL_NASNET || m->desc.kind == HN_KIND_FDL_NASNET01) return !m->knobs.fdl_valu;
  if (m->desc.kind == HN_KIND_NAS) {  // the fused front's patch load (hn_front.hip): no input_norm
    // PIL on the k5 front (two workgroups per CU): its staging barrier and LDS window reads cost more
    // than the separate pass (wang3 23.4-23.6 against 24.4-24.5 Mpatches/s; k3 / max-pool fronts equal)
    if (resize == HN_RESIZE_PIL_BILINEAR && m->front == 1 && !m->layers.empty() && m->layers[0].k == 5) return false;
    return m->front && m->desc.input_norm_eps < 0.f && !m->knobs.front_fold;
  }
  return m->desc.kind == HN_KIND_HARDNET && m->c12 && !m->unfused_stem && (m->knobs.c12_cfg == 12 || m->knobs.c12_cfg == 13 || m->knobs.c12_cfg == kC12Wino || m->knobs.c12_cfg == kC12Split) &&
         !m->knobs.c12_abl;
}

extern "C" int hn_workspace_bytes_u8(const hn_model* m, int64_t batch, size_t* bytes_out) {
  int rc = hn_workspace_bytes(m, batch, bytes_out);
  if (rc) return rc;
  // (the fp32 tail for hn_preprocess unless every resize mode is fused)
  if (!u8_fused(m, HN_RESIZE_PIL_BILINEAR)) *bytes_out += (size_t)std::min<int64_t>(batch, m->chunk) * 1024 * sizeof(float);
  return HN_OK;
}

extern "C" int hn_forward_u8(hn_model* m, const uint8_t* d_in, int64_t batch, int32_t in_hw, int32_t resize,
                             int32_t normalize, float mean, float stdv, float* d_out, void* d_workspace,
                             size_t workspace_bytes, void* hip_stream) {
  if (!m) return fail(HN_ERR_ARG, "model is NULL");
  if (batch < 0) return fail(HN_ERR_ARG, "negative batch");
  if (resize != HN_RESIZE_NONE && resize != HN_RESIZE_CV2_LINEAR && resize != HN_RESIZE_PIL_BILINEAR)
    return fail(HN_ERR_ARG, "unknown resize mode " + std::to_string(resize));
  const int want = resize == HN_RESIZE_NONE ? 32 : 64;
  if (in_hw != want)
    return fail(HN_ERR_ARG, "in_hw must be " + std::to_string(want) + " for this resize mode, got " +
                                std::to_string(in_hw));
  if (normalize && !(stdv != 0.0f)) return fail(HN_ERR_ARG, "std must be nonzero");
  if (batch == 0) return HN_OK;
  if (!d_in || !d_out || !d_workspace) return fail(HN_ERR_ARG, "NULL device pointer");
  if ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_out) |
       reinterpret_cast<uintptr_t>(d_workspace)) & 15)
    return fail(HN_ERR_ARG, "device pointers must be 16-byte aligned");
  size_t need = 0;
  hn_workspace_bytes_u8(m, batch, &need);
  if (workspace_bytes < need)
    return fail(HN_ERR_WORKSPACE, "workspace too small: need " + std::to_string(need) + " bytes");
  hipStream_t st = static_cast<hipStream_t>(hip_stream);
  KnobScope knobs(&m->knobs);
  const bool fused = u8_fused(m, resize);
  const size_t inb = (size_t)in_hw * in_hw;
  float* ws = static_cast<float*>(d_workspace);
  size_t base = 0;
  hn_workspace_bytes(m, batch, &base);
  float* pre = reinterpret_cast<float*>(static_cast<char*>(d_workspace) + base);  // unfused: fp32 patches
  const int pmax = (int)std::min<int64_t>(m->chunk, batch);
  for (int64_t off = 0; off < batch; off += m->chunk) {
    const int P = (int)std::min<int64_t>(m->chunk, batch - off);
    const uint8_t* in = d_in + off * inb;
    float* out = d_out + off * 128;
    int rc;
    if (fused) {
      const HnU8In u8{in, resize, normalize, mean, stdv};
      rc = m->desc.kind == HN_KIND_HARDNET ? forward_hardnet(m, nullptr, P, pmax, out, ws, st, &u8)
                                           : forward_nas(m, nullptr, P, pmax, out, ws, st, &u8);
    } else {
      STAGE("preprocess", hn_launch_preprocess(in, P, resize, normalize, mean, stdv, pre, st));
      rc = m->desc.kind == HN_KIND_HARDNET ? forward_hardnet(m, pre, P, pmax, out, ws, st)
                                           : forward_nas(m, pre, P, pmax, out, ws, st);
    }
    if (rc) return rc;
  }
  return HN_OK;
}

// ---------------------------------------------------------------------------------------
// train-mode stock HardNet (hn_train.hip)
// ---------------------------------------------------------------------------------------
extern "C" int hn_hardnet_train_workspace_bytes(int64_t batch, size_t* saved_bytes_out, size_t* scratch_bytes_out) {
  if (!saved_bytes_out || !scratch_bytes_out || batch < 2 || batch > (1 << 24))
    return fail(HN_ERR_ARG, "batch must be 2 .. 2^24 (and both size pointers given)");
  const HnTrainWs L = hn_train_layout((long)batch);
  *saved_bytes_out = L.saved_total;
  *scratch_bytes_out = L.scratch_total;
  return HN_OK;
}

static int train_args(int64_t batch, const void* const* ptrs, int n, void* saved, size_t saved_bytes, void* scratch,
                      size_t scratch_bytes) {
  size_t need_sv = 0, need_sc = 0;
  int rc = hn_hardnet_train_workspace_bytes(batch, &need_sv, &need_sc);
  if (rc) return rc;
  if (!saved || !scratch) return fail(HN_ERR_ARG, "NULL workspace");
  if (saved_bytes < need_sv)
    return fail(HN_ERR_WORKSPACE, "saved workspace too small: need " + std::to_string(need_sv) + " bytes");
  if (scratch_bytes < need_sc)
    return fail(HN_ERR_WORKSPACE, "scratch workspace too small: need " + std::to_string(need_sc) + " bytes");
  if (!ptrs) return fail(HN_ERR_ARG, "NULL weight pointer array");
  for (int i = 0; i < n; ++i)
    if (!ptrs[i]) return fail(HN_ERR_ARG, "NULL weight pointer " + std::to_string(i));
  return HN_OK;
}

extern "C" int hn_hardnet_train_forward(const float* d_in, int64_t batch, const float* const* d_weights,
                                        float* const* d_running_mean, float* const* d_running_var, float momentum,
                                        float dropout_p, uint64_t seed, float* d_out, void* d_saved,
                                        size_t saved_bytes, void* d_scratch, size_t scratch_bytes,
                                        void* hip_stream) {
  int rc = train_args(batch, reinterpret_cast<const void* const*>(d_weights), 7, d_saved, saved_bytes, d_scratch,
                      scratch_bytes);
  if (rc) return rc;
  if (!d_in || !d_out) return fail(HN_ERR_ARG, "NULL device pointer");
  if ((d_running_mean == nullptr) != (d_running_var == nullptr))
    return fail(HN_ERR_ARG, "running_mean and running_var must both be given or both NULL");
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(HN_ERR_ARG, "dropout_p must be in [0, 1)");
  HIPCHK(hn_train_forward(d_in, (long)batch, d_weights, d_running_mean, d_running_var, momentum, 1e-5f, 1e-7f,
                          1e-10f, dropout_p, (unsigned long long)seed, d_out, static_cast<char*>(d_saved),
                          static_cast<char*>(d_scratch), static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_hardnet_train_backward(const float* d_dout, int64_t batch, const float* const* d_weights,
                                         float* const* d_dweights, float* d_din, float dropout_p, uint64_t seed,
                                         void* d_saved, size_t saved_bytes, void* d_scratch, size_t scratch_bytes,
                                         void* hip_stream) {
  int rc = train_args(batch, reinterpret_cast<const void* const*>(d_weights), 7, d_saved, saved_bytes, d_scratch,
                      scratch_bytes);
  if (rc) return rc;
  if (!d_dout) return fail(HN_ERR_ARG, "NULL device pointer");
  if (!d_dweights) return fail(HN_ERR_ARG, "NULL gradient pointer array");
  for (int i = 0; i < 7; ++i)
    if (!d_dweights[i]) return fail(HN_ERR_ARG, "NULL gradient pointer " + std::to_string(i));
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(HN_ERR_ARG, "dropout_p must be in [0, 1)");
  HIPCHK(hn_train_backward(d_dout, (long)batch, d_weights, d_dweights, d_din, 1e-10f, dropout_p,
                           (unsigned long long)seed, static_cast<char*>(d_saved), static_cast<char*>(d_scratch),
                           static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

// ---------------------------------------------------------------------------------------
// train-mode hardnetNAS (hn_nas_train.hip)
// ---------------------------------------------------------------------------------------
static int nas_train_desc_ok(const hn_arch_desc* d) {
  if (!d) return fail(HN_ERR_ARG, "NULL desc");
  const bool fdl = d->kind == HN_KIND_FDL_NASNET || d->kind == HN_KIND_FDL_NASNET01;
  if (d->kind != HN_KIND_NAS && d->kind != HN_KIND_NAS_SUPERNET && !fdl)
    return fail(HN_ERR_ARG, "train mode: desc kind must be HN_KIND_NAS, HN_KIND_NAS_SUPERNET or an FDL kind");
  if (d->n_layers < 1 || d->n_layers > HN_MAX_LAYERS) return fail(HN_ERR_ARG, "bad n_layers");
  if (fdl && !(d->input_norm_eps >= 0.f)) return fail(HN_ERR_ARG, "FDL: input_norm_eps must be >= 0");
  int hw = fdl ? 8 : 32, c = fdl ? 64 : 32;  // the FDL fronts leave 64 channels at 8x8
  for (int i = 0; i < d->n_layers; ++i) {
    if (d->kind != HN_KIND_NAS_SUPERNET && (d->op[i] < 0 || d->op[i] >= 17)) return fail(HN_ERR_ARG, "bad op index");
    if (d->c_in[i] != c || (d->stride[i] != 1 && d->stride[i] != 2) || hw % d->stride[i])
      return fail(HN_ERR_ARG, "layer " + std::to_string(i) + ": channels / stride do not chain");
    if (d->c_out[i] < 1 || d->c_out[i] > 128 || d->c_in[i] % 4 || d->c_out[i] % 4)
      return fail(HN_ERR_ARG, "layer " + std::to_string(i) + ": channel count");
    c = d->c_out[i];
    hw /= d->stride[i];
  }
  if (hw != 4) return fail(HN_ERR_ARG, "the layers must reduce the front's output to the 4x4 head input");
  return HN_OK;
}

extern "C" int hn_nas_train_tensor_count(const hn_arch_desc* desc, size_t* n_out) {
  int rc = nas_train_desc_ok(desc);
  if (rc) return rc;
  if (!n_out) return fail(HN_ERR_ARG, "NULL n_out");
  hn_nas_train_plan(*desc, 2, n_out, nullptr, nullptr);
  return HN_OK;
}

extern "C" int hn_nas_train_workspace_bytes(const hn_arch_desc* desc, int64_t batch, size_t* saved_bytes_out,
                                            size_t* scratch_bytes_out) {
  int rc = nas_train_desc_ok(desc);
  if (rc) return rc;
  if (!saved_bytes_out || !scratch_bytes_out || batch < 2 || batch > (1 << 22))
    return fail(HN_ERR_ARG, "batch must be 2 .. 2^22 (and both size pointers given)");
  hn_nas_train_plan(*desc, (long)batch, nullptr, saved_bytes_out, scratch_bytes_out);
  return HN_OK;
}

static int nas_train_args(const hn_arch_desc* desc, int64_t batch, float* const* tensors, void* saved,
                          size_t saved_bytes, void* scratch, size_t scratch_bytes, const float* soft) {
  size_t need_sv = 0, need_sc = 0, nt = 0;
  int rc = hn_nas_train_workspace_bytes(desc, batch, &need_sv, &need_sc);
  if (rc) return rc;
  hn_nas_train_plan(*desc, (long)batch, &nt, nullptr, nullptr);
  if (!saved || !scratch) return fail(HN_ERR_ARG, "NULL workspace");
  if (saved_bytes < need_sv)
    return fail(HN_ERR_WORKSPACE, "saved workspace too small: need " + std::to_string(need_sv) + " bytes");
  if (scratch_bytes < need_sc)
    return fail(HN_ERR_WORKSPACE, "scratch workspace too small: need " + std::to_string(need_sc) + " bytes");
  if (!tensors) return fail(HN_ERR_ARG, "NULL tensor pointer array");
  for (size_t i = 0; i < nt; ++i)
    if (!tensors[i]) return fail(HN_ERR_ARG, "NULL tensor pointer " + std::to_string(i));
  if (desc->kind == HN_KIND_NAS_SUPERNET && !soft) return fail(HN_ERR_ARG, "the supernet needs d_soft");
  return HN_OK;
}

extern "C" int hn_nas_train_forward(const hn_arch_desc* desc, const float* d_in, int64_t batch, float* const* d_tensors,
                                    float momentum, const float* d_soft, float* d_out, void* d_saved,
                                    size_t saved_bytes, void* d_scratch, size_t scratch_bytes, void* hip_stream) {
  int rc = nas_train_args(desc, batch, d_tensors, d_saved, saved_bytes, d_scratch, scratch_bytes, d_soft);
  if (rc) return rc;
  if (!d_in || !d_out) return fail(HN_ERR_ARG, "NULL device pointer");
  HIPCHK(hn_nas_train_forward_impl(*desc, d_in, (long)batch, d_tensors, momentum, d_soft, d_out,
                                   static_cast<char*>(d_saved), static_cast<char*>(d_scratch),
                                   static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_nas_train_backward(const hn_arch_desc* desc, const float* d_dout, const float* d_in, int64_t batch,
                                     float* const* d_tensors, const float* d_soft, float* const* d_grads,
                                     float* d_dsoft, void* d_saved, size_t saved_bytes, void* d_scratch,
                                     size_t scratch_bytes, void* hip_stream) {
  int rc = nas_train_args(desc, batch, d_tensors, d_saved, saved_bytes, d_scratch, scratch_bytes, d_soft);
  if (rc) return rc;
  if (!d_dout || !d_in) return fail(HN_ERR_ARG, "NULL device pointer");
  if (!d_grads) return fail(HN_ERR_ARG, "NULL gradient pointer array");
  if (const int slot = hn_nas_train_null_grad_slot(*desc, d_grads); slot >= 0) {
    return fail(HN_ERR_ARG, "d_grads[" + std::to_string(slot) + "] is NULL: every weight slot needs a gradient buffer");
  }
  if (desc->kind == HN_KIND_NAS_SUPERNET && !d_dsoft) return fail(HN_ERR_ARG, "the supernet needs d_dsoft");
  HIPCHK(hn_nas_train_backward_impl(*desc, d_dout, (long)batch, d_in, d_tensors, d_soft, d_grads, d_dsoft,
                                    static_cast<char*>(d_saved), static_cast<char*>(d_scratch),
                                    static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_hardnet_loss_train_workspace_bytes(int64_t batch, size_t* bytes_out) {
  if (!bytes_out || batch < 1 || batch > (1 << 22)) return fail(HN_ERR_ARG, "batch out of range");
  *bytes_out = hn_loss_train_saved_bytes((long)batch);
  return HN_OK;
}

static int loss_train_args(const float* a, const float* p, int64_t batch, int32_t dim, int32_t loss_type,
                           void* saved, size_t saved_bytes) {
  if (!a || !p || !saved) return fail(HN_ERR_ARG, "NULL device pointer");
  if (batch < 1 || batch > (1 << 22)) return fail(HN_ERR_ARG, "batch out of range");
  if (dim != 128) return fail(HN_ERR_ARG, "dim must be 128");
  if (loss_type < 0 || loss_type > 2) return fail(HN_ERR_ARG, "unknown loss_type");
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(saved)) & 15)
    return fail(HN_ERR_ARG, "device pointers must be 16-byte aligned");
  if (saved_bytes < hn_loss_train_saved_bytes((long)batch)) return fail(HN_ERR_WORKSPACE, "saved workspace too small");
  return HN_OK;
}

extern "C" int hn_hardnet_loss_train_forward(const float* d_anchor, const float* d_positive, int64_t batch,
                                             int32_t dim, int32_t anchor_swap, float margin, int32_t loss_type,
                                             float* d_loss, void* d_saved, size_t saved_bytes, void* hip_stream) {
  if (int rc = loss_train_args(d_anchor, d_positive, batch, dim, loss_type, d_saved, saved_bytes)) return rc;
  if (!d_loss) return fail(HN_ERR_ARG, "NULL device pointer");
  HIPCHK(hn_launch_loss_train_fwd(d_anchor, d_positive, (int)batch, anchor_swap ? 1 : 0, margin, loss_type, d_loss,
                                  d_saved, static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_hardnet_loss_backward(const float* d_anchor, const float* d_positive, int64_t batch, int32_t dim,
                                        int32_t anchor_swap, float margin, int32_t loss_type, const float* d_dloss,
                                        float* d_grad_anchor, float* d_grad_positive, void* d_saved,
                                        size_t saved_bytes, void* hip_stream) {
  if (int rc = loss_train_args(d_anchor, d_positive, batch, dim, loss_type, d_saved, saved_bytes)) return rc;
  if (!d_dloss || !d_grad_anchor || !d_grad_positive) return fail(HN_ERR_ARG, "NULL device pointer");
  if ((reinterpret_cast<uintptr_t>(d_grad_anchor) | reinterpret_cast<uintptr_t>(d_grad_positive)) & 7)
    return fail(HN_ERR_ARG, "gradient pointers must be 8-byte aligned");
  HIPCHK(hn_launch_loss_train_bwd(d_anchor, d_positive, (int)batch, anchor_swap ? 1 : 0, margin, loss_type, d_dloss,
                                  d_grad_anchor, d_grad_positive, d_saved, static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_pairdist_workspace_bytes(int64_t batch, size_t* bytes_out) {
  if (!bytes_out || batch < 0) return fail(HN_ERR_ARG, "bad argument");
  // column minima (padded to 64 entries) + the row kernel's workspace (hn_pairdist_rows_ws_bytes)
  const long b = batch > 0 ? (long)batch : 1;
  *bytes_out = (size_t)((b + 63) / 64 * 64) * sizeof(float) + hn_pairdist_rows_ws_bytes(b, b);
  return HN_OK;
}

extern "C" int hn_pairdist_hardneg(const float* d_anchor, const float* d_positive, int64_t batch,
                                   int32_t dim, int32_t anchor_swap, float* d_pos,
                                   float* d_min_neg, void* d_workspace, size_t workspace_bytes,
                                   void* hip_stream) {
  if (!d_anchor || !d_positive || !d_pos || !d_min_neg || !d_workspace)
    return fail(HN_ERR_ARG, "NULL device pointer");
  if (batch < 2 || batch > (1 << 30)) return fail(HN_ERR_ARG, "batch out of range");
  if (dim != 128) return fail(HN_ERR_ARG, "dim must be 128");
  size_t need = 0;
  hn_pairdist_workspace_bytes(batch, &need);
  if (workspace_bytes < need) return fail(HN_ERR_WORKSPACE, "workspace too small");
  HIPCHK(hn_launch_pairdist(d_anchor, d_positive, (int)batch, dim, anchor_swap, d_pos, d_min_neg,
                            d_workspace, static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_pairdist_rows_workspace_bytes(int64_t n_rows, int64_t batch, size_t* bytes_out) {
  if (!bytes_out || n_rows < 1 || batch < 2 || batch > (1 << 30) || n_rows > batch)
    return fail(HN_ERR_ARG, "bad n_rows / batch");
  *bytes_out = hn_pairdist_rows_ws_bytes((long)n_rows, (long)batch);
  return HN_OK;
}

extern "C" int hn_pairdist_rows(const float* d_anchor_rows, int64_t n_rows, int64_t row0,
                                const float* d_positive, int64_t batch, int32_t dim, float* d_pos,
                                float* d_row_min, float* d_col_min, void* d_workspace,
                                size_t workspace_bytes, void* hip_stream) {
  if (!d_anchor_rows || !d_positive || !d_pos || !d_row_min || !d_workspace)
    return fail(HN_ERR_ARG, "NULL device pointer");
  if (dim != 128) return fail(HN_ERR_ARG, "dim must be 128");
  size_t need = 0;
  int rc = hn_pairdist_rows_workspace_bytes(n_rows, batch, &need);
  if (rc) return rc;
  if (row0 < 0 || row0 + n_rows > batch) return fail(HN_ERR_ARG, "rows [row0, row0 + n_rows) outside the batch");
  if (workspace_bytes < need) return fail(HN_ERR_WORKSPACE, "workspace too small");
  if ((reinterpret_cast<uintptr_t>(d_anchor_rows) | reinterpret_cast<uintptr_t>(d_positive)) & 15)
    return fail(HN_ERR_ARG, "descriptor pointers must be 16-byte aligned");
  HIPCHK(hn_launch_pairdist_rows(d_anchor_rows, (int)n_rows, (int)row0, d_positive, (int)batch, d_pos,
                                 d_row_min, d_col_min, d_workspace, static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_hardnet_loss(const float* d_pos, const float* d_row_min, const float* d_col_min,
                               int64_t n, float margin, int32_t loss_type, float scale,
                               float* d_min_neg, float* d_loss, void* hip_stream) {
  if (!d_pos || !d_row_min || !d_loss) return fail(HN_ERR_ARG, "NULL device pointer");
  if (n < 1 || n > (1 << 30)) return fail(HN_ERR_ARG, "n out of range");
  if (loss_type < HN_LOSS_TRIPLET_MARGIN || loss_type > HN_LOSS_CONTRASTIVE)
    return fail(HN_ERR_ARG, "unknown loss_type " + std::to_string(loss_type) +
                                " (Losses.py:142-152: triplet_margin, softmax, contrastive)");
  HIPCHK(hn_launch_loss(d_pos, d_row_min, d_col_min, (int)n, margin, loss_type, scale, d_min_neg, d_loss,
                        static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_fpr95_workspace_bytes(int64_t n, size_t* bytes_out) {
  if (!bytes_out || n < 1 || n > (int64_t)1 << 30) return fail(HN_ERR_ARG, "n out of range");
  HIPCHK(hn_fpr95_ws_bytes(n, bytes_out));
  return HN_OK;
}

extern "C" int hn_fpr95(const float* d_anchor, const float* d_positive, const int32_t* d_labels,
                        int64_t n, int32_t dim, float* d_dists, double* d_fpr, void* d_workspace,
                        size_t workspace_bytes, void* hip_stream) {
  if (!d_anchor || !d_positive || !d_labels || !d_fpr || !d_workspace)
    return fail(HN_ERR_ARG, "NULL device pointer");
  if (n < 1 || n > (int64_t)1 << 30 || dim < 1) return fail(HN_ERR_ARG, "bad n / dim");
  size_t need = 0;
  HIPCHK(hn_fpr95_ws_bytes(n, &need));
  if (workspace_bytes < need) return fail(HN_ERR_WORKSPACE, "workspace too small");
  HIPCHK(hn_launch_fpr95(d_anchor, d_positive, d_labels, n, dim, d_dists, d_fpr, d_workspace,
                         workspace_bytes, static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_preprocess(const uint8_t* d_in, int64_t n, int32_t in_hw, int32_t resize,
                             int32_t normalize, float mean, float stdv, float* d_out,
                             void* hip_stream) {
  if (n < 0) return fail(HN_ERR_ARG, "n < 0");
  if (resize != HN_RESIZE_NONE && resize != HN_RESIZE_CV2_LINEAR && resize != HN_RESIZE_PIL_BILINEAR)
    return fail(HN_ERR_ARG, "unknown resize mode " + std::to_string(resize));
  const int want = resize == HN_RESIZE_NONE ? 32 : 64;
  if (in_hw != want)
    return fail(HN_ERR_ARG, "in_hw must be " + std::to_string(want) + " for this resize mode, got " +
                                std::to_string(in_hw));
  if (n == 0) return HN_OK;
  if (!d_in || !d_out) return fail(HN_ERR_ARG, "NULL device pointer");
  if ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_out)) & 15)
    return fail(HN_ERR_ARG, "d_in / d_out must be 16-byte aligned");
  if (normalize && !(stdv != 0.0f)) return fail(HN_ERR_ARG, "std must be nonzero");
  HIPCHK(hn_launch_preprocess(d_in, n, resize, normalize, mean, stdv, d_out,
                              static_cast<hipStream_t>(hip_stream)));
  return HN_OK;
}

extern "C" int hn_set_profiling(hn_model* m, int enable) {
  if (!m) return fail(HN_ERR_ARG, "model is NULL");
  m->prof.on = enable != 0;
  return HN_OK;
}

extern "C" int hn_stage_times(hn_model* m, int max_stages, const char** names_out,
                              double* total_ms_out, int64_t* launches_out) {
  if (!m) return -fail(HN_ERR_ARG, "model is NULL");
  Prof& p = m->prof;
  for (auto& e : p.pend) {
    HIPCHK(hipEventSynchronize(e.b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e.a, e.b));
    p.ms[e.stage] += ms;
    p.cnt[e.stage] += 1;
    p.pool.push_back(e.a);
    p.pool.push_back(e.b);
  }
  p.pend.clear();
  const int n = (int)std::min<size_t>(p.names.size(), (size_t)std::max(0, max_stages));
  for (int i = 0; i < n; ++i) {
    if (names_out) names_out[i] = p.names[i].c_str();
    if (total_ms_out) total_ms_out[i] = p.ms[i];
    if (launches_out) launches_out[i] = p.cnt[i];
    p.ms[i] = 0.0;
    p.cnt[i] = 0;
  }
  return n;
}

extern "C" void hn_destroy(hn_model* m) { delete m; }

extern "C" const char* hn_last_error(void) { return g_err.c_str(); }

extern "C" int hn_abi_version(void) { return HN_ABI_VERSION; }
