// Internal host-side interface between the C ABI (hn_api.hip) and the kernel files.
#pragma once
#include <hip/hip_runtime.h>

#include "hardnet_mi355x.h"

// A/B switches of the launchers.  Read from the environment once per model in hn_create (and
// once per process for the model-less entry points); hn_forward makes the calling model's
// set current for the duration of the call (thread-local), so launchers never call getenv.
// Every switch selects a parity-tested alternative kernel; the ablation switches (c12_abl,
// dbg: timing-only builds with wrong results) exist only in the HN_EXPERIMENTS library.
struct HnKnobs {
  int c12_cfg = 15;            // HN_C12_CFG: k_c12 configuration (0..15, all within the parity bar; 15 = k_c12s)
  int head = 4;                // HN_HEAD: head GEMM form (1 k_head, 2 k_head2, 3 k_head3 LDS-DMA rings, 4 k_head4 256-patch rings)
  bool head_pf = true;         // HN_HEAD_PF: k_head4 reads chunk c + 1 from LDS while chunk c runs (0: off)
  bool fdl_valu = false;       // HN_FDL_VALU: FDLNet front as fp32 VALU
  bool naive_pw = false;       // HN_NAIVE_PW: untiled 1x1 conv kernel
  bool naive_dw = false;       // HN_NAIVE_DW: untiled depthwise kernel
  bool no_skipfuse = false;    // HN_NO_SKIPFUSE: maxpool + pw instead of k_skip_s2 (and no k_irf_skip)
  bool no_irfskip = false;     // HN_NO_IRFSKIP: k_irf + k_skip_s2 instead of k_irf_skip
  bool pairdist_valu = false;  // HN_PAIRDIST_VALU: fp32 VALU pair-distance kernel
  bool pairdist_reg = false;   // HN_PAIRDIST_REG: register-staged positives instead of the LDS-DMA ring
  bool pairdist_spread = true;  // HN_PAIRDIST_SPREAD: the ring's DMA issued inside the MFMA chain (0: before it)
  bool front_fold = false;     // HN_FRONT_FOLD: the NAS front's pwl with the LDS partial-sum fold
  bool u8_apart = false;       // HN_U8_APART: uint8 input preprocessed into the workspace first (A/B)
  bool front_xch3 = false;     // HN_FRONT_XCH3: the k3 front's dw per channel group (SGPR weights, s_x; two
                               // workgroups per CU instead of three: wang2 front 5.05 -> 5.57 ms, not the default)
  bool no_mpfront = false;     // HN_NO_MPFRONT: k_front (max-pool) + k_irf instead of k_mpfront_irf
  bool pipeline = false;       // HN_PIPELINE=1: HardNet batches of several chunks overlap chunk k + 1's k_c12s (second
                               // stream) with chunk k's conv3 .. head (opt-in: measured within noise)
  bool irf3 = false;           // HN_IRF3 (HN_EXPERIMENTS only): k_irf3 for layers 3 -> 4 -> 5 (measured slower)
  int train_splitk = 1024;     // HN_TRAIN_SPLITK: K per split-K slice of the train GEMMs
  int train_f32 = 17;          // HN_TRAIN_F32: bit 0 train forward convs, bit 1 stride-1 dgrads as f32-MFMA
                               // GEMMs (else the bf16x3 conv kernels); 1 = every product f32; default 17 =
                               // f32 forwards, the stride-1 dgrads on the bf16x3 conv kernels;
                               // bit 2: stride-1 weight gradients as the generic GEMM (else k_wgrad3);
                               // bit 3: stride-1 f32 forwards as the generic GEMM (else k_fwd3);
                               // bit 4: stride-1 dgrads not as k_fwd3 over dY (then bit 1 decides);
                               // bit 5: stride-2 layers as the generic GEMM + col2im (else k_fwd2 /
                               // k_wgrad2 / k_dgrad2); bit 6: conv0 as the generic GEMM (else
                               // k_fwd0 / k_wgrad0); bit 7: swaps the one-ring-per-wave and the
                               // shared-ring-per-patch forms (default shared: conv3 / conv5 k_fwd3s,
                               // conv4 k_dgrad2; per wave: conv2 / conv4 k_fwd2)
  int c12w_pd = 11;            // HN_C12W_PD: k_c12w's P2 / P3 B-fragment prefetch distances (tens / units)
  int c12_abl = 0;             // HN_C12_ABL (HN_EXPERIMENTS only)
  int dbg = 0;                 // HN_DEBUG (HN_EXPERIMENTS only)
};
void hn_read_knobs(HnKnobs* k);
const HnKnobs& hn_knobs();

// Resident workgroups of `fn` on the current device at `nthreads` threads and `lds` bytes of
// dynamic LDS (also raises the function's dynamic-LDS limit to `lds` on that device).  Cached
// per (function, device) under a mutex.
hipError_t hn_resident_blocks(const void* fn, int nthreads, int lds, int* resident);

// Device-resident, BN-folded, packed HardNet parameters.
struct HardnetDev {
  float* stem_w = nullptr;   // [9][32]   conv0 folded
  float* stem_b = nullptr;   // [32]
  void* wpack[7] = {};       // conv1..5: bf16 hi/lo MFMA fragments; [6] = head
  float* bias[7] = {};       // folded BN bias per conv
  void* c12_w1 = nullptr;    // conv1 / conv2 as 16x16x32 A operands for the fused k_c12
  void* c12_w2 = nullptr;
  void* c12_w1w = nullptr;   // conv1 as 1-D Winograd F(4,3) U fragments for k_c12w
  void* wino[7] = {};        // conv3 / conv5: Winograd F(2x2,3x3) U fragments (hn_wino.hip)
  void* wino1[7] = {};       // conv3 / conv5: 1-D Winograd F(2,3) U fragments (hn_wino1.hip)
  void* wino4[7] = {};       // conv3: 1-D Winograd F(4,3) U fragments (hn_wino1.hip k_conv_w4)
};
// uint8 patches for the fused preprocessing load (hn_forward_u8)
struct HnU8In {
  const uint8_t* in;  // this chunk's patches
  int resize;         // enum hn_resize
  int normalize;
  float mean, stdv;
};
// fused input_norm + conv0 + conv1 + conv2 (hn_c12.hip): [P,1,32,32] -> a2 [P,16,16,64]; with
// u8 the patches are uint8 and preprocessed in the load (production configuration only)
hipError_t hn_launch_c12(const float* in, float* out, const HardnetDev& d, int P, float eps,
                         hipStream_t st, const HnU8In* u8 = nullptr);

hipError_t hn_launch_stem(const float* in, float* out, const float* w, const float* b, int P,
                          bool norm, float eps, hipStream_t st);
bool hn_hardnet_variant_ok(int layer, int variant);
bool hn_c12_cfg_ok(int cfg, int abl);
// HN_C12_CFG 14: k_c12w (hn_c12w.hip), conv1 as a 1-D Winograd F(4,3)
constexpr int kC12Wino = 14;
// HN_C12_CFG 15: k_c12s (hn_c12w.hip), k_c12w's arithmetic with conv1 / conv2+stem waves per SIMD
constexpr int kC12Split = 15;
hipError_t hn_launch_c12s(const float* in, float* out, const HardnetDev& d, int P, float eps, hipStream_t st,
                          const HnU8In* u8);
hipError_t hn_launch_c12w(const float* in, float* out, const HardnetDev& d, int P, float eps, hipStream_t st,
                          const HnU8In* u8, int abl);
hipError_t hn_launch_hardnet_conv(int layer, int variant, const HardnetDev& d, const float* in,
                                  float* out, int P, float eps, hipStream_t st);
// part: scratch for the split-K partials of small batches (P <= kHeadSplitMaxP: head_split(K) x P x 128
// floats), or null for the unsplit forms
constexpr int kHeadSplitMaxP = 16384;
constexpr int head_split(int K) { return K / 128; }  // 64 (HardNet, K = 8,192) / 16 (NAS, K = 2,048): 4 K-chunks each
hipError_t hn_launch_head(const float* a, float* out, const void* wp, const float* bias, int P,
                          int K, float l2eps, hipStream_t st, bool f16 = false, float* part = nullptr);
int hn_conv_lds_bytes(int layer);
// train mode: conv layer 1..5 as a plain NHWC convolution (no bias, no ReLU), bf16x3 fragments
// in the pack_conv3x3 layout
hipError_t hn_launch_conv_raw(int layer, const void* wp, const float* zero_bias, const float* in, float* out,
                              int P, hipStream_t st);
// 1-D Winograd F(2,3) conv3 / conv5 (hn_wino1.hip; HN_VARIANT digit j)
hipError_t hn_launch_wino1(int layer, int wd, const HardnetDev& d, const float* in, float* out, int P,
                           hipStream_t st);
int hn_wino1_lds_bytes(int layer);
// conv3 as 1-D Winograd F(4,3) (hn_wino1.hip k_conv_w4; HN_VARIANT digits w / x)
hipError_t hn_launch_wino4(int layer, int wd, const HardnetDev& d, const float* in, float* out, int P,
                           hipStream_t st);
// Winograd F(2x2,3x3) conv3 / conv5 (hn_wino.hip; HN_VARIANT digit h)
hipError_t hn_launch_wino(int layer, const HardnetDev& d, const float* in, float* out, int P, hipStream_t st);

hipError_t hn_launch_pw(const float* in, float* out, const float* wt, const float* bias,
                        const float* res, long npix, int cin, int cout, int groups, bool relu,
                        int shuffle_g, hipStream_t st);
hipError_t hn_launch_dw(const float* in, float* out, const float* wd, const float* bias, int P,
                        int hin, int c, int k, int s, hipStream_t st);
hipError_t hn_launch_maxpool(const float* in, float* out, int P, int hin, int c, hipStream_t st);
// fused MaxPool2d(3, 2, 1) + ConvBNRelu 1x1 of the channel-changing "skip" op (hn_nas.hip)
bool hn_skip_s2_supported(int hin, int cin, int cout);
hipError_t hn_launch_skip_s2(const float* in, float* out, const float* wt, const float* bias, int P, int hin,
                             int cin, int cout, hipStream_t st);
hipError_t hn_launch_se(float* y, const float* w1, const float* b1, const float* w2,
                        const float* b2, int P, int hw, int c, int mid, hipStream_t st);
hipError_t hn_launch_nas_head(const float* a, float* out, const float* wt, const float* bias,
                              int P, int K, float l2eps, hipStream_t st);

hipError_t hn_launch_pairdist(const float* a, const float* p, int B, int D, int swap,
                              float* pos, float* minneg, void* ws, hipStream_t st);
// rows [row0, row0 + NA) of the B x B matrix (a = those NA anchors, p = all B positives);
// colmin (float bits, atomicMin; may be NULL) gets the column minima over these rows
size_t hn_pairdist_rows_ws_bytes(long NA, long B);
hipError_t hn_launch_pairdist_rows(const float* a, int NA, int row0, const float* p, int B, float* pos,
                                   float* rowmin, float* colmin, void* ws, hipStream_t st);
hipError_t hn_launch_loss(const float* pos, const float* rmin, const float* cmin, int n, float margin,
                          int type, float scale, float* min_neg, float* loss, hipStream_t st);

hipError_t hn_fpr95_ws_bytes(int64_t n, size_t* bytes);
// fused NAS front (stem + layer 0), hn_front.hip
struct HnFrontArgs {
  const float* in;
  float* out;
  const uint4* spack;   // stem A operand, [plane 2][lane 64] x 8 fp16 (taps 8h..8h+7)
  const float* stem_b;
  const uint4* apack;   // pw A operand, [MID/32][kstep 2][plane 2][lane 64] x 8 fp16
  const float* pw_b;    // [MID], dw channel order
  const float* dw_w;    // [K*K][MID]
  const float* dw_b;
  const uint4* pwl_a;   // pwl A operand, [1][MID/16][plane 2][lane 64] x 8 fp16
  const float* pwl_b;   // [32]
  const uint4* pwl_a16; // pwl A operand for 16x16x32: [MID/32][out tile 2][plane 2][lane 64] x 8 fp16
};
bool hn_front_supported(int k, int mid);
// u8: uint8 patches preprocessed in the front's patch load (the production forms without
// input_norm, HN_FRONT_FOLD off; hn_api.hip u8_fused)
hipError_t hn_launch_front(const HnFrontArgs& a, int P, int k, int mid, bool maxpool, bool norm,
                           float eps, hipStream_t st, const HnU8In* u8 = nullptr);
// FDLNet HardNetNeiMask front (32x32 patch -> 8x8x64), hn_fdl.hip; mode 0 = NASNet, 1 = NASNet_0.1
struct HnFdlFrontArgs {
  const float* in;
  float* out;
  const float *stem_w, *stem_b;  // [9][32], [32]
  const float *w1, *b1;          // [32][32], [32] (mode 0)
  const float *w2, *b2;          // [32][64], [64]
};
// u8: uint8 patches preprocessed in the patch load (hn_forward_u8), else a.in (fp32)
hipError_t hn_launch_fdl_front(const HnFdlFrontArgs& a, int P, int mode, float eps, hipStream_t st,
                               const HnU8In* u8 = nullptr);
// fused IRF block (pw -> dw -> pwl [+ residual]) for layers 1..5, hn_irf.hip
struct HnIrfArgs {
  const float* x;
  float* y;
  const uint4* pw_a;   // [MID/32][CIN/16][plane 2][lane 64] x 8 fp16, rows in dw order
  const float* pw_b;   // [MID] dw order
  const float* dw_w;   // [K*K][MID]
  const float* dw_b;
  const uint4* pwl_a;  // [COUT/32][MID/16][plane 2][lane 64] x 8 fp16
  const float* pwl_b;  // [COUT]
};
bool hn_irf_supported(int cin, int cout, int hin, int s, int k, int mid);
// two consecutive blocks in one kernel (hn_irf.hip k_irf2): A (ca -> ca, stride 1) then B (ca -> cb, stride 2)
bool hn_irf2_supported(int ca, int hi, int ka, int ma, int cb, int kb, int mb);
hipError_t hn_launch_irf2(const HnIrfArgs& a, const HnIrfArgs& b, int P, int ca, int hi, int ka, int ma, int cb,
                          int kb, int mb, hipStream_t st);
hipError_t hn_launch_irf(const HnIrfArgs& a, int P, int cin, int cout, int hin, int s, int k, int mid,
                         hipStream_t st);
// a 16x16 stride-2 32 -> 64 block and the 8x8 64 -> 128 stride-2 skip that follows it (after identity
// skips) in one kernel (hn_irf.hip k_irf_skip); a.y receives the skip's [P,4,4,128] output
bool hn_irf_skip_supported(int cin, int cout, int hin, int s, int k, int mid);
// k_irf2's 8x8 pair (64 -> 64 s1, 64 -> 128 s2, mid 64) and the 4x4 128 -> 128 e1 block in one kernel (k_irf3,
// experiments library only)
bool hn_irf3_supported(int ka, int ma, int kb, int mb, int kc, int mc);
hipError_t hn_launch_irf3(const HnIrfArgs& a, const HnIrfArgs& b, const HnIrfArgs& c, int P, int ka, int kb, int kc,
                          hipStream_t st);
// the max-pool front + the first (16x16 stride-2 32 -> 64) IRF block in one kernel (hn_irf.hip k_mpfront_irf)
bool hn_mpfront_irf_supported(int cin, int cout, int hin, int s, int k, int mid);
hipError_t hn_launch_mpfront_irf(const float* in, const uint4* spack, const float* stem_b, const HnIrfArgs& a, int P,
                                 int k, int mid, bool norm, float eps, hipStream_t st);
hipError_t hn_launch_irf_skip(const HnIrfArgs& a, const uint4* skip_a, const float* skip_b, int P, int k, int mid,
                              hipStream_t st);
hipError_t hn_launch_preprocess(const uint8_t* in, int64_t n, int resize, int norm, float mean,
                                float stdv, float* out, hipStream_t st);
hipError_t hn_launch_fpr95(const float* a, const float* p, const int* labels, int64_t n, int dim,
                           float* dists, double* fpr, void* ws, size_t ws_bytes, hipStream_t st);

// train-mode stock HardNet (hn_train.hip): conv shapes and workspace layout
struct HnTrainLayer {
  int cin, cout, hin, ks, s, pad;
};
extern const HnTrainLayer kHardnetTrainLayers[7];
// CANDIDATE_BLOCKS (lookup_table_builder.py:18-20) as (skip, expansion, kernel, pw groups, SE);
// the ChannelShuffle runs iff groups > 1 (fbnet_builder.py:36-191); defined in hn_api.hip
struct HnOpSpec {
  const char* name;
  int skip, e, k, g, se;
};
extern const HnOpSpec kHnOps[17];

struct HnTrainWs {  // byte offsets into the train workspace's saved region (xn .. rstd) / scratch region
  size_t xn, inv_sd, z[7], rstd[7], saved_total;
  size_t g0, g1, col, part, bnpart, bnmean, wt, nhwc0, nhwc1, wpack, zero, scratch_total;
};
HnTrainWs hn_train_layout(long B);
// train-mode hardnetNAS (hn_nas_train.hip): tensors consumed, saved / scratch workspace bytes
int hn_nas_train_plan(const hn_arch_desc& d, long B, size_t* n_tensors, size_t* saved, size_t* scratch);
int hn_nas_train_null_grad_slot(const hn_arch_desc& d, float* const* grads);
hipError_t hn_nas_train_forward_impl(const hn_arch_desc& d, const float* in, long B, float* const* tensors,
                                     float momentum, const float* soft, float* out, char* saved, char* scratch,
                                     hipStream_t st);
hipError_t hn_nas_train_backward_impl(const hn_arch_desc& d, const float* dout, long B, const float* in,
                                      float* const* tensors, const float* soft, float* const* grads, float* dsoft,
                                      char* saved, char* scratch, hipStream_t st);
hipError_t hn_train_forward(const float* in, long B, const float* const* W, float* const* rmean, float* const* rvar,
                            float mom, float bn_eps, float in_eps, float l2_eps, float drop_p,
                            unsigned long long seed, float* out, char* saved, char* scratch, hipStream_t st);
hipError_t hn_train_backward(const float* dout, long B, const float* const* W, float* const* dW, float* din,
                             float l2_eps, float drop_p, unsigned long long seed, char* saved, char* scratch,
                             hipStream_t st);

// train-mode loss_HardNet 'min' reduce and its backward (hn_loss.hip)
size_t hn_loss_train_saved_bytes(long B);
hipError_t hn_launch_loss_train_fwd(const float* a, const float* p, int B, int swap, float margin, int type,
                                    float* loss, void* saved, hipStream_t st);
hipError_t hn_launch_loss_train_bwd(const float* a, const float* p, int B, int swap, float margin, int type,
                                    const float* dloss, float* ga, float* gp, void* saved, hipStream_t st);
