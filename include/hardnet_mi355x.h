/*
 * hardnet_mi355x.h -- C ABI of the MI355X-native HardNet / hardnetNAS descriptor forward.
 *
 * This is the drop-in boundary for the reference hot path
 *   hardnet/HardNet.py:312-315          HardNet.forward(input [B,1,32,32]) -> [B,128]
 *   hardnet/HardNet.py:306-310          HardNet.input_norm (fused into hn_forward)
 *   hardnet/Utils.py:15-22              L2Norm (fused into hn_forward)
 *   hardnetNAS/supernet_functions/model_supernet.py:70-85
 *                                       sampled-supernet forward (argmax op per layer)
 *   hardnet/Losses.py:5-13,87-154       distance_matrix_vector + loss_HardNet 'min' reduce
 *                                       (hn_pairdist_hardneg)
 * The reference is pure PyTorch and has no FFI of its own; the Python host package
 * (hardnetnas_amd/_native.py) binds these entry points with ctypes -- see
 * INTEGRATION.md for the binding a maintainer adds to the reference.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Device pointers are HIP device memory owned by the
 *    caller; nothing is copied host<->device inside hn_forward.
 *  - Every call is ordered on the caller's HIP stream (hipStream_t passed as void*;
 *    NULL = the legacy default stream).  No allocation or synchronisation happens inside
 *    hn_forward / hn_pairdist_hardneg, so they can be captured in a hipGraph.
 *  - Return value 0 = success; nonzero = error, message in hn_last_error() (thread-local).
 *    The library never exits the process.
 */
#ifndef HARDNET_MI355X_H
#define HARDNET_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HN_ABI_VERSION 2

enum hn_status {
  HN_OK = 0,
  HN_ERR_ARG = 1,      /* invalid argument / shape / size mismatch */
  HN_ERR_HIP = 2,      /* HIP runtime error (message has the HIP error string) */
  HN_ERR_NOMEM = 3,    /* device allocation failed */
  HN_ERR_WORKSPACE = 4 /* workspace too small for the requested batch */
};

enum hn_kind {
  HN_KIND_HARDNET = 0,      /* stock HardNet, hardnet/HardNet.py:275-304 */
  HN_KIND_NAS = 1,          /* sampled hardnetNAS net, model_supernet.py:53-85 */
  HN_KIND_FDL_NASNET = 2,   /* FDLNet HardNetNeiMask, FDLNet-master/latency/NASNet/model/des.py:8-55 */
  HN_KIND_FDL_NASNET01 = 3, /* FDLNet HardNetNeiMask, FDLNet-master/latency/NASNet_0.1/model/des.py:10-55 */
  HN_KIND_NAS_SUPERNET = 4  /* train mode only: FBNet_Stochastic_SuperNet, model_supernet.py:53-85 (every layer
                               a MixedOperation over all 17 CANDIDATE_BLOCKS, :10-36) */
};

#define HN_MAX_LAYERS 8

/* Architecture description.
 *  HardNet: only kind, input_norm_eps, l2_eps, bn_eps are read.
 *  NAS:     op[i] = index into CANDIDATE_BLOCKS (lookup_table_builder.py:18-20);
 *           c_in/c_out/stride from SEARCH_SPACE2 (lookup_table_builder.py:22-45).
 *  FDL:     a fixed front (des.py) to 8x8x64, then op/c_in/c_out/stride of its IRFBlocks in the
 *           same CANDIDATE_BLOCKS vocabulary (NASNet: ir_k5_e1 64->64, ir_k3_e3 64->128 s2,
 *           ir_k5_s2 128->128), then the 4x4 head; input_norm_eps 1e-8, l2_eps 0.
 *  input_norm_eps < 0 disables input_norm (the NAS nets have none);
 *  l2_eps: HardNet 1e-10 inside the sqrt (Utils.py:18); NAS 0 (torch.norm, model_supernet.py:84). */
typedef struct hn_arch_desc {
  int32_t kind;
  int32_t n_layers;
  int32_t op[HN_MAX_LAYERS];
  int32_t c_in[HN_MAX_LAYERS];
  int32_t c_out[HN_MAX_LAYERS];
  int32_t stride[HN_MAX_LAYERS];
  float input_norm_eps;
  float l2_eps;
  float bn_eps;
} hn_arch_desc;

typedef struct hn_model hn_model;

/* Number of floats hn_create expects in host_params for this architecture. */
int hn_param_count(const hn_arch_desc* desc, size_t* n_out);

/* Build a device model on the current HIP device from host fp32 parameters.
 * host_params is the concatenation, in state_dict order, of every conv weight and
 * BatchNorm tensor of the module (HardNet: for each of the 7 convs
 *   features.{c}.weight, features.{b}.running_mean, features.{b}.running_var;
 * NAS / FDL: see hardnetnas_amd/_native.py::state_dict_blob, which documents the order).
 * BatchNorm (eval) is folded into the conv weights/bias here, once. */
int hn_create(const hn_arch_desc* desc, const float* host_params, size_t n_params,
              hn_model** out);

/* Bytes of device workspace hn_forward needs for a batch of B patches.  The forward walks the batch in
 * chunks of min(B, 65,536) patches and sizes the workspace for one chunk; for the stock HardNet at the
 * defaults that is 160 KiB per patch: 10 GiB from 65,536 patches up, 80 MiB at the reference eval loop's
 * 512.  Two environment knobs, read by hn_create, bound it for the stock HardNet (both default 65,536; any
 * values give bit-identical descriptors): HN_C12_GROUP (patches per fused stem+conv1+conv2 launch) and
 * HN_SUBCHUNK (patches per conv3..conv5 launch); the footprint is (HN_SUBCHUNK + HN_C12_GROUP) x 64 KiB +
 * chunk x 32 KiB, e.g. 4 GiB per 65,536-patch chunk at 16,384 / 16,384 (about 4 % slower end to end).
 * HN_PIPELINE=1 (opt-in) overlaps a multi-chunk HardNet batch's chunks over a second, internally created
 * stream (forked from and joined back into hip_stream, so graph capture holds) and adds one more
 * chunk x 64 KiB buffer for batches of more than one chunk.
 * NAS / FDL descriptors need four buffers of their largest per-patch activation. */
int hn_workspace_bytes(const hn_model* m, int64_t batch, size_t* bytes_out);

/* d_in: [B,1,32,32] fp32 contiguous (device); d_out: [B,128] fp32 (device).
 * Eval-mode forward of the whole descriptor network (HardNet: input_norm, 7 conv+BN
 * stages, ReLU, L2Norm; NAS: stem, 6 searched blocks, 4x4 head, BN, L2). */
int hn_forward(hn_model* m, const float* d_in, int64_t batch, float* d_out,
               void* d_workspace, size_t workspace_bytes, void* hip_stream);

/* Fused distance_matrix_vector + hardest-in-batch negative (loss_HardNet 'min' reduce,
 * hardnet/Losses.py:87-154) without materialising the B x B matrix.
 * d_anchor, d_positive: [B,D] fp32.  Outputs (device, [B] fp32 each):
 *   d_pos[i]     = dist(a_i, p_i) + 1e-8              (pos1)
 *   d_min_neg[i] = min_j masked dist(a_i, p_j)        (row min, or min(row,col) if anchor_swap)
 * d_workspace needs hn_pairdist_workspace_bytes(B). */
int hn_pairdist_workspace_bytes(int64_t batch, size_t* bytes_out);
int hn_pairdist_hardneg(const float* d_anchor, const float* d_positive, int64_t batch, int32_t dim,
                        int32_t anchor_swap, float* d_pos, float* d_min_neg,
                        void* d_workspace, size_t workspace_bytes, void* hip_stream);

/* Row block of the same computation, for a batch sharded over ranks: rows
 * [row0, row0 + n_rows) of the batch x batch distance matrix between this rank's anchors
 * d_anchor_rows [n_rows, dim] and ALL positives d_positive [batch, dim] (all-gathered).
 * Outputs for the local rows: d_pos[i] = dist(a_i, p_{row0+i}) + 1e-8, d_row_min[i] = masked
 * row minimum; if d_col_min is not NULL it receives, for every column j of the batch, the
 * masked minimum over these rows (reduce it across ranks with an all-reduce(MIN), then
 * min_neg = min(row_min, col_min[row0 + i]) for anchor_swap; hn_hardnet_loss does that).
 * The single-GPU hn_pairdist_hardneg is this call with row0 = 0, n_rows = batch. */
int hn_pairdist_rows_workspace_bytes(int64_t n_rows, int64_t batch, size_t* bytes_out);
int hn_pairdist_rows(const float* d_anchor_rows, int64_t n_rows, int64_t row0, const float* d_positive,
                     int64_t batch, int32_t dim, float* d_pos, float* d_row_min, float* d_col_min,
                     void* d_workspace, size_t workspace_bytes, void* hip_stream);

/* loss_HardNet's margin loss over the 'min' reduce (hardnet/Losses.py:142-153) for n rows:
 * min_neg = d_col_min ? min(d_row_min, d_col_min) : d_row_min (written to d_min_neg if not
 * NULL); *d_loss = scale * sum_i loss_i (scale = 1/B for torch.mean; with a sharded batch
 * every rank passes 1/B_total and the partial sums are all-reduced).  One workgroup, fixed
 * summation order (deterministic). */
enum hn_loss_type { HN_LOSS_TRIPLET_MARGIN = 0, HN_LOSS_SOFTMAX = 1, HN_LOSS_CONTRASTIVE = 2 };
int hn_hardnet_loss(const float* d_pos, const float* d_row_min, const float* d_col_min, int64_t n,
                    float margin, int32_t loss_type, float scale, float* d_min_neg, float* d_loss,
                    void* hip_stream);

/* Train-mode loss_HardNet, batch_reduce 'min' (hardnet/Losses.py:87-154 as the training loop calls
 * it, HardNet.py:408-413) and its backward (HardNet.py:421-423), without a B x B matrix.
 *   forward : *d_loss = mean_i loss(pos_i, min_neg_i) over d_anchor / d_positive [B,128] fp32
 *             (exact fp32 dot products; the hardest negatives and their argmins -- the first index
 *             on a tie -- are kept in d_saved);
 *   backward: d_dloss (one float on the device: d L / d loss) -> d_grad_anchor, d_grad_positive
 *             [B,128] (overwritten), as autograd differentiates the reference formulation: the
 *             gradient reaches each row's positive entry and its selected negative (the row
 *             minimum's argmin, the column minimum's for anchor_swap; halves on a row / column
 *             tie, as torch.minimum's backward).  Deterministic: no atomics in the backward.
 * d_saved (hn_hardnet_loss_train_workspace_bytes) is written by the forward and read by the
 * backward with the same anchors, positives and arguments; 1 <= batch <= 2^22. */
int hn_hardnet_loss_train_workspace_bytes(int64_t batch, size_t* bytes_out);
int hn_hardnet_loss_train_forward(const float* d_anchor, const float* d_positive, int64_t batch, int32_t dim,
                                  int32_t anchor_swap, float margin, int32_t loss_type, float* d_loss,
                                  void* d_saved, size_t saved_bytes, void* hip_stream);
int hn_hardnet_loss_backward(const float* d_anchor, const float* d_positive, int64_t batch, int32_t dim,
                             int32_t anchor_swap, float margin, int32_t loss_type, const float* d_dloss,
                             float* d_grad_anchor, float* d_grad_positive, void* d_saved, size_t saved_bytes,
                             void* hip_stream);

/* FPR at 95 % recall of an evaluation batch of descriptor pairs (hardnet/HardNet.py:450-472
 * + hardnet/EvalMetrics.py:6-19): per-pair L2 distance, scores -> distances transform, sort,
 * first index reaching 95 % recall, FP / (FP + TN).
 * d_anchor, d_positive: [n,dim] fp32; d_labels: [n] int32 (1 = match).  Outputs: d_dists
 * ([n] fp32 pair distances, may be NULL) and d_fpr (one double; NaN if there are no
 * negatives).  Ties are ordered stably (numpy's quicksort order is unspecified). */
int hn_fpr95_workspace_bytes(int64_t n, size_t* bytes_out);
int hn_fpr95(const float* d_anchor, const float* d_positive, const int32_t* d_labels, int64_t n,
             int32_t dim, float* d_dists, double* d_fpr, void* d_workspace, size_t workspace_bytes,
             void* hip_stream);

/* Patch preprocessing: uint8 patches -> fp32 [n,1,32,32] network input,
 * bit-exact with the reference loaders.
 *   HN_RESIZE_CV2_LINEAR   hardnet/HardNet.py:345-349 'transform' + Utils.py:10-11 cv2_scale:
 *                          64x64 -> 32x32 cv2 INTER_LINEAR (= OpenCV's 2x area-fast path)
 *   HN_RESIZE_PIL_BILINEAR hardnet/HardNet.py:333-337 'transform_test': PIL Resize(32), bilinear
 *   HN_RESIZE_NONE         input already 32x32 (cv2.resize to the same size is a copy)
 * then ToTensor (/255) and, if normalize != 0, Normalize((mean,), (std,)) in fp32.
 * d_in: [n, in_hw, in_hw] uint8 (in_hw 64 for the resizing modes, 32 for NONE). */
enum hn_resize { HN_RESIZE_NONE = 0, HN_RESIZE_CV2_LINEAR = 1, HN_RESIZE_PIL_BILINEAR = 2 };
int hn_preprocess(const uint8_t* d_in, int64_t n, int32_t in_hw, int32_t resize, int32_t normalize,
                  float mean, float std, float* d_out, void* hip_stream);

/* Descriptor forward from uint8 patches (the loader transforms of
 * hardnet/HardNet.py:333-337 / 345-349 + Utils.py:10-11 fused into the network's patch load):
 * d_in [B, in_hw, in_hw] uint8; resize / normalize / mean / std as hn_preprocess.  Equals
 * hn_preprocess followed by hn_forward bit for bit.  For the stock HardNet, FDLNet and the
 * hardnetNAS descriptors (every resize mode) the preprocessing runs inside the first fused kernel
 * (k_c12 / the FDLNet and NAS fronts: 4 / 1 KiB of input HBM per patch and no fp32 copy); the k5
 * NAS front in PIL mode (measured faster apart) and the A/B configurations (HN_NO_FRONT,
 * HN_FRONT_FOLD, HN_FDL_VALU, HN_U8_APART) preprocess each chunk into the workspace tail first.
 * Workspace: hn_workspace_bytes_u8. */
int hn_workspace_bytes_u8(const hn_model* m, int64_t batch, size_t* bytes_out);
int hn_forward_u8(hn_model* m, const uint8_t* d_in, int64_t batch, int32_t in_hw, int32_t resize,
                  int32_t normalize, float mean, float std, float* d_out, void* d_workspace,
                  size_t workspace_bytes, void* hip_stream);

/* Train-mode stock HardNet (the module of hardnet/HardNet.py:275-315 in
 * model.train() as the training loop :379-441 runs it through autograd).
 *  forward : input_norm (mean / std detached), 7 x [conv -> BatchNorm2d(affine=False) with the
 *            batch's statistics (running_mean / running_var updated in place with `momentum`,
 *            unbiased variance) -> ReLU], Dropout(dropout_p) before conv6, L2Norm.
 *  backward: d_dout [B,128] -> d_dweights[l] (each [Cout,Cin,k,k] like the module's weights,
 *            overwritten), and d_din [B,1,32,32] if not NULL.
 * d_weights / d_running_* / d_dweights are host arrays of 7 device pointers (features.{0,3,6,9,
 * 12,15,19}.weight and the matching BN buffers, fp32 contiguous).  The workspace has two parts:
 *   d_saved   -- written by the forward, read by its backward: keep it unchanged between a
 *                forward and its backward (the training loop's two forwards, anchors and
 *                positives, HardNet.py:392-393, each need their own);
 *   d_scratch -- transient: any buffer of the size asked for, reusable by every call.
 * The backward must get the forward's batch, dropout_p and seed (the dropout mask is a counter
 * hash of (seed, element), recomputed).  It only reads d_saved, so it may run more than once.
 * Batch >= 2 (train-mode BatchNorm of the 1x1 conv6 output needs more than one value). */
int hn_hardnet_train_workspace_bytes(int64_t batch, size_t* saved_bytes_out, size_t* scratch_bytes_out);
int hn_hardnet_train_forward(const float* d_in, int64_t batch, const float* const* d_weights,
                             float* const* d_running_mean, float* const* d_running_var, float momentum,
                             float dropout_p, uint64_t seed, float* d_out, void* d_saved, size_t saved_bytes,
                             void* d_scratch, size_t scratch_bytes, void* hip_stream);
int hn_hardnet_train_backward(const float* d_dout, int64_t batch, const float* const* d_weights,
                              float* const* d_dweights, float* d_din, float dropout_p, uint64_t seed,
                              void* d_saved, size_t saved_bytes, void* d_scratch, size_t scratch_bytes,
                              void* hip_stream);

/* Train-mode hardnetNAS (second half; hardnetNAS/supernet_functions/
 * training_functions_supernet.py:88-103 runs the module in train() through autograd):
 *   desc->kind HN_KIND_NAS           the sampled descriptor (op[i] per layer), model_supernet.py:53-85
 *                                    with each MixedOperation replaced by its arch op;
 *   desc->kind HN_KIND_NAS_SUPERNET  the supernet: layer i outputs sum_j m[i][j] op_j(x) over all 17
 *                                    CANDIDATE_BLOCKS (MixedOperation.forward, model_supernet.py:23-36);
 *                                    d_soft = the soft weights m [n_layers][17] (the caller's
 *                                    Gumbel-softmax draw, :24), d_dsoft receives d loss / d m.
 *   desc->kind HN_KIND_FDL_NASNET / _FDL_NASNET01  FDLNet HardNetNeiMask (des.py:8-55 / NASNet_0.1
 *                                    des.py:10-55): input_norm (desc->input_norm_eps), conv0 3x3 + bias,
 *                                    then BN(affine=False) -> 1x1 s2 BN ReLU -> 1x1 s2 BN ReLU (NASNet) or
 *                                    MaxPool(3,2,1) -> 1x1 s2 BN ReLU (NASNet_0.1), then the layers at 8x8.
 * forward : front -> the layers -> 4x4 head conv -> BatchNorm2d(affine=False) -> y / ||y||,
 *           every BatchNorm with the batch's statistics (running stats updated with `momentum`,
 *           unbiased variance).  d_in [B,1,32,32] fp32 (NAS: no input_norm, the NAS loaders normalise;
 *           FDL: input_norm in the forward).
 * backward: d_dout [B,128] -> d_grads (every conv weight, BN weight / bias and SE weight / bias,
 *           overwritten); no input gradient.
 * d_tensors: host array of hn_nas_train_tensor_count() device pointers, one per float tensor of the
 * module's state_dict in order (num_batches_tracked and the supernet's `thetas` left out): conv
 * weights, BN weight, bias, running_mean, running_var (updated in place), SE weights / biases.
 * d_grads: the same length; entries for running buffers are ignored (may be NULL); every weight
 * slot (conv / SE weights and biases) needs a buffer, frozen parameters included (HN_ERR_ARG if NULL).
 * Workspace: d_saved is written by the forward and read by its backward (one per forward call);
 * d_scratch is transient. */
int hn_nas_train_tensor_count(const hn_arch_desc* desc, size_t* n_out);
int hn_nas_train_workspace_bytes(const hn_arch_desc* desc, int64_t batch, size_t* saved_bytes_out,
                                 size_t* scratch_bytes_out);
int hn_nas_train_forward(const hn_arch_desc* desc, const float* d_in, int64_t batch, float* const* d_tensors,
                         float momentum, const float* d_soft, float* d_out, void* d_saved, size_t saved_bytes,
                         void* d_scratch, size_t scratch_bytes, void* hip_stream);
int hn_nas_train_backward(const hn_arch_desc* desc, const float* d_dout, const float* d_in, int64_t batch,
                          float* const* d_tensors, const float* d_soft, float* const* d_grads, float* d_dsoft,
                          void* d_saved, size_t saved_bytes, void* d_scratch, size_t scratch_bytes,
                          void* hip_stream);

/* Per-stage timing (profiling aid used by bench.py): when enabled, hn_forward records a
 * hipEvent pair around every kernel launch on the caller's stream.  hn_stage_times
 * waits for the recorded events, accumulates their durations per stage name and returns
 * the number of stages (<= max_stages); it then clears the accumulators.
 * names_out[i] points to storage owned by the model. */
int hn_set_profiling(hn_model* m, int enable);
int hn_stage_times(hn_model* m, int max_stages, const char** names_out, double* total_ms_out,
                   int64_t* launches_out);

void hn_destroy(hn_model* m);

/* Message of the last failing call on this thread ("" if none). */
const char* hn_last_error(void);

/* HN_ABI_VERSION of the loaded library. */
int hn_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* HARDNET_MI355X_H */
