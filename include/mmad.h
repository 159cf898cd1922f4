/*
 * mmad.h -- C ABI of libmmad_hip.so, the MI355X (gfx950) kernels behind the
 * multimodal_alzheimer 3D-volume training hot path.
 *
 * The reference (Liz490/multimodal_alzheimer) is pure Python: its hot path is the
 * torch.nn call chain of MedicalNet's 3D-ResNet + the reference heads and losses.
 * Each entry point below replaces one op of that chain; the reference call site it
 * stands in for is cited next to it (paths relative to the reference root).  There
 * is no reference FFI to mirror, so the binding is ctypes (INTEGRATION.md shows it).
 *
 * Conventions
 *   - Every function is asynchronous on the caller's HIP stream (`stream`, a
 *     hipStream_t passed as void*; NULL = the legacy default stream) and returns an
 *     int status: MMAD_OK, one of the MMAD_E* codes, or MMAD_EHIP + hipError_t.
 *   - The library never allocates, frees or synchronises device memory and keeps no
 *     mutable global state: every buffer (including workspaces sized by the
 *     *_workspace / *_parts queries) is owned by the caller.
 *   - Activation, packed-weight and workspace buffers of the conv entry points are
 *     16-byte aligned (they move as 16-byte vectors); a misaligned one is refused with
 *     MMAD_EBADSHAPE before anything is launched.
 *   - Activations are NDHWC ("voxel-major": channels contiguous per voxel) in the
 *     compute dtype (MMAD_F32 or MMAD_BF16); a logical (N,C,D,H,W) torch tensor in
 *     torch.channels_last_3d memory format is exactly this layout.
 *   - Conv weights enter in the torch layout [Co][Ci][kd][kh][kw] fp32 and are packed
 *     per step (mmad_conv_pack_weight); weight gradients leave in the same torch
 *     layout, fp32.  BN statistics, scale/shift and all reductions are fp32 (f64 for
 *     the final per-channel sums); logits and the loss are f64 as in the reference
 *     (pkg/models/mri_models/anat_cnn.py:104).
 */
#ifndef MMAD_H
#define MMAD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { MMAD_OK = 0, MMAD_EBADSHAPE = 1001, MMAD_EBADDTYPE = 1002, MMAD_ENULL = 1003,
       MMAD_EUNSUPPORTED = 1004, MMAD_EHIP = 2000 };

enum { MMAD_F32 = 0, MMAD_BF16 = 1, MMAD_F64 = 2 };

/* One 3D convolution (torch.nn.Conv3d semantics, groups = 1).  `do_` is the output
 * depth (`do` is a C keyword). */
typedef struct mmad_conv_desc {
  int32_t n;
  int32_t ci, di, hi, wi;
  int32_t co, do_, ho, wo;
  int32_t kd, kh, kw;
  int32_t sd, sh, sw;
  int32_t pd, ph, pw;
  int32_t dd, dh, dw;
} mmad_conv_desc;

int mmad_abi_version(void);                 /* == MMAD_ABI_VERSION */
#define MMAD_ABI_VERSION 1
const char* mmad_strerror(int status);
/* Kernel-variant switch (the run-time twin of the MMAD_* environment A/B switches; no
 * reference counterpart): "lattice_zp" = 1 plane-pair residue-class conv (default), 0 the
 * one-plane form, 2 plane-pair at any size; "lattice" / "lattice8" / "lattice5" = 1
 * residue-class convs where their tiles fill the CUs (default), 2 at any size, 0 off;
 * "pool_run" = the stem BN+ReLU+max-pool forward: 2 the z-walking kernel (default), other
 * values the per-output rows kernel; "patchz" = 1 the persistent z-walking layer1 conv where
 * its work items fill the CUs (default), 2 at any size, 0 the per-box patch conv;
 * "pw_wg3_dedup" = 1 the stride-2 3^3 weight gradient on 16-wide rows with de-duplicated
 * input columns (default), 0 its three-image form.  value < 0 only queries.
 * Returns the previous value, -1 for an unknown name.  Not thread-safe against concurrent
 * launches. */
int mmad_set_kernel_variant(const char* name, int value);

/* ---- 3D convolution as MFMA implicit GEMM --------------------------------------
 * Replaces nn.Conv3d forward/backward: MedicalNet conv1 / BasicBlock / Bottleneck /
 * shortcut-B convs (used at pkg/models/mri_models/anat_cnn.py:29-31,
 * pet_resnet_cnn.py:33-35), the 'same'-padded head convs (anat_cnn.py:55-63) and the
 * Small_PET_CNN convs (pkg/models/pet_models/pet_cnn.py:20-22).
 * Requirements: ci % 8 == 0 or ci == 1; co % 8 == 0 for dgrad; channel counts powers
 * of two.  ci == 1 convs run on a W-unfolded input: x must be the output of
 * mmad_conv_unfold_input (layout [n][di][hi][wo][8]).                              */
int64_t mmad_conv_packed_elems(const mmad_conv_desc* d, int dtype, int for_dgrad);
int mmad_conv_pack_weight(const mmad_conv_desc* d, int dtype, const float* w,
                          void* w_packed, int for_dgrad, void* stream);
/* Batched packing: one launch repacks every listed weight (a model's whole conv set per
 * step).  mmad_conv_pack_job fills one job on the host (MMAD_EUNSUPPORTED when this
 * geometry needs the per-call path: padded K rows or a ci == 1 conv); the job array is
 * copied to device memory once and reused while the pointers stay valid.            */
typedef struct mmad_pack_job {
  const float* w;
  void* w_packed;
  /* source row i of batch entry b is row i % rdiv of packed block b * rows / rdiv + i / rdiv
   * (forward jobs fold every output channel into one rows = co * ci matrix)            */
  int32_t rows, cols, batch, jdiv, ostride_j2, tiles_x, tiles_y, pad_, rdiv;
  int64_t ostride_b, ostride_j1, tile0;
} mmad_pack_job;
int mmad_conv_pack_job(const mmad_conv_desc* d, int dtype, int for_dgrad, const float* w,
                       void* w_packed, int64_t tile0, mmad_pack_job* job);
int64_t mmad_pack_job_tiles(const mmad_pack_job* job);
/* Both bf16 layouts of one conv weight from a single read (16 co x 16 ci x taps tiles):
 * forward [co][tap][ci] into w_fwd and input-gradient [ci][tap'][co] into w_dgrad (tap'
 * reversed when the dgrad runs as a forward conv), bit-identical to two
 * mmad_conv_pack_weight calls.  MMAD_EUNSUPPORTED unless both layouts are unpadded and
 * ci, co are multiples of 16 (bf16 only). */
typedef struct mmad_pack_dual {
  const float* w;
  void* w_fwd;
  void* w_dgrad;
  int32_t co, ci, taps, flip;
  int64_t tile0;
} mmad_pack_dual;
int mmad_conv_pack_dual_job(const mmad_conv_desc* d, int dtype, const float* w, void* w_fwd,
                            void* w_dgrad, int64_t tile0, mmad_pack_dual* job);
int64_t mmad_pack_dual_tiles(const mmad_pack_dual* job);
int mmad_conv_pack_dual_batch(int dtype, int njobs, const mmad_pack_dual* jobs_device,
                              int64_t total_tiles, void* stream);
int mmad_conv_pack_batch(int dtype, int njobs, const mmad_pack_job* jobs_device,
                         int64_t total_tiles, void* stream);
/* Adam step fused with the bf16 repack (the captured training step's optimizer,
 * fused_optim.AdamRepack): replaces torch.optim.Adam(fused=True, capturable=True).step()
 * over the reference's param groups (anat_cnn.py:111-126; amsgrad, maximize and grad
 * scaling off) -- bit-identical update of param, exp_avg, exp_avg_sq and the device step --
 * and, for a job with w_fwd != NULL, the updated conv weight's two bf16 layouts exactly as
 * mmad_conv_pack_dual_batch writes them (co, ci multiples of 16, taps <= 27); for a job with
 * unf_kw > 0 (the Cin = 1 stem: co rows, taps = kd*kh, kpad; one block per row) the
 * unfolded forward layout mmad_conv_pack_weight writes into w_fwd.  Blocks [tile0, tile0 + ntiles) of the launch
 * belong to a job (jobs sorted by tile0; ntiles from mmad_adam_job_tiles); block_job (device,
 * may be NULL: a binary search over tile0 then) = each block's job index; `arrivals` is one
 * zeroed int per job, left zeroed. */
typedef struct mmad_adam_job {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  float* step;                  /* the parameter's device step counter (float32) */
  const float* lr;              /* the group's device learning rate (float32) */
  double beta1, beta2, eps, weight_decay;
  void* w_fwd;                  /* NULL: no repack */
  void* w_dgrad;
  int32_t co, ci, taps, flip;
  int32_t unf_kw, kpad;         /* unfolded stem repack (unf_kw > 0) */
  int64_t numel, tile0, ntiles;
} mmad_adam_job;
int64_t mmad_adam_job_tiles(const mmad_adam_job* job);
int mmad_adam_repack(int njobs, const mmad_adam_job* jobs_device, const int* block_job,
                     int64_t total_tiles, int* arrivals, void* stream);
int64_t mmad_conv_unfolded_elems(const mmad_conv_desc* d);
int mmad_conv_unfold_input(const mmad_conv_desc* d, int in_dtype, const void* x,
                           int dtype, void* x_unf, void* stream);
/* rows of the BN-statistics partial buffer written by mmad_conv3d_fwd: [rows][2][co] */
int64_t mmad_conv3d_stats_rows(const mmad_conv_desc* d, int dtype);
int mmad_conv3d_fwd(const mmad_conv_desc* d, int dtype, const void* x,
                    const void* w_packed, const float* bias, void* y, float* stats,
                    void* stream);
/* Eval-mode fused conv + BN (+ residual) + ReLU (BasicBlock / shortcut in .eval(), running
 * statistics): weights packed with the BN scale folded in (mmad_conv_pack_weight_scaled,
 * forward layout), `bias` = the folded BN shift (mmad_bn_fold); the epilogue adds `res`
 * (output-shaped NDHWC, may be NULL) and applies ReLU when `relu` != 0.  Not for the
 * Cin = 1 stem.  Replaces the eval forward of anat_cnn.py:29-31's backbone blocks. */
int mmad_conv3d_fwd_ex(const mmad_conv_desc* d, int dtype, const void* x,
                       const void* w_packed, const float* bias, const void* res, int relu,
                       void* y, float* stats, void* stream);
int mmad_conv_pack_weight_scaled(const mmad_conv_desc* d, int dtype, const float* w,
                                 const float* scale, void* w_packed, int for_dgrad,
                                 void* stream);
int mmad_bn_fold(int c, const float* gamma, const float* beta, const float* running_mean,
                 const float* running_var, float eps, const float* conv_bias, float* scale,
                 float* bias, void* stream);
int mmad_conv3d_dgrad(const mmad_conv_desc* d, int dtype, const void* dy,
                      const void* w_packed_t, void* dx, void* stream);
/* Input gradient of a conv whose input was relu(bn(y)) -- a BN+ReLU without residual, as
 * MedicalNet's BasicBlock runs bn1 -> relu -> conv2 (reference call site anat_cnn.py:30-31;
 * replaces the column-sum pass of that BN's backward, mmad_bn_relu_bwd_reduce) -- with the
 * BN backward's partial sums from the dgrad epilogue: parts [rows][2][ci] holds per tile
 * (sum g', sum g' * xhat), g' = dx * (fma(y, scale, shift) > 0), xhat = (y - mean) * invstd,
 * g = dx as stored (bf16); feed them to mmad_bn_bwd_finalize with nparts = rows.
 * rows = mmad_conv3d_dgrad_bnsum_rows(d, dtype): -1 when this conv's dgrad route has no such
 * epilogue (then mmad_conv3d_dgrad + mmad_bn_relu_bwd_reduce).  bf16 only; y NDHWC like dx,
 * scale / shift / mean / invstd [ci] fp32, 16-byte aligned. */
int64_t mmad_conv3d_dgrad_bnsum_rows(const mmad_conv_desc* d, int dtype);
int mmad_conv3d_dgrad_bnsum(const mmad_conv_desc* d, int dtype, const void* dy, const void* wpt,
                            void* dx, const void* y, const float* scale, const float* shift,
                            const float* mean, const float* invstd, float* parts, void* stream);
int64_t mmad_conv3d_wgrad_workspace(const mmad_conv_desc* d, int dtype); /* bytes */
int mmad_conv3d_wgrad(const mmad_conv_desc* d, int dtype, const void* x, const void* dy,
                      float* dw, float* dbias, void* workspace, void* stream);
/* Same, with the split-K slab reduction (and dbias) queued on reduce_stream after an event
 * on stream: the memory-bound reduction overlaps the kernels that follow on stream.  The
 * caller keeps workspace / dy alive for reduce_stream and joins it before reading dw. */
int mmad_conv3d_wgrad_split(const mmad_conv_desc* d, int dtype, const void* x, const void* dy,
                            float* dw, float* dbias, void* workspace, void* stream,
                            void* reduce_stream);
/* MedicalNet stem (Cin 1, 7^3, stride 2, pad 3; the descriptor mmad_conv_unfold_input
 * takes) straight from the raw volume (n, 1, D, H, W) in `in_dtype` MMAD_F64 (as the
 * reference DataLoader delivers it, dataloader.py:213-277 -> anat_cnn.py:29) or MMAD_F32,
 * bf16 compute: the kernels unfold each input row in registers, so no unfolded copy is
 * written or read.  Results are bit-identical to unfold + mmad_conv3d_fwd / _wgrad.
 * mmad_stem_raw_ok: 1 when this path applies (even W <= 128, bf16, the stem geometry). */
int mmad_stem_raw_ok(const mmad_conv_desc* d, int in_dtype, int dtype);
int mmad_conv3d_fwd_raw(const mmad_conv_desc* d, int in_dtype, const void* x, int dtype,
                        const void* w_packed, const float* bias, void* y, float* stats,
                        void* stream);
/* Deferred slab reduction (round 5): the weight gradient's split-K kernel runs now, its
 * slab reduction is described in *job (kind != 0) instead of launched, and
 * mmad_wgrad_reduce_batch later runs the pending reductions of many convs (the whole
 * backward's, or one data-parallel stage's) as ONE launch -- the same per-element sums in the
 * same fixed order, so dW is bit-identical to mmad_conv3d_wgrad.  Where a path has no
 * separate reduction to defer (the stem's two-level sum, bias gradients, no split) it runs
 * inline and job->kind = 0.  The caller keeps workspace and dw alive, and reads dw only
 * after the batch.  Replaces the per-conv reduction launches behind loss.backward()
 * (anat_cnn.py:99-109 via Lightning's training_step). */
typedef struct mmad_wgrad_job {
  const float* ws;
  float* dw;
  int32_t splits, nd, k, cs, taps, tper, kind, gx, gy, gz;
} mmad_wgrad_job;
int mmad_conv3d_wgrad_deferred(const mmad_conv_desc* d, int dtype, const void* x,
                               const void* dy, float* dw, void* workspace, mmad_wgrad_job* job,
                               void* stream);
/* the same for the stem straight from the raw volume (mmad_conv3d_wgrad_raw) */
int mmad_conv3d_wgrad_raw_deferred(const mmad_conv_desc* d, int in_dtype, const void* x,
                                   int dtype, const void* dy, float* dw, void* workspace,
                                   mmad_wgrad_job* job, void* stream);
/* jobs: host array (copied into the launch's arguments, so a captured launch replays the
 * same jobs); any njobs (16 per launch) */
int mmad_wgrad_reduce_batch(int njobs, const mmad_wgrad_job* jobs, void* stream);
/* reduce_stream may be NULL (everything on stream); see mmad_conv3d_wgrad_split */
int mmad_conv3d_wgrad_raw(const mmad_conv_desc* d, int in_dtype, const void* x, int dtype,
                          const void* dy, float* dw, float* dbias, void* workspace,
                          void* stream, void* reduce_stream);

/* ---- BatchNorm3d / BatchNorm1d (+ fused ReLU and residual add) -------------------
 * Replaces nn.BatchNorm3d/1d + nn.ReLU + the residual `out += residual; relu`
 * of MedicalNet BasicBlock, the stem bn1+relu, and the head BNs
 * (anat_cnn.py:50-51, :69-70).  torch semantics: biased batch variance to normalise,
 * unbiased variance into running_var, momentum update.  Layout [m][c], m = N*D*H*W.  */
int64_t mmad_bn_stats_parts(int64_t m, int c);
int mmad_bn_stats(int dtype, int64_t m, int c, const void* y, float* parts, void* stream);
/* fold groups of `group` partial rows into one: out has cdiv(nparts, group) rows */
int mmad_bn_parts_fold(int c, int nparts, const float* parts, int group, float* out,
                       void* stream);
int mmad_bn_finalize(int c, int64_t count, int nparts, const float* parts,
                     const float* gamma, const float* beta, float* running_mean,
                     float* running_var, float momentum, float eps, int training,
                     float* mean, float* invstd, float* scale, float* shift,
                     int64_t* num_batches_tracked, void* stream);
                     /* num_batches_tracked (nullable) += 1 with the running-stat update */
/* mmad_bn_finalize's arguments for one BN (all but c / count) */
typedef struct mmad_bn_fin {
  int nparts;
  const float* parts;
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float momentum;
  float eps;
  int training;
  float* mean;
  float* invstd;
  float* scale;
  float* shift;
  int64_t* num_batches_tracked;
} mmad_bn_fin;
/* the two BNs of a residual pair (same c and count: bn2 and the shortcut BN) in one launch;
 * each set exactly as one mmad_bn_finalize call */
int mmad_bn_finalize2(int c, int64_t count, const mmad_bn_fin* a, const mmad_bn_fin* b,
                      void* stream);
/* out = act(y*scale + shift + R), R = res*rscale + rshift | res | 0; act = relu|id */
int mmad_scale_shift_act(int dtype, int64_t m, int c, const void* y, const float* scale,
                         const float* shift, const void* res, const float* rscale,
                         const float* rshift, int relu, void* out, void* stream);
int64_t mmad_bn_bwd_parts(int64_t m, int c);
/* partial sums of g' and g'*xhat with g' = g * (relu_out > 0 | 1) */
/* g2 (may be NULL, here and in every BN / BN+pool backward below that takes it): a second
 * gradient of the same output (a block input read by both conv1 and the shortcut); the
 * kernels use as_stored(g + g2) -- the value torch's own gradient accumulation would hand
 * them -- so the separate add pass disappears.  Generic (non fixed-channel) layouts of
 * mmad_bn_bwd_apply return MMAD_EUNSUPPORTED with g2: the caller adds it first. */
int mmad_bn_bwd_reduce(int dtype, int64_t m, int c, const void* g, const void* g2,
                       const void* relu_out, const void* y, const float* mean,
                       const float* invstd, float* parts, void* stream);
/* dgamma, dbeta (fp32, may be NULL) and the apply coefficients for mmad_bn_bwd_apply */
int mmad_bn_bwd_finalize(int c, int64_t count, int nparts, const float* parts,
                         const float* gamma, const float* invstd, int training,
                         float* dgamma, float* dbeta, float* coef, void* stream);
/* dy = coef0[c]*g' - coef1[c] - xhat*coef2[c]; optionally also gmask_out = g' */
int mmad_bn_bwd_apply(int dtype, int64_t m, int c, const void* g, const void* g2,
                      const void* relu_out, const void* y, const float* mean,
                      const float* invstd, const float* coef, void* dy, void* gmask_out,
                      void* stream);
/* Residual pair relu(bn(y) + bn2(y2)) (BasicBlock with the shortcut-B downsample BN): both
 * BNs' backward in one pass each over g / relu_out -- reduce2 writes both part buffers
 * (parts2 = sums of g' and g'*xhat2), finalize2 both coefficient sets, apply2 dy and dy2.
 * Bit-identical to the per-BN calls; fixed-channel layouts only (else MMAD_EUNSUPPORTED). */
/* g_rows > 0 (reduce2 / apply2): g is the compact (N, C) gradient of a global average pool
 * (mmad_gap_bwd_compact) and row r of the BN input reads its sample's row g[r / g_rows]
 * -- the same values as the broadcast mmad_gap_bwd output, never materialised; requires
 * m % g_rows == 0 and m < 2^31.  0: g is a dense [m][c] gradient. */
int mmad_bn_bwd_reduce2(int dtype, int64_t m, int c, const void* g, const void* g2,
                        int64_t g_rows, const void* relu_out, const void* y, const float* mean,
                        const float* invstd, const void* y2,
                        const float* mean2, const float* invstd2, float* parts, float* parts2,
                        void* stream);
int mmad_bn_bwd_finalize2(int c, int64_t count, int nparts, const float* parts,
                          const float* gamma, const float* invstd, int training, float* dgamma,
                          float* dbeta, float* coef, const float* parts2, const float* gamma2,
                          const float* invstd2, int training2, float* dgamma2, float* dbeta2,
                          float* coef2, void* stream);
int mmad_bn_bwd_apply2(int dtype, int64_t m, int c, const void* g, const void* g2,
                       int64_t g_rows, const void* relu_out, const void* y, const float* mean, const float* invstd, const float* coef,
                       void* dy, const void* y2, const float* mean2, const float* invstd2,
                       const float* coef2, void* dy2, void* stream);
/* BN + ReLU without residual (bn1 of every BasicBlock): the same two passes with the ReLU
 * mask recomputed from y as fma(y, scale, shift) > 0 (the forward's affine, so the mask
 * equals out > 0) instead of read from the ReLU output -- one tensor fewer per pass. */
int mmad_bn_relu_bwd_reduce(int dtype, int64_t m, int c, const void* g, const void* y,
                            const float* mean, const float* invstd, const float* scale,
                            const float* shift, float* parts, void* stream);
int mmad_bn_relu_bwd_apply(int dtype, int64_t m, int c, const void* g, const void* y,
                           const float* mean, const float* invstd, const float* scale,
                           const float* shift, const float* coef, void* dy, void* stream);
int mmad_relu_fwd(int dtype, int64_t n, const void* x, void* y, void* stream);
int mmad_relu_bwd(int dtype, int64_t n, const void* g, const void* out, void* dx, void* stream);
int mmad_add(int dtype, int64_t n, const void* a, const void* b, void* out, void* stream);

/* ---- pooling -------------------------------------------------------------------
 * MaxPool3d(3,2,1) stem pool and MaxPool3d(2) head/PET pools (pet_cnn.py:26),
 * AdaptiveAvgPool3d(1) (anat_cnn.py:66, pet_cnn.py:33).  Max-pool ties resolve to the
 * first window position in (kd,kh,kw) scan order, as torch's CPU kernel does.       */
int mmad_colsum_ws(int dtype, int64_t m, int c, const void* y, float* parts, float* out,
                   void* stream);   /* out[c] = sum_m y[m][c]; parts: bn_stats_parts rows */
int mmad_maxpool3d_fwd(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho,
                       int wo, int k, int s, int p, const void* x, void* y,
                       uint8_t* argmax, void* stream);
int mmad_maxpool3d_bwd(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho,
                       int wo, int k, int s, int p, const void* dy, const uint8_t* argmax,
                       void* dx, void* stream);
/* Fused MedicalNet stem tail maxpool(relu(bn1(conv1 y))) (MedicalNet resnet.py forward:
 * conv1 -> bn1 -> relu -> maxpool, reached from anat_cnn.py:29-31): the full-resolution
 * BN+ReLU output is never written.  argmax = window index | 0x80 when the max passed the
 * ReLU; ymax = the raw y at the argmax.  Backward: mmad_bnpool_bwd_reduce over the pooled
 * grid -> mmad_bn_bwd_finalize (count = full-resolution rows) -> mmad_bnpool_bwd_apply. */
int mmad_bnpool_fwd(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho, int wo,
                    int k, int s, int p, const void* y, const float* scale, const float* shift,
                    void* out, uint8_t* argmax, void* ymax, void* stream);
/* m = pooled rows; with g2 the summed gradient as_stored(g + g2) is also written to gsum
 * (the apply then reads gsum as its g: the pool backward reads each pooled gradient from up
 * to 8 cells, so it takes one summed tensor, not two) */
int mmad_bnpool_bwd_reduce(int dtype, int64_t m, int c, const void* g, const void* g2,
                           void* gsum, const uint8_t* argmax, const void* ymax,
                           const float* mean, const float* invstd, float* parts, void* stream);
int mmad_bnpool_bwd_apply(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho,
                          int wo, int k, int s, int p, const void* g, const uint8_t* argmax,
                          const void* y, const float* mean, const float* invstd,
                          const float* coef, void* dy, void* stream);
int mmad_gap_fwd(int dtype, int n, int64_t s, int c, const void* x, float* y, void* stream);
/* same, partitioned over voxel slabs so small batches still fill the GPU; ws holds
 * mmad_gap_fwd_ws_elems(n, s, c) floats of partial sums (summed in a fixed order) */
int64_t mmad_gap_fwd_ws_elems(int n, int64_t s, int c);
int mmad_gap_fwd_ws(int dtype, int n, int64_t s, int c, const void* x, float* y, float* ws,
                    void* stream);
int mmad_gap_bwd(int dtype, int n, int64_t s, int c, const float* dy, void* dx, void* stream);
/* The same values without the broadcast: dx[n][c] = (dtype) (dy[n][c] / s), for consumers
 * that take a pooled gradient as broadcast rows (g_rows in mmad_bn_bwd_reduce2 / _apply2). */
int mmad_gap_bwd_compact(int dtype, int n, int64_t s, int c, const float* dy, void* dx,
                         void* stream);
/* conv_seg's AdaptiveAvgPool3d(1) -> Flatten -> Linear (-> ReLU) (anat_cnn.py:66-76) as two
 * launches forward and one backward, same values as mmad_gap_fwd_ws + mmad_linear_fwd and
 * mmad_linear_bwd_ex + mmad_gap_bwd_compact:
 *   mmad_gap_partial   the GAP's first level into ws (mmad_gap_fwd_ws_elems floats):
 *                      mmad_gap_parts(n, s, c) = P partial rows per sample (the pooled means
 *                      themselves when P == 1);
 *   mmad_gap_linear_fwd  folds them (xs[b][i] = pooled input, kept for the backward) and
 *                      y = act(xs W^T + bias) (in <= 4096, else MMAD_EUNSUPPORTED);
 *   mmad_linear_gap_bwd  dW, dbias and the input gradient as compact GAP rows
 *                      rows[b][i] = (rows_dtype) ((dy' W)[b][i] / s), dy' = ReLU-masked dy
 *                      (ymask = the forward output, or NULL). */
int mmad_gap_parts(int n, int64_t s, int c);
int mmad_gap_partial(int dtype, int n, int64_t s, int c, const void* x, float* ws,
                     void* stream);
int mmad_gap_linear_fwd(int b, int in, int out, int parts, int64_t s, const float* ws,
                        const float* w, const float* bias, int relu, float* xs, float* y,
                        void* stream);
int mmad_linear_gap_bwd(int b, int in, int out, int64_t s, const float* x, const float* w,
                        const float* dy, const float* ymask, int rows_dtype, void* rows,
                        float* dw, float* dbias, void* stream);

/* ---- fusion / classifier MLP head (fp32) ----------------------------------------
 * nn.Linear (+ReLU) of conv_seg (anat_cnn.py:68-76), reduce_dim_mri / stage2out /
 * cls2 of Anat_PET_CNN (pkg/models/fusion_models/anat_pet_fusion.py:42-51) and the
 * concat of the two branch features (anat_pet_fusion.py:76).                       */
int mmad_linear_fwd(int b, int in, int out, const float* x, const float* w,
                    const float* bias, int relu, float* y, void* stream);
int mmad_linear_bwd(int b, int in, int out, const float* x, const float* w,
                    const float* dy, float* dx, float* dw, float* dbias, void* stream);
/* Same in one launch, with the backward of a fused ReLU: ymask = the forward output of
 * mmad_linear_fwd(relu=1) (NULL: no ReLU); the gradient is taken as ymask > 0 ? dy : 0. */
int mmad_linear_bwd_ex(int b, int in, int out, const float* x, const float* w,
                       const float* dy, const float* ymask, float* dx, float* dw, float* dbias,
                       void* stream);
int mmad_concat_cols(int b, int n_in, const float* const* srcs, const int* widths,
                     float* dst, void* stream);
int mmad_split_cols(int b, int n_out, const float* src, float* const* dsts,
                    const int* widths, void* stream);

/* ---- voxel-level PET-MRI fusion (fusion.hip) ----------------------------------------
 * mmad_gather_channels: torch.stack((x_pet, x_mri), dim=1).to(float32) of PET_MRI_EF
 * (pkg/models/fusion_models/early_fusion.py:77-80) written straight into the NDHWC layout
 * of the Cin = 2 conv (:35), channels padded to cpad = 8 with zeros: source plane c is
 * srcs[c] + b*batch_stride + v*vox_stride (elements), v over the n*vox voxels; in dtype
 * f64/f32/bf16 -> out dtype f32/bf16 (f64 -> f32 -> bf16 rounding, as torch).
 * mmad_pad_rows: dst[r][j] = j < cin ? src[r][j] : 0 for j < cout (pads a conv weight's
 * Ci -- [Co][Ci*taps] rows -- and cuts the padded weight gradient back).
 * mmad_concat_channels / mmad_split_channels: torch.cat((a, b), dim=1) of two NDHWC
 * volumes and its backward ('concatenate' fusion, anat_pet_featuremapfusion.py:112-113).
 * mmad_max2_fwd / _bwd: torch.max(torch.stack((a, b)), dim=0) ('maxout' fusion, :115-117):
 * ties and NaN follow torch (ties -> a; NaN propagates); sel[i] = 1 where b was taken; the
 * gradient goes to the selected operand only.  n % (16 / sizeof(dtype)) == 0.          */
int mmad_gather_channels(int in_dtype, int nsrc, const void* const* srcs,
                         int64_t batch_stride, int64_t vox_stride, int n, int64_t vox,
                         int cpad, int out_dtype, void* dst, void* stream);
int mmad_pad_rows(int rows, int cin, int cout, const float* src, float* dst, void* stream);
int mmad_concat_channels(int dtype, int64_t rows, int ca, const void* a, int cb,
                         const void* b, void* dst, void* stream);
int mmad_split_channels(int dtype, int64_t rows, int ca, int cb, const void* src, void* a,
                        void* b, void* stream);
int mmad_max2_fwd(int dtype, int64_t n, const void* a, const void* b, void* y, uint8_t* sel,
                  void* stream);
int mmad_max2_bwd(int dtype, int64_t n, const void* g, const uint8_t* sel, void* ga, void* gb,
                  void* stream);

/* ---- dtype casts / dropout ------------------------------------------------------ */
int mmad_cast(int in_dtype, int out_dtype, int64_t n, const void* x, void* y, void* stream);
int mmad_dropout_fwd(int dtype, int64_t n, float p, uint64_t seed, const void* x, void* y,
                     uint8_t* keep, void* stream);
/* as mmad_dropout_fwd with the seed read from device memory when the kernel runs
 * (pet_cnn.py:27-29, :38-39 under HIP-graph replay: each replay draws a fresh mask) */
int mmad_dropout_fwd_dev(int dtype, int64_t n, float p, const uint64_t* seed, const void* x,
                         void* y, uint8_t* keep, void* stream);
int mmad_dropout_bwd(int dtype, int64_t n, float p, const void* g, const uint8_t* keep,
                     void* dx, void* stream);

/* ---- losses (f64, one workgroup) -----------------------------------------------
 * mode 0: weighted cross entropy, nn.CrossEntropyLoss(weight=w) 'mean' reduction
 *         = sum_i w[y_i]*nll_i / sum_i w[y_i]   (anat_cnn.py:84-85);
 * mode 1: FocalLoss(gamma), alpha None, mean, with pt DETACHED
 *         (pkg/loss_functions/focalloss.py:19-39).
 * Writes the loss and d loss / d logits (the backward is a scale of `dlogits`).     */
int mmad_loss_fwd(int b, int c, const double* logits, const int64_t* labels,
                  const double* weight, double gamma, int mode, double* loss,
                  double* dlogits, void* stream);
/* Same on MMAD_F32 or MMAD_F64 logits (fp32 widened exactly on load); logits64 (may be
 * NULL) receives the f64 logits -- general_step's f64 cast of the model output
 * (anat_cnn.py:102-104) fused into the loss launch. */
int mmad_loss_fwd_ex(int b, int c, int logits_dtype, const void* logits,
                     const int64_t* labels, const double* weight, double gamma, int mode,
                     double* logits64, double* loss, double* dlogits, void* stream);
/* d logits = (out_dtype) (dlogits * gloss[0] (+ gout[i] when gout != NULL)): the loss
 * backward and the f64 cast's backward in one pass (n = B*C). */
int mmad_loss_bwd(int64_t n, const double* dlogits, const double* gloss, const double* gout,
                  int out_dtype, void* dx, void* stream);

/* ---- test-set bootstrap (Base_Model.bootstrap_metric, pkg/models/base_model.py:219-239) --
 * For each of ndraw drawings d (idx[d][0..n) = the drawing's sample indices, as drawn by
 * torch.randint(0, n, (n,)) in the reference loop): f1[d] = torchmetrics-0.10 macro F1 and
 * mcc[d] = multiclass Matthews correlation of argmax(logits[idx]) vs labels[idx], f32.
 * c <= 16.  mmad_mean_std: out = (mean, unbiased std) of v in f64.                      */
int mmad_bootstrap_cls_metrics(int n, int c, const double* logits, const int64_t* labels,
                               int ndraw, const int64_t* idx, float* f1, float* mcc,
                               void* stream);
int mmad_mean_std(int n, const float* v, double* out, void* stream);

/* ---- input pipeline normalisation (float64, batched over scans) -------------------
 * Replaces MultiModalDataset.__getitem__'s per-sample CPU normalisation
 * (pkg/utils/dataloader.py:213-215 PET, :244-270 MRI per-scan, :272-277 MRI all-scan).
 * x, mask, out: [nscan][vox] float64 (out may alias x).  ws: mmad_norm_ws_bytes bytes.
 * min_max: v = nonzero(x*mask); lo/hi = torch.quantile(v, 1-q / q, 'linear') as exact
 *          order statistics (radix select) -> out = clamp((x-lo)/(hi-lo), 0, 1) * mask;
 *          q_out (optional, device) receives (lo, hi) per scan.  Bit-exact with the
 *          reference.  A scan with no nonzero masked voxel: out = NaN (torch raises).
 * zscore : out = (x - mean(v)) / std(v) * mask, unbiased std.
 * affine : out = (x - mean) / std over n elements (PET split statistics, all-scan MRI). */
int64_t mmad_norm_ws_bytes(int nscan, int64_t vox);
int mmad_mri_minmax_norm(int nscan, int64_t vox, const double* x, const double* mask,
                         double q, double* out, void* ws, double* q_out, void* stream);
int mmad_mri_zscore_norm(int nscan, int64_t vox, const double* x, const double* mask,
                         double* out, void* ws, void* stream);
int mmad_affine_norm(int64_t n, const double* x, double mean, double stdv, double* out,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MMAD_H */
