/*
 * libstx — MI355X (gfx950 / CDNA4) kernels for the tupini07/StyleTransfer hot
 * path, behind a plain C ABI.  All pointers are DEVICE pointers to fp32 NCHW
 * contiguous tensors unless stated; `stream` is a hipStream_t (NULL = legacy
 * default stream).  Every entry point is asynchronous on `stream`, performs no
 * allocation and no host synchronisation, and returns 0 on success or a
 * non-zero STX_E_* / hipError_t code (message via stx_last_error_string()).
 * Kernels are graph-capturable.
 *
 * Reference interfaces replaced (all in /root/reference, tupini07/StyleTransfer):
 *   conv2d fwd/dgrad/wgrad  <- torchvision vgg19 `.features` Conv2d layers sliced in
 *                              stransfer/network.py:246-314 and the ImageTransformNet
 *                              Conv2d layers stransfer/network.py:468-481,525-609
 *   gram / style loss       <- StyleLoss.gram_matrix / forward  stransfer/network.py:92-123
 *   mse losses              <- ContentLoss.forward :155-164, FeatureReconstructionLoss.forward :186-201
 *   maxpool / relu          <- VGG MaxPool2d / ReLU(inplace=False) stransfer/network.py:270-271
 *   adam                    <- torch.optim.Adam via get_content_optimizer :403-409, get_optimizer :643-649
 *   instance norm           <- nn.InstanceNorm2d(affine=True) stransfer/network.py:474,483,531,...,600
 *   residual add            <- ResidualBlock.forward `out += residual` :502
 *   upsample nearest x2     <- nn.Upsample(mode='nearest', scale_factor=2) :580-581,592-593
 *   total variation         <- get_total_variation_regularization_loss :621-641
 *   temporal loss           <- VideoTransformNet.get_temporal_loss :885-903
 *   image conditioning      <- img_utils.image_loader_transform stransfer/img_utils.py:13-44
 *                              (COCO loader stransfer/dataset.py:141-197)
 */
#ifndef STX_H_
#define STX_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Every max|.| bound in this API ("amax": in_amax, w_amax, out_amax, p2_amax,
 * z_amax, stx_amax's out) is a group of STX_AMAX_SLOTS floats whose maximum is the
 * value; producers spread their atomics over the group, a zeroed group reads 0. */
#define STX_AMAX_SLOTS 32

#define STX_OK 0
#define STX_E_INVALID 1001   /* bad argument / unsupported shape */
#define STX_E_WORKSPACE 1002 /* workspace too small */

/* input-loader modes for stx_conv2d: how the virtual conv input is formed
 * from the physical tensor x (fused into the LDS halo load) */
#define STX_IN_RAW 0        /* v = x                                            */
#define STX_IN_RELU 1       /* v = max(x, 0)              (VGG ReLU, not in-place) */
#define STX_IN_RELU_POOL2 2 /* v = maxpool2x2(max(x,0))   (VGG ReLU + MaxPool2d) */
#define STX_IN_UPSAMPLE2 3  /* v = x[y/2][x/2]            (nn.Upsample nearest x2) */
#define STX_IN_DILATE2 4    /* v = x[y/2][x/2] at even y,x else 0 (stride-2 dgrad) */

typedef struct stx_conv_params {
  const float* x;     /* physical input [n][cin][h][w] */
  const float* wt;    /* prepped weights [cin_pad*ks*ks][cout_pad] (stx_conv_weight_prep);
                         may be NULL when wt16 selects the split path */
  const float* bias;  /* [cout] or NULL */
  float* y;           /* output [n][cout][ho][wo]; NULL with pool_out (split path, plain
                         epilogue): only pool_out is written */
  const float* mask;  /* NULL or [n][cout][ho][wo]: value *= (mask > 0)   (ReLU backward) */
  const float* aux;   /* NULL or [n][cout][ho][wo]: value += aux_scale*aux */
  float aux_scale;
  const float* acc_scale; /* NULL or device scalar: value = acc * (*acc_scale) first */
  int accumulate;     /* value += old y */
  int relu_out;       /* y = max(value, 0) */
  int n, cin, h, w;   /* physical input dims */
  int cout, ks, stride, pad;
  int in_mode;        /* STX_IN_* */
  int hv, wv;         /* virtual input dims (after the in_mode transform) */
  int ho, wo;         /* output dims */
  int cin_pad, cout_pad;
  long long wt_batch_stride; /* floats between per-image weight matrices (0 = shared) */
  /* optional fused second GEMM phase (Gram backward inside the data-gradient conv):
   * after the main K loop the mask is applied, then
   *   value += (*p2_scale) * sum_c A[n][c][co] * p2_z[n][c][oy][ox]
   * A = p2_wt + n*p2_wt_batch_stride, laid out [c (padded to cin_pad rule of a 1x1 conv)]
   * [cout_pad]; p2_z [n][p2_c][ho][wo].  p2_z == NULL disables it.  stride 1 only. */
  const float* p2_z;
  const float* p2_wt;
  const float* p2_scale;
  int p2_c;
  long long p2_wt_batch_stride;
  /* optional fused ReLU+MaxPool2d backward epilogue:
   *   value += unpool(up_dp)[co][oy][ox] * (up_z > 0)
   * with the 2x2 argmax (first max of relu(up_z), row-major) recomputed from up_z
   * [n][cout][ho][wo]; up_dp [n][cout][ho/2][wo/2].  up_dp == NULL disables it. */
  const float* up_dp;
  const float* up_z;
  /* fp16 hi/lo split path (3x3 stride-1 convs, cin >= 16, cout > 4): when wt16 is
   * non-NULL the conv runs on v_mfma_f32_32x32x16_f16 with both operands split as
   * s*v = hi + lo (fp16 each, s a per-tensor power of two) and the three products
   * hi*hi + hi*lo + lo*hi accumulated in fp32 (fp32-level accuracy).
   * wt16/w_amax come from stx_conv_weight_prep16; in_amax is a device scalar
   * >= max|x| over the physical input (stx_amax, or a producer's out_amax). */
  const void* wt16;
  const float* w_amax;
  const float* in_amax;
  /* optional: *out_amax = max(*out_amax, max|y|) over the values this call writes
   * (caller zeroes it first) — the next split conv's in_amax at no extra pass. */
  float* out_amax;
  /* optional fused VGG ReLU + MaxPool2d(2,2) output: pool_out [n][cout][ho/2][wo/2] =
   * maxpool(relu(y)) (torch floor mode), written beside y.  Split path (wt16) with
   * wo > 32 only; the next conv then reads it with STX_IN_RAW. */
  float* pool_out;
  /* split path only: device scalar >= max|p2_z| (required with p2_z and wt16; the
   * Gram-backward phase then also runs on the fp16 hi/lo split MFMA, A scaled per
   * block by its own max).  A 1x1 conv with per-image weights (the Gram backward
   * dz = s*A[n].z, stx_gram_bwd) given in_amax and wt16 = (void*)1 runs as that
   * phase alone on the split kernel (no ReLU mask allowed there). */
  const float* p2_amax;
  /* optional fused Gram partials of the output (StyleLoss.gram_matrix of a 64- or
   * 128-channel VGG tap, stransfer/network.py:92-108, computed where the tile is produced
   * instead of re-reading y): split path, stride 1, cout == 64 or 128, wo > 32, and the
   * plain epilogue (no mask / aux / accumulate / acc_scale / up_dp / p2_z / relu_out;
   * cout 128: raw or ReLU input).  Block t of image n writes sum over its output pixels
   * of y y^T (fp32, fp16 hi/lo MFMA with a block-local power-of-two scale) as U 64 x 64
   * tiles: tile u to gram_part + ((n * U + u) * T + t) * 4096, T = stx_conv_gram_tiles(p),
   * U = 1 (cout 64) or 3 (cout 128: tiles (0,0), (0,1), (1,1) of the 128 x 128 matrix,
   * diagonal tiles whole); stx_style_loss_from_parts reduces them. */
  float* gram_part;
  /* with pool_out: pool_out = the 2x2 SUM of the output (no ReLU) and y is not written
   * -- the backward of nearest x2 upsampling (torch.nn.Upsample(scale_factor=2), the
   * ImageTransformNet's UpsampleConvLayer, stransfer/network.py:583-605) fused into the
   * data-gradient conv of the upsampled conv.  Split path, stride 1, wo > 32, even
   * ho / wo, plain epilogue only (no mask / aux / accumulate / acc_scale / up_dp / p2_z /
   * relu_out / gram_part / out_amax). */
  int pool_sum;
  /* optional with gram_part: per-group arrival counters, n * stx_conv_gram_groups(p)
   * uint32 words, zeroed once by the caller (every call leaves them zero again).  The
   * partials of tiles g*STX_GRAM_GROUP .. g*STX_GRAM_GROUP+7 of image n form group g;
   * the last block of a group to finish sums the group's partials in tile order and
   * writes that sum to gram_part + (n_total * T + n * NG + g) * 4096 (NG =
   * stx_conv_gram_groups(p)), so stx_style_loss_from_parts reads NG sums per image
   * instead of T partials.  The per-tile slots then hold three of the four 32 x 32
   * blocks only (scratch); the gram_part slab needs (T + NG) * 4096 floats per image. */
  unsigned int* gram_cnt;
  /* optional with p2_z on the split path: device amax group >= max|s * A[n]| over every
   * image n (stx_gram_fin_job.coef_amax of the finalize that wrote A, times |p2_scale|
   * folded in by the kernel).  The Gram-backward phase then runs on the fp16 hi/lo
   * split MFMA with this precomputed scale instead of the fp32 MFMA. */
  const float* p2_wt_amax;
  /* optional with gram_part on a 128-channel tap (the content layer conv2_2,
   * stransfer/network.py:134-201): the content target ref [n][cout][ho][wo]; block t of
   * image n then also writes sum (y - ref)^2 and sum (relu y - relu ref)^2 over its
   * outputs to mse_parts[2 (n T + t) + 0 / 1] (n * T * 2 floats), which
   * stx_style_content_loss_from_parts reduces into the content / feature losses. */
  const float* mse_ref;
  float* mse_parts;
  /* optional with in_mode STX_IN_UPSAMPLE2 on the split path (wt16 / w_amax of the same
   * weights): the parity-class slab (stx_conv_weight_prep16_up).  The conv then runs as
   * four output-parity 2x2 convs over the un-upsampled input (64 x 8 output tiles of one
   * row parity per block); plain epilogue only (bias, relu_out, out_amax), wo > 32. */
  const void* wt16_up;
  /* unpool_out = 1 (split path, raw-input 3x3 stride-1 data gradient, cout C = 64 or 128,
   * wo % 32 == 0, ho % 4 == 0): the conv's result d (the gradient of a MaxPool2d(2,2)(ReLU
   * (.)) output, [n][C][ho][wo]) is not stored; y receives, at full resolution
   * [n][C][2ho][2wo],
   *   y[co][Y][X] = d[co][Y/2][X/2] * [(Y, X) is the first max of its 2x2 window of relu(z)]
   *                 * [z[co][Y][X] > 0]  +  s * sum_c A[n][c][co] z[c][Y][X]
   *                 (+ aux_scale * aux[co][Y][X] with aux, full resolution)
   * with z = up_z, A = p2_wt (p2_wt_batch_stride, pitch cout_pad = C), p2_c = C, s =
   * *p2_scale (or 1), p2_amax >= max|z| and p2_wt_amax >= max|A| -- the ReLU+MaxPool
   * backward and the Gram backward (+ the folded content term) of the pooled VGG tap
   * (stransfer/network.py:110-164 through :264-275) in the producing conv's epilogue, so d
   * never reaches HBM.  out_amax receives max|y|; no bias / mask / accumulate / relu_out /
   * pool / Gram outputs. */
  int unpool_out;
} stx_conv_params;

#define STX_GRAM_GROUP 8

int stx_version(void);
/* sizeof and the offset of the last member of each ABI struct, in this order:
 * stx_conv_params, stx_wprep_job, stx_loss_parts, stx_gram_fin_job, stx_in_pgrad_job,
 * stx_image_meta -- 12 values, min(n, 12) written to out; returns 12.  Bindings check
 * their struct mirrors against it. */
int stx_abi_layout(long long* out, int n);
const char* stx_last_error_string(void);
/* The ABI revision of this header (STX_ABI_VERSION): a host binding refuses a library of
 * another revision rather than pass arguments whose meaning changed (round 6:
 * stx_instnorm_bwd's second argument is beta, not y; 7: stx_conv_params.unpool_out). */
#define STX_ABI_VERSION 7
int stx_abi_version(void);

/* Padded GEMM dims the conv kernels expect for a (cin, cout, ks) conv. */
int stx_conv_weight_dims(int cin, int cout, int ks, int* cin_pad, int* cout_pad);

/* w [cout][cin][ks][ks] -> wt [cin_pad*ks*ks][cout_pad] (zero padded).
 * transpose=1 builds the data-gradient weights of the same layer instead:
 * wt'[co*ks*ks + kh*ks + kw][ci] = w[co][ci][ks-1-kh][ks-1-kw] with dims
 * (cin'=cout, cout'=cin) padded by stx_conv_weight_dims(cout, cin, ks). */
int stx_conv_weight_prep(const float* w, float* wt, int cout, int cin, int ks, int transpose,
                         void* stream);

/* fp16 hi/lo split weight slab for the wt16 path: bytes of the slab for GEMM dims
 * (cin', cout') = (cin, cout), or (cout, cin) for transpose=1, ks = 3. */
size_t stx_conv_weight16_bytes(int cin, int cout, int ks, int transpose);
/* w [cout][cin][3][3] -> split slab wt16 ([cin'/16][tap][hi,lo][cin' group of 8]
 * [cout' padded to 64][8] fp16, scaled by 2^(15-e), max|w| < 2^e) and *w_amax =
 * max|w| (device scalar).  transpose=1: the data-gradient weights (as
 * stx_conv_weight_prep). */
int stx_conv_weight_prep16(const float* w, void* wt16, float* w_amax, int cout, int cin, int ks,
                           int transpose, void* stream);
/* The data-gradient split slab of a composed weight, for a Gram-backward operator that
 * feeds a 3x3 conv's data gradient with nothing in between (VGG conv3_1: dZ5 = A5 Z5,
 * then dP4 = conv3_1^T(dZ5); stransfer/network.py:92-123 StyleLoss backward through
 * :264-314 the conv3_1 piece):  conv^T_w(A . z) = conv^T_{w'}(z) with
 *   w'[c][ci][kh][kw] = s * sum_co A[c*pitch + co] * w[co][ci][kh][kw]   (s = *scale or 1)
 * so the data gradient reads z directly and dZ = A z is never formed.  The identity as
 * written needs A symmetric, which the Gram-backward operator is (coef = c (G - T) with
 * the diagonal alpha term; G and T symmetric); for a general A the launch computes
 * conv^T_w(A^T . z).  A is one image's
 * [cout][pitch] operator (pitch >= cout; stx_style_loss's coef), a_amax an amax group
 * >= max|A| (the finalize's coef_amax), w [cout][cin][3][3] with w_amax >= max|w|.  One
 * launch writes the transposed split slab wtT16 (stx_conv_weight16_bytes(cin, cout, 3, 1)
 * bytes) at the power-of-two scale of the bound |s| * cout * max|A| * max|w| >= max|w'|,
 * and stores that bound into every slot of the group out_amax: the conv takes
 * wt16 = wtT16, w_amax = out_amax.  cout <= 256, cin % 4 == 0, w 16-byte aligned; fixed
 * summation order. */
int stx_conv_weight_compose16(const float* A, int pitch, const float* a_amax, const float* w,
                              const float* w_amax, int cout, int cin, const float* scale,
                              void* wtT16, float* out_amax, void* stream);
/* Both split slabs of one weight (forward and data gradient) and their shared w_amax in
 * two launches (one max pass, one conversion) -- a trained layer re-preps every step. */
int stx_conv_weight_prep16_pair(const float* w, void* wt16, void* wtT16, float* w_amax,
                                int cout, int cin, int ks, void* stream);
/* The parity-class split slab of a 3x3 conv that reads a nearest x2 upsampled input
 * (UpsampleConvLayer, stransfer/network.py:578-600): each output parity class (a, b) of
 * the conv over the upsampled image is a 2x2 conv over the input with summed weights
 * W'[a][b][ry][rx] (16 instead of 36 tap MACs per 2x2 output group).  w [cout][cin][3][3]
 * -> wt16_up (stx_conv_weight16up_bytes(cin, cout) bytes), *w_amax = max|w| (the slab is
 * split at 2^(13 - e), |W'| <= 4 max|w|); stx_conv_params.wt16_up takes it. */
size_t stx_conv_weight16up_bytes(int cin, int cout);
int stx_conv_weight_prep16_up(const float* w, void* wt16_up, float* w_amax, int cout, int cin,
                              void* stream);
/* Every slab of a trained network in two launches (one max|w| pass over the distinct
 * split-slab weights, one conversion pass over all jobs) instead of two launches per
 * slab: the per-step re-prep of ImageTransformNet's 14 conv weights after each Adam
 * update (stransfer/network.py:765 optimizer.step -> the next static_train closure).
 * kind STX_WPREP_F32: slab as stx_conv_weight_prep(w, slab, cout, cin, ks, transpose);
 * kind STX_WPREP_F16: as stx_conv_weight_prep16(w, slab, w_amax, ...) (ks = 3).  The
 * forward and data-gradient split slabs of one weight may share w_amax (computed
 * once).  `jobs` is a host array read at call time (graph-capturable). */
#define STX_WPREP_MAX 48
#define STX_WPREP_F32 0
#define STX_WPREP_F16 1
#define STX_WPREP_F16UP 2 /* the parity-class slab (stx_conv_weight_prep16_up), transpose 0 */
typedef struct stx_wprep_job {
  const float* w;
  void* slab;
  float* w_amax;
  int kind, cout, cin, ks, transpose;
  int pad_;
} stx_wprep_job;
int stx_conv_weight_prep_batch(const stx_wprep_job* jobs, int njobs, void* stream);
/* *out = max |x[i]| over n floats (device scalar; NaN propagates). */
int stx_amax(const float* x, long long n, float* out, void* stream);

/* Gram partials per image a stx_conv2d call with these params writes through
 * gram_part (its 256-pixel output tiles), or 0 when the fused Gram does not apply. */
int stx_conv_gram_tiles(const stx_conv_params* p);
/* Gram group sums per image written with gram_cnt (ceil(T / STX_GRAM_GROUP)), 0 when
 * the fused Gram does not apply. */
int stx_conv_gram_groups(const stx_conv_params* p);

/* Implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32), fused input
 * transform (in_mode) and epilogue (bias, mask, aux, accumulate, relu). */
int stx_conv2d(const stx_conv_params* p, void* stream);

/* Weight gradient: dw[cout][cin][ks][ks] (+)= sum_{n,oy,ox} dy * xv  (xv = in_mode(x)).
 * Split-K partial slabs in ws (fp32), reduced in fixed order (deterministic).
 * Supported: ks=3 stride 1/2, ks=9 stride 1.  Workspace: stx_conv2d_wgrad_ws(). */
size_t stx_conv2d_wgrad_ws(int n, int cin, int cout, int ks, int stride, int ho, int wo);
int stx_conv2d_wgrad(const float* x, const float* dy, float* dw, int accumulate,
                     int n, int cin, int h, int w, int cout, int ks, int stride, int pad,
                     int in_mode, int hv, int wv, int ho, int wo,
                     void* ws, size_t ws_bytes, void* stream);
/* Weight gradient of a 3x3 stride-1 pad-1 conv on the fp16 hi/lo split MFMA
 * (in_mode RAW / RELU / UPSAMPLE2, hv x wv = dy's spatial size with wv % 16 == 0,
 * cin and cout >= 16); x_amax / dy_amax are amax groups of x and dy.  Split-K
 * partials in ws (stx_conv2d_wgrad16_ws, 0 = unsupported shape), fixed-order sum. */
size_t stx_conv2d_wgrad16_ws(int n, int cin, int cout, int in_mode, int hv, int wv);
int stx_conv2d_wgrad16(const float* x, const float* dy, float* dw, int accumulate, int n,
                       int cin, int h, int w, int cout, int in_mode, int hv, int wv,
                       const float* x_amax, const float* dy_amax, void* ws, size_t ws_bytes,
                       void* stream);
/* Weight gradient of the 3x3 stride-2 pad-1 downsampling convs of ImageTransformNet
 * (stransfer/network.py:528-533; replaces the autograd conv2d weight gradient of
 * static_train :690-765) on the fp16 hi/lo split MFMA: raw input x [n][cin][h][w]
 * with h = 2 ho, w = 2 wo, dy [n][cout][ho][wo], wo % 16 == 0, cin / cout >= 16.
 * Workspace: stx_conv2d_wgrad16_s2_ws (0 = unsupported shape). */
size_t stx_conv2d_wgrad16_s2_ws(int n, int cin, int cout, int ho, int wo);
int stx_conv2d_wgrad16_s2(const float* x, const float* dy, float* dw, int accumulate, int n,
                          int cin, int h, int w, int cout, int ho, int wo, const float* x_amax,
                          const float* dy_amax, void* ws, size_t ws_bytes, void* stream);

/* dW of the ImageTransformNet 9x9 stride-1 pad-4 layers whose one side has 1..3
 * channels and the other 32 (conv0 3->32, conv22 32->3; stransfer/network.py:525-527,
 * 605-609, trained by static_train :690-765) on the fp16 hi/lo split MFMA: the
 * 3-channel tensor is expanded per tap row in LDS, the 32-channel one streamed.
 * x_amax / dy_amax: amax groups (>= max|x|, max|dy|).  ws: per-block partials
 * (stx_conv2d_wgrad_few16_ws, 0 = unsupported shape), summed in a fixed order. */
size_t stx_conv2d_wgrad_few16_ws(int n, int cin, int cout, int ks, int h, int w);
int stx_conv2d_wgrad_few16(const float* x, const float* dy, float* dw, int accumulate, int n,
                           int cin, int h, int w, int cout, int ks, int pad, const float* x_amax,
                           const float* dy_amax, void* ws, size_t ws_bytes, void* stream);
/* db[c] (+)= sum_{n,p} dy[n][c][p]  (conv bias gradient) */
size_t stx_bias_grad_ws(int n, int c);
int stx_bias_grad(const float* dy, float* db, int n, int c, int hw, int accumulate,
                  void* ws, size_t ws_bytes, void* stream);

/* Gram: G[b] = F_b F_b^T * scale, F_b = z[b] viewed [c][hw].  Split-K MFMA +
 * deterministic reduction.  z_amax (optional device scalar >= max|z|, e.g. the
 * producing conv's out_amax): with it and hw % 8 == 0 the partials run on the fp16
 * hi/lo split MFMA (fp32-level accuracy), else on fp32 MFMA. */
size_t stx_gram_ws(int b, int c, int hw);
int stx_gram(const float* z, float* g, int b, int c, int hw, float scale,
             const float* z_amax, void* ws, size_t ws_bytes, void* stream);

/* Style loss forward + backward coefficients (StyleLoss.forward):
 *   G = gram(z)/(c*hw);  loss = mean((G - T)^2) over b*c*c  -> *loss (device scalar)
 *   A[b] = weight*4/(b*c*c*c*hw) * (G[b]-T) + diag_alpha*I     (A is [b][cpad][cpad])
 * so that dz = A·z (+ aux) is d(weight*loss)/dz; g_out (optional) receives G.
 * cpad = stx_gram_coef_pitch(c).  ws: stx_gram_ws(b, c, hw). */
int stx_gram_coef_pitch(int c);
/* With loss == NULL stx_style_loss leaves its loss partials in ws: *nparts floats at
 * byte offset stx_style_loss_parts(b, c, hw, &nparts), loss = sum * 1/(b*c*c). */
size_t stx_style_loss_parts(int b, int c, int hw, int* nparts);
/* Deferred loss reductions in one launch (the 5 StyleLoss values of a forward, then
 * the weighted total of get_total_current_{style,content}_loss):
 *   losses[i] = inv[i] * sum(parts[i][0 .. nparts[i]))          i < k (fixed order)
 *   *total    = sum_i w[i] losses[i] + sum_j w[k+j] extra[j]    (if total != NULL)
 * extra: m device scalars (e.g. the content loss); w_host: k + m host floats. */
typedef struct stx_loss_parts {
  const float* parts[8];
  int nparts[8];
  float inv[8];
  int k;
} stx_loss_parts;
int stx_loss_finalize(const stx_loss_parts* lp, float* losses, const float* extra, int m,
                      const float* w_host, float* total, void* stream);
int stx_style_loss(const float* z, const float* target, float* g_out, float* coef,
                   float* loss, int b, int c, int hw, int target_batched, float weight,
                   float diag_alpha, const float* z_amax, void* ws, size_t ws_bytes,
                   void* stream);
/* dz (+)= s * A[b]·z[b] (+ aux_scale*aux) — Gram backward as a 1x1 MFMA conv with
 * per-image weights; z viewed [b][c][h][w]; s = *acc_scale_dev (or 1 if NULL) */
int stx_gram_bwd(const float* coef, const float* z, float* dz, int b, int c, int h, int w,
                 const float* acc_scale_dev, const float* mask, const float* aux,
                 float aux_scale, int accumulate, void* stream);

/* Sum-of-squared-difference reductions (ContentLoss / FeatureReconstructionLoss):
 *   s = sum((f(a) - f(b))^2), f = relu if relu_inputs else identity
 *   mode 0: *out = s / n                        (F.mse_loss, mean)
 *   mode 1: out[0] = (s / n)^2 / n, out[1] = s / n   (FeatureReconstructionLoss)
 *   mode 2: both from one pass (16-B aligned a, b; relu_inputs ignored):
 *           out[0] = mean((a-b)^2), out[1] = mean((relu a - relu b)^2)^2 / n,
 *           out[2] = mean((relu a - relu b)^2)   (content + feature at conv2_2)
 * grad (optional, mode 0): grad = gscale * 2*(a-b)/n. */
size_t stx_mse_ws(long long n);
int stx_mse(const float* a, const float* b, long long n, int relu_inputs, int mode,
            float* out, float* grad, float gscale, void* ws, size_t ws_bytes, void* stream);
/* grad (+)= s0 * (*s1) * (*s2) * (f(a) - f(b)) [* (a>0) if relu]; s1/s2 device scalars or NULL */
int stx_diff_scale(const float* a, const float* b, float* grad, long long n, float s0,
                   const float* s1_dev, const float* s2_dev, int relu, int accumulate,
                   void* stream);
/* stx_style_loss(z, ...) and stx_mse(z, content, b*c*hw, 0, 2, mse_out, ...) (the content,
 * feature and feature-mse values of ContentLoss / FeatureReconstructionLoss at the
 * content tap, stransfer/network.py:155-164, 186-201) in one pass over z where the
 * Gram kernel allows it (c = 128 on the split path), else as the two calls.
 * ws >= stx_style_content_ws(b, c, hw); the deferred style-loss partials sit where
 * stx_style_loss_parts says, as for stx_style_loss. */
size_t stx_style_content_ws(int b, int c, int hw);
int stx_style_content_loss(const float* z, const float* target, float* coef, float* loss,
                           int b, int c, int hw, int target_batched, float weight,
                           float diag_alpha, const float* z_amax, const float* content,
                           float* mse_out, void* ws, size_t ws_bytes, void* stream);
/* stx_style_loss from precomputed Gram partials (stx_conv_params.gram_part; c <= 64 or
 * c == 128): parts [b][U][nparts][64][64] (U = 1, or 3 tiles for c = 128) summed in a
 * fixed order, then the same G, coef, loss and deferred loss partials
 * (ws >= stx_gram_ws(b, c, hw); stx_style_loss_parts). */
int stx_style_loss_from_parts(const float* parts, int nparts, const float* target,
                              float* g_out, float* coef, float* loss, int b, int c, int hw,
                              int target_batched, float weight, float diag_alpha, void* ws,
                              size_t ws_bytes, void* stream);
/* stx_style_loss_from_parts plus the content tap's content / feature / feature-mse values
 * (stx_style_content_loss's mse_out) from the conv epilogue's MSE sums
 * (stx_conv_params.mse_parts: b * nparts pairs), finalized by the same launch. */
int stx_style_content_loss_from_parts(const float* parts, int nparts, const float* target,
                                      float* coef, float* loss, int b, int c, int hw,
                                      int target_batched, float weight, float diag_alpha,
                                      const float* mse_parts, float* mse_out, void* ws,
                                      size_t ws_bytes, void* stream);
/* Deferred Gram finalizes.  The *_deferred forms of stx_style_loss,
 * stx_style_content_loss and stx_style_loss_from_parts launch only their partial
 * kernel(s) (if any) and describe the finalize (G, coef, loss partials, the fused content
 * MSE) in *job; stx_gram_finalize_batch then runs up to STX_FIN_MAX such finalizes -- the
 * five StyleLoss taps of a forward -- in ONE launch, block for block the same arithmetic
 * (bit-identical to the immediate forms).  The loss partials land where
 * stx_style_loss_parts says; reduce them with stx_loss_finalize. */
#define STX_FIN_MAX 8
typedef struct stx_gram_fin_job {
  const float* parts;      /* partial slabs [b][ntiles][nsplit][64][64] */
  float* g_out;            /* optional G */
  const float* target;
  float* coef;
  float* loss_parts;
  const float* mse_parts;  /* fused content pass (or NULL) */
  float* mse_out;
  long long t_bstride;
  double mse_n;
  float scale, cA, alpha;
  int c, nsplit, b, cpad, mse_nparts;
  float* coef_amax;        /* optional amax group (zeroed): >= max|coef| over the batch */
} stx_gram_fin_job;
int stx_style_loss_deferred(const float* z, const float* target, float* coef, int b, int c,
                            int hw, int target_batched, float weight, float diag_alpha,
                            const float* z_amax, void* ws, size_t ws_bytes, stx_gram_fin_job* job,
                            void* stream);
int stx_style_content_loss_deferred(const float* z, const float* target, float* coef, int b,
                                    int c, int hw, int target_batched, float weight,
                                    float diag_alpha, const float* z_amax, const float* content,
                                    float* mse_out, void* ws, size_t ws_bytes,
                                    stx_gram_fin_job* job, void* stream);
int stx_style_loss_from_parts_deferred(const float* parts, int nparts, const float* target,
                                       float* coef, int b, int c, int hw, int target_batched,
                                       float weight, float diag_alpha, void* ws, size_t ws_bytes,
                                       stx_gram_fin_job* job, void* stream);
int stx_style_content_loss_from_parts_deferred(const float* parts, int nparts,
                                               const float* target, float* coef, int b, int c,
                                               int hw, int target_batched, float weight,
                                               float diag_alpha, const float* mse_parts,
                                               float* mse_out, void* ws, size_t ws_bytes,
                                               stx_gram_fin_job* job, void* stream);
int stx_gram_finalize_batch(const stx_gram_fin_job* jobs, int njobs, void* stream);

/* *out = sum_i w_host[i] * s[i]   (k <= 16 device scalars, fixed order) */
int stx_loss_combine(const float* s, int k, const float* w_host, float* out, void* stream);

/* Vector kernels of the on-device L-BFGS (StyleNetwork.train_gatys' optimiser,
 * stransfer/network.py:435; torch.optim.LBFGS semantics):
 *   stx_vec_reduce: r = dot(a,b) (op 0), sum|a| (op 1) or max|a| (op 2) over n floats
 *     (fixed-order two-stage reduction, ws >= stx_vec_ws()), then
 *     *out = (add ? *add : 0) + sgn * r * (mul ? *mul : 1)   (device scalars)
 *   stx_vec_axpby: y = alpha*x + b*y, alpha = a_dev ? a_sgn * (*a_dev) * a : a
 *   stx_scalar_op: s[k] = s[i] op s[j]  (0 div, 1 mul, 2 sub, 3 add, 4 1/s[i],
 *     5 min(s[j], 1/s[i])) on a device scalar array */
size_t stx_vec_ws(void);
int stx_vec_reduce(const float* a, const float* b, long long n, int op, float* out,
                   const float* mul, const float* add, float sgn, void* ws, size_t ws_bytes,
                   void* stream);
int stx_vec_axpby(float* y, const float* x, long long n, float a, const float* a_dev,
                  float a_sgn, float b, void* stream);
int stx_scalar_op(float* s, int op, int i, int j, int k, void* stream);

/* L-BFGS in the compact form (lbfgs.hip): torch.optim.LBFGS's search direction, step
 * size and parameter update without line search (StyleNetwork.train_gatys,
 * stransfer/network.py:435-456; torch/optim/lbfgs.py's two-loop recursion) in a fixed
 * launch sequence whatever the history length.
 *   hist   [2][m + 1][npad] floats (stx_lbfgs_hist_bytes): S slots then Y slots, a ring
 *          of m committed pairs + one candidate; npad = n rounded up to 1024
 *   state  stx_lbfgs_state_bytes(m) bytes, zeroed by the caller before the first call:
 *          pair order, R = [s_i.y_j], Y^T Y, H_diag, t, torch's n_iter
 *   prev_g npad floats (the previous gradient)
 *   scal   >= 16 device floats the host reads: 0 loss, 1 max|g|, 2 sum|g|, 3 g.d, 4 t,
 *          5 max|t d|, 6 stop flag (g.d > -tol_change: x not moved), 7 y.s, 8 pairs,
 *          9 n_iter, 10 H_diag
 * stx_lbfgs_grad_stats (after each closure evaluation): scal[0] = *loss (if loss),
 *   scal[1] = max|g|, scal[2] = sum|g|; zeroes clear[0 .. clear_n).
 * stx_lbfgs_direction (one torch loop iteration up to the next closure): n_iter += 1;
 *   y = g - prev_g, s = t_prev d_prev, accept when y.s > 1e-10 (H_diag = y.s / y.y); t =
 *   min(1, 1/sum|g|) * lr on the first iteration, else lr; d = -H g; g.d; x += t d unless
 *   g.d > -tol_change.  1 <= m <= 256; 16-byte aligned vectors. */
size_t stx_lbfgs_state_bytes(int m);
size_t stx_lbfgs_hist_bytes(long long n, int m);
size_t stx_lbfgs_ws(long long n, int m);
int stx_lbfgs_direction(float* x, const float* g, float* prev_g, float* hist, long long n, int m,
                        float lr, float tol_change, void* state, float* scal, void* ws,
                        size_t ws_bytes, void* stream);
int stx_lbfgs_grad_stats(const float* g, long long n, const float* loss, float* scal, float* clear,
                         int clear_n, void* ws, size_t ws_bytes, void* stream);

/* MaxPool2d(2,2) on (optionally relu'd) input; idx = flat y*w+x argmax per plane,
 * torch CPU semantics (first max in row-major window order; NaN propagates). idx may be NULL. */
int stx_maxpool2x2_fwd(const float* x, float* y, long long* idx, int nc, int h, int w,
                       int relu_input, void* stream);
/* dx = scatter(dy at idx)  (dx fully written, gather form) */
int stx_maxpool2x2_bwd(const float* dy, const long long* idx, float* dx, int nc, int h, int w,
                       void* stream);
/* dz = unpool(dp) * (z > 0): backward of ReLU + MaxPool2d(2,2) with the argmax
 * recomputed from z (dz fully written; z is the pre-ReLU tensor [nc][h][w]) */
int stx_relupool_bwd(const float* dp, const float* z, float* dz, int nc, int h, int w,
                     void* stream);
int stx_relu_fwd(const float* x, float* y, long long n, void* stream);
/* dx = dy * (y > 0) */
int stx_relu_bwd(const float* dy, const float* y, float* dx, long long n, void* stream);

/* Adam (torch.optim.Adam semantics, in place; 16-byte aligned buffers).
 * step_dev: device int32 step counter, incremented on the device by every call so
 * a captured graph replays correctly.  ws: stx_adam_ws() bytes of device scratch. */
size_t stx_adam_ws(void);
int stx_adam_step(float* p, const float* g, float* m, float* v, long long n, float lr,
                  float beta1, float beta2, float eps, int* step_dev, void* ws, void* stream);
/* the same, and zeroes clear[0 .. clear_n) in the step-counter launch (the Gatys
 * engine's per-iteration amax groups, which are next produced by the following
 * iteration's forward): one launch fewer per iteration than a separate fill. */
int stx_adam_step_clear(float* p, const float* g, float* m, float* v, long long n, float lr,
                        float beta1, float beta2, float eps, int* step_dev, void* ws,
                        float* clear, int clear_n, void* stream);

/* InstanceNorm2d(affine) forward, per (n,c) plane over hw (biased var, eps):
 *   u = x (+ res);  y = (u-mean)*rstd*gamma + beta, formed as fma(u, gsc, sh) with
 *   gsc = gamma rstd, sh = fma(-mean, gsc, beta);  y = max(y,0) if relu.
 * mean/rstd [n*c] saved for the backward (may be NULL).  out_amax (amax group, zeroed
 * by the caller, may be NULL) receives max|y| -- the next split conv's input scale. */
int stx_instnorm_fwd(const float* x, const float* res, const float* gamma, const float* beta,
                     float* y, float* mean, float* rstd, int n, int c, int hw, float eps,
                     int relu, float* out_amax, void* stream);
/* backward: dy = grad wrt y; beta = the forward's beta (NULL if none).  With relu the
 * mask y > 0 is recomputed from u = x (+ res), mean, rstd, gamma and beta exactly as the
 * forward formed y (y = fma(u, gsc, sh), gsc = gamma rstd, sh = fma(-mean, gsc, beta):
 * the same bits), so y itself is not read.  du = grad wrt u (= grad of x and of res).  dgamma/dbeta (may be NULL) (+)= sums over n (fixed order).  dbias_in
 * (may be NULL) (+)= sum_{n,p} du: the bias gradient of the conv that produced x
 * (stransfer/network.py:471-611, every Conv2d followed by InstanceNorm2d), so that
 * conv needs no separate bias-gradient pass.  out_amax (amax group or NULL) receives
 * max|du| -- the split dgrad/wgrad scale of du. */
size_t stx_instnorm_bwd_ws(int n, int c);
/* The parameter reductions of many stx_instnorm_bwd calls in one launch: each such
 * call ran with dgamma = dbeta = dbias_in = NULL into its own workspace `parts`
 * (>= stx_instnorm_bwd_ws(n, c) bytes, kept until this call); each job then writes /
 * accumulates its dgamma, dbeta, dbias_in (any may be NULL) with the same fixed-order
 * sums over n -- one launch per training step instead of one per InstanceNorm2d
 * layer (stransfer/network.py:474-600, 15 layers in ImageTransformNet). */
#define STX_PGRAD_MAX 32
typedef struct stx_in_pgrad_job {
  const float* parts;
  float* dgamma;
  float* dbeta;
  float* dbias_in;
  int n, c, accumulate, pad_;
} stx_in_pgrad_job;
int stx_instnorm_param_grads(const stx_in_pgrad_job* jobs, int njobs, void* stream);
int stx_instnorm_bwd(const float* dy, const float* beta, const float* x, const float* res,
                     const float* gamma, const float* mean, const float* rstd, float* du,
                     float* dgamma, float* dbeta, float* dbias_in, int n, int c, int hw, int relu,
                     int accumulate_params, float* out_amax, void* ws, size_t ws_bytes,
                     void* stream);

/* nearest x2 upsample: y [nc][2h][2w];  backward dx[y][x] = sum of dy's 2x2 block */
int stx_upsample2x_fwd(const float* x, float* y, int nc, int h, int w, void* stream);
int stx_upsample2x_bwd(const float* dy, float* dx, int nc, int h, int w, void* stream);

/* Total variation, batch SUM (stransfer/network.py:621-641):
 *   *loss = factor*(sum|y[..,x]-y[..,x+1]| + sum|y[..,y,:]-y[..,y+1,:]|)
 *   grad (optional) = gscale * (*gscale_dev or 1) * d loss / dy */
size_t stx_tv_ws(int n, int c, int h, int w);
int stx_tv_loss(const float* y, float* loss, float* grad, float gscale, const float* gscale_dev,
                int n, int c, int h, int w, float factor, void* ws, size_t ws_bytes,
                void* stream);

/* Temporal loss of the video network (VideoTransformNet.get_temporal_loss,
 * stransfer/network.py:885-903), Frobenius norms over the whole batch:
 *   out[0] = ||y - y_old|| / (||x - x_old|| + 1) * weight,  out[1] = ||y - y_old||,
 *   out[2] = ||x - x_old||   (one streaming pass, fixed-order reduction)
 * Backward: grad (+)= (*g_dev or 1) * weight / ((out[2] + 1) * out[1]) * (y - y_old)
 * (0 where out[1] == 0, torch's norm backward); fwd = the forward's out.
 * All four tensors hold n floats, 16-byte aligned. */
size_t stx_temporal_loss_ws(void);
int stx_temporal_loss(const float* y, const float* y_old, const float* x, const float* x_old,
                      long long n, float weight, float* out, void* ws, size_t ws_bytes,
                      void* stream);
int stx_temporal_loss_bwd(const float* y, const float* y_old, long long n, const float* fwd,
                          float weight, const float* g_dev, float* grad, int accumulate,
                          void* stream);

/* Image conditioning (img_utils.image_loader_transform, stransfer/img_utils.py:13-44)
 * of a batch of decoded 8-bit RGB images on the GPU: centre crop, Pillow-exact
 * BILINEAR resize to size x size (its 8-bit fixed-point two-pass resampler: output
 * bytes equal PIL's), ToTensor (/255) and (x - mean) / std -> out [b][3][size][size].
 * src: device buffer of packed HWC uint8 images; meta: device array of b entries;
 * coef: device int tables, per axis [out][2] bounds (first tap, taps) followed by
 * [out][k] coefficients, built with stx_resample_coeffs (host function: returns the
 * kernel size k, or with NULL outputs only the size query); mean/std: HOST arrays
 * of 3; tmp: device workspace holding every image's horizontally resampled rows
 * (max_rows = the largest y1 - y0; 0 when no image needs the horizontal pass). */
typedef struct {
  long long offset;        /* byte offset of the image in src */
  int h, w;                /* decoded size */
  int top, left;           /* centre-crop origin */
  int y0, y1;              /* crop rows read by the vertical pass */
  int resize_w, resize_h;  /* passes needed (0: the crop side already equals size) */
  int xcoef, ycoef;        /* int offsets of the two axis tables in coef */
  int xk, yk;              /* their kernel sizes */
  long long tmp_offset;    /* byte offset of this image's rows in tmp ([rows][size][3]) */
} stx_image_meta;
int stx_resample_coeffs(int in_size, int out_size, int* bounds, int* kk, int kk_stride);
int stx_image_condition(const void* src, const stx_image_meta* meta, int b, int max_rows,
                        const int* coef, int size, const float* mean, const float* std_,
                        float* out, void* tmp, size_t tmp_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* STX_H_ */
