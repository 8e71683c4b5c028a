/*
 * adaptseg.h — C ABI of the MI355X-native AdaptSegNet adversarial-step kernels.
 *
 * One shared library (adaptsegnet_amd/lib/libadaptseg.so), gfx950 only.  Every entry
 * point takes plain device pointers, sizes and a hipStream_t (passed as void*), returns
 * an int status (ADAPTSEG_OK = 0) and never throws.  No global allocation happens
 * behind the caller's back: ops that need scratch take a caller-owned workspace whose
 * size is reported by the matching *_workspace_size() call.  Nothing here synchronises
 * the device, so every call is graph-capturable.
 *
 * Activation layout: NHWC fp32 ("channels_last" of the reference's NCHW tensors).
 * Weight layout: [Cout][KH][KW][Cin] (= torch channels_last of the reference's
 * [Cout][Cin][KH][KW] parameters, so state_dict shapes are unchanged).
 *
 * The reference (sahngmin/AdaptSegNet) is pure PyTorch; each entry point below names
 * the torch.nn call site whose arithmetic it replaces.
 */
#ifndef ADAPTSEG_H
#define ADAPTSEG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *adaptseg_stream_t; /* hipStream_t */

enum adaptseg_status {
  ADAPTSEG_OK = 0,
  ADAPTSEG_ERR_ARG = 1,         /* bad shape / null pointer / misaligned */
  ADAPTSEG_ERR_UNSUPPORTED = 2, /* valid request this build does not implement */
  ADAPTSEG_ERR_HIP = 3,         /* launch or runtime error (see adaptseg_last_error) */
  ADAPTSEG_ERR_WORKSPACE = 4    /* workspace smaller than *_workspace_size() */
};

/* Human-readable description of the last error raised on the calling thread. */
const char *adaptseg_last_error(void);
/* Library build string, e.g. "adaptseg 0.1 gfx950". */
const char *adaptseg_version(void);

/* ------------------------------------------------------------------------------------ */
/* Convolution (implicit GEMM on the MFMA: by default F32X3 = fp32-accurate products on   */
/* v_mfma_f32_32x32x16_bf16 through exact 3-term bf16 splits, conv_x3.hpp / conv_x3r.hpp; */
/* v_mfma_f32_32x32x2_f32 under ADAPTSEG_MATH_F32; bf16 operands under ADAPTSEG_MATH_BF16). */
/* Replaces nn.Conv2d in model/deeplab_multi.py:64,70-71,75,128,158-159 (Bottleneck,    */
/* stem, downsample), Classifier_Module model/deeplab_multi.py:106-121 (ASPP: nseg=4    */
/* branches summed into one GEMM with concatenated K) and model/discriminator.py:10-14.  */
/* ------------------------------------------------------------------------------------ */
typedef struct adaptseg_conv_desc {
  int n, c, h, w;          /* input batch, channels, height, width                       */
  int64_t in_stride[4];    /* input element strides for (n, c, h, w); NHWC = {HWC,1,WC,C} */
  int k, oh, ow;           /* output channels and spatial size; output is NHWC-contiguous */
  int kh, kw;              /* kernel size (same for every segment)                       */
  int stride;              /* spatial stride (both dims)                                 */
  int nseg;                /* 1, or the number of summed branches (ASPP: 4)              */
  int pad[4];              /* per-segment padding (both dims)                            */
  int dil[4];              /* per-segment dilation (both dims)                           */
} adaptseg_conv_desc;

enum adaptseg_conv_op { ADAPTSEG_CONV_FWD = 0, ADAPTSEG_CONV_BWD_DATA = 1, ADAPTSEG_CONV_BWD_WEIGHT = 2 };

/* Epilogue flags (bitwise OR). */
enum adaptseg_conv_flags {
  ADAPTSEG_EPI_LEAKY = 1,      /* fwd: y = leaky_relu(y, 0.2)  (discriminator.py:21-29)    */
  ADAPTSEG_EPI_ACCUMULATE = 2, /* out += result instead of out = result                    */
  ADAPTSEG_EPI_LEAKY_GRAD = 4, /* bwd_data: dx *= (aux > 0 ? 1 : 0.2)                      */
  ADAPTSEG_EPI_RESIDUAL = 8,   /* out = result + res (same NHWC shape as out)              */
  ADAPTSEG_EPI_RELU = 16,      /* fwd: y = relu(y)  (deeplab_vgg.py:34-43 conv + ReLU)     */
  ADAPTSEG_EPI_RELU_GRAD = 32, /* bwd_data: dx *= (aux > 0 ? 1 : 0)                        */
  ADAPTSEG_WGRAD_DEFER_SUM = 64 /* bwd_weight: leave a split-K sum pending (adaptseg_splitk_flush) */
};

/* Conv arithmetic, process-wide (set before sizing workspaces; every conv entry point and
   *_workspace_size() reads it).  The library default is F32X3 (conv_igemm.hip).  F32: fp32
   MFMA, exact fp32 products.  BF16: the
   operands of each product are rounded to bf16 (RNE) as they are staged into LDS and
   multiplied on v_mfma_f32_32x32x16_bf16 with fp32 accumulation — torch.autocast(bfloat16)
   conv semantics; activations, gradients and epilogues stay fp32 (BASELINE config c5).
   Products the bf16 kernel does not cover (Cin or Cout not a multiple of 64 for the forward /
   data-gradient, per-element operands) stay on the fp32 path. */
enum adaptseg_conv_math {
  ADAPTSEG_MATH_F32 = 0,
  ADAPTSEG_MATH_BF16 = 1,
  ADAPTSEG_MATH_BF16_WIDE = 2, /* BF16 with 128x256 tiles for fwd / data-grad products with N >= 256 */
  ADAPTSEG_MATH_F32X3 = 3,     /* fp32 on the bf16 MFMA: exact 3-term bf16 splits of both operands,
                                  the 6 products above 2^-23 relative (fp32-accurate; conv_x3.hpp) */
  ADAPTSEG_MATH_F32X3_PRESPLIT = 4 /* F32X3 arithmetic (bitwise the same results where neither
                                  splits K) with every product the 256x128x32 term-image kernel
                                  covers on it (conv_x3r.hpp, LDS-DMA of PRE-SPLIT bf16 term
                                  images written by the producing BN passes) */
};
int adaptseg_conv_set_math(int math);
int adaptseg_conv_get_math(int *math);
/* Kernel-selection options, process-wide (set before sizing workspaces, like the maths); the
   initial values come from the environment variables named below.
     ADAPTSEG_OPT_X3H (ADAPTSEG_X3H, default 0): F32X3 maths, bit 1 / 2 / 4 = forward / data-gradient
       / weight-gradient products that the 256x128x32 term-image tiles cover (a 32-deep K step inside
       one tap) run on igemm_x3h_kernel / igemm_x3hw_kernel<128> — those tiles with the fp32 operands
       split in-kernel, no term images — instead of the register-staged 128x128x16 kernel.  Same
       arithmetic (bitwise the term-image kernels' results on the same plan).
     ADAPTSEG_OPT_G16_WIDE (ADAPTSEG_G16_WIDE, default 1): BF16 maths, bit 1 = forward /
       data-gradient products with N >= 256 and K >= 2048 on the 256x256x64 two-stage LDS-DMA
       tile, bit 2 = weight gradients with Cout >= 256 and N >= 256 on the 256x256 tile with
       64-pixel K steps. */
enum adaptseg_conv_option { ADAPTSEG_OPT_X3H = 1, ADAPTSEG_OPT_G16_WIDE = 2 };
int adaptseg_conv_set_option(int option, int value);
int adaptseg_conv_get_option(int option, int *value);

int adaptseg_conv2d_workspace_size(const adaptseg_conv_desc *d, int op, size_t *bytes);
/* Kernel selector (see adaptseg_timing_enable) and K-split count the library would use. */
int adaptseg_conv2d_kernel_id(const adaptseg_conv_desc *d, int op, int *kernel_id, int *splits);
/* The same for a call of the _x forms that passes the operand copies (with_copies != 0): under
   the F32X3 maths the products the 256x128x32 term-image kernel covers move to it (selector
   100*op + 88, + 89 for the stride-2 parity path / 128-row weight gradients). */
int adaptseg_conv2d_kernel_id_x(const adaptseg_conv_desc *d, int op, int with_copies, int *kernel_id, int *splits);

/* y[n,oh,ow,k] = sum_seg conv(x, w[seg]) + sum_seg bias[seg]   (bias may be NULL) */
int adaptseg_conv2d_fwd(const adaptseg_conv_desc *d, const float *x, const float *const *w,
                        const float *const *bias, const float *res, float *y, int flags,
                        void *ws, size_t ws_bytes, adaptseg_stream_t stream);

/* Forward conv (no bias / epilogue flags) that also emits the per-row-tile BatchNorm
   statistics of y for adaptseg_bn_fwd_train_tiles: stats = [ntiles] row counts, then
   [k][ntiles] tile means, then [k][ntiles] tile sums of squared deviations.  *ntiles = 0
   when the chosen kernel cannot produce them (split-K, unaligned operands, tap-GEMM path):
   y is still computed and the caller runs adaptseg_bn_fwd_train.  The BN statistics pass
   over y is skipped otherwise (model/deeplab_multi.py:83-103: every Bottleneck conv feeds a
   BatchNorm). */
int adaptseg_conv2d_bnstats_size(const adaptseg_conv_desc *d, size_t *bytes);
/* The row-tile count adaptseg_conv2d_fwd_bnstats will produce for `d` (0: no fused
   statistics for this geometry), assuming 16-byte aligned operands: lets a caller size and
   plan the BatchNorm that follows before launching (host-side, no GPU). */
int adaptseg_conv2d_bnstats_tiles(const adaptseg_conv_desc *d, int *ntiles);
/* ... for adaptseg_conv2d_fwd_bnstats_x called with (with_copy != 0) or without x's copy: under
   the F32X3 maths the copy moves the product to a kernel with 256-row tiles. */
int adaptseg_conv2d_bnstats_tiles_x(const adaptseg_conv_desc *d, int with_copy, int *ntiles);
int adaptseg_conv2d_fwd_bnstats(const adaptseg_conv_desc *d, const float *x, const float *const *w,
                                float *y, float *stats, size_t stats_bytes, int *ntiles, void *ws,
                                size_t ws_bytes, adaptseg_stream_t stream);

/* bf16 operand copies (conv math ADAPTSEG_MATH_BF16, config c5).  The _x forms take, beside
   the fp32 activation operand, an optional bf16 (RNE) copy of it as written by the producing
   BatchNorm pass (adaptseg_bn_*_x): contiguous NHWC, 16-byte aligned; NULL = none.  The bf16
   LDS-DMA kernel (forward and stride-1 data gradient with N >= 128) then reads it instead of
   converting the operand itself, one pass over the activation less per call; every other
   kernel ignores it.  The results are bitwise those of the plain forms (the copy holds
   exactly the values the kernel would have rounded).  The fp32 operand itself may then be
   NULL — its producer skipped writing it — but only when the product runs on that kernel
   (adaptseg_conv2d_kernel_id selector 100*op + 94 / 97-99, or 192 / 193 for the stride-2
   data gradient); otherwise ADAPTSEG_ERR_ARG, checked on the host before any launch.  Same
   interfaces otherwise (model/deeplab_multi.py:83-103: the Bottleneck convs consume BN+ReLU
   outputs).
   y_bf16 / dx_bf16 (optional, NULL = none): a bf16 (RNE) copy of the fp32 output, written by
   the GEMM epilogue or split-K reduce beside y / dx (a separate pass on the thin and tap-GEMM
   paths), so that a consumer conv's _x operand needs no conversion pass: the discriminator
   convs (model/discriminator.py:14-27) chain conv -> LeakyReLU -> conv with no BatchNorm
   between.  Contiguous NHWC like y; 2-byte alignment suffices.  bf16 activation storage (config
   c5): the forward forms take y == NULL with y_bf16 given — the conv output is stored in bf16
   only (fused BN statistics still come from the fp32 accumulators) — on the implicit-GEMM
   kernels (not the thin / tap-GEMM paths, which return ADAPTSEG_ERR_ARG for it). */
/* *only = 1 when product `op` of `d` (16-byte aligned operands) runs on a kernel that reads
   ONLY the operand copies of the _x forms (the LDS-DMA kernels; the register-staged bf16
   forward; a tap-GEMM forward / weight gradient whose inner GEMM is on an LDS-DMA kernel), so
   the fp32 operand may be NULL and its producer need not write it; 0 otherwise (thin,
   per-element and register-staged fp32 kernels, the tap-GEMM data gradient read fp32).  Host-side planning, no GPU.  The same plan
   the _x entry points check against. */
int adaptseg_conv2d_copy_operand_only(const adaptseg_conv_desc *d, int op, int *only);

/* Operand BatchNorm (round 6): a train-mode BatchNorm + ReLU folded into the consuming conv's
   operand gather, so the BN's output is never written.  The conv reads x_pre, the BN's INPUT
   (fp32 NHWC, contiguous), and uses relu((x_pre - mean) * invstd * weight + bias) per element —
   the expression of the BN apply pass (adaptseg_bn_fwd_train*: bitwise the conv of that pass's
   output); positions outside the image read 0.  Two products have such a kernel (F32X3 maths):
   the forward on the 256x128x32 x3h tile and the register-staged weight gradient, for a BN of at
   most 512 channels; adaptseg_conv2d_operand_bn_ok reports whether product `op` of `d` runs on
   one (host-side planning, 16-byte aligned operands), and the _abn entry points return
   ADAPTSEG_ERR_ARG otherwise.  The reference's pair is model/deeplab_multi.py:92-95
   (out = relu(bn2(conv2(..))); out = conv3(out)). */
typedef struct {
  const float *mean, *invstd;   /* the BN's batch statistics (adaptseg_bn_fwd_train_tiles_stats) */
  const float *weight, *bias;   /* its affine parameters (NULL: 1 / 0) */
} adaptseg_operand_bn;
int adaptseg_conv2d_operand_bn_ok(const adaptseg_conv_desc *d, int op, int *ok);
/* adaptseg_conv2d_fwd_bnstats_x with the operand BN on x_pre (fp32 output, the row-tile
   statistics of y as there) */
int adaptseg_conv2d_fwd_bnstats_abn(const adaptseg_conv_desc *d, const float *x_pre, const adaptseg_operand_bn *abn,
                                    const float *const *w, const void *w_pack, float *y, float *stats,
                                    size_t stats_bytes, int *ntiles, void *ws, size_t ws_bytes,
                                    adaptseg_stream_t stream);
/* adaptseg_conv2d_bwd_weight with the operand BN on x_pre (no bias gradient) */
int adaptseg_conv2d_bwd_weight_abn(const adaptseg_conv_desc *d, const float *dy, const float *x_pre,
                                   const adaptseg_operand_bn *abn, float *const *dw, int flags, void *ws,
                                   size_t ws_bytes, adaptseg_stream_t stream);
/* Caller-owned weight packs.  The F32X3 and bf16 kernels read the weights of the forward and
   data-gradient products as a pack (the exact three-term bf16 split, or bf16 rows, laid out in
   the kernels' tile order) which the entry points otherwise build per call
   (optimizer.step in train_gta2cityscapes_multi.py:532-540 is the only writer of the weights:
   a training step calls each conv's forward 2-3 times and its data gradient 1-3 times on
   unchanged weights).  adaptseg_conv2d_wpack_size: *bytes = 0 when product `op` of `d` (16-byte
   aligned operands) reads no pack (fp32-input, thin and tap-GEMM kernels, the weight gradient);
   adaptseg_conv2d_wpack builds it (same kernel as the per-call pack, same bytes).  The `w_pack`
   argument of the _x forms takes one (NULL = build per call); it is valid for the weights it
   was built from until they are written — keeping that promise is the caller's side (the
   trainer rebuilds every pack once per step, adaptsegnet_amd.kernels.weight_pack_scope).  A
   plan that ends on a kernel without a pack (misaligned operands) ignores it;
   adaptseg_conv2d_wpack rejects misaligned weights (ADAPTSEG_ERR_ARG). */
int adaptseg_conv2d_wpack_size(const adaptseg_conv_desc *d, int op, size_t *bytes);
int adaptseg_conv2d_wpack(const adaptseg_conv_desc *d, int op, const float *const *w, void *pack, size_t bytes,
                          adaptseg_stream_t stream);
int adaptseg_conv2d_fwd_x(const adaptseg_conv_desc *d, const float *x, const uint16_t *x_bf16,
                          const float *const *w, const void *w_pack, const float *const *bias, const float *res,
                          float *y, uint16_t *y_bf16, int flags, void *ws, size_t ws_bytes,
                          adaptseg_stream_t stream);
int adaptseg_conv2d_fwd_bnstats_x(const adaptseg_conv_desc *d, const float *x, const uint16_t *x_bf16,
                                  const float *const *w, const void *w_pack, float *y, uint16_t *y_bf16,
                                  float *stats, size_t stats_bytes, int *ntiles, void *ws, size_t ws_bytes,
                                  adaptseg_stream_t stream);
int adaptseg_conv2d_bwd_data_x(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16,
                               const float *const *w, const void *w_pack, const float *res, const float *aux,
                               float *dx, uint16_t *dx_bf16, int flags, void *ws, size_t ws_bytes,
                               adaptseg_stream_t stream);
/* adaptseg_conv2d_bwd_data_x with bf16 GRADIENT storage (BF16 conv maths, config c5: under
   torch.autocast(bfloat16) the data gradients of the convs and the residual gradient of a
   Bottleneck, model/deeplab_multi.py:83-103, are bf16 tensors).  The residual read by
   ADAPTSEG_EPI_RESIDUAL is fp32 (res) or bf16 (res_bf16, 16-byte aligned; at most one of them);
   dx == NULL stores the output in bf16 only (dx_bf16: RNE of the fp32 epilogue value), and then
   ADAPTSEG_EPI_ACCUMULATE adds to dx_bf16.  The thin (Cout <= 4) and tap-GEMM products keep fp32
   gradients (ADAPTSEG_ERR_ARG for res_bf16 / dx == NULL there, and under the F32X3 maths).
   res_bits (any conv maths; Cin % 32 == 0; NULL = none): a ReLU mask bitmap [rows][Cin / 32] of
   the residual (written by adaptseg_bn_fwd_*_xm) — the epilogue adds res only where the bit is
   set, i.e. the masked residual gradient g = gout * [out > 0] of a Bottleneck (deeplab_multi.py:
   96-103) read straight from gout, so the BN backward need not write g out.
   adaptseg_conv2d_bwd_data_x is this with res_bf16 = res_bits = NULL and dx != NULL. */
int adaptseg_conv2d_bwd_data_xg(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16,
                                const float *const *w, const void *w_pack, const float *res, const uint16_t *res_bf16,
                                const uint32_t *res_bits, const float *aux, float *dx, uint16_t *dx_bf16, int flags,
                                void *ws, size_t ws_bytes, adaptseg_stream_t stream);
/* The BatchNorm backward reduction fused into the data gradient that produces the BN's incoming
   gradient (a Bottleneck's conv3 -> bn2 and conv2 -> bn1 data gradients, the next block's conv1
   data gradient -> bn3; model/deeplab_multi.py:83-103 under torch's batch_norm_backward): the
   epilogue also sums, per row tile and channel, g' and g' * (x - mean), where g' is the output
   value masked as the BN backward masks it.  adaptseg_bn_bwd_sums then skips its own reduction
   pass over dy and x.  Replaces the separate read of dy (and the reduction launch) per BN. */
typedef struct {
  const float *x;          /* the BN input [rows][c] (the conv output it normalised): fp32 ...  */
  const uint16_t *x_bf16;  /* ... or bf16 (bf16 activation storage): exactly one                 */
  const float *mean, *invstd;      /* the forward's saved statistics (16-byte aligned)        */
  const float *weight, *bias;      /* affine parameters (NULL: 1 / 0)                          */
  const uint32_t *bits;    /* mask 2: bitmap [rows][c / 32] (adaptseg_bn_fwd_*_xm relu_bits)      */
  int mask;                /* 0 none; 1 ReLU of the BN output, recomputed from x (bn_bwd's mask
                              from x); 2 the bitmap (bn_bwd_xg's dy_bits)                       */
  float *partial;          /* out: [2][c][ntiles] per-row-tile sums                             */
  size_t partial_bytes;
} adaptseg_bnsum_desc;
/* Row tiles the fused sums of product `d` come in (0: its plan cannot fuse them — thin /
   tap-GEMM / split-K / stride-2 / per-element products); with_copy as for bnstats_tiles_x
   (the plan with the caller's copy of dY).  Host-side planning, no GPU. */
int adaptseg_conv2d_bnsum_tiles(const adaptseg_conv_desc *d, int with_copy, int *ntiles);
/* adaptseg_conv2d_bwd_data_xg (no activation-gradient epilogue) that also writes the fused sums
   of `bs` when its final plan can (*ntiles = the row tiles written, else 0: the caller runs the
   BN backward's own reduction).  Tiles count rows of the output; every (channel, tile) is
   written exactly once. */
int adaptseg_conv2d_bwd_data_bnsum(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16,
                                   const float *const *w, const void *w_pack, const float *res,
                                   const uint16_t *res_bf16, const uint32_t *res_bits, float *dx, uint16_t *dx_bf16,
                                   int flags, const adaptseg_bnsum_desc *bs, int *ntiles, void *ws, size_t ws_bytes,
                                   adaptseg_stream_t stream);
/* Weight gradient with bf16 copies of BOTH operands (dY from adaptseg_bn_bwd_x, x from the
   forward's adaptseg_bn_*_x; either NULL = neither used): the LDS-DMA weight-gradient kernel
   (Cin and Cout multiples of 8) reads them; other kernels ignore them.  Exception: the
   tap-GEMM path of the multi-branch dilated classifier (model/deeplab_multi.py:112-121; its dY
   operand is a buffer it builds itself) uses x_bf16 alone, as adaptseg_conv2d_fwd_x does. */
int adaptseg_conv2d_bwd_weight_x(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16,
                                 const float *x, const uint16_t *x_bf16, float *const *dw,
                                 float *const *db, int flags, void *ws, size_t ws_bytes,
                                 adaptseg_stream_t stream);

/* dx[n,h,w,c] = conv_transpose(dy, w)  (NHWC, contiguous).  aux: LEAKY_/RELU_GRAD source. */
int adaptseg_conv2d_bwd_data(const adaptseg_conv_desc *d, const float *dy, const float *const *w,
                             const float *res, const float *aux, float *dx, int flags, void *ws,
                             size_t ws_bytes, adaptseg_stream_t stream);

/* dw[seg][k,kh,kw,c] (+)= sum_{n,oh,ow} dy * x_gathered; db[seg][k] (+)= sum dy.
   db may be NULL.  Only ADAPTSEG_EPI_ACCUMULATE and ADAPTSEG_WGRAD_DEFER_SUM are honoured. */
int adaptseg_conv2d_bwd_weight(const adaptseg_conv_desc *d, const float *dy, const float *x,
                               float *const *dw, float *const *db, int flags, void *ws,
                               size_t ws_bytes, adaptseg_stream_t stream);

/* Deferred split-K sums of weight gradients (round 6).  With ADAPTSEG_WGRAD_DEFER_SUM in
   `flags`, a weight gradient whose plan splits K writes its partial outputs into `ws` and
   returns with their sum into dw pending on `stream` (a call that also computes a bias gradient
   db sums immediately: its bias partials reuse the workspace);
   adaptseg_splitk_flush(stream) launches every pending sum of that stream on it, in the order
   the products were issued, and clears the list — bitwise the same dw as the immediate sum.
   Until the flush the caller keeps each deferred call's workspace alive and unshared (the
   partial outputs live there) and reads no deferred dw.  A product that does not split K
   writes dw in its GEMM as usual.  The PyTorch binding: ops.splitk_flush(); the engine's weight
   gradient stream flushes when it joins (engine.WgradStream, ADAPTSEG_DEFER_SPLITK).
   Replaces nothing in the reference (its weight gradients are cuDNN's, inside autograd). */
int adaptseg_splitk_flush(adaptseg_stream_t stream);
/* number of sums pending on `stream` */
int adaptseg_splitk_pending(adaptseg_stream_t stream, int *count);

/* ------------------------------------------------------------------------------------ */
/* BatchNorm2d, train mode (batch statistics) with fused residual add and ReLU.          */
/* Replaces nn.BatchNorm2d + ReLU + "out += residual" in model/deeplab_multi.py:65-101, */
/* 130-134, 160 (affine params frozen, eps 1e-5, momentum 0.1).                          */
/* ------------------------------------------------------------------------------------ */
int adaptseg_bn_workspace_size(int64_t rows, int c, size_t *bytes);

/* x,y: [rows][c].  Writes save_mean/save_invstd[c]; updates running stats (may be NULL).
   y = act((x-mean)*invstd*weight + bias (+ res)).  The `relu` argument of every BN entry point
   selects the activation: 0 none, 1 ReLU, 2 LeakyReLU(0.2) (the warper's DownConvolution,
   model/custom_layers.py:83-96). */
int adaptseg_bn_fwd_train(int64_t rows, int c, const float *x, const float *weight,
                          const float *bias, float *running_mean, float *running_var,
                          float momentum, float eps, float *save_mean, float *save_invstd,
                          const float *res, float *y, int relu, void *ws, size_t ws_bytes,
                          adaptseg_stream_t stream);

/* bn_fwd_train from row-tile statistics (adaptseg_conv2d_fwd_bnstats): a Chan merge of the
   tiles' (count, mean, M2) in fp64 replaces the statistics pass over x; then the same apply. */
int adaptseg_bn_fwd_train_tiles(int64_t rows, int c, const float *stats, int ntiles, const float *x,
                                const float *weight, const float *bias, float *running_mean,
                                float *running_var, float momentum, float eps, float *save_mean,
                                float *save_invstd, const float *res, float *y, int relu,
                                adaptseg_stream_t stream);

/* The forward BN passes with bf16 activation storage (conv math BF16 = config c5, autocast
   semantics: the convs store bf16, BatchNorm reads bf16 and normalises in fp32).  Activation
   operands are fp32 (x, res) or bf16 (x_bf16, res_bf16) — exactly one of x / x_bf16, and the
   residual stored like x.  Outputs: y (fp32) and / or y_bf16 (a bf16 RNE copy, contiguous
   [rows][c]), at least one. */
int adaptseg_bn_fwd_train_x(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *weight,
                            const float *bias, float *running_mean, float *running_var, float momentum, float eps,
                            float *save_mean, float *save_invstd, const float *res, const uint16_t *res_bf16,
                            float *y, uint16_t *y_bf16, int relu, void *ws, size_t ws_bytes,
                            adaptseg_stream_t stream);
/* The statistics half of adaptseg_bn_fwd_train_tiles alone (batch mean / invstd from the
   producing conv's row tiles, running statistics updated): for a BN whose apply is folded into
   its consumer conv (adaptseg_operand_bn), so y is never written. */
int adaptseg_bn_fwd_train_tiles_stats(int64_t rows, int c, const float *stats, int ntiles, float *running_mean,
                                      float *running_var, float momentum, float eps, float *save_mean,
                                      float *save_invstd, adaptseg_stream_t stream);
int adaptseg_bn_fwd_train_tiles_x(int64_t rows, int c, const float *stats, int ntiles, const float *x,
                                  const uint16_t *x_bf16, const float *weight, const float *bias,
                                  float *running_mean, float *running_var, float momentum, float eps,
                                  float *save_mean, float *save_invstd, const float *res, const uint16_t *res_bf16,
                                  float *y, uint16_t *y_bf16, int relu, adaptseg_stream_t stream);
int adaptseg_bn_fwd_infer_x(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *weight,
                            const float *bias, const float *running_mean, const float *running_var, float eps,
                            const float *res, const uint16_t *res_bf16, float *y, uint16_t *y_bf16, int relu,
                            adaptseg_stream_t stream);
/* The _x forward passes that also write the ReLU mask bitmap of y (relu_bits, [rows][c / 32]
   uint32, c % 32 == 0; bit c % 32 of word (row, c / 32) = y > 0): the backward then reads 1 bit
   per element instead of the stored y (adaptseg_bn_bwd_xg dy_bits, adaptseg_conv2d_bwd_data_xg
   res_bits). */
int adaptseg_bn_fwd_train_xm(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *weight,
                             const float *bias, float *running_mean, float *running_var, float momentum, float eps,
                             float *save_mean, float *save_invstd, const float *res, const uint16_t *res_bf16,
                             float *y, uint16_t *y_bf16, uint32_t *relu_bits, int relu, void *ws, size_t ws_bytes,
                             adaptseg_stream_t stream);
int adaptseg_bn_fwd_train_tiles_xm(int64_t rows, int c, const float *stats, int ntiles, const float *x,
                                   const uint16_t *x_bf16, const float *weight, const float *bias,
                                   float *running_mean, float *running_var, float momentum, float eps,
                                   float *save_mean, float *save_invstd, const float *res, const uint16_t *res_bf16,
                                   float *y, uint16_t *y_bf16, uint32_t *relu_bits, int relu, adaptseg_stream_t stream);
int adaptseg_bn_fwd_infer_xm(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *weight,
                             const float *bias, const float *running_mean, const float *running_var, float eps,
                             const float *res, const uint16_t *res_bf16, float *y, uint16_t *y_bf16,
                             uint32_t *relu_bits, int relu, adaptseg_stream_t stream);

/* Eval-mode BN (running statistics): y = (x-rm)/sqrt(rv+eps)*w + b (+res), ReLU if relu. */
int adaptseg_bn_fwd_infer(int64_t rows, int c, const float *x, const float *weight,
                          const float *bias, const float *running_mean, const float *running_var,
                          float eps, const float *res, float *y, int relu,
                          adaptseg_stream_t stream);

/* Backward of bn_fwd_train.  g = dy * act'(y) (relu: 0 none, 1 ReLU, 2 LeakyReLU(0.2)).
   dx = weight*invstd*(g - mean(g) - xhat*mean(g*xhat)); dres = g if dres != NULL.
   y == NULL with relu (train mode, BN without residual): the mask is recomputed from x as
   (x-mean)*invstd*weight + bias > 0 — one tensor read less in both passes.
   If train == 0 the eval-mode backward dx = g*weight*invstd is computed. */
int adaptseg_bn_bwd(int64_t rows, int c, const float *dy, const float *y, const float *x,
                    const float *weight, const float *bias, const float *save_mean,
                    const float *save_invstd, float *dx, float *dres, int relu, int train,
                    void *ws, size_t ws_bytes, adaptseg_stream_t stream);

/* adaptseg_bn_bwd with bf16 activation storage and an optional bf16 (RNE) copy of dx
   (dx_bf16, NULL = none: the data-gradient operand of the conv that produced x, under bf16
   conv math; dx may be NULL when dx_bf16 is given).  The saved activations x and y are both
   fp32 or both bf16 (y_bf16 / x_bf16); the gradients dy, dres stay fp32. */
int adaptseg_bn_bwd_x(int64_t rows, int c, const float *dy, const float *y, const uint16_t *y_bf16, const float *x,
                      const uint16_t *x_bf16, const float *weight, const float *bias, const float *save_mean,
                      const float *save_invstd, float *dx, uint16_t *dx_bf16, float *dres, int relu, int train,
                      void *ws, size_t ws_bytes, adaptseg_stream_t stream);

/* adaptseg_bn_bwd_x with bf16 GRADIENT storage (BF16 conv maths with bf16 activation storage,
   config c5): the incoming gradient is dy (fp32) or dy_bf16 (exactly one), and the residual
   gradient dres is written like it (dres / dres_bf16; it may alias dy of the same storage).  dx
   is fp32 and / or its bf16 copy, as in adaptseg_bn_bwd_x (for bf16 storage: dx_bf16 only).
   dy_bits (any maths; C % 32 == 0; NULL = none): a mask bitmap [rows][c / 32] applied to dy
   first, g = dy * bit (then the `relu` mask as usual) — the Bottleneck's BN3 backward with its
   ReLU mask from the forward's bitmap (relu = 0), and the downsample BN's, whose incoming
   gradient is that same masked g. */
int adaptseg_bn_bwd_xg(int64_t rows, int c, const float *dy, const uint16_t *dy_bf16, const uint32_t *dy_bits,
                       const float *y, const uint16_t *y_bf16, const float *x, const uint16_t *x_bf16,
                       const float *weight, const float *bias, const float *save_mean, const float *save_invstd,
                       float *dx, uint16_t *dx_bf16, float *dres, uint16_t *dres_bf16, int relu, int train, void *ws,
                       size_t ws_bytes, adaptseg_stream_t stream);

/* adaptseg_bn_bwd_xg in train mode with the reduction already done: `partial` [2][c][ntiles]
   from adaptseg_conv2d_bwd_data_bnsum over this dy (same mask: relu with y == NULL <-> bnsum
   mask 1, dy_bits <-> mask 2).  Runs the finalisation and the apply pass only. */
int adaptseg_bn_bwd_sums(int64_t rows, int c, const float *dy, const uint16_t *dy_bf16, const uint32_t *dy_bits,
                         const float *y, const uint16_t *y_bf16, const float *x, const uint16_t *x_bf16,
                         const float *weight, const float *bias, const float *save_mean, const float *save_invstd,
                         float *dx, uint16_t *dx_bf16, float *dres, uint16_t *dres_bf16, int relu,
                         const float *partial, int ntiles, void *ws, size_t ws_bytes, adaptseg_stream_t stream);

/* adaptseg_bn_bwd in train mode for a BN whose affine parameters are trainable (the warper's
   NaiveConvolution norms, model/custom_layers.py:25-33): additionally dbias[c] += sum(g),
   dweight[c] += sum(g * xhat) (accumulated, as torch's AccumulateGrad; either may be NULL).
   act: 0 none, 1 ReLU, 2 LeakyReLU(0.2); its mask comes from y, or from x when y == NULL. */
int adaptseg_bn_bwd_affine(int64_t rows, int c, const float *dy, const float *y, const float *x,
                           const float *weight, const float *bias, const float *save_mean,
                           const float *save_invstd, float *dx, float *dres, int act, float *dweight,
                           float *dbias, void *ws, size_t ws_bytes, adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* Evaluation: evaluate_cityscapes.py:153-169 (interp to 1024x2048 + argmax) and          */
/* compute_iou.py:15-28 (label_mapping + fast_hist).                                      */
/* ------------------------------------------------------------------------------------ */
/* out[n][oh][ow] = argmax_c bilinear_align_corners(x)[n][oh][ow][c]; x NHWC [n][h][w][c]. */
int adaptseg_upsample_argmax(int n, int c, int h, int w, int oh, int ow, const float *x,
                             uint8_t *out, adaptseg_stream_t stream);
/* hist[a][b] += #pixels with a = lut[gt] (or gt if lut == NULL) in [0, ncls), b = pred;
   hist is int64 [ncls][ncls] (accumulated, never cleared). */
int adaptseg_confusion_hist(int64_t npix, const uint8_t *gt, const int32_t *lut,
                            const uint8_t *pred, int ncls, int64_t *hist, adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* Input pipeline: GTA5DataSet.__getitem__ after file decode (dataset/gta5_dataset.py:47-71) */
/* and the target loader's image path (train_gta2cityscapes_multi.py:333-336, 520-523).    */
/* Bit-exact with Pillow's Image.resize(crop, BICUBIC) / (crop, NEAREST) 8-bit resampler.   */
/* ------------------------------------------------------------------------------------ */
int adaptseg_preprocess_workspace_size(int n, int in_h, int in_w, int out_h, int out_w, size_t *bytes);
/* rgb: [n][in_h][in_w][3] uint8 (decoded RGB).  image: [n][3][out_h][out_w] float32 =
   BGR(resize_bicubic(rgb)) - (mean_b, mean_g, mean_r) in float32 (image -= IMG_MEAN).
   label_ids (optional, with labels): [n][in_h][in_w] uint8 class ids -> labels [n][out_h][out_w]
   int64 = lut[resize_nearest(ids)] (lut: int32[256] id -> trainId; NULL keeps the ids). */
int adaptseg_gta5_preprocess(int n, int in_h, int in_w, int out_h, int out_w, const uint8_t *rgb, float mean_b,
                             float mean_g, float mean_r, float *image, const uint8_t *label_ids, const int32_t *lut,
                             int64_t *labels, void *ws, size_t ws_bytes, adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* MaxPool2d (model/deeplab_multi.py:135: kernel 3, stride 2, pad 1, floor mode), NHWC.  */
/* ------------------------------------------------------------------------------------ */
int adaptseg_maxpool2d_fwd(int n, int c, int h, int w, int oh, int ow, int k, int s, int p,
                           const float *x, float *y, uint8_t *argmax, adaptseg_stream_t stream);
int adaptseg_maxpool2d_bwd(int n, int c, int h, int w, int oh, int ow, int k, int s, int p,
                           const float *dy, const uint8_t *argmax, float *dx,
                           adaptseg_stream_t stream);
/* The same with the output's F32X3 term images (the _x operand copies of the conv consuming it,
   [..., 3, C] pixel-interleaved; NULL = none): the pooled activation for the next conv's
   products (DeeplabVGG's 2x2 pools, model/deeplab_vgg.py: pool -> conv), the routed gradient for
   the pooled conv's weight / data gradients.  Terms need C % 4 == 0 and 16-B aligned fp32
   tensors (8-B aligned term images), else ADAPTSEG_ERR_ARG. */
int adaptseg_maxpool2d_fwd_x(int n, int c, int h, int w, int oh, int ow, int k, int s, int p,
                             const float *x, float *y, uint8_t *argmax, uint16_t *y_terms,
                             adaptseg_stream_t stream);
int adaptseg_maxpool2d_bwd_x(int n, int c, int h, int w, int oh, int ow, int k, int s, int p,
                             const float *dy, const uint8_t *argmax, float *dx, uint16_t *dx_terms,
                             adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* nn.Upsample(mode='bilinear', align_corners=True), NHWC (model/deeplab_multi.py:188). */
/* The backward is a deterministic two-pass gather (no atomics).                         */
/* ------------------------------------------------------------------------------------ */
int adaptseg_upsample_workspace_size(int n, int c, int h, int w, int oh, int ow, size_t *bytes);
int adaptseg_upsample_bilinear_fwd(int n, int c, int h, int w, int oh, int ow, const float *x,
                                   float *y, adaptseg_stream_t stream);
int adaptseg_upsample_bilinear_bwd(int n, int c, int h, int w, int oh, int ow, const float *dy,
                                   float *dx, int flags, void *ws, size_t ws_bytes,
                                   adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* Channel softmax (F.softmax(pred), train_gta2cityscapes_multi.py:423,617-618), NHWC.   */
/* ------------------------------------------------------------------------------------ */
int adaptseg_softmax_fwd(int64_t rows, int c, const float *x, float *y, adaptseg_stream_t stream);
int adaptseg_softmax_bwd(int64_t rows, int c, const float *y, const float *dy, float *dx,
                         int flags, adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* Cross entropy over channels with ignore label (utils/loss.py:14-36 CrossEntropy2d;    */
/* nn.CrossEntropyLoss(ignore_index=255), train_gta2cityscapes_multi.py:359,546).        */
/* logits [rows][c], labels int64 [rows].  A label < 0 or == ignore is skipped.           */
/* class_weight may be NULL.  out[0] = loss, out[1] = denominator (valid count or         */
/* summed class weight).  All-ignored input gives NaN, as the reference does.            */
/* ------------------------------------------------------------------------------------ */
int adaptseg_ce_workspace_size(int64_t rows, size_t *bytes);
int adaptseg_softmax_ce_fwd(int64_t rows, int c, const float *logits, const int64_t *labels,
                            int ignore, const float *class_weight, float *out, void *ws,
                            size_t ws_bytes, adaptseg_stream_t stream);
/* dlogits = grad_loss[0] / out[1] * w[label] * (softmax - onehot); grad_loss, out on device */
int adaptseg_softmax_ce_bwd(int64_t rows, int c, const float *logits, const int64_t *labels,
                            int ignore, const float *class_weight, const float *out,
                            const float *grad_loss, float *dlogits, int flags,
                            adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* Adversarial losses against a constant target (train_gta2cityscapes_multi.py:542-545, */
/* 620-624, 648-650, 668-670): kind 0 = BCEWithLogitsLoss, 1 = MSELoss, mean reduction.  */
/* ------------------------------------------------------------------------------------ */
int adaptseg_adv_workspace_size(int64_t n, size_t *bytes);
int adaptseg_adv_loss_fwd(int64_t n, const float *x, float target, int kind, float *loss,
                          void *ws, size_t ws_bytes, adaptseg_stream_t stream);
int adaptseg_adv_loss_bwd(int64_t n, const float *x, float target, int kind,
                          const float *grad_loss, float *dx, int flags, adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* Optimisers over flat fp32 arenas (train_gta2cityscapes_multi.py:532-540).             */
/* ------------------------------------------------------------------------------------ */
/* torch.optim.SGD(momentum, weight_decay, dampening 0, nesterov False) applied `multiplicity`
   times in sequence, as torch does for a parameter listed that many times in its group
   (the reference's get_1x_lr_params_NOscale yields block weights 3x and downsample weights
   4x, model/deeplab_multi.py:216-222).  first_step != 0: no momentum buffer exists yet, so
   every repetition starts from a fresh copy of its own d_p (torch's clone path).
   grad is multiplied by grad_scale first (1/world for data-parallel averaging). */
int adaptseg_sgd_step(int64_t n, float *param, const float *grad, float *mom, float lr,
                      float momentum, float weight_decay, float grad_scale, int multiplicity,
                      int first_step, adaptseg_stream_t stream);
/* torch.optim.Adam(betas, eps, weight_decay 0, amsgrad False); step counts from 1. */
int adaptseg_adam_step(int64_t n, float *param, const float *grad, float *exp_avg,
                       float *exp_avg_sq, float lr, float beta1, float beta2, float eps,
                       int step, float grad_scale, adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* The fork's Warper: model/warper.py:216-267, its decoder blocks  */
/* model/custom_layers.py:117-188 and the prediction warp model/deeplab_multi.py:238-255.  */
/* ------------------------------------------------------------------------------------ */
/* out[n][2h][2w][cs+cd] = Upsample(x2, bilinear, align_corners=False)(ReLU(cat(s, d), dim=C)):
   one decoder block's input (SkipConnectionDecode.forward, model/warper.py:130-144, then
   UpConvolution's ReLU(inplace) + nn.Upsample).  s [n][h][w][cs] may be NULL with cs = 0 (the
   DecoderInput / DecoderOutput blocks); d [n][h][w][cd].  cs, cd multiples of 4. */
int adaptseg_up2_relu_cat_fwd(int n, int h, int w, int cs, int cd, const float *s, const float *d,
                              float *out, adaptseg_stream_t stream);
/* Adjoint: ds = dS * (s > 0), dd = dD * (d > 0) where (dS, dD) = the channel split of
   Upsample^T(dout); written (not accumulated), fixed summation order. */
int adaptseg_up2_relu_cat_bwd(int n, int h, int w, int cs, int cd, const float *s, const float *d,
                              const float *dout, float *ds, float *dd, adaptseg_stream_t stream);
/* ResNetMulti.warp: grid = clamp(tanh(flow[..., last channel pair]) + meshgrid(linspace(-1, 1,
   w), linspace(-1, 1, h)), -1, 1); y = grid_sample(x, grid) (bilinear, zeros padding,
   align_corners=False).  x, y NHWC [n][h][w][c] (c <= 256); flow NHWC [n][h][w][fc] (fc even).  Two
   inputs share one grid (the two heads, deeplab_multi.py:190-192); x1/y1 may be NULL. */
int adaptseg_grid_warp_fwd(int n, int c, int h, int w, int fc, const float *flow, const float *x1,
                           const float *x2, float *y1, float *y2, adaptseg_stream_t stream);
int adaptseg_grid_warp_bwd_workspace_size(int n, int c, int h, int w, size_t *bytes);
/* dflow (written; [n][h][w][fc], zero outside the last pair) = the warp field's gradient summed
   over both heads (needs x1/x2 for every given dy; c <= 256); dx1/dx2 (written, optional) = the input
   gradients.  The input gradient is a data-dependent scatter: it accumulates in 64-bit fixed
   point (integer atomics, so the result is independent of scheduling), with the scale chosen
   per call from max|dy| so no sum can overflow; rounding <= 2^-42 * max|dy| at 1024x2048. */
int adaptseg_grid_warp_bwd(int n, int c, int h, int w, int fc, const float *flow, const float *x1,
                           const float *x2, const float *dy1, const float *dy2, float *dflow,
                           float *dx1, float *dx2, void *ws, size_t ws_bytes,
                           adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* Plumbing kernels.                                                                      */
/* ------------------------------------------------------------------------------------ */
int adaptseg_zero(void *ptr, size_t bytes, adaptseg_stream_t stream);
/* dst[n][h][w][c] = src(n, c, h, w) read through arbitrary element strides. */
int adaptseg_to_nhwc(int n, int c, int h, int w, const int64_t *src_stride, const float *src,
                     float *dst, adaptseg_stream_t stream);
/* to_nhwc with channel padding (c_dst >= c: channels c..c_dst-1 written as 0) and, with
   ADAPTSEG_EPI_ACCUMULATE, dst += instead of dst =.  Pads a thin conv's input / weight to a
   vector-friendly channel count (the stem's Cin 3 -> 4, D.conv1's Cin 19 -> 32) and folds a
   padded weight gradient back into the unpadded one (src = its first c channels).  Stands in
   for no reference call: the reference convs take the unpadded tensors directly. */
int adaptseg_to_nhwc_pad(int n, int c, int h, int w, const int64_t *src_stride, const float *src, int c_dst,
                         float *dst, int flags, adaptseg_stream_t stream);
/* dst[i] += src[i] (or dst = src when flags lacks ADAPTSEG_EPI_ACCUMULATE). */
int adaptseg_axpy(int64_t n, float alpha, const float *src, float *dst, int flags,
                  adaptseg_stream_t stream);

/* p[i] += v for i < n (BatchNorm num_batches_tracked counters, kept in one arena). */
int adaptseg_add_i64(int64_t *p, int64_t n, int64_t v, adaptseg_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* Live kernel timing for the benchmark: when enabled, every launch of the selected          */
/* implicit-GEMM conv kernel symbol is launched through hipExtLaunchKernel with an event     */
/* pair, which records the kernel's own execution (start to end, as rocprofv3 reports it,   */
/* not the stream time it spent queued behind other streams' work); the summed durations    */
/* and summed algorithmic FLOPs (2*N*OH*OW*K*C*KH*KW*nseg per launch) are read              */
/* back after a device synchronise.  selector = -1: every igemm launch; otherwise           */
/* selector = 100*op + 10*tile + variant names ONE kernel symbol: op 0 fwd, 1 bwd-data,     */
/* 2 bwd-weight; tile 0 = 128x128, 1 = 256x32, 2 = 32x256, 3 = 64x256, 4 = 256x64;          */
/* variant 0..3 = generic gather (2*vecA + vecB), 4 = FAST, 5 = FAST stride-2 parity path;    */
/* tile 9 = the bf16-MFMA kernels: variant 0 / 1 bf16 operands (stride-2 parity path),      */
/* 2 / 3 the same on the 128x256 tile, 5 / 6 the F32X3 kernel (3-term bf16 splits).          */
/* ------------------------------------------------------------------------------------ */
int adaptseg_timing_enable(int enable, int selector);
int adaptseg_timing_read(double *total_ms, double *total_flops, int64_t *launches);
/* Create `pairs` event pairs now, so a timed region records into existing events (creating one
   inside it costs milliseconds). */
int adaptseg_timing_reserve(int64_t pairs);
/* HBM-bound kernels (the interp / loss / BN passes): when enabled, every launch of upsample
   fwd (id 1000) / bwd (1001), softmax fwd (1002) / bwd (1003), cross-entropy fwd (1004) / bwd
   (1005), BN apply (1006) / backward apply (1007), the warper's up2_relu_cat fwd (1008) / bwd
   (1009), grid warp fwd (1010) / field gradient (1011) / input-gradient scatter (1012, all of its
   passes), BN statistics reduce (1013) / backward-sums reduce (1014) and the conv split-K
   reduce (1015) is bracketed the same way with its
   ALGORITHMIC bytes (compulsory reads + writes at the op interface) as units. */
int adaptseg_timing_enable_mem(int enable);
int adaptseg_timing_read_id(int kernel_id, double *total_ms, double *total_units, int64_t *launches);
/* Conv GEMMs: also bracket each timed launch with stream events (the time from the launch's
   position in its stream to its end, which includes waiting for CU slots beside other streams'
   work); read per kernel id with adaptseg_timing_read_id_stream. */
int adaptseg_timing_enable_stream(int enable);
int adaptseg_timing_read_id_stream(int kernel_id, double *total_ms, int64_t *launches);

/* A stream restricted to a subset of the device's compute units (hipExtStreamCreateWithCUMask):
   CU i is enabled when i % d < k (a stride pattern, so every XCD keeps k / d of its CUs whatever
   the logical CU numbering).  For the engine's weight-gradient stream (ADAPTSEG_WGRAD_CU_MASK):
   its GEMM blocks then occupy only those CUs, and the main chain's one-block-per-CU tiles keep
   the rest.  The stream lives until adaptseg_stream_destroy. */
int adaptseg_stream_create_cu_mask(int k, int d, adaptseg_stream_t *stream);
int adaptseg_stream_destroy(adaptseg_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* ADAPTSEG_H */
