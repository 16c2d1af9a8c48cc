/* libhgk — MI355X (gfx950) stacked-hourglass kernels behind a plain C ABI.
 *
 * Drop-in boundary for the reference's training hot path: the arithmetic of
 * ResidualBlock / hourglass / lin / creatModel.forward (+ autograd backward) and the per-stack
 * nn.MSELoss of /root/reference/try_with_torch.py:179-298,305-343. The reference has no FFI of
 * its own (it is pure PyTorch); each entry point below names the reference operator it replaces.
 *
 * Conventions
 *  - Activations are NHWC, element type `dtype` (HGK_F32 or HGK_BF16); BN statistics, BN
 *    parameters, biases and every gradient of a parameter are fp32.
 *  - All pointers are device pointers owned by the caller (PyTorch caching allocator); the library
 *    never allocates, frees or retains a pointer past return. Workspaces are passed in.
 *  - Every launch goes to the caller's `stream` (a hipStream_t), with no implicit synchronisation,
 *    so a caller may capture any sequence of calls into a hipGraph.
 *  - Return 0 on success, a negative HGK_ERR_* code otherwise; hgk_last_error() then holds a
 *    thread-local message. No C++ exception crosses the ABI. Deterministic: no float atomics;
 *    every cross-workgroup sum is a fixed-order reduction of per-workgroup partial slabs.
 *  - "stats partials": a CHANNEL-major float buffer [C][3][rows] (rows = the count the producing
 *    call reports) of per-workgroup (sum, M2 = sum of squared
 *    deviations from the workgroup's own mean, count) of a tensor's channels — merged in fp64 with
 *    Chan's rule, so a BatchNorm over very few values (1x1 innermost level) keeps full precision;
 *    the producing call reports `rows` through *rows_out (host int).
 */
#ifndef HGK_H_
#define HGK_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HGK_ABI_VERSION 39

enum { HGK_F32 = 0, HGK_BF16 = 1 };
enum { HGK_OK = 0, HGK_ERR_ARG = -1, HGK_ERR_UNSUPPORTED = -2, HGK_ERR_HIP = -3 };
enum { HGK_UP_BILINEAR_AC = 0, HGK_UP_NEAREST = 1 };

typedef void* hgk_stream_t; /* hipStream_t */

int hgk_abi_version(void);
const char* hgk_last_error(void);

/* Kernel routing. Every routing decision is a compiled-in default; nothing is read from the
 * environment. An A/B experiment or a test that needs another route sets it explicitly here
 * (process-wide, takes effect at the next call; not thread-safe against concurrent launches).
 *   HGK_ROUTE_RING_NW       4 (default): two 4-wave ring workgroups per CU where Cout <= 128;
 *                           8: one 8-wave workgroup everywhere
 *   HGK_ROUTE_RING_MINM     rows from which a 1x1 launch takes the ring kernel (16384: the 32x32
 *                           level too — at N = 32 +0.6 % img/s over 65536, at the N = 16 of
 *                           try_with_aspp +1.7 % over 32768); 0 = off
 *   HGK_ROUTE_RING_SMALL    1 (default): the 4-wave ring for the 32x32 / 16+8 launches; 0 = off
 *   HGK_ROUTE_ROW3          row-streaming 3x3: 0 off, 1 every supported launch, 2 (default)
 *                           launches whose first segment is 64 wide, 3 single 64-wide only
 *   HGK_ROUTE_SPLITK_FIXUP  1 (default): split-K sums inside the conv launch; 0 = epilogue kernel
 *   HGK_ROUTE_IMG           image-tile kernel (1x1 / 3x3 of the small levels, whole images or
 *                           row strips of 64 pixels per workgroup) for launches of at most this
 *                           many output pixels per segment (8192: 16x16 at N = 32); 0 = off
 *   HGK_ROUTE_WG_FULL       1x1 bf16 weight gradients (128x256 / 256x128 weights) with the whole
 *                           weight in one workgroup tile (dy and x read once per use instead of
 *                           once per k- / co-tile) for launches of at least this many pixels;
 *                           0 = off
 *   HGK_ROUTE_WG_DMA        3x3 halo weight gradients with LDS-DMA staging (dy and the raw input
 *                           halo DMA'd, the BN+ReLU transform in place; bitwise the register-staged
 *                           kernel): 1 on, 0 = off
 *   HGK_ROUTE_WG_BATCH_TARGET  hgk_conv_wgrad_accum_batch: workgroups one batched launch aims for
 *                           over all its jobs (few pixel splits per weight, small fp32 slabs);
 *                           0 = every job planned alone
 *   HGK_ROUTE_ROW3_ALT      row-streaming 3x3: odd workgroups take their rows bottom-up (shared
 *                           boundary rows hit L2: fewer HBM bytes, bitwise); 1 on, 0 = off
 *   HGK_ROUTE_HALO_BN64     3x3 halo launches with 64-channel output tiles (twice the
 *                           workgroups): 16x16 level with one 4-wave group (1) or two k-groups
 *                           (2: outputs bitwise the 128-channel tiles'), + 4 (default 6): also
 *                           the 8-row-tile launches of <= 128 workgroups (32x32 at N <= 16); 0 off
 *   HGK_ROUTE_WG_BATCH_SLAB_X10  hgk_conv_wgrad_accum_batch's split plan: a job's fp32 partial
 *                           slabs capped at this / 10 x the bytes of dy + input it reads
 *                           (default 5; every other weight gradient: 2x)
 *   HGK_ROUTE_STEM          1 (default): the 7x7 / stride-2 stem over the channel-padded input
 *                           (8 stored channels, 64 outputs, 128-pixel output rows) takes the
 *                           row-tile stem kernel; 0 = the implicit GEMM's SMALLC path
 *   HGK_ROUTE_IMG_NARROW    image-tile 1x1 launches of at most this many rows (both segments of
 *                           a twin) take 32-channel output tiles; 0 (default) = 64 everywhere
 *   HGK_ROUTE_WG_RING       multi-use 1x1 bf16 weight gradients (128x256 / 256x128 / 256x256
 *                           weights, every use's pixels a multiple of 32) of at least this many
 *                           pixels in total take the LDS-DMA ring kernel (hgk_wgrad_ring.hip: the
 *                           whole K per workgroup, 3-4 blocks of dy / x in flight per CU);
 *                           default 65536 (+0.8 % img/s same-box, profiles/r06_wg_ring_ab.txt); 0 = off
 *   HGK_ROUTE_WG_HALO_MULTI multi-use bf16 3x3 weight gradients: the uses of H % 8 == 0 and
 *                           W % 16 == 0, when they hold at least this many 8x16-pixel tiles in
 *                           total, go to ONE halo launch whose splits run over the concatenated
 *                           tiles (each slab read-modified-written once per launch, not per use;
 *                           the other uses take the implicit GEMM multi launch); default 128; 0 = off
 * hgk_set_route returns the previous value (HGK_ERR_ARG for an unknown knob); a negative value
 * restores the default. */
enum {
  HGK_ROUTE_RING_NW = 0,
  HGK_ROUTE_RING_MINM = 1,
  HGK_ROUTE_RING_SMALL = 2,
  HGK_ROUTE_ROW3 = 3,
  HGK_ROUTE_SPLITK_FIXUP = 4,
  HGK_ROUTE_IMG = 5,
  HGK_ROUTE_WG_FULL = 6,
  HGK_ROUTE_WG_DMA = 7,
  HGK_ROUTE_WG_BATCH_TARGET = 8,
  HGK_ROUTE_ROW3_ALT = 9,
  HGK_ROUTE_HALO_BN64 = 10,
  HGK_ROUTE_WG_BATCH_SLAB_X10 = 11,
  HGK_ROUTE_STEM = 12,
  HGK_ROUTE_IMG_NARROW = 13,
  HGK_ROUTE_WG_RING = 14,
  HGK_ROUTE_WG_HALO_MULTI = 15,
  HGK_ROUTE_COUNT = 16
};
long hgk_set_route(int knob, long value);
long hgk_get_route(int knob);
/* kernel family a forward convolution (twin when N1 > 0) of this geometry takes under the current
 * routes, without launching anything (tests, tooling): HGK_KFAM_* below, negative on bad args */
enum {
  HGK_KFAM_IMPLICIT = 0, /* implicit GEMM (tiled / all-ahead / split-K) */
  HGK_KFAM_SMALLC = 1,   /* channel-padded RGB stem */
  HGK_KFAM_HALO = 2,     /* 3x3 halo tiles */
  HGK_KFAM_RING = 3,     /* LDS-DMA ring 1x1 */
  HGK_KFAM_ROW3 = 4,     /* row-streaming 3x3 */
  HGK_KFAM_IMG = 5,      /* image-tile kernel of the small levels */
  HGK_KFAM_SPLIT = 6,    /* twin: the two segments launch separately */
  HGK_KFAM_STEM = 7      /* row-tile 7x7 / stride-2 stem kernel */
};
int hgk_conv_fwd_kernel_family(int dtype, int N0, int H0, int W0, int N1, int H1, int W1, int Cin,
                               int Cout, int KH, int KW, int stride, int pad, int dil);
/* upper bound of the `rows` any stats-producing call below reports (size partial buffers by it) */
int hgk_max_stats_rows(void);

/* ---- convolution (replaces nn.Conv2d forward, try_with_torch.py:186,189,192,193,248,262,271-273)
 * y[N,Ho,Wo,Cout] = conv(pre(x), w) + bias[Cout] (+ res) (then ReLU if post_relu), NHWC.
 * pre(x)[..c] = relu?(x*pre_scale[c] + pre_shift[c]) on in-bounds taps (the conv's zero padding is
 * applied AFTER the transform, as in BN->ReLU->Conv); pre_scale == NULL -> identity.
 * This fuses the BatchNorm-apply + ReLU in front of every bottleneck conv (:196-205).
 * w: packed by hgk_pack_conv_weight, row stride w_ld (>= KH*KW*Cin, multiple of 64).
 * res may alias y (in-place accumulate: y += conv(...)); bias may be NULL.
 * stats (nullable): partials of the stored y for a following BatchNorm.
 * workspace (nullable): >= hgk_conv_fwd_workspace() bytes enables split-K for small-M launches
 * (the 8x8 / 4x4 hourglass levels), reduced in a fixed split order by the last-arriving split of
 * each tile inside the same launch. Its first 4096 bytes are tile counters: they must be zero
 * when a workspace is first used, and every call leaves them zero (allocate it zeroed once). */
int hgk_conv_fwd(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                 const float* bias, const void* res, void* y, const float* pre_scale,
                 const float* pre_shift, int pre_relu, int post_relu, float* stats, int* rows_out,
                 int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                 int dil, void* workspace, size_t ws_bytes);
/* hgk_conv_fwd (no bias / pre-transform / statistics) that is the input gradient dA of a
 * BatchNorm(+ReLU) output, with that BN's backward reduction fused into its epilogue: writes
 * bn_partial [*bn_rows][2][Cout] = (sum g, sum g*xhat) per tile, g = dA * [relu(bn_y*scale+shift)
 * > 0], xhat = (bn_y - mean) * invstd — exactly what hgk_bn_bwd_reduce produces, so the result
 * feeds hgk_bn_bwd_finalize unchanged. bn_y is the BN input ([M][Cout], same layout as y). */
int hgk_conv_fwd_bnbwd(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                       const void* res, void* y, int N, int H, int W, int Cin, int Cout, int KH,
                       int KW, int stride, int pad, int dil, void* workspace, size_t ws_bytes,
                       const void* bn_y, const float* bn_scale, const float* bn_shift, int bn_relu,
                       const float* bn_mean, const float* bn_invstd, float* bn_partial,
                       int* bn_rows);
/* The train-mode BatchNorm(+ReLU) backward APPLY of this conv's input, folded into its operand
 * staging (the conv is the input gradient of a conv whose output fed that BN, e.g. conv1's input
 * gradient in front of bn2, try_with_torch.py:186-188): x = the BN's upstream gradient dA; the conv
 * consumes dy = hgk_bn_bwd_apply(dA, y, scale, shift, relu, coef) (same bits) and also writes dy
 * to `out` [M][C] for the weight gradient. Replaces hgk_bn_bwd_apply + a read of its output. */
typedef struct hgk_bn_vgrad {
  const void* y;       /* BN input [M][C] */
  const float* scale;  /* forward BN scale / shift: the ReLU mask y*scale+shift > 0 */
  const float* shift;
  const float* coef;   /* [4][C] from hgk_bn_bwd_finalize (or rows 0-3 of a twin segment's);
                          ignored when `partial` is set */
  int relu;
  void* out;           /* dy [M][C], written */
  /* ABI 27 — the BN-backward FINALIZE folded too (replaces hgk_bn_bwd_finalize_apply at the small
   * hourglass levels, try_with_torch.py:186-192): when partial != NULL every workgroup computes
   * the coefficients from the BN-backward partial rows [rows][2][C] (what the producing
   * input-gradient conv's epilogue wrote) with hgk_bn_bwd_finalize_apply's arithmetic, and one
   * workgroup accumulates dgamma / dbeta (nullable). A twin launch accumulates segment 0's sums
   * then segment 1's, as two single launches in that order would. Image-tile route only
   * (hgk_conv_vgrad_fin_ok). */
  const float* partial;
  int rows;
  long M;              /* values per channel of the BN */
  const float* mean;   /* forward batch mean / invstd [C] */
  const float* invstd;
  int training;
  float* dgamma;
  float* dbeta;
  /* ABI 28 (with `partial`): nullable gradient already accumulated for the BN's input (a
   * ResidualBlock's skip gradient in front of bn1, try_with_torch.py:183-185,207): dy = apply + add,
   * as hgk_bn_bwd_finalize_apply's `add` (`out` must not alias it). 256-channel 1x1 only. */
  const void* add;
} hgk_bn_vgrad;
/* hgk_conv_fwd_bnbwd with the folded apply of its input (bf16; shapes with
 * hgk_conv_vgrad_ok() only, else HGK_ERR_UNSUPPORTED and nothing is launched) */
int hgk_conv_fwd_bnbwd_vg(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                          const void* res, void* y, int N, int H, int W, int Cin, int Cout, int KH,
                          int KW, int stride, int pad, int dil, void* workspace, size_t ws_bytes,
                          const void* bn_y, const float* bn_scale, const float* bn_shift,
                          int bn_relu, const float* bn_mean, const float* bn_invstd,
                          float* bn_partial, int* bn_rows, const hgk_bn_vgrad* vg);
/* A train-mode BatchNorm FINALIZE folded into the consuming conv (the conv's input is
 * relu?(bn(x)), try_with_torch.py:196-205, at the small hourglass levels): every workgroup
 * computes the BN's scale / shift from the producer's channel-major statistics partials
 * [C][3][rows] (what hgk_bn_finalize_deferred reads), mean = sum S / M and
 * M2 = sum (M2_r + n_r (S_r / n_r - mean)^2) in fp64; the first workgroup writes stat [4][C]
 * (mean | invstd | scale | shift) and rec [2][C] (fp64 mean | unbiased variance, for
 * hgk_bn_running_update). Replaces the hgk_bn_finalize_deferred launch. rows <= 32, % 4 == 0. */
typedef struct hgk_bn_fold {
  const float* partial;
  int rows;
  long M;
  const float* gamma; /* nullable (affine = False) */
  const float* beta;
  float eps;
  float* stat;
  double* rec;
} hgk_bn_fold;
/* hgk_conv_fwd whose input transform is the folded finalize's (bf16, shapes with
 * hgk_conv_fold_ok() only — else HGK_ERR_UNSUPPORTED, nothing launched; workspace required) */
int hgk_conv_fwd_fold(hgk_stream_t stream, int dtype, const void* x, const void* w, int w_ld,
                      const float* bias, const void* res, void* y, int pre_relu, int post_relu,
                      float* stats, int* rows_out, int N, int H, int W, int Cin, int Cout, int KH,
                      int KW, int stride, int pad, int dil, void* workspace, size_t ws_bytes,
                      const hgk_bn_fold* fold);
/* 1 when a (twin, N1 > 0) forward launch of this geometry can fold the finalizes (rows0 / rows1
 * partial rows of the segments' BN inputs) */
int hgk_conv_fold_ok(int dtype, int N0, int H0, int W0, int N1, int H1, int W1, int Cin, int Cout,
                     int KH, int KW, int stride, int pad, int dil, int rows0, int rows1);
/* 1 when a (twin, N1 > 0) input-gradient launch of this geometry can fold the apply; bn_bwd: with
 * the fused BN-backward reduction of its own output (hgk_conv_fwd_bnbwd) */
int hgk_conv_vgrad_ok(int dtype, int N0, int H0, int W0, int N1, int H1, int W1, int Cin, int Cout,
                      int KH, int KW, int stride, int pad, int dil, int bn_bwd);
/* 1 when a (twin, N1 > 0) input-gradient launch of this geometry can fold the BN-backward finalize
 * AND apply of its input (hgk_bn_vgrad.partial set) with rows0 / rows1 partial rows; bn_bwd as in
 * hgk_conv_vgrad_ok; add: with hgk_bn_vgrad.add (ABI 28) */
int hgk_conv_vgrad_fin_ok(int dtype, int N0, int H0, int W0, int N1, int H1, int W1, int Cin,
                          int Cout, int KH, int KW, int stride, int pad, int dil, int bn_bwd,
                          int rows0, int rows1, int add);
size_t hgk_conv_fwd_workspace(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                              int stride, int pad, int dil);
/* One segment of a twin convolution: the per-use operands of hgk_conv_fwd (x, res, y, pre
 * transform, statistics, N/H/W) and, when bb_partial != NULL, those of hgk_conv_fwd_bnbwd. */
typedef struct hgk_conv_seg {
  const void* x;
  const void* res;
  void* y;
  const float* pre_scale;
  const float* pre_shift;
  float* stats;
  int* rows_out;
  int N, H, W;
  const void* bb_y;
  const float* bb_scale;
  const float* bb_shift;
  const float* bb_mean;
  const float* bb_invstd;
  float* bb_partial;
  int bb_relu;
  int* bb_rows;
  const hgk_bn_vgrad* vg; /* nullable: folded BN-backward apply (both segments or neither) */
  const hgk_bn_fold* fold; /* nullable: folded BN finalize of the input (both segments or neither) */
} hgk_conv_seg;
/* Two convolutions with the SAME weights / bias / kernel geometry on two inputs (an hourglass
 * level's up-branch and down-branch blocks share one ResidualBlock, try_with_torch.py:217-237):
 * each segment's result is exactly what hgk_conv_fwd (or hgk_conv_fwd_bnbwd) gives for it, in ONE
 * launch when both route to the implicit-GEMM kernel, else one launch per segment. Both segments
 * have statistics or neither; both a BN-backward epilogue or neither. workspace: >=
 * hgk_conv_fwd_twin_workspace() bytes. */
int hgk_conv_fwd_twin(hgk_stream_t stream, int dtype, const void* w, int w_ld, const float* bias,
                      int pre_relu, int post_relu, int Cin, int Cout, int KH, int KW, int stride,
                      int pad, int dil, const hgk_conv_seg* seg, void* workspace, size_t ws_bytes);
size_t hgk_conv_fwd_twin_workspace(int dtype, int N0, int H0, int W0, int N1, int H1, int W1,
                                   int Cin, int Cout, int KH, int KW, int stride, int pad, int dil);

/* Pack canonical fp32 nn.Conv2d weight [Cout][Cin][KH][KW] into the conv_fwd layout
 * [round_up(Cout_store,128)][w_ld] (k = (kh*KW+kw)*Cin_store + ci, zero padded), or — with
 * for_dgrad=1 — the spatially flipped, in/out-transposed weight that turns the stride-1
 * input-gradient into a forward conv ([round_up(Cin_store,128)][w_ld], k = (kh*KW+kw)*Cout_store
 * + co). *_store >= the logical counts: activations may be stored channel-padded (the 17-channel
 * heatmaps are kept as 64 channels so every head conv runs the vectorised MFMA path). */
int hgk_pack_conv_weight(hgk_stream_t stream, int dtype, const float* w, void* packed, int w_ld,
                         int Cout, int Cin, int KH, int KW, int for_dgrad, int Cout_store,
                         int Cin_store);
/* one weight layout to pack (the arguments of hgk_pack_conv_weight; rows_store = Cin_store for
 * a dgrad layout, else Cout_store) */
typedef struct hgk_pack_desc {
  const float* w;
  void* packed;
  int w_ld, Cout, Cin, KH, KW, for_dgrad, Cout_store, Cin_store, rows_store;
} hgk_pack_desc;
/* hgk_pack_conv_weight for n layouts, in ceil(n / 48) launches */
int hgk_pack_conv_weight_multi(hgk_stream_t stream, int dtype, const hgk_pack_desc* descs, int n);
/* w_ld the packer/conv expect for a given K = KH*KW*C (rounded up to 64) */
int hgk_conv_w_ld(int K);

/* ---- weight gradient (autograd of nn.Conv2d weight/bias) with ACCUMULATION, because the
 * reference reuses one module for up to 32 calls per step (try_with_torch.py:217,224-237,268,286):
 * dw[Cout_log][Cin_log][KH][KW] += sum_m dy[m][co] * pre(x)(m,k); db[Cout_log] += sum_m dy[m][co].
 * Cin / Cout are the STORED channel counts of x / dy (>= the logical Cin_log / Cout_log).
 * workspace: hgk_conv_wgrad_workspace() bytes (stored counts). */
size_t hgk_conv_wgrad_workspace(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                                int stride, int pad, int dil);
int hgk_conv_wgrad(hgk_stream_t stream, int dtype, const void* x, const void* dy,
                   const float* pre_scale, const float* pre_shift, int pre_relu, float* dw,
                   float* db, void* workspace, size_t ws_bytes, int N, int H, int W, int Cin,
                   int Cout, int KH, int KW, int stride, int pad, int dil, int Cin_log,
                   int Cout_log);
/* Deferred form for shared weights: every use of one weight accumulates its split-K partials
 * into the weight's own slab set ([slab_cap][Cout][K] + bias [slab_cap][Cout], fp32); slabs
 * [0, slabs_init) already hold earlier uses' partials (added to), the rest are overwritten.
 * *splits_out = slabs this use touched. One hgk_conv_wgrad_finish per weight and step then
 * reduces the slabs (fixed order) into dw / db (+=): ~40 reductions per step instead of ~360. */
int hgk_conv_wgrad_max_splits(void);
size_t hgk_conv_wgrad_slab_bytes(int Cin, int Cout, int KH, int KW, int slab_cap);
int hgk_conv_wgrad_accum(hgk_stream_t stream, int dtype, const void* x, const void* dy,
                         const float* pre_scale, const float* pre_shift, int pre_relu,
                         void* slabs, int slab_cap, int slabs_init, int with_bias, int* splits_out,
                         int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                         int pad, int dil);
int hgk_conv_wgrad_finish(hgk_stream_t stream, const void* slabs, int slab_cap, int nslabs,
                          float* dw, float* db, int Cin, int Cout, int KH, int KW, int Cin_log,
                          int Cout_log);
/* the arguments of one hgk_conv_wgrad_finish */
typedef struct hgk_wgrad_fin {
  const void* slabs;
  int slab_cap, nslabs;
  float* dw;
  float* db;
  int Cin, Cout, KH, KW, Cin_log, Cout_log;
} hgk_wgrad_fin;
/* hgk_conv_wgrad_finish for n weights in ceil(n / 32) launches, bitwise equal to the n single
 * calls (the weights of one flush point: ~30 launches per step become 2) */
int hgk_conv_wgrad_finish_multi(hgk_stream_t stream, const hgk_wgrad_fin* f, int n);
/* One use of a weight for hgk_conv_wgrad_accum_multi: input x [N,H,W,Cin] (with its fused
 * BN(+ReLU) transform, or NULL) and output grad dy [N,Ho,Wo,Cout]. */
typedef struct hgk_wgrad_src {
  const void* x;
  const void* dy;
  const float* pre_scale;
  const float* pre_shift;
  int pre_relu;
  int N, H, W;
} hgk_wgrad_src;
/* hgk_conv_wgrad_accum for nsrc uses of ONE weight in one launch (per 24 uses): the uses' pixels
 * are concatenated and split over workgroups, so many small (latency-bound) weight-grad GEMMs of
 * the small hourglass levels become one full-GPU launch. Same slab semantics as
 * hgk_conv_wgrad_accum; the per-slab summation order is the concatenated pixel order
 * (deterministic). Implicit-GEMM path only: Cin % 64 == 0, Cout % 8 == 0, same geometry for all
 * uses except N, H, W. */
int hgk_conv_wgrad_accum_multi(hgk_stream_t stream, int dtype, const hgk_wgrad_src* src, int nsrc,
                               void* slabs, int slab_cap, int slabs_init, int with_bias,
                               int* splits_out, int Cin, int Cout, int KH, int KW, int stride,
                               int pad, int dil);
/* One use of ONE weight for hgk_conv_wgrad_accum_batch: the hgk_conv_wgrad_accum_multi call
 * (nsrc = 1) of that weight. */
typedef struct hgk_wgrad_job {
  hgk_wgrad_src src;
  void* slabs;
  int slab_cap, slabs_init, with_bias;
  int Cin, Cout, KH, KW, stride, pad, dil;
} hgk_wgrad_job;
/* hgk_conv_wgrad_accum_multi(nsrc = 1) for n DIFFERENT weights, several per launch (jobs with the
 * same tile plan share a launch, up to 12): the unshared weights of hourglass_compare / train.py
 * (one use each, hourglass_compare.py:492-538) no longer cost a launch each. Every job's slabs are
 * bitwise those of its single call when the split plan is the single call's
 * (HGK_ROUTE_WG_BATCH_SLAB_X10 = 20, HGK_ROUTE_WG_BATCH_TARGET = 0); the default cap (5) takes
 * fewer pixel splits: another fp32 summation order. splits_out[i] = slabs job i touched. Every
 * job is validated before the first launch: an invalid job returns an error with nothing
 * accumulated and splits_out untouched. Jobs of 256-wide tiles (HGK_ROUTE_WG_FULL) and bf16 3x3
 * jobs the halo weight gradient tiles (HGK_ROUTE_WG_HALO_MULTI's size) take their own launch:
 * bitwise their single call. */
int hgk_conv_wgrad_accum_batch(hgk_stream_t stream, int dtype, const hgk_wgrad_job* jobs, int n,
                               int* splits_out);

/* ---- BatchNorm2d, training statistics (try_with_torch.py:184,187,190,249; PyTorch semantics:
 * biased variance to normalise, unbiased variance into running_var, momentum, eps) ---- */
int hgk_bn_stats(hgk_stream_t stream, int dtype, const void* x, long M, int C, float* partial,
                 int* rows_out);
/* Reduce partials -> mean, invstd and the fused affine scale = gamma*invstd,
 * shift = beta - mean*scale; update running stats if running_mean != NULL (training).
 * training == 0: eval mode, scale/shift from running stats (partial ignored). */
int hgk_bn_finalize(hgk_stream_t stream, const float* partial, int rows, long M, int C,
                    const float* gamma, const float* beta, float* running_mean,
                    float* running_var, float momentum, float eps, int training, float* mean,
                    float* invstd, float* scale, float* shift, float* scratch);
/* bytes of `scratch` the finalisers may use for `rows` partial rows. The forward statistics are
 * channel-major and never need it; the backward finaliser merges its row-major partials 64:1 into
 * it only when the workgroup-per-channel path is off (NULL scratch = single-stage) */
size_t hgk_bn_finalize_scratch(int rows, int C);
/* y = relu?(x*scale + shift): materialises a BN(+ReLU) output when no conv consumes it */
int hgk_bn_apply(hgk_stream_t stream, int dtype, const void* x, long M, int C, const float* scale,
                 const float* shift, int relu, void* y);
/* Backward of relu?(bn(y)): g = dA * [y*scale+shift > 0]; partials of (sum g, sum g*xhat) */
int hgk_bn_bwd_reduce(hgk_stream_t stream, int dtype, const void* dA, const void* y, long M,
                      int C, const float* scale, const float* shift, int relu, const float* mean,
                      const float* invstd, float* partial, int* rows_out);
/* dgamma += sum g*xhat, dbeta += sum g; coef[4][C] so that
 * dy = coef0*g + coef1*(y - coef3) + coef2   (coef3 = batch mean) */
int hgk_bn_bwd_finalize(hgk_stream_t stream, const float* partial, int rows, long M, int C,
                        const float* scale, const float* mean, const float* invstd, int training,
                        float* dgamma, float* dbeta, float* coef, float* scratch);
/* dy (= or +=, per accumulate) coef0*g + coef1*(y - coef3) + coef2 (+ add[m][c] if add) */
int hgk_bn_bwd_apply(hgk_stream_t stream, int dtype, const void* dA, const void* y, long M, int C,
                     const float* scale, const float* shift, int relu, const float* coef,
                     const void* add, void* dy, int accumulate);
/* ---- a BN pair whose outputs are summed: hourglass_compare's / train.py's ResidualBlock output
 * bn4(conv3(..)) + downsaple-BN(conv(x)) (hourglass_compare.py:437-440, train.py:444-447) ---- */
typedef struct hgk_bn_side {
  const void* y;       /* the BN input [M][C] (activation dtype) */
  const float* scale;  /* [C] forward scale / shift (BNUse stat rows 2 / 3) */
  const float* shift;
  const float* mean;   /* [C] batch mean / invstd (backward only) */
  const float* invstd;
  int relu;
  float* partial;      /* backward: [rows][2][C] sums (hgk_bn_bwd_reduce's format) */
} hgk_bn_side;
/* out = relu_a?(a*scale_a + shift_a) + relu_b?(b*scale_b + shift_b): each term rounded to the
 * activation dtype as hgk_bn_apply writes it, their sum as hgk_add; with partial != NULL also the
 * statistics partials of `out` exactly as hgk_bn_stats computes them (same rows, same order).
 * Bitwise equal to hgk_bn_apply x2 + hgk_add (+ hgk_bn_stats), in one pass: reads a and b once,
 * writes out once. (replaces BatchNorm2d x2 + the add of hourglass_compare.py:437-440) */
int hgk_bn_apply2_add(hgk_stream_t stream, int dtype, const hgk_bn_side* a, const hgk_bn_side* b,
                      void* out, long M, int C, float* partial, int* rows_out);
/* hgk_bn_bwd_reduce for both sides of such a pair over their common upstream gradient dA (read
 * once): a->partial and b->partial bitwise equal to two hgk_bn_bwd_reduce calls */
int hgk_bn_bwd_reduce2(hgk_stream_t stream, int dtype, const void* dA, long M, int C,
                       const hgk_bn_side* a, const hgk_bn_side* b, int* rows_out);
/* Several DIFFERENT BatchNorms' deferred finalizes in one launch (a host that finalizes each BN
 * only when its consumer needs it batches the ones pending then: hourglass_compare's bn4 and the
 * projection BN, hourglass_compare.py:437-440). Per job exactly hgk_bn_finalize_deferred's result
 * for that one BN (bitwise): stat [4][C] and the running-statistics record [2][C]. */
typedef struct hgk_bn_fin_job {
  const float* partial;
  int rows;
  long M;
  int C;
  const float *gamma, *beta;
  float eps;
  double* rec;
  float* stat;
} hgk_bn_fin_job;
int hgk_bn_finalize_multi(hgk_stream_t stream, const hgk_bn_fin_job* jobs, int n);
/* ... and their backward finalizes (coef [4][C], dgamma / dbeta accumulated), bitwise
 * hgk_bn_bwd_finalize per job; every job needs rows >= hgk_bn_bwd_finalize_multi_min_rows(). */
typedef struct hgk_bnb_fin_job {
  const float* partial;
  int rows;
  long M;
  int C;
  const float *scale, *mean, *invstd;
  int training;
  float *dgamma, *dbeta, *coef;
} hgk_bnb_fin_job;
int hgk_bn_bwd_finalize_multi(hgk_stream_t stream, const hgk_bnb_fin_job* jobs, int n);
int hgk_bn_bwd_finalize_multi_min_rows(void);
/* The pair's backward after hgk_bn_bwd_reduce2: per side the coefficients — from its partial rows
 * in-kernel when partial != NULL (rows <= hgk_bn_bwd_fused_max_rows(); workgroup 0 adds the sums to
 * dgamma / dbeta), else from coef (hgk_bn_bwd_finalize's [4][C]) — and dy_side = its apply of the
 * common upstream gradient dA, in ONE pass reading dA once. Bitwise equal to two
 * hgk_bn_bwd_finalize_apply (resp. two hgk_bn_bwd_apply) calls. Both sides in the same mode. */
typedef struct hgk_bnb_side {
  const void* y;
  const float *scale, *shift, *mean, *invstd;
  int relu;
  const float* partial;
  int rows;
  const float* coef;
  float *dgamma, *dbeta;
  void* dy;
} hgk_bnb_side;
int hgk_bn_bwd_pair(hgk_stream_t stream, int dtype, const void* dA, long M, int C, int training,
                    const hgk_bnb_side* a, const hgk_bnb_side* b);
/* hgk_bn_bwd_finalize + hgk_bn_bwd_apply in one launch (every workgroup reduces the partial rows
 * itself; workgroup 0 accumulates dgamma / dbeta): rows <= hgk_bn_bwd_fused_max_rows(),
 * C % 8 == 0, C <= 512, 256 % (C/2) == 0. */
int hgk_bn_bwd_fused_max_rows(void);
int hgk_bn_bwd_finalize_apply(hgk_stream_t stream, int dtype, const float* partial, int rows,
                              long M, int C, const float* scale, const float* shift, int relu,
                              const float* mean, const float* invstd, int training, float* dgamma,
                              float* dbeta, const void* dA, const void* y, const void* add,
                              void* dy, int accumulate);

/* ---- twin / deferred BatchNorm: two uses of ONE BatchNorm2d module per launch (the shared
 * ResidualBlock of an hourglass level, try_with_torch.py:217-237) ---- */
typedef struct hgk_bn_seg {
  const float* partial; /* stats partials [C][3][rows] of the use's input */
  int rows;
  long M;
  double* rec; /* out [2][C]: batch mean | unbiased variance (fp64) */
  float* stat; /* out [4][C]: mean | invstd | scale | shift */
} hgk_bn_seg;
/* hgk_bn_finalize(training=1) for nseg (1 or 2) uses, except that the running statistics are NOT
 * updated: each use's record goes to rec, applied later by hgk_bn_running_update in call order */
int hgk_bn_finalize_deferred(hgk_stream_t stream, const hgk_bn_seg* seg, int nseg, int C,
                             const float* gamma, const float* beta, float eps);
typedef struct hgk_bn_running {
  float* running_mean;
  float* running_var;
  const double* rec; /* a hgk_bn_finalize_deferred record */
  int C;
  float momentum;
} hgk_bn_running;
/* running = (1-momentum)*running + momentum*rec for the n entries IN ORDER (entries with the same
 * running_mean are sequential; the result equals hgk_bn_finalize's immediate updates bitwise) */
int hgk_bn_running_update(hgk_stream_t stream, const hgk_bn_running* e, int n);
typedef struct hgk_bnb_seg {
  const float* partial; /* BN-backward partials [rows][2][C] (hgk_conv_fwd_bnbwd) */
  int rows;
  long M;
  const float* stat; /* [4][C] of the forward use */
  const void* dA;
  const void* y;
  const void* add;
  void* dy;
  int accumulate;
} hgk_bnb_seg;
/* hgk_bn_bwd_finalize + hgk_bn_bwd_apply for nseg uses of one module; dgamma / dbeta accumulate
 * segment 0 then segment 1. rows <= hgk_bn_bwd_fused_max_rows() for every segment: one launch,
 * else finalize + apply launches through coef ([nseg][6][C] fp32 scratch). dy == NULL in every
 * segment (more rows than that only): coef + dgamma / dbeta only, one launch — the apply is then
 * folded into the consuming convolution (hgk_bn_vgrad, coefficients = rows 0-3 of coef[q]). */
int hgk_bn_bwd_twin(hgk_stream_t stream, int dtype, const hgk_bnb_seg* seg, int nseg, int C,
                    int relu, int training, float* dgamma, float* dbeta, float* coef);

/* ---- data side of the path ----
 * Gaussian heatmap targets, try_with_torch.py:104-130 (myImageDataset_COCO.__getitem__):
 * kps [B][P][K][3] = (x, y, v) in original-image pixels, counts[B] annotations per image, wh[B][2]
 * original (w, h). As the reference: only the LAST annotation of an image counts (its map buffer
 * is re-created per annotation), coordinates are scaled to the map and truncated toward zero in
 * float64, v == 0 gives an all-zero map, out[b][k][r][c] = (float)exp(-((c-x)^2+(r-y)^2)/(2s^2)). */
int hgk_gauss_targets(hgk_stream_t stream, const float* kps, const int* counts, const float* wh,
                      int B, int P, int K, int Hm, int Wm, float sigma, float* out);
/* PCKh, train.py:759-791: x [B][C][H][W] heatmaps (channel j+1 <-> joint j), target [B][H][W]
 * int32 label map (j+1 marks joint j), rect [B][4] head box (float64). preds / labels [B][C][2]
 * (x, y) of the first row-major maximum / label pixel (0 for an unlabelled joint); acc [B][11]
 * = correct/total at thresholds np.arange(0, 0.55, 0.05) (float32 distance arithmetic as the
 * reference's tensors; nan when an image has no labelled joint). scratch: B*C ints. */
int hgk_pckh(hgk_stream_t stream, const float* x, const int* target, const double* rect, int B,
             int C, int H, int W, int* preds, int* labels, int* scratch, double* acc);

/* ---- MaxPool2d(2) (try_with_torch.py:220,226,265) ---- */
int hgk_maxpool2_fwd(hgk_stream_t stream, int dtype, const void* x, void* y, int N, int H, int W,
                     int C);
/* maxpool2 that also emits the stats partials (channel-major [C][3][*rows_out]) of y for the
 * BatchNorm that consumes it (the next residual block's bn1) — no separate hgk_bn_stats pass */
int hgk_maxpool2_fwd_stats(hgk_stream_t stream, int dtype, const void* x, void* y, int N, int H,
                           int W, int C, float* partial, int* rows_out);
/* dx (= or +=) routes dy to the first maximum of each 2x2 window (PyTorch CPU tie rule) */
int hgk_maxpool2_bwd(hgk_stream_t stream, int dtype, const void* x, const void* dy, void* dx,
                     int N, int H, int W, int C, int accumulate);

/* ---- x2 up-sampling + skip-add (try_with_torch.py:238-239: interpolate(bilinear,
 * align_corners=True) then up1 + up2; mode NEAREST for hourglass_compare.py:532-542) ----
 * out[N,2h,2w,C] = skip + up(low[N,h,w,C]);  skip may alias out. */
int hgk_upsample2_add_fwd(hgk_stream_t stream, int dtype, int mode, const void* low,
                          const void* skip, void* out, int N, int h, int w, int C);
/* upsample2_add that also emits the stats partials of out (as hgk_maxpool2_fwd_stats) */
int hgk_upsample2_add_fwd_stats(hgk_stream_t stream, int dtype, int mode, const void* low,
                                const void* skip, void* out, int N, int h, int w, int C,
                                float* partial, int* rows_out);
/* dlow (= or +=) up^T(dout), gather form (no atomics) */
int hgk_upsample2_bwd(hgk_stream_t stream, int dtype, int mode, const void* dout, void* dlow,
                      int N, int h, int w, int C, int accumulate);

/* ---- per-stack nn.MSELoss (try_with_torch.py:305-308,333-341), fused forward+backward ----
 * out, target, grad: NCHW fp32 [numel]. loss_partial[rows] += nothing: writes per-workgroup
 * partial sums of (o-t)^2; grad = grad_scale * 2 (o - t) / numel. */
int hgk_mse_fwd_bwd(hgk_stream_t stream, const float* out, const float* target, long numel,
                    float* loss_partial, int* rows_out, float* grad, float grad_scale);
/* loss[0] (= or +=) sum(loss_partial[0:rows]) / numel */
int hgk_mse_finalize(hgk_stream_t stream, const float* loss_partial, int rows, long numel,
                     float* loss, int accumulate);

/* All nheads per-stack MSE losses of one step in one launch + one finalize (round 6; ABI 38), on
 * the engine's NHWC heads: heads[h] NHWC dtype [N][H][W][C_store] (the first K channels are the
 * logical heatmaps), target NCHW fp32 [N][K][H][W] (shared by every head), grads[h] NHWC dtype
 * (written: grad_scale * 2 (o - t) / (N K H W), pad channels 0 — the values hgk_nhwc_to_nchw +
 * hgk_mse_fwd_bwd + hgk_nchw_to_nhwc produce); loss[0] = sum over heads of each head's mean
 * (hgk_mse_finalize's arithmetic; the per-head partial sums run in another order). loss_partial:
 * hgk_mse_heads_partial_rows() floats. nheads <= 8, K <= 64, C_store % 8 == 0, 16-B aligned
 * heads / grads. */
int hgk_mse_heads_nhwc(hgk_stream_t stream, int dtype, const void* const* heads, void* const* grads,
                       int nheads, const float* target, int N, int K, int H, int W, int C_store,
                       float grad_scale, float* loss_partial, float* loss);
int hgk_mse_heads_partial_rows(void);

/* ---- layout / elementwise glue ---- */
/* NCHW fp32 [N][C][H][W] -> NHWC dtype [N][H][W][C_store] (pad channels zeroed) */
int hgk_nchw_to_nhwc(hgk_stream_t stream, int dtype, const float* src, void* dst, int N, int C,
                     int H, int W, int C_store);
/* NHWC dtype [N][H][W][C_store] -> NCHW fp32 [N][C][H][W] */
int hgk_nhwc_to_nchw(hgk_stream_t stream, int dtype, const void* src, float* dst, int N, int C,
                     int H, int W, int C_store);
/* dst[m][dst_c0 + c] (= or +=) src[m][src_c0 + c] for c < nch, m < M: NHWC channel-range copy,
 * i.e. torch.cat(dim=1) and its backward for the progressive heads (replaces the reference's
 * torch.cat([ll, tmpOut], dim=1), try_with_aspp.py:327-334 / try_different_stack.py:316-328) */
int hgk_channel_copy(hgk_stream_t stream, int dtype, const void* src, int src_C, int src_c0,
                     void* dst, int dst_C, int dst_c0, int nch, long M, int accumulate);
/* y = a + b  (or y += a if b == NULL and accumulate), elementwise over n elements */
int hgk_add(hgk_stream_t stream, int dtype, const void* a, const void* b, void* y, long n,
            int accumulate);

/* dst[n, j, l, :] = src[n, j/stride, l/stride, :] where stride divides j and l (and the source
 * pixel exists), else 0; src NHWC [N, h, w, C], dst [N, Hz, Wz, C]. The input-gradient of a
 * stride-s conv is then the stride-1 conv of dst with the flipped / transposed weight at padding
 * dil*(K-1)-pad, Hz = H + 2 pad - dil (K-1): the strided residual blocks of train.py:411-447
 * (3x3/2 conv2 and the 1x1/2 projection) */
int hgk_zero_insert(hgk_stream_t stream, int dtype, const void* src, void* dst, int N, int h, int w,
                    int C, int stride, int Hz, int Wz);
/* y[n, c] = scale * sum_{p < HW} x[n, p, c] (+ y[n, c] if accumulate), x NHWC [N, HW, C]:
 * nn.AdaptiveAvgPool2d((1, 1)) forward (scale = 1/HW) and the backward of a 1x1 -> HxW broadcast
 * (scale = 1) — the live ASPP image-pool branch, try_more_layer.py:266-268,286-287 */
int hgk_spatial_sum(hgk_stream_t stream, int dtype, const void* x, void* y, int N, int HW, int C,
                    float scale, int accumulate);
/* y[n, p, c] = scale * x[n, c] (+ y if accumulate): F.interpolate(1x1 -> HxW, bilinear,
 * align_corners=True) forward (scale = 1, try_more_layer.py:287) and the average pool's backward
 * (scale = 1/HW) */
int hgk_spatial_broadcast(hgk_stream_t stream, int dtype, const void* x, void* y, int N, int HW,
                          int C, float scale, int accumulate);

/* ---- progressive-head losses (train.py:343-408), NCHW fp32 outputs ---- */
/* loss[n, p] = (mask[n, p] *) CE of pixel p: logsumexp_k logits[n, k, p] - logits[n, target, p];
 * logits [N, K, P], target int64 [N, P] (-100 = ignored: 0; any other out-of-range class sets
 * *bad = 1 and gives 0), mask [N, P] or NULL. P = H * W. */
int hgk_ce_pixels(hgk_stream_t stream, const float* logits, const long* target, const float* mask,
                  int N, int K, long P, float* loss, int* bad);
/* dlogits = g * mult * weight[n, p] (* mask) * (softmax - onehot(target)); g = *gscale (device
 * scalar, the incoming loss gradient; NULL = 1), weight / mask NULL = 1; ignored pixels get 0 */
int hgk_ce_grad(hgk_stream_t stream, const float* logits, const long* target, const float* weight,
                const float* mask, int N, int K, long P, const float* gscale, float mult,
                float* dlogits);
/* Fused nn.CrossEntropyLoss forward + backward for the Trainer's progressive heads
 * (try_with_aspp.py:356-358,393-396): loss_partial[0:*rows_out] = per-workgroup sums of the pixel
 * losses (finish with hgk_mse_finalize(numel = N P) for the mean); dlogits = grad_scale / (N P) *
 * (softmax - onehot(target)). logits NCHW fp32 [N, K, P], target int64 [N, P]; a target outside
 * [0, K) sets *bad = 1 (device int) and contributes nothing. *rows_out <= 1024. */
int hgk_ce_fwd_bwd(hgk_stream_t stream, const float* logits, const long* target, int N, int K,
                   long P, float* loss_partial, int* rows_out, float* dlogits, float grad_scale,
                   int* bad);
/* out = (mask[n, p] *) (a - b)^2 elementwise over [N, C, P] */
int hgk_sqdiff(hgk_stream_t stream, const float* a, const float* b, const float* mask, int N, int C,
               long P, float* out);
/* da = g * mult * 2 (a - b) (* weight[i]) (* mask[n, p]) */
int hgk_sqdiff_grad(hgk_stream_t stream, const float* a, const float* b, const float* weight,
                    const float* mask, int N, int C, long P, const float* gscale, float mult,
                    float* da);
/* per row of values [rows, L]: sel = 1 for the k largest (ties at the k-th value: lowest indices
 * first), else 0; sums[row] = sum of the selected values (fixed order) — torch.topk(..., k) of
 * the bootstrapped losses; 1 <= k <= L */
int hgk_topk_select(hgk_stream_t stream, const float* values, int rows, long L, long k,
                    float* sel, float* sums);

/* ---- optimizer: Adam (torch.optim.Adam semantics, try_with_torch.py:317), flat fp32 ---- */
/* step_state: device float[4] zero-initialised by the caller; [0] counts steps on the device
 * (graph-replay safe), [1],[2] hold the bias corrections of the current step. */
int hgk_adam_step(hgk_stream_t stream, float* param, const float* grad, float* exp_avg,
                  float* exp_avg_sq, long n, float lr, float beta1, float beta2, float eps,
                  float weight_decay, float* step_state);

#ifdef __cplusplus
}
#endif
#endif /* HGK_H_ */
