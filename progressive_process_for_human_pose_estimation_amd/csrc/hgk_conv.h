// Definitions shared by the convolution translation units (hgk_conv.hip: implicit-GEMM, halo and
// weight-grad kernels; hgk_conv_ring.hip: the streaming 1x1 kernel of the big levels).
#pragma once
#include "hgk_common.h"

namespace hgk {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

static constexpr int kMaxPreC = 512;  // max channels of a fused BN(+ReLU) input transform
static constexpr int kHaloPreC = 256;  // ... on the 3x3 halo path (staged in LDS: 2 KB)
static constexpr int kSplitCtrBytes = 4096;  // split-K tile counters at the head of a conv workspace
static constexpr int kMaxStatsRows = 65536;
// folded BN finalize (hgk_conv_fwd_fold): at most this many producer partial rows (the 8x8 / 4x4
// levels: 32 / 8), a multiple of 4 (16-B loads)
static constexpr int kFoldRows = 32;  // partial rows of one launch (384x384 stem at N=16: 9216)

// BN affine (+ReLU) of one 16-byte chunk, result packed back to T. For bf16 the ReLU runs on the
// packed result as a signed-int16 max with 0 (a bf16 is negative iff its int16 image is), one
// v_pk_max_i16 per 2 elements instead of 2 v_max_f32; round(relu(x)) == relu(round(x)).
template <typename T>
__device__ __forceinline__ typename Vec16<T>::type bn_relu_chunk(const typename Vec16<T>::type& v,
                                                               const float* ps, const float* pb,
                                                               bool relu);
template <>
__device__ __forceinline__ float4 bn_relu_chunk<float>(const float4& v, const float* ps,
                                                       const float* pb, bool relu) {
  float4 r = make_float4(fmaf(v.x, ps[0], pb[0]), fmaf(v.y, ps[1], pb[1]), fmaf(v.z, ps[2], pb[2]),
                         fmaf(v.w, ps[3], pb[3]));
  if (relu) r = make_float4(fmaxf(r.x, 0.f), fmaxf(r.y, 0.f), fmaxf(r.z, 0.f), fmaxf(r.w, 0.f));
  return r;
}
template <>
__device__ __forceinline__ uint4 bn_relu_chunk<bf16_t>(const uint4& v, const float* ps,
                                                       const float* pb, bool relu) {
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  const uint32_t in[4] = {v.x, v.y, v.z, v.w};
  uint32_t out[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = fmaf(__uint_as_float(in[i] << 16), ps[2 * i], pb[2 * i]);
    const float hi = fmaf(__uint_as_float(in[i] & 0xffff0000u), ps[2 * i + 1], pb[2 * i + 1]);
    bf16x2_t h = {(__bf16)lo, (__bf16)hi};
    s16x2 q = __builtin_bit_cast(s16x2, h);
    if (relu) q = __builtin_elementwise_max(q, (s16x2){0, 0});
    out[i] = __builtin_bit_cast(uint32_t, q);
  }
  return make_uint4(out[0], out[1], out[2], out[3]);
}

struct ConvFwdArgs {
  const void* x;
  const void* w;
  const float* bias;
  const void* res;
  void* y;
  const float* pre_scale;
  const float* pre_shift;
  float* stats;
  int pre_relu, post_relu;
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, dil;
  int K, w_ld;
  long M;
  FastDiv fd_howo, fd_wo, fd_cin, fd_kw;
  float* split_ws;   // split-K fp32 partials [ksplit][M][Cout] (small-M launches only)
  int ksplit, kt_per_split;
  // split-K fix-up in the conv launch (no epilogue kernel): per-tile arrival counters (zero on
  // entry, left zero: the last-arriving split of a tile resets its counter), null = epilogue kernel
  int* split_ctr;
  // fused BatchNorm-backward reduction over the produced tensor dA (this launch is the input
  // gradient of a BN(+ReLU) output): per channel sum g and sum g*xhat, g = dA * [relu mask],
  // xhat = (bb_y - mean) * invstd -> partial rows [rows][2][Cout] (hgk_bn_bwd_reduce's format)
  const void* bb_y;
  const float *bb_scale, *bb_shift, *bb_mean, *bb_invstd;
  float* bb_partial;
  int bb_relu;
  // folded BatchNorm-backward apply (hgk_conv_fwd_bnbwd_vg): x is the upstream gradient dA of a
  // train-mode BN(+ReLU) whose input is vg_y [M][Cin]; the conv consumes dy = bnb_apply(dA, vg_y,
  // vg_scale, vg_shift, coefficients vg_coef [4][Cin]) and also stores it to vg_out
  const void* vg_y;
  const float *vg_scale, *vg_shift, *vg_coef;
  void* vg_out;
  int vg_relu;
  // folded BatchNorm finalize (hgk_conv_fwd_fold): the input transform's scale / shift are
  // computed by every workgroup from the producer's channel-major statistics partials
  // [Cin][3][fold_rows] (fold_M values per channel); the first workgroup of the launch (of the
  // segment) publishes mean | invstd | scale | shift (fold_stat [4][Cin]) and the fp64
  // running-statistics record (fold_rec [2][Cin]: mean | unbiased variance)
  const float* fold_part;
  int fold_rows;
  long fold_M;
  const float *fold_gamma, *fold_beta;
  float fold_eps;
  float* fold_stat;
  double* fold_rec;
  // statistics partials are CHANNEL-major, [Cout][3][stats_R] (stats_R = partial rows of the
  // launch): a finaliser's per-channel reads are contiguous instead of one 128-B line per row
  int stats_R;
};

// One 16-B-per-lane LDS-DMA (global_load_lds_dwordx4; LDS destination = wave-uniform M0 base +
// 16 * lane). Issued from inline asm on purpose: hipcc cannot tell which stage buffer a DMA
// writes, and for the builtin it drains every DMA in flight (vmcnt(0)) before each fragment
// ds_read; the kernel orders DMA and ds_read itself with counted vmcnt + s_barrier.
__device__ __forceinline__ void dma16(const void* src, char* lds_wave_base) {
  const uint32_t l = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds_wave_base;
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
               ::"s"(__builtin_amdgcn_readfirstlane(l)), "v"(src)
               : "memory", "m0");
}

// v of the partner lane (every lane has one for the patterns below); written as update_dpp with
// bound_ctrl so the compiler folds `x + dpp_mov(v)` into one v_add_f32_dpp
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}
// partners inside a row of 16 lanes: quad_perm(1,0,3,2) = lane ^ 1, quad_perm(3,2,1,0) = ^ 3,
// row_half_mirror = ^ 7, row_mirror = ^ 15
constexpr int kDppX1 = 0xB1, kDppX3 = 0x1B, kDppX7 = 0x141, kDppX15 = 0x140;

// sum over the 16 lanes of a row; stage-major so a DPP never reads a VGPR written by the
// instruction right before it (no hazard nops)
template <int CTRL, int N>
__device__ __forceinline__ void row_add_stage(float* v) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] += dpp_mov<CTRL>(v[i]);
}
template <int N>
__device__ __forceinline__ void row_allreduce(float* v) {
  row_add_stage<kDppX1, N>(v);
  row_add_stage<kDppX3, N>(v);
  row_add_stage<kDppX7, N>(v);
  row_add_stage<kDppX15, N>(v);
}
// streaming 1x1 path (hgk_conv_ring.hip): shape check and launch of one convolution or a twin pair
// (a1 != nullptr: the second segment, same weights)
bool ring_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1 = nullptr);
int launch_ring(hipStream_t st, ConvFwdArgs& a0, ConvFwdArgs* a1, int* rows0, int* rows1);
// row-streaming 3x3 path (hgk_conv_row3.hip): the 128 -> 128 3x3 at the 64x64 / 32x32 levels
bool row3_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1 = nullptr);
int launch_row3(hipStream_t st, ConvFwdArgs& a0, ConvFwdArgs* a1, int* rows0, int* rows1);

}  // namespace hgk
