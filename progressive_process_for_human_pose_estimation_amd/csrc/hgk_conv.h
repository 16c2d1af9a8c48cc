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

// Read-modify-write of a workgroup's MFMA accumulators (16x16 fragments, FM x FN per wave, element
// r of lane (lg, lr) at row co_base + i*16 + r, column kc_base + j*16) into its fp32 partial slab
// [Cout][K]. Every load is issued before the first store: as far as the compiler knows a store
// may alias the next element's load, so the natural `*d = *d + v` loop serialises one L2/HBM
// round trip per element. Loads use clamped indices (no guarded loads); only stores are guarded.
template <int FM, int FN>
__device__ __forceinline__ void slab_rmw(float* __restrict__ slab, int K, int Cout, bool accum,
                                         int co_base, int kc_base, const f32x4 (&acc)[FM][FN]) {
  float old[FM][FN][4];
  if (accum) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = min(co_base + i * 16 + r, Cout - 1);
          const int kc = min(kc_base + j * 16, K - 1);
          old[i][j][r] = slab[(long)co * K + kc];
        }
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co_base + i * 16 + r, kc = kc_base + j * 16;
        if (co < Cout && kc < K)
          slab[(long)co * K + kc] = accum ? old[i][j][r] + acc[i][j][r] : acc[i][j][r];
      }
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
  // with vg_part the BN-backward finalize is folded too (image-tile kernel only): the coefficients
  // come from the partial rows [vg_rows][2][Cin] with hgk_bn_bwd_finalize_apply's arithmetic, and
  // the segment's first workgroup accumulates vg_dgamma / vg_dbeta (twin: segment 0's first
  // workgroup, for both segments in order)
  const float* vg_part;
  int vg_rows, vg_training;
  long vg_M;
  const float *vg_mean, *vg_invstd;
  float *vg_dgamma, *vg_dbeta;
  const void* vg_add;  // nullable: gradient already accumulated for the BN input, added to dy
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
// ---- twin launches: two convolutions with the same weights in one grid ----
static constexpr int kNoTwin = 1 << 30;

// segment `s` of a twin launch as a local ConvFwdArgs, picked word by word (constant offsets, so it
// lives in registers; a reference selected between the two kernel arguments made the compiler
// copy them to scratch)
static constexpr int kArgWords = (int)(sizeof(ConvFwdArgs) / 4);
__device__ __forceinline__ void twin_pick(const ConvFwdArgs& a0, const ConvFwdArgs& a1, bool s,
                                          uint32_t* wr) {
  static_assert(sizeof(ConvFwdArgs) % 4 == 0, "word-wise pick");
  const uint32_t* w0 = reinterpret_cast<const uint32_t*>(&a0);
  const uint32_t* w1 = reinterpret_cast<const uint32_t*>(&a1);
#pragma unroll
  for (int i = 0; i < kArgWords; ++i) wr[i] = s ? w1[i] : w0[i];
}


// Epilogue, second half: the tile's HROWS x BN values (acc + bias, rounded to T) are staged in Cs;
// add the residual, ReLU, store with 16-B coalesced accesses, and emit the BN statistics partial
// row (sum, M2 about this half's mean, count) — shared by the fused and the split-K epilogues.
// TILE_W > 0: the tile is a spatial block of rows of TILE_W output pixels (3x3 halo kernel);
// tile row r is pixel m0 + (r / TILE_W) * Wo + r % TILE_W (always inside the image).
template <typename T, int BM, int BN, int NT, int HROWS, int NH, int TILE_W = 0>
__device__ __forceinline__ void epi_store_half(const ConvFwdArgs& a, T* Cs, float* red,
                                               float* bmean, long m0, int n0, int h, int tid,
                                               long mtile, bool active = true) {
  constexpr int VEC = Vec16<T>::N;
  constexpr int LDC = BN + 16 / (int)sizeof(T);
  constexpr int ECH = BN / VEC;
  constexpr int ERPP = NT / ECH;
  T* __restrict__ y = reinterpret_cast<T*>(a.y);
  const T* res = reinterpret_cast<const T*>(a.res);
  const int ecv = tid % ECH, er0 = tid / ECH;
  const bool vec_ok = (a.Cout % VEC) == 0;
  // 2) coalesced: + residual, ReLU, store; per-thread channel sums for the BN statistics
    const long hm0 = m0 + h * HROWS;
    const long nrows = TILE_W ? (long)HROWS : max(0L, min((long)HROWS, a.M - hm0));
    const int cb = n0 + ecv * VEC;
    float s1[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) s1[e] = 0.f;
    const bool bb = a.bb_partial != nullptr;  // host guarantees vec_ok when set
    float g1[VEC], gx[VEC], bsc[VEC], bsh[VEC], bmu[VEC], bis[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      g1[e] = 0.f; gx[e] = 0.f;
      bsc[e] = 0.f; bsh[e] = 0.f; bmu[e] = 0.f; bis[e] = 0.f;
    }
    if (bb && active) {
      // this thread's VEC channels, loaded once (16-B loads, clamped column) before the row loop
      const int cbc = min(cb, a.Cout - VEC);
#pragma unroll
      for (int e = 0; e < VEC; e += 4) {
        const float4 q0 = *reinterpret_cast<const float4*>(a.bb_scale + cbc + e);
        const float4 q1 = *reinterpret_cast<const float4*>(a.bb_shift + cbc + e);
        const float4 q2 = *reinterpret_cast<const float4*>(a.bb_mean + cbc + e);
        const float4 q3 = *reinterpret_cast<const float4*>(a.bb_invstd + cbc + e);
        bsc[e] = q0.x; bsc[e + 1] = q0.y; bsc[e + 2] = q0.z; bsc[e + 3] = q0.w;
        bsh[e] = q1.x; bsh[e + 1] = q1.y; bsh[e + 2] = q1.z; bsh[e + 3] = q1.w;
        bmu[e] = q2.x; bmu[e + 1] = q2.y; bmu[e + 2] = q2.z; bmu[e + 3] = q2.w;
        bis[e] = q3.x; bis[e + 1] = q3.y; bis[e + 2] = q3.z; bis[e + 3] = q3.w;
      }
    }
    // residual and BN-input rows of this thread: every load issued before the first store (a
    // store to y may alias a later row's load as far as the compiler knows, which would
    // serialise one round trip per row); clamped rows/columns, so no load is guarded
    constexpr int RPT = HROWS / ERPP;
    typedef typename Vec16<T>::type V;
    const int cbc = min(cb, a.Cout - VEC);
    auto prefetch = [&](int u, V* rr, V* ry) {
      const int r = er0 + u * ERPP;
      long row = TILE_W ? hm0 + (long)(r / TILE_W) * a.Wo + (r % TILE_W) : hm0 + r;
      if (!TILE_W) row = min(row, a.M - 1);
      if (res) rr[u] = load16(res + row * a.Cout + cbc);
      if (bb) ry[u] = load16(reinterpret_cast<const T*>(a.bb_y) + row * a.Cout + cbc);
    };
    V rres[RPT], rby[RPT];
#ifndef HGK_ABL_NO_EPI_PREFETCH
    if (vec_ok && active) {
#pragma unroll
      for (int u = 0; u < RPT; ++u) prefetch(u, rres, rby);
    }
#endif
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int r = er0 + u * ERPP;
      const long row = TILE_W ? hm0 + (long)(r / TILE_W) * a.Wo + (r % TILE_W) : hm0 + r;
      if (!active || (!TILE_W && row >= a.M)) break;
#ifdef HGK_ABL_NO_EPI_PREFETCH
      if (vec_ok) prefetch(u, rres, rby);
#endif
      T* cp = &Cs[r * LDC + ecv * VEC];
      float f[VEC];
      unpack16<T>(*reinterpret_cast<const V*>(cp), f);
      const long off = row * a.Cout + cb;
      if (vec_ok) {
        if (cb < a.Cout) {
          if (res) {
            float rv[VEC];
            unpack16<T>(rres[u], rv);
#pragma unroll
            for (int e = 0; e < VEC; ++e) f[e] += rv[e];
          }
          if (a.post_relu)
#pragma unroll
            for (int e = 0; e < VEC; ++e) f[e] = fmaxf(f[e], 0.f);
          const typename Vec16<T>::type pv = pack16<T>(f);
          store16(y + off, pv);
          unpack16<T>(pv, f);
          *reinterpret_cast<typename Vec16<T>::type*>(cp) = pv;  // keep stored value for stats
#pragma unroll
          for (int e = 0; e < VEC; ++e) s1[e] += f[e];
          if (bb) {
            // BN backward partial sums on the STORED dA (what hgk_bn_bwd_reduce would read)
            float yv[VEC];
            unpack16<T>(rby[u], yv);
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
              float g = f[e];
              if (a.bb_relu && !(fmaf(yv[e], bsc[e], bsh[e]) > 0.f)) g = 0.f;
              g1[e] += g;
              gx[e] += g * ((yv[e] - bmu[e]) * bis[e]);
            }
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          if (cb + e >= a.Cout) break;
          float v = f[e];
          if (res) v += to_f(res[off + e]);
          if (a.post_relu) v = fmaxf(v, 0.f);
          const T tv = from_f<T>(v);
          y[off + e] = tv;
          cp[e] = tv;
          s1[e] += to_f(tv);
        }
      }
    }
    if (bb) {
      // fixed-order block reduction of the per-thread BN-backward sums -> one partial row
#pragma unroll
      for (int q2 = 0; q2 < 2; ++q2) {
        if (active) {
#pragma unroll
          for (int e = 0; e < VEC; ++e) red[er0 * BN + ecv * VEC + e] = q2 ? gx[e] : g1[e];
        }
        __syncthreads();
        for (int c = tid; active && c < BN; c += NT) {
          float sm = 0.f;
          for (int i = 0; i < ERPP; ++i) sm += red[i * BN + c];
          const int col = n0 + c;
          if (col < a.Cout) a.bb_partial[((mtile * NH + h) * 2 + q2) * a.Cout + col] = sm;
        }
        __syncthreads();
      }
    }
    if (a.stats) {
      // two-pass (sum, M2, n) of this half's rows, per channel (see bn_finalize)
      if (active) {
#pragma unroll
        for (int e = 0; e < VEC; ++e) red[er0 * BN + ecv * VEC + e] = s1[e];
      }
      __syncthreads();
      for (int c = tid; active && c < BN; c += NT) {
        float sm = 0.f;
        for (int i = 0; i < ERPP; ++i) sm += red[i * BN + c];
        bmean[c] = nrows > 0 ? sm / (float)nrows : 0.f;
        const int col = n0 + c;
        if (col < a.Cout) {
          const long prow = (TILE_W ? mtile : xcd_slot(mtile, a.stats_R / NH)) * NH + h;
          a.stats[((long)col * 3 + 0) * a.stats_R + prow] = sm;
          a.stats[((long)col * 3 + 2) * a.stats_R + prow] = (float)nrows;
        }
      }
      __syncthreads();
      float q[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) q[e] = 0.f;
      for (int r = er0; active && r < nrows; r += ERPP) {
        float f[VEC];
        unpack16<T>(*reinterpret_cast<const typename Vec16<T>::type*>(&Cs[r * LDC + ecv * VEC]), f);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const float d = f[e] - bmean[ecv * VEC + e];
          q[e] += d * d;
        }
      }
      if (active) {
#pragma unroll
        for (int e = 0; e < VEC; ++e) red[er0 * BN + ecv * VEC + e] = q[e];
      }
      __syncthreads();
      for (int c = tid; active && c < BN; c += NT) {
        float qq = 0.f;
        for (int i = 0; i < ERPP; ++i) qq += red[i * BN + c];
        const int col = n0 + c;
        if (col < a.Cout) {
          const long prow = (TILE_W ? mtile : xcd_slot(mtile, a.stats_R / NH)) * NH + h;
          a.stats[((long)col * 3 + 1) * a.stats_R + prow] = qq;
        }
      }
    }
}


// ---- folded BN finalize (hgk_conv_fwd_fold), shared by the all-ahead implicit GEMM and the
// image-tile kernel: every workgroup merges the producer's channel-major partials [Cin][3][rows]
// of its input BN in fp64 (one thread per channel, two per channel when Cin <= NT / 2) ----
template <int FV>
struct FoldRegs {
  float4 fsum[FV], fm2[FV], fcnt[FV];
  float fg, fb;
  bool ftwo;
  int fh, fc, fstep;
};

template <int FV>
__device__ __forceinline__ void fold_setup(const ConvFwdArgs& a, bool fold, int tid, int NT,
                                           FoldRegs<FV>& r) {
  r.fg = 1.f;
  r.fb = 0.f;
  r.ftwo = fold && 2 * a.Cin <= NT;
  r.fh = r.ftwo && tid >= a.Cin ? 1 : 0;
  // clamped: with Cin < NT / 2 the threads past 2 Cin compute a copy of the last channel's
  // half (never published or staged) instead of reading past the partials
  r.fc = min(r.fh ? tid - a.Cin : tid, a.Cin - 1);
  r.fstep = r.ftwo ? 2 : 1;
}

// this thread's share of its channel's partial rows (sum | M2 | n runs, 16-B loads, clamped);
// issue only — fold_merge consumes them. PRED: skip the row quads past this thread's share
// (wave-uniform: the two threads of a channel sit in different waves) instead of re-loading the
// last one — fewer load instructions where the issue rate bounds the prologue
template <int FV, bool PRED = false>
__device__ __forceinline__ void fold_issue(const ConvFwdArgs& a, FoldRegs<FV>& r) {
  const int nv = a.fold_rows >> 2;
  const int myq = (nv - r.fh + r.fstep - 1) / r.fstep;
  const float4* p = reinterpret_cast<const float4*>(a.fold_part + (long)r.fc * 3 * a.fold_rows);
#pragma unroll
  for (int j = 0; j < FV; ++j) {
    if (PRED && j >= myq) break;
    const int jj = min(j * r.fstep + r.fh, nv - 1);
    r.fsum[j] = p[jj];
    r.fm2[j] = p[nv + jj];
    r.fcnt[j] = p[2 * nv + jj];
  }
  if (a.fold_gamma) r.fg = a.fold_gamma[r.fc];
  if (a.fold_beta) r.fb = a.fold_beta[r.fc];
}

// mean = sum S / M, M2 = sum (M2_r + n_r (S_r / n_r - mean)^2), in fp64 -> this thread's
// channel's scale / shift; `publish`: also write mean | invstd | scale | shift and the fp64
// running-statistics record. Workgroup-uniform call (barriers when two threads share a channel).
template <int FV>
__device__ __forceinline__ void fold_merge(const ConvFwdArgs& a, const FoldRegs<FV>& r, int tid,
                                           double* sFold, bool publish, float& scale, float& shift) {
  const int fh = r.fh, fstep = r.fstep;
  const int nv = a.fold_rows >> 2;
  const int myq = (nv - fh + fstep - 1) / fstep;  // row quads of this thread
  // four independent accumulators (one per float4 lane): short dependent fp64 chains
  double S4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 0; j < FV; ++j) {
    if (j < myq) {
      S4[0] += (double)r.fsum[j].x; S4[1] += (double)r.fsum[j].y;
      S4[2] += (double)r.fsum[j].z; S4[3] += (double)r.fsum[j].w;
    }
  }
  double S = (S4[0] + S4[1]) + (S4[2] + S4[3]);
  if (r.ftwo) {  // the pair's halves, in a fixed order (fh 0 first)
    sFold[tid] = S;
    __syncthreads();
    S = fh ? sFold[tid - a.Cin] + S : S + sFold[tid + a.Cin];
  }
  const double M = (double)a.fold_M;
  const double mu = S / M;
  // sum over rows of M2_r + n_r (S_r / n_r - mu)^2; rows of equal count n0 (every full tile):
  // sum M2_r + (sum (S_r - n0 mu)^2) / n0 — one division instead of one per row
  const float n0 = r.fcnt[0].x;
  bool same = n0 > 0.f;
#pragma unroll
  for (int j = 0; j < FV; ++j)
    if (j < myq)
      same = same && r.fcnt[j].x == n0 && r.fcnt[j].y == n0 && r.fcnt[j].z == n0 && r.fcnt[j].w == n0;
  double Q4[4] = {0.0, 0.0, 0.0, 0.0};
  double R4[4] = {0.0, 0.0, 0.0, 0.0};
  const double nm = (double)n0 * mu;
  auto addq = [&](int e, float s_, float q_, float n_) __attribute__((always_inline)) {
    if (same) {
      const double d = (double)s_ - nm;
      Q4[e] += (double)q_;
      R4[e] += d * d;
    } else {
      const double d = n_ > 0.f ? (double)s_ / (double)n_ - mu : 0.0;
      Q4[e] += (double)q_ + (double)n_ * d * d;
    }
  };
#pragma unroll
  for (int j = 0; j < FV; ++j) {
    if (j < myq) {
      addq(0, r.fsum[j].x, r.fm2[j].x, r.fcnt[j].x);
      addq(1, r.fsum[j].y, r.fm2[j].y, r.fcnt[j].y);
      addq(2, r.fsum[j].z, r.fm2[j].z, r.fcnt[j].z);
      addq(3, r.fsum[j].w, r.fm2[j].w, r.fcnt[j].w);
    }
  }
  double Q = (Q4[0] + Q4[1]) + (Q4[2] + Q4[3]);
  if (same) Q += ((R4[0] + R4[1]) + (R4[2] + R4[3])) / (double)n0;
  if (r.ftwo) {
    __syncthreads();  // every read of the S exchange is done
    sFold[tid] = Q;
    __syncthreads();
    Q = fh ? sFold[tid - a.Cin] + Q : Q + sFold[tid + a.Cin];
  }
  const double var = Q / M;
  const float is = (float)(1.0 / sqrt(var + (double)a.fold_eps));
  scale = r.fg * is;
  shift = r.fb - (float)mu * scale;
  if (publish && tid < a.Cin) {
    const int C = a.Cin;
    a.fold_stat[tid] = (float)mu;
    a.fold_stat[C + tid] = is;
    a.fold_stat[2 * C + tid] = scale;
    a.fold_stat[3 * C + tid] = shift;
    a.fold_rec[tid] = mu;
    a.fold_rec[C + tid] = a.fold_M > 1 ? Q / (M - 1.0) : var;
  }
}

// streaming 1x1 path (hgk_conv_ring.hip): shape check and launch of one convolution or a twin pair
// (a1 != nullptr: the second segment, same weights)
bool ring_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1 = nullptr);
int launch_ring(hipStream_t st, ConvFwdArgs& a0, ConvFwdArgs* a1, int* rows0, int* rows1);
// row-streaming 3x3 path (hgk_conv_row3.hip): the 128 -> 128 3x3 at the 64x64 / 32x32 levels
bool row3_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1 = nullptr);
int launch_row3(hipStream_t st, ConvFwdArgs& a0, ConvFwdArgs* a1, int* rows0, int* rows1);
// image-tile path (hgk_conv_img.hip): 1x1 and 3x3 at the small levels, 64 output pixels of whole
// images / row strips per workgroup, everything staged in one burst (folds a BN finalize too)
bool img_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1 = nullptr);
int launch_img(hipStream_t st, ConvFwdArgs& a0, ConvFwdArgs* a1, int* rows0, int* rows1);
// the 7x7 / stride-2 stem over the channel-padded input (hgk_conv_stem.hip): one output row per
// workgroup, weights in registers
bool stem_ok(const ConvFwdArgs& a);
int launch_stem(hipStream_t st, ConvFwdArgs& a, int* rows_out);

// the LDS-DMA ring weight gradient of big multi-use 1x1 bf16 weights (hgk_wgrad_ring.hip)
bool wgrad_ring_shape_ok(int Cout, int Cin);
int launch_wgrad_ring(hipStream_t st, const void* const* xs, const void* const* dys,
                      const float* const* pscale, const float* const* pshift, const int* prelu,
                      const long* Ms, int nsrc, float* slab, float* slab_b, int slab_cap, int s_init,
                      int Cout, int Cin);

}  // namespace hgk
