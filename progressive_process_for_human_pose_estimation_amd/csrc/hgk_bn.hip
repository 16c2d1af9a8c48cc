// Train-mode BatchNorm2d (+ fused ReLU) statistics, finalisation and backward, NHWC.
// Reference semantics: torch.nn.BatchNorm2d as used by try_with_torch.py:184,187,190,249 —
// batch mean / biased variance to normalise, unbiased variance into running_var, momentum 0.1,
// eps 1e-5; ReLU(True) after it (:185). All cross-workgroup sums go through per-workgroup
// partial slabs reduced in a fixed order (fp64 in the finalisers).
#include <algorithm>

#include "hgk_common.h"

namespace hgk {

static constexpr int kStatsNT = 256;
static constexpr int kRowU = 4;  // rows whose loads a thread keeps in flight together
static constexpr int kMaxRows = 8192;

struct RowPlan {
  int tpr, rpp, G;
  long rows_per_block;
};

#ifndef HGK_APPLY_PASSES
#define HGK_APPLY_PASSES 8
#endif
// passes per block of the BN-backward apply kernels (4 = one batch of kRowU rows per thread;
// 8 = two batches, the second's loads overlapping the first's stores)
static constexpr int kApplyPasses = HGK_APPLY_PASSES;

template <typename T>
static bool row_plan(long M, int C, RowPlan& p, int passes = 4) {
  constexpr int VEC = Vec16<T>::N;
  if (C % VEC != 0) return false;
  p.tpr = C / VEC;
  if (kStatsNT % p.tpr != 0) return false;
  p.rpp = kStatsNT / p.tpr;
  // >= `passes` passes per block (4 = one batch of kRowU rows in flight per thread), <= 2048
  // blocks
  long per = std::max<long>((long)p.rpp * passes, (M + 2047) / 2048);
  per = ((per + p.rpp - 1) / p.rpp) * p.rpp;
  p.G = (int)((M + per - 1) / per);
  p.rows_per_block = per;
  return true;
}

// Statistics partials, CHANNEL-major layout [C][3][G]: (sum, M2 about the block mean, count) of
// block b's rows at [c][.][b] (the conv epilogues write the same layout with G = their row count).
// Each thread accumulates its rows shifted by its first value (well conditioned), the threads of
// a channel are merged with Chan's parallel rule, and bn_finalize merges the blocks the same way
// in fp64: no E[x^2]-E[x]^2 cancellation even for a BN over 2 values (1x1 innermost level, N=2).
template <typename T>
__global__ __launch_bounds__(kStatsNT) void bn_stats_kernel(const T* __restrict__ x, long M, int C,
                                                            long rows_per_block, int tpr, int rpp,
                                                            float* __restrict__ partial) {
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [rpp][C][3]
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float k[VEC], s[VEC], q[VEC];
  int n = 0;
#pragma unroll
  for (int e = 0; e < VEC; ++e) { k[e] = 0.f; s[e] = 0.f; q[e] = 0.f; }
  if (r_begin + rp < r_end) unpack16<T>(load16(x + (r_begin + rp) * C + cv * VEC), k);
  typedef typename Vec16<T>::type V;
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    V v[kRowU];
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) v[u] = load16(x + r * C + cv * VEC);
    }
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      if (r0 + u * rpp >= r_end) break;
      float f[VEC];
      unpack16<T>(v[u], f);
      ++n;
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float d = f[e] - k[e];
        s[e] += d;
        q[e] += d * d;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    float* dst = &red[((long)rp * C + cv * VEC + e) * 3];
    const float mean = n ? k[e] + s[e] / (float)n : 0.f;
    dst[0] = (float)n;
    dst[1] = mean;
    dst[2] = n ? fmaxf(q[e] - s[e] * s[e] / (float)n, 0.f) : 0.f;
  }
  __syncthreads();
  const long slot = xcd_slot(blockIdx.x, gridDim.x);
  for (int c = tid; c < C; c += kStatsNT) {
    float na = 0.f, ma = 0.f, m2a = 0.f;
    for (int i = 0; i < rpp; ++i) {
      const float* src = &red[((long)i * C + c) * 3];
      const float nb = src[0];
      if (nb == 0.f) continue;
      const float nab = na + nb;
      const float delta = src[1] - ma;
      ma += delta * (nb / nab);
      m2a += src[2] + delta * delta * (na * nb / nab);
      na = nab;
    }
    // channel-major [C][3][G]
    partial[((long)c * 3 + 0) * gridDim.x + slot] = ma * na;
    partial[((long)c * 3 + 1) * gridDim.x + slot] = m2a;
    partial[((long)c * 3 + 2) * gridDim.x + slot] = na;
  }
}

// Finalisers: one WAVE per channel, its 64 lanes stride over the partial rows (4 rows in flight
// per lane), fp64 accumulation, a fixed-order wave shuffle tree — no LDS, no barriers. Rows above
// kFinDirect are first merged 64:1 by bn_partial_merge_kernel (coalesced, lane = channel), so a
// wave never walks more than kFinDirect strided rows. Per-channel parameters are loaded before the
// reduction so their latency overlaps it; the Chan weights nb/(na+nb) are fp32 quotients (counts
// are exact integers in fp32; a 1-ulp weight moves the merged mean by 6e-8 of a between-block
// difference), the accumulators stay fp64.
static constexpr int kFinWaves = 4;
static constexpr int kFinDirect = 256;
static constexpr int kMergeRows = 64;

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// (n, m, m2) += (nb, mb, m2b), Chan's rule. Branch-free (an empty operand has nb = m2b = 0 and
// a finite mb): a divergent branch here makes the compiler sink the operand loads into it and wait
// for each one separately.
__device__ __forceinline__ void chan_merge(double& n, double& m, double& m2, float nbf, double mb,
                                          double m2b) {
  const float nnf = (float)n + nbf;
  const double w = nbf > 0.f ? (double)(nbf / nnf) : 0.0;
  const double d = mb - m;
  m += d * w;
  m2 += m2b + d * d * (n * w);
  n += (double)nbf;
}

// level-2 partials: block (g, cg) merges rows [64g, 64g+64) of channels [64cg, 64cg+64) into row g.
// NV = 3: (sum, M2, n) statistics rows; NV = 2: (sum g, sum g*xhat) backward rows.
template <int NV>
__global__ __launch_bounds__(256) void bn_partial_merge_kernel(const float* __restrict__ partial,
                                                               int rows, int C,
                                                               float* __restrict__ out) {
  __shared__ double red[4][3][64];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const int r0 = blockIdx.x * kMergeRows;
  const int r1 = min(rows, r0 + kMergeRows);
  constexpr int PER = kMergeRows / 4;
  float v[PER][NV];
  // clamped, unconditional loads: a guarded load would make the compiler wait for each one
  const int cc = min(c, C - 1);
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int r = r0 + ph + 4 * u;
    const int rc = min(r, r1 - 1);
#pragma unroll
    for (int k = 0; k < NV; ++k) v[u][k] = partial[((long)rc * NV + k) * C + cc];
  }
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const bool ok = r0 + ph + 4 * u < r1 && c < C;
#pragma unroll
    for (int k = 0; k < NV; ++k) v[u][k] = ok ? v[u][k] : 0.f;
  }
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  if (NV == 3) {
#pragma unroll
    for (int u = 0; u < PER; ++u)
      chan_merge(a2, a0, a1, v[u][2], (double)v[u][0] / (double)fmaxf(v[u][2], 1.f), v[u][1]);
  } else {
#pragma unroll
    for (int u = 0; u < PER; ++u) { a0 += v[u][0]; a1 += v[u][1]; }
  }
  red[ph][0][lane] = a0; red[ph][1][lane] = a1; red[ph][2][lane] = a2;
  __syncthreads();
  if (ph != 0 || c >= C) return;
  for (int q = 1; q < 4; ++q) {
    if (NV == 3) {
      chan_merge(a2, a0, a1, (float)red[q][2][lane], red[q][0][lane], red[q][1][lane]);
    } else {
      a0 += red[q][0][lane]; a1 += red[q][1][lane];
    }
  }
  const long g = blockIdx.x;
  if (NV == 3) {
    out[(g * 3 + 0) * C + c] = (float)(a0 * a2);
    out[(g * 3 + 1) * C + c] = (float)a1;
    out[(g * 3 + 2) * C + c] = (float)a2;
  } else {
    out[(g * 2 + 0) * C + c] = (float)a0;
    out[(g * 2 + 1) * C + c] = (float)a1;
  }
}

__global__ __launch_bounds__(64 * kFinWaves) void bn_finalize_kernel(
    const float* __restrict__ partial, int rows, long M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* running_mean, float* running_var, float momentum,
    float eps, int training, float* mean, float* invstd, float* scale, float* shift) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * kFinWaves + (threadIdx.x >> 6);
  if (c >= C) return;  // whole wave exits together
  // parameter loads issued up front and unconditionally (a null pointer reads a valid stand-in
  // and the value is replaced): they overlap the reduction instead of serialising after it
  const float* any = training ? partial : running_mean;
  const float g0 = (gamma ? gamma : any)[c], b0 = (beta ? beta : any)[c];
  const float rm0 = (running_mean ? running_mean : any)[c];
  const float rv0 = (running_var ? running_var : any)[c];
  const float g = gamma ? g0 : 1.f, b = beta ? b0 : 0.f;
  const float rm = running_mean ? rm0 : 0.f, rv = running_var ? rv0 : 1.f;
  double mu, var;
  if (training) {
    // single pass: each lane Chan-merges its rows' (count, mean, M2); then a fixed-order wave
    // shuffle tree merges the lanes (lane 0's result is the one used -> deterministic)
    double n = 0.0, m = 0.0, m2 = 0.0;
    for (int r0 = lane; r0 < rows; r0 += 64 * 4) {
      float ps[4], pq[4], pn[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int rc = min(r0 + 64 * u, rows - 1);  // clamped: no per-load branch + wait
        ps[u] = partial[((long)c * 3 + 0) * rows + rc];
        pq[u] = partial[((long)c * 3 + 1) * rows + rc];
        pn[u] = partial[((long)c * 3 + 2) * rows + rc];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = r0 + 64 * u < rows;
        pn[u] = ok ? pn[u] : 0.f;
        pq[u] = ok ? pq[u] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        chan_merge(n, m, m2, pn[u], (double)ps[u] / (double)fmaxf(pn[u], 1.f), pq[u]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double nb = __shfl_xor(n, o, 64), mb = __shfl_xor(m, o, 64), qb = __shfl_xor(m2, o, 64);
      chan_merge(n, m, m2, (float)nb, mb, qb);
    }
    mu = m;
    var = m2 / (double)M;
    if (lane == 0 && running_mean) {
      const double unbiased = M > 1 ? m2 / (double)(M - 1) : var;
      running_mean[c] = (float)((1.0 - momentum) * rm + momentum * mu);
      running_var[c] = (float)((1.0 - momentum) * rv + momentum * unbiased);
    }
  } else {
    mu = rm;
    var = rv;
  }
  if (lane != 0) return;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = g * is;
  mean[c] = (float)mu;
  invstd[c] = is;
  scale[c] = sc;
  shift[c] = b - (float)mu * sc;
}

// Finalisers for many partial rows (rows > kFinDirect, the 64x64 / 32x32 levels): one WORKGROUP
// per channel, so no separate merge launch. Each thread walks rows tid, tid + kFinWgNT, ... with
// kFinWgU rows' loads in flight (2048 rows = one round trip), then a fixed-order wave shuffle tree
// and a fixed-order merge of the 4 wave results (deterministic).
static constexpr int kFinWgNT = 256;
static constexpr int kFinWgU = 8;

__global__ __launch_bounds__(kFinWgNT) void bn_finalize_wg_kernel(
    const float* __restrict__ partial, int rows, long M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* running_mean, float* running_var, float momentum,
    float eps, float* mean, float* invstd, float* scale, float* shift) {
  __shared__ double red[3][kFinWgNT / 64];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float g0 = (gamma ? gamma : partial)[c], b0 = (beta ? beta : partial)[c];
  const float rm0 = (running_mean ? running_mean : partial)[c];
  const float rv0 = (running_var ? running_var : partial)[c];
  double n = 0.0, m = 0.0, m2 = 0.0;
  for (int r0 = tid; r0 < rows; r0 += kFinWgNT * kFinWgU) {
    float ps[kFinWgU], pq[kFinWgU], pn[kFinWgU];
#pragma unroll
    for (int u = 0; u < kFinWgU; ++u) {
      const int rc = min(r0 + kFinWgNT * u, rows - 1);
      ps[u] = partial[((long)c * 3 + 0) * rows + rc];
      pq[u] = partial[((long)c * 3 + 1) * rows + rc];
      pn[u] = partial[((long)c * 3 + 2) * rows + rc];
    }
#pragma unroll
    for (int u = 0; u < kFinWgU; ++u) {
      const bool ok = r0 + kFinWgNT * u < rows;
      pn[u] = ok ? pn[u] : 0.f;
      pq[u] = ok ? pq[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kFinWgU; ++u)
      chan_merge(n, m, m2, pn[u], (double)ps[u] / (double)fmaxf(pn[u], 1.f), pq[u]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double nb = __shfl_xor(n, o, 64), mb = __shfl_xor(m, o, 64), qb = __shfl_xor(m2, o, 64);
    chan_merge(n, m, m2, (float)nb, mb, qb);
  }
  if (lane == 0) { red[0][wv] = n; red[1][wv] = m; red[2][wv] = m2; }
  __syncthreads();
  if (tid != 0) return;
  for (int q = 1; q < kFinWgNT / 64; ++q) chan_merge(n, m, m2, (float)red[0][q], red[1][q], red[2][q]);
  const double mu = m, var = m2 / (double)M;
  if (running_mean) {
    const double unbiased = M > 1 ? m2 / (double)(M - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * rm0 + momentum * mu);
    running_var[c] = (float)((1.0 - momentum) * rv0 + momentum * unbiased);
  }
  const float g = gamma ? g0 : 1.f, b = beta ? b0 : 0.f;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = g * is;
  mean[c] = (float)mu;
  invstd[c] = is;
  scale[c] = sc;
  shift[c] = b - (float)mu * sc;
}

// backward partials: g = dA * [y*scale+shift > 0]; sum g, sum g*xhat
template <typename T>
__global__ __launch_bounds__(kStatsNT) void bn_bwd_reduce_kernel(
    const T* __restrict__ dA, const T* __restrict__ y, long M, int C, long rows_per_block, int tpr,
    int rpp, const float* __restrict__ scale, const float* __restrict__ shift, int relu,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ partial) {
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float sc[VEC], sh[VEC], mu[VEC], is[VEC], s[VEC], q[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int c = cv * VEC + e;
    sc[e] = scale[c]; sh[e] = shift[c]; mu[e] = mean[c]; is[e] = invstd[c];
    s[e] = 0.f; q[e] = 0.f;
  }
  typedef typename Vec16<T>::type V;
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    V vd[kRowU], vy[kRowU];
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) {
        vd[u] = load16(dA + r * C + cv * VEC);
        vy[u] = load16(y + r * C + cv * VEC);
      }
    }
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      if (r0 + u * rpp >= r_end) break;
      float fd[VEC], fy[VEC];
      unpack16<T>(vd[u], fd);
      unpack16<T>(vy[u], fy);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float g = fd[e];
        if (relu && !(fmaf(fy[e], sc[e], sh[e]) > 0.f)) g = 0.f;
        s[e] += g;
        q[e] += g * ((fy[e] - mu[e]) * is[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    red[((long)rp * C + cv * VEC + e) * 2 + 0] = s[e];
    red[((long)rp * C + cv * VEC + e) * 2 + 1] = q[e];
  }
  __syncthreads();
  for (int c = tid; c < C; c += kStatsNT) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < rpp; ++i) {
      a += red[((long)i * C + c) * 2 + 0];
      b += red[((long)i * C + c) * 2 + 1];
    }
    partial[((long)blockIdx.x * 2 + 0) * C + c] = a;
    partial[((long)blockIdx.x * 2 + 1) * C + c] = b;
  }
}

// dgamma += sum g*xhat, dbeta += sum g, and the apply coefficients of channel c
__device__ __forceinline__ void bn_bwd_coef(int c, int C, long M, int training, double sc, float mu,
                                            double is, double sg, double sgx, float dg0, float db0,
                                            float* dgamma, float* dbeta, float* coef) {
  if (dgamma) dgamma[c] = dg0 + (float)sgx;
  if (dbeta) dbeta[c] = db0 + (float)sg;
  double c1 = 0.0, c2 = 0.0;
  if (training) {
    // dy = scale * (g - mean(g) - xhat * mean(g*xhat)),  xhat = (y - mean) * invstd
    //    = coef0*g + coef1*(y - mean) + coef2   (centred form: no cancellation when y ~ mean)
    c1 = -sc * is * sgx / (double)M;
    c2 = -sc * sg / (double)M;
  }
  coef[c] = (float)sc;
  coef[C + c] = (float)c1;
  coef[2 * C + c] = (float)c2;
  coef[3 * C + c] = mu;
}

__global__ __launch_bounds__(64 * kFinWaves) void bn_bwd_finalize_kernel(
    const float* __restrict__ partial, int rows, long M, int C, const float* __restrict__ scale,
    const float* __restrict__ mean, const float* __restrict__ invstd, int training, float* dgamma,
    float* dbeta, float* coef) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * kFinWaves + (threadIdx.x >> 6);
  if (c >= C) return;
  const double sc = scale[c];
  const float mu = mean[c];
  const double is = invstd[c];
  const float dg0 = (dgamma ? dgamma : scale)[c], db0 = (dbeta ? dbeta : scale)[c];
  double sg = 0.0, sgx = 0.0;
  for (int r0 = lane; r0 < rows; r0 += 64 * 4) {
    float a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int rc = min(r0 + 64 * u, rows - 1);
      a[u] = partial[((long)rc * 2 + 0) * C + c];
      b[u] = partial[((long)rc * 2 + 1) * C + c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = r0 + 64 * u < rows;
      a[u] = ok ? a[u] : 0.f;
      b[u] = ok ? b[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { sg += (double)a[u]; sgx += (double)b[u]; }
  }
  sg = wave_sum_d(sg);
  sgx = wave_sum_d(sgx);
  if (lane != 0) return;
  bn_bwd_coef(c, C, M, training, sc, mu, is, sg, sgx, dg0, db0, dgamma, dbeta, coef);
}

// bn_bwd_finalize_wg_kernel's sums of channel c by the whole workgroup (thread 0: the result)
__device__ __forceinline__ void bwd_wg_merge(const float* __restrict__ partial, int rows, int C,
                                             int c, int tid, double (*red)[kFinWgNT / 64],
                                             double& sg_out, double& sgx_out) {
  const int lane = tid & 63, wv = tid >> 6;
  double sg = 0.0, sgx = 0.0;
  for (int r0 = tid; r0 < rows; r0 += kFinWgNT * kFinWgU) {
    float a[kFinWgU], b[kFinWgU];
#pragma unroll
    for (int u = 0; u < kFinWgU; ++u) {
      const int rc = min(r0 + kFinWgNT * u, rows - 1);
      a[u] = partial[((long)rc * 2 + 0) * C + c];
      b[u] = partial[((long)rc * 2 + 1) * C + c];
    }
#pragma unroll
    for (int u = 0; u < kFinWgU; ++u) {
      const bool ok = r0 + kFinWgNT * u < rows;
      sg += ok ? (double)a[u] : 0.0;
      sgx += ok ? (double)b[u] : 0.0;
    }
  }
  sg = wave_sum_d(sg);
  sgx = wave_sum_d(sgx);
  if (lane == 0) { red[0][wv] = sg; red[1][wv] = sgx; }
  __syncthreads();
  if (tid == 0) {
    sg = red[0][0]; sgx = red[1][0];
    for (int q = 1; q < kFinWgNT / 64; ++q) { sg += red[0][q]; sgx += red[1][q]; }
  }
  sg_out = sg;
  sgx_out = sgx;
}

// bn_bwd_finalize for many partial rows: one workgroup per channel (see bn_finalize_wg_kernel)
__global__ __launch_bounds__(kFinWgNT) void bn_bwd_finalize_wg_kernel(
    const float* __restrict__ partial, int rows, long M, int C, const float* __restrict__ scale,
    const float* __restrict__ mean, const float* __restrict__ invstd, int training, float* dgamma,
    float* dbeta, float* coef) {
  __shared__ double red[2][kFinWgNT / 64];
  const int c = blockIdx.x, tid = threadIdx.x;
  const double sc = scale[c];
  const float mu = mean[c];
  const double is = invstd[c];
  const float dg0 = (dgamma ? dgamma : scale)[c], db0 = (dbeta ? dbeta : scale)[c];
  double sg, sgx;
  bwd_wg_merge(partial, rows, C, c, tid, red, sg, sgx);
  if (tid != 0) return;
  bn_bwd_coef(c, C, M, training, sc, mu, is, sg, sgx, dg0, db0, dgamma, dbeta, coef);
}

// Several BatchNorms' backward finalizes (each > kFinDirect partial rows) in one launch
// (hgk_bn_bwd_finalize_multi): a workgroup per (job, channel), bn_bwd_finalize_wg_kernel's sums.
struct BnbFinJobK {
  const float* partial;
  int rows;
  long M;
  int C;
  const float *scale, *mean, *invstd;
  int training;
  float *dgamma, *dbeta, *coef;
  int blk0;
};
struct BnbFinMultiArgs {
  BnbFinJobK j[8];
  int n;
};

__global__ __launch_bounds__(kFinWgNT) void bn_bwd_finalize_multi_kernel(BnbFinMultiArgs a) {
  __shared__ double red[2][kFinWgNT / 64];
  int q = 0;
  while (q + 1 < a.n && (int)blockIdx.x >= a.j[q + 1].blk0) ++q;
  const BnbFinJobK& J = a.j[q];
  const int c = blockIdx.x - J.blk0, tid = threadIdx.x;
  const double sc = J.scale[c];
  const float mu = J.mean[c];
  const double is = J.invstd[c];
  const float dg0 = (J.dgamma ? J.dgamma : J.scale)[c], db0 = (J.dbeta ? J.dbeta : J.scale)[c];
  double sg, sgx;
  bwd_wg_merge(J.partial, J.rows, J.C, c, tid, red, sg, sgx);
  if (tid != 0) return;
  bn_bwd_coef(c, J.C, J.M, J.training, sc, mu, is, sg, sgx, dg0, db0, J.dgamma, J.dbeta, J.coef);
}

// Apply kernels: the same row plan as the reductions — a thread owns VEC channels for the whole
// launch, so its per-channel constants live in registers; rows are streamed with 16-B accesses.
template <typename T>
__global__ __launch_bounds__(kStatsNT) HGK_WPE_BWDAPPLY void bn_bwd_apply_kernel(
    const T* __restrict__ dA, const T* __restrict__ y, long M, int C, long rows_per_block, int tpr,
    int rpp, const float* __restrict__ scale, const float* __restrict__ shift, int relu,
    const float* __restrict__ coef, const T* add, T* dy, int accumulate) {
  constexpr int VEC = Vec16<T>::N;
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float sc[VEC], sh[VEC], k0[VEC], k1[VEC], k2[VEC], mu[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int c = cv * VEC + e;
    sc[e] = scale[c]; sh[e] = shift[c];
    k0[e] = coef[c]; k1[e] = coef[C + c]; k2[e] = coef[2 * C + c]; mu[e] = coef[3 * C + c];
  }
  typedef typename Vec16<T>::type V;
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    V vd[kRowU], vy[kRowU], va[kRowU], vo[kRowU];
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) {
        const long off = r * C + cv * VEC;
        vd[u] = load16(dA + off);
        vy[u] = load16(y + off);
        if (add) va[u] = load16(add + off);
        if (accumulate) vo[u] = load16(dy + off);
      }
    }
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r >= r_end) break;
      float fd[VEC], fy[VEC], fa[VEC], fo[VEC], o[VEC];
      unpack16<T>(vd[u], fd);
      unpack16<T>(vy[u], fy);
      if (add) unpack16<T>(va[u], fa);
      if (accumulate) unpack16<T>(vo[u], fo);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float v = bnb_apply(fd[e], fy[e], sc[e], sh[e], k0[e], k1[e], k2[e], mu[e], relu);
        if (add) v += fa[e];
        if (accumulate) v += fo[e];
        o[e] = v;
      }
      store16(dy + r * C + cv * VEC, pack16<T>(o));
    }
  }
}

// bn_bwd_finalize + bn_bwd_apply in ONE launch for few partial rows (the <= 16x16 hourglass
// levels: 8..128 rows): every workgroup first reduces ALL partial rows itself — coalesced float4
// loads, thread t owns float4 column t % (C/2) of rows g, g+G, ... (G = 512/C groups), U loads in
// flight, fp64 sums, a fixed-order merge of the G group sums through LDS (identical in every
// workgroup, so deterministic) — then applies like bn_bwd_apply_kernel. Workgroup 0 alone
// accumulates dgamma / dbeta. Saves the finalize launch and its dependent round trip.
static constexpr int kFusedFinMaxRows = 128;
#ifndef HGK_FINAPPLY_U
#define HGK_FINAPPLY_U 8
#endif

template <typename T>
__global__ __launch_bounds__(kStatsNT) HGK_WPE_BWDAPPLY void bn_bwd_fin_apply_kernel(
    const float* __restrict__ partial, int rows, const float* __restrict__ mean,
    const float* __restrict__ invstd, int training, float* dgamma, float* dbeta,
    const T* __restrict__ dA, const T* __restrict__ y, long M, int C, long rows_per_block, int tpr,
    int rpp, const float* __restrict__ scale, const float* __restrict__ shift, int relu,
    const T* add, T* dy, int accumulate) {
  constexpr int VEC = Vec16<T>::N;
  constexpr int U = HGK_FINAPPLY_U;  // partial rows in flight per thread (16: measured 0.4 % slower)
  __shared__ double red[1024];        // [G][2C]
  __shared__ float scoef[4 * 512];   // [4][C]
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  typedef typename Vec16<T>::type V;
  V vd[kRowU], vy[kRowU], va[kRowU], vo[kRowU];
  auto load_batch = [&](long r0) {
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) {
        const long off = r * C + cv * VEC;
        vd[u] = load16(dA + off);
        vy[u] = load16(y + off);
        if (add) va[u] = load16(add + off);
        if (accumulate) vo[u] = load16(dy + off);
      }
    }
  };
  // the first batch of rows is loaded BEFORE the partial-row reduction: both round trips overlap
  load_batch(r_begin + rp);
  // per-channel constants, also before the reduction: this thread's VEC apply channels and the
  // (up to 2) channels whose coefficients it computes
  float sc[VEC], sh[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) { sc[e] = scale[cv * VEC + e]; sh[e] = shift[cv * VEC + e]; }
  float csc[2], cis[2], cmu[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = min(tid + k * kStatsNT, C - 1);
    csc[k] = scale[c]; cis[k] = invstd[c]; cmu[k] = mean[c];
  }
  float dg0[2] = {0.f, 0.f}, db0[2] = {0.f, 0.f};
  if (blockIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = min(tid + k * kStatsNT, C - 1);
      if (dgamma) dg0[k] = dgamma[c];
      if (dbeta) db0[k] = dbeta[c];
    }
  }
  {
    const int F4 = C >> 1;            // float4 columns per partial row
    const int G = kStatsNT / F4;
    const int q = tid % F4, g = tid / F4;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    const float4* p4 = reinterpret_cast<const float4*>(partial);
    for (int r0 = g; r0 < rows; r0 += G * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p4[(long)min(r0 + G * u, rows - 1) * F4 + q];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = r0 + G * u < rows;
        a0 += ok ? (double)v[u].x : 0.0;
        a1 += ok ? (double)v[u].y : 0.0;
        a2 += ok ? (double)v[u].z : 0.0;
        a3 += ok ? (double)v[u].w : 0.0;
      }
    }
    double* rr = red + g * 2 * C + 4 * q;
    rr[0] = a0; rr[1] = a1; rr[2] = a2; rr[3] = a3;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = tid + k * kStatsNT;
      if (c >= C) break;
      double sg = 0.0, sgx = 0.0;
      for (int gg = 0; gg < G; ++gg) { sg += red[gg * 2 * C + c]; sgx += red[gg * 2 * C + C + c]; }
      const double sc = csc[k], is = cis[k];
      const float mu = cmu[k];
      if (blockIdx.x == 0) {
        if (dgamma) dgamma[c] = dg0[k] + (float)sgx;
        if (dbeta) dbeta[c] = db0[k] + (float)sg;
      }
      double c1 = 0.0, c2 = 0.0;
      if (training) {
        c1 = -sc * is * sgx / (double)M;
        c2 = -sc * sg / (double)M;
      }
      scoef[c] = (float)sc;
      scoef[C + c] = (float)c1;
      scoef[2 * C + c] = (float)c2;
      scoef[3 * C + c] = mu;
    }
    __syncthreads();
  }
  float k0[VEC], k1[VEC], k2[VEC], mu[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int c = cv * VEC + e;
    k0[e] = scoef[c]; k1[e] = scoef[C + c]; k2[e] = scoef[2 * C + c]; mu[e] = scoef[3 * C + c];
  }
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    if (r0 != r_begin + rp) load_batch(r0);
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r >= r_end) break;
      float fd[VEC], fy[VEC], fa[VEC], fo[VEC], o[VEC];
      unpack16<T>(vd[u], fd);
      unpack16<T>(vy[u], fy);
      if (add) unpack16<T>(va[u], fa);
      if (accumulate) unpack16<T>(vo[u], fo);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float v = bnb_apply(fd[e], fy[e], sc[e], sh[e], k0[e], k1[e], k2[e], mu[e], relu);
        if (add) v += fa[e];
        if (accumulate) v += fo[e];
        o[e] = v;
      }
      store16(dy + r * C + cv * VEC, pack16<T>(o));
    }
  }
}

// the backward of a summed BN pair (hgk_bn_bwd_pair): per side bn_bwd_fin_apply_kernel's
// coefficients (FIN) or hgk_bn_bwd_finalize's (coef), and both applies over ONE read of dA
struct BnbSideK {
  const void* y;
  const float *scale, *shift, *mean, *invstd;
  int relu;
  const float* partial;
  int rows;
  const float* coef;
  float *dgamma, *dbeta;
  void* dy;
};

// bn_bwd_fin_apply_kernel's prologue for one side: scoef[4][C] (coef0..2, mean), dgamma / dbeta
// accumulated by workgroup 0; every workgroup computes the same values in the same order
template <int U>
__device__ __forceinline__ void bnb_side_coef(const BnbSideK& s, long M, int C, int training,
                                              double* red, float* scoef) {
  const int tid = threadIdx.x;
  float csc[2], cis[2], cmu[2], dg0[2] = {0.f, 0.f}, db0[2] = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = min(tid + k * kStatsNT, C - 1);
    csc[k] = s.scale[c]; cis[k] = s.invstd[c]; cmu[k] = s.mean[c];
    if (blockIdx.x == 0) {
      if (s.dgamma) dg0[k] = s.dgamma[c];
      if (s.dbeta) db0[k] = s.dbeta[c];
    }
  }
  const int F4 = C >> 1, G = kStatsNT / F4;
  const int q = tid % F4, g = tid / F4;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  const float4* p4 = reinterpret_cast<const float4*>(s.partial);
  for (int r0 = g; r0 < s.rows; r0 += G * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p4[(long)min(r0 + G * u, s.rows - 1) * F4 + q];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = r0 + G * u < s.rows;
      a0 += ok ? (double)v[u].x : 0.0;
      a1 += ok ? (double)v[u].y : 0.0;
      a2 += ok ? (double)v[u].z : 0.0;
      a3 += ok ? (double)v[u].w : 0.0;
    }
  }
  double* rr = red + g * 2 * C + 4 * q;
  rr[0] = a0; rr[1] = a1; rr[2] = a2; rr[3] = a3;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = tid + k * kStatsNT;
    if (c >= C) break;
    double sg = 0.0, sgx = 0.0;
    for (int gg = 0; gg < G; ++gg) { sg += red[gg * 2 * C + c]; sgx += red[gg * 2 * C + C + c]; }
    const double sc = csc[k], is = cis[k];
    if (blockIdx.x == 0) {
      if (s.dgamma) s.dgamma[c] = dg0[k] + (float)sgx;
      if (s.dbeta) s.dbeta[c] = db0[k] + (float)sg;
    }
    double c1 = 0.0, c2 = 0.0;
    if (training) {
      c1 = -sc * is * sgx / (double)M;
      c2 = -sc * sg / (double)M;
    }
    scoef[c] = (float)sc;
    scoef[C + c] = (float)c1;
    scoef[2 * C + c] = (float)c2;
    scoef[3 * C + c] = cmu[k];
  }
  __syncthreads();  // red is reused by the next side
}

template <typename T, bool FIN>
__global__ __launch_bounds__(kStatsNT) HGK_WPE_BWDAPPLY void bn_bwd_pair_kernel(
    const T* __restrict__ dA, BnbSideK A, BnbSideK B, long M, int C, int training,
    long rows_per_block, int tpr, int rpp) {
  constexpr int VEC = Vec16<T>::N;
  __shared__ double red[1024];
  // both sides' per-channel constants [side][k0 | k1 | k2 | mean | scale | shift][C]: read per
  // row batch, one side at a time (held in registers for both sides the kernel needed 256 VGPRs
  // and ran one wave per SIMD)
  __shared__ __attribute__((aligned(16))) float sp[2][6 * 512];
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  typedef typename Vec16<T>::type V;
  V vd[kRowU], vy[2][kRowU];
  const T* const ys[2] = {reinterpret_cast<const T*>(A.y), reinterpret_cast<const T*>(B.y)};
  T* const dys[2] = {reinterpret_cast<T*>(A.dy), reinterpret_cast<T*>(B.dy)};
  auto load_batch = [&](long r0) {
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) {
        const long off = r * C + cv * VEC;
        vd[u] = load16(dA + off);
        vy[0][u] = load16(ys[0] + off);
        vy[1][u] = load16(ys[1] + off);
      }
    }
  };
  load_batch(r_begin + rp);
  if constexpr (FIN) {
    bnb_side_coef<HGK_FINAPPLY_U>(A, M, C, training, red, sp[0]);
    bnb_side_coef<HGK_FINAPPLY_U>(B, M, C, training, red, sp[1]);
  } else {
    for (int i = tid; i < 4 * C; i += kStatsNT) { sp[0][i] = A.coef[i]; sp[1][i] = B.coef[i]; }
  }
  for (int c = tid; c < C; c += kStatsNT) {
    sp[0][4 * C + c] = A.scale[c]; sp[0][5 * C + c] = A.shift[c];
    sp[1][4 * C + c] = B.scale[c]; sp[1][5 * C + c] = B.shift[c];
  }
  __syncthreads();
  const int relu[2] = {A.relu, B.relu};
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    if (r0 != r_begin + rp) load_batch(r0);
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      float k0[VEC], k1[VEC], k2[VEC], mu[VEC], sc[VEC], sh[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const int c = cv * VEC + e;
        k0[e] = sp[sd][c]; k1[e] = sp[sd][C + c]; k2[e] = sp[sd][2 * C + c];
        mu[e] = sp[sd][3 * C + c]; sc[e] = sp[sd][4 * C + c]; sh[e] = sp[sd][5 * C + c];
      }
#pragma unroll
      for (int u = 0; u < kRowU; ++u) {
        const long r = r0 + u * rpp;
        if (r >= r_end) break;
        float fd[VEC], fy[VEC], o[VEC];
        unpack16<T>(vd[u], fd);
        unpack16<T>(vy[sd][u], fy);
#pragma unroll
        for (int e = 0; e < VEC; ++e)
          o[e] = bnb_apply(fd[e], fy[e], sc[e], sh[e], k0[e], k1[e], k2[e], mu[e], relu[sd]);
        store16(dys[sd] + r * C + cv * VEC, pack16<T>(o));
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kStatsNT) void bn_apply_kernel(
    const T* __restrict__ x, long M, int C, long rows_per_block, int tpr, int rpp,
    const float* __restrict__ scale, const float* __restrict__ shift, int relu, T* __restrict__ y) {
  constexpr int VEC = Vec16<T>::N;
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float sc[VEC], sh[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) { sc[e] = scale[cv * VEC + e]; sh[e] = shift[cv * VEC + e]; }
  typedef typename Vec16<T>::type V;
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    V v[kRowU];
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) v[u] = load16(x + r * C + cv * VEC);
    }
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r >= r_end) break;
      float f[VEC];
      unpack16<T>(v[u], f);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float t = f[e] * sc[e] + sh[e];
        f[e] = relu ? fmaxf(t, 0.f) : t;
      }
      store16(y + r * C + cv * VEC, pack16<T>(f));
    }
  }
}

// --------------------------------------------------------------------------------------------
// A BN pair whose outputs are summed (hgk_bn_apply2_add / hgk_bn_bwd_reduce2): hourglass_compare's
// block output bn4(y3) + bn_ds(s). Each side's arithmetic is bn_apply_kernel's (forward) /
// bn_bwd_reduce_kernel's (backward) and the sum is add_kernel's; the statistics of the sum follow
// bn_stats_kernel's row plan and per-thread order exactly, so the results are bitwise those of
// the separate passes, with one read of each operand and one write.
// --------------------------------------------------------------------------------------------
struct BnSideK {
  const void* y;
  const float *scale, *shift, *mean, *invstd;
  int relu;
  float* partial;
};

template <typename T>
__global__ __launch_bounds__(kStatsNT) void bn_apply2_add_kernel(BnSideK A, BnSideK B, T* __restrict__ out,
                                                                 long M, int C, long rows_per_block,
                                                                 int tpr, int rpp,
                                                                 float* __restrict__ partial) {
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [rpp][C][3]
  const T* __restrict__ ya = reinterpret_cast<const T*>(A.y);
  const T* __restrict__ yb = reinterpret_cast<const T*>(B.y);
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float sa[VEC], ha[VEC], sb[VEC], hb[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    sa[e] = A.scale[cv * VEC + e]; ha[e] = A.shift[cv * VEC + e];
    sb[e] = B.scale[cv * VEC + e]; hb[e] = B.shift[cv * VEC + e];
  }
  const bool stats = partial != nullptr;
  float k[VEC], s[VEC], q[VEC];
  int n = 0;
#pragma unroll
  for (int e = 0; e < VEC; ++e) { k[e] = 0.f; s[e] = 0.f; q[e] = 0.f; }
  typedef typename Vec16<T>::type V;
  bool first = true;
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    V va[kRowU], vb[kRowU];
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) {
        va[u] = load16(ya + r * C + cv * VEC);
        vb[u] = load16(yb + r * C + cv * VEC);
      }
    }
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r >= r_end) break;
      float fa[VEC], fb[VEC];
      unpack16<T>(va[u], fa);
      unpack16<T>(vb[u], fb);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float ta = fa[e] * sa[e] + ha[e];
        fa[e] = A.relu ? fmaxf(ta, 0.f) : ta;
        const float tb = fb[e] * sb[e] + hb[e];
        fb[e] = B.relu ? fmaxf(tb, 0.f) : tb;
      }
      // each BN output rounded as hgk_bn_apply stores it, then add_kernel's sum (+ 0 accumulate)
      float xa[VEC], xb[VEC];
      unpack16<T>(pack16<T>(fa), xa);
      unpack16<T>(pack16<T>(fb), xb);
#pragma unroll
      for (int e = 0; e < VEC; ++e) xa[e] += xb[e] + 0.f;
      const V vo = pack16<T>(xa);
      store16(out + r * C + cv * VEC, vo);
      if (stats) {
        float f[VEC];
        unpack16<T>(vo, f);
        if (first) {  // bn_stats_kernel's shift: this thread's first row
#pragma unroll
          for (int e = 0; e < VEC; ++e) k[e] = f[e];
          first = false;
        }
        ++n;
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const float d = f[e] - k[e];
          s[e] += d;
          q[e] += d * d;
        }
      }
    }
  }
  if (!stats) return;
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    float* dst = &red[((long)rp * C + cv * VEC + e) * 3];
    const float mean = n ? k[e] + s[e] / (float)n : 0.f;
    dst[0] = (float)n;
    dst[1] = mean;
    dst[2] = n ? fmaxf(q[e] - s[e] * s[e] / (float)n, 0.f) : 0.f;
  }
  __syncthreads();
  const long slot = xcd_slot(blockIdx.x, gridDim.x);
  for (int c = tid; c < C; c += kStatsNT) {
    float na = 0.f, ma = 0.f, m2a = 0.f;
    for (int i = 0; i < rpp; ++i) {
      const float* src = &red[((long)i * C + c) * 3];
      const float nb = src[0];
      if (nb == 0.f) continue;
      const float nab = na + nb;
      const float delta = src[1] - ma;
      ma += delta * (nb / nab);
      m2a += src[2] + delta * delta * (na * nb / nab);
      na = nab;
    }
    partial[((long)c * 3 + 0) * gridDim.x + slot] = ma * na;
    partial[((long)c * 3 + 1) * gridDim.x + slot] = m2a;
    partial[((long)c * 3 + 2) * gridDim.x + slot] = na;
  }
}

template <typename T>
__global__ __launch_bounds__(kStatsNT) void bn_bwd_reduce2_kernel(const T* __restrict__ dA, BnSideK A,
                                                                  BnSideK B, long M, int C,
                                                                  long rows_per_block, int tpr,
                                                                  int rpp) {
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [2][rpp][C][2]
  const T* __restrict__ ya = reinterpret_cast<const T*>(A.y);
  const T* __restrict__ yb = reinterpret_cast<const T*>(B.y);
  const int tid = threadIdx.x;
  const int cv = tid % tpr, rp = tid / tpr;
  const long r_begin = (long)blockIdx.x * rows_per_block;
  const long r_end = min(M, r_begin + rows_per_block);
  float sca[VEC], sha[VEC], mua[VEC], isa[VEC], s_a[VEC], q_a[VEC];
  float scb[VEC], shb[VEC], mub[VEC], isb[VEC], s_b[VEC], q_b[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int c = cv * VEC + e;
    sca[e] = A.scale[c]; sha[e] = A.shift[c]; mua[e] = A.mean[c]; isa[e] = A.invstd[c];
    scb[e] = B.scale[c]; shb[e] = B.shift[c]; mub[e] = B.mean[c]; isb[e] = B.invstd[c];
    s_a[e] = 0.f; q_a[e] = 0.f; s_b[e] = 0.f; q_b[e] = 0.f;
  }
  typedef typename Vec16<T>::type V;
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    V vd[kRowU], va[kRowU], vb[kRowU];
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) {
        vd[u] = load16(dA + r * C + cv * VEC);
        va[u] = load16(ya + r * C + cv * VEC);
        vb[u] = load16(yb + r * C + cv * VEC);
      }
    }
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      if (r0 + u * rpp >= r_end) break;
      float fd[VEC], fa[VEC], fb[VEC];
      unpack16<T>(vd[u], fd);
      unpack16<T>(va[u], fa);
      unpack16<T>(vb[u], fb);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float g = fd[e];
        if (A.relu && !(fmaf(fa[e], sca[e], sha[e]) > 0.f)) g = 0.f;
        s_a[e] += g;
        q_a[e] += g * ((fa[e] - mua[e]) * isa[e]);
        float h = fd[e];
        if (B.relu && !(fmaf(fb[e], scb[e], shb[e]) > 0.f)) h = 0.f;
        s_b[e] += h;
        q_b[e] += h * ((fb[e] - mub[e]) * isb[e]);
      }
    }
  }
  float* ra = red;
  float* rb = red + (long)rpp * C * 2;
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    ra[((long)rp * C + cv * VEC + e) * 2 + 0] = s_a[e];
    ra[((long)rp * C + cv * VEC + e) * 2 + 1] = q_a[e];
    rb[((long)rp * C + cv * VEC + e) * 2 + 0] = s_b[e];
    rb[((long)rp * C + cv * VEC + e) * 2 + 1] = q_b[e];
  }
  __syncthreads();
  for (int c = tid; c < C; c += kStatsNT) {
    float a = 0.f, b = 0.f, a2 = 0.f, b2 = 0.f;
    for (int i = 0; i < rpp; ++i) {
      a += ra[((long)i * C + c) * 2 + 0];
      b += ra[((long)i * C + c) * 2 + 1];
      a2 += rb[((long)i * C + c) * 2 + 0];
      b2 += rb[((long)i * C + c) * 2 + 1];
    }
    A.partial[((long)blockIdx.x * 2 + 0) * C + c] = a;
    A.partial[((long)blockIdx.x * 2 + 1) * C + c] = b;
    B.partial[((long)blockIdx.x * 2 + 0) * C + c] = a2;
    B.partial[((long)blockIdx.x * 2 + 1) * C + c] = b2;
  }
}

// --------------------------------------------------------------------------------------------
// Twin / deferred BatchNorm (hgk_bn_finalize_deferred, hgk_bn_running_update, hgk_bn_bwd_twin).
// An hourglass level's up-branch and down-branch blocks use ONE ResidualBlock (shared BN modules,
// try_with_torch.py:217-237); the engine runs them side by side, so each BN launch serves two
// independent uses ("segments"). Running statistics: the finaliser writes each use's (mean,
// unbiased variance) in fp64 to a record and hgk_bn_running_update applies the records in the
// reference's call order — the EMA is order dependent and the twin schedule interleaves uses.
// Every per-segment arithmetic step is the single-use kernels' own, so a twin launch is bitwise
// equal to the two single launches in segment order (dgamma / dbeta: segment 0 first).
// --------------------------------------------------------------------------------------------
struct BnDefSeg {
  const float* partial;
  int rows;
  long M;
  double* rec;  // [2][C]: mean | unbiased variance
  float* stat;  // [4][C]: mean | invstd | scale | shift
};
struct BnDefArgs {
  BnDefSeg s[2];
  int nseg, C;
  const float *gamma, *beta;
  float eps;
};

__device__ __forceinline__ void bn_def_out(const BnDefArgs& a, const BnDefSeg& s, int c, double m,
                                           double m2, float g, float b) {
  const double mu = m, var = m2 / (double)s.M;
  s.rec[c] = mu;
  s.rec[a.C + c] = s.M > 1 ? m2 / (double)(s.M - 1) : var;
  const float is = (float)(1.0 / sqrt(var + (double)a.eps));
  const float sc = g * is;
  s.stat[c] = (float)mu;
  s.stat[a.C + c] = is;
  s.stat[2 * a.C + c] = sc;
  s.stat[3 * a.C + c] = b - (float)mu * sc;
}

// bn_finalize_def_kernel's merge of channel c: every lane of the wave ends with the result
__device__ __forceinline__ void def_wave_merge(const float* partial, int rows, int c, int lane,
                                               double& n, double& m, double& m2) {
  n = 0.0; m = 0.0; m2 = 0.0;
  {
    for (int r0 = lane; r0 < rows; r0 += 64 * 4) {
      float ps[4], pq[4], pn[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int rc = min(r0 + 64 * u, rows - 1);
        ps[u] = partial[((long)c * 3 + 0) * rows + rc];
        pq[u] = partial[((long)c * 3 + 1) * rows + rc];
        pn[u] = partial[((long)c * 3 + 2) * rows + rc];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = r0 + 64 * u < rows;
        pn[u] = ok ? pn[u] : 0.f;
        pq[u] = ok ? pq[u] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        chan_merge(n, m, m2, pn[u], (double)ps[u] / (double)fmaxf(pn[u], 1.f), pq[u]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double nb = __shfl_xor(n, o, 64), mb = __shfl_xor(m, o, 64), qb = __shfl_xor(m2, o, 64);
      chan_merge(n, m, m2, (float)nb, mb, qb);
    }
  }
}

// wave per (channel, segment) (bn_finalize_kernel's merge)
__global__ __launch_bounds__(64 * kFinWaves) void bn_finalize_def_kernel(BnDefArgs a) {
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * kFinWaves + (threadIdx.x >> 6);
  const int q = wid / a.C, c = wid - q * a.C;
  if (q >= a.nseg) return;  // whole wave exits together
  const float g = a.gamma ? a.gamma[c] : 1.f, b = a.beta ? a.beta[c] : 0.f;
  const BnDefSeg& s = a.s[q];
  double n, m, m2;
  def_wave_merge(s.partial, s.rows, c, lane, n, m, m2);
  if (lane == 0) bn_def_out(a, s, c, m, m2, g, b);
}

// bn_finalize_def_wg_kernel's merge of channel c by the whole workgroup: thread 0 ends with the
// result (red: the kernel's LDS)
__device__ __forceinline__ void def_wg_merge(const float* partial, int rows, int c, int tid,
                                             double (*red)[kFinWgNT / 64], double& n, double& m,
                                             double& m2) {
  const int lane = tid & 63, wv = tid >> 6;
  n = 0.0; m = 0.0; m2 = 0.0;
  {
    for (int r0 = tid; r0 < rows; r0 += kFinWgNT * kFinWgU) {
      float ps[kFinWgU], pq[kFinWgU], pn[kFinWgU];
#pragma unroll
      for (int u = 0; u < kFinWgU; ++u) {
        const int rc = min(r0 + kFinWgNT * u, rows - 1);
        ps[u] = partial[((long)c * 3 + 0) * rows + rc];
        pq[u] = partial[((long)c * 3 + 1) * rows + rc];
        pn[u] = partial[((long)c * 3 + 2) * rows + rc];
      }
#pragma unroll
      for (int u = 0; u < kFinWgU; ++u) {
        const bool ok = r0 + kFinWgNT * u < rows;
        pn[u] = ok ? pn[u] : 0.f;
        pq[u] = ok ? pq[u] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kFinWgU; ++u)
        chan_merge(n, m, m2, pn[u], (double)ps[u] / (double)fmaxf(pn[u], 1.f), pq[u]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double nb = __shfl_xor(n, o, 64), mb = __shfl_xor(m, o, 64), qb = __shfl_xor(m2, o, 64);
      chan_merge(n, m, m2, (float)nb, mb, qb);
    }
    if (lane == 0) { red[0][wv] = n; red[1][wv] = m; red[2][wv] = m2; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < kFinWgNT / 64; ++w) chan_merge(n, m, m2, (float)red[0][w], red[1][w], red[2][w]);
    }
  }
}

// workgroup per (channel, segment) (bn_finalize_wg_kernel's merge)
__global__ __launch_bounds__(kFinWgNT) void bn_finalize_def_wg_kernel(BnDefArgs a) {
  __shared__ double red[3][kFinWgNT / 64];
  const int q = blockIdx.x / a.C, c = blockIdx.x - q * a.C;
  const int tid = threadIdx.x;
  const float g = a.gamma ? a.gamma[c] : 1.f, b = a.beta ? a.beta[c] : 0.f;
  const BnDefSeg& s = a.s[q];
  double n, m, m2;
  def_wg_merge(s.partial, s.rows, c, tid, red, n, m, m2);
  if (tid == 0) bn_def_out(a, s, c, m, m2, g, b);
}

// Several DIFFERENT BatchNorms' deferred finalizes in one launch (hgk_bn_finalize_multi): per job
// the merge hgk_bn_finalize_deferred would run for it alone (workgroup per channel above
// kFinDirect rows, else wave per channel), bitwise, and the same record / stat outputs.
static constexpr int kFinMulti = 8;
struct BnFinJobK {
  const float* partial;
  int rows;
  long M;
  int C;
  const float *gamma, *beta;
  float eps;
  double* rec;
  float* stat;
  int blk0, wg;
};
struct BnFinMultiArgs {
  BnFinJobK j[kFinMulti];
  int n;
};

__global__ __launch_bounds__(kFinWgNT) void bn_finalize_multi_kernel(BnFinMultiArgs a) {
  __shared__ double red[3][kFinWgNT / 64];
  int q = 0;
  while (q + 1 < a.n && (int)blockIdx.x >= a.j[q + 1].blk0) ++q;
  const BnFinJobK& J = a.j[q];
  const int lb = blockIdx.x - J.blk0, tid = threadIdx.x, lane = tid & 63;
  const int c = J.wg ? lb : lb * kFinWaves + (tid >> 6);
  if (c >= J.C) return;  // wave mode: whole waves (no barrier in that mode)
  const float g = J.gamma ? J.gamma[c] : 1.f, b = J.beta ? J.beta[c] : 0.f;
  BnDefArgs da;
  da.C = J.C; da.eps = J.eps;
  const BnDefSeg sg{J.partial, J.rows, J.M, J.rec, J.stat};
  double n, m, m2;
  if (J.wg) {
    def_wg_merge(J.partial, J.rows, c, tid, red, n, m, m2);
    if (tid == 0) bn_def_out(da, sg, c, m, m2, g, b);
  } else {
    def_wave_merge(J.partial, J.rows, c, lane, n, m, m2);
    if (lane == 0) bn_def_out(da, sg, c, m, m2, g, b);
  }
}

// running-statistics records applied in order: entries of one module (same running_mean) run
// sequentially in one workgroup, modules in parallel (96 entries: 3.4 KB of kernel arguments)
static constexpr int kRunMax = 96;
struct RunArgs {
  float* rm[kRunMax];
  float* rv[kRunMax];
  const double* rec[kRunMax];
  int C[kRunMax];
  float mom[kRunMax];
  int gbeg[kRunMax + 1];
};

// The module's running mean / var stay in registers across its records (one load, one store per
// channel; a read-modify-write per record made every record a dependent HBM round trip), and
// the records' (mean, unbiased var) are loaded kRunU at a time; same arithmetic per record.
static constexpr int kRunU = 8;
__global__ __launch_bounds__(256) void bn_running_update_kernel(RunArgs a) {
  const int g = blockIdx.x;
  const int i0 = a.gbeg[g], i1 = a.gbeg[g + 1];
  float* rm = a.rm[i0];
  float* rv = a.rv[i0];
  const int C = a.C[i0];  // host-checked equal over the group
  for (int c = threadIdx.x; c < C; c += 256) {
    float m = rm[c], v = rv[c];
    for (int i = i0; i < i1; i += kRunU) {
      double rmu[kRunU], rva[kRunU];
#pragma unroll
      for (int u = 0; u < kRunU; ++u) {
        const double* rec = a.rec[min(i + u, i1 - 1)];
        rmu[u] = rec[c];
        rva[u] = rec[C + c];
      }
#pragma unroll
      for (int u = 0; u < kRunU; ++u) {
        if (i + u < i1) {
          const float momentum = a.mom[i + u];
          m = (float)((1.0 - momentum) * m + momentum * rmu[u]);
          v = (float)((1.0 - momentum) * v + momentum * rva[u]);
        }
      }
    }
    rm[c] = m;
    rv[c] = v;
  }
}

struct BnbSeg {
  const float* partial;
  int rows;
  long M;
  const float* stat;  // [4][C] mean | invstd | scale | shift of the forward use
  const void* dA;
  const void* y;
  const void* add;
  void* dy;
  int accumulate;
  long rows_per_block;
  int G;
};
struct BnbArgs {
  BnbSeg s[2];
  int nseg, C, tpr, rpp, relu, training;
  float *dgamma, *dbeta;
  float* coef;  // [nseg][4][C] (unfused path)
};

// bn_bwd_fin_apply_kernel for 1-2 segments. Two segments: workgroup 0 only reduces both
// segments' rows and accumulates dgamma / dbeta (segment 0 then segment 1: the two single launches'
// order); workgroups [1, 1 + G0) apply segment 0, the rest segment 1 (each reduces its own rows,
// so no apply workgroup waits for a second reduction). One segment: workgroup 0 also owns dgamma.
template <typename T>
__global__ __launch_bounds__(kStatsNT) HGK_WPE_BWDAPPLY void bn_bwd_fin_apply_twin_kernel(BnbArgs a) {
  constexpr int VEC = Vec16<T>::N;
  constexpr int U = HGK_FINAPPLY_U;  // partial rows in flight per thread (16: measured 0.4 % slower)
  __shared__ double red[1024];        // [G][2C]
  __shared__ float scoef[4 * 512];   // [4][C]
  const int C = a.C;
  const int tid = threadIdx.x;
  const int F4 = C >> 1;  // float4 columns per partial row
  const int G = kStatsNT / F4;
  const int q4 = tid % F4, g4 = tid / F4;
  // sums of one segment's partial rows -> sg / sgx of this thread's (up to 2) channels
  auto reduce = [&](const float* partial, int rows, double* sg, double* sgx) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    const float4* p4 = reinterpret_cast<const float4*>(partial);
    for (int r0 = g4; r0 < rows; r0 += G * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p4[(long)min(r0 + G * u, rows - 1) * F4 + q4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = r0 + G * u < rows;
        a0 += ok ? (double)v[u].x : 0.0;
        a1 += ok ? (double)v[u].y : 0.0;
        a2 += ok ? (double)v[u].z : 0.0;
        a3 += ok ? (double)v[u].w : 0.0;
      }
    }
    __syncthreads();  // red free
    double* rr = red + g4 * 2 * C + 4 * q4;
    rr[0] = a0; rr[1] = a1; rr[2] = a2; rr[3] = a3;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = tid + k * kStatsNT;
      sg[k] = 0.0; sgx[k] = 0.0;
      if (c >= C) continue;
      for (int gg = 0; gg < G; ++gg) { sg[k] += red[gg * 2 * C + c]; sgx[k] += red[gg * 2 * C + C + c]; }
    }
  };
  const bool two = a.nseg == 2;
  if (two && blockIdx.x == 0) {
    float dg0[2], db0[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = min(tid + k * kStatsNT, C - 1);
      dg0[k] = a.dgamma ? a.dgamma[c] : 0.f;
      db0[k] = a.dbeta ? a.dbeta[c] : 0.f;
    }
    double s0[2], x0[2], s1[2], x1[2];
    reduce(a.s[0].partial, a.s[0].rows, s0, x0);
    reduce(a.s[1].partial, a.s[1].rows, s1, x1);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = tid + k * kStatsNT;
      if (c >= C) break;
      if (a.dgamma) a.dgamma[c] = (dg0[k] + (float)x0[k]) + (float)x1[k];
      if (a.dbeta) a.dbeta[c] = (db0[k] + (float)s0[k]) + (float)s1[k];
    }
    return;
  }
  const int b = (int)blockIdx.x - (two ? 1 : 0);
  const bool seg1 = b >= a.s[0].G;
  const BnbSeg& s = a.s[seg1 ? 1 : 0];
  const int bx = b - (seg1 ? a.s[0].G : 0);
  const bool lead = !two && blockIdx.x == 0;  // dgamma / dbeta owner (one segment)
  const int cv = tid % a.tpr, rp = tid / a.tpr;
  const int rpp = a.rpp;
  const long r_begin = (long)bx * s.rows_per_block;
  const long r_end = min(s.M, r_begin + s.rows_per_block);
  const T* __restrict__ dA = reinterpret_cast<const T*>(s.dA);
  const T* __restrict__ y = reinterpret_cast<const T*>(s.y);
  const T* add = reinterpret_cast<const T*>(s.add);
  T* dy = reinterpret_cast<T*>(s.dy);
  const int accumulate = s.accumulate;
  const float* mean = s.stat;
  const float* invstd = s.stat + C;
  const float* scale = s.stat + 2 * C;
  const float* shift = s.stat + 3 * C;
  typedef typename Vec16<T>::type V;
  V vd[kRowU], vy[kRowU], va[kRowU], vo[kRowU];
  auto load_batch = [&](long r0) {
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) {
        const long off = r * C + cv * VEC;
        vd[u] = load16(dA + off);
        vy[u] = load16(y + off);
        if (add) va[u] = load16(add + off);
        if (accumulate) vo[u] = load16(dy + off);
      }
    }
  };
  load_batch(r_begin + rp);
  float sc[VEC], sh[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) { sc[e] = scale[cv * VEC + e]; sh[e] = shift[cv * VEC + e]; }
  float csc[2], cis[2], cmu[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = min(tid + k * kStatsNT, C - 1);
    csc[k] = scale[c]; cis[k] = invstd[c]; cmu[k] = mean[c];
  }
  float dg0[2] = {0.f, 0.f}, db0[2] = {0.f, 0.f};
  if (lead) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = min(tid + k * kStatsNT, C - 1);
      if (a.dgamma) dg0[k] = a.dgamma[c];
      if (a.dbeta) db0[k] = a.dbeta[c];
    }
  }
  double sg[2], sgx[2];
  reduce(s.partial, s.rows, sg, sgx);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = tid + k * kStatsNT;
    if (c >= C) break;
    const double scd = csc[k], is = cis[k];
    const float mu = cmu[k];
    if (lead) {
      if (a.dgamma) a.dgamma[c] = dg0[k] + (float)sgx[k];
      if (a.dbeta) a.dbeta[c] = db0[k] + (float)sg[k];
    }
    double c1 = 0.0, c2 = 0.0;
    if (a.training) {
      c1 = -scd * is * sgx[k] / (double)s.M;
      c2 = -scd * sg[k] / (double)s.M;
    }
    scoef[c] = (float)scd;
    scoef[C + c] = (float)c1;
    scoef[2 * C + c] = (float)c2;
    scoef[3 * C + c] = mu;
  }
  __syncthreads();
  float k0[VEC], k1[VEC], k2[VEC], mu[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int c = cv * VEC + e;
    k0[e] = scoef[c]; k1[e] = scoef[C + c]; k2[e] = scoef[2 * C + c]; mu[e] = scoef[3 * C + c];
  }
  const int relu = a.relu;
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    if (r0 != r_begin + rp) load_batch(r0);
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r >= r_end) break;
      float fd[VEC], fy[VEC], fa[VEC], fo[VEC], o[VEC];
      unpack16<T>(vd[u], fd);
      unpack16<T>(vy[u], fy);
      if (add) unpack16<T>(va[u], fa);
      if (accumulate) unpack16<T>(vo[u], fo);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float v = bnb_apply(fd[e], fy[e], sc[e], sh[e], k0[e], k1[e], k2[e], mu[e], relu);
        if (add) v += fa[e];
        if (accumulate) v += fo[e];
        o[e] = v;
      }
      store16(dy + r * C + cv * VEC, pack16<T>(o));
    }
  }
}

// bn_bwd_finalize_wg_kernel for 1-2 segments: one workgroup per (channel, segment) writes the
// segment's coefficients and its (float) sums; the dgamma / dbeta accumulation (segment order)
// happens in workgroup 0 of bn_bwd_apply_twin_kernel. coef: [nseg][6][C] = 4 coefficient rows +
// (float) sum g, (float) sum g*xhat.
__global__ __launch_bounds__(kFinWgNT) void bn_bwd_finalize_twin_kernel(BnbArgs a) {
  __shared__ double red[2][kFinWgNT / 64];
  const int C = a.C;
  const int q = blockIdx.x / C, c = blockIdx.x - q * C;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const BnbSeg& s = a.s[q];
  const float* partial = s.partial;
  const int rows = s.rows;
  double sg = 0.0, sgx = 0.0;
  for (int r0 = tid; r0 < rows; r0 += kFinWgNT * kFinWgU) {
    float x0[kFinWgU], x1[kFinWgU];
#pragma unroll
    for (int u = 0; u < kFinWgU; ++u) {
      const int rc = min(r0 + kFinWgNT * u, rows - 1);
      x0[u] = partial[((long)rc * 2 + 0) * C + c];
      x1[u] = partial[((long)rc * 2 + 1) * C + c];
    }
#pragma unroll
    for (int u = 0; u < kFinWgU; ++u) {
      const bool ok = r0 + kFinWgNT * u < rows;
      sg += ok ? (double)x0[u] : 0.0;
      sgx += ok ? (double)x1[u] : 0.0;
    }
  }
  sg = wave_sum_d(sg);
  sgx = wave_sum_d(sgx);
  if (lane == 0) { red[0][wv] = sg; red[1][wv] = sgx; }
  __syncthreads();
  if (tid != 0) return;
  sg = red[0][0]; sgx = red[1][0];
  for (int w = 1; w < kFinWgNT / 64; ++w) { sg += red[0][w]; sgx += red[1][w]; }
  float* coef = a.coef + (long)q * 6 * C;
  const double sc = s.stat[2 * C + c];
  const float mu = s.stat[c];
  const double is = s.stat[C + c];
  double c1 = 0.0, c2 = 0.0;
  if (a.training) {
    c1 = -sc * is * sgx / (double)s.M;
    c2 = -sc * sg / (double)s.M;
  }
  coef[c] = (float)sc;
  coef[C + c] = (float)c1;
  coef[2 * C + c] = (float)c2;
  coef[3 * C + c] = mu;
  coef[4 * C + c] = (float)sg;
  coef[5 * C + c] = (float)sgx;
}

// coefficients only (the apply is folded into the consuming convolution, hgk_conv_fwd_bnbwd_vg):
// one workgroup per channel runs bn_bwd_finalize_twin_kernel's reduction for each segment in turn
// and then accumulates dgamma / dbeta segment 0 first — the same operations, in the same order, as
// bn_bwd_finalize_twin_kernel + workgroup 0 of bn_bwd_apply_twin_kernel (same bits)
__global__ __launch_bounds__(kFinWgNT) void bn_bwd_coef_twin_kernel(BnbArgs a) {
  __shared__ double red[2][kFinWgNT / 64];
  const int C = a.C, c = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float sgf[2] = {0.f, 0.f}, sgxf[2] = {0.f, 0.f};
  for (int q = 0; q < a.nseg; ++q) {
    const BnbSeg& s = a.s[q];
    const float* partial = s.partial;
    const int rows = s.rows;
    double sg = 0.0, sgx = 0.0;
    for (int r0 = tid; r0 < rows; r0 += kFinWgNT * kFinWgU) {
      float x0[kFinWgU], x1[kFinWgU];
#pragma unroll
      for (int u = 0; u < kFinWgU; ++u) {
        const int rc = min(r0 + kFinWgNT * u, rows - 1);
        x0[u] = partial[((long)rc * 2 + 0) * C + c];
        x1[u] = partial[((long)rc * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < kFinWgU; ++u) {
        const bool ok = r0 + kFinWgNT * u < rows;
        sg += ok ? (double)x0[u] : 0.0;
        sgx += ok ? (double)x1[u] : 0.0;
      }
    }
    sg = wave_sum_d(sg);
    sgx = wave_sum_d(sgx);
    __syncthreads();  // the previous segment's red[] reads are done
    if (lane == 0) { red[0][wv] = sg; red[1][wv] = sgx; }
    __syncthreads();
    if (tid == 0) {
      sg = red[0][0]; sgx = red[1][0];
      for (int w = 1; w < kFinWgNT / 64; ++w) { sg += red[0][w]; sgx += red[1][w]; }
      float* coef = a.coef + (long)q * 6 * C;
      const double sc = s.stat[2 * C + c];
      const float mu = s.stat[c];
      const double is = s.stat[C + c];
      double c1 = 0.0, c2 = 0.0;
      if (a.training) {
        c1 = -sc * is * sgx / (double)s.M;
        c2 = -sc * sg / (double)s.M;
      }
      coef[c] = (float)sc;
      coef[C + c] = (float)c1;
      coef[2 * C + c] = (float)c2;
      coef[3 * C + c] = mu;
      coef[4 * C + c] = (float)sg;
      coef[5 * C + c] = (float)sgx;
      sgf[q] = (float)sg;
      sgxf[q] = (float)sgx;
    }
  }
  if (tid == 0) {
    float dg = a.dgamma ? a.dgamma[c] : 0.f, db = a.dbeta ? a.dbeta[c] : 0.f;
    for (int q = 0; q < a.nseg; ++q) {
      db = db + sgf[q];
      dg = dg + sgxf[q];
    }
    if (a.dgamma) a.dgamma[c] = dg;
    if (a.dbeta) a.dbeta[c] = db;
  }
}

// bn_bwd_apply_kernel for 1-2 segments (coefficients from bn_bwd_finalize_twin_kernel);
// workgroup 0 accumulates dgamma / dbeta from the per-segment sums, segment 0 first
template <typename T>
__global__ __launch_bounds__(kStatsNT) HGK_WPE_BWDAPPLY void bn_bwd_apply_twin_kernel(BnbArgs a) {
  constexpr int VEC = Vec16<T>::N;
  const int C = a.C;
  const int tid = threadIdx.x;
  if (blockIdx.x == 0) {
    for (int c = tid; c < C; c += kStatsNT) {
      float dg = a.dgamma ? a.dgamma[c] : 0.f, db = a.dbeta ? a.dbeta[c] : 0.f;
      for (int q = 0; q < a.nseg; ++q) {
        db = db + a.coef[((long)q * 6 + 4) * C + c];
        dg = dg + a.coef[((long)q * 6 + 5) * C + c];
      }
      if (a.dgamma) a.dgamma[c] = dg;
      if (a.dbeta) a.dbeta[c] = db;
    }
    return;
  }
  const int b = (int)blockIdx.x - 1;
  const bool seg1 = b >= a.s[0].G;
  const BnbSeg& s = a.s[seg1 ? 1 : 0];
  const int bx = b - (seg1 ? a.s[0].G : 0);
  const int cv = tid % a.tpr, rp = tid / a.tpr;
  const int rpp = a.rpp;
  const long r_begin = (long)bx * s.rows_per_block;
  const long r_end = min(s.M, r_begin + s.rows_per_block);
  const T* __restrict__ dA = reinterpret_cast<const T*>(s.dA);
  const T* __restrict__ y = reinterpret_cast<const T*>(s.y);
  const T* add = reinterpret_cast<const T*>(s.add);
  T* dy = reinterpret_cast<T*>(s.dy);
  const int accumulate = s.accumulate, relu = a.relu;
  const float* coef = a.coef + (seg1 ? 6L * C : 0L);
  float sc[VEC], sh[VEC], k0[VEC], k1[VEC], k2[VEC], mu[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) {
    const int c = cv * VEC + e;
    sc[e] = s.stat[2 * C + c]; sh[e] = s.stat[3 * C + c];
    k0[e] = coef[c]; k1[e] = coef[C + c]; k2[e] = coef[2 * C + c]; mu[e] = coef[3 * C + c];
  }
  typedef typename Vec16<T>::type V;
  for (long r0 = r_begin + rp; r0 < r_end; r0 += kRowU * rpp) {
    V vd[kRowU], vy[kRowU], va[kRowU], vo[kRowU];
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r < r_end) {
        const long off = r * C + cv * VEC;
        vd[u] = load16(dA + off);
        vy[u] = load16(y + off);
        if (add) va[u] = load16(add + off);
        if (accumulate) vo[u] = load16(dy + off);
      }
    }
#pragma unroll
    for (int u = 0; u < kRowU; ++u) {
      const long r = r0 + u * rpp;
      if (r >= r_end) break;
      float fd[VEC], fy[VEC], fa[VEC], fo[VEC], o[VEC];
      unpack16<T>(vd[u], fd);
      unpack16<T>(vy[u], fy);
      if (add) unpack16<T>(va[u], fa);
      if (accumulate) unpack16<T>(vo[u], fo);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        float v = bnb_apply(fd[e], fy[e], sc[e], sh[e], k0[e], k1[e], k2[e], mu[e], relu);
        if (add) v += fa[e];
        if (accumulate) v += fo[e];
        o[e] = v;
      }
      store16(dy + r * C + cv * VEC, pack16<T>(o));
    }
  }
}

// rows > kFinDirect: one workgroup per channel (measured faster than a 64:1 merge launch into
// `scratch` first, bn_partial_merge_kernel, which remains for the backward partials' fallback)
static constexpr bool fin_wg() { return true; }

// partial rows > kFinDirect: merge them 64:1 into `scratch` first (see bn_partial_merge_kernel)
template <int NV>
static const float* merge_partials(hipStream_t st, const float* partial, int& rows, int C,
                                   float* scratch) {
  if (rows <= kFinDirect || scratch == nullptr) return partial;
  const int g = ceil_div(rows, kMergeRows);
  hipLaunchKernelGGL(bn_partial_merge_kernel<NV>, dim3(g, ceil_div(C, 64)), dim3(256), 0, st,
                     partial, rows, C, scratch);
  rows = g;
  return scratch;
}

}  // namespace hgk

using namespace hgk;

extern "C" {

int hgk_bn_stats(hgk_stream_t stream, int dtype, const void* x, long M, int C, float* partial,
                 int* rows_out) {
  HGK_CHECK_ARG(x && partial && M > 0 && C > 0, "bn_stats: bad args");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_stats: unsupported C=%d", C);
    HGK_CHECK_ARG(p.G <= kMaxRows, "bn_stats: too many rows");
    size_t lds = (size_t)p.rpp * C * 3 * sizeof(float);
    hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(p.G), dim3(kStatsNT), lds, st,
                       reinterpret_cast<const T*>(x), M, C, p.rows_per_block, p.tpr, p.rpp,
                       partial);
    if (rows_out) *rows_out = p.G;
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

size_t hgk_bn_finalize_scratch(int rows, int C) {
  // forward statistics are channel-major: the finalisers read them directly (no merge scratch);
  // the backward partials ([rows][2][C]) would take the 64:1 merge without the workgroup path
  return rows > kFinDirect ? (size_t)ceil_div(rows, kMergeRows) * 2 * C * sizeof(float) : 0;
}

int hgk_bn_finalize(hgk_stream_t stream, const float* partial, int rows, long M, int C,
                    const float* gamma, const float* beta, float* running_mean,
                    float* running_var, float momentum, float eps, int training, float* mean,
                    float* invstd, float* scale, float* shift, float* scratch) {
  HGK_CHECK_ARG(mean && invstd && scale && shift, "bn_finalize: null outputs");
  HGK_CHECK_ARG(!training || (partial && rows > 0), "bn_finalize: partials missing");
  HGK_CHECK_ARG(training || (running_mean && running_var), "bn_finalize: eval needs running stats");
  HGK_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr), "bn_finalize: running pair");
  hipStream_t st = (hipStream_t)stream;
  if (training && rows > kFinDirect) {
    hipLaunchKernelGGL(bn_finalize_wg_kernel, dim3(C), dim3(kFinWgNT), 0, st, partial, rows, M, C,
                       gamma, beta, running_mean, running_var, momentum, eps, mean, invstd, scale,
                       shift);
    HGK_LAUNCH_CHECK();
    return HGK_OK;
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(C, kFinWaves)), dim3(64 * kFinWaves), 0, st, partial, rows,
                     M, C, gamma, beta, running_mean, running_var, momentum, eps, training, mean,
                     invstd, scale, shift);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_apply(hgk_stream_t stream, int dtype, const void* x, long M, int C, const float* scale,
                 const float* shift, int relu, void* y) {
  HGK_CHECK_ARG(x && y && scale && shift, "bn_apply: null");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_apply: unsupported C=%d", C);
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(p.G), dim3(kStatsNT), 0, st,
                       reinterpret_cast<const T*>(x), M, C, p.rows_per_block, p.tpr, p.rpp, scale,
                       shift, relu, reinterpret_cast<T*>(y));
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_bwd_reduce(hgk_stream_t stream, int dtype, const void* dA, const void* y, long M,
                      int C, const float* scale, const float* shift, int relu, const float* mean,
                      const float* invstd, float* partial, int* rows_out) {
  HGK_CHECK_ARG(dA && y && scale && shift && mean && invstd && partial, "bn_bwd_reduce: null");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_bwd_reduce: unsupported C=%d", C);
    HGK_CHECK_ARG(p.G <= kMaxRows, "bn_bwd_reduce: too many rows");
    size_t lds = (size_t)p.rpp * C * 2 * sizeof(float);
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<T>, dim3(p.G), dim3(kStatsNT), lds, st,
                       reinterpret_cast<const T*>(dA), reinterpret_cast<const T*>(y), M, C,
                       p.rows_per_block, p.tpr, p.rpp, scale, shift, relu, mean, invstd, partial);
    if (rows_out) *rows_out = p.G;
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

static BnSideK side_k(const hgk_bn_side* s) {
  return BnSideK{s->y, s->scale, s->shift, s->mean, s->invstd, s->relu, s->partial};
}

int hgk_bn_apply2_add(hgk_stream_t stream, int dtype, const hgk_bn_side* a, const hgk_bn_side* b,
                      void* out, long M, int C, float* partial, int* rows_out) {
  HGK_CHECK_ARG(a && b && out && a->y && b->y && a->scale && a->shift && b->scale && b->shift &&
                    M > 0 && C > 0,
                "bn_apply2_add: null / bad args");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_apply2_add: unsupported C=%d", C);
    HGK_CHECK_ARG(p.G <= kMaxRows, "bn_apply2_add: too many rows");
    size_t lds = partial ? (size_t)p.rpp * C * 3 * sizeof(float) : 0;
    hipLaunchKernelGGL(bn_apply2_add_kernel<T>, dim3(p.G), dim3(kStatsNT), lds, st, side_k(a),
                       side_k(b), reinterpret_cast<T*>(out), M, C, p.rows_per_block, p.tpr, p.rpp,
                       partial);
    if (rows_out) *rows_out = partial ? p.G : 0;
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_bwd_reduce2(hgk_stream_t stream, int dtype, const void* dA, long M, int C,
                       const hgk_bn_side* a, const hgk_bn_side* b, int* rows_out) {
  HGK_CHECK_ARG(dA && a && b && M > 0 && C > 0, "bn_bwd_reduce2: null / bad args");
  for (const hgk_bn_side* s : {a, b})
    HGK_CHECK_ARG(s->y && s->scale && s->shift && s->mean && s->invstd && s->partial,
                  "bn_bwd_reduce2: null side");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_bwd_reduce2: unsupported C=%d", C);
    HGK_CHECK_ARG(p.G <= kMaxRows, "bn_bwd_reduce2: too many rows");
    size_t lds = (size_t)p.rpp * C * 2 * 2 * sizeof(float);
    HGK_CHECK_ARG(lds <= 64 * 1024, "bn_bwd_reduce2: C=%d too wide", C);
    hipLaunchKernelGGL(bn_bwd_reduce2_kernel<T>, dim3(p.G), dim3(kStatsNT), lds, st,
                       reinterpret_cast<const T*>(dA), side_k(a), side_k(b), M, C, p.rows_per_block,
                       p.tpr, p.rpp);
    if (rows_out) *rows_out = p.G;
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_bwd_finalize(hgk_stream_t stream, const float* partial, int rows, long M, int C,
                        const float* scale, const float* mean, const float* invstd, int training,
                        float* dgamma, float* dbeta, float* coef, float* scratch) {
  HGK_CHECK_ARG(partial && scale && mean && invstd && coef && rows > 0, "bn_bwd_finalize: null");
  hipStream_t st = (hipStream_t)stream;
  if (rows > kFinDirect && fin_wg()) {
    hipLaunchKernelGGL(bn_bwd_finalize_wg_kernel, dim3(C), dim3(kFinWgNT), 0, st, partial, rows, M,
                       C, scale, mean, invstd, training, dgamma, dbeta, coef);
    HGK_LAUNCH_CHECK();
    return HGK_OK;
  }
  partial = merge_partials<2>(st, partial, rows, C, scratch);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(ceil_div(C, kFinWaves)), dim3(64 * kFinWaves), 0, st, partial,
                     rows, M, C, scale, mean, invstd, training, dgamma, dbeta, coef);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_bwd_apply(hgk_stream_t stream, int dtype, const void* dA, const void* y, long M, int C,
                     const float* scale, const float* shift, int relu, const float* coef,
                     const void* add, void* dy, int accumulate) {
  HGK_CHECK_ARG(dA && y && scale && shift && coef && dy, "bn_bwd_apply: null");
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p, kApplyPasses), "bn_bwd_apply: unsupported C=%d", C);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(p.G), dim3(kStatsNT), 0, st,
                       reinterpret_cast<const T*>(dA), reinterpret_cast<const T*>(y), M, C,
                       p.rows_per_block, p.tpr, p.rpp, scale, shift, relu, coef,
                       reinterpret_cast<const T*>(add), reinterpret_cast<T*>(dy), accumulate);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_bwd_fused_max_rows(void) { return kFusedFinMaxRows; }

int hgk_bn_bwd_finalize_apply(hgk_stream_t stream, int dtype, const float* partial, int rows,
                              long M, int C, const float* scale, const float* shift, int relu,
                              const float* mean, const float* invstd, int training, float* dgamma,
                              float* dbeta, const void* dA, const void* y, const void* add,
                              void* dy, int accumulate) {
  HGK_CHECK_ARG(partial && scale && shift && mean && invstd && dA && y && dy && rows > 0,
                "bn_bwd_finalize_apply: null");
  HGK_CHECK_ARG(rows <= kFusedFinMaxRows, "bn_bwd_finalize_apply: %d partial rows > %d", rows,
                kFusedFinMaxRows);
  HGK_CHECK_ARG(C % 8 == 0 && C <= 512 && kStatsNT % (C / 2) == 0,
                "bn_bwd_finalize_apply: unsupported C=%d", C);
  hipStream_t st = (hipStream_t)stream;
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p), "bn_bwd_finalize_apply: unsupported C=%d", C);
    hipLaunchKernelGGL(bn_bwd_fin_apply_kernel<T>, dim3(p.G), dim3(kStatsNT), 0, st, partial, rows,
                       mean, invstd, training, dgamma, dbeta, reinterpret_cast<const T*>(dA),
                       reinterpret_cast<const T*>(y), M, C, p.rows_per_block, p.tpr, p.rpp, scale,
                       shift, relu, reinterpret_cast<const T*>(add), reinterpret_cast<T*>(dy),
                       accumulate);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_bwd_pair(hgk_stream_t stream, int dtype, const void* dA, long M, int C, int training,
                    const hgk_bnb_side* a, const hgk_bnb_side* b) {
  HGK_CHECK_ARG(dA && a && b && M > 0 && C > 0, "bn_bwd_pair: null / bad args");
  const bool fin = a->partial != nullptr;
  HGK_CHECK_ARG((b->partial != nullptr) == fin, "bn_bwd_pair: both sides fused or neither");
  for (const hgk_bnb_side* s : {a, b}) {
    HGK_CHECK_ARG(s->y && s->scale && s->shift && s->dy, "bn_bwd_pair: null side");
    if (fin)
      HGK_CHECK_ARG(s->mean && s->invstd && s->rows > 0 && s->rows <= kFusedFinMaxRows,
                    "bn_bwd_pair: fused finalize needs mean / invstd and 1..%d rows", kFusedFinMaxRows);
    else
      HGK_CHECK_ARG(s->coef, "bn_bwd_pair: coef missing");
  }
  HGK_CHECK_ARG(C % 8 == 0 && C <= 512 && kStatsNT % (C / 2) == 0, "bn_bwd_pair: unsupported C=%d", C);
  hipStream_t st = (hipStream_t)stream;
  const BnbSideK A{a->y, a->scale, a->shift, a->mean, a->invstd, a->relu, a->partial, a->rows, a->coef,
                   a->dgamma, a->dbeta, a->dy};
  const BnbSideK B{b->y, b->scale, b->shift, b->mean, b->invstd, b->relu, b->partial, b->rows, b->coef,
                   b->dgamma, b->dbeta, b->dy};
  HGK_DISPATCH_DTYPE(dtype, T, {
    RowPlan p;
    HGK_CHECK_ARG(row_plan<T>(M, C, p, fin ? 4 : kApplyPasses), "bn_bwd_pair: unsupported C=%d", C);
    if (fin)
      hipLaunchKernelGGL((bn_bwd_pair_kernel<T, true>), dim3(p.G), dim3(kStatsNT), 0, st,
                         reinterpret_cast<const T*>(dA), A, B, M, C, training, p.rows_per_block, p.tpr,
                         p.rpp);
    else
      hipLaunchKernelGGL((bn_bwd_pair_kernel<T, false>), dim3(p.G), dim3(kStatsNT), 0, st,
                         reinterpret_cast<const T*>(dA), A, B, M, C, training, p.rows_per_block, p.tpr,
                         p.rpp);
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_finalize_multi(hgk_stream_t stream, const hgk_bn_fin_job* jobs, int n) {
  HGK_CHECK_ARG(n >= 0 && (n == 0 || jobs), "bn_finalize_multi: bad args");
  hipStream_t st = (hipStream_t)stream;
  for (int i0 = 0; i0 < n; i0 += kFinMulti) {
    BnFinMultiArgs a;
    a.n = std::min(kFinMulti, n - i0);
    int blk = 0;
    for (int q = 0; q < a.n; ++q) {
      const hgk_bn_fin_job& g = jobs[i0 + q];
      HGK_CHECK_ARG(g.partial && g.rows > 0 && g.M > 0 && g.C > 0 && g.rec && g.stat,
                    "bn_finalize_multi: job %d incomplete", i0 + q);
      const int wg = g.rows > kFinDirect;
      a.j[q] = BnFinJobK{g.partial, g.rows, g.M, g.C, g.gamma, g.beta, g.eps, g.rec, g.stat, blk, wg};
      blk += wg ? g.C : ceil_div(g.C, kFinWaves);
    }
    hipLaunchKernelGGL(bn_finalize_multi_kernel, dim3(blk), dim3(kFinWgNT), 0, st, a);
    HGK_LAUNCH_CHECK();
  }
  return HGK_OK;
}

int hgk_bn_bwd_finalize_multi(hgk_stream_t stream, const hgk_bnb_fin_job* jobs, int n) {
  HGK_CHECK_ARG(n >= 0 && (n == 0 || jobs), "bn_bwd_finalize_multi: bad args");
  hipStream_t st = (hipStream_t)stream;
  for (int i0 = 0; i0 < n; i0 += 8) {
    BnbFinMultiArgs a;
    a.n = std::min(8, n - i0);
    int blk = 0;
    for (int q = 0; q < a.n; ++q) {
      const hgk_bnb_fin_job& g = jobs[i0 + q];
      HGK_CHECK_ARG(g.partial && g.scale && g.mean && g.invstd && g.coef && g.C > 0 && g.M > 0,
                    "bn_bwd_finalize_multi: job %d incomplete", i0 + q);
      HGK_CHECK_ARG(g.rows > kFinDirect && fin_wg(),
                    "bn_bwd_finalize_multi: job %d has %d partial rows (needs > %d)", i0 + q, g.rows,
                    kFinDirect);
      a.j[q] = BnbFinJobK{g.partial, g.rows, g.M, g.C, g.scale, g.mean, g.invstd, g.training,
                          g.dgamma, g.dbeta, g.coef, blk};
      blk += g.C;
    }
    hipLaunchKernelGGL(bn_bwd_finalize_multi_kernel, dim3(blk), dim3(kFinWgNT), 0, st, a);
    HGK_LAUNCH_CHECK();
  }
  return HGK_OK;
}

int hgk_bn_bwd_finalize_multi_min_rows(void) { return fin_wg() ? kFinDirect + 1 : 1 << 30; }

int hgk_bn_finalize_deferred(hgk_stream_t stream, const hgk_bn_seg* seg, int nseg, int C,
                             const float* gamma, const float* beta, float eps) {
  HGK_CHECK_ARG(seg && (nseg == 1 || nseg == 2) && C > 0, "bn_finalize_deferred: bad args");
  BnDefArgs a;
  a.nseg = nseg; a.C = C; a.gamma = gamma; a.beta = beta; a.eps = eps;
  int most = 0;
  for (int q = 0; q < 2; ++q) {
    const hgk_bn_seg& g = seg[q < nseg ? q : 0];
    if (q < nseg)
      HGK_CHECK_ARG(g.partial && g.rows > 0 && g.M > 0 && g.rec && g.stat,
                    "bn_finalize_deferred: segment %d incomplete", q);
    a.s[q] = BnDefSeg{g.partial, g.rows, g.M, g.rec, g.stat};
    most = std::max(most, g.rows);
  }
  hipStream_t st = (hipStream_t)stream;
  if (most > kFinDirect)
    hipLaunchKernelGGL(bn_finalize_def_wg_kernel, dim3(C * nseg), dim3(kFinWgNT), 0, st, a);
  else
    hipLaunchKernelGGL(bn_finalize_def_kernel, dim3(ceil_div((long)C * nseg, kFinWaves)),
                       dim3(64 * kFinWaves), 0, st, a);
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

int hgk_bn_running_update(hgk_stream_t stream, const hgk_bn_running* e, int n) {
  HGK_CHECK_ARG(n >= 0 && (n == 0 || e), "bn_running_update: bad args");
  hipStream_t st = (hipStream_t)stream;
  for (int b = 0; b < n; b += kRunMax) {
    const int cnt = std::min(kRunMax, n - b);
    // group the chunk's entries by module (running_mean), keeping each module's order
    int order[kRunMax], gstart[kRunMax + 1], ng = 0;
    bool taken[kRunMax] = {};
    int k = 0;
    for (int i = 0; i < cnt; ++i) {
      if (taken[i]) continue;
      gstart[ng++] = k;
      for (int j = i; j < cnt; ++j)
        if (!taken[j] && e[b + j].running_mean == e[b + i].running_mean) {
          HGK_CHECK_ARG(e[b + j].running_var == e[b + i].running_var && e[b + j].C == e[b + i].C,
                        "bn_running_update: entries %d / %d share running_mean only", b + i, b + j);
          order[k++] = j;
          taken[j] = true;
        }
    }
    gstart[ng] = k;
    RunArgs a;
    for (int i = 0; i < cnt; ++i) {
      const hgk_bn_running& r = e[b + order[i]];
      HGK_CHECK_ARG(r.running_mean && r.running_var && r.rec && r.C > 0, "bn_running_update: entry %d", b + order[i]);
      a.rm[i] = r.running_mean; a.rv[i] = r.running_var; a.rec[i] = r.rec; a.C[i] = r.C;
      a.mom[i] = r.momentum;
    }
    for (int g = 0; g <= ng; ++g) a.gbeg[g] = gstart[g];
    hipLaunchKernelGGL(bn_running_update_kernel, dim3(ng), dim3(256), 0, st, a);
    HGK_LAUNCH_CHECK();
  }
  return HGK_OK;
}

static int most_rows(const hgk_bnb_seg* seg, int nseg) {
  int m = 0;
  for (int q = 0; q < nseg; ++q) m = std::max(m, seg[q].rows);
  return m;
}

int hgk_bn_bwd_twin(hgk_stream_t stream, int dtype, const hgk_bnb_seg* seg, int nseg, int C,
                    int relu, int training, float* dgamma, float* dbeta, float* coef) {
  HGK_CHECK_ARG(seg && (nseg == 1 || nseg == 2) && C > 0, "bn_bwd_twin: bad args");
  // dy == NULL in every segment: coefficients + dgamma / dbeta only (the apply is folded into the
  // consuming convolution, hgk_bn_vgrad); needs the unfused path's coef scratch
  const bool coef_only = seg[0].dy == nullptr;
  for (int q = 0; q < nseg; ++q)
    HGK_CHECK_ARG((seg[q].dy == nullptr) == coef_only, "bn_bwd_twin: dy NULL in only some segments");
  if (coef_only) {
    HGK_CHECK_ARG(coef != nullptr && most_rows(seg, nseg) > kFusedFinMaxRows,
                  "bn_bwd_twin: coefficients-only needs the coef scratch and > %d partial rows",
                  kFusedFinMaxRows);
    BnbArgs a;
    memset(&a, 0, sizeof(a));
    a.nseg = nseg; a.C = C; a.relu = relu; a.training = training; a.dgamma = dgamma;
    a.dbeta = dbeta; a.coef = coef;
    for (int q = 0; q < nseg; ++q) {
      const hgk_bnb_seg& g = seg[q];
      HGK_CHECK_ARG(g.partial && g.rows > 0 && g.M > 0 && g.stat, "bn_bwd_twin: segment %d incomplete", q);
      a.s[q] = BnbSeg{g.partial, g.rows, g.M, g.stat, nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
    }
    hipLaunchKernelGGL(bn_bwd_coef_twin_kernel, dim3(C), dim3(kFinWgNT), 0, (hipStream_t)stream, a);
    HGK_LAUNCH_CHECK();
    return HGK_OK;
  }
  BnbArgs a;
  a.nseg = nseg; a.C = C; a.relu = relu; a.training = training; a.dgamma = dgamma; a.dbeta = dbeta;
  a.coef = coef;
  hipStream_t st = (hipStream_t)stream;
  int most = 0;
  long blocks = 0;
  HGK_DISPATCH_DTYPE(dtype, T, {
    for (int q = 0; q < 2; ++q) {
      const hgk_bnb_seg& g = seg[q < nseg ? q : 0];
      if (q < nseg)
        HGK_CHECK_ARG(g.partial && g.rows > 0 && g.M > 0 && g.stat && g.dA && g.y && g.dy,
                      "bn_bwd_twin: segment %d incomplete", q);
      RowPlan p;
      HGK_CHECK_ARG(row_plan<T>(g.M, C, p, most_rows(seg, nseg) <= kFusedFinMaxRows ? 4 : kApplyPasses),
                    "bn_bwd_twin: unsupported C=%d", C);
      a.tpr = p.tpr; a.rpp = p.rpp;
      a.s[q] = BnbSeg{g.partial, g.rows, g.M, g.stat, g.dA, g.y, g.add, g.dy, g.accumulate,
                      p.rows_per_block, q < nseg ? p.G : 0};
      if (q < nseg) { most = std::max(most, g.rows); blocks += p.G; }
    }
    const bool fused = most <= kFusedFinMaxRows && C % 8 == 0 && C <= 512 && kStatsNT % (C / 2) == 0;
    if (fused) {
      hipLaunchKernelGGL(bn_bwd_fin_apply_twin_kernel<T>, dim3((unsigned)(blocks + (nseg == 2 ? 1 : 0))),
                         dim3(kStatsNT), 0, st, a);
    } else {
      HGK_CHECK_ARG(coef != nullptr, "bn_bwd_twin: %d partial rows need the coef scratch", most);
      hipLaunchKernelGGL(bn_bwd_finalize_twin_kernel, dim3(C * nseg), dim3(kFinWgNT), 0, st, a);
      HGK_LAUNCH_CHECK();
      hipLaunchKernelGGL(bn_bwd_apply_twin_kernel<T>, dim3((unsigned)(blocks + 1)), dim3(kStatsNT), 0,
                         st, a);
    }
  });
  HGK_LAUNCH_CHECK();
  return HGK_OK;
}

}  // extern "C"
