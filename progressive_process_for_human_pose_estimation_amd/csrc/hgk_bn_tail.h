// In-kernel BatchNorm finalisation ("BN tail") for kernels that emit BN partial rows.
//
// A conv launch whose output feeds a train-mode BatchNorm (forward statistics) or whose output
// is a BN's input gradient (backward sums, see hgk_conv_fwd_bnbwd) writes one partial row per
// workgroup tile. Instead of a separate merge + finalize launch (each ~5 us of launch-bound work
// on the hot path, ~700 per training step), the workgroups finish the job themselves:
//   level 1: the LAST workgroup (ticket counter) to complete a group of kTailGroup partial rows
//            merges them (fixed order, fp64) into one level-2 row;
//   level 2: the last group-merger merges the level-2 rows and finalises: mean / invstd / scale /
//            shift + running statistics (forward), or dgamma / dbeta / coef (backward) —
//            exactly hgk_bn_finalize / hgk_bn_bwd_finalize semantics.
// Cross-workgroup hand-off (any XCD placement): partial rows are stored write-through (sc1),
// every storing wave drains them (vmcnt(0)), barrier, one lane takes a relaxed agent-scope ticket;
// the winner reads every handed-off value with sc1 loads (cdna_hip_programming.md §6 G16 R1).
// Tickets are reset by the winner, so the caller's zeroed ticket buffer stays zero across
// launches (graph-replay safe).
// Deterministic: the merge order is fixed (rows in index order, phases in index order).
#pragma once
#include "hgk_common.h"

namespace hgk {

static constexpr int kTailGroup = 64;     // partial rows per level-1 group
static constexpr int kTailMaxGroups = 128;  // -> at most 8192 rows (= kMaxStatsRows)

// Hand-off of the partial rows: WRITE-THROUGH (sc1, agent-scope relaxed atomic) stores, drained
// by every storing wave before the workgroup barrier and the relaxed ticket add; the winner reads
// them with sc1 loads (bypassing this CU's L1), so neither side needs a release/acquire fence
// (cdna_hip_programming.md §6 G16 R1: an agent release per workgroup costs an L2 write-back).
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}

// Returns true (in every thread) if this workgroup is the last of `expected` arrivals on *cnt
// (and then resets *cnt to 0). The caller's sc1 stores must be issued before the call.
__device__ __forceinline__ bool tail_ticket(unsigned* cnt, unsigned expected, int* sflag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == expected - 1;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sflag = last;
  }
  __syncthreads();
  const bool last = *sflag != 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the sc1 loads below the ticket
  return last;
}

// Merge rows [r0, r1) of a [rows][NV][C] partial buffer. NV = 3: (sum, M2, n) rows -> per channel
// (S, M2, N) in fp64 via the exact decomposition M2 = sum_b M2_b + n_b (mean_b - mean)^2
// (two passes, no dependent chain of divisions). NV = 2: (a, b) sums. Results in res[c*3 + q].
template <int NV, int NT>
__device__ void tail_merge(const float* __restrict__ part, int r0, int r1, int C, double* red,
                           double* res) {
  const int tid = threadIdx.x;
  const int CH = C < NT ? C : NT;
  const int P = NT / CH;
  const int c_in = tid % CH, p = tid / CH;
  for (int cb = 0; cb < C; cb += CH) {
    const int c = cb + c_in;
    const bool act = p < P && c < C;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    if (act) {
      int r = r0 + p;
      for (; r + 3 * P < r1; r += 4 * P) {  // 4 rows' loads in flight
        float a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[u] = ld_sc1(&part[((long)(r + u * P) * NV + 0) * C + c]);
          b[u] = ld_sc1(&part[((long)(r + u * P) * NV + (NV == 3 ? 2 : 1)) * C + c]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          s0 += (double)a[u];
          if (NV == 3) s2 += (double)b[u];
          else s1 += (double)b[u];
        }
      }
      for (; r < r1; r += P) {
        s0 += (double)ld_sc1(&part[((long)r * NV + 0) * C + c]);
        if (NV == 3) s2 += (double)ld_sc1(&part[((long)r * NV + 2) * C + c]);
        else s1 += (double)ld_sc1(&part[((long)r * NV + 1) * C + c]);
      }
    }
    red[(p * CH + c_in) * 3 + 0] = s0;
    red[(p * CH + c_in) * 3 + 1] = s1;
    red[(p * CH + c_in) * 3 + 2] = s2;
    __syncthreads();
    if (p == 0 && c < C) {
      double a0 = 0.0, a1 = 0.0, a2 = 0.0;
      for (int q = 0; q < P; ++q) {
        a0 += red[(q * CH + c_in) * 3 + 0];
        a1 += red[(q * CH + c_in) * 3 + 1];
        a2 += red[(q * CH + c_in) * 3 + 2];
      }
      res[c * 3 + 0] = a0;
      res[c * 3 + 1] = a1;
      res[c * 3 + 2] = a2;
    }
    __syncthreads();
    if (NV == 3) {
      // second pass: M2 about the merged mean
      double m2 = 0.0;
      if (act) {
        const double mean = res[c * 3 + 2] > 0.0 ? res[c * 3 + 0] / res[c * 3 + 2] : 0.0;
        int r = r0 + p;
        for (; r + 3 * P < r1; r += 4 * P) {
          float sb[4], qb[4], nb[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            sb[u] = ld_sc1(&part[((long)(r + u * P) * 3 + 0) * C + c]);
            qb[u] = ld_sc1(&part[((long)(r + u * P) * 3 + 1) * C + c]);
            nb[u] = ld_sc1(&part[((long)(r + u * P) * 3 + 2) * C + c]);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const double d = nb[u] > 0.f ? (double)sb[u] / (double)nb[u] - mean : 0.0;
            m2 += (double)qb[u] + (double)nb[u] * d * d;
          }
        }
        for (; r < r1; r += P) {
          const float sb = ld_sc1(&part[((long)r * 3 + 0) * C + c]);
          const float qb = ld_sc1(&part[((long)r * 3 + 1) * C + c]);
          const float nb = ld_sc1(&part[((long)r * 3 + 2) * C + c]);
          const double d = nb > 0.f ? (double)sb / (double)nb - mean : 0.0;
          m2 += (double)qb + (double)nb * d * d;
        }
      }
      red[(p * CH + c_in) * 3 + 0] = m2;
      __syncthreads();
      if (p == 0 && c < C) {
        double a = 0.0;
        for (int q = 0; q < P; ++q) a += red[(q * CH + c_in) * 3 + 0];
        res[c * 3 + 1] = a;
      }
      __syncthreads();
    }
  }
}

// The whole tail for one workgroup that just wrote its partial row(s) [prow0, prow0 + nh).
// rows = total partial rows of the launch (gridDim.x * nh); gy workgroups (column tiles) write
// disjoint channel ranges of each row.
template <int NT>
__device__ void bn_tail(const hgk_bn_tail& t, const float* part, int NV, int rows, int C, long M,
                        int prow0, int nh, int gy, char* smem) {
  int* sflag = reinterpret_cast<int*>(smem);
  double* red = reinterpret_cast<double*>(smem + 16);   // [NT][3]
  double* res = red + NT * 3;                           // [C][3]
  const int G = (rows + kTailGroup - 1) / kTailGroup;
  const int g = prow0 / kTailGroup;
  const int g0 = g * kTailGroup, g1 = min(rows, g0 + kTailGroup);
  __syncthreads();  // the caller's LDS use is over
  // arrivals for group g: its rows / nh tiles (nh rows per workgroup) x gy column tiles
  if (!tail_ticket(&t.tickets[g], (unsigned)((g1 - g0) / nh * gy), sflag)) return;
  float* l2 = t.level2;
  if (G > 1) {
    if (NV == 3) tail_merge<3, NT>(part, g0, g1, C, red, res);
    else tail_merge<2, NT>(part, g0, g1, C, red, res);
    for (int c = threadIdx.x; c < C; c += NT) {
      if (NV == 3) {
        st_sc1(&l2[((long)g * 3 + 0) * C + c], (float)res[c * 3 + 0]);
        st_sc1(&l2[((long)g * 3 + 1) * C + c], (float)res[c * 3 + 1]);
        st_sc1(&l2[((long)g * 3 + 2) * C + c], (float)res[c * 3 + 2]);
      } else {
        st_sc1(&l2[((long)g * 2 + 0) * C + c], (float)res[c * 3 + 0]);
        st_sc1(&l2[((long)g * 2 + 1) * C + c], (float)res[c * 3 + 1]);
      }
    }
    if (!tail_ticket(&t.tickets[kTailMaxGroups], (unsigned)G, sflag)) return;
    if (NV == 3) tail_merge<3, NT>(l2, 0, G, C, red, res);
    else tail_merge<2, NT>(l2, 0, G, C, red, res);
  } else {
    if (NV == 3) tail_merge<3, NT>(part, 0, rows, C, red, res);
    else tail_merge<2, NT>(part, 0, rows, C, red, res);
  }
  // finalise (hgk_bn_finalize / hgk_bn_bwd_finalize semantics)
  for (int c = threadIdx.x; c < C; c += NT) {
    if (NV == 3) {
      const double n = res[c * 3 + 2];
      const double mu = n > 0.0 ? res[c * 3 + 0] / n : 0.0;
      const double var = res[c * 3 + 1] / (double)M;
      if (t.running_mean) {
        const double unbiased = M > 1 ? res[c * 3 + 1] / (double)(M - 1) : var;
        t.running_mean[c] = (float)((1.0 - t.momentum) * t.running_mean[c] + t.momentum * mu);
        t.running_var[c] = (float)((1.0 - t.momentum) * t.running_var[c] + t.momentum * unbiased);
      }
      const float is = (float)(1.0 / sqrt(var + (double)t.eps));
      const float gm = t.gamma ? t.gamma[c] : 1.f;
      const float bt = t.beta ? t.beta[c] : 0.f;
      const float sc = gm * is;
      t.stat[c] = (float)mu;
      t.stat[C + c] = is;
      t.stat[2 * C + c] = sc;
      t.stat[3 * C + c] = bt - (float)mu * sc;
    } else {
      const double sg = res[c * 3 + 0], sgx = res[c * 3 + 1];
      if (t.dgamma) t.dgamma[c] += (float)sgx;
      if (t.dbeta) t.dbeta[c] += (float)sg;
      const double sc = t.bn_scale[c];
      double c1 = 0.0, c2 = 0.0;
      if (t.training) {
        c1 = -sc * (double)t.bn_invstd[c] * sgx / (double)M;
        c2 = -sc * sg / (double)M;
      }
      t.coef[c] = (float)sc;
      t.coef[C + c] = (float)c1;
      t.coef[2 * C + c] = (float)c2;
      t.coef[3 * C + c] = t.bn_mean[c];
    }
  }
}

}  // namespace hgk
