// Image-tile convolution for the small hourglass levels (bf16, 1x1 and 3x3 / stride 1 / pad 1).
//
// At 16x16 and below (N = 32: M = 8192 .. 512 output pixels) a convolution is a chain of memory
// latencies, not work: the all-ahead implicit GEMM spent 0.5 us per 64-deep k-step in a barrier /
// transform / wait round trip, and its split-K seam (fp32 partial slabs, arrival counter, the
// last arriver re-reading every split cross-XCD) made a 3x3 at 8x8 or 4x4 a 14-16 us launch for
// 150 MFLOP (scripts/fwd_trace.py, profiles/r04_fwd_trace.txt).
//
// Here a workgroup owns 64 consecutive output pixels — R = 64 / W full image rows, i.e. whole
// images at 8x8 (one) and 4x4 (four), four-row strips at 16x16 — and BN output channels, and
// moves everything it needs into LDS in ONE burst:
//   * every weight k-chunk of its BN channels by LDS-DMA (global_load_lds_dwordx4, 128-B rows,
//     16-B slot c of row n at c ^ (n & 7): conflict-free fragment reads), the whole K at once
//     (3x3 128 -> 32 channels: 72 KB);
//   * the input halo of its rows ((R + 2) x (W + 2) positions per image, zero padding applied
//     after the BN(+ReLU) transform, every input pixel staged once per workgroup — not once per
//     tap as in the implicit GEMM), through registers so the transform runs on the way in;
//   * the input BN's constants, or its folded finalize (fold_merge, as the all-ahead kernel).
// One vmcnt(0) + one barrier later the MFMA stream (v_mfma_f32_16x16x32_bf16, 4 waves of 32
// pixels x BN / 2 channels) runs with no further synchronisation, over all taps and channel
// chunks; no split-K, so no cross-workgroup seam. The epilogue is the shared staged / coalesced /
// statistics / BN-backward-sums path (epi_store_half), so outputs, statistics partial rows
// (one per 64-pixel tile, as the 64-row implicit-GEMM tiles wrote them) and fused BN-backward
// sums have the formats every consumer already reads. Twin launches (an hourglass level's two
// chains, e.g. 8x8 + 4x4) run both segments' tiles in one grid.
#include "hgk_common.h"
#include "hgk_conv.h"

namespace hgk {

static constexpr int kImgBM = 64;      // output pixels per workgroup
static constexpr int kImgMaxHP = 160;  // halo positions per 64-channel chunk (4x4 images: 144)
static constexpr int kImgVgMaxRows = 32;  // folded BN-backward finalize: partial rows
#ifdef HGK_ABL_IMG_NOSTRIP  // ablation: no row strips
static constexpr long kImgStripMaxM = 0;
#else
static constexpr long kImgStripMaxM = 4096;  // 3x3 row strips: 64 tiles x 4 channel tiles = 256 WGs
#endif

// tile geometry of a 3x3 launch (rows of width W; whole images when H W <= 64)
struct ImgGeom {
  int R;    // output rows per tile (per image when the tile holds several images)
  int IMG;  // images per tile
  int HPI;  // halo positions per image: (R + 2) (W + 2)
  int HP;   // halo positions per tile
};

// floor(n / d) for 0 <= n < 2^22 from a float reciprocal of d (<= 1024): (n + 0.5) / d sits at
// least 0.5 / d from an integer, far above the float error — no integer division sequence
__device__ __forceinline__ int fdiv(int n, float rcp) { return (int)(((float)n + 0.5f) * rcp); }

__host__ __device__ inline ImgGeom img_geom(int H, int W) {
  ImgGeom g;
  const int hw = H * W;
  g.IMG = hw <= kImgBM ? kImgBM / hw : 1;
  g.R = hw <= kImgBM ? H : kImgBM / W;
  g.HPI = (g.R + 2) * (W + 2);
  g.HP = g.IMG * g.HPI;
  return g;
}

#ifdef HGK_FWD_TRACE  // timing build (scripts/fwd_trace.py): phase stamps of workgroups 0-511
__device__ unsigned long long g_imgtrace[512 * 16];
#define IT_STAMP(k)                                                                        \
  do {                                                                                     \
    const unsigned it_b = blockIdx.y * gridDim.x + blockIdx.x;                              \
    if (threadIdx.x == 0 && it_b < 512) g_imgtrace[it_b * 16 + (k)] = wall_clock64();       \
  } while (0)
#else
#define IT_STAMP(k)
#endif

// seg: 0 single launch, 1 / 2 segment 0 / 1 of a twin launch; part1 / rows1: segment 1's
// folded-finalize partials (for segment 0's dgamma owner)
template <int KS, int CIN, int BN, int VG>
__device__ __forceinline__ void img_body(const ConvFwdArgs& a, int mx, int ny, int seg,
                                         const float* part1, int rows1);

// VG: the input is the upstream gradient dA of a train-mode BN(+ReLU) whose backward APPLY (and,
// with vg_part, its finalize) is folded into the staging (hgk_bn_vgrad); VG = 2: plus the
// gradient already accumulated for the BN input (vg_add: bn1's skip gradient)
template <int KS, int CIN, int BN, bool TWIN, int VG>
__global__ __launch_bounds__(256, 1) void conv_img_kernel(ConvFwdArgs a0, ConvFwdArgs a1, int t0) {
  IT_STAMP(0);
  // the gy output-channel tiles of one pixel tile get block ids b, b + 8, ... (one XCD: the
  // halo rows they share are fetched into one L2)
  int mx = blockIdx.x, ny = blockIdx.y;
  if (gridDim.y > 1) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int b = blockIdx.y * gx + blockIdx.x;
    const int g = b / (8 * gy);
    const int cnt = min(8, gx - g * 8);
    const int r = b - g * 8 * gy;
    ny = r / cnt;
    mx = g * 8 + (r - ny * cnt);
  }
  if constexpr (TWIN) {
    const bool seg1 = mx >= t0;
    alignas(8) uint32_t wr[kArgWords];
    twin_pick(a0, a1, seg1, wr);
    // segment 0's first workgroup accumulates both segments' dgamma / dbeta (folded finalize)
    img_body<KS, CIN, BN, VG>(*reinterpret_cast<const ConvFwdArgs*>(wr), seg1 ? mx - t0 : mx, ny,
                              seg1 ? 2 : 1, a1.vg_part, a1.vg_rows);
  } else {
    img_body<KS, CIN, BN, VG>(a0, mx, ny, 0, nullptr, 0);
  }
}

// sums of a folded finalize's BN-backward partial rows [rows][2][CIN], in
// bn_bwd_fin_apply_kernel's order (thread (q, g) of G = 256 / (CIN / 2) groups adds rows g, g + G,
// ... in fp64; the group sums meet in LDS in group order): the coefficients are bit-identical
template <int CIN, int VFR>
__device__ __forceinline__ void vg_load_partials(const float* part, int rows, int tid, float4* pv) {
  constexpr int F4 = CIN / 2, GG = 256 / F4;
  const float4* p4 = reinterpret_cast<const float4*>(part);
  const int q = tid % F4, g = tid / F4;
#pragma unroll
  for (int u = 0; u < VFR; ++u) pv[u] = p4[(long)min(g + GG * u, rows - 1) * F4 + q];
}
template <int CIN, int VFR>
__device__ __forceinline__ void vg_group_sums(const float4* pv, int rows, int tid, double* red) {
  constexpr int F4 = CIN / 2, GG = 256 / F4;
  const int q = tid % F4, g = tid / F4;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
  for (int u = 0; u < VFR; ++u) {
    const bool ok = g + GG * u < rows;
    s0 += ok ? (double)pv[u].x : 0.0;
    s1 += ok ? (double)pv[u].y : 0.0;
    s2 += ok ? (double)pv[u].z : 0.0;
    s3 += ok ? (double)pv[u].w : 0.0;
  }
  double* rr = red + g * 2 * CIN + 4 * q;
  rr[0] = s0; rr[1] = s1; rr[2] = s2; rr[3] = s3;
}
// channel c's (sum g, sum g xhat) from the group sums (after a barrier)
template <int CIN>
__device__ __forceinline__ void vg_channel_sums(const double* red, int c, double& sg, double& sgx) {
  constexpr int GG = 256 / (CIN / 2);
  sg = 0.0; sgx = 0.0;
#pragma unroll
  for (int gg = 0; gg < GG; ++gg) { sg += red[gg * 2 * CIN + c]; sgx += red[gg * 2 * CIN + CIN + c]; }
}

template <int KS, int CIN, int BN, int VG>
__device__ __forceinline__ void img_body(const ConvFwdArgs& a, int mx, int ny, int seg,
                                         const float* part1, int rows1) {
  typedef bf16_t T;
  constexpr int NT = 256, BM = kImgBM;
  constexpr int TAPS = KS * KS, NCC = CIN / 64, NKC = TAPS * NCC;
  // KSPLIT (3x3): each wave computes the whole 64 x BN tile over a quarter of the k-steps
  // (k32 steps w, w + 4, ...), the four partial tiles are summed through LDS in a fixed order:
  // every A and B fragment is read from LDS once per workgroup (the 2 x 2 wave grid read each
  // twice — the MFMA stream was LDS-bandwidth bound). 1x1: the 2 x 2 wave grid.
  constexpr bool KSPLIT = KS == 3;
  constexpr int WM = KSPLIT ? 1 : 2, WN = KSPLIT ? 1 : 2;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int HPMAX = KS == 3 ? kImgMaxHP : BM;
  constexpr int WBYTES = NKC * BN * 128;
  constexpr int HBYTES = NCC * HPMAX * 128;
  constexpr int HLD = (NCC * HPMAX * 8 + NT - 1) / NT;  // halo 16-B chunks per thread
  constexpr int NU = NKC * BN / 8;                       // weight DMA units of 8 rows (1 KB)
  static_assert(NU % 4 == 0, "weight DMA units per wave");
  constexpr int LDC = BN + 8, ECH = BN / 8, ERPP = NT / ECH;
  constexpr int EPI = BM * LDC * 2 + ERPP * BN * 4 + BN * 4;
  static_assert(EPI <= WBYTES + HBYTES, "epilogue fits the main LDS");
  static_assert(FN >= 1 && CIN <= NT, "tile shape");
  __shared__ __attribute__((aligned(16))) char smem[WBYTES + HBYTES];
  __shared__ __attribute__((aligned(16))) float sPre[2 * CIN];  // BN scale | shift
  __shared__ float sBias[BN];
  __shared__ double sFold[NT];
  // VG: per channel k0 | k1 | k2 | mu (hgk_bn_bwd_finalize's coefficients) | forward scale | shift
  __shared__ __attribute__((aligned(16))) float sVg[VG ? 6 * CIN : 1];
  // folded finalize: partial rows per thread (rows <= kImgVgMaxRows = 256 / (CIN / 2) * VFR)
  constexpr int VFR = 32 / (256 / (CIN / 2));
  static_assert(!VG || CIN == 128 || (CIN == 256 && KS == 1), "folded BN-backward apply: 128 channels, 256 (1x1)");
  static_assert(!VG || (256 / (CIN / 2)) * 2 * CIN * 8 <= HBYTES, "finalize group sums fit the halo region");
  char* Wl = smem;
  char* Hl = smem + WBYTES;

  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ w = reinterpret_cast<const T*>(a.w);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = KSPLIT ? 0 : wave / WN, wn = KSPLIT ? 0 : wave % WN;  // tile position
  const int lr = lane & 15, lg = lane >> 4;
  const long m0 = (long)mx * BM;
  const int n0 = ny * BN;
  const int W = a.W, H = a.H;
  const ImgGeom gm = img_geom(H, W);
  const int HW2 = W + 2;
  const int hw = H * W;
  const float rW = 1.f / (float)W, rHW2 = 1.f / (float)HW2, rHW = 1.f / (float)hw;
  const float rHPI = 1.f / (float)gm.HPI, rPER = 1.f / (float)(gm.R * W);
  const int n_first = fdiv((int)m0, rHW);                    // first image of the tile
  const int h_first = fdiv((int)m0 - n_first * hw, rW);     // its first row (strips)

  // ---- halo geometry (ALU only, before any load is in flight) ----
  const int c8 = tid & 7;
  int hoff[HLD], hdst[HLD];
#pragma unroll
  for (int j = 0; j < HLD; ++j) {
    const int q = tid + j * NT;
    const int prow = q >> 3;  // (chunk, position) row
    const int cc = prow / HPMAX, pos = prow - cc * HPMAX;
    bool in = cc < NCC;
    int n = 0, hi = 0, wi = 0;
    if (KS == 3) {
      const int img = fdiv(pos, rHPI), rem = pos - img * gm.HPI;
      const int hr = fdiv(rem, rHW2), hc = rem - hr * HW2;
      n = n_first + img;
      hi = h_first - 1 + hr;
      wi = hc - 1;
      in = in && pos < gm.HP && hi >= 0 && hi < H && wi >= 0 && wi < W && n < a.N;
      hdst[j] = (cc < NCC && pos < gm.HP) ? cc * HPMAX * 128 + pos * 128 + ((c8 ^ (pos & 7)) << 4) : -1;
    } else {
      const int m = (int)m0 + pos;
      n = fdiv(m, rHW);
      const int rem = m - n * hw;
      hi = fdiv(rem, rW);
      wi = rem - hi * W;
      hdst[j] = cc < NCC ? cc * HPMAX * 128 + pos * 128 + ((c8 ^ (pos & 7)) << 4) : -1;
    }
    hoff[j] = in ? ((n * H + hi) * W + wi) * CIN + cc * 64 + c8 * 8 : -1;
  }
  // A-fragment base positions of this lane's pixel rows (top-left tap)
  int hb[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int p = wm * WTM + i * 16 + lr;
    if (KS == 3) {
      const int per = gm.R * W;
      const int img = fdiv(p, rPER), rem = p - img * per;
      const int r = fdiv(rem, rW), c = rem - r * W;
      hb[i] = img * gm.HPI + r * HW2 + c;
    } else {
      hb[i] = p;
    }
  }

  IT_STAMP(1);
  // ---- one burst: halo, BN constants / folded-finalize partials, bias, weights (LDS-DMA); the
  // halo first (it is needed first: transform and staging run while the weights stream in) ----
  uint4 hreg[HLD];
#pragma unroll
  for (int j = 0; j < HLD; ++j)
    if (hdst[j] >= 0) hreg[j] = *reinterpret_cast<const uint4*>(x + (hoff[j] >= 0 ? hoff[j] : c8 * 8));
  // VG: the BN input at the same positions, the finalize's partial rows, the channel constants
  uint4 yreg[VG ? HLD : 1];
  uint4 areg[VG == 2 ? HLD : 1];
  float4 pv[VG ? VFR : 1];
  const bool vfin = VG && a.vg_part != nullptr;
  // the dgamma / dbeta owner: the segment's first workgroup (twin: segment 0's, for both)
  const bool vown = vfin && mx == 0 && ny == 0 && seg != 2 &&
                    (a.vg_dgamma != nullptr || a.vg_dbeta != nullptr);
  float vsc = 0.f, vsh = 0.f, vk0 = 0.f, vk1 = 0.f, vk2 = 0.f, vmu = 0.f, vis = 0.f, vdg = 0.f, vdb = 0.f;
  if constexpr (VG) {
    const T* __restrict__ vy = reinterpret_cast<const T*>(a.vg_y);
#pragma unroll
    for (int j = 0; j < HLD; ++j)
      if (hdst[j] >= 0) yreg[j] = *reinterpret_cast<const uint4*>(vy + (hoff[j] >= 0 ? hoff[j] : c8 * 8));
    if constexpr (VG == 2) {
      const T* __restrict__ va = reinterpret_cast<const T*>(a.vg_add);
#pragma unroll
      for (int j = 0; j < HLD; ++j)
        if (hdst[j] >= 0) areg[j] = *reinterpret_cast<const uint4*>(va + (hoff[j] >= 0 ? hoff[j] : c8 * 8));
    }
    if (vfin) vg_load_partials<CIN, VFR>(a.vg_part, a.vg_rows, tid, pv);
    const int c = min(tid, CIN - 1);
    vsc = a.vg_scale[c];
    vsh = a.vg_shift[c];
    if (vfin) {
      vmu = a.vg_mean[c];
      vis = a.vg_invstd[c];
      if (vown) {
        vdg = a.vg_dgamma ? a.vg_dgamma[c] : 0.f;
        vdb = a.vg_dbeta ? a.vg_dbeta[c] : 0.f;
      }
    } else {
      vk0 = a.vg_coef[c];
      vk1 = a.vg_coef[CIN + c];
      vk2 = a.vg_coef[2 * CIN + c];
      vmu = a.vg_coef[3 * CIN + c];
    }
  }
  const bool fold = a.fold_part != nullptr;
  const bool has_pre = a.pre_scale != nullptr || fold;
  FoldRegs<kFoldRows / 4> fr;
  fold_setup(a, fold, tid, NT, fr);
  float pre_s = 0.f, pre_b = 0.f;
  if (fold) {
    fold_issue<kFoldRows / 4, true>(a, fr);
  } else if (has_pre) {
    const int c = min(tid, CIN - 1);
    pre_s = a.pre_scale[c];
    pre_b = a.pre_shift[c];
  }
  const float bias_v = (a.bias && tid < BN) ? a.bias[min(n0 + tid, a.Cout - 1)] : 0.f;
  {
    const int gch = (lane & 7) ^ (lane >> 3);
#pragma unroll
    for (int u0 = 0; u0 < NU; u0 += 4) {
      const int u = u0 + wave;
      const int kc = u / (BN / 8), rg = u - kc * (BN / 8);
      const int row = rg * 8 + (lane >> 3);
      dma16(w + (long)(n0 + row) * a.w_ld + kc * 64 + gch * 8, Wl + (kc * BN + rg * 8) * 128);
    }
  }

  IT_STAMP(2);
  if constexpr (VG) {
    if (vfin) {
      // hgk_bn_bwd_finalize_apply's coefficients (same fp64 sums, same expressions)
      double* red = reinterpret_cast<double*>(Hl);  // the halo region is written after 2 barriers
      vg_group_sums<CIN, VFR>(pv, a.vg_rows, tid, red);
      __syncthreads();
      if (tid < CIN) {
        double sg, sgx;
        vg_channel_sums<CIN>(red, tid, sg, sgx);
        const double sc = vsc, is = vis;
        double c1 = 0.0, c2 = 0.0;
        if (a.vg_training) {
          c1 = -sc * is * sgx / (double)a.vg_M;
          c2 = -sc * sg / (double)a.vg_M;
        }
        vk0 = (float)sc;
        vk1 = (float)c1;
        vk2 = (float)c2;
        if (vown) {
          vdg = vdg + (float)sgx;
          vdb = vdb + (float)sg;
          if (seg == 0) {  // single launch: final
            if (a.vg_dgamma) a.vg_dgamma[tid] = vdg;
            if (a.vg_dbeta) a.vg_dbeta[tid] = vdb;
          }
        }
      }
    }
    if (tid < CIN) {
      sVg[tid] = vk0;
      sVg[CIN + tid] = vk1;
      sVg[2 * CIN + tid] = vk2;
      sVg[3 * CIN + tid] = vmu;
      sVg[4 * CIN + tid] = vsc;
      sVg[5 * CIN + tid] = vsh;
    }
  }
  if (fold) fold_merge(a, fr, tid, sFold, mx == 0 && ny == 0, pre_s, pre_b);
  if (has_pre && tid < CIN) {
    sPre[tid] = pre_s;
    sPre[CIN + tid] = pre_b;
  }
  if (tid < BN) sBias[tid] = (n0 + tid < a.Cout) ? bias_v : 0.f;
  IT_STAMP(3);
  __syncthreads();
  IT_STAMP(4);

  // halo: BN(+ReLU) transform, zero padding AFTER it (the conv pads the activated input)
  const bool relu = a.pre_relu != 0;
#pragma unroll
  for (int j = 0; j < HLD; ++j) {
    if (hdst[j] < 0) continue;
    uint4 v = hreg[j];
    if constexpr (VG) {
      // dy = bn_bwd_apply(dA, y) (bnb_apply: the apply kernels' bits); the segment's first
      // channel tile also stores it for the weight gradient (halo positions >= 0 are this tile's
      // own pixels: whole images / 1x1)
      const int cb = (hdst[j] / (HPMAX * 128)) * 64 + c8 * 8;
      float fd[8], fy[8], o[8];
      unpack16<T>(v, fd);
      unpack16<T>(yreg[j], fy);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o[e] = bnb_apply(fd[e], fy[e], sVg[4 * CIN + cb + e], sVg[5 * CIN + cb + e], sVg[cb + e],
                         sVg[CIN + cb + e], sVg[2 * CIN + cb + e], sVg[3 * CIN + cb + e], a.vg_relu != 0);
      if constexpr (VG == 2) {
        float fa[8];
        unpack16<T>(areg[j], fa);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += fa[e];
      }
      v = pack16<T>(o);
      if (ny == 0 && hoff[j] >= 0) store16(reinterpret_cast<T*>(a.vg_out) + hoff[j], v);
    } else if (has_pre) {
      const int cc = hdst[j] / (HPMAX * 128);
      const float* sp = sPre + cc * 64 + c8 * 8;
      float ps[8], pb[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ps[e] = sp[e];
        pb[e] = sp[CIN + e];
      }
      v = bn_relu_chunk<bf16_t>(v, ps, pb, relu);
    }
    const uint32_t keep = hoff[j] >= 0 ? 0xffffffffu : 0u;
    v.x &= keep; v.y &= keep; v.z &= keep; v.w &= keep;
    *reinterpret_cast<uint4*>(Hl + hdst[j]) = v;
  }
  IT_STAMP(5);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's weight DMAs have landed
  IT_STAMP(6);
  __syncthreads();
  IT_STAMP(7);

  // ---- MFMA stream: every tap and channel chunk, no synchronisation ----
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragments of k32 step (kc, kk); software-pipelined: step s + 1's LDS reads are issued before
  // step s's MFMAs (counted lgkmcnt waits from the straight-line schedule), so LDS latency hides
  // behind the matrix work instead of adding to it once per step
  auto kload = [&](int kc, int kk, bf16x8* av, bf16x8* bv) __attribute__((always_inline)) {
    const int tap = kc / NCC, cc = kc - tap * NCC;
    const int kh = tap / KS, kw = tap - kh * KS;
    const int toff = KS == 3 ? kh * HW2 + kw : 0;
    const int cidx = kk * 4 + lg;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int pos = hb[i] + toff;
      av[i] = *reinterpret_cast<const bf16x8*>(Hl + cc * HPMAX * 128 + pos * 128 +
                                               ((cidx ^ (pos & 7)) << 4));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = wn * WTN + j * 16 + lr;
      bv[j] = *reinterpret_cast<const bf16x8*>(Wl + (kc * BN + n) * 128 + ((cidx ^ (n & 7)) << 4));
    }
  };
  auto kmma = [&](const bf16x8* av, const bf16x8* bv) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
  };
  // this wave's k32 steps: KSPLIT the steps w, w + 4, ... of 2 NKC; else all of them
  constexpr int NSW = KSPLIT ? 2 * NKC / 4 : 2 * NKC;
  static_assert(!KSPLIT || (2 * NKC) % 4 == 0, "k-steps per wave");
  auto step_of = [&](int i) __attribute__((always_inline)) { return KSPLIT ? wave + 4 * i : i; };
  bf16x8 Ab[2][FM], Bb[2][FN];
  kload(step_of(0) >> 1, step_of(0) & 1, Ab[0], Bb[0]);
#pragma unroll
  for (int i = 0; i < NSW; ++i) {
    if (i + 1 < NSW) {
      const int sn = step_of(i + 1);
      kload(sn >> 1, sn & 1, Ab[(i + 1) & 1], Bb[(i + 1) & 1]);
    }
    kmma(Ab[i & 1], Bb[i & 1]);
  }
  IT_STAMP(8);
  __syncthreads();  // every fragment read of the main LDS is done
  if constexpr (KSPLIT) {
    // the four waves' partial tiles -> LDS [wave][frag][lane][4]; each wave then sums a quarter
    // of the fragments over the waves in order 0..3 (deterministic) into acc
    constexpr int NF = FM * FN;
    static_assert(NF % 4 == 0, "fragments per wave in the reduction");
    f32x4* part = reinterpret_cast<f32x4*>(smem);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) part[(wave * NF + i * FN + j) * 64 + lane] = acc[i][j];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int f = i * FN + j;
        if (f / (NF / 4) != wave) continue;
        f32x4 v = part[f * 64 + lane];
#pragma unroll
        for (int w2 = 1; w2 < 4; ++w2) {
          const f32x4 q = part[(w2 * NF + f) * 64 + lane];
          v[0] += q[0]; v[1] += q[1]; v[2] += q[2]; v[3] += q[3];
        }
        acc[i][j] = v;
      }
  }

  // ---- epilogue: the shared staged / coalesced / statistics path ----
  // (KSPLIT: behind the partial tiles, which are still being read)
  constexpr int EPI0 = KSPLIT ? 4 * FM * FN * 64 * 16 : 0;
  static_assert(EPI0 + EPI <= WBYTES + HBYTES, "epilogue behind the partial tiles");
  T* Cs = reinterpret_cast<T*>(smem + EPI0);
  float* red = reinterpret_cast<float*>(smem + EPI0 + BM * LDC * sizeof(T));
  float* bmean = red + ERPP * BN;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = wn * WTN + j * 16 + lr;
    const float bj = sBias[c];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (KSPLIT && (i * FN + j) / (FM * FN / 4) != wave) continue;  // this wave's reduced fragments
      const int rbase = wm * WTM + i * 16;
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(rbase + lg * 4 + r) * LDC + c] = from_f<T>(acc[i][j][r] + bj);
    }
  }
  __syncthreads();
  IT_STAMP(9);
  epi_store_half<T, BM, BN, NT, BM, 1>(a, Cs, red, bmean, m0, n0, 0, tid, mx);
  if constexpr (VG) {
    if (vown && seg == 1) {
      // twin: segment 1's sums, then dgamma = (dgamma + x0) + x1 (hgk_bn_bwd_twin's order)
      float4 pv1[VFR];
      vg_load_partials<CIN, VFR>(part1, rows1, tid, pv1);
      double* red1 = reinterpret_cast<double*>(smem);
      __syncthreads();  // the epilogue's LDS reads are done
      vg_group_sums<CIN, VFR>(pv1, rows1, tid, red1);
      __syncthreads();
      if (tid < CIN) {
        double sg, sgx;
        vg_channel_sums<CIN>(red1, tid, sg, sgx);
        if (a.vg_dgamma) a.vg_dgamma[tid] = vdg + (float)sgx;
        if (a.vg_dbeta) a.vg_dbeta[tid] = vdb + (float)sg;
      }
    }
  }
  IT_STAMP(15);
}

// ---------------------------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------------------------
static int img_bn(int ks) { return ks == 3 ? 32 : 64; }

static bool img_shape_ok(const ConvFwdArgs& a) {
  const int ks = a.KH;
  if (!(ks == 1 || ks == 3) || a.KW != ks || a.stride != 1 || a.dil != 1 || a.pad != (ks == 3 ? 1 : 0))
    return false;
  if (a.H != a.Ho || a.W != a.Wo || a.M % kImgBM != 0 || a.w_ld % 8 != 0) return false;
  // folded BN-backward apply: 128 channels; its folded finalize: <= 32 partial rows (one batch of
  // loads per thread in the prologue)
  // (+ add: the 256-channel 1x1 only, with the folded finalize)
  if (a.vg_y) {
    const bool c128 = a.Cin == 128 && !a.vg_add;
#ifdef HGK_ABL_IMG_NOADD  // ablation: no skip-gradient fold (bn1 keeps its finalize+apply launch)
    const bool c256 = false;
#else
    const bool c256 = a.Cin == 256 && ks == 1 && a.vg_add && a.vg_part;
#endif
    if (!(c128 || c256) || (a.vg_part && a.vg_rows > kImgVgMaxRows)) return false;
  }
  if (ks == 3 ? a.Cin != 128 : (a.Cin != 128 && a.Cin != 256)) return false;
  if (a.Cout % img_bn(ks) != 0) return false;
  if (ks == 3) {
    // whole images (8x8, 4x4), or row strips (16x16) where the launch is one round of
    // workgroups (M <= kImgStripMaxM: the N = 16 of try_with_aspp); at N = 32 (two rounds) the
    // halo kernel is faster on 16x16 (13.2 vs 18.5 us, scripts/img_bench.py). A folded
    // BN-backward apply needs whole images (its dy stores cover the halo's own pixels only)
    if (a.W > kImgBM || kImgBM % a.W != 0) return false;
    const int hw = a.H * a.W;
    if (hw > kImgBM) {
      if (a.M > kImgStripMaxM || a.vg_y || a.H % (kImgBM / a.W) != 0) return false;
    } else if (kImgBM % hw != 0) {
      return false;
    }
    if (img_geom(a.H, a.W).HP > kImgMaxHP) return false;
  }
  return (long)a.M / kImgBM <= kMaxStatsRows;
}

// route HGK_ROUTE_IMG: the largest M (per segment) that takes this kernel; 0 = off
bool img_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1) {
  const long maxm = route(HGK_ROUTE_IMG);
  if (maxm <= 0 || !img_shape_ok(a) || a.M > maxm) return false;
  if (!a1) return true;
  return img_shape_ok(*a1) && a1->M <= maxm && a1->KH == a.KH && a1->Cin == a.Cin &&
         a1->Cout == a.Cout && a1->pre_relu == a.pre_relu && (a1->fold_part == nullptr) == (a.fold_part == nullptr) &&
         (a1->vg_y == nullptr) == (a.vg_y == nullptr) && (a1->vg_part == nullptr) == (a.vg_part == nullptr) &&
         (a1->vg_add == nullptr) == (a.vg_add == nullptr) &&
         a1->vg_relu == a.vg_relu;
}

template <int KS, int CIN, int BN, int VG>
static void img_launch_t(hipStream_t st, ConvFwdArgs& a, ConvFwdArgs* b, int g0, int g1, int gy) {
  if (b)
    hipLaunchKernelGGL((conv_img_kernel<KS, CIN, BN, true, VG>), dim3(g0 + g1, gy), dim3(256), 0, st, a, *b, g0);
  else
    hipLaunchKernelGGL((conv_img_kernel<KS, CIN, BN, false, VG>), dim3(g0, gy), dim3(256), 0, st, a, a,
                       kNoTwin);
}

// route HGK_ROUTE_IMG_NARROW: 1x1 launches of at most this many rows (both segments) take
// 32-channel output tiles — twice the workgroups, half the weight burst and MFMA chain per
// workgroup (the 8x8 / 4x4 levels: 8-64 workgroups of a latency-bound launch); 0 = off
static bool img_narrow(const ConvFwdArgs& a, const ConvFwdArgs* b) {
  return a.KH == 1 && a.Cout % 32 == 0 && a.M + (b ? b->M : 0) <= route(HGK_ROUTE_IMG_NARROW);
}

int launch_img(hipStream_t st, ConvFwdArgs& a, ConvFwdArgs* b, int* rows0, int* rows1) {
  const int g0 = (int)(a.M / kImgBM), g1 = b ? (int)(b->M / kImgBM) : 0;
  a.stats_R = g0;
  if (b) b->stats_R = g1;
  const bool narrow = img_narrow(a, b);
  const int ks = a.KH, bn = narrow ? 32 : img_bn(ks);
  const int gy = a.Cout / bn;
  const bool vg = a.vg_y != nullptr;  // img_ok: both segments or neither
  if (narrow) {
    if (a.Cin == 128) {
      if (vg)
        img_launch_t<1, 128, 32, 1>(st, a, b, g0, g1, gy);
      else
        img_launch_t<1, 128, 32, 0>(st, a, b, g0, g1, gy);
    } else {
      if (vg)
        img_launch_t<1, 256, 32, 2>(st, a, b, g0, g1, gy);
      else
        img_launch_t<1, 256, 32, 0>(st, a, b, g0, g1, gy);
    }
  } else if (ks == 3) {
    if (vg)
      img_launch_t<3, 128, 32, 1>(st, a, b, g0, g1, gy);
    else
      img_launch_t<3, 128, 32, 0>(st, a, b, g0, g1, gy);
  } else if (a.Cin == 128) {
    if (vg)
      img_launch_t<1, 128, 64, 1>(st, a, b, g0, g1, gy);
    else
      img_launch_t<1, 128, 64, 0>(st, a, b, g0, g1, gy);
  } else {
    if (vg)  // img_ok: the add variant only (bn1's skip gradient)
      img_launch_t<1, 256, 64, 2>(st, a, b, g0, g1, gy);
    else
      img_launch_t<1, 256, 64, 0>(st, a, b, g0, g1, gy);
  }
  HGK_LAUNCH_CHECK();
  if (rows0) *rows0 = (a.stats || a.bb_partial) ? g0 : 0;
  if (rows1) *rows1 = (b && (b->stats || b->bb_partial)) ? g1 : 0;
  return HGK_OK;
}

}  // namespace hgk

#ifdef HGK_FWD_TRACE
extern "C" int hgk_debug_img_trace(void* dst, int reset) {
  if (reset) {
    static unsigned long long zero[512 * 16];
    return hipMemcpyToSymbol(HIP_SYMBOL(hgk::g_imgtrace), zero, sizeof(zero)) == hipSuccess ? 0 : 1;
  }
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(hgk::g_imgtrace), sizeof(hgk::g_imgtrace)) == hipSuccess ? 0 : 1;
}
#endif
