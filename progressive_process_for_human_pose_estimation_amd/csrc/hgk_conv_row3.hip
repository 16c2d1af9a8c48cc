// Row-streaming 3x3 convolution: the ResidualBlock's 128 -> 128 3x3 (try_with_torch.py:189, conv2)
// at the 64x64 and 32x32 levels, forward (BN+ReLU input transform, statistics out) and input
// gradient (BN-backward partial sums of the produced dA), single or twin (two segments, one grid).
//
// The halo kernel (hgk_conv.hip) re-streams the 295 KB weight tensor through LDS for every
// 128-pixel tile and runs each tile's phases (halo load, 18 weight steps, epilogue) back to back:
// with neither the weight DMA nor the MFMAs it still took 37.5 of its 60 us at 64x64
// (profiles/r03_halo_ablation2.txt). Here the weights stay in REGISTERS for the whole launch and
// the input streams through: one workgroup per CU (8 waves; wave w owns output channels
// 16w..16w+15 and holds their 9 taps x 128 input channels, 144 VGPRs), a contiguous run of output
// rows per workgroup, and a 6-slot LDS ring of input rows (every input row loaded once per
// workgroup, W+2 positions with zero pads, one LDS-DMA round per row). Output row r reads rows
// r-1, r, r+1; per 16-pixel tile every wave runs 36 MFMAs (16x16x32) whose B fragments are
// ds_read_b128 at the tap's shifted position: LDS row layout 256 B per position with 16-B chunk c
// of position p in slot c ^ (p & 15). Per iteration ONE barrier: row i+3 has landed (counted vmcnt)
// and is transformed (BN+ReLU, in place) behind row i's MFMAs; the slot of row i-1 takes the DMA
// of row i+R-1. The input gradient's BN-backward sums read the BN input row through one more
// LDS-DMA row (a second barrier per iteration). Partial rows: one per output row (channel-major statistics [128][3][N*H]; BN-
// backward [N*H][2][128]), reduced over the stored (bf16) outputs.
#include "hgk_conv.h"

namespace hgk {

static constexpr int kR3C = 128;               // channels in and out
static constexpr int kR3WMax = 64;
static constexpr int kR3SlotB = (kR3WMax + 2) * 256;
// ring + zero row (+ BN input row) + partial-sum exchange: 7 rows + 32 KB
static constexpr int kR3Lds = 7 * kR3SlotB + 8 * (kR3WMax / 16) * 1024;
#ifndef HGK_ROW3_PF
#define HGK_ROW3_PF 6  // B fragments in flight per wave
#endif

#ifdef HGK_R3_TRACE  // timing build (scripts only): per-iteration phase stamps of wave 0, 4 workgroups
__device__ unsigned long long g_r3trace[4 * 16 * 6];
#define R3_STAMP(k)                                                                     \
  if (trace_on && i < 16) {                                                             \
    const unsigned long long c = clock64();                                             \
    if (lane == 0) g_r3trace[(wg * 16 + i) * 6 + (k)] = c;                              \
  }
#else
#define R3_STAMP(k)
#endif

struct Row3Seg {
  const bf16_t* x;
  bf16_t* y;
  const float *pre_scale, *pre_shift;
  float* stats;
  const bf16_t* bby;
  const float *bsc, *bsh, *bmu, *bis;
  float* bpart;
  // folded BN-backward apply of the input (mode 16): x is the upstream gradient dA of a
  // train-mode BN(+ReLU) whose input is vgy; the conv consumes dy = bnb_apply(dA, vgy, ...) and
  // also stores it to vout (the weight gradient's operand)
  const bf16_t* vgy;
  const float *vsc, *vsh, *vco;
  bf16_t* vout;
  int N, H, W;
};

struct Row3Args {
  Row3Seg s[2];
  const bf16_t* w;
  const float* bias;
  int w_ld, pre_relu, bb_relu, vg_relu;
  int g0, g1;  // workgroups of segment 0 / 1
  int alt_order;
};

template <int MODE, int W>
__device__ __forceinline__ void row3_body(const Row3Args& ra, const Row3Seg& sg, int wg, int G,
                                          char* smem, float* sPre, float* sBb, float* sVg) {
  constexpr bool PRE = MODE & 1, BBM = (MODE & 4) != 0, STATS = (MODE & 8) != 0,
                 VG = (MODE & 16) != 0;
  static_assert(!VG || (BBM && !PRE), "the folded apply comes with the BN-backward sums");
  constexpr int NT = 512, NW = 8;
  // input-row ring slots (BBM: one row of LDS for bby; VG: one more for the BN input rows)
  constexpr int R = VG ? 4 : BBM ? 5 : 6;
  constexpr int D = W * 256 / (NW * 1024);  // 1-KB DMA pieces per wave per row
  constexpr int TPR = W / 16;               // 16-pixel tiles per row
  constexpr int XC = W * 16 / NT;           // transform chunks per thread per row
  constexpr int ZS = R;                     // the zero row
  static_assert(D >= 1 && D * NW * 1024 == W * 256 && XC >= 1, "row geometry");
  static_assert((R + 1 + (BBM ? 1 : 0) + (VG ? 1 : 0)) * kR3SlotB + NW * TPR * 1024 <= kR3Lds,
                "LDS plan");
  // LDS: ring [R slots + zero row] | BBM: BN input row | partial-sum exchange [wave][tile][lane]
  char* const ring = smem;
  char* const bybuf = smem + (R + 1) * kR3SlotB;
  char* const yslot = smem + (R + 2) * kR3SlotB;  // VG: the BN input row of the row in flight
  char* const xch = smem + (R + 1 + (BBM ? 1 : 0) + (VG ? 1 : 0)) * kR3SlotB;
  // ops of one iteration on the vm counter: the BN input row's DMA (BBM), the input row's DMA,
  // the output stores + the partial-row store. Every load of the loop is an LDS-DMA issued from
  // asm: a compiler-visible global load would make hipcc wait for all of them
  constexpr int BD = BBM ? D : 0, ST = TPR + ((STATS || BBM) ? 1 : 0), XI = BD + D + ST;
  // at iteration i, loaded row i + NEED must have landed (PRE: transformed one iteration ahead)
  constexpr int NEED = PRE ? 3 : 2, K0 = R - 1 - NEED;
  static_assert(VG || (K0 >= 1 && K0 <= 3), "ring depth");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
  // wave = (g, h): partial sums of output channels 32g .. 32g+31 over input channels 64h .. 64h+63;
  // after the exchange it owns channels co .. co+15 of every pixel
  const int g = wave & 3, h = wave >> 2;
  const int co = 32 * g + 16 * h;
  const int H = sg.H, rows = sg.N * H;
  const int o0 = (int)((long)wg * rows / G), o1 = (int)((long)(wg + 1) * rows / G);
  const int nrow = o1 - o0;
  if (nrow <= 0) return;  // workgroup-uniform, before any barrier
  // route row3_alt (ra.alt_order): odd workgroups run their rows bottom-up, so two neighbouring
  // runs (same XCD, see the kernel) read their shared boundary rows at about the same time — both
  // at their first rows or both at their last — and the second read hits the XCD's L2: HBM bytes
  // 1.40x -> 1.21x the algorithmic, but +1 us per 64x64 launch (profiles/r05_row3_alt_order.txt),
  // so off by default. Every output row is computed the same way in either order (bitwise).
  const bool rev = ra.alt_order && (wg & 1) != 0;
  // row key of loaded index n (0 .. nrow + 1) and of output row i (0 .. nrow - 1)
  auto lkey = [&](int n) __attribute__((always_inline)) { return rev ? o1 - n : o0 - 1 + n; };
#ifdef HGK_R3_TRACE
  const bool trace_on = wg < 4 && wave == 0 && sg.W == W && (&sg == &ra.s[0]);
#endif
  // loaded index n <-> input row key o0 - 1 + n (key = image * H + row), n = 0 .. nrow + 1; keys
  // outside [0, rows) load a clamped row into their (unused) slot, keeping the op count fixed
  const bf16_t* __restrict__ x = sg.x;
  int soff[D];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const int o = (j * NW + wave) * 1024 + lane * 16;  // byte offset from position 1
    const int p = 1 + o / 256, js = (o % 256) / 16;
    soff[j] = (p - 1) * kR3C + ((js ^ (p & 15)) * 8);
  }
  auto issue_by = [&](int key) __attribute__((always_inline)) {
    const bf16_t* src = sg.bby + (long)key * W * kR3C;
#pragma unroll
    for (int j = 0; j < D; ++j) dma16(src + soff[j], bybuf + 256 + (j * NW + wave) * 1024);
  };
  auto issue = [&](int n) __attribute__((always_inline)) {
    const int key = min(max(lkey(n), 0), rows - 1);
    const bf16_t* src = x + (long)key * W * kR3C;
    char* dst = ring + (n % R) * kR3SlotB + 256;
#pragma unroll
    for (int j = 0; j < D; ++j) dma16(src + soff[j], dst + (j * NW + wave) * 1024);
  };
  // VG: the BN input row of loaded row n into ybuf (same pieces as the row's own DMA)
  auto issue_y = [&](int n, char* ybuf) __attribute__((always_inline)) {
    const int key = min(max(lkey(n), 0), rows - 1);
    const bf16_t* src = sg.vgy + (long)key * W * kR3C;
#pragma unroll
    for (int j = 0; j < D; ++j) dma16(src + soff[j], ybuf + 256 + (j * NW + wave) * 1024);
  };
  // VG: dy = bnb_apply(dA, y) of loaded row n in place, over the pieces THIS wave loaded (its own
  // counted vmcnt orders them; no barrier); rows the workgroup owns (n = 1 .. nrow) also go to vout
  const bool vrelu = ra.vg_relu != 0;
  auto transform_vg = [&](int n, const char* ybuf) __attribute__((always_inline)) {
    const bool own = n >= 1 && n <= nrow;
    const long rowbase = (long)lkey(n) * W * kR3C;
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int o = (j * NW + wave) * 1024 + lane * 16;
      const int p = 1 + o / 256, c = ((o % 256) / 16) ^ (p & 15);
      char* cp = ring + (n % R) * kR3SlotB + 256 + o;
      float fd[8], fy[8], out[8];
      unpack16<bf16_t>(*reinterpret_cast<const uint4*>(cp), fd);
      unpack16<bf16_t>(*reinterpret_cast<const uint4*>(ybuf + 256 + o), fy);
      // four channels at a time: the weights hold 144 registers
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        // asm reads: the coefficients are loop invariant, and hoisted they took 96 registers
        float k[6][4];
        f32x4 kv[6];
        const uint32_t ka = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)(sVg + c * 8 + 4 * hf);
#pragma unroll
        for (int q = 0; q < 6; ++q)
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kv[q]) : "v"(ka), "i"(q * kR3C * 4));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kv[0]), "+v"(kv[1]), "+v"(kv[2]), "+v"(kv[3]), "+v"(kv[4]), "+v"(kv[5]));
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          k[q][0] = kv[q][0]; k[q][1] = kv[q][1]; k[q][2] = kv[q][2]; k[q][3] = kv[q][3];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
          out[4 * hf + e] = bnb_apply(fd[4 * hf + e], fy[4 * hf + e], k[0][e], k[1][e], k[2][e],
                                      k[3][e], k[4][e], k[5][e], vrelu);
      }
      const uint4 pk = pack16<bf16_t>(out);
      *reinterpret_cast<uint4*>(cp) = pk;
      if (own) store16(sg.vout + rowbase + soff[j], pk);
    }
  };

  // ---- prologue: zero pads / zero row, first R-1 rows in flight, constants, weights ----
  {
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    // pads (positions 0 and W+1) of the R ring slots: 2 x 16 chunks each
    if (tid < R * 32) {
      const int sl = tid / 32, c = tid % 32;
      const int pos = c < 16 ? 0 : W + 1;
      *reinterpret_cast<uint4*>(ring + sl * kR3SlotB + pos * 256 + (c % 16) * 16) = z;
    }
    for (int c = tid; c < (W + 2) * 16; c += NT)
      *reinterpret_cast<uint4*>(ring + ZS * kR3SlotB + c * 16) = z;
  }
#pragma unroll
  for (int n = 0; n < R - 1; ++n) issue(n);
  if constexpr (VG) {
    // the BN input rows of loaded rows 0, 1, 2: the y slot, the bby buffer and ring slot 3 (all
    // free until iteration 0)
    static_assert(R == 4, "prologue buffers assume 4 ring slots");
    issue_y(0, yslot);
    issue_y(1, bybuf);
    issue_y(2, ring + 3 * kR3SlotB);
  }
  float vg_v[2] = {0.f, 0.f};
  if constexpr (VG) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i6 = tid + u * NT;
      if (i6 < 6 * kR3C) {
        const int part = i6 / kR3C, c = i6 % kR3C;
        vg_v[u] = part == 0 ? sg.vsc[c] : part == 1 ? sg.vsh[c] : sg.vco[(part - 2) * kR3C + c];
      }
    }
  }
  float pv_s = 0.f, pv_b = 0.f;
  if (PRE && tid < kR3C) {
    pv_s = sg.pre_scale[tid];
    pv_b = sg.pre_shift[tid];
  }
  float bias4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bias4[i] = ra.bias ? ra.bias[co + 4 * lg + i] : 0.f;
  // BN-backward constants -> LDS [scale | shift | invstd | -mean * invstd][128] (read per tile)
  float bb_v = 0.f;
  if (BBM) {
    const int part = tid / kR3C, c = tid % kR3C;
    bb_v = part == 0 ? sg.bsc[c] : part == 1 ? sg.bsh[c] : part == 2 ? sg.bis[c] : -sg.bmu[c] * sg.bis[c];
  }
  // weights: A fragment of (tap, k-step kq of this half, channel tile j) = rows 32g + 16j + lr,
  // input channels 64h + 32kq + 8lg .. +7
  bf16x8 wreg[9][2][2];
  {
    const bf16_t* wp = ra.w + (long)(32 * g + lr) * ra.w_ld + 64 * h + lg * 8;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int kq = 0; kq < 2; ++kq)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          wreg[t][kq][j] =
              *reinterpret_cast<const bf16x8*>(wp + (long)16 * j * ra.w_ld + t * kR3C + kq * 32);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (PRE && tid < kR3C) { sPre[tid] = pv_s; sPre[kR3C + tid] = pv_b; }
  if (BBM) sBb[tid] = bb_v;
  if constexpr (VG) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (tid + u * NT < 6 * kR3C) sVg[tid + u * NT] = vg_v[u];
  }
  __syncthreads();
  if constexpr (VG) {
    transform_vg(0, yslot);
    transform_vg(1, bybuf);
    transform_vg(2, ring + 3 * kR3SlotB);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // BN(+ReLU) of loaded row n, in place (positions 1..W; the pads stay zero)
  const bool relu = ra.pre_relu != 0;
  auto transform = [&](int n) __attribute__((always_inline)) {
    char* base = ring + (n % R) * kR3SlotB + 256;
#pragma unroll
    for (int u = 0; u < XC; ++u) {
      const int ci = tid + u * NT;
      const int p = 1 + ci / 16, c = (ci % 16) ^ (p & 15);
      float ps[8], pb[8];
      const float4 s0 = *reinterpret_cast<const float4*>(sPre + c * 8);
      const float4 s1 = *reinterpret_cast<const float4*>(sPre + c * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(sPre + kR3C + c * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(sPre + kR3C + c * 8 + 4);
      ps[0] = s0.x; ps[1] = s0.y; ps[2] = s0.z; ps[3] = s0.w;
      ps[4] = s1.x; ps[5] = s1.y; ps[6] = s1.z; ps[7] = s1.w;
      pb[0] = b0.x; pb[1] = b0.y; pb[2] = b0.z; pb[3] = b0.w;
      pb[4] = b1.x; pb[5] = b1.y; pb[6] = b1.z; pb[7] = b1.w;
      uint4* cp = reinterpret_cast<uint4*>(base + ci * 16);
      *cp = bn_relu_chunk<bf16_t>(*cp, ps, pb, relu);
    }
  };
  if constexpr (PRE) {
    transform(0);
    transform(1);
    transform(2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // B fragment of (kw, kq) in a row, tile 0: position lr + kw, chunk (2h + kq) * 4 + lg
  int loff[3][2];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int kq = 0; kq < 2; ++kq) {
      const int p = lr + kw;
      loff[kw][kq] = p * 256 + ((((2 * h + kq) * 4 + lg) ^ (p & 15)) << 4);
    }

#ifdef HGK_ABL_R3_PROLOGUE  // ablation: prologue only (wrong results; timing only)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return;
#endif
#pragma unroll 1
  for (int i = 0; i < nrow; ++i) {
    R3_STAMP(0)
    // loaded row i + NEED landed for this wave. Issue order per iteration j: [BN input DMA]
    // [input DMA of row j + R - 1] [stores]; younger than that row's DMA: the rest of its
    // iteration's ops and every op of the iterations after it
    if constexpr (VG) {
      // rows i .. i + 2 were transformed by their own waves at the end of earlier iterations
    } else if (i >= K0)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ST + (R - 2 - NEED) * XI) : "memory");
    else if (i == 0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (i == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(XI) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * XI) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    R3_STAMP(1)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    R3_STAMP(2)
    const int key = rev ? o1 - 1 - i : o0 + i, r = key % H;
    const long pix0 = (long)key * W;
    if constexpr (BBM) issue_by(key);  // the buffer's last reader was iteration i - 1
    // the slot of row i - 1 (last read at iteration i - 1) takes row i + R - 1
    issue(i + R - 1);
    if constexpr (VG) issue_y(i + R - 1, yslot);  // this wave's last reads of it: lgkmcnt(0) above
    if constexpr (PRE) transform(i + 3);
    // loaded i / i + 2 hold the rows above / below the output row (swapped bottom-up)
    const int above = rev ? (i + 2) % R : i % R, below = rev ? i % R : (i + 2) % R;
    const char* rowp[3] = {ring + (r > 0 ? above : ZS) * kR3SlotB, ring + ((i + 1) % R) * kR3SlotB,
                           ring + (r < H - 1 ? below : ZS) * kR3SlotB};
    // the row's TPR x 18 B fragments as one unrolled stream, two MFMAs (channel tiles) each; the
    // fragment of step s + P is read while step s multiplies. Reads, their address adds and the
    // waits are asm: hipcc otherwise sinks every read to its MFMA (one exposed LDS latency per
    // MFMA) and keeps all per-row addresses live
    constexpr int NS = TPR * 18, P = VG ? HGK_ROW3_PF - 3 : BBM ? HGK_ROW3_PF - 2 : HGK_ROW3_PF;
    static_assert(P >= 2 && P <= 16, "lgkmcnt range");
    uint32_t rb[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
      rb[kh] = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)rowp[kh]);
    auto rd = [&](int s) __attribute__((always_inline)) {
      const int t = s / 18, q = s % 18, kh = q / 6, kw = (q / 2) % 3, kq = q % 2;
      const uint32_t base = rb[kh] + t * 4096;  // scalar
      uint32_t addr;
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(addr) : "s"(base), "v"(loff[kw][kq]));
      bf16x8 v;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
      return v;
    };
    bf16x8 bq[P];
#pragma unroll
    for (int s = 0; s < P; ++s) bq[s] = rd(s);
    f32x4 acc[TPR][2];
#pragma clang loop unroll(full)
    for (int s = 0; s < NS; ++s) {
      const int t = s / 18, q = s % 18, kh = q / 6, kw = (q / 2) % 3, kq = q % 2;
      if (q == 0) {
        acc[t][0] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      // reads younger than step s's: P - 1 (fewer at the tail: wait for all)
      if (s + P <= NS)
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(bq[s % P]) : "n"(P - 1));
      else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(bq[s % P]));
#ifdef HGK_ABL_R3_NOMFMA  // ablation: no MFMAs (wrong results; timing only)
      asm volatile("" ::"v"(bq[s % P]), "v"(wreg[kh * 3 + kw][kq][0]), "v"(wreg[kh * 3 + kw][kq][1]));
#else
      acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[kh * 3 + kw][kq][0], bq[s % P], acc[t][0], 0, 0, 0);
      acc[t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[kh * 3 + kw][kq][1], bq[s % P], acc[t][1], 0, 0, 0);
#endif
#ifndef HGK_ABL_R3_NOREAD  // ablation: B fragments read once per row (wrong results; timing only)
      if (s + P < NS) bq[s % P] = rd(s + P);
#endif
    }
    R3_STAMP(3)
    // exchange: the partner (h ^ 1) gets this wave's sums for ITS channel tile; lane-linear
    // 16-B slots [wave][tile][lane]
#pragma unroll
    for (int t = 0; t < TPR; ++t)
      *reinterpret_cast<f32x4*>(xch + ((wave * TPR + t) * 64 + lane) * 16) = h ? acc[t][0] : acc[t][1];
    if constexpr (BBM) {
      // ... and the BN input row of every wave landed (only this iteration's input DMA and, VG,
      // the BN input row of the row in flight are younger)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(VG ? 2 * D : D) : "memory");
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    R3_STAMP(4)
    uint2 keep[TPR];
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < TPR; ++t) {
      // h = 0 part + h = 1 part, in that order for both owners
      const f32x4 oth = *reinterpret_cast<const f32x4*>(xch + (((wave ^ 4) * TPR + t) * 64 + lane) * 16);
      const f32x4 sum = h ? oth + acc[t][1] : acc[t][0] + oth;
      // epilogue: lane = channels co + 4 lg .. +3 of pixel t * 16 + lr
      float f[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) f[e] = sum[e] + bias4[e];
      const bf16x2_t h0 = {(__bf16)f[0], (__bf16)f[1]}, h1 = {(__bf16)f[2], (__bf16)f[3]};
      const uint2 pk = make_uint2(__builtin_bit_cast(uint32_t, h0), __builtin_bit_cast(uint32_t, h1));
      *reinterpret_cast<uint2*>(sg.y + (pix0 + t * 16 + lr) * kR3C + co + 4 * lg) = pk;
      keep[t] = pk;
      if constexpr (BBM) {
        // BN-backward partial sums over the STORED dA: g = dA [relu mask of the BN output]
        const int pos = t * 16 + lr + 1, c = (co + 4 * lg) >> 3;
        const uint2 yb = *reinterpret_cast<const uint2*>(
            bybuf + pos * 256 + ((c ^ (pos & 15)) << 4) + (((co + 4 * lg) >> 2) & 1) * 8);
        const float dv[4] = {__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u),
                             __uint_as_float(pk.y << 16), __uint_as_float(pk.y & 0xffff0000u)};
        const float yv[4] = {__uint_as_float(yb.x << 16), __uint_as_float(yb.x & 0xffff0000u),
                             __uint_as_float(yb.y << 16), __uint_as_float(yb.y & 0xffff0000u)};
        const float4 bsc = *reinterpret_cast<const float4*>(sBb + co + 4 * lg);
        const float4 bsh = *reinterpret_cast<const float4*>(sBb + kR3C + co + 4 * lg);
        const float4 bis = *reinterpret_cast<const float4*>(sBb + 2 * kR3C + co + 4 * lg);
        const float4 bmis = *reinterpret_cast<const float4*>(sBb + 3 * kR3C + co + 4 * lg);
        const float sc4[4] = {bsc.x, bsc.y, bsc.z, bsc.w}, sh4[4] = {bsh.x, bsh.y, bsh.z, bsh.w};
        const float is4[4] = {bis.x, bis.y, bis.z, bis.w}, mi4[4] = {bmis.x, bmis.y, bmis.z, bmis.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gv = (ra.bb_relu && !(fmaf(yv[e], sc4[e], sh4[e]) > 0.f)) ? 0.f : dv[e];
          s1[e] += gv;
          s2[e] = fmaf(gv, fmaf(yv[e], is4[e], mi4[e]), s2[e]);
        }
      }
    }
    // one partial row per output row; ONE store instruction per wave (lanes pick their value)
    if constexpr (STATS) {
      float v[TPR][4];
#pragma unroll
      for (int t = 0; t < TPR; ++t) {
        v[t][0] = __uint_as_float(keep[t].x << 16); v[t][1] = __uint_as_float(keep[t].x & 0xffff0000u);
        v[t][2] = __uint_as_float(keep[t].y << 16); v[t][3] = __uint_as_float(keep[t].y & 0xffff0000u);
      }
      float o1[4], o2[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < TPR; ++t) sum += v[t][e];
        o1[e] = sum;
      }
      row_allreduce<4>(o1);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float mu = o1[e] * (1.f / W);
        float d2 = 0.f;
#pragma unroll
        for (int t = 0; t < TPR; ++t) {
          const float d = v[t][e] - mu;
          d2 = fmaf(d, d, d2);
        }
        o2[e] = d2;
      }
      row_allreduce<4>(o2);
      // lane lr < 12: channel co + 4 lg + lr / 3, value lr % 3 (sum | M2 | count)
      const int e = lr / 3, k = lr - 3 * e;
      const float a1 = e == 0 ? o1[0] : e == 1 ? o1[1] : e == 2 ? o1[2] : o1[3];
      const float a2 = e == 0 ? o2[0] : e == 1 ? o2[1] : e == 2 ? o2[2] : o2[3];
      const float val = k == 0 ? a1 : k == 1 ? a2 : (float)W;
      if (lr < 12) sg.stats[((long)(co + 4 * lg + e) * 3 + k) * rows + key] = val;
    }
    if constexpr (BBM) {
      row_allreduce<4>(s1);
      row_allreduce<4>(s2);
      // lane lr < 8: channel co + 4 lg + (lr & 3), value lr >> 2 (sum g | sum g xhat)
      const int e = lr & 3, part = (lr >> 2) & 1;
      const float a1 = e == 0 ? s1[0] : e == 1 ? s1[1] : e == 2 ? s1[2] : s1[3];
      const float a2 = e == 0 ? s2[0] : e == 1 ? s2[1] : e == 2 ? s2[2] : s2[3];
      if (lr < 8) sg.bpart[((long)key * 2 + part) * kR3C + co + 4 * lg + e] = part ? a2 : a1;
    }
    if constexpr (VG) {
      // row i + 3 and its BN input landed for this wave (younger: this iteration's stores)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ST) : "memory");
      transform_vg(i + 3, yslot);
    }
    R3_STAMP(5)
  }
  // the tail's clamped DMAs: drained before the workgroup retires
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int MODE, int W0, int W1>
__global__ __launch_bounds__(512) void conv3x3_row_kernel(Row3Args ra) {
  __shared__ __attribute__((aligned(16))) char smem[kR3Lds];
  __shared__ __attribute__((aligned(16))) float sPre[2 * kR3C];
  __shared__ __attribute__((aligned(16))) float sBb[(MODE & 4) ? 4 * kR3C : 4];
  __shared__ __attribute__((aligned(16))) float sVg[(MODE & 16) ? 6 * kR3C : 4];
  // XCD-contiguous order: the workgroups of one XCD take neighbouring row runs (shared boundary
  // rows hit that XCD's L2)
  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int vid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  if (vid < ra.g0)
    row3_body<MODE, W0>(ra, ra.s[0], vid, ra.g0, smem, sPre, sBb, sVg);
  else
    row3_body<MODE, W1>(ra, ra.s[1], vid - ra.g0, ra.g1, smem, sPre, sBb, sVg);
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static int row3_mode(const ConvFwdArgs& a) {
  return (a.pre_scale ? 1 : 0) | (a.bb_partial ? 4 : 0) | (a.stats ? 8 : 0) | (a.vg_y ? 16 : 0);
}

static bool row3_shape_ok(const ConvFwdArgs& a) {
  const int mode = row3_mode(a);
  return a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.dil == 1 && a.Cin == kR3C &&
         a.Cout == kR3C && (a.W == 64 || a.W == 32) && a.H == a.Ho && a.W == a.Wo && a.H >= 2 &&
         !a.res && !a.post_relu && !a.fold_part && a.w_ld % 8 == 0 && a.w_ld >= 9 * kR3C &&
#ifdef HGK_ABL_R3_NOVG  // ablation build: no folded apply on this route
         mode != 20 &&
#endif
         (mode == 0 || mode == 1 || mode == 4 || mode == 8 || mode == 9 || mode == 20) &&
         (long)a.N * a.H <= kMaxStatsRows;
}

// route HGK_ROUTE_ROW3: 0 disables the route (A/B and tests), 1 every supported launch, 2
// (default) launches whose (first) segment is 64 wide: at 32x32 alone the halo kernel is faster;
// 3 single 64-wide only
static int row3_policy() { return (int)route(HGK_ROUTE_ROW3); }

bool row3_ok(const ConvFwdArgs& a, const ConvFwdArgs* a1) {
  const int pol = row3_policy();
  if (pol == 0 || !row3_shape_ok(a) || (pol >= 2 && a.W != 64)) return false;
  if (a.vg_part || (a1 && a1->vg_part)) return false;  // no folded BN-backward finalize
  if (!a1) return true;
  if (pol == 3) return false;  // 3: 64-wide single launches only (twins on the halo kernel)
  return row3_shape_ok(*a1) && row3_mode(*a1) == row3_mode(a) && a1->pre_relu == a.pre_relu &&
         a1->bb_relu == a.bb_relu && a1->vg_relu == a.vg_relu;
}

static int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <int MODE, int W0, int W1>
static void row3_launch_t(hipStream_t st, const Row3Args& ra) {
  hipLaunchKernelGGL((conv3x3_row_kernel<MODE, W0, W1>), dim3(ra.g0 + ra.g1), dim3(512), 0, st, ra);
}

template <int W0, int W1>
static bool row3_dispatch(hipStream_t st, const Row3Args& ra, int mode) {
  switch (mode) {
    case 0: row3_launch_t<0, W0, W1>(st, ra); return true;
    case 1: row3_launch_t<1, W0, W1>(st, ra); return true;
    case 4: row3_launch_t<4, W0, W1>(st, ra); return true;
    case 8: row3_launch_t<8, W0, W1>(st, ra); return true;
    case 9: row3_launch_t<9, W0, W1>(st, ra); return true;
    case 20: row3_launch_t<20, W0, W1>(st, ra); return true;
    default: return false;
  }
}

int launch_row3(hipStream_t st, ConvFwdArgs& a0, ConvFwdArgs* a1, int* rows0, int* rows1) {
  if (!row3_ok(a0, a1)) {
    set_error("conv_fwd row3: unsupported shape");
    return HGK_ERR_UNSUPPORTED;
  }
  const int mode = row3_mode(a0);
  Row3Args ra;
  memset(&ra, 0, sizeof(ra));
  long px[2] = {0, 0};
  for (int s = 0; s < 2; ++s) {
    const ConvFwdArgs* a = s == 0 ? &a0 : a1;
    if (!a) break;
    Row3Seg& g = ra.s[s];
    g.x = reinterpret_cast<const bf16_t*>(a->x);
    g.y = reinterpret_cast<bf16_t*>(a->y);
    g.pre_scale = a->pre_scale;
    g.pre_shift = a->pre_shift;
    g.stats = a->stats;
    g.bby = reinterpret_cast<const bf16_t*>(a->bb_y);
    g.bsc = a->bb_scale; g.bsh = a->bb_shift; g.bmu = a->bb_mean; g.bis = a->bb_invstd;
    g.bpart = a->bb_partial;
    g.vgy = reinterpret_cast<const bf16_t*>(a->vg_y);
    g.vsc = a->vg_scale; g.vsh = a->vg_shift; g.vco = a->vg_coef;
    g.vout = reinterpret_cast<bf16_t*>(a->vg_out);
    g.N = a->N; g.H = a->H; g.W = a->W;
    px[s] = a->M;
  }
  ra.w = reinterpret_cast<const bf16_t*>(a0.w);
  ra.bias = a0.bias;
  ra.w_ld = a0.w_ld;
  ra.pre_relu = a0.pre_relu;
  ra.bb_relu = a0.bb_relu;
  ra.vg_relu = a0.vg_relu;
  ra.alt_order = route(HGK_ROUTE_ROW3_ALT) != 0;
  // one workgroup per CU; a twin splits them in proportion to the segments' pixels
  const int ncu = cu_count();
  const int rows_a = a0.N * a0.H;
  if (!a1) {
    ra.g0 = std::min(ncu, rows_a);
    ra.g1 = 0;
    ra.s[1] = ra.s[0];
  } else {
    const int rows_b = a1->N * a1->H;
    int g0 = (int)((double)ncu * px[0] / (double)(px[0] + px[1]) + 0.5);
    g0 = std::max(1, std::min(g0, ncu - 1));
    ra.g0 = std::min(g0, rows_a);
    ra.g1 = std::min(ncu - g0, rows_b);
  }
  bool ok;
  const int wa = a0.W, wb = a1 ? a1->W : a0.W;
  if (wa == 64 && wb == 64) ok = row3_dispatch<64, 64>(st, ra, mode);
  else if (wa == 32 && wb == 32) ok = row3_dispatch<32, 32>(st, ra, mode);
  else if (wa == 64 && wb == 32) ok = row3_dispatch<64, 32>(st, ra, mode);
  else ok = false;
  if (!ok) {
    set_error("conv_fwd row3: no kernel for widths %d / %d, mode %d", wa, wb, mode);
    return HGK_ERR_UNSUPPORTED;
  }
  HGK_LAUNCH_CHECK();
  a0.stats_R = rows_a;
  if (a1) a1->stats_R = a1->N * a1->H;
  const bool part = (mode & 12) != 0;
  if (rows0) *rows0 = part ? rows_a : 0;
  if (rows1) *rows1 = part && a1 ? a1->N * a1->H : 0;
  return HGK_OK;
}

}  // namespace hgk

#ifdef HGK_R3_TRACE
extern "C" int hgk_debug_row3_trace(void* dst) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(hgk::g_r3trace), sizeof(hgk::g_r3trace)) == hipSuccess ? 0 : 1;
}
#endif
