// Host-side sanitizer check of libhgk (AddressSanitizer + UndefinedBehaviorSanitizer on the HOST
// code only; GPU sanitizers are not available on this pool). Built by scripts/asan_host.sh from
// the library sources compiled host-only, so every kernel launch fails cleanly (no code object /
// no device) AFTER the host-side work it depends on has run: argument validation, launch planning
// (split-K / tile / workspace plans), descriptor packing of the multi-entry calls and the grouping
// of the running-statistics records. Any out-of-bounds host access or UB aborts with a report.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hgk.h"

static int fails = 0;
#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++fails;                                                         \
    }                                                                  \
  } while (0)

int main() {
  // fake, never dereferenced "device" pointers: the launches fail before touching them
  std::vector<char> dummy(1 << 20);
  void* p = dummy.data();
  float* f = reinterpret_cast<float*>(dummy.data());
  double* d = reinterpret_cast<double*>(dummy.data());
  int rows = 0;

  EXPECT(hgk_abi_version() == HGK_ABI_VERSION);
  // argument validation
  EXPECT(hgk_conv_fwd(nullptr, HGK_BF16, nullptr, nullptr, 64, nullptr, nullptr, nullptr, nullptr,
                      nullptr, 0, 0, nullptr, nullptr, 1, 8, 8, 64, 64, 1, 1, 1, 0, 1, nullptr, 0) ==
         HGK_ERR_ARG);
  EXPECT(hgk_last_error() != nullptr);
  EXPECT(hgk_conv_fwd(nullptr, 7, p, p, 64, nullptr, nullptr, p, nullptr, nullptr, 0, 0, nullptr,
                      nullptr, 1, 8, 8, 64, 64, 1, 1, 1, 0, 1, nullptr, 0) < 0);
  EXPECT(hgk_bn_finalize_deferred(nullptr, nullptr, 2, 128, nullptr, nullptr, 1e-5f) == HGK_ERR_ARG);
  EXPECT(hgk_bn_bwd_twin(nullptr, HGK_BF16, nullptr, 3, 128, 1, 1, nullptr, nullptr, nullptr) ==
         HGK_ERR_ARG);
  EXPECT(hgk_add(nullptr, 7, p, nullptr, p, 4, 0) < 0);

  // planning queries over every hourglass level and both dtypes
  for (int dt = 0; dt < 2; ++dt)
    for (int hw = 4; hw <= 128; hw *= 2)
      for (int k = 1; k <= 3; k += 2) {
        size_t a = hgk_conv_fwd_workspace(dt, 32, hw, hw, 128, 128, k, k, 1, k / 2, 1);
        size_t b = hgk_conv_fwd_twin_workspace(dt, 32, hw, hw, 32, hw / 2, hw / 2, 128, 128, k, k, 1,
                                               k / 2, 1);
        EXPECT(b >= a);
        EXPECT(hgk_conv_wgrad_workspace(dt, 32, hw, hw, 128, 128, k, k, 1, k / 2, 1) > 0);
      }
  EXPECT(hgk_conv_wgrad_slab_bytes(256, 128, 1, 1, 256) == (size_t)256 * 128 * 256 * 4 + 256 * 128 * 4);

  // full host paths up to the (failing) launch
  hgk_conv_seg seg[2] = {};
  for (int s = 0; s < 2; ++s) {
    seg[s].x = p; seg[s].y = p; seg[s].stats = f; seg[s].rows_out = &rows;
    seg[s].pre_scale = f; seg[s].pre_shift = f;
    seg[s].N = 32; seg[s].H = 16 >> s; seg[s].W = 16 >> s;
  }
  int rc = hgk_conv_fwd_twin(nullptr, HGK_BF16, p, 1152, f, 1, 0, 128, 128, 3, 3, 1, 1, 1, seg, p,
                             1 << 20);
  EXPECT(rc == HGK_OK || rc == HGK_ERR_HIP);
  seg[1].stats = nullptr;  // statistics on one segment only: rejected
  EXPECT(hgk_conv_fwd_twin(nullptr, HGK_BF16, p, 1152, f, 1, 0, 128, 128, 3, 3, 1, 1, 1, seg, p,
                           1 << 20) == HGK_ERR_ARG);

  std::vector<hgk_bn_running> run(100);
  for (int i = 0; i < 100; ++i) run[i] = {f + (i % 7) * 512, f + 4096 + (i % 7) * 512, d, 256, 0.1f};
  rc = hgk_bn_running_update(nullptr, run.data(), (int)run.size());
  EXPECT(rc == HGK_OK || rc == HGK_ERR_HIP);

  std::vector<hgk_wgrad_fin> fin(70);
  for (int i = 0; i < 70; ++i) fin[i] = {p, 8, 1 + i % 8, f, (i & 1) ? f : nullptr, 64, 64, 1 + 2 * (i % 2),
                                        1 + 2 * (i % 2), 64, 17};
  rc = hgk_conv_wgrad_finish_multi(nullptr, fin.data(), (int)fin.size());
  EXPECT(rc == HGK_OK || rc == HGK_ERR_HIP);

  std::vector<hgk_pack_desc> pk(100);
  for (int i = 0; i < 100; ++i) pk[i] = {f, p, 1152, 128, 128, 3, 3, i & 1, 128, 128, 128};
  rc = hgk_pack_conv_weight_multi(nullptr, HGK_BF16, pk.data(), (int)pk.size());
  EXPECT(rc == HGK_OK || rc == HGK_ERR_HIP);

  hgk_bn_seg bs[2] = {{f, 64, 2048, d, f}, {f, 600, 512, d, f}};
  rc = hgk_bn_finalize_deferred(nullptr, bs, 2, 128, f, f, 1e-5f);
  EXPECT(rc == HGK_OK || rc == HGK_ERR_HIP);
  hgk_bnb_seg bb[2] = {{f, 128, 8192, f, p, p, nullptr, p, 0}, {f, 300, 2048, f, p, p, p, p, 1}};
  rc = hgk_bn_bwd_twin(nullptr, HGK_BF16, bb, 2, 128, 1, 1, f, f, f);
  EXPECT(rc == HGK_OK || rc == HGK_ERR_HIP);

  std::printf("asan host check: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}
