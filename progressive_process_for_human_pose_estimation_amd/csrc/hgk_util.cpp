// Thread-local error string and version for the libhgk C-ABI.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/hgk.h"

namespace hgk {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// compiled routing defaults (include/hgk.h, HGK_ROUTE_*); changed only through hgk_set_route
static constexpr long kRouteDefault[HGK_ROUTE_COUNT] = {4, 16384, 1, 2, 1, 8192, 0, 0, 0, 0, 6, 5, 1, 0, 65536, 128};
static long g_route[HGK_ROUTE_COUNT] = {4, 16384, 1, 2, 1, 8192, 0, 0, 0, 0, 6, 5, 1, 0, 65536, 128};
long route(int knob) { return g_route[knob]; }
}  // namespace hgk

extern "C" {
int hgk_abi_version(void) { return HGK_ABI_VERSION; }
const char* hgk_last_error(void) { return hgk::g_err; }

long hgk_set_route(int knob, long value) {
  if (knob < 0 || knob >= HGK_ROUTE_COUNT) {
    hgk::set_error("set_route: unknown knob %d", knob);
    return HGK_ERR_ARG;
  }
  const long prev = hgk::g_route[knob];
  hgk::g_route[knob] = value < 0 ? hgk::kRouteDefault[knob] : value;
  return prev;
}

long hgk_get_route(int knob) {
  if (knob < 0 || knob >= HGK_ROUTE_COUNT) {
    hgk::set_error("get_route: unknown knob %d", knob);
    return HGK_ERR_ARG;
  }
  return hgk::g_route[knob];
}
}
