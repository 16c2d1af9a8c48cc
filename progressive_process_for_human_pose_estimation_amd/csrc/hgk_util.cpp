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
}  // namespace hgk

extern "C" {
int hgk_abi_version(void) { return HGK_ABI_VERSION; }
const char* hgk_last_error(void) { return hgk::g_err; }
}
