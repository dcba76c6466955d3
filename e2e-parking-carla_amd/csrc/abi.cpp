// C-ABI bookkeeping shared by every kernel file: version + thread-local error message.
#include <stdarg.h>
#include <stdio.h>

#include "e2ep.h"

namespace e2ep {
static thread_local char g_err[512] = "";
void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace e2ep

extern "C" {
int e2ep_abi_version(void) { return 1; }
const char *e2ep_last_error(void) { return e2ep::g_err; }
}
