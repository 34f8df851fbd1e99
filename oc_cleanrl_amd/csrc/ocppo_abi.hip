// C-ABI housekeeping: ABI version and the thread-local error message behind ocppo_last_error().
#include "ocppo_common.h"

namespace ocppo {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

}  // namespace ocppo

extern "C" int ocppo_abi_version(void) { return OCPPO_ABI_VERSION; }
extern "C" const char* ocppo_last_error(void) { return ocppo::g_err; }
