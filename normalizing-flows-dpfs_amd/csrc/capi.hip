// capi.hip -- error plumbing and version of the C ABI (include/nfdpf.h).
#include <cstdarg>
#include <cstdio>

#include "common.hpp"

namespace nfdpf {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int launch_status(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return NFDPF_ELAUNCH;
  }
  return NFDPF_OK;
}

}  // namespace nfdpf

extern "C" int nfdpf_version(void) { return 1; }
extern "C" int64_t nfdpf_filter_desc_size(void) { return (int64_t)sizeof(nfdpf_filter_desc); }
extern "C" const char *nfdpf_last_error(void) { return nfdpf::g_err; }
