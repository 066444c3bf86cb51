// capi.hip -- error plumbing and version of the C ABI (include/nfdpf.h).
#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <set>
#include <utility>

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

void ensure_max_dynamic_lds(const void *fn, int bytes) {
  // per (kernel, current device): the attribute belongs to the device's module
  static std::mutex mu;
  static std::set<std::pair<const void *, int>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  std::lock_guard<std::mutex> lock(mu);
  if (done.insert({fn, dev}).second) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

}  // namespace nfdpf

extern "C" int nfdpf_version(void) { return 1; }
extern "C" int64_t nfdpf_filter_desc_size(void) { return (int64_t)sizeof(nfdpf_filter_desc); }
extern "C" const char *nfdpf_last_error(void) { return nfdpf::g_err; }
