// last-error stub for standalone probe builds of single library sources
#include <cstdio>
extern "C" __attribute__((visibility("default"))) const char* sl_probe_last_error();
static char g_err[512];
void sl_set_last_error(const char* msg) { snprintf(g_err, sizeof g_err, "%s", msg); }
extern "C" const char* sl_probe_last_error() { return g_err; }
// the library's once-per-kernel LDS attribute setter (dev_util.cpp), simplified
#include <hip/hip_runtime.h>
int sl_lds_attr(const void* fn, int bytes) {
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess ? 0 : -1;
}
