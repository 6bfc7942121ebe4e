// pt_error.cpp — the thread-local last-error message of the C ABI (host only).
#include "pt_error.h"

#include "../../include/ptgpu.h"

namespace {
thread_local std::string g_err;
}  // namespace

int pt_fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

extern "C" const char* pt_last_error(void) { return g_err.c_str(); }
