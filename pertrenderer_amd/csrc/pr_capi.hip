// C-ABI plumbing: version, thread-local error message, launch checks.
#include "pr_common.h"

namespace pr {

static thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(PR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  return PR_OK;
}

}  // namespace pr

extern "C" int pr_abi_version(void) { return PR_ABI_VERSION; }

extern "C" const char* pr_last_error(void) { return pr::g_last_error.c_str(); }
