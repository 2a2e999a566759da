// C-ABI plumbing: version, thread-local error message, launch checks.
#include <string.h>

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

// ------------------------------------------------------------ live kernel timer
constexpr int kTimerSlots = 256;
struct KTimer {
  hipEvent_t ev[2] = {nullptr, nullptr};
  const char* kernel = "";
  int device = -1;
};
static KTimer g_timers[kTimerSlots];
static thread_local int g_armed = -1;

void ktimer_mark(int which, const char* kernel, hipStream_t st) {
  if (g_armed < 0) return;
  KTimer& t = g_timers[g_armed];
  if (which == 0) t.kernel = kernel;
  (void)hipEventRecord(t.ev[which], st);
  if (which == 1) g_armed = -1;
}

}  // namespace pr

extern "C" int pr_ktimer_arm(int32_t slot) {
  using namespace pr;
  if (slot == -1) {  // disarm
    g_armed = -1;
    return PR_OK;
  }
  if (slot < 0 || slot >= kTimerSlots) return set_error(PR_ERR_ARG, "ktimer: slot out of range");
  KTimer& t = g_timers[slot];
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (t.device != dev) {
    for (auto& e : t.ev) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
      if (hipEventCreate(&e) != hipSuccess) return set_error(PR_ERR_HIP, "ktimer: hipEventCreate failed");
    }
    t.device = dev;
  }
  t.kernel = "";
  g_armed = slot;
  return PR_OK;
}

extern "C" int pr_ktimer_read(int32_t slot, float* ms, char* name, int32_t name_cap) {
  using namespace pr;
  if (slot < 0 || slot >= kTimerSlots || !g_timers[slot].ev[0]) return set_error(PR_ERR_ARG, "ktimer: slot not armed");
  KTimer& t = g_timers[slot];
  if (!t.kernel[0]) return set_error(PR_ERR_ARG, "ktimer: no kernel was timed in this slot");
  const hipError_t e = hipEventElapsedTime(ms, t.ev[0], t.ev[1]);
  if (e != hipSuccess) return set_error(PR_ERR_HIP, std::string("ktimer: ") + hipGetErrorString(e));
  if (name && name_cap > 0) {
    strncpy(name, t.kernel, name_cap - 1);
    name[name_cap - 1] = 0;
  }
  return PR_OK;
}

extern "C" int pr_abi_version(void) { return PR_ABI_VERSION; }

extern "C" const char* pr_last_error(void) { return pr::g_last_error.c_str(); }
