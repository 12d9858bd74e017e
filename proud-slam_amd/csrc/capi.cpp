// psvo C-ABI plumbing: thread-local error state and launch checking.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "psvo_common.h"
#include "lookback.h"

namespace psvo {

static thread_local char g_err[512] = "";
thread_local hipEvent_t g_stop_event = nullptr;
thread_local bool g_stop_share = false;
thread_local hipEvent_t g_stop_bound = nullptr;

int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(PSVO_E_LAUNCH, "%s: %s", what, hipGetErrorString(e));
    return PSVO_OK;
}

// tests only: look-back controls for the sites in `mask` (lookback.h)
static int g_lb_debug_mask = 0, g_lb_debug_bound = -1, g_lb_debug_delay = 0;
LbCtl lb_ctl(int site) {
    const bool on = (g_lb_debug_mask & site) != 0;
    return LbCtl{on && g_lb_debug_bound >= 0 ? g_lb_debug_bound : kLbSpinMax, on ? g_lb_debug_delay : 0};
}

}  // namespace psvo

extern "C" int psvo_debug_set_lookback(int mask, int spin_bound, int delay_us) {
    PSVO_REQUIRE(mask >= 0 && mask <= 7 && spin_bound >= -1 && delay_us >= 0 && delay_us <= 100000,
                 "debug_set_lookback: bad arguments");
    psvo::g_lb_debug_mask = mask;
    psvo::g_lb_debug_bound = spin_bound;
    psvo::g_lb_debug_delay = delay_us;
    return PSVO_OK;
}

extern "C" int psvo_debug_lb_helps(int64_t *out3, int reset) {
    PSVO_REQUIRE(out3, "debug_lb_helps: null argument");
    const int rc = psvo::lb_helps_query(out3, reset != 0);
    if (rc != PSVO_OK) return rc;
    return psvo::lb_helps_select(out3 + 2, reset != 0);
}

extern "C" const char *psvo_last_error(void) { return psvo::g_err; }

extern "C" const char *psvo_version(void) { return "psvo 0.1.0 (gfx950)"; }
