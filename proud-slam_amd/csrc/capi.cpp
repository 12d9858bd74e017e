// psvo C-ABI plumbing: thread-local error state and launch checking.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "psvo_common.h"

namespace psvo {

static thread_local char g_err[512] = "";

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

}  // namespace psvo

extern "C" const char *psvo_last_error(void) { return psvo::g_err; }

extern "C" const char *psvo_version(void) { return "psvo 0.1.0 (gfx950)"; }
