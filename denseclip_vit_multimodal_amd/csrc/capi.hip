// Error reporting and version of the C ABI (include/dclip.h).
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

static thread_local char g_err[1024] = "";

void dclip_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

extern "C" const char* dclip_last_error(void) { return g_err; }

extern "C" int dclip_abi_version(void) { return 1; }
