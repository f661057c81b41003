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

extern "C" int dclip_abi_version(void) { return 7; }

// Tuning options (variant selection for A/B benchmarking in one process); 0 = default.
static int g_opts[DCLIP_OPT_COUNT] = {0};

int dclip_option(int id) { return (id >= 0 && id < DCLIP_OPT_COUNT) ? g_opts[id] : 0; }

extern "C" int dclip_set_option(int id, int value) {
    DCLIP_HOST_CHECK(id >= 0 && id < DCLIP_OPT_COUNT, "dclip_set_option: unknown option %d", id);
    g_opts[id] = value;
    return 0;
}
