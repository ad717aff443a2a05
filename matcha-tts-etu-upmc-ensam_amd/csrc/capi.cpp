// Library identity and the thread-local error slot behind mtts_last_error().
#include <cstdarg>
#include <cstdio>

#include "mtts_common.h"

namespace {
thread_local char g_last_error[512] = "";
}

namespace mtts {
void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}
}  // namespace mtts

extern "C" int mtts_abi_version(void) { return MTTS_ABI_VERSION; }

extern "C" const char *mtts_last_error(void) { return g_last_error; }
