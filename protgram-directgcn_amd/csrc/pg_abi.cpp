// Error channel and version of the C ABI (include/pg_directgcn.h).
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "pg_common.h"

namespace {
thread_local char g_err[512] = {0};
}

namespace pg {

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

void clear_error() { g_err[0] = 0; }

}  // namespace pg

extern "C" {

const char* pg_last_error(void) { return g_err; }

int pg_abi_version(void) { return PG_ABI_VERSION; }

}  // extern "C"
