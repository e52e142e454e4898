// sgx_errors.cpp — the thread-local error message behind sgx_last_error() (host only).
// Error convention of the C ABI (include/sgx.h): negative codes map to the JVM exceptions /
// OperationStatus.FAILURE of the reference (ShuffleTransport.scala:49-51,71).
#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/sgx.h"
#include "sgx_host.h"

static thread_local std::string t_last_error;

int sgx::fail_msg(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_last_error = buf;
    return code;
}

extern "C" const char *sgx_last_error(void) { return t_last_error.c_str(); }
extern "C" int32_t sgx_abi_version(void) { return SGX_ABI_VERSION; }
