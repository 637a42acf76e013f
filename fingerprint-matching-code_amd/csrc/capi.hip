// C-ABI plumbing: thread-local last-error string and launch checking.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "fpm_common.h"

namespace fpm {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return 2;
    }
    return 0;
}

}  // namespace fpm

extern "C" {

const char* fpm_last_error(void) { return fpm::g_err; }

int fpm_version(void) { return 100; }

int fpm_device_sync(void) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        fpm::set_error("hipDeviceSynchronize: %s", hipGetErrorString(e));
        return 2;
    }
    return 0;
}

}  // extern "C"
