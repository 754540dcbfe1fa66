// errors.cpp — error state and version of libpamg (host only, so the host setup routines
// build and run without the HIP runtime, e.g. under the sanitizers of tests/test_sanitizers.py).
#include "pamg_common.h"

std::string& pamg::last_error() {
    static thread_local std::string msg;
    return msg;
}

extern "C" {
const char* pamg_version(void) { return "pamg 0.1 (gfx950)"; }
const char* pamg_last_error(void) { return pamg::last_error().c_str(); }
}
