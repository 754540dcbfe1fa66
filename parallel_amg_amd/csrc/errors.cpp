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

// Debug aid (PAMG_SEGV_TRACE=1 in the environment): on SIGSEGV print the native call stack of
// the faulting thread to stderr before the default action (Python's faulthandler shows only
// the Python frames of a crash inside this library or a library it calls).
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>

namespace {
void segv_trace(int sig) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char head[] = "[pamg] SIGSEGV native stack:\n";
    (void)!write(2, head, sizeof(head) - 1);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
struct SegvTraceInstaller {
    SegvTraceInstaller() {
        const char* e = std::getenv("PAMG_SEGV_TRACE");
        if (e && std::strcmp(e, "0") != 0) signal(SIGSEGV, segv_trace);
    }
} segv_trace_installer;
}  // namespace
