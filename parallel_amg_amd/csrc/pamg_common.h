// pamg_common.h — shared host-side helpers of libpamg (error state, host CSR type).
#pragma once

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/pamg.h"

namespace pamg {

// Thread-local message of the last failure (pamg_last_error).
std::string& last_error();

inline int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    last_error() = buf;
    return code;
}

}  // namespace pamg

// Host CSR (SPEC §S1): int64 row pointers, int32 global column ids, fp64 values.
struct pamg_hcsr {
    int64_t nr = 0, nc = 0;
    std::vector<int64_t> rp;
    std::vector<int32_t> col;
    std::vector<double> val;
    int64_t nnz() const { return rp.empty() ? 0 : rp.back(); }
};
