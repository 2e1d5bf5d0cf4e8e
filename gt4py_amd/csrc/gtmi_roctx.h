// gtmi_roctx.h -- optional ROCTX ranges around every stencil call and halo copy
// (rocprofv3 --marker-trace shows them by stencil name).
//
// Compiled in only when the build found rocprofiler-sdk-roctx (runtime/jit.py passes
// -DGTMI_ROCTX=1 and the link flags then) and the header is present; GTMI_ROCTX=0 in the
// environment turns the ranges off at run time (read once per library).
#pragma once
#if defined(GTMI_ROCTX) && GTMI_ROCTX && __has_include(<rocprofiler-sdk-roctx/roctx.h>)
#include <rocprofiler-sdk-roctx/roctx.h>
#include <stdlib.h>
static inline bool gtmi_roctx_on() {
    static const bool on = [] {
        const char* e = getenv("GTMI_ROCTX");
        return !(e && e[0] == '0');
    }();
    return on;
}
#define GTMI_RANGE_PUSH(name)                   \
    do {                                        \
        if (gtmi_roctx_on()) roctxRangePushA(name); \
    } while (0)
#define GTMI_RANGE_POP()                      \
    do {                                      \
        if (gtmi_roctx_on()) roctxRangePop(); \
    } while (0)
#else
#define GTMI_RANGE_PUSH(name) \
    do {                      \
        (void)(name);         \
    } while (0)
#define GTMI_RANGE_POP() \
    do {                 \
    } while (0)
#endif
