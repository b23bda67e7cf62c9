// Developer and test overrides of libkwmatch, read through one gate (host code only).
//
//   KW_TEST_*  the tests' capacity / table overrides (tests/test_gpu_capacity.py and others): honoured only in
//              a process that sets KW_TEST_HOOKS=1;
//   KW_*       profiling and A/B knobs (KW_SERIAL, KW_TASK_G, KW_HT_SCALE, ...): honoured only
//              with KW_DEV=1.
//
// A production process sets neither, so nothing in its environment changes a scan.
#pragma once
#include <cstdlib>
#include <cstring>

static inline const char *kw_env(const char *name)
{
    const bool test = strncmp(name, "KW_TEST_", 8) == 0;
    const char *gate = getenv(test ? "KW_TEST_HOOKS" : "KW_DEV");
    if (!gate || strcmp(gate, "1") != 0) return nullptr;
    return getenv(name);
}
