/* Test-only entry points of the MI355X FFA engine.  They exist only in the
 * test build of the library (riptide_amd/libriptide_amd_testhooks.so, the
 * same kernels and host code compiled with -DRT_TEST_HOOKS); the product
 * library libriptide_amd.so does not export them. */
#pragma once
#include "riptide_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* No reference counterpart: while `on` is non-zero, every plan uploaded to a
 * device carries one unit that breaks the cone kernel's budget, so the kernel
 * refuses it and raises the plan's error flag -- exercises rt_plan_check and
 * the host-buffer API's error path
 * (tests/test_gpu_e2e.py::test_plan_device_error_flag). */
int rt_test_corrupt_next_plans(int on);

#ifdef __cplusplus
}
#endif
