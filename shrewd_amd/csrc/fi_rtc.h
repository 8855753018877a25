// fi_rtc.h -- the few declarations the kernel sources need from the C/HIP
// headers, in a form that compiles both under hipcc (static library) and
// under hipRTC (the load-time build with translated golden blocks).
#pragma once
#ifdef __HIPCC_RTC__
using namespace __hip_internal;
typedef unsigned long uintptr_t;
#ifndef INT64_MIN
#define INT64_MIN (-9223372036854775807LL - 1)
#endif
#ifndef INT32_MIN
#define INT32_MIN (-2147483647 - 1)
#endif
#else
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif
