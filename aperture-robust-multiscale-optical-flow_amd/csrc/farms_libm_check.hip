// farms_libm_check.hip — host build of csrc/farms_libm.h for tests/test_libm.py:
// evaluates the correctly rounded atan2 / sin / cos next to the host glibc
// (looked up in libm.so.6 at run time, so no compiler builtin stands in) and
// counts the arguments where the two differ.  Test infrastructure only.
#include <dlfcn.h>

#include <cstdint>

static int64_t g_fallbacks = 0;
#define FARMS_LIBM_FALLBACK() (++g_fallbacks)
#include "farms_libm.h"

extern "C" {

// host builds of the three functions (tests swap them into the oracle,
// oracle/farms_oracle.h farms_oracle_set_libm)
double farms_cr_atan2(double y, double x) { return farms_libm::cr_atan2(y, x); }
double farms_cr_sin(double x) { return farms_libm::cr_sin(x); }
double farms_cr_cos(double x) { return farms_libm::cr_cos(x); }

// fn 0: atan2(a, b); 1: sin(a); 2: cos(a), each by the fast path (with its
// fallback) and by the full double-double evaluation alone.  Returns the number
// of bitwise differences between the two; *fallbacks = the calls whose fast
// path could not decide the rounding.
int64_t farms_libm_fast_check(int fn, const double *a, const double *b, int64_t n, int64_t *fallbacks) {
    g_fallbacks = 0;
    int64_t diff = 0;
    for (int64_t i = 0; i < n; ++i) {
        double f, s;
        if (fn == 0) { f = farms_libm::cr_atan2(a[i], b[i]); s = farms_libm::atan2_dd(a[i], b[i]); }
        else if (fn == 1) { f = farms_libm::cr_sin(a[i]); s = farms_libm::sin_dd(a[i]); }
        else { f = farms_libm::cr_cos(a[i]); s = farms_libm::cos_dd(a[i]); }
        uint64_t uf, us;
        __builtin_memcpy(&uf, &f, 8);
        __builtin_memcpy(&us, &s, 8);
        diff += uf != us && !(f != f && s != s);
    }
    *fallbacks = g_fallbacks;
    return diff;
}

// fn 0: atan2(a, b); 1: sin(a); 2: cos(a).  out_cr / out_glibc may be NULL.
// Returns the number of i with bitwise-different results, -1 if libm is missing.
int64_t farms_libm_check(int fn, const double *a, const double *b, int64_t n, double *out_cr, double *out_glibc) {
    void *lm = dlopen("libm.so.6", RTLD_NOW | RTLD_LOCAL);
    if (!lm) return -1;
    double (*g1)(double) = nullptr;
    double (*g2)(double, double) = nullptr;
    if (fn == 0) g2 = (double (*)(double, double))dlsym(lm, "atan2");
    else g1 = (double (*)(double))dlsym(lm, fn == 1 ? "sin" : "cos");
    if (!g1 && !g2) return -1;
    int64_t diff = 0;
    for (int64_t i = 0; i < n; ++i) {
        double c, g;
        if (fn == 0) { c = farms_libm::cr_atan2(a[i], b[i]); g = g2(a[i], b[i]); }
        else if (fn == 1) { c = farms_libm::cr_sin(a[i]); g = g1(a[i]); }
        else { c = farms_libm::cr_cos(a[i]); g = g1(a[i]); }
        if (out_cr) out_cr[i] = c;
        if (out_glibc) out_glibc[i] = g;
        uint64_t uc, ug;
        __builtin_memcpy(&uc, &c, 8);
        __builtin_memcpy(&ug, &g, 8);
        diff += uc != ug && !(c != c && g != g);
    }
    return diff;
}
}
