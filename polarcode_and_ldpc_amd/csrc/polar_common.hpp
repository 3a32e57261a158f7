// Polar f / g / path-metric arithmetic shared by the lane-per-path kernels
// (polar_lane.hip, polar_tree.hip).  Each is the reference's fp64 operation:
//   f  src/polar/decoder.py:121-127 (SCDecoder._upper_llr) and :408-410
//   g  src/polar/decoder.py:129-144 (SCDecoder._lower_llr) and :412-417
//   metric increments src/polar/decoder.py:374-406 (SCLDecoder._log_likelihood)
#pragma once
#include "common.hpp"

namespace pl {

// min-sum f with the reference's value semantics: sign(a)*sign(b)*min(|a|,|b|);
// zeros give a zero, NaN in either input gives NaN.  Exact (no rounding).
PL_DEV double f_ms(double a, double b) {
    const double x = fabs(a), y = fabs(b);
    const double mn = (y < x) ? y : x;
    const uint64_t sb = ((uint64_t)__double_as_longlong(a) ^ (uint64_t)__double_as_longlong(b)) & 0x8000000000000000ull;
    const double r = __longlong_as_double((long long)((uint64_t)__double_as_longlong(mn) | sb));
    return __builtin_isunordered(a, b) ? __builtin_nan("") : r;
}
// g: btm + top if bit == 0 else btm - top (one rounding, as the reference)
PL_DEV double g_op(double top, double btm, uint32_t bit) {
    const uint64_t flip = (uint64_t)(bit & 1u) << 63;
    return btm + __longlong_as_double((long long)((uint64_t)__double_as_longlong(top) ^ flip));
}

// Path-metric increments.  t = log1p(exp(-|lam|)) is skipped when
// exp(-|lam|) < 2^(e-56), e = min(ilogb pm, ilogb |lam|), pm != 0: then t is
// below a quarter ulp of every quantity it is added to and the rounded metrics
// are exactly pm, pm + lam, pm - lam as in the reference.
template <bool WANT1>
PL_DEV void path_metrics(double pm, double lam, double& m0, double& m1) {
    const double x = fabs(lam);
    int e = ilogb(pm);
    const int ex = ilogb(x);
    e = e < ex ? e : ex;
    e = e < -1100 ? -1100 : (e > 1100 ? 1100 : e);  // ilogb(0) = INT_MIN: keep 56 - e finite
    const bool skip = (pm != 0.0) && (x > (double)(56 - e) * 0.6931471805599453);
    double t = 0.0;
    if (!skip) t = log1p(exp(-x));
    m0 = pm + ((lam >= 0.0) ? -t : lam - t);
    if (WANT1) m1 = pm + ((lam >= 0.0) ? -lam - t : -t);
}

}  // namespace pl
