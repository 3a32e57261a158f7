// Lean fp64 transcendental building blocks shared by the LDPC BP check update
// (ldpc.hip) and the polar path metrics (polar_common.hpp).
#pragma once
#include "common.hpp"

namespace pl {

// ---- lean fp64 transcendentals -----------------------------------------------
// The reference evaluates np.tanh / np.arctanh (NumPy's SIMD kernels); ocml's
// versions cost ~160 VALU each (double-double internals) and made this kernel
// VALU-bound.  These are <= ~2 ulp (NumPy's own differ from libm by 1-2 ulp in
// ~20 % of inputs), and decisions are checked bit-exact against the
// reference fixtures (tests/test_gpu_ldpc.py).  PL_LDPC_MATH=ocml restores ocml.
//
// log1p for x >= 0: the classic reduction 1+x = 2^k (1+f), sqrt(2)/2 <= 1+f <
// sqrt(2), with the rounding of 1+x carried as a correction c, and log(1+f) =
// 2s + s R(s^2), s = f/(2+f), R the published minimax fit (Lg1..Lg7, the
// coefficients of the Sun fdlibm log kernel).
// x / y to <= 1 ulp: hardware reciprocal, two Newton steps, one residual step
// (8 VALU against 13 for the IEEE-exact sequence); y finite, nonzero, normal.
PL_DEV double div_fast(double x, double y) {
    double r = __builtin_amdgcn_rcp(y);
    double e = fma(-y, r, 1.0);
    r = fma(r, e, r);
    e = fma(-y, r, 1.0);
    r = fma(r, e, r);
    const double q = x * r;
    return fma(fma(-y, q, x), r, q);
}
PL_DEV double lg_R(double z) {
    const double w = z * z;
    const double t1 = w * fma(w, fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01), 3.999999999940941908e-01);
    const double t2 = z * fma(w, fma(w, fma(w, 1.479819860511658591e-01, 1.818357216161805012e-01),
                                     2.857142874366239149e-01), 6.666666666666735130e-01);
    return t2 + t1;
}
PL_DEV double log1p_pos(double x) {
    constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    double f, c = 0.0;
    int k = 0;
    if (x < 0.41421356237309503) {
        f = x;
    } else {
        const double u = 1.0 + x;
        k = __builtin_amdgcn_frexp_exp(u) - 1;  // u = 2^k * m, m in [1, 2)
        c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
        c *= __builtin_amdgcn_rcp(u);  // rounding correction, a few bits suffice
        double m = __builtin_amdgcn_ldexp(u, -k);
        if (m >= 1.4142135623730951) { m *= 0.5; k += 1; }
        f = m - 1.0;
    }
    const double hfsq = 0.5 * f * f;
    const double s = div_fast(f, 2.0 + f);
    const double R = lg_R(s * s);
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    const double dk = (double)k;
    return dk * LN2_HI - ((hfsq - (s * (hfsq + R) + (dk * LN2_LO + c))) - f);
}

}  // namespace pl
