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
// fma(a, b, c) as one VOP3 v_fma_f64 with all operands in VGPRs (VOP3 = true).
// For a Horner step whose addend c is a constant the compiler otherwise emits
// the two-address v_fmac_f64 plus a v_mov_b64 copy of the constant (2 VALU);
// worth it in the VALU-bound LDPC kernel, harmful in the register-bound polar
// tree kernel (the constants then occupy VGPRs), hence opt-in.
template <bool VOP3>
PL_DEV double fma_k(double a, double b, double c) {
    if constexpr (VOP3) {
        double d;
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
        return d;
    } else {
        return fma(a, b, c);
    }
}
// x / y to <= 1 ulp: hardware reciprocal, one Newton step, one residual step
// (6 VALU against 13 for the IEEE-exact sequence); y finite, nonzero, normal.
// v_rcp_f64 is good to ~2^-25 (2.5e8 ulp measured); one Newton step brings r
// to ~2^-50 and the residual step then rounds q as two steps would: the same
// two_atanh on 8.4 M inputs across its domain (tools/probes/atanh_probe.hip,
// profiles/r05/atanh_probe.json; without the Newton step 3 % differ).
PL_DEV double div_fast(double x, double y) {
    double r = __builtin_amdgcn_rcp(y);
    const double e = fma(-y, r, 1.0);
    r = fma(r, e, r);
    const double q = x * r;
    return fma(fma(-y, q, x), r, q);
}
// exp(-x) for x >= 0 (finite or +inf): x = k ln2 + r with |r| <= ln2/2
// (Cody-Waite two-constant reduction), e^-r by the degree-13 Taylor polynomial
// (truncation < 2^-57), scaled by 2^-k.  <= 1 ulp, ~19 VALU against ocml's 42.
PL_DEV double exp_neg(double x) {
    constexpr double INV_LN2 = 1.4426950408889634074, LN2_HI = 6.93147180369123816490e-01,
                     LN2_LO = 1.90821492927058770002e-10;
    const double xc = x < 746.0 ? x : 746.0;  // e^-746 underflows to 0 either way
    const double k = __builtin_rint(xc * INV_LN2);
    double r = fma(-k, LN2_HI, xc);
    r = -fma(-k, LN2_LO, r);  // r = k ln2 - x, |r| <= ln2/2
    double p = 1.6059043836821614599e-10;        // 1/13!
    p = fma(p, r, 2.0876756987868098979e-09);  // 1/12!
    p = fma(p, r, 2.5052108385441718775e-08);  // 1/11!
    p = fma(p, r, 2.7557319223985890653e-07);  // 1/10!
    p = fma(p, r, 2.7557319223985890653e-06);  // 1/9!
    p = fma(p, r, 2.4801587301587301566e-05);  // 1/8!
    p = fma(p, r, 1.9841269841269841253e-04);  // 1/7!
    p = fma(p, r, 1.3888888888888888889e-03);  // 1/6!
    p = fma(p, r, 8.3333333333333333333e-03);  // 1/5!
    p = fma(p, r, 4.1666666666666666667e-02);  // 1/4!
    p = fma(p, r, 1.6666666666666666667e-01);  // 1/3!
    p = fma(p, r, 0.5);                            // 1/2!
    p = fma(p, r, 1.0);                            // 1/1!
    const double e = fma(p, r, 1.0);             // e^r
    return __builtin_amdgcn_ldexp(e, -(int)k);
}

// expm1(x) for x <= 0: the exp_neg reduction, e^r - 1 = r + r^2 P(r) (degree-13
// Taylor), then 2^-k (1 + (e^r - 1)) - 1 for k > 0.  <= 2 ulp, ~22 VALU (ocml: 53).
PL_DEV double expm1_neg(double x) {
    constexpr double INV_LN2 = 1.4426950408889634074, LN2_HI = 6.93147180369123816490e-01,
                     LN2_LO = 1.90821492927058770002e-10;
    const double ax = -x < 746.0 ? -x : 746.0;
    const double k = __builtin_rint(ax * INV_LN2);
    double r = fma(-k, LN2_HI, ax);
    r = -fma(-k, LN2_LO, r);  // r = k ln2 - |x|
    double p = 1.6059043836821614599e-10;        // 1/13!
    p = fma(p, r, 2.0876756987868098979e-09);
    p = fma(p, r, 2.5052108385441718775e-08);
    p = fma(p, r, 2.7557319223985890653e-07);
    p = fma(p, r, 2.7557319223985890653e-06);
    p = fma(p, r, 2.4801587301587301566e-05);
    p = fma(p, r, 1.9841269841269841253e-04);
    p = fma(p, r, 1.3888888888888888889e-03);
    p = fma(p, r, 8.3333333333333333333e-03);
    p = fma(p, r, 4.1666666666666666667e-02);
    p = fma(p, r, 1.6666666666666666667e-01);
    p = fma(p, r, 0.5);                            // 1/2!
    const double em = fma(p * r, r, r);          // e^r - 1
    if (k == 0.0) return em;
    return __builtin_amdgcn_ldexp(1.0 + em, -(int)k) - 1.0;
}

template <bool VOP3 = false>
PL_DEV double lg_R(double z) {
    const double w = z * z;
    const double t1 = w * fma_k<VOP3>(w, fma_k<VOP3>(w, 1.531383769920937332e-01, 2.222219843214978396e-01), 3.999999999940941908e-01);
    const double t2 = z * fma_k<VOP3>(w, fma_k<VOP3>(w, fma_k<VOP3>(w, 1.479819860511658591e-01, 1.818357216161805012e-01),
                                         2.857142874366239149e-01), 6.666666666666735130e-01);
    return t2 + t1;
}
PL_DEV double log1p_pos(double x) {
    // branch-free (a wavefront's lanes mix both ranges): u = 1 + x rounded,
    // c = the rounding error of u relative to u, 1 + x = 2^k (1 + f) (1 + c)
    constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    const double u = 1.0 + x;
    int k = __builtin_amdgcn_frexp_exp(u) - 1;  // u = 2^k * m, m in [1, 2)
    double c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
    c *= __builtin_amdgcn_rcp(u);  // rounding correction, a few bits suffice
    double m = __builtin_amdgcn_ldexp(u, -k);
    const bool hi = m >= 1.4142135623730951;
    m = hi ? 0.5 * m : m;
    k += hi ? 1 : 0;
    const double f = m - 1.0;
    const double hfsq = 0.5 * f * f;
    const double s = div_fast(f, 2.0 + f);
    const double R = lg_R(s * s);
    const double dk = (double)k;
    return dk * LN2_HI - ((hfsq - (s * (hfsq + R) + (dk * LN2_LO + c))) - f);
}

// log1p(exp(-x)) for x >= 0 (finite or +inf), the SCL path-metric term
// (src/polar/decoder.py:374-406).  u = e^-x by exp_neg; then, as u <= 1,
// 1 + u = 2^j (1 + f) with j = 0, f = u below sqrt(2) - 1 and j = 1,
// f = (u - 1)/2 above -- both exact (Sterbenz), so the rounding correction of
// the general log1p (frexp, ldexp, a reciprocal) is not needed; the same fdlibm
// log kernel on f.  <= 1 ulp.
PL_DEV double log1p_exp_neg(double x) {
    constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    const double u = exp_neg(x);
    // (measured, not kept: lanes with x > 8 taking the log1p series u - u^2/2 +
    // ... - u^6/6 instead of the log kernel -- correctly rounded, 7 VALU instead
    // of ~25, but the per-lane branch cost the tree kernel registers: N = 1024 L =
    // 8 5.34 -> 6.70 ms, profiles/r06_b/ab_split.log)
    const bool big = u > 0.41421356237309503;
    const double f = big ? 0.5 * (u - 1.0) : u;
    const double hfsq = 0.5 * f * f;
    const double s = div_fast(f, 2.0 + f);
    const double R = lg_R(s * s);
    const double j = big ? 1.0 : 0.0;
    return j * LN2_HI - ((hfsq - (s * (hfsq + R) + j * LN2_LO)) - f);
}

}  // namespace pl
