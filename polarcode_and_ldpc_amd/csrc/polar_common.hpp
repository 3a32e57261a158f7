// Polar f / g / path-metric arithmetic shared by the lane-per-path kernels
// (polar_lane.hip, polar_tree.hip).  Each is the reference's fp64 operation:
//   f  src/polar/decoder.py:121-127 (SCDecoder._upper_llr) and :408-410
//   g  src/polar/decoder.py:129-144 (SCDecoder._lower_llr) and :412-417
//   metric increments src/polar/decoder.py:374-406 (SCLDecoder._log_likelihood)
#pragma once
#include "common.hpp"
#include "fp64_math.hpp"
#include "internal.hpp"  // PL_METRIC_FUSED_NMAX

namespace pl {

// min-sum f with the reference's value semantics: sign(a)*sign(b)*min(|a|,|b|)
// (Python min keeps |a| unless |b| < |a|); NaN in either input gives NaN.  The
// sign of a zero result may differ from NumPy's, which never changes a value or
// decision downstream (x + -0 = x + 0 for x != 0, and -0 >= 0).  Exact.
// 7 VALU: cmp, 2 selects, xor + bfi for the sign, unordered cmp + select.
PL_DEV double f_ms(double a, double b) {
    const bool lt = fabs(b) < fabs(a);
    const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
    const uint32_t lo = lt ? (uint32_t)ub : (uint32_t)ua;
    const uint32_t hs = lt ? (uint32_t)(ub >> 32) : (uint32_t)(ua >> 32);
    const uint32_t sg = (uint32_t)(ua >> 32) ^ (uint32_t)(ub >> 32);
    uint32_t hi = (hs & 0x7FFFFFFFu) | (sg & 0x80000000u);
    hi = __builtin_isunordered(a, b) ? 0x7FF80000u : hi;
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
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

// whether path_metrics_fast must evaluate log1p(e^-|lam|) for this lane (else
// the term is below a quarter ulp of every addend, or the lane is idle)
PL_DEV bool metric_needs_t(double pm, double lam, bool active) {
    const double x = fabs(lam);
    const int ep = __builtin_amdgcn_frexp_exp(pm);
    const int ex = __builtin_amdgcn_frexp_exp(x);
    const int e = ep < ex ? ep : ex;
    const bool finite_pm = __builtin_isfinite(pm);
    return !(!active || (!finite_pm && !__builtin_isnan(x)) ||
             (finite_pm && pm != 0.0 && x > (double)(57 - e) * 0.6931471805599453));
}


// Same increments for the tree kernel, with a cheaper skip test (hardware
// frexp exponents: frexp_exp = ilogb + 1 for finite nonzero values, so the
// threshold is identical) and two more skips that cannot change a result:
// inactive list slots (their metrics are never read) and pm = +-inf with a
// non-NaN LLR (t is finite, so pm + anything finite = pm as in the reference).
// t = log1p(exp(-x)), x >= 0, in the list kernels' evaluations (fp64_math.hpp):
// FORM 0 lean exp + log1p, 1 fused
template <int FORM>
PL_DEV double metric_t(double x) {
    if constexpr (FORM == 1) return log1p_exp_neg(x);
    else return log1p_pos(exp_neg(x));
}

template <bool WANT1, int FORM = 0>
PL_DEV void path_metrics_fast(double pm, double lam, bool active, double& m0, double& m1) {
    const double x = fabs(lam);
    const bool skip = !metric_needs_t(pm, lam, active);
    double t = 0.0;
    if (!skip) t = metric_t<FORM>(x);
    m0 = pm + ((lam >= 0.0) ? -t : lam - t);
    if (WANT1) m1 = pm + ((lam >= 0.0) ? -lam - t : -t);
}

// CRC register of u_hat[info bits] for this lane's path, from its root partial
// sum x_hat (u = x_hat F^{(x)n} and the bit-serial CRC of src/polar/utils.py:
// 86-163 are both GF(2)-linear with zero initial register, so the CRC is the
// XOR of the host table g[j] over the set bits j of x_hat).  `root` points at
// word 0 of the lane's x_hat, consecutive words `stride` u32 apart.
PL_DEV uint32_t crc_of_xhat(const uint32_t* root, int stride, int words, const uint32_t* __restrict__ g) {
    uint32_t crc = 0;
    for (int w = 0; w < words; ++w) {
        const uint32_t x = root[w * stride];
#pragma unroll 8
        for (int b = 0; b < 32; ++b) crc ^= ((x >> b) & 1u) ? g[32 * w + b] : 0u;
    }
    return crc;
}

// Issue priority 0..3 by the quarter of [0, n) that i falls in (the list
// kernels' frame-group schedule, polar_tree.hip / polar_lane.hpp): s_setprio
// takes an immediate, so one branch per level (wave-uniform).
PL_DEV void set_prio_quarter(unsigned int i, unsigned int n) {
    const unsigned int q = (unsigned int)(((uint64_t)i * 4u) / n);
    if (q >= 3) __builtin_amdgcn_s_setprio(3);
    else if (q == 2) __builtin_amdgcn_s_setprio(2);
    else if (q == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

}  // namespace pl
