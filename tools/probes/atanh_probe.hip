// Accuracy probe (diagnostic, not product): ldpc.hip's two_atanh with the
// division refined by two Newton steps (product) and by one, against
// 2*atanhl(p) in long double on the host, over p in [-0.999999, 0.999999]
// (uniform, log-uniform near 0 and near the clip bound).  Prints max ulp error
// and the share of results that differ between the two variants.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "../../polarcode_and_ldpc_amd/csrc/fp64_math.hpp"

namespace {
template <int NEWTON>
__device__ double div_n(double x, double y) {
    double r = __builtin_amdgcn_rcp(y);
    double e;
    if (NEWTON >= 1) { e = fma(-y, r, 1.0); r = fma(r, e, r); }
    if (NEWTON >= 2) { e = fma(-y, r, 1.0); r = fma(r, e, r); }
    const double q = x * r;
    return fma(fma(-y, q, x), r, q);
}
template <int NEWTON>
__device__ double two_atanh_n(double p) {
    constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    const double a = fabs(p);
    const float yf = (float)(1.0 + a) * __builtin_amdgcn_rcpf((float)(1.0 - a));
    const int k = __builtin_amdgcn_frexp_expf(yf * 1.41421356f) - 1;
    const double tk = __builtin_amdgcn_ldexp(1.0, k);
    const double s = div_n<NEWTON>(fma(a, 1.0 + tk, 1.0 - tk), fma(a, 1.0 - tk, 1.0 + tk));
    const double dk = (double)k;
    const double r = dk * LN2_HI + ((s + s) + (s * pl::lg_R<false>(s * s) + dk * LN2_LO));
    return __builtin_isnan(p) ? p : __builtin_copysign(r, p);
}
__global__ void k(const double* p, double* o2, double* o1, double* o0, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { o2[i] = two_atanh_n<2>(p[i]); o1[i] = two_atanh_n<1>(p[i]); o0[i] = two_atanh_n<0>(p[i]); }
}
// the reciprocal alone: v_rcp_f64 against 1/y in long double, y in [1, 2) and (0, 2^30)
__global__ void krcp(const double* y, double* r, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) r[i] = __builtin_amdgcn_rcp(y[i]);
}
double ulp_err(double got, long double ref) {
    const double r = (double)ref;
    const double u = std::nextafter(std::fabs(r), INFINITY) - std::fabs(r);
    return (double)std::fabs((long double)got - ref) / u;
}
}  // namespace

int main() {
    const int n = 1 << 23;
    std::vector<double> p(n);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-0.999999, 0.999999), lu(-40.0, 0.0);
    for (int i = 0; i < n; ++i) {
        const int kind = i % 3;
        double v = kind == 0 ? u(g) : (kind == 1 ? std::pow(2.0, lu(g)) : 0.999999 - std::pow(2.0, lu(g)) * 0.5);
        if (v > 0.999999) v = 0.999999;
        p[i] = (g() & 1) ? v : -v;
    }
    double *dp, *d2, *d1, *d0;
    hipMalloc(&dp, n * 8); hipMalloc(&d2, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d0, n * 8);
    hipMemcpy(dp, p.data(), n * 8, hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(dp, d2, d1, d0, n);
    std::vector<double> o2(n), o1(n), o0(n);
    hipMemcpy(o2.data(), d2, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(o1.data(), d1, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(o0.data(), d0, n * 8, hipMemcpyDeviceToHost);
    double m2 = 0, m1 = 0, m0 = 0;
    long diff1 = 0, diff0 = 0, cr2 = 0;
    for (int i = 0; i < n; ++i) {
        const long double ref = 2.0L * atanhl((long double)p[i]);
        const double e2 = ulp_err(o2[i], ref), e1 = ulp_err(o1[i], ref), e0 = ulp_err(o0[i], ref);
        m2 = std::max(m2, e2); m1 = std::max(m1, e1); m0 = std::max(m0, e0);
        cr2 += e2 <= 0.5;
        diff1 += o1[i] != o2[i];
        diff0 += o0[i] != o2[i];
    }
    // v_rcp_f64 itself
    std::uniform_real_distribution<double> e(0.0, 30.0);
    for (int i = 0; i < n; ++i) p[i] = (i & 1) ? 1.0 + (double)(g() >> 11) * 0x1p-53 : std::pow(2.0, e(g));
    hipMemcpy(dp, p.data(), n * 8, hipMemcpyHostToDevice);
    krcp<<<(n + 255) / 256, 256>>>(dp, d0, n);
    hipMemcpy(o0.data(), d0, n * 8, hipMemcpyDeviceToHost);
    double mr = 0;
    for (int i = 0; i < n; ++i) mr = std::max(mr, ulp_err(o0[i], 1.0L / (long double)p[i]));
    std::printf("{\"n\": %d, \"max_ulp_two_newton\": %.3f, \"max_ulp_one_newton\": %.3f, \"max_ulp_no_newton\": %.3f, "
                "\"correctly_rounded_two\": %.5f, \"differ_frac_one\": %.3g, \"differ_frac_none\": %.3g, "
                "\"v_rcp_f64_max_ulp\": %.3f}\n",
                n, m2, m1, m0, (double)cr2 / n, (double)diff1 / n, (double)diff0 / n, mr);
    return 0;
}
