// Shared device helpers for the gfx950 decoder kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PL_DEV __device__ __forceinline__

// PL_DIAG=1 (make DIAG=1, a separate library for tools/): adds the stamped /
// alternative-geometry polar tree instances, the thread-per-check LDPC kernel
// and the ocml BP path.  The product library (PL_DIAG=0) carries none of them.
#ifndef PL_DIAG
#define PL_DIAG 0
#endif

// np.sign semantics: +1 / -1 / 0 (NaN propagates).
PL_DEV double np_sign(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x)); }

// Min-sum f of src/polar/decoder.py:121-127:  sign(a)*sign(b)*min(|a|,|b|).
// Python's min(x, y) returns x unless y < x.  Exact (no rounding).
PL_DEV double f_minsum(double a, double b) {
    const double x = fabs(a), y = fabs(b);
    const double mn = (y < x) ? y : x;
    return np_sign(a) * np_sign(b) * mn;
}

// 64-bit value of another lane (lane index wave-uniform) -> scalar registers.
PL_DEV double readlane_d(double v, int l) {
    const long long x = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)x, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(x >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Spread the low 16 bits of x to the even bit positions of a 32-bit word.
PL_DEV uint32_t spread16(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// In-word stages of the polar transform x[t] ^= x[t+s] (t with bit s clear),
// s = 1..16 (src/polar/utils.py:193-229, natural index, bit t = position t).
PL_DEV uint32_t polar_word_transform(uint32_t x) {
    x ^= (x >> 1) & 0x55555555u;
    x ^= (x >> 2) & 0x33333333u;
    x ^= (x >> 4) & 0x0F0F0F0Fu;
    x ^= (x >> 8) & 0x00FF00FFu;
    x ^= (x >> 16) & 0x0000FFFFu;
    return x;
}

// ---- Philox4x32-10 (Salmon et al., SC'11) ---------------------------------
struct pl_u4 { uint32_t x, y, z, w; };
PL_DEV pl_u4 philox4x32_10(pl_u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = pl_u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}
