// Batched LDPC flooding decoder (sum-product BP and normalised min-sum) for
// gfx950 (MI355X).
//
// Semantics: src/ldpc/decoder.py of the reference --
//   BPDecoder.decode :124-202   check update :62-96  (t = clip(tanh(m/2), +-0.999999);
//                               leave-one-out product in ascending neighbour order,
//                               sequential, no divide-out; clip; 2*atanh; nan_to_num),
//                               variable update :98-122 (total = llr + np.sum(msgs));
//                               decision total <= 0 -> 1; syndrome early stop.
//   MSDecoder.decode :289-352   check update :257-287 (sign product * leave-one-out
//                               min * normalization).
// np.sum over the incoming messages is NumPy's pairwise_sum (sequential below 8
// terms, 8 accumulators up to 128); reproduced exactly.
//
// Mapping (DESIGN.md §4 LDPC kernels): one workgroup decodes one frame.  State
// T[E] (check inputs) + C[E] (check-to-variable) in LDS, v2c = total - c2v
// exactly as the reference forms it; edges check-major (CSR of H, checks
// degree-sorted) so a check's inputs are contiguous.  Kernels:
//   ldpc_reg_kernel<ALGO, DV, EPT, VPT>  constant variable degree: adjacency and
//                                        channel LLRs in registers, BP tanh via a
//                                        compacted work list (the BASELINE codes);
//   ldpc_decode_kernel<ALGO, GLOBAL, ..> any code, LDS or global-workspace state;
//   ldpc_ms_compact_kernel               min-sum for codes whose T/C exceed LDS:
//                                        compressed per-check statistics in LDS;
//   ldpc_ms36_kernel<VPT>                the same for (3,6)-regular n = 1024 VPT
//                                        (the BASELINE n = 8192 code);
//   ldpc_check_kernel<ALGO>              thread-per-check variant (diagnostic).
#include "common.hpp"
#include "internal.hpp"
#include "fp64_math.hpp"

#include <cstdlib>
#include <string>
#include <type_traits>

namespace pl {

PL_DEV double clip999(double x) {
    const double c = 0.999999;
    return x < -c ? -c : (x > c ? c : x);
}


// OR of `pred` over the workgroup behind one barrier (__syncthreads_or costs
// three: a reduction, then two barriers around an LDS word): each wavefront's
// ballot goes to its own LDS word, words[parity][wave] (double-buffered by the
// caller's iteration parity, so a word is rewritten only after every wavefront
// has passed the barriers of the iteration that read it), then every thread
// reads them all.  words: 2 * 16 u32 of LDS.
PL_DEV bool wg_any(bool pred, uint32_t* words, int parity) {
    const bool any_w = __ballot(pred) != 0;
    if (__lane_id() == 0) words[parity * 16 + (threadIdx.x >> 6)] = any_w ? 1u : 0u;
    __syncthreads();
    const uint4* w4 = reinterpret_cast<const uint4*>(words + parity * 16);
    uint32_t any = 0;
    const int nw4 = (blockDim.x + 255) >> 8;  // wavefronts / 4
    for (int k = 0; k < nw4; ++k) {
        const uint4 v = w4[k];
        any |= v.x | v.y | v.z | v.w;
    }
    return any != 0u;
}

// 2*atanh(p), |p| <= 0.999999 (after the reference's clip), NaN -> NaN.
// 2 atanh(a) = log(y), y = (1+a)/(1-a) = 2^k m, m in [sqrt(2)/2, sqrt(2)) with k
// from an fp32 estimate of y; log(m) = 2s + s R(s^2) (the fdlibm log kernel),
// s = (m-1)/(m+1) = (a(1+2^k) + (1-2^k)) / (a(1-2^k) + (1+2^k)): numerator and
// denominator are single fmas of exact constants (correctly rounded, no
// cancellation), so one division serves the whole evaluation.  k = 0 gives
// s = a exactly (the atanh series).  <= 2 ulp, ~97 % correctly rounded.
PL_DEV double two_atanh(double p) {
    constexpr double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
    const double a = fabs(p);
    const float yf = (float)(1.0 + a) * __builtin_amdgcn_rcpf((float)(1.0 - a));  // 1 - a >= 1e-6
    const int k = __builtin_amdgcn_frexp_expf(yf * 1.41421356f) - 1;               // 0 <= k <= 21
    const double tk = __builtin_amdgcn_ldexp(1.0, k);
    const double s = div_fast(fma(a, 1.0 + tk, 1.0 - tk), fma(a, 1.0 - tk, 1.0 + tk));
    const double dk = (double)k;
    const double r = dk * LN2_HI + ((s + s) + (s * lg_R<true>(s * s) + dk * LN2_LO));
    return __builtin_isnan(p) ? p : __builtin_copysign(r, p);
}
// clip(tanh(x/2), +-0.999999).  e^-|x| = 2^-k e^r (Cody-Waite, |r| <= ln2/2) and
// e^r = (R + r)/(R - r) with R = r coth(r/2) = 2 + Rp(r^2), Rp the fdlibm exp
// minimax fit (P1..P5), so tanh(|x|/2) = (2^k - e^r)/(2^k + e^r) is one division:
//   k <= 1: ((2^k-1)R - (2^k+1)r) / ((2^k+1)R - (2^k-1)r)
//   k >= 2: 1 - 2(R + r) / ((2^k+1)R - (2^k-1)r)   (small correction, no cancellation)
// <= 4 ulp, 84 % correctly rounded (the expm1 form it replaces: 57 %).  For
// |x| > 14.52 tanh(|x|/2) exceeds the clip bound by > 1e-8 (>> any rounding).
PL_DEV double tanh_half_clip(double x) {
    constexpr double INV_LN2 = 1.4426950408889634074, LN2_HI = 6.93147180369123816490e-01,
                     LN2_LO = 1.90821492927058770002e-10;
    const double ax = fabs(x);
    double t = 0.999999;
    if (ax <= 14.52) {
        const double k = __builtin_rint(ax * INV_LN2);
        double r = fma(-k, LN2_HI, ax);
        r = -fma(-k, LN2_LO, r);  // k ln2 - |x|
        const double z = r * r;
        const double Rp = z * fma_k<true>(z, fma_k<true>(z, fma_k<true>(z, fma_k<true>(z, 4.13813679705723846039e-08, -1.65339022054652515390e-06),
                                                        6.61375632143793436117e-05), -2.77777777770155933842e-03),
                                    1.66666666666666019037e-01);
        const double tk = __builtin_amdgcn_ldexp(1.0, (int)k), A = tk - 1.0, B = tk + 1.0;
        const bool big = k >= 2.0;
        const double num = big ? 2.0 * ((2.0 + r) + Rp) : fma(A, Rp, fma(-B, r, A + A));
        const double q = div_fast(num, fma(B, Rp, fma(-A, r, B + B)));
        t = __builtin_fmin(big ? 1.0 - q : q, 0.999999);  // x NaN: replaced below
    }
    return __builtin_isnan(x) ? x : __builtin_copysign(t, x);
}

// numpy add.reduce (pairwise_sum) over msgs gathered through var_edge.
PL_DEV double np_sum_gather(const double* C, const int32_t* __restrict__ ve, int dv) {
    if (dv < 8) {
        double res = 0.;
        for (int k = 0; k < dv; ++k) res += C[ve[k]];
        return res;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = C[ve[j]];
    int i = 8;
    for (; i < dv - (dv % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += C[ve[i + j]];
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < dv; ++i) res += C[ve[i]];
    return res;
}

// Min-sum check output for edge i of a degree-d check (decoder.py:270-287):
// (prod_{k != i} np.sign(x_k)) * min_{k != i} |x_k| * normalization.  The
// sequential sign product is +-1 by the parity of negatives, +-0 (same parity)
// if any factor is zero (np.sign(+-0) = +0), NaN if any is NaN; the min is
// NaN-propagating like np.min.  Same value as the loop it restates.
PL_DEV double ms_check(const double* x, int i, int d, double norm) {
    const double* hi = x + 1;
    double mn = 0.0;
    uint32_t neg = 0, zero = 0, nan = 0;
    for (int k = 0; k < d - 1; ++k) {
        const double v = (k < i ? x : hi)[k];
        neg ^= v < 0.0 ? 1u : 0u;
        zero |= v == 0.0 ? 1u : 0u;
        nan |= __builtin_isnan(v) ? 1u : 0u;
        const double av = fabs(v);
        mn = (k == 0 || av < mn) ? av : mn;
    }
    double sp = neg ? -1.0 : 1.0;
    sp = zero ? sp * 0.0 : sp;
    sp = nan ? __builtin_nan("") : sp;
    return sp * mn * norm;
}

// Flooding decoder, one workgroup per frame.  State: T[E] (check inputs:
// clip(tanh(v2c/2)) for BP, v2c for MS), C[E] (check-to-variable), bt[n]
// (decisions), syn[2][m] (syndrome parity, double-buffered).  Per iteration:
//   vote (early stop, it > 0): OR of the previous variable pass's syndrome
//     parities in a __syncthreads_or -> all checks satisfied: stop with
//     iterations = it (the reference's break after iteration it-1,
//     decoder.py:194-198);
//   check pass (thread = edge): C[e] = leave-one-out over the check's T in
//     ascending neighbour order (two loops around e: the same left-to-right
//     product as np.prod over the masked messages, decoder.py:87);
//   variable pass (thread = variable): total = llr + np.sum(C over its checks)
//     (NumPy pairwise order), decision total <= 0 (decoder.py:191), the next
//     check inputs T[e] = f(total - C[e]) (v2c exactly as decoder.py:120 forms
//     it), and the syndrome parity toggled with LDS atomics.
template <int ALGO, bool GLOBAL, bool OCML>
__global__ void __launch_bounds__(1024)
ldpc_decode_kernel(LdpcGeom g, LdpcDev dv, const double* __restrict__ llr, int64_t ld,
                   uint8_t* __restrict__ bits, int32_t* __restrict__ iters, int64_t batch,
                   double* __restrict__ work) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t frame = blockIdx.x;
    if (frame >= batch) return;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int E = g.E, n = g.n, m = g.m;
    double* T;
    unsigned char* lds = smem;
    if constexpr (GLOBAL) {
        T = work + (int64_t)blockIdx.x * (2 * (int64_t)E);
    } else {
        T = reinterpret_cast<double*>(smem);
        lds += (size_t)2 * E * sizeof(double);
    }
    double* C = T + E;
    uint32_t* syn = reinterpret_cast<uint32_t*>(lds);  // [2][m]
    uint8_t* bt = lds + (size_t)8 * m;                  // [n]
    const double* __restrict__ ch = llr + frame * ld;
    auto tin = [&](double x) -> double {
        if (ALGO != 0) return x;
        return OCML ? clip999(tanh(x / 2.0)) : tanh_half_clip(x);
    };

    for (int c = tid; c < 2 * m; c += nt) syn[c] = 0u;
    for (int v = tid; v < n; v += nt) {  // v2c = llr (decoder.py:144-146), c2v = 0
        const int a0 = dv.var_ptr[v], d = dv.var_ptr[v + 1] - a0;
        const double t = tin(ch[v]);
        for (int k = 0; k < d; ++k) {
            const int e = dv.var_edge[a0 + k];
            T[e] = t;
            C[e] = 0.0;
        }
    }
    __syncthreads();
    int done = g.max_iter;
    for (int it = 0; it < g.max_iter; ++it) {
        uint32_t* sprev = syn + ((it + 1) & 1) * m;  // toggled by the previous variable pass
        uint32_t* scur = syn + (it & 1) * m;         // toggled by this iteration's variable pass
        if (g.early_stop && it > 0) {                // decoder.py:194-198, after iteration it-1
            int bad = 0;
            for (int c = tid; c < m; c += nt) bad |= (int)sprev[c];
            if (!__syncthreads_or(bad)) { done = it; break; }
        }
        // ---- check pass
        for (int c = tid; c < m; c += nt) scur[c] = 0u;
        for (int e = tid; e < E; e += nt) {
            const int meta = dv.edge_meta[e];
            const int e0 = meta & 0xFFFFF, d = meta >> 20, i = e - e0;
            double o;
            if (ALGO == 0) {
                // np.prod over the masked messages, left to right (see ldpc_reg_kernel)
                const double* lo = T + e0;
                const double* hi = lo + 1;
                const int nf = d - 1;
                double p = 1.0;
                int k = 0;
                for (; k + 4 <= nf; k += 4, lo += 4, hi += 4) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) p *= (k + c < i ? lo : hi)[c];
                }
                for (; k < nf; ++k, ++lo, ++hi) p *= (k < i ? lo : hi)[0];
                const bool pn = __builtin_isnan(p);
                p = __builtin_fmax(__builtin_fmin(p, 0.999999), -0.999999);
                o = OCML ? 2.0 * atanh(p) : two_atanh(p);
                o = pn ? 0.0 : o;  // nan_to_num; 2*atanh is finite after the clip
            } else {
                o = ms_check(T + e0, i, d, g.norm);
            }
            C[e] = o;
        }
        __syncthreads();
        // ---- variable pass
        for (int v = tid; v < n; v += nt) {
            const int a0 = dv.var_ptr[v], d = dv.var_ptr[v + 1] - a0;
            const double total = ch[v] + np_sum_gather(C, dv.var_edge + a0, d);
            const bool one = total <= 0.0;
            bt[v] = one ? 1 : 0;
            for (int k = 0; k < d; ++k) {
                const int e = dv.var_edge[a0 + k];
                T[e] = tin(total - C[e]);
                if (one) atomicXor(&scur[dv.var_chk[a0 + k]], 1u);
            }
        }
        __syncthreads();
    }
    uint8_t* o = bits + frame * (int64_t)n;
    for (int v = tid; v < n; v += nt) o[v] = bt[v];
    if (iters && tid == 0) iters[frame] = done;
}

#ifndef PL_MS_PRIO
// ldpc_ms_compact_kernel: issue priority falling with a wavefront's progress
// through each pass, 1 = per batch of checks, 2 = per check (16 384 frames of
// n = 8192: 12.61 -> 11.78 -> 11.40 ms, profiles/r04_a/ab_bp_prio.log,
// ab_ms_prio2.log)
#define PL_MS_PRIO 2
#endif
// s_setprio 3..0 as step i of n passes its quarters: the wavefronts of a SIMD
// belong to one workgroup and meet at the next barrier, so the ones behind
// get the issue slots (age-ordered arbitration otherwise lets the oldest run ahead)
PL_DEV void ms_prio(int i, int n) {
    const int q = (4 * i) / n;
    if (q == 0) __builtin_amdgcn_s_setprio(3);
    else if (q == 1) __builtin_amdgcn_s_setprio(2);
    else if (q == 2) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

#ifndef PL_MS_REGIDX
#define PL_MS_REGIDX 1  // regular min-sum codes: adjacency indices cached in registers
#endif

// Register-cached variant of ldpc_decode_kernel for codes whose variable degree
// is a constant DV < 8 (np.sum is then sequential) and whose state fits LDS:
// 256 threads, thread tid owns edges tid + j*256 (j < EPT) and variables
// tid + j*256 (j < VPT); their edge metadata, var_edge / var_chk lists and
// channel LLRs are loaded once into registers instead of once per iteration.
// Same passes and arithmetic as ldpc_decode_kernel (bit-identical).  BP on
// codes with check degrees <= 15 runs ldpc_bp_grp_kernel below instead; this
// one serves min-sum and the other BP codes (and PL_LDPC_KERNEL=reg).
// Measured and not kept: products over all d inputs with the
// own factor replaced by 1.0 (8.18 against 7.00 ms), 2 / 4 frames per
// workgroup sharing its barriers (8.10 / 9.83), progress-based issue priority
// (+1.4 %).
template <int ALGO, int DV, int EPT, int VPT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
ldpc_reg_kernel(LdpcGeom g, LdpcDev dv, const double* __restrict__ llr, int64_t ld,
                uint8_t* __restrict__ bits, int32_t* __restrict__ iters, int64_t batch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NT = 256;
    const int64_t frame = blockIdx.x;
    if (frame >= batch) return;
    const int tid = threadIdx.x;
    const int E = g.E, n = g.n, m = g.m;
    double* T = reinterpret_cast<double*>(smem);
    double* C = T + E;
    uint32_t* syn = reinterpret_cast<uint32_t*>(smem + (size_t)16 * E);  // [2][m]
    uint8_t* bt = reinterpret_cast<uint8_t*>(syn + 2 * m);               // [n]
    // BP: per-wavefront lists of the edges whose v2c needs a tanh (|x| <= 14.52
    // or NaN), 16-bit edge indices (E < 65536), 64*VPT*DV per wavefront: each
    // wavefront compacts and evaluates its own, so the tanh pass needs no
    // workgroup barrier (capi.cpp sizes it with ldpc_reg_list_bytes)
    uint16_t* work = reinterpret_cast<uint16_t*>(smem + (((size_t)16 * E + (size_t)8 * m + n + 15) & ~(size_t)15));
    uint32_t* vote = reinterpret_cast<uint32_t*>(smem + g.lds_bytes - 128);  // [2][16] (wg_any)
    const double* __restrict__ ch = llr + frame * ld;
    auto tin = [&](double x) -> double { return ALGO == 0 ? tanh_half_clip(x) : x; };
    const int lane = __lane_id();

    int meta[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const int e = tid + j * NT;
        meta[j] = e < E ? dv.edge_meta[e] : 0;
    }
    int ve[VPT][DV], vc[VPT][DV];
    double chv[VPT];
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
        const int v = tid + j * NT;
        const bool ok = v < n;
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            ve[j][k] = ok ? dv.var_edge[v * DV + k] : 0;
            vc[j][k] = ok ? dv.var_chk[v * DV + k] : 0;
        }
        chv[j] = ok ? ch[v] : 0.0;
    }
    for (int c = tid; c < 2 * m; c += NT) syn[c] = 0u;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
        if (tid + j * NT < n) {
            const double t = tin(chv[j]);
#pragma unroll
            for (int k = 0; k < DV; ++k) {
                T[ve[j][k]] = t;
                C[ve[j][k]] = 0.0;
            }
        }
    }
    __syncthreads();
    int done = g.max_iter;
    for (int it = 0; it < g.max_iter; ++it) {
        uint32_t* sprev = syn + ((it + 1) & 1) * m;
        uint32_t* scur = syn + (it & 1) * m;
        if (g.early_stop && it > 0) {
            int bad = 0;
            for (int c = tid; c < m; c += NT) bad |= (int)sprev[c];
            if (!wg_any(bad != 0, vote, it & 1)) { done = it; break; }
        }
        for (int c = tid; c < m; c += NT) scur[c] = 0u;
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int e = tid + j * NT;
            if (e >= E) break;
            const int e0 = meta[j] & 0xFFFFF, d = meta[j] >> 20, i = e - e0;
            double o;
            if (ALGO == 0) {
                // np.prod over the masked messages, left to right: factor k of
                // d-1 is T[e0 + k] before the own edge, T[e0 + k + 1] after it
                // (two running LDS pointers, one select per factor; a guarded
                // tail instead of a remainder loop)
                const double* lo = T + e0;
                const double* hi = lo + 1;
                const int nf = d - 1;
                double p = 1.0;
                int k = 0;
                for (; k + 4 <= nf; k += 4, lo += 4, hi += 4) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) p *= (k + c < i ? lo : hi)[c];
                }
                if (k < nf) {
                    p *= (k < i ? lo : hi)[0];
                    if (k + 1 < nf) {
                        p *= (k + 1 < i ? lo : hi)[1];
                        if (k + 2 < nf) p *= (k + 2 < i ? lo : hi)[2];
                    }
                }
                // clip, 2*atanh, nan_to_num: after the clip 2*atanh is finite,
                // so only a NaN product (NaN channel LLRs) maps to 0
                const bool pn = __builtin_isnan(p);
                o = two_atanh(__builtin_fmax(__builtin_fmin(p, 0.999999), -0.999999));
                o = pn ? 0.0 : o;
            } else {
                o = ms_check(T + e0, i, d, g.norm);
            }
            C[e] = o;
        }
        __syncthreads();
        uint16_t* const wl = work + (tid >> 6) * (64 * VPT * DV);  // this wavefront's tanh list
        int wn = 0;                                                 // its length (wavefront-uniform)
#pragma unroll
        for (int j = 0; j < VPT; ++j) {
            const int v = tid + j * NT;
            const bool vok = v < n;  // lanes past n run along (ve = 0) with every store masked
            if (!__ballot(vok)) break;
            double c2v[DV];
            double sum = 0.0;  // np.sum over DV < 8 messages: sequential
#pragma unroll
            for (int k = 0; k < DV; ++k) {
                c2v[k] = C[ve[j][k]];
                sum += c2v[k];
            }
            const double total = chv[j] + sum;
            const bool one = total <= 0.0;
            if (vok) bt[v] = one ? 1 : 0;
#pragma unroll
            for (int k = 0; k < DV; ++k) {
                const double x = total - c2v[k];  // v2c as decoder.py:120 forms it
                if (ALGO == 0) {
                    // saturated inputs take the clip value now; the rest are
                    // appended to the wavefront's list and get their tanh below
                    const bool sat = fabs(x) > 14.52;
                    if (vok) T[ve[j][k]] = sat ? __builtin_copysign(0.999999, x) : x;
                    const bool need = vok && !sat;
                    const uint64_t nb = __ballot(need);
                    const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(nb >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)nb, 0u));
                    if (need) wl[wn + pre] = (uint16_t)ve[j][k];
                    wn += (int)__popcll(nb);
                } else if (vok) {
                    T[ve[j][k]] = x;
                }
                if (vok && one) atomicXor(&scur[vc[j][k]], 1u);
            }
        }
        if (ALGO == 0) {
            // the list and its T entries were written by this wavefront, and LDS
            // runs a wavefront's operations in order: no barrier
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int w = lane; w < wn; w += 64) {
                const int e = wl[w];
                T[e] = tanh_half_clip(T[e]);
            }
        }
        __syncthreads();  // T and the syndrome parities for the next iteration's vote / check pass
    }
    uint8_t* o = bits + frame * (int64_t)n;
    for (int v = tid; v < n; v += NT) o[v] = bt[v];
    if (iters && tid == 0) iters[frame] = done;
}

// ---- BP with degree-grouped check products (ldpc_bp_grp_kernel)
// The edge slots of ldpc_reg_kernel (slot s = 4 j + wavefront: edges 64 s ..
// 64 s + 63 of the degree-sorted check-major order) span one or two check
// degrees each.  The host gives every slot its maximum degree D_s and lays the
// check inputs out per check, 16-byte aligned and padded with 1.0 up to the
// largest D_s among the slots holding the check's edges (T'[], C'[] of length
// tl; the pads are written once and never change).  A lane's product is then
// the same instruction stream for its whole wavefront: the D_s inputs of its
// check read as D_s/2 ds_read_b128 at immediate offsets, multiplied left to
// right with the lane's own factor skipped through the exec mask.  x * 1.0 = x,
// so every lane gets exactly the sequential product over its check's other
// inputs (decoder.py:87) -- no per-factor pointer select, no per-lane trip
// count, one LDS round trip per product.

// p *= t0 (then t1) on the lanes whose position i is not K (resp. K + 1): the
// compare, the exec mask and the multiplies in one block (the compare kept
// inside, so it is not hoisted out of the iteration loop into SGPRs)
template <int K>
PL_DEV double mul_skip1(double p, double t0, int i) {
    uint64_t sv, m0;
    asm("v_cmp_ne_u32_e64 %[m0], %[k0], %[i]\n\t"
        "s_and_saveexec_b64 %[sv], %[m0]\n\t"
        "v_mul_f64 %[p], %[p], %[t0]\n\t"
        "s_mov_b64 exec, %[sv]"
        : [p] "+v"(p), [sv] "=&s"(sv), [m0] "=&s"(m0)
        : [k0] "n"(K), [i] "v"(i), [t0] "v"(t0)
        : "scc");
    return p;
}
template <int K>
PL_DEV double mul_skip2(double p, double2 t, int i) {
    uint64_t sv, m0, m1;
    asm("v_cmp_ne_u32_e64 %[m0], %[k0], %[i]\n\t"
        "v_cmp_ne_u32_e64 %[m1], %[k1], %[i]\n\t"
        "s_and_saveexec_b64 %[sv], %[m0]\n\t"
        "v_mul_f64 %[p], %[p], %[t0]\n\t"
        "s_and_b64 exec, %[sv], %[m1]\n\t"
        "v_mul_f64 %[p], %[p], %[t1]\n\t"
        "s_mov_b64 exec, %[sv]"
        : [p] "+v"(p), [sv] "=&s"(sv), [m0] "=&s"(m0), [m1] "=&s"(m1)
        : [k0] "n"(K), [k1] "n"(K + 1), [i] "v"(i), [t0] "v"(t.x), [t1] "v"(t.y)
        : "scc");
    return p;
}
template <int Q, int D>
PL_DEV double grp_mul_pairs(double p, const double2* t, int i) {
    if constexpr (2 * Q + 1 < D) return grp_mul_pairs<Q + 1, D>(mul_skip2<2 * Q>(p, t[Q], i), t, i);
    else if constexpr (2 * Q + 1 == D) return mul_skip1<2 * Q>(p, t[Q].x, i);
    else return p;
}
// the product over positions k < D, k != i, of the check inputs at tb
template <int D>
PL_DEV double grp_prod(const double* tb, int i) {
    const double2* t2 = reinterpret_cast<const double2*>(tb);
    double2 t[(D + 1) / 2];
#pragma unroll
    for (int q = 0; q < (D + 1) / 2; ++q) t[q] = t2[q];
    return grp_mul_pairs<0, D>(1.0, t, i);
}

// STAMPS (diagnostic build): per-phase s_memtime cycles of every wavefront,
// summed into stamps[wavefront][8] (init, vote, check pass, its barrier,
// variable pass, tanh list, closing barrier, output).
// FPG frames per workgroup, one after the other: the frame-independent tables
// (edge slots, variable slots, pads) are loaded / written once per workgroup
// and the next frame's channel LLRs are fetched while the current one decodes.
template <int DV, int EPT, int VPT, bool STAMPS = false, int FPG = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
ldpc_bp_grp_kernel(LdpcGeom g, LdpcDev dv, const double* __restrict__ llr, int64_t ld,
                   uint8_t* __restrict__ bits, int32_t* __restrict__ iters, int64_t batch,
                   unsigned long long* __restrict__ stamps) {
    unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tprev = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
#define PL_GSTAMP(k)                                               \
    if constexpr (STAMPS) {                                        \
        const unsigned long long tn = __builtin_amdgcn_s_memtime(); \
        st[k] += tn - tprev;                                       \
        tprev = tn;                                                \
    }
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NT = 256;
    const int64_t frame0 = (int64_t)blockIdx.x * FPG;
    if (frame0 >= batch) return;
    const int tid = threadIdx.x;
    const int n = g.n, m = g.m, tl = g.tl;
    double* T = reinterpret_cast<double*>(smem);  // T'[tl]: check inputs, per check, padded
    double* C = T + tl;                           // C'[tl]: check-to-variable, same positions
    // syndrome of the current decisions, kept across iterations: a variable
    // whose decision flips toggles its checks' parities (no per-iteration reset,
    // and the LDS atomics only where a decision changed)
    const int mp = (m + 3) & ~3;
    uint32_t* syn = reinterpret_cast<uint32_t*>(smem + (size_t)16 * tl);  // [mp]
    uint16_t* work = reinterpret_cast<uint16_t*>(smem + (((size_t)16 * tl + (size_t)4 * mp + 15) & ~(size_t)15));
    const int lane = __lane_id();

    int meta[EPT];  // T' position of the edge's check | position in the check << 16 | D_s << 20
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const int e = tid + j * NT;
        meta[j] = dv.grp_meta[e];  // [256 EPT], host-assigned edges (position 15: none)
    }
    // variables by thread slot q = tid + 256 j (host-chosen order):
    // var_tpos = [T' positions of the slot's DV edges][their checks][variable or -1]
    int ve[VPT][DV], vc[VPT][DV], vid[VPT];
    double chv[VPT], nchv[FPG > 1 ? VPT : 1];
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
        const int q = tid + j * NT;
        vid[j] = dv.var_tpos[2 * DV * NT * VPT + q];
        const bool ok = vid[j] >= 0;
#pragma unroll
        for (int k = 0; k < DV; ++k) {
            ve[j][k] = dv.var_tpos[q * DV + k];
            vc[j][k] = dv.var_tpos[DV * NT * VPT + q * DV + k];
        }
        chv[j] = ok ? llr[frame0 * ld + vid[j]] : 0.0;
    }
    {
        // the pads (positions no edge writes: no barrier before the edges' writes)
        const int32_t* __restrict__ pads = dv.var_tpos + (2 * DV + 1) * NT * VPT;
        for (int q = tid; q < g.npad; q += NT) {
            const int x = pads[q];
            if (x >= 0) T[x] = 1.0;
        }
    }
  for (int fk = 0; fk < FPG; ++fk) {
    const int64_t frame = frame0 + fk;
    if (frame >= batch) break;  // workgroup-uniform
    if (fk > 0) {
        __syncthreads();  // every wavefront is done with the previous frame's T', C', syndrome
#pragma unroll
        for (int j = 0; j < VPT; ++j) chv[j] = nchv[j];
    }
    for (int c = tid; c < mp; c += NT) syn[c] = 0u;  // H * 0
    uint32_t decs = 0;  // bit j: the decision of variable tid + 256 j (initially 0)
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
        if (vid[j] >= 0) {
            const double t = tanh_half_clip(chv[j]);
#pragma unroll
            for (int k = 0; k < DV; ++k) {
                T[ve[j][k]] = t;
                C[ve[j][k]] = 0.0;
            }
        }
    }
    __syncthreads();
    if constexpr (FPG > 1) {  // the next frame's channel LLRs, in flight while this one decodes
        if (frame + 1 < batch && fk + 1 < FPG) {
#pragma unroll
            for (int j = 0; j < VPT; ++j) nchv[j] = vid[j] >= 0 ? llr[(frame + 1) * ld + vid[j]] : 0.0;
        }
    }
    PL_GSTAMP(0)
    int done = g.max_iter;
    for (int it = 0; it < g.max_iter; ++it) {
        if (g.early_stop && it > 0) {
            // every wavefront reads all m parities itself (the previous closing
            // barrier made them complete) and reaches the same verdict: no
            // cross-wavefront vote, no barrier (__syncthreads_or costs three)
            uint32_t bad = 0;
            for (int c = 4 * lane; c < m; c += 256) {
                if (c + 4 <= m) {
                    const uint4 w4 = *reinterpret_cast<const uint4*>(syn + c);
                    bad |= w4.x | w4.y | w4.z | w4.w;
                } else {
                    for (int k = c; k < m; ++k) bad |= syn[k];
                }
            }
            if (!__ballot(bad != 0u)) { done = it; break; }
        }
        PL_GSTAMP(1)
        // the product of slot j over its D_s inputs (one instruction stream per wavefront)
        auto slot_prod = [&](int j, int& base, int& i) -> double {
            const int D = __builtin_amdgcn_readfirstlane(meta[j] >> 20);  // the slot's D_s
            base = meta[j] & 0xFFFF;
            i = (meta[j] >> 16) & 15;
            const double* tb = T + base;
            switch (D) {
                case 0: return 0.0;  // slot past the last edge (not stored)
                case 1: return grp_prod<1>(tb, i);
                case 2: return grp_prod<2>(tb, i);
                case 3: return grp_prod<3>(tb, i);
                case 4: return grp_prod<4>(tb, i);
                case 5: return grp_prod<5>(tb, i);
                case 6: return grp_prod<6>(tb, i);
                case 7: return grp_prod<7>(tb, i);
                case 8: return grp_prod<8>(tb, i);
                case 9: return grp_prod<9>(tb, i);
                case 10: return grp_prod<10>(tb, i);
                case 11: return grp_prod<11>(tb, i);
                case 12: return grp_prod<12>(tb, i);
                case 13: return grp_prod<13>(tb, i);
                case 14: return grp_prod<14>(tb, i);
                default: return grp_prod<15>(tb, i);
            }
        };
        // clip, 2*atanh, nan_to_num: after the clip 2*atanh is finite, so
        // only a NaN product (NaN channel LLRs) maps to 0.  (This form -- the
        // uniform skip of an empty slot ahead of the product, the product as a
        // function returning from its switch -- schedules 3 % faster than the
        // same operations written inline, 6.21 -> 6.03 ms, bits identical; two
        // slots' 2*atanh chains side by side: 6.14, profiles/r05_b/ab_bp_pair.log)
        auto c2v_of = [](double p) -> double {
            const double o = two_atanh(__builtin_fmax(__builtin_fmin(p, 0.999999), -0.999999));
            return __builtin_isnan(p) ? 0.0 : o;
        };
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            if (__builtin_amdgcn_readfirstlane(meta[j] >> 20) == 0) continue;  // slot past the last edge
            int base, i;
            const double p = slot_prod(j, base, i);
            C[base + i] = c2v_of(p);  // lanes without an edge: the sink
        }
        PL_GSTAMP(2)
        __syncthreads();
        PL_GSTAMP(3)
        uint16_t* const wl = work + (tid >> 6) * (64 * VPT * DV);  // this wavefront's tanh list
        int wn = 0;
#pragma unroll
        for (int j = 0; j < VPT; ++j) {
            const bool vok = vid[j] >= 0;
            if (!__ballot(vok)) continue;
            double c2v[DV];
            double sum = 0.0;  // np.sum over DV < 8 messages: sequential
#pragma unroll
            for (int k = 0; k < DV; ++k) {
                c2v[k] = C[ve[j][k]];
                sum += c2v[k];
            }
            const double total = chv[j] + sum;
            const bool one = total <= 0.0;
            const bool flip = vok && (one != (((decs >> j) & 1u) != 0u));
            decs ^= flip ? (1u << j) : 0u;
#pragma unroll
            for (int k = 0; k < DV; ++k) {
                const double x = total - c2v[k];  // v2c as decoder.py:120 forms it
                const bool sat = fabs(x) > 14.52;
                if (vok) T[ve[j][k]] = sat ? __builtin_copysign(0.999999, x) : x;
                const bool need = vok && !sat;
                const uint64_t nb = __ballot(need);
                const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(nb >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)nb, 0u));
                if (need) wl[wn + pre] = (uint16_t)ve[j][k];
                wn += (int)__popcll(nb);
                if (flip) atomicXor(&syn[vc[j][k]], 1u);
            }
        }
        PL_GSTAMP(4)
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int w = lane; w < wn; w += 64) {
            const int e = wl[w];
            T[e] = tanh_half_clip(T[e]);
        }
        PL_GSTAMP(5)
        __syncthreads();
        PL_GSTAMP(6)
    }
    uint8_t* o = bits + frame * (int64_t)n;
#pragma unroll
    for (int j = 0; j < VPT; ++j)
        if (vid[j] >= 0) o[vid[j]] = (uint8_t)((decs >> j) & 1u);
    if (iters && tid == 0) iters[frame] = done;
  }
    PL_GSTAMP(7)
    if constexpr (STAMPS) {
        if (lane == 0)
            for (int k = 0; k < 8; ++k) atomicAdd(&stamps[(tid >> 6) * 8 + k], st[k]);
    }
#undef PL_GSTAMP
}

// (DV, EPT, VPT) instances of ldpc_reg_kernel: E <= 256*EPT, n <= 256*VPT
struct RegVariant { int dv, ept, vpt; void* k[4]; };  // BP, MS, BP degree-grouped (1, 2 frames per group)
template <int DV, int EPT, int VPT>
static RegVariant reg_variant() {
    return {DV, EPT, VPT,
            {(void*)ldpc_reg_kernel<0, DV, EPT, VPT>, (void*)ldpc_reg_kernel<1, DV, EPT, VPT>,
             (void*)ldpc_bp_grp_kernel<DV, EPT, VPT>, (void*)ldpc_bp_grp_kernel<DV, EPT, VPT, false, 2>}};
}
static const RegVariant* reg_table(int& count) {
    // E = DV n for a constant variable degree, so (3, 8, 2) and (3, 16, 4) could
    // never be picked ahead of (3, 6, 2) / (3, 12, 4): not built
    static const RegVariant t[] = {reg_variant<3, 6, 2>(), reg_variant<3, 12, 4>(), reg_variant<4, 8, 2>(),
                                   reg_variant<4, 16, 4>()};
    count = (int)(sizeof(t) / sizeof(t[0]));
    return t;
}
size_t ldpc_reg_list_bytes(int variant) {
    int cnt;
    const RegVariant* t = reg_table(cnt);
    return variant > 0 && variant <= cnt ? (size_t)256 * t[variant - 1].vpt * t[variant - 1].dv * 2 : 0;
}
int ldpc_reg_vpt(int variant) {
    int cnt;
    const RegVariant* t = reg_table(cnt);
    return variant > 0 && variant <= cnt ? t[variant - 1].vpt : 0;
}
int ldpc_reg_ept(int variant) {
    int cnt;
    const RegVariant* t = reg_table(cnt);
    return variant > 0 && variant <= cnt ? t[variant - 1].ept : 0;
}
int ldpc_reg_variant(int dv, int E, int n) {
    int cnt;
    const RegVariant* t = reg_table(cnt);
    for (int i = 0; i < cnt; ++i)
        if (t[i].dv == dv && E <= 256 * t[i].ept && n <= 256 * t[i].vpt) return i + 1;
    return 0;
}

// ---- min-sum with compressed check state (codes whose T/C arrays exceed LDS)
// Min-sum check outputs are determined by a few statistics of the check's
// inputs, so instead of T[E] and C[E] (393 KB for n = 8192) the state is
// total[n] (fp64) plus, per check, (min1, min2) and a 32-bit word:
//   bits 0-3 idx1 (first position attaining min1), 4-5 NaN count (saturating
//   at 2), 6-9 position of the first NaN, 10-11 zero count, 12-15 position of
//   the first zero, 16 parity of negatives, 17-31 negative flag per position.
// NaN inputs are left out of (min1, min2).  ms_c2v rebuilds the exact output
// of ms_check for position i from it (same sign product, same min, same
// multiplications), so the decoder stays bit-identical; 8n + 20m bytes of LDS
// (144 KB at n = 8192) hold the whole state, no global workspace.
PL_DEV double ms_c2v(double2 mm, uint32_t meta, int i, double norm) {
    const int idx1 = (int)(meta & 15u), ncnt = (int)((meta >> 4) & 3u), nidx = (int)((meta >> 6) & 15u);
    const int zcnt = (int)((meta >> 10) & 3u), zidx = (int)((meta >> 12) & 15u);
    const uint32_t neg = ((meta >> 16) ^ (meta >> (17 + i))) & 1u;  // parity of negatives over k != i
    const double mn = (i == idx1) ? mm.y : mm.x;
    double sp = neg ? -1.0 : 1.0;
    sp = (zcnt >= 2 || (zcnt == 1 && zidx != i)) ? sp * 0.0 : sp;
    sp = (ncnt >= 2 || (ncnt == 1 && nidx != i)) ? __builtin_nan("") : sp;
    return sp * mn * norm;
}

#ifndef PL_MS_CB
#define PL_MS_CB 2  // regular codes: checks whose loads are issued together in the check pass (-6 %)
#endif
#ifndef PL_MS_VB
#define PL_MS_VB 1  // regular codes: variables whose state loads are issued together (2: +15 %)
#endif
#ifndef PL_MS_VFAST
#define PL_MS_VFAST 1  // variable pass: sign-flip c2v when the check saw no zero / NaN input
#endif
#ifndef PL_MS_SFAST
#define PL_MS_SFAST 1  // check-state update without the zero / NaN bookkeeping when no input needs it (-11.5 %)
#endif
#ifndef PL_MS_PRE
#define PL_MS_PRE 1  // regular codes, |norm| <= 1: check state pre-multiplied by the normalization
#endif

// All DC outputs of a check from its state, equal to ms_c2v position by
// position: with no zero and no NaN input (the usual case) the sign product is
// +-1, so (sp * mn) * norm = +-(mn * norm) -- two multiplies per check instead
// of one per position (rounding is sign-symmetric).
// PRE: the state holds (min1 * norm, min2 * norm) (|norm| <= 1, so no product
// overflows): c2v = sp * (mn * norm), the same value as (sp * mn) * norm for
// sp = +-1 (sign-symmetric rounding), +-0 (signs agree, 0 * inf = NaN on both
// sides) and NaN, and with sp = +-1 just a sign flip -- no multiply per edge.
PL_DEV double ms_c2v_pre(double2 mm, uint32_t meta, int i) {
    const int idx1 = (int)(meta & 15u), ncnt = (int)((meta >> 4) & 3u), nidx = (int)((meta >> 6) & 15u);
    const int zcnt = (int)((meta >> 10) & 3u), zidx = (int)((meta >> 12) & 15u);
    const uint32_t neg = ((meta >> 16) ^ (meta >> (17 + i))) & 1u;
    const double mn = (i == idx1) ? mm.y : mm.x;
    double sp = neg ? -1.0 : 1.0;
    sp = (zcnt >= 2 || (zcnt == 1 && zidx != i)) ? sp * 0.0 : sp;
    sp = (ncnt >= 2 || (ncnt == 1 && nidx != i)) ? __builtin_nan("") : sp;
    return sp * mn;
}

template <int DC, bool PRE = false>
PL_DEV void ms_c2v_all(double2 mm, uint32_t meta, double norm, double* out) {
    if ((meta & 0x0C30u) == 0u) {
        const double a1 = PRE ? mm.x : mm.x * norm, a2 = PRE ? mm.y : mm.y * norm;
        const int idx1 = (int)(meta & 15u);
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const double mag = k == idx1 ? a2 : a1;
            const uint64_t sgn = (uint64_t)(((meta >> 16) ^ (meta >> (17 + k))) & 1u) << 63;
            out[k] = __longlong_as_double((long long)((uint64_t)__double_as_longlong(mag) ^ sgn));
        }
    } else {
#pragma unroll
        for (int k = 0; k < DC; ++k) out[k] = PRE ? ms_c2v_pre(mm, meta, k) : ms_c2v(mm, meta, k, norm);
    }
}

// Check-state update from a check's DC inputs x_k (min-sum statistics, see
// ms_c2v); syndrome of the decisions rides along in `s`.
template <int DC>
PL_DEV void ms_state(const double* x, double2& mm, uint32_t& meta) {
#if PL_MS_SFAST
    // no zero and no NaN input (|x| > 0 is false for both): no NaN / zero
    // bookkeeping, min2 by fmin, the sign bits as the negative flags -- the same
    // (min1, min2, idx1, parity, flags) as the general scan below
    bool ord = true;
#pragma unroll
    for (int k = 0; k < DC; ++k) ord &= fabs(x[k]) > 0.0;
    if (ord) {
        double min1 = __builtin_inf(), min2 = __builtin_inf();
        uint32_t idx1 = 0, negs = 0;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const double a = fabs(x[k]);
            const bool lt = a < min1;
            min2 = lt ? min1 : __builtin_fmin(min2, a);
            min1 = lt ? a : min1;
            idx1 = lt ? (uint32_t)k : idx1;
            negs |= ((uint32_t)((uint64_t)__double_as_longlong(x[k]) >> 63)) << k;
        }
        mm = make_double2(min1, min2);
        meta = idx1 | ((uint32_t)(__popc(negs) & 1) << 16) | (negs << 17);
        return;
    }
#endif
    double min1 = __builtin_inf(), min2 = __builtin_inf();
    uint32_t idx1 = 0, ncnt = 0, nidx = 0, zcnt = 0, zidx = 0, par = 0, negs = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        if (__builtin_isnan(x[k])) {
            if (ncnt == 0) nidx = (uint32_t)k;
            ncnt = ncnt < 2 ? ncnt + 1 : 2;
        } else {
            const double a = fabs(x[k]);
            if (a < min1) { min2 = min1; min1 = a; idx1 = (uint32_t)k; }
            else if (a < min2) min2 = a;
        }
        if (x[k] == 0.0) {
            if (zcnt == 0) zidx = (uint32_t)k;
            zcnt = zcnt < 2 ? zcnt + 1 : 2;
        }
        if (x[k] < 0.0) { par ^= 1u; negs |= 1u << k; }
    }
    mm = make_double2(min1, min2);
    meta = idx1 | (ncnt << 4) | (nidx << 6) | (zcnt << 10) | (zidx << 12) | (par << 16) | (negs << 17);
}

// One workgroup (1024 threads) per frame.  Per iteration: check pass (thread =
// check: v2c_k = total[v_k] - c2v_k(old state) as decoder.py:120 forms it --
// llr itself at iteration 0 -- new state in place, syndrome of the decisions of
// total rides along), vote (early stop, as ldpc_check_kernel), variable pass
// (thread = variable: total = llr + np.sum of the rebuilt c2v in the reference's
// order).  Decisions total <= 0.
// VPT > 0 (n <= 1024 * VPT): each thread keeps the channel LLRs of its
// variables tid + 1024 j in registers instead of re-reading them every iteration.
// DV, DC > 0: a (DV, DC)-regular code (every variable / check degree equal, as
// the BASELINE n = 8192 code): edge offsets are c * DC and v * DV, no row/column
// pointer loads, and the edge loops unroll so their index loads issue together.
template <int VPT, int DV, int DC, bool PRE = false>
__global__ void __launch_bounds__(1024)
ldpc_ms_compact_kernel(LdpcGeom g, LdpcDev dv, const double* __restrict__ llr, int64_t ld,
                       uint8_t* __restrict__ bits, int32_t* __restrict__ iters, int64_t batch) {
    static_assert(!PRE || (PL_MS_CB > 0 && PL_MS_VB > 0 && DV > 0 && DC > 0), "pre-scaled state: batched regular passes only");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t frame = blockIdx.x;
    if (frame >= batch) return;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int n = g.n, m = g.m;
    double* tot = reinterpret_cast<double*>(smem);
    double2* smin = reinterpret_cast<double2*>(smem + (((size_t)8 * n + 15) & ~(size_t)15));
    uint32_t* smeta = reinterpret_cast<uint32_t*>(smin + m);
    uint32_t* vote = reinterpret_cast<uint32_t*>(smem + ((((size_t)8 * n + 15) & ~(size_t)15) + (size_t)20 * m + 15) / 16 * 16);  // [2][16]
    const double* __restrict__ ch = llr + frame * ld;
    const int32_t* __restrict__ rp = dv.row_ptr;
    const int32_t* __restrict__ ci = dv.col_idx;
    double chv[VPT > 0 ? VPT : 1];
    if constexpr (VPT > 0) {
#pragma unroll
        for (int j = 0; j < VPT; ++j) chv[j] = tid + 1024 * j < n ? ch[tid + 1024 * j] : 0.0;
    }
    for (int v = tid; v < n; v += nt) tot[v] = ch[v];
    // Regular codes (the BASELINE n = 8192 one): every adjacency index this
    // thread uses -- the DC columns of its checks tid + 1024 q and the DV
    // (check << 4 | position) entries of its variables -- packed two per
    // register, loaded once instead of from L2 every iteration (n <= 65536).
    constexpr bool RI = (PL_MS_REGIDX & 1) && DV > 0 && DC > 0 && VPT > 0 && (DC % 2) == 0;
    constexpr int MQ = RI ? (VPT * DV + DC - 1) / DC : 1;  // checks per thread (m = n DV / DC)
    uint32_t ccol[RI ? MQ : 1][RI ? DC / 2 : 1];
    constexpr bool RV = RI && (PL_MS_REGIDX & 2);
    uint32_t vcp[RV ? VPT : 1][RV ? (DV + 1) / 2 : 1];
    if constexpr (RI) {
#pragma unroll
        for (int q = 0; q < MQ; ++q) {
            const int c = tid + 1024 * q;
#pragma unroll
            for (int k = 0; k < DC / 2; ++k)
                ccol[q][k] = c < m ? ((uint32_t)ci[c * DC + 2 * k] | ((uint32_t)ci[c * DC + 2 * k + 1] << 16)) : 0u;
        }
#pragma unroll
        for (int j = 0; j < (RV ? VPT : 0); ++j) {
            const int v = tid + 1024 * j;
#pragma unroll
            for (int k = 0; k < (DV + 1) / 2; ++k) {
                const uint32_t lo = v < n ? (uint32_t)dv.var_cp[v * DV + 2 * k] : 0u;
                const uint32_t hi = (v < n && 2 * k + 1 < DV) ? (uint32_t)dv.var_cp[v * DV + 2 * k + 1] : 0u;
                vcp[j][k] = lo | (hi << 16);
            }
        }
    }
    __syncthreads();
    int done = g.max_iter;
    for (int it = 0; it < g.max_iter; ++it) {
        int syn = 0;
        if constexpr (RI) {
            // opaque to the compiler each iteration: the packed indices stay packed
            // (hoisted out of the loop as 24 unpacked LDS addresses they pushed the
            // kernel to 44 B of scratch per lane, whose stores reached HBM: +2.9 GB
            // per launch at n = 8192)
#pragma unroll
            for (int q = 0; q < MQ; ++q)
#pragma unroll
                for (int k = 0; k < DC / 2; ++k) asm volatile("" : "+v"(ccol[q][k]));
        }
        if constexpr (RI && DV > 0 && DV < 8 && PL_MS_CB > 0) {
            // regular code, indices in registers: the loads of PL_MS_CB checks
            // (their old state and DC totals) issue before any of them is
            // reduced (a store to the state would otherwise order every later
            // load behind it); same arithmetic as the loop below
            constexpr int CB = PL_MS_CB < MQ ? (PL_MS_CB > 0 ? PL_MS_CB : 1) : MQ;
#pragma unroll
            for (int q0 = 0; q0 < MQ; q0 += CB) {
                if constexpr (PL_MS_PRIO == 1) ms_prio(q0, MQ);
                double2 om[CB];
                uint32_t ometa[CB];
                double tv[CB][DC];
#pragma unroll
                for (int b = 0; b < CB; ++b) {
                    const int c = tid + 1024 * (q0 + b);
                    const bool ok = q0 + b < MQ && c < m;
                    om[b] = ok ? smin[c] : make_double2(0.0, 0.0);
                    ometa[b] = ok ? smeta[c] : 0u;
#pragma unroll
                    for (int k = 0; k < DC; ++k)
                        tv[b][k] = ok ? tot[(int)((ccol[(q0 + b) < MQ ? q0 + b : 0][k >> 1] >> (16 * (k & 1))) & 0xFFFFu)] : 1.0;
                }
#pragma unroll
                for (int b = 0; b < CB; ++b) {
                    if constexpr (PL_MS_PRIO >= 2) ms_prio(q0 + b, MQ);
                    const int c = tid + 1024 * (q0 + b);
                    if (q0 + b >= MQ || c >= m) continue;
                    double x[DC];
                    int sp = 0;
                    if (it == 0) {
#pragma unroll
                        for (int k = 0; k < DC; ++k) x[k] = tv[b][k];
                    } else {
                        double c2v[DC];
                        ms_c2v_all<DC, PRE>(om[b], ometa[b], g.norm, c2v);
#pragma unroll
                        for (int k = 0; k < DC; ++k) x[k] = tv[b][k] - c2v[k];
                    }
#pragma unroll
                    for (int k = 0; k < DC; ++k) sp ^= (tv[b][k] <= 0.0) ? 1 : 0;
                    syn |= sp;
                    double2 mm;
                    uint32_t meta;
                    ms_state<DC>(x, mm, meta);
                    smin[c] = PRE ? make_double2(mm.x * g.norm, mm.y * g.norm) : mm;
                    smeta[c] = meta;
                }
            }
        } else {
#pragma unroll
        for (int q = 0; q < (RI ? MQ : 1); ++q)
        for (int c = tid + 1024 * q; c < m; c += (RI ? m : nt)) {
            const int e0 = DC > 0 ? c * DC : rp[c], d = DC > 0 ? DC : rp[c + 1] - e0;
            const double2 om = smin[c];
            const uint32_t ometa = smeta[c];
            double min1 = __builtin_inf(), min2 = __builtin_inf();
            uint32_t idx1 = 0, ncnt = 0, nidx = 0, zcnt = 0, zidx = 0, par = 0, negs = 0;
            int s = 0;
            int cidx[DC > 0 ? DC : 1];
            if constexpr (RI) {
#pragma unroll
                for (int k = 0; k < DC; ++k) cidx[k] = (int)((ccol[q][k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
            } else if constexpr (DC > 0) {
#pragma unroll
                for (int k = 0; k < DC; ++k) cidx[k] = ci[e0 + k];
            }
#pragma unroll
            for (int k = 0; k < (DC > 0 ? DC : d); ++k) {
                const double tv = tot[DC > 0 ? cidx[k] : ci[e0 + k]];
                s ^= (tv <= 0.0) ? 1 : 0;
                const double x = it == 0 ? tv : tv - ms_c2v(om, ometa, k, g.norm);
                if (__builtin_isnan(x)) {
                    if (ncnt == 0) nidx = (uint32_t)k;
                    ncnt = ncnt < 2 ? ncnt + 1 : 2;
                } else {
                    const double a = fabs(x);
                    if (a < min1) { min2 = min1; min1 = a; idx1 = (uint32_t)k; }
                    else if (a < min2) min2 = a;
                }
                if (x == 0.0) {
                    if (zcnt == 0) zidx = (uint32_t)k;
                    zcnt = zcnt < 2 ? zcnt + 1 : 2;
                }
                if (x < 0.0) { par ^= 1u; negs |= 1u << k; }
            }
            syn |= s;
            smin[c] = make_double2(min1, min2);
            smeta[c] = idx1 | (ncnt << 4) | (nidx << 6) | (zcnt << 10) | (zidx << 12) | (par << 16) | (negs << 17);
        }
        }
        if (g.early_stop && it > 0) {
            if (!wg_any(syn != 0, vote, it & 1)) { done = it; break; }
        } else {
            __syncthreads();
        }
        if constexpr (RI && DV > 0 && DV < 8 && PL_MS_VB > 0) {
            // regular code: the state loads of PL_MS_VB variables issue together
            constexpr int VB = PL_MS_VB < VPT ? (PL_MS_VB > 0 ? PL_MS_VB : 1) : VPT;
#pragma unroll
            for (int j0 = 0; j0 < VPT; j0 += VB) {
                if constexpr (PL_MS_PRIO) ms_prio(j0, VPT);
                double2 mm[VB][DV];
                uint32_t mt[VB][DV];
                int pos[VB][DV];
#pragma unroll
                for (int b = 0; b < VB; ++b) {
                    const int v = tid + 1024 * (j0 + b);
                    const bool ok = j0 + b < VPT && v < n;
#pragma unroll
                    for (int k = 0; k < DV; ++k) {
                        const int cpk = RV ? (int)((vcp[RV && (j0 + b) < VPT ? j0 + b : 0][k >> 1] >> (16 * (k & 1))) & 0xFFFFu)
                                           : (ok ? dv.var_cp[v * DV + k] : 0);
                        pos[b][k] = cpk & 15;
                        mm[b][k] = ok ? smin[cpk >> 4] : make_double2(0.0, 0.0);
                        mt[b][k] = ok ? smeta[cpk >> 4] : 0u;
                    }
                }
#pragma unroll
                for (int b = 0; b < VB; ++b) {
                    const int v = tid + 1024 * (j0 + b);
                    if (j0 + b >= VPT || v >= n) continue;
                    double sum = 0.0;  // np.sum over DV < 8 terms: sequential
#pragma unroll
                    for (int k = 0; k < DV; ++k) {
                        double c2v;
                        if (PRE && PL_MS_VFAST && (mt[b][k] & 0x0C30u) == 0u) {
                            // no zero / NaN input at the check: +-(scaled min), a sign flip
                            const double mag = pos[b][k] == (int)(mt[b][k] & 15u) ? mm[b][k].y : mm[b][k].x;
                            const uint64_t sgn = (uint64_t)(((mt[b][k] >> 16) ^ (mt[b][k] >> (17 + pos[b][k]))) & 1u) << 63;
                            c2v = __longlong_as_double((long long)((uint64_t)__double_as_longlong(mag) ^ sgn));
                        } else {
                            c2v = PRE ? ms_c2v_pre(mm[b][k], mt[b][k], pos[b][k]) : ms_c2v(mm[b][k], mt[b][k], pos[b][k], g.norm);
                        }
                        sum += c2v;
                    }
                    tot[v] = chv[j0 + b] + sum;
                }
            }
        } else {
#pragma unroll
        for (int jv = 0; jv < (VPT > 0 ? VPT : 1); ++jv) {
          for (int v = tid + 1024 * jv; v < n; v += (VPT > 0 ? n : nt)) {
            const int a0 = DV > 0 ? v * DV : dv.var_ptr[v], d = DV > 0 ? DV : dv.var_ptr[v + 1] - a0;
            const int32_t* __restrict__ cp = dv.var_cp + a0;
            auto c2v = [&](int k) -> double {
                const int c = cp[k] >> 4;
                return ms_c2v(smin[c], smeta[c], cp[k] & 15, g.norm);
            };
            double sum;
            if constexpr (DV > 0 && DV < 8) {  // sequential np.sum, loads issued together
                int cpk[DV];
#pragma unroll
                for (int k = 0; k < DV; ++k)
                    cpk[k] = RV ? (int)((vcp[RV ? jv : 0][k >> 1] >> (16 * (k & 1))) & 0xFFFFu) : cp[k];
                sum = 0.0;
#pragma unroll
                for (int k = 0; k < DV; ++k)
                    sum += ms_c2v(smin[cpk[k] >> 4], smeta[cpk[k] >> 4], cpk[k] & 15, g.norm);
            } else if (d < 8) {  // np.sum: sequential below 8 terms, pairwise (8 accumulators) above
                sum = 0.0;
                for (int k = 0; k < d; ++k) sum += c2v(k);
            } else {
                double r[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) r[j] = c2v(j);
                int k = 8;
                for (; k < d - (d % 8); k += 8) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) r[j] += c2v(k + j);
                }
                sum = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                for (; k < d; ++k) sum += c2v(k);
            }
            tot[v] = (VPT > 0 ? chv[jv] : ch[v]) + sum;
          }
        }
        }
        __syncthreads();
    }
    uint8_t* o = bits + frame * (int64_t)n;
    for (int v = tid; v < n; v += nt) o[v] = tot[v] <= 0.0 ? 1 : 0;
    if (iters && tid == 0) iters[frame] = done;
}

// ---- min-sum on (3,6)-regular codes of n = 1024 VPT (ldpc_ms36_kernel) ------
// The BASELINE n = 8192 code (configs[4]): the passes, state size and
// arithmetic of ldpc_ms_compact_kernel, with the check state stored in the form
// both passes rebuild a check-to-variable message from in a few instructions
// (the compact kernel spent ~46 VALU lane-operations per edge-iteration, 94 %
// of them integer / select / move: VERDICT r05).
//   rec[c] = (A, B), meta[c] (u32): output k of check c is (k == idx1 ? B : A)
//   with its sign bit XORed with flip_k.  meta bits: flip_k at bit (3k + 31) mod
//   32, sel_k = (k == idx1) at bit 3k + 3, 3 idx1 at bits 20-23.
// Every min-sum check fits this form.  No zero and no NaN input: A, B = min1 *
// norm, min2 * norm, idx1 the first position of min1, flip_k = parity of the
// negative inputs XOR input k's sign (sp * mn * norm with sp = +-1 is exactly
// +-(mn * norm)).  Otherwise (ms_c2v's rules, decoder.py:257-287): two or more
// NaN inputs -> every output NaN; one -> every output but the NaN position's
// NaN; no NaN, two or more zeros -> every output +-0; one zero -> every output
// but the zero's +-0: at most one position differs from the rest, so the
// outputs, computed exactly by ms_c2v, are encoded as |A| | |B| | signs.  The
// rebuilt messages are therefore bit-identical to ms_c2v's.
// Odd checks store meta rotated by 16 bits: a variable's edge word (the check's
// rec address | 3 pos; bit 4 of it is the check's parity) is then the rotation
// that brings flip_pos to bit 31 and sel_pos to bit 3 (v_alignbit), and the rec
// address of its magnitude is (word & ~15) | (rotated & 8).
// LDS: tot[n] at 0 (16-bit byte addresses 8v, two per register), rec[m] at 8n,
// meta[m] at 16n, vote words at 18n (n = 8192: 144.1 KB, as the compact kernel).
struct Ms36State {
    double2 st;
    uint32_t meta0;
};

// ldpc_ms36_kernel's check state for a check with a zero or NaN input (rare:
// out of line, so its registers do not weigh on the kernel's common path): the
// exact outputs (ms_c2v), encoded as (A, B, idx1, signs).
#ifndef PL_MS36_NOINLINE
#define PL_MS36_NOINLINE 0
#endif
#if PL_MS36_NOINLINE
__device__ __noinline__
#else
__device__ __forceinline__
#endif
Ms36State ms36_special(double x0, double x1, double x2, double x3, double x4, double x5,
                                               double norm) {
    constexpr int DC = 6;
    const double x[DC] = {x0, x1, x2, x3, x4, x5};
    double2 mm;
    uint32_t gm;
    ms_state<DC>(x, mm, gm);
    uint64_t u[DC];
    uint32_t f = 0;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const uint64_t b = (uint64_t)__double_as_longlong(ms_c2v(mm, gm, k, norm));
        u[k] = b & 0x7FFFFFFFFFFFFFFFull;
        f |= (uint32_t)(b >> 63) << ((3 * k + 31) & 31);
    }
    uint32_t id = 0;
    uint64_t A, B;
    if (u[0] == u[1]) {  // position 0 is not the odd one: the first differing position is
        A = u[0];
#pragma unroll
        for (int k = DC - 1; k >= 2; --k) id = u[k] != A ? (uint32_t)k : id;
        B = u[id];
    } else if (u[2] == u[0]) {
        A = u[0]; id = 1; B = u[1];
    } else {
        A = u[1]; id = 0; B = u[0];
    }
    Ms36State r;
    r.st = make_double2(__longlong_as_double((long long)A), __longlong_as_double((long long)B));
    r.meta0 = f | (8u << (3 * id)) | ((3 * id) << 20);
    return r;
}

#ifndef PL_MS36_CB
#define PL_MS36_CB 2  // checks whose loads issue together
#endif
#ifndef PL_MS36_CREG
#define PL_MS36_CREG 0  // 1: check adjacency in registers (spills), 0: one 16-byte load per check
#endif
#ifndef PL_MS36_CHREG
// 1: the channel LLRs in registers across iterations (125 VGPRs, no spills):
// n = 8192 8.91 -> 8.34 ms per 16 384 frames and 84 -> ~10 GB of memory-side
// traffic per 131 072 (re-read per iteration, the rows 64 KB apart missed L2 about
// half the time); 0: re-read per iteration (profiles/r06_d/ab_chreg.log)
#define PL_MS36_CHREG 1
#endif
template <int VPT>
__global__ void __launch_bounds__(1024)
ldpc_ms36_kernel(LdpcGeom g, LdpcDev dv, const double* __restrict__ llr, int64_t ld,
                 uint8_t* __restrict__ bits, int32_t* __restrict__ iters, int64_t batch) {
    constexpr int N = 1024 * VPT, M = N / 2, MQ = VPT / 2, DC = 6;
    constexpr uint32_t REC = 8u * N, MET = REC + 16u * M, VOTE = MET + 4u * M;
    constexpr uint32_t FMASK = 0x80004924u;  // flip bits of positions 0..5: 31, 2, 5, 8, 11, 14
    static_assert(8 * (N - 1) < 65536 && REC % 32 == 0 && MQ >= 1, "ldpc_ms36_kernel geometry");
    // static LDS: its base address is the constant 0, so the byte addresses need no base added
    __shared__ __attribute__((aligned(16))) unsigned char smem[VOTE + 128];
    const int64_t frame = blockIdx.x;
    if (frame >= batch) return;
    const int tid = threadIdx.x;
    double* tot = reinterpret_cast<double*>(smem);
    double2* rec = reinterpret_cast<double2*>(smem + REC);
    uint32_t* met = reinterpret_cast<uint32_t*>(smem + MET);
    uint32_t* vote = reinterpret_cast<uint32_t*>(smem + VOTE);
    const double* __restrict__ ch = llr + frame * ld;
    const int32_t* __restrict__ ci = dv.col_idx;
    const uint4* __restrict__ vw = reinterpret_cast<const uint4*>(dv.ms_vw);
    const double norm = g.norm;
    double chr[PL_MS36_CHREG ? VPT : 1];
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
        const double c0 = ch[tid + 1024 * j];
        if constexpr (PL_MS36_CHREG) chr[j] = c0;
        tot[tid + 1024 * j] = c0;
    }
    // the tot byte addresses of the DC variables of checks tid + 1024 q, two per
    // word: in registers (PL_MS36_CREG) or read per check from the plan (ms_cw)
    uint32_t ccol[PL_MS36_CREG ? MQ : 1][DC / 2];
    if constexpr (PL_MS36_CREG) {
#pragma unroll
        for (int q = 0; q < MQ; ++q) {
            const int c = tid + 1024 * q;
#pragma unroll
            for (int k = 0; k < DC / 2; ++k)
                ccol[q][k] = (8u * (uint32_t)ci[c * DC + 2 * k]) | ((8u * (uint32_t)ci[c * DC + 2 * k + 1]) << 16);
        }
    }
    const uint4* __restrict__ cw = reinterpret_cast<const uint4*>(dv.ms_vw + 8 * N);
    const uint32_t rot = 16u * (uint32_t)(tid & 1);  // this thread's checks' parity (c = tid + 1024 q)
    __syncthreads();

    // one check: its DC inputs (x = tv - c2v, or tv at iteration 0) -> new state
    auto check_state = [&](const double* x, double2& st, uint32_t& meta0) {
        bool ord = true;
#pragma unroll
        for (int k = 0; k < DC; ++k) ord &= fabs(x[k]) > 0.0;  // false for +-0 and NaN
        if (ord) {
            // no NaN and no zero: (min1, min2) = (min(min1, a), min(min2, max(min1, a)))
            // is the reference scan's (lt ? a : min1, lt ? min1 : min(min2, a)), as
            // three v_min/v_max_f64 (inline: no NaN can reach them, so minnum's
            // quieting canonicalisations are not needed)
            double min1 = fabs(x[0]), min2 = __builtin_inf();
            uint32_t i3 = 0, ng = (uint32_t)__double2hiint(x[0]) & 0x80000000u;
#pragma unroll
            for (int k = 1; k < DC; ++k) {
                const bool lt = fabs(x[k]) < min1;
                double mx;
                asm("v_max_f64 %0, %1, |%2|" : "=v"(mx) : "v"(min1), "v"(x[k]));
                asm("v_min_f64 %0, %1, %2" : "=v"(min2) : "v"(min2), "v"(mx));
                asm("v_min_f64 %0, %1, |%2|" : "=v"(min1) : "v"(min1), "v"(x[k]));
                i3 = lt ? 3u * k : i3;
                ng |= ((uint32_t)__double2hiint(x[k]) >> 31) << (3 * k - 1);
            }
            const uint32_t flips = ng ^ ((__popc(ng) & 1) ? FMASK : 0u);
            meta0 = flips | (8u << i3) | (i3 << 20);
            st = make_double2(min1 * norm, min2 * norm);
        } else {
            const Ms36State r = ms36_special(x[0], x[1], x[2], x[3], x[4], x[5], norm);
            st = r.st;
            meta0 = r.meta0;
        }
    };

    // check pass: checks tid + 1024 q; the loads of two checks issue before either is reduced
    auto check_pass = [&](auto first_tag) -> int {
        constexpr bool FIRST = decltype(first_tag)::value;
        int syn = 0;
        int ct = tid;  // opaque: the check words are re-read every iteration (see the variable pass)
        asm volatile("" : "+v"(ct));
        constexpr int CB = MQ >= PL_MS36_CB ? PL_MS36_CB : 1;
#pragma unroll
        for (int q0 = 0; q0 < MQ; q0 += CB) {
            double tv[CB][DC];
            double2 om[CB];
            uint32_t omt[CB];
#pragma unroll
            for (int b = 0; b < CB; ++b) {
                const int c = tid + 1024 * (q0 + b);
                uint32_t cc[DC / 2];
                if constexpr (PL_MS36_CREG) {
#pragma unroll
                    for (int k = 0; k < DC / 2; ++k) cc[k] = ccol[q0 + b][k];
                } else {
                    const uint4 w4 = cw[ct + 1024 * (q0 + b)];
                    cc[0] = w4.x; cc[1] = w4.y; cc[2] = w4.z;
                }
#pragma unroll
                for (int k = 0; k < DC; ++k) {
                    const uint32_t a = (cc[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                    tv[b][k] = *reinterpret_cast<const double*>(smem + a);
                }
                if (!FIRST) {
                    om[b] = rec[c];
                    omt[b] = met[c];
                }
            }
#pragma unroll
            for (int b = 0; b < CB; ++b) {
                if constexpr (PL_MS_PRIO >= 2) ms_prio(q0 + b, MQ);
                const int c = tid + 1024 * (q0 + b);
                double x[DC];
                if constexpr (FIRST) {
#pragma unroll
                    for (int k = 0; k < DC; ++k) x[k] = tv[b][k];
                } else {
                    const uint32_t m0 = __builtin_amdgcn_alignbit(omt[b], omt[b], rot);
                    const uint32_t i3 = (m0 >> 20) & 15u;
#pragma unroll
                    for (int k = 0; k < DC; ++k) {
                        const double mag = i3 == 3u * k ? om[b].y : om[b].x;
                        const uint32_t s = k == 0 ? m0 : m0 << (32 - 3 * k);
                        const double c2v = __hiloint2double(__double2hiint(mag) ^ (int)(s & 0x80000000u),
                                                            __double2loint(mag));
                        x[k] = tv[b][k] - c2v;
                    }
                }
                int sp = 0;
#pragma unroll
                for (int k = 0; k < DC; ++k) sp ^= (tv[b][k] <= 0.0) ? 1 : 0;
                syn |= sp;
                double2 st;
                uint32_t meta0;
                check_state(x, st, meta0);
                rec[c] = st;
                met[c] = __builtin_amdgcn_alignbit(meta0, meta0, rot);
            }
        }
        return syn;
    };

    int done = g.max_iter;
    for (int it = 0; it < g.max_iter; ++it) {
        // opaque each iteration: the packed addresses stay packed (see ldpc_ms_compact_kernel)
        if constexpr (PL_MS36_CREG) {
#pragma unroll
            for (int q = 0; q < MQ; ++q)
#pragma unroll
                for (int k = 0; k < DC / 2; ++k) asm volatile("" : "+v"(ccol[q][k]));
        }
        const int syn = it == 0 ? check_pass(std::integral_constant<bool, true>())
                                : check_pass(std::integral_constant<bool, false>());
        // the variable pass reads its edge words again every iteration (L2): an
        // opaque index keeps the compiler from holding them in registers across
        // iterations (with the channel values: spilled 40 VGPRs)
        int vt = tid;
        asm volatile("" : "+v"(vt));
        if (g.early_stop && it > 0) {
            if (!wg_any(syn != 0, vote, it & 1)) { done = it; break; }
        } else {
            __syncthreads();
        }
        // variable pass: total = llr + np.sum of the 3 rebuilt messages (sequential)
#pragma unroll
        for (int j = 0; j < VPT; ++j) {
            if constexpr (PL_MS_PRIO) ms_prio(j, VPT);
            const int v = tid + 1024 * j;
            const int vo = vt + 1024 * j;
            const uint4 wa = vw[2 * vo], wb = vw[2 * vo + 1];  // w0 w1 w2 ma0 | ma1 ma2 - -
            const double chv = PL_MS36_CHREG ? chr[PL_MS36_CHREG ? j : 0] : ch[vo];
            const uint32_t w[3] = {wa.x, wa.y, wa.z}, ma[3] = {wa.w, wb.x, wb.y};
            double sum = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint32_t mt = *reinterpret_cast<const uint32_t*>(smem + ma[k]);
                const uint32_t t = __builtin_amdgcn_alignbit(mt, mt, w[k]);
                const double mag = *reinterpret_cast<const double*>(smem + ((w[k] & ~15u) | (t & 8u)));
                sum += __hiloint2double(__double2hiint(mag) ^ (int)(t & 0x80000000u), __double2loint(mag));
            }
            tot[v] = chv + sum;
        }
        __syncthreads();
    }
    uint8_t* o = bits + frame * (int64_t)N;
#pragma unroll
    for (int j = 0; j < VPT; ++j) o[tid + 1024 * j] = tot[tid + 1024 * j] <= 0.0 ? 1 : 0;
    if (iters && tid == 0) iters[frame] = done;
}

// LDS bytes of ldpc_ms36_kernel<n / 1024> (0: no instance for this code)
int ldpc_ms36_lds(int n) {
    return (n == 2048 || n == 4096 || n == 8192) ? 18 * n + 128 : 0;
}

#if PL_DIAG
// Thread-per-check kernel: one workgroup (256 threads) per frame, all state in
// LDS: C[E] (check-to-variable), T[E] (check inputs), tot[n].  Checks are
// degree-sorted by the host so a wavefront's check loops have equal length.
// Per iteration:
//   check pass (thread = check): x_k = tot[v_k] - C[e_k] (v2c as the reference
//     forms it), T = clip(tanh(x/2)) (BP) or x (MS); leave-one-out outputs with
//     the running prefix product shared: p_i = (t_0...t_{i-1}) * t_{i+1} * ...,
//     the same left-to-right order as np.prod over the masked messages; the
//     syndrome of the decisions of tot (the previous iteration's) rides along;
//   vote (__syncthreads_or): all checks satisfied -> stop (iterations = it);
//   variable pass (thread = variable): tot = llr + np.sum(C over its checks).
// Two barriers per iteration (the reference's check / variable / decision /
// syndrome sequence, decoder.py:148-198, with the syndrome of iteration it
// evaluated at the start of iteration it+1 -- same stop point, same bits).
template <int ALGO>
__global__ void __launch_bounds__(256)
ldpc_check_kernel(LdpcGeom g, LdpcDev dv, const double* __restrict__ llr, int64_t ld,
                  uint8_t* __restrict__ bits, int32_t* __restrict__ iters, int64_t batch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int E = g.E, n = g.n, m = g.m;
    double* C = reinterpret_cast<double*>(smem);
    double* T = C + E;
    double* tot = T + E;
    const int32_t* __restrict__ rp = dv.row_ptr;
    const int32_t* __restrict__ ci = dv.col_idx;
    for (int64_t frame = blockIdx.x; frame < batch; frame += gridDim.x) {
        const double* __restrict__ ch = llr + frame * ld;
        for (int e = tid; e < E; e += nt) C[e] = 0.0;
        for (int v = tid; v < n; v += nt) tot[v] = ch[v];  // decoder.py:144-146 (v2c = llr)
        __syncthreads();
        int done = g.max_iter;
        for (int it = 0; it < g.max_iter; ++it) {
            int syn = 0;
            for (int c = tid; c < m; c += nt) {
                const int e0 = rp[c], d = rp[c + 1] - e0;
                int s = 0;
                for (int k = 0; k < d; ++k) {
                    const double tv = tot[ci[e0 + k]];
                    s ^= (tv <= 0.0) ? 1 : 0;
                    const double x = tv - C[e0 + k];
                    T[e0 + k] = (ALGO == 0) ? tanh_half_clip(x) : x;
                }
                syn |= s;
                if (ALGO == 0) {
                    double P = 1.0;  // t_0 * ... * t_{i-1}, sequential
                    for (int i = 0; i < d; ++i) {
                        double p = P;
                        for (int k = i + 1; k < d; ++k) p *= T[e0 + k];
                        p = clip999(p);
                        double o = two_atanh(p);
                        if (isnan(o)) o = 0.0;
                        else if (isinf(o)) o = o > 0.0 ? 20.0 : -20.0;
                        C[e0 + i] = o;
                        P *= T[e0 + i];
                    }
                } else {
                    for (int i = 0; i < d; ++i) {
                        double sp = 1.0, mn = 0.0;
                        bool first = true;
                        for (int k = 0; k < d; ++k) {
                            if (k == i) continue;
                            const double x = T[e0 + k];
                            sp *= np_sign(x);
                            const double ax = fabs(x);
                            if (first) { mn = ax; first = false; }
                            else if (isnan(ax) || isnan(mn)) mn = __builtin_nan("");
                            else if (ax < mn) mn = ax;
                        }
                        C[e0 + i] = sp * mn * g.norm;
                    }
                }
            }
            if (g.early_stop && it > 0) {
                if (!__syncthreads_or(syn)) { done = it; break; }
            } else {
                __syncthreads();
            }
            for (int v = tid; v < n; v += nt) {
                const int a0 = dv.var_ptr[v], d = dv.var_ptr[v + 1] - a0;
                tot[v] = ch[v] + np_sum_gather(C, dv.var_edge + a0, d);
            }
            __syncthreads();
        }
        uint8_t* o = bits + frame * (int64_t)n;
        for (int v = tid; v < n; v += nt) o[v] = tot[v] <= 0.0 ? 1 : 0;
        if (iters && tid == 0) iters[frame] = done;
        __syncthreads();
    }
}

#endif  // PL_DIAG

size_t ldpc_work_bytes_per_frame(const LdpcGeom& g) {
    return g.use_global ? (size_t)(2 * (size_t)g.E) * sizeof(double) : 0;
}

template <int ALGO>
static void* pick(bool global) {
#if PL_DIAG
    const char* m = std::getenv("PL_LDPC_MATH");  // diagnostic: ocml tanh / atanh
    if (ALGO == 0 && m && std::string(m) == "ocml")
        return global ? (void*)ldpc_decode_kernel<ALGO, true, true> : (void*)ldpc_decode_kernel<ALGO, false, true>;
#endif
    return global ? (void*)ldpc_decode_kernel<ALGO, true, false> : (void*)ldpc_decode_kernel<ALGO, false, false>;
}

static void* pick_kernel(const LdpcGeom& g) {
    if (g.ms36) {
        if (g.ms36 == 2) return (void*)ldpc_ms36_kernel<2>;
        if (g.ms36 == 4) return (void*)ldpc_ms36_kernel<4>;
        return (void*)ldpc_ms36_kernel<8>;
    }
    if (g.compact) {
        if (g.n <= 8192 && g.regular && g.maxdv == 3 && g.maxdc == 6) {
            // pre-scaled check state for |normalization| <= 1 (every BASELINE min-sum decode)
            if (PL_MS_PRE && PL_MS_CB > 0 && PL_MS_VB > 0 && fabs(g.norm) <= 1.0)
                return (void*)ldpc_ms_compact_kernel<8, 3, 6, (PL_MS_PRE && PL_MS_CB > 0 && PL_MS_VB > 0)>;
            return (void*)ldpc_ms_compact_kernel<8, 3, 6>;
        }
        return g.n <= 8192 ? (void*)ldpc_ms_compact_kernel<8, 0, 0> : (void*)ldpc_ms_compact_kernel<0, 0, 0>;
    }
    if (g.reg_variant) {
        int cnt;
        return reg_table(cnt)[g.reg_variant - 1].k[g.algo != 0 ? 1 : (g.grp ? (g.fpg == 2 ? 3 : 2) : 0)];
    }
#if PL_DIAG
    if (g.check_kernel) return g.algo == 0 ? (void*)ldpc_check_kernel<0> : (void*)ldpc_check_kernel<1>;
#endif
    return g.algo == 0 ? pick<0>(g.use_global) : pick<1>(g.use_global);
}


#if PL_DIAG
// the degree-grouped BP kernel of a grp plan with per-phase stamps (4 x 8 u64)
hipError_t ldpc_launch_stamped(const LdpcGeom& g, const LdpcDev& d, const double* llr, int64_t ld, uint8_t* bits,
                               int32_t* iters, int64_t batch, unsigned long long* stamps, hipStream_t s) {
    if (!g.grp || g.reg_variant != 1) return hipErrorInvalidValue;
    void* k = (void*)ldpc_bp_grp_kernel<3, 6, 2, true>;
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, g.lds_bytes);
    if (e != hipSuccess) return e;
    LdpcGeom gg = g;
    LdpcDev dd = d;
    void* args[] = {&gg, &dd, (void*)&llr, (void*)&ld, (void*)&bits, (void*)&iters, (void*)&batch, (void*)&stamps};
    return hipLaunchKernel(k, dim3((unsigned)batch), dim3(256), args, g.lds_bytes, s);
}
#endif

// ldpc_ms36_kernel's LDS is static (declared in the kernel); the others' dynamic
static int dyn_lds(const LdpcGeom& g) { return g.ms36 ? 0 : g.lds_bytes; }

hipError_t ldpc_prepare(const LdpcGeom& g) {
    void* k = pick_kernel(g);
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, dyn_lds(g));
}

hipError_t ldpc_launch(const LdpcGeom& g, const LdpcDev& d, const double* llr, int64_t ld,
                       uint8_t* bits, int32_t* iters, int64_t batch, double* work, hipStream_t s) {
    void* k = pick_kernel(g);
    LdpcGeom gg = g;
    LdpcDev dd = d;
    void* args[] = {&gg, &dd, (void*)&llr, (void*)&ld, (void*)&bits, (void*)&iters, (void*)&batch,
                    (void*)&work};
    const int fpg = g.fpg > 1 ? g.fpg : 1;  // frames per workgroup
    return hipLaunchKernel(k, dim3((unsigned)((batch + fpg - 1) / fpg)), dim3(g.threads), args, dyn_lds(g), s);
}

}  // namespace pl
