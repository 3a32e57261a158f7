// polar_lane.hpp -- the lane-per-path kernel template (see the comment below);
// instantiated in polar_lane.hip (SC, lists 1..8), polar_lane_mid.hip (16, 32)
// and polar_lane_big.hip (64..1024) so the three compile in parallel.
// Batched polar SC / SCL decoder for gfx950 (MI355X) -- lane-per-path kernel.
//
// Semantics: src/polar/decoder.py of the reference --
//   SCDecoder.decode  :38-71   (min-sum f :121-127, g :129-144, u = 0 if L >= 0)
//   SCLDecoder.decode :225-262 (frozen :264-281, info :283-339, metric :374-406,
//                               stable descending sort, survivors renumbered in
//                               sorted order, final np.argmax = first maximum)
// Every LLR is produced by the same fp64 f/g operation on the same operands as
// the reference (f exact, g one rounding), every path metric by the same fp64
// formula; exp/log1p come from ocml instead of NumPy (<= 1-2 ulp apart) and are
// skipped where their value provably cannot change the rounded metric.
//
// Mapping (DESIGN.md §Polar kernel):
//   * one wavefront decodes FPW = 64/LCAP frames; lane l = (frame l/LCAP, list
//     slot l%LCAP): every lane runs ONE decoding path sequentially, so no
//     per-leaf work is replicated across lanes (SC: 64 frames per wave);
//   * all tree arrays are lane-interleaved ([element][64 lanes]): the 64 lanes
//     touch 64 consecutive doubles -> conflict-free LDS / coalesced global;
//   * LLR arrays are pooled per depth with per-path slot pointers: a clone copies
//     a 32-byte pointer row (64-byte above 256 paths; ds_bpermute or LDS), never data.  A path only writes depths
//     whose previous contents are dead for every path of its frame;
//   * depth tiers: the top F depths are recomputed from the channel LLRs, depths
//     [F, Dl) live in a per-wave global workspace (L2/MALL resident), depths
//     [Dl, D] in LDS, and the bottom B = n - D depths are recomputed per leaf in
//     registers from the depth-D node;
//   * partial sums (beta) are bit-packed words pooled like the LLRs (single-word
//     depths in LDS, multi-word depths in the workspace) and built by a walk up
//     the trailing-ones path of each leaf;
//   * pruning: rank of each of the 2*nact candidates in the stable descending
//     order via ds_bpermute within the frame's LCAP lanes;
//   * u_hat is never stored: the root partial sum of the best path is x_hat and
//     u = x_hat * F^{(x)n} (an involution), computed once per frame.
#pragma once
#include "common.hpp"
#include "internal.hpp"
#include "polar_common.hpp"

namespace pl {

namespace {

// Pointer row of a path: field d of a[] = LLR pool slot of depth d, field d of
// b[] = beta slot of depth d (depths 0..kMaxDepth).  FB bits per field: 8 for
// lists up to 256, 16 above.
template <int FB>
struct RowT {
    static constexpr int PW = 64 / FB;                       // fields per word
    static constexpr int NW = (kMaxDepth + 1 + PW - 1) / PW;  // words per kind
    static constexpr uint64_t M = (1ull << FB) - 1ull;
    static constexpr uint64_t REP = FB == 8 ? 0x0101010101010101ull : 0x0001000100010001ull;
    uint64_t a[NW], b[NW];
};
template <class R>
PL_DEV uint64_t row_word(const uint64_t* w, int d) {  // the word holding field d (selects, no dynamic index)
    uint64_t x = w[0];
#pragma unroll
    for (int k = 1; k < R::NW; ++k) x = d >= k * R::PW ? w[k] : x;
    return x;
}
template <class R>
PL_DEV int row_llr(const R& r, int d) {
    return (int)((row_word<R>(r.a, d) >> ((d % R::PW) * (64 / R::PW))) & R::M);
}
template <class R>
PL_DEV int row_beta(const R& r, int d) {
    return (int)((row_word<R>(r.b, d) >> ((d % R::PW) * (64 / R::PW))) & R::M);
}
template <class R>
PL_DEV uint64_t field_range_mask(int a, int b) {  // fields [a, b) of one word
    constexpr int FB = 64 / R::PW;
    a = a < 0 ? 0 : (a > R::PW ? R::PW : a);
    b = b < 0 ? 0 : (b > R::PW ? R::PW : b);
    if (b <= a) return 0ull;
    const uint64_t hi = (b >= R::PW) ? ~0ull : ((1ull << (FB * b)) - 1ull);
    const uint64_t lo = (a <= 0) ? 0ull : ((1ull << (FB * a)) - 1ull);
    return hi & ~lo;
}
template <class R>
PL_DEV void fill_fields(uint64_t* w, int lo, int hi, int val) {  // depths [lo, hi) := val
    const uint64_t rep = (uint64_t)(uint32_t)val * R::REP;
#pragma unroll
    for (int k = 0; k < R::NW; ++k) {
        const uint64_t m = field_range_mask<R>(lo - k * R::PW, hi - k * R::PW);
        w[k] = (w[k] & ~m) | (rep & m);
    }
}
PL_DEV uint32_t bperm(int src_lane, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}
PL_DEV uint64_t bperm64(int src_lane, uint64_t x) {
    const uint64_t lo = bperm(src_lane, (uint32_t)x), hi = bperm(src_lane, (uint32_t)(x >> 32));
    return (hi << 32) | lo;
}
PL_DEV double bperm_d(int src_lane, double v) {
    return __longlong_as_double((long long)bperm64(src_lane, (uint64_t)__double_as_longlong(v)));
}

PL_DEV void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

struct Ctx {
    const LaneGeom* g;
    unsigned char* smem;
    unsigned char* ws;  // this workgroup's global workspace
    int lane, base;     // base = first lane of this frame's group
    int lw;             // lanes per workgroup (the stride of every lane-interleaved array)
};

// element t of lane-slot s at pool depth d (tier by d)
PL_DEV double* pool(const Ctx& c, int d, int t, int s) {
    const LaneGeom& g = *c.g;
    if (d >= g.Dl) return reinterpret_cast<double*>(c.smem + g.lds_pool[d]) + t * c.lw + s;
    return reinterpret_cast<double*>(c.ws + g.ws_pool[d]) + (size_t)t * c.lw + s;
}
// word w of the beta array of lane-slot s at depth d
PL_DEV uint32_t* blw(const Ctx& c, int d, int w, int s) {
    const LaneGeom& g = *c.g;
    if (g.bl_words[d] == 1) return reinterpret_cast<uint32_t*>(c.smem + g.lds_bl[d]) + s;
    return reinterpret_cast<uint32_t*>(c.ws + g.ws_bl[d]) + (size_t)w * c.lw + s;
}
PL_DEV uint32_t* walkbuf(const Ctx& c, int par, int w) {
    return reinterpret_cast<uint32_t*>(c.ws + c.g->ws_walk) + ((size_t)par * c.g->cw + w) * c.lw + c.lane;
}

// child depth cd (size S = 2^(n-cd)) from parent depth cd-1 in lane-slot ps, own
// slot os.  Loads of a chunk of U outputs are issued before any store, so the
// (possibly aliasing, as far as the compiler knows) stores do not serialise them.
template <bool PLDS, bool CLDS>
PL_DEV void level(const Ctx& c, int cd, bool right, int ps, int bs, int os) {
    const LaneGeom& g = *c.g;
    const int S = 1 << (g.n - cd);
    const int lw = c.lw;
    const double* __restrict__ P = PLDS ? reinterpret_cast<const double*>(c.smem + g.lds_pool[cd - 1]) + ps
                                        : reinterpret_cast<const double*>(c.ws + g.ws_pool[cd - 1]) + ps;
    double* __restrict__ C = CLDS ? reinterpret_cast<double*>(c.smem + g.lds_pool[cd]) + os
                                  : reinterpret_cast<double*>(c.ws + g.ws_pool[cd]) + os;
    constexpr int U = 8;
    if (S < U) {
        uint32_t bw = right ? *blw(c, cd, 0, bs) : 0u;
        for (int t = 0; t < S; ++t) {
            const double a = P[2 * t * lw], b = P[(2 * t + 1) * lw];
            C[t * lw] = right ? g_op(a, b, bw >> t) : f_ms(a, b);
        }
        return;
    }
    for (int t0 = 0; t0 < S; t0 += U) {
        double a[U], b[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            a[k] = P[(2 * (t0 + k)) * lw];
            b[k] = P[(2 * (t0 + k) + 1) * lw];
        }
        const uint32_t bw = right ? (*blw(c, cd, t0 >> 5, bs) >> (t0 & 31)) : 0u;
#pragma unroll
        for (int k = 0; k < U; ++k) C[(t0 + k) * lw] = right ? g_op(a[k], b[k], bw >> k) : f_ms(a[k], b[k]);
    }
}

PL_DEV void level_any(const Ctx& c, int cd, bool right, int ps, int bs, int os) {
    const int Dl = c.g->Dl;
    if (cd - 1 >= Dl) level<true, true>(c, cd, right, ps, bs, os);
    else if (cd >= Dl) level<false, true>(c, cd, right, ps, bs, os);
    else level<false, false>(c, cd, right, ps, bs, os);
}

// depth-F node for leaf i straight from the channel (depths 1..F recomputed)
template <int F, class R>
PL_DEV double fused_top(const Ctx& c, int i, const double* __restrict__ ch, const R& row, int os) {
    const LaneGeom& g = *c.g;
    const int n = g.n;
    const int S = 1 << (n - F);
    bool right[F + 1];
    int bsl[F + 1];
#pragma unroll
    for (int d = 1; d <= F; ++d) {
        right[d] = (i >> (n - d)) & 1;
        bsl[d] = c.base + row_beta(row, d);
    }
    double lam = 0.0;
    double* __restrict__ C = (F < n) ? pool(c, F, 0, os) : nullptr;
    for (int t = 0; t < S; ++t) {
        double v[1 << F];
        const double* src = ch + ((size_t)t << F);
#pragma unroll
        for (int k = 0; k < (1 << F); ++k) v[k] = src[k];
#pragma unroll
        for (int d = 1; d <= F; ++d) {
            const int e0 = t << (F - d);  // depth-d element index of v[0]
            const uint32_t bw = right[d] ? (*blw(c, d, e0 >> 5, bsl[d]) >> (e0 & 31)) : 0u;
#pragma unroll
            for (int k = 0; k < (1 << (F - d)); ++k)
                v[k] = right[d] ? g_op(v[2 * k], v[2 * k + 1], bw >> k) : f_ms(v[2 * k], v[2 * k + 1]);
        }
        if (F < n) C[(size_t)t * c.lw] = v[0];
        else lam = v[0];
    }
    return lam;
}

}  // namespace

#ifndef PL_LANE_DYN_LCAP
#define PL_LANE_DYN_LCAP 1024  // list capacities whose frame groups come from the counter
#endif
#ifndef PL_LANE_PRIO_LCAP
// ... and run at issue priorities by dispatch / claim order (up to 32: at 64 and
// 128 +2 / +5 %, equal without; profiles/r04_a/ab_lane_dyn2.log)
#define PL_LANE_PRIO_LCAP 32
#endif
// LCAP <= 64: 64/LCAP frames per wavefront, list exchanges by ds_bpermute.
// LCAP > 64: one frame per workgroup of LCAP lanes (LCAP/64 wavefronts), list
// exchanges through LDS (g.lds_xchg) behind workgroup barriers.
template <int LCAP, bool SC, int F, int B>
__global__ void __launch_bounds__(LCAP > 64 ? LCAP : 64)
polar_lane_kernel(LaneGeom g, const double* __restrict__ llr, int64_t ld, uint8_t* __restrict__ out,
                  const uint32_t* __restrict__ frozen_dec, const int32_t* __restrict__ info_pos, int64_t batch,
                  unsigned char* __restrict__ workspace, const uint32_t* __restrict__ crc_g,
                  uint64_t* __restrict__ nan_masks) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int FPW = LCAP >= 64 ? 1 : 64 / LCAP;
    constexpr int LW = LCAP > 64 ? LCAP : 64;  // lanes per workgroup
    using Row = RowT<(LCAP > 256 ? 16 : 8)>;
    const int lane = threadIdx.x;
    const int fw = lane / LCAP, slot = lane % LCAP;
    const int n = g.n, N = g.N;
    const int D = n - B;
    Ctx c;
    c.g = &g;
    c.smem = smem;
    c.ws = workspace + (size_t)blockIdx.x * g.ws_bytes;
    c.lane = lane;
    c.base = fw * LCAP;
    c.lw = LW;

    // Frame groups as in polar_tree.hip: group blockIdx.x first, every later
    // one from the workspace counter (kSchedBytes before the slices, zeroed by
    // lane_launch); issue priority by dispatch quarter, then by claim order
    // (the SIMD's age-ordered arbitration otherwise makes its youngest
    // wavefront the launch's tail).  NaN mask word of group grp: [grp % grid][grp / grid].
    const int64_t ngrp = (batch + FPW - 1) / FPW;
    constexpr bool DYN = LCAP <= PL_LANE_DYN_LCAP, PRIO = LCAP <= PL_LANE_PRIO_LCAP;
    unsigned int* const sched = reinterpret_cast<unsigned int*>(workspace - kSchedBytes);
    __shared__ unsigned int claim;
    if constexpr (PRIO) set_prio_quarter(blockIdx.x, gridDim.x);
    for (int64_t grp = blockIdx.x; grp < ngrp;) {
        const int64_t f0 = grp * FPW;
        const uint32_t pass = (uint32_t)(grp / gridDim.x), mwave = (uint32_t)(grp % gridDim.x);
        const int64_t frame = f0 + fw;
        const bool live = frame < batch;
        const double* __restrict__ ch = llr + (live ? frame : batch - 1) * ld;
        bool nanf = false;  // a NaN candidate / final metric: redone by polar_nan.hip
        Row row;
#pragma unroll
        for (int k = 0; k < Row::NW; ++k) row.a[k] = row.b[k] = (uint64_t)(uint32_t)slot * Row::REP;
        double pm = (slot == 0) ? 0.0 : -INFINITY;
        int nact = 1;
        int root_par = 0;

        for (int i = 0; i < N; ++i) {
            // -------------------------------------------- LLRs down to leaf i
            const int dstart = (i == 0) ? 1 : n - __builtin_ctz(i);
            double lam;
            if (B == 0) {
                lam = fused_top<F, Row>(c, i, ch, row, lane);  // F == n
            } else {
                int src;
                if (dstart <= D) {
                    int d;
                    if (dstart < c.g->Dl) __syncthreads();  // workspace written by other lanes: vmcnt(0)
                    if (dstart <= F) {
                        fused_top<F, Row>(c, i, ch, row, lane);
                        d = F;
                    } else {
                        level_any(c, dstart, true, c.base + row_llr(row, dstart - 1), c.base + row_beta(row, dstart),
                                  lane);
                        d = dstart;
                    }
                    for (; d < D; ++d) level_any(c, d + 1, false, lane, lane, lane);
                    fill_fields<Row>(row.a, dstart > F ? dstart : F, D + 1, slot);
                    src = lane;
                } else {
                    src = c.base + row_llr(row, D);
                }
                double v[8];
                if (D < c.g->Dl) __syncthreads();  // bottom node in the workspace (tiny LDS budget)
                const double* node = pool(c, D, 0, src);
#pragma unroll
                for (int k = 0; k < (1 << B); ++k) v[k] = node[k * LW];
#pragma unroll
                for (int s = 0; s < B; ++s) {
                    const int d = D + 1 + s;
                    const bool right = (i >> (n - d)) & 1;
                    const uint32_t bw = right ? *blw(c, d, 0, c.base + row_beta(row, d)) : 0u;
#pragma unroll
                    for (int k = 0; k < (1 << (B - 1 - s)); ++k)
                        v[k] = right ? g_op(v[2 * k], v[2 * k + 1], bw >> k) : f_ms(v[2 * k], v[2 * k + 1]);
                }
                lam = v[0];
            }

            // -------------------------------------------- decision at leaf i
            const bool frozen = (frozen_dec[i >> 5] >> (i & 31)) & 1u;
            int bit;
            if constexpr (SC) {
                bit = frozen ? 0 : (lam >= 0.0 ? 0 : 1);
            } else if (frozen) {
                double m0, m1;
                path_metrics<false>(pm, lam, m0, m1);
                if (slot < nact) pm = m0;
                bit = 0;
            } else {
                double m0, m1;
                path_metrics<true>(pm, lam, m0, m1);
                nanf |= (slot < nact) & (__builtin_isnan(m0) | __builtin_isnan(m1));
                const int nsurv = (2 * nact < g.Lsz) ? 2 * nact : g.Lsz;
              if constexpr (LCAP > 64) {
                // the same ranks through LDS: publish (m0, m1) and the pointer
                // row, rank against every active path, publish the ranks, find
                // the candidate this slot receives
                double2* const xm = reinterpret_cast<double2*>(smem + g.lds_xchg);
                uint64_t* const xr = reinterpret_cast<uint64_t*>(xm + LW);
                int2* const xk = reinterpret_cast<int2*>(xr + 2 * Row::NW * LW);
                constexpr int RW = 2 * Row::NW;  // u64 words of a pointer row
                xm[lane] = make_double2(m0, m1);
#pragma unroll
                for (int k = 0; k < Row::NW; ++k) {
                    xr[RW * lane + k] = row.a[k];
                    xr[RW * lane + Row::NW + k] = row.b[k];
                }
                __syncthreads();
                int r0 = 0, r1 = 0;
                for (int q = 0; q < nact; ++q) {
                    const double2 v = xm[q];
                    r0 += (v.x > m0) | ((v.x == m0) & (q < slot));
                    r0 += v.y > m0;
                    r1 += v.x >= m1;
                    r1 += (v.y > m1) | ((v.y == m1) & (q < slot));
                }
                xk[lane] = make_int2(r0, r1);
                __syncthreads();
                int par = 0;
                bit = 0;
                for (int q = 0; q < nact; ++q) {
                    const int2 k = xk[q];
                    if (k.x == slot) { par = q; bit = 0; }
                    if (k.y == slot) { par = q; bit = 1; }
                }
                if (slot < nsurv) {
                    const double2 pv = xm[par];
                    pm = bit ? pv.y : pv.x;
#pragma unroll
                    for (int k = 0; k < Row::NW; ++k) {
                        row.a[k] = xr[RW * par + k];
                        row.b[k] = xr[RW * par + Row::NW + k];
                    }
                } else {
                    pm = -INFINITY;
                }
                nact = nsurv;
                __syncthreads();  // exchange reads done before the next leaf's writes
              } else {
                // rank of (slot, b) in the stable descending order of
                // [(m0, p) for active p] + [(m1, p) for active p]; all lane fetches of
                // a chunk are issued before use (one LDS-crossbar round trip per chunk)
                constexpr int QC = LCAP < 8 ? LCAP : 8;
                int r0 = 0, r1 = 0;
                for (int q0 = 0; q0 < nact; q0 += QC) {
                    double a[QC], b[QC];
#pragma unroll
                    for (int k = 0; k < QC; ++k) {
                        a[k] = bperm_d(c.base + q0 + k, m0);
                        b[k] = bperm_d(c.base + q0 + k, m1);
                    }
#pragma unroll
                    for (int k = 0; k < QC; ++k) {
                        const int q = q0 + k;
                        const bool v = q < nact;
                        r0 += v & ((a[k] > m0) | ((a[k] == m0) & (q < slot)));
                        r0 += v & (b[k] > m0);
                        r1 += v & (a[k] >= m1);
                        r1 += v & ((b[k] > m1) | ((b[k] == m1) & (q < slot)));
                    }
                }
                int par = 0;
                bit = 0;
                for (int q0 = 0; q0 < nact; q0 += QC) {
                    int a[QC], b[QC];
#pragma unroll
                    for (int k = 0; k < QC; ++k) {
                        a[k] = (int)bperm(c.base + q0 + k, (uint32_t)r0);
                        b[k] = (int)bperm(c.base + q0 + k, (uint32_t)r1);
                    }
#pragma unroll
                    for (int k = 0; k < QC; ++k) {
                        const int q = q0 + k;
                        if (q < nact && a[k] == slot) { par = q; bit = 0; }
                        if (q < nact && b[k] == slot) { par = q; bit = 1; }
                    }
                }
                const int sl = c.base + par;
                const double pa = bperm_d(sl, m0), pb = bperm_d(sl, m1);
                Row nr;
#pragma unroll
                for (int k = 0; k < Row::NW; ++k) {
                    nr.a[k] = bperm64(sl, row.a[k]);
                    nr.b[k] = bperm64(sl, row.b[k]);
                }
                if (slot < nsurv) {
                    pm = bit ? pb : pa;
                    row = nr;
                } else {
                    pm = -INFINITY;
                }
                nact = nsurv;
              }
            }

            // -------------------------------------------- partial-sum walk
            {
                const int to = __builtin_ctz(~(unsigned)i);
                const int steps = to < n ? to : n;
                int dd = n;
                uint32_t cur = (uint32_t)bit;
                int k = 0;
                for (; k < steps && k < 5; ++k) {
                    const uint32_t left = *blw(c, dd, 0, c.base + row_beta(row, dd));
                    const uint32_t msk = (1u << (1 << k)) - 1u;
                    cur = spread16((left ^ cur) & msk) | (spread16(cur & msk) << 1);
                    --dd;
                }
                if (k == steps) {
                    if (dd > 0) *blw(c, dd, 0, lane) = cur;
                    else { *walkbuf(c, 0, 0) = cur; root_par = 0; }
                } else {
                    int parity = 0;
                    __syncthreads();  // multi-word beta words of other lanes live in the workspace
                    *walkbuf(c, 0, 0) = cur;
                    for (; k < steps; ++k) {
                        const int cwc = 1 << (k - 5);
                        const int ls = c.base + row_beta(row, dd);
                        const bool last = (k + 1 == steps);
                        for (int w = 0; w < 2 * cwc; ++w) {
                            const uint32_t cwv = *walkbuf(c, parity, w >> 1), lw = *blw(c, dd, w >> 1, ls);
                            const int sh = (w & 1) * 16;
                            const uint32_t r = spread16((lw ^ cwv) >> sh) | (spread16(cwv >> sh) << 1);
                            if (last && dd - 1 > 0) *blw(c, dd - 1, w, lane) = r;
                            else *walkbuf(c, parity ^ 1, w) = r;
                        }
                        parity ^= 1;
                        --dd;
                        __syncthreads();  // left words of other lanes at the next depth
                    }
                    if (dd == 0) root_par = parity;
                }
                if (dd > 0) fill_fields<Row>(row.b, dd, dd + 1, slot);
            }
            if constexpr (LCAP > 64) __syncthreads();  // other wavefronts' beta words
            else wave_fence();  // LDS is in order within a wave; only stop compiler reordering
        }

        // ------------------------------------------------ best path, output
        int best = 0;
        if constexpr (!SC) {
            nanf |= (slot < nact) & __builtin_isnan(pm);
            if constexpr (LCAP > 64) {
                const bool any = __syncthreads_or(nanf);
                if (nan_masks && pass < (uint32_t)kNanMaskPasses && lane == 0)
                    nan_masks[(size_t)mwave * kNanMaskPasses + pass] = any ? 1ull : 0ull;
            } else {
                const uint64_t bal = __ballot(nanf);
                if (nan_masks && pass < (uint32_t)kNanMaskPasses) {
                    constexpr uint64_t GM = LCAP >= 64 ? ~0ull : ((1ull << LCAP) - 1ull);
                    uint64_t fm = 0;
#pragma unroll
                    for (int f = 0; f < FPW; ++f) fm |= (uint64_t)(((bal >> (f * LCAP)) & GM) != 0ull) << f;
                    if (lane == 0) nan_masks[(size_t)mwave * kNanMaskPasses + pass] = fm;
                }
            }
        }
        if constexpr (!SC && LCAP > 64) {
            double* const xp = reinterpret_cast<double*>(smem + g.lds_xchg);
            uint32_t* const xkey = reinterpret_cast<uint32_t*>(xp + LW);
            xp[lane] = pm;
            __syncthreads();  // also: root partial sums in the workspace
            if (crc_g) {
                const uint32_t crc = crc_of_xhat(walkbuf(c, root_par, 0), LW, g.cw, crc_g);
                int rank = 0;
                for (int q = 0; q < nact; ++q) {
                    const double v = xp[q];
                    rank += (v > pm) | ((v == pm) & (q < slot));
                }
                xkey[lane] = slot >= nact ? 0xFFFFFFFFu : (uint32_t)(crc == 0u ? rank : LW + rank);
                __syncthreads();
                uint32_t bk = xkey[0];
                for (int q = 1; q < nact; ++q) {
                    const uint32_t k = xkey[q];
                    if (k < bk) { bk = k; best = q; }
                }
            } else {
                double bm = xp[0];
                for (int q = 1; q < nact; ++q) {
                    const double v = xp[q];
                    if (v > bm) { bm = v; best = q; }
                }
            }
            __syncthreads();  // scratch reads done before X (which may alias nothing) is written
        } else if constexpr (!SC) {
            if (crc_g) {
                // CRC-aided selection, as polar_tree.hip
                __syncthreads();  // root partial sums in the workspace
                const uint32_t crc = crc_of_xhat(walkbuf(c, root_par, 0), LW, g.cw, crc_g);
                int rank = 0;
                for (int q = 0; q < LCAP; ++q) {
                    const double v = bperm_d(c.base + q, pm);
                    if (q < nact) rank += (v > pm) | ((v == pm) & (q < slot));
                }
                const uint32_t key = slot >= nact ? 0xFFFFu : (uint32_t)(crc == 0u ? rank : 64 + rank);
                uint32_t bk = bperm(c.base, key);
                for (int q = 1; q < LCAP; ++q) {
                    const uint32_t k = bperm(c.base + q, key);
                    if (q < nact && k < bk) { bk = k; best = q; }
                }
            } else {
                double bm = bperm_d(c.base, pm);
                for (int q = 1; q < nact; ++q) {
                    const double v = bperm_d(c.base + q, pm);
                    if (v > bm) { bm = v; best = q; }
                }
            }
        }
        uint32_t* X = reinterpret_cast<uint32_t*>(smem + g.lds_final) + fw * g.cw;
        if (slot == best)
            for (int w = 0; w < g.cw; ++w) X[w] = polar_word_transform(*walkbuf(c, root_par, w));
        __syncthreads();
        for (int sw = 1; sw < g.cw; sw <<= 1) {
            for (int w = slot; w < g.cw; w += LCAP)
                if (!(w & sw)) X[w] ^= X[w + sw];
            __syncthreads();
        }
        if (live) {
            uint8_t* o = out + frame * (int64_t)g.K;
            for (int k = slot; k < g.K; k += LCAP) {
                const int p = info_pos[k];
                o[k] = (uint8_t)((X[p >> 5] >> (p & 31)) & 1u);
            }
        }
        if constexpr (!DYN) {
            __syncthreads();
            grp += gridDim.x;
            continue;
        }
        // the next group (a counter read past the end skips the claim)
        unsigned int nx = 0xFFFFFFFFu;
        if (threadIdx.x == 0) {
            const unsigned int seen = __hip_atomic_load(sched, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((int64_t)gridDim.x + (int64_t)seen < ngrp)
                nx = __hip_atomic_fetch_add(sched, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if constexpr (LCAP > 64) claim = nx;
        }
        if constexpr (LCAP > 64) {
            __syncthreads();
            nx = claim;
            __syncthreads();  // read by every wavefront before the next claim overwrites it
        } else {
            nx = (unsigned int)__builtin_amdgcn_readfirstlane((int)nx);
            __syncthreads();
        }
        grp = nx == 0xFFFFFFFFu ? ngrp : (int64_t)gridDim.x + (int64_t)nx;
        if (PRIO && nx != 0xFFFFFFFFu) set_prio_quarter(nx % gridDim.x, gridDim.x);
    }
}


// ---- instance pickers (each translation unit instantiates the ones it calls)
template <int LCAP, bool SC, int F>
static void* lane_pick_b(int B) {
    switch (B) {
        case 0: return (void*)polar_lane_kernel<LCAP, SC, F, 0>;
        case 1: return (void*)polar_lane_kernel<LCAP, SC, F, 1>;
        case 2: return (void*)polar_lane_kernel<LCAP, SC, F, 2>;
        default: return (void*)polar_lane_kernel<LCAP, SC, F, 3>;
    }
}
template <int LCAP, bool SC>
static void* lane_pick_f(int F, int B) {
    switch (F) {
        case 1: return lane_pick_b<LCAP, SC, 1>(B);
        case 2: return lane_pick_b<LCAP, SC, 2>(B);
        case 3: return lane_pick_b<LCAP, SC, 3>(B);
        default: return lane_pick_b<LCAP, SC, 4>(B);
    }
}
// lists of 64+ (one frame per wavefront / workgroup): F = min(3, n) only
template <int LCAP>
static void* lane_pick_big(int F, int B) {
    if (F == 1) return (void*)polar_lane_kernel<LCAP, false, 1, 0>;
    if (F == 2) return (void*)polar_lane_kernel<LCAP, false, 2, 0>;
    return lane_pick_b<LCAP, false, 3>(B);
}

// defined in polar_lane_mid.hip (lists 16, 32) and polar_lane_big.hip (64..1024)
void* lane_pick_mid(int lcap, int F, int B);
void* lane_pick_large(int lcap, int F, int B);


}  // namespace pl
