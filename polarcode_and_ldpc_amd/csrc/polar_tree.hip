// Batched polar SC / SCL decoder for gfx950 (MI355X) -- v4 "tree" kernel:
// lane-per-path like polar_lane.hip, with the whole tree geometry fixed at
// compile time (template on n = log2 N and the list capacity).
//
// Semantics: src/polar/decoder.py of the reference --
//   SCDecoder.decode  :38-71   (min-sum f :121-127, g :129-144, u = 0 if L >= 0)
//   SCLDecoder.decode :225-262 (frozen :264-281, info :283-339, metric :374-406,
//                               stable descending sort, survivors renumbered in
//                               sorted order, final np.argmax = first maximum)
// Every LLR is the same fp64 f/g of the same operands as the reference; the
// path-metric rule is shared with polar_lane.hip (polar_common.hpp).
//
// What differs from polar_lane.hip:
//   * streaming descend: the LLR update of leaf i computes depths dstart..n in
//     chains of up to 3-4 levels per pass over the parent array -- each parent
//     element is loaded once and folded through the whole chain in registers,
//     every level is stored once (for the later g of its right sibling) but the
//     left child (f) never re-reads it.  Halves workspace reads and removes the
//     level-by-level load->store->load latency chain;
//   * tiers by depth, all offsets compile-time constants:
//       depth 0        channel LLRs (global, the caller's rows),
//       depths 1..F-1  recomputed from the channel ("fused top"),
//       depths F..DL-1 per-wave global workspace (L2 / MALL),
//       depths DL..n-1 LDS, depth n (the leaf LLR) a register;
//   * pointer rows are two u64 (5-bit slot per depth) and the leaf-level left
//     partial sum is bit 63 of the beta row, so a clone is 16 bytes;
//   * pruning runs through LDS: lanes publish (m0, m1, rows), read their frame's
//     metrics with 16-byte LDS broadcasts, rank, and scatter survivors to a slot
//     table -- no cross-lane shuffles.
#include "common.hpp"
#include "internal.hpp"
#include "polar_common.hpp"

namespace pl {

namespace {

constexpr int RB = 5;  // bits per slot field of a pointer row (list capacity <= 32)

template <int NL, int LCAP, int F, int DL>
struct TG {
    static constexpr int n = NL, N = 1 << NL, FPW = 64 / LCAP;
    static constexpr int CW = (N / 32) < 1 ? 1 : N / 32;
    static constexpr int BW1 = (n - 5) > 1 ? (n - 5) : 1;  // first single-word beta depth
    static_assert(F >= 1 && F < DL && DL <= n - 1, "tiers: 1 <= F < DL <= n-1");
    static_assert(n <= 12, "pointer rows hold depths < 12");
    static_assert(DL >= BW1, "LDS pool depths must have single-word partial sums");
    // ---- LDS (bytes)
    static constexpr int L_LLR_BYTES = 1024 * ((1 << (n - DL)) - 1);  // pools DL..n-1, [S_d][64] f64
    static constexpr int L_BL = L_LLR_BYTES;                           // single-word beta BW1..n-1, [64] u32
    static constexpr int L_MET = L_BL + (n - BW1) * 256;              // [64] (m0, m1)
    static constexpr int L_ROW = L_MET + 64 * 16;                      // [64] (lrow, brow)
    static constexpr int L_SURV = L_ROW + 64 * 16;                     // [64] u32 survivor entries
    static constexpr int L_FINAL = L_MET;                              // [FPW][CW] u32 (aliases pruning scratch)
    static constexpr int L_END0 = L_SURV + 64 * 4;
    static constexpr int L_END1 = L_FINAL + FPW * CW * 4;
    static constexpr int LDS = (((L_END0 > L_END1) ? L_END0 : L_END1) + 15) & ~15;
    // ---- workspace (bytes per wave)
    static constexpr int64_t W_LLR_BYTES = 1024LL * ((1LL << (n - F)) - (1LL << (n - DL)));  // pools F..DL-1
    static constexpr int64_t W_BL = W_LLR_BYTES;  // multi-word beta depths 1..BW1-1, [W_d][64] u32
    static constexpr int64_t W_BL_BYTES = 8LL * ((1LL << n) - (1LL << (n - BW1 + 1)));
    static constexpr int64_t W_WALK = W_BL + W_BL_BYTES;  // [2][CW][64] u32
    static constexpr int64_t WS = (W_WALK + 2LL * CW * 256 + 255) & ~255LL;

    PL_DEV static int l_llr(int d) { return 1024 * ((1 << (n - DL)) - (1 << (n - d))); }
    PL_DEV static int64_t w_llr(int d) { return 1024LL * ((1LL << (n - F)) - (1LL << (n - d))); }
    PL_DEV static int l_bl(int d) { return L_BL + (d - BW1) * 256; }
    PL_DEV static int64_t w_bl(int d) { return W_BL + 8LL * ((1LL << n) - (1LL << (n - d + 1))); }
};

PL_DEV int field(uint64_t row, int d) { return (int)((row >> (RB * d)) & 31u); }
PL_DEV uint64_t range_mask(int lo, int hi) {  // fields [lo, hi)
    const uint64_t h = (RB * hi >= 64) ? ~0ull : ((1ull << (RB * hi)) - 1ull);
    const uint64_t l = (1ull << (RB * lo)) - 1ull;
    return h & ~l;
}
PL_DEV uint64_t set_range(uint64_t row, uint64_t own, int lo, int hi) {
    const uint64_t m = range_mask(lo, hi);
    return (row & ~m) | (own & m);
}

// Global workspace written by other lanes of this wave: wait for this wave's
// outstanding stores (s_waitcnt vmcnt(0)) before reading it.
PL_DEV void ws_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}
// LDS written by other lanes of this wave: LDS executes a wave's operations in
// order, so only compiler reordering has to be stopped.
PL_DEV void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// One streaming chain of C levels: parent values ld(e) at depth p; level k (1..C)
// is depth p+k; level 1 is g (bits from bits(t), bit j = element t*2^(C-1)+j)
// when GF, all other levels f.  st(k, idx, v) stores level k element idx, except
// the last level when LAST (the leaf LLR, returned).
template <int C, bool GF, bool LAST, class LD, class ST, class BT>
PL_DEV double chain(int nout, const LD& ld, const ST& st, const BT& bits) {
    double lam = 0.0;
    for (int t = 0; t < nout; ++t) {
        double v[1 << C];
#pragma unroll
        for (int k = 0; k < (1 << C); ++k) v[k] = ld(t * (1 << C) + k);
        const uint32_t bw = GF ? bits(t) : 0u;
#pragma unroll
        for (int lv = 1; lv <= C; ++lv) {
            const int m = 1 << (C - lv);
#pragma unroll
            for (int k = 0; k < m; ++k) {
                v[k] = (GF && lv == 1) ? g_op(v[2 * k], v[2 * k + 1], bw >> k) : f_ms(v[2 * k], v[2 * k + 1]);
                if (!(LAST && lv == C)) st(lv, t * m + k, v[k]);
            }
        }
        lam = v[0];
    }
    return lam;
}

}  // namespace

template <int NL, int LCAP, bool SC, int F, int DL, bool STAMPS>
__global__ void __launch_bounds__(64)
polar_tree_kernel(const double* __restrict__ llr, int64_t ld, uint8_t* __restrict__ out,
                  const uint32_t* __restrict__ frozen_dec, const int32_t* __restrict__ info_pos, int64_t batch,
                  int K, int Lsz, unsigned char* __restrict__ workspace, unsigned long long* __restrict__ stamps) {
    using G = TG<NL, LCAP, F, DL>;
    constexpr int n = G::n, N = G::N, FPW = G::FPW, BW1 = G::BW1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int fw = lane / LCAP, slot = lane % LCAP, base = fw * LCAP;
    unsigned char* const ws = workspace + (size_t)blockIdx.x * G::WS;
    uint64_t own = 0;
#pragma unroll
    for (int d = 0; d < 12; ++d) own |= (uint64_t)slot << (RB * d);

    unsigned long long acc[5] = {0, 0, 0, 0, 0};
    unsigned long long tprev = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
#define STAMP(k)                                                   \
    if constexpr (STAMPS) {                                        \
        const unsigned long long tn = __builtin_amdgcn_s_memtime(); \
        acc[k] += tn - tprev;                                      \
        tprev = tn;                                                \
    }

    for (int64_t f0 = (int64_t)blockIdx.x * FPW; f0 < batch; f0 += (int64_t)gridDim.x * FPW) {
        const int64_t frame = f0 + fw;
        const bool live = frame < batch;
        const double* __restrict__ ch = llr + (live ? frame : batch - 1) * ld;
        uint64_t lrow = own, brow = own & ~(1ull << 63);
        double pm = (slot == 0) ? 0.0 : -INFINITY;
        int nact = 1;
        int root_par = 0;

        for (int i = 0; i < N; ++i) {
            // ================================================ LLRs down to leaf i
            const int dstart = (i == 0) ? 1 : n - __builtin_ctz(i);
            double lam;
            {
                int p;
                bool gfirst;
                if (dstart <= DL) ws_sync();  // workspace data of other lanes (pools, multi-word betas)
                if (dstart <= F) {
                    // ---- fused top: depth F from the channel, levels 1..F (g where the
                    // ancestor at that depth is a right child), stored in the workspace
                    double* __restrict__ dst = reinterpret_cast<double*>(ws + G::w_llr(F)) + lane;
                    bool right[F + 1];
                    const uint32_t* bsrc[F + 1];
#pragma unroll
                    for (int d = 1; d <= F; ++d) {
                        right[d] = (i >> (n - d)) & 1;
                        const int bs = base + field(brow, d);
                        bsrc[d] = (d >= BW1) ? reinterpret_cast<const uint32_t*>(smem + G::l_bl(d)) + bs
                                             : reinterpret_cast<const uint32_t*>(ws + G::w_bl(d)) + bs;
                    }
                    constexpr int SF = 1 << (n - F);
#pragma unroll 2
                    for (int t = 0; t < SF; ++t) {
                        double v[1 << F];
                        const double* src = ch + ((size_t)t << F);
#pragma unroll
                        for (int k = 0; k < (1 << F); ++k) v[k] = src[k];
#pragma unroll
                        for (int d = 1; d <= F; ++d) {
                            const int e0 = t << (F - d);  // depth-d element index of v[0]
                            const int m = 1 << (F - d);
                            if (right[d]) {
                                const uint32_t bw = bsrc[d][(d >= BW1) ? 0 : (e0 >> 5) * 64] >> (e0 & 31);
#pragma unroll
                                for (int k = 0; k < m; ++k) v[k] = g_op(v[2 * k], v[2 * k + 1], bw >> k);
                            } else {
#pragma unroll
                                for (int k = 0; k < m; ++k) v[k] = f_ms(v[2 * k], v[2 * k + 1]);
                            }
                        }
                        dst[(size_t)t * 64] = v[0];
                    }
                    lrow = set_range(lrow, own, F, F + 1);
                    p = F;
                    gfirst = false;
                } else {
                    p = dstart - 1;
                    gfirst = true;
                }
                // ---- workspace chains: depths p+1 .. DL-1
                while (p < DL - 1) {
                    const int C = (DL - 1 - p) < 3 ? (DL - 1 - p) : 3;
                    const int ps = base + (gfirst ? field(lrow, p) : slot);  // parent slot
                    const double* P = reinterpret_cast<const double*>(ws + G::w_llr(p)) + ps;
                    const int bsl = base + field(brow, p + 1);
                    const int d1 = p + 1;
                    auto ld = [&](int e) { return P[(size_t)e * 64]; };
                    auto st = [&](int k, int idx, double v) {
                        reinterpret_cast<double*>(ws + G::w_llr(p + k))[(size_t)idx * 64 + lane] = v;
                    };
                    const int nout = 1 << (n - p - C);
                    if (gfirst) {
                        auto bits = [&](int t) -> uint32_t {
                            const int e0 = t << (C - 1);
                            const uint32_t w = (d1 >= BW1)
                                ? reinterpret_cast<const uint32_t*>(smem + G::l_bl(d1))[bsl]
                                : reinterpret_cast<const uint32_t*>(ws + G::w_bl(d1))[(e0 >> 5) * 64 + bsl];
                            return w >> (e0 & 31);
                        };
                        if (C == 3) chain<3, true, false>(nout, ld, st, bits);
                        else if (C == 2) chain<2, true, false>(nout, ld, st, bits);
                        else chain<1, true, false>(nout, ld, st, bits);
                    } else {
                        auto nb = [](int) -> uint32_t { return 0u; };
                        if (C == 3) chain<3, false, false>(nout, ld, st, nb);
                        else if (C == 2) chain<2, false, false>(nout, ld, st, nb);
                        else chain<1, false, false>(nout, ld, st, nb);
                    }
                    lrow = set_range(lrow, own, p + 1, p + 1 + C);
                    p += C;
                    gfirst = false;
                }
                // ---- LDS chains ending at the leaf: depths p+1 .. n-1 stored, depth n returned
                {
                    const int C = n - p;
                    const int ps = base + (gfirst ? field(lrow, p) : slot);
                    const bool pws = (p < DL);
                    const double* P = pws ? reinterpret_cast<const double*>(ws + G::w_llr(p)) + ps
                                          : reinterpret_cast<const double*>(smem + G::l_llr(p)) + ps;
                    const int d1 = p + 1;
                    const int bsl = base + field(brow, d1 < n ? d1 : 0);
                    auto st = [&](int k, int idx, double v) {
                        reinterpret_cast<double*>(smem + G::l_llr(p + k))[idx * 64 + lane] = v;
                    };
                    auto bits = [&](int) -> uint32_t {
                        if (d1 == n) return (uint32_t)(brow >> 63);
                        return reinterpret_cast<const uint32_t*>(smem + G::l_bl(d1))[bsl];
                    };
                    auto nb = [](int) -> uint32_t { return 0u; };
                    if (pws) {
                        auto ld = [&](int e) { return P[(size_t)e * 64]; };
                        constexpr int CC = n - DL + 1;  // p == DL-1
                        lam = gfirst ? chain<CC, true, true>(1, ld, st, bits) : chain<CC, false, true>(1, ld, st, nb);
                    } else {
                        auto ld = [&](int e) { return P[e * 64]; };
                        // from an LDS parent the chain always starts with g (dstart > DL)
                        static_assert(n - DL <= 4, "LDS tier deeper than 4 levels");
                        if (C == 1) lam = chain<1, true, true>(1, ld, st, bits);
                        else if (C == 2 || n - DL < 3) lam = chain<(n - DL < 2 ? n - DL : 2), true, true>(1, ld, st, bits);
                        else if (C == 3 || n - DL < 4) lam = chain<(n - DL < 3 ? n - DL : 3), true, true>(1, ld, st, bits);
                        else lam = chain<4, true, true>(1, ld, st, bits);
                    }
                    if (C > 1) lrow = set_range(lrow, own, p + 1, n);
                }
            }
            STAMP(0);

            // ================================================ decision at leaf i
            const bool frozen = (frozen_dec[i >> 5] >> (i & 31)) & 1u;
            int bit;
            if constexpr (SC) {
                bit = frozen ? 0 : (lam >= 0.0 ? 0 : 1);
                STAMP(1);
            } else if (frozen) {
                double m0, m1;
                path_metrics<false>(pm, lam, m0, m1);
                if (slot < nact) pm = m0;
                bit = 0;
                STAMP(1);
            } else {
                double m0, m1;
                path_metrics<true>(pm, lam, m0, m1);
                STAMP(1);
                double2* metv = reinterpret_cast<double2*>(smem + G::L_MET);
                uint64_t* rowv = reinterpret_cast<uint64_t*>(smem + G::L_ROW);
                uint32_t* surv = reinterpret_cast<uint32_t*>(smem + G::L_SURV);
                metv[lane] = make_double2(m0, m1);
                rowv[2 * lane] = lrow;
                rowv[2 * lane + 1] = brow;
                lds_sync();
                // rank of (slot, b) in the stable descending order of
                // [(m0, q) for active q] + [(m1, q) for active q]
                int r0 = 0, r1 = 0;
                constexpr int QC = LCAP < 8 ? LCAP : 8;
                for (int q0 = 0; q0 < nact; q0 += QC) {
                    double2 mq[QC];
#pragma unroll
                    for (int k = 0; k < QC; ++k) mq[k] = metv[base + q0 + k];
#pragma unroll
                    for (int k = 0; k < QC; ++k) {
                        const int q = q0 + k;
                        const bool v = q < nact;
                        const double a = mq[k].x, b = mq[k].y;
                        r0 += v & ((a > m0) | ((a == m0) & (q < slot)));
                        r0 += v & (b > m0);
                        r1 += v & (a >= m1);
                        r1 += v & ((b > m1) | ((b == m1) & (q < slot)));
                    }
                }
                const int nsurv = (2 * nact < Lsz) ? 2 * nact : Lsz;
                if (slot < nact) {
                    if (r0 < nsurv) surv[base + r0] = (uint32_t)(slot << 1);
                    if (r1 < nsurv) surv[base + r1] = (uint32_t)((slot << 1) | 1);
                }
                lds_sync();
                bit = 0;
                if (slot < nsurv) {
                    const uint32_t e = surv[base + slot];
                    const int par = base + (int)(e >> 1);
                    bit = (int)(e & 1u);
                    const double2 pmv = metv[par];
                    pm = bit ? pmv.y : pmv.x;
                    lrow = rowv[2 * par];
                    brow = rowv[2 * par + 1];
                } else {
                    pm = -INFINITY;
                }
                nact = nsurv;
                lds_sync();  // scratch reads done before the next leaf's writes
                STAMP(2);
            }

            // ================================================ partial-sum walk
            {
                const int to = __builtin_ctz(~(unsigned)i);
                const int steps = to < n ? to : n;
                int dd = n;
                uint32_t cur = (uint32_t)bit;
                int k = 0;
                for (; k < steps && k < 5; ++k) {
                    const uint32_t left = (dd == n)
                        ? (uint32_t)(brow >> 63)
                        : reinterpret_cast<const uint32_t*>(smem + G::l_bl(dd))[base + field(brow, dd)];
                    const uint32_t msk = (1u << (1 << k)) - 1u;
                    cur = spread16((left ^ cur) & msk) | (spread16(cur & msk) << 1);
                    --dd;
                }
                uint32_t* walk = reinterpret_cast<uint32_t*>(ws + G::W_WALK) + lane;  // [2][CW][64]
                if (k == steps) {
                    if (dd == n) {
                        brow = (brow & ~(1ull << 63)) | ((uint64_t)bit << 63);
                    } else if (dd > 0) {
                        reinterpret_cast<uint32_t*>(smem + G::l_bl(dd))[lane] = cur;
                        brow = set_range(brow, own, dd, dd + 1);
                    } else {
                        walk[0] = cur;
                        root_par = 0;
                    }
                } else {
                    int parity = 0;
                    ws_sync();  // multi-word betas of other lanes live in the workspace
                    walk[0] = cur;
                    for (; k < steps; ++k) {
                        const int cwc = 1 << (k - 5);
                        const int ls = base + field(brow, dd);
                        const bool last = (k + 1 == steps);
                        for (int w = 0; w < 2 * cwc; ++w) {
                            const uint32_t cwv = walk[(parity * G::CW + (w >> 1)) * 64];
                            const uint32_t lw = (dd >= BW1)
                                ? reinterpret_cast<const uint32_t*>(smem + G::l_bl(dd))[ls]
                                : reinterpret_cast<const uint32_t*>(ws + G::w_bl(dd))[(w >> 1) * 64 + ls];
                            const int sh = (w & 1) * 16;
                            const uint32_t r = spread16((lw ^ cwv) >> sh) | (spread16(cwv >> sh) << 1);
                            if (last && dd - 1 > 0)
                                reinterpret_cast<uint32_t*>(ws + G::w_bl(dd - 1))[w * 64 + lane] = r;
                            else
                                walk[((parity ^ 1) * G::CW + w) * 64] = r;
                        }
                        parity ^= 1;
                        --dd;
                    }
                    if (dd == 0) root_par = parity;
                    else brow = set_range(brow, own, dd, dd + 1);
                    ws_sync();
                }
            }
            lds_sync();
            STAMP(3);
        }

        // ================================================ best path, output
        int best = 0;
        if constexpr (!SC) {
            double2* metv = reinterpret_cast<double2*>(smem + G::L_MET);
            metv[lane] = make_double2(pm, 0.0);
            lds_sync();
            double bm = metv[base].x;
            for (int q = 1; q < nact; ++q) {
                const double v = metv[base + q].x;
                if (v > bm) { bm = v; best = q; }
            }
            lds_sync();
        }
        uint32_t* X = reinterpret_cast<uint32_t*>(smem + G::L_FINAL) + fw * G::CW;
        const uint32_t* walk = reinterpret_cast<const uint32_t*>(ws + G::W_WALK) + lane;
        if (slot == best)
            for (int w = 0; w < G::CW; ++w) X[w] = polar_word_transform(walk[(root_par * G::CW + w) * 64]);
        lds_sync();
        for (int sw = 1; sw < G::CW; sw <<= 1) {
            for (int w = slot; w < G::CW; w += LCAP)
                if (!(w & sw)) X[w] ^= X[w + sw];
            lds_sync();
        }
        if (live) {
            uint8_t* o = out + frame * (int64_t)K;
            for (int k = slot; k < K; k += LCAP) {
                const int p = info_pos[k];
                o[k] = (uint8_t)((X[p >> 5] >> (p & 31)) & 1u);
            }
        }
        lds_sync();
        STAMP(4);
    }
    if constexpr (STAMPS) {
        if (lane == 0)
            for (int k = 0; k < 5; ++k) atomicAdd(stamps + k, acc[k]);
    }
#undef STAMP
}

// ------------------------------------------------------------------- host
namespace {

struct TreeEntry {
    int n, lcap;
    bool sc;
    int F, DL;
    void* fn;
    void* fn_stamps;
    int lds;
    int64_t ws;
};

template <int NL, int LCAP, bool SC, int F, int DL>
TreeEntry make_entry() {
    using G = TG<NL, LCAP, F, DL>;
    return TreeEntry{NL, LCAP, SC, F, DL, (void*)polar_tree_kernel<NL, LCAP, SC, F, DL, false>,
                     (void*)polar_tree_kernel<NL, LCAP, SC, F, DL, true>, G::LDS, G::WS};
}

const TreeEntry* tree_table(int* count) {
    static const TreeEntry tab[] = {
        make_entry<10, 8, false, 3, 7>(),
    };
    *count = (int)(sizeof(tab) / sizeof(tab[0]));
    return tab;
}

}  // namespace

bool tree_lookup(int n, int lcap, bool sc, TreeInfo* info) {
    int cnt = 0;
    const TreeEntry* t = tree_table(&cnt);
    for (int k = 0; k < cnt; ++k)
        if (t[k].n == n && t[k].lcap == lcap && t[k].sc == sc) {
            info->fn = t[k].fn;
            info->fn_stamps = t[k].fn_stamps;
            info->lds_bytes = t[k].lds;
            info->ws_bytes = t[k].ws;
            info->F = t[k].F;
            info->DL = t[k].DL;
            info->fpw = 64 / lcap;
            return true;
        }
    return false;
}

hipError_t tree_prepare(const TreeInfo& t, int* max_blocks_per_cu) {
    hipError_t e = hipFuncSetAttribute(t.fn, hipFuncAttributeMaxDynamicSharedMemorySize, t.lds_bytes);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute(t.fn_stamps, hipFuncAttributeMaxDynamicSharedMemorySize, t.lds_bytes);
    if (e != hipSuccess) return e;
    int nb = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, t.fn, 64, t.lds_bytes);
    if (e != hipSuccess) return e;
    *max_blocks_per_cu = nb < 1 ? 1 : nb;
    return hipSuccess;
}

hipError_t tree_launch(const TreeInfo& t, const double* llr, int64_t ld, uint8_t* out, const uint32_t* frozen_dec,
                       const int32_t* info_pos, int64_t batch, int K, int Lsz, unsigned char* ws, int grid,
                       unsigned long long* stamps, hipStream_t s) {
    void* args[] = {(void*)&llr, (void*)&ld, (void*)&out, (void*)&frozen_dec, (void*)&info_pos, (void*)&batch,
                    (void*)&K, (void*)&Lsz, (void*)&ws, (void*)&stamps};
    return hipLaunchKernel(stamps ? t.fn_stamps : t.fn, dim3((unsigned)grid), dim3(64), args, t.lds_bytes, s);
}

}  // namespace pl
