// Batched polar SC / SCL decoder for gfx950 (MI355X) -- the "tree" kernel:
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
// Design:
//   * one wavefront = 64/LCAP frames, lane = one list path (LCAP lanes/frame);
//   * streaming descend: the LLR update of leaf i is ONE pass over the parent
//     array of depth dstart-1: each parent pair is loaded once, combined (g for
//     the right child at dstart; f/g from the channel for the fused top) and
//     folded down to the leaf through per-depth pending registers (binary-
//     counter order).  Every depth is stored once, as 16-byte pairs, for the
//     later g of its right sibling; no depth is re-read by its left child;
//   * tiers by depth, offsets compile-time constants:
//       depth 0        channel LLRs: read in place from aligned input rows by
//                      the de-duplicated fused top (n <= 10), else staged per
//                      wave transposed [N/2][frames] (one line per load),
//       depths 1..F-1  recomputed from the channel (fused top),
//       depths F..DL-1 per-wave global workspace, [S/2][64 lanes] f64 pairs,
//       depths DL..n-1 LDS, same pair-interleaved layout,
//       depth n        a register (the leaf LLR);
//   * partial sums (beta) of depths n-5..n live in two registers per lane, the
//     multi-word depths 1..n-6 in the workspace behind 5-bit slot pointers, as
//     the LLR pools.  A list clone copies 24 bytes (rows + beta registers);
//   * pruning: strict ranks from fp32 roundings of the metrics (ties and fp32
//     collisions detected and redone exactly), read through DPP lane exchanges
//     at LCAP 8 and from LDS with 16-byte broadcasts otherwise; survivors are
//     scattered to an LDS slot table and take their parent's rows, partial-sum
//     registers and metric from LDS;
//   * rate-0 nodes of 2..8 leaves (all frozen) are decoded at their first leaf:
//     the other leaves' LLRs from the node's stored array (beta = 0), their
//     metric increments added in leaf order;
//   * lane columns are slot-major and, while the list grows, lanes beyond the
//     active paths shadow slot 0 (TG::SHADOW), so inactive paths cost no memory
//     traffic.
#include "common.hpp"
#include "internal.hpp"
#include "polar_common.hpp"

#include <cstdlib>

namespace pl {

namespace {

#ifndef RANK_STRICT_LCAP
#define RANK_STRICT_LCAP 8  // list capacities ranked with strict comparisons
#endif
#ifndef PL_TREE_PRIO
// issue priority (s_setprio) against the SIMD's age-ordered arbitration: 1 =
// a group claimed in the last quarters of its round runs at priority 1..3;
// 2 = also the first group by dispatch quarter (kernel: group loop)
#define PL_TREE_PRIO 2
#endif
#ifndef PL_ORDERED_PRUNE
#define PL_ORDERED_PRUNE 16  // list capacities >= this skip ranking when the full list stays ordered (ordered_prune)
#endif
// SC instances hold 31 KB of LDS per wave (5 waves per CU, ~1 per SIMD), so
// nothing hides a wave's latencies but its own loads in flight: a 256-VGPR
// budget, 32 workspace pairs per g batch and the channel loop unrolled 16
// (against 8 pairs / unroll 2: N=1024 -5 %, default set -4 %, N=256 -7 %,
// N=4096 -12 %, bits identical; profiles/r03_e/ab_sc_knobs*.log)
#ifndef PL_T12_WPE
#define PL_T12_WPE 4  // the N = 4096 L = 8 instance's register budget (waves per SIMD)
#endif
#ifndef PL_SC_WPE
#define PL_SC_WPE 2  // SC instances: waves per SIMD their register budget is built for
#endif
#ifndef PL_SC_U
#define PL_SC_U 32  // SC instances: workspace parent pairs in flight per g-chain batch
#endif
#ifndef PL_LIST_U
#define PL_LIST_U 8  // list instances: workspace parent pairs in flight per g-chain batch
#endif
#ifndef PL_FT_UNR32
#define PL_FT_UNR32 2  // L = 32: the fused top's element-loop unroll
#endif
#ifndef PL_SC_FUNROLL
#define PL_SC_FUNROLL 16  // SC instances: unroll of the depth-1 loop over the channel
#endif

// Lane exchanges inside the 8-lane group of a frame (LCAP = 8) without LDS:
// quad_perm xor 1/2/3 and row_half_mirror (lane i <- 7 - i = i ^ 7 in each
// half-row); xor 4/5/6 are a quad_perm of the mirrored value.
template <int CTRL>
PL_DEV int dpp_i(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, false); }
constexpr int DPP_X1 = 0xB1, DPP_X2 = 0x4E, DPP_X3 = 0x1B, DPP_MIRROR8 = 0x141;
// fn(x of lane slot ^ k) for k = 1..7 of the lane's 8-lane group
template <class Fn>
PL_DEV void group8_each(int x, Fn fn) {
    const int m = dpp_i<DPP_MIRROR8>(x);
    fn(dpp_i<DPP_X1>(x));
    fn(dpp_i<DPP_X2>(x));
    fn(dpp_i<DPP_X3>(x));
    fn(dpp_i<DPP_X3>(m));
    fn(dpp_i<DPP_X2>(m));
    fn(dpp_i<DPP_X1>(m));
    fn(m);
}

// ---- LCAP = 32: survivors by a bitonic sort of the frame's 64 candidate keys
// across its 32 lanes (two keys per lane), lane exchanges by DPP / ds_swizzle
// instead of LDS broadcasts.  Element e of lane s holds sorted position
// 32 e + s; the network sorts descending, so lane s ends with position s --
// survivor s -- in element 0 (model: 64-key bitonic network, 21 stages).
// x of lane s ^ STRIDE (within the lane's 32-lane group)
template <int STRIDE>
PL_DEV int bit_partner(int x) {
    if constexpr (STRIDE == 1) return dpp_i<DPP_X1>(x);
    else if constexpr (STRIDE == 2) return dpp_i<DPP_X2>(x);
    else if constexpr (STRIDE == 4) return dpp_i<DPP_X3>(dpp_i<DPP_MIRROR8>(x));  // (s ^ 7) ^ 3
    else if constexpr (STRIDE == 8) return dpp_i<0x128>(x);                       // row_ror:8
    else return __builtin_amdgcn_ds_swizzle(x, 0x401F);                           // xor 16 (32-lane groups)
}
constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }
// One compare-exchange stage.  Element e of lane s is position p = 32 e + s;
// it keeps the smaller key when it is the upper element of a descending block
// or the lower one of an ascending block (blocks of SIZE descend where p & SIZE
// is 0; every block of the final merge descends): the same select for both
// elements except in the SIZE = 32 merge, where element 1's block ascends.
template <int SIZE, int STRIDE>
PL_DEV void bit_stage(int& k0, int& k1, int s) {
    if constexpr (STRIDE == 32) {
        const int a = k0, b = k1;
        k0 = a > b ? a : b;
        k1 = a > b ? b : a;
    } else {
        const int p0 = bit_partner<STRIDE>(k0), p1 = bit_partner<STRIDE>(k1);
        const int lo0 = min(k0, p0), hi0 = max(k0, p0), lo1 = min(k1, p1), hi1 = max(k1, p1);
        const bool upper = (s & STRIDE) != 0;
        if constexpr (SIZE == 64) {
            k0 = upper ? lo0 : hi0;
            k1 = upper ? lo1 : hi1;
        } else if constexpr (SIZE == 32) {
            k0 = upper ? lo0 : hi0;
            k1 = upper ? hi1 : lo1;
        } else {
            const bool tmin = (((s >> ilog2(STRIDE)) ^ (s >> ilog2(SIZE))) & 1) == 0;
            k0 = tmin ? lo0 : hi0;
            k1 = tmin ? lo1 : hi1;
        }
    }
}
template <int SIZE, int STRIDE>
PL_DEV void bit_merge(int& k0, int& k1, int s) {
    bit_stage<SIZE, STRIDE>(k0, k1, s);
    if constexpr (STRIDE > 1) bit_merge<SIZE, STRIDE / 2>(k0, k1, s);
}
template <int SIZE = 2>
PL_DEV void bit_sort64_desc(int& k0, int& k1, int s) {
    bit_merge<SIZE, SIZE / 2>(k0, k1, s);
    if constexpr (SIZE < 64) bit_sort64_desc<SIZE * 2>(k0, k1, s);
}
// Sort key of candidate list index cidx (0..63, the reference's candidate order
// b * nact + q up to a monotone relabelling): the fp32 rounding of its metric as
// an order-preserving int (-0 taken as +0), low 6 bits replaced by 63 - cidx, so
// that equal truncated metrics order by ascending list index (the stable sort).
PL_DEV int bit_key(double m, int cidx) {
    const int b = __float_as_int((float)m + 0.0f);
    const int s = b ^ ((b >> 31) & 0x7FFFFFFF);
    return (s & ~63) | (63 - cidx);
}

// ---- pruning without reordering (the list is full and ordered) ------------
// True (wave-uniform) when in every frame of the wave the best child of each
// path (max(m0, m1)) is strictly below the best child of the path in the slot
// before it and the last path's best child is strictly above every path's
// other child (all finite): then the reference's stable descending sort of the
// 2L candidates starts with exactly the L best children in slot order, so
// survivor s is path s with its better bit -- no ranks, no exchange.  Lanes of
// a frame are lanes LCAP*f .. LCAP*f + LCAP - 1; every lane active.
template <int LCAP>
PL_DEV bool ordered_prune(double m0, double m1, int slot, int lane) {
    const double A = m1 > m0 ? m1 : m0, B = m1 > m0 ? m0 : m1;
    bool ok = A > B && !__builtin_isnan(m0) && !__builtin_isnan(m1);
    // the previous slot's best child
    const long long ab = __double_as_longlong(A);
    int plo, phi;
    if constexpr (LCAP <= 16) {  // groups inside 16-lane rows: row_shr:1
        plo = __builtin_amdgcn_update_dpp(0, (int)ab, 0x111, 0xF, 0xF, false);
        phi = __builtin_amdgcn_update_dpp(0, (int)(ab >> 32), 0x111, 0xF, 0xF, false);
    } else {
        plo = __builtin_amdgcn_ds_bpermute((lane - 1) << 2, (int)ab);
        phi = __builtin_amdgcn_ds_bpermute((lane - 1) << 2, (int)(ab >> 32));
    }
    const double Ap = __longlong_as_double((long long)(((unsigned long long)(unsigned)phi << 32) | (unsigned)plo));
    // max over the frame of the other children (butterfly)
    double mb = B;
#define PL_OP_MAXB(S)                                                                                   \
    if constexpr (LCAP > S) {                                                                           \
        const long long x = __double_as_longlong(mb);                                                   \
        const int lo = bit_partner<S>((int)x), hi = bit_partner<S>((int)(x >> 32));                     \
        const double o = __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo)); \
        mb = o > mb ? o : mb;                                                                           \
    }
    PL_OP_MAXB(1)
    PL_OP_MAXB(2)
    PL_OP_MAXB(4)
    PL_OP_MAXB(8)
    PL_OP_MAXB(16)
#undef PL_OP_MAXB
    ok = ok && (slot == 0 || Ap > A) && (slot + 1 < LCAP || A > mb);
    return __ballot(!ok) == 0;
}

constexpr int RB = 5;  // bits per slot field of a pointer row (list capacity <= 32)

template <int NL, int LCAP_, int F_, int DL_, int DS_ = 0>
struct TG {
    static constexpr int n = NL, N = 1 << NL, LCAP = LCAP_, FPW = 64 / LCAP_, F = F_, DL = DL_;
    static constexpr int DS = DS_;  // dead-store record / replay instance (diagnostic, kernel comment)
    // path-metric term form (metric_t): fused, or lean above PL_METRIC_FUSED_NMAX.  (A
    // table form -- 20 fp64 operations and a 16-byte gather from a 770-row
    // table instead of ~45 -- measured 35 % slower at N = 1024 L = 8: the gather
    // waits on a saturated memory system, profiles/r06_b/ab_tab.log)
    static constexpr int MF = NL <= PL_METRIC_FUSED_NMAX ? 1 : 0;
    static constexpr int CW = N / 32;
    static constexpr int NB = n - 6;          // multi-word beta depths 1..NB (workspace)
    static constexpr bool STAGE = LCAP > 1;   // stage channel rows shared by a frame's lanes
    static_assert(n >= 7 && n <= 12, "tree kernel: 7 <= n <= 12");
    static_assert(F >= 1 && F < DL && DL <= n - 1, "tiers: 1 <= F < DL <= n-1");
    static_assert(F <= 4, "fused top at most 4 levels");
    // ---- LDS (bytes)
    static constexpr int L_LLR_BYTES = 1024 * ((1 << (n - DL)) - 1);  // pools DL..n-1
    static constexpr int GS = LCAP * 16 + 16;                          // padded group stride (16-B entries)
    static constexpr int L_MET = L_LLR_BYTES;                          // [FPW][GS]: (m0, m1)
    static constexpr int L_ROW = L_MET + FPW * GS;                     // [FPW][GS]: (lrow, brow)
    static constexpr int L_BR = L_ROW + FPW * GS;                      // [64] u64: beta registers
    static constexpr int L_SURV = L_BR + 64 * 8;                       // [64] u32: survivor entries
    // [FPW][CW] u32: the final transform's words, written once the best path
    // is known, alias the LDS pools and the pruning scratch (all dead by then).
    // Before round 5 they sat after the pools, which put n = 12 L = 8 at 11 KB
    // (14 waves per CU instead of 16) and SC N = 2048 / 4096 at 47 / 63 KB
    static constexpr int L_FINAL = 0;
    static constexpr int L_END0 = L_SURV + 64 * 4;
    static constexpr int L_END1 = L_FINAL + FPW * CW * 4;
    static constexpr int LDS = (((L_END0 > L_END1) ? L_END0 : L_END1) + 15) & ~15;
    static_assert(!STAGE || 2 * FPW * GS >= 1024, "metric/row scratch holds a 1 KB staging chunk");
    // ---- workspace (bytes per wave)
    // staged channel depth 0 and its path-independent f-only depths 1..NS
    // (the left-most nodes): depth d as [S_d/2][FPW] f64 pairs at st_off(d)
    static constexpr int NS = STAGE ? (F - 1 < 3 ? F - 1 : 3) : 0;
    static constexpr int64_t st_off(int d) {  // sum_{k<d} N/2^k values
        return (int64_t)FPW * 8 * (2 * N - (2 * N >> d));
    }
    static constexpr int64_t W_CH_BYTES = STAGE ? st_off(NS + 1) : 0;
    static constexpr int64_t W_LLR = W_CH_BYTES;                               // pools F..DL-1
    static constexpr int64_t W_LLR_BYTES = 1024LL * ((1LL << (n - F)) - (1LL << (n - DL)));
    static constexpr int64_t W_BL = W_LLR + W_LLR_BYTES;  // beta depths 1..NB: [W_d][64] u32
    static constexpr int64_t W_BL_BYTES = 8LL * ((1LL << n) - (1LL << (n - NB)));
    static constexpr int64_t W_WALK = W_BL + W_BL_BYTES;  // [2][CW][64] u32
    static constexpr int64_t WS = (W_WALK + 2LL * CW * 256 + 255) & ~255LL;

    // byte offset of the pool of depth d (LDS if d >= DL, else workspace);
    // pair j of lane-slot s sits at offset + (j * 64 + s) * 16
    static constexpr int64_t llr_off(int d) {
        return d >= DL ? (int64_t)1024 * ((1 << (n - DL)) - (1 << (n - d)))
                       : W_LLR + 1024LL * ((1LL << (n - F)) - (1LL << (n - d)));
    }
    // byte offset of the beta pool of multi-word depth d (1..NB); word w of slot s at + (w*64 + s)*4
    static constexpr int64_t bl_off(int d) { return W_BL + 8LL * ((1LL << n) - (1LL << (n - d + 1))); }
    // Shadow lanes + slot-major lane columns (kernel comment at `plane`): on for
    // every instance but LCAP = 16, where they measured slower (7.3 against
    // 6.8 ms at N = 1024); there inactive slots keep their own state and planes
    // and the columns are frame-major, as before.
    static constexpr bool SHADOW = LCAP != 16;
    // Streaming (nt) accesses for the traffic with the longest reuse distance,
    // so it does not evict the deeper pools' lines from L2 (round 5; A/B on one
    // box, bits identical, profiles/r05_b/ab_nt*.log, ab_ntr*.log):
    //   NTD: the g reads of the NTD shallowest workspace pool depths (F ..
    //        F+NTD-1) as nt loads -- 2 at n = 10, 3 at n >= 11 (4 at n = 12 and
    //        3 at n = 10 measured slower), none at L = 16 (slower) nor SC;
    //   NT_ST: at n <= 10 also those depths' stores (at n >= 11 slower);
    //   PL_NT_CH: the fused top's chunk prefetch (channel rows / staged nodes).
    // N = 4096 L = 8 61.1 -> 57.8 ms, N = 2048 7.27 -> 6.85, N = 1024 L = 8
    // 5.53 -> 5.40, L = 32 18.85 -> 17.95.  (Round 2 had found nt stores
    // slower, before the dynamic group counter and the issue priorities.)
#ifndef PL_NT_DEPTHS
#define PL_NT_DEPTHS -1  // -1: the per-instance rule
#endif
#ifndef PL_NT_SC
#define PL_NT_SC 0
#endif
    static constexpr int NTD = PL_NT_DEPTHS >= 0 ? PL_NT_DEPTHS
                               : (LCAP == 1 ? PL_NT_SC : (LCAP == 16 ? 0 : (n >= 11 ? 3 : 2)));
#ifndef PL_NT_ST
#define PL_NT_ST -1  // -1: the per-instance rule
#endif
#ifndef PL_NT_CH
#define PL_NT_CH 1
#endif
    static constexpr bool NT_ST = PL_NT_ST >= 0 ? PL_NT_ST != 0 : n <= 10;
#ifndef PL_NT_ST_DEPTHS
#define PL_NT_ST_DEPTHS -1  // -1: NT_ST ? NTD : 0
#endif
    // the stores of the NTS shallowest workspace depths as nt stores
    static constexpr int NTS = PL_NT_ST_DEPTHS >= 0 ? PL_NT_ST_DEPTHS : (NT_ST ? NTD : 0);
    // fused top from staged depth D0 with de-duplicated chunk reads: a chunk is
    // LCAP pairs of every frame, W / 2 = 2^(F-D0-1) of them per depth-F
    // element, and the depth-F array (2^(n-F) elements) must fill at least one
    // chunk (round 3 measured it slower at N = 2048 / 4096, L = 8; with round
    // 5's 16 waves per CU and issue priorities at n = 12 it is faster there)
    static constexpr bool dedup(int D0) {
        return STAGE && LCAP >= (1 << (F - D0)) / 2 && (1 << (n - F)) * ((1 << (F - D0)) / 2) >= LCAP;
    }
    static PL_DEV int pl(int s, int f) { return SHADOW ? s * FPW + f : f * LCAP + s; }
};

PL_DEV int field(uint64_t row, int d) { return (int)((row >> (RB * d)) & 31u); }
PL_DEV uint64_t set_field(uint64_t row, int d, int v) {
    return (row & ~(31ull << (RB * d))) | ((uint64_t)v << (RB * d));
}
PL_DEV uint64_t set_range(uint64_t row, uint64_t own, int lo, int hi) {  // fields [lo, hi) := own
    const uint64_t h = (RB * hi >= 64) ? ~0ull : ((1ull << (RB * hi)) - 1ull);
    const uint64_t m = h & ~((1ull << (RB * lo)) - 1ull);
    return (row & ~m) | (own & m);
}

// Partial sums of depths n-5..n in registers: bb holds depth n-k (k = 0..4) at
// bit offset 2^k - 1 (width 2^k); bw5 is the 32-bit word of depth n-5.
template <int n>
PL_DEV uint32_t beta_get(int d, uint32_t bb, uint32_t bw5) {
    const int k = n - d;
    if (k == 5) return bw5;
    return (bb >> ((1 << k) - 1)) & ((1u << (1 << k)) - 1u);
}
template <int n>
PL_DEV void beta_set(int d, uint32_t v, uint32_t& bb, uint32_t& bw5) {
    const int k = n - d;
    if (k == 5) { bw5 = v; return; }
    const uint32_t m = ((1u << (1 << k)) - 1u) << ((1 << k) - 1);
    bb = (bb & ~m) | ((v << ((1 << k) - 1)) & m);
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

template <class G>
struct Fold {
    double pend[G::n + 1];  // pending even element per depth
    double lam;             // the leaf LLR (depth n)
    uint32_t skip;          // G::DS == 2 only: bit d = do not store depth d (dead-store bound)
};

// Element idx of depth D has been computed: if even, hold it; if odd, store the
// (even, odd) pair to this lane's slot and continue one depth down with f.
// Compile-time recursion keeps every pending value in a register.
template <class G, int D>
PL_DEV void fold(Fold<G>& st, double v, int idx, unsigned char* smem, unsigned char* ws, int plane) {
    if constexpr (D == G::n) {
        st.lam = v;
    } else {
        if (idx & 1) {
            double2* dst = reinterpret_cast<double2*>((D >= G::DL ? smem : ws) + G::llr_off(D));
            if (G::DS != 2 || !((st.skip >> D) & 1u)) {
                if constexpr (D < G::F + G::NTS && D < G::DL) {
                    double2* a = dst + (idx >> 1) * 64 + plane;
                    __builtin_nontemporal_store(st.pend[D], &a->x);
                    __builtin_nontemporal_store(v, &a->y);
                } else {
                    dst[(idx >> 1) * 64 + plane] = make_double2(st.pend[D], v);
                }
            }
            fold<G, D + 1>(st, f_ms(st.pend[D], v), idx >> 1, smem, ws, plane);
        } else {
            st.pend[D] = v;
        }
    }
}

// Right child at depth Q = P+1: g over the parent pairs (slot ps) with the left
// sibling's partial sums, then the f-chain down to the leaf.
template <class G, int P>
PL_DEV double descend_g(unsigned char* smem, unsigned char* ws, int plane, int ps, int bs, uint32_t bb,
                        uint32_t bw5, uint32_t skip) {
    constexpr int n = G::n, Q = P + 1, SQ = 1 << (n - Q);
    Fold<G> st;
    st.lam = 0.0;
    if constexpr (G::DS == 2) st.skip = skip;
    const double2* src = reinterpret_cast<const double2*>((P >= G::DL ? smem : ws) + G::llr_off(P)) + ps;
    uint32_t w = 0;
    if constexpr (Q > G::NB) w = beta_get<n>(Q, bb, bw5);
    const uint32_t* bsrc = reinterpret_cast<const uint32_t*>(ws + G::bl_off(Q <= G::NB ? Q : 1)) + bs;
    constexpr int UM = G::LCAP == 1 ? PL_SC_U : PL_LIST_U;
    constexpr int U = SQ < UM ? SQ : UM;  // parent pairs in flight
#pragma unroll 1
    for (int t0 = 0; t0 < SQ; t0 += U) {
        // the partial-sum word first: waiting for it then leaves the pair
        // loads in flight (each pair is waited for at its own fold)
        if constexpr (Q <= G::NB) {
            if ((t0 & 31) == 0) w = bsrc[(t0 >> 5) * 64];
        }
        double2 pr[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            // the shallowest workspace depths' g reads as streaming loads (TG::NTD)
            if constexpr (G::NTD > 0 && P < G::F + G::NTD && P < G::DL) {
                const double2* a = src + (t0 + k) * 64;
                pr[k] = make_double2(__builtin_nontemporal_load(&a->x), __builtin_nontemporal_load(&a->y));
            } else {
                pr[k] = src[(t0 + k) * 64];
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
            fold<G, Q>(st, g_op(pr[k].x, pr[k].y, w >> ((t0 + k) & 31)), t0 + k, smem, ws, plane);
    }
    return st.lam;
}

// Fused top from staged depth D0 (0 = channel; 1, 2 = the path-independent
// left-most f-only nodes, valid when the ancestors at depths 1..D0 are left
// children): depth-F elements from 2^(F-D0) values each (level d is g where the
// depth-d ancestor of leaf i is a right child), then the f-chain to the leaf.
template <class G, int D0>
PL_DEV double fused_loop(unsigned char* smem, unsigned char* ws, int lane, int fw, int plane, const double* ch,
                         const double2* raw, const bool* right, const uint32_t* const* bsrc, uint32_t* bw,
                         uint32_t skip) {
    constexpr int n = G::n, F = G::F, SF = 1 << (n - F), W = 1 << (F - D0);
    Fold<G> st;
    st.lam = 0.0;
    if constexpr (G::DS == 2) st.skip = skip;
    if constexpr (G::dedup(D0)) {
        // De-duplicated staged reads: the staged depth is [S/2][FPW] pairs, so
        // a 1 KB chunk (LCAP pairs of every frame of the wave) is contiguous.
        // Each lane fetches one distinct 16-byte pair of it (instead of the
        // frame's LCAP lanes all fetching the same pairs), parks the chunk in
        // the metric/row scratch (idle during a descend) and every lane reads
        // its frame's pairs back as LDS broadcasts.  Next chunk prefetched.
        constexpr int CH = 1;  // pairs per lane per chunk (CH = 2: 7.5 ms against 7.06)
        constexpr int PPI = W / 2, IPC = CH * G::LCAP / PPI, NCH = SF / IPC;
        // depth 0 straight from the input rows when they are 16-byte aligned
        // (`raw`: pair lane / FPW of frame lane % FPW; chunk c at + c * LCAP):
        // the same 8 lines per chunk as the staged copy, which is then not stored
        const bool from_raw = D0 == 0 && raw != nullptr;
        const double2* src = from_raw ? raw : reinterpret_cast<const double2*>(ws + G::st_off(D0)) + lane;
        const int cstr = from_raw ? G::LCAP : 64;
        double2* stg = reinterpret_cast<double2*>(smem + G::L_MET);
        double2 nxt[CH];
#pragma unroll
        for (int h = 0; h < CH; ++h) nxt[h] = src[h * cstr];
#pragma unroll 1
        for (int c = 0; c < NCH; ++c) {
            lds_sync();  // the previous chunk's reads are issued before the overwrite
#pragma unroll
            for (int h = 0; h < CH; ++h) stg[h * 64 + lane] = nxt[h];
            // The chunk's partial-sum words (a chunk's elements lie in one word
            // per depth), loaded BEFORE the next chunk's prefetch: the wait for
            // a word then leaves the prefetch in flight.  (Loaded inside the
            // element loop, after the prefetch, every word's join drained the
            // prefetch with vmcnt(0) and each chunk paid a full memory latency.)
#pragma unroll
            for (int d = D0 + 1; d <= F; ++d) {
                static_assert(32 % (IPC << (F - D0 - 1)) == 0, "a chunk's elements share one partial-sum word per depth");
                const int e0 = (c * IPC) << (F - d);
                if (d <= G::NB && right[d] && (e0 & 31) == 0) bw[d] = bsrc[d][(e0 >> 5) * 64];
            }
            // the next chunk's prefetch: unconditional (the last chunk re-reads
            // itself; a conditional one made the compiler's wait for the words
            // above a vmcnt(0) on the path without it, draining the prefetch)
            constexpr int UNR = G::LCAP == 16 ? 4 : (G::LCAP == 32 ? PL_FT_UNR32 : 2);  // element-loop unroll (4 at L = 32: +20 %)
            auto prefetch = [&]() {
                const int cn = c + 1 < NCH ? c + 1 : c;
#pragma unroll
                for (int h = 0; h < CH; ++h) {
                    if constexpr (PL_NT_CH) {
                        const double2* a = src + (cn * CH + h) * cstr;
                        nxt[h] = make_double2(__builtin_nontemporal_load(&a->x), __builtin_nontemporal_load(&a->y));
                    } else {
                        nxt[h] = src[(cn * CH + h) * cstr];
                    }
                }
            };
            // no inner loop (IPC <= UNR): issued here.  Otherwise (LCAP >= 16)
            // inside the loop's first iteration: the loop preheader waits
            // vmcnt(0) for the words above and would drain a prefetch issued
            // before it (L = 16 -2.3 %, L = 32 -1 %; at LCAP = 8, whose inner
            // loops are the short D0 = 1, 2 passes, +3 %: spills).
            constexpr bool PF_IN = IPC > UNR && G::LCAP >= 16;
            if constexpr (!PF_IN) prefetch();
            lds_sync();
            // (unrolled 2, 4 at LCAP = 16: the D0 = 0 chunks (IPC = 2, 4) run
            // without an inner loop, whose preheader would drain the prefetch
            // with vmcnt(0); full unrolling spills at LCAP = 8 / 32)
#pragma unroll UNR
            for (int u = 0; u < IPC; ++u) {
                if constexpr (PF_IN) {
                    if (u == 0) prefetch();
                }
                const int t = c * IPC + u;
                double v[W];
#pragma unroll
                for (int k = 0; k < PPI; ++k) {
                    const double2 pr = stg[(u * PPI + k) * G::FPW + fw];
                    v[2 * k] = pr.x;
                    v[2 * k + 1] = pr.y;
                }
#pragma unroll
                for (int d = D0 + 1; d <= F; ++d) {
                    const int e0 = t << (F - d);
                    const int m = 1 << (F - d);
                    if (right[d]) {
                        const uint32_t b = bw[d] >> (e0 & 31);
#pragma unroll
                        for (int k = 0; k < m; ++k) v[k] = g_op(v[2 * k], v[2 * k + 1], b >> k);
                    } else {
#pragma unroll
                        for (int k = 0; k < m; ++k) v[k] = f_ms(v[2 * k], v[2 * k + 1]);
                    }
                }
                fold<G, F>(st, v[0], t, smem, ws, plane);
            }
        }
        return st.lam;
    }
    const double2* src = reinterpret_cast<const double2*>(ws + G::st_off(D0)) + fw;
    constexpr int kChUnroll = G::LCAP == 1 ? PL_SC_FUNROLL : 2;
#pragma unroll kChUnroll
    for (int t = 0; t < SF; ++t) {
        double v[W];
        if constexpr (G::STAGE) {
#pragma unroll
            for (int k = 0; k < W / 2; ++k) {
                const double2 pr = src[((t * (W / 2)) + k) * G::FPW];
                v[2 * k] = pr.x;
                v[2 * k + 1] = pr.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < W; ++k) v[k] = ch[t * W + k];
        }
#pragma unroll
        for (int d = D0 + 1; d <= F; ++d) {
            const int e0 = t << (F - d);  // depth-d element index of v[0]
            const int m = 1 << (F - d);
            if (right[d]) {
                if (d <= G::NB && (e0 & 31) == 0) bw[d] = bsrc[d][(e0 >> 5) * 64];
                const uint32_t b = bw[d] >> (e0 & 31);
#pragma unroll
                for (int k = 0; k < m; ++k) v[k] = g_op(v[2 * k], v[2 * k + 1], b >> k);
            } else {
#pragma unroll
                for (int k = 0; k < m; ++k) v[k] = f_ms(v[2 * k], v[2 * k + 1]);
            }
        }
        fold<G, F>(st, v[0], t, smem, ws, plane);
    }
    return st.lam;
}

template <class G>
PL_DEV double descend_fused(unsigned char* smem, unsigned char* ws, int lane, int fw, int plane, int i,
                            const double* ch, const double2* raw, uint64_t brow, uint32_t bb, uint32_t bw5,
                            uint32_t skip = 0) {
    constexpr int n = G::n, F = G::F;
    bool right[F + 1];
    const uint32_t* bsrc[F + 1];
    uint32_t bw[F + 1];
#pragma unroll
    for (int d = 1; d <= F; ++d) {
        right[d] = (i >> (n - d)) & 1;
        bsrc[d] = reinterpret_cast<const uint32_t*>(ws + G::bl_off(d <= G::NB ? d : 1)) +
                  G::pl(field(brow, d), fw);
        bw[d] = (d > G::NB) ? beta_get<n>(d, bb, bw5) : 0u;
    }
    if constexpr (G::NS >= 3) {
        if (!right[1] && !right[2] && !right[3]) return fused_loop<G, 3>(smem, ws, lane, fw, plane, ch, raw, right, bsrc, bw, skip);
    }
    if constexpr (G::NS >= 2) {
        if (!right[1] && !right[2]) return fused_loop<G, 2>(smem, ws, lane, fw, plane, ch, raw, right, bsrc, bw, skip);
    }
    if constexpr (G::NS >= 1) {
        if (!right[1]) return fused_loop<G, 1>(smem, ws, lane, fw, plane, ch, raw, right, bsrc, bw, skip);
    }
    return fused_loop<G, 0>(smem, ws, lane, fw, plane, ch, raw, right, bsrc, bw, skip);
}

// Size 2^k (k <= 3) of the rate-0 node (all leaves frozen) whose first leaf is
// decode-order leaf i, 0 if none: i a multiple of 2^k, leaves i .. i+2^k-1
// frozen (one mask word holds them).
PL_DEV int rate0_k(const uint32_t* __restrict__ frozen_dec, int i) {
    const uint32_t w = frozen_dec[i >> 5] >> (i & 31);
    return ((i & 7) == 0 && (w & 0xFFu) == 0xFFu)  ? 3
           : ((i & 3) == 0 && (w & 0xFu) == 0xFu) ? 2
           : ((i & 1) == 0 && (w & 3u) == 3u)     ? 1
                                                  : 0;
}

// Leaf LLRs of a rate-0 node (every leaf frozen, so every partial sum inside
// it is 0 and the g of a right child is btm + top): the leaves of A are the
// leaves of its f-child, then those of its g-child -- the very f / g the leaf
// by leaf schedule evaluates on the same operands.
template <int S>
PL_DEV void rate0_leaves(const double* A, double* out) {
    if constexpr (S == 1) {
        out[0] = A[0];
    } else {
        double L[S / 2], R[S / 2];
#pragma unroll
        for (int t = 0; t < S / 2; ++t) {
            L[t] = f_ms(A[2 * t], A[2 * t + 1]);
            R[t] = g_op(A[2 * t], A[2 * t + 1], 0u);
        }
        rate0_leaves<S / 2>(L, out);
        rate0_leaves<S / 2>(R, out + S / 2);
    }
}

// Leaves i+1 .. i+2^K-1 of the rate-0 node at depth n-K whose first leaf i was
// just decoded: its LLR array is the depth-(n-K) pool the descent to leaf i
// stored (this lane's plane); their path-metric increments (bit 0) are added
// in leaf order.  SC: nothing to evaluate.
template <class G, int K, bool SC>
PL_DEV void rate0_rest(const unsigned char* smem, const unsigned char* ws, int plane, bool active, double& pm) {
    if constexpr (!SC) {
        constexpr int S = 1 << K, D = G::n - K;
        const double2* src = reinterpret_cast<const double2*>((D >= G::DL ? smem : ws) + G::llr_off(D)) + plane;
        double a[S], ll[S];
#pragma unroll
        for (int j = 0; j < S / 2; ++j) {
            const double2 pr = src[j * 64];
            a[2 * j] = pr.x;
            a[2 * j + 1] = pr.y;
        }
        rate0_leaves<S>(a, ll);
        // increments of two leaves evaluated together (independent chains),
        // always computed: where path_metrics_fast skips t it is below a quarter
        // ulp of every addend and the sums are the same
        constexpr int IL = 2;
#pragma unroll
        for (int j0 = 1; j0 < S; j0 += IL) {
            double inc[IL];
#pragma unroll
            for (int u = 0; u < IL; ++u) {
                if (j0 + u < S) {
                    const double lam = ll[j0 + u];
                    const double t = metric_t<G::MF>(fabs(lam));
                    inc[u] = (lam >= 0.0) ? -t : lam - t;
                }
            }
#pragma unroll
            for (int u = 0; u < IL; ++u)
                if (j0 + u < S && active) pm = pm + inc[u];
        }
    }
}

template <class G, int P>
PL_DEV double descend_from(int p, unsigned char* smem, unsigned char* ws, int plane, int ps, int bs, uint32_t bb,
                           uint32_t bw5, uint32_t skip = 0) {
    if constexpr (P >= G::n) {
        return 0.0;
    } else {
        if (p == P) return descend_g<G, P>(smem, ws, plane, ps, bs, bb, bw5, skip);
        return descend_from<G, P + 1>(p, smem, ws, plane, ps, bs, bb, bw5, skip);
    }
}

}  // namespace

// DS (diagnostic build, the dead-store bound of DESIGN.md §4.1): 1 records in
// `stamps` (u32 words, [group][read, stored][node of depths F..DL-1][64 planes]
// bits) every workspace pool array a right child's g reads and every one
// stored; 2 replays the same frames with every store of an unread array
// skipped (same bits by construction).
template <int NL, int LCAP, bool SC, int F, int DL, bool STAMPS, int WPE, int DS = 0>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
polar_tree_kernel(const double* __restrict__ llr, int64_t ld, uint8_t* __restrict__ out,
                  const uint32_t* __restrict__ frozen_dec, const int32_t* __restrict__ info_pos, int64_t batch,
                  int K, int Lsz, unsigned char* __restrict__ workspace, unsigned long long* __restrict__ stamps,
                  const uint32_t* __restrict__ crc_g, const uint32_t* __restrict__ aux) {
    // aux: SC -- the rate-0 node table r0k; lists -- the NaN mask words,
    // u64 [gridDim.x][kNanMaskPasses], zero on entry (polar_nan.hip re-zeroes the
    // words it reads).  One argument for both: a separate mask pointer kept live
    // across the leaf loop cost the list instances 8-24 spilled bytes per lane.
    const uint32_t* __restrict__ r0k = SC ? aux : nullptr;
    using G = TG<NL, LCAP, F, DL, DS>;
    constexpr int n = G::n, N = G::N, FPW = G::FPW;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int fw = lane / LCAP, slot = lane % LCAP, base = fw * LCAP;
    // Workspace / LDS pools, partial sums and walk buffers are slot-major: path
    // slot s of the wave's frame f lives in plane s * FPW + f, so the wave's
    // slot-0 entries share one 128-byte line.  While the list is still growing
    // (slot >= nact) a lane shadows slot 0: it takes slot 0's survivor entry at
    // every pruning (same rows, partial sums and bit; metric -inf), uses slot
    // 0's plane, and so loads the lines slot 0 loads and stores the values
    // slot 0 stores to the same addresses -- no memory traffic of its own.
    unsigned char* const ws = workspace + (size_t)blockIdx.x * G::WS;
    uint64_t own = 0;
#pragma unroll
    for (int d = 0; d < 12; ++d) own |= (uint64_t)slot << (RB * d);
    double2* const met = reinterpret_cast<double2*>(smem + G::L_MET + fw * G::GS);    // [LCAP] of this frame
    uint64_t* const rowx = reinterpret_cast<uint64_t*>(smem + G::L_ROW + fw * G::GS);  // [LCAP][2]
    uint64_t* const brx = reinterpret_cast<uint64_t*>(smem + G::L_BR) + base;          // [LCAP]
    uint32_t* const surv = reinterpret_cast<uint32_t*>(smem + G::L_SURV) + base;       // [LCAP]
    uint32_t* const walk0 = reinterpret_cast<uint32_t*>(ws + G::W_WALK) + (G::SHADOW ? fw : 0);  // [2][CW][64]

    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // STAMPS: metric evaluations -- [0] path_metrics_fast calls (per wave), [1] of
    // them with a lane that needs log1p(e^-x), [2] such lanes, [3] active lanes
    unsigned long long mcnt[4] = {0, 0, 0, 0};
    auto count_metric = [&](double pmv, double lamv, bool act) {
        if constexpr (STAMPS) {
            const uint64_t need = __ballot(metric_needs_t(pmv, lamv, act)), on = __ballot(act);
            mcnt[0] += 1;
            mcnt[1] += need ? 1 : 0;
            mcnt[2] += (unsigned long long)__popcll(need);
            mcnt[3] += (unsigned long long)__popcll(on);
        }
    };
    unsigned long long tprev = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
#define STAMP(k)                                                    \
    if constexpr (STAMPS) {                                         \
        const unsigned long long tn = __builtin_amdgcn_s_memtime(); \
        acc[k] += tn - tprev;                                       \
        tprev = tn;                                                 \
    }

    // Frame groups (FPW frames each): group blockIdx.x first; then the next
    // unclaimed group from one counter (kSchedBytes before the slices, zeroed by
    // tree_launch), so that wavefronts slowed by harder frames, a busier SIMD or
    // a busier XCD take fewer groups instead of stretching the launch's tail
    // (the static b, b + grid, b + 2 grid, ... measured 8.5 % slower at L = 32)
    const int64_t ngrp = (batch + FPW - 1) / FPW;
    unsigned int* const sched = reinterpret_cast<unsigned int*>(workspace - kSchedBytes);
    // (at n = 12 with 14 waves per CU it cost 3-5 %, profiles/r04_a/ab_prio_4096.log;
    // with 16 it gains 2.4 %, profiles/r05_b/ab_t12*.log)
    constexpr int PRIO = PL_TREE_PRIO;
#if PL_TREE_PRIO >= 2
    // the first group: later-dispatched wavefronts (younger on their SIMD, so
    // behind in the age-ordered issue arbitration) start at a higher priority
    if constexpr (PRIO >= 2) set_prio_quarter(blockIdx.x, gridDim.x);
#endif
    for (int64_t grp = blockIdx.x; grp < ngrp;) {
        const int64_t f0 = grp * FPW;
        const int64_t frame = f0 + fw;
        const bool live = frame < batch;
        const double* __restrict__ ch = llr + (live ? frame : batch - 1) * ld;
        const double2* raw = nullptr;  // depth-0 pairs read in place (fused_loop)
        if constexpr (G::STAGE) {
            // channel rows of this wave's frames -> [N/2][FPW] pairs, plus the
            // path-independent left-most f-only nodes of depths 1..NS.
            // Lane: frame l % FPW, CV consecutive channel values per step.
            const int sf = lane % FPW;
            const int64_t fr = f0 + sf < batch ? f0 + sf : batch - 1;
            const double* row = llr + fr * ld;
            if (G::dedup(0) && (ld & 1) == 0 && ((uintptr_t)llr & 15) == 0)
                raw = reinterpret_cast<const double2*>(row) + lane / FPW;
            constexpr int CV = 2 << G::NS;    // channel values per lane per step
            constexpr int CPI = 64 / FPW;     // chunks per frame per step
            // NaN path metrics need a NaN LLR at a leaf, i.e. a NaN input or an
            // inf - inf in a g.  The two operands of a g descend from disjoint
            // halves of its node's inputs, and an LLR whose inputs are all below
            // 2^1000 in magnitude is finite (<= 12 levels at most double it), so
            // with no NaN input and at most ONE input of magnitude >= 2^1000 (or
            // inf) no g meets two infinities: every LLR is finite or +-inf and
            // every metric a sum of non-positive terms (-inf at worst, never NaN).
            // Frames with a NaN input or two such inputs are flagged in this
            // pass's mask word (aux) and decoded again by polar_nan.hip in the
            // reference's exact candidate order (list.sort, decoder.py:306-307);
            // a frame with one erasure-style +-inf stays on this kernel.
            int ext = 0;  // this lane's inputs of magnitude >= 2^1000 or inf, + 2 per NaN
#pragma unroll 1
            for (int cb = 0; cb < N / CV; cb += CPI) {
                const int cc = cb + lane / FPW;
                double v[CV];
#pragma unroll
                for (int k = 0; k < CV; ++k) v[k] = row[CV * cc + k];
#pragma unroll
                for (int k = 0; k < CV; ++k) ext += !(fabs(v[k]) < 0x1p1000) ? (__builtin_isnan(v[k]) ? 2 : 1) : 0;
                // depth d of the chunk: CV >> d values = CV >> (d+1) pairs
#pragma unroll
                for (int d = 0; d <= G::NS; ++d) {
                    double2* dst = reinterpret_cast<double2*>(ws + G::st_off(d)) + sf;
                    const int np = CV >> (d + 1);
                    if (d > 0 || raw == nullptr) {
#pragma unroll
                        for (int k = 0; k < np; ++k) dst[(np * cc + k) * FPW] = make_double2(v[2 * k], v[2 * k + 1]);
                    }
                    if (d < G::NS) {
#pragma unroll
                        for (int k = 0; k < np; ++k) v[k] = f_ms(v[2 * k], v[2 * k + 1]);
                    }
                }
            }
            // lane l stages frame l % FPW: a frame is flagged when a lane saw a NaN
            // or two extreme inputs, or two of its lanes saw one each
            const uint64_t b1 = __ballot(ext >= 1), b2 = __ballot(ext >= 2);
            if (!SC && b1) {
                uint64_t lanes = 0;
#pragma unroll
                for (int sft = 0; sft < 64; sft += FPW) lanes |= 1ull << sft;
                uint64_t fm = 0;
#pragma unroll
                for (int f = 0; f < FPW; ++f)
                    if ((b2 & (lanes << f)) || __popcll(b1 & (lanes << f)) >= 2) fm |= 1ull << f;
                // word [grp % grid][grp / grid], where the static schedule's pass
                // grp / grid of wavefront grp % grid keeps it (polar_nan.hip)
                const uint32_t ps = (uint32_t)grp / gridDim.x, wv = (uint32_t)grp % gridDim.x;
                if (fm && lane == 0 && ps < (uint32_t)kNanMaskPasses)
                    atomicOr(reinterpret_cast<unsigned long long*>(const_cast<uint32_t*>(aux)) +
                                 (size_t)wv * kNanMaskPasses + ps,
                             (unsigned long long)fm);
            }
        }
        uint64_t lrow = G::SHADOW ? 0 : own, brow = lrow;  // shadows start on slot 0's rows
        uint32_t bb = 0, bw5 = 0;
        double pm = (slot == 0) ? 0.0 : -INFINITY;
        int nact = 1;
        int root_par = 0;
        STAMP(7);
        int nextK = (SC && r0k) ? (int)(r0k[0] & 15u) : 0;  // SC: r0k of the next leaf (scalar load, a leaf ahead)

        for (int i = 0; i < N; ++i) {
            // ================================================ LLRs down to leaf i
            const int dstart = (i == 0) ? 1 : n - __builtin_ctz(i);
            const int pslot = (!G::SHADOW || slot < nact) ? slot : 0;  // shadows use slot 0's planes
            const int plane = G::pl(pslot, fw);
            // SC: leaves i .. i + 2^skipK - 1 form the largest all-frozen node
            // that starts at leaf i (host table, decode order).  SC decides a
            // frozen bit without its LLR and nothing inside the node is read
            // after it, so those leaves are not decoded at all: the descent to
            // leaf i is skipped when every array it would store lies inside the
            // node (skipK = ctz i), and otherwise runs only for the ancestors'
            // arrays it stores on the way; the node's partial sums are zeros.
            const int skipK = SC ? nextK : 0;
            const bool skip_descend = SC && skipK > 0 && i > 0 && skipK >= __builtin_ctz(i);
            double lam = 0.0;
            // DS: the pool arrays of node i >> (n - d), depths F..DL-1, as bits of
            // this group's words: [read][stored], DSW words each
            constexpr int DSW = ((1 << DL) - (1 << F)) * 2;
            uint32_t* const dsm = DS ? reinterpret_cast<uint32_t*>(stamps) + grp * 2 * DSW : nullptr;
            uint32_t dskip = 0;
            if constexpr (DS == 1) {
                if (!skip_descend) {
#pragma unroll
                    for (int d = F; d < DL; ++d)
                        if (d >= dstart)
                            atomicOr(dsm + DSW + ((1 << d) - (1 << F) + (i >> (n - d))) * 2 + (plane >> 5),
                                     1u << (plane & 31));
                }
            }
            if constexpr (DS == 2) {
                // (depth, node) is wave-uniform: one scalar 8-byte load per depth,
                // the lane's plane bit extracted from it (no per-lane gather)
                const uint64_t* __restrict__ dsm64 = reinterpret_cast<const uint64_t*>(stamps) + grp * DSW;
#pragma unroll
                for (int d = F; d < DL; ++d) {
                    if (d >= dstart) {
                        const uint64_t mk = dsm64[(1 << d) - (1 << F) + (i >> (n - d))];
                        if (!((mk >> plane) & 1u)) dskip |= 1u << d;
                    }
                }
            }
            if (!skip_descend) {
                if (dstart <= DL) ws_sync();  // workspace written by other lanes
                STAMP(7);
                if (dstart <= F) {
                    lam = descend_fused<G>(smem, ws, lane, fw, plane, i, ch, raw, brow, bb, bw5, dskip);
                    lrow = set_range(lrow, (!G::SHADOW || slot < nact) ? own : 0ull, F, n);
                    STAMP(0);
                } else {
                    const int p = dstart - 1;
                    const int ps = G::pl(field(lrow, p), fw);
                    const int bs = G::pl(field(brow, dstart <= G::NB ? dstart : 0), fw);
                    if constexpr (DS == 1) {
                        if (p >= F && p < DL)
                            atomicOr(dsm + ((1 << p) - (1 << F) + (i >> (n - p))) * 2 + (ps >> 5), 1u << (ps & 31));
                    }
                    lam = descend_from<G, F>(p, smem, ws, plane, ps, bs, bb, bw5, dskip);
                    lrow = set_range(lrow, (!G::SHADOW || slot < nact) ? own : 0ull, dstart, n);
                    if (p < DL) { STAMP(1); } else { STAMP(2); }
                }
            }

            // ================================================ decision at leaf i
            const bool frozen = (frozen_dec[i >> 5] >> (i & 31)) & 1u;
            int bit;
            if constexpr (SC) {
                bit = frozen ? 0 : (lam >= 0.0 ? 0 : 1);
                STAMP(3);
            } else if (frozen) {
                double m0, m1;
                count_metric(pm, lam, slot < nact);
                path_metrics_fast<false, G::MF>(pm, lam, slot < nact, m0, m1);
                if (slot < nact) pm = m0;
                bit = 0;
                STAMP(3);
            } else {
                double m0, m1;
                count_metric(pm, lam, slot < nact);
                path_metrics_fast<true, G::MF>(pm, lam, slot < nact, m0, m1);
                STAMP(3);
                // a full, ordered list keeps its order: survivor s = path s
                // with its better bit (ordered_prune), nothing exchanged
                bool kept = false;
                // (measured: L = 16 / 32 at N = 1024 -4.5 % / -4.7 %, L = 8 at N = 4096 -3.7 %,
                // L = 8 at N = 1024 +1.8 %: eight frames per wave rarely all stay ordered)
                if constexpr (LCAP >= PL_ORDERED_PRUNE || (NL >= 11 && LCAP >= 8)) {
                    if (nact == LCAP && Lsz == LCAP) kept = ordered_prune<LCAP>(m0, m1, slot, lane);
                }
                if (kept) {
                    bit = m1 > m0 ? 1 : 0;
                    pm = bit ? m1 : m0;
                } else {
                constexpr bool STRICT = LCAP >= RANK_STRICT_LCAP || NL >= 11;
                constexpr bool F32 = STRICT;
                // DPP: the fp32 ranks from lane exchanges inside the frame's 8
                // lanes instead of an LDS round trip (N=1024 6.42 -> 6.38 ms,
                // N=4096 11.69 -> 11.51 ms).  Finding each survivor the same way
                // (a search over the 8 lanes' ranks instead of the LDS survivor
                // table) measured slower: 6.52 ms.
                constexpr bool DPP = F32 && LCAP == 8;
                constexpr bool BITONIC = F32 && LCAP == 32;
                if constexpr (F32 && !DPP && !BITONIC) reinterpret_cast<float2*>(met)[slot] = make_float2((float)m0, (float)m1);
                else met[slot] = make_double2(m0, m1);
                rowx[2 * slot] = lrow;
                rowx[2 * slot + 1] = brow;
                brx[slot] = (uint64_t)bb | ((uint64_t)bw5 << 32);
                if constexpr (!DPP && !BITONIC) lds_sync();
                // rank of (slot, b) in the stable descending order of
                // [(m0, q) for active q] + [(m1, q) for active q]
                constexpr int QC = LCAP < 8 ? LCAP : 8;
                auto exact_ranks = [&](int& r0, int& r1) {
                    r0 = 0;
                    r1 = 0;
                    for (int q0 = 0; q0 < nact; q0 += QC) {
                        double2 mq[QC];
#pragma unroll
                        for (int k = 0; k < QC; ++k) mq[k] = met[q0 + k];
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
                };
                const int nsurv = (2 * nact < Lsz) ? 2 * nact : Lsz;
                const uint32_t id0 = (uint32_t)(slot << 1), id1 = id0 | 1u;
                // survivor this lane takes (decoder.py:323-336); lanes beyond the
                // survivors shadow survivor 0 (see `plane`)
                const int tgt = slot < nsurv ? slot : 0;
                uint32_t e = 0;  // survivor entry: parent slot << 1 | bit
                int r0, r1;
                if constexpr (BITONIC) {
                    // LCAP = 32: sort the 64 keys (bit_key) across the frame's
                    // lanes; lane s then holds survivor s.  Two candidates whose
                    // fp32 metrics agree in all but the 6 label bits at or above
                    // the survivor boundary (or a NaN metric) send the wave to the
                    // exact fp64 ranks below, as a tie does on the LDS path.
                    const bool act = slot < nact;
                    int k0 = act ? bit_key(m0, slot) : (int)0x80000000;  // (m0, slot): list index slot
                    int k1 = act ? bit_key(m1, 32 + slot) : (int)0x80000000;  // (m1, slot): after every m0
                    const bool bad = act && (__builtin_isnan(m0) || __builtin_isnan(m1));
                    bit_sort64_desc(k0, k1, slot);
                    // position s + 1: element 0 of lane s + 1, or element 1 of lane 0 for s = 31
                    const int x = slot == 0 ? k1 : k0;
                    const int nxt = __builtin_amdgcn_ds_bpermute((((slot + 1) & 31) + fw * 32) * 4, x);
                    const bool lost = slot < nsurv && ((k0 ^ nxt) & ~63) == 0;
                    const int cidx = 63 - (k0 & 63);
                    const uint32_t eo = (uint32_t)(((cidx & 31) << 1) | (cidx >> 5));
                    const uint32_t e0 = (uint32_t)__builtin_amdgcn_readlane((int)eo, 0);
                    const uint32_t e32 = (uint32_t)__builtin_amdgcn_readlane((int)eo, 32);
                    e = slot < nsurv ? eo : (fw ? e32 : e0);  // beyond the survivors: shadow survivor 0
                    if (__ballot(lost || bad)) {
                        lds_sync();  // the fp64 metrics of every lane
                        exact_ranks(r0, r1);
                        if (slot < nact) {
                            if (r0 < nsurv) surv[r0] = id0;
                            if (r1 < nsurv) surv[r1] = id1;
                        }
                        lds_sync();
                        e = surv[tgt];
                    }
                } else if constexpr (STRICT) {
                    // Lists of 8+ / long codes: strict comparisons only -- exact unless two
                    // candidates tie (inactive slots publish -inf and never
                    // count).  A tie makes two candidates claim one survivor
                    // slot; the wave sees it and redoes the ranks with the
                    // stable tie-break.  (L = 32: 9.1 -> 7.5 ms, L = 16:
                    // 7.7 -> 7.0 ms, N = 2048 / 4096 L = 8: ~2 %, N = 1024 L = 8
                    // with shadow lanes: 6.72 -> 6.54 ms.)
                    // F32: the comparisons use the fp32 roundings, half the LDS
                    // bytes of the rank loop.  Rounding is monotone, so a > b in
                    // fp32 implies a > b; two candidates that round equal get
                    // the same rank and collide like a tie, and ranks at or past
                    // the survivors cannot hide one below them.
                    r0 = 0;
                    r1 = 0;
                    if constexpr (DPP) {
                        const float f0 = (float)m0, f1 = (float)m1;
                        r0 = f1 > f0;  // own pair (f0 > f0 never counts)
                        r1 = f0 > f1;
                        auto cmp = [&](int v) {
                            const float c = __int_as_float(v);
                            r0 += c > f0;
                            r1 += c > f1;
                        };
                        group8_each(__float_as_int(f0), cmp);
                        group8_each(__float_as_int(f1), cmp);
                    } else if constexpr (F32) {
                        const float f0 = (float)m0, f1 = (float)m1;
                        const float2* const met32 = reinterpret_cast<const float2*>(met);
                        for (int q0 = 0; q0 < nact; q0 += QC) {
                            float2 mq[QC];
#pragma unroll
                            for (int k = 0; k < QC; ++k) mq[k] = met32[q0 + k];
#pragma unroll
                            for (int k = 0; k < QC; ++k) {
                                const float a = mq[k].x, b = mq[k].y;
                                r0 += (a > f0) + (b > f0);
                                r1 += (a > f1) + (b > f1);
                            }
                        }
                    } else {
                        for (int q0 = 0; q0 < nact; q0 += QC) {
                            double2 mq[QC];
#pragma unroll
                            for (int k = 0; k < QC; ++k) mq[k] = met[q0 + k];
#pragma unroll
                            for (int k = 0; k < QC; ++k) {
                                const double a = mq[k].x, b = mq[k].y;
                                r0 += (a > m0) + (b > m0);
                                r1 += (a > m1) + (b > m1);
                            }
                        }
                    }
                    if (slot < nact) {
                        if (r0 < nsurv) surv[r0] = id0;
                        if (r1 < nsurv) surv[r1] = id1;
                    }
                    lds_sync();
                    // fp64 metrics over the fp32 copies (all read before the sync)
                    if constexpr (F32 && !DPP) met[slot] = make_double2(m0, m1);
                    // a lost claim = a tie; the survivor entry is read in the same trip
                    const bool lost =
                        slot < nact && ((r0 < nsurv && surv[r0] != id0) || (r1 < nsurv && surv[r1] != id1));
                    e = surv[tgt];
                    if (__ballot(lost)) {
                        lds_sync();  // the fp64 metrics of every lane; surv reads done
                        exact_ranks(r0, r1);
                        if (slot < nact) {
                            if (r0 < nsurv) surv[r0] = id0;
                            if (r1 < nsurv) surv[r1] = id1;
                        }
                        lds_sync();
                        e = surv[tgt];
                    }
                } else {
                    exact_ranks(r0, r1);
                    if (slot < nact) {
                        if (r0 < nsurv) surv[r0] = id0;
                        if (r1 < nsurv) surv[r1] = id1;
                    }
                    lds_sync();
                    e = surv[tgt];
                }
                lds_sync();  // met / rows of every lane written
                if (G::SHADOW || slot < nsurv) {
                    const int par = (int)(e >> 1);
                    bit = (int)(e & 1u);
                    const double2 pmv = met[par];
                    pm = slot < nsurv ? (bit ? pmv.y : pmv.x) : -INFINITY;
                    lrow = rowx[2 * par];
                    brow = rowx[2 * par + 1];
                    const uint64_t br = brx[par];
                    bb = (uint32_t)br;
                    bw5 = (uint32_t)(br >> 32);
                } else {
                    pm = -INFINITY;  // LCAP = 16: inactive slots keep their own state
                    bit = 0;
                }
                nact = nsurv;
                lds_sync();  // scratch reads done before the next leaf's writes
                }
                STAMP(4);
            }

            // ========================================= rate-0 node from leaf i
            // Leaves i .. i+2^k-1 all frozen (k <= 3, i a multiple of 2^k): their
            // bits are 0, so every partial sum inside the node is 0 and nothing
            // the later leaves' descents, walks or pointer rows would produce
            // is read after the node except the zeros walked up from its last
            // leaf.  Their LLRs follow from the node's array (depth n-k, stored by
            // the descent to leaf i) without a descent each; the metrics are
            // added in leaf order.  Same operations on the same operands as the
            // leaf-by-leaf schedule.
            if constexpr (SC) {
                if (skipK > 0) i += (1 << skipK) - 1;  // the walk below runs for the node's last leaf
                nextK = (r0k && i + 1 < N) ? (int)((r0k[(i + 1) >> 3] >> (4 * ((i + 1) & 7))) & 15u) : 0;
            } else {
                if (frozen) {
                    const int k = rate0_k(frozen_dec, i);
                    if (k > 0) {
                        const int pslot = (!G::SHADOW || slot < nact) ? slot : 0;
                        const int plane = G::pl(pslot, fw);
                        if (k == 3) rate0_rest<G, 3, SC>(smem, ws, plane, slot < nact, pm);
                        else if (k == 2) rate0_rest<G, 2, SC>(smem, ws, plane, slot < nact, pm);
                        else rate0_rest<G, 1, SC>(smem, ws, plane, slot < nact, pm);
                        bb &= ~((1u << ((1 << k) - 1)) - 1u);  // partial sums of depths n-k+1..n: 0
                        i += (1 << k) - 1;                     // the walk below runs for the node's last leaf
                        STAMP(3);
                    }
                }
            }

            // ================================================ partial-sum walk
            {
                const int to = __builtin_ctz(~(unsigned)i);
                const int steps = to < n ? to : n;
                // SC, skipped node of 2^skipK leaves: the walk starts at the node's
                // own depth with its 2^skipK zero partial sums (skipK <= steps)
                int dd = n - skipK;
                uint32_t cur = (uint32_t)bit;
                int k = skipK;
                if (SC && skipK > 5 && k == steps) {
                    // the node is a left child at a multi-word depth: store its
                    // zero words as that depth's partial sums (read by the right
                    // sibling's g), nothing to combine
                    uint32_t* dst = reinterpret_cast<uint32_t*>(ws + G::bl_off(dd)) + G::pl(slot, fw);
                    for (int w = 0; w < (1 << (skipK - 5)); ++w) dst[w * 64] = 0u;
                    brow = set_field(brow, dd, slot);
                    k = steps + 1;  // done (no register store either)
                }
                for (; k < steps && k < 5; ++k) {
                    const uint32_t left = beta_get<n>(dd, bb, bw5);
                    const uint32_t msk = (1u << (1 << k)) - 1u;
                    cur = spread16((left ^ cur) & msk) | (spread16(cur & msk) << 1);
                    --dd;
                }
                if (k > steps) {
                    // SC skipped node stored above
                } else if (k == steps) {
                    beta_set<n>(dd, cur, bb, bw5);  // dd >= n-5: a left child, kept in registers
                } else {
                    // dd == n-5, cur = one word: multi-word combine through the workspace.
                    // Planes from the list size after this leaf's pruning: a lane that
                    // just stopped shadowing slot 0 writes its own.
                    const int wslot = (!G::SHADOW || slot < nact) ? slot : 0;
                    uint32_t* const walkw = walk0 + (G::SHADOW ? wslot * FPW : lane);
                    int parity = 0;
                    ws_sync();  // multi-word betas of other lanes live in the workspace
                    walkw[0] = cur;
                    if (SC && skipK > 5) {  // the skipped node's zero words (k = skipK)
                        for (int w = 1; w < (1 << (skipK - 5)); ++w) walkw[w * 64] = 0u;
                    }
                    for (; k < steps; ++k) {
                        const int cwc = 1 << (k - 5);
                        const int ls = G::pl(field(brow, dd <= G::NB ? dd : 0), fw);
                        const bool last = (k + 1 == steps);
                        const uint32_t* lsrc = reinterpret_cast<const uint32_t*>(ws + G::bl_off(dd <= G::NB ? dd : 1)) + ls;
                        uint32_t* ldst = reinterpret_cast<uint32_t*>(ws + G::bl_off(dd - 1 >= 1 ? dd - 1 : 1)) +
                                         G::pl(wslot, fw);
                        // word j of the step's input gives output words 2j, 2j+1
                        // (one round trip per input word instead of per output
                        // word; batching WB = 2 / 4 input words measured 7 / 16 %
                        // slower at L = 8: spills)
                        constexpr int WB = 1;
                        uint32_t* const wdst = (last && dd - 1 > 0) ? ldst : walkw + (parity ^ 1) * G::CW * 64;
#pragma unroll 1
                        for (int j0 = 0; j0 < cwc; j0 += WB) {
                            uint32_t cv[WB], lv[WB];
#pragma unroll
                            for (int u = 0; u < WB; ++u) {
                                if (j0 + u < cwc) {  // wave-uniform
                                    cv[u] = walkw[(parity * G::CW + j0 + u) * 64];
                                    lv[u] = (dd > G::NB) ? bw5 : lsrc[(j0 + u) * 64];
                                }
                            }
#pragma unroll
                            for (int u = 0; u < WB; ++u) {
                                if (j0 + u < cwc) {
                                    const uint32_t x = lv[u] ^ cv[u];
                                    wdst[(2 * (j0 + u)) * 64] = spread16(x) | (spread16(cv[u]) << 1);
                                    wdst[(2 * (j0 + u) + 1) * 64] = spread16(x >> 16) | (spread16(cv[u] >> 16) << 1);
                                }
                            }
                        }
                        parity ^= 1;
                        --dd;
                    }
                    if (dd == 0) root_par = parity;
                    else brow = set_field(brow, dd, wslot);
                }
            }
            lds_sync();
            STAMP(5);
        }

        // ================================================ best path, output
        uint32_t* const walk = walk0 + (G::SHADOW ? (slot < nact ? slot : 0) * FPW : lane);
        int best = 0;
        if constexpr (!SC) {
            met[slot] = make_double2(pm, 0.0);
            lds_sync();
            if (crc_g) {
                // CRC-aided selection (build-defined extension): the
                // first path in descending-metric order (ties: lower slot) whose
                // u_hat[info] passes the CRC; none -> that order's first = argmax
                const uint32_t crc = crc_of_xhat(walk + root_par * G::CW * 64, 64, G::CW, crc_g);
                int rank = 0;
                for (int q = 0; q < nact; ++q) {
                    const double v = met[q].x;
                    rank += (v > pm) | ((v == pm) & (q < slot));
                }
                surv[slot] = slot >= nact ? 0xFFFFu : (uint32_t)(crc == 0u ? rank : 64 + rank);
                lds_sync();
                uint32_t bk = surv[0];
                for (int q = 1; q < nact; ++q) {
                    const uint32_t k = surv[q];
                    if (k < bk) { bk = k; best = q; }
                }
            } else {
                double bm = met[0].x;
                for (int q = 1; q < nact; ++q) {
                    const double v = met[q].x;
                    if (v > bm) { bm = v; best = q; }
                }
            }
            lds_sync();
        }
        ws_sync();  // the root partial sum was written to the walk buffer
        uint32_t* X = reinterpret_cast<uint32_t*>(smem + G::L_FINAL) + fw * G::CW;
        if (slot == best) {
            // LCAP >= 16 at n <= 10: 32 words loaded before the first of them
            // is transformed (one round trip per 32 words): L=32 -2.2 %; at
            // LCAP = 8 equal, at N = 4096 +3.8 % (spills)
            constexpr bool XBATCH = G::LCAP >= 16 && n <= 10;
            if constexpr (XBATCH) {
            constexpr int XB = G::CW < 32 ? G::CW : 32;
#pragma unroll 1
            for (int w0 = 0; w0 < G::CW; w0 += XB) {
                uint32_t xw[XB];
#pragma unroll
                for (int w = 0; w < XB; ++w) xw[w] = walk[(root_par * G::CW + w0 + w) * 64];
                asm volatile("" ::: "memory");
#pragma unroll
                for (int w = 0; w < XB; ++w) X[w0 + w] = polar_word_transform(xw[w]);
            }
            } else {
            for (int w = 0; w < G::CW; ++w) X[w] = polar_word_transform(walk[(root_par * G::CW + w) * 64]);
            }
        }
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
        ws_sync();  // staging of the next frames overwrites workspace read above
        STAMP(6);
        // a counter read past the end (it only grows: a stale value is never
        // too large) ends the loop without a claim, so the wavefronts finishing
        // together at the end do not queue on one atomic
        unsigned int nx = 0xFFFFFFFFu;
        if (lane == 0) {
            const unsigned int seen = __hip_atomic_load(sched, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((int64_t)gridDim.x + (int64_t)seen < ngrp)
                nx = __hip_atomic_fetch_add(sched, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        nx = (unsigned int)__builtin_amdgcn_readfirstlane((int)nx);
        grp = nx == 0xFFFFFFFFu ? ngrp : (int64_t)gridDim.x + (int64_t)nx;
#if PL_TREE_PRIO
        // claims come in finishing order: a wavefront in the last quarters of
        // its round runs the next group at a higher issue priority
        if (PRIO >= 1 && nx != 0xFFFFFFFFu) set_prio_quarter(nx % gridDim.x, gridDim.x);
#endif
    }
    if constexpr (STAMPS && !DS) {
        if (lane == 0) {
            for (int k = 0; k < 8; ++k) atomicAdd(stamps + k, acc[k]);
            for (int k = 0; k < 4; ++k) atomicAdd(stamps + 8 + k, mcnt[k]);
        }
    }
#undef STAMP
}

// ------------------------------------------------------------------- host
namespace {

struct TreeEntry {
    int n, lcap;
    bool sc;
    int F, DL;
    void* fn;         // compiled for 4 waves/SIMD (<= 128 VGPRs; measured fastest)
    void* fn_stamps;  // PL_DIAG only: per-phase s_memtime stamps
    void* fn_wpe1;    // PL_DIAG only: compiler's own register budget (3 waves/SIMD), PL_TREE_WPE=1
    void* fn_ds[2];   // PL_DIAG only (the headline instance): dead-store record / replay
    int lds;
    int64_t ws;
};

template <int NL, int LCAP, bool SC, int F, int DL, bool VARIANTS = false, int WPE = 4>
TreeEntry make_entry() {
    using G = TG<NL, LCAP, F, DL>;
    void* st = nullptr;
    void* w1 = nullptr;
    void* ds1 = nullptr;
    void* ds2 = nullptr;
#if PL_DIAG
    st = (void*)polar_tree_kernel<NL, LCAP, SC, F, DL, true, WPE>;
    if constexpr (VARIANTS) {
        w1 = (void*)polar_tree_kernel<NL, LCAP, SC, F, DL, false, 1>;
        ds1 = (void*)polar_tree_kernel<NL, LCAP, SC, F, DL, false, WPE, 1>;
        ds2 = (void*)polar_tree_kernel<NL, LCAP, SC, F, DL, false, WPE, 2>;
    }
#endif
    return TreeEntry{NL, LCAP, SC, F, DL, (void*)polar_tree_kernel<NL, LCAP, SC, F, DL, false, WPE>, st, w1,
                     {ds1, ds2}, G::LDS, G::WS};
}

// (n, list capacity) pairs built with the tree kernel: the BASELINE.json
// configurations (N=256 SC, N=1024 SC / SCL L=8 / L=32, N=4096 SCL L=8), SCL
// L=4/16 at N=1024, L=8 at N=2048, SC at N=128..4096; the diagnostic build adds
// the tier alternatives measured against them (PL_TREE_F, PL_TREE_DL, PL_TREE_DLOFF).
// polar_lane.hip serves every other (N, L).
const TreeEntry* tree_table(int* count) {
    static const TreeEntry tab[] = {
        make_entry<10, 8, false, 3, 7, true>(),
#if PL_DIAG
        make_entry<10, 8, false, 2, 7>(),
        make_entry<10, 8, false, 4, 7>(),
        make_entry<12, 8, false, 3, 9>(),
#endif
        make_entry<10, 32, false, 3, 7>(),
        make_entry<10, 16, false, 3, 7>(),
        make_entry<10, 4, false, 3, 7>(),
        make_entry<11, 8, false, 3, 8>(),
        make_entry<12, 8, false, 4, 9, false, PL_T12_WPE>(),  // N = 4096: F = 4 11.63 vs F = 3 11.89 ms (16 384 frames)
        make_entry<8, 2, false, 3, 5>(),
        make_entry<8, 4, false, 3, 5>(),
        make_entry<8, 8, false, 3, 5>(),
        make_entry<8, 16, false, 3, 5>(),
        make_entry<8, 32, false, 3, 5>(),
        make_entry<9, 8, false, 3, 6>(),
        make_entry<9, 16, false, 3, 6>(),
        make_entry<10, 2, false, 3, 7>(),
        make_entry<7, 8, false, 3, 4>(),
        make_entry<7, 32, false, 3, 4>(),
        // SC: no fused top (a lane's frame shares its channel row with no other
        // lane) and five LDS depths (62 doubles per frame, 31 KB per wave, 5
        // waves per CU): N=1024 1.88 -> 1.28 ms, N=4096 5.78 -> 4.47 ms against
        // F = 3, DL = n-3 (profiles/r03_d/ab_sc_tiers.log)
        make_entry<7, 1, true, 1, 2, false, PL_SC_WPE>(),
        make_entry<8, 1, true, 1, 3, false, PL_SC_WPE>(),
        make_entry<9, 1, true, 1, 4, false, PL_SC_WPE>(),
        make_entry<10, 1, true, 1, 5, false, PL_SC_WPE>(),
        make_entry<11, 1, true, 1, 6, false, PL_SC_WPE>(),
        make_entry<12, 1, true, 1, 7, false, PL_SC_WPE>(),
#if PL_DIAG  // after the product entries: picked only through PL_TREE_F / PL_TREE_DL(OFF)
        make_entry<10, 32, false, 4, 7>(),
        make_entry<10, 32, false, 2, 7>(),
        make_entry<10, 1, true, 3, 7>(),
        make_entry<10, 1, true, 2, 7>(),
        make_entry<10, 1, true, 1, 6, false, PL_SC_WPE>(),
        make_entry<10, 1, true, 1, 4, false, PL_SC_WPE>(),
#endif
    };
    *count = (int)(sizeof(tab) / sizeof(tab[0]));
    return tab;
}

// Small-batch instances: one more LDS depth (DL - 1) and a 2-wave register
// budget (no spills; the LDS allows 8 waves per CU).  A batch whose wavefronts
// fit the device at 8 per CU runs at that occupancy either way, and then the
// depth kept out of the workspace wins: A/B on one box, bits identical
// (profiles/r06_d/ab_sb*.log): N=4096 L=8 16 384 / 8 192 frames 9.75 -> 8.34 /
// 7.10 -> 6.41 ms, N=2048 16 384 4.05 -> 3.71, N=1024 L=8 16 384 1.88 -> 1.76,
// L=32 4 096 1.70 -> 1.59, L=16 8 192 1.80 -> 1.59, L=4 32 768 2.17 -> 1.97,
// N=512 L=8 16 384 0.857 -> 0.817, L=16 8 192 0.760 -> 0.713 (ab_smore.log).
// Above one such pass the product entries win (N=4096
// at 131 072 frames: 76.7 against 57.8 ms at 4 waves per SIMD, ab_dl12.log).
const TreeEntry* tree_table_small(int* count) {
    static const TreeEntry tab[] = {
        make_entry<12, 8, false, 4, 8, false, 2>(),
        make_entry<11, 8, false, 3, 7, false, 2>(),
        make_entry<10, 8, false, 3, 6, false, 2>(),
        make_entry<10, 32, false, 3, 6, false, 2>(),
        make_entry<10, 16, false, 3, 6, false, 2>(),
        make_entry<10, 4, false, 3, 6, false, 2>(),
        make_entry<9, 8, false, 3, 5, false, 2>(),
        make_entry<9, 16, false, 3, 5, false, 2>(),
    };
    *count = (int)(sizeof(tab) / sizeof(tab[0]));
    return tab;
}

}  // namespace

bool tree_lookup(int n, int lcap, bool sc, TreeInfo* info) {
    int cnt = 0;
    const TreeEntry* t = tree_table(&cnt);
    const char* fe = PL_DIAG ? std::getenv("PL_TREE_F") : nullptr;  // diagnostic: pick the fused-top depth
    const int want_f = fe ? std::atoi(fe) : 0;
    const char* de = PL_DIAG ? std::getenv("PL_TREE_DL") : nullptr;  // diagnostic: pick the first LDS depth
    const char* doff = PL_DIAG ? std::getenv("PL_TREE_DLOFF") : nullptr;  // diagnostic: first LDS depth n - value
    const int want_dl = de ? std::atoi(de) : (doff ? n - std::atoi(doff) : 0);
    for (int k = 0; k < cnt; ++k)
        if (t[k].n == n && t[k].lcap == lcap && t[k].sc == sc && (!want_f || t[k].F == want_f) &&
            (!want_dl || t[k].DL == want_dl)) {
            const char* w = PL_DIAG ? std::getenv("PL_TREE_WPE") : nullptr;
            const int wpe = w ? std::atoi(w) : 4;
            info->fn = (wpe == 1 && t[k].fn_wpe1) ? t[k].fn_wpe1 : t[k].fn;
            info->fn_stamps = t[k].fn_stamps;
            info->fn_ds[0] = t[k].fn_ds[0];
            info->fn_ds[1] = t[k].fn_ds[1];
            info->lds_bytes = t[k].lds;
            info->ws_bytes = t[k].ws;
            info->F = t[k].F;
            info->DL = t[k].DL;
            info->fpw = 64 / lcap;
            return true;
        }
    return false;
}

// the small-batch instance for (n, lcap) if there is one (tree_table_small);
// PL_TREE_SMALL=0 turns them off, as does a diagnostic tier choice (PL_TREE_F / DL / DLOFF)
bool tree_lookup_small(int n, int lcap, bool sc, TreeInfo* info) {
    const char* off = std::getenv("PL_TREE_SMALL");
    if (sc || (off && std::atoi(off) == 0)) return false;
    if (PL_DIAG && (std::getenv("PL_TREE_F") || std::getenv("PL_TREE_DL") || std::getenv("PL_TREE_DLOFF"))) return false;
    int cnt = 0;
    const TreeEntry* t = tree_table_small(&cnt);
    for (int k = 0; k < cnt; ++k)
        if (t[k].n == n && t[k].lcap == lcap && t[k].sc == sc) {
            *info = TreeInfo{};
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
    if (t.fn_stamps) {
        e = hipFuncSetAttribute(t.fn_stamps, hipFuncAttributeMaxDynamicSharedMemorySize, t.lds_bytes);
        if (e != hipSuccess) return e;
    }
    int nb = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, t.fn, 64, t.lds_bytes);
    if (e != hipSuccess) return e;
    *max_blocks_per_cu = nb < 1 ? 1 : nb;
    return hipSuccess;
}

hipError_t tree_launch(const TreeInfo& t, const double* llr, int64_t ld, uint8_t* out, const uint32_t* frozen_dec,
                       const int32_t* info_pos, int64_t batch, int K, int Lsz, unsigned char* ws, int grid,
                       unsigned long long* stamps, const uint32_t* crc_g, const void* aux, hipStream_t s,
                       int ds_mode) {
    void* args[] = {(void*)&llr, (void*)&ld, (void*)&out, (void*)&frozen_dec, (void*)&info_pos, (void*)&batch,
                    (void*)&K,   (void*)&Lsz, (void*)&ws, (void*)&stamps,     (void*)&crc_g,    (void*)&aux};
    void* fn = stamps ? t.fn_stamps : t.fn;
#if PL_DIAG
    if (ds_mode) {  // pl_debug_polar_deadstore: `stamps` is the record / replay bitmask
        fn = t.fn_ds[ds_mode - 1];
        if (!fn || !stamps) return hipErrorInvalidValue;
        if (hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, t.lds_bytes);
            e != hipSuccess)
            return e;
    }
#else
    if (ds_mode) return hipErrorInvalidValue;
#endif
    if (!fn) return hipErrorInvalidValue;
    // the frame-group counter (kernel: group loop)
    if (hipError_t e = hipMemsetAsync(ws - kSchedBytes, 0, 4, s); e != hipSuccess) return e;
    return hipLaunchKernel(fn, dim3((unsigned)grid), dim3(64), args, t.lds_bytes, s);
}

}  // namespace pl
