// Batched polar SC / SCL decoder for gfx950 (MI355X).
//
// Semantics: src/polar/decoder.py of the reference --
//   SCDecoder.decode  :38-71   (min-sum f :121-127, g :129-144, u = 0 if L >= 0)
//   SCLDecoder.decode :225-262 (frozen :264-281, info :283-339, metric :374-406,
//                               stable descending sort, survivors renumbered in
//                               sorted order, final np.argmax = first maximum)
// The decision sequence is reproduced exactly: every LLR is produced by the same
// fp64 f/g operation on the same operands as the reference (f is exact, g one
// rounding), metrics by the same fp64 formula; only exp/log1p come from ocml
// instead of NumPy (<= 1-2 ulp apart), and they are
// skipped where their value provably cannot change the rounded metric.
//
// Mapping (DESIGN.md §Polar kernel):
//   * one wavefront (= one workgroup) decodes one frame; the 64 lanes are split
//     into LCAP lane groups of G = 64/LCAP lanes, group p = list slot p;
//   * tree arrays use the reference's own element layout, so a child element t
//     reads the adjacent parent pair (2t, 2t+1): one ds_read_b128;
//   * LLR arrays are pooled per depth with per-path slot pointers (no copies on
//     path cloning).  A path only ever writes depths whose previous contents are
//     dead for every path, so clones share arrays by pointer only.  The pointer
//     rows live in registers and are cloned with ds_bpermute;
//   * the top F depths are never stored: the depth-F node is recomputed straight
//     from the channel LLRs in HBM (2^F contiguous doubles per output);
//   * the bottom B <= 3 depths are never stored either: every leaf recomputes its
//     chain from the pooled depth-(n-B) node in registers (no LDS round trip, no
//     barrier on the per-leaf path);
//   * list pruning (rank in the stable descending order of the 2*nact candidate
//     metrics, survivors renumbered by rank) runs on readlane/bpermute;
//   * partial sums (beta) are bit-packed, pooled per depth like the LLRs, and
//     built by a walk up the trailing-ones path of each leaf;
//   * u_hat is never stored: the root partial sum of the best path is the
//     re-encoded codeword x_hat and u = x_hat * F^{(x)n} (an involution).
#include "common.hpp"
#include "internal.hpp"

namespace pl {

// ------------------------------------------------------------------ helpers
// Slot-pointer row of one path: byte d of (a0|a1) = LLR-pool slot of depth d,
// byte d of (b0|b1) = beta-pool slot of depth d (d < 16).  Four named 64-bit
// words, so every access is a shift (no indexable array -> no scratch).
struct Row {
    uint64_t a0, a1, b0, b1;
};

PL_DEV int row_llr(const Row& r, int d) {  // d wave-uniform
    const uint64_t w = (d < 8) ? r.a0 : r.a1;
    return (int)((w >> ((d & 7) * 8)) & 0xFFu);
}
PL_DEV int row_beta(const Row& r, int d) {
    const uint64_t w = (d < 8) ? r.b0 : r.b1;
    return (int)((w >> ((d & 7) * 8)) & 0xFFu);
}

PL_DEV uint64_t byte_range_mask(int a, int b) {  // bytes [a, b) of a 64-bit word, 0 <= a, b <= 8
    if (b <= a) return 0ull;
    const uint64_t hi = (b >= 8) ? ~0ull : ((1ull << (8 * b)) - 1ull);
    const uint64_t lo = (a <= 0) ? 0ull : ((1ull << (8 * a)) - 1ull);
    return hi & ~lo;
}

PL_DEV void fill_pair(uint64_t& w0, uint64_t& w1, int lo, int hi, int val) {  // depths [lo, hi) := val
    const uint64_t rep = (uint64_t)(uint32_t)val * 0x0101010101010101ull;
    const int a0 = lo < 0 ? 0 : (lo > 8 ? 8 : lo), b0 = hi < 0 ? 0 : (hi > 8 ? 8 : hi);
    const int a1 = lo - 8 < 0 ? 0 : (lo - 8 > 8 ? 8 : lo - 8), b1 = hi - 8 < 0 ? 0 : (hi - 8 > 8 ? 8 : hi - 8);
    const uint64_t m0 = byte_range_mask(a0, b0), m1 = byte_range_mask(a1, b1);
    w0 = (w0 & ~m0) | (rep & m0);
    w1 = (w1 & ~m1) | (rep & m1);
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

// Path-metric increment (decoder.py:374-406): t = log1p(exp(-|lam|));
//   LL0 = lam >= 0 ? -t : lam - t ;  LL1 = lam >= 0 ? -lam - t : -t.
// Returns m0 = pm + LL0 and (if want1) m1 = pm + LL1, rounded exactly like the
// reference.  When exp(-|lam|) < 2^(e-56) for e = min(ilogb pm, ilogb |lam|)
// (pm != 0), t is below a quarter ulp of every quantity it is added to, so the
// rounded results do not depend on it and the transcendentals are skipped.
template <bool WANT1>
PL_DEV void metrics(double pm, double lam, double& m0, double& m1) {
    const double x = fabs(lam);
    int e = ilogb(pm);
    const int ex = ilogb(x);
    e = e < ex ? e : ex;
    e = e < -1100 ? -1100 : (e > 1100 ? 1100 : e);  // ilogb(0) = INT_MIN: keep 56 - e finite
    const bool skip = (pm != 0.0) && (x > (double)(56 - e) * 0.6931471805599453);
    double t = 0.0;
    if (!skip) t = log1p(exp(-x));
    const double ll0 = (lam >= 0.0) ? -t : lam - t;
    m0 = pm + ll0;
    if (WANT1) {
        const double ll1 = (lam >= 0.0) ? -lam - t : -t;
        m1 = pm + ll1;
    }
}

struct SurvEntry {
    double m;
    int pb;
    int pad;
};

template <int F, int G>
PL_DEV double fused_top(const PolarGeom& g, int i, const double* __restrict__ ch, const Row& row, int slot,
                        int lg, unsigned char* smem) {
    const int n = g.n;
    const int S = 1 << (n - F);  // depth-F node size
    bool right[F + 1];
    const uint32_t* beta[F + 1];
#pragma unroll
    for (int d = 1; d <= F; ++d) {
        right[d] = (i >> (n - d)) & 1;
        beta[d] = reinterpret_cast<const uint32_t*>(smem + g.bl_off[d]) + row_beta(row, d) * g.bl_words[d];
    }
    double lam = 0.0;
    double* dst = (F < n) ? reinterpret_cast<double*>(smem + g.llr_off[F]) + slot * S : nullptr;
    for (int t = (S == 1 ? 0 : lg); t < S; t += G) {
        double v[1 << F];
        const double* src = ch + ((size_t)t << F);
#pragma unroll
        for (int k = 0; k < (1 << F); ++k) v[k] = src[k];
#pragma unroll
        for (int d = 1; d <= F; ++d) {
            const int base = t << (F - d);
            const uint32_t bw = right[d] ? (beta[d][base >> 5] >> (base & 31)) : 0u;
#pragma unroll
            for (int k = 0; k < (1 << (F - d)); ++k) {
                const double a = v[2 * k], b = v[2 * k + 1];
                v[k] = right[d] ? (((bw >> k) & 1u) ? b - a : b + a) : f_minsum(a, b);
            }
        }
        if (F < n) dst[t] = v[0];
        else lam = v[0];
    }
    return lam;
}

// Chain from a node of 2^B values (v) down to leaf i (depths D+1..n), in registers.
template <int B>
PL_DEV double bottom_chain(const PolarGeom& g, int i, double (&v)[8], const Row& row, unsigned char* smem) {
    const int n = g.n;
#pragma unroll
    for (int s = 0; s < B; ++s) {
        const int d = n - B + 1 + s;  // child depth
        const bool right = (i >> (n - d)) & 1;
        uint32_t bw = 0;
        if (right) bw = *(reinterpret_cast<const uint32_t*>(smem + g.bl_off[d]) + row_beta(row, d) * g.bl_words[d]);
#pragma unroll
        for (int k = 0; k < (1 << (B - 1 - s)); ++k) {
            const double a = v[2 * k], b = v[2 * k + 1];
            v[k] = right ? (((bw >> k) & 1u) ? b - a : b + a) : f_minsum(a, b);
        }
    }
    return v[0];
}

template <int LCAP, bool SC, int F, int B, bool STAMPS>
__global__ void __launch_bounds__(64)
polar_decode_kernel(PolarGeom g, const double* __restrict__ llr, int64_t ld, uint8_t* __restrict__ out,
                    const uint32_t* __restrict__ frozen_dec, const int32_t* __restrict__ info_pos,
                    int64_t batch, unsigned long long* __restrict__ stamps) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int G = 64 / LCAP;
    const int64_t frame = blockIdx.x;
    if (frame >= batch) return;
    const int lane = threadIdx.x;
    const int slot = lane / G;
    const int lg = lane & (G - 1);
    const int n = g.n, N = g.N;
    const int D = n - B;  // deepest pooled depth (node of 2^B values), D >= F
    const double* __restrict__ ch = llr + frame * ld;
    unsigned long long acc[5] = {0, 0, 0, 0, 0};
    unsigned long long tprev = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
#define STAMP(k)                                                   \
    if constexpr (STAMPS) {                                        \
        const unsigned long long tn = __builtin_amdgcn_s_memtime(); \
        acc[k] += tn - tprev;                                      \
        tprev = tn;                                                \
    }

    Row row;
    row.a0 = row.a1 = row.b0 = row.b1 = (uint64_t)(uint32_t)slot * 0x0101010101010101ull;

    double pm = (slot == 0) ? 0.0 : -INFINITY;
    int nact = 1;
    int root_par = 0;

    for (int i = 0; i < N; ++i) {
        // ------------------------------------------------ LLRs down to leaf i
        const int dstart = (i == 0) ? 1 : n - __builtin_ctz(i);  // depth of the first child computed
        double lam;
        if (B == 0 && dstart <= F) {
            lam = fused_top<F, G>(g, i, ch, row, slot, lg, smem);  // F == n
        } else {
            int src_slot;
            if (dstart <= D) {
                int d;
                if (dstart <= F) {
                    fused_top<F, G>(g, i, ch, row, slot, lg, smem);
                    d = F;
                } else {
                    const int d0 = dstart - 1;
                    const int S = 1 << (n - dstart);
                    const double* par =
                        reinterpret_cast<const double*>(smem + g.llr_off[d0]) + row_llr(row, d0) * (2 * S);
                    const uint32_t* beta = reinterpret_cast<const uint32_t*>(smem + g.bl_off[dstart]) +
                                           row_beta(row, dstart) * g.bl_words[dstart];
                    double* dst = reinterpret_cast<double*>(smem + g.llr_off[dstart]) + slot * S;
                    for (int t = lg; t < S; t += G) {
                        const double2 ab = reinterpret_cast<const double2*>(par)[t];
                        dst[t] = ((beta[t >> 5] >> (t & 31)) & 1u) ? ab.y - ab.x : ab.y + ab.x;
                    }
                    d = dstart;
                }
                for (; d < D; ++d) {  // left children: f
                    __syncthreads();
                    const int S = 1 << (n - d - 1);
                    const double2* par =
                        reinterpret_cast<const double2*>(smem + g.llr_off[d]) + slot * S;
                    double* dst = reinterpret_cast<double*>(smem + g.llr_off[d + 1]) + slot * S;
                    for (int t = lg; t < S; t += G) {
                        const double2 ab = par[t];
                        dst[t] = f_minsum(ab.x, ab.y);
                    }
                }
                __syncthreads();
                fill_pair(row.a0, row.a1, dstart > F ? dstart : F, D + 1, slot);
                src_slot = slot;
            } else {
                src_slot = row_llr(row, D);
            }
            double v[8];
            const double2* node = reinterpret_cast<const double2*>(smem + g.llr_off[D]) + src_slot * (1 << B) / 2;
#pragma unroll
            for (int k = 0; k < (1 << B) / 2; ++k) {
                const double2 ab = node[k];
                v[2 * k] = ab.x;
                v[2 * k + 1] = ab.y;
            }
            lam = bottom_chain<B>(g, i, v, row, smem);
        }
        STAMP(0);

        // ------------------------------------------------ decision at leaf i
        const bool frozen = (frozen_dec[i >> 5] >> (i & 31)) & 1u;
        int bit;
        if constexpr (SC) {
            bit = frozen ? 0 : (lam >= 0.0 ? 0 : 1);  // decoder.py:61-64, :117-119
            STAMP(1);
        } else {
            if (frozen) {                               // decoder.py:264-281
                double m0, m1;
                metrics<false>(pm, lam, m0, m1);
                if (slot < nact) pm = m0;
                bit = 0;
                STAMP(1);
            } else {                                    // decoder.py:283-339
                double m0, m1;
                metrics<true>(pm, lam, m0, m1);
                STAMP(1);
                // rank of (slot, b) in the stable descending order of
                // [(m0, p) for active p] + [(m1, p) for active p]
                int r0 = 0, r1 = 0;
                for (int q = 0; q < nact; ++q) {
                    const double a = readlane_d(m0, q * G), b = readlane_d(m1, q * G);
                    r0 += (a > m0) | ((a == m0) & (q < slot));
                    r0 += (b > m0);
                    r1 += (a >= m1);
                    r1 += (b > m1) | ((b == m1) & (q < slot));
                }
                const int nsurv = (2 * nact < g.Lsz) ? 2 * nact : g.Lsz;
                // survivor `slot` = the candidate of rank `slot`
                int par = 0;
                bit = 0;
                for (int q = 0; q < nact; ++q) {
                    const int a = __builtin_amdgcn_readlane(r0, q * G), b = __builtin_amdgcn_readlane(r1, q * G);
                    if (a == slot) { par = q; bit = 0; }
                    if (b == slot) { par = q; bit = 1; }
                }
                const int src = par * G + lg;
                const double pa = bperm_d(src, m0), pb = bperm_d(src, m1);
                Row nr;
                nr.a0 = bperm64(src, row.a0); nr.a1 = bperm64(src, row.a1);
                nr.b0 = bperm64(src, row.b0); nr.b1 = bperm64(src, row.b1);
                if (slot < nsurv) {
                    pm = bit ? pb : pa;
                    row = nr;
                } else {
                    pm = -INFINITY;
                }
                nact = nsurv;
                STAMP(2);
            }
        }

        // ------------------------------------------------ partial-sum walk
        // Leaf i closes the nodes on its trailing-ones path; their beta is
        // [left ^ right, right] interleaved (decoder.py:96-115).
        {
            const int to = __builtin_ctz(~(unsigned)i);
            const int steps = to < n ? to : n;
            int dd = n;
            uint32_t cur = (uint32_t)bit;
            int k = 0;
            for (; k < steps && k < 5; ++k) {
                const uint32_t left =
                    *(reinterpret_cast<const uint32_t*>(smem + g.bl_off[dd]) + row_beta(row, dd) * g.bl_words[dd]);
                const uint32_t msk = (1u << (1 << k)) - 1u;
                cur = spread16((left ^ cur) & msk) | (spread16(cur & msk) << 1);
                --dd;
            }
            if (k == steps) {
                if (dd == 0) root_par = 0;
                if (lg == 0) {
                    if (dd > 0) *(reinterpret_cast<uint32_t*>(smem + g.bl_off[dd]) + slot * g.bl_words[dd]) = cur;
                    else *(reinterpret_cast<uint32_t*>(smem + g.cur_off) + slot * 2 * g.cw) = cur;
                }
            } else {
                uint32_t* buf = reinterpret_cast<uint32_t*>(smem + g.cur_off) + slot * 2 * g.cw;
                int parity = 0;
                if (lg == 0) buf[0] = cur;
                for (; k < steps; ++k) {
                    __syncthreads();
                    const int cwc = 1 << (k - 5);
                    const uint32_t* left =
                        reinterpret_cast<const uint32_t*>(smem + g.bl_off[dd]) + row_beta(row, dd) * g.bl_words[dd];
                    const uint32_t* srcw = buf + parity * g.cw;
                    const bool last = (k + 1 == steps);
                    uint32_t* dst = (last && dd - 1 > 0)
                                        ? reinterpret_cast<uint32_t*>(smem + g.bl_off[dd - 1]) + slot * g.bl_words[dd - 1]
                                        : buf + (parity ^ 1) * g.cw;
                    for (int w = lg; w < 2 * cwc; w += G) {
                        const uint32_t cwv = srcw[w >> 1], lw = left[w >> 1];
                        const int sh = (w & 1) * 16;
                        dst[w] = spread16((lw ^ cwv) >> sh) | (spread16(cwv >> sh) << 1);
                    }
                    parity ^= 1;
                    --dd;
                }
                if (dd == 0) root_par = parity;
            }
            if (dd > 0) fill_pair(row.b0, row.b1, dd, dd + 1, slot);
        }
        __syncthreads();
        STAMP(3);
    }

    // ---------------------------------------------------- best path, output
    int best = 0;
    if constexpr (!SC) {
        double bm = readlane_d(pm, 0);
        for (int q = 1; q < nact; ++q) {
            const double v = readlane_d(pm, q * G);
            if (v > bm) { bm = v; best = q; }
        }
    }
    uint32_t* X = reinterpret_cast<uint32_t*>(smem + g.cur_off) + (best * 2 + root_par) * g.cw;
    for (int w = lane; w < g.cw; w += 64) X[w] = polar_word_transform(X[w]);
    for (int sw = 1; sw < g.cw; sw <<= 1) {
        __syncthreads();
        for (int w = lane; w < g.cw; w += 64)
            if (!(w & sw)) X[w] ^= X[w + sw];
    }
    __syncthreads();
    uint8_t* o = out + frame * (int64_t)g.K;
    for (int k = lane; k < g.K; k += 64) {
        const int p = info_pos[k];
        o[k] = (uint8_t)((X[p >> 5] >> (p & 31)) & 1u);
    }
    STAMP(4);
    if constexpr (STAMPS) {
        if (lane == 0)
            for (int k = 0; k < 5; ++k) atomicAdd(stamps + k, acc[k]);
    }
#undef STAMP
}

// ------------------------------------------------------------------- host
int polar_lcap(int list_size) {
    int l = list_size < 1 ? 1 : list_size;
    int c = 1;
    while (c < l) c <<= 1;
    return c;
}

static int bottom_depths(int n, int F) { int b = n - F; return b > 3 ? 3 : (b < 0 ? 0 : b); }

int polar_geom(int N, int K, int list_size, int F, PolarGeom* g) {
    int n = 0;
    while ((1 << n) < N) ++n;
    const int lcap = polar_lcap(list_size);
    if (F > n) F = n;
    if (F < 1) F = 1;
    const int B = bottom_depths(n, F);
    const int D = n - B;
    g->N = N; g->n = n; g->K = K; g->Lsz = list_size < 1 ? 1 : list_size; g->F = F; g->lcap = lcap;
    int off = 0;
    for (int d = 0; d < kMaxDepth + 2; ++d) { g->llr_off[d] = 0; g->bl_off[d] = 0; g->bl_words[d] = 0; }
    if (B > 0)
        for (int d = F; d <= D; ++d) { g->llr_off[d] = off; off += lcap * (1 << (n - d)) * 8; }
    for (int d = 1; d <= n; ++d) {
        const int w = (1 << (n - d)) / 32;
        g->bl_words[d] = w < 1 ? 1 : w;
        g->bl_off[d] = off;
        off += lcap * g->bl_words[d] * 4;
    }
    g->cw = N / 32 < 1 ? 1 : N / 32;
    g->cur_off = off; off += lcap * 2 * g->cw * 4;
    g->tab_off = off;
    off = (off + 15) & ~15;
    g->surv_off = off;
    g->lds_bytes = off;
    return off;
}

template <int LCAP, bool SC, int F, bool ST>
static void* pick_b(int B) {
    switch (B) {
        case 0: return (void*)polar_decode_kernel<LCAP, SC, F, 0, ST>;
        case 1: return (void*)polar_decode_kernel<LCAP, SC, F, 1, ST>;
        case 2: return (void*)polar_decode_kernel<LCAP, SC, F, 2, ST>;
        default: return (void*)polar_decode_kernel<LCAP, SC, F, 3, ST>;
    }
}

template <int LCAP, bool SC, bool ST>
static void* pick_f(int F, int B) {
    switch (F) {
        case 1: return pick_b<LCAP, SC, 1, ST>(B);
        case 2: return pick_b<LCAP, SC, 2, ST>(B);
        case 3: return pick_b<LCAP, SC, 3, ST>(B);
        default: return pick_b<LCAP, SC, 4, ST>(B);
    }
}

static void* pick_kernel(const PolarGeom& g, bool sc, bool stamps) {
    const int B = bottom_depths(g.n, g.F);
    if (stamps) {
        if (sc) return pick_f<1, true, true>(g.F, B);
        return g.lcap == 8 ? pick_f<8, false, true>(g.F, B) : nullptr;
    }
    if (sc) return pick_f<1, true, false>(g.F, B);
    switch (g.lcap) {
        case 1: return pick_f<1, false, false>(g.F, B);
        case 2: return pick_f<2, false, false>(g.F, B);
        case 4: return pick_f<4, false, false>(g.F, B);
        case 8: return pick_f<8, false, false>(g.F, B);
        case 16: return pick_f<16, false, false>(g.F, B);
        case 32: return pick_f<32, false, false>(g.F, B);
        default: return nullptr;
    }
}

hipError_t polar_prepare(const PolarGeom& g, bool sc) {
    void* k = pick_kernel(g, sc, false);
    if (!k) return hipErrorInvalidValue;
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, g.lds_bytes);
    if (e != hipSuccess) return e;
    if (void* ks = pick_kernel(g, sc, true))
        e = hipFuncSetAttribute(ks, hipFuncAttributeMaxDynamicSharedMemorySize, g.lds_bytes);
    return e;
}

hipError_t polar_launch(const PolarGeom& g, bool sc, const double* llr, int64_t ld, uint8_t* out,
                        const uint32_t* frozen_dec, const int32_t* info_pos, int64_t batch, hipStream_t s,
                        unsigned long long* stamps) {
    void* k = pick_kernel(g, sc, stamps != nullptr);
    if (!k) return hipErrorInvalidValue;
    const int64_t maxgrid = 1ll << 30;
    for (int64_t b0 = 0; b0 < batch; b0 += maxgrid) {
        const int64_t nb = (batch - b0) < maxgrid ? (batch - b0) : maxgrid;
        PolarGeom gg = g;
        const double* l = llr + b0 * ld;
        uint8_t* o = out + b0 * g.K;
        void* args[] = {&gg, (void*)&l, (void*)&ld, (void*)&o, (void*)&frozen_dec, (void*)&info_pos,
                        (void*)&nb, (void*)&stamps};
        hipError_t e = hipLaunchKernel(k, dim3((unsigned)nb), dim3(64), args, g.lds_bytes, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace pl
