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
// instead of NumPy (<= 1-2 ulp apart).
//
// Mapping (DESIGN.md §Polar kernel):
//   * one wavefront (= one workgroup) decodes one frame; the 64 lanes are split
//     into LCAP lane groups of G = 64/LCAP lanes, group p = list slot p;
//   * tree arrays use the reference's own element layout, so a child element t
//     always reads the adjacent parent pair (2t, 2t+1): one ds_read_b128;
//   * LLR arrays are pooled per depth with per-path slot pointers (no copies on
//     path cloning).  A path only ever writes depths whose previous contents are
//     dead for every path, so clones share arrays by pointer only;
//   * the top F depths are never stored: the depth-F node is recomputed straight
//     from the channel LLRs in HBM (2^F contiguous doubles per output) -- this
//     halves/quarters the LDS footprint to raise occupancy;
//   * partial sums (beta) are bit-packed, pooled per depth like the LLRs, and
//     built by a walk up the trailing-ones path of each leaf;
//   * u_hat is never stored: at the end the root partial sum of the best path is
//     the re-encoded codeword x_hat and u = x_hat * F^{(x)n} (an involution).
#include "common.hpp"
#include "internal.hpp"

namespace pl {

struct SurvEntry {
    double m;
    int pb;  // parent * 2 + bit
    int pad;
};

template <int F, int G>
PL_DEV double fused_top(const PolarGeom& g, int i, const double* __restrict__ ch,
                        const uint8_t* tab, int slot, int lg, unsigned char* smem) {
    const int n = g.n;
    const int S = 1 << (n - F);  // depth-F node size
    bool right[F + 1];
    const uint32_t* beta[F + 1];
#pragma unroll
    for (int d = 1; d <= F; ++d) {
        right[d] = (i >> (n - d)) & 1;
        beta[d] = reinterpret_cast<const uint32_t*>(smem + g.bl_off[d]) + tab[16 + d] * g.bl_words[d];
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
            const int base = t << (F - d);  // depth-d element index of v[0]
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

template <int LCAP, bool SC, int F>
__global__ void __launch_bounds__(64)
polar_decode_kernel(PolarGeom g, const double* __restrict__ llr, int64_t ld, uint8_t* __restrict__ out,
                    const uint32_t* __restrict__ frozen_dec, const int32_t* __restrict__ info_pos,
                    int64_t batch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int G = 64 / LCAP;
    const int64_t frame = blockIdx.x;
    if (frame >= batch) return;
    const int lane = threadIdx.x;
    const int slot = lane / G;
    const int lg = lane & (G - 1);
    const int n = g.n, N = g.N;
    const double* __restrict__ ch = llr + frame * ld;
    uint8_t* tab = smem + g.tab_off + slot * 32;
    for (int w = lg; w < 8; w += G) reinterpret_cast<uint32_t*>(tab)[w] = (uint32_t)slot * 0x01010101u;

    double pm = (slot == 0) ? 0.0 : -INFINITY;
    int nact = 1;
    int root_par = 0;
    __syncthreads();

    for (int i = 0; i < N; ++i) {
        // ------------------------------------------------ LLRs down to leaf i
        const int dstart = (i == 0) ? 1 : n - __builtin_ctz(i);  // depth of the first child computed
        double lam = 0.0;
        int d;
        if (dstart <= F) {
            lam = fused_top<F, G>(g, i, ch, tab, slot, lg, smem);
            d = F;
        } else {
            const int d0 = dstart - 1;
            const int S = 1 << (n - dstart);
            const double* par = reinterpret_cast<const double*>(smem + g.llr_off[d0]) + tab[d0] * (2 * S);
            const uint32_t* beta =
                reinterpret_cast<const uint32_t*>(smem + g.bl_off[dstart]) + tab[16 + dstart] * g.bl_words[dstart];
            if (dstart == n) {
                const double2 ab = *reinterpret_cast<const double2*>(par);
                lam = (beta[0] & 1u) ? ab.y - ab.x : ab.y + ab.x;
            } else {
                double* dst = reinterpret_cast<double*>(smem + g.llr_off[dstart]) + slot * S;
                for (int t = lg; t < S; t += G) {
                    const double2 ab = reinterpret_cast<const double2*>(par)[t];
                    dst[t] = ((beta[t >> 5] >> (t & 31)) & 1u) ? ab.y - ab.x : ab.y + ab.x;
                }
            }
            d = dstart;
        }
        for (; d < n; ++d) {  // left children: f
            __syncthreads();
            const int S = 1 << (n - d - 1);
            const double* par = reinterpret_cast<const double*>(smem + g.llr_off[d]) + slot * (2 * S);
            if (d + 1 == n) {
                const double2 ab = *reinterpret_cast<const double2*>(par);
                lam = f_minsum(ab.x, ab.y);
            } else {
                double* dst = reinterpret_cast<double*>(smem + g.llr_off[d + 1]) + slot * S;
                for (int t = lg; t < S; t += G) {
                    const double2 ab = reinterpret_cast<const double2*>(par)[t];
                    dst[t] = f_minsum(ab.x, ab.y);
                }
            }
        }
        if (lg == 0) {
            for (int dd = (dstart > F ? dstart : F); dd < n; ++dd) tab[dd] = (uint8_t)slot;
        }

        // ------------------------------------------------ decision at leaf i
        const bool frozen = (frozen_dec[i >> 5] >> (i & 31)) & 1u;
        int bit;
        if constexpr (SC) {
            bit = frozen ? 0 : (lam >= 0.0 ? 0 : 1);  // decoder.py:61-64, :117-119
        } else {
            const double t = log1p(exp(-fabs(lam)));      // decoder.py:391-406
            const double ll0 = (lam >= 0.0) ? -t : lam - t;
            if (frozen) {                                   // decoder.py:264-281
                if (slot < nact) pm = pm + ll0;
                bit = 0;
            } else {                                        // decoder.py:283-339
                const double ll1 = (lam >= 0.0) ? -lam - t : -t;
                const double m0 = pm + ll0, m1 = pm + ll1;
                // rank in the stable descending order of the candidate list
                // [(m0,p) for active p] + [(m1,p) for active p]
                int r0 = 0, r1 = 0;
                for (int q = 0; q < nact; ++q) {
                    const double mq = readlane_d(m0, q * G);
                    r0 += (mq > m0) | ((mq == m0) & (q < slot));
                    r1 += (mq >= m1);
                }
                for (int q = 0; q < nact; ++q) {
                    const double mq = readlane_d(m1, q * G);
                    r0 += (mq > m0);
                    r1 += (mq > m1) | ((mq == m1) & (q < slot));
                }
                const int nsurv = (2 * nact < g.Lsz) ? 2 * nact : g.Lsz;
                SurvEntry* st = reinterpret_cast<SurvEntry*>(smem + g.surv_off);
                __syncthreads();
                if (slot < nact && lg == 0) {
                    if (r0 < nsurv) { st[r0].m = m0; st[r0].pb = slot * 2; }
                    if (r1 < nsurv) { st[r1].m = m1; st[r1].pb = slot * 2 + 1; }
                }
                __syncthreads();
                uint32_t row[8 / (G < 8 ? G : 8)];
                bit = 0;
                if (slot < nsurv) {
                    const double em = st[slot].m;
                    const int pb = st[slot].pb;
                    const uint32_t* prow = reinterpret_cast<const uint32_t*>(smem + g.tab_off + (pb >> 1) * 32);
#pragma unroll
                    for (int k = 0; k < 8 / (G < 8 ? G : 8); ++k) {
                        const int w = lg + k * G;
                        row[k] = (w < 8) ? prow[w] : 0u;
                    }
                    pm = em;
                    bit = pb & 1;
                }
                __syncthreads();
                if (slot < nsurv) {
#pragma unroll
                    for (int k = 0; k < 8 / (G < 8 ? G : 8); ++k) {
                        const int w = lg + k * G;
                        if (w < 8) reinterpret_cast<uint32_t*>(tab)[w] = row[k];
                    }
                }
                nact = nsurv;
            }
        }
        __syncthreads();

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
                    *(reinterpret_cast<const uint32_t*>(smem + g.bl_off[dd]) + tab[16 + dd] * g.bl_words[dd]);
                const uint32_t msk = (1u << (1 << k)) - 1u;
                cur = spread16((left ^ cur) & msk) | (spread16(cur & msk) << 1);
                --dd;
            }
            if (k == steps) {
                if (dd == 0) root_par = 0;
                if (lg == 0) {
                    if (dd > 0) {
                        *(reinterpret_cast<uint32_t*>(smem + g.bl_off[dd]) + slot * g.bl_words[dd]) = cur;
                        tab[16 + dd] = (uint8_t)slot;
                    } else {
                        *(reinterpret_cast<uint32_t*>(smem + g.cur_off) + slot * 2 * g.cw) = cur;
                    }
                }
            } else {
                uint32_t* buf = reinterpret_cast<uint32_t*>(smem + g.cur_off) + slot * 2 * g.cw;
                int par = 0;
                if (lg == 0) buf[0] = cur;
                for (; k < steps; ++k) {
                    __syncthreads();
                    const int cwc = 1 << (k - 5);
                    const uint32_t* left =
                        reinterpret_cast<const uint32_t*>(smem + g.bl_off[dd]) + tab[16 + dd] * g.bl_words[dd];
                    const uint32_t* src = buf + par * g.cw;
                    const bool last = (k + 1 == steps);
                    uint32_t* dst = (last && dd - 1 > 0)
                                        ? reinterpret_cast<uint32_t*>(smem + g.bl_off[dd - 1]) + slot * g.bl_words[dd - 1]
                                        : buf + (par ^ 1) * g.cw;
                    for (int w = lg; w < 2 * cwc; w += G) {
                        const uint32_t cwv = src[w >> 1], lw = left[w >> 1];
                        const int sh = (w & 1) * 16;
                        dst[w] = spread16((lw ^ cwv) >> sh) | (spread16(cwv >> sh) << 1);
                    }
                    par ^= 1;
                    --dd;
                }
                if (dd > 0) {
                    if (lg == 0) tab[16 + dd] = (uint8_t)slot;
                } else {
                    root_par = par;
                }
            }
        }
        __syncthreads();
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
}

// ------------------------------------------------------------------- host
int polar_lcap(int list_size) {
    int l = list_size < 1 ? 1 : list_size;
    int c = 1;
    while (c < l) c <<= 1;
    return c;
}

int polar_geom(int N, int K, int list_size, int F, PolarGeom* g) {
    int n = 0;
    while ((1 << n) < N) ++n;
    const int lcap = polar_lcap(list_size);
    if (F > n) F = n;
    if (F < 1) F = 1;
    g->N = N; g->n = n; g->K = K; g->Lsz = list_size < 1 ? 1 : list_size; g->F = F; g->lcap = lcap;
    int off = 0;
    for (int d = 0; d < kMaxDepth + 2; ++d) { g->llr_off[d] = 0; g->bl_off[d] = 0; g->bl_words[d] = 0; }
    for (int d = F; d < n; ++d) { g->llr_off[d] = off; off += lcap * (1 << (n - d)) * 8; }
    for (int d = 1; d <= n; ++d) {
        const int w = (1 << (n - d)) / 32;
        g->bl_words[d] = w < 1 ? 1 : w;
        g->bl_off[d] = off;
        off += lcap * g->bl_words[d] * 4;
    }
    g->cw = N / 32 < 1 ? 1 : N / 32;
    g->cur_off = off; off += lcap * 2 * g->cw * 4;
    g->tab_off = off; off += lcap * 32;
    off = (off + 15) & ~15;
    g->surv_off = off; off += lcap * 16;
    off = (off + 15) & ~15;
    g->lds_bytes = off;
    return off;
}

template <int LCAP, bool SC>
static void* pick_f(int F) {
    switch (F) {
        case 1: return (void*)polar_decode_kernel<LCAP, SC, 1>;
        case 2: return (void*)polar_decode_kernel<LCAP, SC, 2>;
        case 3: return (void*)polar_decode_kernel<LCAP, SC, 3>;
        default: return (void*)polar_decode_kernel<LCAP, SC, 4>;
    }
}

static void* pick_kernel(const PolarGeom& g, bool sc) {
    if (sc) return pick_f<1, true>(g.F);
    switch (g.lcap) {
        case 1: return pick_f<1, false>(g.F);
        case 2: return pick_f<2, false>(g.F);
        case 4: return pick_f<4, false>(g.F);
        case 8: return pick_f<8, false>(g.F);
        case 16: return pick_f<16, false>(g.F);
        case 32: return pick_f<32, false>(g.F);
        default: return nullptr;
    }
}

hipError_t polar_prepare(const PolarGeom& g, bool sc) {
    void* k = pick_kernel(g, sc);
    if (!k) return hipErrorInvalidValue;
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, g.lds_bytes);
}

hipError_t polar_launch(const PolarGeom& g, bool sc, const double* llr, int64_t ld, uint8_t* out,
                        const uint32_t* frozen_dec, const int32_t* info_pos, int64_t batch,
                        hipStream_t s) {
    void* k = pick_kernel(g, sc);
    if (!k) return hipErrorInvalidValue;
    const int64_t maxgrid = 1ll << 30;
    for (int64_t b0 = 0; b0 < batch; b0 += maxgrid) {
        const int64_t nb = (batch - b0) < maxgrid ? (batch - b0) : maxgrid;
        PolarGeom gg = g;
        const double* l = llr + b0 * ld;
        uint8_t* o = out + b0 * g.K;
        void* args[] = {&gg, (void*)&l, (void*)&ld, (void*)&o, (void*)&frozen_dec, (void*)&info_pos,
                        (void*)&nb};
        hipError_t e = hipLaunchKernel(k, dim3((unsigned)nb), dim3(64), args, g.lds_bytes, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace pl
