// polar_fpw.hip -- DIAGNOSTIC ONLY (make DIAG=1): the frame-per-wavefront SCL
// mapping, built to measure it against the product's lane-per-path tree kernel
// (DESIGN.md §4.1 "frame per wavefront, measured").
//
// One wavefront decodes one N=1024 frame with an L=8 list: eight lanes per
// path (lane = 8 p + s), so every descent level runs eight lanes wide on a
// path's array; all LLR pools of depths 3..9 (254 doubles per path slot, 16 KB
// per frame), the partial sums and the list bookkeeping live in LDS -- no
// workspace traffic at all; depths 1..2 are recomputed from the channel when a
// descent reaches depth 3 (the product's fused top); the leaf LLR, the metric
// and the pointer row of a path are computed redundantly by its eight lanes.
// Same f / g / metric arithmetic as the product (polar_common.hpp), stable
// ranks over the 16 candidates through LDS, pointer rows as the product's
// (a clone copies a row; a path only writes its own slot), so the decoded bits
// match the product kernel's on frames without NaN metrics.  s_memtime stamps
// per phase: descent, metric, prune, partial-sum walk, output.
#include "common.hpp"
#include "internal.hpp"
#include "polar_common.hpp"

namespace pl {

#if PL_DIAG

namespace {

constexpr int FN = 10, FNN = 1 << FN, FL = 8;
// LDS layout (bytes) of one wavefront
PL_DEV constexpr int fpw_S(int d) { return FNN >> d; }
PL_DEV constexpr int fpw_pool_off(int d) {  // pools of depths 3..9, [slot][S_d] f64
    int o = 0;
    for (int k = 3; k < d; ++k) o += FL * fpw_S(k) * 8;
    return o;
}
constexpr int FPW_POOL_BYTES = FL * (128 + 64 + 32 + 16 + 8 + 4 + 2) * 8;  // 16 256
PL_DEV constexpr int fpw_bw(int d) { return (FNN >> d) >= 32 ? (FNN >> d) / 32 : 1; }  // beta words of depth d
PL_DEV constexpr int fpw_beta_off(int d) {  // partial sums of depths 1..10, [slot][words] u32
    int o = FPW_POOL_BYTES;
    for (int k = 1; k < d; ++k) o += FL * fpw_bw(k) * 4;
    return o;
}
constexpr int FPW_WALK = FPW_POOL_BYTES + FL * (16 + 8 + 4 + 2 + 1 + 1 + 1 + 1 + 1 + 1) * 4;  // [path][2][32] u32
constexpr int FPW_MET = FPW_WALK + FL * 2 * 32 * 4;  // [8] double2
constexpr int FPW_ROW = FPW_MET + FL * 16;           // [8] u64 llr rows, [8] u64 beta rows
constexpr int FPW_SURV = FPW_ROW + FL * 16;          // [8] u32
constexpr int FPW_X = FPW_SURV + FL * 4;             // [32] u32 output transform
constexpr int FPW_LDS = FPW_X + 32 * 4;

PL_DEV int fld(uint64_t row, int d) { return (int)((row >> (4 * d)) & 15u); }
PL_DEV uint64_t fset(uint64_t row, int d, int v) { return (row & ~(15ull << (4 * d))) | ((uint64_t)v << (4 * d)); }
PL_DEV void wfence() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__global__ void __launch_bounds__(64) polar_fpw_kernel(const double* __restrict__ llr, int64_t ld,
                                                       uint8_t* __restrict__ out,
                                                       const uint32_t* __restrict__ frozen_dec,
                                                       const int32_t* __restrict__ info_pos, int64_t batch, int K,
                                                       unsigned long long* __restrict__ stamps) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x, p = lane >> 3, s = lane & 7;
    auto pool = [&](int d, int slot) { return reinterpret_cast<double*>(smem + fpw_pool_off(d)) + slot * fpw_S(d); };
    auto beta = [&](int d, int slot) { return reinterpret_cast<uint32_t*>(smem + fpw_beta_off(d)) + slot * fpw_bw(d); };
    uint32_t* const walk = reinterpret_cast<uint32_t*>(smem + FPW_WALK) + p * 64;  // [2][32] of this path
    double2* const met = reinterpret_cast<double2*>(smem + FPW_MET);
    uint64_t* const rowx = reinterpret_cast<uint64_t*>(smem + FPW_ROW);
    uint32_t* const surv = reinterpret_cast<uint32_t*>(smem + FPW_SURV);
    uint32_t* const X = reinterpret_cast<uint32_t*>(smem + FPW_X);
    unsigned long long acc[5] = {0, 0, 0, 0, 0};
    unsigned long long tp = __builtin_amdgcn_s_memtime();
#define FSTAMP(k)                                                 \
    {                                                             \
        const unsigned long long tn = __builtin_amdgcn_s_memtime(); \
        acc[k] += tn - tp;                                        \
        tp = tn;                                                  \
    }
    for (int64_t frame = blockIdx.x; frame < batch; frame += gridDim.x) {
        const double* __restrict__ ch = llr + frame * ld;
        uint64_t lrow = 0, brow = 0;  // every field = slot 0 (path 0's)
        double pm = p == 0 ? 0.0 : -INFINITY;
        int nact = 1, par = 0;
        for (int i = 0; i < FNN; ++i) {
            // ---------------------------------------------------- descent
            const int dstart = i == 0 ? 1 : FN - __builtin_ctz(i);
            const bool act = p < nact;
            int d = dstart;
            if (dstart <= 3) {
                // depth-3 node of this path from the channel: 16 outputs per lane
                const bool r1 = (i >> 9) & 1, r2 = (i >> 8) & 1, r3 = (i >> 7) & 1;
                const uint32_t* b1 = beta(1, fld(brow, 1));
                const uint32_t* b2 = beta(2, fld(brow, 2));
                const uint32_t* b3 = beta(3, fld(brow, 3));
                double* C = pool(3, p);
                for (int t = s; t < 128; t += 8) {
                    double v[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[k] = ch[8 * t + k];
                    const int e1 = 4 * t, e2 = 2 * t;
                    const uint32_t w1 = r1 ? b1[e1 >> 5] >> (e1 & 31) : 0u, w2 = r2 ? b2[e2 >> 5] >> (e2 & 31) : 0u;
                    const uint32_t w3 = r3 ? b3[t >> 5] >> (t & 31) : 0u;
#pragma unroll
                    for (int k = 0; k < 4; ++k) v[k] = r1 ? g_op(v[2 * k], v[2 * k + 1], w1 >> k) : f_ms(v[2 * k], v[2 * k + 1]);
#pragma unroll
                    for (int k = 0; k < 2; ++k) v[k] = r2 ? g_op(v[2 * k], v[2 * k + 1], w2 >> k) : f_ms(v[2 * k], v[2 * k + 1]);
                    const double o = r3 ? g_op(v[0], v[1], w3) : f_ms(v[0], v[1]);
                    if (act) C[t] = o;
                }
                lrow = fset(lrow, 3, p);
                d = 4;
                wfence();
            }
            for (; d <= 9; ++d) {
                const int S = fpw_S(d);
                const bool right = d == dstart && ((i >> (FN - d)) & 1);
                const double* P = pool(d - 1, fld(lrow, d - 1));
                double* C = pool(d, p);
                const uint32_t* bl = beta(d, fld(brow, d));
                for (int t = s; t < S; t += 8) {
                    const double a = P[2 * t], b = P[2 * t + 1];
                    const double o = right ? g_op(a, b, bl[t >> 5] >> (t & 31)) : f_ms(a, b);
                    if (act) C[t] = o;
                }
                lrow = fset(lrow, d, p);
                wfence();
            }
            double lam;
            {
                const double* P = pool(9, fld(lrow, 9));
                const double a = P[0], b = P[1];
                lam = (i & 1) ? g_op(a, b, beta(10, fld(brow, 10))[0]) : f_ms(a, b);
            }
            FSTAMP(0);
            // ---------------------------------------------------- decision
            const bool frozen = (frozen_dec[i >> 5] >> (i & 31)) & 1u;
            int bit = 0;
            double m0, m1;
            path_metrics_fast<true, (FN <= PL_METRIC_FUSED_NMAX)>(pm, lam, act, m0, m1);
            FSTAMP(1);
            if (frozen) {
                if (act) pm = m0;
            } else {
                if (s == 0) {
                    met[p] = make_double2(m0, m1);
                    rowx[2 * p] = lrow;
                    rowx[2 * p + 1] = brow;
                }
                wfence();
                int r0 = 0, r1 = 0;
                for (int q = 0; q < nact; ++q) {
                    const double2 v = met[q];
                    r0 += (v.x > m0) | ((v.x == m0) & (q < p));
                    r0 += v.y > m0;
                    r1 += v.x >= m1;
                    r1 += (v.y > m1) | ((v.y == m1) & (q < p));
                }
                const int nsurv = 2 * nact < FL ? 2 * nact : FL;
                if (s == 0 && act) {
                    if (r0 < nsurv) surv[r0] = (uint32_t)(p << 1);
                    if (r1 < nsurv) surv[r1] = (uint32_t)((p << 1) | 1);
                }
                wfence();
                if (p < nsurv) {
                    const uint32_t e = surv[p];
                    const int q = (int)(e >> 1);
                    bit = (int)(e & 1u);
                    const double2 v = met[q];
                    pm = bit ? v.y : v.x;
                    lrow = rowx[2 * q];
                    brow = rowx[2 * q + 1];
                } else {
                    pm = -INFINITY;
                }
                nact = nsurv;
                wfence();
            }
            FSTAMP(2);
            // ---------------------------------------------------- partial sums
            {
                const int to = __builtin_ctz(~(unsigned)i);
                const int steps = to < FN ? to : FN;
                int dd = FN, k = 0;
                uint32_t cur = (uint32_t)bit;
                for (; k < steps && k < 5; ++k) {
                    const uint32_t left = beta(dd, fld(brow, dd))[0];
                    const uint32_t msk = (1u << (1 << k)) - 1u;
                    cur = spread16((left ^ cur) & msk) | (spread16(cur & msk) << 1);
                    --dd;
                }
                if (k == steps) {
                    if (dd > 0) {
                        if (s == 0 && p < nact) beta(dd, p)[0] = cur;
                        brow = fset(brow, dd, p);
                    } else {
                        if (s == 0 && p < nact) walk[0] = cur;
                        par = 0;
                    }
                } else {
                    // multi-word depths: the path's lanes split the output words
                    int pr = 0;
                    if (s == 0 && p < nact) walk[0] = cur;
                    wfence();
                    for (; k < steps; ++k) {
                        const int cwc = 1 << (k - 5);  // input words
                        const uint32_t* lsrc = beta(dd, fld(brow, dd));
                        const bool last = k + 1 == steps;
                        uint32_t* dst = (last && dd - 1 > 0) ? beta(dd - 1, p) : walk + (pr ^ 1) * 32;
                        for (int w = s; w < 2 * cwc; w += 8) {
                            const uint32_t cv = walk[pr * 32 + (w >> 1)], lv = lsrc[w >> 1];
                            const int sh = (w & 1) * 16;
                            const uint32_t r = spread16((lv ^ cv) >> sh) | (spread16(cv >> sh) << 1);
                            if (p < nact) dst[w] = r;
                        }
                        pr ^= 1;
                        --dd;
                        wfence();
                    }
                    if (dd > 0) brow = fset(brow, dd, p);
                    else par = pr;
                }
                wfence();
            }
            FSTAMP(3);
        }
        // -------------------------------------------------------- output
        int best = 0;
        {
            if (s == 0) met[p] = make_double2(pm, 0.0);
            wfence();
            double bm = met[0].x;
            for (int q = 1; q < nact; ++q) {
                const double v = met[q].x;
                if (v > bm) { bm = v; best = q; }
            }
        }
        const uint32_t* root = reinterpret_cast<uint32_t*>(smem + FPW_WALK) + best * 64 + par * 32;
        if (lane < 32) X[lane] = polar_word_transform(root[lane]);
        wfence();
        for (int sw = 1; sw < 32; sw <<= 1) {
            uint32_t v = 0;
            if (lane < 32 && !(lane & sw)) v = X[lane] ^ X[lane + sw];
            wfence();
            if (lane < 32 && !(lane & sw)) X[lane] = v;
            wfence();
        }
        uint8_t* o = out + frame * (int64_t)K;
        for (int k = lane; k < K; k += 64) {
            const int ps = info_pos[k];
            o[k] = (uint8_t)((X[ps >> 5] >> (ps & 31)) & 1u);
        }
        wfence();
        FSTAMP(4);
    }
    if (stamps && lane == 0)
        for (int k = 0; k < 5; ++k) atomicAdd(stamps + k, acc[k]);
#undef FSTAMP
}

}  // namespace

hipError_t fpw_launch(const double* llr, int64_t ld, uint8_t* out, const uint32_t* frozen_dec,
                      const int32_t* info_pos, int64_t batch, int K, unsigned long long* stamps, int grid,
                      hipStream_t st) {
    hipError_t e = hipFuncSetAttribute((const void*)polar_fpw_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       FPW_LDS);
    if (e != hipSuccess) return e;
    if (grid <= 0) {
        int nb = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)polar_fpw_kernel, 64, FPW_LDS);
        if (e != hipSuccess) return e;
        hipDeviceProp_t prop;
        int dev = 0;
        hipGetDevice(&dev);
        hipGetDeviceProperties(&prop, dev);
        grid = (nb < 1 ? 1 : nb) * prop.multiProcessorCount;
    }
    if (grid > batch) grid = (int)batch;
    void* args[] = {(void*)&llr, (void*)&ld, (void*)&out, (void*)&frozen_dec, (void*)&info_pos, (void*)&batch,
                    (void*)&K, (void*)&stamps};
    return hipLaunchKernel((const void*)polar_fpw_kernel, dim3((unsigned)grid), dim3(64), args, FPW_LDS, st);
}

#endif  // PL_DIAG

}  // namespace pl
