// polar_nan.hip -- SCL frames whose path metrics became NaN, decoded again with
// the reference's own candidate order.
//
// +-inf LLRs meeting in a g give inf - inf = NaN (src/polar/decoder.py:412-417),
// and a NaN LLR gives NaN metrics (:374-406).  The reference then orders its
// candidates with list.sort(key=metric, reverse=True) (:306-307), where NaN keys
// compare false both ways, and picks np.argmax of the final metrics (:258), the
// first NaN.  The fast list kernels (polar_tree.hip, polar_lane.hpp) rank
// candidates in parallel, which is the stable descending order only for
// comparable keys; a frame in which any active path's candidate or final metric
// is NaN is flagged in a per-(wavefront, pass) mask.  This kernel reads the
// masks and decodes each flagged frame again: one workgroup per frame, the list
// state in global scratch, thread 0 running CPython's sort (pysort.hpp) on the
// candidates, survivors renumbered in that order, argmax = first NaN else first
// maximum.  f, g and the metric increments are the list kernels' own
// (polar_common.hpp), each frame with the metric evaluation of the kernel that
// flagged it (RedoArgs::metric: the lane kernel's libm-style log1p(exp(-x)),
// or the tree instance's fused / lean one), so on finite values a flagged frame
// decodes exactly as that kernel decodes it.
//
// Scratch per workgroup (nan_redo_unit): for each of the L physical path
// buffers, the LLR arrays of depths 1..n (N - 1 doubles: depth d at offset
// N - (N >> (d - 1)), 2^(n-d) values), the partial sums of the last completed
// node at each depth (N - 1 bytes, same offsets), and two N-byte walk buffers.
// A clone claims its parent's buffer if no earlier survivor did, else copies it
// into a buffer no survivor uses (Tal & Vardy's lazy copy without reference
// counts: at most one copy per extra child).
//
// The same kernel, launched without masks, is the decoder of lists above 1024
// paths (the list kernels hold one lane per path in one workgroup): every
// frame, one workgroup each.  Up to kMaxRedoList paths the frame's list state
// (candidates, sort scratch, metrics, buffer tables: lds_frame_bytes) sits in
// LDS; above that (polar_nan_redo_kernel<true>, lists of up to kMaxListSize
// paths) it sits in the workgroup's global scratch after the path buffers --
// the same code on flat pointers, a correctness path like the rest of this file.
#include <algorithm>
#include <mutex>

#include "common.hpp"
#include "internal.hpp"
#include "polar_common.hpp"
#include "pysort.hpp"

namespace pl {

namespace {

constexpr int kRedoThreads = 256;

struct RedoArgs {
    const double* llr;
    int64_t ld;
    uint8_t* out;
    int64_t batch;  // frames of this launch (chunk)
    int N, n, K, Lsz;
    const uint32_t* frozen_dec;
    const int32_t* info_pos;
    const uint32_t* crc_g;   // CA-SCL table, or null
    uint64_t* masks;         // [grid][kNanMaskPasses]: bit f of word p = frame f of pass p flagged
    int grid, fpw;           // the list kernel's grid and frames per wavefront
    int metric;              // RedoMetric of the kernel whose frames these are
    unsigned char* scratch;  // nan_redo_unit bytes per redo workgroup
    size_t unit;
};

PL_DEV int dep_off(int N, int d) { return N - (N >> (d - 1)); }

// LDS of redo_frame: candidates [2L] + sort scratch [L+1] (16 B items), metrics
// [L] f64, five [L] int arrays, four shared ints
__host__ __device__ inline size_t lds_frame_bytes(int L) {
    const size_t b = sizeof(PsItem) * (3 * (size_t)L + 1) + 8 * (size_t)L + 4 * (5 * (size_t)L + 4);
    return (b + 15) & ~(size_t)15;
}

struct Bufs {
    unsigned char* base;
    int N;
    size_t pbytes;  // bytes per physical path buffer
    PL_DEV double* llr(int b) const { return reinterpret_cast<double*>(base + (size_t)b * pbytes); }
    PL_DEV uint8_t* beta(int b) const { return base + (size_t)b * pbytes + (size_t)8 * (N - 1 > 0 ? N - 1 : 1); }
    PL_DEV uint8_t* walk(int b, int par) const {
        return beta(b) + (N - 1 > 0 ? N - 1 : 1) + (size_t)par * N;
    }
};

__host__ __device__ inline size_t path_bytes(int N) {
    const size_t e = (size_t)(N - 1 > 0 ? N - 1 : 1);
    return (8 * e + e + 2 * (size_t)N + 15) & ~(size_t)15;
}

// one frame, all threads of the workgroup; smem = the frame state (LDS or scratch)
PL_DEV void redo_frame(const RedoArgs& a, int64_t frame, const Bufs& bf, unsigned char* smem) {
    const int N = a.N, n = a.n, L = a.Lsz, tid = threadIdx.x;
    PsItem* cand = reinterpret_cast<PsItem*>(smem);               // [2L]
    PsItem* tmp = cand + 2 * L;                                    // [L + 1]
    double* pm = reinterpret_cast<double*>(tmp + L + 1);           // [L]
    int* phys = reinterpret_cast<int*>(pm + L);                    // [L]
    int* nphys = phys + L;                                         // [L]
    int* src = nphys + L;                                          // [L] copy source buffer or -1
    int* nbit = src + L;                                           // [L]
    int* flag = nbit + L;                                          // [L] claimed / used scratch
    int* shared = flag + L;                                        // [4]
    const double* ch = a.llr + frame * a.ld;

    for (int p = tid; p < L; p += kRedoThreads) {
        phys[p] = p;
        pm[p] = p == 0 ? 0.0 : -INFINITY;
    }
    __syncthreads();
    int nact = 1;
    int par_root = 0;
    for (int i = 0; i < N; ++i) {
        // ---- LLRs of every active path down to leaf i
        const int dstart = i == 0 ? 1 : n - __builtin_ctz(i);
        for (int d = dstart; d <= n; ++d) {
            const int sh = n - d, S = 1 << sh;
            const bool right = (i >> (n - d)) & 1;
            for (int idx = tid; idx < nact * S; idx += kRedoThreads) {
                const int p = idx >> sh, t = idx & (S - 1);
                const int b = phys[p];
                const double* P = d == 1 ? ch : bf.llr(b) + dep_off(N, d - 1);
                const double x0 = P[2 * t], x1 = P[2 * t + 1];
                double* C = bf.llr(b) + dep_off(N, d);
                C[t] = right ? g_op(x0, x1, bf.beta(b)[dep_off(N, d) + t]) : f_ms(x0, x1);
            }
            __syncthreads();
        }
        // ---- decision
        const bool frozen = (a.frozen_dec[i >> 5] >> (i & 31)) & 1u;
        if (frozen) {
            for (int p = tid; p < nact; p += kRedoThreads) {
                const double lam = bf.llr(phys[p])[dep_off(N, n)];
                double m0, m1;
                if (a.metric == kRedoMetricFused) path_metrics_fast<false, true>(pm[p], lam, true, m0, m1);
                else if (a.metric == kRedoMetricLean) path_metrics_fast<false, false>(pm[p], lam, true, m0, m1);
                else path_metrics<false>(pm[p], lam, m0, m1);
                pm[p] = m0;
                nbit[p] = 0;
            }
            __syncthreads();
        } else {
            for (int p = tid; p < nact; p += kRedoThreads) {
                const double lam = bf.llr(phys[p])[dep_off(N, n)];
                double m0, m1;
                if (a.metric == kRedoMetricFused) path_metrics_fast<true, true>(pm[p], lam, true, m0, m1);
                else if (a.metric == kRedoMetricLean) path_metrics_fast<true, false>(pm[p], lam, true, m0, m1);
                else path_metrics<true>(pm[p], lam, m0, m1);
                cand[p] = PsItem{m0, p, 0};             // path_metrics_0 (decoder.py:300-303)
                cand[nact + p] = PsItem{m1, nact + p, 0};  // path_metrics_1, after every bit-0 candidate
            }
            __syncthreads();
            const int ns = 2 * nact < L ? 2 * nact : L;
            if (tid == 0) {
                py_sort_desc(cand, 2 * nact, tmp);
                for (int q = 0; q < L; ++q) flag[q] = 0;  // q < nact: parent claimed; buffer used
                for (int k = 0; k < ns; ++k) {
                    const int v = cand[k].v, q = v < nact ? v : v - nact;
                    if (!(flag[q] & 1)) {
                        flag[q] |= 1;
                        nphys[k] = phys[q];
                        src[k] = -1;
                    } else {
                        src[k] = phys[q];
                    }
                    nbit[k] = v >= nact;
                    pm[k] = cand[k].k;
                }
                // buffers of unclaimed parents and never-used slots take the copies
                int fi = 0;
                for (int k = 0; k < ns; ++k) {
                    if (src[k] < 0) continue;
                    while (fi < L && fi < nact && (flag[fi] & 1)) ++fi;
                    nphys[k] = phys[fi];  // fi < nact: an unclaimed parent; else an unused slot
                    ++fi;
                }
                for (int k = 0; k < L; ++k) flag[k] = 0;
                for (int k = 0; k < ns; ++k) flag[nphys[k]] = 1;
                int u = ns;
                for (int b = 0; b < L; ++b)
                    if (!flag[b]) nphys[u++] = b;
                for (int k = 0; k < L; ++k) phys[k] = nphys[k];
                for (int k = ns; k < L; ++k) pm[k] = -INFINITY;
            }
            __syncthreads();
            // clones: copy the parent's arrays (partial sums included) into the new buffer
            const int E = N - 1 > 0 ? N - 1 : 1;
            for (int k = 0; k < ns; ++k) {
                const int s = src[k];
                if (s < 0) continue;
                const int b = phys[k];
                for (int e = tid; e < E; e += kRedoThreads) {
                    bf.llr(b)[e] = bf.llr(s)[e];
                    bf.beta(b)[e] = bf.beta(s)[e];
                }
            }
            nact = ns;
            __syncthreads();
        }
        // ---- partial sums: walk up the trailing ones of i
        const int to = __builtin_ctz(~(unsigned)i);
        const int steps = to < n ? to : n;
        for (int p = tid; p < nact; p += kRedoThreads) bf.walk(phys[p], 0)[0] = (uint8_t)nbit[p];
        __syncthreads();
        int par = 0, dd = n;
        for (int s = 0; s < steps; ++s) {
            const int S = 1 << s;
            for (int idx = tid; idx < nact * S; idx += kRedoThreads) {
                const int p = idx >> s, t = idx & (S - 1);
                const int b = phys[p];
                const uint8_t c = bf.walk(b, par)[t], l = bf.beta(b)[dep_off(N, dd) + t];
                bf.walk(b, par ^ 1)[2 * t] = l ^ c;
                bf.walk(b, par ^ 1)[2 * t + 1] = c;
            }
            par ^= 1;
            --dd;
            __syncthreads();
        }
        if (dd > 0) {
            const int S = 1 << steps;
            for (int idx = tid; idx < nact * S; idx += kRedoThreads) {
                const int p = idx >> steps, t = idx & (S - 1);
                const int b = phys[p];
                bf.beta(b)[dep_off(N, dd) + t] = bf.walk(b, par)[t];
            }
            __syncthreads();
        } else {
            par_root = par;
        }
    }

    // ---- best path: np.argmax (first NaN, else first maximum); CA-SCL: the first
    // path in list.sort(key=metric, reverse=True) order whose CRC is 0
    int* best_p = shared;
    if (a.crc_g) {
        for (int p = tid; p < nact; p += kRedoThreads) {
            const uint8_t* x = bf.walk(phys[p], par_root);
            uint32_t crc = 0;
            for (int j = 0; j < N; ++j) crc ^= x[j] ? a.crc_g[j] : 0u;
            src[p] = (int)crc;
        }
        __syncthreads();
    }
    if (tid == 0) {
        int best = 0;
        for (int p = 1; p < L && !__builtin_isnan(pm[best]); ++p)
            if (__builtin_isnan(pm[p]) || pm[p] > pm[best]) best = p;
        if (a.crc_g) {
            for (int p = 0; p < nact; ++p) cand[p] = PsItem{pm[p], p, 0};
            py_sort_desc(cand, nact, tmp);
            for (int k = 0; k < nact; ++k)
                if (src[cand[k].v] == 0) {
                    best = cand[k].v;
                    break;
                }
        }
        *best_p = best;
    }
    __syncthreads();
    const int bb = phys[*best_p];
    // u = x_hat F^{(x)n}: butterflies in the other walk buffer, then u[info]
    uint8_t* u = bf.walk(bb, par_root ^ 1);
    for (int j = tid; j < N; j += kRedoThreads) u[j] = bf.walk(bb, par_root)[j];
    __syncthreads();
    for (int h = 1; h < N; h <<= 1) {
        for (int idx = tid; idx < N / 2; idx += kRedoThreads) {
            const int j = (idx / h) * 2 * h + idx % h;
            u[j] ^= u[j + h];
        }
        __syncthreads();
    }
    uint8_t* o = a.out + frame * (int64_t)a.K;
    for (int k = tid; k < a.K; k += kRedoThreads) o[k] = u[a.info_pos[k]];
    __syncthreads();
}

template <bool GSTATE>
__global__ void __launch_bounds__(kRedoThreads) polar_nan_redo_kernel(RedoArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const Bufs bf{a.scratch + (size_t)blockIdx.x * a.unit, a.N, path_bytes(a.N)};
    if constexpr (GSTATE) {  // lists above kMaxRedoList: state after the path buffers, every frame here
        unsigned char* const st = bf.base + (size_t)a.Lsz * bf.pbytes;
        for (int64_t f = blockIdx.x; f < a.batch; f += gridDim.x) redo_frame(a, f, bf, st);
        return;
    }
    // flagged (mask, first frame) pairs of one scan round, after the frame state
    uint64_t* const xw = reinterpret_cast<uint64_t*>(smem + lds_frame_bytes(a.Lsz));
    int* const xn = reinterpret_cast<int*>(xw + 2 * kRedoThreads);
    if (a.masks == nullptr) {  // lists above 1024: every frame here
        for (int64_t f = blockIdx.x; f < a.batch; f += gridDim.x) redo_frame(a, f, bf, smem);
        return;
    }
    const int64_t stride_frames = (int64_t)a.grid * a.fpw;
    // mask words of wavefronts w = blockIdx.x, + gridDim.x, ...: 256 at a time
    const int64_t wpb = (a.grid + gridDim.x - 1) / gridDim.x;  // wavefronts of this workgroup (at most)
    for (int64_t r0 = 0; r0 < wpb * kNanMaskPasses; r0 += kRedoThreads) {
        if (threadIdx.x == 0) *xn = 0;
        __syncthreads();
        const int64_t r = r0 + threadIdx.x;
        const int64_t w = (int64_t)blockIdx.x + (r / kNanMaskPasses) * gridDim.x;
        const int p = (int)(r % kNanMaskPasses);
        if (r < wpb * kNanMaskPasses && w < a.grid) {
            // pass p of wavefront w ran iff its first frame is inside the batch
            const int64_t f0 = w * a.fpw + (int64_t)p * stride_frames;
            if (f0 < a.batch) {
                uint64_t* const mw = a.masks + w * kNanMaskPasses + p;
                const uint64_t m = *mw;
                if (m) {
                    *mw = 0ull;  // zero for the next decode (the list kernels only OR)
                    const int slot = atomicAdd(xn, 1);
                    xw[2 * slot] = m;
                    xw[2 * slot + 1] = (uint64_t)f0;
                }
            }
        }
        __syncthreads();
        const int cnt = *xn;
        for (int e = 0; e < cnt; ++e) {
            uint64_t m = xw[2 * e];
            const int64_t f0 = (int64_t)xw[2 * e + 1];
            while (m) {
                const int f = __builtin_ctzll(m);
                m &= m - 1;
                if (f0 + f < a.batch) redo_frame(a, f0 + f, bf, smem);
            }
        }
        __syncthreads();
    }
}

}  // namespace

size_t nan_redo_unit(int N, int list_size) {
    return path_bytes(N) * (size_t)list_size + (list_size > kMaxRedoList ? lds_frame_bytes(list_size) : 0);
}

int nan_redo_lds_bytes(int list_size) {
    return list_size > kMaxRedoList ? 0 : (int)(lds_frame_bytes(list_size) + 16 * kRedoThreads + 16);
}

// The kernel's dynamic-LDS limit is a per-function attribute: raise it to what
// this plan's list needs (never lower it under another plan), per device.
hipError_t nan_redo_prepare(int list_size) {
    static std::mutex mu;
    static int set_bytes[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const int need = nan_redo_lds_bytes(list_size);
    if (list_size > kMaxRedoList) return hipSuccess;  // state in scratch, no dynamic LDS
    std::lock_guard<std::mutex> lk(mu);
    if (dev >= 0 && dev < 64 && need <= set_bytes[dev]) return hipSuccess;
    int optin = 0;
    if ((e = hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev)) != hipSuccess) return e;
    if (need > optin) return hipErrorInvalidValue;  // this list's state does not fit the device's LDS
    e = hipFuncSetAttribute((const void*)polar_nan_redo_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, need);
    if (e == hipSuccess && dev >= 0 && dev < 64) set_bytes[dev] = need;
    return e;
}

hipError_t nan_redo_launch(const double* llr, int64_t ld, uint8_t* out, int64_t batch, int N, int K, int Lsz,
                           const uint32_t* frozen_dec, const int32_t* info_pos, const uint32_t* crc_g,
                           uint64_t* masks, int grid, int fpw, int metric, unsigned char* scratch,
                           size_t scratch_bytes, int max_blocks, hipStream_t s) {
    int n = 0;
    while ((1 << n) < N) ++n;
    RedoArgs a{llr, ld, out, batch, N, n, K, Lsz, frozen_dec, info_pos, crc_g, masks, grid, fpw, metric, scratch,
               nan_redo_unit(N, Lsz)};
    const int64_t fit = (int64_t)(scratch_bytes / a.unit);
    // masks: one workgroup per list-kernel wavefront at most; no masks: per frame
    const int64_t want = masks ? (int64_t)grid : batch;
    int blocks = (int)std::min<int64_t>(std::min<int64_t>(want, fit), max_blocks);
    if (blocks < 1) return hipErrorInvalidValue;
    void* args[] = {(void*)&a};
    if (Lsz > kMaxRedoList) {
        if (masks) return hipErrorInvalidValue;  // such lists decode every frame here, never flagged
        return hipLaunchKernel((const void*)polar_nan_redo_kernel<true>, dim3((unsigned)blocks), dim3(kRedoThreads),
                               args, 0, s);
    }
    return hipLaunchKernel((const void*)polar_nan_redo_kernel<false>, dim3((unsigned)blocks), dim3(kRedoThreads),
                           args, nan_redo_lds_bytes(Lsz), s);
}

}  // namespace pl
