// C-ABI of libpolarldpc.so (include/polarldpc.h): plan lifetime, argument
// checking (mirroring the reference's assertions), dispatch to the kernels.
#include "../../include/polarldpc.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "internal.hpp"

// Device workspace of one stream (polar: per resident wavefront; LDPC codes
// whose messages exceed LDS: per frame of a chunk).  Grown lazily to the batch.
// Its own mutex serialises the decodes of that stream only, so a stream that
// drains and regrows its buffer never stalls decodes on other streams.
struct Workspace {
    std::mutex mu;
    void* ptr = nullptr;
    // written under `mu`; atomic so pl_plan_workspace_stats may read it under the map mutex only
    std::atomic<size_t> bytes{0};
    // after an out-of-memory fallback: the request that did not fit.  Later decodes
    // needing no more than it run on the smaller buffer (decode_impl clamps the grid)
    // instead of draining and retrying the allocation every call; pl_plan_reserve,
    // or a larger request, retries.
    size_t failed_need = 0;
    ~Workspace() {
        if (ptr) hipFree(ptr);  // hipFree waits for work that still uses it
    }
};

struct pl_plan {
    int kind = 0;  // 0 polar, 1 ldpc
    int device = 0;
    // polar
    pl::PolarGeom pg{};  // N, K, F, lds_bytes of the chosen kernel
    bool sc = false;
    int list_size = 0;
    uint32_t* d_frozen_dec = nullptr;  // decode-order frozen bitmask [ceil(N/32)]
    int32_t* d_info_pos = nullptr;     // [K] ascending info indices
    uint32_t* d_crc_g = nullptr;       // CA-SCL: CRC contribution of x_hat bit j [N] (null = plain SCL)
    uint32_t* d_r0k = nullptr;         // SC tree kernel: log2 size of the largest all-frozen node at leaf i (4-bit fields)
    std::vector<int32_t> h_info;       // ascending info positions (host copy)
    bool tree = false;      // compile-time-geometry kernel (polar_tree.hip); else polar_lane.hip
    pl::TreeInfo tinfo{};
    // the small-batch tree instance (polar_tree.hip tree_table_small): used for a
    // decode whose wavefronts all fit the device at its occupancy, small_grid_max
    bool tree_small = false;
    pl::TreeInfo tinfo_small{};
    int small_grid_max = 0;
    pl::LaneGeom lgeo{};
    int fpw = 1;            // frames per wavefront
    int lane_grid_max = 0;  // resident wavefronts (persistent grid)
    // ldpc
    pl::LdpcGeom lg{};
    pl::LdpcDev ld{};
    int32_t* d_ldpc = nullptr;
    int64_t ldpc_chunk = 16384;  // frames per launch of the global-workspace kernel
    // workspace: bytes per unit (polar: one resident wave; LDPC global: one
    // frame), one buffer per stream (plans are shared across host threads that
    // use distinct streams; a decode only ever touches its stream's buffer)
    size_t ws_unit = 0;
    // polar list decoders: NaN-frame masks (kNanMaskPasses u64 per resident
    // wavefront, at the start of the workspace) and the scratch one workgroup of
    // polar_nan_redo_kernel needs (it reuses the list kernel's slices after it)
    size_t mask_bytes = 0, redo_unit = 0;
    size_t head_bytes = 0;  // polar: NaN masks + the tree kernel's frame-group counter, before the slices
    bool generic = false;  // list_size > 1024: polar_nan.hip decodes every frame
    int redo_blocks = 0;
    std::mutex mu;  // guards the map only; each entry has its own mutex
    std::unordered_map<hipStream_t, std::shared_ptr<Workspace>> ws;
};

static thread_local std::string g_err;

// HIP caps a launch at 2^32 work-items per grid dimension; per-frame kernels
// (one workgroup per frame) are launched in chunks below 2^31 work-items.
constexpr int64_t kMaxLaunchItems = 1LL << 31;

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
static int hipfail(hipError_t e, const char* what) {
    return fail(e == hipErrorOutOfMemory ? PL_ENOMEM : PL_EHIP,
                std::string(what) + ": " + hipGetErrorString(e));
}

extern "C" const char* pl_last_error(void) { return g_err.c_str(); }

static int bitrev(int v, int nb) {
    int r = 0;
    for (int i = 0; i < nb; ++i) { r = (r << 1) | (v & 1); v >>= 1; }
    return r;
}

template <typename T>
static hipError_t upload(T** dst, const std::vector<T>& src) {
    const size_t bytes = (src.empty() ? 1 : src.size()) * sizeof(T);
    hipError_t e = hipMalloc((void**)dst, bytes);
    if (e != hipSuccess) return e;
    if (!src.empty()) e = hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
    return e;
}

static int env_int(const char* name, int dflt) {
    const char* s = std::getenv(name);
    return (s && *s) ? std::atoi(s) : dflt;
}

// Every call that touches a plan's device memory must run on the plan's device
// (the one current at plan creation): a workspace allocated, or a kernel
// launched, on another device would use foreign pointers.
static int check_device(const pl_plan* p) {
    int cur = -1;
    const hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess) return hipfail(e, "hipGetDevice");
    if (cur != p->device)
        return fail(PL_EINVAL, "current device " + std::to_string(cur) + " is not the plan's device " +
                                   std::to_string(p->device) + " (hipSetDevice first)");
    return PL_OK;
}

// the metric evaluation of the list kernel a plan's NaN frames come from (polar_nan.hip)
static int redo_metric(const pl_plan* p) {
    if (!p->tree && !p->generic) return pl::kRedoMetricLane;
    return p->pg.N <= (1 << PL_METRIC_FUSED_NMAX) ? pl::kRedoMetricFused : pl::kRedoMetricLean;
}

// ldpc_bp_grp_kernel's variable -> thread-slot map (slot q = 256 j + tid;
// nslots >= n, -1 = empty).  The variable pass stores T'[tpos] (ds_write_b64:
// lane groups of 16, bank pair tpos mod 16) and reads C'[tpos] (ds_read_b64:
// lane groups of 32, element (tl + tpos) mod 32) for each of its DV edges; a
// group's cost is, per edge k, the largest number of its lanes on one bank.
// Greedy fill (each slot takes the unplaced variable that adds the fewest
// same-bank lanes to its two groups), then hill climbing over slot swaps
// (deterministic xorshift, sideways moves kept).  Any map gives the same
// decoding; only the LDS conflicts change (MI355X_MICROARCH.md, LDS).
static std::vector<int> ldpc_var_slots(int n, int dv, const std::vector<int32_t>& tp, int tl, int nslots) {
    std::vector<int> vm(nslots, -1);
    {
        std::vector<char> used(n, 0);
        std::vector<int> wcnt((size_t)dv * 16), rcnt((size_t)dv * 32);
        const int empty = nslots - n;  // empty slots go to the end of the last groups
        for (int q = 0; q < nslots - empty; ++q) {
            if ((q & 15) == 0) std::fill(wcnt.begin(), wcnt.end(), 0);
            if ((q & 31) == 0) std::fill(rcnt.begin(), rcnt.end(), 0);
            int best = -1, bc = 1 << 30;
            for (int v = 0; v < n; ++v) {
                if (used[v]) continue;
                int c = 0;
                for (int k = 0; k < dv; ++k) {
                    const int t = tp[(size_t)v * dv + k];
                    c += wcnt[(size_t)k * 16 + t % 16] + rcnt[(size_t)k * 32 + (t + tl) % 32];
                }
                if (c < bc) { bc = c; best = v; if (c == 0) break; }
            }
            used[best] = 1;
            vm[q] = best;
            for (int k = 0; k < dv; ++k) {
                const int t = tp[(size_t)best * dv + k];
                ++wcnt[(size_t)k * 16 + t % 16];
                ++rcnt[(size_t)k * 32 + (t + tl) % 32];
            }
        }
    }
    auto gcost = [&](int start, int size, int mod, int add) {
        int c = 0;
        for (int k = 0; k < dv; ++k) {
            int cnt[32] = {0}, mx = 0;
            for (int q = start; q < start + size; ++q) {
                const int v = vm[q];
                if (v < 0) continue;
                const int b = (tp[(size_t)v * dv + k] + add) % mod;
                mx = std::max(mx, ++cnt[b]);
            }
            c += mx;
        }
        return c;
    };
    auto groups_cost = [&](int a, int b) {
        const int wa = a & ~15, wb = b & ~15, ra = a & ~31, rb = b & ~31;
        int c = gcost(wa, 16, 16, 0) + gcost(ra, 32, 32, tl);
        if (wb != wa) c += gcost(wb, 16, 16, 0);
        if (rb != ra) c += gcost(rb, 32, 32, tl);
        return c;
    };
    uint64_t x = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    const int iters = 40 * nslots;
    for (int it = 0; it < iters; ++it) {
        const int a = (int)(rnd() % (uint64_t)nslots), b = (int)(rnd() % (uint64_t)nslots);
        if (a == b || (vm[a] < 0 && vm[b] < 0)) continue;
        const int before = groups_cost(a, b);
        std::swap(vm[a], vm[b]);
        if (groups_cost(a, b) > before) std::swap(vm[a], vm[b]);
    }
    return vm;
}

static int device_cus(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
        return prop.multiProcessorCount;
    return 256;
}

extern "C" int pl_polar_plan_create(int32_t N, int32_t K, const uint8_t* frozen_mask, int32_t list_size,
                                    int32_t flags, pl_plan** out) {
    if (!out) return fail(PL_EINVAL, "out is NULL");
    *out = nullptr;
    if (N < 2 || (N & (N - 1)) || N > (1 << pl::kMaxDepth))
        return fail(PL_EINVAL, "N must be a power of 2 in [2, 32768]");
    if (!(0 < K && K <= N)) return fail(PL_EINVAL, "K (info positions) must be in [1, N]");
    if (list_size < 0) return fail(PL_EINVAL, "list_size must be >= 1 (0 = SC)");
    if (list_size > pl::kMaxListSize || (int64_t)list_size * N > pl::kMaxListTimesN)
        return fail(PL_EUNSUPPORTED, "list_size > 65536 or list_size * N > 2^30 not supported by this build");
    if (!frozen_mask) return fail(PL_EINVAL, "frozen_mask is NULL");
    int n = 0;
    while ((1 << n) < N) ++n;
    std::vector<int32_t> info;
    for (int j = 0; j < N; ++j)
        if (!frozen_mask[j]) info.push_back(j);
    if ((int)info.size() != K) return fail(PL_EINVAL, "number of unfrozen positions != K");
    std::vector<uint32_t> fdec((N + 31) / 32, 0u);
    for (int i = 0; i < N; ++i)
        if (frozen_mask[bitrev(i, n)]) fdec[i >> 5] |= 1u << (i & 31);

    pl_plan* p = new pl_plan();
    p->kind = 0;
    p->h_info = info;
    p->sc = (list_size == 0);
    p->list_size = list_size;
    hipGetDevice(&p->device);
    const char* kern = std::getenv("PL_POLAR_KERNEL");
    int lcap = 1;
    while (lcap < (p->sc ? 1 : list_size)) lcap <<= 1;
    // lists above 1024 (one frame per workgroup no longer holds one lane per
    // path): every frame through the exact single-workgroup decoder of polar_nan.hip
    p->generic = list_size > 1024;
    p->tree = !p->generic && !(kern && std::string(kern) == "lane") && !(flags & 0x3F) &&
              pl::tree_lookup(n, lcap, p->sc, &p->tinfo);
    hipError_t e;
    if ((e = upload(&p->d_frozen_dec, fdec)) != hipSuccess || (e = upload(&p->d_info_pos, info)) != hipSuccess) {
        pl_plan_destroy(p);
        return hipfail(e, "plan upload");
    }
    p->pg.N = N;
    p->pg.K = K;
    if (p->tree && p->sc) {
        // r0k[i] (decode order): the largest k with i a multiple of 2^k (any k
        // for i = 0) and leaves i .. i + 2^k - 1 all frozen.  K >= 1 info bits,
        // so k < n <= 15: eight 4-bit fields per word, which the kernel reads
        // with scalar loads.
        std::vector<uint32_t> r0k((size_t)(N + 7) / 8, 0u);
        for (int i = 0; i < N; ++i) {
            int k = 0;
            while (k + 1 < n + 1 && (i & ((1 << (k + 1)) - 1)) == 0 && i + (1 << (k + 1)) <= N) {
                bool all = true;
                for (int t = i; t < i + (1 << (k + 1)) && all; ++t) all = (fdec[t >> 5] >> (t & 31)) & 1u;
                if (!all) break;
                ++k;
            }
            r0k[(size_t)i >> 3] |= (uint32_t)k << (4 * (i & 7));
        }
        if ((e = upload(&p->d_r0k, r0k)) != hipSuccess) {
            pl_plan_destroy(p);
            return hipfail(e, "plan upload");
        }
    }
    int per_cu = 1;
    if (p->generic) {
        p->pg.F = 0;
        p->pg.lds_bytes = pl::nan_redo_lds_bytes(list_size);
        p->fpw = 1;
        p->ws_unit = 0;
        e = hipSuccess;
    } else if (p->tree) {
        p->pg.F = p->tinfo.F;
        p->pg.lds_bytes = p->tinfo.lds_bytes;
        p->fpw = p->tinfo.fpw;
        p->ws_unit = (size_t)p->tinfo.ws_bytes;
        e = pl::tree_prepare(p->tinfo, &per_cu);
    } else {
        // lane-per-path kernel for every (N, L) without a tree instance; flags
        // bits 0..3 pick its fused-top depth (diagnostic), 0x10 / 0x20 force it
        int F = flags & 0xF;
        if (!F) F = env_int("PL_POLAR_FUSED", 3);
        pl::lane_geom(N, K, p->sc ? 1 : list_size, F, env_int("PL_POLAR_LDS_BUDGET", 8 * 1024), &p->lgeo);
        p->pg.F = p->lgeo.F;
        p->pg.lds_bytes = p->lgeo.lds_bytes;
        p->fpw = p->lgeo.lcap >= 64 ? 1 : 64 / p->lgeo.lcap;
        p->ws_unit = (size_t)p->lgeo.ws_bytes;
        e = pl::lane_prepare(p->lgeo, p->sc, &per_cu);
    }
    if (e != hipSuccess) {
        pl_plan_destroy(p);
        return hipfail(e, "polar kernel prepare");
    }
    p->lane_grid_max = per_cu * device_cus(p->device);
    const int waves_env = env_int("PL_POLAR_WAVES", 0);
    if (waves_env > 0) p->lane_grid_max = waves_env;
    if (p->tree && waves_env <= 0 && pl::tree_lookup_small(n, lcap, p->sc, &p->tinfo_small) &&
        p->tinfo_small.ws_bytes <= p->tinfo.ws_bytes && p->tinfo_small.fpw == p->fpw) {
        // its slices fit the main instance's (the workspace is sized for that one)
        int per_cu_small = 0;
        if ((e = pl::tree_prepare(p->tinfo_small, &per_cu_small)) != hipSuccess) {
            pl_plan_destroy(p);
            return hipfail(e, "polar kernel prepare");
        }
        p->small_grid_max = std::min(per_cu_small * device_cus(p->device), p->lane_grid_max);
        p->tree_small = p->small_grid_max > 0;
    }
    if (!p->sc) {
        p->mask_bytes = p->generic ? 0 : pl::nan_mask_region(p->lane_grid_max);
        p->redo_unit = pl::nan_redo_unit(N, list_size);
        p->redo_blocks = device_cus(p->device);
        if (p->generic) {  // scratch of up to 2 GB (at least one frame's): a 2048-path list of N = 1024 holds 23 MB
            // one frame's list state must fit the device (list_size * N = 2^30 needs ~11 GB)
            size_t free_b = 0, total_b = 0;
            if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && p->redo_unit > total_b) {
                pl_plan_destroy(p);
                return fail(PL_EUNSUPPORTED, "list_size: one frame's list state exceeds this device's memory");
            }
            const size_t cap = (size_t)2 << 30;
            p->redo_blocks = (int)std::max<size_t>(1, std::min<size_t>((size_t)p->redo_blocks, cap / p->redo_unit));
            p->lane_grid_max = p->redo_blocks;
        }
        // the redo kernel's dynamic-LDS limit (a per-function attribute) raised to this list's need;
        // a list whose state does not fit the device's LDS is refused here, so that any error
        // of the prepare call itself is a HIP error
        int optin = 0;
        if ((e = hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, p->device)) != hipSuccess) {
            pl_plan_destroy(p);
            return hipfail(e, "device attribute query");
        }
        if (pl::nan_redo_lds_bytes(list_size) > optin) {
            pl_plan_destroy(p);
            return fail(PL_EUNSUPPORTED, "list_size: the redo kernel's list state exceeds this device's LDS");
        }
        if ((e = pl::nan_redo_prepare(list_size)) != hipSuccess) {
            pl_plan_destroy(p);
            return hipfail(e, "NaN redo kernel prepare");
        }
    }
    p->head_bytes = p->mask_bytes + (p->generic ? 0 : (size_t)pl::kSchedBytes);
    *out = p;
    return PL_OK;
}

extern "C" int pl_ldpc_plan_create(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx,
                                   int32_t algo, int32_t max_iter, int32_t early_stop, double normalization,
                                   int32_t flags, pl_plan** out) {
    (void)flags;
    if (!out) return fail(PL_EINVAL, "out is NULL");
    *out = nullptr;
    if (m < 0 || n < 1 || !row_ptr || (!col_idx && row_ptr[m] > 0)) return fail(PL_EINVAL, "bad H");
    if (algo != PL_LDPC_BP && algo != PL_LDPC_MS) return fail(PL_EINVAL, "algo must be BP or MS");
    if (max_iter < 1) return fail(PL_EINVAL, "max_iter must be >= 1");
    const int E = row_ptr[m];
    if (row_ptr[0] != 0 || E < 0) return fail(PL_EINVAL, "row_ptr[0] must be 0");
    std::vector<int32_t> edge_chk(E), var_ptr(n + 1, 0), var_edge(E);
    int maxdc = 0;
    for (int c = 0; c < m; ++c) {
        const int d = row_ptr[c + 1] - row_ptr[c];
        if (d < 0) return fail(PL_EINVAL, "row_ptr not monotone");
        if (d > maxdc) maxdc = d;
        if (algo == PL_LDPC_MS && d == 1)
            return fail(PL_EUNSUPPORTED, "min-sum on a degree-1 check (reference raises ValueError)");
        for (int e = row_ptr[c]; e < row_ptr[c + 1]; ++e) {
            if (col_idx[e] < 0 || col_idx[e] >= n) return fail(PL_EINVAL, "column index out of range");
            if (e > row_ptr[c] && col_idx[e] <= col_idx[e - 1]) return fail(PL_EINVAL, "columns must ascend");
            edge_chk[e] = c;
            var_ptr[col_idx[e] + 1]++;
        }
    }
    for (int v = 0; v < n; ++v) var_ptr[v + 1] += var_ptr[v];
    int maxdv = 0;
    for (int v = 0; v < n; ++v) maxdv = std::max(maxdv, var_ptr[v + 1] - var_ptr[v]);
    if (maxdv > 128) return fail(PL_EUNSUPPORTED, "variable degree > 128");
    // Device edge order: checks sorted by degree (stable), so the lanes of a
    // wavefront run check loops of equal length; columns stay ascending within a
    // check (the reference's product order).  No result depends on the check
    // order: var_edge lists each variable's edges by ascending ORIGINAL check
    // index, the order of the reference's np.sum over them (decoder.py:110-116).
    std::vector<int32_t> order(m);
    for (int c = 0; c < m; ++c) order[c] = c;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        return (row_ptr[a + 1] - row_ptr[a]) < (row_ptr[b + 1] - row_ptr[b]);
    });
    std::vector<int32_t> prow(m + 1, 0), pcol(E), new_edge(E);  // new_edge[original edge]
    for (int k = 0; k < m; ++k) {
        const int c = order[k];
        prow[k + 1] = prow[k] + (row_ptr[c + 1] - row_ptr[c]);
        for (int e = row_ptr[c], j = prow[k]; e < row_ptr[c + 1]; ++e, ++j) {
            pcol[j] = col_idx[e];
            new_edge[e] = j;
            edge_chk[j] = k;
        }
    }
    {
        std::vector<int32_t> fill(var_ptr.begin(), var_ptr.end() - 1);
        for (int c = 0; c < m; ++c)  // original check order
            for (int e = row_ptr[c]; e < row_ptr[c + 1]; ++e) var_edge[fill[col_idx[e]]++] = new_edge[e];
    }
    row_ptr = prow.data();
    col_idx = pcol.data();
    pl_plan* p = new pl_plan();
    p->kind = 1;
    hipGetDevice(&p->device);
    pl::LdpcGeom& g = p->lg;
    g.m = m; g.n = n; g.E = E; g.max_iter = max_iter; g.early_stop = early_stop ? 1 : 0; g.algo = algo;
    g.maxdc = maxdc; g.maxdv = maxdv; g.norm = normalization;
    g.regular = 1;
    for (int c = 0; c < m && g.regular; ++c) g.regular = (row_ptr[c + 1] - row_ptr[c]) == maxdc;
    for (int v = 0; v < n && g.regular; ++v) g.regular = (var_ptr[v + 1] - var_ptr[v]) == maxdv;
    g.threads = E <= 4096 ? 256 : 1024;
    if (E >= (1 << 20) || maxdc >= (1 << 11)) { delete p; return fail(PL_EUNSUPPORTED, "code too large"); }
    const size_t lds_small = (size_t)8 * m + n;                 // syndrome [2][m] u32 + decisions [n]
    const size_t lds_all = (size_t)2 * (size_t)E * 8 + lds_small;  // + T[E], C[E]
    g.use_global = lds_all > 64 * 1024 ? 1 : 0;
    g.lds_bytes = (int)(((g.use_global ? lds_small : lds_all) + 15) & ~(size_t)15);
    // check-per-thread kernel (ldpc.hip ldpc_check_kernel): diagnostic build only, PL_LDPC_KERNEL=check
    const char* lk = std::getenv("PL_LDPC_KERNEL");
    g.check_kernel = PL_DIAG && !g.use_global && lk && std::string(lk) == "check" ? 1 : 0;
    // register-cached kernel: constant variable degree < 8, LDS-resident state
    g.reg_variant = 0;
    if (!g.use_global && !g.check_kernel && !(lk && std::string(lk) == "generic")) {
        bool regular = true;
        for (int v = 0; v < n && regular; ++v) regular = (var_ptr[v + 1] - var_ptr[v]) == maxdv;
        if (regular && maxdv < 8 && E < 65536) g.reg_variant = pl::ldpc_reg_variant(maxdv, E, n);
        if (g.reg_variant) {
            g.threads = 256;
            // + the per-wavefront BP tanh lists (ldpc_reg_kernel)
            const size_t base = ((size_t)2 * E * 8 + lds_small + 15) & ~(size_t)15;
            g.lds_bytes = (int)((base + pl::ldpc_reg_list_bytes(g.reg_variant) + 15) & ~(size_t)15) + 128;  // + vote words
        }
    }
    // BP on a reg variant: degree-grouped check products (ldpc_bp_grp_kernel).
    // Slot s holds edges 64 s .. 64 s + 63 (degree-sorted, check-major); D_s =
    // the largest check degree among them; check c's inputs sit at T' offset
    // off[c] (even), padded with 1.0 to the largest D_s of the slots holding its
    // edges.  PL_LDPC_KERNEL=reg keeps ldpc_reg_kernel's per-lane products.
    std::vector<int32_t> grp_meta, var_tpos;
    g.grp = 0;
    g.tl = 0;
    if (g.reg_variant && algo == PL_LDPC_BP && maxdc <= 15 && !(lk && std::string(lk) == "reg")) {
        const int slots = 4 * pl::ldpc_reg_ept(g.reg_variant);
        std::vector<int> dslot(slots, 0), dpad(m, 0), off(m + 1, 0);
        for (int e = 0; e < E; ++e) {
            const int c = edge_chk[e], d = row_ptr[c + 1] - row_ptr[c];
            dslot[e / 64] = std::max(dslot[e / 64], d);
        }
        for (int e = 0; e < E; ++e) dpad[edge_chk[e]] = std::max(dpad[edge_chk[e]], dslot[e / 64]);
        for (int c = 0; c < m; ++c) off[c + 1] = off[c] + ((dpad[c] + 1) & ~1);
        // T', C' positions [0, off[m]) hold the checks, [off[m], off[m] + 16) is a sink
        // for the lanes of a slot past the last edge (they read it and store into it)
        const int sink = off[m], tl = off[m] + 16;
        const size_t base = ((size_t)16 * tl + (size_t)4 * ((m + 3) & ~3) + 15) & ~(size_t)15;  // T', C', syndrome
        const size_t lds = (base + pl::ldpc_reg_list_bytes(g.reg_variant) + 15) & ~(size_t)15;
        if (tl < 65536 && lds <= 64 * 1024) {
            g.grp = 1;
            // two frames per workgroup, one after the other (ldpc_bp_grp_kernel FPG):
            // valid codewords (early stop) 0.777 -> 0.742 ms per 65 536 frames, the
            // harness frames (20 iterations) equal; PL_BP_FPG=1 restores one.  Only
            // the (DV, EPT, VPT) = (3, 6, 2) instance: the larger ones' two-frame
            // builds spill 24-41 more VGPRs than their one-frame builds
            const bool fpg2 = maxdv == 3 && pl::ldpc_reg_ept(g.reg_variant) == 6;
            g.fpg = env_int("PL_BP_FPG", fpg2 ? 2 : 1) == 1 ? 1 : 2;
            g.tl = tl;
            g.lds_bytes = (int)lds;
            // sorted slot s goes to the thread slot (j = s / 4, wavefront w) in snake
            // order (w = s % 4 for even j, 3 - s % 4 for odd j), so the four
            // wavefronts -- one per SIMD -- get products of about equal total length
            grp_meta.assign((size_t)slots * 64, 0);
            for (int s = 0; s < slots; ++s) {
                const int j = s / 4, w = (j & 1) ? 3 - (s & 3) : (s & 3);
                for (int l = 0; l < 64; ++l) {
                    const int e = 64 * s + l, q = 256 * j + 64 * w + l;
                    if (e < E) {
                        const int c = edge_chk[e];
                        grp_meta[q] = off[c] | ((e - row_ptr[c]) << 16) | (dslot[s] << 20);
                    } else {  // reads and stores the sink (position 15 skips no factor)
                        grp_meta[q] = sink | (15 << 16) | (dslot[s] << 20);
                    }
                }
            }
            // variables in thread-slot order (slot q = 256 j + tid): T' position and
            // check of each edge, variable index (-1: empty); the order chosen so
            // the variable pass's scattered LDS accesses conflict little
            std::vector<int32_t> tp((size_t)n * maxdv), vck((size_t)n * maxdv);
            for (int v = 0; v < n; ++v)
                for (int k = 0; k < maxdv; ++k) {
                    const int e = var_edge[var_ptr[v] + k], c = edge_chk[e];
                    tp[(size_t)v * maxdv + k] = off[c] + (e - row_ptr[c]);
                    vck[(size_t)v * maxdv + k] = c;
                }
            const int nslots = 256 * pl::ldpc_reg_vpt(g.reg_variant);
            const std::vector<int> vmap = ldpc_var_slots(n, maxdv, tp, tl, nslots);
            // + the pad positions (T' = 1.0 from the first write on), -1 filled to 256
            std::vector<char> real(sink, 0);
            for (int e = 0; e < E; ++e) real[off[edge_chk[e]] + (e - row_ptr[edge_chk[e]])] = 1;
            std::vector<int32_t> pads;
            for (int q = 0; q < sink; ++q)
                if (!real[q]) pads.push_back(q);
            g.npad = (int)((pads.size() + 255) / 256 * 256);
            pads.resize(g.npad, -1);
            var_tpos.assign((size_t)nslots * (2 * maxdv + 1), 0);
            for (int q = 0; q < nslots; ++q) {
                const int v = vmap[q];
                var_tpos[(size_t)2 * maxdv * nslots + q] = v;
                for (int k = 0; k < maxdv; ++k) {
                    var_tpos[(size_t)q * maxdv + k] = v >= 0 ? tp[(size_t)v * maxdv + k] : 0;
                    var_tpos[(size_t)maxdv * nslots + (size_t)q * maxdv + k] = v >= 0 ? vck[(size_t)v * maxdv + k] : 0;
                }
            }
            var_tpos.insert(var_tpos.end(), pads.begin(), pads.end());
        }
    }
    // min-sum codes whose T/C arrays exceed LDS: compressed check state in LDS
    g.compact = 0;
    if (g.use_global && algo == 1 && maxdc <= 15 && !(lk && std::string(lk) == "generic")) {
        const size_t lds_c = (((((size_t)8 * n + 15) & ~(size_t)15) + (size_t)20 * m + 15) & ~(size_t)15) + 128;  // + vote words
        if (lds_c <= 160 * 1024) {
            g.compact = 1;
            g.use_global = 0;
            g.threads = 1024;
            g.lds_bytes = (int)((lds_c + 15) & ~(size_t)15);
        }
    }
    // (3,6)-regular min-sum of n = 2048 / 4096 / 8192 (the BASELINE n = 8192 code):
    // ldpc_ms36_kernel (PL_LDPC_KERNEL=compact keeps ldpc_ms_compact_kernel)
    g.ms36 = 0;
    std::vector<int32_t> ms_vw;
    if (g.compact && g.regular && maxdv == 3 && maxdc == 6 && 2 * m == n && pl::ldpc_ms36_lds(n) > 0 &&
        !(lk && std::string(lk) == "compact")) {
        g.ms36 = n / 1024;
        g.lds_bytes = pl::ldpc_ms36_lds(n);
        const uint32_t REC = 8u * (uint32_t)n, MET = 16u * (uint32_t)n;  // ldpc_ms36_kernel's LDS layout
        // [n][8]: per variable its three edge words and meta addresses; then
        // [m][4]: per check the LDS byte addresses 8v of its six variables, two per word
        ms_vw.assign((size_t)n * 8 + (size_t)m * 4, 0);
        for (int v = 0; v < n; ++v)
            for (int k = 0; k < 3; ++k) {
                const int e = var_edge[var_ptr[v] + k], c = edge_chk[e], pos = e - row_ptr[c];
                ms_vw[(size_t)v * 8 + k] = (int32_t)((REC + 16u * (uint32_t)c) | (3u * (uint32_t)pos));
                ms_vw[(size_t)v * 8 + 3 + k] = (int32_t)(MET + 4u * (uint32_t)c);
            }
        for (int c = 0; c < m; ++c)
            for (int k = 0; k < 3; ++k)
                ms_vw[(size_t)n * 8 + (size_t)c * 4 + k] =
                    (int32_t)((8u * (uint32_t)col_idx[row_ptr[c] + 2 * k]) | ((8u * (uint32_t)col_idx[row_ptr[c] + 2 * k + 1]) << 16));
    }
    if (g.check_kernel) {
        g.threads = 256;
        g.lds_bytes = (int)(((size_t)(2 * (size_t)E + n) * 8 + 15) & ~(size_t)15);
    }
    std::vector<int32_t> all;
    all.insert(all.end(), row_ptr, row_ptr + m + 1);
    all.insert(all.end(), col_idx, col_idx + E);
    all.insert(all.end(), edge_chk.begin(), edge_chk.end());
    all.insert(all.end(), var_ptr.begin(), var_ptr.end());
    all.insert(all.end(), var_edge.begin(), var_edge.end());
    std::vector<int32_t> edge_meta(E), var_chk(E);
    for (int k = 0; k < m; ++k)
        for (int e = row_ptr[k]; e < row_ptr[k + 1]; ++e) edge_meta[e] = row_ptr[k] | ((row_ptr[k + 1] - row_ptr[k]) << 20);
    for (int k = 0; k < E; ++k) var_chk[k] = edge_chk[var_edge[k]];
    std::vector<int32_t> var_cp(E);
    for (int k = 0; k < E; ++k) {
        const int e = var_edge[k], c = edge_chk[e];
        var_cp[k] = (c << 4) | ((e - row_ptr[c]) & 15);
    }
    all.insert(all.end(), edge_meta.begin(), edge_meta.end());
    all.insert(all.end(), var_chk.begin(), var_chk.end());
    all.insert(all.end(), var_cp.begin(), var_cp.end());
    const size_t grp_at = all.size();
    all.insert(all.end(), grp_meta.begin(), grp_meta.end());
    all.insert(all.end(), var_tpos.begin(), var_tpos.end());
    all.resize((all.size() + 3) & ~(size_t)3, 0);  // ms_vw: 16-byte aligned (uint4 loads)
    const size_t vw_at = all.size();
    all.insert(all.end(), ms_vw.begin(), ms_vw.end());
    hipError_t e = upload(&p->d_ldpc, all);
    if (e != hipSuccess) { pl_plan_destroy(p); return hipfail(e, "plan upload"); }
    p->ld.row_ptr = p->d_ldpc;
    p->ld.col_idx = p->ld.row_ptr + (m + 1);
    p->ld.edge_chk = p->ld.col_idx + E;
    p->ld.var_ptr = p->ld.edge_chk + E;
    p->ld.var_edge = p->ld.var_ptr + (n + 1);
    p->ld.edge_meta = p->ld.var_edge + E;
    p->ld.var_chk = p->ld.edge_meta + E;
    p->ld.var_cp = p->ld.var_chk + E;
    p->ld.grp_meta = g.grp ? p->d_ldpc + grp_at : nullptr;
    p->ld.var_tpos = g.grp ? p->d_ldpc + grp_at + grp_meta.size() : nullptr;
    p->ld.ms_vw = g.ms36 ? reinterpret_cast<const uint32_t*>(p->d_ldpc + vw_at) : nullptr;
    if ((e = pl::ldpc_prepare(g)) != hipSuccess) { pl_plan_destroy(p); return hipfail(e, "hipFuncSetAttribute"); }
    p->ws_unit = pl::ldpc_work_bytes_per_frame(g);
    p->ldpc_chunk = std::max(1, env_int("PL_LDPC_CHUNK", 16384));
    *out = p;
    return PL_OK;
}

// Polar workspace layout for a grid of `grid` resident wavefronts: a list
// plan's NaN masks first (for its largest grid, so they stay in place, and
// zero, from one decode to the next), then the tree / lane kernel's frame-group
// counter (zeroed by tree_launch / lane_launch before each launch), then the list kernel's
// slices, which the NaN redo kernel reuses as its scratch once the list kernel
// is done.
static size_t polar_bytes(const pl_plan* p, int64_t grid) {
    return p->head_bytes + std::max<size_t>(p->ws_unit * (size_t)grid, p->redo_unit);
}
// the smallest workspace a decode can run on (one wavefront's slice)
static size_t ws_min(const pl_plan* p) {
    if (p->kind == 0 && p->generic) return p->redo_unit;
    return p->kind == 0 ? polar_bytes(p, 1) : p->ws_unit;
}

// Workspace bytes a decode of `batch` frames uses at full speed.
static size_t ws_need(const pl_plan* p, int64_t batch) {
    if (batch <= 0 || (p->ws_unit == 0 && p->redo_unit == 0)) return 0;
    if (p->kind == 0 && p->generic) return p->redo_unit * (size_t)std::min<int64_t>(batch, p->redo_blocks);
    if (p->kind == 0) {
        const int64_t waves = (batch + p->fpw - 1) / p->fpw;
        return polar_bytes(p, std::min<int64_t>(waves, p->lane_grid_max));
    }
    return p->ws_unit * (size_t)std::min<int64_t>(batch, p->ldpc_chunk);
}

// Diagnostic-build options of one decode call (none in the product entry points):
// stamps = the tree kernel's stamp buffer (or, with ds_mode 1 / 2, the dead-store
// record / replay bitmask); flagged = a host array of `batch` bytes that receives,
// per frame, whether the list kernel flagged it for the NaN-order redo decoder.
struct DecodeDiag {
    unsigned long long* stamps = nullptr;
    int ds_mode = 0;
    uint8_t* flagged = nullptr;
};

// Decode with an explicit workspace of ws_bytes (>= one unit when one is needed):
// the polar grid / LDPC chunk is clamped to what the workspace holds.
static int decode_impl(pl_plan* p, const double* llr, int64_t batch, int64_t ld, uint8_t* bits, int32_t* iters,
                       void* ws, size_t ws_bytes, hipStream_t s, bool zero_masks = false,
                       const DecodeDiag& dg = DecodeDiag()) {
    unsigned long long* const stamps = dg.stamps;
    const size_t wmin = ws_min(p);
    if (wmin > 0 && (ws == nullptr || ws_bytes < wmin))
        return fail(PL_EINVAL, "workspace smaller than one unit (pl_plan_workspace_bytes)");
    if (p->kind == 0 && p->generic) {
        if (stamps) return fail(PL_EUNSUPPORTED, "stamps only for the tree kernel");
        // one workgroup per frame, masks = null: every frame
        hipError_t e = pl::nan_redo_launch(llr, ld, bits, batch, p->pg.N, p->pg.K, p->list_size, p->d_frozen_dec,
                                           p->d_info_pos, p->d_crc_g, nullptr, 0, 1, redo_metric(p),
                                           (unsigned char*)ws, ws_bytes, p->redo_blocks, s);
        return e == hipSuccess ? PL_OK : hipfail(e, "polar generic list launch");
    }
    if (p->kind == 0) {
        if (!p->tree && stamps) return fail(PL_EUNSUPPORTED, "stamps only for the tree kernel");
        const int64_t waves = (batch + p->fpw - 1) / p->fpw;
        // every wavefront of the decode resident at the small instance's occupancy:
        // that instance (not for the dead-store diagnostics, headline instance only)
        const bool small = p->tree_small && waves <= p->small_grid_max && dg.ds_mode == 0;
        const pl::TreeInfo& ti = small ? p->tinfo_small : p->tinfo;
        int64_t grid = std::min<int64_t>(waves, p->lane_grid_max);
        while (grid > 1 && polar_bytes(p, grid) > ws_bytes) grid = std::min<int64_t>(grid - 1, grid * ws_bytes / polar_bytes(p, grid));
        unsigned char* const base = (unsigned char*)ws;
        uint64_t* const masks = p->mask_bytes ? (uint64_t*)base : nullptr;
        unsigned char* const slices = base + p->head_bytes;  // the group counter: slices - kSchedBytes
        if (masks && zero_masks) {  // a caller-owned workspace: the masks may hold anything
            hipError_t e = hipMemsetAsync(masks, 0, (size_t)grid * 8 * pl::kNanMaskPasses, s);
            if (e != hipSuccess) return hipfail(e, "NaN mask reset");
        }
        // a list launch runs at most kNanMaskPasses passes of its grid (the masks' depth)
        const int64_t step = masks ? grid * p->fpw * pl::kNanMaskPasses : batch;
        for (int64_t b0 = 0; b0 < batch; b0 += step) {
            const int64_t nb = std::min<int64_t>(step, batch - b0);
            const double* l0 = llr + b0 * ld;
            uint8_t* o0 = bits + b0 * p->pg.K;
            hipError_t e;
            if (p->tree)
                e = pl::tree_launch(ti, l0, ld, o0, p->d_frozen_dec, p->d_info_pos, nb, p->pg.K,
                                    p->sc ? 1 : p->list_size, slices, (int)grid, stamps, p->d_crc_g,
                                    p->sc ? (const void*)p->d_r0k : (const void*)masks, s, dg.ds_mode);
            else
                e = pl::lane_launch(p->lgeo, p->sc, l0, ld, o0, p->d_frozen_dec, p->d_info_pos, nb, slices, (int)grid,
                                    p->d_crc_g, masks, s);
            if (e != hipSuccess) return hipfail(e, "polar decode launch");
            if (masks && dg.flagged) {  // diagnostic: which frames of this pass group were flagged
                std::vector<uint64_t> mw((size_t)grid * pl::kNanMaskPasses);
                e = hipMemcpyAsync(mw.data(), masks, mw.size() * 8, hipMemcpyDeviceToHost, s);
                if (e == hipSuccess) e = hipStreamSynchronize(s);
                if (e != hipSuccess) return hipfail(e, "NaN mask readback");
                // word [w][ps] bit f = frame (ps * grid + w) * fpw + f (polar_tree.hip, polar_nan.hip)
                for (int64_t w = 0; w < grid; ++w)
                    for (int ps = 0; ps < pl::kNanMaskPasses; ++ps)
                        for (int f = 0; f < 64; ++f)
                            if ((mw[(size_t)w * pl::kNanMaskPasses + ps] >> f) & 1) {
                                const int64_t fr = ((int64_t)ps * grid + w) * p->fpw + f;
                                if (fr < nb) dg.flagged[b0 + fr] = 1;
                            }
            }
            if (masks) {
                // frames whose list saw a NaN metric, in the reference's candidate order
                e = pl::nan_redo_launch(l0, ld, o0, nb, p->pg.N, p->pg.K, p->list_size, p->d_frozen_dec,
                                        p->d_info_pos, p->d_crc_g, masks, (int)grid, p->fpw, redo_metric(p), slices,
                                        ws_bytes - p->head_bytes, p->redo_blocks, s);
                if (e != hipSuccess) return hipfail(e, "polar NaN redo launch");
            }
        }
        return PL_OK;
    }
    if (!p->lg.use_global) {
        // one workgroup per frame; HIP caps a grid at 2^32 work-items
        const int64_t step = kMaxLaunchItems / p->lg.threads;
        for (int64_t b0 = 0; b0 < batch; b0 += step) {
            const int64_t nb = std::min<int64_t>(step, batch - b0);
            hipError_t e = pl::ldpc_launch(p->lg, p->ld, llr + b0 * ld, ld, bits + b0 * p->lg.n,
                                           iters ? iters + b0 : nullptr, nb, nullptr, s);
            if (e != hipSuccess) return hipfail(e, "ldpc decode launch");
        }
        return PL_OK;
    }
    const int64_t chunk = std::min<int64_t>(p->ldpc_chunk, (int64_t)(ws_bytes / p->ws_unit));
    for (int64_t b0 = 0; b0 < batch; b0 += chunk) {
        const int64_t nb = std::min<int64_t>(chunk, batch - b0);
        hipError_t e = pl::ldpc_launch(p->lg, p->ld, llr + b0 * ld, ld, bits + b0 * p->lg.n,
                                       iters ? iters + b0 : nullptr, nb, (double*)ws, s);
        if (e != hipSuccess) return hipfail(e, "ldpc decode launch");
    }
    return PL_OK;
}

// The calling stream's workspace entry (created empty on first use).
static std::shared_ptr<Workspace> stream_entry(pl_plan* p, hipStream_t s) {
    std::lock_guard<std::mutex> lk(p->mu);
    std::shared_ptr<Workspace>& w = p->ws[s];
    if (!w) w = std::make_shared<Workspace>();
    return w;
}

// Grow `w` (its mutex held by the caller) to `need` bytes.  A buffer is only
// ever used by its own stream.  The new buffer is allocated while the old one
// is still held; only if the device is out of memory is the old one released
// (after draining its stream) before retrying, then halved down to one unit (the
// decode then runs fewer resident wavefronts / smaller chunks: decode_impl
// clamps to what the buffer holds).  A failure other than out-of-memory leaves
// the old buffer in place.  `retry`: also retry a request that fell back before.
static int grow_ws(pl_plan* p, Workspace* w, hipStream_t s, size_t need, bool retry) {
    if (w->bytes >= need) return PL_OK;
    if (!retry && w->ptr && w->failed_need && need <= w->failed_need) return PL_OK;  // fell back for this size
    const size_t unit = std::max<size_t>(ws_min(p), 1);
    size_t want = need;
    for (;;) {
        void* np = nullptr;
        hipError_t e = hipMalloc(&np, want);
        if (e == hipSuccess) {
            if (w->ptr) {
                // the old buffer may still be read by work queued on this stream
                hipError_t se = hipStreamSynchronize(s);
                hipFree(w->ptr);
                w->ptr = nullptr;
                w->bytes = 0;
                if (se != hipSuccess) {
                    hipFree(np);
                    return hipfail(se, "workspace regrow: stream synchronize");
                }
            }
            if (p->mask_bytes) {  // NaN masks start at zero (the decodes keep them so), before the buffer is published
                hipError_t me = hipMemsetAsync(np, 0, p->mask_bytes, s);
                if (me != hipSuccess) {
                    hipFree(np);  // the workspace stays empty: the next decode retries
                    return hipfail(me, "NaN mask reset");
                }
            }
            w->ptr = np;
            w->bytes = want;
            w->failed_need = want < need ? need : 0;
            return PL_OK;
        }
        (void)hipGetLastError();  // clear the sticky allocation error before retrying
        if (e != hipErrorOutOfMemory) return hipfail(e, "decode workspace");
        if (w->ptr) {  // make room: drain this stream, release its buffer, retry the same size
            hipError_t se = hipStreamSynchronize(s);
            hipFree(w->ptr);
            w->ptr = nullptr;
            w->bytes = 0;
            if (se != hipSuccess) return hipfail(se, "workspace regrow: stream synchronize");
            continue;
        }
        if (want <= unit) return hipfail(e, "decode workspace");
        want = std::max(unit, (want / 2) / unit * unit);
    }
}

static int check_decode_args(const pl_plan* p, int64_t batch, int64_t ld, const void* llr, const void* bits) {
    if (!p) return fail(PL_EINVAL, "plan is NULL");
    if (batch < 0) return fail(PL_EINVAL, "batch < 0");
    if (batch > 0 && (!llr || !bits)) return fail(PL_EINVAL, "NULL buffer");
    if (p->kind == 0 && ld < p->pg.N) return fail(PL_EINVAL, "ld < N");
    if (p->kind == 1 && ld < p->lg.n) return fail(PL_EINVAL, "ld < n");
    return PL_OK;
}

extern "C" int pl_plan_reserve(pl_plan* p, int64_t max_batch, void* stream) {
    if (!p) return fail(PL_EINVAL, "plan is NULL");
    if (max_batch < 0) return fail(PL_EINVAL, "max_batch < 0");
    if (max_batch == 0) return pl_plan_release(p, stream);
    int rc = check_device(p);
    if (rc) return rc;
    const size_t need = ws_need(p, max_batch);
    if (need == 0) return PL_OK;
    const hipStream_t s = (hipStream_t)stream;
    std::shared_ptr<Workspace> w = stream_entry(p, s);
    std::lock_guard<std::mutex> lk(w->mu);
    return grow_ws(p, w.get(), s, need, true);
}

extern "C" int pl_plan_release(pl_plan* p, void* stream) {
    if (!p) return fail(PL_EINVAL, "plan is NULL");
    if (int rc = check_device(p)) return rc;
    const hipStream_t s = (hipStream_t)stream;
    std::shared_ptr<Workspace> w;
    {
        std::lock_guard<std::mutex> lk(p->mu);
        auto it = p->ws.find(s);
        if (it == p->ws.end()) return PL_OK;
        w = it->second;
        p->ws.erase(it);
    }
    std::lock_guard<std::mutex> lk(w->mu);  // a decode in flight on this stream finishes its launch first
    if (w->ptr) {
        hipError_t e = hipStreamSynchronize(s);
        hipFree(w->ptr);
        w->ptr = nullptr;
        w->bytes = 0;
        if (e != hipSuccess) return hipfail(e, "workspace release: stream synchronize");
    }
    return PL_OK;
}

extern "C" int pl_plan_workspace_stats(const pl_plan* p, int64_t* streams, int64_t* bytes) {
    if (!p || !streams || !bytes) return fail(PL_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(const_cast<pl_plan*>(p)->mu);
    *streams = 0;
    *bytes = 0;
    for (const auto& kv : p->ws) {
        ++*streams;
        *bytes += (int64_t)kv.second->bytes.load();
    }
    return PL_OK;
}

extern "C" int pl_plan_workspace_bytes(const pl_plan* p, int64_t batch, int64_t* bytes) {
    if (!p || !bytes) return fail(PL_EINVAL, "NULL argument");
    if (batch < 0) return fail(PL_EINVAL, "batch < 0");
    *bytes = (int64_t)ws_need(p, batch);
    return PL_OK;
}

extern "C" int pl_decode(pl_plan* p, const double* llr, int64_t batch, int64_t ld, uint8_t* bits,
                         int32_t* iters, void* stream) {
    int rc = check_decode_args(p, batch, ld, llr, bits);
    if (rc || batch == 0) return rc;
    if ((rc = check_device(p))) return rc;
    const hipStream_t s = (hipStream_t)stream;
    const size_t need = ws_need(p, batch);
    if (!need) return decode_impl(p, llr, batch, ld, bits, iters, nullptr, 0, s);
    std::shared_ptr<Workspace> w = stream_entry(p, s);
    std::lock_guard<std::mutex> lk(w->mu);
    if ((rc = grow_ws(p, w.get(), s, need, false))) return rc;
    return decode_impl(p, llr, batch, ld, bits, iters, w->ptr, w->bytes, s);
}

extern "C" int pl_decode_ws(pl_plan* p, const double* llr, int64_t batch, int64_t ld, uint8_t* bits,
                            int32_t* iters, void* workspace, int64_t workspace_bytes, void* stream) {
    int rc = check_decode_args(p, batch, ld, llr, bits);
    if (rc || batch == 0) return rc;
    if (workspace_bytes < 0) return fail(PL_EINVAL, "workspace_bytes < 0");
    if ((rc = check_device(p))) return rc;
    return decode_impl(p, llr, batch, ld, bits, iters, workspace, (size_t)workspace_bytes, (hipStream_t)stream,
                       true);
}

extern "C" int pl_debug_polar_stamps(pl_plan* p, const double* llr, int64_t batch, int64_t ld, uint8_t* bits,
                                     unsigned long long* stamps_dev, void* stream) {
    if (!p || p->kind != 0 || !stamps_dev) return fail(PL_EINVAL, "polar plan and stamp buffer required");
#if !PL_DIAG
    (void)llr; (void)batch; (void)ld; (void)bits; (void)stream;
    return fail(PL_EUNSUPPORTED, "stamped kernels are in the diagnostic build only (make DIAG=1)");
#else
    int rc = check_decode_args(p, batch, ld, llr, bits);
    if (rc || batch == 0) return rc;
    if ((rc = check_device(p))) return rc;
    const hipStream_t s = (hipStream_t)stream;
    std::shared_ptr<Workspace> w = stream_entry(p, s);
    std::lock_guard<std::mutex> lk(w->mu);
    if ((rc = grow_ws(p, w.get(), s, ws_need(p, batch), false))) return rc;
    DecodeDiag dg;
    dg.stamps = stamps_dev;
    return decode_impl(p, llr, batch, ld, bits, nullptr, w->ptr, w->bytes, s, false, dg);
#endif
}

extern "C" int pl_debug_polar_deadstore(pl_plan* p, const double* llr, int64_t batch, int64_t ld, uint8_t* bits,
                                        uint32_t* mask_dev, int32_t mode, void* stream) {
    if (!p || p->kind != 0 || !mask_dev || (mode != 1 && mode != 2)) return fail(PL_EINVAL, "polar plan, mask, mode 1|2");
#if !PL_DIAG
    (void)llr; (void)batch; (void)ld; (void)bits; (void)stream;
    return fail(PL_EUNSUPPORTED, "dead-store instances are in the diagnostic build only (make DIAG=1)");
#else
    int rc = check_decode_args(p, batch, ld, llr, bits);
    if (rc || batch == 0) return rc;
    if ((rc = check_device(p))) return rc;
    if (!p->tree || !p->tinfo.fn_ds[0]) return fail(PL_EUNSUPPORTED, "dead-store instances: N=1024 L=8 tree plans only");
    const hipStream_t s = (hipStream_t)stream;
    std::shared_ptr<Workspace> w = stream_entry(p, s);
    std::lock_guard<std::mutex> lk(w->mu);
    if ((rc = grow_ws(p, w.get(), s, ws_need(p, batch), false))) return rc;
    DecodeDiag dg;
    dg.stamps = reinterpret_cast<unsigned long long*>(mask_dev);
    dg.ds_mode = mode;
    return decode_impl(p, llr, batch, ld, bits, nullptr, w->ptr, w->bytes, s, false, dg);
#endif
}

// Diagnostic build: an ordinary list decode that also reports, per frame, whether
// the list kernel flagged it for the NaN-order redo decoder (flagged_host: `batch`
// bytes, 1 = flagged).  The decode itself is the product path, bits included.
extern "C" int pl_debug_polar_flagged(pl_plan* p, const double* llr, int64_t batch, int64_t ld, uint8_t* bits,
                                      uint8_t* flagged_host, void* stream) {
    if (!p || p->kind != 0 || !flagged_host) return fail(PL_EINVAL, "polar plan and flag array required");
#if !PL_DIAG
    (void)llr; (void)batch; (void)ld; (void)bits; (void)stream;
    return fail(PL_EUNSUPPORTED, "test hook: diagnostic build only (make DIAG=1)");
#else
    int rc = check_decode_args(p, batch, ld, llr, bits);
    if (rc || batch == 0) return rc;
    if ((rc = check_device(p))) return rc;
    if (p->generic || p->mask_bytes == 0) return fail(PL_EUNSUPPORTED, "plan has no NaN masks (SC or generic list plan)");
    std::memset(flagged_host, 0, (size_t)batch);
    const hipStream_t s = (hipStream_t)stream;
    std::shared_ptr<Workspace> w = stream_entry(p, s);
    std::lock_guard<std::mutex> lk(w->mu);
    if ((rc = grow_ws(p, w.get(), s, ws_need(p, batch), false))) return rc;
    DecodeDiag dg;
    dg.flagged = flagged_host;
    return decode_impl(p, llr, batch, ld, bits, nullptr, w->ptr, w->bytes, s, false, dg);
#endif
}

extern "C" int pl_debug_ldpc_stamps(pl_plan* p, const double* llr, int64_t batch, int64_t ld, uint8_t* bits,
                                    int32_t* iters, unsigned long long* stamps_dev, void* stream) {
    if (!p || p->kind != 1 || !stamps_dev) return fail(PL_EINVAL, "LDPC plan and stamp buffer required");
#if !PL_DIAG
    (void)llr; (void)batch; (void)ld; (void)bits; (void)iters; (void)stream;
    return fail(PL_EUNSUPPORTED, "stamped kernels are in the diagnostic build only (make DIAG=1)");
#else
    int rc = check_decode_args(p, batch, ld, llr, bits);
    if (rc || batch == 0) return rc;
    if ((rc = check_device(p))) return rc;
    if (!p->lg.grp || p->lg.reg_variant != 1) return fail(PL_EUNSUPPORTED, "stamps only for the grouped (504,252)-size BP kernel");
    hipError_t e = pl::ldpc_launch_stamped(p->lg, p->ld, llr, ld, bits, iters, batch, stamps_dev, (hipStream_t)stream);
    return e == hipSuccess ? PL_OK : hipfail(e, "stamped LDPC launch");
#endif
}

// Diagnostic build: the frame-per-wavefront prototype (polar_fpw.hip) on a
// polar N=1024 L=8 plan's device constants; stamps_dev: 5 u64 cycle sums
// (descent, metric, prune, partial sums, output); grid 0 = fill the device.
extern "C" int pl_debug_polar_fpw(pl_plan* p, const double* llr, int64_t batch, int64_t ld, uint8_t* bits,
                                  unsigned long long* stamps_dev, int32_t grid, void* stream) {
#if !PL_DIAG
    (void)p; (void)llr; (void)batch; (void)ld; (void)bits; (void)stamps_dev; (void)grid; (void)stream;
    return fail(PL_EUNSUPPORTED, "the frame-per-wavefront prototype is in the diagnostic build only (make DIAG=1)");
#else
    if (!p || p->kind != 0 || p->pg.N != 1024 || p->list_size != 8) return fail(PL_EINVAL, "N=1024 L=8 polar plan");
    int rc = check_decode_args(p, batch, ld, llr, bits);
    if (rc || batch == 0) return rc;
    if ((rc = check_device(p))) return rc;
    hipError_t e = pl::fpw_launch(llr, ld, bits, p->d_frozen_dec, p->d_info_pos, batch, p->pg.K, stamps_dev, grid,
                                  (hipStream_t)stream);
    return e == hipSuccess ? PL_OK : hipfail(e, "fpw launch");
#endif
}

extern "C" int pl_debug_set_plan_device(pl_plan* p, int32_t device) {
    if (!p) return fail(PL_EINVAL, "plan is NULL");
#if !PL_DIAG
    (void)device;
    return fail(PL_EUNSUPPORTED, "test hook: diagnostic build only (make DIAG=1)");
#else
    p->device = device;
    return PL_OK;
#endif
}

extern "C" int pl_polar_plan_set_crc(pl_plan* p, int32_t crc_len, uint32_t poly) {
    if (!p || p->kind != 0) return fail(PL_EINVAL, "not a polar plan");
    if (p->sc) return fail(PL_EINVAL, "CRC-aided selection needs a list decoder (list_size >= 1)");
    if (crc_len < 0 || crc_len > 32) return fail(PL_EINVAL, "crc_len must be in [0, 32]");
    if (int rc = check_device(p)) return rc;
    if (p->d_crc_g) { hipFree(p->d_crc_g); p->d_crc_g = nullptr; }
    if (crc_len == 0) return PL_OK;
    const int N = p->pg.N;
    // g[j] = CRC register (src/polar/utils.py:86-125, zero initial register) of
    // the info bits of u = e_j F^{(x)n}; u_k = 1 iff k is a bit-submask of j.
    const uint32_t top = 1u << (crc_len - 1), mask = crc_len == 32 ? 0xFFFFFFFFu : ((1u << crc_len) - 1u);
    std::vector<uint32_t> g((size_t)N);
    for (int j = 0; j < N; ++j) {
        uint32_t crc = 0;
        for (const int32_t k : p->h_info) {
            const uint32_t bit = ((k & j) == k) ? 1u : 0u;
            crc ^= bit << (crc_len - 1);
            crc = (crc & top) ? ((crc << 1) ^ poly) : (crc << 1);
            crc &= mask;
        }
        g[(size_t)j] = crc;
    }
    hipError_t e = upload(&p->d_crc_g, g);
    return e == hipSuccess ? PL_OK : hipfail(e, "crc table upload");
}

extern "C" int pl_plan_get_info(const pl_plan* p, pl_plan_info* info) {
    if (!p || !info) return fail(PL_EINVAL, "NULL argument");
    *info = pl_plan_info{};
    if (p->kind == 0) {
        info->kind = 0; info->n_in = p->pg.N; info->n_out = p->pg.K; info->list_size = p->list_size;
        info->lds_bytes = p->pg.lds_bytes; info->fused_top = p->pg.F;
        info->frames_per_block = p->fpw;
        info->reserved = p->generic ? 6 : (p->tree ? 4 : 3);  // kernel: 4 tree, 3 lane, 6 single-workgroup exact
    } else {
        info->kind = 1; info->n_in = p->lg.n; info->n_out = p->lg.n; info->list_size = 0;
        info->lds_bytes = p->lg.lds_bytes; info->fused_top = 0; info->frames_per_block = p->lg.fpg > 1 ? p->lg.fpg : 1;
        // kernel: 2 register-cached, 7 register-cached BP with degree-grouped products,
        // 1 generic (LDS or global workspace), 3 thread-per-check, 5 min-sum with compressed check state,
        // 8 (3,6)-regular min-sum with rebuild-ready check state
        info->reserved = p->lg.ms36 ? 8 : p->lg.compact ? 5 : (p->lg.check_kernel ? 3 : (p->lg.grp ? 7 : (p->lg.reg_variant ? 2 : 1)));
    }
    return PL_OK;
}

extern "C" int pl_polar_plan_small_batch(const pl_plan* p, int64_t* max_frames) {
    if (!p || !max_frames) return fail(PL_EINVAL, "NULL argument");
    *max_frames = (p->kind == 0 && p->tree_small) ? (int64_t)p->small_grid_max * p->fpw : 0;
    return PL_OK;
}

extern "C" int pl_plan_destroy(pl_plan* p) {
    if (!p) return PL_OK;
    if (p->d_frozen_dec) hipFree(p->d_frozen_dec);
    if (p->d_info_pos) hipFree(p->d_info_pos);
    if (p->d_crc_g) hipFree(p->d_crc_g);
    if (p->d_r0k) hipFree(p->d_r0k);
    if (p->d_ldpc) hipFree(p->d_ldpc);
    p->ws.clear();  // each Workspace frees its buffer (hipFree waits for work that still uses it)
    delete p;
    return PL_OK;
}

extern "C" int pl_random_bits(uint64_t seed, int64_t frame_offset, int64_t batch, int32_t k, uint8_t* bits,
                              void* stream) {
    if (batch < 0 || k < 0 || (!bits && batch * k > 0)) return fail(PL_EINVAL, "bad argument");
    hipError_t e = pl::random_bits_launch(seed, frame_offset, batch, k, bits, (hipStream_t)stream);
    return e == hipSuccess ? PL_OK : hipfail(e, "random bits launch");
}

extern "C" int pl_polar_encode(const pl_plan* p, const uint8_t* msg, int64_t batch, uint8_t* cw, void* stream) {
    if (!p || p->kind != 0) return fail(PL_EINVAL, "not a polar plan");
    if (batch < 0 || (batch > 0 && (!msg || !cw))) return fail(PL_EINVAL, "bad argument");
    if (int rc = check_device(p)) return rc;
    const int64_t step = kMaxLaunchItems / 64;  // one wavefront per frame
    for (int64_t b0 = 0; b0 < batch; b0 += step) {
        const int64_t nb = std::min<int64_t>(step, batch - b0);
        hipError_t e = pl::polar_encode_launch(p->pg.N, p->pg.K, p->d_info_pos, msg + b0 * p->pg.K, nb,
                                               cw + b0 * p->pg.N, (hipStream_t)stream);
        if (e != hipSuccess) return hipfail(e, "polar encode launch");
    }
    return PL_OK;
}

extern "C" int pl_awgn_llr(const uint8_t* cw, int32_t n, int64_t batch, double snr_db, uint64_t seed,
                           int64_t frame_offset, double* llr, int64_t ld, void* stream) {
    if (n < 1 || batch < 0 || ld < n || (!llr && batch > 0)) return fail(PL_EINVAL, "bad argument");
    // src/channel/awgn.py:27-32 -- same double-precision expression order
    const double snr_linear = std::pow(10.0, snr_db / 10.0);
    const double sigma = std::sqrt(1.0 / (2.0 * snr_linear));
    const double sigma2 = sigma * sigma;
    hipError_t e = pl::awgn_launch(cw, n, batch, sigma, sigma2, seed, frame_offset, llr, ld, (hipStream_t)stream);
    return e == hipSuccess ? PL_OK : hipfail(e, "awgn launch");
}

extern "C" int pl_rayleigh_llr(const uint8_t* cw, int32_t n, int64_t batch, double snr_db, uint64_t seed,
                               int64_t frame_offset, double* llr, int64_t ld, void* stream) {
    if (n < 1 || batch < 0 || ld < n || (!llr && batch > 0)) return fail(PL_EINVAL, "bad argument");
    const double snr_linear = std::pow(10.0, snr_db / 10.0);  // src/channel/fading.py:21-23
    const double sigma = std::sqrt(1.0 / (2.0 * snr_linear));
    hipError_t e = pl::rayleigh_launch(cw, n, batch, sigma, sigma * sigma, seed, frame_offset, llr, ld,
                                       (hipStream_t)stream);
    return e == hipSuccess ? PL_OK : hipfail(e, "rayleigh launch");
}

extern "C" int pl_bsc(const uint8_t* cw, int32_t n, int64_t batch, double crossover_prob, uint64_t seed,
                      int64_t frame_offset, uint8_t* out, int64_t ld, void* stream) {
    if (n < 1 || batch < 0 || ld < n || !(crossover_prob >= 0.0 && crossover_prob <= 1.0) || (!out && batch > 0))
        return fail(PL_EINVAL, "bad argument (crossover probability must be in [0, 1])");  // bsc.py:26
    hipError_t e = pl::bsc_launch(cw, n, batch, crossover_prob, seed, frame_offset, out, ld, (hipStream_t)stream);
    return e == hipSuccess ? PL_OK : hipfail(e, "bsc launch");
}

extern "C" int pl_crc_append(uint8_t* msg, int64_t ld, int64_t batch, int32_t k_data, int32_t crc_len,
                             uint32_t poly, void* stream) {
    if (batch < 0 || k_data < 0 || crc_len < 1 || crc_len > 32 || ld < (int64_t)k_data + crc_len ||
        (batch > 0 && !msg))
        return fail(PL_EINVAL, "bad argument");
    hipError_t e = pl::crc_append_launch(msg, ld, batch, k_data, crc_len, poly, (hipStream_t)stream);
    return e == hipSuccess ? PL_OK : hipfail(e, "crc append launch");
}

extern "C" int pl_gf2_encode(const uint32_t* g_dev, int32_t k, int32_t n, const uint8_t* msg, int64_t ld_msg,
                             int64_t batch, uint8_t* cw, int64_t ld_cw, void* stream) {
    if (batch < 0 || k < 1 || n < 1 || ld_msg < k || ld_cw < n || (batch > 0 && (!g_dev || !msg || !cw)))
        return fail(PL_EINVAL, "bad argument");
    const int64_t step = kMaxLaunchItems / 64;  // one wavefront per frame
    for (int64_t b0 = 0; b0 < batch; b0 += step) {
        const int64_t nb = std::min<int64_t>(step, batch - b0);
        hipError_t e = pl::gf2_encode_launch(g_dev, k, n, msg + b0 * ld_msg, ld_msg, nb, cw + b0 * ld_cw, ld_cw,
                                             (hipStream_t)stream);
        if (e != hipSuccess) return hipfail(e, "gf2 encode launch");
    }
    return PL_OK;
}

extern "C" int pl_count_errors(const uint8_t* ref, int64_t ldr, const uint8_t* dec, int64_t ldd, int32_t width,
                               int64_t batch, int64_t* counts, void* stream) {
    if (batch < 0 || width < 0 || !counts || (batch > 0 && (!ref || !dec))) return fail(PL_EINVAL, "bad argument");
    hipError_t e = pl::count_errors_launch(ref, ldr, dec, ldd, width, batch, counts, (hipStream_t)stream);
    return e == hipSuccess ? PL_OK : hipfail(e, "count errors launch");
}
