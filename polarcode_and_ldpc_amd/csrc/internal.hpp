// Host-side internal interface between the C-ABI (capi.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef PL_METRIC_FUSED_NMAX
// polar tree instances with n <= this use the fused log1p(exp(-x))
// (log1p_exp_neg): N=1024 L=8 -1.9 %, L=32 -2.6 % (round 4); N=4096 L=8 +3.6 %
// then (register allocation), -0.6 % with round 5's 16 waves per CU and
// de-duplicated fused top -- every tree instance (n <= 12) now uses it
#define PL_METRIC_FUSED_NMAX 12
#endif

namespace pl {

constexpr int kMaxDepth = 15;  // N <= 2^15

// What pl_plan_get_info reports about a polar plan's kernel.
struct PolarGeom {
    int N, K, F;
    int lds_bytes;
};

// Lane-per-path decoder (polar_lane.hip): one lane = one list path, 64/lcap
// frames per wavefront; tree depths tiered over registers / LDS / workspace.
struct LaneGeom {
    int N, n, K, Lsz, lcap, F, B, D, Dl, cw;
    int lw;                        // lanes per workgroup: 64, or lcap (> 64: one frame per workgroup)
    int lds_bytes, lds_final;
    int lds_xchg;                  // lcap > 64: metric / row / rank exchange scratch [lw]
    int lds_pool[kMaxDepth + 2];   // byte offset of LDS pool depth d (Dl <= d <= D): [2^(n-d)][lw] f64
    int lds_bl[kMaxDepth + 2];     // byte offset of single-word beta depth d: [lw] u32
    int bl_words[kMaxDepth + 2];   // beta words per slot at depth d
    int64_t ws_pool[kMaxDepth + 2];  // workspace byte offset of pool depth d (F <= d < Dl)
    int64_t ws_bl[kMaxDepth + 2];    // workspace byte offset of multi-word beta depth d: [words][lw] u32
    int64_t ws_walk;                 // [2][cw][lw] u32 walk buffers
    int64_t ws_bytes;                // workspace bytes per workgroup
};
int lane_geom(int N, int K, int list_size, int F, int lds_budget, LaneGeom* g);
hipError_t lane_prepare(const LaneGeom& g, bool sc, int* max_blocks_per_cu);
hipError_t lane_launch(const LaneGeom& g, bool sc, const double* llr, int64_t ld, uint8_t* out,
                       const uint32_t* frozen_dec, const int32_t* info_pos, int64_t batch, unsigned char* ws,
                       int grid, const uint32_t* crc_g, uint64_t* nan_masks, hipStream_t s);

// v4 lane-per-path decoder with compile-time geometry (polar_tree.hip); built
// for the (n, list capacity) pairs in its table, polar_lane.hip covers the rest.
struct TreeInfo {
    void* fn;
    void* fn_stamps;
    void* fn_ds[2];  // PL_DIAG: dead-store record / replay instances (headline geometry only)
    int lds_bytes;
    int64_t ws_bytes;  // workspace bytes per resident wavefront
    int F, DL, fpw;
};
bool tree_lookup(int n, int lcap, bool sc, TreeInfo* info);
// a list instance for batches that fit the device at its 8 waves per CU (one
// more LDS depth, 2-wave register budget), if (n, lcap) has one
bool tree_lookup_small(int n, int lcap, bool sc, TreeInfo* info);
// The tree and lane kernels' frame groups (FPW frames) past the first one per
// wavefront come from a u32 counter in the kSchedBytes just before their
// slices (polar_tree.hip, polar_lane.hpp); tree_launch / lane_launch zero it.
constexpr int kSchedBytes = 4096;
hipError_t tree_prepare(const TreeInfo& t, int* max_blocks_per_cu);
hipError_t tree_launch(const TreeInfo& t, const double* llr, int64_t ld, uint8_t* out, const uint32_t* frozen_dec,
                       const int32_t* info_pos, int64_t batch, int K, int Lsz, unsigned char* ws, int grid,
                       unsigned long long* stamps, const uint32_t* crc_g, const void* aux, hipStream_t s,
                       int ds_mode = 0);  // ds_mode 1 / 2 (PL_DIAG): the dead-store record / replay instance

// SCL frames with NaN path metrics (polar_nan.hip): the list kernels set bit f
// of masks[wave][pass] for frame f of that pass; polar_nan_redo_kernel decodes
// those frames again in the reference's candidate order.  A launch runs at most
// kNanMaskPasses passes of its persistent grid.
constexpr int kNanMaskPasses = 64;
constexpr int kMaxRedoList = 2048;  // the redo kernel's list state of one frame fits LDS up to here
// lists above kMaxRedoList keep that state in global scratch; list_size * N is
// bounded so that the kernel's int indices (path x element) stay below 2^31
constexpr int kMaxListSize = 1 << 16;
constexpr int64_t kMaxListTimesN = (int64_t)1 << 30;
// Bytes of the mask words of up to `grid` wavefronts, u64 [grid][kNanMaskPasses]
// (a multiple of 64 KB, at the start of a list plan's workspace).  They are zero
// between decodes: zeroed when the workspace is allocated, ORed by the list
// kernels, re-zeroed by the redo kernel after it reads them.
inline size_t nan_mask_region(int64_t grid) { return ((size_t)grid * 8 * kNanMaskPasses + 65535) / 65536 * 65536; }
size_t nan_redo_unit(int N, int list_size);  // scratch bytes per redo workgroup
int nan_redo_lds_bytes(int list_size);
hipError_t nan_redo_prepare(int list_size);
// path-metric evaluation of the list kernel whose frames are redone: the lane
// kernel's path_metrics (libm-style log1p(exp(-x))), or the tree instances'
// path_metrics_fast with the fused (n <= PL_METRIC_FUSED_NMAX) or lean form
enum RedoMetric { kRedoMetricLane = 0, kRedoMetricFused = 1, kRedoMetricLean = 2 };
hipError_t nan_redo_launch(const double* llr, int64_t ld, uint8_t* out, int64_t batch, int N, int K, int Lsz,
                           const uint32_t* frozen_dec, const int32_t* info_pos, const uint32_t* crc_g,
                           uint64_t* masks, int grid, int fpw, int metric, unsigned char* scratch,
                           size_t scratch_bytes, int max_blocks, hipStream_t s);

#if PL_DIAG
// frame-per-wavefront SCL N=1024 L=8 prototype (polar_fpw.hip, diagnostic build)
hipError_t fpw_launch(const double* llr, int64_t ld, uint8_t* out, const uint32_t* frozen_dec,
                      const int32_t* info_pos, int64_t batch, int K, unsigned long long* stamps, int grid,
                      hipStream_t st);
#endif

hipError_t polar_encode_launch(int N, int K, const int32_t* info_pos, const uint8_t* msg,
                               int64_t batch, uint8_t* cw, hipStream_t s);
hipError_t random_bits_launch(uint64_t seed, int64_t off, int64_t batch, int k, uint8_t* bits,
                              hipStream_t s);
hipError_t awgn_launch(const uint8_t* cw, int n, int64_t batch, double sigma, double sigma2,
                       uint64_t seed, int64_t off, double* llr, int64_t ld, hipStream_t s);
hipError_t rayleigh_launch(const uint8_t* cw, int n, int64_t batch, double sigma, double sigma2, uint64_t seed,
                           int64_t off, double* llr, int64_t ld, hipStream_t s);
hipError_t bsc_launch(const uint8_t* cw, int n, int64_t batch, double p, uint64_t seed, int64_t off, uint8_t* out,
                      int64_t ld, hipStream_t s);
hipError_t gf2_encode_launch(const uint32_t* g, int k, int n, const uint8_t* msg, int64_t ldm, int64_t batch,
                             uint8_t* cw, int64_t ldc, hipStream_t s);
hipError_t crc_append_launch(uint8_t* msg, int64_t ld, int64_t batch, int k_data, int crc_len, uint32_t poly,
                             hipStream_t s);
hipError_t count_errors_launch(const uint8_t* ref, int64_t ldr, const uint8_t* dec, int64_t ldd,
                               int width, int64_t batch, int64_t* counts, hipStream_t s);

// ---- LDPC ----
struct LdpcGeom {
    int m, n, E, max_iter, early_stop, algo, maxdc, maxdv;
    double norm;
    int threads;       // threads per workgroup (one frame per workgroup)
    int lds_bytes;     // 0 => messages live in the global workspace
    int use_global;
    int check_kernel;  // 1: ldpc_check_kernel (thread per check, state in LDS)
    int reg_variant;   // > 0: ldpc_reg_kernel instance (constant variable degree, LDS state)
    int compact;       // 1: ldpc_ms_compact_kernel (min-sum, compressed check state in LDS)
    int regular;       // every check has degree maxdc and every variable degree maxdv
    int grp;           // BP reg variant: ldpc_bp_grp_kernel (degree-grouped products, padded T'/C')
    int tl;            // grp: length of the padded T'/C' arrays (doubles)
    int npad;          // grp: pad positions listed after the variable slots (a multiple of 256, -1 filled)
    int ms36;          // > 0: ldpc_ms36_kernel<ms36> ((3,6)-regular min-sum, n = 1024 ms36)
    int fpg;           // grp: frames per workgroup (1 or 2)
};
struct LdpcDev {
    const int32_t* row_ptr;   // [m+1]
    const int32_t* col_idx;   // [E]   (check-major edge -> variable)
    const int32_t* edge_chk;  // [E]   edge -> check
    const int32_t* var_ptr;   // [n+1]
    const int32_t* var_edge;  // [E]   var-major list of check-major edge ids (ascending check)
    const int32_t* edge_meta; // [E]   first edge of the edge's check | check degree << 20
    const int32_t* var_chk;   // [E]   check of var_edge[k]
    const int32_t* var_cp;    // [E]   check << 4 | position in the check, of var_edge[k]
    // grp (ldpc_bp_grp_kernel): per edge slot (256 EPT of them) the T' position
    // of the edge's check | position in the check << 16 | its slot's D_s << 20;
    // per variable slot q (256 VPT of them): [q][DV] T' positions, [q][DV]
    // checks, then [q] the variable (-1: none); then npad pad positions
    const int32_t* grp_meta;  // [256 EPT]
    const int32_t* var_tpos;  // [256 VPT (2 DV + 1)]
    // ms36 (ldpc_ms36_kernel), 16-byte aligned: per variable [8] u32, its three
    // edge words (LDS rec address of the check | 3 * position) then the three
    // LDS meta addresses, in the reference's np.sum order (ascending check);
    // then per check [4] u32, the LDS addresses 8v of its six variables, two per word
    const uint32_t* ms_vw;    // [n][8] + [m][4]
};
hipError_t ldpc_launch(const LdpcGeom& g, const LdpcDev& d, const double* llr, int64_t ld,
                       uint8_t* bits, int32_t* iters, int64_t batch, double* work, hipStream_t s);
hipError_t ldpc_prepare(const LdpcGeom& g);
#if PL_DIAG
hipError_t ldpc_launch_stamped(const LdpcGeom& g, const LdpcDev& d, const double* llr, int64_t ld, uint8_t* bits,
                               int32_t* iters, int64_t batch, unsigned long long* stamps, hipStream_t s);
#endif
size_t ldpc_work_bytes_per_frame(const LdpcGeom& g);
int ldpc_reg_variant(int dv, int E, int n);  // 0: none fits
size_t ldpc_reg_list_bytes(int variant);      // BP tanh lists of an ldpc_reg_kernel instance
int ldpc_reg_ept(int variant);                // edges per thread of an ldpc_reg_kernel instance
int ldpc_reg_vpt(int variant);                // variables per thread
int ldpc_ms36_lds(int n);                     // LDS of the ldpc_ms36_kernel instance for n (0: none)

}  // namespace pl
