/*
 * polarldpc.h -- C-ABI of libpolarldpc.so, the MI355X (gfx950) batched
 * channel decoder.  Plain pointers and sizes only; device pointers are
 * hipMalloc'd (e.g. torch tensors' data_ptr()); `stream` is a hipStream_t
 * passed as void* (NULL = legacy default stream).
 *
 * The reference (B1ear/PolarCode_and_LDPC) is pure Python/NumPy and has no FFI;
 * each entry point below replaces the body of a reference Python method.  The
 * Python drop-in classes (polarcode_and_ldpc_amd.polar.SCDecoder, ...) bind
 * these with ctypes; INTEGRATION.md shows the binding.
 *
 * Return codes: 0 ok, <0 error (PL_E*); pl_last_error() gives a thread-local
 * message for the last failing call on the calling thread.
 */
#ifndef POLARLDPC_H
#define POLARLDPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PL_OK 0
#define PL_EINVAL (-1)       /* bad argument (reference: AssertionError)        */
#define PL_ENOMEM (-2)       /* device allocation failed                         */
#define PL_EHIP (-3)         /* HIP runtime error (launch, copy)                 */
#define PL_EUNSUPPORTED (-4) /* valid for the reference but not for this build,  */
                             /* or MS on a degree-1 check (reference ValueError) */

#define PL_LDPC_BP 0 /* BPDecoder: sum-product, tanh rule   (src/ldpc/decoder.py:11-205)  */
#define PL_LDPC_MS 1 /* MSDecoder: (normalised) min-sum     (src/ldpc/decoder.py:208-355) */

typedef struct pl_plan pl_plan;

typedef struct {
    int32_t kind;       /* 0 polar, 1 ldpc                                         */
    int32_t n_in;       /* LLRs per frame (N or n)                                 */
    int32_t n_out;      /* output bits per frame: K (polar) or n (ldpc)            */
    int32_t list_size;  /* polar: 0 = SC, >=1 = SCL list size                      */
    int32_t lds_bytes;  /* dynamic LDS per workgroup of the decode kernel          */
    int32_t fused_top;  /* polar: tree depths fused into the channel read (>=1)    */
    int32_t frames_per_block; /* frames one workgroup decodes                     */
    int32_t reserved;   /* polar: kernel (4 tree, 3 lane, 6 single-workgroup exact);
                           LDPC: 2 register-cached, 7 register-cached BP with
                           degree-grouped check products, 1 generic,
                           3 thread-per-check, 5 min-sum with compressed check state */
} pl_plan_info;

/* Polar SC / SCL plan.
 *   Replaces SCDecoder.__init__ (src/polar/decoder.py:16-36) when list_size == 0
 *   and SCLDecoder.__init__ (src/polar/decoder.py:191-223) when list_size >= 1.
 *   frozen_mask: host array [N], nonzero = frozen (the reference's frozen_bits
 *   index set as a mask; info bits = the complement, ascending).
 *   N power of two (2..32768); K = number of unfrozen positions, 1 <= K <= N
 *   (the reference's 0 < K < N assertion, decoder.py:17-18, is made by the
 *   Python layer on its K argument, exactly as the reference does).
 *   list_size: lists above 64 run one frame per workgroup of list_size/64
 *   wavefronts (16-bit path slots above 256); lists above 1024 run every frame
 *   through the exact single-workgroup decoder of polar_nan.hip (milliseconds
 *   per frame; its per-frame list state in LDS up to 2048 paths, in the
 *   workspace above).  list_size > 65536 or list_size * N > 2^30 returns
 *   PL_EUNSUPPORTED (the reference accepts any L, its scripts use <= 32).
 *   Cost of the largest lists: one frame's list state takes about
 *   list_size * N * 11 bytes of workspace (path LLR + bit arrays; 11 GB at
 *   list_size * N = 2^30, refused when larger than the device's memory), and
 *   one thread sorts the 2 * list_size candidates of every information bit,
 *   so such a frame takes seconds to minutes.  Tested up to list_size 4096.
 *   flags: 0 = fastest kernel built for (N, list size).  Diagnostics: bits 0-3
 *   force the lane kernel (polar_lane.hip) with that fused-top depth, 0x10 or
 *   0x20 the lane kernel with its default depth.
 *   The plan owns device constants only; decode workspace is per stream (grown
 *   lazily to the batch, see pl_decode) or caller-supplied (pl_decode_ws). */
int pl_polar_plan_create(int32_t N, int32_t K, const uint8_t* frozen_mask, int32_t list_size,
                         int32_t flags, pl_plan** out);

/* CRC-aided list selection (build-defined extension: the reference stores
 *   SCLDecoder's use_crc / crc_polynomial but never reads them, decoder.py:202-203,
 *   259).  With crc_len > 0 the decoded path is the first one, in descending
 *   final-metric order (ties: lower list index), whose u_hat[info bits] passes
 *   crc_check of src/polar/utils.py:128-163 (bit-serial, MSB first, zero initial
 *   register, generator `poly` without its x^crc_len term, e.g. CRC-8 0x1D,
 *   CRC-16 0x1021, CRC-24 0x1864CFB); if none passes, the argmax path.
 *   crc_len == 0 restores plain SCL.  List plans only (list_size >= 1). */
int pl_polar_plan_set_crc(pl_plan* plan, int32_t crc_len, uint32_t poly);

/* LDPC plan.  Replaces BPDecoder.__init__/_build_tanner_graph
 *   (src/ldpc/decoder.py:18-60) for algo PL_LDPC_BP and MSDecoder.__init__
 *   (:215-255) for PL_LDPC_MS.  H given as CSR over its m rows with ascending
 *   column indices: row_ptr[m+1], col_idx[row_ptr[m]] (host arrays).
 *   normalization is MSDecoder's factor (ignored for BP). */
int pl_ldpc_plan_create(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx,
                        int32_t algo, int32_t max_iter, int32_t early_stop, double normalization,
                        int32_t flags, pl_plan** out);

/* Batched decode: replaces SCDecoder.decode (decoder.py:38-71),
 *   SCLDecoder.decode (:225-262), BPDecoder.decode (src/ldpc/decoder.py:124-202)
 *   and MSDecoder.decode (:289-352) applied to `batch` frames.
 *   llr_dev : fp64 [batch][ld] device, row b = channel LLRs of frame b (n_in used)
 *   bits_dev: uint8 [batch][n_out] device, rows contiguous (pitch n_out).
 *             Polar: u_hat[info_bits] ascending; LDPC: the full hard-decision
 *             word (decoded = total <= 0).
 *   iters_dev: int32 [batch] device or NULL; LDPC: iterations run (BPDecoder's
 *             return_iterations); polar: ignored.
 *   Asynchronous on `stream`.  Deterministic bits: the decode path's atomics
 *   (the polar list kernels' frame-group counter and NaN mask ORs, LDPC
 *   syndrome XORs in LDS) decide which wavefront decodes which frames, never
 *   what a frame decodes to.
 *   Workspace: the plan keeps one device buffer per stream, sized on first use
 *   to this batch (polar: one slice per resident wavefront, at most the
 *   persistent grid; LDPC codes whose messages exceed LDS: one per frame of a
 *   chunk) and grown when a larger batch arrives (after draining that stream).
 *   Host threads may share a plan when each uses its own stream; calls on one
 *   stream are serialised by the plan. */
int pl_decode(pl_plan* plan, const double* llr_dev, int64_t batch, int64_t ld, uint8_t* bits_dev,
              int32_t* iters_dev, void* stream);

/* Workspace bytes pl_decode_ws needs to decode `batch` frames at full speed
 * (0: the kernel needs none).  Any size >= one unit works: a smaller
 * workspace runs fewer resident wavefronts / smaller LDPC chunks. */
int pl_plan_workspace_bytes(const pl_plan* plan, int64_t batch, int64_t* bytes);

/* pl_decode with a caller-supplied device workspace (the caller owns it and
 * must not use it concurrently elsewhere); no allocation, so safe inside
 * hipGraph capture. */
int pl_decode_ws(pl_plan* plan, const double* llr_dev, int64_t batch, int64_t ld, uint8_t* bits_dev,
                 int32_t* iters_dev, void* workspace_dev, int64_t workspace_bytes, void* stream);

/* Pre-allocate `stream`'s workspace for batches up to max_batch, so that
 * pl_decode on that stream never allocates (max_batch == 0: pl_plan_release).
 * If the device cannot hold the full-speed size, the largest halving of at
 * least one unit is kept (fewer resident wavefronts, same results) and later
 * decodes of up to max_batch frames run on it without retrying the allocation;
 * only another pl_plan_reserve (or a larger batch) retries. */
int pl_plan_reserve(pl_plan* plan, int64_t max_batch, void* stream);

/* Free `stream`'s workspace (after draining that stream).  A finished stream's
 * buffer is otherwise kept until pl_plan_destroy, invisible to torch's
 * caching allocator.  No-op for a stream the plan has not decoded on. */
int pl_plan_release(pl_plan* plan, void* stream);

/* Number of per-stream workspaces the plan holds and their total bytes. */
int pl_plan_workspace_stats(const pl_plan* plan, int64_t* streams, int64_t* bytes);

int pl_plan_get_info(const pl_plan* plan, pl_plan_info* info);
/* Build-defined extension (no reference counterpart): the largest batch a
 * pl_decode of this polar plan runs on its small-batch tree instance (one more
 * LDS depth and a 2-wave register budget, polar_tree.hip tree_table_small;
 * bits identical to the product instance), 0 if it has none.  Such batches fit
 * the device at 8 wavefronts per CU, where that instance is 6-15 % faster;
 * larger ones run the product instance (16 per CU).  PL_TREE_SMALL=0 at plan
 * creation turns it off. */
int pl_polar_plan_small_batch(const pl_plan* plan, int64_t* max_frames);
int pl_plan_destroy(pl_plan* plan);
const char* pl_last_error(void);

/* Calls that touch a plan's device memory -- pl_decode, pl_decode_ws,
 * pl_plan_reserve, pl_plan_release, pl_polar_plan_set_crc, pl_polar_encode,
 * pl_debug_polar_stamps -- must run with the plan's device current (the device
 * current at plan creation); otherwise they return PL_EINVAL and do nothing.
 * pl_plan_get_info, pl_plan_workspace_bytes and pl_plan_workspace_stats read
 * host state only; pl_plan_destroy may run on any device. */

/* Diagnostic build only (make DIAG=1; the product library returns
 * PL_EUNSUPPORTED): pl_decode of a polar plan through an instrumented kernel that adds
 * per-phase s_memtime cycle totals (summed over all frames) into stamps_dev[16]:
 * tree kernel (pl_plan_info.reserved == 4): [0] fused top, [1] workspace chains,
 * [2] LDS chain, [3] path metrics, [4] pruning/cloning, [5] partial-sum walk,
 * [6] final selection/output, [7] workspace fences; then counts of the
 * path-metric evaluations: [8] per-wave calls, [9] calls with a lane that
 * evaluates log1p(e^-x), [10] such lanes, [11] active lanes.  Timing differs
 * from pl_decode; read shares. */
int pl_debug_polar_stamps(pl_plan* plan, const double* llr_dev, int64_t batch, int64_t ld, uint8_t* bits_dev,
                          unsigned long long* stamps_dev, void* stream);

/* Diagnostic build only (the product library returns PL_EUNSUPPORTED): the
 * frame-per-wavefront SCL prototype (one wavefront per frame, eight lanes per
 * list path, every LLR pool in LDS) on a polar N=1024 L=8
 * plan, for timing against pl_decode.  stamps_dev[5] (may be NULL) receives
 * per-phase s_memtime cycle totals: descent, metric, pruning, partial sums,
 * output.  grid <= 0: one wavefront per LDS slot of the device. */
int pl_debug_polar_fpw(pl_plan* plan, const double* llr_dev, int64_t batch, int64_t ld, uint8_t* bits_dev,
                       unsigned long long* stamps_dev, int32_t grid, void* stream);

/* Diagnostic build only (the product library returns PL_EUNSUPPORTED): the
 * dead-store bound of the SCL N=1024 L=8 tree kernel.  mode 1
 * decodes recording, per frame group of 8 frames, which workspace pool arrays
 * (depths F..DL-1, one bit per node and lane plane) a right child's g reads and
 * which were stored: mask_dev u32 [ceil(batch/8)][2][words], zeroed by the
 * caller; mode 2 decodes the same frames again with every store of an array
 * not read in mode 1 skipped.  Bits equal pl_decode's by construction. */
int pl_debug_polar_deadstore(pl_plan* plan, const double* llr_dev, int64_t batch, int64_t ld, uint8_t* bits_dev,
                             uint32_t* mask_dev, int32_t mode, void* stream);

/* Diagnostic build only (the product library returns PL_EUNSUPPORTED): BP
 * decode of a (504,252)-class LDPC plan on the degree-grouped kernel with
 * per-phase s_memtime cycle totals added into stamps_dev[4][8] (per wavefront
 * index of the workgroup = per SIMD): [0] init, [1] early-stop vote, [2] check
 * pass, [3] its barrier, [4] variable pass, [5] tanh list, [6] closing
 * barrier, [7] output.  Timing differs from pl_decode; read shares. */
int pl_debug_ldpc_stamps(pl_plan* plan, const double* llr_dev, int64_t batch, int64_t ld, uint8_t* bits_dev,
                         int32_t* iters_dev, unsigned long long* stamps_dev, void* stream);

/* Test hook, diagnostic build only (the product library returns
 * PL_EUNSUPPORTED): pl_decode of a list plan that also reports which frames the
 * list kernel flagged for the exact NaN-order redo decoder (frames with a NaN
 * input or two inputs of magnitude >= 2^1000 / inf; polar_tree.hip).
 * flagged_host: `batch` host bytes, 1 = flagged.  Bits are the product path's. */
int pl_debug_polar_flagged(pl_plan* plan, const double* llr_dev, int64_t batch, int64_t ld, uint8_t* bits_dev,
                           uint8_t* flagged_host, void* stream);

/* Test hook, diagnostic build only (the product library returns
 * PL_EUNSUPPORTED): overwrite the device id a plan is bound to, so the
 * wrong-device check can be exercised on a one-GPU machine.  UNSAFE: it turns
 * the wrong-device protection off for that plan. */
int pl_debug_set_plan_device(pl_plan* plan, int32_t device);

/* ---- Monte-Carlo frame source (replaces src/channel/awgn.py:91-112 and the
 *      message/encode loop of benchmarks/ber_simulation.py:167-177) ---------- */

/* Random message bits, uint8 [batch][k], Philox4x32-10 keyed by (seed, global
 * frame index = frame_offset + b): identical for any sharding of the frames. */
int pl_random_bits(uint64_t seed, int64_t frame_offset, int64_t batch, int32_t k, uint8_t* bits_dev,
                   void* stream);

/* Polar encoder (src/polar/encoder.py:63-95 without CRC): u[info] = msg,
 * u[frozen] = 0, x = u * F^{(x)n} (src/polar/utils.py:193-229).
 * msg_dev uint8 [batch][K]; codeword_dev uint8 [batch][N]. */
int pl_polar_encode(const pl_plan* plan, const uint8_t* msg_dev, int64_t batch, uint8_t* codeword_dev,
                    void* stream);

/* BPSK (0 -> +1, 1 -> -1) + AWGN with sigma = sqrt(1/(2*10^(snr_db/10)))
 * (awgn.py:27-32, :47, :88), LLR = 2*y/sigma^2 (:75).  codeword_dev uint8 (bit 0 of each byte)
 * [batch][n] or NULL for the all-zero codeword.  Noise: Philox4x32-10 keyed by
 * (seed, frame_offset + b) + Box-Muller; statistically equivalent to the
 * reference's np.random.normal, not stream-identical. */
int pl_awgn_llr(const uint8_t* codeword_dev, int32_t n, int64_t batch, double snr_db, uint64_t seed,
                int64_t frame_offset, double* llr_dev, int64_t ld, void* stream);

/* Rayleigh fading + BPSK + AWGN (src/channel/fading.py:31-63): per bit
 * |h| (h complex Gaussian, E|h|^2 = 1), y = |h| s + N(0, sigma), LLR =
 * 2 y |h| / sigma^2, sigma = sqrt(1/(2*10^(snr_db/10))).  Philox keyed by (seed,
 * frame_offset + b, bit); statistically equivalent, not stream-identical. */
int pl_rayleigh_llr(const uint8_t* codeword_dev, int32_t n, int64_t batch, double snr_db, uint64_t seed,
                    int64_t frame_offset, double* llr_dev, int64_t ld, void* stream);

/* Binary symmetric channel (src/channel/bsc.py:33-49): out[b][j] = cw[b][j] ^
 * (u < crossover_prob), u uniform per bit; codeword_dev NULL = all-zero word. */
int pl_bsc(const uint8_t* codeword_dev, int32_t n, int64_t batch, double crossover_prob, uint64_t seed,
           int64_t frame_offset, uint8_t* out_dev, int64_t ld, void* stream);

/* CRC append (src/polar/utils.py:86-125 crc_encode, the message layout of
 * PolarEncoder(use_crc=True), src/polar/encoder.py:74-78): for each row b of the
 * uint8 device matrix msg [batch][ld], writes the crc_len CRC bits of
 * msg[b][0:k_data] (MSB first) to msg[b][k_data : k_data+crc_len]. */
int pl_crc_append(uint8_t* msg_dev, int64_t ld, int64_t batch, int32_t k_data, int32_t crc_len, uint32_t poly,
                  void* stream);

/* GF(2) block encoding (LDPC valid codewords; replaces LDPCEncoder.encode,
 * src/ldpc/encoder.py:56-95, whose direct-solving fallback :97-187 emits
 * non-codewords for rank-deficient H): cw[b][j] = XOR_i msg[b][i] & G[i][j] for
 * a k x n generator G given bit-packed column-wise in device memory,
 * g_dev[w * n + j] bit i = G[32 w + i][j], w < ceil(k / 32).  msg [batch][ld_msg]
 * and cw [batch][ld_cw] are uint8 0/1 device matrices. */
int pl_gf2_encode(const uint32_t* g_dev, int32_t k, int32_t n, const uint8_t* msg_dev, int64_t ld_msg,
                  int64_t batch, uint8_t* cw_dev, int64_t ld_cw, void* stream);

/* Error counting (benchmarks/ber_simulation.py:180-189):
 * counts_dev[0] += bit errors, [1] += frame errors, [2] += frames, over the
 * first `width` entries of each row.  counts_dev int64[3], device. */
int pl_count_errors(const uint8_t* ref_dev, int64_t ld_ref, const uint8_t* dec_dev, int64_t ld_dec,
                    int32_t width, int64_t batch, int64_t* counts_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* POLARLDPC_H */
