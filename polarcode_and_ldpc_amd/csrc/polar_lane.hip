// Batched polar SC / SCL decoder, lane-per-path kernel: host side (geometry,
// launch) and the SC / list 1..8 instances.  The kernel is in polar_lane.hpp.
#include "polar_lane.hpp"

namespace pl {

// ------------------------------------------------------------------- host
static int lane_bottom(int n, int F) { int b = n - F; return b > 3 ? 3 : (b < 0 ? 0 : b); }

int lane_geom(int N, int K, int list_size, int F, int lds_budget, LaneGeom* g) {
    int n = 0;
    while ((1 << n) < N) ++n;
    int lcap = 1;
    while (lcap < (list_size < 1 ? 1 : list_size)) lcap <<= 1;
    if (lcap >= 64) F = 3;  // large lists: one fused-top depth is built (lane_pick_big)
    if (F > n) F = n;
    if (F < 1) F = 1;
    *g = LaneGeom{};
    g->N = N; g->n = n; g->K = K; g->Lsz = list_size < 1 ? 1 : list_size; g->lcap = lcap;
    g->lw = lcap > 64 ? lcap : 64;
    g->F = F; g->B = lane_bottom(n, F); g->D = n - g->B;
    g->cw = N / 32 < 1 ? 1 : N / 32;
    const int fpw = lcap >= 64 ? 1 : 64 / lcap;
    const int lw = g->lw;
    // LDS: single-word beta depths + final transform buffer (+ list exchange
    // scratch for lcap > 64: (m0, m1), pointer row, ranks per lane) + pool depths [Dl, D]
    int lds = 0;
    for (int d = 1; d <= n; ++d) {
        const int w = (1 << (n - d)) / 32;
        g->bl_words[d] = w < 1 ? 1 : w;
        if (g->bl_words[d] == 1) { g->lds_bl[d] = lds; lds += lw * 4; }
    }
    g->lds_final = lds; lds += fpw * g->cw * 4;
    lds = (lds + 15) & ~15;
    if (lcap > 64) { g->lds_xchg = lds; lds += lw * (16 + (lcap > 256 ? 64 : 32) + 8); }  // (m0, m1), pointer row, ranks
    int Dl = g->D + 1;
    if (g->B > 0) {
        // deepest depths first, while they fit the LDS budget
        while (Dl - 1 >= F && lds + (1 << (n - (Dl - 1))) * lw * 8 <= lds_budget) {
            --Dl;
            g->lds_pool[Dl] = lds;
            lds += (1 << (n - Dl)) * lw * 8;
        }
    }
    g->Dl = Dl;
    g->lds_bytes = (lds + 15) & ~15;
    // workspace per wave: pool depths [F, Dl), multi-word beta depths, walk buffers
    int64_t ws = 0;
    if (g->B > 0)
        for (int d = F; d < Dl; ++d) { g->ws_pool[d] = ws; ws += (int64_t)(1 << (n - d)) * lw * 8; }
    for (int d = 1; d <= n; ++d)
        if (g->bl_words[d] > 1) { g->ws_bl[d] = ws; ws += (int64_t)g->bl_words[d] * lw * 4; }
    g->ws_walk = ws; ws += (int64_t)2 * g->cw * lw * 4;
    g->ws_bytes = (ws + 255) & ~(int64_t)255;
    return g->lds_bytes;
}

static void* lane_kernel(const LaneGeom& g, bool sc) {
    if (sc) return lane_pick_f<1, true>(g.F, g.B);
    switch (g.lcap) {
        case 1: return lane_pick_f<1, false>(g.F, g.B);
        case 2: return lane_pick_f<2, false>(g.F, g.B);
        case 4: return lane_pick_f<4, false>(g.F, g.B);
        case 8: return lane_pick_f<8, false>(g.F, g.B);
        case 16:
        case 32: return lane_pick_mid(g.lcap, g.F, g.B);
        case 64:   // one frame per wave
        case 128:  // one frame per workgroup of 2 waves
        case 256:                                             // 4 waves
        case 512:                                             // 8 waves (16-bit row fields)
        case 1024: return lane_pick_large(g.lcap, g.F, g.B);  // 16 waves
        default: return nullptr;
    }
}

hipError_t lane_prepare(const LaneGeom& g, bool sc, int* max_blocks_per_cu) {
    void* k = lane_kernel(g, sc);
    if (!k) return hipErrorInvalidValue;
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, g.lds_bytes);
    if (e != hipSuccess) return e;
    int nb = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, g.lw, g.lds_bytes);
    if (e != hipSuccess) return e;
    *max_blocks_per_cu = nb < 1 ? 1 : nb;
    return hipSuccess;
}

hipError_t lane_launch(const LaneGeom& g, bool sc, const double* llr, int64_t ld, uint8_t* out,
                       const uint32_t* frozen_dec, const int32_t* info_pos, int64_t batch, unsigned char* ws,
                       int grid, const uint32_t* crc_g, uint64_t* nan_masks, hipStream_t s) {
    void* k = lane_kernel(g, sc);
    if (!k) return hipErrorInvalidValue;
    LaneGeom gg = g;
    void* args[] = {&gg,           (void*)&llr,   (void*)&ld, (void*)&out, (void*)&frozen_dec, (void*)&info_pos,
                    (void*)&batch, (void*)&ws,    (void*)&crc_g, (void*)&nan_masks};
    // the frame-group counter (polar_lane.hpp: group loop)
    if (hipError_t e = hipMemsetAsync(ws - kSchedBytes, 0, 4, s); e != hipSuccess) return e;
    return hipLaunchKernel(k, dim3((unsigned)grid), dim3((unsigned)g.lw), args, g.lds_bytes, s);
}

}  // namespace pl
