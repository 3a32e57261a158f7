// polar_lane_kernel instances for lists of 33..256: one frame per wavefront
// (64) or per workgroup of 2 / 4 wavefronts (128 / 256).
#include "polar_lane.hpp"

namespace pl {

void* lane_pick_large(int lcap, int F, int B) {
    switch (lcap) {
        case 64: return lane_pick_big<64>(F, B);
        case 128: return lane_pick_big<128>(F, B);
        default: return lane_pick_big<256>(F, B);
    }
}

}  // namespace pl
