// polar_lane_kernel instances for lists of 33..1024: one frame per wavefront
// (64) or per workgroup of 2 / 4 / 8 / 16 wavefronts (128 .. 1024).
#include "polar_lane.hpp"

namespace pl {

void* lane_pick_large(int lcap, int F, int B) {
    switch (lcap) {
        case 64: return lane_pick_big<64>(F, B);
        case 128: return lane_pick_big<128>(F, B);
        case 256: return lane_pick_big<256>(F, B);
        case 512: return lane_pick_big<512>(F, B);
        default: return lane_pick_big<1024>(F, B);
    }
}

}  // namespace pl
