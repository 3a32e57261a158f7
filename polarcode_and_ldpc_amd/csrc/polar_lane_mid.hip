// polar_lane_kernel instances for lists of 9..32 (16 / 32 lanes per frame);
// a translation unit of its own so it compiles beside polar_lane.hip.
#include "polar_lane.hpp"

namespace pl {

void* lane_pick_mid(int lcap, int F, int B) {
    return lcap == 16 ? lane_pick_f<16, false>(F, B) : lane_pick_f<32, false>(F, B);
}

}  // namespace pl
