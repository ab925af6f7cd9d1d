// sdr_cost3k2.hip -- CN = 3 cost-volume instantiations for D > 128 (two disparity pairs per lane);
// see sdr_cost3.hip.
#include "sdr_cost_kernel.hpp"

namespace sdr {

void launch_cost_cn3_k2(const Geometry& g, const CostArgs& a, int F, hipStream_t st) {
    switch (2 * g.SH2 + 1) {
        case 1: launch_cost_t<1, 2, 3>(g, a, F, st); break;
        case 3: launch_cost_t<3, 2, 3>(g, a, F, st); break;
        case 5: launch_cost_t<5, 2, 3>(g, a, F, st); break;
        case 7: launch_cost_t<7, 2, 3>(g, a, F, st); break;
        case 9: launch_cost_t<9, 2, 3>(g, a, F, st); break;
        case 11: launch_cost_t<11, 2, 3>(g, a, F, st); break;
        default: break;
    }
}

}  // namespace sdr
