// sdr_cost3.hip -- the cost-volume kernel for 3-channel input (calcPixelCostBT's cn == 3 branch:
// each channel's Sobel and raw BT costs are summed into the pixel cost).  The kernel template is
// sdr_cost_kernel.hpp; this file holds its CN = 3 instantiations for D <= 128 (K = 1) and the
// dispatch; sdr_cost3k2.hip the D > 128 ones (two translation units that compile in parallel).
#include "sdr_cost_kernel.hpp"

namespace sdr {

void launch_cost_cn3_k2(const Geometry& g, const CostArgs& a, int F, hipStream_t st);

void launch_cost_cn3(const Geometry& g, const CostArgs& a, int F, hipStream_t st) {
    if (g.D > 128) return launch_cost_cn3_k2(g, a, F, st);
    switch (2 * g.SH2 + 1) {
        case 1: launch_cost_t<1, 1, 3>(g, a, F, st); break;
        case 3: launch_cost_t<3, 1, 3>(g, a, F, st); break;
        case 5: launch_cost_t<5, 1, 3>(g, a, F, st); break;
        case 7: launch_cost_t<7, 1, 3>(g, a, F, st); break;
        case 9: launch_cost_t<9, 1, 3>(g, a, F, st); break;
        case 11: launch_cost_t<11, 1, 3>(g, a, F, st); break;
        default: break;
    }
}

}  // namespace sdr
