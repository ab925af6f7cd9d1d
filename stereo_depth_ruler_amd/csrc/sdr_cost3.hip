// sdr_cost3.hip -- the cost-volume kernel for 3-channel input (calcPixelCostBT's cn == 3 branch:
// each channel's Sobel and raw BT costs are summed into the pixel cost).  The kernel template is
// sdr_cost_kernel.hpp; this file holds its CN = 3 instantiations.
#include "sdr_cost_kernel.hpp"

namespace sdr {

void launch_cost_cn3(const Geometry& g, const CostArgs& a, int F, hipStream_t st) {
    const int NR = 2 * g.SH2 + 1;
    const bool k2 = g.D > 128;
#define SDR_COST(NRV)                                                 \
    case NRV:                                                         \
        if (k2) launch_cost_t<NRV, 2, 3>(g, a, F, st);                \
        else launch_cost_t<NRV, 1, 3>(g, a, F, st);                   \
        break;
    switch (NR) {
        SDR_COST(1) SDR_COST(3) SDR_COST(5) SDR_COST(7) SDR_COST(9) SDR_COST(11)
        default: break;
    }
#undef SDR_COST
}

}  // namespace sdr
