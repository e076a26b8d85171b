// render_f64_lgrid.hip -- parity-mode (f64) instantiation of the render
// kernels with the light BVH / light grid (C3, C5 and other long light
// lists).  Built like render_f64.hip (-ffp-contract=off); its own unit so
// that these kernels keep the plain IEEE quotients (RTW_FASTDIV 0: the shared-
// divisor sequence of rtw_device.hpp div3 measured C3 f64 +1.1 % here, where
// the walk's registers are tight, and -1.3 % in the Book-1 kernels).
#ifndef RTW_FASTDIV_LGRID
#define RTW_FASTDIV_LGRID 0
#endif
#undef RTW_FASTDIV
#define RTW_FASTDIV RTW_FASTDIV_LGRID
#include "render_kernel.hpp"

namespace rtw {

int launch_render_f64_lgrid(const KParams<double>& p, int world, size_t lds_bytes, hipStream_t stream, int kopt) {
    return launch_lgrid_impl<double>(p, world, lds_bytes, stream, kopt);
}

}  // namespace rtw
