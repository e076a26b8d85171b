// render_f32.hip -- speed-mode (f32) instantiation of the render kernels.
// Built with -ffp-contract=on (FMA within a source expression) and native
// sqrt/rcp/rsq/sin/cos.
#include "render_kernel.hpp"

namespace rtw {

int launch_render_f32(const KParams<float>& p, int world, size_t lds_bytes, float* out,
                      hipStream_t stream, hipEvent_t mid) {
    return launch_render_impl<float>(p, world, lds_bytes, out, stream, mid);
}

}  // namespace rtw
