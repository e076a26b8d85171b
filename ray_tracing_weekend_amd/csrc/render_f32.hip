// render_f32.hip -- speed-mode (f32) instantiation of the render kernels.
// Built with -ffp-contract=on (FMA within a source expression) and native
// sqrt/rcp/rsq/sin/cos.
#include "render_kernel.hpp"

namespace rtw {

int launch_render_f32(const KParams<float>& p, int world, size_t lds_bytes, float* out,
                      hipStream_t stream, hipEvent_t mid) {
    return launch_render_impl<float>(p, world, lds_bytes, out, stream, mid);
}

int launch_assemble_f32(const float* ranks, size_t rank_stride, uint32_t nranks, uint32_t W, uint32_t H,
                        const uint32_t* slot, float* img, hipStream_t stream) {
    return launch_assemble_impl<float>(ranks, rank_stride, nranks, W, H, slot, img, stream);
}

}  // namespace rtw
