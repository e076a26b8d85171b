// render_f64.hip -- parity-mode (f64) instantiation of the render kernels.
// Built with -ffp-contract=off: every a*b+c rounds twice, in the reference's
// operation order, so the output is bit-comparable with the CPU oracle.
#include "render_kernel.hpp"

namespace rtw {

int launch_render_f64(const KParams<double>& p, int world, size_t lds_bytes, double* out,
                      hipStream_t stream, hipEvent_t mid) {
    return launch_render_impl<double>(p, world, lds_bytes, out, stream, mid);
}

int launch_assemble_f64(const double* ranks, size_t rank_stride, uint32_t nranks, uint32_t W, uint32_t H,
                        const uint32_t* slot, double* img, hipStream_t stream) {
    return launch_assemble_impl<double>(ranks, rank_stride, nranks, W, H, slot, img, stream);
}

}  // namespace rtw
