// Instantiations of the decode attention for F16, head dims 64, 80, 96, 256
#include "attention.cuh"
namespace illm {
template void launch_d<F16, 64>(const AttnDecodeArgs&, hipStream_t);
template void launch_d<F16, 80>(const AttnDecodeArgs&, hipStream_t);
template void launch_d<F16, 96>(const AttnDecodeArgs&, hipStream_t);
template void launch_d<F16, 256>(const AttnDecodeArgs&, hipStream_t);
}  // namespace illm
