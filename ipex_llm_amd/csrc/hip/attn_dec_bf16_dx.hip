// Instantiations of the decode attention for BF16, head dims 64, 80, 96, 256
#include "attention.cuh"
namespace illm {
template void launch_d<BF16, 64>(const AttnDecodeArgs&, hipStream_t);
template void launch_d<BF16, 80>(const AttnDecodeArgs&, hipStream_t);
template void launch_d<BF16, 96>(const AttnDecodeArgs&, hipStream_t);
template void launch_d<BF16, 256>(const AttnDecodeArgs&, hipStream_t);
}  // namespace illm
