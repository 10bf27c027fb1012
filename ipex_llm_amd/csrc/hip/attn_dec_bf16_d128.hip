// Instantiations of the decode attention for BF16, head dims 128
#include "attention.cuh"
namespace illm {
template void launch_d<BF16, 128>(const AttnDecodeArgs&, hipStream_t);
}  // namespace illm
