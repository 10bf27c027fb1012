// Instantiations of the decode attention for F16, head dims 128
#include "attention.cuh"
namespace illm {
template void launch_d<F16, 128>(const AttnDecodeArgs&, hipStream_t);
}  // namespace illm
