// Instantiations of the low-bit GEMV for decoder kinds: DK_INT8S,DK_INT8A
#include "lowbit_gemv.cuh"
namespace illm {
template void launch_gemv_dk<DK_INT8S>(bool, int, int, dim3, const GemvArgs&, hipStream_t);
template void launch_gemv_dk<DK_INT8A>(bool, int, int, dim3, const GemvArgs&, hipStream_t);
template void launch_gemv5_dk<DK_INT8S>(bool, int, int, dim3, size_t, const GemvArgs&, hipStream_t);
template void launch_gemv5_dk<DK_INT8A>(bool, int, int, dim3, size_t, const GemvArgs&, hipStream_t);
}  // namespace illm
