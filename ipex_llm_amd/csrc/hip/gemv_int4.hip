// Instantiations of the low-bit GEMV for decoder kinds: DK_INT4S,DK_INT4A
#include "lowbit_gemv.cuh"
namespace illm {
template void launch_gemv_dk<DK_INT4S>(bool, int, int, dim3, const GemvArgs&, hipStream_t);
template void launch_gemv_dk<DK_INT4A>(bool, int, int, dim3, const GemvArgs&, hipStream_t);
template void launch_gemv5_dk<DK_INT4S>(bool, int, int, dim3, size_t, const GemvArgs&, hipStream_t);
template void launch_gemv5_dk<DK_INT4A>(bool, int, int, dim3, size_t, const GemvArgs&, hipStream_t);
}  // namespace illm
