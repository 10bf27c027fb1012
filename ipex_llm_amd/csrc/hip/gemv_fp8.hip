// Instantiations of the low-bit GEMV for decoder kinds: DK_FP8E4,DK_FP8E5
#include "lowbit_gemv.cuh"
namespace illm {
template void launch_gemv_dk<DK_FP8E4>(bool, int, int, dim3, const GemvArgs&, hipStream_t);
template void launch_gemv_dk<DK_FP8E5>(bool, int, int, dim3, const GemvArgs&, hipStream_t);
template void launch_gemv5_dk<DK_FP8E4>(bool, int, int, dim3, size_t, const GemvArgs&, hipStream_t);
template void launch_gemv5_dk<DK_FP8E5>(bool, int, int, dim3, size_t, const GemvArgs&, hipStream_t);
}  // namespace illm
