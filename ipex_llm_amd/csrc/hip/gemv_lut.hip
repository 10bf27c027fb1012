// Instantiations of the low-bit GEMV for decoder kinds: DK_LUT4,DK_FP4
#include "lowbit_gemv.cuh"
namespace illm {
template void launch_gemv_dk<DK_LUT4>(bool, int, int, dim3, const GemvArgs&, hipStream_t);
template void launch_gemv_dk<DK_FP4>(bool, int, int, dim3, const GemvArgs&, hipStream_t);
template void launch_gemv5_dk<DK_LUT4>(bool, int, int, dim3, size_t, const GemvArgs&, hipStream_t);
template void launch_gemv5_dk<DK_FP4>(bool, int, int, dim3, size_t, const GemvArgs&, hipStream_t);
}  // namespace illm
