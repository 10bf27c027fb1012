// The decode GEMV XM instantiations (sym_int4, bf16; lowbit_gemv5.cuh
// launch5_xm_int4s), apart from the generic kernels: this unit is built without
// -amdgpu-mfma-vgpr-form (_build.py), with which hipcc miscompiles some of them
#define ILLM_GEMV5_XM_IMPL 1
#include "lowbit_gemv.cuh"
