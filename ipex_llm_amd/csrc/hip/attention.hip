// Decode attention dispatch by head dim and dtype; the kernels are in
// attention.cuh and instantiated per (dtype, head dim) in attn_dec_*.hip so
// the variants compile in parallel.
#include "attention.cuh"

namespace illm {

extern template void launch_d<BF16, 64>(const AttnDecodeArgs&, hipStream_t);
extern template void launch_d<BF16, 80>(const AttnDecodeArgs&, hipStream_t);
extern template void launch_d<BF16, 96>(const AttnDecodeArgs&, hipStream_t);
extern template void launch_d<BF16, 128>(const AttnDecodeArgs&, hipStream_t);
extern template void launch_d<BF16, 256>(const AttnDecodeArgs&, hipStream_t);
extern template void launch_d<F16, 64>(const AttnDecodeArgs&, hipStream_t);
extern template void launch_d<F16, 80>(const AttnDecodeArgs&, hipStream_t);
extern template void launch_d<F16, 96>(const AttnDecodeArgs&, hipStream_t);
extern template void launch_d<F16, 128>(const AttnDecodeArgs&, hipStream_t);
extern template void launch_d<F16, 256>(const AttnDecodeArgs&, hipStream_t);

template <typename T>
static void launch_t(const AttnDecodeArgs& a, hipStream_t st) {
  switch (a.D) {
    case 64: launch_d<T, 64>(a, st); break;
    case 80: launch_d<T, 80>(a, st); break;
    case 96: launch_d<T, 96>(a, st); break;
    case 128: launch_d<T, 128>(a, st); break;
    case 256: launch_d<T, 256>(a, st); break;
  }
}

void launch_attn_decode(bool bf16, const AttnDecodeArgs& a, hipStream_t st) {
  if (bf16) launch_t<BF16>(a, st); else launch_t<F16>(a, st);
}

}  // namespace illm
