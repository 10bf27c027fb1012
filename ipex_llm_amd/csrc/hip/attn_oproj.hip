// Decode attention -> o projection as ONE launch (batch <= 16, fused-RoPE v3
// attention with its in-kernel combine, then the o_proj split-K atomic GEMV).
//
// Reference: the decode step of SRC/transformers/models/llama.py:129-205
// (attention, then o_proj); the VERDICT's "persistent launch" item for the
// launch-ramp-bound small GEMVs.
//
// Workgroups [0, nA) are the attention's (split, kv head, batch) workgroups,
// the rest are the o_proj GEMV's.  A GEMV workgroup requests its first weight
// chunks (independent of the attention), then waits until every (batch, kv
// head) merge has signalled (the attention's merging workgroups store their
// output rows write-through and add one to a counter after their stores are
// acknowledged), and stages its x slice through the write-through path: the
// o_proj's launch ramp and weight round trip overlap the attention instead of
// following it.  Workgroups are dispatched in id order on each XCD, so every
// attention workgroup is resident before any waiting GEMV workgroup can hold
// its slot: no deadlock; the wait is bounded anyway (ERR_CHAIN).  The last
// GEMV workgroup past the wait resets the counters for the next launch.
// One 256-thread shape: the attention runs 4-wave splits, the GEMV 4-wave
// groups; both views share the dynamic LDS.
#include "attention.cuh"
#include "lowbit_gemv.cuh"

namespace illm {

namespace {

struct AOChain {
  int nA, ns, gx, gy;
  int* cnt;
  int* dep;
  int* err;
};

template <typename T, int RQ, int DK>
__global__ void __launch_bounds__(256, 3) attn_oproj_kernel(const AttnDecodeArgs aa, const GemvArgs ga,
                                                            const AOChain c) {
  extern __shared__ __attribute__((aligned(16))) uint8_t ao_smem[];
  const int id = (int)blockIdx.x;
  if (id < c.nA) {
    const int split = id % c.ns, r = id / c.ns;
    attn_v3_body<T, 128, 4, RQ, true>(aa, split, r % aa.Hkv, r / aa.Hkv, c.ns,
                                      *reinterpret_cast<V3Smem<128, 4, RQ>*>(ao_smem), c.cnt);
    return;
  }
  const int j = id - c.nA;
  const G5Wait w{c.cnt, aa.B * aa.Hkv, c.dep, c.gx * c.gy, c.err};
  gemv5_body<DK, T, EPI_ATOMIC, 1, 1, false, 4, 4, false>(ga, G5Blk{j % c.gx, j / c.gx, 0, c.gx, c.gy, 1}, &w);
}

template <typename T, int RQ, int DK>
void launch_ao(const AttnDecodeArgs& aa, const GemvArgs& ga0, dim3 ggrid, size_t gshmem, int* cnt, hipStream_t st) {
  using C = typename std::conditional<DK == DK_LUT4, F16, T>::type;
  GemvArgs ga = ga0;
  ga.nib_mask = 0x000F000Fu;
  ga.nib_magic = Raw<C>::k4;
  ga.nw = 4;
  const int ns = (aa.nsplit * SPLIT + V3_KPW * 4 - 1) / (V3_KPW * 4);
  const AOChain c{ns * aa.Hkv * aa.B, ns, (int)ggrid.x, (int)ggrid.y, cnt, cnt + 1, aa.err};
  const size_t sh = std::max(sizeof(V3Smem<128, 4, RQ>), gshmem);
  hipLaunchKernelGGL((attn_oproj_kernel<T, RQ, DK>), dim3((unsigned)(c.nA + c.gx * c.gy)), dim3(256), sh, st, aa,
                     ga, c);
}

template <typename T, int RQ>
bool launch_ao_dk(int dk, const AttnDecodeArgs& aa, const GemvArgs& ga, dim3 g, size_t sh, int* cnt, hipStream_t st) {
  switch (dk) {
    case DK_INT4S: launch_ao<T, RQ, DK_INT4S>(aa, ga, g, sh, cnt, st); return true;
    case DK_INT4A: launch_ao<T, RQ, DK_INT4A>(aa, ga, g, sh, cnt, st); return true;
    default: return false;
  }
}

}  // namespace

bool launch_attn_oproj(int dk, bool bf16, const AttnDecodeArgs& aa, const GemvArgs& ga, dim3 ggrid, size_t gshmem,
                       int* cnt, hipStream_t st) {
  // the fused-RoPE v3 path with its in-kernel combine, head dim 128, 4-wave splits
  if (aa.D != 128 || aa.Tq != 1 || aa.rq_part == nullptr || aa.v3_counters == nullptr || !v3_ok(aa, 128) ||
      ga.M != aa.B || gshmem > 64 * 1024)
    return false;
  const int rq = aa.rq_prerot && aa.rq_bias == nullptr ? 2 : 1;
  if (bf16) return rq == 2 ? launch_ao_dk<BF16, 2>(dk, aa, ga, ggrid, gshmem, cnt, st)
                           : launch_ao_dk<BF16, 1>(dk, aa, ga, ggrid, gshmem, cnt, st);
  return rq == 2 ? launch_ao_dk<F16, 2>(dk, aa, ga, ggrid, gshmem, cnt, st)
                 : launch_ao_dk<F16, 1>(dk, aa, ga, ggrid, gshmem, cnt, st);
}

}  // namespace illm
