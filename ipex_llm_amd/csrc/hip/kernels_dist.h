// Host-callable launchers of the expert-parallel peer all-to-all (ep_a2a.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace illm {

constexpr int EP_MAX_RANKS = 8;
constexpr int EP_BLOCKS = 64;
constexpr int64_t EP_SIG_BYTES = 2 * EP_BLOCKS * EP_MAX_RANKS * 4;   // [2 phases][blocks][src] u32
constexpr int64_t EP_CNT_BYTES = 256;                                 // i32 counts [src]
// bytes of one rank's EP buffer: signals | counts | meta [W][cap] i32 | recv [W][cap][H] | ret [W][cap][H]
constexpr int64_t ep_buffer_bytes(int world, int64_t cap, int64_t H) {
  return EP_SIG_BYTES + EP_CNT_BYTES + (int64_t)world * cap * 4 + 2 * (int64_t)world * cap * H * 2;
}

struct EpA2AArgs {
  uint8_t* bufs[EP_MAX_RANKS];  // every rank's EP buffer (own included), mapped
  int rank, world;
  int64_t cap;                  // slots per (source, destination) region
  int H;                        // hidden size (16-bit elements, % 8 == 0)
  int bf16;
  const uint16_t* x;            // [T, H] this rank's tokens
  int T, k, el;                 // tokens, top-k, experts per rank
  const int32_t* ids;           // [T * k] global expert ids
  const int32_t* off;           // [W + 1] pairs per destination (moe_align over dst ranks)
  const int32_t* rows;          // [T * k] pair ids sorted by destination
  int32_t* pos;                 // [T * k] sorted position of every pair (dispatch writes)
  int32_t* counts;              // [W + 1] received pairs per source; [W] = return status
  const uint16_t* out_rows;     // [W * cap, H] expert outputs by received slot (return)
  const float* w;               // [T * k] routing weights (combine)
  uint16_t* y;                  // [T, H] combined output
  const uint32_t* epoch;        // device epoch of this call (advanced once per call)
  int* err;                     // kernel error word
  uint64_t timeout;             // peer wait bound, 100 MHz wall-clock ticks
};

void launch_ep_dispatch(const EpA2AArgs& a, hipStream_t st);   // dispatch + wait / mask
void launch_ep_return(const EpA2AArgs& a, hipStream_t st);
void launch_ep_combine(const EpA2AArgs& a, hipStream_t st);    // wait + weighted combine

}  // namespace illm
