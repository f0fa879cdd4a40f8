// Device-side synchronisation between the compute stream and the comm stream of the overlapped decode / prefill
// schedules (models/decoder.py _DevSync).
//
// Measured on MI355X (bench/xq_probe.py, profiles/r5_tbo): inside a HIP graph every edge from a kernel on one
// queue to a kernel on another queue (an event record + stream wait under capture) stalls the SOURCE queue for
// ~9 us after that kernel, whatever the HIP runtime settings. The two-micro-batch decode schedule has 8 such
// edges per layer, 4 of them on the compute queue. Here the streams hand off through flags in device memory
// instead: the producer stream runs flag_signal (flag[i] = current epoch, release), the consumer stream runs
// flag_wait (spin until flag[i] == epoch, acquire) before the dependent kernel. No queue barrier, no
// cross-queue edge, one 1-lane launch on each side.
//
// The epoch (one int, bumped by epoch_bump at the start of every forward) makes the flags reusable across graph
// replays without a reset. flag_wait gives up after ~1 s (err = 1, read by DecoderLM.sync_error()) so a
// schedule bug ends in a reported error instead of a hung GPU. Reference: the synchronous all-reduce of
// layers.py:175-179, which this overlap replaces.
#include "common.h"

namespace {
constexpr int kSpinLimit = 1 << 22;  // polls of ~0.2 us (s_sleep 8) before flag_wait reports a timeout

__global__ void epoch_bump_kernel(int* __restrict__ epoch) {
  if (threadIdx.x == 0) {
    const int v = __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(epoch, v + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void flag_signal_kernel(int* __restrict__ flags, int idx, const int* __restrict__ epoch) {
  if (threadIdx.x == 0) {
    const int e = __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(flags + idx, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void flag_wait_kernel(const int* __restrict__ flags, int idx, const int* __restrict__ epoch,
                                 int* __restrict__ err) {
  if (threadIdx.x == 0) {
    const int e = __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int n = 0;
    while (__hip_atomic_load(flags + idx, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != e) {
      __builtin_amdgcn_s_sleep(8);
      if (++n > kSpinLimit) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
}
}  // namespace

void launch_epoch_bump(void* epoch, hipStream_t st) {
  epoch_bump_kernel<<<1, 64, 0, st>>>((int*)epoch);
  HIP_CHECK_LAUNCH();
}

void launch_flag_signal(void* flags, int idx, const void* epoch, hipStream_t st) {
  flag_signal_kernel<<<1, 64, 0, st>>>((int*)flags, idx, (const int*)epoch);
  HIP_CHECK_LAUNCH();
}

void launch_flag_wait(const void* flags, int idx, const void* epoch, void* err, hipStream_t st) {
  flag_wait_kernel<<<1, 64, 0, st>>>((const int*)flags, idx, (const int*)epoch, (int*)err);
  HIP_CHECK_LAUNCH();
}
