// A modelled collective for the simulated TP=N shard (bench.py --simulate-tp N --sim-comm LAT,GBPS,CHANNELS): the
// stand-in for an RCCL all-reduce that, like RCCL's kernels, occupies CHANNELS workgroups on as many CUs and streams
// memory - instead of one sleeping workgroup (torch.cuda._sleep), which leaves every other CU and the whole memory
// system to the compute that the schedules overlap with it ("a model that is too kind"). Each
// workgroup copies its share of the collective's local memory traffic through a scratch buffer, then holds its CU
// until the modelled time has passed on the device's constant wall clock; every workgroup reaches the same
// deadline, so the grid drains by construction.
#include "common.h"

__global__ __launch_bounds__(256) void comm_model_kernel(f32x4* __restrict__ buf, int64_t vec_per_wg, int reps,
                                                         int64_t ticks) {
  const int64_t t0 = (int64_t)wall_clock64();
  f32x4* src = buf + (int64_t)blockIdx.x * 2 * vec_per_wg;
  f32x4* dst = src + vec_per_wg;
  for (int r = 0; r < reps; ++r)  // the collective's memory traffic, spread over its channels
    for (int64_t i = threadIdx.x; i < vec_per_wg; i += blockDim.x) {
      f32x4 v = __builtin_nontemporal_load(src + i);
      v[0] += 1.f;
      __builtin_nontemporal_store(v, dst + i);
    }
  while ((int64_t)wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(4);  // then hold the CU until it "lands"
}

// Model of one collective moving `nbytes` of payload in `us`: `channels` workgroups read and write 2 x nbytes in all
// (a ring all-reduce's local traffic is ~4x its payload: the input read, the peer's writes, the reduce, the output),
// then keep their CUs until `us` has passed. buf: >= channels x 2 x slice bytes (comm_model_slice).
int64_t comm_model_slice(int channels, int64_t nbytes) {
  const int64_t per = (2 * nbytes / channels + 15) / 16 * 16;
  return std::max<int64_t>(16, std::min<int64_t>(per, 4 << 20));
}
void launch_comm_model(void* buf, int channels, int64_t nbytes, double us, hipStream_t st) {
  if (channels < 1 || channels > 1024) throw std::runtime_error("comm_model: 1-1024 channels");
  static int rate_khz = 0;  // wall-clock rate (kHz): a device attribute, read once
  if (!rate_khz) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || rate_khz <= 0)
      throw std::runtime_error("comm_model: cannot read the device wall-clock rate");
  }
  const int64_t slice = comm_model_slice(channels, nbytes);
  const int64_t want = 2 * nbytes / channels;
  const int reps = (int)std::max<int64_t>(1, (want + slice - 1) / slice);
  const int64_t ticks = std::max<int64_t>(1, (int64_t)(us * rate_khz / 1000.0));
  comm_model_kernel<<<channels, 256, 0, st>>>((f32x4*)buf, slice / 16, reps, ticks);
  HIP_CHECK_LAUNCH();
}
