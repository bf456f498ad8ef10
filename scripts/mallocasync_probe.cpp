// mallocasync_probe.cpp -- does the stream-ordered allocator hand a block
// freed on stream A (behind work still running there) to an allocation on
// stream B without making B wait for A?  That is the pattern of round 5's
// sf_index_files stages on two streams when each fused many-file launch took
// its stage counters from hipMallocAsync and gave them back with
// hipFreeAsync on its own stream (sf_capi.hip batch_staged): if B got A's
// counters and zeroed them while A's kernel still ran, A's blocks_hash lanes
// would wait for a count that never comes.
//
//   hipcc --offload-arch=gfx950 -O2 -I include scripts/mallocasync_probe.cpp \
//     -L syncfast_amd/lib -lsyncfast_amd -Wl,-rpath,$PWD/syncfast_amd/lib -o scripts/mallocasync_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <unistd.h>

#include "syncfast_amd.h"

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const uint64_t len = 4ull << 30;
  void *big = nullptr, *dig = nullptr;
  CK(hipMalloc(&big, len));
  CK(hipMalloc(&dig, (len / 4096) * 20));
  if (sf_fill_splitmix_device(big, len, 1, 0, nullptr) != 0) return 1;
  CK(hipDeviceSynchronize());
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t eb;
  CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
  int mempool_reuse[3] = {-1, -1, -1};
  hipMemPool_t pool;
  int dev = 0;
  CK(hipDeviceGetDefaultMemPool(&pool, dev));
  const hipMemPoolAttr attrs[3] = {hipMemPoolReuseFollowEventDependencies, hipMemPoolReuseAllowOpportunistic,
                                   hipMemPoolReuseAllowInternalDependencies};
  for (int i = 0; i < 3; i++) (void)hipMemPoolGetAttribute(pool, attrs[i], &mempool_reuse[i]);
  printf("{\"pool_attrs\": {\"follow_event_dependencies\": %d, \"allow_opportunistic\": %d, "
         "\"allow_internal_dependencies\": %d}}\n",
         mempool_reuse[0], mempool_reuse[1], mempool_reuse[2]);
  int same = 0, hazard = 0, trials = 20;
  for (int t = 0; t < trials; t++) {
    uint64_t nb = 0;
    for (int k = 0; k < 6; k++)  // ~7 ms of kernels queued on a
      if (sf_index_device_fixed(big, len, 4096, dig, len / 4096, &nb, a) != 0) return 1;
    void *p1 = nullptr, *p2 = nullptr;
    CK(hipMallocAsync(&p1, 128, a));
    CK(hipMemsetAsync(p1, 0, 128, a));
    CK(hipFreeAsync(p1, a));
    CK(hipMallocAsync(&p2, 128, b));
    CK(hipMemsetAsync(p2, 0xFF, 128, b));
    CK(hipEventRecord(eb, b));
    usleep(500);  // b's memset runs at once unless b was made to wait for a
    const bool a_busy = hipStreamQuery(a) == hipErrorNotReady;
    const bool b_done = hipEventQuery(eb) == hipSuccess;
    (void)hipGetLastError();
    same += p1 == p2;
    hazard += (p1 == p2) && a_busy && b_done;
    printf("{\"trial\": %d, \"same_block\": %d, \"a_still_running\": %d, \"b_memset_done\": %d}\n", t, p1 == p2,
           a_busy, b_done);
    CK(hipFreeAsync(p2, b));
    CK(hipStreamSynchronize(a));
    CK(hipStreamSynchronize(b));
  }
  printf("{\"summary\": {\"trials\": %d, \"same_block\": %d, \"reused_while_a_ran\": %d}}\n", trials, same, hazard);
  return 0;
}
