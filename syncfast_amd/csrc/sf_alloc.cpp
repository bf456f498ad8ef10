// sf_alloc.cpp -- the library's stream-ordered scratch (sort workspaces,
// chain states, wire offsets, block-set slots): stream_alloc / stream_free.
//
// Every such buffer is allocated, used and freed on ONE stream.  Until round
// 6 they came from hipMallocAsync, i.e. the device's default pool, whose
// release threshold is 0: at every synchronisation the pool gives its freed
// blocks back, and the next call's allocation maps memory again.  With the
// explicit-list sort's workspace allocated that way in every call (round 6
// sorts every list of two waves or more), calls read wrong data through it:
// a loop of sf_index_fds_blocks + sf_index_fd_cut calls in one process
// (scripts/sort_race_stress.py, profiles/r06/scratch_pool/) went wrong in
// 58-60 of 60 iterations in 7 of 8 processes, from the default pool and from
// a pool of our own with the threshold left at 0 alike, and in 0 of 480 from
// a pool of our own that keeps its freed blocks (a 1 GiB threshold in that
// measurement), whether or not the runtime may reuse a block across streams;
// with no scratch at all (the sort off) 0 of 240.  So the library takes its
// scratch from a pool of its own per device that keeps every freed block
// mapped (no threshold: nothing is given back and mapped again), and reuses
// a block only on the stream that freed it.  SF_TEST_STREAM_POOL (test
// hook): 1 that pool (default); 0 hipMallocAsync on the default pool; 2 the
// pool with cross-stream reuse on; 3 the pool releasing at every
// synchronisation.
#include <stdint.h>

#include <mutex>

#include "sf_internal.hpp"

namespace sfi {

namespace {

std::mutex g_pool_mu;
// [mode - 1][device]: mode 1 is the shipped pool; 2 and 3 exist for the A/B
// that found which of its settings matters
hipMemPool_t g_pool[3][kMaxDevices] = {};

int stream_device(hipStream_t s, int* dev) {
  if (s) {
    hipDevice_t d = 0;
    if (hipStreamGetDevice(s, &d) == hipSuccess) {
      *dev = (int)d;
      return SF_OK;
    }
    (void)hipGetLastError();
  }
  SF_HIP(hipGetDevice(dev));
  return SF_OK;
}

// The library's pool of device `dev` (created on first use, kept: freeing it
// from a static destructor could run after the HIP runtime is gone).
//   mode 1 (shipped): blocks reused on the freeing stream only, every freed
//     block kept mapped (the pool holds its peak: the largest scratch is a
//     sort workspace of at most ~0.6-1 GiB for a 2^27-block launch piece, by
//     the class-key width);
//   mode 2: the same pool with the runtime's cross-stream reuse left on;
//   mode 3: reuse on the freeing stream only, freed blocks released at every
//     synchronisation (the runtime's default threshold, 0).
int pool_of(int mode, int dev, hipMemPool_t* out) {
  if (dev < 0 || dev >= kMaxDevices || mode < 1 || mode > 3) return SF_EINVAL;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  hipMemPool_t& slot = g_pool[mode - 1][dev];
  if (!slot) {
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t p = nullptr;
    SF_HIP(hipMemPoolCreate(&p, &props));
    hipError_t e = hipSuccess;
    if (mode != 2) {
      int off = 0;
      e = hipMemPoolSetAttribute(p, hipMemPoolReuseAllowOpportunistic, &off);
      if (e == hipSuccess) e = hipMemPoolSetAttribute(p, hipMemPoolReuseAllowInternalDependencies, &off);
      if (e == hipSuccess) e = hipMemPoolSetAttribute(p, hipMemPoolReuseFollowEventDependencies, &off);
    }
    // keep every freed block (mode 1, 2): the measurement ties the wrong data
    // to pools that give freed blocks back at synchronisation points, and a
    // finite threshold would still give back what lies above it
    uint64_t keep = mode == 3 ? 0 : UINT64_MAX;
    if (e == hipSuccess) e = hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep);
    if (e != hipSuccess) {
      (void)hipMemPoolDestroy(p);
      return hip_err(e);
    }
    slot = p;
  }
  *out = slot;
  return SF_OK;
}

}  // namespace

int stream_alloc(void** p, size_t bytes, hipStream_t s) {
  *p = nullptr;
  const int64_t mode = knob(K_TEST_STREAM_POOL);
  if (mode == 0) return hip_err(hipMallocAsync(p, bytes, s));
  int dev = 0, rc = stream_device(s, &dev);
  hipMemPool_t pool = nullptr;
  if (rc == SF_OK) rc = pool_of((int)mode, dev, &pool);
  if (rc != SF_OK) return rc;
  return hip_err(hipMallocFromPoolAsync(p, bytes, pool, s));
}

void stream_free(void* p, hipStream_t s) {
  if (p) (void)hipFreeAsync(p, s);
}

}  // namespace sfi
