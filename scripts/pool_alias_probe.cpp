// pool_alias_probe.cpp -- round 6: can a stream-ordered allocation overlap a
// live hipMalloc allocation?  The library's scratch used to come from the
// device's default pool (release threshold 0: freed blocks go back at every
// synchronisation); with the explicit-list sort's workspace allocated there
// in every call, file calls read wrong data.  Here, per trial:
// a block from the pool (hipMallocAsync, or hipMallocFromPoolAsync on a pool
// of our own that keeps 1 GiB) is freed and the stream synchronised; a
// hipMalloc buffer of another size is taken and KEPT; the pool is asked for a
// block again; the two live ranges are compared, and a pattern written
// through each is read back through both.  One JSON line per pool.
//
//   hipcc --offload-arch=gfx950 -O2 scripts/pool_alias_probe.cpp -o scripts/pool_alias_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

static int run(const char* name, hipMemPool_t pool, int trials) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<void*> kept;
  std::vector<size_t> kept_len;
  int overlaps = 0, clobbered = 0;
  const size_t sizes[] = {4u << 20, 1u << 20, 12u << 20, 256u << 10, 33u << 20};
  for (int t = 0; t < trials; t++) {
    const size_t a = sizes[t % 5], b = sizes[(t + 2) % 5];
    void* p = nullptr;
    if (pool) CK(hipMallocFromPoolAsync(&p, a, pool, s));
    else CK(hipMallocAsync(&p, a, s));
    CK(hipMemsetAsync(p, 0x11, a, s));
    CK(hipFreeAsync(p, s));
    CK(hipStreamSynchronize(s));
    void* q = nullptr;
    CK(hipMalloc(&q, b));
    kept.push_back(q);
    kept_len.push_back(b);
    void* r = nullptr;
    if (pool) CK(hipMallocFromPoolAsync(&r, a, pool, s));
    else CK(hipMallocAsync(&r, a, s));
    const uintptr_t r0 = (uintptr_t)r, r1 = r0 + a;
    for (size_t i = 0; i < kept.size(); i++) {
      const uintptr_t k0 = (uintptr_t)kept[i];
      if (k0 < r1 && r0 < k0 + kept_len[i]) overlaps++;
    }
    // write through r, then through q, read r back: a shared page would show q's bytes
    CK(hipMemsetAsync(r, 0x22, a, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemset(q, 0x33, b));
    CK(hipDeviceSynchronize());
    uint8_t probe[4096];
    for (size_t off = 0; off < a; off += a / 8) {
      CK(hipMemcpy(probe, (uint8_t*)r + off, sizeof probe, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < sizeof probe; i++)
        if (probe[i] != 0x22) {
          clobbered++;
          break;
        }
    }
    CK(hipFreeAsync(r, s));
    CK(hipStreamSynchronize(s));
    if (kept.size() > 16) {
      CK(hipFree(kept.front()));
      kept.erase(kept.begin());
      kept_len.erase(kept_len.begin());
    }
  }
  for (void* k : kept) CK(hipFree(k));
  CK(hipStreamDestroy(s));
  printf("{\"pool\": \"%s\", \"trials\": %d, \"overlapping_live_ranges\": %d, \"pool_bytes_changed_by_hipMalloc_writes\": %d}\n",
         name, trials, overlaps, clobbered);
  fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 200;
  if (run("default (hipMallocAsync, release threshold 0)", nullptr, trials)) return 1;
  hipMemPoolProps props = {};
  props.allocType = hipMemAllocationTypePinned;
  props.handleTypes = hipMemHandleTypeNone;
  props.location.type = hipMemLocationTypeDevice;
  props.location.id = 0;
  for (int keep = 0; keep < 2; keep++) {
    hipMemPool_t pool = nullptr;
    CK(hipMemPoolCreate(&pool, &props));
    uint64_t thr = keep ? (1ull << 30) : 0;
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
    if (run(keep ? "own, keeps 1 GiB" : "own, release threshold 0", pool, trials)) return 1;
    CK(hipMemPoolDestroy(pool));
  }
  return 0;
}
