// sf_knobs.cpp -- the library's environment knobs, read ONCE when the library
// is loaded (a static initializer) into g_knob[]; nothing on a launch or copy
// path calls getenv.  Two kinds ("Environment knobs"):
//   * performance A/B knobs (SF_*): change how a call runs, never its result;
//   * test hooks (SF_TEST_*): shrink stages, force a sort, a launch split, a
//     chain timeout or a page-lock failure -- they change the shape of a call
//     or its error behaviour, so they carry the SF_TEST_ prefix and are meant
//     for the test suite only.
// Tests change a knob inside one process with sf_test_set_knob
// (include/syncfast_amd_test.h), not with the environment.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sf_internal.hpp"
#include "../../include/syncfast_amd_test.h"

namespace sfi __attribute__((visibility("hidden"))) {

const KnobDef kKnobDefs[K_COUNT] = {
    {"SF_IO_THREADS", 0},               // K_IO_THREADS: pread threads (0 = 16)
    {"SF_INPLACE_MIN_MIB", -1},         // K_INPLACE_MIN_MIB: smallest in-place buffer (-1 = 1 MiB)
    {"SF_INPLACE_SERIAL", 0},           // K_INPLACE_SERIAL: lock whole range first, rows at the end
    {"SF_FADVISE", 1},                  // K_FADVISE: sequential / will-need hints on the pread route
    {"SF_NO_HOSTREG", 0},               // K_NO_HOSTREG: never page-lock caller memory
    {"SF_TABLE_CLASS_BITS", 4},         // K_TABLE_CLASS_BITS: mantissa bits of the length class (<= 4: 8-bit key)
    {"SF_TRACE", 0},                    // K_TRACE: sf_index_files / sf_index_fds_blocks phase times on stderr
    {"SF_BATCH_FUSED", 1},              // K_BATCH_FUSED: sf_index_device_batch's two halves (0: blocks, then chains)
    {"SF_TEST_INPLACE_FAIL_AT", -1},    // K_TEST_INPLACE_FAIL_AT: region k "fails" to page-lock
    {"SF_TEST_WIRE_CHUNK", 0},          // K_TEST_WIRE_CHUNK: messages per streamed chunk (0 = 2^18)
    {"SF_TEST_STREAM_STAGE_MIB", 0},    // K_TEST_STREAM_STAGE_MIB: pipeline stage size (0 = 256)
    {"SF_TEST_LAUNCH_MAX_BLOCKS", 0},   // K_TEST_LAUNCH_MAX_BLOCKS: blocks per launch (0 = 2^31)
    {"SF_TEST_TABLE_SORT", -1},         // K_TEST_TABLE_SORT: -1 auto (> 64 blocks), 0 never, 1 always
    {"SF_TEST_MULTI_SELF_GATHER", 0},   // K_TEST_MULTI_SELF_GATHER: one-device multi gather through RCCL (self send/recv)
    {"SF_TEST_CUT_WINDOW_MIB", 0},      // K_TEST_CUT_WINDOW_MIB: sf_index_fd_cut's window (0 = 512 MiB)
    {"SF_TEST_STREAM_POOL", 1},         // K_TEST_STREAM_POOL: scratch pool (1 own, keeps blocks; 0 / 3 known wrong)
};

std::atomic<int64_t> g_knob[K_COUNT];
std::atomic<int64_t> g_stat[S_COUNT];

namespace {
std::atomic<sf_test_read_hook_fn> g_read_hook{nullptr};
std::atomic<void*> g_read_hook_arg{nullptr};
}  // namespace

void read_hook(uint64_t window) {
  const sf_test_read_hook_fn fn = g_read_hook.load(std::memory_order_acquire);
  if (fn) fn(g_read_hook_arg.load(std::memory_order_relaxed), window);
}
static const char* const kStatNames[S_COUNT] = {"pages_locked", "not_anon_refused"};

namespace {
struct LoadKnobs {
  LoadKnobs() {
    for (int k = 0; k < K_COUNT; k++) {
      const char* e = getenv(kKnobDefs[k].env);
      g_knob[k].store(e && *e ? strtoll(e, nullptr, 10) : kKnobDefs[k].dflt, std::memory_order_relaxed);
    }
  }
} load_knobs;  // runs when the library is loaded
}  // namespace

}  // namespace sfi

using namespace sfi;

extern "C" {

int sf_test_set_knob(const char* name, int64_t value, int64_t* old_value) {
  if (!name) return SF_EINVAL;
  for (int k = 0; k < K_COUNT; k++)
    if (strcmp(name, kKnobDefs[k].env) == 0) {
      const int64_t o = g_knob[k].exchange(value, std::memory_order_relaxed);
      if (old_value) *old_value = o;
      return SF_OK;
    }
  return SF_EINVAL;
}

int sf_test_get_stat(const char* name, int64_t* value) {
  if (!name || !value) return SF_EINVAL;
  for (int k = 0; k < S_COUNT; k++)
    if (strcmp(name, kStatNames[k]) == 0) {
      *value = g_stat[k].load(std::memory_order_relaxed);
      return SF_OK;
    }
  return SF_EINVAL;
}

int sf_test_set_read_hook(sf_test_read_hook_fn fn, void* arg) {
  g_read_hook_arg.store(arg, std::memory_order_relaxed);
  g_read_hook.store(fn, std::memory_order_release);
  return SF_OK;
}

int sf_test_get_knob(const char* name, int64_t* value) {
  if (!name || !value) return SF_EINVAL;
  for (int k = 0; k < K_COUNT; k++)
    if (strcmp(name, kKnobDefs[k].env) == 0) {
      *value = g_knob[k].load(std::memory_order_relaxed);
      return SF_OK;
    }
  return SF_EINVAL;
}

}  // extern "C"
