// CPU stress test of the library's host worker pool (syncfast_amd/csrc/
// sf_pool.cpp, run_pool in sf_internal.hpp), built and run by
// tests/test_capi.py::test_host_pool_stress: concurrent callers, nested
// calls from a helper, workers that throw, and callers that finish their
// work before any helper starts.  Every work item must run exactly once.
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../../syncfast_amd/csrc/sf_internal.hpp"

using sfi::run_pool;

static int fail(const char* what) {
  std::fprintf(stderr, "pool_stress: %s\n", what);
  return 1;
}

// n items over up to t threads; each item's slot is bumped once
static bool sweep(unsigned t, unsigned n, bool nested) {
  std::vector<std::atomic<int>> hits(n);
  for (auto& h : hits) h.store(0);
  std::atomic<unsigned> next{0};
  run_pool(t, [&] {
    for (unsigned i; (i = next.fetch_add(1)) < n;) {
      if (nested && i % 97 == 0) {  // a helper (or the caller) runs a pool of its own
        std::atomic<unsigned> in{0}, sum{0};
        run_pool(4, [&] {
          for (unsigned k; (k = in.fetch_add(1)) < 100;) sum.fetch_add(k);
        });
        if (sum.load() != 4950) hits[i].fetch_add(100);
      }
      hits[i].fetch_add(1);
    }
  });
  for (auto& h : hits)
    if (h.load() != 1) return false;
  return true;
}

int main() {
  for (unsigned t : {1u, 2u, 16u, 64u})
    for (unsigned n : {0u, 1u, 5u, 1000u})
      if (!sweep(t, n, false)) return fail("single caller");
  if (!sweep(16, 5000, true)) return fail("nested");
  // concurrent callers, some nesting
  {
    std::atomic<int> bad{0};
    std::vector<std::thread> callers;
    for (int c = 0; c < 8; c++)
      callers.emplace_back([&, c] {
        for (int r = 0; r < 200; r++)
          if (!sweep(1 + (unsigned)((c * 7 + r) % 17), 1 + (unsigned)((r * 13) % 300), r % 5 == 0)) bad++;
      });
    for (auto& th : callers) th.join();
    if (bad.load()) return fail("concurrent callers");
  }
  // an exception in a worker reaches the caller, after every helper is done
  for (int r = 0; r < 50; r++) {
    std::atomic<unsigned> next{0}, finished{0};
    bool caught = false;
    try {
      run_pool(8, [&] {
        for (unsigned i; (i = next.fetch_add(1)) < 64;) {
          if (i == 13) throw std::runtime_error("item 13");
          finished.fetch_add(1);
        }
      });
    } catch (const std::runtime_error&) {
      caught = true;
    }
    if (!caught) return fail("exception not rethrown");
  }
  // a fork()ed child (no helpers of its own; the parent's mutex may have been
  // copied locked) runs its pools on a fresh pool (not under ThreadSanitizer,
  // which does not support threads started after a multi-threaded fork)
#ifndef __SANITIZE_THREAD__
  {
    std::atomic<bool> stop{false};
    std::thread busy([&] {  // keeps the parent's pool mutex busy while we fork
      while (!stop.load()) sweep(16, 64, false);
    });
    for (int r = 0; r < 20; r++) {
      const pid_t pid = fork();
      if (pid == 0) _exit(sweep(16, 1000, true) ? 0 : 3);
      int st = 0;
      if (pid < 0 || waitpid(pid, &st, 0) != pid || !WIFEXITED(st) || WEXITSTATUS(st) != 0) {
        stop = true;
        busy.join();
        return fail("fork child");
      }
    }
    stop = true;
    busy.join();
  }
#endif
  std::printf("pool_stress ok\n");
  return 0;
}
