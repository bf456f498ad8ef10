// Per-call cost of a 16-thread host pool with an empty worker: threads
// started and joined per call (the host pipelines' form until round 5) vs
// the library's kept helpers (run_pool, syncfast_amd/csrc/sf_pool.cpp).
// g++ -O2 -std=c++17 -pthread -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
//   scripts/pool_probe.cpp syncfast_amd/csrc/sf_pool.cpp -o /tmp/pool_probe
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#include "../syncfast_amd/csrc/sf_internal.hpp"

int main() {
  constexpr int kCalls = 200;
  std::atomic<unsigned> items{0};
  auto work = [&] {
    for (int i = 0; i < 64; i++) items.fetch_add(1, std::memory_order_relaxed);
  };
  for (int rep = 0; rep < 3; rep++) {
    auto t0 = std::chrono::steady_clock::now();
    for (int c = 0; c < kCalls; c++) {
      std::vector<std::thread> th;
      for (int t = 1; t < 16; t++) th.emplace_back(work);
      work();
      for (auto& t : th) t.join();
    }
    auto t1 = std::chrono::steady_clock::now();
    for (int c = 0; c < kCalls; c++) sfi::run_pool(16, work);
    auto t2 = std::chrono::steady_clock::now();
    std::printf("16 threads per call: started per call %.1f us, kept %.1f us\n",
                std::chrono::duration<double, std::micro>(t1 - t0).count() / kCalls,
                std::chrono::duration<double, std::micro>(t2 - t1).count() / kCalls);
  }
  return 0;
}
