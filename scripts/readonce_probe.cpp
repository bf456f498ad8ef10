// Default mode, host side only: what the chunker costs when it cuts bytes it
// has just read into their final (pinned) stage location, against the 64 KiB
// reused buffer it uses today.  16 threads over 1024 files of 8 MiB (page
// cache), the stand-in chunker (examples/zpaq_standin.h):
//   reused  pread 64 KiB into a per-thread buffer, cut it (today; the library
//           then reads every file again into its pinned stages)
//   pinned  pread 64 KiB straight into a hipHostMalloc'd batch buffer at the
//           file's place, cut it while it is in cache (no second read needed)
//   heap    the same into a malloc'd buffer
// hipcc -O2 -std=c++17 scripts/readonce_probe.cpp -o /tmp/readonce_probe -lpthread
#include <hip/hip_runtime_api.h>
#include <fcntl.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../examples/zpaq_standin.h"

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp/sf_ro";
  const int nfiles = 1024, threads = 16;
  const size_t fsz = 8u << 20, piece = 64u << 10;
  std::vector<std::string> paths;
  for (int k = 0; k < nfiles; k++) paths.push_back(std::string(dir) + "/f" + std::to_string(k));
  uint8_t* pinned = nullptr;
  if (hipHostMalloc((void**)&pinned, (size_t)nfiles * fsz, hipHostMallocDefault) != hipSuccess) return 1;
  uint8_t* heap = (uint8_t*)malloc((size_t)nfiles * fsz);
  for (size_t i = 0; i < (size_t)nfiles * fsz; i += 4096) heap[i] = 0;  // fault in
  for (int rep = 0; rep < 3; rep++)
    for (int mode = 0; mode < 3; mode++) {
      std::atomic<int> next{0};
      std::atomic<uint64_t> cuts{0};
      const double t0 = now();
      std::vector<std::thread> th;
      for (int t = 0; t < threads; t++)
        th.emplace_back([&] {
          std::vector<uint8_t> small(piece);
          for (int k; (k = next.fetch_add(1)) < nfiles;) {
            const int fd = open(paths[k].c_str(), O_RDONLY);
            sf_zpaq z;
            sf_zpaq_init(&z, 13, 32768);
            uint64_t c = 0;
            for (size_t off = 0; off < fsz; off += piece) {
              uint8_t* dst = mode == 0 ? small.data() : (mode == 1 ? pinned : heap) + (size_t)k * fsz + off;
              const ssize_t r = pread(fd, dst, piece, (off_t)off);
              if (r <= 0) break;
              for (size_t q = 0; q < (size_t)r;) {
                const size_t m = sf_zpaq_next(&z, dst + q, (size_t)r - q);
                if (!m) break;
                q += m;
                c++;
              }
            }
            close(fd);
            cuts += c;
          }
        });
      for (auto& t : th) t.join();
      const double dt = now() - t0;
      std::printf("rep %d %-6s %.3f s  %.2f GB/s  cuts %llu\n", rep, mode == 0 ? "reused" : mode == 1 ? "pinned" : "heap",
                  dt, (double)nfiles * fsz / dt / 1e9, (unsigned long long)cuts.load());
      std::fflush(stdout);
    }
  return 0;
}
