// sf_pool.cpp -- the library's host worker threads (run_pool, sf_internal.hpp).
//
// The host pipelines split each stage's reads, copies, stats and row writes
// over up to io_threads() threads.  Starting those threads per stage cost
// ~0.6 ms per 16-thread pool (scripts/pool_probe.cpp): a 256 MiB stage reads
// in ~5 ms, and a many-file call of small files runs several pools per stage.
// The threads are started once, on first use, and kept: a job hands its
// worker to as many idle helpers as it asks for, runs the worker on the
// calling thread too, and at its end takes back the helpers that have not
// started it yet, so it never waits for a thread that is busy elsewhere.
// The workers share an atomic work counter, so a call that got fewer helpers
// (others busy, or the system refused a thread) only loses parallelism; a
// helper that starts after the work is taken finds none and returns.
// Helpers are never stopped: the pool lives until the process exits (it is
// never destroyed from a static destructor, like the device resources); a
// fork()ed child starts a fresh one.
#include <pthread.h>

#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "sf_internal.hpp"

namespace sfi {
namespace {

struct Job {
  const std::function<void()>* fn;
  unsigned want = 0;     // helpers asked for that have not started it
  unsigned running = 0;  // helpers running it now
  std::exception_ptr err;
};

constexpr unsigned kMaxHelpers = 256;

struct Pool {
  std::mutex mu;
  std::condition_variable work;  // a job wants helpers
  std::condition_variable done;  // a helper finished a job
  std::vector<Job*> jobs;        // jobs still wanting helpers, oldest first
  unsigned helpers = 0, busy = 0, wanted = 0;

  void helper() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      work.wait(lk, [&] { return !jobs.empty(); });
      Job* j = jobs.front();
      if (--j->want == 0) jobs.erase(jobs.begin());
      wanted--;
      j->running++;
      busy++;
      lk.unlock();
      std::exception_ptr e;
      try {
        (*j->fn)();
      } catch (...) {
        e = std::current_exception();
      }
      lk.lock();
      if (e && !j->err) j->err = e;
      busy--;
      if (--j->running == 0) done.notify_all();
    }
  }
};

// The pool: never freed, its helpers wait in it until exit.  A child made by
// fork() has none of the parent's helpers, and may have copied the mutex
// locked: it starts from a fresh pool (the old one is left as it is).
std::atomic<Pool*> g_pool{nullptr};
std::once_flag g_pool_once;

void fresh_pool_in_child() { g_pool.store(new Pool, std::memory_order_release); }

Pool* pool() {
  std::call_once(g_pool_once, [] {
    g_pool.store(new Pool, std::memory_order_release);
    pthread_atfork(nullptr, nullptr, fresh_pool_in_child);
  });
  return g_pool.load(std::memory_order_acquire);
}

}  // namespace

void run_pool_fn(unsigned nthreads, const std::function<void()>& fn) {
  Pool* P = pool();
  Job j;
  j.fn = &fn;
  {
    std::lock_guard<std::mutex> lk(P->mu);
    const unsigned ask = std::min(nthreads - 1, kMaxHelpers);
    // enough idle helpers for this job and the ones still waiting for theirs
    while (P->helpers - P->busy < P->wanted + ask && P->helpers < kMaxHelpers) {
      try {
        std::thread(&Pool::helper, P).detach();
      } catch (...) {
        break;  // the system refused a thread: fewer helpers
      }
      P->helpers++;
    }
    j.want = std::min(ask, P->helpers);
    if (j.want) {
      P->jobs.push_back(&j);
      P->wanted += j.want;
      P->work.notify_all();
    }
  }
  std::exception_ptr mine;
  try {
    fn();
  } catch (...) {
    mine = std::current_exception();
  }
  {
    std::unique_lock<std::mutex> lk(P->mu);
    if (j.want) {  // helpers that never started it: take them back
      for (size_t i = 0; i < P->jobs.size(); i++)
        if (P->jobs[i] == &j) {
          P->jobs.erase(P->jobs.begin() + (long)i);
          break;
        }
      P->wanted -= j.want;
      j.want = 0;
    }
    P->done.wait(lk, [&] { return j.running == 0; });
  }
  if (mine) std::rethrow_exception(mine);
  if (j.err) std::rethrow_exception(j.err);
}

}  // namespace sfi
