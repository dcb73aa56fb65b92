// parallel.cpp — the CPU backend's worker pool.  Children of a generation are
// independent (counter-based RNG: every draw is a function of the child, not
// of an execution order), so a generation splits into contiguous child
// ranges over persistent worker threads and stays bit-identical to the serial
// loop; the packed best is a max, so its combination order is irrelevant.
//
// PGA_CPU_THREADS=N sets the thread count; default min(8, CPUs in the affinity
// mask).  OneMax-64 pop 1024 on the MI355X host: 11.5k gens/s on 1 thread,
// 19.9k on 4, 24.3k on 8, 13.2k on 16 (wake-up cost outgrows the work).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

#include <sched.h>
#include <unistd.h>

#include <exception>

#include "pga/cpu.hpp"

namespace pga {
namespace cpu {
namespace {

class WorkerPool {
 public:
  explicit WorkerPool(unsigned n) {
    for (unsigned i = 1; i < n; ++i) threads_.emplace_back([this, i] { loop(i); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  unsigned size() const { return (unsigned)threads_.size() + 1; }

  // run job(slot) for slot in [0, n): slot 0 on the caller, the rest on
  // workers.  Every slot runs to its end before run() returns, a throwing one
  // included; the first exception (caller's or a worker's) is rethrown here.
  void run(unsigned n, const std::function<void(unsigned)>& job) {
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &job;
      active_ = n;
      pending_ = n - 1;
      error_ = nullptr;
      ++epoch_;
    }
    cv_.notify_all();
    std::exception_ptr mine;
    try {
      job(0);
    } catch (...) {
      mine = std::current_exception();
    }
    std::unique_lock<std::mutex> l(m_);
    done_.wait(l, [&] { return pending_ == 0; });
    job_ = nullptr;
    std::exception_ptr e = mine ? mine : error_;
    error_ = nullptr;
    l.unlock();
    if (e) std::rethrow_exception(e);
  }

  std::mutex busy;  // one generation at a time; concurrent callers run serially

 private:
  void loop(unsigned id) {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> l(m_);
      cv_.wait(l, [&] { return stop_ || epoch_ != seen; });
      if (stop_) return;
      seen = epoch_;
      if (id >= active_) continue;
      const std::function<void(unsigned)>* job = job_;
      l.unlock();
      std::exception_ptr e;
      try {
        (*job)(id);
      } catch (...) {
        e = std::current_exception();
      }
      l.lock();
      if (e && !error_) error_ = e;
      if (--pending_ == 0) done_.notify_one();
    }
  }

  std::vector<std::thread> threads_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(unsigned)>* job_ = nullptr;
  unsigned active_ = 0, pending_ = 0;
  std::exception_ptr error_;  // first worker exception of the current run
  uint64_t epoch_ = 0;
  bool stop_ = false;
};

unsigned configured_threads() {
  if (const char* e = std::getenv("PGA_CPU_THREADS")) {
    const long v = std::strtol(e, nullptr, 10);
    if (v >= 1) return (unsigned)std::min<long>(v, 256);
  }
  cpu_set_t set;
  unsigned n = 0;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = (unsigned)CPU_COUNT(&set);
  if (n == 0) n = std::thread::hardware_concurrency();
  return std::max(1u, std::min(n, 8u));
}

// one pool per process: a child forked from a process that had started the
// workers has none of its threads, so it builds its own (the parent's object
// is left alone, never joined)
WorkerPool& pool() {
  static std::mutex m;
  static WorkerPool* p = nullptr;
  static pid_t owner = 0;
  std::lock_guard<std::mutex> g(m);
  if (!p || owner != getpid()) {
    p = new WorkerPool(configured_threads());
    owner = getpid();
  }
  return *p;
}

}  // namespace

unsigned cpu_threads() { return pool().size(); }

void parallel_for(uint64_t n, uint64_t grain, const std::function<void(uint64_t, uint64_t, unsigned)>& fn) {
  WorkerPool& p = pool();
  const uint64_t want = grain ? (n + grain - 1) / grain : 1;
  const unsigned slots = (unsigned)std::min<uint64_t>(p.size(), std::max<uint64_t>(want, 1));
  if (slots <= 1 || !p.busy.try_lock()) {
    fn(0, n, 0);
    return;
  }
  std::lock_guard<std::mutex> g(p.busy, std::adopt_lock);
  const uint64_t per = (n + slots - 1) / slots;
  p.run(slots, [&](unsigned s) {
    const uint64_t b = std::min<uint64_t>(n, (uint64_t)s * per), e = std::min<uint64_t>(n, b + per);
    if (b < e) fn(b, e, s);
  });
}

}  // namespace cpu
}  // namespace pga
