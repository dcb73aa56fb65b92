// comm.cpp — migration plans and the loopback transport of the C API island
// model (see pga/comm.hpp).
//
// Reference: pga_migrate / pga_migrate_between / pga_run_islands are empty
// (src/pga.cu:368-374, :393-395); the header only says "randomly migrate top
// %pct between populations" (include/pga.h:108-115, :145-150).
#include <algorithm>
#include <cstring>
#include <numeric>

#include "pga/comm.hpp"
#include "pga/core.hpp"

namespace pga {

uint32_t plan_migrants(int topology, int nranks, uint32_t k) {
  if (nranks < 1 || k == 0) return 0;
  if (nranks == 1) return k;  // self-exchange (fault-injection test mode)
  if (topology == TOPO_ALL_TO_ALL) {
    const uint32_t peers = (uint32_t)nranks - 1;
    return std::max<uint32_t>(1, k / peers) * peers;
  }
  return k;
}

std::vector<Xfer> migration_plan(int topology, int nranks, uint32_t k, uint64_t seed, uint32_t epoch) {
  std::vector<Xfer> plan;
  if (nranks < 1 || k == 0) return plan;
  if (nranks == 1) return {{0, 0, 0, 0, k}};  // a 1-rank ring: to itself
  const int n = nranks;
  if (topology == TOPO_ALL_TO_ALL) {
    // rank r's j-th peer (peers in rank order, r skipped) gets slice j of r's
    // emigrants and stores it at slot (index of r among that peer's peers)
    const uint32_t per = plan_migrants(topology, n, k) / (uint32_t)(n - 1);
    for (int r = 0; r < n; ++r) {
      uint32_t j = 0;
      for (int p = 0; p < n; ++p) {
        if (p == r) continue;
        const uint32_t slot = (uint32_t)(r < p ? r : r - 1);
        plan.push_back({r, p, j * per, slot * per, per});
        ++j;
      }
    }
    return plan;
  }
  std::vector<int> ring(n);
  std::iota(ring.begin(), ring.end(), 0);
  if (topology == TOPO_RANDOM) {
    // Fisher-Yates from the shared seed: every rank draws the same ring
    const RngKey key{(uint32_t)seed, (uint32_t)(seed >> 32), epoch, 0xFFFFu};
    for (int i = n - 1; i >= 1; --i) {
      const uint32_t j = word_to_index(draw(key, ST_MIGRATE, 1, (uint32_t)i).x, (uint32_t)i + 1);
      std::swap(ring[i], ring[j]);
    }
  }
  for (int i = 0; i < n; ++i) plan.push_back({ring[i], ring[(i + 1) % n], 0, 0, k});
  return plan;
}

namespace {

class LoopbackComm final : public Comm {
 public:
  explicit LoopbackComm(int n) : n_(n) {}
  int size() const override { return n_; }
  const char* name() const override { return "loopback"; }
  bool drives_all_ranks() const override { return true; }

  void exchange(const std::vector<Xfer>& plan, std::vector<LocalRank>& local) override {
    ++count_;
    failed_ = false;
    const bool fault = every_ > 0 && count_ % (uint64_t)every_ == 0;
    if (fault && mode_ == 1) {
      failed_ = true;  // dropped: nothing arrives
      return;
    }
    auto find = [&](int r) -> LocalRank& {
      for (LocalRank& l : local)
        if (l.rank == r) return l;
      throw std::runtime_error("loopback exchange: rank not driven by this call");
    };
    for (LocalRank& l : local)
      if (l.device >= 0) PGA_COMM_HIP(hipStreamSynchronize(l.stream));
    for (const Xfer& x : plan) {
      LocalRank &s = find(x.src), &d = find(x.dst);
      const size_t rb = s.row_bytes;
      const char* sr = (const char*)s.send_rows + rb * x.src_off;
      char* dr = (char*)d.recv_rows + rb * x.dst_off;
      const float* ss = s.send_scores + x.src_off;
      float* ds = d.recv_scores + x.dst_off;
      if (s.device < 0 && d.device < 0) {
        std::memcpy(dr, sr, rb * x.n);
        std::memcpy(ds, ss, 4ull * x.n);
      } else {
        // unified addressing: host<->device and peer copies alike
        PGA_COMM_HIP(hipMemcpy(dr, sr, rb * x.n, hipMemcpyDefault));
        PGA_COMM_HIP(hipMemcpy(ds, ss, 4ull * x.n, hipMemcpyDefault));
      }
      bytes_sent += (rb + 4) * x.n;
      if (fault && mode_ == 2) {
        std::vector<float> bad(x.n, 3e38f);
        if (d.device < 0) std::memcpy(ds, bad.data(), 4ull * x.n);
        else PGA_COMM_HIP(hipMemcpy(ds, bad.data(), 4ull * x.n, hipMemcpyHostToDevice));
      }
    }
  }

  bool wait(std::vector<LocalRank>&, double) override { return !failed_; }

  bool allgather(const std::vector<LocalRank>& local, const std::vector<uint32_t>& mine, uint32_t count,
                 std::vector<uint32_t>& all, double) override {
    if (count == 0 || count > kGatherMaxWords) throw std::invalid_argument("allgather: bad word count");
    all.assign((size_t)n_ * count, 0u);
    for (size_t i = 0; i < local.size(); ++i)
      std::memcpy(&all[(size_t)local[i].rank * count], &mine[i * count], 4ull * count);
    return true;
  }

  bool broadcast(const std::vector<LocalRank>& local, const std::vector<void*>& bufs, size_t bytes, int root,
                 double) override {
    size_t r = local.size();
    for (size_t i = 0; i < local.size(); ++i)
      if (local[i].rank == root) r = i;
    if (r == local.size()) throw std::runtime_error("loopback broadcast: root not driven by this call");
    for (const LocalRank& l : local)
      if (l.device >= 0) PGA_COMM_HIP(hipStreamSynchronize(l.stream));
    for (size_t i = 0; i < local.size(); ++i) {
      if (i == r) continue;
      if (local[i].device < 0 && local[r].device < 0) std::memcpy(bufs[i], bufs[r], bytes);
      else PGA_COMM_HIP(hipMemcpy(bufs[i], bufs[r], bytes, hipMemcpyDefault));
    }
    return true;
  }

  void set_fault(int every, int mode) override {
    if (mode < 0 || mode > 2) throw std::invalid_argument("loopback fault mode must be 0 (none), 1 (drop) or 2 (corrupt)");
    every_ = every;
    mode_ = mode;
  }

 private:
  int n_;
  uint64_t count_ = 0;
  int every_ = 0, mode_ = 0;
  bool failed_ = false;
};

}  // namespace

std::shared_ptr<Comm> loopback_comm(int nranks) {
  if (nranks < 1) throw std::invalid_argument("loopback: nranks < 1");
  return std::make_shared<LoopbackComm>(nranks);
}


}  // namespace pga
