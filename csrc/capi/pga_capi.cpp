// pga_capi.cpp — the C API (include/pga.h, include/pga_ext.h) on top of the
// native Island runtime.
//
// Reference: include/pga.h:17-156 and src/pga.cu:148-395.  Parity notes:
//   * pga_create_population: NULL at MAX_POPULATIONS or genome_len < 4
//     (src/pga.cu:180-186); genes U(0, 1].
//   * pga_run evolves population 0 only (src/pga.cu:376-391); one fused
//     generation kernel per generation instead of fill_rand + 3 stage
//     kernels x ceil(S/512) launches + 3 device syncs.
//   * pga_get_best prints the best score with "%f\n" (src/pga.cu:230) unless
//     pga_set_quiet(p, 1), and returns a malloc'd copy the caller frees.
//   * NULL mutate / crossover restore the built-in defaults (the header says
//     so, include/pga.h:74-85; the original stored NULL).
//   * The stubs of the original (pga_get_best_top*, pga_get_best_all,
//     pga_migrate*, pga_run_islands, src/pga.cu:238-248, :368-374, :393-395)
//     are implemented.
//   * Errors: print + exit(1) by default, like the original's gpuAssert
//     (src/pga.cu:25-33); pga_set_abort_on_error(p, 0) records them for
//     pga_last_error() instead.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <memory>
#include <string>
#include <vector>

#include "pga.h"
#include "pga/comm.hpp"
#include "pga/island.hpp"
#include "pga/ops.hpp"
#include "pga_ext.h"

struct pga_population {
  std::unique_ptr<pga::Island> isl;
  pga_t* owner = nullptr;
  hipStream_t stream = nullptr;  // own stream: islands of pga_run_islands evolve concurrently
  hipEvent_t done = nullptr;
  // persistent emigrant staging of intra-solver migration (grown, never freed
  // per call: hipFree would synchronise the whole device)
  void* emi_rows = nullptr;
  float* emi_scores = nullptr;
  uint32_t emi_cap = 0;
  ~pga_population() {
    if (emi_rows && isl) {
      if (isl->on_gpu()) {
        (void)hipFree(emi_rows);
        (void)hipFree(emi_scores);
      } else {
        std::free(emi_rows);
        std::free(emi_scores);
      }
    }
    if (done) (void)hipEventDestroy(done);
    if (stream) (void)hipStreamDestroy(stream);
  }
  int builtin = -1;  // built-in objective id, -1: the pga-level obj_f callback, -2: hipRTC source
};

struct pga_solver {
  int device = 0;
  uint64_t seed = 0;
  bool quiet = false;
  bool abort_on_error = true;
  std::vector<population_t*> pops;
  obj_f objective = nullptr;
  mutate_f mutate = nullptr;
  crossover_f crossover = nullptr;
  hipStream_t stream = nullptr;
  uint32_t migration_epoch = 0;
  // inter-rank island model (pga_comm_*): the communicator may be shared by
  // several solvers of this process (InitAll / loopback groups)
  std::shared_ptr<pga::Comm> comm;
  std::shared_ptr<std::vector<pga_t*>> comm_members;  // solvers driven together (drives_all_ranks)
  int comm_rank = 0;
  int topology = pga::TOPO_RING;
  double comm_timeout = 0.0;
  bool validate_migrants = true;
  bool degraded = false;
  uint32_t comm_failures = 0;
  uint32_t comm_epoch = 0;
  uint64_t migrants_received = 0;
  // migration staging (device of population 0)
  void* mig_send_rows = nullptr;
  void* mig_recv_rows = nullptr;
  float* mig_send_scores = nullptr;
  float* mig_recv_scores = nullptr;
  uint32_t mig_cap = 0;
  // an exchange posted and not yet received (run_islands overlaps it with
  // the next generation), of mig_k migrants
  bool mig_pending = false;
  uint32_t mig_k = 0;
  // one row of device staging for the cross-rank best genome (broadcast)
  void* best_row = nullptr;
  // pga_run_islands: same-shape islands as one batched launch per generation
  bool batch_islands = true;
  uint64_t batched_gens = 0;
};

namespace {

thread_local std::string g_last_error;

void fail(pga_t* p, const char* what) {
  g_last_error = what;
  if (!p || p->abort_on_error) {
    std::fprintf(stderr, "pga error: %s\n", what);
    std::exit(1);
  }
}

template <typename F>
void guard(pga_t* p, F&& f) {
  try {
    f();
  } catch (const std::exception& e) {
    fail(p, e.what());
  }
}
template <typename R, typename F>
R guard_r(pga_t* p, R bad, F&& f) {
  try {
    return f();
  } catch (const std::exception& e) {
    fail(p, e.what());
    return bad;
  }
}

bool valid_pop(pga_t* p, population_t* pop) {
  return p && pop && pop->owner == p && std::find(p->pops.begin(), p->pops.end(), pop) != p->pops.end();
}

// push the current callbacks / built-in objective into a population
void sync_callbacks(pga_t* p, population_t* pop) {
  pga::Island& isl = *pop->isl;
  pga::Config c = isl.config();
  if (pop->builtin == -1) {
    c.objective = p->objective ? pga::OBJ_USER_FNPTR : pga::OBJ_NONE;
    isl.set_user_fn((void*)p->objective);
    if (c.encoding == pga::ENC_REAL) isl.set_user_operators((void*)p->crossover, (void*)p->mutate);
  }
  isl.set_operators(c);
  isl.stream = p->stream;
}

float fraction(float pct) { return pct > 1.f ? pct / 100.f : pct; }

uint32_t migrants(uint64_t from_S, uint64_t to_S, float pct) {
  const double f = fraction(pct);
  if (f <= 0) return 0;
  uint64_t k = (uint64_t)std::llround(f * (double)from_S);
  k = std::max<uint64_t>(k, 1);
  k = std::min<uint64_t>(k, std::min(from_S, to_S) / 2 ? std::min(from_S, to_S) / 2 : 1);
  return (uint32_t)k;
}

// row -> float genes (BINARY: one float per bit, PERMUTATION: city ids)
gene* decode_row(const pga::Island& isl, const std::vector<uint32_t>& row) {
  const uint32_t L = isl.config().L;
  gene* g = (gene*)std::malloc(sizeof(gene) * L);
  if (!g) throw std::bad_alloc();
  switch (isl.config().encoding) {
    case pga::ENC_REAL: std::memcpy(g, row.data(), sizeof(float) * L); break;
    case pga::ENC_BINARY:
      for (uint32_t i = 0; i < L; ++i) g[i] = (float)((row[i / 32] >> (i % 32)) & 1u);
      break;
    default: {
      const uint16_t* h = (const uint16_t*)row.data();
      for (uint32_t i = 0; i < L; ++i) g[i] = (float)h[i];
    }
  }
  return g;
}

void* dev_alloc(pga::Island& isl, size_t bytes) {
  void* ptr = nullptr;
  if (isl.on_gpu()) PGA_HIP_CHECK(hipMalloc(&ptr, bytes));
  else ptr = std::malloc(bytes);
  if (!ptr) throw std::bad_alloc();
  return ptr;
}
void dev_free(pga::Island& isl, void* ptr) {
  if (!ptr) return;
  if (isl.on_gpu()) (void)hipFree(ptr);
  else std::free(ptr);
}

// Intra-solver migration, fully stream-ordered on the solver stream: the
// top-k emigrants of a population go to its own persistent staging, the
// destination's bottom-k are replaced from there.  No allocation, free or host
// synchronisation per call, so concurrent island streams are not serialised.
void ensure_emigrant_staging(population_t* pop, uint32_t k) {
  if (pop->emi_cap >= k) return;
  pga::Island& isl = *pop->isl;
  if (pop->emi_rows) {
    isl.synchronize();  // a previous epoch may still read the old staging
    dev_free(isl, pop->emi_rows);
    dev_free(isl, pop->emi_scores);
  }
  pop->emi_rows = pop->emi_scores = nullptr;
  pop->emi_cap = 0;
  pop->emi_rows = dev_alloc(isl, isl.row_bytes() * k);
  pop->emi_scores = (float*)dev_alloc(isl, 4ull * k);
  pop->emi_cap = k;
}

void take_best(population_t* pop, uint32_t k) {
  ensure_emigrant_staging(pop, k);
  pop->isl->emigrate(k, pop->emi_rows, pop->emi_scores);
}

void replace_worst(pga::Island& isl, const population_t* from, uint32_t k) {
  isl.immigrate(k, from->emi_rows, from->emi_scores);
}

int default_device() {
  const char* e = std::getenv("PGA_DEVICE");
  if (e && *e) return std::atoi(e);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return -1;
  return 0;
}

uint64_t default_seed() {
  const char* e = std::getenv("PGA_SEED");
  if (e && *e) return std::strtoull(e, nullptr, 10);
  return (uint64_t)std::time(nullptr);  // reference: time(NULL) (src/pga.cu:154)
}

population_t* create(pga_t* p, unsigned long size, unsigned genome_len, int encoding) {
  if (!p) return nullptr;
  if (p->pops.size() >= MAX_POPULATIONS) return nullptr;
  if (genome_len < 4 || size == 0) return nullptr;
  return guard_r<population_t*>(p, nullptr, [&]() -> population_t* {
    pga::Config c;
    c.encoding = encoding;
    c.S = size;
    c.L = genome_len;
    c.seed = p->seed;
    c.island = (uint32_t)p->pops.size();
    c.objective = pga::OBJ_NONE;
    c.selection = pga::SEL_TOURNAMENT;
    c.tour_k = 2;
    if (encoding == pga::ENC_REAL) {  // reference semantics
      c.lo = 0.f;
      c.hi = 1.f;
      c.crossover = pga::XO_UNIFORM;
      c.mutation = pga::MUT_RESET_ONE;
      c.mut_rate = 0.01f;
    } else if (encoding == pga::ENC_BINARY) {
      c.crossover = pga::XO_UNIFORM;
      c.mutation = pga::MUT_BIT_FLIP;
    } else {
      c.crossover = pga::XO_OX;
      c.mutation = pga::MUT_INVERSION;
      c.mut_rate = 0.3f;
      c.tour_k = 4;
    }
    auto pop = std::make_unique<pga_population>();
    pop->owner = p;
    pop->isl = std::make_unique<pga::Island>(c, p->device);
    pop->isl->stream = p->stream;
    pop->isl->initialize();
    population_t* raw = pop.release();
    p->pops.push_back(raw);
    return raw;
  });
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ lifetime
pga_t* pga_init_device(int device) {
  pga_t* p = new (std::nothrow) pga_solver;
  if (!p) return nullptr;
  p->device = device;
  p->seed = default_seed();
  if (device >= 0) {
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
      g_last_error = "cannot initialise the GPU";
      delete p;
      return nullptr;
    }
  }
  return p;
}

pga_t* pga_init(void) { return pga_init_device(default_device()); }

int pga_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

void pga_deinit(pga_t* p) {
  if (!p) return;
  if (!p->pops.empty() && p->mig_cap) {
    pga::Island& isl = *p->pops[0]->isl;
    if (isl.on_gpu()) (void)hipStreamSynchronize(p->stream);  // a posted exchange may still read the staging
    for (void* b : {p->mig_send_rows, p->mig_recv_rows, (void*)p->mig_send_scores, (void*)p->mig_recv_scores})
      dev_free(isl, b);
  }
  if (!p->pops.empty() && p->best_row) dev_free(*p->pops[0]->isl, p->best_row);
  for (population_t* pop : p->pops) delete pop;
  p->pops.clear();
  if (p->comm_members) {
    auto& m = *p->comm_members;
    m.erase(std::remove(m.begin(), m.end(), p), m.end());
  }
  p->comm.reset();
  if (p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
}

void pga_set_seed(pga_t* p, uint64_t seed) {
  if (p) p->seed = seed;
}
void pga_set_quiet(pga_t* p, int quiet) {
  if (p) p->quiet = quiet != 0;
}
void pga_set_abort_on_error(pga_t* p, int a) {
  if (p) p->abort_on_error = a != 0;
}
const char* pga_last_error(void) { return g_last_error.c_str(); }

// --------------------------------------------------------------- populations
population_t* pga_create_population(pga_t* p, unsigned long size, unsigned genome_len, enum population_type type) {
  if (type != RANDOM_POPULATION) return nullptr;
  return create(p, size, genome_len, pga::ENC_REAL);
}

population_t* pga_create_population_ext(pga_t* p, unsigned long size, unsigned genome_len, enum pga_encoding e) {
  if (e != PGA_BINARY && e != PGA_REAL && e != PGA_PERMUTATION) return nullptr;
  if (genome_len == 0 || size == 0 || !p || p->pops.size() >= MAX_POPULATIONS) return nullptr;
  return create(p, size, genome_len < 4 && e == PGA_REAL ? 4 : genome_len, (int)e);
}

void pga_set_objective_function(pga_t* p, obj_f f) {
  if (p) p->objective = f;
}
void pga_set_mutate_function(pga_t* p, mutate_f f) {
  if (p) p->mutate = f;
}
void pga_set_crossover_function(pga_t* p, crossover_f f) {
  if (p) p->crossover = f;
}

int pga_set_objective_builtin(pga_t* p, population_t* pop, enum pga_objective obj, const float* data, size_t n,
                              const float* data2, size_t n2, int iparam, float f0, float f1) {
  if (!valid_pop(p, pop)) return -1;
  return guard_r<int>(p, -1, [&]() {
    pga::Island& isl = *pop->isl;
    isl.stream = p->stream;
    if (data) isl.set_objective_data(data, n, 0);
    if (data2) isl.set_objective_data(data2, n2, 1);
    pga::Config c = isl.config();
    c.objective = (int32_t)obj;
    c.obj_i = iparam;
    c.obj_f0 = f0;
    c.obj_f1 = f1;
    isl.set_operators(c);
    pop->builtin = (int)obj;
    return 0;
  });
}

int pga_set_objective_source(pga_t* p, population_t* pop, const char* source, const char* name, const float* data,
                             size_t n) {
  if (!valid_pop(p, pop) || !source || !name) return -1;
  return guard_r<int>(p, -1, [&]() {
    pga::Island& isl = *pop->isl;
    isl.stream = p->stream;
    auto k = pga::jit_compile(isl.config().encoding, source, name, {});
    if (data) isl.set_objective_data(data, n, 0);
    pga::Config c = isl.config();
    c.objective = pga::OBJ_NONE;
    isl.set_operators(c);
    isl.set_jit_objective(k);
    pop->builtin = -2;
    return 0;
  });
}

int pga_set_operators(pga_t* p, population_t* pop, enum pga_selection sel, unsigned k, enum pga_crossover xo,
                      float xo_prob, enum pga_mutation mut, float rate, float sigma, unsigned elitism) {
  if (!valid_pop(p, pop)) return -1;
  return guard_r<int>(p, -1, [&]() {
    pga::Config c = pop->isl->config();
    c.selection = (int32_t)sel;
    c.tour_k = k ? k : 2;
    c.crossover = (int32_t)xo;
    c.xo_prob = xo_prob;
    c.mutation = (int32_t)mut;
    c.mut_rate = rate;
    c.sigma = sigma;
    c.n_elite = elitism;
    pop->isl->stream = p->stream;
    pop->isl->set_operators(c);
    return 0;
  });
}

int pga_set_bounds(pga_t* p, population_t* pop, float lo, float hi) {
  if (!valid_pop(p, pop) || !(lo < hi)) return -1;
  return guard_r<int>(p, -1, [&]() {
    pga::Config c = pop->isl->config();
    c.lo = lo;
    c.hi = hi;
    pop->isl->set_operators(c);
    return 0;
  });
}

int pga_set_blend_alpha(pga_t* p, population_t* pop, float alpha) {
  if (!valid_pop(p, pop)) return -1;
  return guard_r<int>(p, -1, [&]() {
    pga::Config c = pop->isl->config();
    c.blend_alpha = alpha;
    pop->isl->set_operators(c);
    return 0;
  });
}

int pga_set_rank_pressure(pga_t* p, population_t* pop, float sp) {
  if (!valid_pop(p, pop) || !(sp >= 1.f && sp <= 2.f)) return -1;
  return guard_r<int>(p, -1, [&]() {
    pga::Config c = pop->isl->config();
    c.rank_pressure = sp;
    pop->isl->set_operators(c);
    return 0;
  });
}

// -------------------------------------------------------------------- stages
void pga_evaluate(pga_t* p, population_t* pop) {
  if (!valid_pop(p, pop)) return;
  guard(p, [&]() {
    sync_callbacks(p, pop);
    pop->isl->evaluate();
  });
}

void pga_evaluate_all(pga_t* p) {
  if (!p) return;
  for (population_t* pop : p->pops) pga_evaluate(p, pop);
}

void pga_crossover(pga_t* p, population_t* pop, enum crossover_selection_type type) {
  (void)type;  // TOURNAMENT is the only selection of the original enum; see pga_set_operators
  if (!valid_pop(p, pop)) return;
  guard(p, [&]() {
    sync_callbacks(p, pop);
    pop->isl->crossover_stage();
  });
}

void pga_crossover_all(pga_t* p, enum crossover_selection_type type) {
  if (!p) return;
  for (population_t* pop : p->pops) pga_crossover(p, pop, type);
}

void pga_mutate(pga_t* p, population_t* pop) {
  if (!valid_pop(p, pop)) return;
  guard(p, [&]() {
    sync_callbacks(p, pop);
    pop->isl->mutate_stage();
  });
}

void pga_mutate_all(pga_t* p) {
  if (!p) return;
  for (population_t* pop : p->pops) pga_mutate(p, pop);
}

void pga_swap_generations(pga_t* p, population_t* pop) {
  if (!valid_pop(p, pop)) return;
  pop->isl->swap();
}

void pga_fill_random_values(pga_t* p, population_t* pop) {
  // Randomness is counter-based; this only re-keys the population's streams
  // so repeated stage calls within one generation draw fresh numbers.
  if (!valid_pop(p, pop)) return;
  pop->isl->bump_epoch();
}

// ------------------------------------------------------------------- results
gene* pga_get_best(pga_t* p, population_t* pop) {
  if (!valid_pop(p, pop)) return nullptr;
  return guard_r<gene*>(p, nullptr, [&]() {
    pga::Island& isl = *pop->isl;
    isl.stream = p->stream;
    const unsigned long long b = isl.best_packed();
    if (!p->quiet) std::printf("%f\n", (double)pga::best_score(b));
    return decode_row(isl, isl.row_host(pga::best_index(b)));
  });
}

gene** pga_get_best_top(pga_t* p, population_t* pop, unsigned length) {
  if (!valid_pop(p, pop) || length == 0) return nullptr;
  return guard_r<gene**>(p, nullptr, [&]() -> gene** {
    pga::Island& isl = *pop->isl;
    isl.stream = p->stream;
    const uint32_t k = (uint32_t)std::min<uint64_t>(length, isl.config().S);
    std::vector<uint32_t> idx = isl.topk_host(k, true);
    gene** out = (gene**)std::calloc(length, sizeof(gene*));
    if (!out) throw std::bad_alloc();
    for (uint32_t i = 0; i < k; ++i) out[i] = decode_row(isl, isl.row_host(idx[i]));
    return out;
  });
}

gene* pga_get_best_all(pga_t* p) {
  if (!p || p->pops.empty()) return nullptr;
  return guard_r<gene*>(p, nullptr, [&]() -> gene* {
    population_t* bp = nullptr;
    unsigned long long best = 0;
    for (population_t* pop : p->pops) {
      pop->isl->stream = p->stream;
      const unsigned long long b = pop->isl->best_packed();
      if (!bp || pga::best_score(b) > pga::best_score(best)) {
        bp = pop;
        best = b;
      }
    }
    if (!p->quiet) std::printf("%f\n", (double)pga::best_score(best));
    return decode_row(*bp->isl, bp->isl->row_host(pga::best_index(best)));
  });
}

gene** pga_get_best_top_all(pga_t* p, unsigned length) {
  if (!p || p->pops.empty() || length == 0) return nullptr;
  return guard_r<gene**>(p, nullptr, [&]() -> gene** {
    // per population: top-k on the device, the k winners' rows and scores
    // gathered there, ONE copy of k rows + k scores to the host
    struct Cand {
      float score;
      size_t pop;
      uint32_t slot;
    };
    std::vector<Cand> all;
    std::vector<std::vector<uint32_t>> rows(p->pops.size());
    for (size_t i = 0; i < p->pops.size(); ++i) {
      pga::Island& isl = *p->pops[i]->isl;
      isl.stream = p->stream;
      const uint32_t k = (uint32_t)std::min<uint64_t>(length, isl.config().S);
      const size_t rb = isl.row_bytes();
      // rows at a 16-byte boundary: the gather kernel stores them as uint4
      const size_t roff = (4ull * k + 15) & ~(size_t)15, soff = roff + ((rb * k + 15) & ~(size_t)15);
      char* buf = (char*)isl.scratch(soff + 4ull * k);
      uint32_t* idx = (uint32_t*)buf;
      void* rdev = buf + roff;
      float* sdev = (float*)(buf + soff);
      isl.topk(k, true, idx, /*sorted=*/true);
      isl.gather(idx, k, rdev, sdev);
      rows[i].resize(rb / 4 * k);
      std::vector<float> sc(k);
      isl.copy_to_host(rows[i].data(), rdev, rb * k);
      isl.copy_to_host(sc.data(), sdev, 4ull * k);
      for (uint32_t j = 0; j < k; ++j) all.push_back({sc[j], i, j});
    }
    std::stable_sort(all.begin(), all.end(), [](const Cand& a, const Cand& b) { return a.score > b.score; });
    gene** out = (gene**)std::calloc(length, sizeof(gene*));
    if (!out) throw std::bad_alloc();
    for (size_t i = 0; i < std::min<size_t>(length, all.size()); ++i) {
      const pga::Island& isl = *p->pops[all[i].pop]->isl;
      const size_t rw = isl.row_bytes() / 4;
      std::vector<uint32_t> r(rows[all[i].pop].begin() + rw * all[i].slot, rows[all[i].pop].begin() + rw * (all[i].slot + 1));
      out[i] = decode_row(isl, r);
    }
    return out;
  });
}

// -------------------------------------------------------------------- islands
void pga_migrate_between(pga_t* p, population_t* from, population_t* to, float pct) {
  if (!valid_pop(p, from) || !valid_pop(p, to) || from == to) return;
  guard(p, [&]() {
    pga::Island &a = *from->isl, &b = *to->isl;
    if (a.config().encoding != b.config().encoding || a.config().L != b.config().L)
      throw std::invalid_argument("migration needs populations of the same encoding and genome length");
    a.stream = b.stream = p->stream;
    const uint32_t k = migrants(a.config().S, b.config().S, pct);
    if (!k) return;
    take_best(from, k);
    replace_worst(b, from, k);
  });
}

void pga_migrate(pga_t* p, float pct) {
  if (!p || p->pops.size() < 2) return;
  guard(p, [&]() {
    // random island ring, drawn from the seed so runs are reproducible;
    // every population's emigrants are taken before any is replaced
    const size_t n = p->pops.size();
    std::vector<uint32_t> perm(n);
    for (uint32_t i = 0; i < n; ++i) perm[i] = i;
    pga::RngKey key{(uint32_t)p->seed, (uint32_t)(p->seed >> 32), p->migration_epoch++, 0};
    for (uint32_t i = (uint32_t)n - 1; i >= 1; --i) {
      const uint32_t j = pga::word_to_index(pga::draw(key, pga::ST_MIGRATE, 0, i).x, i + 1);
      std::swap(perm[i], perm[j]);
    }
    std::vector<uint32_t> ks(n, 0);
    for (size_t i = 0; i < n; ++i) {
      population_t* src = p->pops[perm[i]];
      population_t* dst = p->pops[perm[(i + 1) % n]];
      src->isl->stream = p->stream;
      ks[i] = migrants(src->isl->config().S, dst->isl->config().S, pct);
      if (ks[i]) take_best(src, ks[i]);
    }
    for (size_t i = 0; i < n; ++i) {
      population_t* dst = p->pops[perm[(i + 1) % n]];
      if (ks[i]) {
        dst->isl->stream = p->stream;
        replace_worst(*dst->isl, p->pops[perm[i]], ks[i]);
      }
    }
  });
}

extern "C++" {
namespace {
void use_device(pga_t* p) {
  if (p->device >= 0) PGA_HIP_CHECK(hipSetDevice(p->device));
}

void ensure_staging(pga_t* p, pga::Island& isl, uint32_t k) {
  if (p->mig_cap >= k) return;
  for (void* b : {p->mig_send_rows, p->mig_recv_rows, (void*)p->mig_send_scores, (void*)p->mig_recv_scores})
    dev_free(isl, b);
  p->mig_send_rows = p->mig_recv_rows = nullptr;
  p->mig_send_scores = p->mig_recv_scores = nullptr;
  p->mig_cap = 0;
  p->mig_send_rows = dev_alloc(isl, isl.row_bytes() * k);
  p->mig_recv_rows = dev_alloc(isl, isl.row_bytes() * k);
  p->mig_send_scores = (float*)dev_alloc(isl, 4ull * k);
  p->mig_recv_scores = (float*)dev_alloc(isl, 4ull * k);
  p->mig_cap = k;
}

// Inter-rank migration of population 0 of every solver in `solvers` (all the
// ranks this call drives: one per process with ncclCommInitRank, all of them
// with InitAll / loopback), in two phases so the transfer overlaps compute:
//   post_ranks    per rank: emigrants (island policy: exact top-k by default)
//                 packed on the compute stream -> the epoch's plan posted on
//                 the transport (RCCL: the rank's communication stream, which
//                 waits only for the packed emigrants)
//   finish_ranks  [host poll against the deadline, after whatever the caller
//                 enqueued meanwhile] -> compute stream ordered after the
//                 transfer -> received rows re-scored with the LOCAL
//                 objective (a forged score never enters) -> bottom-k
//                 replaced
// run_islands posts at a migration point, enqueues the next generation, then
// finishes: the exchange runs beside that generation and the host waits (if
// at all) only once it is queued.  A failure or expiry aborts the
// communicator and leaves every rank of the call degraded.
void degrade(const std::vector<pga_t*>& solvers, const char* what) {
  for (pga_t* p : solvers) {
    if (!p->degraded) ++p->comm_failures;
    p->degraded = true;
    p->mig_pending = false;
  }
  std::fprintf(stderr, "pga: %s over %s failed (%s); islands continue without migration\n", what,
               solvers.front()->comm ? solvers.front()->comm->name() : "?", g_last_error.c_str());
}

bool comm_active(const pga_t* p0) {
  return p0->comm && !(p0->comm->size() == 1 && !p0->comm->self_exchange) && !p0->degraded;
}

std::vector<pga::LocalRank> local_ranks(const std::vector<pga_t*>& solvers) {
  std::vector<pga::LocalRank> local;
  for (pga_t* p : solvers) {
    pga::Island& isl = *p->pops[0]->isl;
    pga::LocalRank l;
    l.rank = p->comm_rank;
    l.device = p->device;
    l.stream = p->stream;
    l.row_bytes = isl.row_bytes();
    l.send_rows = p->mig_send_rows;
    l.send_scores = p->mig_send_scores;
    l.recv_rows = p->mig_recv_rows;
    l.recv_scores = p->mig_recv_scores;
    local.push_back(l);
  }
  return local;
}

bool post_ranks(const std::vector<pga_t*>& solvers, float pct) {
  pga_t* p0 = solvers.front();
  // a 1-rank communicator exchanges only in self-exchange (test) mode
  if (!comm_active(p0) || p0->mig_pending) return false;
  pga::Comm& comm = *p0->comm;
  const uint64_t S = p0->pops[0]->isl->config().S;
  const uint32_t k0 = migrants(S, S, pct);
  const uint32_t k = pga::plan_migrants(p0->topology, comm.size(), k0);
  if (!k) return false;
  if (k > S / 2) throw std::invalid_argument("migration: too many migrants for the population size");
  const std::vector<pga::Xfer> plan = pga::migration_plan(p0->topology, comm.size(), k0, p0->seed, p0->comm_epoch);
  for (pga_t* p : solvers) {
    use_device(p);
    pga::Island& isl = *p->pops[0]->isl;
    if (isl.config().S != S || isl.row_bytes() != p0->pops[0]->isl->row_bytes())
      throw std::invalid_argument("migration: ranks need populations of the same size and genome length");
    isl.stream = p->stream;
    ensure_staging(p, isl, k);
    isl.emigrate(k, p->mig_send_rows, p->mig_send_scores);
  }
  std::vector<pga::LocalRank> local = local_ranks(solvers);
  try {
    comm.exchange(plan, local);
  } catch (const std::exception& e) {
    g_last_error = e.what();
    for (pga_t* p : solvers) ++p->comm_epoch;
    degrade(solvers, "migration");
    return false;
  }
  for (pga_t* p : solvers) {
    p->mig_pending = true;
    p->mig_k = k;
  }
  return true;
}

void finish_ranks(const std::vector<pga_t*>& solvers) {
  pga_t* p0 = solvers.front();
  if (!p0->mig_pending) return;
  pga::Comm& comm = *p0->comm;
  const uint32_t k = p0->mig_k;
  std::vector<pga::LocalRank> local = local_ranks(solvers);
  bool ok = true;
  try {
    ok = comm.wait(local, p0->comm_timeout);
  } catch (const std::exception& e) {
    g_last_error = e.what();
    ok = false;
  }
  for (pga_t* p : solvers) {
    ++p->comm_epoch;
    p->mig_pending = false;
  }
  if (!ok) {
    if (g_last_error.empty()) g_last_error = "transfer failed or timed out";
    degrade(solvers, "migration");
    return;
  }
  for (pga_t* p : solvers) {
    use_device(p);
    pga::Island& isl = *p->pops[0]->isl;
    isl.stream = p->stream;
    if (p->validate_migrants) isl.evaluate_rows(p->mig_recv_rows, p->mig_recv_scores, k);
    isl.immigrate(k, p->mig_recv_rows, p->mig_recv_scores);
    p->migrants_received += k;
  }
}

// the serial form (pga_comm_exchange): post and receive at once
void migrate_ranks(const std::vector<pga_t*>& solvers, float pct) {
  if (post_ranks(solvers, pct)) finish_ranks(solvers);
}
}  // namespace
}  // extern "C++"

void pga_run(pga_t* p, unsigned n) {
  if (!p || p->pops.empty()) return;
  guard(p, [&]() {
    population_t* pop = p->pops[0];
    sync_callbacks(p, pop);
    pop->isl->stream = p->stream;
    pop->isl->evaluate();  // reference: evaluate precedes every crossover (src/pga.cu:383)
    pop->isl->run(n);      // each fused generation leaves its children evaluated
  });
}

int pga_run_until(pga_t* p, unsigned n, float target, unsigned check_every) {
  if (!p || p->pops.empty()) return -1;
  return guard_r<int>(p, -1, [&]() {
    population_t* pop = p->pops[0];
    sync_callbacks(p, pop);
    pop->isl->stream = p->stream;
    pop->isl->evaluate();
    if (pop->isl->best_score() >= target) return 0;
    return (int)pop->isl->run_until(n, target, check_every);
  });
}

// Islands evolve concurrently, one HIP stream each, between migration points;
// a migration joins them on the solver stream (events), exchanges, and forks
// them again.  Small islands are launch/latency bound, so running them side by
// side on the 256 CUs is what makes many-island runs cheap on one MI355X.
namespace {
void fork_islands(pga_t* p) {
  hipEvent_t ev;
  PGA_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  PGA_HIP_CHECK(hipEventRecord(ev, p->stream));
  for (population_t* pop : p->pops) {
    if (!pop->stream) {
      PGA_HIP_CHECK(hipStreamCreateWithFlags(&pop->stream, hipStreamNonBlocking));
      PGA_HIP_CHECK(hipEventCreateWithFlags(&pop->done, hipEventDisableTiming));
    }
    PGA_HIP_CHECK(hipStreamWaitEvent(pop->stream, ev, 0));
    pop->isl->stream = pop->stream;
  }
  PGA_HIP_CHECK(hipEventDestroy(ev));
}

void join_islands(pga_t* p) {
  for (population_t* pop : p->pops) {
    PGA_HIP_CHECK(hipEventRecord(pop->done, pop->stream));
    PGA_HIP_CHECK(hipStreamWaitEvent(p->stream, pop->done, 0));
    pop->isl->stream = p->stream;
  }
}
}  // namespace

namespace {
// n generations of every population of every solver in `solvers`, migrating
// every m generations: first between the populations of each solver
// (pga_migrate), then between ranks (migrate_ranks).  Each solver's islands
// run on their own streams; solvers on different GPUs run concurrently
// because nothing here waits on the host between migration points.
// best score over every population of `solvers` and, with a communicator that
// is still healthy, over every rank (the same value on all of them)
float global_best(const std::vector<pga_t*>& solvers) {
  std::vector<uint32_t> mine;
  float all_best = -INFINITY;
  for (pga_t* q : solvers) {
    use_device(q);
    float b = -INFINITY;
    for (population_t* pop : q->pops) {
      pop->isl->stream = q->stream;
      b = std::max(b, pop->isl->best_score());
    }
    uint32_t w;
    std::memcpy(&w, &b, 4);
    mine.push_back(w);
    all_best = std::max(all_best, b);
  }
  pga_t* p0 = solvers.front();
  if (!comm_active(p0)) return all_best;
  std::vector<uint32_t> all;
  bool ok = false;
  try {
    ok = p0->comm->allgather(local_ranks(solvers), mine, 1, all, p0->comm_timeout);
  } catch (const std::exception& e) {
    g_last_error = e.what();
  }
  if (!ok) {  // a dead or withheld peer: every local rank continues alone on its own best
    if (g_last_error.empty()) g_last_error = "all-gather failed or timed out";
    degrade(solvers, "global best all-gather");
    return all_best;
  }
  for (uint32_t w : all) {
    float v;
    std::memcpy(&v, &w, 4);
    all_best = std::max(all_best, v);
  }
  return all_best;
}

// n generations of every population of every solver in `solvers`, migrating
// every m generations (see below); with a target (not NaN) the run stops at
// the first check point (every m generations, 10 when m == 0) whose global
// best reaches it.  Returns the generations run.
unsigned run_islands_until(const std::vector<pga_t*>& solvers, unsigned n, unsigned m, float pct, float target) {
  for (pga_t* p : solvers) {
    use_device(p);
    for (population_t* pop : p->pops) {
      sync_callbacks(p, pop);
      pop->isl->stream = p->stream;
      pop->isl->evaluate();
    }
  }
  const bool until = !std::isnan(target);
  const unsigned every = m > 0 ? m : 10u;  // check points of a target run
  if (until && global_best(solvers) >= target) return 0;
  auto generations = [&](unsigned k) {
    for (pga_t* p : solvers) {
      use_device(p);
      const bool gpu = p->device >= 0;
      if (gpu && p->pops.size() > 1 && p->batch_islands) {
        // same-shape islands: one launch per generation for all of them
        std::vector<pga::Island*> v;
        for (population_t* pop : p->pops) v.push_back(pop->isl.get());
        if (pga::Island::run_batched(v, k, p->stream)) {
          p->batched_gens += k;
          continue;
        }
      }
      if (gpu) fork_islands(p);
      for (population_t* pop : p->pops) pop->isl->run(k);
      if (gpu) join_islands(p);
    }
  };
  unsigned g = 0;
  while (g < n) {
    // generations until the next migration / check point (or the end)
    unsigned step = n - g;
    const unsigned period = m > 0 ? m : (until ? every : 0u);
    if (period > 0) {
      const unsigned next = (g / period + 1) * period;
      if (next < n) step = next - g;
    }
    if (solvers.front()->mig_pending) {
      // the exchange posted at the last migration point runs beside this
      // generation; its migrants enter the population that generation made
      generations(1);
      finish_ranks(solvers);
      ++g;
      --step;
    }
    if (step > 0) generations(step);
    g += step;
    if (until && global_best(solvers) >= target) break;
    if (m > 0 && g % m == 0 && g < n) {
      for (pga_t* p : solvers) {
        use_device(p);
        pga_migrate(p, pct);
      }
      post_ranks(solvers, pct);
    }
  }
  finish_ranks(solvers);  // nothing is left in flight (a no-op unless a check point ended the run)
  return g;
}
}  // namespace

int pga_set_batch_islands(pga_t* p, int on) {
  if (!p) return -1;
  p->batch_islands = on != 0;
  return 0;
}

unsigned long long pga_batched_generations(const pga_t* p) { return p ? p->batched_gens : 0ull; }

void pga_run_islands(pga_t* p, unsigned n, unsigned m, float pct) {
  if (!p || p->pops.empty()) return;
  guard(p, [&]() {
    if (p->comm && p->comm->drives_all_ranks() && p->comm->size() > 1)
      throw std::invalid_argument("this communicator drives all ranks from one process: use pga_run_islands_multi");
    (void)run_islands_until({p}, n, m, pct, NAN);
  });
}

int pga_run_islands_until(pga_t* p, unsigned n, unsigned m, float pct, float target) {
  if (!p || p->pops.empty()) return -1;
  return guard_r<int>(p, -1, [&]() {
    if (p->comm && p->comm->drives_all_ranks() && p->comm->size() > 1)
      throw std::invalid_argument("this communicator drives all ranks from one process: use pga_run_islands_multi");
    if (std::isnan(target)) throw std::invalid_argument("pga_run_islands_until: target is NaN");
    return (int)run_islands_until({p}, n, m, pct, target);
  });
}

namespace {
int run_multi(pga_t** solvers, int count, unsigned n, unsigned m, float pct, float target) {
  if (!solvers || count < 1 || !solvers[0]) return -1;
  pga_t* p0 = solvers[0];
  return guard_r<int>(p0, -1, [&]() {
    std::vector<pga_t*> v(solvers, solvers + count);
    for (pga_t* p : v) {
      if (!p || p->pops.empty()) throw std::invalid_argument("pga_run_islands_multi: solver without populations");
      if (p->comm != p0->comm) throw std::invalid_argument("pga_run_islands_multi: solvers of different communicators");
    }
    if (p0->comm && p0->comm->size() > 1 && (!p0->comm->drives_all_ranks() || count != p0->comm->size()))
      throw std::invalid_argument("pga_run_islands_multi: pass every rank of an InitAll / loopback group");
    std::sort(v.begin(), v.end(), [](pga_t* a, pga_t* b) { return a->comm_rank < b->comm_rank; });
    return (int)run_islands_until(v, n, m, pct, target);
  });
}
}  // namespace

int pga_run_islands_multi(pga_t** solvers, int count, unsigned n, unsigned m, float pct) {
  return run_multi(solvers, count, n, m, pct, NAN) < 0 ? -1 : 0;
}

int pga_run_islands_multi_until(pga_t** solvers, int count, unsigned n, unsigned m, float pct, float target) {
  if (std::isnan(target)) return -1;
  return run_multi(solvers, count, n, m, pct, target);
}

// -------------------------------------------------------------------- queries
unsigned long pga_population_size(const population_t* pop) { return pop ? (unsigned long)pop->isl->config().S : 0; }
unsigned pga_genome_length(const population_t* pop) { return pop ? pop->isl->config().L : 0; }
unsigned pga_generation(const population_t* pop) { return pop ? pop->isl->generation() : 0; }
size_t pga_row_bytes(const population_t* pop) { return pop ? pop->isl->row_bytes() : 0; }

float pga_best_score(pga_t* p, population_t* pop) {
  if (!valid_pop(p, pop)) return NAN;
  return guard_r<float>(p, NAN, [&]() {
    pop->isl->stream = p->stream;
    return pop->isl->best_score();
  });
}

unsigned long pga_best_index(pga_t* p, population_t* pop) {
  if (!valid_pop(p, pop)) return 0;
  return guard_r<unsigned long>(p, 0, [&]() {
    pop->isl->stream = p->stream;
    return (unsigned long)pop->isl->best_index();
  });
}

int pga_get_scores(pga_t* p, population_t* pop, float* out) {
  if (!valid_pop(p, pop) || !out) return -1;
  return guard_r<int>(p, -1, [&]() {
    pop->isl->stream = p->stream;
    pop->isl->copy_to_host(out, pop->isl->scores(0), 4ull * pop->isl->config().S);
    return 0;
  });
}

int pga_get_genome(pga_t* p, population_t* pop, unsigned long i, void* out) {
  if (!valid_pop(p, pop) || !out) return -1;
  return guard_r<int>(p, -1, [&]() {
    pop->isl->stream = p->stream;
    std::vector<uint32_t> r = pop->isl->row_host(i);
    std::memcpy(out, r.data(), 4 * r.size());
    return 0;
  });
}

int pga_set_stats_history(pga_t* p, population_t* pop, int on) {
  if (!valid_pop(p, pop)) return -1;
  return guard_r<int>(p, -1, [&]() {
    pop->isl->set_stats_history(on != 0);
    return 0;
  });
}

long pga_get_stats_history(pga_t* p, population_t* pop, float* out, unsigned long max_rows) {
  if (!valid_pop(p, pop)) return -1;
  return guard_r<long>(p, -1, [&]() {
    pop->isl->stream = p->stream;
    const std::vector<float> h = pop->isl->history();
    const unsigned long rows = h.size() / 4;
    if (out) std::memcpy(out, h.data(), 16ull * std::min(rows, max_rows));
    return (long)rows;
  });
}

int pga_stats(pga_t* p, population_t* pop, float out[4]) {
  if (!valid_pop(p, pop) || !out) return -1;
  return guard_r<int>(p, -1, [&]() {
    pop->isl->stream = p->stream;
    pop->isl->stats(out);
    return 0;
  });
}

int pga_synchronize(pga_t* p) {
  if (!p) return -1;
  if (p->stream) return hipStreamSynchronize(p->stream) == hipSuccess ? 0 : -1;
  return 0;
}

int pga_save(pga_t* p, population_t* pop, const char* path) {
  if (!valid_pop(p, pop) || !path) return -1;
  return guard_r<int>(p, -1, [&]() {
    pop->isl->stream = p->stream;
    pop->isl->save(path);
    return 0;
  });
}

int pga_load(pga_t* p, population_t* pop, const char* path) {
  if (!valid_pop(p, pop) || !path) return -1;
  return guard_r<int>(p, -1, [&]() {
    pop->isl->stream = p->stream;
    pop->isl->load(path);
    return 0;
  });
}

// ---------------------------------------------------------------------- comm
int pga_comm_unique_id(char id[128]) {
  try {
    return pga::rccl_unique_id(id);
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return -1;
  }
}

int pga_comm_init(pga_t* p, int nranks, int rank, const char id[128]) {
  if (!p || p->device < 0 || !id) return -1;
  return guard_r<int>(p, -1, [&]() {
    p->comm = pga::rccl_comm_rank(nranks, rank, id, p->device);
    p->comm_rank = rank;
    p->comm_members.reset();
    return 0;
  });
}

namespace {
int init_group(pga_t** solvers, int n, bool loopback) {
  if (!solvers || n < 1) return -1;
  for (int i = 0; i < n; ++i)
    if (!solvers[i]) return -1;
  return guard_r<int>(solvers[0], -1, [&]() {
    std::shared_ptr<pga::Comm> c;
    if (loopback) {
      c = pga::loopback_comm(n);
    } else {
      std::vector<int> devs(n);
      for (int i = 0; i < n; ++i) {
        if (solvers[i]->device < 0) throw std::invalid_argument("pga_comm_init_local needs GPU solvers");
        devs[i] = solvers[i]->device;
      }
      c = pga::rccl_comm_all(devs);
    }
    auto members = std::make_shared<std::vector<pga_t*>>(solvers, solvers + n);
    for (int i = 0; i < n; ++i) {
      solvers[i]->comm = c;
      solvers[i]->comm_rank = i;
      solvers[i]->comm_members = members;
      solvers[i]->topology = solvers[0]->topology;
      solvers[i]->seed = solvers[0]->seed;  // identical random-ring draws on every rank
    }
    return 0;
  });
}
}  // namespace

int pga_comm_init_local(pga_t** solvers, int n) { return init_group(solvers, n, false); }
int pga_comm_init_loopback(pga_t** solvers, int n) { return init_group(solvers, n, true); }

int pga_comm_rank(const pga_t* p) { return p && p->comm ? p->comm_rank : 0; }
int pga_comm_size(const pga_t* p) { return p && p->comm ? p->comm->size() : 1; }

static_assert((int)PGA_MIGRATE_TOPK == pga::MIG_TOPK && (int)PGA_MIGRATE_STRIPE == pga::MIG_STRIPE,
              "pga_ext.h migration policies mirror core.hpp");

int pga_set_migration_policy(pga_t* p, population_t* pop, enum pga_migration_policy policy) {
  if (!valid_pop(p, pop)) return -1;
  return guard_r<int>(p, -1, [&]() {
    pop->isl->set_migration_policy((int)policy);
    return 0;
  });
}

int pga_comm_set_topology(pga_t* p, enum pga_topology t) {
  if (!p || (t != PGA_TOPO_RING && t != PGA_TOPO_RANDOM && t != PGA_TOPO_ALL_TO_ALL)) return -1;
  if (p->comm_members)
    for (pga_t* q : *p->comm_members) q->topology = (int)t;
  p->topology = (int)t;
  return 0;
}

int pga_comm_set_timeout(pga_t* p, double seconds) {
  if (!p || seconds < 0) return -1;
  p->comm_timeout = seconds;
  return 0;
}

int pga_comm_set_validation(pga_t* p, int on) {
  if (!p) return -1;
  p->validate_migrants = on != 0;
  return 0;
}

int pga_comm_degraded(const pga_t* p) { return p && p->degraded ? 1 : 0; }

int pga_comm_info(const pga_t* p, struct pga_comm_stats* out) {
  if (!p || !out) return -1;
  out->epochs = p->comm_epoch;
  out->failures = p->comm_failures;
  out->degraded = p->degraded ? 1 : 0;
  out->migrants_received = p->migrants_received;
  out->bytes_sent = p->comm ? p->comm->bytes_sent : 0;
  return 0;
}

int pga_comm_set_fault(pga_t* p, int every, int mode) {
  if (!p || !p->comm) return -1;
  return guard_r<int>(p, -1, [&]() {
    p->comm->set_fault(every, mode);
    return 0;
  });
}

int pga_comm_exchange(pga_t** solvers, int count, float pct) {
  if (!solvers || count < 1 || !solvers[0]) return -1;
  pga_t* p0 = solvers[0];
  return guard_r<int>(p0, -1, [&]() {
    std::vector<pga_t*> v(solvers, solvers + count);
    for (pga_t* p : v) {
      if (!p || p->pops.empty()) throw std::invalid_argument("pga_comm_exchange: solver without populations");
      if (p->comm != p0->comm) throw std::invalid_argument("pga_comm_exchange: solvers of different communicators");
    }
    if (p0->comm && p0->comm->size() > 1 && p0->comm->drives_all_ranks() && count != p0->comm->size())
      throw std::invalid_argument("pga_comm_exchange: pass every rank of an InitAll / loopback group");
    std::sort(v.begin(), v.end(), [](pga_t* a, pga_t* b) { return a->comm_rank < b->comm_rank; });
    migrate_ranks(v, pct);
    return 0;
  });
}

extern "C++" {
namespace {
// the solvers this process drives for p's communicator (all ranks of an
// InitAll / loopback group, else p alone)
std::vector<pga_t*> comm_solvers(pga_t* p) {
  std::vector<pga_t*> solvers{p};
  if (p->comm && p->comm->drives_all_ranks() && p->comm_members) solvers = *p->comm_members;
  std::sort(solvers.begin(), solvers.end(), [](pga_t* a, pga_t* b) { return a->comm_rank < b->comm_rank; });
  return solvers;
}

// (score, index) of every local rank's population-0 best, all-gathered: the
// global best = the highest score, ties to the lowest rank.  false: the
// all-gather failed or timed out (the group is degraded, *score / *rank / *idx
// describe the local best).
bool comm_best_of(pga_t* p, const std::vector<pga_t*>& solvers, float* score, int* rank, uint32_t* idx) {
  std::vector<uint32_t> mine;
  for (pga_t* q : solvers) {
    use_device(q);
    pga::Island& isl = *q->pops[0]->isl;
    isl.stream = q->stream;
    const unsigned long long b = isl.best_packed();
    const float s = pga::best_score(b);
    uint32_t w;
    std::memcpy(&w, &s, 4);
    mine.push_back(w);
    mine.push_back((uint32_t)pga::best_index(b));
  }
  std::vector<uint32_t> all = mine;
  bool ok = true;
  if (comm_active(p)) {
    try {
      ok = p->comm->allgather(local_ranks(solvers), mine, 2, all, p->comm_timeout);
    } catch (const std::exception& e) {
      g_last_error = e.what();
      ok = false;
    }
    if (!ok) {
      degrade(solvers, "global best all-gather");
      all = mine;
    }
  }
  const int nr = ok && comm_active(p) ? p->comm->size() : (int)solvers.size();
  int br = 0;
  float bs = -INFINITY;
  for (int i = 0; i < nr; ++i) {
    float v;
    std::memcpy(&v, &all[2 * i], 4);
    if (i == 0 || v > bs) {
      bs = v;
      br = i;
    }
  }
  if (score) *score = bs;
  if (rank) *rank = ok && comm_active(p) ? br : solvers[br]->comm_rank;
  if (idx) *idx = all[2 * br + 1];
  return ok;
}
}  // namespace
}  // extern "C++"

int pga_comm_best(pga_t* p, float* score, int* rank) {
  if (!p || p->pops.empty()) return -1;
  return guard_r<int>(p, -1, [&]() {
    (void)comm_best_of(p, comm_solvers(p), score, rank, nullptr);
    return 0;
  });
}

int pga_comm_get_best(pga_t* p, float* score, int* rank, void* row_out) {
  if (!p || p->pops.empty()) return -1;
  return guard_r<int>(p, -1, [&]() {
    const std::vector<pga_t*> solvers = comm_solvers(p);
    float bs = 0.f;
    int br = 0;
    uint32_t bi = 0;
    const bool ok = comm_best_of(p, solvers, &bs, &br, &bi);
    if (score) *score = bs;
    if (rank) *rank = br;
    if (!row_out) return 0;
    pga_t* self = p;
    if (!ok || !comm_active(p)) {  // local only: the winner is one of our own solvers
      for (pga_t* q : solvers)
        if (q->comm_rank == br) self = q;
      pga::Island& isl = *self->pops[0]->isl;
      std::vector<uint32_t> r = isl.row_host(bi);
      std::memcpy(row_out, r.data(), isl.row_bytes());
      return 0;
    }
    // the winning rank copies its row into the staging, the communicator
    // broadcasts it, every rank reads it back
    std::vector<void*> bufs;
    for (pga_t* q : solvers) {
      use_device(q);
      pga::Island& isl = *q->pops[0]->isl;
      if (!q->best_row) q->best_row = dev_alloc(isl, isl.row_bytes());
      if (q->comm_rank == br) {
        const char* src = (const char*)isl.rows(0) + (size_t)bi * isl.row_bytes();
        if (isl.on_gpu())
          PGA_HIP_CHECK(hipMemcpyAsync(q->best_row, src, isl.row_bytes(), hipMemcpyDeviceToDevice, q->stream));
        else
          std::memcpy(q->best_row, src, isl.row_bytes());
      }
      bufs.push_back(q->best_row);
    }
    std::vector<pga::LocalRank> local = local_ranks(solvers);
    const size_t rb = p->pops[0]->isl->row_bytes();
    bool bok = false;
    try {
      bok = p->comm->broadcast(local, bufs, rb, br, p->comm_timeout);
    } catch (const std::exception& e) {
      g_last_error = e.what();
    }
    if (!bok) {
      degrade(solvers, "best-genome broadcast");
      return -1;
    }
    pga::Island& isl = *p->pops[0]->isl;
    isl.stream = p->stream;
    isl.copy_to_host(row_out, p->best_row, rb);
    return 0;
  });
}

int pga_comm_set_self_exchange(pga_t* p, int on) {
  if (!p || !p->comm) return -1;
  p->comm->self_exchange = on != 0;
  return 0;
}

}  // extern "C"
