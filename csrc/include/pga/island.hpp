// island.hpp — the native GA runtime: one population (an "island") resident on
// one device (or on the host for the CPU reference backend).
//
// An Island owns its memory (double-buffered rows + scores, per-block best
// partials, mutation tables, objective data, top-k/roulette workspaces) and
// enqueues every stage on ONE stream without host synchronisation, so a run
// of n generations is n back-to-back fused kernel launches.  It is the
// engine behind both the reference-compatible C API (csrc/capi/pga.cpp,
// include/pga.h) and the torch bindings (csrc/python/bindings.cpp).
//
// Reference counterparts: struct population / struct pga (src/pga.cu:37-56),
// __fill_population (:107-118), pga_run (:376-391), pga_get_best (:218-236).
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "pga/core.hpp"
#include "pga/jit.hpp"
#include "pga/ops.hpp"

namespace pga {
struct TopkFused;  // ops.hpp
}

namespace pga {

struct Config {
  int32_t encoding = ENC_BINARY;
  uint64_t S = 0;
  uint32_t L = 0;
  int32_t selection = SEL_TOURNAMENT;
  uint32_t tour_k = 2;
  int32_t crossover = XO_UNIFORM;
  float xo_prob = 1.f;
  float blend_alpha = 0.5f;
  int32_t mutation = MUT_BIT_FLIP;
  float mut_rate = -1.f;  // < 0: 1/L per gene (BIT_FLIP/GAUSSIAN/UNIFORM), 0.01 per individual (RESET_ONE...)
  float sigma = 0.1f;
  float rank_pressure = 1.5f;  // SEL_RANK: expected copies of the best individual, in [1, 2]
  float lo = 0.f, hi = 1.f;
  int32_t objective = OBJ_ONEMAX;
  int32_t obj_i = 0;
  float obj_f0 = 0.f, obj_f1 = 0.f;
  uint32_t n_elite = 0;
  uint64_t seed = 0;
  uint32_t island = 0;
};

// words per row and gene chunks for an encoding
void row_geometry(int32_t encoding, uint32_t L, uint32_t* row_words, uint32_t* chunks);

struct Buffer {
  void* ptr = nullptr;
  size_t bytes = 0;
};

class Island {
 public:
  // device >= 0: GPU ordinal; device < 0: CPU reference backend
  Island(const Config& cfg, int device);
  ~Island();
  Island(const Island&) = delete;
  Island& operator=(const Island&) = delete;

  const Config& config() const { return cfg_; }
  bool on_gpu() const { return device_ >= 0; }
  int device() const { return device_; }
  uint32_t row_words() const { return row_words_; }
  uint32_t chunks() const { return chunks_; }
  uint32_t generation() const { return gen_; }
  void set_generation(uint32_t g) { gen_ = g; }
  uint32_t epoch() const { return epoch_; }
  void bump_epoch() { ++epoch_; }

  hipStream_t stream = nullptr;

  // ---- configuration (may be changed between generations) ----
  void set_operators(const Config& c);  // selection/crossover/mutation/objective scalars
  void set_objective_data(const float* host, size_t n, int which);  // which = 0 or 1
  void set_user_fn(void* f) {
    user_fn_ = f;
    invalidate();
  }
  // reference-ABI crossover_f / mutate_f device pointers (nullptr = built-in)
  void set_user_operators(void* xo, void* mut);
  // hipRTC-compiled objective (jit.hpp); needs objective OBJ_NONE and the GPU.
  // Its data pointer is objective data slot 0.  nullptr detaches.
  void set_jit_objective(std::shared_ptr<JitKernel> k);
  bool has_jit() const { return (bool)jit_; }
  // generations whose JIT objective ran inside the generation kernel (fused),
  // and why fusion is off when it is ("" while it works or was never tried)
  uint64_t jit_fused_generations() const { return jit_fused_gens_; }
  std::string jit_fused_error() const { return jit_ ? jit_->fused_error() : std::string(); }

  // ---- stages ----
  void initialize();          // random population + evaluation (generation 0)
  void evaluate();            // scores(cur) <- objective(rows(cur))
  void run(uint32_t n);       // n fused generations
  // n generations of several islands of one device as ONE launch per
  // generation (binary_launch_batch: BINARY, same shape / operators, built-in
  // integer objective); every island's stream is set to s.  Returns false
  // (nothing run) when the islands do not qualify: run them one by one.
  static bool run_batched(const std::vector<Island*>& isls, uint32_t n, hipStream_t s);
  // up to n generations, stopping once the best score reaches `target`; the
  // best is read (one stream sync) every `check_every` generations (0: 10).
  // Returns the generations run.
  uint32_t run_until(uint32_t n, float target, uint32_t check_every);
  void crossover_stage();     // next <- crossover(select(cur))  (no mutation / evaluation)
  void mutate_stage();        // mutate next in place
  void swap();                // cur <-> next, generation++
  void rebest();              // recompute best partials (and tournament keys) of cur from its scores

  // ---- queries (synchronise the stream) ----
  unsigned long long best_packed();
  float best_score() { return pga::best_score(best_packed()); }
  uint64_t best_index() { return pga::best_index(best_packed()); }
  void stats(float out4[4]);  // min, max, sum, count of current scores
  // Per-generation statistics history: when on, every generation appends its
  // {min, max, sum, count} row on the device (from the generation kernel's
  // fused partials, no pass over the scores); history() copies the rows out.
  // Turning it on clears the history and disables hipGraph replay.
  void set_stats_history(bool on);
  // manual history: generations append no row themselves; the caller appends
  // one per generation with record_history_row() once the scores are final
  // (an objective evaluated outside the island, e.g. GeneticAlgorithm's
  // torch_objective)
  void set_history_manual(bool on) { hist_manual_ = on; }
  void record_history_row() {
    if (hist_on_) append_history();
  }
  bool stats_history() const { return hist_on_; }
  std::vector<float> history();
  std::vector<uint32_t> topk_host(uint32_t k, bool largest);
  std::vector<uint32_t> row_host(uint64_t i);

  // ---- device-side building blocks (no sync) ----
  // idx_out: device (or host for CPU) memory.  sorted: best first (ties by
  // index); unsorted: selection order, cheaper (migration, elitism)
  void topk(uint32_t k, bool largest, uint32_t* idx_out, bool sorted = true);
  void gather(const uint32_t* idx, uint32_t n, void* out_rows, float* out_scores);
  void scatter(const uint32_t* idx, uint32_t n, const void* in_rows, const float* in_scores);
  // Island migration, stream-ordered: emigrate = the top-k rows + scores
  // (selection order) into out buffers; immigrate = the k given rows replace
  // the bottom-k (then best partials follow).  On the GPU, integer objectives
  // do each in ONE selection kernel with the row moves fused in; otherwise
  // topk + gather / scatter.  `idx_scratch` (k words, device) may be null.
  void emigrate(uint32_t k, void* out_rows, float* out_scores);
  // MIG_TOPK (default: the reference's "top pct%") or MIG_STRIPE, see core.hpp MigrationPolicy
  void set_migration_policy(int p);
  int migration_policy() const { return mig_policy_; }
  void immigrate(uint32_t k, const void* in_rows, const float* in_scores);
  // score n external rows (e.g. received migrants) with this island's
  // objective, in place; false when the objective is not native (OBJ_NONE)
  bool evaluate_rows(void* rows, float* scores, uint32_t n);
  // Fused key histogram (GenArgs::key_hist): when on, the BINARY generation
  // kernel of an integer objective also produces the value histogram of the
  // keys it writes, and the exact top-k / bottom-k selections of that
  // population (migration, elitism > 1, unsorted top-k) skip their histogram
  // pass over the keys.  On by default with elitism > 1; island models turn it
  // on for migration.  Results are identical either way.
  void set_fused_histogram(bool on);
  bool fused_histogram() const { return fhist_on_; }
  // a fused histogram of the current population is available (tests, benches)
  bool fused_histogram_ready() const { return fhist_of_[cur_] >= 0; }
  // Persistent multi-generation launches of the headline kernel (run(n) as
  // ONE launch with a device-wide barrier between generations); off by
  // default: measured slower than one launch per generation on MI355X
  bool persistent() const { return persistent_; }
  void set_persistent(bool on) { persistent_ = on; }

  // raw buffers (cur = current generation)
  void* rows(int which) { return rows_[which ^ cur_].ptr; }
  float* scores(int which) { return (float*)scores_[which ^ cur_].ptr; }
  unsigned long long* best_parts() { return (unsigned long long*)best_[cur_].ptr; }
  uint32_t n_best() const { return n_best_[cur_]; }
  void set_n_best(uint32_t n) {
    n_best_[cur_] = n;
    stats_ok_[cur_] = false;
  }
  size_t row_bytes() const { return 4ull * row_words_; }

  // scratch buffers for callers (migration staging)
  void* scratch(size_t bytes);

  // hipGraph replay: run() records G generations once per (parity, epoch,
  // configuration) and replays the graph; 0 disables.  Default: PGA_GRAPH
  // env (generations per graph), else 0.  Bit-identical to plain launches.
  // Off by default because it measured no gain on MI355X: even the smallest
  // populations (S=100) are bound by the kernel's own dependent memory chain
  // (~4.8 us/gen with or without the graph), not by host launch cost
  // (profiles/README.md).
  void set_graph_generations(uint32_t g);
  uint32_t graph_generations() const { return graph_g_; }
  uint64_t graph_replays() const { return graph_replays_; }
  // BINARY knapsack: int8 digits per value of the matrix-core evaluation
  // (0: the instance is not integer-exact and runs the scalar evaluation)
  uint32_t knapsack_digits() const { return knap_dig_; }

  // checkpoint: header + current rows + scores
  void save(const std::string& path);
  void load(const std::string& path);

  void synchronize();
  void copy_to_host(void* dst, const void* src, size_t bytes);
  void copy_to_device(void* dst, const void* src, size_t bytes);

 private:
  GenArgs make_args(int mode);
  uint32_t launch(int mode, const GenArgs& a, unsigned long long* parts);
  void prepare_generation();  // elitism indices, roulette prefix
  Buffer alloc(size_t bytes);
  void release(Buffer& b);
  void rebuild_mut_table();
  void ensure_topk_ws(uint32_t k);

  Config cfg_;
  int device_;
  uint32_t row_words_ = 0, chunks_ = 0;
  int cur_ = 0;
  uint32_t gen_ = 0, epoch_ = 0;
  Buffer rows_[2], scores_[2], best_[2], keys_[2];
  uint32_t n_best_[2] = {0, 0};
  Buffer mut_thr_, obj_data_[2], elite_idx_, cumfit_, cum_ws_, topk_ws_, stats_, out_best_, scratch_;
  Buffer rank_order_, rank_ws_;
  Buffer roul_guide_;  // roulette guide table (GPU), S + 1 entries
  // REAL on the GPU: quantized u16 tournament keys in keys_[p] (qkey), valid
  // when qk_valid_[p]; qk_ws_ = {min, max, sum, count} of the current
  // generation (+ score_stats workspace), the range the GEN kernel quantizes
  // the next generation's keys over
  bool real_qk() const;
  void invalidate_qk() {
    qk_valid_[cur_] = false;
    fhist_of_[cur_] = -1;  // the keys of the current population change
    if (rank_cnt_of_ == cur_) rank_cnt_of_ = -1;
  }
  Buffer qk_ws_;
  bool qk_valid_[2] = {false, false};
  Buffer qubo_qt_;               // QUBO: int8 Q^T packed from objective data slot 0 (GPU)
  uint32_t obj_version_ = 0, qubo_version_ = ~0u;
  void prepare_objective();      // derived objective data (QUBO packing)
  size_t obj_len_[2] = {0, 0};
  std::vector<float> obj_host0_;  // host copy of objective data slot 0 (derived tables)
  Buffer knap_tab_;               // BINARY knapsack: matrix-core digit table (GPU, integer instances)
  uint32_t knap_version_ = ~0u, knap_dig_ = 0, knap_cols_ = 0;
  // fused statistics partials per parity ({min, sum} per block of the kernel
  // that wrote best_[p]); stats_ok_[p]: they belong to the current best_[p]
  Buffer stats_parts_[2];
  bool stats_ok_[2] = {false, false};
  // stats_part_[p]: the block partition of the binary_gen_tp launch whose
  // partials stats_parts_[p] holds (grid 0: another kernel wrote them)
  TpPartition stats_part_[2] = {{0, 0, 0}, {0, 0, 0}};
  void set_stats_ok(int p, bool ok) {
    stats_ok_[p] = ok;
    stats_part_[p] = TpPartition{0, 0, 0};
  }
  static bool roul_fused_off();  // PGA_ROUL_FUSED=0: the three-launch roulette prefix (A/B knob)
  bool roul_packed() const;      // the GEN kernels read the packed guide table (GenArgs::roul_packed; off)
  bool fused_stats() const;  // the evaluating kernels of this configuration store them
  void append_history();
  Buffer hist_;
  std::vector<float> hist_host_;  // CPU backend
  uint64_t hist_n_ = 0;
  bool hist_on_ = false, hist_manual_ = false;
  int mig_policy_ = MIG_TOPK;
  float mut_inv_ = 0.f;
  bool mut_sparse_ = false;  // BINARY bit-flip uses the sparse (Binomial) sampler
  float mut_rate_eff_ = 0.f;
  void* user_fn_ = nullptr;
  void* user_xo_fn_ = nullptr;
  void* user_mut_fn_ = nullptr;
  Buffer compat_rand_, ev_parts_;
  std::shared_ptr<JitKernel> jit_;
  // JIT evaluation of `n` rows at `rows` -> scores, block bests -> parts; returns the grid
  uint32_t jit_eval(const void* rows, float* scores, uint64_t n, unsigned long long* parts);
  bool fused_jit_generation(GenArgs& a);
  uint32_t qk_age_ = 0;  // REAL quantized keys: generations since the range was refreshed
  bool jit_fused_off_ = false;
  uint64_t jit_fused_gens_ = 0;
  u32x4 last_mask_{0, 0, 0, 0};

  // graph replay state
  void run_plain(uint32_t n);
  bool run_tiny(uint32_t n);
  bool run_multi(uint32_t n);  // n headline generations in one persistent launch (binary_gen_tp_multi)
  bool persistent_ = false;    // run_multi on (PGA_TP_MULTI=1 or set_persistent)
  bool run_graph(uint32_t reps, bool fresh);
  bool capture_graph();
  void drop_graph();
  void invalidate() {
    ++version_;
    fhist_of_[0] = fhist_of_[1] = -1;
    rank_cnt_of_ = -1;
  }
  // fused key histograms: three buffers of fused_hist_words(L + 1) words
  // rotated by the generations that produce one (each zeroes the next);
  // fhist_of_[p] = the buffer with the histogram of parity p's population
  Buffer fhist_[3];
  int fhist_of_[2] = {-1, -1};
  bool fhist_clean_[3] = {true, true, true};  // its selection status words are still zero
  uint32_t fhist_rot_ = 0;
  bool fhist_on_ = false, fhist_user_ = false;
  bool fhist_ready_for(const GenArgs& a) const;  // this GEN launch produces the histogram
  // rank selection of an integer objective: the GEN kernel also stores the
  // next rank sort's tile counts into rank_ws_ (GenArgs::rank_counts);
  // rank_cnt_of_ = the parity whose keys they count (-1: none), consumed by
  // the next prepare_generation's sort
  int rank_cnt_of_ = -1;
  uint32_t* rank_counts_for_gen() const;
  const TopkFused* fused_select(TopkFused& f);    // the current population's histogram for a select
  uint32_t graph_g_ = 0, version_ = 0;
  bool graph_broken_ = false, capturing_ = false;
  uint32_t capture_base_ = 0;
  Buffer gen_dev_;
  Buffer tp_pool_;        // binary_gen_tp pair-pool counters (tp.hpp), GPU BINARY only
  Buffer multi_bar_;      // binary_gen_tp_multi's grid-barrier counter
  Buffer obj_aux_;        // derived objective table (TSP: the integer matrix as u16, GenArgs::obj_aux)
  uint32_t aux_kind_ = 0, aux_bytes_ = 0, aux_version_ = ~0u;
  bool aux_on_ = true;    // PGA_TSP_NO_LDS unset at construction
  uint32_t batch_n_ = 1;  // islands of the batch this one runs in (run_batched), else 1
  uint32_t tp_seq_ = 0;   // their per-launch stamp
  hipStream_t cap_stream_ = nullptr;
  hipGraphExec_t gexec_ = nullptr;
  int g_cur_ = -1;
  uint32_t g_epoch_ = 0, g_version_ = 0, g_nbest_ = 0, g_len_ = 0;
  uint64_t graph_replays_ = 0;
};

}  // namespace pga
