// island.cpp — native GA runtime (see island.hpp).
#include "pga/island.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "pga/cpu.hpp"
#include "pga/ops.hpp"
#include "pga/trace.hpp"

namespace pga {

void row_geometry(int32_t encoding, uint32_t L, uint32_t* row_words, uint32_t* chunks) {
  uint32_t c = 0;
  switch (encoding) {
    case ENC_BINARY: c = (L + 127) / 128; break;
    case ENC_REAL: c = (L + 3) / 4; break;
    case ENC_PERMUTATION: c = (L + 7) / 8; break;
    default: throw std::invalid_argument("unknown encoding");
  }
  if (c == 0) c = 1;
  *chunks = c;
  *row_words = 4 * c;
}

namespace {
bool per_individual_mutation(int32_t m) { return m == MUT_RESET_ONE || m == MUT_SWAP || m == MUT_INVERSION; }
uint32_t prob_thresh(float p) {
  double v = std::floor((double)p * 4294967296.0);
  return v >= 4294967295.0 ? 0xFFFFFFFFu : (v <= 0 ? 0u : (uint32_t)v);
}
}  // namespace

Island::Island(const Config& cfg, int device) : cfg_(cfg), device_(device) {
  if (cfg_.S == 0) throw std::invalid_argument("population size must be > 0");
  if (cfg_.S >= (1ull << 32)) throw std::invalid_argument("population size must be < 2^32");
  if (cfg_.L == 0) throw std::invalid_argument("genome length must be > 0");
  if (cfg_.encoding == ENC_PERMUTATION && cfg_.L > 65536) throw std::invalid_argument("permutation length > 65536");
  if (cfg_.island >= 65536) throw std::invalid_argument("island id must be < 65536");
  row_geometry(cfg_.encoding, cfg_.L, &row_words_, &chunks_);
  if (on_gpu()) PGA_HIP_CHECK(hipSetDevice(device_));
  const uint64_t Sp = cfg_.S + kRowPad;  // padded (ops.hpp kRowPad)
  const size_t rb = 4ull * row_words_ * Sp;
  for (int i = 0; i < 2; ++i) {
    rows_[i] = alloc(rb);
    scores_[i] = alloc(4ull * Sp);
    best_[i] = alloc(8ull * kMaxGrid);
    if (on_gpu()) stats_parts_[i] = alloc(8ull * kMaxGrid);
    keys_[i] = alloc(2ull * Sp);
  }
  out_best_ = alloc(64);
  stats_ = alloc(4ull * (4 + 3 * 1024));
  aux_on_ = std::getenv("PGA_TSP_NO_LDS") == nullptr;  // verification: the f32 L2 matrix path
  persistent_ = [] {
    const char* e = std::getenv("PGA_TP_MULTI");
    return e && e[0] == '1';
  }();
  if (on_gpu() && cfg_.encoding == ENC_BINARY) {  // binary_gen_tp's pair-pool counters (stamp 0 = stale)
    tp_pool_ = alloc(tp_pool_bytes(kMaxGrid));
    PGA_HIP_CHECK(hipMemset(tp_pool_.ptr, 0, tp_pool_.bytes));
  }
  if (cfg_.encoding == ENC_BINARY) {
    const uint32_t rem = cfg_.L - 128 * (chunks_ - 1);
    uint32_t m[4];
    for (uint32_t j = 0; j < 4; ++j) m[j] = range_mask32(32 * j, 0, rem);
    last_mask_ = u32x4{m[0], m[1], m[2], m[3]};
  } else {
    last_mask_ = u32x4{~0u, ~0u, ~0u, ~0u};
  }
  set_operators(cfg_);
  if (const char* e = std::getenv("PGA_GRAPH")) set_graph_generations((uint32_t)std::strtoul(e, nullptr, 10));
}

Island::~Island() {
  Buffer* all[] = {&rows_[0],   &rows_[1],     &scores_[0],   &scores_[1],  &best_[0],  &best_[1],   &mut_thr_,
                   &obj_data_[0], &obj_data_[1], &keys_[0], &keys_[1], &elite_idx_, &cumfit_, &cum_ws_, &roul_guide_, &topk_ws_, &stats_,
                   &out_best_,  &scratch_, &compat_rand_, &ev_parts_, &gen_dev_, &rank_order_, &rank_ws_, &qubo_qt_,
                   &knap_tab_, &stats_parts_[0], &stats_parts_[1], &hist_, &qk_ws_, &tp_pool_, &obj_aux_,
                   &fhist_[0], &fhist_[1], &fhist_[2], &multi_bar_};
  drop_graph();
  if (cap_stream_) (void)hipStreamDestroy(cap_stream_);
  for (Buffer* b : all) {
    try {
      release(*b);
    } catch (...) {
    }
  }
}

Buffer Island::alloc(size_t bytes) {
  Buffer b;
  b.bytes = bytes;
  if (bytes == 0) return b;
  if (on_gpu()) {
    PGA_HIP_CHECK(hipMalloc(&b.ptr, bytes));
  } else {
    b.ptr = std::aligned_alloc(64, (bytes + 63) & ~(size_t)63);
    if (!b.ptr) throw std::bad_alloc();
    std::memset(b.ptr, 0, bytes);
  }
  return b;
}

void Island::release(Buffer& b) {
  if (!b.ptr) return;
  if (on_gpu()) PGA_HIP_CHECK(hipFree(b.ptr));
  else std::free(b.ptr);
  b.ptr = nullptr;
  b.bytes = 0;
}

void* Island::scratch(size_t bytes) {
  if (scratch_.bytes < bytes) {
    if (on_gpu() && scratch_.ptr) synchronize();
    release(scratch_);
    scratch_ = alloc(bytes);
  }
  return scratch_.ptr;
}

void Island::copy_to_host(void* dst, const void* src, size_t bytes) {
  if (on_gpu()) {
    PGA_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream));
    PGA_HIP_CHECK(hipStreamSynchronize(stream));
  } else {
    std::memcpy(dst, src, bytes);
  }
}

void Island::copy_to_device(void* dst, const void* src, size_t bytes) {
  if (on_gpu()) {
    PGA_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream));
    PGA_HIP_CHECK(hipStreamSynchronize(stream));
  } else {
    std::memcpy(dst, src, bytes);
  }
}

void Island::synchronize() {
  if (on_gpu()) PGA_HIP_CHECK(hipStreamSynchronize(stream));
}

void Island::rebuild_mut_table() {
  const bool per_ind = per_individual_mutation(cfg_.mutation);
  mut_rate_eff_ = cfg_.mut_rate >= 0.f ? cfg_.mut_rate : (per_ind ? 0.01f : 1.f / (float)cfg_.L);
  if (mut_rate_eff_ > 1.f) mut_rate_eff_ = 1.f;
  std::vector<uint32_t> thr(kMutCap);
  build_mut_table(per_ind ? 0.f : mut_rate_eff_, kMutCap, thr.data(), &mut_inv_);
  // sparse samplers (K ~ Binomial(L, p), then K distinct positions): BINARY
  // bit-flip and REAL per-gene mutation at the usual ~1/L rates
  const bool per_gene = (cfg_.encoding == ENC_BINARY && cfg_.mutation == MUT_BIT_FLIP) ||
                        (cfg_.encoding == ENC_REAL && (cfg_.mutation == MUT_GAUSSIAN || cfg_.mutation == MUT_UNIFORM));
  mut_sparse_ = per_gene && bin_sparse_mutation(cfg_.L, mut_rate_eff_);
  if (mut_sparse_) build_binom_table(mut_rate_eff_, cfg_.L, thr.data());
  if (!mut_thr_.ptr) mut_thr_ = alloc(4ull * kMutCap);
  if (on_gpu()) synchronize();
  copy_to_device(mut_thr_.ptr, thr.data(), 4ull * kMutCap);
}

void Island::set_operators(const Config& c) {
  invalidate();
  if (c.S != cfg_.S || c.L != cfg_.L || c.encoding != cfg_.encoding)
    throw std::invalid_argument("set_operators cannot change S, L or encoding");
  if (c.selection == SEL_TOURNAMENT && (c.tour_k < 1 || c.tour_k > 64))
    throw std::invalid_argument("tournament size must be in [1, 64]");
  if (c.n_elite > c.S) throw std::invalid_argument("elitism count exceeds population");
  if (c.selection < SEL_TOURNAMENT || c.selection > SEL_RANK) throw std::invalid_argument("unknown selection");
  if (c.selection == SEL_RANK && !(c.rank_pressure >= 1.f && c.rank_pressure <= 2.f))
    throw std::invalid_argument("rank pressure must be in [1, 2]");
  const float old_rate = cfg_.mut_rate;
  const int32_t old_mut = cfg_.mutation;
  cfg_ = c;
  if (!mut_thr_.ptr || old_rate != c.mut_rate || old_mut != c.mutation) rebuild_mut_table();
  fhist_on_ = fhist_user_ || cfg_.n_elite > 1;  // elitism > 1 selects top-k every generation
  if (cfg_.n_elite > 1 && elite_idx_.bytes < 4ull * cfg_.n_elite) {
    release(elite_idx_);
    elite_idx_ = alloc(4ull * cfg_.n_elite);
  }
  if (cfg_.selection == SEL_ROULETTE && !cumfit_.ptr) {
    cumfit_ = alloc(4ull * (cfg_.S + 4));  // + 4: the GEN kernels' 16-byte window loads (tp.hpp)
    if (on_gpu()) {
      cum_ws_ = alloc(4ull * roulette_workspace_floats(cfg_.S));
      roul_guide_ = alloc(8ull * (cfg_.S + 4));  // packed: {guide, cumfit} per entry (roul_packed)
    }
  }
  if (cfg_.selection == SEL_RANK && !rank_order_.ptr) {
    rank_order_ = alloc(4ull * cfg_.S);
    if (on_gpu()) rank_ws_ = alloc(rank_order_workspace_bytes(cfg_.S));
  }
}

void Island::set_user_operators(void* xo, void* mut) {
  invalidate();
  if ((xo || mut) && !on_gpu()) throw std::invalid_argument("device function pointers need the GPU backend");
  if ((xo || mut) && cfg_.encoding != ENC_REAL)
    throw std::invalid_argument("user crossover/mutate callbacks need the REAL (float gene) encoding");
  user_xo_fn_ = xo;
  user_mut_fn_ = mut;
  if ((xo || mut) && !compat_rand_.ptr) compat_rand_ = alloc(4ull * cfg_.S * cfg_.L);
}

void Island::set_objective_data(const float* host, size_t n, int which) {
  invalidate();
  if (which < 0 || which > 1) throw std::invalid_argument("objective data slot must be 0 or 1");
  if (on_gpu()) synchronize();
  release(obj_data_[which]);
  obj_data_[which] = alloc(4ull * (n ? n : 1));
  if (n) copy_to_device(obj_data_[which].ptr, host, 4ull * n);
  obj_len_[which] = n;
  if (which == 0) obj_host0_.assign(host, host + n);
  ++obj_version_;
}

void Island::prepare_objective() {
  if (cfg_.objective == OBJ_KNAPSACK && cfg_.encoding == ENC_BINARY && on_gpu() && knap_version_ != obj_version_) {
    knap_version_ = obj_version_;
    knap_dig_ = knap_cols_ = 0;
    std::vector<uint8_t> tab;
    if (obj_host0_.size() >= 2ull * cfg_.L &&
        build_knap_table(obj_host0_.data(), obj_host0_.data() + cfg_.L, cfg_.L, chunks_, tab, knap_dig_, knap_cols_)) {
      if (knap_tab_.bytes < tab.size()) {
        release(knap_tab_);
        knap_tab_ = alloc(tab.size());
      }
      copy_to_device(knap_tab_.ptr, tab.data(), tab.size());
    }
  }
  if ((cfg_.objective == OBJ_TSP || cfg_.objective == OBJ_TSP_OPEN) && cfg_.encoding == ENC_PERMUTATION && on_gpu() &&
      aux_version_ != obj_version_) {
    // the matrix for the LDS-resident tour evaluation (perm.hip perm_gen_fast
    // TBL): an integer matrix (entries in [0, 65535]) as u16 — the strict
    // lower triangle plus the diagonal when symmetric (kind 1), else the full
    // matrix (kind 2); any other symmetric matrix as the f32 triangle plus
    // diagonal (kind 3); an asymmetric float matrix stays in L2 (kind 0)
    aux_version_ = obj_version_;
    aux_kind_ = aux_bytes_ = 0;
    const uint32_t L = cfg_.L;
    const float* d = obj_host0_.data();
    // (only what can fit one CU's LDS: 160 KiB)
    const size_t tri = (size_t)L * (L + 1) / 2, lds = 160 * 1024;
    const bool have = obj_host0_.size() >= (size_t)L * L && L >= 2 && 2 * tri <= lds;
    bool ints = have, sym = have;
    for (size_t i = 0; ints && i < (size_t)L * L; ++i) ints = d[i] >= 0.f && d[i] <= 65535.f && d[i] == std::floor(d[i]);
    for (uint32_t i = 0; sym && i < L; ++i)
      for (uint32_t j = 0; sym && j < i; ++j)
        sym = std::memcmp(&d[(size_t)i * L + j], &d[(size_t)j * L + i], sizeof(float)) == 0;
    std::vector<uint8_t> t;
    auto put = [&t](const auto v) {
      const size_t o = t.size();
      t.resize(o + sizeof(v));
      std::memcpy(t.data() + o, &v, sizeof(v));
    };
    if (ints && sym) {
      for (uint32_t i = 0; i < L; ++i)  // rows of the lower triangle with the diagonal: (i, j <= i) at i (i + 1) / 2 + j
        for (uint32_t j = 0; j <= i; ++j) put((uint16_t)d[(size_t)i * L + j]);
      aux_kind_ = 1;
    } else if (ints && 2ull * L * L <= lds) {
      for (size_t i = 0; i < (size_t)L * L; ++i) put((uint16_t)d[i]);
      aux_kind_ = 2;
    } else if (sym && !ints && 4 * tri <= lds) {
      for (uint32_t i = 0; i < L; ++i)
        for (uint32_t j = 0; j <= i; ++j) put(d[(size_t)i * L + j]);
      aux_kind_ = 3;
    }
    if (aux_kind_) {
      t.resize((t.size() + 15) / 16 * 16, 0);  // whole 16-byte stores
      if (obj_aux_.bytes < t.size()) {
        release(obj_aux_);
        obj_aux_ = alloc(t.size());
      }
      copy_to_device(obj_aux_.ptr, t.data(), t.size());
      aux_bytes_ = (uint32_t)t.size();
    }
  }
  if (cfg_.objective != OBJ_QUBO) return;
  if (cfg_.encoding != ENC_BINARY) throw std::invalid_argument("the QUBO objective needs the BINARY encoding");
  if (obj_len_[0] < (size_t)cfg_.L * cfg_.L) throw std::invalid_argument("QUBO: objective data must hold the L x L matrix Q");
  if (!on_gpu() || qubo_version_ == obj_version_) return;
  const uint32_t lp = qubo_padded_length(cfg_.L);
  if (lp > kQuboMaxBits) throw std::invalid_argument("QUBO objective supports genomes of at most 1024 bits");
  if (qubo_qt_.bytes < (size_t)lp * lp) {
    release(qubo_qt_);
    qubo_qt_ = alloc((size_t)lp * lp);
  }
  qubo_pack_launch((const float*)obj_data_[0].ptr, cfg_.L, (int8_t*)qubo_qt_.ptr, stream);
  qubo_version_ = obj_version_;
}

GenArgs Island::make_args(int mode) {
  prepare_objective();
  GenArgs a;
  std::memset(&a, 0, sizeof(a));
  a.qubo_qt = (const int8_t*)qubo_qt_.ptr;
  if (aux_kind_ && aux_on_ && (cfg_.objective == OBJ_TSP || cfg_.objective == OBJ_TSP_OPEN)) {
    a.obj_aux = obj_aux_.ptr;
    a.obj_aux_kind = aux_kind_;
    a.obj_aux_bytes = aux_bytes_;
  }
  if (cfg_.objective == OBJ_KNAPSACK && knap_cols_ > 0) {
    a.knap_tab = knap_tab_.ptr;
    a.knap_dig = knap_dig_;
    a.knap_cols = knap_cols_;
  }
  const int nx = cur_ ^ 1;
  a.cur = rows_[cur_].ptr;
  a.next = rows_[nx].ptr;
  a.score_cur = (const float*)scores_[cur_].ptr;
  a.score_next = (float*)scores_[nx].ptr;
  if (mode == MODE_INIT || mode == MODE_EVAL) {
    a.next = rows_[cur_].ptr;
    a.score_next = (float*)scores_[cur_].ptr;
  } else if (mode == MODE_MUTATE) {
    a.cur = rows_[nx].ptr;
    a.next = rows_[nx].ptr;
  }
  a.S = cfg_.S;
  a.L = cfg_.L;
  a.row_words = row_words_;
  a.chunks = chunks_;
  a.encoding = (uint32_t)cfg_.encoding;
  a.key.k0 = (uint32_t)cfg_.seed;
  a.key.k1 = (uint32_t)(cfg_.seed >> 32) ^ (epoch_ * 0x9E3779B9u);
  a.key.gen = gen_;
  a.key.island = cfg_.island;
  a.selection = cfg_.selection;
  a.tour_k = cfg_.tour_k;
  a.cumfit = (const float*)cumfit_.ptr;
  a.roul_guide = (const uint32_t*)roul_guide_.ptr;
  a.roul_packed = roul_guide_.ptr && roul_packed() ? 1u : 0u;
  a.roul_scale = cum_ws_.ptr ? (const float*)cum_ws_.ptr + kRoulScale : nullptr;
  a.rank_order = (const uint32_t*)rank_order_.ptr;
  a.rank_thresh = rank_thresh_of(cfg_.rank_pressure);
  a.crossover = cfg_.crossover;
  a.xo_always = cfg_.xo_prob >= 1.f ? 1u : 0u;
  a.xo_thresh_hi = prob_thresh(cfg_.xo_prob);
  a.blend_alpha = cfg_.blend_alpha;
  a.mutation = cfg_.mutation;
  a.mut_rate = mut_rate_eff_;
  a.mut_ind_thresh = per_individual_mutation(cfg_.mutation) ? prob_thresh(mut_rate_eff_) : 0u;
  a.mut_thr = (const uint32_t*)mut_thr_.ptr;
  a.mut_inv_log2_1mp = mut_inv_;
  a.mut_sparse = mut_sparse_ ? 1u : 0u;
  a.sigma = cfg_.sigma;
  a.lo = cfg_.lo;
  a.hi = cfg_.hi;
  a.objective = cfg_.objective;
  a.obj_i = cfg_.obj_i;
  a.obj_f0 = cfg_.obj_f0;
  a.obj_f1 = cfg_.obj_f1;
  a.obj_data = (const float*)obj_data_[0].ptr;
  a.obj_data2 = (const float*)obj_data_[1].ptr;
  a.user_fn = user_fn_;
  a.user_xo_fn = user_xo_fn_;
  a.user_mut_fn = user_mut_fn_;
  a.compat_rand = (float*)compat_rand_.ptr;
  a.n_elite = cfg_.n_elite;
  a.elite_idx = cfg_.n_elite > 1 ? (const uint32_t*)elite_idx_.ptr : nullptr;
  if (mode == MODE_GEN && tp_pool_.ptr && !capturing_) {
    // a stamp per launch (never 0: zeroed counters are stale); a graph
    // replay would repeat its stamp, so captured generations run without
    a.tp_pool = (unsigned long long*)tp_pool_.ptr;
    if (++tp_seq_ == 0) ++tp_seq_;
    a.tp_seq = tp_seq_;
  }
  a.best_cur = (const unsigned long long*)best_[cur_].ptr;
  a.n_best_cur = n_best_[cur_];
  static const uint32_t nt = [] {
    const char* e = std::getenv("PGA_TP_NT_STORE");
    return e && e[0] == '1' ? 1u : 0u;
  }();
  a.nt_store = nt;
  a.last_mask = last_mask_;
  if (capturing_) {
    a.gen_dev = (const uint32_t*)gen_dev_.ptr;
    a.gen_off = gen_ - capture_base_;
  }
  if (fused_stats()) a.stats_parts = (float*)stats_parts_[(mode == MODE_INIT || mode == MODE_EVAL) ? cur_ : nx].ptr;
  if (integer_objective(cfg_.objective, cfg_.L)) {
    a.key_cur = (const uint16_t*)keys_[cur_].ptr;
    a.key_next = (uint16_t*)keys_[nx].ptr;
    if (mode == MODE_INIT || mode == MODE_EVAL) a.key_next = (uint16_t*)keys_[cur_].ptr;
  } else if (mode == MODE_GEN && real_qk() && qk_valid_[cur_] && qk_ws_.ptr) {
    a.key_cur = (const uint16_t*)keys_[cur_].ptr;
    a.key_next = (uint16_t*)keys_[nx].ptr;
    a.qk = (const float*)qk_ws_.ptr;
  }
  return a;
}

uint32_t Island::launch(int mode, const GenArgs& a, unsigned long long* parts) {
  if (mode != MODE_GEN && a.cur == rows_[cur_].ptr) {  // staged / init / eval
    fhist_of_[0] = fhist_of_[1] = -1;
    rank_cnt_of_ = -1;
  }
  if (on_gpu()) return encoding_launch(mode, a, parts, stream);
  return cpu::encoding_run(mode, a, parts);
}

void Island::initialize() {
  TraceRange tr("pga.initialize");
  invalidate_qk();
  GenArgs a = make_args(MODE_INIT);
  n_best_[cur_] = launch(MODE_INIT, a, (unsigned long long*)best_[cur_].ptr);
  set_stats_ok(cur_, a.stats_parts != nullptr);
  if (jit_) {
    n_best_[cur_] = jit_eval(rows_[cur_].ptr, (float*)scores_[cur_].ptr, cfg_.S, (unsigned long long*)best_[cur_].ptr);
    set_stats_ok(cur_, false);
  } else if (cfg_.objective == OBJ_NONE) {
    rebest();
  }
}

void Island::evaluate() {
  TraceRange tr("pga.evaluate");
  invalidate_qk();
  if (jit_) {
    n_best_[cur_] = jit_eval(rows_[cur_].ptr, (float*)scores_[cur_].ptr, cfg_.S, (unsigned long long*)best_[cur_].ptr);
    set_stats_ok(cur_, false);
    return;
  }
  GenArgs a = make_args(MODE_EVAL);
  n_best_[cur_] = launch(MODE_EVAL, a, (unsigned long long*)best_[cur_].ptr);
  set_stats_ok(cur_, a.stats_parts != nullptr);
}

void Island::rebest() {
  set_stats_ok(cur_, false);
  invalidate_qk();
  const float* sc = (const float*)scores_[cur_].ptr;
  if (on_gpu()) {
    uint16_t* keys = integer_objective(cfg_.objective, cfg_.L) ? (uint16_t*)keys_[cur_].ptr : nullptr;
    n_best_[cur_] = best_of_scores_launch(sc, cfg_.S, (unsigned long long*)best_[cur_].ptr, stream, keys);
  } else {
    ((unsigned long long*)best_[cur_].ptr)[0] = cpu::best_of_scores(sc, cfg_.S);
    n_best_[cur_] = 1;
  }
}

bool Island::real_qk() const {
  // quantized tournament keys feed only the two-phase kernel (real_gen_tp),
  // which small populations do not take: there they would cost a launch
  return on_gpu() && cfg_.encoding == ENC_REAL && cfg_.objective != OBJ_NONE && cfg_.objective != OBJ_USER_FNPTR &&
         !jit_ &&
         cfg_.S * batch_n_ >= real_tp_min_population();
}

void Island::prepare_generation() {
  if (real_qk()) {
    // the current generation's score range (fused partials when its kernel
    // stored them), and its quantized keys if anything rewrote the scores
    if (!qk_ws_.ptr) {
      qk_ws_ = alloc(4ull * (4 + 3 * 1024));
      qk_age_ = 0;
    }
    const float* sc = (const float*)scores_[cur_].ptr;
    // The quantization range only has to be the same for every key of a
    // generation: keys are monotonic in the score and equal keys fall back to
    // the exact f32 compare, so any range gives the same tournaments.  It is
    // refreshed every few generations (a stale range only costs more
    // ties), not every generation: small populations are launch-bound.
    // Every 8 generations (32 below 2^18 children, where the ~5 us refresh
    // launch is a larger share of a short generation: reference E1).
    const uint32_t refresh = cfg_.S * batch_n_ < (1ull << 18) ? 32u : 8u;
    if (qk_age_++ % refresh == 0) {
      if (stats_ok_[cur_])
        stats_from_parts_launch((const float*)stats_parts_[cur_].ptr, (const unsigned long long*)best_[cur_].ptr,
                                n_best_[cur_], cfg_.S, (float*)qk_ws_.ptr, stream);
      else
        score_stats_launch(sc, cfg_.S, (float*)qk_ws_.ptr, stream);
    }
    if (!qk_valid_[cur_]) {
      scores_to_qkeys_launch(sc, cfg_.S, (const float*)qk_ws_.ptr, (uint16_t*)keys_[cur_].ptr, stream);
      qk_valid_[cur_] = true;
    }
  }
  if (cfg_.selection == SEL_ROULETTE) {
    const float* sc = (const float*)scores_[cur_].ptr;
    const bool fused = on_gpu() && stats_ok_[cur_] && stats_parts_[cur_].ptr;  // min from the GEN kernel's partials
    // integer objectives after a two-phase GEN launch: one exact launch
    // (the partials give every block its carry)
    const bool one = fused && stats_part_[cur_].grid && integer_objective(cfg_.objective, cfg_.L) &&
                     cfg_.objective != OBJ_KNAPSACK && !roul_fused_off() &&
                     roulette_fused_launch(sc, cfg_.S, (const float*)stats_parts_[cur_].ptr, stats_part_[cur_], cfg_.L,
                                           (float*)cumfit_.ptr, (uint32_t*)roul_guide_.ptr, (float*)cum_ws_.ptr, stream,
                                           roul_packed());
    if (one) {
    } else if (on_gpu()) {
      roulette_prefix_launch(sc, cfg_.S, fused ? (const float*)stats_parts_[cur_].ptr : nullptr, n_best_[cur_],
                             (float*)cumfit_.ptr, (float*)cum_ws_.ptr, stream, integer_objective(cfg_.objective, cfg_.L));
      roulette_guide_launch((const float*)cumfit_.ptr, cfg_.S, (uint32_t*)roul_guide_.ptr, (float*)cum_ws_.ptr, stream,
                            roul_packed());
    } else {
      cpu::roulette_prefix(sc, cfg_.S, (float*)cumfit_.ptr);
    }
  }
  if (cfg_.selection == SEL_RANK) {
    const float* sc = (const float*)scores_[cur_].ptr;
    if (on_gpu() && integer_objective(cfg_.objective, cfg_.L) && keys_[cur_].ptr) {
      // the tile counts of these keys, when the GEN kernel that wrote them stored them
      const bool ready = rank_cnt_of_ == cur_ && !capturing_;
      rank_cnt_of_ = -1;  // the sort scans them in place
      rank_order16_launch((const uint16_t*)keys_[cur_].ptr, cfg_.S, cfg_.L + 1, (uint32_t*)rank_order_.ptr,
                          rank_ws_.ptr, stream, ready);
    }
    else if (on_gpu()) rank_order_launch(sc, cfg_.S, (uint32_t*)rank_order_.ptr, rank_ws_.ptr, stream);
    else cpu::rank_order(sc, cfg_.S, (uint32_t*)rank_order_.ptr);
  }
  if (cfg_.n_elite > 1) topk(cfg_.n_elite, true, (uint32_t*)elite_idx_.ptr, /*sorted=*/false);
}

void Island::run(uint32_t n) {
  TraceRange tr("pga.run");
  if (run_tiny(n)) return;
  if (on_gpu() && graph_g_ > 0 && !graph_broken_ && !hist_on_ && n >= graph_g_ + 2) {
    const bool fresh = gexec_ && g_cur_ == cur_ && g_epoch_ == epoch_ && g_version_ == version_ &&
                       g_nbest_ == n_best_[cur_] && g_len_ == graph_g_;
    if (!fresh) {
      // two plain generations first: the best-partials count of this parity
      // then equals the GEN kernel's grid, which is what every replay leaves
      run_plain(2);
      n -= 2;
    }
    const uint32_t reps = n / graph_g_;
    fhist_of_[0] = fhist_of_[1] = -1;  // replays do not produce the fused histograms
    rank_cnt_of_ = -1;                 // (nor rank counts; their sorts overwrite the workspace)
    if (run_graph(reps, fresh)) n -= reps * graph_g_;
  }
  if (run_multi(n)) return;
  run_plain(n);
}

bool Island::run_multi(uint32_t n) {
  // off by default (PGA_TP_MULTI=1 turns it on): measured slower on MI355X,
  // the barrier's L2 writeback + invalidate and its polling cost more than the
  // launch ramp it removes (interleaved A/B, profiles/persistent_ab_r06.txt:
  // 94.7 vs 89.5 us/gen over 500 generations, 97.3 vs 91.7 over 20)
  if (!persistent_ || n < 2 || !on_gpu() || cfg_.encoding != ENC_BINARY || jit_ || capturing_ || hist_on_) return false;
  if (!integer_objective(cfg_.objective, cfg_.L) || cfg_.objective == OBJ_KNAPSACK || cfg_.n_elite > 1 ||
      (cfg_.selection != SEL_TOURNAMENT && cfg_.selection != SEL_RANDOM))
    return false;  // (no per-generation host work between the generations: prepare_generation is empty)
  GenArgs a = make_args(MODE_GEN);
  const int nx = cur_ ^ 1;
  MultiGenArgs mg;
  mg.parts[0] = (unsigned long long*)best_[nx].ptr;  // generation i writes the partials of parity cur_ ^ 1 ^ (i & 1)
  mg.parts[1] = (unsigned long long*)best_[cur_].ptr;
  mg.stats[0] = a.stats_parts;
  mg.stats[1] = a.stats_parts ? (float*)stats_parts_[cur_].ptr : nullptr;
  mg.gens = n;
  if (!multi_bar_.ptr) multi_bar_ = alloc(256);
  mg.barrier = (uint32_t*)multi_bar_.ptr;
  bool fh = fhist_ready_for(a);
  if (fh) {
    for (int j = 0; j < 3; ++j) mg.hist[j] = (uint32_t*)fhist_[j].ptr;
    mg.hist_rot = fhist_rot_ % 3;
    mg.hist_bins = cfg_.L + 1;
    mg.hist_zero_words = fused_hist_words(cfg_.L + 1);
  }
  TraceRange tr("pga.generations_multi", 2);
  const uint32_t grid = binary_launch_multi(a, mg, stream);
  if (grid == 0) return false;
  rank_cnt_of_ = -1;
  fh = fh && binary_hist_written();
  for (uint32_t i = 0; i < n; ++i) {  // the bookkeeping of n plain generations
    n_best_[cur_ ^ 1] = grid;
    set_stats_ok(cur_ ^ 1, a.stats_parts != nullptr);
    if (fh) {
      const int w = (int)(fhist_rot_ % 3), z = (int)((fhist_rot_ + 1) % 3);
      ++fhist_rot_;
      fhist_of_[cur_ ^ 1] = w;
      fhist_clean_[w] = true;
      fhist_clean_[z] = true;
      if (fhist_of_[cur_] == z) fhist_of_[cur_] = -1;
    } else {
      fhist_of_[cur_ ^ 1] = -1;
    }
    qk_valid_[cur_ ^ 1] = false;
    swap();
  }
  return true;
}

bool Island::run_tiny(uint32_t n) {
  // REAL populations that fit one block: all n generations in one launch
  // (real_launch_multi); nothing to prepare between generations, so the
  // launch is exactly n run_plain generations
  if (!on_gpu() || n < 2 || cfg_.encoding != ENC_REAL || jit_ || hist_on_ || capturing_ || real_qk()) return false;
  if (cfg_.n_elite > 1 || (cfg_.selection != SEL_TOURNAMENT && cfg_.selection != SEL_RANDOM)) return false;
  GenArgs a = make_args(MODE_GEN);
  const int nx = cur_ ^ 1;
  unsigned long long* const parts[2] = {(unsigned long long*)best_[nx].ptr, (unsigned long long*)best_[cur_].ptr};
  float* const st[2] = {a.stats_parts, a.stats_parts ? (float*)stats_parts_[cur_].ptr : nullptr};
  if (!real_launch_multi(a, parts, st, n, stream)) return false;
  TraceRange tg("pga.generations_tiny", 2);
  // the kernel keeps the population in LDS between generations: only the
  // last generation's buffers (the new current parity) are written
  for (uint32_t i = 0; i < n; ++i) swap();
  // the previous parity's rows / scores / partials were never written (its
  // generations lived in LDS): no valid partials there until a kernel writes them
  n_best_[cur_] = 1;
  n_best_[cur_ ^ 1] = 0;
  set_stats_ok(cur_, a.stats_parts != nullptr);
  set_stats_ok(cur_ ^ 1, false);
  qk_valid_[0] = qk_valid_[1] = false;
  return true;
}

void Island::run_plain(uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    TraceRange tg("pga.generation", 2);
    prepare_generation();
    GenArgs a = make_args(MODE_GEN);
    if (jit_ && fused_jit_generation(a)) {  // the objective linked into the generation kernel
      rank_cnt_of_ = -1;
      swap();
      if (hist_on_ && !hist_manual_ && !capturing_) append_history();
      continue;
    }
    bool fh = fhist_ready_for(a);
    if (fh) {  // this generation may also write the value histogram of its keys (GenArgs::key_hist)
      a.key_hist = (uint32_t*)fhist_[fhist_rot_ % 3].ptr;
      a.hist_zero = (uint32_t*)fhist_[(fhist_rot_ + 1) % 3].ptr;
      a.hist_bins = cfg_.L + 1;
      a.hist_zero_words = fused_hist_words(cfg_.L + 1);
    }
    a.rank_counts = rank_counts_for_gen();
    if (a.rank_counts) a.hist_bins = cfg_.L + 1;
    n_best_[cur_ ^ 1] = launch(MODE_GEN, a, (unsigned long long*)best_[cur_ ^ 1].ptr);
    set_stats_ok(cur_ ^ 1, a.stats_parts != nullptr);
    if (a.stats_parts && cfg_.encoding == ENC_BINARY && on_gpu() && binary_tp_partition().grid == n_best_[cur_ ^ 1])
      stats_part_[cur_ ^ 1] = binary_tp_partition();  // (the roulette prefix's carries, roulette_fused_launch)
    rank_cnt_of_ = a.rank_counts && binary_rank_counts_written() ? (cur_ ^ 1) : -1;
    // valid only when the launcher reports that its kernel took the histogram
    // (binary_gs.hip go_tp), not on the conditions predicted above
    fh = fh && binary_hist_written();
    if (fh) {
      const int w = (int)(fhist_rot_ % 3), z = (int)((fhist_rot_ + 1) % 3);
      ++fhist_rot_;
      fhist_of_[cur_ ^ 1] = w;
      fhist_clean_[w] = true;   // zeroed (bins and status) by the launch before this one
      fhist_clean_[z] = true;   // zeroed by this launch
      if (fhist_of_[cur_] == z) fhist_of_[cur_] = -1;
    } else {
      fhist_of_[cur_ ^ 1] = -1;
    }
    qk_valid_[cur_ ^ 1] = a.qk != nullptr && !jit_;  // every REAL GEN kernel writes the keys it is given
    if (jit_) {
      n_best_[cur_ ^ 1] = jit_eval(rows_[cur_ ^ 1].ptr, (float*)scores_[cur_ ^ 1].ptr, cfg_.S,
                                   (unsigned long long*)best_[cur_ ^ 1].ptr);
      set_stats_ok(cur_ ^ 1, false);
    }
    swap();
    if (hist_on_ && !hist_manual_ && !capturing_) append_history();
  }
}

bool Island::run_batched(const std::vector<Island*>& isls, uint32_t n, hipStream_t s) {
  const size_t N = isls.size();
  if (N < 2 || !isls[0]) return false;
  const Island* i0 = isls[0];
  const bool bin = i0->cfg_.encoding == ENC_BINARY, real = i0->cfg_.encoding == ENC_REAL;
  const bool perm = i0->cfg_.encoding == ENC_PERMUTATION;
  if ((!bin && !real && !perm) || N > (bin ? binary_max_batch() : real ? real_max_batch() : perm_max_batch()))
    return false;
  for (const Island* i : isls) {
    if (!i || !i->on_gpu() || i->device_ != i0->device_ || i->cfg_.encoding != i0->cfg_.encoding || i->jit_ ||
        i->user_fn_ || i->user_xo_fn_ || i->user_mut_fn_ || i->hist_on_ || i->cfg_.S != i0->cfg_.S || i->cfg_.L != i0->cfg_.L)
      return false;
    for (const Island* j : isls)
      if (j != i && j->rows_[0].ptr == i->rows_[0].ptr) return false;  // the same island twice
  }
  {  // the batched kernels' conditions from the configuration alone, before
     // any launch (an island that cannot qualify pays no extra prepare pass)
    const Config& c = i0->cfg_;
    const bool sel_ok = (c.selection == SEL_TOURNAMENT && c.tour_k == 2) || c.selection == SEL_RANDOM ||
                        c.selection == SEL_RANK || c.selection == SEL_ROULETTE;
    const bool o32 = (c.S + kRowPad) * (uint64_t)i0->row_words_ * 4u <= 0xFFFFFFFFull;
    if (perm) {  // perm_gen_fast: every selection; the TSP objectives, one chunk per lane
      if (c.objective != OBJ_TSP && c.objective != OBJ_TSP_OPEN && c.objective != OBJ_TSP_EUC) return false;
      if (i0->chunks_ > 64 || force_generic_kernels()) return false;
      for (const Island* i : isls)
        if (i->cfg_.objective != c.objective) return false;
    } else if (!sel_ok || !o32 || i0->chunks_ > 64 || c.n_elite > 64 || force_generic_kernels()) {
      return false;
    } else if (bin) {
      if (c.objective != OBJ_ONEMAX && c.objective != OBJ_LEADING_ONES && c.objective != OBJ_TRAP) return false;
      for (const Island* i : isls)
        if (!integer_objective(i->cfg_.objective, i->cfg_.L) || !i->keys_[0].ptr || i->cfg_.objective != c.objective)
          return false;
    } else {
      const bool obj_ok = c.objective == OBJ_SPHERE || c.objective == OBJ_RASTRIGIN || c.objective == OBJ_ROSENBROCK ||
                          c.objective == OBJ_ACKLEY || c.objective == OBJ_GRIEWANK || c.objective == OBJ_SCHWEFEL ||
                          c.objective == OBJ_LINEAR || c.objective == OBJ_KNAPSACK_REAL;
      if (!obj_ok || (c.obj_i & 2) || c.S * N < real_tp_min_population()) return false;
      for (const Island* i : isls)
        if (i->cfg_.objective != c.objective || i->cfg_.obj_i != c.obj_i) return false;
    }
  }
  TraceRange tr("pga.run_batched");
  // REAL: the batch takes the two-phase kernel, which tournaments on the
  // quantized keys, so every island keeps them for the batch's population
  for (Island* I : isls) I->batch_n_ = (uint32_t)N;
  struct Reset {
    const std::vector<Island*>& v;
    ~Reset() {
      for (Island* I : v) I->batch_n_ = 1;
    }
  } reset{isls};
  std::vector<GenArgs> args(N);
  std::vector<unsigned long long*> parts(N);
  for (uint32_t g = 0; g < n; ++g) {
    for (size_t k = 0; k < N; ++k) {
      Island& I = *isls[k];
      I.stream = s;
      I.prepare_generation();
      args[k] = I.make_args(MODE_GEN);
      parts[k] = (unsigned long long*)I.best_[I.cur_ ^ 1].ptr;
    }
    const uint32_t grid = bin    ? binary_launch_batch(args.data(), parts.data(), (uint32_t)N, s)
                          : real ? real_launch_batch(args.data(), parts.data(), (uint32_t)N, s)
                                 : perm_launch_batch(args.data(), parts.data(), (uint32_t)N, s);
    if (grid == 0) {
      if (g == 0) return false;  // not eligible (decided on the first generation's arguments)
      throw std::logic_error("batched islands stopped qualifying mid-run");
    }
    for (size_t k = 0; k < N; ++k) {
      Island& I = *isls[k];
      const int nx = I.cur_ ^ 1;
      I.n_best_[nx] = grid;
      I.set_stats_ok(nx, args[k].stats_parts != nullptr);
      I.qk_valid_[nx] = real && args[k].qk != nullptr;  // the REAL kernel writes the keys it is given
      I.fhist_of_[nx] = -1;  // the batched launch produces no fused histogram
      I.rank_cnt_of_ = -1;
      I.swap();
    }
  }
  return true;
}

uint32_t Island::run_until(uint32_t n, float target, uint32_t check_every) {
  TraceRange tr("pga.run_until");
  if (check_every == 0) check_every = 10;
  uint32_t done = 0;
  while (done < n) {
    const uint32_t k = std::min(check_every, n - done);
    run(k);
    done += k;
    if (best_score() >= target) break;  // one sync per check
  }
  return done;
}

bool Island::fused_stats() const {
  // JIT objectives and the QUBO evaluation pass store best partials only
  return on_gpu() && !jit_ && cfg_.objective != OBJ_QUBO && cfg_.objective != OBJ_NONE;
}

void Island::set_stats_history(bool on) {
  hist_on_ = on;
  if (!on) return;  // off keeps the rows so far
  hist_n_ = 0;
  hist_host_.clear();
}

void Island::append_history() {
  if (!on_gpu()) {
    float r[4];
    cpu::score_stats((const float*)scores_[cur_].ptr, cfg_.S, r);
    hist_host_.insert(hist_host_.end(), r, r + 4);
    ++hist_n_;
    return;
  }
  if (hist_.bytes < 16ull * (hist_n_ + 1)) {  // grow (rare): keep the rows so far
    const uint64_t cap = std::max<uint64_t>(1024, 2 * (hist_n_ + 1));
    Buffer nb = alloc(16ull * cap);
    if (hist_n_) PGA_HIP_CHECK(hipMemcpyAsync(nb.ptr, hist_.ptr, 16ull * hist_n_, hipMemcpyDeviceToDevice, stream));
    synchronize();
    release(hist_);
    hist_ = nb;
  }
  float* row = (float*)hist_.ptr + 4 * hist_n_;
  if (stats_ok_[cur_]) {
    stats_from_parts_launch((const float*)stats_parts_[cur_].ptr, (const unsigned long long*)best_[cur_].ptr,
                            n_best_[cur_], cfg_.S, row, stream);
  } else {
    score_stats_launch((const float*)scores_[cur_].ptr, cfg_.S, (float*)stats_.ptr, stream);
    PGA_HIP_CHECK(hipMemcpyAsync(row, stats_.ptr, 16, hipMemcpyDeviceToDevice, stream));
  }
  ++hist_n_;
}

std::vector<float> Island::history() {
  if (!on_gpu()) return hist_host_;
  std::vector<float> out(4 * hist_n_);
  if (hist_n_) copy_to_host(out.data(), hist_.ptr, 16ull * hist_n_);
  return out;
}

void Island::crossover_stage() {
  TraceRange tr("pga.crossover");
  prepare_generation();
  GenArgs a = make_args(MODE_CROSS);
  launch(MODE_CROSS, a, nullptr);
}

void Island::mutate_stage() {
  TraceRange tr("pga.mutate");
  GenArgs a = make_args(MODE_MUTATE);
  launch(MODE_MUTATE, a, nullptr);
}

void Island::swap() {
  cur_ ^= 1;
  ++gen_;
}

unsigned long long Island::best_packed() {
  unsigned long long r = 0;
  if (on_gpu()) {
    reduce_best_launch((const unsigned long long*)best_[cur_].ptr, n_best_[cur_], (unsigned long long*)out_best_.ptr,
                       stream);
    copy_to_host(&r, out_best_.ptr, 8);
  } else {
    r = cpu::reduce_best((const unsigned long long*)best_[cur_].ptr, n_best_[cur_]);
  }
  return r;
}

void Island::stats(float out[4]) {
  const float* sc = (const float*)scores_[cur_].ptr;
  if (on_gpu() && stats_ok_[cur_]) {  // fused partials of the kernel that scored this generation
    stats_from_parts_launch((const float*)stats_parts_[cur_].ptr, (const unsigned long long*)best_[cur_].ptr,
                            n_best_[cur_], cfg_.S, (float*)stats_.ptr, stream);
    copy_to_host(out, stats_.ptr, 16);
  } else if (on_gpu()) {
    score_stats_launch(sc, cfg_.S, (float*)stats_.ptr, stream);
    copy_to_host(out, stats_.ptr, 16);
  } else {
    cpu::score_stats(sc, cfg_.S, out);
  }
}

void Island::ensure_topk_ws(uint32_t k) {
  const size_t need = topk_workspace_bytes(cfg_.S, k);
  if (topk_ws_.bytes >= need) return;
  synchronize();
  release(topk_ws_);
  topk_ws_ = alloc(need);
  PGA_HIP_CHECK(hipMemsetAsync(topk_ws_.ptr, 0, need, stream));  // the value histogram must start zeroed
}

void Island::topk(uint32_t k, bool largest, uint32_t* idx_out, bool sorted) {
  TraceRange tr(largest ? "pga.topk" : "pga.bottomk");
  if (k > cfg_.S) throw std::invalid_argument("k exceeds population size");
  const float* sc = (const float*)scores_[cur_].ptr;
  if (on_gpu()) {
    ensure_topk_ws(k);
    const uint16_t* k16 = integer_objective(cfg_.objective, cfg_.L) ? (const uint16_t*)keys_[cur_].ptr : nullptr;
    TopkFused f;
    topk_launch(sc, k16, cfg_.L + 1, cfg_.S, k, largest, sorted, idx_out, topk_ws_.ptr, stream, nullptr,
                sorted || !k16 ? nullptr : fused_select(f));
  } else {
    cpu::topk(sc, cfg_.S, k, largest, idx_out, sorted);
  }
}

std::vector<uint32_t> Island::topk_host(uint32_t k, bool largest) {
  std::vector<uint32_t> out(k);
  if (k == 0) return out;
  if (on_gpu()) {
    uint32_t* d = (uint32_t*)scratch(4ull * k);
    topk(k, largest, d);
    copy_to_host(out.data(), d, 4ull * k);
  } else {
    topk(k, largest, out.data());
  }
  return out;
}

std::vector<uint32_t> Island::row_host(uint64_t i) {
  if (i >= cfg_.S) throw std::out_of_range("individual index out of range");
  std::vector<uint32_t> out(row_words_);
  copy_to_host(out.data(), (const uint32_t*)rows_[cur_].ptr + i * row_words_, 4ull * row_words_);
  return out;
}

void Island::gather(const uint32_t* idx, uint32_t n, void* out_rows, float* out_scores) {
  TraceRange tr("pga.migrate.gather");
  if (on_gpu())
    gather_rows_launch(rows_[cur_].ptr, (const float*)scores_[cur_].ptr, row_words_, idx, n, out_rows, out_scores,
                       stream);
  else
    cpu::gather_rows(rows_[cur_].ptr, (const float*)scores_[cur_].ptr, row_words_, idx, n, out_rows, out_scores);
}

void Island::scatter(const uint32_t* idx, uint32_t n, const void* in_rows, const float* in_scores) {
  TraceRange tr("pga.migrate.scatter");
  if (on_gpu())
    scatter_rows_launch(rows_[cur_].ptr, (float*)scores_[cur_].ptr, row_words_, idx, n, in_rows, in_scores, stream);
  else
    cpu::scatter_rows(rows_[cur_].ptr, (float*)scores_[cur_].ptr, row_words_, idx, n, in_rows, in_scores);
  rebest();  // best partials and tournament keys follow the new scores
}

void Island::set_migration_policy(int p) {
  if (p != MIG_TOPK && p != MIG_STRIPE) throw std::invalid_argument("migration policy must be MIG_TOPK or MIG_STRIPE");
  mig_policy_ = p;
}

void Island::emigrate(uint32_t k, void* out_rows, float* out_scores) {
  TraceRange tr("pga.migrate.emigrate");
  if (k == 0) return;
  if (k > cfg_.S) throw std::invalid_argument("k exceeds population size");
  if (mig_policy_ == MIG_STRIPE) {
    if (on_gpu())
      stripe_emigrate_launch((const float*)scores_[cur_].ptr, rows_[cur_].ptr, row_words_, cfg_.S, k, out_rows,
                             out_scores, stream);
    else
      cpu::stripe_emigrate((const float*)scores_[cur_].ptr, rows_[cur_].ptr, row_words_, cfg_.S, k, out_rows,
                           out_scores);
    return;
  }
  const uint16_t* k16 = integer_objective(cfg_.objective, cfg_.L) ? (const uint16_t*)keys_[cur_].ptr : nullptr;
  if (on_gpu() && topk_move_supported(k16, cfg_.L + 1, cfg_.S)) {
    ensure_topk_ws(k);
    TopkMove mv;
    mv.mode = TopkMove::GATHER;
    mv.rw16 = row_words_ / 4;
    mv.src_rows = (const uint4*)rows_[cur_].ptr;
    mv.src_scores = (const float*)scores_[cur_].ptr;
    mv.dst_rows = (uint4*)out_rows;
    mv.dst_scores = out_scores;
    TopkFused f;
    topk_launch((const float*)scores_[cur_].ptr, k16, cfg_.L + 1, cfg_.S, k, true, false, nullptr, topk_ws_.ptr, stream,
                &mv, fused_select(f));
    return;
  }
  uint32_t* idx = (uint32_t*)scratch(4ull * k);
  topk(k, true, idx, false);
  gather(idx, k, out_rows, out_scores);
}

void Island::immigrate(uint32_t k, const void* in_rows, const float* in_scores) {
  TraceRange tr("pga.migrate.immigrate");
  if (k == 0) return;
  TopkFused f;
  const TopkFused* fsel = fused_select(f);  // the victims' selection, before the keys change
  invalidate_qk();
  if (k > cfg_.S) throw std::invalid_argument("k exceeds population size");
  uint16_t* k16 = integer_objective(cfg_.objective, cfg_.L) ? (uint16_t*)keys_[cur_].ptr : nullptr;
  if (mig_policy_ == MIG_STRIPE) {
    if (on_gpu()) {
      // victims, their keys, and the island's best partials + statistics in one pass
      float* sp = fused_stats() ? (float*)stats_parts_[cur_].ptr : nullptr;
      n_best_[cur_] = stripe_immigrate_launch((float*)scores_[cur_].ptr, k16, rows_[cur_].ptr, row_words_, cfg_.S, k,
                                              in_rows, in_scores, (unsigned long long*)best_[cur_].ptr, sp, stream);
      set_stats_ok(cur_, sp != nullptr);
    } else {
      cpu::stripe_immigrate((float*)scores_[cur_].ptr, rows_[cur_].ptr, row_words_, cfg_.S, k, in_rows, in_scores);
      rebest();
    }
    return;
  }
  if (on_gpu() && topk_move_supported(k16, cfg_.L + 1, cfg_.S)) {
    ensure_topk_ws(k);
    TopkMove mv;
    mv.mode = TopkMove::SCATTER;
    mv.rw16 = row_words_ / 4;
    mv.src_rows = (const uint4*)in_rows;
    mv.src_scores = in_scores;
    mv.dst_rows = (uint4*)rows_[cur_].ptr;
    mv.dst_scores = (float*)scores_[cur_].ptr;
    mv.dst_keys = k16;
    mv.best_parts = (unsigned long long*)best_[cur_].ptr;  // the new per-block bests, from the selection itself
    const uint32_t nb = topk_launch((const float*)scores_[cur_].ptr, k16, cfg_.L + 1, cfg_.S, k, false, false,
                                    nullptr, topk_ws_.ptr, stream, &mv, fsel);
    // the victims' keys were written with their rows; the best partials came
    // with the selection (else one pass over the scores)
    n_best_[cur_] = nb ? nb
                       : best_of_scores_launch((const float*)scores_[cur_].ptr, cfg_.S,
                                               (unsigned long long*)best_[cur_].ptr, stream, nullptr);
    set_stats_ok(cur_, false);
    return;
  }
  uint32_t* idx = (uint32_t*)scratch(4ull * k);
  topk(k, false, idx, false);
  scatter(idx, k, in_rows, in_scores);
}

void Island::set_fused_histogram(bool on) {
  fhist_user_ = on;
  fhist_on_ = on || cfg_.n_elite > 1;
}

bool Island::roul_packed() const {
  // PGA_ROUL_PACKED=1: the GEN kernel reads one packed {guide, cumfit} table.
  // Off by default: measured much slower (167.7 vs 130.1 us/gen, OneMax-1024
  // roulette; profiles/roulette_r06.md): the guide lookups' lines then hold
  // 16 buckets instead of 32, and the pick's working set doubles
  static const bool on = [] {
    const char* e = std::getenv("PGA_ROUL_PACKED");
    return e && e[0] == '1';
  }();
  return on && cfg_.S < (1ull << 28);
}

bool Island::roul_fused_off() {
  static const bool off = [] {
    const char* e = std::getenv("PGA_ROUL_FUSED");
    return e && e[0] == '0';
  }();
  return off;
}

uint32_t* Island::rank_counts_for_gen() const {
  // the launcher (binary_gs.hip go_tp) takes them only at the sort's tile geometry
  if (cfg_.selection != SEL_RANK || !on_gpu() || capturing_ || jit_ || cfg_.encoding != ENC_BINARY) return nullptr;
  if (!integer_objective(cfg_.objective, cfg_.L) || cfg_.objective == OBJ_KNAPSACK || !keys_[0].ptr) return nullptr;
  if (cfg_.L + 1 > kHistMaxBins || !rank_ws_.ptr) return nullptr;
  static const bool off = [] {  // PGA_RANK_FUSED=0: the sort counts its keys itself (A/B knob)
    const char* e = std::getenv("PGA_RANK_FUSED");
    return e && e[0] == '0';
  }();
  if (off) return nullptr;
  return rank_order16_counts(rank_ws_.ptr, cfg_.S, cfg_.L + 1);
}

bool Island::fhist_ready_for(const GenArgs& a) const {
  // the conditions under which binary_gen_tp runs with u16 keys (binary_gs.hip
  // launch_mode), so the launch really produces the histogram
  if (!fhist_on_ || !on_gpu() || capturing_ || jit_ || cfg_.encoding != ENC_BINARY) return false;
  if (!integer_objective(cfg_.objective, cfg_.L) || cfg_.L + 1 > kHistMaxBins || a.key_cur == nullptr) return false;
  if (cfg_.objective == OBJ_KNAPSACK) return false;
  uint32_t gs = 0;
  bool full = false, dense = false;
  if (!binary_tp_plan(a, gs, full, dense)) return false;
  if (!fhist_[0].ptr) {  // allocated zeroed on first use
    Island* self = const_cast<Island*>(this);
    for (auto& b : self->fhist_) {
      b = self->alloc(4ull * fused_hist_words(cfg_.L + 1));
      PGA_HIP_CHECK(hipMemsetAsync(b.ptr, 0, b.bytes, stream));
    }
  }
  return true;
}

const TopkFused* Island::fused_select(TopkFused& f) {
  const int b = on_gpu() ? fhist_of_[cur_] : -1;
  if (b < 0) return nullptr;
  f.hist = (const uint32_t*)fhist_[b].ptr;
  f.status = (uint32_t*)fhist_[b].ptr + (cfg_.L + 1 + 3) / 4 * 4;
  if (!fhist_clean_[b])  // a selection on this population already used its status words
    PGA_HIP_CHECK(hipMemsetAsync(f.status, 0, 4ull * kTopkStatusWords, stream));
  fhist_clean_[b] = false;
  return &f;
}

bool Island::evaluate_rows(void* rows, float* scores, uint32_t n) {
  if (cfg_.objective == OBJ_NONE && !jit_) return false;
  if (n == 0) return true;
  TraceRange tr("pga.migrate.evaluate");
  if (!ev_parts_.ptr) ev_parts_ = alloc(8ull * kMaxGrid);
  if (jit_) {
    jit_eval(rows, scores, n, (unsigned long long*)ev_parts_.ptr);
    return true;
  }
  GenArgs a = make_args(MODE_EVAL);
  a.cur = rows;
  a.next = rows;
  a.score_cur = scores;
  a.score_next = scores;
  a.S = n;
  a.key_cur = nullptr;
  a.key_next = nullptr;
  a.stats_parts = nullptr;  // the island's own statistics are not these rows'
  a.n_elite = 0;
  a.elite_idx = nullptr;
  launch(MODE_EVAL, a, (unsigned long long*)ev_parts_.ptr);
  return true;
}

// ----------------------------------------------------------------- JIT ---
void Island::set_jit_objective(std::shared_ptr<JitKernel> k) {
  if (k) {
    if (!on_gpu()) throw std::invalid_argument("JIT objectives need the GPU backend");
    if (cfg_.objective != OBJ_NONE) throw std::invalid_argument("a JIT objective needs objective OBJ_NONE");
    if (k->encoding != cfg_.encoding) throw std::invalid_argument("JIT objective compiled for another encoding");
    k->function(device_);  // load the module now: errors surface here, not mid-run
  }
  jit_ = std::move(k);
  jit_fused_off_ = false;
  invalidate();
}

bool Island::fused_jit_generation(GenArgs& a) {
  if (!on_gpu() || (cfg_.encoding != ENC_BINARY && cfg_.encoding != ENC_REAL) || jit_fused_off_) return false;
  uint32_t gs = 0;
  bool full = false, dense = false;
  if (cfg_.encoding == ENC_REAL ? !real_tp_plan(a, gs) : !binary_tp_plan(a, gs, full, dense)) return false;
  // no compile / module load inside a graph capture: there only a variant
  // loaded by an earlier plain generation is used
  hipFunction_t f = jit_->gen_function(device_, gs, full, dense, cfg_.L, !capturing_);
  if (!f) {
    if (!capturing_) jit_fused_off_ = true;  // fall back to generation + evaluation pass (fused_error() says why)
    return false;
  }
  TraceRange tr("pga.jit_generation", 2);
  const int nx = cur_ ^ 1;
  a.stats_parts = (float*)stats_parts_[nx].ptr;  // the fused kernel stores {min, sum} partials like the built-ins
  n_best_[nx] = jit_->gen_launch(f, &a, sizeof(a), cfg_.S, (unsigned long long*)best_[nx].ptr, kMaxGrid, stream);
  set_stats_ok(nx, a.stats_parts != nullptr);
  qk_valid_[nx] = false;
  ++jit_fused_gens_;
  return true;
}

uint32_t Island::jit_eval(const void* rows, float* scores, uint64_t n, unsigned long long* parts) {
  TraceRange tr("pga.jit_eval", 2);
  return jit_->eval(device_, rows, row_words_, n, cfg_.L, (const float*)obj_data_[0].ptr, scores, parts, kMaxGrid,
                    stream);
}

// ------------------------------------------------------------ hipGraph ---
void Island::set_graph_generations(uint32_t g) {
  if (g % 2) ++g;  // even: the graph must end on the parity it started from
  graph_g_ = g;
  drop_graph();
}

void Island::drop_graph() {
  if (gexec_) (void)hipGraphExecDestroy(gexec_);
  gexec_ = nullptr;
  g_cur_ = -1;
}

bool Island::capture_graph() {
  drop_graph();
  if (!gen_dev_.ptr) gen_dev_ = alloc(64);
  if (!cap_stream_) PGA_HIP_CHECK(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking));
  // workspaces that a stage would otherwise (re)allocate synchronously
  if (cfg_.n_elite > 1) {
    ensure_topk_ws(cfg_.n_elite);
  }
  const int cur0 = cur_;
  const uint32_t gen0 = gen_, nb0 = n_best_[cur_];
  hipStream_t user = stream;
  stream = cap_stream_;
  capturing_ = true;
  capture_base_ = gen_;
  hipGraph_t graph = nullptr;
  bool ok = hipStreamBeginCapture(cap_stream_, hipStreamCaptureModeThreadLocal) == hipSuccess;
  if (ok) {
    try {
      run_plain(graph_g_);
      advance_counter_launch((uint32_t*)gen_dev_.ptr, graph_g_, cap_stream_);
    } catch (...) {
      ok = false;
    }
    ok = (hipStreamEndCapture(cap_stream_, &graph) == hipSuccess) && ok && graph;
  }
  capturing_ = false;
  stream = user;
  gen_ = gen0;  // the captured launches ran nothing: restore the host view
  if (cur_ != cur0) cur_ = cur0;
  if (ok) ok = hipGraphInstantiate(&gexec_, graph, nullptr, nullptr, 0) == hipSuccess;
  if (graph) (void)hipGraphDestroy(graph);
  if (!ok) {
    (void)hipGetLastError();
    gexec_ = nullptr;
    graph_broken_ = true;  // fall back to plain launches for good
    return false;
  }
  g_cur_ = cur0;
  g_epoch_ = epoch_;
  g_version_ = version_;
  g_nbest_ = nb0;
  g_len_ = graph_g_;
  return true;
}

bool Island::run_graph(uint32_t reps, bool fresh) {
  if (!fresh && !capture_graph()) return false;
  PGA_HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)gen_dev_.ptr, (int)gen_, 1, stream));
  for (uint32_t r = 0; r < reps; ++r) PGA_HIP_CHECK(hipGraphLaunch(gexec_, stream));
  gen_ += reps * graph_g_;
  graph_replays_ += reps;
  return true;
}

// ------------------------------------------------------------ checkpoint ---
namespace {
struct CkptHeader {
  char magic[8];  // "PGACKPT1"
  uint32_t version, encoding, L, row_words;
  uint64_t S;
  uint32_t gen, epoch, island, pad;
  uint64_t seed;
};
}  // namespace

void Island::save(const std::string& path) {
  TraceRange tr("pga.checkpoint.save");
  CkptHeader h;
  std::memset(&h, 0, sizeof(h));
  std::memcpy(h.magic, "PGACKPT1", 8);
  h.version = 1;
  h.encoding = (uint32_t)cfg_.encoding;
  h.L = cfg_.L;
  h.row_words = row_words_;
  h.S = cfg_.S;
  h.gen = gen_;
  h.epoch = epoch_;
  h.island = cfg_.island;
  h.seed = cfg_.seed;
  std::vector<char> rows(4ull * row_words_ * cfg_.S);
  std::vector<float> sc(cfg_.S);
  copy_to_host(rows.data(), rows_[cur_].ptr, rows.size());
  copy_to_host(sc.data(), scores_[cur_].ptr, 4ull * cfg_.S);
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot open checkpoint for writing: " + path);
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1 && std::fwrite(rows.data(), 1, rows.size(), f) == rows.size() &&
            std::fwrite(sc.data(), 4, cfg_.S, f) == cfg_.S;
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error("short write to checkpoint: " + path);
}

void Island::load(const std::string& path) {
  TraceRange tr("pga.checkpoint.load");
  invalidate();
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open checkpoint: " + path);
  CkptHeader h;
  if (std::fread(&h, sizeof(h), 1, f) != 1 || std::memcmp(h.magic, "PGACKPT1", 8) != 0) {
    std::fclose(f);
    throw std::runtime_error("not a pga checkpoint: " + path);
  }
  if (h.S != cfg_.S || h.L != cfg_.L || h.encoding != (uint32_t)cfg_.encoding || h.row_words != row_words_) {
    std::fclose(f);
    throw std::runtime_error("checkpoint geometry does not match this population");
  }
  std::vector<char> rows(4ull * row_words_ * cfg_.S);
  std::vector<float> sc(cfg_.S);
  bool ok = std::fread(rows.data(), 1, rows.size(), f) == rows.size() && std::fread(sc.data(), 4, cfg_.S, f) == cfg_.S;
  std::fclose(f);
  if (!ok) throw std::runtime_error("truncated checkpoint: " + path);
  copy_to_device(rows_[cur_].ptr, rows.data(), rows.size());
  copy_to_device(scores_[cur_].ptr, sc.data(), 4ull * cfg_.S);
  gen_ = h.gen;
  epoch_ = h.epoch;
  cfg_.seed = h.seed;
  cfg_.island = h.island;
  rebest();
}

}  // namespace pga
