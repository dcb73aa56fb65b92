// ops.hpp — host-side launcher API of the engine's device operators.
//
// Every operator takes raw device pointers and a HIP stream, allocates
// nothing and never synchronises, so callers can capture sequences of them
// into a hipGraph.  The same entry points back the C API runtime
// (csrc/capi) and the torch bindings (csrc/python); the CPU reference
// backend (csrc/cpu) implements identical semantics on host memory.
#pragma once

#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "pga/core.hpp"

#define PGA_HIP_CHECK(expr)                                                                  \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                   \
  } while (0)

namespace pga {

// Max blocks of a persistent grid-stride launch; per-block best arrays must
// hold at least this many entries.
constexpr uint32_t kMaxGrid = 8192;
// Population buffers (rows, scores, tournament keys) carry kRowPad spare
// entries past S: the fast BINARY kernel's last wave writes its tail there
// instead of predicating its stores.
constexpr uint32_t kRowPad = 64;

// grid for `S` work items processed `per_block` at a time: min(ceil, 8*CUs)
uint32_t launch_grid(uint64_t S, uint32_t per_block);
// same, capped at the kernel's resident blocks per CU (hipOccupancy...) so a
// persistent grid-stride launch never leaves a partial second wave
uint32_t launch_grid_occ(uint64_t S, uint32_t per_block, const void* kernel);
uint32_t occupancy_blocks(const void* kernel, int block, size_t dyn_lds = 0);
// Launch geometry of the two-phase kernels (binary_gen_tp, tp.hpp
// tp_block_range): one 16-wave block per CU of an island's share of the
// device when every wave breeds at least one 64-child unit, else 4-wave
// blocks on an occupancy-sized grid with breed units of `unit` children (a
// power of two >= ng = children per step) small enough to reach every
// resident wave; `lds` = the dynamic LDS bytes.  Launchers store `unit` in
// GenArgs::tp_unit.
struct TpGeom {
  uint32_t grid, block, lds, unit;
};
TpGeom tp_geometry(uint64_t S, uint32_t islands, const void* kernel, uint32_t ng, uint32_t pseg = 7);
// the same from the resident 4-wave blocks per CU (occ4; module kernels)
TpGeom tp_geometry_occ(uint64_t S, uint32_t islands, uint32_t occ4, uint32_t ng, uint32_t pseg = 7);
uint32_t tp_dyn_lds_bytes(uint32_t nw, uint32_t pseg = 7);
// LDS a fused BINARY JIT launch adds for its staged children (tp.hpp kJitStageSteps)
uint32_t tp_jit_stage_bytes(uint32_t nw);
// units per block in binary_gen_tp's pair pool for this geometry (tp.hpp;
// PGA_TP_POOL=d: 1/d of a 16-wave block's units; default 0: off)
uint32_t tp_pool_units(const TpGeom& t, uint64_t S);
// share skew for this geometry (tp.hpp tp_share; PGA_TP_SKEW units, default 2)
uint32_t tp_skew_units(const TpGeom& t, uint64_t S);
// bytes of pair-pool counters a launch of up to `grid` blocks needs
inline size_t tp_pool_bytes(uint32_t grid) { return (size_t)(grid + 1) / 2 * 128; }
int device_cu_count();
// raise a kernel's dynamic-LDS limit to what its static LDS leaves of the
// CU's 160 KiB on the current device (once per kernel and device; cheap to
// call per launch); returns that many bytes
size_t allow_dynamic_lds(const void* kernel);
// PGA_FORCE_GENERIC=1: every encoding runs its generic (non-pipelined) GEN
// kernel.  Verification / debugging only: the fast kernels are bit-identical.
bool force_generic_kernels();

// ---- encodings: one launch per call, returns the grid used (= number of
// valid entries written to best_parts, when the mode evaluates) ----
uint32_t binary_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s);
// binary_launch for one group size GS (binary_gs.hip, one translation unit per GS)
template <int GS>
uint32_t binary_launch_group(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s);
// Persistent multi-generation launch of the headline kernel
// (binary_dev.hpp binary_gen_tp_multi): `gens` generations from `a`
// (generation 0), generation i writing best / stats partials parts[i & 1] /
// stats[i & 1]; barrier: 4 device bytes (zeroed by the launch).  Returns the
// grid (every generation's partial count) or 0 when the arguments do not
// qualify (nothing launched: run plain launches).
struct MultiGenArgs {
  unsigned long long* parts[2];
  float* stats[2];
  uint32_t gens;
  uint32_t* barrier;
  // fused key histogram (GenArgs::key_hist) rotation: generation i writes
  // hist[(rot + i) % 3] and zeroes hist[(rot + i + 1) % 3] (hist[0] nullptr: off)
  uint32_t* hist[3] = {nullptr, nullptr, nullptr};
  uint32_t hist_rot = 0, hist_bins = 0, hist_zero_words = 0;
};
uint32_t binary_launch_multi(const GenArgs& a, const MultiGenArgs& mg, hipStream_t s);
template <int GS>
uint32_t binary_launch_multi_group(const GenArgs& a, const MultiGenArgs& mg, hipStream_t s);
// whether the last binary_launch on this host thread handed GenArgs::key_hist
// to its kernel (so the fused key histogram was written and hist_zero
// cleared); the island marks a histogram valid only on this report
bool& binary_hist_written();
// the same report for GenArgs::rank_counts (the next rank sort's tile counts)
bool& binary_rank_counts_written();
// the block partition of the last binary_gen_tp launch on this host thread
// (grid 0: the launch took another kernel): block j wrote children
// tp_share(S, unit, j, skew) and stored their {min, sum} partials at
// stats_parts[2 j] (no pair pool)
struct TpPartition {
  uint32_t grid, unit, skew;
};
TpPartition& binary_tp_partition();
// whether a MODE_GEN launch of these arguments takes the hot two-phase kernel
// (binary_gen_tp) and which variant: group size, full groups, dense mutation.
// For f32-score objectives (the fused JIT generation kernel, jit.hpp).
bool binary_tp_plan(const GenArgs& a, uint32_t& gs, bool& full, bool& dense);
// the same for REAL (real_gen_tp, no rotation): its group size
bool real_tp_plan(const GenArgs& a, uint32_t& gs);
// smallest REAL population that takes real_gen_tp (PGA_TP_MIN_S overrides)
uint64_t real_tp_min_population();
// REAL batched islands (real_batch.hip): whether an island qualifies as one
// of n, and one MODE_GEN launch of up to real_max_batch() same-shape islands
// (returns each island's grid; 0 = not launched, run them one by one)
bool real_tp_batchable(const GenArgs& a, uint32_t n);
uint32_t real_max_batch();
uint32_t real_launch_batch(const GenArgs* args, unsigned long long* const* parts, uint32_t n, hipStream_t s);
// PERMUTATION batched islands (perm.hip perm_gen_fast_batch): TSP objectives,
// genomes of at most 512 cities
uint32_t perm_max_batch();
uint32_t perm_launch_batch(const GenArgs* args, unsigned long long* const* parts, uint32_t n, hipStream_t s);
// batched islands (binary_batch.hip): one MODE_GEN launch of up to
// binary_max_batch() same-shape islands (args[i], best partials parts[i]);
// returns each island's grid (its best-partials count), 0 when the islands do
// not qualify (nothing launched: run them one by one)
uint32_t binary_max_batch();
uint32_t binary_launch_batch(const GenArgs* args, unsigned long long* const* parts, uint32_t n, hipStream_t s);
// Knapsack digit table for the matrix-core evaluation (binary.hip): false
// (table empty) when the instance does not qualify -- non-integer values or
// weights, sums of magnitudes >= 2^24, fewer than 4 lanes per individual, or
// more than 16 digit columns
bool build_knap_table(const float* values, const float* weights, uint32_t L, uint32_t chunks,
                      std::vector<uint8_t>& tab, uint32_t& digits, uint32_t& cols);
uint32_t real_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s);
// REAL tiny populations (every child in one block): n >= 2 MODE_GEN
// generations in one launch (real.hip real_multi_kernel); parts / stats of
// the even and odd generations; false (nothing launched) when `a` does not
// qualify (per-generation host work: rank / roulette / top-k elites, user
// operators, rotation, quantized keys; PGA_TINY_MULTI=0 turns it off)
bool real_launch_multi(const GenArgs& a, unsigned long long* const parts[2], float* const stats[2], uint32_t n,
                       hipStream_t s);
uint32_t perm_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s);

// reference-ABI path: thread-per-individual kernel calling user device
// function pointers (crossover_f / mutate_f / obj_f), REAL encoding only
uint32_t compat_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s);

// QUBO on the int8 matrix cores (qubo.hip): genomes up to kQuboMaxBits bits
constexpr uint32_t kQuboMaxBits = 1024;
uint32_t qubo_padded_length(uint32_t L);  // 64, 128, 256, 512 or 1024
// qt: Lp x Lp int8 (Lp = qubo_padded_length(L)), Q^T of round/clamped q
void qubo_pack_launch(const float* q, uint32_t L, int8_t* qt, hipStream_t s);
// scores[i] = sign * x_i^T Q x_i for S bit rows; per-block bests -> parts; returns the grid
uint32_t qubo_eval_launch(const void* rows, uint32_t row_words, uint64_t S, uint32_t L, const int8_t* qt, float sign,
                          float* scores, unsigned long long* parts, hipStream_t s);

inline uint32_t encoding_launch(int mode, const GenArgs& a, unsigned long long* best_parts, hipStream_t s) {
  switch (a.encoding) {
    case ENC_BINARY:
      if (a.objective == OBJ_QUBO && (mode == MODE_GEN || mode == MODE_INIT || mode == MODE_EVAL)) {
        // the fused kernel writes the children, the matrix cores score them
        GenArgs b = a;
        b.objective = OBJ_NONE;
        b.key_next = nullptr;
        if (mode != MODE_EVAL) binary_launch(mode, b, best_parts, s);
        return qubo_eval_launch(a.next, a.row_words, a.S, a.L, a.qubo_qt, a.obj_f0, a.score_next, best_parts, s);
      }
      return binary_launch(mode, a, best_parts, s);
    case ENC_REAL:
      if (a.user_xo_fn || a.user_mut_fn) return compat_launch(mode, a, best_parts, s);
      return real_launch(mode, a, best_parts, s);
    default: return perm_launch(mode, a, best_parts, s);
  }
}

// ---- reductions / selection helpers (util.hip) ----
// out[0] = max over parts[0..n)
void reduce_best_launch(const unsigned long long* parts, uint32_t n, unsigned long long* out, hipStream_t s);
// per-block best over arbitrary scores (for externally evaluated populations)
uint32_t best_of_scores_launch(const float* scores, uint64_t S, unsigned long long* parts, hipStream_t s,
                               uint16_t* keys = nullptr);  // keys: also refresh u16 tournament keys
// keys[i] = (uint16)scores[i] (integer objectives' tournament keys)
void scores_to_keys_launch(const float* scores, uint64_t S, uint16_t* keys, hipStream_t s);
// keys[i] = qkey(scores[i]) over the range {min, max} = mm[0..1] (device):
// the quantized tournament keys of a float objective (core.hpp qkey)
void scores_to_qkeys_launch(const float* scores, uint64_t S, const float* mm, uint16_t* keys, hipStream_t s);
// *counter += delta (graph replay: the device-resident generation counter)
void advance_counter_launch(uint32_t* counter, uint32_t delta, hipStream_t s);
// stats[0..3] = {min, max, sum, count} of scores (count as float)
void score_stats_launch(const float* scores, uint64_t S, float* stats, hipStream_t s);
// the same 4 floats from a generation kernel's fused partials (n blocks)
void stats_from_parts_launch(const float* parts, const unsigned long long* best, uint32_t n, uint64_t S, float* out,
                             hipStream_t s);
// roulette: cumfit = inclusive prefix sum of max(score - min, 0); then the
// guide table guide[0..S] for O(1) picks (GenArgs::roul_guide).  workspace:
// roulette_workspace_floats(S); its word kRoulScale holds the bucket scale.
// The minimum comes from the generation kernel's fused {min, sum} partials
// (parts, nparts blocks) when given, else from a score pass.
constexpr uint32_t kRoulScale = 4 + 3 * 1024 + 1024;
size_t roulette_workspace_floats(uint64_t S);
// integer = true: the scores are integers (integer_objective): u64 sums, the
// exact prefix rounded once per entry
void roulette_prefix_launch(const float* scores, uint64_t S, const float* parts, uint32_t nparts, float* cumfit,
                            float* workspace, hipStream_t s, bool integer = false);
// packed: guide is the packed table of GenArgs::roul_packed (8 bytes per
// entry, S + 4 entries; S < 2^28)
void roulette_guide_launch(const float* cumfit, uint64_t S, uint32_t* guide, float* workspace, hipStream_t s,
                           bool packed = false);
// Both in ONE launch for an integer objective whose current population came
// from binary_gen_tp with partition `part`: its {min, sum} partials (parts,
// part.grid blocks) give every block its carry, so no pass precedes the scan.
// The weights and prefix sums are exact integers (cumfit[i] = the prefix
// rounded to f32 once).  max_score: the objective's largest score; returns
// false (nothing launched) when a partial sum could be inexact in f32.
bool roulette_fused_launch(const float* scores, uint64_t S, const float* parts, const TpPartition& part,
                           uint32_t max_score, float* cumfit, uint32_t* guide, float* workspace, hipStream_t s,
                           bool packed = false);
// stable LSD radix sort (sort.hip: reduce-then-scan, digits of up to 8 bits,
// count / scan / scatter launches per pass): (keys, vals) by the low `bits`
// bits of the keys, ascending, or descending (all 32 bits; equal keys keep
// their order).  vals == nullptr: the values are 0..n-1.  n < 2^32.
size_t radix_sort_workspace_bytes(uint64_t n);
void radix_sort_pairs(const uint32_t* keys, const uint32_t* vals, uint64_t n, uint32_t bits, bool descending,
                      uint32_t* keys_out, uint32_t* vals_out, void* workspace, hipStream_t s);
// rank selection: order = indices by ascending (score_key, index); workspace: rank_order_workspace_bytes(S)
size_t rank_order_workspace_bytes(uint64_t S);
void rank_order_launch(const float* scores, uint64_t S, uint32_t* order, void* workspace, hipStream_t s);
// the same order from the u16 tournament keys of an integer objective (keys
// < key_range: only their bits are sorted, 2 passes for OneMax-1024)
void rank_order16_launch(const uint16_t* keys16, uint64_t S, uint32_t key_range, uint32_t* order, void* workspace,
                         hipStream_t s, bool counts_ready = false);
// The sort's per-tile key counts (counts[key * tiles + tile], tiles of
// kRankTile keys) in the workspace, when the u16 sort of this key range is a
// single pass whose digit is the whole key; else nullptr.  A producer that
// stores exactly these counts (binary_gen_tp's GenArgs::rank_counts) lets
// the next rank_order16_launch run with counts_ready, skipping its count pass.
constexpr uint32_t kRankTile = 4096;
uint32_t* rank_order16_counts(void* workspace, uint64_t S, uint32_t key_range);
// top-k by score (descending, ties -> lower index); idx_out[k]; workspace: topk_workspace_bytes(S)
size_t topk_workspace_bytes(uint64_t S, uint32_t k);
// sorted = false: the k indices in selection order (keys above the threshold by
// index, then threshold ties by index) — cheaper, used by migration / elitism.
// keys16 (optional): the u16 tournament keys of an integer objective (2 passes)
// key_range: keys16 take values in [0, key_range) (L + 1 for the integer
// objectives); <= kTopkMaxRange enables the one-pass value histogram
constexpr uint32_t kTopkMaxRange = 8192;
// Optional fused row move of the selection (u16-key selection-order path
// only, see topk_move_supported): emigrants gathered into a send buffer, or
// immigrants scattered over the selected victims (rows, scores, keys).
struct TopkMove {
  enum Mode : int32_t { NONE = 0, GATHER = 1, SCATTER = 2 };
  int32_t mode = NONE;
  uint32_t rw16 = 0;  // row stride in 16-byte units
  const uint4* src_rows = nullptr;
  const float* src_scores = nullptr;
  uint4* dst_rows = nullptr;
  float* dst_scores = nullptr;
  uint16_t* dst_keys = nullptr;
  // SCATTER (integer objectives: key == score): when set, the selection also
  // writes the population's new per-block packed bests (one per selection
  // block, topk_launch returns their count): the best survivor of each block
  // and the immigrants placed in it — no pass over the scores afterwards
  unsigned long long* best_parts = nullptr;
};
bool topk_move_supported(const uint16_t* keys16, uint32_t key_range, uint64_t S);
// A value histogram of the keys produced by the generation kernel (GenArgs::
// key_hist, key_range bins in value order, read only) with its selection's
// status words (fused_status_words(), zero on entry): the u16 selection-order
// path then skips its histogram pass over the keys.
struct TopkFused {
  const uint32_t* hist = nullptr;
  uint32_t* status = nullptr;
};
// words of a fused-histogram buffer: key_range bins + the select kernel's status
constexpr uint32_t kTopkStatusWords = 2 * 1024 + 4;
inline uint32_t fused_hist_words(uint32_t key_range) { return (key_range + 3u) / 4u * 4u + kTopkStatusWords; }
// returns the packed-best partials written (TopkMove::best_parts), else 0
uint32_t topk_launch(const float* scores, const uint16_t* keys16, uint32_t key_range, uint64_t S, uint32_t k,
                     bool largest, bool sorted, uint32_t* idx_out, void* workspace, hipStream_t s,
                     const TopkMove* mv = nullptr, const TopkFused* fused = nullptr);
// rows: out[i] = rows[idx[i]] (row_words 32-bit words per row), optional scores
// MIG_STRIPE migration (util.hip): stripe i of k = individuals [i*S/k, (i+1)*S/k).
// emigrate: the best of every stripe (ties: lowest index) -> out rows/scores[i].
// immigrate: in row/score i replaces the worst of stripe i (ties: lowest
// index), the tournament key follows, and the kernel writes the island's new
// per-block best partials (+ {min, sum} statistics when stats_parts is set) —
// the stripes cover the population, so they are complete.  Returns their count.
void stripe_emigrate_launch(const float* scores, const void* rows, uint32_t row_words, uint64_t S, uint32_t k,
                            void* out_rows, float* out_scores, hipStream_t s);
uint32_t stripe_immigrate_launch(float* scores, uint16_t* keys, void* rows, uint32_t row_words, uint64_t S, uint32_t k,
                                 const void* in_rows, const float* in_scores, unsigned long long* best_parts,
                                 float* stats_parts, hipStream_t s);
void gather_rows_launch(const void* rows, const float* scores, uint32_t row_words, const uint32_t* idx, uint32_t n,
                        void* out_rows, float* out_scores, hipStream_t s);
// rows[idx[i]] = in[i]
void scatter_rows_launch(void* rows, float* scores, uint32_t row_words, const uint32_t* idx, uint32_t n,
                         const void* in_rows, const float* in_scores, hipStream_t s);

// mutation threshold table for geometric skips: thr[m-1] = floor((1-p)^m 2^32), m = 1..L
void build_mut_table(float p, uint32_t L, uint32_t* host_out, float* inv_log2_1mp);
// sparse BINARY bit-flip: kMutCap-entry Binomial(L, p) CDF table (binom_count)
void build_binom_table(float p, uint32_t L, uint32_t* host_out);

}  // namespace pga
