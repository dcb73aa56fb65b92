// core.hpp — definitions shared by the gfx950 kernels, the CPU reference backend,
// the C API runtime and the torch bindings.
//
// Everything random in the engine comes from ONE counter-based generator,
// Philox4x32-10 (bit-identical to rocrand's `philox4x32_10_engine::ten_rounds`,
// checked by tests/test_rng.py via tools/rng_check.cpp).  A draw is addressed by
//   key     = 64-bit seed
//   counter = {block | stream<<24, child_lo, child_hi | island<<16, generation}
// so a value depends only on (seed, generation, island, individual, purpose,
// block) and never on launch geometry.  This is what lets the CPU reference
// backend reproduce a GPU generation bit for bit (BINARY / PERMUTATION) and
// what makes checkpoints exactly resumable (the generation counter IS the
// RNG state).
//
// Reference: the reference draws one process-global cuRAND XORWOW buffer of
// S*L floats per generation (src/pga.cu:35, :99-101) and re-uses the same slice
// for selection, crossover and mutation (src/pga.cu:298, :306-307, :341); see
// SURVEY.md §5.2 for why that is replaced.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PGA_HD __host__ __device__ __forceinline__
#define PGA_DEVICE_COMPILE 1
#else
#define PGA_HD inline
#endif

namespace pga {

// ---------------------------------------------------------------- enums ----
// Values are part of the C ABI (pga_ext.h mirrors them) and of the python
// bindings; append only.
enum Encoding : int32_t {
  ENC_BINARY = 0,       // bit-packed, 128-bit chunks, row stride multiple of 16 B
  ENC_REAL = 1,         // f32 genes, 4-gene chunks
  ENC_PERMUTATION = 2,  // u16 genes, each row a permutation of 0..L-1
};

enum Selection : int32_t {
  SEL_TOURNAMENT = 0,  // k-way tournament, with replacement, first max wins
  SEL_ROULETTE = 1,    // fitness proportional (scores shifted by the minimum)
  SEL_RANDOM = 2,      // uniform parent choice (no pressure) — testing/baseline
  SEL_RANK = 3,        // linear ranking, pressure sp in [1, 2] (Config::rank_pressure)
};

enum Crossover : int32_t {
  XO_UNIFORM = 0,     // per gene/bit: parent A with p=1/2 (reference default)
  XO_ONE_POINT = 1,   // prefix from A, suffix from B
  XO_TWO_POINT = 2,   // [a,b) from B, rest from A
  XO_BLEND = 3,       // REAL: BLX-alpha
  XO_ARITHMETIC = 4,  // REAL: child = A + u*(B-A), one u per child
  XO_PMX = 5,         // PERMUTATION: partially mapped crossover
  XO_OX = 6,          // PERMUTATION: ordered crossover (OX1)
  XO_NONE = 7,        // child = copy of parent A
};

enum Mutation : int32_t {
  MUT_BIT_FLIP = 0,     // BINARY: each bit flipped independently with rate p
  MUT_GAUSSIAN = 1,     // REAL: each gene += sigma*N(0,1) with rate p (clamped)
  MUT_UNIFORM = 2,      // REAL: each gene reset to U(lo,hi) with rate p
  MUT_RESET_ONE = 3,    // reference default: with prob p per individual reset ONE gene
  MUT_SWAP = 4,         // PERMUTATION: with prob p per individual swap two positions
  MUT_INVERSION = 5,    // PERMUTATION: with prob p per individual reverse a segment (2-opt)
  MUT_NONE = 6,
};

enum Objective : int32_t {
  OBJ_NONE = 0,          // no fused evaluation (scores provided externally)
  OBJ_ONEMAX = 1,        // BINARY: popcount
  OBJ_KNAPSACK = 2,      // BINARY: 0/1 knapsack, data = [values L | weights L], p0 = capacity
  OBJ_TRAP = 3,          // BINARY: concatenated deceptive trap, block size param_i (2,4,8)
  OBJ_LEADING_ONES = 4,  // BINARY: number of leading one bits
  OBJ_QUBO = 5,          // BINARY: obj_f0 * x^T Q x, data = L*L Q (integers in [-128,127]); int8 MFMA
  OBJ_SPHERE = 16,       // REAL: -sum z^2
  OBJ_RASTRIGIN = 17,    // REAL: -(10 D + sum z^2 - 10 cos(2 pi z))
  OBJ_ROSENBROCK = 18,   // REAL: -sum 100 (z_{i+1} - z_i^2)^2 + (1 - z_i)^2
  OBJ_ACKLEY = 19,       // REAL: -(ackley)
  OBJ_GRIEWANK = 20,     // REAL
  OBJ_SCHWEFEL = 21,     // REAL: -(418.9829 D - sum z sin(sqrt|z|))
  OBJ_LINEAR = 22,       // REAL: w . x  (the float-gene sum of reference E1 when w = 1)
  OBJ_KNAPSACK_REAL = 23,// REAL: reference E2 semantics: count=(int)(g*max_count)
  OBJ_TSP_RANDOM_KEY = 24,// REAL: reference E3 semantics (decode (int)(g*L), dup penalty)
  OBJ_TSP = 32,          // PERMUTATION: -(closed tour length), data = L*L distance matrix
  OBJ_TSP_OPEN = 33,     // PERMUTATION: -(open path length) (reference E3 metric)
  OBJ_TSP_EUC = 34,      // PERMUTATION: -(closed tour length), data = L (x, y) city coordinates
  OBJ_USER_FNPTR = 64,   // REAL: reference-ABI device function pointer obj_f
};

// Island migration policy (Island::emigrate / immigrate)
enum MigrationPolicy : int32_t {
  MIG_TOPK = 0,    // exact: the top-k emigrate, the bottom-k are replaced (two radix selections)
  MIG_STRIPE = 1,  // the population is cut into k contiguous stripes; stripe i's best
                   // emigrates and its worst is replaced by immigrant i (one pass each)
};

// Philox streams (purpose tags, high byte of counter word 0)
enum Stream : uint32_t {
  ST_INIT = 1,     // initial population
  ST_XO = 2,       // crossover masks / per-gene crossover values
  ST_CHILD = 3,    // per-child word pool (see word layout below)
  ST_MUTX = 4,     // extra per-gene mutation values (gaussian etc.)
  ST_MIGRATE = 5,  // migration pairing / victim choice
  ST_COMPAT = 6,   // reference-ABI rand slices handed to user callbacks
  ST_PERM = 7,     // permutation crossover helpers
  ST_SEL = 8,      // BINARY: selection words, 4 per block
  ST_BMUT = 9,     // BINARY: mutation words (positions, per-chunk geometric draws)
};

// Per-child randomness (stream ST_CHILD, one Philox block b per index):
//   child words  t = 0,1,2,...  = register (t % 3) of block (t / 3)   [.x .y .z]
//   mutation word of chunk c    = register .w of block c
// so the lane that owns chunk c of an individual holds that chunk's first
// mutation draw in its own register, and child words are fetched with one
// group-uniform ds_bpermute.  Child-word layout:
//   0      crossover-probability test
//   1, 2   cut points / blend parameter
//   3      per-individual mutation test (RESET_ONE / SWAP / INVERSION)
//   4      per-individual mutation position
//   5..    selection words (2k for tournament-k, 2 otherwise)
// Further geometric skips of a BINARY chunk come from mut_skip_word(r0, n);
// REAL mutation values come from stream ST_MUTX, block (chunk << 6) | (32 + n)
// for the n-th mutated gene of the chunk, whose .w word is the next skip.
constexpr uint32_t W_XOPROB = 0, W_CUT1 = 1, W_CUT2 = 2, W_MUTIND = 3, W_MUTPOS = 4, W_SEL = 5;
constexpr uint32_t kMutCap = 128;  // geometric-skip table length (one BINARY chunk)

// ---------------------------------------------------------------- Philox ---
struct u32x4 {
  uint32_t x, y, z, w;
};

PGA_HD void mulhilo32(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

// NH ("no hoist"): the key words pass through an empty asm, so the compiler
// cannot precompute the 20 round keys of a loop-invariant key outside a
// loop (20 SGPRs pinned for the whole loop); the hot BINARY kernel uses it.
template <bool NH = false>
PGA_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (NH) asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c.x, hi0, lo0);
    mulhilo32(0xCD9E8D57u, c.z, hi1, lo1);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

struct RngKey {
  uint32_t k0, k1;     // seed
  uint32_t gen;        // generation counter
  uint32_t island;     // island id (< 65536)
};

template <bool NH = false>
PGA_HD u32x4 draw(const RngKey& key, uint32_t stream, uint64_t ind, uint32_t block) {
  u32x4 c{(block & 0x00FFFFFFu) | (stream << 24), (uint32_t)ind,
          (uint32_t)(ind >> 32) | (key.island << 16), key.gen};
  return philox4x32_10<NH>(c, key.k0, key.k1);
}

// by value + value selects: a select over field REFERENCES becomes a select of
// addresses, which forces the struct into scratch memory on the device
PGA_HD uint32_t sel4(u32x4 v, uint32_t i) {
  uint32_t r = v.w;
  r = i == 2 ? v.z : r;
  r = i == 1 ? v.y : r;
  return i == 0 ? v.x : r;
}
PGA_HD uint32_t sel3(u32x4 v, uint32_t i) {
  uint32_t r = v.z;
  r = i == 1 ? v.y : r;
  return i == 0 ? v.x : r;
}

// child word t (reference definition; kernels fetch it from the owner lane)
PGA_HD uint32_t child_word(const RngKey& key, uint64_t child, uint32_t t) {
  return sel3(draw(key, ST_CHILD, child, t / 3u), t % 3u);
}
// first mutation draw of chunk c
PGA_HD uint32_t chunk_mut_word(const RngKey& key, uint64_t child, uint32_t c) {
  return draw(key, ST_CHILD, child, c).w;
}
// n-th further geometric-skip word of a BINARY chunk whose first mutation
// word was r0 (only reached when r0 already placed a flip, ~12% of chunks at
// rate 1/L = 1/1024).  A murmur3 finalizer of (r0, n) instead of another
// Philox block: in a wave of 64 chunks SOME lane almost always needs it, so a
// Philox here cost the whole wave a third Philox per child (measured: the
// largest single VALU item of the headline kernel after the two mandatory
// draws).  r0 is a Philox word spread over ~5e8 values, and the finalizer is
// a bijection with full avalanche, so successive skips are uniform and
// independent for every practical purpose.
PGA_HD uint32_t mut_skip_word(uint32_t r0, uint32_t n) {
  uint32_t h = r0 ^ (0x9E3779B9u * (n + 1u));
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// uniform index in [0, n) from a 32-bit word (n < 2^32)
PGA_HD uint32_t word_to_index(uint32_t w, uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  // One v_mul_hi_u32.  The empty asm makes the result opaque: otherwise hipcc
  // folds zext(mulhi)*4 into a 64-bit shift of a register PAIR whose low half
  // may be an in-flight load destination, which forces s_waitcnt vmcnt(0).
  uint32_t r = __umulhi(w, n);
  asm("" : "+v"(r));
  return r;
#else
  return (uint32_t)(((uint64_t)w * (uint64_t)n) >> 32);
#endif
}

// uniform float in (0, 1], exactly representable, identical on host and device
PGA_HD float word_to_unit(uint32_t w) {
  return (float)((w >> 8) + 1u) * (1.0f / 16777216.0f);
}

// ------------------------------------------------------- geometric skips ---
// Bernoulli(p)-per-position mutation is simulated by geometric skips.  The skip
// distribution is inverted EXACTLY with an integer threshold table
//   thr[m] = floor((1-p)^m * 2^32)  for m = 1..cap   (thr[0] = 2^32 implied)
//   skip(r) = #{ m in [1,cap] : r < thr[m] }
// P(skip >= m) = thr[m]/2^32 = (1-p)^m.  A float log estimate seeds the
// search and two integer correction loops make the result exact, so device
// and host agree bit for bit.
PGA_HD uint32_t geom_skip(uint32_t r, const uint32_t* thr, uint32_t cap, float inv_log2_1mp) {
  // thr is 1-indexed: thr[m-1] holds thr[m]
  if (cap == 0) return 0;
  if (r >= thr[0]) return 0;  // flip at the very next position
  float est = __builtin_log2f(((float)r + 0.5f) * (1.0f / 4294967296.0f)) * inv_log2_1mp;
  uint32_t m = est <= 0.f ? 0u : (est >= (float)cap ? cap : (uint32_t)est);
  while (m < cap && r < thr[m]) ++m;         // thr[m] == threshold for m+1
  while (m > 0 && !(r < thr[m - 1])) --m;    // thr[m-1] == threshold for m
  return m;
}

// ------------------------------------------------------------ arguments ----
// One POD for every encoding.  Passed by value to kernels (fits the 4 KB
// kernarg segment) and by const-ref to the CPU reference.
struct GenArgs {
  // population buffers (current generation read, next generation written)
  const void* cur;
  void* next;
  const float* score_cur;
  float* score_next;
  unsigned long long* best_next;  // packed (orderable score << 32 | ~index), reset by launcher

  uint64_t S;          // individuals
  uint32_t L;          // genes (bits for BINARY)
  uint32_t row_words;  // row stride in 32-bit words (multiple of 4)
  uint32_t chunks;     // 16-byte chunks per row that hold genes
  uint32_t encoding;

  RngKey key;

  // selection
  int32_t selection;
  uint32_t tour_k;
  const float* cumfit;  // roulette: inclusive prefix sums of shifted scores (S)
  // roulette guide table (util.hip roulette_guide_launch): roul_guide[b] = the
  // first individual whose cumfit bucket is >= b, bucket(t) =
  // roulette_bucket(t, *roul_scale, S); nullptr: binary search only
  const uint32_t* roul_guide;
  const float* roul_scale;
  const uint32_t* rank_order;  // rank: individuals by ascending (score_key, index)
  uint32_t rank_thresh;        // rank: uniform-branch threshold (2 - sp) * 2^32

  // crossover
  int32_t crossover;
  uint32_t xo_thresh_hi;  // crossover happens iff word < xo_thresh (xo_thresh = p_c * 2^32,
  uint32_t xo_always;     //  xo_always = 1 when p_c >= 1)
  float blend_alpha;

  // mutation
  int32_t mutation;
  float mut_rate;            // per gene (BIT_FLIP/GAUSSIAN/UNIFORM) or per individual
  uint32_t mut_ind_thresh;   // per-individual threshold (RESET_ONE/SWAP/INVERSION)
  const uint32_t* mut_thr;   // geometric skip thresholds (cap = L entries)
  float mut_inv_log2_1mp;    // 1/log2(1-p)
  float sigma;               // gaussian sigma
  float lo, hi;              // REAL gene bounds

  // objective
  int32_t objective;
  int32_t obj_i;         // integer parameter (trap order, rotated flag, ...)
  float obj_f0, obj_f1;  // float parameters (capacity, max count, ...)
  const float* obj_data; // problem data (weights, distance matrix, rotation, shift)
  const float* obj_data2;
  void* user_fn;         // reference-ABI device function pointer (OBJ_USER_FNPTR)
  void* user_xo_fn;      // reference-ABI crossover_f (compat kernel), nullptr = built-in
  void* user_mut_fn;     // reference-ABI mutate_f (compat kernel), nullptr = built-in
  float* compat_rand;    // S*L scratch for the rand slices handed to user callbacks

  // elitism: children [0, n_elite) copy elite_idx[i] (E==1 may use best_cur)
  uint32_t n_elite;
  const uint32_t* elite_idx;
  const unsigned long long* best_cur;  // per-block packed bests of the current generation
  uint32_t n_best_cur;

  // Tournament keys: for integer-valued objectives with scores in [0, 65535]
  // (OneMax, LeadingOnes, Trap) every individual also carries key = score as
  // u16.  The 2 MiB key array of a 1M population stays L2-resident, the 4 MiB
  // f32 array does not, and tournament reads are random; comparisons are
  // unchanged because the key is exact.  nullptr when disabled.
  const uint16_t* key_cur;
  uint16_t* key_next;
  // float objectives on the GPU (REAL): key_cur / key_next hold QUANTIZED
  // keys (qkey) and qk -> {min, max} of the current generation's scores, the
  // range the kernel quantizes the next generation's keys over
  const float* qk;

  // derived objective data built by the runtime (QUBO: int8 Q^T padded to
  // qubo_padded_length(L) square); nullptr when unused
  const int8_t* qubo_qt;
  // BINARY knapsack on the matrix cores (binary.hip knap_mfma): int8 digit
  // table of [values | weights] in B-fragment order, its digit count and
  // column count; nullptr when the instance is not integer-exact
  const void* knap_tab;
  uint32_t knap_dig, knap_cols;

  // fused statistics: when set, evaluating kernels store a {min, sum} pair per
  // block (same blocks as best_parts); see device.hpp ScoreStats
  float* stats_parts;

  // padding mask for the last chunk (BINARY)
  u32x4 last_mask;


  // hipGraph replay: when set, the generation counter is read from device
  // memory (key.gen = *gen_dev + gen_off) so one captured graph of G
  // generations can be replayed without re-recording kernel arguments
  const uint32_t* gen_dev;
  uint32_t gen_off;

  // BINARY bit-flip: 1 = sparse sampler (mut_thr is the Binomial CDF table),
  // 0 = per-chunk geometric skips (mut_thr is the geometric table)
  uint32_t mut_sparse;

  // two-phase kernels (tp.hpp): children per dynamically assigned breed unit,
  // a power of two in [64 / GS, 64] set by the launcher (0 = 64)
  uint32_t tp_unit;
  // pair pool of binary_gen_tp (tp.hpp): per block pair one 64-bit counter
  // (kTpPoolStride apart), this launch's stamp, the units per block in the
  // pool (0 / nullptr: no pool)
  unsigned long long* tp_pool;
  uint32_t tp_seq, tp_pool_units;
  // share skew of binary_gen_tp (tp.hpp tp_share): units each odd block of a
  // pair hands to its even neighbour (0: equal shares)
  uint32_t tp_skew;
  // encoding-specific derived objective table, nullptr when unused
  // (PERMUTATION, perm.hip: the integer distance matrix as u16, kind 1 = a
  // symmetric matrix's strict lower triangle then its diagonal, 2 = the
  // full matrix)
  const void* obj_aux;
  uint32_t obj_aux_kind, obj_aux_bytes;
  // fused key histogram (binary_gen_tp, integer objectives): when set, the
  // generation kernel adds the histogram of the u16 keys it writes (each
  // clamped to hist_bins - 1) to key_hist, which is zero before the launch,
  // and zeroes hist_zero[0, hist_zero_words) — a later generation's buffer
  // and its selection status words (the Island rotates three buffers).
  // Exact top-k / bottom-k selections (migration, elitism,
  // pga_get_best_top) then need no histogram pass over the keys.
  uint32_t* key_hist;
  uint32_t* hist_zero;
  uint32_t hist_bins, hist_zero_words;
  // binary_gen_tp: child rows stored non-temporally (experiment knob,
  // PGA_TP_NT_STORE=1; 0: ordinary stores)
  uint32_t nt_store;
  // rank selection (binary_gen_tp, integer objectives): when set, every block
  // also stores its LDS key histogram, all hist_bins bins, to
  // rank_counts[bin * gridDim.x + blockIdx.x]: the tile counts of the next
  // generation's rank-order sort (sort.hip, rank_order16_counts), whose count
  // pass then reads nothing.  The launcher sets it only when each block's
  // children are exactly one kRankTile sort tile.
  uint32_t* rank_counts;
  // roulette, two-phase kernels: roul_guide is the PACKED table, entry e =
  // {guide[e], cumfit[e] bits} (8 bytes), so a pick's cumfit window usually
  // sits in the guide line it just fetched (util.hip roulette_*_launch)
  uint32_t roul_packed;
};
// the fused histogram's LDS bins (binary_gen_tp): objectives with more key
// values use the separate histogram pass
constexpr uint32_t kHistMaxBins = 2048;

PGA_HD uint32_t sel_words(const GenArgs& a) {
  return a.selection == SEL_TOURNAMENT ? 2u * a.tour_k : (a.selection == SEL_RANK ? 6u : 2u);
}

// Linear ranking selection, exactly and without floating point: the rank
// density of pressure sp, P(r) = (2-sp)/S + (sp-1)(2r+1)/S^2 (r = 0 worst),
// is a mixture of the uniform rank (weight 2-sp) and the maximum of two
// uniform ranks (weight sp-1, P(max = r) = (2r+1)/S^2).  Three words per
// parent: branch, first rank, second rank.  Integer-only, so the CPU backend
// and the kernels agree bit for bit.
PGA_HD uint32_t rank_thresh_of(float sp) {
  const double b = 2.0 - (double)(sp < 1.f ? 1.f : (sp > 2.f ? 2.f : sp));
  const double t = b * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}
PGA_HD uint32_t rank_pick(uint32_t w_branch, uint32_t w1, uint32_t w2, uint32_t S, uint32_t thresh) {
  const uint32_t r1 = word_to_index(w1, S);
  if (w_branch < thresh) return r1;
  const uint32_t r2 = word_to_index(w2, S);
  return r1 > r2 ? r1 : r2;
}

// Bernoulli(p) flips over positions [0, clen) of chunk c (clen <= kMutCap):
// first draw r0 = chunk_mut_word, then geometric skips.  Returns the flip
// positions as a 128-bit mask.
PGA_HD u32x4 chunk_flip_mask(const GenArgs& a, uint64_t child, uint32_t c, uint32_t clen, uint32_t r0,
                             const uint32_t* thr) {
  u32x4 m{0, 0, 0, 0};
  if (r0 < thr[kMutCap - 1]) return m;  // no flip in 128 positions: the common case
  uint32_t pos = geom_skip(r0, thr, kMutCap, a.mut_inv_log2_1mp);
  uint32_t n = 0;
  while (pos < clen) {
    const uint32_t bit = 1u << (pos & 31u);
    switch (pos >> 5) {
      case 0: m.x ^= bit; break;
      case 1: m.y ^= bit; break;
      case 2: m.z ^= bit; break;
      default: m.w ^= bit; break;
    }
    // the next flip lands in this chunk iff skip(h) < rem; skip(h) >= rem
    // <=> h < thr[rem] (1-indexed): one table read decides the common "no
    // second flip" case without the log-seeded search (same result)
    const uint32_t rem = clen - pos - 1u;
    if (rem == 0u) break;
    const uint32_t h = mut_skip_word(r0, n++);
    if (h < thr[rem - 1u]) break;
    pos += 1u + geom_skip(h, thr, kMutCap, a.mut_inv_log2_1mp);
  }
  return m;
}

PGA_HD bool do_crossover(const GenArgs& a, uint32_t w0) { return a.xo_always || w0 < a.xo_thresh_hi; }

// Roulette guide-table bucket of a cumulative weight t (Chen & Asau's
// indexed search): any monotone non-decreasing map into [0, B] works, since
// the pick then scans forward from guide[bucket(target)] to the first
// cumfit >= target -- the same individual as the binary search.
// guide entries (S < 2^31): the individual's index, and kGuideCovered when
// the bucket is not the last one the individual's weight reaches into (its
// cumfit is then above every target in the bucket: no cumfit load)
constexpr uint32_t kGuideCovered = 0x80000000u, kGuideIndexMask = 0x7FFFFFFFu;
PGA_HD uint32_t roulette_bucket(float t, float scale, uint32_t B) {
  const float x = t * scale;
  return x >= (float)B ? B : (x > 0.f ? (uint32_t)x : 0u);
}

// ------------------------------------------------- BINARY randomness layout ---
// The BINARY encoding draws per child (REAL / PERMUTATION keep the ST_CHILD
// word pool above):
//   selection word t      = register t%4 of block t/4 of stream ST_SEL
//   misc block            = block 0 of ST_CHILD: .x crossover test, .y/.z cut
//                           points, .w mutation word (bit-flip count K in the
//                           sparse regime, the per-individual test for RESET_ONE)
//   mutation word j       = register j%4 of block j/4 of ST_BMUT
//   dense chunk draw of c = register .x of block kDenseBlock + c of ST_BMUT
//   crossover mask        = block c of ST_XO (128 bits per chunk)
// so one Philox block yields all four contestants of a binary tournament and
// the kernel can run the tournaments of 64 children with one lane each.
//
// Bit-flip mutation (rate p per bit) has two exact samplers, chosen by L and p:
//   sparse (L <= kSparseMaxL, L*p <= kSparseMaxMean): K ~ Binomial(L, p) by
//     inverse CDF of the misc word (mut_thr holds the CDF table), then the
//     first K distinct values of word_to_index(mutation word j, L), j = 0,1,..
//     (a uniform K-subset: together, independent Bernoulli(p) bits).
//   dense: per 128-bit chunk, geometric skips from the dense chunk draw
//     (chunk_flip_mask, mut_thr holds the geometric table).
constexpr uint32_t kSparseMaxL = 8192;
constexpr float kSparseMaxMean = 1.5f;
constexpr uint32_t kDenseBlock = 0x400000u;  // well above any sparse word block
constexpr uint32_t kRecPos = 8;              // positions a kernel carries per child record

PGA_HD bool bin_sparse_mutation(uint32_t L, float p) {
  return L <= kSparseMaxL && p > 0.f && (double)L * (double)p <= (double)kSparseMaxMean;
}
PGA_HD uint32_t bin_sel_word(const RngKey& key, uint64_t child, uint32_t t) {
  return sel4(draw(key, ST_SEL, child, t >> 2), t & 3u);
}
template <bool NH = false>
PGA_HD u32x4 bin_misc(const RngKey& key, uint64_t child) { return draw<NH>(key, ST_CHILD, child, 0); }
template <bool NH = false>
PGA_HD uint32_t bin_mut_word(const RngKey& key, uint64_t child, uint32_t j) {
  return sel4(draw<NH>(key, ST_BMUT, child, j >> 2), j & 3u);
}
template <bool NH = false>
PGA_HD uint32_t bin_chunk_mut_word(const RngKey& key, uint64_t child, uint32_t c) {
  return draw<NH>(key, ST_BMUT, child, kDenseBlock + c).x;
}
// sparse regime: number of flips from the misc word (thr = CDF table;
// entries of 0xFFFFFFFF end the table)
PGA_HD uint32_t binom_count(uint32_t w, const uint32_t* thr) {
  uint32_t k = 0;
  while (k < kMutCap && thr[k] != 0xFFFFFFFFu && w >= thr[k]) ++k;
  return k;
}

// bits of the 32-bit word starting at bit `base` that fall in [lo, hi)
PGA_HD uint32_t range_mask32(uint32_t base, uint32_t lo, uint32_t hi) {
  uint32_t l = lo <= base ? 0u : (lo - base >= 32u ? 32u : lo - base);
  uint32_t h = hi <= base ? 0u : (hi - base >= 32u ? 32u : hi - base);
  uint32_t mh = h >= 32u ? 0xFFFFFFFFu : ((1u << h) - 1u);
  uint32_t ml = l >= 32u ? 0xFFFFFFFFu : ((1u << l) - 1u);
  return mh & ~ml;
}

// Lanes cooperating on one individual: the smallest power of two >= chunks,
// capped at one wave.  Part of the SEMANTICS (it fixes the float summation
// order of group reductions), so the CPU reference uses it too.
PGA_HD uint32_t group_size(uint32_t chunks) {
  uint32_t g = 1;
  while (g < chunks && g < 64) g <<= 1;
  return g;
}

// Kernel modes
enum Mode : int32_t {
  MODE_GEN = 0,     // select + crossover + mutate + evaluate (fused generation)
  MODE_INIT = 1,    // random init + evaluate
  MODE_EVAL = 2,    // evaluate current rows
  MODE_CROSS = 3,   // select + crossover only (reference pga_crossover)
  MODE_MUTATE = 4,  // mutate rows in place (reference pga_mutate)
};

// objectives whose scores are exact integers in [0, L] (u16 tournament keys)
PGA_HD bool integer_objective(int32_t obj, uint32_t L) {
  return (obj == OBJ_ONEMAX || obj == OBJ_LEADING_ONES || obj == OBJ_TRAP) && L <= 65535u;
}

// QUBO coefficient as used by every backend: round half away from zero, clamp to int8
PGA_HD int32_t qubo_coef(float q) {
  float r = q < 0.f ? -__builtin_floorf(-q + 0.5f) : __builtin_floorf(q + 0.5f);
  r = r < -128.f ? -128.f : (r > 127.f ? 127.f : r);
  return (int32_t)r;
}

// ---- quantized tournament keys (GPU tournaments on float scores) ----
// A 16-bit key per individual, monotone non-decreasing in its score: q(a) <
// q(b) implies a < b, so a tournament decides on the 2-byte keys (an array
// that stays L2-resident, where the f32 scores do not) and only equal keys
// fall back to comparing the f32 scores -- the exact result either way.
// lo / scale come from the population's score range; NaN maps to kQkNan,
// which always falls back.
constexpr uint32_t kQkNan = 0xFFFFu;
PGA_HD void qkey_params(float mn, float mx, float& lo, float& scale) {
  const float d = mx - mn;
  const bool ok = d > 0.f && d < 3.0e38f && mn > -3.0e38f;
  lo = ok ? mn : 0.f;
  scale = ok ? 65534.f / d : 0.f;
}
PGA_HD uint32_t qkey(float s, float lo, float scale) {
  const float x = (s - lo) * scale;
  if (!(x == x)) return kQkNan;
  return x <= 0.f ? 0u : (x >= 65534.f ? 65534u : (uint32_t)x);
}

// orderable encoding of a float score (monotone, -NaN < -inf < ... < +inf)
PGA_HD uint32_t score_key(float s) {
  uint32_t u;
  __builtin_memcpy(&u, &s, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
PGA_HD float key_score(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  float s;
  __builtin_memcpy(&s, &u, 4);
  return s;
}
// packed best: larger is better; ties resolved to the LOWER index (reference
// pga_get_best keeps the first max, src/pga.cu:221-229)
PGA_HD unsigned long long pack_best(float s, uint64_t idx) {
  return ((unsigned long long)score_key(s) << 32) | (0xFFFFFFFFull - (uint32_t)idx);
}
PGA_HD uint64_t best_index(unsigned long long p) { return 0xFFFFFFFFull - (uint32_t)p; }
PGA_HD float best_score(unsigned long long p) { return key_score((uint32_t)(p >> 32)); }

}  // namespace pga
