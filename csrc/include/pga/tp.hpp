// tp.hpp — the first phase of the transposed generation kernels (gfx950).
//
// A wave owns a contiguous range of children; a SEGMENT of up to
// kSegBatches batches of 64 children is selected one lane per child with
// every score / key load of the segment in flight at once (the second phase,
// breeding, is encoding specific: real_dev.hpp real_gen_tp and binary_dev.hpp
// binary_gen_tp both call tp_select_segment for this one).  Selection words are the ST_SEL layout of
// core.hpp, so the result equals st_select_parents() child by child.
#pragma once

#include <type_traits>

#include "pga/device.hpp"

#ifndef PGA_TP_NOSCORES
#define PGA_TP_NOSCORES 0
#endif
// batches (x 64 children) per tournament segment
#ifndef PGA_TP_SEG
#define PGA_TP_SEG 4
#endif

namespace pga {
namespace dev {

constexpr uint32_t kSegBatches = PGA_TP_SEG;
constexpr int kObjJit = 1001;  // launcher-only objective id: a linked user objective (jitgen*.hip)
// launcher-only objective id: the reference ABI's obj_f device function
// pointer (GenArgs::user_fn), called on the staged LDS row like a linked
// objective (real_dev.hpp)
constexpr int kObjUserFn = 1002;
constexpr uint32_t kTpMaxElite = 64;  // elites the transposed kernels route through their records

// element i of a buffer with a 32-bit byte offset (uniform base + one VGPR)
template <typename T>
__device__ __forceinline__ T ld32(const void* base, uint32_t i) {
  return *(const T*)((const char*)base + i * (uint32_t)sizeof(T));
}

// Tournament key modes: the f32 scores; the u16 keys of an integer
// objective (exact); or quantized u16 keys of a float objective (core.hpp
// qkey: equal keys fall back to the f32 scores, the exact result either way)
// (TP_NOKEY: experiment builds only, tournaments on fake keys without loads)
enum TpKeys : int { TP_F32 = 0, TP_KEY16 = 1, TP_QKEY16 = 2, TP_NOKEY = 3 };

// Parents (A, B) of children [begin + 64 B + lane] for the segment's batches
// B < kSegBatches -> par[B * 64 + lane].  ixs: 4 x 64 uint4 of LDS scratch
// (the contestants wait there while the loads fly).
template <int KM>
__device__ __forceinline__ void tp_select_segment(const GenArgs& a, uint32_t begin, uint32_t end, uint32_t lane,
                                                  uint4* ixs, uint2* par) {
  constexpr bool KEY = KM != TP_F32;
  const uint32_t S = (uint32_t)a.S;
  const uint32_t nbatch = (end - begin + 63) / 64;
  const bool tourn = a.selection == SEL_TOURNAMENT;  // tour_k == 2 guaranteed by the launcher
  const bool rank = a.selection == SEL_RANK;
  const bool roul = a.selection == SEL_ROULETTE;  // else random
  // raw keys (u16 zero-extended, or f32 scores), compared only after every
  // load of the segment is issued: a conversion here would make hipcc wait
  // for each batch's loads before issuing the next batch's
  using KT = typename std::conditional<KEY, uint32_t, float>::type;
  KT k0[kSegBatches], k1[kSegBatches], k2[kSegBatches], k3[kSegBatches];
#pragma unroll
  for (uint32_t B = 0; B < kSegBatches; ++B) {
    const uint32_t tc = begin + B * 64u + lane;
    const uint32_t cc = tc < end ? tc : end - 1;
    u32x4 blk{0u, 0u, 0u, 0u};
    if (B < nbatch) blk = draw<true>(a.key, ST_SEL, cc, 0);  // wave-uniform; batches past the end load entry 0
    const uint4 ix = make_uint4(word_to_index(blk.x, S), word_to_index(blk.y, S), word_to_index(blk.z, S),
                                word_to_index(blk.w, S));
    ixs[B * 64u + lane] = ix;
    const uint4 j = tourn ? ix : make_uint4(0, 0, 0, 0);
    if (roul) {  // the two selection words, searched below for every batch at once
      k0[B] = __builtin_bit_cast(KT, blk.x);
      k1[B] = __builtin_bit_cast(KT, blk.y);
    } else if (rank) {  // linear ranking: the two parents straight from the rank order
      const u32x4 b1 = draw<true>(a.key, ST_SEL, cc, 1);
      const uint32_t ra = rank_pick(blk.x, blk.y, blk.z, S, a.rank_thresh);
      const uint32_t rb = rank_pick(blk.w, b1.x, b1.y, S, a.rank_thresh);
      k0[B] = __builtin_bit_cast(KT, ld32<uint32_t>(a.rank_order, ra));
      k1[B] = __builtin_bit_cast(KT, ld32<uint32_t>(a.rank_order, rb));
    } else if constexpr (KM == TP_NOKEY) {
      k0[B] = j.x & 1023u;
      k1[B] = j.y & 1023u;
      k2[B] = j.z & 1023u;
      k3[B] = j.w & 1023u;
    } else if constexpr (KEY) {
      k0[B] = ld32<uint16_t>(a.key_cur, j.x);
      k1[B] = ld32<uint16_t>(a.key_cur, j.y);
      k2[B] = ld32<uint16_t>(a.key_cur, j.z);
      k3[B] = ld32<uint16_t>(a.key_cur, j.w);
    } else if constexpr (PGA_TP_NOSCORES) {  // experiment builds: tournaments without score loads
      k0[B] = (float)(j.x & 1023u);
      k1[B] = (float)(j.y & 1023u);
      k2[B] = (float)(j.z & 1023u);
      k3[B] = (float)(j.w & 1023u);
    } else {
      k0[B] = ld32<float>(a.score_cur, j.x);
      k1[B] = ld32<float>(a.score_cur, j.y);
      k2[B] = ld32<float>(a.score_cur, j.z);
      k3[B] = ld32<float>(a.score_cur, j.w);
    }
  }
  if (roul) {
    // fitness-proportional, by the guide table: the pick is the smallest i
    // with cumfit[i] >= u * total (roulette_pick's binary search); the guide
    // entry of the target's bucket is a lower bound for it, so one guide load,
    // one cumfit load and (rarely) a short forward scan find it.  The
    // 2 x kSegBatches picks of a lane advance in lock step.
    constexpr uint32_t NS = 2 * kSegBatches;
    const float total = a.cumfit[S - 1];
    const float scale = *a.roul_scale;
    const uint32_t gsh = a.roul_packed ? 1u : 0u;  // packed: entry e = {guide[e], cumfit[e]}
    uint32_t ix[NS];
    float tg[NS];
    #pragma unroll
    for (uint32_t i = 0; i < NS; ++i) {
      const uint32_t w = __builtin_bit_cast(uint32_t, (i & 1u) ? k1[i >> 1] : k0[i >> 1]);
      tg[i] = word_to_unit(w) * total;
      ix[i] = total > 0.f ? ld32<uint32_t>(a.roul_guide, roulette_bucket(tg[i], scale, S) << gsh) : word_to_index(w, S);
    }
    // kGuideCovered (S < 2^31): the bucket is not the last of its
    // individual's buckets, so that individual's cumfit is above every target
    // in it: the pick is resolved without a cumfit load
    const bool gflag = S <= kGuideIndexMask;  // wave-uniform
    bool covered[NS];
    #pragma unroll
    for (uint32_t i = 0; i < NS; ++i) {
      covered[i] = gflag && total > 0.f && (ix[i] & kGuideCovered) != 0u;
      ix[i] = gflag && total > 0.f ? ix[i] & kGuideIndexMask : ix[i];
    }
    // the first cumfit load is the aligned 16-byte window holding the guide
    // entry (cumfit is padded by 4 floats): a pick within it is resolved
    // without a dependent load, one past it scans on from the window's end
    float v[NS];
    #pragma unroll
    for (uint32_t i = 0; i < NS; ++i) {
      const uint32_t b = ix[i] & ~3u, off = ix[i] - b;
      float4 w = make_float4(tg[i], tg[i], tg[i], tg[i]);  // (covered: no entry below the target)
      if (!covered[i]) {
        if (gsh) {  // entries b .. b + 3: 32 bytes of the packed table
          const uint4 q0 = *(const uint4*)((const char*)a.roul_guide + b * 8u);
          const uint4 q1 = *(const uint4*)((const char*)a.roul_guide + b * 8u + 16u);
          w = make_float4(__builtin_bit_cast(float, q0.y), __builtin_bit_cast(float, q0.w),
                          __builtin_bit_cast(float, q1.y), __builtin_bit_cast(float, q1.w));
        } else {
          w = *(const float4*)((const char*)a.cumfit + b * 4u);
        }
      }
      // step over the window entries below the target, in order (the padding
      // past cumfit[S - 1] = total is never reached: total >= every target)
      uint32_t p = off;
      p = p == 0u && w.x < tg[i] ? 1u : p;
      p = p == 1u && w.y < tg[i] ? 2u : p;
      p = p == 2u && w.z < tg[i] ? 3u : p;
      p = p == 3u && w.w < tg[i] ? 4u : p;
      const bool live = total > 0.f;
      ix[i] = live ? (p == 4u ? b + 3u : b + p) : ix[i];
      v[i] = live && p == 4u ? -INFINITY : tg[i];  // -inf: step to b + 4 and load it below
    }
    for (uint32_t it = 0; it < S; ++it) {  // wave-uniform: until every pick of every lane is resolved
      bool more = false;
      #pragma unroll
      for (uint32_t i = 0; i < NS; ++i) more |= total > 0.f && v[i] < tg[i];
      if (!__any(more)) break;
      #pragma unroll
      for (uint32_t i = 0; i < NS; ++i) {
        const bool adv = total > 0.f && v[i] < tg[i];
        ix[i] += adv ? 1u : 0u;
        v[i] = gsh ? ld32<float>(a.roul_guide, (ix[i] << 1) + 1u) : ld32<float>(a.cumfit, ix[i]);
      }
    }
    #pragma unroll
    for (uint32_t B = 0; B < kSegBatches; ++B) {
      k0[B] = __builtin_bit_cast(KT, ix[2 * B]);
      k1[B] = __builtin_bit_cast(KT, ix[2 * B + 1]);
    }
  }
#pragma unroll
  for (uint32_t B = 0; B < kSegBatches; ++B) {
    const uint4 ix = ixs[B * 64u + lane];
    uint32_t pa = ix.x, pb = ix.y;
    if (tourn) {
      pa = k0[B] < k1[B] ? ix.y : ix.x;
      pb = k2[B] < k3[B] ? ix.w : ix.z;
      if constexpr (KM == TP_QKEY16) {  // equal quantized keys: the exact compare (rare, divergent)
        const uint32_t q0 = __builtin_bit_cast(uint32_t, k0[B]), q1 = __builtin_bit_cast(uint32_t, k1[B]);
        const uint32_t q2 = __builtin_bit_cast(uint32_t, k2[B]), q3 = __builtin_bit_cast(uint32_t, k3[B]);
        if (q0 == q1 || q0 == kQkNan || q1 == kQkNan)
          pa = ld32<float>(a.score_cur, ix.x) < ld32<float>(a.score_cur, ix.y) ? ix.y : ix.x;
        if (q2 == q3 || q2 == kQkNan || q3 == kQkNan)
          pb = ld32<float>(a.score_cur, ix.z) < ld32<float>(a.score_cur, ix.w) ? ix.w : ix.z;
      }
    } else if (rank || roul) {
      pa = __builtin_bit_cast(uint32_t, k0[B]);
      pb = __builtin_bit_cast(uint32_t, k1[B]);
    }
    par[B * 64u + lane] = make_uint2(pa, pb);
  }
}

// Work distribution of the two-phase kernels (binary_gen_tp, real_gen_tp):
// BLOCK shares with CU-local dynamic breed units.  Block b owns the contiguous children
// [b per, (b + 1) per), per = ceil(S / grid) rounded up to whole UNITS of
// U = GenArgs::tp_unit children (64: one batch; small populations use fewer,
// so that every wave gets a unit), processed in ROUNDS of at most
// tp_par_cap(nw) children: the waves pull the round's 256-child tournament
// segments from one LDS counter, then its units from another until none is
// left; a unit waits for its segment's ready flag (no block barrier between
// the phases).  The headline launch is one
// 16-wave block per CU (its LDS admits no second), so the counter balances
// every wave slot of the CU: the oldest-first issue order only decides WHICH
// wave breeds a unit, and the last ~20 us of thinning grid that equal static
// shares left (phase clocks, round 3) shrink to the last unit of each CU.
// The RNG is keyed per child, so any assignment is bit-identical.  (Round 3
// measured two device-scope balancers and dropped both: 128-child units from
// 64 global ticket heads cost +14 us of atomic latency; shares skewed by
// dispatch order did not move the young waves.)
constexpr uint32_t kTpMaxWaves = 16;
// parents per round: pseg tournament segments per 4 waves (7; 6 for kernels
// with more static LDS)
__host__ __device__ constexpr uint32_t tp_par_cap(uint32_t nw, uint32_t pseg = 7) {
  return nw / 4u * pseg * kSegBatches * 64u;
}
// dynamic LDS of a block of nw waves: records [nw][2][64][2] uint4, the
// round's parents [tp_par_cap] uint2
__host__ __device__ constexpr uint32_t tp_dyn_lds(uint32_t nw, uint32_t pseg = 7) {
  return nw * 4096u + tp_par_cap(nw, pseg) * 8u;
}
static_assert(tp_par_cap(4) % (kSegBatches * 64) == 0, "rounds hold whole segments");
// fused BINARY JIT kernels (binary_dev.hpp): steps of children staged in LDS
// per objective pass, 1 KB per wave per step after the parents (16 waves:
// 120 + 32 KB of dynamic LDS); tp_jit_stage_lds is what the launch adds
constexpr uint32_t kJitStageSteps = 2;
__host__ __device__ constexpr uint32_t tp_jit_stage_lds(uint32_t nw) { return nw * kJitStageSteps * 1024u; }
constexpr uint32_t kTpMaxSegs = tp_par_cap(kTpMaxWaves) / (kSegBatches * 64);  // tournament segments per round

// Breed prefetch depth: parent rows are loaded PD steps ahead (<= 3; a unit
// must hold at least PD steps, so PD <= GS = the steps of a 64-child unit)
#ifndef PGA_TP_PD
#define PGA_TP_PD 2
#endif
__host__ __device__ constexpr uint32_t tp_prefetch_depth(uint32_t gs) { return gs < PGA_TP_PD ? gs : PGA_TP_PD; }

__host__ __device__ inline uint32_t tp_unit(const GenArgs& a, uint32_t NG) {  // (the launchers record it)
  const uint32_t u = a.tp_unit, lo = NG * tp_prefetch_depth(64u / NG);
  return u >= lo && u <= 64u && (u & (u - 1u)) == 0u ? u : 64u;
}

// PRODUCER waves (one 16-wave block per CU): only the first nprod waves of a
// round run its tournament segments, the others breed from the start, each
// unit waiting for its segment's flag.  With every wave producing, the whole
// GPU runs its L2-bound random key reads first (~14 us at the headline, no
// row traffic) and its HBM-bound row gathers after (phase clocks, round 4);
// a few producers keep ahead of the breeders (a segment of 256 children per
// ~1.5 us of key latency against ~70 children per us consumed by a CU) and
// the two kinds of traffic overlap.  The key reads stay concentrated in the
// first ~20 us of the kernel, so the 2 MiB key array stays L2-resident.
#ifndef PGA_TP_PROD
#define PGA_TP_PROD 0
#endif
__device__ __forceinline__ uint32_t tp_producers(uint32_t nw) {
  return PGA_TP_PROD > 0 && nw == kTpMaxWaves ? (uint32_t)PGA_TP_PROD : nw;
}

// One ticket per wave from an LDS counter, with no lane divergence: every
// lane of the (full, converged) wave adds one — the atomic optimizer folds
// the uniform add into ONE ds_add of 64 and hands the first lane the old
// value — so the counter counts in steps of 64 and the ticket is the old
// value / 64.  An `if (lane == 0)` around the atomic inside the kernels'
// ticket loops left hipcc's structurizer a divergent region in a uniform
// loop, and real_gen_tp hung (round 4); a per-lane 0/1 add made the
// optimizer scan the wave with a 64-step scalar loop.
__device__ __forceinline__ uint32_t tp_ticket(uint32_t* ctr, uint32_t lane) {
  (void)lane;
#ifdef PGA_DEBUG  // the steps of 64 need a full, converged wave at every call
  if (__builtin_amdgcn_read_exec() != ~0ull) __builtin_trap();
#endif
  const uint32_t t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return __builtin_amdgcn_readfirstlane(t) >> 6;
}
// publish a ready flag: every lane stores the same value (no divergence)
__device__ __forceinline__ void tp_flag_set(uint32_t* flag) {
  __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the share [bb, be) of block blk.  skew (units, < per / U): in each block
// pair (2p, 2p + 1) the odd block hands `skew` units to the even one.  The
// dispatcher deals a launch's blocks to the XCDs round robin (block b ->
// XCD b % 8), and on every box measured the odd XCDs' blocks finished ~6 us
// behind the even ones' (phase clocks, round 4), so the launcher can skew.
__device__ __forceinline__ void tp_share(uint32_t S, uint32_t U, uint32_t blk, uint32_t& bb, uint32_t& be,
                                         uint32_t skew = 0) {
  uint64_t per = (S + (uint64_t)gridDim.x - 1) / gridDim.x;
  per = (per + U - 1) / U * U;
#ifdef PGA_TP_SWAPSHARE  // experiment builds: neighbouring blocks (XCDs) trade shares
  blk = (blk ^ 1u) < gridDim.x ? (blk ^ 1u) : blk;
#endif
  const uint64_t d = (uint64_t)skew * U < per && (blk | 1u) < gridDim.x ? (uint64_t)skew * U : 0;
  const uint64_t b = (uint64_t)blk * per + ((blk & 1u) ? d : 0), n = (blk & 1u) ? per - d : per + d;
  bb = (uint32_t)(b < S ? b : S);
  be = (uint32_t)(bb + n < S ? bb + n : S);
}
__device__ __forceinline__ void tp_block_range(uint32_t S, uint32_t U, uint32_t& bbegin, uint32_t& bend,
                                               uint32_t skew = 0) {
  tp_share(S, U, blockIdx.x, bbegin, bend, skew);
}

// Pair pool (cross-XCD tail sharing; OFF by default, PGA_TP_POOL=d enables
// 1/d of each block's units): the last P units of each block's share
// are bred by whichever wave of the block PAIR (2p, 2p+1: neighbouring blocks
// land on different XCDs) asks first, through one device-scope counter per
// pair (GenArgs::tp_pool, 128 B apart).  The XCDs do not finish alike: the
// phase clocks put the odd XCDs' blocks ~6 us behind the even ones' on every
// box (round 4), which per-CU counters cannot see.  A counter is 64 bits:
// the launch stamp (GenArgs::tp_seq, unique per launch) above the ticket
// count, so no launch has to clear it: a grab that reads an older stamp
// swaps in (stamp, 1) by compare-exchange (ticket 0); one that reads the
// current stamp takes a ticket with fetch-add.  Lock-free: every failed
// exchange means another wave's succeeded (a stale counter is never
// incremented, so the exchange cannot be starved by concurrent adds), and
// once the stamp is current it stays so for the launch.  Vector atomics from
// one lane (never the scalar cache).  Measured (round 4, interleaved A/B):
// 1/8 pooled 94.3 us/gen vs 89.8 without — a stolen unit runs its own
// tournaments and refills the row pipeline, which costs more than the XCD
// skew it removes, so the launcher leaves it off.
constexpr uint32_t kTpPoolStride = 16;  // u64 per pair counter (128 B)
// first child of the pool part of share [bb, be): its last min(P, units)
// whole units (the own part ends on a unit boundary)
__device__ __forceinline__ uint32_t tp_pool_start(uint32_t bb, uint32_t be, uint32_t U, uint32_t P) {
  const uint32_t nu = (be - bb + U - 1) / U;
  return bb + (nu > P ? nu - P : 0u) * U;
}
__device__ __forceinline__ uint32_t tp_pool_grab(unsigned long long* ctr, uint32_t seq, uint32_t lane) {
  uint32_t t = 0;
  if (lane == 0) {
    const unsigned long long stamp = (unsigned long long)seq << 32;
    unsigned long long v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      if ((v >> 32) == (unsigned long long)seq) {
        t = (uint32_t)__hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      // a stale stamp: claim ticket 0 of this launch (a failure reloads v)
      if (__hip_atomic_compare_exchange_strong(ctr, &v, stamp | 1ull, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        t = 0;
        break;
      }
    }
  }
  return __builtin_amdgcn_readfirstlane(t);
}

}  // namespace dev
}  // namespace pga
