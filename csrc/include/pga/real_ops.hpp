// real_ops.hpp — per-gene semantics of the REAL (f32) encoding, shared by the
// gfx950 kernels (csrc/kernels/real.hip) and the CPU reference backend
// (csrc/cpu/cpu_real.cpp).  A chunk is 4 consecutive genes (16 bytes).
//
// Reference parity: the reference's only genome type is f32 (include/pga.h:29)
// with uniform crossover "rand > 0.5 ? p1 : p2" (src/pga.cu:135-143) and a
// single-gene reset mutation with p = 0.01 per individual (src/pga.cu:127-133);
// both are XO_UNIFORM / MUT_RESET_ONE here, with independent random streams.
//
// REAL randomness layout (every word a pure function of seed, generation,
// island, individual, purpose and position -- never of launch geometry):
//   selection     the BINARY ST_SEL words (core.hpp; one Philox block = the
//                 four contestants of a binary tournament)
//   misc block    draw(ST_CHILD, child, 0): .x crossover test, .y cut point 1 /
//                 arithmetic u, .z cut point 2, .w mutation word (sparse
//                 per-gene mutation: the Binomial(L, p) count K; RESET_ONE:
//                 the per-individual test)
//   positions     sparse per-gene mutation: the first K distinct
//                 word_to_index(mutation word j, L), j = 0, 1, ... (the BINARY
//                 ST_BMUT words); RESET_ONE: position of word 0
//   values        the n-th mutated gene (n in the order above) takes
//                 draw(ST_MUTX, child, n): gaussian z = gauss_z(.x, .y),
//                 uniform / reset value unit_range(.z)
//   dense         per-gene mutation with L p > kSparseMaxMean: per chunk c,
//                 geometric skips from draw(ST_BMUT, child, kDenseBlock + c).x,
//                 the n-th mutated gene of the chunk from ST_MUTX block
//                 (c << 6) | (32 + n), whose .w is the next skip
//   crossover     UNIFORM: gene g from A iff bit g % 32 of xo word g / 32
//                 (word w = register w % 4 of draw(ST_XO, child, w / 4));
//                 BLEND: gene g's u = word_to_unit(mut_skip_word(misc.y, g)),
//                 a murmur3 finalizer of the child's seed word (a bijection with
//                 full avalanche) instead of a Philox block per chunk
// The per-child words need one Philox block each, so the transposed kernel
// (real_gen_tp) computes them one lane per child; a gene-parallel lane draws
// nothing but the UNIFORM mask of genomes beyond 32 genes.
#pragma once

#include <math.h>

#include "pga/core.hpp"

namespace pga {

constexpr float kPi = 3.14159265358979323846f;

// bitwise select: both operands are loaded unconditionally, so the device
// compiler cannot turn "c ? A[j] : B[j]" into a load through a selected
// address (which demotes the arrays to scratch memory)
PGA_HD float fsel(bool c, float x, float y) {
  uint32_t a, b;
  __builtin_memcpy(&a, &x, 4);
  __builtin_memcpy(&b, &y, 4);
  const uint32_t m = 0u - (uint32_t)c;
  const uint32_t r = (a & m) | (b & ~m);
  float f;
  __builtin_memcpy(&f, &r, 4);
  return f;
}
PGA_HD float u2f(uint32_t u) {
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
PGA_HD uint32_t f2u(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return u;
}

// cos(2 pi x) of the Rastrigin / Ackley terms.  On the device this is ONE
// v_cos_f32, whose argument is in revolutions, instead of the range-reduced
// libm cosf (measured: Rastrigin-30D pop 1M 145 -> 132 us/gen, Ackley 157 ->
// 141).  The CPU reference keeps cosf, so REAL scores of these two objectives
// agree with it to float rounding (tests compare them with a tolerance), not
// bit for bit; every GPU kernel uses the same instruction, so GPU paths stay
// bit-identical to each other.  PGA_HW_TRIG=0 restores cosf on the device.
#ifndef PGA_HW_TRIG
#define PGA_HW_TRIG 1
#endif
PGA_HD float cos2pi(float x) {
#if defined(__HIP_DEVICE_COMPILE__) && PGA_HW_TRIG
  return __builtin_amdgcn_cosf(x);  // v_cos_f32: argument in revolutions
#else
  return cosf(2.f * kPi * x);
#endif
}

PGA_HD float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
// explicit fmaf everywhere a gene VALUE is produced: device (-ffp-contract=fast)
// and host compilers then agree bit for bit on the rows
PGA_HD float unit_range(uint32_t w, float lo, float hi) { return fmaf(hi - lo, word_to_unit(w), lo); }

// ---- deterministic gaussian (host == device, bit for bit) ----
// Box-Muller from two Philox words with hand-written elementary functions:
// integer range reduction, f32 multiplies and explicit fmaf only.  Each of
// these is a correctly rounded IEEE operation on the host and on gfx950 and
// no product is left for the device compiler to contract into an fma, so the
// CPU backend reproduces gaussian mutation exactly (libm logf / cosf differ
// between the two by ulps).  Accuracy ~1e-7 relative: far below what a
// mutation step can resolve.
//
// ln(k / 2^24) for k in [1, 2^24]
PGA_HD float det_ln_unit(uint32_t k) {
  uint32_t b = f2u((float)k);  // exact: k < 2^25
  int32_t e = (int32_t)(b >> 23) - 127;
  uint32_t mb = (b & 0x007FFFFFu) | 0x3F800000u;  // m in [1, 2)
  if (mb > 0x3FB504F3u) {                          // m > sqrt(2): m / 2
    mb -= 0x00800000u;
    ++e;
  }
  const float f = u2f(mb) - 1.f;  // exact (Sterbenz), in [sqrt(.5) - 1, sqrt(2) - 1]
  float q = -7.764425129e-02f;
  q = fmaf(q, f, 1.265655756e-01f);
  q = fmaf(q, f, -1.306504160e-01f);
  q = fmaf(q, f, 1.420955658e-01f);
  q = fmaf(q, f, -1.663306952e-01f);
  q = fmaf(q, f, 2.000124156e-01f);
  q = fmaf(q, f, -2.500060499e-01f);
  q = fmaf(q, f, 3.333332837e-01f);
  q = fmaf(q, f, -4.999999702e-01f);
  const float f2 = f * f;
  const float lm = fmaf(f2, q, f);                              // ln(m)
  return fmaf((float)(e - 24), 0.693147180559945309f, lm);      // + (e - 24) ln 2
}
// sqrt(s), s >= 0: bit-trick reciprocal square root + 3 Newton steps
PGA_HD float det_sqrt(float s) {
  float y = u2f(0x5F3759DFu - (f2u(s) >> 1));
  const float h = 0.5f * s;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float hy = h * y;
    y = y * fmaf(-hy, y, 1.5f);
  }
  return s * y;
}
// cos(2 pi u) for u = k / 2^24, k in [1, 2^24] (word_to_unit's lattice):
// quadrant and octant by integer arithmetic, then a polynomial on [0, pi/4]
PGA_HD float det_cos_turn(uint32_t k) {
  const uint32_t t = k & 0x00FFFFFFu;  // 2^24 -> 0 (cos 2 pi = cos 0)
  const uint32_t quad = t >> 22;
  uint32_t r = t & 0x003FFFFFu;        // angle in the quadrant, units of (pi/2) / 2^22
  const bool comp = r > 0x00200000u;   // past pi/4: use the complementary angle
  r = comp ? 0x00400000u - r : r;
  const float x = (float)r * 3.7450702e-07f;  // (pi/2) / 2^22
  const float x2 = x * x;
  float c = -6.427432595e-07f;
  c = fmaf(c, x2, 2.528363802e-05f);
  c = fmaf(c, x2, -1.389097422e-03f);
  c = fmaf(c, x2, 4.166670144e-02f);
  c = fmaf(c, x2, -5.000000000e-01f);
  const float cs = fmaf(x2, c, 1.f);
  float s = 7.040334538e-08f;
  s = fmaf(s, x2, 2.631227289e-06f);
  s = fmaf(s, x2, -1.983589609e-04f);
  s = fmaf(s, x2, 8.333324455e-03f);
  s = fmaf(s, x2, -1.666666716e-01f);
  const float x3 = x2 * x;
  const float sn = fmaf(x3, s, x);
  const float cq = comp ? sn : cs;  // cos of the in-quadrant angle
  const float sq = comp ? cs : sn;  // sin of it
  switch (quad) {
    case 0: return cq;
    case 1: return -sq;
    case 2: return -cq;
    default: return sq;
  }
}
// N(0, 1) from two Philox words (Box-Muller, cosine branch)
PGA_HD float gauss_z(uint32_t w1, uint32_t w2) {
  const float s = -2.f * det_ln_unit((w1 >> 8) + 1u);  // u1 = word_to_unit(w1) in (0, 1]
  return det_sqrt(s) * det_cos_turn((w2 >> 8) + 1u);
}

// ---- initialisation: gene 4c+j = U(lo, hi) ----
PGA_HD void real_init_chunk(const GenArgs& a, uint64_t child, uint32_t c, float v[4]) {
  const u32x4 r = draw(a.key, ST_INIT, child, c);
  v[0] = unit_range(r.x, a.lo, a.hi);
  v[1] = unit_range(r.y, a.lo, a.hi);
  v[2] = unit_range(r.z, a.lo, a.hi);
  v[3] = unit_range(r.w, a.lo, a.hi);
}

// ---- per-child plan from the misc block ----
template <bool NH = false>
PGA_HD u32x4 real_misc(const RngKey& key, uint64_t child) { return draw<NH>(key, ST_CHILD, child, 0); }
// crossover plan word: ONE/TWO_POINT lo | hi << 16 (genes [lo, hi) from B),
// ARITHMETIC the bits of u; 0 otherwise
PGA_HD uint32_t real_cut_word(const GenArgs& a, u32x4 misc) {
  const uint32_t L = a.L;
  if (a.crossover == XO_ONE_POINT) {
    return word_to_index(misc.y, L) | (L << 16);
  } else if (a.crossover == XO_TWO_POINT) {
    const uint32_t c1 = word_to_index(misc.y, L), c2 = word_to_index(misc.z, L);
    const uint32_t lo = c1 < c2 ? c1 : c2, hi = c1 < c2 ? c2 : c1;
    return lo | (hi << 16);
  } else if (a.crossover == XO_ARITHMETIC) {
    return f2u(word_to_unit(misc.y));
  } else if (a.crossover == XO_BLEND) {
    return misc.y;  // the per-gene uniforms' seed
  }
  return 0u;
}
// UNIFORM crossover: the 4 bits of chunk c (bit j = gene 4c+j from A)
template <bool NH = false>
PGA_HD uint32_t real_uniform_bits(const RngKey& key, uint64_t child, uint32_t c) {
  const uint32_t w = c >> 3;  // xo word holding genes 4c..4c+3
  return (sel4(draw<NH>(key, ST_XO, child, w >> 2), w & 3u) >> ((4u * c) & 31u)) & 0xFu;
}
// the 32 bits of genes 0..31 (every chunk of an L <= 32 genome)
template <bool NH = false>
PGA_HD uint32_t real_uniform_word0(const RngKey& key, uint64_t child) { return draw<NH>(key, ST_XO, child, 0).x; }

// ---- crossover of chunk c: genes from parents A, B ----
// cut: real_cut_word; ubits: UNIFORM bits of the chunk (real_uniform_bits)
template <bool NH = false>
PGA_HD void real_cross_chunk(const GenArgs& a, uint64_t child, uint32_t c, const float A[4], const float B[4],
                             bool xo, uint32_t cut, uint32_t ubits, float v[4]) {
  switch (xo ? a.crossover : XO_NONE) {
    case XO_UNIFORM:
      for (int j = 0; j < 4; ++j) v[j] = fsel((ubits >> j) & 1u, A[j], B[j]);
      break;
    case XO_BLEND: {  // BLX-alpha: u in [-alpha, 1 + alpha] per gene, seeded by cut (real_cut_word)
      // one 32-bit hash per gene pair, 16 bits of u each (the hash was a
      // third of the Rastrigin-30D breed step's VALU)
      const uint32_t h0 = mut_skip_word(cut, 2 * c), h1 = mut_skip_word(cut, 2 * c + 1);
      const uint32_t hw[4] = {h0 << 16, h0 & 0xFFFF0000u, h1 << 16, h1 & 0xFFFF0000u};
      for (int j = 0; j < 4; ++j) {
        const float u = fmaf(1.f + 2.f * a.blend_alpha, word_to_unit(hw[j]), -a.blend_alpha);
        v[j] = clampf(fmaf(u, B[j] - A[j], A[j]), a.lo, a.hi);
      }
      break;
    }
    case XO_ARITHMETIC: {
      const float ua = u2f(cut);
      for (int j = 0; j < 4; ++j) v[j] = fmaf(ua, B[j] - A[j], A[j]);
      break;
    }
    case XO_ONE_POINT:
    case XO_TWO_POINT: {
      const uint32_t lo = cut & 0xFFFFu, hi = cut >> 16;
      for (int j = 0; j < 4; ++j) {
        const uint32_t g = 4 * c + j;
        v[j] = fsel(g >= lo && g < hi, B[j], A[j]);
      }
      break;
    }
    default:
      for (int j = 0; j < 4; ++j) v[j] = A[j];
      break;
  }
}

// ---- mutation ----
PGA_HD bool real_per_gene_mutation(const GenArgs& a) {
  return (a.mutation == MUT_GAUSSIAN || a.mutation == MUT_UNIFORM) && a.mut_rate > 0.f;
}
// the n-th mutated gene's draw: gaussian z, or the new value (uniform / reset)
template <bool NH = false>
PGA_HD float real_mut_draw(const GenArgs& a, uint64_t child, uint32_t n) {
  const u32x4 r = draw<NH>(a.key, ST_MUTX, child, n);
  return a.mutation == MUT_GAUSSIAN ? gauss_z(r.x, r.y) : unit_range(r.z, a.lo, a.hi);
}
// applies a real_mut_draw value to the gene's current value
PGA_HD float real_mut_apply(const GenArgs& a, float d, float old) {
  return a.mutation == MUT_GAUSSIAN ? clampf(fmaf(a.sigma, d, old), a.lo, a.hi) : d;
}

// dense per-gene mutation of chunk c (clen valid genes): Bernoulli(p) per
// gene by geometric skips from r0 = draw(ST_BMUT, child, kDenseBlock + c).x
PGA_HD void real_mutate_chunk(const GenArgs& a, uint64_t child, uint32_t c, uint32_t clen, uint32_t r0,
                              const uint32_t* thr, float v[4]) {
  if (r0 < thr[kMutCap - 1]) return;  // common case: no mutation in 128 draws' worth
  uint32_t pos = geom_skip(r0, thr, kMutCap, a.mut_inv_log2_1mp);
  uint32_t n = 0;
  while (pos < clen) {
    const u32x4 r = draw(a.key, ST_MUTX, child, (c << 6) | (32u + n));
    const float old = fsel(pos == 0, v[0], fsel(pos == 1, v[1], fsel(pos == 2, v[2], v[3])));
    const float x = a.mutation == MUT_GAUSSIAN ? clampf(fmaf(a.sigma, gauss_z(r.x, r.y), old), a.lo, a.hi)
                                               : unit_range(r.z, a.lo, a.hi);
    // assign through a branch-free select (no runtime-indexed register array)
    v[0] = fsel(pos == 0, x, v[0]);
    v[1] = fsel(pos == 1, x, v[1]);
    v[2] = fsel(pos == 2, x, v[2]);
    v[3] = fsel(pos == 3, x, v[3]);
    ++n;
    pos += 1u + geom_skip(r.w, thr, kMutCap, a.mut_inv_log2_1mp);  // the value draw's spare word
  }
}

// ---- objectives ----
// Per-lane partial terms over z (already shifted/rotated), combined by a
// GS-lane butterfly.  Up to three partial accumulators.  Products that feed
// a sum are explicit fmaf, so the polynomial objectives (sphere, Rosenbrock,
// linear, knapsack) score bit for bit alike on the host and the device.
struct RealAcc {
  float s0, s1, s2;  // s2 starts at 1 for products
};

PGA_HD bool real_obj_rotatable(int32_t obj) {
  return obj == OBJ_SPHERE || obj == OBJ_RASTRIGIN || obj == OBJ_ROSENBROCK || obj == OBJ_ACKLEY ||
         obj == OBJ_GRIEWANK || obj == OBJ_SCHWEFEL;
}

// per-dimension problem data of the objectives that have any (LINEAR weight;
// KNAPSACK_REAL value w0 and weight w1) — loop-invariant per lane, so the
// fast kernel loads them once instead of inside its loop
PGA_HD void real_obj_data(const GenArgs& a, uint32_t g, float& w0, float& w1) {
  w0 = 1.f;
  w1 = 0.f;
  if (a.objective == OBJ_LINEAR) {
    w0 = a.obj_data ? a.obj_data[g] : 1.f;
  } else if (a.objective == OBJ_KNAPSACK_REAL) {
    w0 = a.obj_data[g];
    w1 = a.obj_data[a.L + g];
  }
}

// term for dimension g (z = its value, zn = value of dimension g+1 when it
// exists, w0/w1 = real_obj_data(g))
PGA_HD void real_obj_term_w(const GenArgs& a, uint32_t g, float z, float zn, float x, float w0, float w1,
                            RealAcc& acc) {
  switch (a.objective) {
    case OBJ_SPHERE: acc.s0 = fmaf(z, z, acc.s0); break;
    case OBJ_RASTRIGIN: acc.s0 += fmaf(z, z, fmaf(-10.f, cos2pi(z), 10.f)); break;
    case OBJ_ROSENBROCK:
      if (g + 1 < a.L) {
        const float t = fmaf(-z, z, zn), u = 1.f - z;
        const float uu = u * u;
        acc.s0 += fmaf(100.f * t, t, uu);
      }
      break;
    case OBJ_ACKLEY:
      acc.s0 = fmaf(z, z, acc.s0);
      acc.s1 += cos2pi(z);
      break;
    case OBJ_GRIEWANK:
      acc.s0 = fmaf(z, z, acc.s0);
      acc.s2 *= cosf(z / sqrtf((float)(g + 1)));
      break;
    case OBJ_SCHWEFEL: acc.s0 = fmaf(z, sinf(sqrtf(fabsf(z))), acc.s0); break;
    case OBJ_LINEAR: acc.s0 = fmaf(w0, x, acc.s0); break;
    case OBJ_KNAPSACK_REAL: {  // reference E2: count = (int)(g * max_count)
      const float cnt = (float)(int)(x * (float)a.obj_i);
      acc.s0 = fmaf(w0, cnt, acc.s0);
      acc.s1 = fmaf(w1, cnt, acc.s1);
      break;
    }
    default: break;
  }
}

PGA_HD void real_obj_term(const GenArgs& a, uint32_t g, float z, float zn, float x, RealAcc& acc) {
  float w0, w1;
  real_obj_data(a, g, w0, w1);
  real_obj_term_w(a, g, z, zn, x, w0, w1, acc);
}

PGA_HD float real_obj_finish(const GenArgs& a, const RealAcc& t) {
  const float D = (float)a.L;
  switch (a.objective) {
    case OBJ_SPHERE: case OBJ_RASTRIGIN: case OBJ_ROSENBROCK: return -t.s0;
    case OBJ_ACKLEY:
      return -(-20.f * expf(-0.2f * sqrtf(t.s0 / D)) - expf(t.s1 / D) + 20.f + 2.71828182845904523536f);
    case OBJ_GRIEWANK: return -(1.f + t.s0 / 4000.f - t.s2);
    case OBJ_SCHWEFEL: return -(418.9828872724339f * D - t.s0);
    case OBJ_LINEAR: return t.s0;
    case OBJ_KNAPSACK_REAL: return t.s1 <= a.obj_f0 ? t.s0 : a.obj_f0 - t.s1;
    default: return 0.f;
  }
}

// reference E3 decode: city = (int)(g * L), clamped (the reference can index L)
PGA_HD uint32_t random_key_city(float g, uint32_t L) {
  int c = (int)(g * (float)L);
  return c < 0 ? 0u : ((uint32_t)c >= L ? L - 1 : (uint32_t)c);
}

}  // namespace pga
