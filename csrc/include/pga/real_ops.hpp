// real_ops.hpp — per-gene semantics of the REAL (f32) encoding, shared by the
// gfx950 kernels (csrc/kernels/real.hip) and the CPU reference backend
// (csrc/cpu/cpu_real.cpp).  A chunk is 4 consecutive genes (16 bytes).
//
// Reference parity: the reference's only genome type is f32 (include/pga.h:29)
// with uniform crossover "rand > 0.5 ? p1 : p2" (src/pga.cu:135-143) and a
// single-gene reset mutation with p = 0.01 per individual (src/pga.cu:127-133);
// both are XO_UNIFORM / MUT_RESET_ONE here, with independent random streams.
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

// ---- initialisation: gene 4c+j = U(lo, hi) ----
PGA_HD void real_init_chunk(const GenArgs& a, uint64_t child, uint32_t c, float v[4]) {
  const u32x4 r = draw(a.key, ST_INIT, child, c);
  v[0] = unit_range(r.x, a.lo, a.hi);
  v[1] = unit_range(r.y, a.lo, a.hi);
  v[2] = unit_range(r.z, a.lo, a.hi);
  v[3] = unit_range(r.w, a.lo, a.hi);
}

// ---- crossover of chunk c: genes from parents A, B ----
// plan: blo/bhi = gene range taken from B (ONE/TWO_POINT); ua = arithmetic u
PGA_HD void real_cross_chunk(const GenArgs& a, uint64_t child, uint32_t c, const float A[4], const float B[4],
                             bool xo, uint32_t blo, uint32_t bhi, float ua, float v[4]) {
  if (!xo) {
    for (int j = 0; j < 4; ++j) v[j] = A[j];
    return;
  }
  switch (a.crossover) {
    case XO_UNIFORM: {
      const uint32_t m = draw(a.key, ST_XO, child, c).x;  // low 4 bits: 1 = parent A
      for (int j = 0; j < 4; ++j) v[j] = fsel((m >> j) & 1u, A[j], B[j]);
      break;
    }
    case XO_BLEND: {  // BLX-alpha: u in [-alpha, 1 + alpha] per gene
      const u32x4 r = draw(a.key, ST_XO, child, c);
      const uint32_t w[4] = {r.x, r.y, r.z, r.w};
      for (int j = 0; j < 4; ++j) {
        const float u = fmaf(1.f + 2.f * a.blend_alpha, word_to_unit(w[j]), -a.blend_alpha);
        v[j] = clampf(fmaf(u, B[j] - A[j], A[j]), a.lo, a.hi);
      }
      break;
    }
    case XO_ARITHMETIC:
      for (int j = 0; j < 4; ++j) v[j] = fmaf(ua, B[j] - A[j], A[j]);
      break;
    default:  // ONE_POINT / TWO_POINT over gene indices
      for (int j = 0; j < 4; ++j) {
        const uint32_t g = 4 * c + j;
        v[j] = fsel(g >= blo && g < bhi, B[j], A[j]);
      }
      break;
  }
}

// ---- mutation of chunk c (clen valid genes): Bernoulli(p) per gene ----
// first draw r0 = chunk_mut_word; n-th mutated gene's values come from
// ST_MUTX block (c << 6) | (32 + n): words 0,1 -> Box-Muller normal, 2 -> uniform, 3 -> next skip
PGA_HD void real_mutate_chunk(const GenArgs& a, uint64_t child, uint32_t c, uint32_t clen, uint32_t r0,
                              const uint32_t* thr, float v[4]) {
  if (r0 < thr[kMutCap - 1]) return;  // common case: no mutation in 128 draws' worth
  uint32_t pos = geom_skip(r0, thr, kMutCap, a.mut_inv_log2_1mp);
  uint32_t n = 0;
  while (pos < clen) {
    const u32x4 r = draw(a.key, ST_MUTX, child, (c << 6) | (32u + n));
    float x;
    if (a.mutation == MUT_GAUSSIAN) {
      const float u1 = word_to_unit(r.x), u2 = word_to_unit(r.y);
      const float z = sqrtf(-2.f * logf(u1)) * cosf(2.f * kPi * u2);
      const float old = fsel(pos == 0, v[0], fsel(pos == 1, v[1], fsel(pos == 2, v[2], v[3])));
      x = clampf(fmaf(a.sigma, z, old), a.lo, a.hi);
    } else {
      x = unit_range(r.z, a.lo, a.hi);
    }
    // assign through a branch-free select (no runtime-indexed register array)
    v[0] = fsel(pos == 0, x, v[0]);
    v[1] = fsel(pos == 1, x, v[1]);
    v[2] = fsel(pos == 2, x, v[2]);
    v[3] = fsel(pos == 3, x, v[3]);
    ++n;
    pos += 1u + geom_skip(r.w, thr, kMutCap, a.mut_inv_log2_1mp);  // the value draw's spare word
  }
}

// RESET_ONE (reference default): gene `pos` <- U(lo, hi) from child word W_MUTPOS+1
PGA_HD float real_reset_value(const GenArgs& a, uint32_t w) { return unit_range(w, a.lo, a.hi); }

// ---- objectives ----
// Per-lane partial terms over z (already shifted/rotated), combined by a
// GS-lane butterfly.  Up to three partial accumulators.
struct RealAcc {
  float s0, s1, s2;  // s2 starts at 1 for products
};

PGA_HD bool real_obj_rotatable(int32_t obj) {
  return obj == OBJ_SPHERE || obj == OBJ_RASTRIGIN || obj == OBJ_ROSENBROCK || obj == OBJ_ACKLEY ||
         obj == OBJ_GRIEWANK || obj == OBJ_SCHWEFEL;
}

// per-dimension problem data of the objectives that have any (LINEAR weight;
// KNAPSACK_REAL value w0 and weight w1) — loop-invariant per lane, so the
// pipelined kernel loads them once instead of inside its loop
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
    case OBJ_SPHERE: acc.s0 += z * z; break;
    case OBJ_RASTRIGIN: acc.s0 += z * z - 10.f * cos2pi(z) + 10.f; break;
    case OBJ_ROSENBROCK:
      if (g + 1 < a.L) {
        const float t = zn - z * z, u = 1.f - z;
        acc.s0 += 100.f * t * t + u * u;
      }
      break;
    case OBJ_ACKLEY:
      acc.s0 += z * z;
      acc.s1 += cos2pi(z);
      break;
    case OBJ_GRIEWANK:
      acc.s0 += z * z;
      acc.s2 *= cosf(z / sqrtf((float)(g + 1)));
      break;
    case OBJ_SCHWEFEL: acc.s0 += z * sinf(sqrtf(fabsf(z))); break;
    case OBJ_LINEAR: acc.s0 += w0 * x; break;
    case OBJ_KNAPSACK_REAL: {  // reference E2: count = (int)(g * max_count)
      const float cnt = (float)(int)(x * (float)a.obj_i);
      acc.s0 += w0 * cnt;
      acc.s1 += w1 * cnt;
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
