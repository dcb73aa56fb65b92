"""hipRTC-compiled objectives (models.JitObjective, csrc/engine/jit.cpp)."""
import pytest
import torch

import libpga_amd as pga

M = pga.models

ONEMAX_SRC = """
__device__ float ones(const unsigned int* w, unsigned int nbits, const float* data) {
  float s = 0.f;
  for (unsigned int i = 0; i < (nbits + 31) / 32; ++i) s += (float)__popc(w[i]);
  return s;
}
"""

RASTRIGIN_SRC = """
__device__ float rastrigin(const float* x, unsigned int n, const float* data) {
  float s = 10.f * n;
  for (unsigned int i = 0; i < n; ++i) s += x[i] * x[i] - 10.f * cosf(6.283185307179586f * x[i]);
  return -s;
}
"""

TSP_SRC = """
__device__ float tour(const unsigned short* p, unsigned int n, const float* d) {
  float len = 0.f;
  for (unsigned int i = 0; i < n; ++i) len += d[p[i] * n + p[(i + 1) % n]];
  return -len;
}
"""


def onemax_jit(L):
    return M.JitObjective("binary", L, ONEMAX_SRC, name="ones", fallback=lambda g: g.float().sum(-1))


def test_jit_compiles_and_reports_errors():
    k = onemax_jit(128).kernel()
    assert k.code_size > 0 and "pga_jit_eval" in k.source
    with pytest.raises(RuntimeError, match="hipRTC compile"):
        M.JitObjective("real", 4, "not c++", name="f").kernel()


def test_jit_fused_generation_object_builds_without_gpu(tmp_path, monkeypatch):
    # the fused-JIT toolchain path (user bitcode + jitgen.hip bitcode, LTO link)
    # needs no GPU: the code object holds the kernel with the objective inlined
    monkeypatch.setenv("PGA_JIT_CACHE", str(tmp_path))
    k = onemax_jit(1024).kernel()
    path = k.build_generation_object(8, True, False, 1024)
    data = open(path, "rb").read()
    assert data[:4] == b"\x7fELF"
    assert b"_ZN3pga6jitgen13binary_gen_tpILi8ELi1001ELb1ELb0EEEvNS_7GenArgsEPy" in data
    assert b"pga_user_objective" not in data  # inlined, no call left
    assert k.build_generation_object(8, True, False, 1024) == path  # cached
    with pytest.raises(ValueError, match="power of two"):
        k.build_generation_object(3, True, False, 1024)


def test_jit_cpu_uses_fallback():
    ga = pga.GeneticAlgorithm(onemax_jit(96), 200, seed=1, device="cpu")
    assert torch.equal(ga.scores, ga.genomes().float().sum(-1))
    s0 = ga.best_score()
    ga.run(10)
    assert ga.best_score() > s0
    with pytest.raises(ValueError, match="JIT objective needs a GPU"):
        pga.GeneticAlgorithm(M.JitObjective("binary", 8, ONEMAX_SRC, name="ones"), 10, device="cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("L,kw,S", [(1024, {}, 1 << 16), (777, {}, 1 << 16), (1024, dict(mutation_rate=0.02), 1 << 16),
                                    (300, dict(selection="rank"), 1 << 16),
                                    # LDS staging: one step per objective pass (GS 1), 32-lane rows
                                    (32, {}, 1 << 16), (4096, {}, 1 << 14),
                                    # the headline geometry (16-wave blocks, XCD skew), a partial last unit
                                    (1024, {}, 1 << 20), (1024, {}, 100003)])
def test_jit_onemax_bit_identical_to_builtin(L, kw, S):
    # the objective is linked into the hot generation kernel (one launch per
    # generation): rows, scores and best equal the built-in OneMax bit for bit
    a = pga.GeneticAlgorithm(M.OneMax(L), S, seed=4, device="cuda:0", elitism=1, **kw)
    b = pga.GeneticAlgorithm(onemax_jit(L), S, seed=4, device="cuda:0", elitism=1, **kw)
    assert b.island.has_jit
    for _ in range(3):
        a.run(7)
        b.run(7)
        torch.cuda.synchronize()
        assert torch.equal(a.rows, b.rows)
        assert torch.equal(a.scores, b.scores)
        assert a.best_score() == b.best_score()
    assert b.island.jit_fused_error == ""
    assert b.island.jit_fused_generations >= 20


WEIGHTED_SRC = """
__device__ float wsum(const unsigned int* w, unsigned int nbits, const float* data) {
  float s = 0.f;
  for (unsigned int i = 0; i < nbits; ++i) s += ((w[i >> 5] >> (i & 31)) & 1u) ? data[i] : 0.f;
  return s;
}
"""


@pytest.mark.gpu
def test_jit_fused_objective_with_data_matches_oracle():
    L = 200
    wts = torch.randn(L, generator=torch.Generator().manual_seed(3))
    p = M.JitObjective("binary", L, WEIGHTED_SRC, name="wsum", data=wts)
    ga = pga.GeneticAlgorithm(p, 1 << 14, seed=5, device="cuda:0", elitism=1)
    s0 = ga.best_score()
    ga.run(15)
    torch.cuda.synchronize()
    assert ga.island.jit_fused_generations >= 15, ga.island.jit_fused_error
    ref = (ga.genomes().float() * wts.to(ga.genomes().device)).sum(-1)
    assert torch.allclose(ref, ga.scores, rtol=1e-4, atol=1e-3)
    assert ga.best_score() > s0


@pytest.mark.gpu
def test_jit_rastrigin_and_tsp_match_oracles():
    p = M.JitObjective("real", 30, RASTRIGIN_SRC, name="rastrigin", bounds=(-5.12, 5.12),
                       fallback=lambda g: M.Rastrigin(30).reference_fitness(g))
    ga = pga.GeneticAlgorithm(p, 1 << 15, seed=2, device="cuda:0", elitism=1)
    ga.run(20)
    torch.cuda.synchronize()
    ref = M.Rastrigin(30).reference_fitness(ga.genomes())
    assert torch.allclose(ref, ga.scores, rtol=2e-4, atol=2e-3)
    d = torch.rand(48, 48, generator=torch.Generator().manual_seed(0))
    q = M.JitObjective("permutation", 48, TSP_SRC, name="tour", data=d.reshape(-1))
    t = pga.GeneticAlgorithm(q, 4096, seed=1, device="cuda:0", elitism=1)
    t0 = t.best_score()
    t.run(30)
    torch.cuda.synchronize()
    ref = M.TSP(d).reference_fitness(t.genomes())
    assert torch.allclose(ref, t.scores, rtol=1e-4, atol=1e-3)
    assert t.best_score() > t0


@pytest.mark.gpu
def test_jit_fusion_unavailable_falls_back(monkeypatch):
    # no generation-kernel bitcode: the island says why and evaluates with the
    # separate hipRTC pass instead, with the same results
    monkeypatch.setenv("PGA_JIT_DIR", "/nonexistent/pga_jit")
    L, S = 512, 1 << 13
    a = pga.GeneticAlgorithm(M.OneMax(L), S, seed=9, device="cuda:0", elitism=1)
    b = pga.GeneticAlgorithm(onemax_jit(L), S, seed=9, device="cuda:0", elitism=1)
    a.run(6)
    b.run(6)
    torch.cuda.synchronize()
    assert b.island.jit_fused_generations == 0
    assert "no generation-kernel bitcode" in b.island.jit_fused_error
    assert torch.equal(a.rows, b.rows) and torch.equal(a.scores, b.scores)


QUAD_SRC = """
__device__ float quad(const float* x, unsigned int n, const float* d) {
  float s = 0.f;
  for (unsigned int i = 0; i < n; ++i) { const float t = x[i] - d[i]; s += t * t; }
  return -s;
}
"""


def test_jit_real_fused_generation_object_builds_without_gpu(tmp_path, monkeypatch):
    # REAL (the reference's float genes): jitgen_real.hip bitcode + the user's
    monkeypatch.setenv("PGA_JIT_CACHE", str(tmp_path))
    k = M.JitObjective("real", 30, RASTRIGIN_SRC, name="rastrigin", bounds=(-5.12, 5.12)).kernel()
    path = k.build_generation_object(8, False, False, 30)
    data = open(path, "rb").read()
    assert data[:4] == b"\x7fELF"
    assert b"_ZN3pga6jitgen11real_gen_tpILi8ELi1001ELb0EEEvNS_7GenArgsEPy" in data
    assert b"pga_user_objective_f32" not in data  # inlined, no call left


def test_jit_cache_must_be_private(tmp_path, monkeypatch):
    import os
    d = tmp_path / "shared"
    d.mkdir()
    os.chmod(d, 0o777)
    monkeypatch.setenv("PGA_JIT_CACHE", str(d))
    k = onemax_jit(256).kernel()
    with pytest.raises(RuntimeError, match="not private"):
        k.build_generation_object(2, True, False, 256)


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1 << 18, 20000])
def test_jit_real_fused_equals_separate_pass(S, monkeypatch):
    """A float-gene source objective fused into real_gen_tp (one launch per
    generation) against the separate evaluation pass: the first generation's
    children are bit-identical (both select on the same initial scores), its
    scores agree to float rounding (two compilations of the objective), and
    the fused run keeps matching the fp32 torch oracle."""
    L = 30
    tgt = torch.linspace(-1, 1, L)
    # the unfused twin gets its own kernel (a different source text, same
    # function) so that no fused variant is cached for it
    mk = lambda tag: M.JitObjective("real", L, QUAD_SRC + tag, name="quad", data=tgt, bounds=(-2.0, 2.0))
    a = pga.GeneticAlgorithm(mk(""), S, seed=6, device="cuda:0", elitism=1)
    a.run(1)
    torch.cuda.synchronize()
    assert a.island.jit_fused_generations == 1, a.island.jit_fused_error
    monkeypatch.setenv("PGA_JIT_DIR", "/nonexistent/pga_jit")
    b = pga.GeneticAlgorithm(mk(f"// unfused {S}\n"), S, seed=6, device="cuda:0", elitism=1)
    b.run(1)
    torch.cuda.synchronize()
    assert b.island.jit_fused_generations == 0
    assert torch.equal(a.rows, b.rows)
    assert torch.allclose(a.scores, b.scores, rtol=1e-6, atol=1e-6)
    a.run(7)
    torch.cuda.synchronize()
    assert a.island.jit_fused_generations == 8
    ref = -((a.genomes().float().cpu() - tgt) ** 2).sum(-1)
    assert torch.allclose(ref, a.scores.cpu(), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_jit_variant_key_distinguishes_lengths():
    # 5000 and 5001 bits share a group size of 64 lanes: one JitKernel (same
    # source) used at both lengths must compile two variants
    src = ONEMAX_SRC + "// variant-key test\n"  # its own kernel: another test's failed fusion is cached per kernel
    for L in (5000, 5001):
        a = pga.GeneticAlgorithm(M.OneMax(L), 4096, seed=3, device="cuda:0", elitism=1)
        b = pga.GeneticAlgorithm(M.JitObjective("binary", L, src, name="ones"), 4096, seed=3, device="cuda:0",
                                 elitism=1)
        a.run(3)
        b.run(3)
        torch.cuda.synchronize()
        assert b.island.jit_fused_generations >= 3, b.island.jit_fused_error
        assert torch.equal(a.rows, b.rows) and torch.equal(a.scores, b.scores)


SCALED_SRC = """
#ifndef SCALE
#define SCALE 1.0f
#endif
__device__ float scaled(const unsigned int* w, unsigned int nbits, const float* data) {
  float s = 0.f;
  for (unsigned int i = 0; i < (nbits + 31) / 32; ++i) s += (float)__popc(w[i]);
  return SCALE * s;
}
"""


@pytest.mark.gpu
def test_jit_options_reach_fused_kernel():
    # -DSCALE=3.0f applies to the fused generation kernel as to the init pass
    p = M.JitObjective("binary", 256, SCALED_SRC, name="scaled", options=["-DSCALE=3.0f"])
    ga = pga.GeneticAlgorithm(p, 1 << 14, seed=2, device="cuda:0", elitism=1)
    ga.run(5)
    torch.cuda.synchronize()
    assert ga.island.jit_fused_generations >= 5, ga.island.jit_fused_error
    assert torch.equal(ga.scores, 3.0 * ga.genomes().float().sum(-1))
