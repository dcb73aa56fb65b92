"""The reference-compatible C API (include/pga.h + pga_ext.h, build/libpga.so).

CPU tests drive libpga.so through ctypes on the CPU reference backend
(device -1) with built-in objectives; GPU tests run the rewritten reference
examples E1/E2/E3 (user __device__ callbacks, linked from libpga.a with
-fgpu-rdc) and the plain-C headline example."""
import ctypes as C
import json
import os
import subprocess

import pytest
import torch  # noqa: F401  (loads the HIP runtime the library links against)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "build", "libpga.so")
EX = os.path.join(ROOT, "build", "examples")

PGA_REAL, PGA_BINARY, PGA_PERM = 1, 0, 2


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.skip("build/libpga.so not built (python tools/build.py)")
    L = C.CDLL(LIB)
    vp = C.c_void_p
    L.pga_init_device.restype = vp
    L.pga_init_device.argtypes = [C.c_int]
    L.pga_deinit.argtypes = [vp]
    L.pga_set_seed.argtypes = [vp, C.c_uint64]
    L.pga_set_quiet.argtypes = [vp, C.c_int]
    L.pga_set_abort_on_error.argtypes = [vp, C.c_int]
    L.pga_last_error.restype = C.c_char_p
    L.pga_create_population.restype = vp
    L.pga_create_population.argtypes = [vp, C.c_ulong, C.c_uint, C.c_int]
    L.pga_create_population_ext.restype = vp
    L.pga_create_population_ext.argtypes = [vp, C.c_ulong, C.c_uint, C.c_int]
    L.pga_set_objective_builtin.argtypes = [vp, vp, C.c_int, C.POINTER(C.c_float), C.c_size_t,
                                            C.POINTER(C.c_float), C.c_size_t, C.c_int, C.c_float, C.c_float]
    L.pga_set_operators.argtypes = [vp, vp, C.c_int, C.c_uint, C.c_int, C.c_float, C.c_int, C.c_float, C.c_float,
                                    C.c_uint]
    L.pga_set_bounds.argtypes = [vp, vp, C.c_float, C.c_float]
    for f in ("pga_evaluate", "pga_mutate", "pga_swap_generations", "pga_fill_random_values"):
        getattr(L, f).argtypes = [vp, vp]
    L.pga_crossover.argtypes = [vp, vp, C.c_int]
    L.pga_evaluate_all.argtypes = [vp]
    L.pga_mutate_all.argtypes = [vp]
    L.pga_crossover_all.argtypes = [vp, C.c_int]
    L.pga_run.argtypes = [vp, C.c_uint]
    L.pga_run_islands.argtypes = [vp, C.c_uint, C.c_uint, C.c_float]
    L.pga_migrate.argtypes = [vp, C.c_float]
    L.pga_migrate_between.argtypes = [vp, vp, vp, C.c_float]
    L.pga_get_best.restype = C.POINTER(C.c_float)
    L.pga_get_best.argtypes = [vp, vp]
    L.pga_get_best_all.restype = C.POINTER(C.c_float)
    L.pga_get_best_all.argtypes = [vp]
    L.pga_get_best_top.restype = C.POINTER(C.POINTER(C.c_float))
    L.pga_get_best_top.argtypes = [vp, vp, C.c_uint]
    L.pga_get_best_top_all.restype = C.POINTER(C.POINTER(C.c_float))
    L.pga_get_best_top_all.argtypes = [vp, C.c_uint]
    L.pga_best_score.restype = C.c_float
    L.pga_best_score.argtypes = [vp, vp]
    L.pga_get_scores.argtypes = [vp, vp, C.POINTER(C.c_float)]
    L.pga_stats.argtypes = [vp, vp, C.POINTER(C.c_float)]
    L.pga_generation.argtypes = [vp]
    L.pga_save.argtypes = [vp, vp, C.c_char_p]
    L.pga_load.argtypes = [vp, vp, C.c_char_p]
    L.pga_set_objective_source.argtypes = [vp, vp, C.c_char_p, C.c_char_p, C.POINTER(C.c_float), C.c_size_t]
    L.pga_run_until.argtypes = [vp, C.c_uint, C.c_float, C.c_uint]
    L.pga_set_migration_policy.argtypes = [vp, vp, C.c_int]
    L.pga_run_islands_until.argtypes = [vp, C.c_uint, C.c_uint, C.c_float, C.c_float]
    L.pga_set_stats_history.argtypes = [vp, vp, C.c_int]
    L.pga_set_batch_islands.argtypes = [vp, C.c_int]
    L.pga_batched_generations.restype = C.c_ulonglong
    L.pga_batched_generations.argtypes = [vp]
    L.pga_get_stats_history.restype = C.c_long
    L.pga_get_stats_history.argtypes = [vp, vp, C.POINTER(C.c_float), C.c_ulong]
    L.free_ = C.CDLL(None).free
    L.free_.argtypes = [vp]
    return L


def fptr(vals):
    arr = (C.c_float * len(vals))(*vals)
    return arr


def new(lib, seed=1):
    p = lib.pga_init_device(-1)
    assert p
    lib.pga_set_seed(p, seed)
    lib.pga_set_quiet(p, 1)
    lib.pga_set_abort_on_error(p, 0)
    return p


def test_create_limits(lib):
    p = new(lib)
    assert not lib.pga_create_population(p, 100, 3, 0)  # genome_len < 4 -> NULL
    pops = [lib.pga_create_population(p, 10, 8, 0) for _ in range(10)]
    assert all(pops)
    assert not lib.pga_create_population(p, 10, 8, 0)  # MAX_POPULATIONS
    lib.pga_deinit(p)


def test_reference_knapsack_builtin(lib):
    """E2 through the C API with the built-in reference knapsack objective."""
    p = new(lib, seed=3)
    pop = lib.pga_create_population(p, 100, 6, 0)
    data = fptr([75, 150, 250, 35, 10, 100, 7, 8, 6, 4, 3, 9])
    assert lib.pga_set_objective_builtin(p, pop, 23, data, 12, None, 0, 2, 10.0, 0.0) == 0
    lib.pga_run(p, 5)
    g = lib.pga_get_best(p, pop)
    counts = [int(g[i] * 2) for i in range(6)]
    lib.free_(g)
    assert lib.pga_best_score(p, pop) == 285.0
    assert counts == [0, 0, 1, 1, 0, 0]
    lib.pga_deinit(p)


def test_stages_and_queries(lib):
    p = new(lib, seed=5)
    pop = lib.pga_create_population(p, 300, 20, 0)
    lib.pga_set_objective_builtin(p, pop, 22, None, 0, None, 0, 0, 0.0, 0.0)  # sum of genes (E1)
    lib.pga_evaluate(p, pop)
    s0 = lib.pga_best_score(p, pop)
    for _ in range(10):
        lib.pga_fill_random_values(p, pop)
        lib.pga_evaluate(p, pop)
        lib.pga_crossover(p, pop, 0)
        lib.pga_mutate(p, pop)
        lib.pga_swap_generations(p, pop)
    lib.pga_evaluate(p, pop)
    assert lib.pga_generation(pop) == 10
    assert lib.pga_best_score(p, pop) > s0
    sc = (C.c_float * 300)()
    assert lib.pga_get_scores(p, pop, sc) == 0
    assert max(sc) == lib.pga_best_score(p, pop)
    st = (C.c_float * 4)()
    lib.pga_stats(p, pop, st)
    assert st[1] == max(sc) and abs(st[2] / st[3] - sum(sc) / 300) < 1e-3
    top = lib.pga_get_best_top(p, pop, 5)
    sums = [sum(top[i][j] for j in range(20)) for i in range(5)]
    assert sums == sorted(sums, reverse=True)
    assert abs(sums[0] - max(sc)) < 1e-3
    for i in range(5):
        lib.free_(top[i])
    lib.free_(top)
    lib.pga_deinit(p)


def test_islands_and_migration(lib):
    p = new(lib, seed=7)
    pops = [lib.pga_create_population(p, 200, 16, 0) for _ in range(4)]
    for pop in pops:
        lib.pga_set_objective_builtin(p, pop, 22, None, 0, None, 0, 0, 0.0, 0.0)
    lib.pga_evaluate_all(p)
    best = [lib.pga_best_score(p, pop) for pop in pops]
    src = max(range(4), key=lambda i: best[i])
    dst = min(range(4), key=lambda i: best[i])
    lib.pga_migrate_between(p, pops[src], pops[dst], 0.05)
    assert lib.pga_best_score(p, pops[dst]) == best[src]
    lib.pga_run_islands(p, 30, 5, 10.0)  # percent form
    b = lib.pga_get_best_all(p)
    total = sum(b[j] for j in range(16))
    lib.free_(b)
    assert abs(total - max(lib.pga_best_score(p, pop) for pop in pops)) < 1e-3
    tops = lib.pga_get_best_top_all(p, 3)
    vals = [sum(tops[i][j] for j in range(16)) for i in range(3)]
    assert vals == sorted(vals, reverse=True)
    lib.pga_migrate(p, 0.1)
    lib.pga_deinit(p)


def test_binary_and_checkpoint(lib, tmp_path):
    p = new(lib, seed=11)
    pop = lib.pga_create_population_ext(p, 512, 64, PGA_BINARY)
    lib.pga_set_objective_builtin(p, pop, 1, None, 0, None, 0, 0, 0.0, 0.0)
    lib.pga_set_operators(p, pop, 0, 2, 2, 1.0, 0, -1.0, 0.0, 1)
    lib.pga_run(p, 5)
    path = str(tmp_path / "pop.ckpt").encode()
    assert lib.pga_save(p, pop, path) == 0
    lib.pga_run(p, 30)
    assert lib.pga_best_score(p, pop) == 64.0
    q = new(lib, seed=11)
    pop2 = lib.pga_create_population_ext(q, 512, 64, PGA_BINARY)
    lib.pga_set_objective_builtin(q, pop2, 1, None, 0, None, 0, 0, 0.0, 0.0)
    lib.pga_set_operators(q, pop2, 0, 2, 2, 1.0, 0, -1.0, 0.0, 1)
    assert lib.pga_load(q, pop2, path) == 0
    assert lib.pga_generation(pop2) == 5
    lib.pga_deinit(p)
    lib.pga_deinit(q)


def onemax_pop(lib, p, S=512, L=64):
    pop = lib.pga_create_population_ext(p, S, L, PGA_BINARY)
    lib.pga_set_objective_builtin(p, pop, 1, None, 0, None, 0, 0, 0.0, 0.0)
    lib.pga_set_operators(p, pop, 0, 2, 2, 1.0, 0, -1.0, 0.0, 1)
    return pop


def test_run_until_target(lib):
    """pga_run_until stops at the first check point whose best reaches the
    target (reference include/pga.h: "until n-generations or
    obj_func(best_genome) == value"); the same seed run to the reported
    generation count reaches it too."""
    p = new(lib, seed=5)
    pop = onemax_pop(lib, p)
    g = lib.pga_run_until(p, 500, 64.0, 5)
    assert 0 < g < 500 and g % 5 == 0
    assert lib.pga_best_score(p, pop) == 64.0
    assert lib.pga_generation(pop) == g
    # checked every 5: the target was not yet reached 5 generations earlier
    q = new(lib, seed=5)
    pop2 = onemax_pop(lib, q)
    lib.pga_run(q, g - 5)
    assert lib.pga_best_score(q, pop2) < 64.0
    # an unreachable target runs every generation
    assert lib.pga_run_until(q, 7, 1e9, 3) == 7
    lib.pga_deinit(p)
    lib.pga_deinit(q)


def test_run_islands_until_target(lib):
    p = new(lib, seed=6)
    pops = [onemax_pop(lib, p, S=256) for _ in range(3)]
    g = lib.pga_run_islands_until(p, 400, 10, 0.05, 64.0)
    assert 0 < g < 400 and g % 10 == 0
    assert max(lib.pga_best_score(p, q) for q in pops) == 64.0
    lib.pga_deinit(p)


@pytest.mark.parametrize("policy", [0, 1])  # PGA_MIGRATE_TOPK, PGA_MIGRATE_STRIPE
def test_migrate_between_policies(lib, policy):
    """Both policies move the source's best into the destination and replace
    only worse individuals: the destination's best becomes the source's, its
    score multiset changes by exactly k entries."""
    p = new(lib, seed=12)
    a, b = onemax_pop(lib, p, S=400), onemax_pop(lib, p, S=400)
    for q in (a, b):
        assert lib.pga_set_migration_policy(p, q, policy) == 0
    lib.pga_run(p, 3)
    sa, sb = (C.c_float * 400)(), (C.c_float * 400)()
    lib.pga_get_scores(p, a, sa)
    lib.pga_get_scores(p, b, sb)
    before = sorted(sb)
    lib.pga_migrate_between(p, a, b, 0.05)  # k = 20
    lib.pga_get_scores(p, b, sb)
    assert max(sb) == max(max(sa), before[-1])
    gone = sum(1 for x, y in zip(sorted(sb), before) if x != y)
    assert 0 < gone <= 20 and sum(sb) >= sum(before)
    assert lib.pga_set_migration_policy(p, a, 7) == -1  # unknown policy refused
    lib.pga_deinit(p)


def test_stats_history(lib):
    """Per-generation {min, max, sum, count} rows equal pga_stats taken after
    each generation."""
    p = new(lib, seed=7)
    pop = onemax_pop(lib, p)
    assert lib.pga_set_stats_history(p, pop, 1) == 0
    ref = []
    out4 = (C.c_float * 4)()
    for _ in range(6):
        lib.pga_run(p, 1)
        lib.pga_stats(p, pop, out4)
        ref.append(list(out4))
    buf = (C.c_float * 40)()
    assert lib.pga_get_stats_history(p, pop, buf, 10) == 6
    rows = [list(buf[4 * i:4 * i + 4]) for i in range(6)]
    assert rows == ref
    assert lib.pga_set_stats_history(p, pop, 1) == 0  # restart clears
    assert lib.pga_get_stats_history(p, pop, None, 0) == 0
    lib.pga_deinit(p)


def run_ex(args, inp=None, timeout=300):
    # a fixed seed: pga_init otherwise seeds from time(NULL) like the reference
    env = dict(os.environ)
    env.setdefault("PGA_SEED", "20261017")
    r = subprocess.run(args, input=inp, capture_output=True, text=True, timeout=timeout, env=env)
    return r.returncode, r.stdout + r.stderr


@pytest.mark.gpu
def test_example_e1_user_objective():
    rc, out = run_ex([os.path.join(EX, "e1_onemax_float"), "100"])
    assert rc == 0, out


@pytest.mark.gpu
def test_example_e1_fnptr_two_phase_matches_generic():
    """The reference user model (a __device__ obj_f function pointer) runs on
    the two-phase kernel at E1's size (test/test.cu:22-43: S = 40,000,
    L = 100); the generic kernel (forced by a population threshold above S)
    calls the same function on the same rows, so every score is identical."""
    def run(extra):
        env = dict(os.environ, PGA_SEED="77", **extra)
        r = subprocess.run([os.path.join(EX, "e1_onemax_float"), "30"], capture_output=True, text=True,
                           timeout=300, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        h = [ln for ln in r.stdout.splitlines() if ln.startswith("E1 scores hash")]
        t = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
        return h[0], t[0]["e1_fnptr_us_per_gen"]
    h_tp, us_tp = run({})
    h_gen, us_gen = run({"PGA_TP_MIN_S": "1000000000"})
    assert h_tp == h_gen
    print(f"E1 fn-ptr: two-phase {us_tp:.1f} us/gen, generic {us_gen:.1f} us/gen")


@pytest.mark.gpu
def test_example_e1_callbacks_4m():
    """User objective + user mutation (the reference-ABI callback kernel) on
    4M individuals: every score must be a real evaluation (grid-stride)."""
    rc, out = run_ex([os.path.join(EX, "e1_onemax_float"), "60", str(4 << 20), "cb"])
    assert rc == 0, out


@pytest.mark.gpu
def test_example_e2_knapsack():
    rc, out = run_ex([os.path.join(EX, "e2_knapsack"), "40"])
    assert rc == 0, out
    assert "0 0 1 1 0 0" in out


@pytest.mark.gpu
def test_example_e3_tsp_user_crossover():
    inst = subprocess.run([os.path.join(EX, "gen_tsp"), "30", "3"], capture_output=True, text=True).stdout
    rc, out = run_ex([os.path.join(EX, "e3_tsp"), "300"], inp=inst)
    assert rc == 0, out
    assert "duplicates: 0" in out


@pytest.mark.gpu
def test_example_onemax_bits_c():
    rc, out = run_ex([os.path.join(EX, "onemax_bits"), "65536", "100"])
    assert rc == 0, out


def test_objective_source_cpu_is_refused(lib):
    p = new(lib)
    pop = lib.pga_create_population_ext(p, 64, 64, PGA_BINARY)
    src = b"__device__ float f(const unsigned int* w, unsigned int n, const float* d) { return 0.f; }"
    assert lib.pga_set_objective_source(p, pop, src, b"f", None, 0) == -1
    assert b"GPU" in lib.pga_last_error()
    lib.pga_deinit(p)


@pytest.mark.gpu
def test_objective_source_gpu(lib):
    """pga_set_objective_source: hipRTC OneMax equals the built-in OneMax run for run."""
    src = (b"__device__ float ones(const unsigned int* w, unsigned int n, const float* d) {"
           b" float s = 0.f; for (unsigned i = 0; i < (n + 31) / 32; ++i) s += __popc(w[i]); return s; }")
    best = []
    for jit in (False, True):
        p = lib.pga_init_device(0)
        lib.pga_set_seed(p, 9)
        lib.pga_set_quiet(p, 1)
        lib.pga_set_abort_on_error(p, 0)
        pop = lib.pga_create_population_ext(p, 4096, 512, PGA_BINARY)
        if jit:
            assert lib.pga_set_objective_source(p, pop, src, b"ones", None, 0) == 0, lib.pga_last_error()
        else:
            assert lib.pga_set_objective_builtin(p, pop, 1, None, 0, None, 0, 0, 0.0, 0.0) == 0
        lib.pga_run(p, 25)
        scores = (C.c_float * 4096)()
        assert lib.pga_get_scores(p, pop, scores) == 0
        best.append(list(scores))
        lib.pga_deinit(p)
    assert best[0] == best[1]


@pytest.mark.gpu
def test_run_islands_batched_launch_matches_streams(lib):
    """pga_run_islands: same-shape BINARY populations run as ONE launch per
    generation (island = grid y) and evolve exactly as on their own streams."""
    def run(batched):
        p = lib.pga_init_device(0)
        lib.pga_set_seed(p, 5)
        lib.pga_set_quiet(p, 1)
        lib.pga_set_abort_on_error(p, 0)
        assert lib.pga_set_batch_islands(p, batched) == 0
        pops = [lib.pga_create_population_ext(p, 4096, 256, PGA_BINARY) for _ in range(4)]
        for pop in pops:
            assert lib.pga_set_objective_builtin(p, pop, 1, None, 0, None, 0, 0, 0.0, 0.0) == 0
        lib.pga_run_islands(p, 25, 5, 0.02)
        out = []
        for pop in pops:
            sc = (C.c_float * 4096)()
            lib.pga_get_scores(p, pop, sc)
            out.append(list(sc))
        n = lib.pga_batched_generations(p)
        lib.pga_deinit(p)
        return out, n

    a, na = run(1)
    b, nb = run(0)
    assert na == 25 and nb == 0
    assert a == b
