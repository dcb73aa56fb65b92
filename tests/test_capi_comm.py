"""Inter-rank island model of the C API (pga_comm_*, csrc/capi/comm*.cpp).

CPU tests drive several solvers of the CPU reference backend through the
loopback transport (the same migration plans and protocol as RCCL: ring,
random ring, all-to-all; re-scoring of received migrants; fault injection
and degraded mode).  GPU tests run the loopback between GPU solvers and the
one-process RCCL transport (ncclCommInitAll) on the box's device.

Reference: the migration entry points are empty stubs
(src/pga.cu:368-374, :393-395) and the README's "GPUs+MPI" has no code
(README.md:4); there is no reference output to pin these against, so the
checks are semantic (parity unpinned)."""
import ctypes as C
import os
import subprocess
import time

import pytest
import torch  # noqa: F401  (loads the HIP runtime the library links against)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "build", "libpga.so")
PGA_BINARY = 0
OBJ_ONEMAX = 1
RING, RANDOM, A2A = 0, 1, 2


class Stats(C.Structure):
    _fields_ = [("epochs", C.c_uint64), ("failures", C.c_uint64), ("migrants_received", C.c_uint64),
                ("bytes_sent", C.c_uint64), ("degraded", C.c_int)]


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
    L.pga_create_population_ext.restype = vp
    L.pga_create_population_ext.argtypes = [vp, C.c_ulong, C.c_uint, C.c_int]
    L.pga_set_objective_builtin.argtypes = [vp, vp, C.c_int, C.POINTER(C.c_float), C.c_size_t,
                                            C.POINTER(C.c_float), C.c_size_t, C.c_int, C.c_float, C.c_float]
    L.pga_set_operators.argtypes = [vp, vp, C.c_int, C.c_uint, C.c_int, C.c_float, C.c_int, C.c_float, C.c_float,
                                    C.c_uint]
    L.pga_run.argtypes = [vp, C.c_uint]
    L.pga_run_islands.argtypes = [vp, C.c_uint, C.c_uint, C.c_float]
    L.pga_best_score.restype = C.c_float
    L.pga_best_score.argtypes = [vp, vp]
    L.pga_get_scores.argtypes = [vp, vp, C.POINTER(C.c_float)]
    L.pga_comm_init_loopback.argtypes = [C.POINTER(vp), C.c_int]
    L.pga_comm_init_local.argtypes = [C.POINTER(vp), C.c_int]
    L.pga_run_islands_multi.argtypes = [C.POINTER(vp), C.c_int, C.c_uint, C.c_uint, C.c_float]
    L.pga_run_islands_multi_until.argtypes = [C.POINTER(vp), C.c_int, C.c_uint, C.c_uint, C.c_float, C.c_float]
    L.pga_comm_set_topology.argtypes = [vp, C.c_int]
    L.pga_comm_set_timeout.argtypes = [vp, C.c_double]
    L.pga_comm_set_validation.argtypes = [vp, C.c_int]
    L.pga_comm_set_fault.argtypes = [vp, C.c_int, C.c_int]
    L.pga_comm_degraded.argtypes = [vp]
    L.pga_comm_info.argtypes = [vp, C.POINTER(Stats)]
    L.pga_comm_best.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(C.c_int)]
    L.pga_comm_get_best.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(C.c_int), vp]
    L.pga_comm_set_self_exchange.argtypes = [vp, C.c_int]
    L.pga_get_genome.argtypes = [vp, vp, C.c_ulong, vp]
    L.pga_best_index.restype = C.c_ulong
    L.pga_best_index.argtypes = [vp, vp]
    L.pga_row_bytes.restype = C.c_size_t
    L.pga_row_bytes.argtypes = [vp]
    L.pga_migrate_between.argtypes = [vp, vp, vp, C.c_float]
    L.pga_run_islands_until.restype = C.c_int
    L.pga_run_islands_until.argtypes = [vp, C.c_uint, C.c_uint, C.c_float, C.c_float]
    L.pga_comm_exchange.argtypes = [C.POINTER(vp), C.c_int, C.c_float]
    L.pga_comm_unique_id.argtypes = [C.c_char_p]
    L.pga_comm_init.argtypes = [vp, C.c_int, C.c_int, C.c_char_p]
    L.pga_generation.restype = C.c_uint
    L.pga_generation.argtypes = [vp]
    L.pga_comm_rank.argtypes = [vp]
    L.pga_comm_size.argtypes = [vp]
    return L


S, LEN = 256, 64


def make_group(lib, n, device=-1, seed=100):
    """n solvers, one OneMax population each (elitism 1), seeds differ per rank."""
    solvers, pops = [], []
    for r in range(n):
        p = lib.pga_init_device(device)
        assert p
        lib.pga_set_seed(p, seed + r)
        lib.pga_set_quiet(p, 1)
        lib.pga_set_abort_on_error(p, 0)
        pop = lib.pga_create_population_ext(p, S, LEN, PGA_BINARY)
        assert lib.pga_set_objective_builtin(p, pop, OBJ_ONEMAX, None, 0, None, 0, 0, 0.0, 0.0) == 0
        assert lib.pga_set_operators(p, pop, 0, 2, 0, 1.0, 0, -1.0, 0.0, 1) == 0
        solvers.append(p)
        pops.append(pop)
    arr = (C.c_void_p * n)(*solvers)
    return solvers, pops, arr


def info(lib, p):
    st = Stats()
    assert lib.pga_comm_info(p, C.byref(st)) == 0
    return st


def test_ring_delivers_the_best(lib):
    solvers, pops, arr = make_group(lib, 3)
    assert lib.pga_comm_init_loopback(arr, 3) == 0
    assert [lib.pga_comm_rank(p) for p in solvers] == [0, 1, 2]
    assert lib.pga_comm_size(solvers[0]) == 3
    lib.pga_run(solvers[1], 60)  # rank 1 far ahead of the others
    b1 = lib.pga_best_score(solvers[1], pops[1])
    assert b1 > lib.pga_best_score(solvers[2], pops[2])
    # 2 generations, one migration at generation 1: ring 1 -> 2 carries rank 1's best
    assert lib.pga_run_islands_multi(arr, 3, 2, 1, 0.05) == 0, lib.pga_last_error()
    assert lib.pga_best_score(solvers[2], pops[2]) >= b1
    for p in solvers:
        st = info(lib, p)
        assert st.epochs == 1 and st.failures == 0 and not st.degraded
        assert st.migrants_received == round(0.05 * S)
    assert info(lib, solvers[0]).bytes_sent == 3 * round(0.05 * S) * (16 + 4)  # 64-bit rows pad to 16 B
    score, rank = C.c_float(), C.c_int()
    assert lib.pga_comm_best(solvers[0], C.byref(score), C.byref(rank)) == 0
    assert score.value == max(lib.pga_best_score(p, q) for p, q in zip(solvers, pops))
    for p in solvers:
        lib.pga_deinit(p)


def test_multi_rank_target_stop(lib):
    """pga_run_islands_multi_until: every rank stops at the same check point,
    the first at which the best over all ranks reaches the target (all-gather
    over the communicator)."""
    solvers, pops, arr = make_group(lib, 3, seed=5)
    assert lib.pga_comm_init_loopback(arr, 3) == 0
    lib.pga_run(solvers[0], 5)  # rank 0 ahead: its best decides the first call
    target = lib.pga_best_score(solvers[0], pops[0])
    assert target < LEN
    assert lib.pga_run_islands_multi_until(arr, 3, 500, 10, 0.05, target) == 0  # already reached
    g = lib.pga_run_islands_multi_until(arr, 3, 500, 10, 0.05, float(LEN))
    assert 0 < g < 500 and g % 10 == 0, g
    assert max(lib.pga_best_score(p, q) for p, q in zip(solvers, pops)) == LEN
    assert len({lib.pga_generation(q) for q in pops[1:]}) == 1  # ranks stopped together
    for p in solvers:
        lib.pga_deinit(p)


def test_all_to_all_and_random_ring(lib):
    for topo in (A2A, RANDOM):
        solvers, pops, arr = make_group(lib, 4, seed=7)
        assert lib.pga_comm_init_loopback(arr, 4) == 0
        assert lib.pga_comm_set_topology(solvers[0], topo) == 0  # applies to the group
        assert lib.pga_run_islands_multi(arr, 4, 31, 10, 0.05) == 0, lib.pga_last_error()
        k = round(0.05 * S)
        want = (k // 3) * 3 if topo == A2A else k
        for p in solvers:
            st = info(lib, p)
            assert st.epochs == 3 and st.migrants_received == 3 * want and not st.degraded
        # elitism + migration never lose the global best
        assert max(lib.pga_best_score(p, q) for p, q in zip(solvers, pops)) >= 50
        for p in solvers:
            lib.pga_deinit(p)


def test_random_ring_is_reproducible(lib):
    finals = []
    for _ in range(2):
        solvers, pops, arr = make_group(lib, 3, seed=21)
        lib.pga_comm_init_loopback(arr, 3)
        lib.pga_comm_set_topology(solvers[0], RANDOM)
        lib.pga_run_islands_multi(arr, 3, 20, 4, 0.1)
        sc = []
        for p, q in zip(solvers, pops):
            buf = (C.c_float * S)()
            lib.pga_get_scores(p, q, buf)
            sc.append(list(buf))
            lib.pga_deinit(p)
        finals.append(sc)
    assert finals[0] == finals[1]


def test_dropped_exchange_degrades(lib):
    solvers, pops, arr = make_group(lib, 2)
    lib.pga_comm_init_loopback(arr, 2)
    assert lib.pga_comm_set_fault(solvers[0], 2, 1) == 0  # the 2nd exchange is lost
    assert lib.pga_run_islands_multi(arr, 2, 40, 5, 0.05) == 0
    for p in solvers:
        st = info(lib, p)
        assert st.degraded == 1 and st.failures == 1
        assert st.epochs == 2 and st.migrants_received == round(0.05 * S)
        assert lib.pga_comm_degraded(p) == 1
    # the islands kept evolving alone
    assert all(lib.pga_best_score(p, q) >= 50 for p, q in zip(solvers, pops))
    for p in solvers:
        lib.pga_deinit(p)


@pytest.mark.parametrize("validate", [1, 0])
def test_forged_scores_are_rescored(lib, validate):
    solvers, pops, arr = make_group(lib, 2)
    lib.pga_comm_init_loopback(arr, 2)
    lib.pga_comm_set_fault(solvers[0], 1, 2)  # every exchange arrives with scores 3e38
    for p in solvers:
        lib.pga_comm_set_validation(p, validate)
    lib.pga_run_islands_multi(arr, 2, 3, 1, 0.05)
    assert lib.pga_comm_exchange(arr, 2, 0.05) == 0  # one more epoch, observed on arrival
    best = max(lib.pga_best_score(p, q) for p, q in zip(solvers, pops))
    if validate:
        assert best <= LEN  # a forged fitness never enters
    else:
        assert best > 1e37  # without re-scoring it does
    # the next generation re-evaluates every child from its genome (elites
    # included), so an unvalidated forged fitness does not outlive it
    lib.pga_run_islands_multi(arr, 2, 1, 0, 0.05)
    assert max(lib.pga_best_score(p, q) for p, q in zip(solvers, pops)) <= LEN
    for p in solvers:
        lib.pga_deinit(p)


def test_get_best_broadcasts_the_winning_genome(lib):
    """pga_comm_get_best: (score, index) all-gathered, the owner's row
    broadcast to every rank -- equal to the owner's own genome."""
    solvers, pops, arr = make_group(lib, 3, seed=31)
    assert lib.pga_comm_init_loopback(arr, 3) == 0
    lib.pga_run(solvers[2], 40)  # rank 2 ahead
    rb = lib.pga_row_bytes(pops[0])
    want = C.create_string_buffer(rb)
    assert lib.pga_get_genome(solvers[2], pops[2], lib.pga_best_index(solvers[2], pops[2]), want) == 0
    for p in solvers:  # every rank sees the same winner and row
        score, rank, row = C.c_float(), C.c_int(), C.create_string_buffer(rb)
        assert lib.pga_comm_get_best(p, C.byref(score), C.byref(rank), row) == 0, lib.pga_last_error()
        assert rank.value == 2 and score.value == lib.pga_best_score(solvers[2], pops[2])
        assert row.raw == want.raw
    for p in solvers:
        lib.pga_deinit(p)


def test_migrate_between_moves_exactly_the_top_k(lib):
    """The pga.h contract (include/pga.h:108-115): pga_migrate_between copies
    the top pct% of `from` over the worst of `to` (exact top-k by default)."""
    p = lib.pga_init_device(-1)
    lib.pga_set_seed(p, 77)
    lib.pga_set_quiet(p, 1)
    a = lib.pga_create_population_ext(p, S, LEN, PGA_BINARY)
    b = lib.pga_create_population_ext(p, S, LEN, PGA_BINARY)
    for q in (a, b):
        assert lib.pga_set_objective_builtin(p, q, OBJ_ONEMAX, None, 0, None, 0, 0, 0.0, 0.0) == 0
    lib.pga_run(p, 25)  # population 0 evolves: its top rows differ from b's
    rb = lib.pga_row_bytes(a)

    def snapshot(q):
        sc = (C.c_float * S)()
        lib.pga_get_scores(p, q, sc)
        rows = []
        for i in range(S):
            r = C.create_string_buffer(rb)
            lib.pga_get_genome(p, q, i, r)
            rows.append(r.raw)
        return list(sc), rows

    sa, ra = snapshot(a)
    sb, rbs = snapshot(b)
    k = round(0.05 * S)
    lib.pga_migrate_between(p, a, b, 0.05)
    sb2, rb2 = snapshot(b)
    # the k lowest-scored slots of b (ties: lower index first) were replaced ...
    worst = sorted(range(S), key=lambda i: (sb[i], i))[:k]
    kept = [i for i in range(S) if i not in set(worst)]
    assert all(rb2[i] == rbs[i] for i in kept)
    # ... by exactly a's top-k rows (as a multiset of (score, row))
    top = sorted(range(S), key=lambda i: (-sa[i], i))[:k]
    assert sorted((sb2[i], rb2[i]) for i in worst) == sorted((sa[i], ra[i]) for i in top)
    lib.pga_deinit(p)


def test_group_needs_the_multi_driver(lib):
    solvers, pops, arr = make_group(lib, 2)
    lib.pga_comm_init_loopback(arr, 2)
    lib.pga_run_islands(solvers[0], 5, 2, 0.05)
    assert b"pga_run_islands_multi" in lib.pga_last_error()
    sub = (C.c_void_p * 1)(solvers[0])
    assert lib.pga_run_islands_multi(sub, 1, 5, 2, 0.05) == -1  # every rank must be passed
    for p in solvers:
        lib.pga_deinit(p)


def test_single_rank_without_comm_is_plain_islands(lib):
    solvers, pops, arr = make_group(lib, 1)
    assert lib.pga_run_islands_multi(arr, 1, 10, 3, 0.05) == 0
    assert info(lib, solvers[0]).epochs == 0
    lib.pga_deinit(solvers[0])


@pytest.mark.gpu
def test_gpu_loopback_matches_cpu(lib):
    """The same loopback ring on GPU solvers reproduces the CPU backend's run
    bit for bit (BINARY generations are bit-exact CPU/GPU)."""
    out = []
    for dev in (-1, 0):
        solvers, pops, arr = make_group(lib, 2, device=dev, seed=3)
        assert lib.pga_comm_init_loopback(arr, 2) == 0
        assert lib.pga_run_islands_multi(arr, 2, 12, 4, 0.05) == 0, lib.pga_last_error()
        sc = []
        for p, q in zip(solvers, pops):
            buf = (C.c_float * S)()
            lib.pga_get_scores(p, q, buf)
            sc.append(sorted(buf))
            lib.pga_deinit(p)
        out.append(sc)
    assert out[0] == out[1]


@pytest.mark.gpu
def test_gpu_rccl_init_all_single_rank(lib):
    """ncclCommInitAll over the box's one GPU: the RCCL transport initialises,
    the group driver runs, and the global best query goes through
    ncclAllGather (one rank: no exchange)."""
    solvers, pops, arr = make_group(lib, 1, device=0)
    assert lib.pga_comm_init_local(arr, 1) == 0, lib.pga_last_error()
    lib.pga_comm_set_timeout(solvers[0], 30.0)
    assert lib.pga_run_islands_multi(arr, 1, 20, 5, 0.05) == 0, lib.pga_last_error()
    score, rank = C.c_float(), C.c_int()
    assert lib.pga_comm_best(solvers[0], C.byref(score), C.byref(rank)) == 0
    assert rank.value == 0 and score.value == lib.pga_best_score(solvers[0], pops[0])
    lib.pga_deinit(solvers[0])


@pytest.mark.gpu
def test_example_islands_multi_gpu():
    import subprocess
    exe = os.path.join(ROOT, "build", "examples", "islands_multi_gpu")
    r = subprocess.run([exe, "65536", "30", "all_to_all"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "GPU islands" in r.stdout


def rccl_rank0(lib, n=1):
    """A GPU solver joined to a fresh n-rank communicator through the
    one-process-per-GPU path (pga_comm_unique_id + pga_comm_init =
    ncclCommInitRank), as rank 0."""
    uid = C.create_string_buffer(128)
    assert lib.pga_comm_unique_id(uid) == 0, lib.pga_last_error()
    solvers, pops, arr = make_group(lib, 1, device=0)
    assert lib.pga_comm_init(solvers[0], n, 0, uid.raw) == 0, lib.pga_last_error()
    return solvers[0], pops[0]


@pytest.mark.gpu
def test_rccl_initrank_self_exchange_gpu(lib):
    """InitRank with one rank; the self-exchange test hook makes every epoch
    run grouped ncclSend/ncclRecv on the communication stream, overlapped
    with the next generation, before the compute stream consumes it."""
    p, pop = rccl_rank0(lib)
    assert lib.pga_comm_size(p) == 1 and lib.pga_comm_rank(p) == 0
    lib.pga_run_islands(p, 10, 5, 0.05)
    assert info(lib, p).epochs == 0  # one rank: no migration ...
    assert lib.pga_comm_set_self_exchange(p, 1) == 0  # ... unless the test hook asks for it
    lib.pga_run_islands(p, 30, 5, 0.05)
    st = info(lib, p)
    k = round(0.05 * S)
    assert st.epochs == 5 and st.failures == 0 and not st.degraded
    assert st.migrants_received == 5 * k and st.bytes_sent == 5 * k * (16 + 4)
    assert lib.pga_generation(pop) == 40 and lib.pga_best_score(p, pop) >= 50
    lib.pga_deinit(p)


@pytest.mark.gpu
def test_rccl_withheld_send_degrades_gpu(lib):
    """The 2nd exchange posts its receive but withholds the matching send:
    the host deadline (2 s) expires, ncclCommAbort runs at once, the pending
    scatter is dropped and the generations continue on the compute stream,
    which never waited for the dead transfer."""
    p, pop = rccl_rank0(lib)
    assert lib.pga_comm_set_self_exchange(p, 1) == 0
    assert lib.pga_comm_set_timeout(p, 2.0) == 0
    assert lib.pga_comm_set_fault(p, 2, 3) == 0
    t0 = time.monotonic()
    lib.pga_run_islands(p, 40, 5, 0.05)
    best = lib.pga_best_score(p, pop)  # synchronises the solver stream
    dt = time.monotonic() - t0
    st = info(lib, p)
    assert st.degraded == 1 and st.failures == 1 and lib.pga_comm_degraded(p) == 1
    assert st.epochs == 2 and st.migrants_received == round(0.05 * S)
    assert lib.pga_generation(pop) == 40 and best >= 50
    assert dt < 30, dt  # one 2 s timeout, not a hang
    lib.pga_deinit(p)


@pytest.mark.gpu
def test_islands_multiproc_example_gpu(tmp_path):
    exe = os.path.join(ROOT, "build", "examples", "islands_multiproc")
    if not os.path.exists(exe):
        pytest.skip("examples not built")
    r = subprocess.run([exe, "0", "1", str(tmp_path / "id"), "65536", "30"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert "rank 0/1 generations 30" in r.stdout


@pytest.mark.gpu
def test_rccl_stalled_allgather_degrades_gpu(lib):
    """A target run whose 2nd check-point all-gather stalls (a peer lost
    between epochs): the deadline expires, the communicator is aborted, the
    run goes on with the local best and returns within the timeout."""
    p, pop = rccl_rank0(lib)
    assert lib.pga_comm_set_self_exchange(p, 1) == 0
    assert lib.pga_comm_set_timeout(p, 2.0) == 0
    assert lib.pga_comm_set_fault(p, 2, 4) == 0
    t0 = time.monotonic()
    g = lib.pga_run_islands_until(p, 60, 10, 0.05, float(LEN + 1))  # unreachable target
    dt = time.monotonic() - t0
    st = info(lib, p)
    assert g == 60, lib.pga_last_error()
    assert st.degraded == 1 and st.failures == 1
    assert dt < 30, dt
    score, rank = C.c_float(), C.c_int()
    assert lib.pga_comm_best(p, C.byref(score), C.byref(rank)) == 0  # degraded: the local best, no hang
    assert score.value == lib.pga_best_score(p, pop)
    lib.pga_deinit(p)


@pytest.mark.gpu
def test_rccl_get_best_genome_single_rank_gpu(lib):
    p, pop = rccl_rank0(lib)
    lib.pga_run(p, 20)
    rb = lib.pga_row_bytes(pop)
    want, row = C.create_string_buffer(rb), C.create_string_buffer(rb)
    assert lib.pga_get_genome(p, pop, lib.pga_best_index(p, pop), want) == 0
    score, rank = C.c_float(), C.c_int()
    assert lib.pga_comm_set_self_exchange(p, 1) == 0  # the RCCL all-gather + broadcast path
    assert lib.pga_comm_get_best(p, C.byref(score), C.byref(rank), row) == 0, lib.pga_last_error()
    assert rank.value == 0 and row.raw == want.raw and score.value == lib.pga_best_score(p, pop)
    lib.pga_deinit(p)
