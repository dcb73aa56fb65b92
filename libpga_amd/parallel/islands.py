"""Island model across ranks: one island per GPU, migration over RCCL/xGMI.

One process per GPU (``torch.distributed``, backend "nccl" = RCCL on ROCm;
"gloo" on CPU for tests).  Every ``migrate_every`` generations each island
exports its top ``migrate_pct`` individuals and imports the same number from
its peer(s), replacing its worst individuals.

Data path per migration (all on-device, no host synchronisation):
  emigrant selection with the row gather fused in (Island.emigrate; policy
  "topk", the default: the exact top-k; "stripe": the best of each of k
  population stripes, one pass) writing
  rows+scores into ONE packed send buffer -> RCCL send/recv on torch's NCCL
  stream -> [next generation kernel runs concurrently on the compute stream]
  -> stream wait on the NCCL work -> re-score -> victims replaced with the
  scatter fused in (Island.immigrate: each stripe's worst, or the bottom-k),
  best partials and statistics written by the same kernel.

Why this shape on MI355X: the 8 GPUs of a node are fully connected by xGMI,
7 point-to-point links of ~153 GB/s each.  A ring migration uses one link per
direction, so it is per-link bound; at 1% of 1M x 128 B that is ~1.3 MB per
epoch (~9 us on one link) — far below one generation's compute, so it hides
behind the overlapped generation entirely.  ``topology="all_to_all"`` spreads
the same volume over all 7 links (``all_to_all_single``) for larger
migrations; ``"random"`` draws a fresh island permutation per epoch from the
shared seed (all ranks agree without communicating).

Failure handling (the reference aborts on any error):
  * received migrants are re-scored with the LOCAL objective before they
    enter the population (``validate=True``), so a corrupted or forged batch
    can never inject a fake fitness;
  * a migration that fails or exceeds ``timeout_s`` puts the model in
    DEGRADED mode: islands are loosely coupled, so each keeps evolving alone
    and ``degraded`` / ``failures`` report it.  The deadline is enforced on
    the host by polling the exchange's completion (``is_completed``, never a
    blocking wait); on expiry the process group is aborted at once and the
    compute stream is never made to wait for the dead transfer, so the
    generations that follow run on (RCCL's ``work.wait(timeout)`` would only
    order the stream, not bound the host);
  * ``fault_hook(recv, epoch) -> bool`` is a test-only injection point that
    may corrupt the received buffer in place or drop it (return False).

Reference: ``pga_migrate`` / ``pga_migrate_between`` / ``pga_run_islands``
are declared but empty in the reference (include/pga.h:108-115, :145-150;
src/pga.cu:368-374, :393-395); the README claims "GPUs+MPI" (README.md:4).
"""
from __future__ import annotations

import datetime
import math
import os
import time
from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

from ..ga import GeneticAlgorithm
from ..utils.log import get_logger
from .local import migration_policy

log = get_logger(__name__)

TOPOLOGIES = ("ring", "random", "all_to_all")


def init_distributed(backend: Optional[str] = None) -> Tuple[int, int, torch.device]:
    """Initialise the default process group from torchrun env vars.

    Returns (rank, world_size, device).  Binds the rank to cuda:LOCAL_RANK
    when GPUs are present.  Safe to call when already initialised or when
    running single-process (returns rank 0 / world 1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    device = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if use_gpu else "gloo")
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    if dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
    return rank, world, device


class IslandModel:
    def __init__(
        self,
        ga: GeneticAlgorithm,
        *,
        migrate_every: int = 10,
        migrate_pct: float = 0.01,
        topology: str = "ring",
        group=None,
        overlap: bool = True,
        side_stream: bool = False,
        seed: int = 0,
        validate: bool = True,
        timeout_s: Optional[float] = None,
        fault_hook: Optional[Callable[[torch.Tensor, int], bool]] = None,
        policy: str = "topk",
        transport: str = "auto",
        self_exchange: bool = False,
        lag: Optional[int] = None,
    ):
        if topology not in TOPOLOGIES:
            raise ValueError(f"topology must be one of {TOPOLOGIES}")
        self.ga = ga
        self.migrate_every = int(migrate_every)
        # lag: generations from an epoch's departure to its arrival.  The
        # exchange overlaps the next generation kernel, but on one device the
        # transfer's kernel only gets the CUs as that generation drains, so it
        # completes at the generation's end; with lag 1 the host then enqueues
        # the immigration while the compute queue sits empty (measured on
        # MI355X: a ~100 us idle gap per epoch, host poll + launch latency).
        # With lag 2 the host checks the exchange only after the generation
        # after it is queued too: the GPU never waits for the host.  Capped at
        # migrate_every - 1 (an epoch ends before the next one starts).
        # (default: 2 for GPU islands, 1 for CPU islands, which have no queue)
        if lag is None:
            lag = int(os.environ.get("PGA_MIG_LAG", "2")) if ga.island.rows(0).device.type == "cuda" else 1
        self.lag = max(1, min(int(lag), self.migrate_every - 1)) if self.migrate_every > 1 else 1
        self._start_gen = 0
        self.topology = topology
        self.group = group
        self.overlap = overlap
        self.seed = seed
        self.validate = validate
        self.timeout = datetime.timedelta(seconds=timeout_s) if timeout_s else None
        self.fault_hook = fault_hook
        self.degraded = False
        self.failures = 0
        self.dropped = 0
        self.distributed = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.world = dist.get_world_size(group) if self.distributed else 1
        self._pg_world = self.world
        # self_exchange (measurement / test mode): ONE process runs the
        # 2-island ring against itself, its migrants sent to and received
        # from its own rank over a 1-rank RCCL communicator, so one GPU pays
        # everything an N-GPU run pays per epoch except the xGMI wire time
        self.self_exchange = bool(self_exchange)
        if self.self_exchange:
            if not (self.distributed and self.world == 1 and topology == "ring"):
                raise ValueError("self_exchange needs a 1-rank process group and the ring topology")
            self.world = 2
        S = ga.pop_size
        k = int(round(migrate_pct * S))
        self.k = max(1, min(k, S // 2)) if migrate_pct > 0 else 0
        if topology == "all_to_all" and self.world > 1:
            per = max(1, self.k // (self.world - 1))
            self.k = per * (self.world - 1)
        isl = ga.island
        isl.migration_policy = migration_policy(policy)  # stripe: one pass each way; topk: exact
        if policy == "topk" and self.world > 1 and self.k > 0 and migrate_every > 0:
            # exact top-k / bottom-k from the generation kernel's fused key
            # histogram: no histogram pass per selection (integer objectives)
            isl.fused_histogram = True
        self.rw = int(isl.row_words)
        dev = isl.rows(0).device
        n = self.k * (self.rw + 1)
        self.send = torch.empty(n, dtype=torch.int32, device=dev)
        self.recv = torch.empty(n, dtype=torch.int32, device=dev)
        # the (rows, scores) views of both buffers, made once: a view costs
        # microseconds of host time, and an epoch's host path is short
        self._send_views = self._views(self.send)
        self._recv_views = self._views(self.recv)
        self._pending = None
        # side_stream=True runs emigrant selection + packing on a side stream,
        # concurrently with the next generation kernel (they only read the
        # current generation; not with elitism > 1: the elite top-k shares the
        # island's selection workspace).  Off by default: measured on MI355X
        # (bench/migration_cost.py, PGA_RCCL_SELF=1, 1M x 1024-bit, every 10
        # generations) the side stream shares the generation's hardware queue,
        # so it overlaps nothing and adds two cross-stream waits per epoch:
        # 11.5% vs 8.6% migration overhead.  The RCCL exchange itself still
        # overlaps the next generation either way.
        use_side = side_stream and dev.type == "cuda" and ga.operators.elitism <= 1
        self._side = torch.cuda.Stream(dev) if use_side else None
        # transport: "torch" = torch.distributed P2P ops (any backend);
        # "engine" = the engine's own RCCL communicator (comm_bind.cpp: one
        # native call packs and posts an epoch, one completes it — a fraction
        # of batch_isend_irecv's host time); "auto" = engine on GPU islands
        # of an RCCL process group for the ring / random topologies (no
        # side stream or fault hook, which need the python path).
        # Permutation islands take it too: the native re-scoring
        # (Island.evaluate_rows) turns a received row that is not a
        # permutation into the identity tour before it can enter.
        if transport not in ("auto", "torch", "engine"):
            raise ValueError("transport must be 'auto', 'torch' or 'engine'")
        self._ec = None
        engine_ok, why = self._engine_supported(ga, dev, topology, fault_hook, group)
        if transport == "engine" and self.distributed and not engine_ok:
            raise ValueError(f"transport='engine' cannot run this model: {why}")
        self._use_engine = engine_ok and self.distributed and (
            transport == "engine" or (transport == "auto" and os.environ.get("PGA_MIGRATION_TRANSPORT", "") != "torch"))
        self.fallbacks = 0  # engine -> torch switches made by connect()
        # test-only fault: post the receive but withhold the matching send, so
        # the exchange can never complete (exercises the deadline + abort path)
        self._withhold_send = False
        if topology == "all_to_all" and self.world > 1:
            others = [p for p in range(self.world) if p != self.rank]
            self._peer_idx = torch.tensor(others, dtype=torch.long, device=dev)
            # persistent [peer][rows | scores] send / receive packing (the self
            # slice stays empty): no allocation or memset per epoch
            per = self.k // (self.world - 1)
            self._a2a_send = torch.zeros(self.world * per * (self.rw + 1), dtype=torch.int32, device=dev)
            self._a2a_recv = torch.empty_like(self._a2a_send)
        self._epoch = 0
        self.migrations = 0
        self.bytes_sent = 0

    # --------------------------------------------------------------- utils --
    def _engine_supported(self, ga, dev, topology, fault_hook, group) -> Tuple[bool, str]:
        if dev.type != "cuda":
            return False, "the engine communicator needs GPU islands"
        if topology not in ("ring", "random"):
            return False, f"topology {topology!r} (the engine plan is ring / random peers)"
        if self._side is not None:
            return False, "side_stream=True (the engine posts on the island's own stream)"
        if fault_hook is not None:
            return False, "a fault_hook (it edits the received buffer in python)"
        if self.distributed and dist.get_backend(group) != "nccl":
            return False, f"process-group backend {dist.get_backend(group)!r} (RCCL needed)"
        return True, ""

    @property
    def transport(self) -> str:
        """The migration transport in use: "engine" or "torch"."""
        return "engine" if self._use_engine else "torch"

    @property
    def rccl_ranks(self) -> int:
        """Ranks of the RCCL communicator that carries the migrants: the
        engine communicator's size, the process group's under backend nccl,
        0 when no RCCL is involved (gloo, one process)."""
        if self._use_engine and self._ec is not None:
            return int(self._ec.nranks)
        if self.distributed and dist.get_backend(self.group) == "nccl":
            return self._pg_world
        return 0

    def reduce_max(self, t: torch.Tensor) -> bool:
        """In-place all-reduce(max) of ``t`` over the islands, bounded by the
        migration deadline; False (and degraded) when it failed or expired."""
        if self.world == 1:
            return True
        if self.degraded:
            return False
        try:
            work = dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group, async_op=True)
        except Exception as e:  # noqa: BLE001
            self._fail(e)
            return False
        return self._bounded(work)

    def _views(self, buf: torch.Tensor):
        rows = buf[: self.k * self.rw]
        scores = buf[self.k * self.rw:].view(torch.float32)
        return rows, scores

    def _peers(self) -> Tuple[int, int]:
        """(send_to, recv_from) for ring / random topologies."""
        r, w = self.rank, self.world
        if self.self_exchange:
            return r, r
        if self.topology == "ring":
            return (r + 1) % w, (r - 1) % w
        g = torch.Generator().manual_seed(self.seed * 1000003 + self._epoch)
        perm = torch.randperm(w, generator=g).tolist()
        pos = perm.index(r)
        return perm[(pos + 1) % w], perm[(pos - 1) % w]

    # ----------------------------------------------------------- migration --
    def _engine(self):
        """The engine communicator (collective: every rank creates it at the
        same migration point, or in connect())."""
        if self._ec is None:
            from .. import _ext

            C = _ext.load()
            uid = [C.rccl_unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(uid, src=dist.get_global_rank(self.group, 0) if self.group else 0,
                                       group=self.group)
            # the process group's own size and rank (tests pretend a peer on a 1-rank group)
            self._ec = C.EngineComm(dist.get_world_size(self.group), dist.get_rank(self.group), uid[0],
                                    self.send.device.index)
        return self._ec

    def start_migration(self) -> None:
        """Pack the top-k emigrants and post the exchange (asynchronous)."""
        if self.world == 1 or self.k == 0 or self.degraded:
            return
        if self._use_engine and not self._withhold_send:
            dst, src = self._peers()
            try:
                self._engine().post(self.ga.island, self.k, *self._send_views, *self._recv_views, dst, src)
            except Exception as e:  # noqa: BLE001 — any comm failure degrades
                self._fail(e)
                return
            self._pending = "engine"
            self._epoch += 1
            self.bytes_sent += self.send.numel() * 4
            return
        if self._side is not None:
            self._side.wait_stream(torch.cuda.current_stream(self._side.device))
            with torch.cuda.stream(self._side):
                ok = self._post()
        else:
            ok = self._post()
        if ok:
            self._epoch += 1
        self.bytes_sent += self.send.numel() * 4

    def _post(self) -> bool:
        isl = self.ga.island
        srows, sscores = self._views(self.send)
        isl.emigrate(self.k, srows, sscores)  # top-k selection with the gather fused in
        if self.topology == "all_to_all":
            self._pending = self._a2a()
            return True
        dst, src = self._peers()
        ops = [dist.P2POp(dist.irecv, self.recv, src, group=self.group)]
        if not self._withhold_send:
            ops.insert(0, dist.P2POp(dist.isend, self.send, dst, group=self.group))
        try:
            self._pending = dist.batch_isend_irecv(ops)
        except Exception as e:  # noqa: BLE001 — any comm failure degrades
            self._fail(e)
            return False
        return True

    def _a2a(self):
        # every peer gets an equal slice of the emigrants, packed as
        # [peer][per rows | per scores] (one indexed copy per part, no
        # per-peer loop); the self slice is empty
        w, per = self.world, self.k // (self.world - 1)
        srows, sscores = self._views(self.send)
        pv = self._a2a_send.view(w, per * (self.rw + 1))
        pv[self._peer_idx, : per * self.rw] = srows.view(w - 1, per * self.rw)
        pv[self._peer_idx, per * self.rw:] = sscores.view(torch.int32).view(w - 1, per)
        return [dist.all_to_all_single(self._a2a_recv, self._a2a_send, group=self.group, async_op=True)]

    def _await(self, works) -> None:
        """Complete the exchange.  Without a timeout: stream-ordered waits
        only.  With one: poll completion on the host until the deadline, then
        abort the group (raising TimeoutError) without ever ordering the
        compute stream after the unfinished transfer."""
        if self.timeout is None:
            for wk in works:
                wk.wait()
            return
        if self.distributed and dist.get_backend(self.group) == "gloo":
            # gloo's P2P works complete only inside wait(), which honours a
            # timeout itself (CPU islands: nothing to keep off the stream)
            try:
                for wk in works:
                    wk.wait(self.timeout)
            except Exception:
                self._abort()
                raise
            return
        deadline = time.monotonic() + self.timeout.total_seconds()
        pending = list(works)
        while pending:
            pending = [wk for wk in pending if not wk.is_completed()]
            if pending and time.monotonic() > deadline:
                self._abort()
                raise TimeoutError(f"migration epoch {self._epoch} exceeded {self.timeout.total_seconds()} s")
            if pending and time.monotonic() > deadline - self.timeout.total_seconds() + 2e-3:
                time.sleep(20e-6)  # spin the first 2 ms, then back off
        for wk in works:
            wk.wait()  # completed: raises a transport error, else just orders the stream

    def _abort(self) -> None:
        try:
            dist.distributed_c10d._abort_process_group(self.group)
        except Exception as e:  # noqa: BLE001 — best effort; the model is degraded either way
            log.warning("process-group abort failed: %s", e)

    def finish_migration(self) -> None:
        """Wait for the exchange and replace the worst individuals."""
        if self._pending is None:
            return
        if isinstance(self._pending, str):  # the engine communicator's epoch
            self._pending = None
            t = self.timeout.total_seconds() if self.timeout is not None else 0.0
            try:
                ok = self._ec.finish(self.ga.island, self.k, t, self.validate)
            except Exception as e:  # noqa: BLE001
                self._fail(e)
                return
            if not ok:
                self._fail(TimeoutError(f"migration epoch {self._epoch} failed or exceeded its deadline"))
                return
            self.migrations += 1
            return
        if self._side is not None:
            # the next generation must not overwrite rows the side stream still packs
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)
        try:
            self._await(self._pending)
        except Exception as e:  # noqa: BLE001
            self._pending = None
            self._fail(e)
            return
        self._pending = None
        isl = self.ga.island
        if self.fault_hook is not None:
            buf = self._a2a_recv if self.topology == "all_to_all" else self.recv
            if self.fault_hook(buf, self._epoch) is False:
                self.dropped += 1
                return
        if self.topology == "all_to_all":
            w, per = self.world, self.k // (self.world - 1)
            pv = self._a2a_recv.view(w, per * (self.rw + 1))[self._peer_idx]
            rows = pv[:, : per * self.rw].reshape(-1)
            scores = pv[:, per * self.rw:].reshape(-1).view(torch.float32)
        else:
            rows, scores = self._views(self.recv)
        rows, scores = rows.contiguous(), scores.contiguous()
        if self.validate:
            # trust nothing from the wire: re-scored with the local objective;
            # a permutation row that is not one becomes the identity tour
            isl.evaluate_rows(rows, scores)
        isl.immigrate(self.k, rows, scores)  # bottom-k replaced (fused scatter), best + keys follow
        self.migrations += 1

    def _fail(self, e: BaseException) -> None:
        self.failures += 1
        self.degraded = True
        log.error("migration failed (%s: %s); island %d continues without migration", type(e).__name__, e, self.rank)

    # ----------------------------------------------------------------- run --
    def run(self, generations: int, *, target: Optional[float] = None, check_every: int = 0) -> int:
        """Run ``generations`` generations with periodic migration.

        Generation counting is global (``ga.generation``), so a run split into
        several calls migrates at the same generations as one long call.
        With ``target``, every ``check_every`` generations (default: the
        migration interval) the islands agree on the global best with one
        all-reduce(max) and all stop together once it reaches ``target``.
        Returns the generations executed."""
        every = check_every or self.migrate_every or 1
        migrates = self.migrate_every > 0 and self.world > 1 and self.k > 0
        done, n = 0, int(generations)
        while done < n:
            g = self.ga.generation
            if migrates and g > 0 and g % self.migrate_every == 0 and self._pending is None and not self.degraded:
                self.start_migration()
                self._start_gen = g
                if not self.overlap:
                    self.finish_migration()
            if self.ga.torch_objective is None and target is None and (
                    self._pending is None or self.ga.generation - self._start_gen < self.lag - 1):
                # nothing to do between generations until the next migration
                # point, or until the generation before the exchange in flight
                # completes: those generations in ONE engine call (C++
                # enqueues them back to back, no per-step Python on the host
                # path)
                step = n - done
                if self._pending is not None:
                    # the first generation alone: _fence() follows it
                    ahead = self.ga.generation - self._start_gen
                    step = min(step, 1 if ahead == 0 else self.lag - 1 - ahead)
                elif migrates:
                    step = min(step, self.migrate_every - g % self.migrate_every)
                self.ga.island.run(step)
                self._fence()
                done += step
                continue
            self.ga.island.run(1)
            self._fence()
            if self.ga.torch_objective is not None:
                self.ga._custom_eval()
            if self._pending is not None and self.ga.generation - self._start_gen >= self.lag:
                self.finish_migration()
            done += 1
            if target is not None and self.ga.generation % every == 0 and self.global_reduce_best() >= target:
                break
        return done

    def _fence(self) -> None:
        """With the engine transport the emigrants are packed on the transport
        stream, concurrently with the generation after their departure; the
        generation after THAT overwrites the population they come from, so
        the compute stream waits for the packing once the first is enqueued."""
        if self._pending is None or self.ga.generation != self._start_gen + 1:
            return
        if self._pending == "engine":
            self._ec.fence(self.ga.island)
        elif self._side is not None:  # the same for the packing on the side stream
            torch.cuda.current_stream(self._side.device).wait_stream(self._side)

    def flush(self) -> None:
        self.finish_migration()

    def connect(self) -> None:
        """Run one migration now: RCCL establishes its point-to-point
        connections lazily on the first exchange, so benchmarks call this
        before timing.

        With the engine transport, a communicator that fails to come up or
        whose first exchange fails on ANY rank (the ranks agree with one
        all-reduce over the process group) is dropped on every rank, and the
        islands fall back to torch P2P ops: the model is left healthy, the
        switch is counted in ``fallbacks``, and nothing is restarted."""
        if self.world == 1 or self.k == 0:
            return
        if self._use_engine:
            ok = 1.0
            try:
                self._engine()
                self.start_migration()
                self.finish_migration()
                ok = 0.0 if self.degraded else 1.0
            except Exception as e:  # noqa: BLE001 — any setup failure: fall back
                log.warning("engine communicator setup failed (%s: %s)", type(e).__name__, e)
                ok = 0.0
            flag = torch.tensor([ok], dtype=torch.float32,
                                device=self.send.device if dist.get_backend(self.group) == "nccl" else "cpu")
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
            if float(flag.item()) > 0.0:
                return
            log.warning("island %d: engine RCCL transport unavailable, falling back to torch P2P", self.rank)
            self._use_engine = False
            self._ec = None
            self._pending = None
            self.degraded, self.failures = False, 0
            self.fallbacks += 1
        self.start_migration()
        self.finish_migration()

    # -------------------------------------------------------------- queries --
    def _bounded(self, work) -> bool:
        """Complete an async collective under the migration deadline (the
        same host poll + abort as an exchange); False: failed or expired, the
        model is now degraded."""
        try:
            self._await([work])
        except Exception as e:  # noqa: BLE001 — a dead peer must never hang a query
            self._fail(e)
            return False
        return True

    def global_best(self) -> Tuple[float, int, torch.Tensor]:
        """(score, owning rank, decoded genome) of the best individual of all
        islands; ties go to the lowest rank.  Bounded by ``timeout_s``: on a
        dead peer the model degrades and this returns the local best."""
        score, genome = self.ga.best()
        if self.world == 1 or self.degraded:
            return score, self.rank, genome
        dev = self.send.device
        t = torch.tensor([score, float(self.rank)], dtype=torch.float64, device=dev)
        allt = [torch.empty_like(t) for _ in range(self._pg_world)]
        if not self._bounded(dist.all_gather(allt, t, group=self.group, async_op=True)):
            return score, self.rank, genome
        vals = torch.stack(allt).cpu()
        best_rank = int(vals[:, 0].argmax().item())
        row = self.ga.island.row(self.ga.best_index()).to(dev)
        if not self._bounded(dist.broadcast(row, src=best_rank, group=self.group, async_op=True)):
            return score, self.rank, genome
        return float(vals[best_rank, 0]), best_rank, self.ga.problem.decode(row.unsqueeze(0).cpu())[0]

    def global_reduce_best(self) -> float:
        """Max of every island's best (the target check).  Bounded by
        ``timeout_s``: on a dead peer the model degrades and this returns the
        local best."""
        s = self.ga.best_score()
        if self.world == 1 or self.degraded:  # an aborted group cannot reduce: the local best
            return s
        t = torch.tensor([s], dtype=torch.float32, device=self.send.device)
        if not self._bounded(dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group, async_op=True)):
            return s
        return float(t.item())


def migrants_for(pop_size: int, pct: float) -> int:
    return max(1, int(math.floor(pct * pop_size + 0.5)))
