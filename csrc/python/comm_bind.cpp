// comm_bind.cpp — the engine's own RCCL communicator for the Python island
// model (libpga_amd/parallel/islands.py, backend "engine").
//
// torch.distributed's batch_isend_irecv costs ~37 us of host time per
// migration epoch (profiles/migration_epoch_host_probe_r04.json: 74 us of
// host calls per epoch against a ~90 us generation).  Here one call packs the
// emigrants (Island::emigrate, exact top-k with the row gather fused in) and
// posts the grouped ncclSend/ncclRecv of the epoch on the rank's
// communication stream (comm_rccl.cpp, the C API's transport), and one call
// completes it: the compute stream waits for the transfer (or, past the
// deadline, the communicator is aborted and the island runs on degraded),
// then the received rows are re-scored and replace the bottom-k.
//
// The communicator is a second RCCL communicator beside torch's process
// group, bootstrapped from torch's: rank 0's ncclUniqueId travels by
// torch.distributed.broadcast_object_list.  _C.so resolves RCCL to the copy
// torch already loaded (same soname), so one RCCL runs in the process.
//
// Reference: the intended pga_run_islands / pga_migrate (include/pga.h:
// 108-115, 145-150) are empty stubs (src/pga.cu:368-374, :393-395).
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "pga/comm.hpp"
#include "pga/island.hpp"
#include "pga/ops.hpp"

namespace py = pybind11;

namespace {

using IslandPtr = std::shared_ptr<pga::Island>;

void check_dev(const torch::Tensor& t, const pga::Island& isl, torch::ScalarType st, const char* what) {
  TORCH_CHECK(t.is_contiguous(), what, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == st, what, " has the wrong dtype");
  TORCH_CHECK(t.is_cuda() && t.device().index() == isl.device(), what, " must live on the island's GPU");
}

// one local rank's staging: the island's current torch stream and the buffers
pga::LocalRank local_of(pga::Island& isl, int rank, torch::Tensor send_rows, torch::Tensor send_scores,
                        torch::Tensor recv_rows, torch::Tensor recv_scores) {
  pga::LocalRank l;
  l.rank = rank;
  l.device = isl.device();
  isl.stream = c10::hip::getCurrentHIPStream(isl.device()).stream();
  l.stream = isl.stream;
  l.row_bytes = isl.row_bytes();
  l.send_rows = send_rows.data_ptr();
  l.send_scores = send_scores.data_ptr<float>();
  l.recv_rows = recv_rows.data_ptr();
  l.recv_scores = recv_scores.data_ptr<float>();
  return l;
}

// the epoch's transfers of this rank: k rows to dst, k rows from src
std::vector<pga::Xfer> ring_plan(int rank, int dst, int src, uint32_t k) {
  if (dst == rank && src == rank) return {pga::Xfer{rank, rank, 0, 0, k}};  // self-exchange (world 1)
  return {pga::Xfer{rank, dst, 0, 0, k}, pga::Xfer{src, rank, 0, 0, k}};
}

struct EngineComm {
  std::shared_ptr<pga::Comm> comm;
  int rank = 0, nranks = 1;
  std::vector<pga::LocalRank> pending;  // the posted epoch (empty: none)
  hipStream_t compute = nullptr;        // the island's stream at post time
  bool on_transport = false;            // the epoch's device work runs on the transport stream
  bool early_eval = false;              // the migrants were re-scored on the transport stream at post time
  hipEvent_t ev_pop = nullptr, ev_out = nullptr, ev_in = nullptr;
  ~EngineComm() {
    for (hipEvent_t ev : {ev_pop, ev_out, ev_in})
      if (ev) (void)hipEventDestroy(ev);
  }
};

// Where the epoch's device work runs.  Emigrant selection only reads the
// current population, and re-scoring only touches the receive buffers, so
// both CAN go on the communicator's transport stream, in order with the
// transfer and beside the next generation kernel (IslandModel._fence orders
// the generation that overwrites the emigrants' population after the
// packing).  Off by default (PGA_MIG_ON_TRANSPORT=1 turns it on): measured
// on MI355X (bench.py --rccl-self, profiles/migration_ab_r06.txt) the
// headline generation kernel holds every CU's LDS, so nothing beside it
// runs until it drains, and the cross-stream hops cost more than they hide
// (OneMax 98.2 vs 95.6 us/gen, TSP-256 147.0 vs 143.8).  Never with
// elitism > 1: the elite top-k of every generation shares the island's
// selection workspace with the emigrant selection.
bool use_transport(EngineComm& e, const pga::Island& isl, const pga::LocalRank& l) {
  if (isl.config().n_elite > 1 || !std::getenv("PGA_MIG_ON_TRANSPORT")) return false;
  if (!e.comm->transport_stream(l)) return false;
  if (!e.ev_pop) {
    PGA_HIP_CHECK(hipEventCreateWithFlags(&e.ev_pop, hipEventDisableTiming));
    PGA_HIP_CHECK(hipEventCreateWithFlags(&e.ev_out, hipEventDisableTiming));
    PGA_HIP_CHECK(hipEventCreateWithFlags(&e.ev_in, hipEventDisableTiming));
  }
  return true;
}

}  // namespace

void bind_comm(py::module& m) {
  m.def("rccl_unique_id", [] {
    char id[128];
    if (pga::rccl_unique_id(id) != 0) throw std::runtime_error("ncclGetUniqueId failed");
    return py::bytes(id, 128);
  });
  py::class_<EngineComm, std::shared_ptr<EngineComm>>(m, "EngineComm")
      .def(py::init([](int nranks, int rank, py::bytes id, int device) {
             const std::string s = id;
             if (s.size() != 128) throw std::invalid_argument("ncclUniqueId must be 128 bytes");
             auto e = std::make_shared<EngineComm>();
             {
               py::gil_scoped_release nogil;  // InitRank blocks until every rank joins
               e->comm = pga::rccl_comm_rank(nranks, rank, s.data(), device);
             }
             e->rank = rank;
             e->nranks = nranks;
             return e;
           }),
           py::arg("nranks"), py::arg("rank"), py::arg("unique_id"), py::arg("device"))
      .def_readonly("rank", &EngineComm::rank)
      .def_readonly("nranks", &EngineComm::nranks)
      .def_property_readonly("bytes_sent", [](const EngineComm& e) { return e.comm->bytes_sent; })
      .def("set_fault", [](EngineComm& e, int every, int mode) { e.comm->set_fault(every, mode); })
      // emigrate the top-k into the send buffers and post the epoch's
      // grouped send / receive (no host wait)
      .def("post",
           [](EngineComm& e, const IslandPtr& isl, uint32_t k, torch::Tensor send_rows, torch::Tensor send_scores,
              torch::Tensor recv_rows, torch::Tensor recv_scores, int dst, int src) {
             TORCH_CHECK(e.pending.empty(), "an exchange is already in flight");
             TORCH_CHECK(isl->on_gpu(), "the engine communicator needs a GPU island");
             check_dev(send_rows, *isl, torch::kInt32, "send_rows");
             check_dev(send_scores, *isl, torch::kFloat32, "send_scores");
             check_dev(recv_rows, *isl, torch::kInt32, "recv_rows");
             check_dev(recv_scores, *isl, torch::kFloat32, "recv_scores");
             const int64_t rw = isl->row_bytes() / 4;
             TORCH_CHECK(send_rows.numel() >= (int64_t)k * rw && recv_rows.numel() >= (int64_t)k * rw &&
                             send_scores.numel() >= k && recv_scores.numel() >= k,
                         "staging buffers too small");
             TORCH_CHECK(dst >= 0 && dst < e.nranks && src >= 0 && src < e.nranks, "peer out of range");
             std::vector<pga::LocalRank> local{local_of(*isl, e.rank, send_rows, send_scores, recv_rows, recv_scores)};
             e.compute = isl->stream;
             e.on_transport = use_transport(e, *isl, local[0]);
             if (e.on_transport) {  // the transport stream waits for the population, then selects the emigrants
               hipStream_t ts = e.comm->transport_stream(local[0]);
               PGA_HIP_CHECK(hipEventRecord(e.ev_pop, e.compute));
               PGA_HIP_CHECK(hipStreamWaitEvent(ts, e.ev_pop, 0));
               isl->stream = ts;
               local[0].stream = ts;
             }
             try {
               isl->emigrate(k, send_rows.data_ptr(), send_scores.data_ptr<float>());
             } catch (...) {
               isl->stream = e.compute;
               throw;
             }
             isl->stream = e.compute;
             // the emigrants are packed: fence() lets the compute stream
             // overwrite the population they came from (generation + 2)
             if (e.on_transport) PGA_HIP_CHECK(hipEventRecord(e.ev_out, local[0].stream));
             e.comm->self_exchange = e.nranks == 1;
             e.comm->exchange(ring_plan(e.rank, dst, src, k), local);
             // PGA_MIG_EVAL_EARLY=1: the re-scoring of the received rows is
             // enqueued now, behind the transfer on the transport stream, so
             // it runs as soon as the rows land (in the drain of the
             // generation beside it) instead of after finish()'s host check
             e.early_eval = false;
             static const bool early = std::getenv("PGA_MIG_EVAL_EARLY") && std::getenv("PGA_MIG_EVAL_EARLY")[0] == '1';
             hipStream_t ts = early ? e.comm->transport_stream(local[0]) : nullptr;
             if (ts) {
               if (!e.ev_in) PGA_HIP_CHECK(hipEventCreateWithFlags(&e.ev_in, hipEventDisableTiming));
               isl->stream = ts;
               try {
                 isl->evaluate_rows(local[0].recv_rows, local[0].recv_scores, k);
               } catch (...) {
                 isl->stream = e.compute;
                 throw;
               }
               isl->stream = e.compute;
               PGA_HIP_CHECK(hipEventRecord(e.ev_in, ts));
               e.early_eval = true;
             }
             e.pending = std::move(local);
           })
      // complete the epoch: false = failed / expired (the communicator was
      // aborted, nothing was received); true = the k received rows were
      // re-scored (validate) and replaced the bottom-k
      .def("finish",
           [](EngineComm& e, const IslandPtr& isl, uint32_t k, double timeout_s, bool validate) {
             TORCH_CHECK(!e.pending.empty(), "no exchange in flight");
             std::vector<pga::LocalRank> local = std::move(e.pending);
             e.pending.clear();
             const hipStream_t compute = c10::hip::getCurrentHIPStream(isl->device()).stream();
             isl->stream = compute;
             // on_transport: local[0].stream is the transport stream itself
             // (the wait orders nothing); else the compute stream waits
             if (!e.on_transport) local[0].stream = compute;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = e.comm->wait(local, timeout_s);
             }
             if (!ok) return false;
             if (e.early_eval) {  // re-scored at post time: the compute stream waits for that
               PGA_HIP_CHECK(hipStreamWaitEvent(compute, e.ev_in, 0));
             } else if (validate) {
               isl->stream = e.on_transport ? local[0].stream : compute;
               try {
                 isl->evaluate_rows(local[0].recv_rows, local[0].recv_scores, k);
               } catch (...) {
                 isl->stream = compute;
                 throw;
               }
               isl->stream = compute;
             }
             if (e.on_transport && !e.early_eval) {  // the compute stream takes the re-scored immigrants
               PGA_HIP_CHECK(hipEventRecord(e.ev_in, local[0].stream));
               PGA_HIP_CHECK(hipStreamWaitEvent(compute, e.ev_in, 0));
             }
             isl->immigrate(k, local[0].recv_rows, local[0].recv_scores);
             return true;
           },
           py::arg("island"), py::arg("k"), py::arg("timeout_s") = 0.0, py::arg("validate") = true)
      // order the compute stream after the epoch's emigrant packing: call
      // once the generation after the epoch's departure is enqueued (the
      // packing reads the population the generation after that overwrites)
      .def("fence",
           [](EngineComm& e, const IslandPtr& isl) {
             if (e.pending.empty() || !e.on_transport) return;
             PGA_HIP_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream(isl->device()).stream(), e.ev_out, 0));
           })
      .def_property_readonly("in_flight", [](const EngineComm& e) { return !e.pending.empty(); });
}
