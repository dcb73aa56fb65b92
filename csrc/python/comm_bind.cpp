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

#include <memory>
#include <string>
#include <vector>

#include "pga/comm.hpp"
#include "pga/island.hpp"

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
};

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
             isl->emigrate(k, send_rows.data_ptr(), send_scores.data_ptr<float>());
             e.comm->self_exchange = e.nranks == 1;
             e.comm->exchange(ring_plan(e.rank, dst, src, k), local);
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
             isl->stream = c10::hip::getCurrentHIPStream(isl->device()).stream();
             local[0].stream = isl->stream;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = e.comm->wait(local, timeout_s);
             }
             if (!ok) return false;
             if (validate) isl->evaluate_rows(local[0].recv_rows, local[0].recv_scores, k);
             isl->immigrate(k, local[0].recv_rows, local[0].recv_scores);
             return true;
           },
           py::arg("island"), py::arg("k"), py::arg("timeout_s") = 0.0, py::arg("validate") = true)
      .def_property_readonly("in_flight", [](const EngineComm& e) { return !e.pending.empty(); });
}
