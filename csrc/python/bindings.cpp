// bindings.cpp — torch extension `libpga_amd._C`.
//
// Exposes the native Island runtime to Python.  Population buffers are
// returned as zero-copy torch tensors (from_blob views that keep the Island
// alive), so the python layer can hand them straight to torch.distributed
// (RCCL over xGMI) for migration, or to a user's vectorised torch objective.
// Every GPU call enqueues on torch's CURRENT stream of the island's device.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>
#include <pybind11/stl.h>

#include <atomic>
#include <memory>
#include <stdexcept>

#include "pga/cpu.hpp"
#include "pga/island.hpp"
#include "pga/trace.hpp"
#include "pga/ops.hpp"
#include "pga/real_ops.hpp"

namespace py = pybind11;
using pga::Island;
using IslandPtr = std::shared_ptr<Island>;

namespace {

void bind_stream(Island& isl) {
  if (isl.on_gpu()) isl.stream = c10::hip::getCurrentHIPStream(isl.device()).stream();
}

torch::Device dev_of(const Island& isl) {
  return isl.on_gpu() ? torch::Device(torch::kCUDA, isl.device()) : torch::Device(torch::kCPU);
}

torch::Tensor view(const IslandPtr& isl, void* ptr, std::vector<int64_t> sizes, torch::ScalarType t) {
  IslandPtr keep = isl;
  return torch::from_blob(
      ptr, sizes, [keep](void*) {}, torch::TensorOptions().dtype(t).device(dev_of(*isl)));
}

void check_tensor(const torch::Tensor& t, const Island& isl, torch::ScalarType st, const char* what) {
  TORCH_CHECK(t.is_contiguous(), what, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == st, what, " has the wrong dtype");
  TORCH_CHECK(t.device() == dev_of(isl), what, " must live on the island's device");
}

}  // namespace

void bind_comm(py::module& m);  // comm_bind.cpp: the engine's RCCL communicator

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X-native parallel genetic algorithm engine (gfx950 HIP kernels + CPU reference)";

#define E(name) m.attr(#name) = (int)pga::name
  E(ENC_BINARY); E(ENC_REAL); E(ENC_PERMUTATION);
  E(SEL_TOURNAMENT); E(SEL_ROULETTE); E(SEL_RANDOM); E(SEL_RANK);
  E(XO_UNIFORM); E(XO_ONE_POINT); E(XO_TWO_POINT); E(XO_BLEND); E(XO_ARITHMETIC); E(XO_PMX); E(XO_OX); E(XO_NONE);
  E(MUT_BIT_FLIP); E(MUT_GAUSSIAN); E(MUT_UNIFORM); E(MUT_RESET_ONE); E(MUT_SWAP); E(MUT_INVERSION); E(MUT_NONE);
  E(MIG_TOPK); E(MIG_STRIPE);
  E(OBJ_NONE); E(OBJ_ONEMAX); E(OBJ_KNAPSACK); E(OBJ_TRAP); E(OBJ_LEADING_ONES); E(OBJ_QUBO);
  E(OBJ_SPHERE); E(OBJ_RASTRIGIN); E(OBJ_ROSENBROCK); E(OBJ_ACKLEY); E(OBJ_GRIEWANK); E(OBJ_SCHWEFEL);
  E(OBJ_LINEAR); E(OBJ_KNAPSACK_REAL); E(OBJ_TSP_RANDOM_KEY); E(OBJ_TSP); E(OBJ_TSP_OPEN); E(OBJ_TSP_EUC); E(OBJ_USER_FNPTR);
  E(MODE_GEN); E(MODE_INIT); E(MODE_EVAL); E(MODE_CROSS); E(MODE_MUTATE);
#undef E
  m.attr("MAX_GRID") = (int)pga::kMaxGrid;

  py::class_<pga::Config>(m, "Config")
      .def(py::init<>())
      .def_readwrite("encoding", &pga::Config::encoding)
      .def_readwrite("S", &pga::Config::S)
      .def_readwrite("L", &pga::Config::L)
      .def_readwrite("selection", &pga::Config::selection)
      .def_readwrite("tour_k", &pga::Config::tour_k)
      .def_readwrite("crossover", &pga::Config::crossover)
      .def_readwrite("xo_prob", &pga::Config::xo_prob)
      .def_readwrite("blend_alpha", &pga::Config::blend_alpha)
      .def_readwrite("mutation", &pga::Config::mutation)
      .def_readwrite("mut_rate", &pga::Config::mut_rate)
      .def_readwrite("sigma", &pga::Config::sigma)
      .def_readwrite("rank_pressure", &pga::Config::rank_pressure)
      .def_readwrite("lo", &pga::Config::lo)
      .def_readwrite("hi", &pga::Config::hi)
      .def_readwrite("objective", &pga::Config::objective)
      .def_readwrite("obj_i", &pga::Config::obj_i)
      .def_readwrite("obj_f0", &pga::Config::obj_f0)
      .def_readwrite("obj_f1", &pga::Config::obj_f1)
      .def_readwrite("n_elite", &pga::Config::n_elite)
      .def_readwrite("seed", &pga::Config::seed)
      .def_readwrite("island", &pga::Config::island);

  m.def("row_geometry", [](int enc, uint32_t L) {
    uint32_t rw, ch;
    pga::row_geometry(enc, L, &rw, &ch);
    return py::make_tuple(rw, ch);
  });
  m.def("group_size", &pga::group_size);
  py::class_<pga::JitKernel, std::shared_ptr<pga::JitKernel>>(m, "JitKernel")
      .def_readonly("encoding", &pga::JitKernel::encoding)
      .def_readonly("name", &pga::JitKernel::name)
      .def_readonly("source", &pga::JitKernel::source)
      .def_readonly("log", &pga::JitKernel::log)
      .def_property_readonly("code_size", [](const pga::JitKernel& k) { return k.code.size(); })
      .def("build_generation_object", &pga::JitKernel::build_gen_object, py::arg("group_size"), py::arg("full"),
           py::arg("dense"), py::arg("length"));
  m.def("jit_compile", &pga::jit_compile, py::arg("encoding"), py::arg("source"), py::arg("name"),
        py::arg("options") = std::vector<std::string>{}, py::call_guard<py::gil_scoped_release>());
  m.def("jit_kernel_source", &pga::jit_kernel_source);
  // several same-shape islands of one device as one launch per generation
  // (Island::run_batched); False (nothing run) when they do not qualify
  m.def("run_islands_batched", [](std::vector<Island*> isls, uint32_t n) {
    if (isls.empty() || !isls[0] || !isls[0]->on_gpu()) return false;
    hipStream_t s = c10::hip::getCurrentHIPStream(isls[0]->device()).stream();
    return Island::run_batched(isls, n, s);
  });
  m.def("max_batched_islands", &pga::binary_max_batch);
  m.def("trace_level", &pga::trace_level);
  m.def("trace_push", [](const std::string& n) { pga::trace_push(n.c_str()); });
  m.def("trace_pop", &pga::trace_pop);
  m.def("trace_mark", [](const std::string& n) { pga::trace_mark(n.c_str()); });
  m.def("philox", [](uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    pga::u32x4 r = pga::philox4x32_10(pga::u32x4{c0, c1, c2, c3}, k0, k1);
    return py::make_tuple(r.x, r.y, r.z, r.w);
  });
  m.def("perm_crossover", [](int op, const std::vector<uint16_t>& A, const std::vector<uint16_t>& B, uint32_t lo,
                             uint32_t hi) {
    if (A.empty() || A.size() != B.size() || hi > A.size() || lo > hi)
      throw std::invalid_argument("perm_crossover: bad arguments");
    // both parents must be permutations of [0, L): the operators index position
    // maps by gene value
    for (const auto* P : {&A, &B}) {
      std::vector<char> seen(A.size(), 0);
      for (uint16_t x : *P) {
        if (x >= A.size() || seen[x]) throw std::invalid_argument("perm_crossover: parents must be permutations of [0, L)");
        seen[x] = 1;
      }
    }
    std::vector<uint16_t> C(A.size());
    pga::cpu::perm_crossover(op, A.data(), B.data(), (uint32_t)A.size(), lo, hi, C.data());
    return C;
  });
  // test hook of the CPU worker pool: sums [0, n) over the pool's slots; the
  // slot holding index throw_at (if < n) throws, which must surface here as
  // one exception after every slot has finished
  m.def("_pool_sum", [](uint64_t n, uint64_t throw_at) {
    std::atomic<uint64_t> sum{0};
    pga::cpu::parallel_for(n, 1, [&](uint64_t b, uint64_t e, unsigned) {
      uint64_t acc = 0;
      for (uint64_t i = b; i < e; ++i) {
        if (i == throw_at) throw std::runtime_error("pool test: slot failed");
        acc += i;
      }
      sum += acc;
    });
    return sum.load();
  });
  // the deterministic Box-Muller of the REAL gaussian mutation (real_ops.hpp)
  m.def("gauss_z", [](uint32_t w1, uint32_t w2) { return pga::gauss_z(w1, w2); });
  m.def("gauss_z_batch", [](torch::Tensor w) {
    auto wc = w.to(torch::kInt64).contiguous();
    TORCH_CHECK(wc.dim() == 2 && wc.size(1) == 2, "gauss_z_batch: [n, 2] words");
    auto out = torch::empty({wc.size(0)}, torch::dtype(torch::kFloat32));
    const int64_t* p = wc.data_ptr<int64_t>();
    float* o = out.data_ptr<float>();
    for (int64_t i = 0; i < wc.size(0); ++i) o[i] = pga::gauss_z((uint32_t)p[2 * i], (uint32_t)p[2 * i + 1]);
    return out;
  });
  m.def("mut_table", [](float p, uint32_t L) {
    auto t = torch::empty({(int64_t)L}, torch::dtype(torch::kInt64));
    std::vector<uint32_t> thr(L);
    float inv;
    pga::build_mut_table(p, L, thr.data(), &inv);
    for (uint32_t i = 0; i < L; ++i) t[i] = (int64_t)thr[i];
    return py::make_tuple(t, inv);
  });

  py::class_<Island, IslandPtr>(m, "Island")
      .def(py::init([](const pga::Config& c, int device) { return std::make_shared<Island>(c, device); }),
           py::arg("config"), py::arg("device"))
      .def_property_readonly("row_words", &Island::row_words)
      .def_property_readonly("chunks", &Island::chunks)
      .def_property_readonly("on_gpu", &Island::on_gpu)
      .def_property_readonly("device", &Island::device)
      .def_property("generation", &Island::generation, &Island::set_generation)
      .def_property_readonly("epoch", &Island::epoch)
      .def("bump_epoch", &Island::bump_epoch)
      .def("set_jit_objective",
           [](Island& i, std::shared_ptr<pga::JitKernel> k) {
             bind_stream(i);
             i.set_jit_objective(std::move(k));
           })
      .def_property_readonly("has_jit", &Island::has_jit)
      .def_property_readonly("jit_fused_generations", &Island::jit_fused_generations)
      .def_property_readonly("jit_fused_error", &Island::jit_fused_error)
      .def_property("graph_generations", &Island::graph_generations, &Island::set_graph_generations)
      .def_property_readonly("graph_replays", &Island::graph_replays)
      .def_property_readonly("knapsack_digits", &Island::knapsack_digits)
      .def_property("migration_policy", &Island::migration_policy, &Island::set_migration_policy)
      .def_property("fused_histogram", &Island::fused_histogram, &Island::set_fused_histogram)
      .def_property_readonly("fused_histogram_ready", &Island::fused_histogram_ready)
      .def_property("persistent", &Island::persistent, &Island::set_persistent)
      .def("config", [](Island& i) { return i.config(); })
      .def("set_operators", [](Island& i, const pga::Config& c) { bind_stream(i); i.set_operators(c); })
      .def("set_objective_data",
           [](Island& i, torch::Tensor t, int which) {
             bind_stream(i);
             auto h = t.to(torch::kCPU, torch::kFloat32).contiguous();
             i.set_objective_data(h.data_ptr<float>(), (size_t)h.numel(), which);
           })
      .def("set_user_fn", [](Island& i, uint64_t f) { i.set_user_fn((void*)f); })
      .def("initialize", [](Island& i) { bind_stream(i); i.initialize(); })
      .def("evaluate", [](Island& i) { bind_stream(i); i.evaluate(); })
      .def("run", [](Island& i, uint32_t n) { bind_stream(i); i.run(n); }, py::arg("n") = 1)
      .def("run_until",
           [](Island& i, uint32_t n, float target, uint32_t every) {
             bind_stream(i);
             return i.run_until(n, target, every);
           },
           py::arg("n"), py::arg("target"), py::arg("check_every") = 10)
      .def("set_stats_history", &Island::set_stats_history)
      .def("set_history_manual", &Island::set_history_manual)
      .def("record_history_row", &Island::record_history_row)
      .def_property_readonly("stats_history", &Island::stats_history)
      .def("history",
           [](Island& i) {
             bind_stream(i);
             std::vector<float> h = i.history();
             torch::Tensor t = torch::empty({(int64_t)(h.size() / 4), 4}, torch::kFloat32);
             if (!h.empty()) std::memcpy(t.data_ptr<float>(), h.data(), 4 * h.size());
             return t;
           })
      .def("crossover_stage", [](Island& i) { bind_stream(i); i.crossover_stage(); })
      .def("mutate_stage", [](Island& i) { bind_stream(i); i.mutate_stage(); })
      .def("swap", &Island::swap)
      .def("rebest", [](Island& i) { bind_stream(i); i.rebest(); })
      .def("best",
           [](Island& i) {
             bind_stream(i);
             unsigned long long p = i.best_packed();
             return py::make_tuple(pga::best_score(p), (uint64_t)pga::best_index(p));
           })
      .def("stats",
           [](Island& i) {
             bind_stream(i);
             float s[4];
             i.stats(s);
             return py::make_tuple(s[0], s[1], s[2], s[3]);
           })
      .def("topk",
           [](const IslandPtr& i, uint32_t k, bool largest, bool sorted) {
             bind_stream(*i);
             auto out = torch::empty({(int64_t)k}, torch::TensorOptions().dtype(torch::kInt32).device(dev_of(*i)));
             i->topk(k, largest, (uint32_t*)out.data_ptr<int32_t>(), sorted);
             return out;
           },
           py::arg("k"), py::arg("largest") = true, py::arg("sorted") = true)
      .def("rows",
           [](const IslandPtr& i, int which) {
             return view(i, i->rows(which), {(int64_t)i->config().S, (int64_t)i->row_words()}, torch::kInt32);
           },
           py::arg("which") = 0)
      .def("scores",
           [](const IslandPtr& i, int which) {
             return view(i, i->scores(which), {(int64_t)i->config().S}, torch::kFloat32);
           },
           py::arg("which") = 0)
      .def("best_parts",
           [](const IslandPtr& i) { return view(i, i->best_parts(), {(int64_t)pga::kMaxGrid}, torch::kInt64); })
      .def_property("n_best", &Island::n_best, &Island::set_n_best)
      .def("gather",
           [](const IslandPtr& i, torch::Tensor idx, torch::Tensor out_rows, torch::Tensor out_scores) {
             bind_stream(*i);
             check_tensor(idx, *i, torch::kInt32, "idx");
             check_tensor(out_rows, *i, torch::kInt32, "out_rows");
             check_tensor(out_scores, *i, torch::kFloat32, "out_scores");
             const int64_t n = idx.numel();
             TORCH_CHECK(out_rows.numel() >= n * i->row_words() && out_scores.numel() >= n, "output too small");
             i->gather((const uint32_t*)idx.data_ptr<int32_t>(), (uint32_t)n, out_rows.data_ptr(),
                       out_scores.data_ptr<float>());
           })
      .def("scatter",
           [](const IslandPtr& i, torch::Tensor idx, torch::Tensor in_rows, torch::Tensor in_scores) {
             bind_stream(*i);
             check_tensor(idx, *i, torch::kInt32, "idx");
             check_tensor(in_rows, *i, torch::kInt32, "in_rows");
             check_tensor(in_scores, *i, torch::kFloat32, "in_scores");
             const int64_t n = idx.numel();
             TORCH_CHECK(in_rows.numel() >= n * i->row_words() && in_scores.numel() >= n, "input too small");
             i->scatter((const uint32_t*)idx.data_ptr<int32_t>(), (uint32_t)n, in_rows.data_ptr(),
                        in_scores.data_ptr<float>());
           })
      .def("emigrate",
           [](const IslandPtr& i, uint32_t k, torch::Tensor out_rows, torch::Tensor out_scores) {
             bind_stream(*i);
             check_tensor(out_rows, *i, torch::kInt32, "out_rows");
             check_tensor(out_scores, *i, torch::kFloat32, "out_scores");
             TORCH_CHECK(out_rows.numel() >= (int64_t)k * i->row_words() && out_scores.numel() >= k, "output too small");
             i->emigrate(k, out_rows.data_ptr(), out_scores.data_ptr<float>());
           })
      .def("immigrate",
           [](const IslandPtr& i, uint32_t k, torch::Tensor in_rows, torch::Tensor in_scores) {
             bind_stream(*i);
             check_tensor(in_rows, *i, torch::kInt32, "in_rows");
             check_tensor(in_scores, *i, torch::kFloat32, "in_scores");
             TORCH_CHECK(in_rows.numel() >= (int64_t)k * i->row_words() && in_scores.numel() >= k, "input too small");
             i->immigrate(k, in_rows.data_ptr(), in_scores.data_ptr<float>());
           })
      .def("evaluate_rows",
           [](const IslandPtr& i, torch::Tensor rows, torch::Tensor scores) {
             bind_stream(*i);
             check_tensor(rows, *i, torch::kInt32, "rows");
             check_tensor(scores, *i, torch::kFloat32, "scores");
             const int64_t n = scores.numel();
             TORCH_CHECK(rows.numel() >= n * i->row_words(), "rows too small");
             return i->evaluate_rows(rows.data_ptr(), scores.data_ptr<float>(), (uint32_t)n);
           })
      .def("row", [](Island& i, uint64_t k) {
        bind_stream(i);
        auto r = i.row_host(k);
        auto t = torch::empty({(int64_t)r.size()}, torch::dtype(torch::kInt32));
        std::memcpy(t.data_ptr<int32_t>(), r.data(), 4 * r.size());
        return t;
      })
      .def("save", [](Island& i, const std::string& p) { bind_stream(i); i.save(p); })
      .def("load", [](Island& i, const std::string& p) { bind_stream(i); i.load(p); })
      .def("synchronize", [](Island& i) { bind_stream(i); i.synchronize(); });
  bind_comm(m);
}
