// jit.cpp — hipRTC compilation of user objectives (see jit.hpp).
#include "pga/jit.hpp"

#include <dlfcn.h>

#include <mutex>
#include <stdexcept>

#include "pga/core.hpp"
#include "pga/ops.hpp"

namespace pga {

namespace {

// --- minimal hipRTC binding (dlopen) ---
typedef int rtc_result;
typedef void* rtc_program;
struct Rtc {
  rtc_result (*create)(rtc_program*, const char*, const char*, int, const char* const*, const char* const*) = nullptr;
  rtc_result (*compile)(rtc_program, int, const char* const*) = nullptr;
  rtc_result (*destroy)(rtc_program*) = nullptr;
  rtc_result (*log_size)(rtc_program, size_t*) = nullptr;
  rtc_result (*get_log)(rtc_program, char*) = nullptr;
  rtc_result (*code_size)(rtc_program, size_t*) = nullptr;
  rtc_result (*get_code)(rtc_program, char*) = nullptr;
  const char* (*error_string)(rtc_result) = nullptr;
  std::string why;
};

Rtc& rtc() {
  static Rtc r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("libhiprtc.so.7", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/libhiprtc.so.7", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("libhiprtc.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      r.why = std::string("cannot load libhiprtc: ") + (e ? e : "?");
      return;
    }
    r.create = (decltype(r.create))dlsym(h, "hiprtcCreateProgram");
    r.compile = (decltype(r.compile))dlsym(h, "hiprtcCompileProgram");
    r.destroy = (decltype(r.destroy))dlsym(h, "hiprtcDestroyProgram");
    r.log_size = (decltype(r.log_size))dlsym(h, "hiprtcGetProgramLogSize");
    r.get_log = (decltype(r.get_log))dlsym(h, "hiprtcGetProgramLog");
    r.code_size = (decltype(r.code_size))dlsym(h, "hiprtcGetCodeSize");
    r.get_code = (decltype(r.get_code))dlsym(h, "hiprtcGetCode");
    r.error_string = (decltype(r.error_string))dlsym(h, "hiprtcGetErrorString");
    if (!r.create || !r.compile || !r.destroy || !r.code_size || !r.get_code) r.why = "libhiprtc lacks symbols";
  });
  return r;
}

const char* gene_type(int encoding) {
  switch (encoding) {
    case ENC_BINARY: return "unsigned int";
    case ENC_REAL: return "float";
    case ENC_PERMUTATION: return "unsigned short";
    default: throw std::invalid_argument("unknown encoding");
  }
}

// The evaluation kernel around the user's function.  The packed best format
// is pga::pack_best (core.hpp): orderable f32 key << 32 | (2^32-1 - index).
const char* kKernelTail = R"(
namespace pga_jit_detail {
__device__ __forceinline__ unsigned int score_key(float s) {
  const unsigned int u = __float_as_uint(s);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }
}  // namespace pga_jit_detail

// Rows are staged through LDS a tile at a time: the tile is copied with
// coalesced dword loads, then work-item t evaluates row t from LDS.  The LDS
// row stride is row_words + 1 so that work-items walking their rows in step
// hit different banks.
extern "C" __global__ __launch_bounds__(256) void pga_jit_eval(const unsigned int* rows, unsigned int row_words,
    unsigned long long S, unsigned int L, const float* data, float* scores, unsigned long long* parts,
    unsigned int tile) {
  extern __shared__ unsigned int lds_rows[];
  __shared__ unsigned long long red[4];
  const unsigned int stride = row_words + 1;
  unsigned long long best = 0;
  for (unsigned long long base = (unsigned long long)blockIdx.x * tile; base < S;
       base += (unsigned long long)gridDim.x * tile) {
    const unsigned int n = (S - base < tile) ? (unsigned int)(S - base) : tile;
    const unsigned int* src = rows + base * row_words;
    for (unsigned int w = threadIdx.x; w < n * row_words; w += 256) {
      const unsigned int r = w / row_words, c = w - r * row_words;
      lds_rows[r * stride + c] = src[w];
    }
    __syncthreads();
    for (unsigned int t = threadIdx.x; t < n; t += 256) {
      const unsigned long long i = base + t;
      const float s = PGA_OBJECTIVE((const PGA_GENE*)(lds_rows + t * stride), L, data);
      scores[i] = s;
      const unsigned long long p = ((unsigned long long)pga_jit_detail::score_key(s) << 32) |
                                   (0xFFFFFFFFull - (unsigned int)i);
      best = pga_jit_detail::umax64(best, p);
    }
    __syncthreads();
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned int lo = __shfl_xor((unsigned int)best, o, 64), hi = __shfl_xor((unsigned int)(best >> 32), o, 64);
    best = pga_jit_detail::umax64(best, ((unsigned long long)hi << 32) | lo);
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    best = pga_jit_detail::umax64(pga_jit_detail::umax64(red[0], red[1]), pga_jit_detail::umax64(red[2], red[3]));
    parts[blockIdx.x] = best;
  }
}
)";

}  // namespace

std::string jit_kernel_source(int encoding, const std::string& source, const std::string& name) {
  std::string s;  // hipRTC provides the HIP device built-ins itself
  s += "#define PGA_GENE " + std::string(gene_type(encoding)) + "\n";
  s += "#define PGA_OBJECTIVE " + name + "\n";
  s += "#line 1 \"user_objective\"\n";
  s += source;
  s += "\n";
  s += kKernelTail;
  return s;
}

std::shared_ptr<JitKernel> jit_compile(int encoding, const std::string& source, const std::string& name,
                                       const std::vector<std::string>& extra_options) {
  Rtc& r = rtc();
  if (!r.why.empty()) throw std::runtime_error(r.why);
  if (name.empty()) throw std::invalid_argument("objective function name is empty");
  auto k = std::make_shared<JitKernel>();
  k->encoding = encoding;
  k->name = name;
  k->source = jit_kernel_source(encoding, source, name);
  rtc_program prog = nullptr;
  if (r.create(&prog, k->source.c_str(), "pga_jit_objective.hip", 0, nullptr, nullptr) != 0)
    throw std::runtime_error("hiprtcCreateProgram failed");
  std::vector<std::string> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
  for (const auto& o : extra_options) opts.push_back(o);
  std::vector<const char*> copts;
  for (const auto& o : opts) copts.push_back(o.c_str());
  const rtc_result rc = r.compile(prog, (int)copts.size(), copts.data());
  size_t ls = 0;
  if (r.log_size && r.log_size(prog, &ls) == 0 && ls > 1) {
    std::string log(ls, '\0');
    if (r.get_log(prog, &log[0]) == 0) k->log = log.c_str();
  }
  if (rc != 0) {
    r.destroy(&prog);
    throw std::runtime_error(std::string("hipRTC compile of objective '") + name + "' failed (" +
                             (r.error_string ? r.error_string(rc) : "?") + "):\n" + k->log);
  }
  size_t cs = 0;
  if (r.code_size(prog, &cs) != 0 || cs == 0) {
    r.destroy(&prog);
    throw std::runtime_error("hipRTC produced no code");
  }
  k->code.resize(cs);
  r.get_code(prog, k->code.data());
  r.destroy(&prog);
  return k;
}

JitKernel::~JitKernel() {
  for (hipModule_t m : modules_)
    if (m) (void)hipModuleUnload(m);
}

hipFunction_t JitKernel::function(int device) {
  if (device < 0) throw std::invalid_argument("JIT objectives need the GPU backend");
  if ((size_t)device >= fns_.size()) {
    modules_.resize(device + 1, nullptr);
    fns_.resize(device + 1, nullptr);
  }
  if (!fns_[device]) {
    PGA_HIP_CHECK(hipSetDevice(device));
    PGA_HIP_CHECK(hipModuleLoadData(&modules_[device], code.data()));
    PGA_HIP_CHECK(hipModuleGetFunction(&fns_[device], modules_[device], "pga_jit_eval"));
  }
  return fns_[device];
}

uint32_t JitKernel::eval(int device, const void* rows, uint32_t row_words, uint64_t S, uint32_t L, const float* data,
                         float* scores, unsigned long long* parts, uint32_t grid, hipStream_t s) {
  hipFunction_t f = function(device);
  const unsigned int* r = (const unsigned int*)rows;
  unsigned int rw = row_words, l = L;
  unsigned long long n = S;
  // rows per LDS tile: up to 256 (one per work-item), at most 64 KiB of LDS
  unsigned int tile = (unsigned int)(65536 / (4ull * (row_words + 1)));
  tile = tile > 256 ? 256 : (tile < 1 ? 1 : tile);
  const size_t lds = 4ull * tile * (row_words + 1);
  if (lds > 65536) throw std::invalid_argument("JIT objective: row too large for LDS staging (> 64 KiB)");
  uint64_t blocks = (S + tile - 1) / tile;
  if (blocks > grid) blocks = grid;
  void* args[] = {&r, &rw, &n, &l, &data, &scores, &parts, &tile};
  PGA_HIP_CHECK(hipModuleLaunchKernel(f, (unsigned)blocks, 1, 1, 256, 1, 1, (unsigned)lds, s, args, nullptr));
  return (uint32_t)blocks;
}

}  // namespace pga
