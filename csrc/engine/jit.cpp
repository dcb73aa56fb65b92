// jit.cpp — hipRTC compilation of user objectives (see jit.hpp).
#include "pga/jit.hpp"

#include <dlfcn.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <stdexcept>

#include "pga/core.hpp"
#include "pga/ops.hpp"

extern char** environ;

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
  k->user_source = source;
  k->options = extra_options;
  rtc_program prog = nullptr;
  if (r.create(&prog, k->source.c_str(), "pga_jit_objective.hip", 0, nullptr, nullptr) != 0)
    throw std::runtime_error("hiprtcCreateProgram failed");
  // -ffp-contract=fast as in the fused build (build_gen_object): both
  // compilations of an objective then form the same fused multiply-adds
  std::vector<std::string> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast"};
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
  for (const GenVariant& v : gen_)
    if (v.mod) (void)hipModuleUnload(v.mod);
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

// ------------------------------------------------------------ fused generation
std::string jit_bitcode_dir() {
  if (const char* e = std::getenv("PGA_JIT_DIR")) return e;
  Dl_info info;
  if (dladdr((const void*)&jit_compile, &info) && info.dli_fname) {
    std::string so = info.dli_fname;
    const size_t k = so.find_last_of('/');
    const std::string dir = k == std::string::npos ? "." : so.substr(0, k);
    for (const std::string& c : {dir + "/jit", dir + "/../build/jit"}) {
      FILE* f = std::fopen((c + "/gen_8_1_0.bc").c_str(), "rb");
      if (f) {
        std::fclose(f);
        return c;
      }
    }
  }
  return "build/jit";
}

namespace {
// the jitgen.hip symbol of binary_gen_tp<GS, kObjJit = 1001, FULL, DENSE>, or
// jitgen_real.hip's real_gen_tp<GS, kObjJit, false>
std::string gen_symbol(int encoding, uint32_t gs, bool full, bool dense) {
  if (encoding == ENC_REAL) return "_ZN3pga6jitgen11real_gen_tpILi" + std::to_string(gs) + "ELi1001ELb0EEEvNS_7GenArgsEPy";
  return "_ZN3pga6jitgen13binary_gen_tpILi" + std::to_string(gs) + "ELi1001ELb" + (full ? "1" : "0") + "ELb" +
         (dense ? "1" : "0") + "EEEvNS_7GenArgsEPy";
}

std::vector<char> read_file(const std::string& path) {
  std::vector<char> v;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return v;
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + n);
  std::fclose(f);
  return v;
}

// Runs `cmd` (a /bin/sh command line) as a child process (posix_spawn, never
// an exec of this process), output appended to `log`; returns its exit status.
int spawn_shell(const std::string& cmd, const std::string& log) {
  const std::string full = cmd + " >> '" + log + "' 2>&1";
  const char* argv[] = {"/bin/sh", "-c", full.c_str(), nullptr};
  pid_t pid = 0;
  if (posix_spawn(&pid, "/bin/sh", nullptr, nullptr, (char* const*)argv, environ) != 0) return -1;
  int st = 0;
  if (waitpid(pid, &st, 0) != pid) return -1;
  return WIFEXITED(st) ? WEXITSTATUS(st) : -1;
}

// The code-object cache: $PGA_JIT_CACHE, else $XDG_CACHE_HOME/pga_jit, else
// ~/.cache/pga_jit.  Code objects found there are loaded and launched, so the
// directory must be private: it is created 0700 and used only if it is a real
// directory (not a symlink) owned by this user and not group/world-writable.
std::string jit_cache_dir() {
  std::string dir;
  if (const char* e = std::getenv("PGA_JIT_CACHE")) {
    dir = e;
  } else if (const char* x = std::getenv("XDG_CACHE_HOME"); x && *x) {
    dir = std::string(x) + "/pga_jit";
  } else if (const char* h = std::getenv("HOME"); h && *h) {
    dir = std::string(h) + "/.cache/pga_jit";
  } else {
    throw std::runtime_error("no private JIT cache directory: set PGA_JIT_CACHE, XDG_CACHE_HOME or HOME");
  }
  while (dir.size() > 1 && dir.back() == '/') dir.pop_back();
  // parents as needed (0700), then the directory itself
  for (size_t k = dir.find('/', 1); k != std::string::npos; k = dir.find('/', k + 1))
    (void)mkdir(dir.substr(0, k).c_str(), 0700);
  (void)mkdir(dir.c_str(), 0700);
  struct stat st;
  if (lstat(dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode))
    throw std::runtime_error("JIT cache " + dir + " is not a directory");
  if (st.st_uid != getuid() || (st.st_mode & (S_IWGRP | S_IWOTH)) != 0)
    throw std::runtime_error("JIT cache " + dir + " is not private (owner " + std::to_string(st.st_uid) +
                             ", mode " + std::to_string(st.st_mode & 0777) + "): refusing to load code from it");
  return dir;
}

std::string shell_quote(const std::string& v) {
  std::string r = "'";
  for (char ch : v) {
    if (ch == '\'') r += "'\\''";
    else r += ch;
  }
  return r + "'";
}

std::string read_text(const std::string& path) {
  std::vector<char> v = read_file(path);
  return std::string(v.begin(), v.end());
}
}  // namespace

// The user objective is compiled to LLVM bitcode and linked with the kernel's
// bitcode by the ROCm toolchain this library was built with (hipcc + clang/lld
// LTO), in a child process, cached on disk by content.  Not hiprtcLink*: in a
// process where another HIP runtime is already loaded (PyTorch bundles its own
// HIP / COMGR) hipRTC links with that older LLVM, which cannot read bitcode
// from this build's compiler.
std::string JitKernel::build_gen_object(uint32_t gs, bool full, bool dense, uint32_t L) {
  if (encoding != ENC_BINARY && encoding != ENC_REAL)
    throw std::invalid_argument("fused generation kernels are BINARY and REAL only");
  if (gs == 0 || gs > 64 || (gs & (gs - 1)) != 0) throw std::invalid_argument("group size must be a power of two <= 64");
  const bool real = encoding == ENC_REAL;
  const std::string variant =
      real ? "real_" + std::to_string(gs) : std::to_string(gs) + "_" + (full ? "1" : "0") + "_" + (dense ? "1" : "0");
  const std::string kbc = jit_bitcode_dir() + "/gen_" + variant + ".bc";
  const std::string kbc_text = read_text(kbc);
  if (kbc_text.empty())
    throw std::runtime_error("no generation-kernel bitcode at " + kbc + " (tools/build.py builds it)");
  const char* rp = std::getenv("ROCM_PATH");
  const std::string rocm = rp && *rp ? rp : "/opt/rocm";
  // the user's source + the external-linkage entry the kernel bitcode calls:
  // the row arrives as an LDS pointer (the kernel stages each step's children
  // there: ds loads, not flat) and the genome length as a constant, so fixed-trip loops over the row unroll with
  // every load in flight (the length is part of the cache key)
  const std::string T = real ? "float" : "unsigned int";
  const std::string src = "#include <hip/hip_runtime.h>\n#line 1 \"user_objective\"\n" + user_source + "\n" +
                          "extern \"C\" __device__ float " + (real ? "pga_user_objective_f32" : "pga_user_objective") +
                          "(__attribute__((address_space(3))) const " + T +
                          "* w, unsigned int, const float* d) { return " +
                          name + "((const " + T + "*)w, " + std::to_string(L) + "u, d); }\n";
  // the user's compile options (-D, -I, ...) apply to the fused objective as
  // they do to the evaluation kernel, and are part of the cache key
  std::string uopts;
  for (const std::string& o : options) uopts += " " + shell_quote(o);
  const std::string h = std::to_string(std::hash<std::string>{}(src + "|" + uopts + "|" + kbc_text));
  const std::string dir = jit_cache_dir();
  const std::string base = dir + "/obj_" + h;
  const std::string co = base + "_" + variant + ".co", log = base + "_" + variant + ".log";
  if (!read_file(co).empty()) return co;
  // per-process intermediates; the code object appears atomically (rename),
  // so concurrent processes compiling the same objective never see a partial one
  const std::string pid = std::to_string((unsigned)getpid());
  const std::string tmp = co + ".tmp" + pid, work = base + "_" + variant + "_" + pid;
  FILE* f = std::fopen((work + ".hip").c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + work + ".hip");
  std::fwrite(src.data(), 1, src.size(), f);
  std::fclose(f);
  // unoptimised bitcode on both sides: the link optimises the whole kernel
  // once, with the objective inlined (optimising twice costs registers)
  const std::string cc = "'" + rocm + "/bin/hipcc' -x hip --offload-arch=gfx950 -O3 -Xclang -disable-llvm-passes "
                         "-std=c++17 -ffp-contract=fast -fgpu-rdc --cuda-device-only -emit-llvm" + uopts + " -c '" +
                         work + ".hip' -o '" + work + ".bc'";
  // -flto: one LTO module, so the objective inlines into the kernel (without
  // it each bitcode is compiled on its own and the objective is a call)
  const std::string ld = "'" + rocm + "/lib/llvm/bin/clang' --target=amdgcn-amd-amdhsa -mcpu=gfx950 -O3 -flto '" + kbc +
                         "' '" + work + ".bc' -o '" + tmp + "' && mv '" + tmp + "' '" + co + "'";
  const bool ok_cc = spawn_shell(cc, log) == 0;
  const bool ok_ld = ok_cc && spawn_shell(ld, log) == 0;
  (void)std::remove((work + ".hip").c_str());
  (void)std::remove((work + ".bc").c_str());
  if (!ok_cc) throw std::runtime_error("compiling the objective to bitcode failed:\n" + read_text(log));
  if (!ok_ld) throw std::runtime_error("linking the fused generation kernel failed:\n" + read_text(log));
  if (read_file(co).empty()) throw std::runtime_error("the linker produced no code object: " + co);
  return co;
}

hipFunction_t JitKernel::gen_function(int device, uint32_t gs, bool full, bool dense, uint32_t L, bool build) {
  if ((encoding != ENC_BINARY && encoding != ENC_REAL) || fused_failed_ || device < 0) return nullptr;
  // (L, gs, full, dense) in disjoint fields: gs * 4 + 3 < 2^16
  const uint64_t key = ((uint64_t)L << 16) | (gs * 4u + (full ? 2u : 0u) + (dense ? 1u : 0u));
  for (const GenVariant& v : gen_)
    if (v.device == device && v.key == key) return v.fn;
  if (!build) return nullptr;
  std::vector<char> image;
  try {
    image = read_file(build_gen_object(gs, full, dense, L));
  } catch (const std::exception& e) {
    fused_failed_ = true;
    fused_error_ = e.what();
    return nullptr;
  }
  PGA_HIP_CHECK(hipSetDevice(device));
  GenVariant v{device, key, nullptr, nullptr, 1, std::make_shared<std::vector<char>>(std::move(image))};
  hipError_t e = hipModuleLoadData(&v.mod, v.image->data());
  if (e == hipSuccess) e = hipModuleGetFunction(&v.fn, v.mod, gen_symbol(encoding, gs, full, dense).c_str());
  if (e != hipSuccess) {
    if (v.mod) (void)hipModuleUnload(v.mod);
    fused_failed_ = true;
    fused_error_ = std::string("loading the fused generation kernel: ") + hipGetErrorString(e);
    return nullptr;
  }
  int occ = 0;  // resident 4-wave blocks per CU (tp_geometry_occ)
  const uint32_t lds4 = tp_dyn_lds_bytes(4) + tp_jit_stage_bytes(4);
  if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&occ, v.fn, 256, lds4) != hipSuccess ||
      occ <= 0)
    occ = 1;
  v.occ = (uint32_t)occ;
  gen_.push_back(v);
  return v.fn;
}

uint32_t JitKernel::gen_launch(hipFunction_t f, const void* args, size_t args_bytes, uint64_t S,
                               unsigned long long* parts, uint32_t max_grid, hipStream_t s) {
  uint32_t occ = 1;
  for (const GenVariant& v : gen_)
    if (v.fn == f) occ = v.occ;
  // the geometry the built-in kernels get (tp_geometry)
  if (args_bytes != sizeof(GenArgs)) throw std::invalid_argument("fused generation: kernel arguments are not a GenArgs");
  GenArgs a;
  std::memcpy(&a, args, sizeof(a));
  const TpGeom t = tp_geometry_occ(S, 1, occ, 64 / group_size(a.chunks));
  a.tp_unit = t.unit;
  const uint32_t grid = std::min(t.grid, max_grid);
  a.tp_pool_units = a.tp_pool && grid == t.grid ? tp_pool_units(t, S) : 0u;
  a.tp_skew = grid == t.grid && a.encoding == ENC_BINARY ? tp_skew_units(t, S) : 0u;
  // kernel arguments as one packed buffer: (GenArgs a, unsigned long long* parts)
  std::vector<char> buf(args_bytes + 16);
  std::memcpy(buf.data(), &a, args_bytes);
  size_t off = (args_bytes + 7) & ~(size_t)7;
  std::memcpy(buf.data() + off, &parts, sizeof(parts));
  size_t total = off + sizeof(parts);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, buf.data(), HIP_LAUNCH_PARAM_BUFFER_SIZE, &total,
                 HIP_LAUNCH_PARAM_END};
  // the kernels stage each step's children in LDS for the objective
  const uint32_t lds = t.lds + tp_jit_stage_bytes(t.block / 64);
  PGA_HIP_CHECK(hipModuleLaunchKernel(f, grid, 1, 1, t.block, 1, 1, lds, s, nullptr, cfg));
  return grid;
}

}  // namespace pga
