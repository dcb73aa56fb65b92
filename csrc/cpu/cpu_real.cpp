#include <stdexcept>
#include "pga/cpu.hpp"
namespace pga { namespace cpu {
uint32_t real_run(int, const GenArgs&, unsigned long long*) { throw std::runtime_error("REAL encoding: not built yet"); }
uint32_t perm_run(int, const GenArgs&, unsigned long long*) { throw std::runtime_error("PERMUTATION encoding: not built yet"); }
}}
