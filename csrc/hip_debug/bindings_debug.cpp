// Diagnostic module _hip_debug (NOT part of the production _hip build): the LDS /
// register poison and LDS canary kernels of debug_poison.hip, used by
// scripts/debug_poison.py and scripts/debug_lds_canary.py. Built on demand by
// ops/build.py build_hip_debug() (or SSA_BUILD_DEBUG=1 with build_all()).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <stdint.h>

namespace ssa {
void poison_lds(uint32_t pat, int blocks, hipStream_t s);
void poison_regs(int blocks, hipStream_t s);
void lds_canary(int iters, unsigned* bad, int blocks, hipStream_t s);
}  // namespace ssa

PYBIND11_MODULE(_hip_debug, m) {
  m.doc() = "gfx950 diagnostic kernels: on-chip state poison and LDS canary";
  m.def("poison_lds", [](uint32_t pat, int blocks, uintptr_t stream) {
    ssa::poison_lds(pat, blocks, reinterpret_cast<hipStream_t>(stream));
  });
  m.def("poison_regs", [](int blocks, uintptr_t stream) {
    ssa::poison_regs(blocks, reinterpret_cast<hipStream_t>(stream));
  });
  m.def("lds_canary", [](int iters, uintptr_t bad, int blocks, uintptr_t stream) {
    ssa::lds_canary(iters, reinterpret_cast<unsigned*>(bad), blocks,
                    reinterpret_cast<hipStream_t>(stream));
  });
}
