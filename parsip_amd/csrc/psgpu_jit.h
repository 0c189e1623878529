// psgpu_jit.h — run-time specialised tree-walk kernels (hiprtc), see psgpu_jit.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <string>

#include "psgpu_model.h"

namespace psgpu {

struct JitKernels {
    hipModule_t mod = nullptr;
    hipFunction_t precheck = nullptr, mpu = nullptr, vertex = nullptr, finish = nullptr, probe = nullptr;
};

// Compiled (cached per structure and device) kernels for the model; nullptr + *err on failure.
// baked: primitive / op parameters compiled in as literals (recompiles when they change).
std::shared_ptr<JitKernels> jit_get(const DevModel& m, bool baked, int device, std::string* err);
// Compile (and cache) without loading: code-object size, or -1 and *err.  No GPU needed.
long jit_compile_only(const DevModel& m, bool baked, std::string* err);
// The generated HIP source (tests and debugging).
std::string jit_source(const DevModel& m, bool baked);

}  // namespace psgpu
