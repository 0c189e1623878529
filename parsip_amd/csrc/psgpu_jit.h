// psgpu_jit.h — run-time specialised tree-walk kernels (hiprtc), see psgpu_jit.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <future>
#include <memory>
#include <string>
#include <vector>

#include "psgpu_model.h"

namespace psgpu {

struct JitKernels {
    hipModule_t mod = nullptr;
    hipFunction_t precheck = nullptr, mpu = nullptr, vertex = nullptr, vertexW = nullptr, finish = nullptr,
                  finishQ = nullptr, finishP = nullptr, probe = nullptr;
    hipFunction_t precheckS = nullptr, mpuS = nullptr;  // tree split at the root (two waves per item)
    hipFunction_t surface = nullptr;  // k_vertex + k_finish in one launch (small launches; with the split kernels)
    hipFunction_t surfaceW = nullptr;  // the same with one lane per vertex (PSGPU_OPT_FUSED_SURFACE 3)
    hipFunction_t front = nullptr, frontS = nullptr;  // k_precheck + k_mpu in one launch (k_front; unsplit / split)
};

extern const char* const kJitArch;  // "gfx950"

// A compiled code object (or the compiler's error) for one generated source.
struct JitCode {
    std::string key;         // source + embedded headers + tuning + toolchain
    std::vector<char> code;  // empty on failure
    std::string error;
};
using JitFuture = std::shared_future<std::shared_ptr<const JitCode>>;

// Request the model's specialised kernels: hiprtc compiles on a host thread (one job per
// distinct source; an on-disk cache serves repeats unless useDisk is false).  No GPU needed.
// baked: primitive / op parameters compiled in as literals (recompiles when they change).
JitFuture jit_request(const DevModel& m, bool baked, bool useDisk = true, bool split = false);
// Load a finished code object on `device` (the calling thread's current device), cached
// per device; nullptr + *err on failure (a stale cached object is dropped from the cache).
std::shared_ptr<JitKernels> jit_load(const JitCode& code, int device, std::string* err);
// Compile (and cache) without loading: code-object size, or -1 and *err.  No GPU needed.
long jit_compile_only(const DevModel& m, bool baked, std::string* err, bool split = false);
// The generated HIP source (tests and debugging).
std::string jit_source(const DevModel& m, bool baked, bool split = false);
// the generated walk splits at the root (TreeEval::kSplit): a binary known op over two ops
bool jit_splittable(const DevModel& m);
// Compat mode: compile a generated compact-tree source (psgpu_gui_jit.cpp) against the
// embedded compat headers, with the same on-disk cache.  Blocking; no GPU needed.
bool jit_compile_gui(const std::string& src, std::vector<char>& code, std::string* err);

}  // namespace psgpu
