// An empty kernel as a code object (hipcc --genco) for tools/launch_cost's module-launch
// rows: the library launches its per-tree kernels through hipModuleLaunchKernel.
#include <hip/hip_runtime.h>
struct Arg {
    unsigned int w[80];
};
extern "C" __global__ void k_empty_mod(Arg a) {
    if (a.w[0] == 0xdeadbeefu && threadIdx.x == 1234567) a.w[1] = 0;
}
