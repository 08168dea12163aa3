// aqlbench_kernels.hip -- the two trivial kernels of tools/aqlbench.cpp (calibration only).
#include <hip/hip_runtime.h>

struct Args {
    int *out;
    int pad[168];
};

extern "C" __global__ __launch_bounds__(256) void k_a(Args a) {
    if (threadIdx.x == 0 && a.pad[blockIdx.x % 168] == 12345) a.out[blockIdx.x] = 1;
}
extern "C" __global__ __launch_bounds__(256) void k_b(Args a) {
    if (threadIdx.x == 0 && a.pad[(blockIdx.x + 1) % 168] == 12345) a.out[blockIdx.x] = 2;
}
