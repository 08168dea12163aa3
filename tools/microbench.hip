// microbench.hip -- calibration of launch / boundary / small-kernel floors on
// the GPU box (not part of the product).  Prints one line per measurement.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -o tools/microbench
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);    \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 1024) p[0] = 1;
}
__global__ void k_write(int *__restrict__ p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    int4 *q = reinterpret_cast<int4 *>(p);
    for (; i < n / 4; i += gridDim.x * blockDim.x) q[i] = make_int4(i, i, i, i);
}
__global__ void k_copy(const int *__restrict__ a, int *__restrict__ b, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int4 *x = reinterpret_cast<const int4 *>(a);
    int4 *y = reinterpret_cast<int4 *>(b);
    for (; i < n / 4; i += gridDim.x * blockDim.x) y[i] = x[i];
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *buf, *buf2;
    const int N = 16 << 20;  // 64 MB of ints
    CK(hipMalloc(&buf, (size_t)N * 4));
    CK(hipMalloc(&buf2, (size_t)N * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int reps = 200;
    // (1) in-packet duration of an empty kernel at several grid sizes
    for (int grid : {1, 64, 256, 1024, 4096}) {
        double tot = 0;
        for (int r = 0; r < reps; ++r) {
            hipExtLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, a, b, 0, (int *)nullptr);
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            tot += ms;
        }
        printf("empty grid=%d: in-packet %.2f us\n", grid, tot / reps * 1e3);
    }
    // (2) write / copy of B bytes, in-packet duration
    for (int mb : {1, 4, 8, 16, 64}) {
        int n = mb << 18;
        for (int grid : {256, 1024, 2048}) {
            double tw = 0, tc = 0;
            for (int r = 0; r < reps; ++r) {
                float ms;
                hipExtLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, s, a, b, 0, buf, n);
                CK(hipEventSynchronize(b));
                CK(hipEventElapsedTime(&ms, a, b));
                tw += ms;
                hipExtLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, s, a, b, 0, (const int *)buf, buf2, n);
                CK(hipEventSynchronize(b));
                CK(hipEventElapsedTime(&ms, a, b));
                tc += ms;
            }
            tw = tw / reps * 1e3;
            tc = tc / reps * 1e3;
            printf("write %d MB grid=%d: %.2f us (%.0f GB/s)   copy: %.2f us (%.0f GB/s)\n", mb, grid, tw,
                   mb * 1.048576e6 / tw / 1e3, tc, 2 * mb * 1.048576e6 / tc / 1e3);
        }
    }
    // (3) back-to-back chains of k dependent empty kernels: wall per chain
    for (int k : {1, 2, 3, 4}) {
        CK(hipStreamSynchronize(s));
        double t0 = now_us();
        for (int r = 0; r < reps; ++r)
            for (int j = 0; j < k; ++j) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, (int *)nullptr);
        CK(hipStreamSynchronize(s));
        double t1 = now_us();
        printf("eager chain of %d empty kernels: %.2f us per chain (host+device)\n", k, (t1 - t0) / reps);
    }
    // (4) the same chains through a captured graph
    for (int k : {1, 3}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int r = 0; r < 50; ++r)
            for (int j = 0; j < k; ++j) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, (int *)nullptr);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        double t0 = now_us();
        for (int r = 0; r < 4; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        double t1 = now_us();
        printf("graph of 50 x chain(%d): %.2f us per chain\n", k, (t1 - t0) / 200);
    }
    // (5) a dependent chain of write 4 MB -> copy 4 MB, eager, wall per pair
    {
        int n = 4 << 18;
        CK(hipStreamSynchronize(s));
        double t0 = now_us();
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, s, buf, n);
            hipLaunchKernelGGL(k_copy, dim3(1024), dim3(256), 0, s, (const int *)buf, buf2, n);
        }
        CK(hipStreamSynchronize(s));
        printf("eager write4MB->copy4MB: %.2f us per pair\n", (now_us() - t0) / reps);
    }
    return 0;
}
