// chainbench.hip -- calibration (not product): durations of small kernels in a
// back-to-back dependent chain, as rocprofv3 --kernel-trace reports them.
//   hipcc --offload-arch=gfx950 -O3 tools/chainbench.hip -o chainbench
//   rocprofv3 --kernel-trace --stats -d out -- ./chainbench
// Every variant is its own kernel name so the stats table separates them.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e = (x);                                                 \
        if (e != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                                       \
        }                                                                   \
    } while (0)

template <int V>
__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 1024) p[0] = V;
}
template <int V>
__global__ void k_write(int *__restrict__ p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    int4 *q = reinterpret_cast<int4 *>(p);
    for (; i < n / 4; i += gridDim.x * blockDim.x) q[i] = make_int4(i, i, V, i);
}
// every block reads the same tbl_words table (16-B loads), sums, writes one word
template <int V>
__global__ void k_table(const int *__restrict__ t, int tbl_words, int *__restrict__ out) {
    const int4 *q = reinterpret_cast<const int4 *>(t);
    int s = 0;
    for (int i = threadIdx.x; i < tbl_words / 4; i += blockDim.x) {
        int4 v = q[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 0x7fffffff) out[blockIdx.x] = s + V;
}
// 4-byte scattered stores: 1M ints in runs of 64 (the emission's store shape)
template <int V>
__global__ void k_scatter(int *__restrict__ p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n; i += gridDim.x * blockDim.x) p[i] = i + V;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *buf, *tbl, *out;
    CK(hipMalloc(&buf, 64 << 20));
    CK(hipMalloc(&tbl, 1 << 20));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(tbl, 0, 1 << 20));
    const int reps = 400;
    auto wall = [&](const char *name, auto fn) -> int {
        for (int r = 0; r < 20; ++r) fn();
        CK(hipStreamSynchronize(s));
        double t0 = now_us();
        for (int r = 0; r < reps; ++r) fn();
        CK(hipStreamSynchronize(s));
        printf("%-40s %.2f us per iteration (wall)\n", name, (now_us() - t0) / reps);
        return 0;
    };
    wall("empty x1 (grid 256)", [&] { hipLaunchKernelGGL(k_empty<1>, dim3(256), dim3(256), 0, s, (int *)nullptr); });
    wall("empty x1 (grid 1024)", [&] { hipLaunchKernelGGL(k_empty<2>, dim3(1024), dim3(256), 0, s, (int *)nullptr); });
    wall("write 4 MB", [&] { hipLaunchKernelGGL(k_write<1>, dim3(1024), dim3(256), 0, s, buf, 1 << 20); });
    wall("write 8 MB", [&] { hipLaunchKernelGGL(k_write<2>, dim3(2048), dim3(256), 0, s, buf, 2 << 20); });
    wall("write 4 MB -> empty", [&] {
        hipLaunchKernelGGL(k_write<3>, dim3(1024), dim3(256), 0, s, buf, 1 << 20);
        hipLaunchKernelGGL(k_empty<3>, dim3(256), dim3(256), 0, s, (int *)nullptr);
    });
    wall("scatter 4 MB (dword stores)", [&] { hipLaunchKernelGGL(k_scatter<1>, dim3(1024), dim3(256), 0, s, buf, 1 << 20); });
    wall("table 28.5 KB x 224 blocks", [&] { hipLaunchKernelGGL(k_table<1>, dim3(224), dim3(256), 0, s, tbl, 7168, out); });
    wall("table 3.6 KB x 224 blocks", [&] { hipLaunchKernelGGL(k_table<2>, dim3(224), dim3(256), 0, s, tbl, 928, out); });
    wall("table 28.5 KB x 224 -> write 4 MB", [&] {
        hipLaunchKernelGGL(k_table<3>, dim3(224), dim3(256), 0, s, tbl, 7168, out);
        hipLaunchKernelGGL(k_write<4>, dim3(1024), dim3(256), 0, s, buf, 1 << 20);
    });
    return 0;
}
