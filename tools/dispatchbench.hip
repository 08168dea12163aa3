// dispatchbench.hip -- calibration (not product): how fast does a grid enter?
// Each block records s_memrealtime (100 MHz, chip-wide) at entry; the spread
// between the first and the p50 / p90 / last entry is printed per variant.
//   hipcc --offload-arch=gfx950 -O3 tools/dispatchbench.hip -o tools/dispatchbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e = (x);                                                 \
        if (e != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                                       \
        }                                                                   \
    } while (0)

struct Big {
    unsigned long long *out;
    int pad[160];  // ~650 B of kernel arguments, like TickArgs
};

// work: spin for `spin` s_memtime ticks after the entry stamp (block lifetime)
template <int LDS>
__global__ __launch_bounds__(256) void k_stamp(unsigned long long *out, int spin) {
    __shared__ int s[LDS / 4 + 1];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t0;
    s[threadIdx.x % (LDS / 4 + 1)] = threadIdx.x;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - c0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(1);
    if (s[(threadIdx.x + 1) % (LDS / 4 + 1)] == -1) out[0] = 0;
}
__global__ __launch_bounds__(256) void k_stamp_big(Big b, int spin) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) b.out[blockIdx.x] = t0 + (unsigned long long)b.pad[blockIdx.x % 160] * 0;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - c0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(1);
}

// every kernel-argument word loaded before the entry stamp (like a copy of TickArgs)
__global__ __launch_bounds__(256) void k_stamp_bigload(Big b, int spin) {
    int acc = 0;
#pragma unroll
    for (int i = 0; i < 160; ++i) acc += b.pad[i];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) b.out[blockIdx.x] = t0 + (acc == 12345 ? 1 : 0);
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - c0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(1);
}

__global__ void k_write4(int *__restrict__ p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    int4 *q = reinterpret_cast<int4 *>(p);
    for (; i < n / 4; i += gridDim.x * blockDim.x) q[i] = make_int4(i, i, 7, i);
}

// a writer that also stores a few words into host-mapped pinned memory (like HostOut)
__global__ void k_write4_host(int *__restrict__ p, int n, long long *hostp) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    int4 *q = reinterpret_cast<int4 *>(p);
    if (blockIdx.x == 0 && threadIdx.x < 8) hostp[threadIdx.x] = n + threadIdx.x;
    for (; i < n / 4; i += gridDim.x * blockDim.x) q[i] = make_int4(i, i, 7, i);
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long *d;
    const int maxg = 4096;
    CK(hipMalloc(&d, maxg * 8));
    std::vector<unsigned long long> h(maxg);
    auto report = [&](const char *name, int g) -> int {
        std::vector<double> acc50, acc90, accmax;
        for (int rep = 0; rep < 30; ++rep) {
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h.data(), d, g * 8, hipMemcpyDeviceToHost));
            std::vector<unsigned long long> v(h.begin(), h.begin() + g);
            std::sort(v.begin(), v.end());
            acc50.push_back((v[g / 2] - v[0]) / 100.0);
            acc90.push_back((v[g * 9 / 10] - v[0]) / 100.0);
            accmax.push_back((v[g - 1] - v[0]) / 100.0);
            break;
        }
        printf("%-44s grid %5d: entry p50 +%.2f us, p90 +%.2f us, last +%.2f us  per id mod 8:", name, g, acc50[0],
               acc90[0], accmax[0]);
        {
            unsigned long long mn = ~0ull;
            for (int i = 0; i < g; ++i) mn = std::min(mn, h[i]);
            for (int x = 0; x < 8; ++x) {
                unsigned long long m = ~0ull;
                for (int i = x; i < g; i += 8) m = std::min(m, h[i]);
                printf(" %.2f", (m - mn) / 100.0);
            }
            printf("\n");
        }
        return 0;
    };
    {
        // the grid right after a kernel that dirtied 4 MB (as k_scan follows k_emit2)
        int *buf;
        CK(hipMalloc(&buf, 16 << 20));
        for (int g : {256, 708, 1024}) {
            for (int r = 0; r < 5; ++r) {
                hipLaunchKernelGGL(k_write4, dim3(1024), dim3(256), 0, s, buf, 1 << 20);
                hipLaunchKernelGGL(k_stamp<8192>, dim3(g), dim3(256), 0, s, d, 4000);
            }
            if (report("after a 4 MB write kernel, spin 4000", g)) return 1;
            for (int r = 0; r < 5; ++r) {
                hipLaunchKernelGGL(k_write4, dim3(1024), dim3(256), 0, s, buf, 1 << 20);
                Big b{};
                b.out = d;
                hipLaunchKernelGGL(k_stamp_bigload, dim3(g), dim3(256), 0, s, b, 4000);
            }
            if (report("after a 4 MB write kernel, all kernarg loaded", g)) return 1;
            long long *hp = nullptr, *hpd = nullptr;
            CK(hipHostMalloc((void **)&hp, 64, hipHostMallocMapped | hipHostMallocCoherent));
            CK(hipHostGetDevicePointer((void **)&hpd, hp, 0));
            for (int r = 0; r < 5; ++r) {
                hipLaunchKernelGGL(k_write4_host, dim3(1024), dim3(256), 0, s, buf, 1 << 20, hpd);
                hipLaunchKernelGGL(k_stamp<8192>, dim3(g), dim3(256), 0, s, d, 4000);
            }
            if (report("after a 4 MB write kernel + 8 host-mapped words", g)) return 1;
            for (int r = 0; r < 5; ++r) {
                hipLaunchKernelGGL(k_write4_host, dim3(1024), dim3(256), 0, s, buf, 64, hpd);
                hipLaunchKernelGGL(k_stamp<8192>, dim3(g), dim3(256), 0, s, d, 4000);
            }
            if (report("after a tiny write kernel + 8 host-mapped words", g)) return 1;
            CK(hipHostFree(hp));
        }
    }
    for (int spin : {0, 4000}) {
        for (int g : {256, 512, 708, 1024, 2048}) {
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_stamp<16>, dim3(g), dim3(256), 0, s, d, spin);
            char nm[96];
            snprintf(nm, sizeof nm, "lds 16 B, spin %d cyc", spin);
            if (report(nm, g)) return 1;
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_stamp<8192>, dim3(g), dim3(256), 0, s, d, spin);
            snprintf(nm, sizeof nm, "lds 8 KB, spin %d cyc", spin);
            if (report(nm, g)) return 1;
            Big b{};
            b.out = d;
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_stamp_big, dim3(g), dim3(256), 0, s, b, spin);
            snprintf(nm, sizeof nm, "650 B kernarg, spin %d cyc", spin);
            if (report(nm, g)) return 1;
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_stamp_bigload, dim3(g), dim3(256), 0, s, b, spin);
            snprintf(nm, sizeof nm, "650 B kernarg all loaded, spin %d cyc", spin);
            if (report(nm, g)) return 1;
        }
    }
    return 0;
}
