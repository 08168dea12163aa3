// kpbench.hip -- calibration (not product): device time per kernel of a dependent
// chain (each kernel reads what the previous one wrote), by argument passing:
// a 680-B struct by value, scalar pointer arguments, and scalar arguments followed
// by the struct.  Build with and without -mllvm -amdgpu-kernarg-preload-count=16
// to separate kernarg preloading from argument size.  The chain is queued behind
// a spin kernel, so host enqueue cost is hidden and events time the device alone.
//   hipcc --offload-arch=gfx950 -O3 tools/kpbench.hip -o tools/kpbench
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e = (x);                                                 \
        if (e != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                                       \
        }                                                                   \
    } while (0)

struct Big {
    const int *in;
    int *out;
    int n;
    int pad[163];
};

__global__ void k_spin(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

__device__ __forceinline__ void body(const int *__restrict__ in, int *__restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int v = in[i];
    const int w = in[(v + 64 * 1021) & (n - 1)];  // dependent second load
    out[i] = w + 1;
}
__global__ __launch_bounds__(256) void k_empty(int *out, int n) {
    if (n == 12345) out[threadIdx.x] = 0;
}
__global__ __launch_bounds__(256) void k_one(const int *__restrict__ in, int *__restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    out[i] = in[i] + 1;
}
__global__ __launch_bounds__(256) void k_three(const int *__restrict__ in, int *__restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int v = in[i];
    const int w = in[(v + 64 * 1021) & (n - 1)];
    const int x = in[(w + 64 * 2039) & (n - 1)];
    out[i] = x + 1;
}
__global__ __launch_bounds__(256) void k_struct(Big a) { body(a.in, a.out, a.n); }
__global__ __launch_bounds__(256) void k_scalar(const int *in, int *out, int n) { body(in, out, n); }
__global__ __launch_bounds__(256) void k_mixed(const int *in, int *out, int n, Big a) {
    body(in, out, n + (a.pad[5] == 77 ? 1 : 0));
}

// hot-spot test: every block reads the same 512-B vector (A) and its own 512-B row,
// after a kernel that wrote both
__global__ __launch_bounds__(256) void k_hot_write(long long *A, long long *rows, int nb) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < 64) A[i] = i;
    if (i < nb * 64) rows[i] = i;
}
template <int SHARED, int SCALAR>
__global__ __launch_bounds__(256) void k_hot_read(const long long *A, const long long *rows, int *out) {
    __shared__ long long s[64];
    const int t = threadIdx.x;
    long long v = 0;
    if (t < 64) {
        v = rows[(size_t)blockIdx.x * 64 + t];
        if (SHARED && !SCALAR) v += A[t];
    }
    if (SHARED && SCALAR) v += A[blockIdx.x & 7];  // uniform address: scalar load
    if (t < 64) s[t] = v;
    __syncthreads();
    if (s[(t + 1) & 63] == 0x7fffffffffffLL) out[blockIdx.x] = 1;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int n = 1 << 16;  // 256 blocks
    int *b0, *b1;
    CK(hipMalloc(&b0, n * 4));
    CK(hipMalloc(&b1, n * 4));
    CK(hipMemset(b0, 0, n * 4));
    CK(hipMemset(b1, 0, n * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int K = 400;
    auto run = [&](const char *name, auto fn) -> int {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 100LL * 20000);  // 20 ms at 100 MHz
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < K; ++r) fn(r);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) printf("%-44s %.3f us per kernel (device, back to back)\n", name, ms * 1e3 / K);
        }
        return 0;
    };
    Big a{};
    a.n = n;
    run("struct 680 B", [&](int r) {
        a.in = r & 1 ? b1 : b0;
        a.out = r & 1 ? b0 : b1;
        hipLaunchKernelGGL(k_struct, dim3(n / 256), dim3(256), 0, s, a);
    });
    run("scalar args 20 B", [&](int r) {
        hipLaunchKernelGGL(k_scalar, dim3(n / 256), dim3(256), 0, s, (const int *)(r & 1 ? b1 : b0),
                           r & 1 ? b0 : b1, n);
    });
    run("empty", [&](int r) { hipLaunchKernelGGL(k_empty, dim3(n / 256), dim3(256), 0, s, b0, n); });
    run("one load", [&](int r) {
        hipLaunchKernelGGL(k_one, dim3(n / 256), dim3(256), 0, s, (const int *)(r & 1 ? b1 : b0), r & 1 ? b0 : b1, n);
    });
    run("three dependent loads", [&](int r) {
        hipLaunchKernelGGL(k_three, dim3(n / 256), dim3(256), 0, s, (const int *)(r & 1 ? b1 : b0), r & 1 ? b0 : b1, n);
    });
    {
        const int nb = 4565;
        long long *A, *rows;
        int *o;
        CK(hipMalloc(&A, 4096));
        CK(hipMalloc(&rows, (size_t)nb * 512));
        CK(hipMalloc(&o, nb * 4));
        CK(hipMemset(rows, 0, (size_t)nb * 512));
        run("hot: write, read own rows", [&](int r) {
            hipLaunchKernelGGL(k_hot_write, dim3(nb / 4 + 1), dim3(256), 0, s, A, rows, nb);
            hipLaunchKernelGGL((k_hot_read<0, 0>), dim3(nb), dim3(256), 0, s, A, rows, o);
        });
        run("hot: write, read own rows + shared vector", [&](int r) {
            hipLaunchKernelGGL(k_hot_write, dim3(nb / 4 + 1), dim3(256), 0, s, A, rows, nb);
            hipLaunchKernelGGL((k_hot_read<1, 0>), dim3(nb), dim3(256), 0, s, A, rows, o);
        });
        run("hot: write, read own rows + shared scalar", [&](int r) {
            hipLaunchKernelGGL(k_hot_write, dim3(nb / 4 + 1), dim3(256), 0, s, A, rows, nb);
            hipLaunchKernelGGL((k_hot_read<1, 1>), dim3(nb), dim3(256), 0, s, A, rows, o);
        });
    }
    run("scalar args + struct", [&](int r) {
        hipLaunchKernelGGL(k_mixed, dim3(n / 256), dim3(256), 0, s, (const int *)(r & 1 ? b1 : b0),
                           r & 1 ? b0 : b1, n, a);
    });
    return 0;
}
