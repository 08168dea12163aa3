// launchbench.hip -- calibration (not product): host cost of enqueueing a
// two-kernel chain with ~700 B of kernel arguments, per launch mechanism.
//   hipcc --offload-arch=gfx950 -O3 tools/launchbench.hip -o tools/launchbench
#include <hip/hip_ext.h>
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

struct Args {
    int *out;
    int pad[168];
};

__global__ __launch_bounds__(256) void k_a(Args a) {
    if (threadIdx.x == 0 && a.pad[blockIdx.x % 168] == 12345) a.out[blockIdx.x] = 1;
}
__global__ __launch_bounds__(256) void k_b(Args a) {
    if (threadIdx.x == 0 && a.pad[(blockIdx.x + 1) % 168] == 12345) a.out[blockIdx.x] = 2;
}

struct Small {
    const Args *a;
    int tick;
};
__global__ __launch_bounds__(256) void k_as(Small s) {
    if (threadIdx.x == 0 && s.a->pad[blockIdx.x % 168] == 12345 + s.tick) s.a->out[blockIdx.x] = 1;
}
__global__ __launch_bounds__(256) void k_bs(Small s) {
    if (threadIdx.x == 0 && s.a->pad[(blockIdx.x + 1) % 168] == 12345 + s.tick) s.a->out[blockIdx.x] = 2;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    Args a{};
    CK(hipMalloc(&a.out, 1 << 20));
    const int K = 2000;
    auto run = [&](const char *name, auto fn) -> int {
        for (int r = 0; r < 50; ++r) fn(r);
        CK(hipStreamSynchronize(s));
        double t0 = now_us();
        for (int r = 0; r < K; ++r) fn(r);
        double t1 = now_us();
        CK(hipStreamSynchronize(s));
        double t2 = now_us();
        printf("%-48s host %.2f us/iter, wall %.2f us/iter\n", name, (t1 - t0) / K, (t2 - t0) / K);
        return 0;
    };
    run("hipLaunchKernelGGL x2 (708 + 345 blocks)", [&](int r) {
        a.pad[0] = r;
        hipLaunchKernelGGL(k_a, dim3(708), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_b, dim3(345), dim3(256), 0, s, a);
    });
    run("hipExtLaunchKernelGGL x2 (no events)", [&](int r) {
        a.pad[0] = r;
        hipExtLaunchKernelGGL(k_a, dim3(708), dim3(256), 0, s, nullptr, nullptr, 0, a);
        hipExtLaunchKernelGGL(k_b, dim3(345), dim3(256), 0, s, nullptr, nullptr, 0, a);
    });
    {
        void *kp[] = {&a};
        run("hipLaunchKernel x2 (void** args)", [&](int r) {
            a.pad[0] = r;
            hipLaunchKernel((const void *)k_a, dim3(708), dim3(256), kp, 0, s);
            hipLaunchKernel((const void *)k_b, dim3(345), dim3(256), kp, 0, s);
        });
    }
    {
        Args *ad;
        CK(hipMalloc(&ad, sizeof(Args)));
        CK(hipMemcpy(ad, &a, sizeof(Args), hipMemcpyHostToDevice));
        Small sm{ad, 0};
        run("hipLaunchKernelGGL x2, 16 B args (pointer to device args)", [&](int r) {
            sm.tick = r;
            hipLaunchKernelGGL(k_as, dim3(708), dim3(256), 0, s, sm);
            hipLaunchKernelGGL(k_bs, dim3(345), dim3(256), 0, s, sm);
        });
        run("hipLaunchKernelGGL x1, 16 B args", [&](int r) {
            sm.tick = r;
            hipLaunchKernelGGL(k_as, dim3(708), dim3(256), 0, s, sm);
        });
        run("hipLaunchKernelGGL x1, 680 B args", [&](int r) {
            a.pad[0] = r;
            hipLaunchKernelGGL(k_a, dim3(708), dim3(256), 0, s, a);
        });
    }
    // graph of the two kernels, replayed as is
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    hipLaunchKernelGGL(k_a, dim3(708), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_b, dim3(345), dim3(256), 0, s, a);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    run("hipGraphLaunch (2 kernel nodes, fixed args)", [&](int) { hipGraphLaunch(ge, s); });
    // graph with per-launch argument updates of both nodes
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    hipGraphNode_t nodes[4];
    CK(hipGraphGetNodes(g, nodes, &nn));
    hipKernelNodeParams p0, p1;
    CK(hipGraphKernelNodeGetParams(nodes[0], &p0));
    CK(hipGraphKernelNodeGetParams(nodes[1], &p1));
    run("hipGraphExecKernelNodeSetParams x2 + launch", [&](int r) {
        a.pad[0] = r;
        void *kp[] = {&a};
        p0.kernelParams = kp;
        p1.kernelParams = kp;
        hipGraphExecKernelNodeSetParams(ge, nodes[0], &p0);
        hipGraphExecKernelNodeSetParams(ge, nodes[1], &p1);
        hipGraphLaunch(ge, s);
    });
    return 0;
}
