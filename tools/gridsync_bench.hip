// gridsync_bench.hip -- calibration (not product): is one kernel with a grid-wide
// barrier cheaper than two dependent kernels for the configs[2] tick shape?
//   hipcc --offload-arch=gfx950 -O3 tools/gridsync_bench.hip -o tools/gridsync_bench
// Shape: 708 workgroups of 256 threads.  Phase A: every block publishes 32 u32
// (its round counts) and writes 1 MB in total; phase B: every block reads the
// whole 708 x 32 table and writes 4 MB in total.  Two variants, K back-to-back
// launches each, wall time per iteration:
//   split: k_a then k_b (kernel boundary = the barrier)
//   fused: k_ab with agent-scope relaxed atomics for the table (write-through,
//          no L2 write-back fence) and monotonic arrival counters spread over
//          64 cache lines (one counter: 708 serialised arrivals, ~36 us).
// Measured on MI355X (round 1): split 15.7 us, fused 18.6 us -- the kernel
// boundary is the cheaper barrier, so the tick stays two kernels.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);    \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr int kG = 708, kR = 32, kBS = 256;

__device__ __forceinline__ void phase_a(unsigned *tab, int *wa, bool atomic_tab, unsigned salt) {
    const int b = blockIdx.x, t = threadIdx.x;
    // 1 MB of ordinary per-thread output (like c_arr / st / ofl)
    for (int i = b * kBS + t; i < (1 << 18); i += kG * kBS) wa[i] = i;
    if (t < kR) {
        const unsigned v = (unsigned)(b * 7 + t) + salt;
        if (atomic_tab) __hip_atomic_store(&tab[b * kR + t], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else tab[b * kR + t] = v;
    }
}

__device__ __forceinline__ void phase_b(const unsigned *tab, int *wb, bool atomic_tab, unsigned *chk) {
    const int b = blockIdx.x, t = threadIdx.x;
    unsigned s = 0;
    for (int i = t; i < kG * kR; i += kBS)
        s += tab[i];  // plain loads: the first touch per XCD misses L2 (invalidated at kernel start)
    // 4 MB of task output
    for (int i = b * kBS + t; i < (1 << 20); i += kG * kBS) wb[i] = i + (int)s;
    if (b == 0 && t == 0) chk[0] = s;
}

__global__ __launch_bounds__(kBS) void k_a(unsigned *tab, int *wa) { phase_a(tab, wa, false, 0); }
__global__ __launch_bounds__(kBS) void k_b(const unsigned *tab, int *wb, unsigned *chk) { phase_b(tab, wb, false, chk + 1); }

constexpr int kNC = 64;  // arrival counters, one per 128-byte line (a single word serialises ~30 ns / arrival)
__global__ __launch_bounds__(kBS) void k_ab(unsigned *tab, int *wa, int *wb, unsigned *ctr, unsigned gen,
                                           unsigned *chk) {
    phase_a(tab, wa, true, gen);
    __builtin_amdgcn_s_waitcnt(0);  // this wave's stores acknowledged
    __syncthreads();
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        if (lane == 0) __hip_atomic_fetch_add(&ctr[(blockIdx.x % kNC) * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // counter i expects gen x (blocks b < G with b mod kNC == i)
        const unsigned per = (unsigned)(kG / kNC + (lane < kG % kNC ? 1 : 0));
        const unsigned want = gen * per;
        unsigned it = 0;
        while (true) {
            const unsigned v = __hip_atomic_load(&ctr[lane * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__ballot(v < want) == 0) break;
            __builtin_amdgcn_s_sleep(1);
            if (++it > (1u << 24)) {  // never hang the device: flag and fall through
                chk[3] = 1;
                break;
            }
        }
    }
    __syncthreads();
    phase_b(tab, wb, true, chk + 2);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned *tab, *ctr, *chk;
    int *wa, *wb;
    CK(hipMalloc(&tab, kG * kR * 4));
    CK(hipMalloc(&ctr, kNC * 128));
    CK(hipMalloc(&chk, 64));
    CK(hipMalloc(&wa, 4 << 18));
    CK(hipMalloc(&wb, 4 << 20));
    CK(hipMemset(ctr, 0, kNC * 128));
    CK(hipMemset(chk, 0, 64));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_ab, kBS, 0));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    printf("k_ab: %d blocks/CU x %d CUs = %d resident (grid %d)\n", occ, p.multiProcessorCount,
           occ * p.multiProcessorCount, kG);
    if (occ * p.multiProcessorCount < kG) return 2;
    const int K = 400;
    unsigned launches = 0;
    for (int rep = 0; rep < 3; ++rep) {
        for (int i = 0; i < 20; ++i) {
            k_a<<<kG, kBS, 0, s>>>(tab, wa);
            k_b<<<kG, kBS, 0, s>>>(tab, wb, chk);
        }
        CK(hipStreamSynchronize(s));
        double t0 = now_us();
        for (int i = 0; i < K; ++i) {
            k_a<<<kG, kBS, 0, s>>>(tab, wa);
            k_b<<<kG, kBS, 0, s>>>(tab, wb, chk);
        }
        CK(hipStreamSynchronize(s));
        const double split = (now_us() - t0) / K;
        for (int i = 0; i < 20; ++i) {
            ++launches;
            k_ab<<<kG, kBS, 0, s>>>(tab, wa, wb, ctr, launches, chk);
        }
        CK(hipStreamSynchronize(s));
        t0 = now_us();
        for (int i = 0; i < K; ++i) {
            ++launches;
            k_ab<<<kG, kBS, 0, s>>>(tab, wa, wb, ctr, launches, chk);
        }
        CK(hipStreamSynchronize(s));
        const double fused = (now_us() - t0) / K;
        unsigned h[4];
        CK(hipMemcpy(h, chk, 16, hipMemcpyDeviceToHost));
        // expected: thread 0's partial of the last launch, entries i = 0, 256, ... (t = 0, b = i / 32)
        unsigned long long e = 0;
        for (int i = 0; i < kG * kR; i += kBS) e += (unsigned)(7 * (i / kR)) + launches;
        printf("split %.2f us/iter   fused %.2f us/iter   (fused sum %u expected %u, timeout flag %u)\n", split, fused,
               h[2], (unsigned)e, h[3]);
    }
    return 0;
}
