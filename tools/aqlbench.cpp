// aqlbench.cpp -- calibration (not product): direct AQL dispatch of a two-kernel
// chain through the HSA runtime, kernel arguments in host (kernarg pool) vs
// device memory, against the HIP launch path (tools/launchbench.hip).
//   hipcc --genco --offload-arch=gfx950 -O3 tools/aqlbench_kernels.hip -o tools/aqlbench.hsaco
//   g++ -O2 -I/opt/rocm/include tools/aqlbench.cpp -L/opt/rocm/lib -lhsa-runtime64 -o tools/aqlbench
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#define HC(x)                                                           \
    do {                                                                \
        hsa_status_t s_ = (x);                                          \
        if (s_ != HSA_STATUS_SUCCESS) {                                 \
            const char *m_ = nullptr;                                   \
            hsa_status_string(s_, &m_);                                 \
            printf("HSA error %s at line %d: %s\n", #x, __LINE__, m_);  \
            return 1;                                                   \
        }                                                               \
    } while (0)

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_amd_memory_pool_t g_karg_pool{}, g_vram_pool{};
static bool g_have_karg = false, g_have_vram = false;

static hsa_status_t find_agents(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_karg(hsa_amd_memory_pool_t p, void *) {
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !g_have_karg) {
        g_karg_pool = p;
        g_have_karg = true;
    }
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_vram(hsa_amd_memory_pool_t p, void *) {
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !g_have_vram) {
        g_vram_pool = p;
        g_have_vram = true;
    }
    return HSA_STATUS_SUCCESS;
}

struct Kern {
    uint64_t obj;
    uint32_t karg, group, priv;
};

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const char *hsaco = argc > 1 ? argv[1] : "tools/aqlbench.hsaco";
    HC(hsa_init());
    HC(hsa_iterate_agents(find_agents, nullptr));
    HC(hsa_amd_agent_iterate_memory_pools(g_cpu, find_karg, nullptr));
    HC(hsa_amd_agent_iterate_memory_pools(g_gpu, find_vram, nullptr));
    if (!g_have_karg || !g_have_vram) {
        printf("pools not found\n");
        return 1;
    }
    std::ifstream f(hsaco, std::ios::binary);
    std::string blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (blob.empty()) {
        printf("no code object at %s\n", hsaco);
        return 1;
    }
    hsa_code_object_reader_t rd;
    HC(hsa_code_object_reader_create_from_memory(blob.data(), blob.size(), &rd));
    hsa_executable_t exe;
    HC(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    HC(hsa_executable_load_agent_code_object(exe, g_gpu, rd, nullptr, nullptr));
    HC(hsa_executable_freeze(exe, nullptr));
    auto get = [&](const char *name, Kern &k) -> int {
        hsa_executable_symbol_t sym;
        HC(hsa_executable_get_symbol_by_name(exe, name, &g_gpu, &sym));
        HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.obj));
        HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.karg));
        HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group));
        HC(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv));
        return 0;
    };
    Kern ka, kb;
    if (get("k_a.kd", ka) || get("k_b.kd", kb)) return 1;
    printf("k_a kernarg %u B group %u priv %u\n", ka.karg, ka.group, ka.priv);
    hsa_queue_t *q;
    HC(hsa_queue_create(g_gpu, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    const int NS = 256, SLOT = 1024;
    char *karg_host = nullptr;
    const bool karg_dev = getenv("AQL_KARG_DEV") && atoi(getenv("AQL_KARG_DEV"));
    int *out = nullptr;
    HC(hsa_amd_memory_pool_allocate(g_vram_pool, 1 << 20, 0, (void **)&out));
    if (karg_dev) {
        // kernel arguments in VRAM, written once by DMA (the test then never rewrites them)
        HC(hsa_amd_memory_pool_allocate(g_vram_pool, NS * SLOT, 0, (void **)&karg_host));
        struct {
            int *out;
            int pad[168];
        } a0{};
        a0.out = out;
        std::vector<char> img(NS * SLOT);
        for (int s = 0; s < NS; ++s) memcpy(img.data() + (size_t)s * SLOT, &a0, sizeof a0);
        char *stage = nullptr;
        HC(hsa_amd_memory_pool_allocate(g_karg_pool, NS * SLOT, 0, (void **)&stage));
        memcpy(stage, img.data(), img.size());
        HC(hsa_memory_copy(karg_host, stage, NS * SLOT));
    } else {
        HC(hsa_amd_memory_pool_allocate(g_karg_pool, NS * SLOT, 0, (void **)&karg_host));
        HC(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, karg_host));
    }
    std::vector<hsa_signal_t> sig(NS);
    const bool gpu_only = getenv("AQL_GPU_ONLY") && atoi(getenv("AQL_GPU_ONLY"));
    for (auto &s : sig) {
        if (gpu_only) HC(hsa_amd_signal_create(0, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &s));
        else HC(hsa_signal_create(0, 0, nullptr, &s));
    }
    const bool sig_last_only = getenv("AQL_SIG_LAST") && atoi(getenv("AQL_SIG_LAST"));
    uint64_t nd = 0;  // dispatches issued
    bool copy_args = !karg_dev;
    auto dispatch = [&](const Kern &k, uint32_t blocks, const void *args, size_t n, bool last) {
        const int slot = (int)(nd % NS);
        while (hsa_signal_load_scacquire(sig[slot]) != 0) {
        }
        char *ka_ = karg_host + (size_t)slot * SLOT;
        if (copy_args) memcpy(ka_, args, n);
        hsa_signal_store_relaxed(sig[slot], 1);
        const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
        }
        auto *p = (hsa_kernel_dispatch_packet_t *)q->base_address + (idx & (q->size - 1));
        p->workgroup_size_x = 256;
        p->workgroup_size_y = 1;
        p->workgroup_size_z = 1;
        p->grid_size_x = blocks * 256;
        p->grid_size_y = 1;
        p->grid_size_z = 1;
        p->private_segment_size = k.priv;
        p->group_segment_size = k.group;
        p->kernel_object = k.obj;
        p->kernarg_address = ka_;
        if (sig_last_only && !last) {
            p->completion_signal.handle = 0;
            hsa_signal_store_relaxed(sig[slot], 0);
        } else {
            p->completion_signal = sig[slot];
        }
        const uint16_t hdr = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                             (1 << HSA_PACKET_HEADER_BARRIER) |
                             (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                             ((last ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT)
                              << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        __atomic_store_n((uint32_t *)p, hdr | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, idx);
        return nd++;
    };
    struct Args {
        int *out;
        int pad[168];
    } a{};
    a.out = out;
    auto wait_all = [&]() {
        for (auto &s : sig)
            while (hsa_signal_load_scacquire(s) != 0) {
            }
    };
    const int K = 2000;
    for (int r = 0; r < 100; ++r) {
        dispatch(ka, 708, &a, sizeof a, false);
        dispatch(kb, 345, &a, sizeof a, true);
    }
    wait_all();
    double t0 = now_us();
    for (int r = 0; r < K; ++r) {
        a.pad[0] = r;
        dispatch(ka, 708, &a, sizeof a, false);
        dispatch(kb, 345, &a, sizeof a, true);
    }
    double t1 = now_us();
    wait_all();
    double t2 = now_us();
    printf("AQL direct x2 (708 + 345 blocks), kernargs in host pool: host %.2f us/iter, wall %.2f us/iter\n",
           (t1 - t0) / K, (t2 - t0) / K);
    copy_args = false;  // kernel arguments already in place: packet write + doorbell only
    t0 = now_us();
    for (int r = 0; r < K; ++r) {
        dispatch(ka, 708, &a, sizeof a, false);
        dispatch(kb, 345, &a, sizeof a, true);
    }
    t1 = now_us();
    wait_all();
    t2 = now_us();
    printf("AQL direct x2, kernel arguments not rewritten: host %.2f us/iter, wall %.2f us/iter\n", (t1 - t0) / K,
           (t2 - t0) / K);
    copy_args = !karg_dev;
    if (!karg_dev) {
        char *dst = karg_host;
        t0 = now_us();
        for (int r = 0; r < K; ++r) memcpy(dst + (size_t)(r % NS) * SLOT, &a, sizeof a);
        t1 = now_us();
        printf("memcpy of %zu B into the kernarg pool: %.2f us\n", sizeof a, (t1 - t0) / K);
        std::vector<char> cached(NS * SLOT);
        t0 = now_us();
        for (int r = 0; r < K; ++r) memcpy(cached.data() + (size_t)(r % NS) * SLOT, &a, sizeof a);
        t1 = now_us();
        printf("memcpy of %zu B into cached host memory: %.3f us\n", sizeof a, (t1 - t0) / K);
        t0 = now_us();
        for (int r = 0; r < K; ++r) hsa_signal_store_relaxed(sig[r % NS], 0);
        t1 = now_us();
        printf("hsa_signal_store_relaxed: %.3f us\n", (t1 - t0) / K);
        t0 = now_us();
        int64_t acc = 0;
        for (int r = 0; r < K; ++r) acc += hsa_signal_load_scacquire(sig[r % NS]);
        t1 = now_us();
        printf("hsa_signal_load_scacquire: %.3f us (%ld)\n", (t1 - t0) / K, (long)acc);
        t0 = now_us();
        for (int r = 0; r < K; ++r) acc += (int64_t)hsa_queue_load_read_index_scacquire(q);
        t1 = now_us();
        printf("hsa_queue_load_read_index_scacquire: %.3f us\n", (t1 - t0) / K);
    }
    // chains of 2 with a host wait per chain (launch latency)
    t0 = now_us();
    for (int r = 0; r < 200; ++r) {
        dispatch(ka, 708, &a, sizeof a, false);
        const uint64_t d = dispatch(kb, 345, &a, sizeof a, true);
        while (hsa_signal_load_scacquire(sig[d % NS]) != 0) {
        }
    }
    t1 = now_us();
    printf("AQL direct x2 + host wait per chain: %.2f us/chain\n", (t1 - t0) / 200);
    hsa_queue_destroy(q);
    return 0;
}
