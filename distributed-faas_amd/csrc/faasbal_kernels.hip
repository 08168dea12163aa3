// faasbal_kernels.hip -- CDNA4 (gfx950) kernels of one balancer tick.
//
// Tick pipeline, every kernel 256 threads = 4 wave64:
//   [E>0]  k_rs_hist / k_rs_scatter   stable LSD radix sort of events by slot (8-11-bit digits)
//   [E>0]  k_ev_apply     per-slot sequential message semantics (task_dispatcher.py:347-387)
//          k_slots        heartbeat purge of every slot (is_alive :209-212, purge_workers :241-249)
//          k_scan         log role: orphan flags per block; queue role: effective free count c
//                         per LRU position + per-block "c > r" counts for every round r
//          k_plan         exclusive scans across blocks (orphans, evictions, one row per round)
//          k_emit         fill level L; water-filling emission of task -> slot in LRU order
//                         (dispatch block :393-419); next LRU queue; orphan/evicted compaction
//          k_commit       (fb_tick_commit) sparse columns hb/registered/epoch
//
// Water-filling: c = max(free,1) for live queued workers,
// round r serves A_r = [q : c_q > r] in queue order, S(r) = sum_q min(c_q, r),
// task k of round r goes to A_r[k - S(r)].  rank_r(q) = qpre[r][blk] + in-block rank.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "faasbal_kernels.h"

namespace fb {

// Diagnostic builds (-DFAASBAL_STAMPS) record s_memtime at phase boundaries of
// thread 0 of every block into a.dbg[block * 16 + slot]; no output reads them.
#ifdef FAASBAL_STAMPS
// slot 0 (entry) and slot 15 (exit) also record s_memrealtime (100 MHz, chip-wide)
// into slots 13 and 14, so kernel spans can be compared across XCDs.
#define STAMP(a, kernel_off, slot)                                                                      \
    do {                                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                                              \
        if (threadIdx.x == 0) {                                                                         \
            unsigned long long *row_ = (a).dbg + ((kernel_off) + blockIdx.x) * 16;                      \
            row_[(slot)] = __builtin_amdgcn_s_memtime();                                                \
            if ((slot) == 0) row_[13] = __builtin_amdgcn_s_memrealtime();                               \
            if ((slot) == 15) row_[14] = __builtin_amdgcn_s_memrealtime();                              \
        }                                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                                              \
    } while (0)
#define STAMPR(a, kernel_off, slot) \
    do {                            \
    } while (0)
// after every outstanding vector memory operation of the wave completed (serialises
// the loads before it against the ones after: diagnostic only)
#define STAMPW(a, kernel_off, slot)                                 \
    do {                                                            \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");            \
        STAMP(a, kernel_off, slot);                                 \
    } while (0)
// realtime at the very top of a kernel, before the argument block is copied (slot 12)
#define STAMP_TOP(a_, kernel_off)                                                                   \
    do {                                                                                            \
        const unsigned long long rt_ = __builtin_amdgcn_s_memrealtime();                            \
        if (threadIdx.x == 0) (a_).dbg[((kernel_off) + blockIdx.x) * 16 + 12] = rt_;              \
    } while (0)
#else
#define STAMP_TOP(a_, kernel_off) \
    do {                          \
    } while (0)
#define STAMPR(a, kernel_off, slot) \
    do {                            \
    } while (0)
#define STAMP(a, kernel_off, slot) \
    do {                           \
    } while (0)
#define STAMPW(a, kernel_off, slot) \
    do {                            \
    } while (0)
#endif

// Output stores of the emission kernel: plain stores.  (Write-through -- agent-scope
// relaxed stores, global_store ... sc1 -- keeps the lines from staying dirty in the writing
// XCD's L2, but cost more than it saved on configs[2]: 11.2 vs 11.0 us per tick.)
template <typename T>
__device__ __forceinline__ void wt_store(T *p, T v) {
    *p = v;
}

// Diagnostic builds only (tools/write_probe.py): k_emit2 output arrays whose stores are
// dropped, to attribute the kernel's WRITE_SIZE per array -- 1 trash rows (inactive lanes
// branch instead), 2 full-round task stores, 4 next free counts, 8 next queue, 16 orphans,
// 32 round-L task stores.  0 in every product build.
#ifndef FAASBAL_DIAG_NOW
#define FAASBAL_DIAG_NOW 0
#endif
constexpr int kDiagNow = FAASBAL_DIAG_NOW;

// k_emit2 after k_plan(2) counts the per-segment round counts of its block in LDS
// (reading the ones k_scan stores would move 2 x 4.7 MB per streaming tick)
// Fused ticks: orphan / eviction totals through atomics into the group rows (reading
// back every per-block count in each emit queue block was slower)

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
__device__ __forceinline__ int popc_lt(uint64_t m) {
    // number of set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Workgroup barrier for LDS traffic only.  __syncthreads() also waits for every
// outstanding global store of the wave (vmcnt(0)); no kernel here reads another
// thread's global stores within a launch, so a barrier need not wait for them.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ---- DPP wave primitives (gfx9 row_shr / row_bcast): no LDS crossbar traffic,
// unlike __shfl_* which lowers to ds_bpermute.
template <int CTRL, int ROWM, int BANKM, bool BC>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWM, BANKM, BC);
}
// Inclusive prefix sum over the 64 lanes.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    uint32_t x = v + dpp<0x111, 0xf, 0xf, true>(v) + dpp<0x112, 0xf, 0xf, true>(v) + dpp<0x113, 0xf, 0xf, true>(v);
    x += dpp<0x114, 0xf, 0xe, false>(x);  // row_shr:4, banks 1-3
    x += dpp<0x118, 0xf, 0xc, false>(x);  // row_shr:8, banks 2-3
    x += dpp<0x142, 0xa, 0xf, false>(x);  // row_bcast:15 into rows 1, 3
    x += dpp<0x143, 0xc, 0xf, false>(x);  // row_bcast:31 into rows 2, 3
    return x;
}
// Inclusive prefix max over the 64 lanes (values >= 0).
__device__ __forceinline__ uint32_t wave_incl_max_u32(uint32_t v) {
    uint32_t x = max(max(v, dpp<0x111, 0xf, 0xf, true>(v)), max(dpp<0x112, 0xf, 0xf, true>(v), dpp<0x113, 0xf, 0xf, true>(v)));
    x = max(x, dpp<0x114, 0xf, 0xe, false>(x));
    x = max(x, dpp<0x118, 0xf, 0xc, false>(x));
    x = max(x, dpp<0x142, 0xa, 0xf, false>(x));
    x = max(x, dpp<0x143, 0xc, 0xf, false>(x));
    return x;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_u32(v), 63);
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max_u32(v), 63);
}
// Sum over the lanes that share (lane mod cls), cls in {8, 16, 32}; every lane
// gets its class total.  DPP row_ror:8 pairs lanes i, i^8 inside a 16-lane row;
// the gfx950 permlane16/32 swaps exchange whole rows / halves without LDS.
__device__ __forceinline__ uint32_t class_sum_u32(uint32_t v, int cls) {
    if (cls <= 8) v += dpp<0x128, 0xf, 0xf, false>(v);
    if (cls <= 16) {
        const auto q = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        v = q[0] + q[1];
    }
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return p[0] + p[1];
}

// Block-wide exclusive prefix sum (u32), one value per thread.
__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t *lds4, uint32_t &total) {
    const uint32_t x = wave_incl_scan_u32(v);
    if (lane_id() == 63) lds4[wave_id()] = x;
    lds_barrier();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const uint32_t t = lds4[w];
        pre += (w < wave_id()) ? t : 0u;
        tot += t;
    }
    lds_barrier();
    total = tot;
    return pre + x - v;
}

// Device self-test of the DPP primitives against a serial LDS reference.
__global__ __launch_bounds__(kBS) void k_selftest(uint32_t *err, uint32_t seed) {
    __shared__ uint32_t vals[kBS];
    __shared__ uint32_t l4[kWaves];
    uint32_t h = (threadIdx.x + 1) * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    const uint32_t v = (seed & 1) ? (h & 0xffu) : (h & 0xffffu);
    vals[threadIdx.x] = v;
    __syncthreads();
    const int wb = wave_id() * 64;
    uint32_t ref = 0, mref = 0;
    for (int i = wb; i <= (int)threadIdx.x; ++i) {
        ref += vals[i];
        mref = vals[i] > mref ? vals[i] : mref;
    }
    uint32_t tot_ref = 0, wsum = 0, wmax = 0, bpre = 0;
    for (int i = 0; i < kBS; ++i) {
        tot_ref += vals[i];
        if (i < (int)threadIdx.x) bpre += vals[i];
        if (i >= wb && i < wb + 64) {
            wsum += vals[i];
            wmax = vals[i] > wmax ? vals[i] : wmax;
        }
    }
    uint32_t bad = 0;
    bad += wave_incl_scan_u32(v) != ref;
    bad += wave_incl_max_u32(v) != mref;
    bad += wave_sum_u32(v) != wsum;
    bad += wave_max_u32(v) != wmax;
    uint32_t tot;
    bad += block_excl_scan_u32(v, l4, tot) != bpre;
    bad += tot != tot_ref;
    for (int cls = 8; cls <= 32; cls <<= 1) {
        uint32_t cref = 0;
        for (int i = wb; i < wb + 64; ++i)
            if (((i - wb) & (cls - 1)) == (lane_id() & (cls - 1))) cref += vals[i];
        bad += class_sum_u32(v, cls) != cref;
    }
    if (bad) atomicAdd(err, bad);
}

// Block-wide exclusive scan of one value per thread (BS = 256 = 4 waves).
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T *lds4, T &total) {
    T x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T y = __shfl_up(x, d, 64);
        if (lane_id() >= d) x += y;
    }
    if (lane_id() == 63) lds4[wave_id()] = x;
    lds_barrier();
    T pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        T t = lds4[w];
        pre += (w < wave_id()) ? t : (T)0;
        tot += t;
    }
    lds_barrier();
    total = tot;
    return pre + x - v;
}

template <typename T>
__device__ __forceinline__ T block_reduce_max(T v, T *lds4) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        T y = __shfl_xor(v, d, 64);
        v = v > y ? v : y;
    }
    if (lane_id() == 0) lds4[wave_id()] = v;
    lds_barrier();
    T m = lds4[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) m = m > lds4[w] ? m : lds4[w];
    lds_barrier();
    return m;
}

// Exclusive scan of n counts cnt[i * cs] into pre[i * ps] by one workgroup;
// returns the total.  Every thread owns a contiguous run of ceil(n / 256)
// entries and issues its loads 16 at a time, so the whole array costs one block
// scan instead of one per 256 entries.  In place (pre == cnt) is allowed: a
// thread reloads a group of its own run before storing into it.
template <typename TO, typename LD>
__device__ __forceinline__ unsigned long long run_excl_scan_ld(const LD &ld, int n, TO *pre, size_t ps,
                                                               unsigned long long *l4);
template <typename TO>
__device__ __forceinline__ unsigned long long run_excl_scan(const uint32_t *cnt, size_t cs, int n, TO *pre,
                                                            size_t ps, unsigned long long *l4) {
    return run_excl_scan_ld<TO>([=](int i) -> uint32_t { return cnt[(size_t)i * cs]; }, n, pre, ps, l4);
}
// the exclusive scan of n counts ld(0 .. n-1) into pre[i * ps] (one workgroup); returns the total
template <typename TO, typename LD>
__device__ __forceinline__ unsigned long long run_excl_scan_ld(const LD &ld, int n, TO *pre, size_t ps,
                                                               unsigned long long *l4) {
    const int per = (n + kBS - 1) / kBS;
    const int i0 = (int)threadIdx.x * per;
    unsigned long long sum = 0;
    if (per <= 16) {
        // one load pass: the run stays in registers across the block scan (a second
        // pass would be another dependent round trip to memory the producer just wrote)
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = min(i0 + j, n - 1);
            v[j] = ld(i);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            v[j] = (j < per && i0 + j < n) ? v[j] : 0u;
            sum += v[j];
        }
        unsigned long long tot;
        unsigned long long run = block_excl_scan<unsigned long long>(sum, l4, tot);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = i0 + j;
            if (j < per && i < n) pre[(size_t)i * ps] = (TO)run;
            run += v[j];
        }
        return tot;
    }
    for (int j0 = 0; j0 < per; j0 += 16) {
        // unconditional loads of clamped indices, masked afterwards: a guarded
        // load compiles to a branch with its own wait, one round trip per entry
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = min(i0 + j0 + j, n - 1);
            v[j] = ld(i);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) sum += (j0 + j < per && i0 + j0 + j < n) ? v[j] : 0u;
    }
    unsigned long long tot;
    unsigned long long run = block_excl_scan<unsigned long long>(sum, l4, tot);
    for (int j0 = 0; j0 < per; j0 += 16) {
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = min(i0 + j0 + j, n - 1);
            v[j] = ld(i);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int i = i0 + j0 + j;
            if (j0 + j < per && i < n) {
                pre[(size_t)i * ps] = (TO)run;
                run += v[j];
            }
        }
    }
    return tot;
}

// The compiler loads a by-value argument block lazily: a field's scalar load is
// placed before its first use, so a kernel whose hot path needs fields spread over
// the ~1 KB block pays one scalar-cache miss round per newly touched 64-byte line,
// in dependent rounds.  Touching one dword of every line up front (a value the
// kernel then depends on) puts the whole block into the scalar cache in one round;
// the later field loads hit it.
template <class A>
__device__ __forceinline__ void prefetch_args(const A &a) {
    {
        constexpr int nl = (int)((sizeof(A) + 63) / 64);
        const uint32_t *w = reinterpret_cast<const uint32_t *>(&a);
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < nl; ++i) x ^= w[i * 16];
        // never true (no grid has 2^31 - 1 blocks): only makes the loads necessary here
        if (blockIdx.x == 0x7fffffffu && x == 0x9e3779b9u) __builtin_trap();
    }
}

// ---------------------------------------------------------------- radix sort
// Stable LSD radix sort of (key = slot, val = event index), `db`-bit digits
// (db <= log2 NB).  NB = 256 for 8-bit passes; 1024 / 2048 let a 20-bit slot
// space (1 M workers) sort in two passes instead of three, each pass being two
// dependent launches.  hist is [block][digit] (the scatter prologue's column
// walk is then one contiguous row segment per wave load).
// (pass 0 also clears the tick's front / back lists, which k_ev_apply fills)
template <int NB>
__global__ __launch_bounds__(kBS) void k_rs_hist(const uint32_t *__restrict__ keys, int n, int shift, int db,
                                                 uint32_t *__restrict__ hist, int nblk, int32_t *__restrict__ zero0,
                                                 int32_t *__restrict__ zero1, uint32_t *__restrict__ zbits, int zwords) {
    constexpr int DPT = NB / kBS;
    __shared__ uint32_t cnt[NB];
#pragma unroll
    for (int k = 0; k < DPT; ++k) cnt[k * kBS + threadIdx.x] = 0;
    __syncthreads();
    const int base = blockIdx.x * kRsTile;
    for (int i = blockIdx.x * kBS + (int)threadIdx.x; i < zwords; i += nblk * kBS) zbits[i] = 0;
    if (zero0) {
#pragma unroll
        for (int j = 0; j < kRsItems; ++j) {
            const int e = base + j * kBS + (int)threadIdx.x;
            if (e < n) {
                zero0[e] = 0;
                zero1[e] = 0;
            }
        }
    }
    const uint32_t mask = (1u << db) - 1u;
    uint32_t kk[kRsItems];  // every key load in flight before the first use
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) kk[j] = keys[min(base + j * kBS + (int)threadIdx.x, n - 1)];
#pragma unroll
    for (int j = 0; j < kRsItems; ++j)
        if (base + j * kBS + (int)threadIdx.x < n) atomicAdd(&cnt[(kk[j] >> shift) & mask], 1u);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
        const int d = k * kBS + threadIdx.x;
        hist[(size_t)blockIdx.x * NB + d] = cnt[d];
    }
}

// Large batches (nblk > kRsScanMin): the column prefixes in their own launch, so a
// scatter block reads its own row and the digit totals (O(NB)) instead of walking
// the whole table (O(nblk NB) per block, O(nblk^2 NB) per pass).  Block j owns
// digits 64 j .. 64 j + 63 (lane = digit, 256-B row segments); its 16 waves take
// consecutive row groups of kRsScanRows, prefix in place, carry across chunks.
constexpr int kRsScanWaves = 16, kRsScanRows = 8;
__global__ __launch_bounds__(64 * kRsScanWaves) void k_rs_scan(uint32_t *__restrict__ hist, int nblk, int NB,
                                                              uint32_t *__restrict__ tot) {
    __shared__ uint32_t ws[kRsScanWaves][64];
    const int lane = lane_id(), w = (int)threadIdx.x >> 6;
    const int d = (int)blockIdx.x * 64 + lane;
    uint32_t carry = 0;
    for (int c0 = 0; c0 < nblk; c0 += kRsScanWaves * kRsScanRows) {
        const int r0 = c0 + w * kRsScanRows;
        uint32_t v[kRsScanRows], s = 0;
#pragma unroll
        for (int j = 0; j < kRsScanRows; ++j) {
            v[j] = hist[(size_t)min(r0 + j, nblk - 1) * NB + d];
            v[j] = r0 + j < nblk ? v[j] : 0u;
            s += v[j];
        }
        ws[w][lane] = s;
        __syncthreads();
        uint32_t ex = carry, all = 0;
#pragma unroll
        for (int q = 0; q < kRsScanWaves; ++q) {
            const uint32_t x = ws[q][lane];
            ex += q < w ? x : 0u;
            all += x;
        }
#pragma unroll
        for (int j = 0; j < kRsScanRows; ++j) {
            if (r0 + j < nblk) hist[(size_t)(r0 + j) * NB + d] = ex;
            ex += v[j];
        }
        carry += all;
        __syncthreads();  // ws reused by the next chunk
    }
    if (w == 0) tot[d] = carry;
}

// scanned: hist holds column prefixes (k_rs_scan) and tot the digit totals
template <int NB>
__global__ __launch_bounds__(kBS) void k_rs_scatter(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                    uint32_t *__restrict__ kout, uint32_t *__restrict__ vout, int n,
                                                    int shift, int db, const uint32_t *__restrict__ hist, int nblk,
                                                    int identity_vals, const uint32_t *__restrict__ scanned) {
    constexpr int DPT = NB / kBS;       // digits per thread
    constexpr int CH = 64 / DPT;        // blocks per batch of 64 loads in flight
    __shared__ uint32_t base[NB];
    __shared__ uint32_t wcnt[kWaves][NB];
    __shared__ uint32_t l4[kWaves];
    const int t = threadIdx.x;
    {
        // this block's base per digit straight from the raw [block][digit] counts
        // (no separate scan launch): thread t sums digits k*256+t over all blocks
        // and over the blocks before this one (each wave load is one contiguous
        // row segment), then one block scan over the digit totals in digit order
        uint32_t tot[DPT], pre[DPT];
#pragma unroll
        for (int k = 0; k < DPT; ++k) tot[k] = pre[k] = 0;
        if (scanned) {
#pragma unroll
            for (int k = 0; k < DPT; ++k) {
                tot[k] = scanned[k * kBS + t];
                pre[k] = hist[(size_t)blockIdx.x * NB + k * kBS + t];
            }
        }
        for (int j0 = 0; !scanned && j0 < nblk; j0 += CH) {
            uint32_t v[DPT][CH];
#pragma unroll
            for (int k = 0; k < DPT; ++k)
#pragma unroll
                for (int j = 0; j < CH; ++j) v[k][j] = hist[(size_t)min(j0 + j, nblk - 1) * NB + k * kBS + t];
#pragma unroll
            for (int k = 0; k < DPT; ++k)
#pragma unroll
                for (int j = 0; j < CH; ++j) {
                    const uint32_t x = (j0 + j < nblk) ? v[k][j] : 0u;
                    tot[k] += x;
                    pre[k] += (j0 + j < (int)blockIdx.x) ? x : 0u;
                }
        }
        if constexpr (DPT == 1) {
            uint32_t all;
            base[t] = block_excl_scan_u32(tot[0], l4, all) + pre[0];
        } else {
            // regroup through LDS so thread t scans the contiguous digits t*DPT ..
#pragma unroll
            for (int k = 0; k < DPT; ++k) {
                base[k * kBS + t] = tot[k];
                wcnt[0][k * kBS + t] = pre[k];
            }
            __syncthreads();
            uint32_t loc[DPT], sum = 0, all;
#pragma unroll
            for (int k = 0; k < DPT; ++k) sum += (loc[k] = base[t * DPT + k]);
            uint32_t ex = block_excl_scan_u32(sum, l4, all);  // its barriers order the reads above
#pragma unroll
            for (int k = 0; k < DPT; ++k) {
                base[t * DPT + k] = ex + wcnt[0][t * DPT + k];
                ex += loc[k];
            }
            __syncthreads();
        }
    }
    if constexpr (NB > 256) {  // the leader-lane updates below keep wcnt zero between items
#pragma unroll
        for (int q = 0; q < kWaves; ++q)
#pragma unroll
            for (int k = 0; k < DPT; ++k) wcnt[q][k * kBS + t] = 0;
    }
    const int tile = blockIdx.x * kRsTile;
    const int w = wave_id();
    const uint32_t mask = (1u << db) - 1u;
    // the tile's keys and values loaded up front (clamped, all in flight at once)
    uint32_t kk[kRsItems], vv[kRsItems];
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) {
        const int e = tile + j * kBS + t, ec = min(e, n - 1);
        kk[j] = kin[ec];
        vv[j] = identity_vals ? (uint32_t)e : vin[ec];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) {
        if constexpr (NB == 256) {
#pragma unroll
            for (int q = 0; q < kWaves; ++q) wcnt[q][t] = 0;
            __syncthreads();
        }
        const int e = tile + j * kBS + t;
        const bool valid = e < n;
        const uint32_t key = kk[j], val = vv[j];
        const uint32_t d = (key >> shift) & mask;
        uint64_t peers = __ballot(valid);
        constexpr int LB = NB == 256 ? 8 : NB == 1024 ? 10 : 11;  // digit bits above db are 0 in every lane
#pragma unroll
        for (int b = 0; b < LB; ++b) {
            const uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const int wrank = popc_lt(peers);
        const bool lead = valid && wrank == 0;
        const uint32_t wn = (uint32_t)__popcll(peers);
        if (lead) wcnt[w][d] = wn;
        __syncthreads();
        if (valid) {
            uint32_t off = base[d] + (uint32_t)wrank;
            for (int q = 0; q < w; ++q) off += wcnt[q][d];
            kout[off] = key;
            vout[off] = val;
        }
        __syncthreads();
        if constexpr (NB == 256) {
            uint32_t add = 0;
#pragma unroll
            for (int q = 0; q < kWaves; ++q) add += wcnt[q][t];
            base[t] += add;
        } else {
            // only the digits this item touched move: each wave's leader lanes advance
            // their digit's base and clear their own count (no NB-wide sweep)
            // (no barrier after: a wave clears only its own wcnt row, and the next
            // item reads base / wcnt only after its first barrier)
            if (lead) {
                atomicAdd(&base[d], wn);
                wcnt[w][d] = 0;
            }
        }
        if constexpr (NB == 256) __syncthreads();
    }
}

// ------------------------------------------------------------ event apply
// One thread per slot segment of the slot-sorted events; processes that
// slot's messages in arrival order (task_dispatcher.py:343-390 per message,
// with the purge of the preceding loop iteration at the same clock).
// Sharded: local log position of global sequence q (entries ascend), or -1.
__device__ __forceinline__ int64_t lseq_find(const uint32_t *lseq, int64_t n, int64_t q) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)lseq[mid] < q) lo = mid + 1;
        else hi = mid;
    }
    return (lo < n && (int64_t)lseq[lo] == q) ? lo : -1;
}

// Slot s got messages this tick (message ticks only: one GPU's bitmap, else the stamp).
template <class A>
__device__ __forceinline__ bool got_msg(const A &a, int s) {
    return a.tbits ? ((a.tbits[s >> 5] >> (s & 31)) & 1u) != 0u : a.touched[s] == a.tick;
}

// The loop without heartbeats, PushDispatcher.start (task_dispatcher.py:251-322), for
// one slot's messages: no liveness; every register(n > 0) inserts a new token at the
// left of the deque (:280-281), a result that brings free to 1 appends one at the
// right (:294-295) -- both whatever tokens the worker already holds.  Each new
// token gets its rank among the slot's tokens in deque order: fronts (newest
// first), then the committed ones, then backs (oldest first).
__device__ void ev_apply_deque(const EvArgs &a, int j, uint32_t s) {
    int nf = 0;
    for (int k = j; k < a.E && a.skeys[k] == s; ++k) {
        const int i = (int)a.svals[k];
        nf += (a.ev_kind[i] == kEvRegister && a.ev_val[i] > 0) ? 1 : 0;
    }
    const int k_old = a.tokcnt_in[s];
    int reg = a.reg[s];
    int32_t fr = a.free_in[s].x;
    double hb = a.hb[s];
    uint32_t epoch = a.epoch[s];
    int mf = 0, nb = 0;
    for (int k = j; k < a.E && a.skeys[k] == s; ++k) {
        const int i = (int)a.svals[k];
        const int kind = a.ev_kind[i];
        uint8_t status = kEvsApplied;
        if (kind == kEvRegister) {                       // :276-281, a fresh PushWorker
            if (!reg) { reg = 1; epoch = (uint32_t)a.head_in; }
            hb = a.ev_ts[i];
            fr = a.ev_val[i];
            if (fr > 0) {
                ++mf;
                a.front_list[a.E - 1 - i] = (int32_t)s + 1;
                a.front_rank[a.E - 1 - i] = nf - mf + 1;
            }
        } else if (kind == kEvResult) {                  // :284-295
            if (!reg) {
                status = kEvsUnknown;                    // KeyError at :291 in the reference
            } else {
                fr += 1;
                const int64_t q = a.ev_seq[i];
                if (q >= 0 && q < a.head_in && a.log_slot[q] == (int32_t)s) a.log_slot[q] = -1;
                if (fr == 1) {
                    ++nb;
                    a.back_list[i] = (int32_t)s + 1;
                    a.back_rank[i] = k_old + nf + nb;
                }
            }
        }                                                // other kinds: no branch in start()
        a.ev_status[i] = status;
    }
    a.post[s] = PostRec{hb, fr, epoch};
    a.post_rf[s] = (uint8_t)(reg | ((kQsKeep << 1) << 1));
    a.touched[s] = a.tick;
    a.post_tok[s] = k_old + nf + nb;
    a.post_nf[s] = nf;
}

// One slot's record while its messages are applied in arrival order
// (task_dispatcher.py:343-390 per message, the purge of the preceding loop
// iteration at the message's own clock first).  s: local slot, gs: global slot.
struct SlotRun {
    int reg, inq, q0, qstat, qidx, cur_is_start, died_start;
    int reg_s;       // registered at tick start (lazy clears: its entries >= ep_s are in flight)
    uint32_t ep_s;
    int32_t fr;
    double hb;
    uint32_t epoch;
    uint32_t infl0;  // defer_clr: in-flight entries of the slot at tick start (bud - free)
    uint32_t ncl;    // defer_clr: distinct entries this tick's results completed
    __device__ __forceinline__ void init(const EvArgs &a, uint32_t s) {
        reg = a.reg[s];
        const int2 fq = a.free_in[s];
        fr = fq.x;
        hb = a.hb[s];
        epoch = a.epoch[s];
        reg_s = reg;
        ep_s = epoch;
        // a slot without a record has no in-flight entries (its budget is stale)
        infl0 = (a.defer_clr && reg) ? (uint32_t)(a.bud[s] - fq.x) : 0u;
        ncl = 0;
        inq = fq.y;
        q0 = fq.y;
        qstat = inq ? kQsKeep : kQsOut;
        qidx = -1;
        cur_is_start = reg;
        died_start = 0;
    }
    // PF: logv = log_slot[seq] loaded by the caller (one GPU, heartbeat loop: defer_clr),
    // dup: an earlier message of this slot in this tick completed the same entry.
    // Returns whether this message completed an in-flight entry.
    template <bool PF = false>
    __device__ __forceinline__ bool step(const EvArgs &a, uint32_t gs, int i, int kind, int32_t val, double ts,
                                         int64_t seq, int32_t logv = 0, bool dup = false) {
        bool cleared = false;
        // purge at ts before the message is polled (:390 of the previous iteration)
        if (reg && (ts - hb) > a.tte) {
            reg = 0;
            inq = 0;
            qstat = kQsOut;
            if (cur_is_start) { died_start = 1; cur_is_start = 0; }
        }
        uint8_t status = kEvsApplied;
        if (kind == kEvRegister) {                       // :347-353
            if (!reg) { reg = 1; epoch = a.head_in; }
            hb = ts;
            fr = val;
            if (val > 0) { inq = 1; qstat = kQsFront; qidx = i; }
        } else if (!reg) {                               // :356-358 unknown id
            reg = 1; epoch = a.head_in; hb = ts; fr = 0;
            status = kEvsReconnect;
        } else if (kind == kEvReconnect) {               // :360-367
            hb = ts;
            fr = val;
            if (val > 0) { inq = 1; qstat = kQsFront; qidx = i; }
        } else if (kind == kEvHeartbeat) {               // :370-371
            hb = ts;
        } else if (kind == kEvResult) {                  // :374-387
            fr += 1;
            hb = ts;
            const int64_t q = seq;
            // lazy clears: an entry of a registration that died before this tick is still in
            // the log naming the slot, but not in flight
            const bool live = !a.live_chk || (reg_s && (uint64_t)q >= (uint64_t)ep_s);
            if (q >= 0 && q < a.head_in && live) {
                if (PF) {
                    // one GPU: the entry's slot loaded ahead.  defer_clr: the log stays as
                    // committed (the commit clears the entry), ctag names the entry for this
                    // launch; else cleared in place (clearing it twice is harmless)
                    if (logv == (int32_t)gs && !dup) {
                        cleared = true;
                        if (a.defer_clr) a.ctag[q] = a.lstamp;
                        else a.log_slot[q] = -1;
                    }
                } else if (a.defer_clr) {
                    // sorted path, one GPU: a slot may carry any number of results; the
                    // first to stamp ctag[q] in this launch counts the entry
                    if (a.log_slot[q] == (int32_t)gs) cleared = atomicExch(&a.ctag[q], a.lstamp) != a.lstamp;
                } else {
                    const int64_t li = a.shard ? lseq_find(a.lseq, a.head_local, q) : q;
                    if (li >= 0 && a.log_slot[li] == (int32_t)gs) a.log_slot[li] = -1;
                }
            }
            if (fr == 1 && !inq) { inq = 1; qstat = kQsBack; qidx = i; }
        }
        a.ev_status[i] = status;
        if (a.defer_clr) a.ev_clr[i] = cleared ? (int32_t)seq : -1;
        ncl += cleared ? 1u : 0u;
        return cleared;
    }
    // the purge at the tick's clock of this touched slot (k_ev_apply_ll's launch)
    __device__ __forceinline__ bool purge(const EvArgs &a, uint32_t s, int reg0, bool &evicted);
    __device__ __forceinline__ void finish(const EvArgs &a, uint32_t s, uint32_t gs) {
        a.post[s] = PostRec{hb, fr, epoch};
        a.post_rf[s] = (uint8_t)(reg | ((died_start | (qstat << 1)) << 1) | (ncl ? kRfCleared : 0) | (q0 ? kRfQ0 : 0));
        if (a.defer_clr) a.post_infl[s] = infl0 - ncl;
        if (a.tbits) atomicOr(&a.tbits[s >> 5], 1u << (s & 31));  // the bitmap is the stamp
        else a.touched[s] = a.tick;
        if (qstat == kQsFront) a.front_list[a.E - 1 - qidx] = (int32_t)gs + 1;
        if (qstat == kQsBack) a.back_list[qidx] = (int32_t)gs + 1;
    }
};

__global__ __launch_bounds__(kBS) void k_ev_apply(EvArgs a) {
    prefetch_args(a);
    const int j = blockIdx.x * kBS + threadIdx.x;
    if (j >= a.E) return;
    // this position's key, its neighbours and its event index in one load round
    const uint32_t gs = a.skeys[j], gprev = a.skeys[max(j - 1, 0)], gnext = a.skeys[min(j + 1, a.E - 1)];
    const int i0 = (int)a.svals[j];
    if (j > 0 && gprev == gs) return;
    if (a.deque) {
        ev_apply_deque(a, j, gs);
        return;
    }
    if (a.shard && ((int)gs < a.slot_base || (int)gs >= a.slot_base + a.W)) return;  // another rank's worker
    const uint32_t s = a.shard ? gs - (uint32_t)a.slot_base : gs;
    // the first message's payload, loaded alongside the slot record (most slots
    // get one message: the chain is key -> {record, payload} -> log entry)
    int kind = a.ev_kind[i0];
    int32_t val = a.ev_val[i0];
    double ts = a.ev_ts[i0];
    int64_t seq = a.ev_seq[i0];
    int i = i0;
    SlotRun r;
    r.init(a, s);
    for (int k = j;;) {
        r.step(a, gs, i, kind, val, ts, seq);
        if (++k >= a.E || (k == j + 1 ? gnext : a.skeys[k]) != gs) break;
        i = (int)a.svals[k];
        kind = a.ev_kind[i];
        val = a.ev_val[i];
        ts = a.ev_ts[i];
        seq = a.ev_seq[i];
    }
    r.finish(a, s, gs);
}

// ------------------------------------------------------------ commit
// One slot's commit: t = the slot got messages this tick.
__device__ __forceinline__ void commit_slot(const CommitArgs &a, int s, bool t, int64_t wq_head) {
    const uint8_t stt = a.st[s];
    // the second load round at once, branch-free (clamped addresses: an untouched slot
    // reads slot 0's line, a slot not queued at tick start slot 0's position): the
    // post-message record and flags of a touched slot, the committed position of a queued one
    const int sc = t ? s : 0;
    const PostRec pr = a.post[sc];
    const uint8_t rf = a.win ? a.post_rf[sc] : (uint8_t)0;
    const int32_t p = a.win ? a.pos[(stt & kStQ0) ? s : 0] : -1;  // exact for a queued slot
    const int32_t bn = a.bud ? a.bud_next[sc] : 0;
    if (a.win) {
        // window tick: the committed position of a slot queued at tick start that the tick
        // did not serve -- tombstoned when the slot died or its messages took it out of the
        // queue, refreshed with its post-message free count and heartbeat when they kept it
        // there (a queued slot that lives on untouched keeps its position as it is).  Slots
        // moved to the front or the back were recorded by k_emit_win (the tomb list above):
        // they may also be appended, so their pos is rewritten in this launch.
        if ((stt & kStQ0) && (t || !(stt & kStAlive))) {
            const int qs = t ? (rf >> 2) & 3 : kQsKeep;
            if (!(stt & kStAlive) || qs == kQsOut || qs == kQsKeep) {
                if (p >= wq_head && p < a.wq_tail) {
                    if (!(stt & kStAlive) || qs == kQsOut) {
                        a.wqf[p] = kTomb;
                    } else {
                        a.wqf[p] = pr.free;
                        a.wqh[p] = pr.hb;
                    }
                }
            }
        }
    }
    // committed hb is NaN for slots without a record (k_scan's log role relies on it)
    if (t) {
        const bool alive = (stt & kStAlive) != 0;
        a.reg[s] = alive ? 1 : 0;
        a.hb[s] = alive ? pr.hb : __builtin_nan("");
        a.epoch[s] = pr.epoch;
        if (a.bud) a.bud[s] = bn;
    } else if (stt & kStEvicted) {
        a.reg[s] = 0;
        a.hb[s] = __builtin_nan("");
    }
}

// wq_head / napp: the window's new head and appended positions (a.wq_head / a.napp, or
// read from the tick's results by an eager commit)
__device__ __forceinline__ void commit_body(const CommitArgs &a, int blk, int64_t wq_head, int64_t napp) {
    const int nclr = (a.n_clr + kBS - 1) / kBS;
    if (a.win && blk >= a.nbw + a.nbo + nclr) {
        const int rb = blk - a.nbw - a.nbo - nclr;
        if (rb < a.nbap) {
            // window tick: the slot at each appended position has its position there
            for (int64_t i = (int64_t)rb * kBS + threadIdx.x; i < napp; i += (int64_t)a.nbap * kBS)
                a.pos[a.wq_buf[a.wq_tail + i]] = (int32_t)(a.wq_tail + i);
            return;
        }
        // the committed positions of queued slots a front / back insertion moved (recorded
        // by k_emit_win per list entry, before any position changed) become tombstones
        const int ntb = (a.n_tomb + kBS - 1) / kBS;
        if (rb < a.nbap + ntb) {
            const int64_t j = (int64_t)(rb - a.nbap) * kBS + threadIdx.x;
            if (j < a.n_tomb) {
                const int32_t p = a.tomb[j];
                if (p >= wq_head && p < a.wq_tail) a.wqf[p] = kTomb;
            }
        }
        return;
    }
    if (blk >= a.nbw + a.nbo) {
        // entries the committed tick's results completed (one-GPU heartbeat contexts keep
        // the log read-only during the tick): they leave the in-flight log now
        const int64_t e = (int64_t)(blk - a.nbw - a.nbo) * kBS + threadIdx.x;
        if (e >= a.n_clr) return;
        const int32_t q = a.ev_clr[e];
        if (q >= 0) a.log_slot[q] = -1;
        return;
    }
    if (blk >= a.nbw && a.oseg) {
        // orphans in per-tile segments (fused one-GPU and window ticks): a wave per 64 tiles
        // (one count load each), then the tiles that hold orphans one after another
        // a wave per tile: 64 orphans per round (a fused tick leaves ~100 per tile, a
        // window tick ~1; most of a window tick's waves read one count and stop)
        const int t = (blk - a.nbw) * kWaves + wave_id();
        const uint32_t n = t < a.oseg_tiles ? a.oseg[t] : 0u;
        for (uint32_t i = lane_id(); i < n; i += 64) a.log_slot[a.orphans[(int64_t)t * kFTile + i]] = -1;
        return;
    }
    if (blk >= a.nbw) {
        // the committed tick redistributed these entries: their tasks now run under new
        // sequence numbers, so the old entries leave the in-flight log
        const int64_t i = (int64_t)(blk - a.nbw) * kBS + threadIdx.x;
        if (i >= a.n_orph) return;
        const int64_t q = a.orphans[i];
        const int64_t li = a.shard ? lseq_find(a.lseq, a.head_local, q) : q;
        if (li >= 0) a.log_slot[li] = -1;
        return;
    }
    const int s = blk * kBS + threadIdx.x;
    if (s >= a.W) return;
    commit_slot(a, s, a.E > 0 && got_msg(a, s), wq_head);
}

__global__ __launch_bounds__(kBS) void k_commit(CommitArgs a) {
    prefetch_args(a);
    int64_t wq_head = a.wq_head, napp = a.napp;
    if (a.eager) {
        // enqueued behind the window tick before the host waited for it: the tick's commit
        // word (device memory: {failed, window head, window length}; a failure -- written by
        // k_ev_link, k_ev_apply_ll or k_emit_win -- stores the launch's link stamp, so the
        // word is never cleared) says whether it finished as a window tick -- if not,
        // nothing is committed and the host reruns it -- and where the window moved
        const int64_t *cw = a.eager;
        if (cw[0] == a.cw_tag) return;
        wq_head = cw[1];
        napp = cw[1] + cw[2] - a.wq_tail;
    }
    commit_body(a, blockIdx.x, wq_head, napp);
}

// ------------------------------------------------------------ event grouping without a sort
// One GPU, heartbeat loop: the messages of a slot are grouped by a linked list
// instead of the radix sort.  k_ev_link: every message exchanges its index into
// its slot's head word (tagged with a per-launch stamp, so nothing is cleared);
// next[e] is the index it displaced, or -1 when it was the first of its slot --
// that message's thread owns the slot in k_ev_apply_ll, walks head -> ... -> itself
// (at most kLinkMax messages), sorts the indices (arrival order) in registers and
// applies them.  A slot with more messages sets hout->resort and the host reruns
// the tick through the sort (fb_tick_wait).  Also does the sort's first-pass
// clears: this tick's front / back lists and the touched bitmap.
constexpr int kLinkMax = 16;
__global__ __launch_bounds__(kBS) void k_ev_link(EvArgs a) {
    prefetch_args(a);
    const int lb = (int)gridDim.x - a.cm_blocks;  // link blocks; the rest commit the previous tick
    if ((int)blockIdx.x >= lb) {
        commit_body(a.cm, (int)blockIdx.x - lb, a.cm.wq_head, a.cm.napp);
        return;
    }
    const int t = blockIdx.x * kBS + (int)threadIdx.x, nt = lb * kBS;
    if (t == 0) {
        a.hout->resort = 0;
        a.hout->win_ovf = 0;
    }
    // window ticks: the purge's partial counts (words 0 and 1 of 64 lines), k_emit_win's
    // look-back granules and its ticket
    if (a.wpart && t < 128) a.wpart[(t >> 1) * 32 + (t & 1)] = 0u;
    for (int i = t; i < a.wlb_n; i += nt) a.wlb[i] = 0ull;
    if (a.wlb_n && t == 0) *a.wticket = 0u;
    for (int w = t; w < a.tbits_words; w += nt) a.tbits[w] = 0u;
    // the counters k_ev_apply_ll's slot purge accumulates with atomics
    for (int w = t; w < a.nbw; w += nt) a.wcnt[w] = 0u;
    if (a.dmask)
        for (int w = t; w < (a.W + 63) >> 6; w += nt) a.dmask[w] = 0ull;
    if (t < a.E) {
        uint32_t s = (uint32_t)a.ev_slot[t];
        if (a.check_ev) {
            // a pinned batch the host did not read: slot in range, known kind, timestamps
            // non-decreasing and <= now; an invalid message is made harmless (slot 0, a
            // heartbeat) for the rest of the launch, whose tick the host then refuses
            const uint8_t k = a.ev_kind[t];
            const double tt = a.ev_ts[t], tp = a.ev_ts[t > 0 ? t - 1 : 0];
            const bool bad_sk = s >= (uint32_t)a.W || k > kEvOther;
            if (bad_sk || !(tt <= a.now) || tt < tp) {
                a.hout->bad_ev = 1;
                if (a.cw) a.cw[0] = a.link;
                if (a.bad_min) atomicMin(a.bad_min, t);
            }
            if (bad_sk) {
                s = 0;
                a.ev_slot[t] = 0;
                a.ev_kind[t] = kEvHeartbeat;
            }
        }
        a.front_list[t] = 0;
        a.back_list[t] = 0;
        const unsigned long long old =
            atomicExch(&a.ev_head[s], ((unsigned long long)a.link << 32) | (unsigned long long)(uint32_t)t);
        a.ev_next[t] = (uint32_t)(old >> 32) == a.link ? (int32_t)(uint32_t)old : -1;
    }
}

// log_slot[seq] of a result, loaded branch-free (clamped index; the value is only
// compared when seq is a dispatched sequence)
__device__ __forceinline__ int32_t log_peek(const EvArgs &a, int64_t seq) {
    const int64_t q = seq < 0 ? 0 : (seq >= a.head_in ? (a.head_in > 0 ? a.head_in - 1 : 0) : seq);
    return a.head_in > 0 ? a.log_slot[q] : -1;
}

// purge_workers (:241-249) at the tick's clock for one slot, as k_scan's slots_body
// (task_dispatcher.py:209-212 for liveness): status byte, next {free, queued}, the
// died-at-start bit and the eviction count.  Untouched slots (t = false) from the
// committed record, touched ones from the owner thread's post-message registers.
// infl: the slot's in-flight entries after its messages; returns the orphans it leaves
// (the entries of a registration that died), and writes the next in-flight count.
// q0: the slot was in the committed queue at tick start (kStQ0, read by a window commit);
// queued_out: a live position of this tick's LRU queue (window ticks count them).
__device__ __forceinline__ uint32_t purge_slot(const EvArgs &a, int s, bool t, int reg0, int reg, double hb,
                                               int32_t fr, int died_flag, bool queued_if_alive, int q0, uint32_t infl,
                                               bool &died, bool &evicted, bool &alive_out, bool &queued_out) {
    const bool dead = reg && ((a.now - hb) > a.tte);
    const bool alive = reg && !dead;
    died = reg0 && (dead || died_flag);
    evicted = (reg0 || t) && !alive;
    a.st[s] = (uint8_t)((alive ? kStAlive : 0) | (died ? kStDiedStart : 0) | (evicted ? kStEvicted : 0) |
                        (q0 ? kStQ0 : 0));
    queued_out = alive && queued_if_alive;
    a.free_out[s] = make_int2(alive ? fr : INT32_MIN, queued_out ? 1 : 0);
    alive_out = alive;
    return died ? infl : 0u;
}
// window ticks: a wave's evictions and live queued slots into partial `part` (one line each)
__device__ __forceinline__ void count_wpart(const EvArgs &a, int part, uint32_t ne, uint32_t nq) {
    uint32_t *w = a.wpart + (size_t)(part & 63) * 32;
    if (ne) atomicAdd(w, ne);
    if (nq) atomicAdd(w + 1, nq);
}
__device__ __forceinline__ void count_evicted(const EvArgs &a, int tile, uint32_t n) {
    atomicAdd(&a.wcnt[tile], n);
    if (a.grp) atomicAdd(&a.grp[(tile % a.ngrp) * a.gstride + a.R + 2], n);
}
// orphans of dead registrations into column R + 1 of a group row (f_emit ticks: k_emit2
// sums every row for O before the fill level; no log scan precedes it)
__device__ __forceinline__ void count_orphans(const EvArgs &a, int tile, uint32_t n) {
    if (a.orph_grp && n) atomicAdd(&a.grp[(tile % a.ngrp) * a.gstride + a.R + 1], n);
}

__device__ __forceinline__ bool SlotRun::purge(const EvArgs &a, uint32_t s, int reg0, bool &evicted) {
    bool died, alive, queued;
    const uint32_t no = purge_slot(a, (int)s, true, reg0, reg, hb, fr, died_start, qstat != kQsOut, q0, infl0 - ncl,
                                   died, evicted, alive, queued);
    // the budget the commit installs: a new registration after a death starts with no
    // in-flight entries (a dead slot's budget is never read)
    if (a.bud_next) a.bud_next[s] = (int32_t)((alive && !died) ? infl0 - ncl : 0u) + fr;
    if (died && a.dmask) atomicOr(&a.dmask[s >> 6], 1ull << (s & 63));
    if (died && a.died_tag) *a.died_tag = a.lstamp;  // (the same value from every writer)
    if (evicted) count_evicted(a, (int)(s >> 8), 1u);
    count_orphans(a, (int)(s >> 8), no);
    return queued;
}

__device__ __forceinline__ bool apply_run(const EvArgs &a, SlotRun &r, uint32_t s, int e, int hidx, int kind0,
                                          int32_t val0, double ts0, int64_t seq0, int reg0, bool &ev);

// k_ev_apply_ll's slot blocks: the purge of untouched slots, one slot per thread, NT tiles
// of 256 slots from tile blk0 (every tile's loads issued before the first tile's purge)
template <int NT>
__device__ __forceinline__ void apply_slot_tiles(const EvArgs &a, int blk0) {
    bool tv[NT];
    int regv[NT];
    double hbv[NT];
    int2 fqv[NT];
    int32_t bv[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int s = (blk0 + j) * kBS + (int)threadIdx.x;
        const int sc = s < a.W ? s : (a.W > 0 ? a.W - 1 : 0);
        // the link stamp says whether the slot got messages (its owner purges it); the
        // committed record loaded with it (no dependent round)
        tv[j] = (uint32_t)(a.ev_head[sc] >> 32) == a.link;
        regv[j] = a.reg[sc];
        hbv[j] = a.hb[sc];
        fqv[j] = a.free_in[sc];
        bv[j] = a.bud ? a.bud[sc] : 0;
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int blk = blk0 + j;
        const int s = blk * kBS + (int)threadIdx.x;
        bool died = false, evicted = false, queued = false;
        uint32_t no = 0;
        if (s < a.W) {
            const int reg0 = regv[j];
            const int2 fq0 = fqv[j];
            const uint32_t in0 = (a.bud && reg0) ? (uint32_t)(bv[j] - fq0.x) : 0u;
            bool alive;
            if (!tv[j])
                no = purge_slot(a, s, false, reg0, reg0, hbv[j], fq0.x, 0, fq0.y != 0, fq0.y, in0, died, evicted,
                                alive, queued);
        }
        const uint64_t dm = __ballot(died);
        const uint32_t ne = (uint32_t)__popcll(__ballot(evicted));
        const uint32_t nq = (uint32_t)__popcll(__ballot(queued));
        const uint32_t nw = a.orph_grp ? wave_sum_u32(no) : 0u;
        if (lane_id() == 0) {
            if (a.dmask && dm) atomicOr(&a.dmask[s >> 6], (unsigned long long)dm);
            if (a.died_tag && dm) *a.died_tag = a.lstamp;
            if (ne) count_evicted(a, blk, ne);
            count_orphans(a, blk, nw);
            if (a.wpart) count_wpart(a, blk * kWaves + wave_id(), ne, nq);
        }
    }
}

#ifdef FAASBAL_STAMPS
// entry: thread 0's stamps; exit: the block's last thread (realtime, atomicMax into slot 14)
#define APPLY_STAMP(slot)                                   \
    do {                                                    \
        if (a.dbg) STAMP(a, 0, slot);                       \
    } while (0)
#define APPLY_EXIT()                                                                                  \
    do {                                                                                              \
        if (a.dbg) atomicMax(&a.dbg[blockIdx.x * 16 + 14], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
    } while (0)
#else
#define APPLY_STAMP(slot) \
    do {                  \
    } while (0)
#define APPLY_EXIT() \
    do {             \
    } while (0)
#endif
__global__ __launch_bounds__(kBS) void k_ev_apply_ll(EvArgs a) {
    prefetch_args(a);
    APPLY_STAMP(0);
    const int nwb = a.wtiles == 4 ? (a.nbw + 3) / 4 : a.nbw;
    const int nba = (int)gridDim.x - nwb;  // apply blocks; the rest purge untouched slots
    if ((int)blockIdx.x >= nba) {
        if (a.wtiles == 4) apply_slot_tiles<4>(a, 4 * ((int)blockIdx.x - nba));
        else apply_slot_tiles<1>(a, (int)blockIdx.x - nba);
        APPLY_EXIT();
        return;
    }
    const int e = blockIdx.x * kBS + threadIdx.x;
    if (e >= a.E) {
        APPLY_EXIT();
        return;
    }
    // slot, link and payload of this message in one load round
    const uint32_t s = (uint32_t)a.ev_slot[e];
    const int32_t nx = a.ev_next[e];
    const int kind0 = a.ev_kind[e];
    const int32_t val0 = a.ev_val[e];
    const double ts0 = a.ev_ts[e];
    const int64_t seq0 = a.ev_seq[e];
    if (nx >= 0) {  // another message of this slot owns it
        APPLY_EXIT();
        return;
    }
    // second round: the slot's head, its record and this message's log entry together
    const int hidx = (int)(uint32_t)a.ev_head[s];
    const int32_t logv0 = log_peek(a, seq0);
    SlotRun r;
    r.init(a, s);
    const int reg0 = r.reg;
    bool qd = false, ev = false;  // window ticks: this slot queued after the purge / evicted
    if (hidx == e) {  // the slot's only message (most slots)
        r.step<true>(a, s, e, kind0, val0, ts0, seq0, logv0);
        r.finish(a, s, s);
        if (a.nbw) qd = r.purge(a, s, reg0, ev);
    } else {
        qd = apply_run(a, r, s, e, hidx, kind0, val0, ts0, seq0, reg0, ev);
    }
    if (a.wpart) {
        // one atomic per wave, by its first owner lane (the others returned above)
        const uint64_t act = __ballot(true);
        const uint32_t ne = (uint32_t)__popcll(__ballot(ev)), nq = (uint32_t)__popcll(__ballot(qd));
        if (lane_id() == (int)__builtin_ctzll(act)) count_wpart(a, (int)blockIdx.x * kWaves + wave_id(), ne, nq);
    }
    APPLY_EXIT();
}

// A slot with several messages (k_ev_apply_ll): walk head -> ... -> e, restore arrival
// order, apply them in order, purge.  Returns whether the slot is queued after the purge.
__device__ __forceinline__ bool apply_run(const EvArgs &a, SlotRun &r, uint32_t s, int e, int hidx, int kind0,
                                          int32_t val0, double ts0, int64_t seq0, int reg0, bool &ev) {
    // walk head -> ... -> e (link order), each message's payload loaded with its link
    int idx[kLinkMax], kd[kLinkMax];
    int32_t vl[kLinkMax];
    double tt[kLinkMax];
    int64_t sq[kLinkMax];
    int n = 0, cur = hidx;
    bool done = false;
#pragma unroll
    for (int k = 0; k < kLinkMax; ++k) {
        const bool own = cur == e;
        const int c = done ? e : cur;
        idx[k] = done ? INT32_MAX : cur;
        kd[k] = own ? kind0 : a.ev_kind[c];
        vl[k] = own ? val0 : a.ev_val[c];
        tt[k] = own ? ts0 : a.ev_ts[c];
        sq[k] = own ? seq0 : a.ev_seq[c];
        if (!done) {
            ++n;
            if (own) done = true;
            else cur = a.ev_next[cur];
        }
    }
    if (!done) {  // too many messages for the registers: the host reruns through the sort
        a.hout->resort = 1;
        if (a.cw) a.cw[0] = a.link;
        return false;
    }
    // sort the messages into arrival order (bitonic network, static register indices;
    // padding entries carry INT32_MAX and stay last).  n <= 4: the first four suffice.
    auto cx = [&](int i, int l, bool up) {
        const bool sw = up ? (idx[i] > idx[l]) : (idx[i] < idx[l]);
        int t = idx[i]; idx[i] = sw ? idx[l] : t; idx[l] = sw ? t : idx[l];
        t = kd[i]; kd[i] = sw ? kd[l] : t; kd[l] = sw ? t : kd[l];
        int32_t v = vl[i]; vl[i] = sw ? vl[l] : v; vl[l] = sw ? v : vl[l];
        double d = tt[i]; tt[i] = sw ? tt[l] : d; tt[l] = sw ? d : tt[l];
        int64_t q = sq[i]; sq[i] = sw ? sq[l] : q; sq[l] = sw ? q : sq[l];
    };
    if (n <= 4) {
#pragma unroll
        for (int k = 2; k <= 4; k <<= 1)
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if ((i ^ j) > i) cx(i, i ^ j, (i & k) == 0);
    } else {
#pragma unroll
        for (int k = 2; k <= kLinkMax; k <<= 1)
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
                for (int i = 0; i < kLinkMax; ++i)
                    if ((i ^ j) > i) cx(i, i ^ j, (i & k) == 0);
    }
    // every result's log entry in one load round, then the messages in order; dp[k]: an
    // earlier message of the slot completed message k's entry (a repeated result)
    int32_t lv[kLinkMax];
    bool dp[kLinkMax];
#pragma unroll
    for (int k = 0; k < kLinkMax; ++k) {
        lv[k] = k < n ? log_peek(a, sq[k]) : -1;
        dp[k] = false;
    }
    for (int m = 0; m < n; ++m) {
        const bool cl = r.step<true>(a, s, idx[0], kd[0], vl[0], tt[0], sq[0], lv[0], dp[0]);
#pragma unroll
        for (int k = 1; k < kLinkMax; ++k) dp[k] = dp[k] || (cl && sq[k] == sq[0]);
#pragma unroll
        for (int k = 0; k + 1 < kLinkMax; ++k) {
            idx[k] = idx[k + 1];
            kd[k] = kd[k + 1];
            vl[k] = vl[k + 1];
            tt[k] = tt[k + 1];
            sq[k] = sq[k + 1];
            lv[k] = lv[k + 1];
            dp[k] = dp[k + 1];
        }
    }
    r.finish(a, s, s);
    return a.nbw ? r.purge(a, s, reg0, ev) : false;
}


// ------------------------------------------------------------ slot state

// Current record of slot s after this tick's messages (touched) or as committed.
struct Cur {
    int reg0, reg, flags, q0;  // q0: in the committed LRU queue
    bool t;
    double hb;
    int32_t fr;
};

__device__ __forceinline__ Cur cur_slot(const TickArgs &a, int s) {
    Cur c;
    c.reg0 = a.reg[s];
    const double hb0 = a.hb[s];
    const int2 fq0 = a.free_in[s];
    const int32_t fr0 = fq0.x;
    c.q0 = fq0.y;
    if (a.E > 0) {
        // message tick: committed and post-message records loaded together and
        // selected afterwards (a load behind the touched test would wait for it) --
        // except for large tables (a.post_lazy), where the kernel is bandwidth-bound
        // and only the few touched slots read their 17-byte post record
        const bool tk = got_msg(a, s);
        uint8_t rf = 0;
        PostRec pr{0.0, 0, 0u};
        if (!a.post_lazy || tk) {
            rf = a.post_rf[s];
            pr = a.post[s];
        }
        c.t = tk;
        c.reg = c.t ? (rf & 1) : c.reg0;
        c.hb = c.t ? pr.hb : hb0;
        c.fr = c.t ? pr.free : fr0;
        c.flags = c.t ? (rf >> 1) : 0;
    } else {
        c.t = false;
        c.reg = c.reg0;
        c.hb = hb0;
        c.fr = fr0;
        c.flags = 0;
    }
    return c;
}

// PushWorker.is_alive (task_dispatcher.py:209-212): time.time() - last_heartbeat > time_to_expire,
// fp64 subtract then compare, exactly as written.
__device__ __forceinline__ bool is_dead(const TickArgs &a, const Cur &c) { return c.reg && ((a.now - c.hb) > a.tte); }

// Global slot at logical LRU position pos of fronts ++ queue ++ backs, or -1.
// One load from the list the position falls in (no branch per list).  The list
// pointers go through registers first: a select between the fields' addresses
// would keep the kernels' argument copy in scratch.
__device__ __forceinline__ int lq_slot(const TickArgs &a, int64_t pos) {
    const bool fr = pos < a.E, qu = !fr && pos < a.E + a.Qn;
    const int32_t *pf = a.front_list, *pq = a.queue_in, *pb = a.back_list;
    asm("" : "+s"(pf), "+s"(pq), "+s"(pb));
    const int32_t *p = fr ? pf : (qu ? pq : pb);
    const int64_t i = fr ? pos : (qu ? pos - a.E : pos - a.E - a.Qn);
    return p[i] - (qu ? 0 : 1);
}
// Local index of global slot s if this rank owns it, else -1 (one GPU: s itself).
__device__ __forceinline__ int own_slot(const TickArgs &a, int s) {
    if (!a.shard) return s;
    const int ls = s - a.slot_base;
    return (s >= 0 && ls >= 0 && ls < a.W) ? ls : -1;
}

// ------------------------------------------------------------ helpers
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const T y = __shfl_xor(v, d, 64);
        v = v > y ? v : y;
    }
    return v;
}

// Counts of "c > r" in this wave for rounds r0 .. r0+rn-1 (rn <= 64): lane i
// receives the count of round r0 + i (one ballot per round, no LDS traffic).
__device__ __forceinline__ uint32_t wave_round_counts(int c, int r0, int rn) {
    uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
    const int lane = lane_id();
    int i = 0;
    for (; i + 3 < rn; i += 4) {
        const uint32_t n0 = (uint32_t)__popcll(__ballot(c > r0 + i));
        const uint32_t n1 = (uint32_t)__popcll(__ballot(c > r0 + i + 1));
        const uint32_t n2 = (uint32_t)__popcll(__ballot(c > r0 + i + 2));
        const uint32_t n3 = (uint32_t)__popcll(__ballot(c > r0 + i + 3));
        m0 = (lane == i) ? n0 : m0;
        m1 = (lane == i + 1) ? n1 : m1;
        m2 = (lane == i + 2) ? n2 : m2;
        m3 = (lane == i + 3) ? n3 : m3;
    }
    for (; i < rn; ++i) {
        const uint32_t n = (uint32_t)__popcll(__ballot(c > r0 + i));
        m0 = (lane == i) ? n : m0;
    }
    return m0 | m1 | m2 | m3;  // each lane is set by exactly one chain (others stay 0)
}

// wave_round_counts for two predicates at once: lane i gets the counts of
// c > r0 + i over all lanes and over the lanes in own (one ballot per round).
__device__ __forceinline__ void wave_round_counts2(int c, uint64_t own, int r0, int rn, uint32_t &all,
                                                   uint32_t &mine) {
    uint32_t a0 = 0, m0 = 0;
    const int lane = lane_id();
    for (int i = 0; i < rn; ++i) {
        const uint64_t m = __ballot(c > r0 + i);
        const uint32_t na = (uint32_t)__popcll(m), nm = (uint32_t)__popcll(m & own);
        a0 = (lane == i) ? na : a0;
        m0 = (lane == i) ? nm : m0;
    }
    all = a0;
    mine = m0;
}

// Sum of cnt[i] over i < n with all loads in flight at once (n <= kPeel*256 on
// the fused path; a tail loop covers larger n); also the sum over i < lim.
template <int PEEL = kPeel, int BS = kBS>
__device__ __forceinline__ void peeled_sum(const uint32_t *__restrict__ cnt, int n, int lim,
                                           unsigned long long &tot, unsigned long long &pre) {
    uint32_t v[PEEL];
#pragma unroll
    for (int k = 0; k < PEEL; ++k) {
        const int i = threadIdx.x + k * BS;
        v[k] = i < n ? cnt[i] : 0u;
    }
    tot = pre = 0;
#pragma unroll
    for (int k = 0; k < PEEL; ++k) {
        const int i = threadIdx.x + k * BS;
        tot += v[k];
        pre += i < lim ? v[k] : 0u;
    }
    for (int i = threadIdx.x + PEEL * BS; i < n; i += BS) {
        const uint32_t x = cnt[i];
        tot += x;
        pre += i < lim ? x : 0u;
    }
}

// ------------------------------------------------------------ specialisations
// The tick kernels are instantiated per tick kind: idle (no messages -- every
// message path folds away, the benchmark's headline tick), message ticks, and
// the deque loop (PushDispatcher.start).  The launcher picks the instance that
// matches the argument block; each kernel works on a copy with those fields
// fixed, so the inlined helpers constant-fold on them -- and the copy loads the
// whole block once at entry instead of one scalar fetch (and wait) per field at
// its first use.
constexpr int kModeIdle = 0, kModeEvents = 1, kModeDeque = 2;

template <int MODE>
__device__ __forceinline__ TickArgs specialise(TickArgs a) {
    if (MODE == kModeIdle) a.E = 0;
    a.deque = MODE == kModeDeque ? 1 : 0;
    return a;
}

// Sharded exchange of the effective free counts: one byte per LRU position while the
// round table has at most 128 rows (every c that matters is below the 255 clamp), two
// bytes (clamp 65535) for wider tables.  Either way one rank writes each position.
__device__ __forceinline__ int xc_get(const TickArgs &a, int64_t pos) {
    return a.xcw == 2 ? (int)reinterpret_cast<const uint16_t *>(a.xc8)[pos] : (int)a.xc8[pos];
}
__device__ __forceinline__ void xc_put(const TickArgs &a, int64_t pos, int c) {
    if (a.xcw == 2) reinterpret_cast<uint16_t *>(a.xc8)[pos] = (uint16_t)(c < 65535 ? c : 65535);
    else a.xc8[pos] = (uint8_t)(c < 255 ? c : 255);
}

// ------------------------------------------------------------ slot purge
// Heartbeat purge of every slot (purge_workers, :241-249): liveness, the
// died-registration bitmap, next free_processes (INT32_MIN = no live record).
// Its own launch (k_slots) or the W-role blocks of k_scan (a.slots_in_scan).
// NT tiles of 256 slots per workgroup (k_scan's W role, fb_set_path("wtiles")), every
// tile's loads issued before the first tile's stores.
template <int NT = 1>
__device__ __forceinline__ void slots_body(const TickArgs &a, int blk0, uint32_t (*l4)[kWaves]) {
    Cur cv[NT];
    int32_t b0v[NT];
    uint32_t ipv[NT];
    uint8_t st0[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int s = (blk0 + j) * kBS + threadIdx.x;
        const int sc = s < a.W ? s : (a.W > 0 ? a.W - 1 : 0);
        cv[j] = cur_slot(a, sc);
        st0[j] = a.cm_fold ? a.st[sc] : (uint8_t)0;
        // in-flight entries after the messages (loaded with the record, selected after)
        b0v[j] = a.bud ? a.bud[sc] : 0;
        ipv[j] = (a.bud && a.E > 0) ? a.post_infl[sc] : 0u;
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int blk = blk0 + j;
        const int s = blk * kBS + threadIdx.x;
        bool died_start = false, evicted = false;
        uint32_t no = 0;  // orphans: in-flight entries of this slot's dead registration
        if (s < a.W) {
            Cur c = cv[j];
            if (a.cm_fold && (st0[j] & kStEvicted)) {
                // the previous tick deleted this record (its commit, folded in here):
                // del self.workers[remove_id] (task_dispatcher.py:246-247)
                c.reg0 = c.reg = 0;
                c.hb = __builtin_nan("");
                const_cast<uint8_t *>(a.reg)[s] = 0;  // (the committed record arrays: read-only elsewhere in a tick)
                const_cast<double *>(a.hb)[s] = c.hb;
            }
            const int32_t b0 = b0v[j];
            const uint32_t ip = ipv[j];
            const bool dead = is_dead(a, c);
            const bool alive = c.reg && !dead;
            died_start = c.reg0 && (dead || (c.flags & kPfDiedStart));
            evicted = !a.deque && (c.reg0 || c.t) && !alive;  // start() never deletes a record
            a.st[s] = (uint8_t)((alive ? kStAlive : 0) | (died_start ? kStDiedStart : 0) | (evicted ? kStEvicted : 0) |
                                (c.q0 ? kStQ0 : 0));
            // queued: a live position of this tick's LRU queue (committed and kept, or a
            // front / back insertion) -- k_emit2 then rewrites only the slots it serves
            const bool queued = !a.deque && !a.shard && alive && (c.t ? ((c.flags >> 1) & 3) != kQsOut : c.q0 != 0);
            const int32_t cq = c.fr > 1 ? c.fr : 1;  // its position's c
            a.free_out[s] = (a.free_pre && queued) ? make_int2(c.fr - cq, 0)
                                                   : make_int2(alive ? c.fr : INT32_MIN, queued ? 1 : 0);
            if (a.bud) {
                // untouched: the committed free count is c.fr; a slot without a record has none
                const uint32_t pin = c.t ? ip : (c.reg0 ? (uint32_t)(b0 - c.fr) : 0u);
                no = died_start ? pin : 0u;
                // a touched slot's budget after the tick (a new registration starts empty);
                // an untouched one keeps its budget: dispatches move free into in flight
                if (c.t) a.bud_next[s] = (int32_t)((alive && !died_start) ? pin : 0u) + c.fr;
            }
            if (a.deque) {  // the emit kernel counts the surviving tokens per slot into these
                a.tokcnt_out[s] = 0;
                a.xw_out[s] = 0;
            }
        }
        const uint64_t dm = __ballot(died_start);
        if ((!a.slots_in_scan || a.f_sep || a.f_emit) && lane_id() == 0 && blk * kBS + wave_id() * 64 < a.W) {
            a.dmask[(blk * kBS) / 64 + wave_id()] = dm;
        }
        if (a.f_emit) {
            // O for the fill level: the dead registrations' in-flight counts (k_emit2's log
            // tiles find the same entries, for the compaction)
            const uint32_t nw = wave_sum_u32(no);
            if (lane_id() == 0 && nw) atomicAdd(&a.grp[(blk % a.ngrp) * a.gstride + a.R + 1], nw);
        }
        const uint32_t ev = (uint32_t)__popcll(__ballot(evicted));
        if (lane_id() == 0) l4[j][wave_id()] = ev;
    }
    lds_barrier();
    if (threadIdx.x < NT && blk0 + (int)threadIdx.x < a.nbw) {
        const int j = threadIdx.x, blk = blk0 + j;
        const uint32_t n = l4[j][0] + l4[j][1] + l4[j][2] + l4[j][3];
        a.wcnt[blk] = n;
        // fused: evictions into column R + 2 of a group row (k_emit2 sums every row)
        if (a.grp_on && n) atomicAdd(&a.grp[(blk % a.ngrp) * a.gstride + a.R + 2], n);
    }
}

template <int MODE>
__global__ __launch_bounds__(kBS) void k_slots(TickArgs a_) {
    prefetch_args(a_);
    const TickArgs a = specialise<MODE>(a_);
    __shared__ uint32_t l4[1][kWaves];
    STAMP(a, 0, 0);
    slots_body(a, blockIdx.x, l4);
    STAMP(a, 0, 15);
}

// One-GPU message ticks: in-flight entry q of slot s was completed by one of this
// tick's results (the log keeps it until the commit).  Only asked for entries whose
// slot died this tick, so the gathers behind the touched test are rare.
template <class A>
__device__ __forceinline__ bool completed_now(const A &a, int s, int64_t q) {
    return got_msg(a, s) && (a.post_rf[s] & kRfCleared) && a.ctag[q] == a.lstamp;
}
// drop the completed entries from a tile row's orphan flags (bit j: entry base + j)
template <class A>
__device__ __forceinline__ uint32_t drop_completed(const A &a, uint32_t flags, const int32_t *v, int64_t base) {
    if (a.E == 0 || !a.ctag) return flags;
    for (uint32_t m = flags; m; m &= m - 1) {
        const int j = __builtin_ctz(m);
        if (completed_now(a, v[j], base + j)) flags &= ~(1u << j);
    }
    return flags;
}

// Lazy clears (one-GPU heartbeat contexts): drop from a row's orphan flags the entries older
// than their died slot's registration -- entries of an earlier, dead registration that its
// commit left in the log (bit j: entry base + j, slot v[j]).  Only once such entries may exist.
template <int N, class A>
__device__ __forceinline__ uint32_t drop_stale(const A &a, uint32_t flags, const int32_t *v, int64_t base) {
    if (!a.live_chk || !flags) return flags;
    uint32_t e[N];
#pragma unroll
    for (int j = 0; j < N; ++j) e[j] = a.epoch[((flags >> j) & 1u) ? v[j] : 0];  // (every gather in flight)
#pragma unroll
    for (int j = 0; j < N; ++j)
        if (((flags >> j) & 1u) && (uint64_t)(base + j) < (uint64_t)e[j]) flags &= ~(1u << j);
    return flags;
}

// The registration of slot s alive at tick start died during this tick (read
// straight from the record: used by k_scan's log role when no bitmap exists).
// Committed hb is NaN for unregistered slots, so the untouched case is one load.
__device__ __forceinline__ bool died_touched(const TickArgs &a, int s) {
    if (!a.reg[s]) return false;
    const uint8_t rf = a.post_rf[s];
    if ((rf >> 1) & kPfDiedStart) return true;
    return (rf & 1) && ((a.now - a.post[s].hb) > a.tte);
}

// k_scan's Q role for a position that is not a committed entry with ride-along records (a
// front / back insertion, or no qaos): its slot from the lists, the free count and heartbeat
// from the slot's record.  raw stays INT32_MIN without a live record (or not mine).
__device__ __forceinline__ void q_raw_slow(const TickArgs &a, int64_t pos, bool inq, int32_t &raw, double &hbq) {
    const int s = lq_slot(a, pos);
    const int ls = s >= 0 ? own_slot(a, s) : -1;
    if (ls >= 0) {
        if (a.slots_in_scan) {
            const Cur cu = cur_slot(a, ls);
            raw = (cu.reg && !is_dead(a, cu)) ? cu.fr : INT32_MIN;
            hbq = cu.hb;
        } else {
            raw = a.free_out[ls].x;
            // the heartbeat after this tick's messages rides along into the next queue
            const double h0 = a.hb[ls], h1 = a.post[ls].hb;
            hbq = (a.E > 0 && got_msg(a, ls)) ? h1 : h0;
        }
    }
    // an old queue entry moved to the front, re-appended or removed by this tick's messages
    if (raw != INT32_MIN && a.E > 0 && inq && got_msg(a, ls) && ((a.post_rf[ls] >> 2) & 3) != kQsKeep)
        raw = INT32_MIN;
}

// k_scan's Q role, QT queue blocks per workgroup (one GPU, unfused tables with ride-along
// queue records, R <= kRFused): every block's position loads in one round, the touched
// tests in a second, then per block the wave histograms of min(c, R), one barrier for all
// blocks, and the blocks' round counts, capacity and max c -- the values the one-block form
// writes (configs[3]: 3 547 one-block workgroups of ~2 us of dependent phases each).
template <int QT>
__device__ __forceinline__ void queue_tiles(const TickArgs &a, int b0) {
    __shared__ uint32_t qh[kWaves][kRFused + 1];
    __shared__ uint8_t qwc[QT][kWaves][kRFused];  // per-wave counts (<= 64): bytes keep k_scan at 8 workgroups per CU
    __shared__ uint32_t qm[QT][kWaves], qsum[QT][kWaves];
    const int t = threadIdx.x, lane = lane_id(), w = wave_id(), R = a.R;
    int sqv[QT];
    double hqv[QT];
    int32_t fqv[QT];
    bool tqv[QT];
#pragma unroll
    for (int j = 0; j < QT; ++j) {
        const int64_t q = (int64_t)(b0 + j) * kBS + t - a.E;
        const int64_t qc = q < 0 ? 0 : (q < a.Qn ? q : (a.Qn > 0 ? a.Qn - 1 : 0));
        sqv[j] = a.queue_in[qc];
        hqv[j] = a.qhb_in[qc];
        fqv[j] = a.qfree_in[qc];
    }
#pragma unroll
    for (int j = 0; j < QT; ++j) tqv[j] = a.E > 0 && got_msg(a, sqv[j]);
#pragma unroll
    for (int j = 0; j < QT; ++j) {
        const int64_t pos = (int64_t)(b0 + j) * kBS + t;
        int c = 0;
        if (pos < a.Qlog) {
            int32_t raw = INT32_MIN;
            double hbq = 0.0;
            const int64_t q = pos - a.E;
            if (q >= 0 && q < a.Qn) {
                // a committed entry (as the one-block form)
                const int sq = sqv[j];
                if (!tqv[j]) {
                    hbq = hqv[j];
                    raw = ((a.now - hqv[j]) > a.tte) ? INT32_MIN : fqv[j];
                } else {
                    const uint8_t rf = a.post_rf[sq];
                    const PostRec pr = a.post[sq];
                    hbq = pr.hb;
                    raw = ((rf & 1) && !((a.now - pr.hb) > a.tte)) ? pr.free : INT32_MIN;
                    if (((rf >> 2) & 3) != kQsKeep || fqv[j] == kTomb) raw = INT32_MIN;
                }
            } else {
                q_raw_slow(a, pos, false, raw, hbq);
            }
            if (raw != INT32_MIN) c = raw > 1 ? raw : 1;  // free <= 0 still takes one task (:409-419)
            if (!a.cq_direct) {
                a.c_arr[pos] = raw;
                a.c_hb[pos] = hbq;
            }
        }
        // the wave's counts of c > r for every round r < R from a histogram of min(c, R)
        uint32_t *h = qh[w];
        for (int i = lane; i <= R; i += 64) h[i] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        atomicAdd(&h[c < R ? c : R], 1u);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        uint32_t carry = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int r = 64 * k + lane;
            const uint32_t hv = h[r < R ? r : R];
            const uint32_t P = carry + wave_incl_scan_u32(r < R ? hv : 0u);
            if (r < R) qwc[j][w][r] = (uint8_t)(64u - P);
            carry = (uint32_t)__builtin_amdgcn_readlane((int)P, 63);
        }
        // capacity sum_r count(c > r) over r < R = sum of min(c, R); max c
        const uint32_t ws = wave_sum_u32((uint32_t)(c < R ? c : R)), wm = wave_max_u32((uint32_t)c);
        if (lane == 0) {
            qsum[j][w] = ws;
            qm[j][w] = wm;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < QT; ++j) {
        const int b = b0 + j;
        if (b >= a.nbq) break;  // (uniform)
        if (t < R) {
            const uint32_t n = (uint32_t)qwc[j][0][t] + qwc[j][1][t] + qwc[j][2][t] + qwc[j][3][t];
            a.qcnt[(size_t)b * R + t] = n;
            // the group's row of round totals (memory-side atomics, no return)
            if (a.grp_on && n) atomicAdd(&a.grp[(b >> a.gshift) * a.gstride + t], n);
        }
    }
    if (t < QT && b0 + t < a.nbq) {
        const int b = b0 + t;
        const uint32_t bm = max(max(qm[t][0], qm[t][1]), max(qm[t][2], qm[t][3]));
        a.qbm_raw[b] = (int32_t)bm;
        a.csum[b] = (unsigned long long)qsum[t][0] + qsum[t][1] + qsum[t][2] + qsum[t][3];
        if (a.grp_on && bm > 0) atomicMax(&a.grp[(b >> a.gshift) * a.gstride + R], bm);
    }
}

// ------------------------------------------------------------ k_scan
// F-blocks flag orphaned log entries (died bitmap in LDS); Q-blocks compute the
// effective free count c of every LRU position and the block's count of c > r
// for every round r (table laid out [block][round]).
template <int MODE, int WT>
__global__ __launch_bounds__(kBS, (WT == 4 ? 8 : 1)) void k_scan(TickArgs a_) {
    STAMP_TOP(a_, a_.nbw);
    prefetch_args(a_);
    const TickArgs a = specialise<MODE>(a_);
    extern __shared__ __attribute__((aligned(16))) unsigned long long dyn[];
    __shared__ uint32_t l4[kWaves];
    __shared__ int32_t m4[kWaves];
    __shared__ unsigned long long s4[kWaves];
    __shared__ uint32_t wc[kWaves][kBS];
    const int nbf = (a.shard == 2 || a.f_sep || a.f_emit) ? 0 : a.nbf;  // phase 2 re-derives only the queue counts
    // Q-role workgroups (a.qtiles queue blocks each in the 4-tile instance)
    const int nqb = (WT == 4 && a.qtiles == 4) ? (a.nbq + 3) >> 2 : a.nbq;
    // grid: queue blocks first (the critical path: their loads go out before the log
    // role's gathers fill the memory queues), then log blocks, then slot blocks.  Sharded
    // phase 1 (a.wfirst): the log and slot blocks first -- there they are the longer ones
    // (4-5 us against the queue blocks' 3 at configs[3], N = 8) and nothing waits on the
    // queue role before the exchange
    const int nfw = (int)gridDim.x - nqb - (a.cm_fold ? a.cm_blocks : 0);
    const int bid = !a.wfirst ? (int)blockIdx.x
                              : ((int)blockIdx.x < nfw ? nqb + (int)blockIdx.x
                                                       : ((int)blockIdx.x < nfw + nqb ? (int)blockIdx.x - nfw
                                                                                       : (int)blockIdx.x));
    const int SO = a.nbw;
    STAMP(a, SO, 0);
    if (bid >= nqb && bid - nqb < nbf) {
        // ---- F-role: orphan flags of log entries [b*2048 + t*8, +8)
        const int b = bid - nqb;
        const int64_t nlog = a.shard ? a.head_local : a.head_in;
        const int64_t base = (int64_t)b * kFTile + (int64_t)threadIdx.x * kFItems;
        int32_t v[kFItems];
        if (base + kFItems <= nlog) {
            const int4 x0 = *reinterpret_cast<const int4 *>(a.log_slot + base);
            const int4 x1 = *reinterpret_cast<const int4 *>(a.log_slot + base + 4);
            v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
            v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
        } else {
#pragma unroll
            for (int j = 0; j < kFItems; ++j) v[j] = (base + j < nlog) ? a.log_slot[base + j] : -1;
        }
        if (a.shard) {  // log slots are global ids; this rank's bitmap and epochs are local
#pragma unroll
            for (int j = 0; j < kFItems; ++j) v[j] = v[j] < 0 ? -1 : v[j] - a.slot_base;
        }
        // an entry is an orphan iff its slot's registration alive at tick start died this
        // tick (entries of earlier registrations were cleared when their tick committed, or --
        // lazy clears -- are older than the slot's epoch: drop_stale)
        uint32_t died = 0;
        if (a.slots_in_scan) {
            // died-at-start straight from the heartbeats: 8 independent 8-byte gathers per
            // thread (the committed hb is NaN for a slot without a record: never dead)
            double h[kFItems];
            uint32_t tc[kFItems];
#pragma unroll
            for (int j = 0; j < kFItems; ++j) {
                const int sj = v[j] < 0 ? 0 : v[j];
                h[j] = a.hb[sj];
                tc[j] = a.E > 0 ? (got_msg(a, sj) ? 1u : 0u) : 0u;
            }
#pragma unroll
            for (int j = 0; j < kFItems; ++j) {
                bool d = false;
                if (v[j] >= 0) d = (a.E > 0 && tc[j] != 0u) ? died_touched(a, v[j]) : ((a.now - h[j]) > a.tte);
                died |= d ? (1u << j) : 0u;
            }
        } else {
        const int nwords = (a.W + 63) >> 6;
        const unsigned long long *dm = a.dmask;
        if (a.lds_bitmap) {
            // <= 2048 words = 1024 int4: at most 4 loads per thread, all in flight together
            const int n4 = (nwords + 1) >> 1;
            const uint4 *src = reinterpret_cast<const uint4 *>(a.dmask);
            uint4 t[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = threadIdx.x + k * kBS;
                t[k] = src[i < n4 ? i : n4 - 1];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = threadIdx.x + k * kBS;
                if (i < n4) reinterpret_cast<uint4 *>(dyn)[i] = t[k];
            }
            lds_barrier();
            dm = dyn;
        }
#pragma unroll
        for (int j = 0; j < kFItems; ++j) {
            const int sj = v[j] < 0 ? 0 : v[j];
            const unsigned long long wd = dm[sj >> 6];
            died |= (v[j] >= 0 && ((wd >> (sj & 63)) & 1ull)) ? (1u << j) : 0u;
        }
        }
        const uint32_t flags = drop_completed(a, drop_stale<kFItems>(a, died, v, base), v, base);
        a.ofl[(size_t)b * kBS + threadIdx.x] = (uint8_t)flags;
        const uint32_t wv = wave_sum_u32((uint32_t)__popc(flags));
        if (lane_id() == 0) l4[wave_id()] = wv;
        lds_barrier();
        if (threadIdx.x == 0) {
            const uint32_t n = l4[0] + l4[1] + l4[2] + l4[3];
            a.fcnt[b] = n;
            // fused: orphans into column R + 1 of a group row (k_emit2 sums every row)
            if (a.grp_on && n) atomicAdd(&a.grp[(b % a.ngrp) * a.gstride + a.R + 1], n);
            if (a.shard && n)
                atomicAdd(&a.xrec[a.rank * kXRecWords + (b & (kXRecLines - 1)) * 16], (unsigned long long)n);
        }
        STAMP(a, SO, 15);
        return;
    }
    if (a.cm_fold && bid >= (int)gridDim.x - a.cm_blocks) {
        // ---- the previous tick's orphaned log entries leave the log (its folded commit)
        // (a dense list; per-tile segments are cleared by k_emit2's log workgroup of each tile)
        const int64_t i = (int64_t)(bid - ((int)gridDim.x - a.cm_blocks)) * kBS + threadIdx.x;
        if (i < a.cm_n_orph) a.log_slot[a.orphans[i]] = -1;
        return;
    }
    if (bid >= nqb) {
        // ---- W-role: heartbeat purge of slots [b*256, +256)
        // WT tiles per workgroup (a.wtiles; its own instance, so the one-tile form -- fused
        // ticks -- keeps its registers and occupancy)
        __shared__ uint32_t l4w[WT][kWaves];
        slots_body<WT>(a, WT * (bid - nqb - nbf), l4w);
        STAMP(a, SO, 15);
        return;
    }
    // ---- Q-role: LRU positions [b*256, +256) of fronts ++ queue ++ backs
    const int b = bid;
    const int64_t pos = (int64_t)b * kBS + threadIdx.x;
    int c = 0, oc = 0;
    if (a.qtiles == 4 && WT == 4) {
        queue_tiles<4>(a, 4 * b);
        STAMP(a, SO, 15);
        return;
    }
    if (a.shard == 2) {
        // phase 2 of a sharded tick: every rank's effective free counts arrived in the exchange
        // both loads issued together (a guarded slot load would wait for the c byte first)
        const int64_t pq = pos < a.Qlog ? pos : (a.Qlog > 0 ? a.Qlog - 1 : 0);
        const int cq = xc_get(a, pq);
        const int sq = lq_slot(a, pq);
        if (pos < a.Qlog) {
            c = cq;
            oc = (c > 0 && own_slot(a, sq) >= 0) ? c : 0;
        }
    } else if (a.deque) {
        // start(): c of every deque token from its worker's free count f, token count k and
        // the token's rank j (gpu_model.token_c): c = m + 1 + (j <= q), m = max(0, ceil(f/k) - 1),
        // q = f - m k - 1 (f <= 0: every token is served once)
        int32_t cc = INT32_MIN;
        int4 tk = make_int4(0, 0, 0, 0);
        if (pos < a.Qlog) {
            const int s = lq_slot(a, pos);
            if (s >= 0) {
                const Cur cu = cur_slot(a, s);
                int jr;
                if (pos < a.E) {
                    jr = a.front_rank[pos];
                } else if (pos < a.E + a.Qn) {
                    const uint32_t raw = a.qrank_in[pos - a.E];
                    const int j0 = (int)(raw & (kPart2 - 1)), x = a.xw_in[s];
                    jr = ((raw & kPart2) ? j0 - x : a.kl_in[s] - x + j0) + (cu.t ? a.post_nf[s] : 0);
                } else {
                    jr = a.back_rank[pos - a.E - a.Qn];
                }
                const int k = cu.t ? a.post_tok[s] : a.tokcnt_in[s];
                const int f = cu.fr;
                // q = f - m k - 1 also for f <= 0 (m = 0): then j <= q never holds and emit
                // recovers f = q + m k + 1 from the record
                int m = 0;
                if (f > 0) {
                    m = (f + k - 1) / k - 1;
                    m = m > 0 ? m : 0;
                }
                const int q = f - m * k - 1;
                cc = m + 1 + (jr <= q ? 1 : 0);
                tk = make_int4(jr, m, q, k);
            }
            a.c_arr[pos] = cc;
            a.c_tok[pos] = tk;
        }
        c = cc != INT32_MIN ? cc : 0;
    } else if (pos < a.Qlog) {
        int32_t raw = INT32_MIN;  // INT32_MIN: no live record (or not mine)
        double hbq = 0.0;
        const int64_t q = pos - a.E;  // committed queue position (fronts come first)
        const bool inq = q >= 0 && q < a.Qn;
        const int64_t qc = q < 0 ? 0 : (q < a.Qn ? q : (a.Qn > 0 ? a.Qn - 1 : 0));
        if (a.qaos && inq) {
            // a committed entry: slot, free count and heartbeat ride along by position
            // (queued slots are registered) -- three coalesced loads issued together,
            // then one 4-byte stamp gather; only slots that got a message this tick
            // gather their post-message record
            const int sq = a.queue_in[qc];
            const double hq = a.qhb_in[qc];
            const int32_t fq = a.qfree_in[qc];
            // touched: the bitmap word (L2-resident) when there is one, else the slot's stamp
            const bool tq = a.E > 0 && got_msg(a, sq);
            if (!tq) {
                hbq = hq;
                raw = ((a.now - hq) > a.tte) ? INT32_MIN : fq;
            } else {
                const uint8_t rf = a.post_rf[sq];
                const PostRec pr = a.post[sq];
                hbq = pr.hb;
                raw = ((rf & 1) && !((a.now - pr.hb) > a.tte)) ? pr.free : INT32_MIN;
                // moved to the front, re-appended or removed by this tick's messages; or a
                // window position whose slot had left the queue (kTomb: its slot may be queued
                // again at a later position)
                if (((rf >> 2) & 3) != kQsKeep || fq == kTomb) raw = INT32_MIN;
            }
        } else {
            q_raw_slow(a, pos, inq, raw, hbq);
        }
        if (raw != INT32_MIN) c = raw > 1 ? raw : 1;  // free <= 0 still takes one task (:409-419)
        if (!a.cq_direct) {
            a.c_arr[pos] = raw;
            if (!a.shard) a.c_hb[pos] = hbq;
        }
        if (a.shard == 1) xc_put(a, pos, c);
    }
    STAMP(a, SO, 1);
    if (a.shard == 1) {
        // phase 1 ends with the c values: phase 2 re-derives capacity and max c from
        // them (exact below the round table: its rows stay below the clamp).
        // Per-wave atomics on one exchange word cost ~10 ns each, serialised --
        // 14 K of them per tick at 8 ranks.
        if (a.xrows) {
            // ... and, with exchanged block rows, this block's counts of c > r (own
            // positions; r <= R): per wave from a histogram of min(c, R + 1) in LDS
            // (k_scan's scheme), summed over the waves; the row as 4-bit digits into the
            // exchange (the SUM over ranks: every rank's counts), the own counts as words
            __shared__ uint32_t xh[kWaves][kRFused + 2];
            const int R = a.R, lane = lane_id(), w = wave_id();
            uint32_t *h = xh[w];
            for (int i = lane; i <= R + 1; i += 64) h[i] = 0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            atomicAdd(&h[c < R + 1 ? c : R + 1], 1u);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            uint32_t carry = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int r = 64 * k + lane;
                const uint32_t P = carry + wave_incl_scan_u32(r <= R ? h[r] : 0u);
                if (r < kBS) wc[w][r] = r <= R ? 64u - P : 0u;
                carry = (uint32_t)__builtin_amdgcn_readlane((int)P, 63);
            }
            // max c (the byte's clamp, as exchanged) into word 1 of one of the rank's record
            // lines (8 lines: same-line device atomics serialise)
            const uint32_t wmx = wave_max_u32((uint32_t)(c < 255 ? c : 255));
            if (lane == 0) m4[w] = (int32_t)wmx;
            lds_barrier();
            const int xs = xr_stride(R), t = threadIdx.x;
            if (t == 0) {
                const int32_t bm = max(max(m4[0], m4[1]), max(m4[2], m4[3]));
                if (bm > 0)
                    atomicMax(&a.xrec[a.rank * kXRecWords + (b & (kXRecLines - 1)) * 16 + 1], (unsigned long long)bm);
            }
            uint8_t *const row = a.xrows + (size_t)b * xr_row(R);
            const uint32_t n = t < xs ? wc[0][t] + wc[1][t] + wc[2][t] + wc[3][t] : 0u;  // 0 past R
            if (t < xs) {
#pragma unroll
                for (int d = 0; d < kXRowDigits; ++d) row[d * xs + t] = (uint8_t)((n >> (4 * d)) & 15u);
                if (t < R) a.ocnt[(size_t)b * R + t] = n;
            } else if (t < xs + xr_row(R) - kXRowDigits * xs) {
                row[kXRowDigits * xs + (t - xs)] = 0;  // the row's padding
            }
            if (a.xgrows) {
                // the group's sums: memory-side adds, then a ticket; the group's last block
                // takes the sums (resetting them for the next tick) and writes the group's
                // digit row into the exchange and this rank's group row
                __shared__ int xlast;
                const int g = b / kXGroupBlocks;
                const int nbg = min(kXGroupBlocks, a.nbq - g * kXGroupBlocks);
                // the adds are device-scope atomics, performed at the coherence point before
                // each wave's vmcnt wait; the ticket is an agent-scope acq_rel RMW after every
                // wave's wait (the memory model's release / acquire pair, not just the
                // hardware's ordering), and the last block reads the sums with atomics
                uint32_t *acc = a.xg_acc + (size_t)g * kXgAccStride;
                if (t <= R && n) atomicAdd(&acc[t], n);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (t == 0)
                    xlast = __hip_atomic_fetch_add(&a.xg_tk[g], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                                    (uint32_t)(nbg - 1)
                                ? 1
                                : 0;
                __syncthreads();
                if (xlast) {
                    uint8_t *const gr = a.xgrows + (size_t)g * xg_row(R);
                    if (t < xs) {
                        const uint32_t v = t <= R ? atomicExch(&acc[t], 0u) : 0u;
#pragma unroll
                        for (int d = 0; d < kXGroupDigits; ++d) gr[d * xs + t] = (uint8_t)((v >> (4 * d)) & 15u);
                        if (t < R) a.ogrp[(size_t)g * R + t] = v;
                    } else if (t < xs + xg_row(R) - kXGroupDigits * xs) {
                        gr[kXGroupDigits * xs + (t - xs)] = 0;
                    }
                    if (t == 0) a.xg_tk[g] = 0u;
                }
            }
        }
        STAMP(a, SO, 15);
        return;
    }
    const uint32_t wmx = wave_max_u32((uint32_t)c);
    if (lane_id() == 0) m4[wave_id()] = (int32_t)wmx;
    unsigned long long csum = 0;
    if (a.shard == 2) {
        // phase 2: the round counts of all positions and of this rank's, one ballot per
        // round for both, 256 rounds (four 64-round groups) per pass
        __shared__ uint32_t owc[kWaves][kBS];
        const uint64_t own = __ballot(oc > 0);
        for (int rc = 0; rc < a.R; rc += kBS) {
            const int rn = (a.R - rc) < kBS ? (a.R - rc) : kBS;
#pragma unroll
            for (int g = 0; g < kBS / 64; ++g) {
                const int r0 = rc + g * 64;
                uint32_t cnt = 0, ocnt = 0;
                if (r0 < rc + rn && r0 < (int)wmx) {
                    int k = rc + rn - r0;
                    k = k < 64 ? k : 64;
                    k = k < (int)wmx - r0 ? k : (int)wmx - r0;
                    wave_round_counts2(c, own, r0, k, cnt, ocnt);
                }
                wc[wave_id()][g * 64 + lane_id()] = cnt;
                owc[wave_id()][g * 64 + lane_id()] = ocnt;
                // per 64-position segment: k_emit_shard's in-block rank bases
                if (g * 64 + lane_id() < rn) {
                    const size_t si = (size_t)(4 * b + wave_id()) * a.R + r0 + lane_id();
                    a.segcnt[si] = cnt;
                    a.osegcnt[si] = ocnt;
                }
            }
            lds_barrier();
            uint32_t t = 0;
            if ((int)threadIdx.x < rn) {
                const int r = threadIdx.x;
                t = wc[0][r] + wc[1][r] + wc[2][r] + wc[3][r];
                const uint32_t ot = owc[0][r] + owc[1][r] + owc[2][r] + owc[3][r];
                a.qcnt[(size_t)b * a.R + rc + r] = t;
                a.ocnt[(size_t)b * a.R + rc + r] = ot;
                // group rows (no k_plan): all positions in columns [0, R), this rank's in [R, 2R)
                if (a.grp_on) {
                    uint32_t *row = a.grp + (size_t)(b >> a.gshift) * a.gstride;
                    if (t) atomicAdd(&row[rc + r], t);
                    if (ot) atomicAdd(&row[a.R + rc + r], ot);
                }
            }
            const uint32_t ts = wave_sum_u32(t);
            if (lane_id() == 0) l4[wave_id()] = ts;
            lds_barrier();
            csum += (unsigned long long)l4[0] + l4[1] + l4[2] + l4[3];
            lds_barrier();
        }
    } else {
    // R <= 128: the wave's counts of c > r for every round from a histogram of
    // min(c, R) in LDS -- one LDS atomic per lane and a wave scan instead of one
    // ballot per round: count(c > r) = 64 - #(lanes with min(c, R) <= r)
    uint32_t hcnt[2] = {0u, 0u};
    if (a.R <= kRFused) {
        __shared__ uint32_t hist[kWaves][kRFused + 1];
        uint32_t *h = hist[wave_id()];
        const int lane = lane_id();
        for (int i = lane; i <= a.R; i += 64) h[i] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        atomicAdd(&h[c < a.R ? c : a.R], 1u);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        uint32_t carry = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int r = 64 * k + lane;
            const uint32_t hv = h[r < a.R ? r : a.R];
            const uint32_t P = carry + wave_incl_scan_u32(r < a.R ? hv : 0u);
            hcnt[k] = r < a.R ? 64u - P : 0u;
            carry = (uint32_t)__builtin_amdgcn_readlane((int)P, 63);
        }
    }
    for (int rc = 0; rc < a.R; rc += kBS) {
        const int rn = (a.R - rc) < kBS ? (a.R - rc) : kBS;
        for (int tab = 0; tab < 1; ++tab) {
            const int cc = tab ? oc : c;
#pragma unroll
            for (int g = 0; g < kBS / 64; ++g) {
                const int r0 = rc + g * 64;
                uint32_t cnt = 0;
                if (a.R <= kRFused) {
                    cnt = g < 2 ? hcnt[g] : 0u;
                } else if (r0 < rc + rn && r0 < (int)wmx) {
                    int k = rc + rn - r0;
                    k = k < 64 ? k : 64;
                    k = k < (int)wmx - r0 ? k : (int)wmx - r0;
                    cnt = wave_round_counts(cc, r0, k);
                }
                wc[wave_id()][g * 64 + lane_id()] = cnt;
                // per 64-position segment (k_emit2 derives its rank bases from these rows)
                if (a.fused && a.segw && tab == 0 && r0 < rc + rn && g * 64 + lane_id() < rn)
                    a.segcnt[(size_t)(4 * b + wave_id()) * a.R + r0 + lane_id()] = cnt;
            }
            lds_barrier();
            uint32_t t = 0;
            if ((int)threadIdx.x < rn) {
                t = wc[0][threadIdx.x] + wc[1][threadIdx.x] + wc[2][threadIdx.x] + wc[3][threadIdx.x];
                uint32_t *tabp = tab ? a.ocnt : a.qcnt;
                tabp[(size_t)b * a.R + rc + threadIdx.x] = t;
                // fused: the group's row of round totals (memory-side atomics, no return)
                if (a.grp_on && t) atomicAdd(&a.grp[(b >> a.gshift) * a.gstride + rc + threadIdx.x], t);
            }
            if (tab == 0 && !a.fused) {
                // sum_r count(c > r) over r < R = sum of min(c, R): the block's capacity when c <= R
                // (k_plan's; a fused k_emit2 sums the totals of the group rows itself)
                const uint32_t ts = wave_sum_u32(t);
                if (lane_id() == 0) l4[wave_id()] = ts;
                lds_barrier();
                csum += (unsigned long long)l4[0] + l4[1] + l4[2] + l4[3];
            }
            if (rc + kBS < a.R) lds_barrier();  // (wc is rewritten by the next column chunk)
        }
    }
    }
    if (threadIdx.x == 0) {
        int bm = m4[0];
        for (int w = 1; w < kWaves; ++w) bm = m4[w] > bm ? m4[w] : bm;
        a.qbm_raw[b] = bm;
        a.csum[b] = csum;
        if (a.shard == 2 && a.grp_on) {  // max c and capacity into columns 2R, 2R + 1
            uint32_t *row = a.grp + (size_t)(b >> a.gshift) * a.gstride;
            if (bm) atomicMax(&row[2 * a.R], (uint32_t)bm);
            if (csum) atomicAdd(&row[2 * a.R + 1], (uint32_t)csum);
        }
        if (a.grp_on && a.shard != 2 && bm > 0) atomicMax(&a.grp[(b >> a.gshift) * a.gstride + a.R], (uint32_t)bm);
    }
    STAMP(a, SO, 15);
}

// ------------------------------------------------------------ window ticks
// A level-0 tick serves the first N = O + T live positions of fronts ++ queue ++ backs
// and its next queue is the rest followed by the served workers with c > 1, so when
// every front is served and the N-th live position falls inside the committed window,
// the tick touches only the window's served prefix: the suffix stays where it is, the
// live backs and then the served workers with c > 1 are appended at the window's tail.
// The elements are numbered in the order [backs][fronts][window]: 1024-element chunks,
// one k_emit_win workgroup each.
struct WinEl {
    int s;        // slot, -1: a hole of a list
    int32_t raw;  // free count of a live queued position, INT32_MIN otherwise
    double hb;
    bool t;       // the slot got messages this tick
    int32_t mv;   // list entries: the committed position the slot left (-1: it was not queued)
};
// region of chunk ch: 0 backs, 1 fronts, 2 window; [i0, i1) its element range in the region
__device__ __forceinline__ int win_region(const TickArgs &a, int ch, int64_t &i0, int64_t &i1) {
    if (ch < a.nchB) {
        i0 = (int64_t)ch * kWinCh;
        i1 = min(i0 + kWinCh, (int64_t)a.E);
        return 0;
    }
    if (ch < a.nchB + a.nchF) {
        i0 = (int64_t)(ch - a.nchB) * kWinCh;
        i1 = min(i0 + kWinCh, (int64_t)a.E);
        return 1;
    }
    i0 = a.wq_off + (int64_t)(ch - a.nchB - a.nchF) * kWinCh;
    i1 = min(i0 + kWinCh, a.wq_tail);
    return 2;
}
// The element's slot and raw free count, as k_scan's queue role classifies a position:
// a list entry (a front / back insertion of this tick) from the purge's next free count,
// a committed window position from its ride-along free count and heartbeat unless the
// slot got messages (then its post-message record) or the position is a tombstone.
// Loads are issued before the tests (clamped indices).
__device__ __forceinline__ WinEl win_elem(const TickArgs &a, int reg, int64_t i, bool in) {
    WinEl e;
    if (reg < 2) {
        const int32_t *lst = reg == 0 ? a.back_list : a.front_list;
        const int64_t ic = in ? i : 0;
        const int s1 = a.E > 0 ? lst[ic] : 0;
        const int sc = s1 > 0 ? s1 - 1 : 0;
        const int32_t fr = a.free_out[sc].x;
        const double h = a.post[sc].hb;
        const uint8_t rf = a.post_rf[sc];
        const int32_t p0 = a.pos_in[sc];
        e.s = s1 - 1;
        e.raw = (in && s1 > 0) ? fr : INT32_MIN;
        e.hb = h;
        e.t = true;
        e.mv = (s1 > 0 && (rf & kRfQ0)) ? p0 : -1;
    } else {
        const int64_t ic = in ? i : a.wq_off;
        const int sq = a.wq_buf[ic];
        const int32_t fq = a.wqf_buf[ic];
        const double hq = a.wqh_buf[ic];
        // the touched bit and the post-message record in one load round (the record of an
        // untouched slot is loaded and ignored: a dependent round costs more than the line)
        const bool tq = got_msg(a, sq);
        const uint8_t rf = a.post_rf[sq];
        const PostRec pr = a.post[sq];
        int32_t raw = ((a.now - hq) > a.tte) ? INT32_MIN : fq;
        double hb = hq;
        if (tq) {
            hb = pr.hb;
            raw = ((rf & 1) && !((a.now - pr.hb) > a.tte) && ((rf >> 2) & 3) == kQsKeep) ? pr.free : INT32_MIN;
        }
        if (fq == kTomb || !in) raw = INT32_MIN;
        e.s = sq;
        e.raw = raw;
        e.hb = hb;
        e.t = tq;
        e.mv = -1;
    }
    return e;
}
__device__ __forceinline__ int win_c(int32_t raw) { return raw != INT32_MIN ? (raw > 1 ? raw : 1) : 0; }

// ------------------------------------------------------------ k_logscan
// The log role of k_scan as its own launch for large tables (a.f_sep): past 128K
// slots a gather per in-flight entry -- into the 16-byte records or the global
// bitmap -- costs a 64-byte L2 request each.  One 16-wave workgroup per CU
// instead copies the whole died bitmap (W/8 bytes, <= the 160 KB of LDS) once,
// then every wave flags the orphans of whole 2048-entry tiles alone (lane: 4
// groups of 8 consecutive entries, 8 int4 loads in flight), with k_scan's
// per-tile ofl / fcnt layout so k_emit's orphan compaction is unchanged.
__global__ __launch_bounds__(kLsBS) void k_logscan(TickArgs a) {
    prefetch_args(a);
    extern __shared__ __attribute__((aligned(16))) unsigned long long bm[];
    const int SO = 3 * (a.nbw + a.nbf + a.nbq);  // diagnostic stamp rows
    STAMP(a, SO, 0);
    const int lblk = (int)blockIdx.x, nlblk = (int)gridDim.x;
    if (a.died_tag && *a.died_tag != a.lstamp) {
        // window tick in which no registration died: no entry is an orphan, so the log is
        // not read -- every tile's count and every workgroup's partial are zero
        for (int b = lblk * kLsBS + (int)threadIdx.x; b < a.nbf; b += nlblk * kLsBS) a.fcnt[b] = 0;
        if (threadIdx.x == 0) a.lpart[lblk] = 0;
        STAMP(a, SO, 15);
        return;
    }
    const int n4 = (((a.W + 63) >> 6) + 1) >> 1;
    const uint4 *src = reinterpret_cast<const uint4 *>(a.dmask);
    for (int i0 = 0; i0 < n4; i0 += kLsBS * 8) {
        uint4 t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + k * kLsBS + (int)threadIdx.x;
            t[k] = src[i < n4 ? i : n4 - 1];
        }
        // stores past the bitmap go to one spare slot, not behind a branch: a
        // guarded store lets the compiler sink its load into the branch, one
        // round trip per load
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + k * kLsBS + (int)threadIdx.x;
            reinterpret_cast<uint4 *>(bm)[i < n4 ? i : n4] = t[k];
        }
    }
    __syncthreads();
    STAMP(a, SO, 1);
    const int lane = lane_id();
    constexpr int nw = kLsBS / 64;
    const int64_t nlog = a.shard ? a.head_local : a.head_in;
    uint32_t wtot = 0;  // this wave's orphans (window ticks: the workgroup's partial)
    for (int b = lblk * nw + (int)(threadIdx.x >> 6); b < a.nbf; b += nlblk * nw) {
        int32_t v[4][kFItems];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t base = (int64_t)b * kFTile + (int64_t)(k * 64 + lane) * kFItems;
            if (base + kFItems <= nlog) {
                const int4 x0 = *reinterpret_cast<const int4 *>(a.log_slot + base);
                const int4 x1 = *reinterpret_cast<const int4 *>(a.log_slot + base + 4);
                v[k][0] = x0.x; v[k][1] = x0.y; v[k][2] = x0.z; v[k][3] = x0.w;
                v[k][4] = x1.x; v[k][5] = x1.y; v[k][6] = x1.z; v[k][7] = x1.w;
            } else {
#pragma unroll
                for (int j = 0; j < kFItems; ++j) v[k][j] = (base + j < nlog) ? a.log_slot[base + j] : -1;
            }
        }
        // died bits from LDS: an entry is an orphan iff its slot's registration alive at
        // tick start died (entries of earlier registrations: cleared at commit, or older than
        // the slot's epoch under lazy clears -- drop_stale)
        uint32_t cnt = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t flags = 0;
#pragma unroll
            for (int j = 0; j < kFItems; ++j) {
                int sj = v[k][j];
                if (a.shard && sj >= 0) sj -= a.slot_base;  // log slots are global ids
                const int sc = sj < 0 ? 0 : sj;
                // (32-bit LDS reads: one bank per lane instead of two)
                const uint32_t *bm32 = reinterpret_cast<const uint32_t *>(bm);
                flags |= (sj >= 0 && ((bm32[sc >> 5] >> (sc & 31)) & 1u)) ? (1u << j) : 0u;
            }
            const int64_t fb0 = (int64_t)b * kFTile + (int64_t)(k * 64 + lane) * kFItems;
            flags = drop_completed(a, drop_stale<kFItems>(a, flags, v[k], fb0), v[k], fb0);
            if (a.wseg) {
                // the tile's orphans, ascending, into its own segment (orphans[b*2048 + i]):
                // entry order is k, then lane, then j
                const uint32_t n = (uint32_t)__popc(flags);
                const uint32_t inc = wave_incl_scan_u32(n);
                int64_t o = (int64_t)b * kFTile + cnt + inc - n;
                const int64_t e0 = (int64_t)b * kFTile + (int64_t)(k * 64 + lane) * kFItems;
                for (uint32_t m = flags; m; m &= m - 1) a.orphans[o++] = e0 + __builtin_ctz(m);
                cnt += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            } else {
                a.ofl[(size_t)b * kBS + k * 64 + lane] = (uint8_t)flags;
                cnt += (uint32_t)__popc(flags);
            }
        }
        if (!a.wseg) cnt = wave_sum_u32(cnt);
        wtot += cnt;
        if (lane == 0) {
            a.fcnt[b] = cnt;
            if (a.grp_on && cnt) atomicAdd(&a.grp[(b % a.ngrp) * a.gstride + a.R + 1], cnt);
            if (a.shard && cnt)
                atomicAdd(&a.xrec[a.rank * kXRecWords + (b & (kXRecLines - 1)) * 16], (unsigned long long)cnt);
        }
    }
    if (a.wseg) {
        // the workgroup's orphans (k_emit_win sums the partials for O)
        __shared__ uint32_t lp[kLsBS / 64];
        if (lane == 0) lp[threadIdx.x >> 6] = wtot;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (int q = 0; q < kLsBS / 64; ++q) t += lp[q];
            a.lpart[lblk] = t;
        }
    }
    STAMP(a, SO, 15);
}

// ------------------------------------------------------------ k_plan (large grids only)
// wg 0: orphan block offsets + O; wg 1: evicted block offsets; wg 2: max c and
// capacity; wg 3+r: exclusive scan of round r's counts across queue blocks.
__global__ __launch_bounds__(kBS) void k_plan(TickArgs a) {
    prefetch_args(a);
    __shared__ unsigned long long l4[kWaves];
    __shared__ int32_t m4[kWaves];
    const int bid = blockIdx.x;
    const int SO = 3 * (a.nbw + a.nbf + a.nbq) + 512;  // diagnostic stamp rows
    STAMP(a, SO, 0);
    if (bid <= 1) {
        const unsigned long long tot = bid == 0 ? run_excl_scan(a.fcnt, 1, a.nbf, a.fpre, 1, l4)
                                                : run_excl_scan(a.wcnt, 1, a.nbw, a.wpre, 1, l4);
        if (threadIdx.x == 0) {
            if (bid == 0) {
                a.P->O_local = (int64_t)tot;
                if (!a.shard) a.P->O = (int64_t)tot;
            } else {
                a.P->n_evicted = (int64_t)tot;
            }
        }
        return;
    }
    if (bid == 2) {
        // capacity and max c from the queue blocks (sharded phase 2: of the exchanged
        // c bytes); sharded: every rank's orphan count from the exchange records
        int32_t mx = 0;
        unsigned long long sum = 0;
        // sharded: the ranks' orphan-count partials (kXRecLines per rank), one load per
        // thread issued up front -- a serial loop over them costs a round trip each
        uint32_t op = 0;
        if (a.shard)
            for (int g = threadIdx.x; g < a.world * kXRecLines; g += kBS) op += (uint32_t)a.xrec[(size_t)g * 16];
        for (int i0 = 0; i0 < a.nbq; i0 += 8 * kBS) {
            int32_t m[8];
            unsigned long long cs[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = i0 + k * kBS + (int)threadIdx.x;
                m[k] = a.qbm_raw[min(i, a.nbq - 1)];
                cs[k] = a.csum[min(i, a.nbq - 1)];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool ok = i0 + k * kBS + (int)threadIdx.x < a.nbq;
                mx = (ok && m[k] > mx) ? m[k] : mx;
                sum += ok ? cs[k] : 0ull;
            }
        }
        __shared__ uint32_t ow[kWaves];
        op = wave_sum_u32(op);
        if (lane_id() == 0) ow[wave_id()] = op;
        mx = block_reduce_max<int32_t>(mx, m4);
        unsigned long long tot;
        block_excl_scan<unsigned long long>(sum, l4, tot);
        if (threadIdx.x == 0) {
            a.P->maxc = mx;
            a.P->cap_total = (int64_t)tot;
            if (a.shard) a.P->O = (int64_t)ow[0] + ow[1] + ow[2] + ow[3];
        }
        return;
    }
    // rows: r < R of all positions, then (sharded) r < R of this rank's positions
    const int rr = bid - 3;
    const bool mine = rr >= a.R;
    const int r = mine ? rr - a.R : rr;
    if (r >= a.R || (mine && !a.shard)) return;
    const uint32_t *cnt = mine ? a.ocnt : a.qcnt;
    int64_t *pre = mine ? a.opre : a.qpre;
    const unsigned long long tot = run_excl_scan(cnt + r, (size_t)a.R, a.nbq, pre + r, (size_t)a.R, l4);
    if (threadIdx.x == 0) (mine ? a.oA : a.A)[r] = (int64_t)tot;
    STAMP(a, SO, 15);
}

// ------------------------------------------------------------ k_xscan (sharded phase 2, large queues)
// The per-block prefixes of the exchanged round counts (xrows_mode 2: > kXRowsMaxBlocks
// queue blocks, R = kXGroupR): one workgroup per chunk of kXsBlocks = 64 queue blocks, lane l
// of every wave the rows of block 64 ch + l; wave w the 16 columns [16 w, 16 w + 16) of the
// 2R = 64 (waves 0-1: every rank's counts, decoded from the block's 4-bit digit row; waves
// 2-3: this rank's own row), each column one DPP scan across the wave's lanes -- no LDS
// transpose.  The chunk-local exclusive prefixes go out as 64 contiguous bytes per lane, the
// chunk totals into xct.  The last workgroup (an agent-scope acq_rel ticket) turns the chunk
// totals into exclusive prefixes over the chunks -- four parts per column, each part's chunks
// loaded at once -- and writes the totals A(r).  (k_plan's one workgroup per column walked
// 3.5 K rows with a 64-line gather per wave load: 13-17 us at configs[3]; an LDS transpose per
// 256-block chunk 11-14 us; counting the exchanged c bytes here instead of in phase 1 -- a
// phase 1 without a queue role -- 20-31 us: NOTES_r05.md.)
template <int R>
__global__ __launch_bounds__(kBS) void k_xscan(TickArgs a) {
    prefetch_args(a);
    const int SO = 3 * (a.nbw + a.nbf + a.nbq) + 6000;  // diagnostic stamp rows (stamps builds)
    STAMP(a, SO, 0);
    static_assert(2 * R == 4 * 16 && kXsBlocks == 64, "four waves of 16 columns, a lane per block");
    constexpr int C = 2 * R, XS = xr_stride(R), NQ = xr_row(R) / 16;
    __shared__ int last;
    __shared__ uint32_t psum[kWaves][C];
    const int ch = blockIdx.x, t = threadIdx.x, lane = lane_id(), w = wave_id();
    const int b = ch * kXsBlocks + lane;
    const bool in = b < a.nbq;
    const int bc = in ? b : a.nbq - 1;
    uint32_t v[16];
    auto word = [](const uint4 &q, int i) -> uint32_t { return i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w; };
    if (w < 2) {
        // every rank's counts of rounds 16 w .. 16 w + 15: digit bytes r, XS + r, 2 XS + r
        uint4 d[NQ];
        const uint4 *dr = reinterpret_cast<const uint4 *>(a.xrows + (size_t)bc * xr_row(R));
#pragma unroll
        for (int k = 0; k < NQ; ++k) d[k] = dr[k];
        auto byte = [&](int k) -> uint32_t { return (word(d[k >> 4], (k >> 2) & 3) >> (8 * (k & 3))) & 0xffu; };
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            // (w is wave-uniform: both forms unrolled with constant byte indices)
            const uint32_t x0 = byte(j) + (byte(XS + j) << 4) + (byte(2 * XS + j) << 8);
            const uint32_t x1 = byte(16 + j) + (byte(XS + 16 + j) << 4) + (byte(2 * XS + 16 + j) << 8);
            v[j] = in ? (w == 0 ? x0 : x1) : 0u;
        }
    } else {
        // this rank's own counts of rounds 16 (w - 2) .. +15: words of its own row
        const uint4 *orw = reinterpret_cast<const uint4 *>(a.ocnt + (size_t)bc * R) + 4 * (w - 2);
        uint4 o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = orw[k];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = in ? word(o[j >> 2], j & 3) : 0u;
    }
    STAMPW(a, SO, 1);
    uint32_t tot[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t inc = wave_incl_scan_u32(v[j]);
        tot[j] = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        v[j] = inc - v[j];
    }
    STAMP(a, SO, 2);
    if (in) {
        uint4 *dst = reinterpret_cast<uint4 *>(a.xpre + (size_t)b * C + 16 * w);
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
    uint32_t my = 0;  // lane j < 16: column 16 w + j's chunk total
#pragma unroll
    for (int j = 0; j < 16; ++j) my = lane == j ? tot[j] : my;
    if (lane < 16) a.xct[(size_t)ch * C + 16 * w + lane] = my;
    if (a.xself) {  // k_emit_shard_xp sums the chunk totals itself
        STAMP(a, SO, 15);
        return;
    }
    // every wave's stores done, then the ticket (release / acquire at agent scope)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    STAMP(a, SO, 4);
    if (t == 0) last = __hip_atomic_fetch_add(a.xtk, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                           (uint32_t)(gridDim.x - 1);
    __syncthreads();
    STAMP(a, SO, 5);
    if (!last) {
        STAMP(a, SO, 15);
        return;
    }
    // exclusive prefixes over the chunks: column col = t % C, part t / C of kBS / C, each
    // part's chunks loaded at once (up to 64 in registers), then the parts' offsets
    constexpr int NP = kBS / C;
    const int col = t % C, part = t / C;
    const int nch = (int)gridDim.x, per = (nch + NP - 1) / NP;
    const int c0 = part * per;
    if (per <= 64) {
        uint32_t x[64];
        uint32_t sum = 0;
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            x[k] = a.xct[(size_t)min(c0 + k, nch - 1) * C + col];
            x[k] = (k < per && c0 + k < nch) ? x[k] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 64; ++k) sum += x[k];
        psum[part][col] = sum;
        __syncthreads();
        uint32_t run = 0, all = 0;
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            run += q < part ? psum[q][col] : 0u;
            all += psum[q][col];
        }
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            if (k < per && c0 + k < nch) a.xct[(size_t)(c0 + k) * C + col] = run;
            run += x[k];
        }
        if (part == 0) a.xA[col] = all;
    } else if (t < C) {
        // (past 64 x NP chunks: one thread per column, 16 chunks in flight per pass)
        uint32_t run = 0;
        for (int b0 = 0; b0 < nch; b0 += 16) {
            uint32_t x[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] = a.xct[(size_t)min(b0 + k, nch - 1) * C + t];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (b0 + k < nch) a.xct[(size_t)(b0 + k) * C + t] = run;
                run += b0 + k < nch ? x[k] : 0u;
            }
        }
        a.xA[t] = run;
    }
    if (t == 0) *a.xtk = 0u;
    STAMP(a, SO, 15);
}

// ------------------------------------------------------------ k_plan2 (large grids, R <= 128)
// k_plan for k_emit2 when k_scan's queue blocks also added their counts into
// group rows (<= 64 groups of 2^gshift blocks): one workgroup per group reads
// the group rows (totals A(r), the prefix of the earlier groups, max c, orphan
// and eviction totals), finds the fill level L as k_emit2 does, and scans the
// rows of its own group for rounds r <= L + 1 only -- the rounds k_emit2 reads
// (a streaming tick: 2 of 64 columns) -- instead of k_plan's one workgroup per
// round walking a column of every block.  Two more workgroups scan the orphan /
// eviction tile counts.  Group 0 publishes the totals (A, P).
constexpr int kGrpLd = 4;     // group / block row loads per thread per batch (k_plan2, k_emit2)
constexpr int kP2Rows = kBS;  // rows per pass of a group's scan (one per thread)
// k_plan2's group scan for groups of <= 64 blocks (one wave; lane l = block b0 + l)
template <int R>
__device__ __forceinline__ void plan2_group_rows(const TickArgs &a, int g, int b0, int b1, int nr,
                                                 const uint32_t *gp_r) {
    const int lane = lane_id();
    const int b = b0 + lane;
    const bool in = b < b1;
    const uint4 *rp = reinterpret_cast<const uint4 *>(a.qcnt + (size_t)min(b, b1 - 1) * R);
    uint32_t v[R];
#pragma unroll
    for (int k = 0; k < R / 4; ++k) {
        const uint4 q = rp[k];
        v[4 * k] = q.x;
        v[4 * k + 1] = q.y;
        v[4 * k + 2] = q.z;
        v[4 * k + 3] = q.w;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t x = (in && r < nr) ? v[r] : 0u;
        const uint32_t inc = wave_incl_scan_u32(x);
        if (in && r < nr) a.qpre[(size_t)b * R + r] = (int64_t)gp_r[r] + (int64_t)(inc - x);
    }
}
__global__ __launch_bounds__(kBS) void k_plan2(TickArgs a) {
    prefetch_args(a);
    __shared__ unsigned long long l4[kWaves];
    __shared__ uint32_t gpre[kBS], gtot[kBS];
    __shared__ uint32_t gp_r[kRFused];           // prefix of the earlier groups, round r
    __shared__ uint32_t red[kWaves][4];
    __shared__ uint32_t wtot[kWaves][4];
    __shared__ int nr_s;
    const int bid = blockIdx.x;
    const int ng = a.ngrp;
    if (bid >= ng) {
        const bool f = bid == ng;
        const unsigned long long tot =
            f ? run_excl_scan(a.fcnt, 1, a.nbf, a.fpre, 1, l4) : run_excl_scan(a.wcnt, 1, a.nbw, a.wpre, 1, l4);
        (void)tot;
        return;
    }
    const int g = bid, R = a.R, gs = a.gstride;
    const int lane = lane_id(), w = wave_id();
    // ---- group rows: thread t sums round r = t mod R over parts p = t / R
    {
        const int P = kBS / R, r = (int)threadIdx.x & (R - 1), p = (int)threadIdx.x / R;
        uint32_t pre = 0, tot = 0;
        for (int j0 = 0; j0 * P < ng; j0 += kGrpLd) {
            uint32_t v[kGrpLd];
#pragma unroll
            for (int j = 0; j < kGrpLd; ++j) v[j] = a.grp[min(p + P * (j0 + j), ng - 1) * gs + r];
#pragma unroll
            for (int j = 0; j < kGrpLd; ++j) {
                const int gg = p + P * (j0 + j);
                tot += gg < ng ? v[j] : 0u;
                pre += gg < g ? v[j] : 0u;
            }
        }
        gpre[threadIdx.x] = pre;
        gtot[threadIdx.x] = tot;
        // max c, orphans, evictions: columns R .. R + 2 (ng <= 64: wave 0 holds them)
        const int gi = min((int)threadIdx.x, ng - 1) * gs + R;
        const bool gin = (int)threadIdx.x < ng;
        const uint32_t mg = gin ? a.grp[gi] : 0u, og = gin ? a.grp[gi + 1] : 0u, eg = gin ? a.grp[gi + 2] : 0u;
        uint32_t fo = og, wo = eg;
        const uint32_t mo = wave_max_u32(mg);
        fo = wave_sum_u32(fo);
        wo = wave_sum_u32(wo);
        if (lane == 0) {
            red[w][0] = fo;
            red[w][1] = wo;
            red[w][3] = mo;
        }
        lds_barrier();
    }
    const int64_t O = (int64_t)red[0][0] + red[1][0] + red[2][0] + red[3][0];
    const int64_t nev = (int64_t)red[0][1] + red[1][1] + red[2][1] + red[3][1];
    const int maxc = (int)max(max(red[0][3], red[1][3]), max(red[2][3], red[3][3]));
    const int rlim = maxc < R ? maxc : R;
    if (w == 0) {
        // per round r (lane i of chunk k: r = 64 k + i): A(r), the earlier groups' prefix,
        // S(r) and the fill level L -- k_emit2's computation
        const int P = kBS / R;
        int64_t carry = 0, S1v[2];
        uint32_t Av[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int r = 64 * k + lane;
            uint32_t sp = 0, st_ = 0;
            if (r < R)
                for (int q = 0; q < P; ++q) {
                    sp += gpre[q * R + r];
                    st_ += gtot[q * R + r];
                }
            if (r < R) gp_r[r] = sp;
            Av[k] = st_;
            const uint32_t v = r < rlim ? st_ : 0u;
            const uint32_t incl = wave_incl_scan_u32(v);
            S1v[k] = carry + (int64_t)incl;
            carry += (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        const int64_t cap = maxc > R ? INT64_MAX : carry;
        const int64_t N = (a.redist ? O : 0) + a.T;
        const int64_t N_eff = N < cap ? N : cap;
        int L = 0;
#pragma unroll
        for (int k = 0; k < 2; ++k) L += __popcll(__ballot(64 * k + lane < rlim && S1v[k] <= N_eff));
        if (lane == 0) nr_s = min(L + 2, R);
        if (g == 0 || a.repl) {
            int64_t *Ad = a.repl ? a.A_rep + (size_t)g * kRFused : a.A;
            DevTotals *Pd = a.repl ? a.P_rep + g : a.P;
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (64 * k + lane < R) Ad[64 * k + lane] = (int64_t)(64 * k + lane < rlim ? Av[k] : 0u);
            if (lane == 0) {
                Pd->O = O;
                Pd->O_local = O;
                Pd->n_evicted = nev;
                Pd->cap_total = cap;
                Pd->maxc = maxc;
            }
        }
    }
    lds_barrier();
    const int nr = nr_s;
    // ---- this group's rows, rounds r < nr: prefix = earlier groups + earlier rows
    const int gsz = 1 << a.gshift, b0 = g * gsz, b1 = min(b0 + gsz, a.nbq);
    if (gsz <= 64 && (R == 32 || R == 64)) {
        // a group of <= 64 blocks (configs[3]: 56 groups of 64): wave 0, lane l = block b0 + l,
        // its whole row in one load round (16-byte loads), then one DPP scan across the lanes
        // per round -- instead of a load round and a block barrier per 4 rounds (8.6 us at
        // configs[3])
        if (w == 0) {
            if (R == 32) plan2_group_rows<32>(a, g, b0, b1, nr, gp_r);
            else plan2_group_rows<64>(a, g, b0, b1, nr, gp_r);
        }
        return;
    }
    for (int r0 = 0; r0 < nr; r0 += 4) {
        uint32_t carry4[4] = {0u, 0u, 0u, 0u};
        for (int c0 = b0; c0 < b1; c0 += kP2Rows) {
            const int b = c0 + (int)threadIdx.x;
            const int bc = min(b, b1 - 1);
            uint32_t v[4], x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = a.qcnt[(size_t)bc * R + min(r0 + u, R - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                v[u] = (b < b1 && r0 + u < nr) ? v[u] : 0u;
                x[u] = wave_incl_scan_u32(v[u]);
                if (lane == 63) wtot[w][u] = x[u];
            }
            lds_barrier();
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                uint32_t before = carry4[u], all = 0;
#pragma unroll
                for (int q = 0; q < kWaves; ++q) {
                    before += q < w ? wtot[q][u] : 0u;
                    all += wtot[q][u];
                }
                if (b < b1 && r0 + u < nr)
                    a.qpre[(size_t)b * R + r0 + u] = (int64_t)gp_r[r0 + u] + (int64_t)(before + x[u] - v[u]);
                carry4[u] += all;
            }
            lds_barrier();  // wtot reused
        }
    }
}

// Deque mode: the end of a token's tick.  Tokens of one worker share its count
// (atomic), survivors carry their rank from before the round-L split plus the
// part they sat in; per slot, x_w = highest rank served in round L and K_L =
// tokens with c > L let the next tick re-rank them (gpu_model.tick_deque).
__device__ __forceinline__ void deque_finish(const TickArgs &a, int64_t pos, int s, int c, int L, int64_t n_q,
                                             bool servedL, int64_t np) {
    const int4 tk = a.c_tok[pos];  // {j, m, q, k}; f = q + m k + 1
    if (tk.w == 1) {
        // the worker's only token: plain stores
        a.free_out[s].x = tk.z + tk.y + 1 - (int32_t)n_q;
        if (np >= 0) a.tokcnt_out[s] = 1;
        if (c > L && servedL) a.xw_out[s] = 1;
    } else {
        atomicSub(&a.free_out[s].x, (int32_t)n_q);
        if (np >= 0) atomicAdd(&a.tokcnt_out[s], 1);
        if (c > L && servedL) atomicMax(&a.xw_out[s], tk.x);
    }
    if (c > L) a.kl_out[s] = L < tk.y + 1 ? tk.w : (L == tk.y + 1 ? tk.z : 0);
    if (np >= 0 && np < a.q_cap) {
        a.queue_out[np] = s;
        a.qrank_out[np] = (uint32_t)tk.x | (servedL ? 0u : kPart2);
    }
}

// The tick's assignments in compact form (fb_get_outputs_compact): per LRU position its
// slot and min(c, L + 1) -- with the fill level, every task's slot in closed form
// (task k of round r <= L is A_r[k - S(r)]) in 5 bytes per queued worker instead of 4
// bytes per task.  c = 0: no live queued worker at this position.
__device__ __forceinline__ void compact_out(const TickArgs &a, int64_t pos, int s, int c, int L) {
    const int cl = c < L + 1 ? c : L + 1;
    a.rb_slot[pos] = c > 0 ? s : -1;
    a.rb_c[pos] = (uint8_t)(cl < 255 ? cl : 255);
}

// ------------------------------------------------------------ k_emit
// Water-filling emission for one queue block once the fill level is known:
// rounds [0, rfull) in full, round L partially (ranks < p), round L+1 ranks.
// pre(i) / Srd(i): this block's prefix and S(r) of round r = rc + i.
struct EmitLds {
    uint32_t wc[kWaves][kBS];   // per-wave counts of c > r
    int32_t wbase[kWaves][kBS]; // rank base of a wave in A_r
    int32_t wpos[kWaves][kBS];  // S(r) + rank base (task index base), r <= L
};

template <int MODE>
__global__ __launch_bounds__(kBS) void k_emit(TickArgs a_) {
    prefetch_args(a_);
    const TickArgs a = specialise<MODE>(a_);
    __shared__ EmitLds E_;
    __shared__ uint32_t red[kWaves][4];
    __shared__ unsigned long long red64[kWaves];
    __shared__ int64_t S_l[kBS + 1];             // S(r) of the current round chunk
    __shared__ int64_t pre_c[kBS];               // this block's prefix of round r (chunk)
    __shared__ int32_t misc[8];
    const int bid = blockIdx.x;
    const int SO = a.nbw + a.nbf + a.nbq + (a.slots_in_scan ? a.nbw : 0);
    STAMP(a, SO, 0);
    const int lane = lane_id(), w = wave_id();
    if (bid < a.nbq) {
        const int b = bid;
        const int64_t pos = (int64_t)b * kBS + threadIdx.x;
        int32_t raw = INT32_MIN;
        double hbp = 0.0;
        int s = -1;
        int64_t O, nev = 0, cap;
        int maxc, bm;
        int rlim;
        int L = 0;
        int64_t S_L = 0, N_eff;
        {
            // ---- totals and the scanned round table from k_plan
            if (pos < a.Qlog) {
                raw = a.c_arr[pos];
                hbp = a.c_hb[pos];
                s = lq_slot(a, pos);
            }
            bm = a.qbm_raw[b];
            O = a.P->O;
            nev = a.P->n_evicted;
            cap = a.P->cap_total;
            maxc = a.P->maxc;
            rlim = maxc < a.R ? maxc : a.R;
            if (maxc > a.R) cap = INT64_MAX;
            const int64_t N = (a.redist ? O : 0) + a.T;  // purge-only ticks report orphans, dispatch none
            N_eff = N < cap ? N : cap;
            int64_t carry = 0;  // S(rc)
            for (int rc = 0; rc < rlim; rc += kBS) {
                const int r = rc + threadIdx.x;
                const unsigned long long v = r < rlim ? (unsigned long long)a.A[r] : 0ull;
                unsigned long long tot;
                const unsigned long long ex = block_excl_scan<unsigned long long>(v, red64, tot);
                const int64_t S1 = carry + (int64_t)(ex + v);  // S(r + 1)
                const bool ok = r < rlim && S1 <= N_eff;
                const int k_w = __popcll(__ballot(ok));
                if (lane == 0) misc[w] = k_w;
                S_l[threadIdx.x + 1] = S1;
                if (threadIdx.x == 0) S_l[0] = carry;
                lds_barrier();
                const int k = misc[0] + misc[1] + misc[2] + misc[3];
                L += k;
                S_L = S_l[k];
                lds_barrier();
                if (k < kBS) break;
                carry += (int64_t)tot;
            }
        }
        int status = 0;
        if (maxc > a.R && L >= a.R - 1) status = 1;   // rows beyond the table needed: rerun wider
        else if (a.head_in + N_eff > a.log_cap) status = 2;  // never write past the in-flight log (N_eff exact once R is)
        const int64_t p = N_eff - S_L;
        auto getA = [&](int r) -> int64_t { return r < rlim ? a.A[r] : (int64_t)0; };
        const int64_t AL = (L < maxc && L < rlim) ? getA(L) : 0;
        STAMP(a, SO, 2);
        if (b == 0 && threadIdx.x == 0) {
            a.hout->O = O;
            a.hout->n_evicted = nev;
            a.hout->cap_total = cap;
            a.hout->maxc = maxc;
            a.hout->L = L;
            a.hout->status = status;
            a.hout->N_eff = status ? 0 : N_eff;
            a.hout->p = p;
            a.hout->AL = AL;
            if (AL == 0) a.hout->new_qlen = 0;
        }
        if (status) return;
        // ---- water-filling emission, 256 rounds per chunk, rounds 0 .. L+1
        const int c = raw != INT32_MIN ? (a.deque ? raw : (raw > 1 ? raw : 1)) : 0;
        if (a.rb_slot && pos < a.Qlog) compact_out(a, pos, s, c, L);
        int32_t *const out = a.log_slot + a.head_in;
        int64_t rankL = -1, exL1 = 0;
        int64_t carryS = 0;  // S(rc)
        const int wmx = (int)wave_max_u32((uint32_t)c);
        for (int rc = 0; rc <= L + 1; rc += kBS) {
            const int rn = (L + 2 - rc) < kBS ? (L + 2 - rc) : kBS;
            {
                // chunk tables from k_plan: pre(r), S(r)
                const int r = rc + threadIdx.x;
                int64_t pr = 0, Av = 0;
                if ((int)threadIdx.x < rn && r < rlim) {
                    pr = a.qpre[(size_t)b * a.R + r];
                    Av = a.A[r];
                }
                unsigned long long tot;
                const unsigned long long ex = block_excl_scan<unsigned long long>((unsigned long long)Av, red64, tot);
                pre_c[threadIdx.x] = pr;
                S_l[threadIdx.x] = carryS + (int64_t)ex;
                carryS += (int64_t)tot;
            }
            STAMP(a, SO, 5);
            // per-wave counts of c > r for the chunk's rounds
#pragma unroll
            for (int g = 0; g < kBS / 64; ++g) {
                const int r0 = rc + g * 64;
                uint32_t cnt = 0;
                if (r0 < rc + rn && r0 < wmx) {
                    int k = rc + rn - r0;
                    k = k < 64 ? k : 64;
                    k = k < wmx - r0 ? k : wmx - r0;
                    cnt = wave_round_counts(c, r0, k);
                }
                E_.wc[w][g * 64 + lane] = cnt;
            }
            lds_barrier();
            STAMP(a, SO, 6);
            // rank base of every (wave, round) and its task index base
            for (int e = threadIdx.x; e < kWaves * rn; e += kBS) {
                const int ww = e / rn, i = e - ww * rn;
                const int r = rc + i;
                int64_t rb = pre_c[i];
                const int64_t Sr = S_l[i];
                for (int q = 0; q < ww; ++q) rb += E_.wc[q][i];
                E_.wbase[ww][i] = (int32_t)rb;
                E_.wpos[ww][i] = (r <= L) ? (int32_t)(Sr + rb) : 0;
            }
            lds_barrier();
            STAMP(a, SO, 7);
            // full rounds: every active lane takes one task; the wave's task index
            // bases for 64 rounds sit in one register (lane i: round rc + i0 + i)
            int rfull = L < bm ? L : bm;
            rfull = rfull < rc + rn ? rfull : rc + rn;
            for (int i0 = 0; rc + i0 < rfull; i0 += 64) {
                const int bases = E_.wpos[w][(i0 + lane) < kBS ? (i0 + lane) : kBS - 1];
                const int nr = (rfull - rc - i0) < 64 ? (rfull - rc - i0) : 64;
                int i = 0;
                for (; i + 3 < nr; i += 4) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const bool act = c > rc + i0 + i + u;
                        const uint64_t m = __ballot(act);
                        const int base = __builtin_amdgcn_readlane(bases, i + u);
                        if (act) out[base + popc_lt(m)] = s;
                    }
                }
                for (; i < nr; ++i) {
                    const bool act = c > rc + i0 + i;
                    const uint64_t m = __ballot(act);
                    const int base = __builtin_amdgcn_readlane(bases, i);
                    if (act) out[base + popc_lt(m)] = s;
                }
            }
            STAMP(a, SO, 8);
            // round L (partial: ranks < p) and round L+1 (ranks for the next queue)
            if (L >= rc && L < rc + rn) {
                const int iL = L - rc;
                const bool act = c > L;
                const uint64_t m = __ballot(act);
                rankL = (int64_t)E_.wbase[w][iL] + popc_lt(m);
                if (act && rankL < p) out[E_.wpos[w][iL] + popc_lt(m)] = s;
            }
            if (L + 1 >= rc && L + 1 < rc + rn) {
                const int i1 = L + 1 - rc;
                exL1 = (int64_t)E_.wbase[w][i1] + popc_lt(__ballot(c > L + 1));
            }
            lds_barrier();
        }
        STAMP(a, SO, 4);
        if (c > 0) {
            int64_t n_q = c < L ? c : L;
            if (c > L && rankL < p) n_q += 1;
            int64_t np = -1;
            if (c > L) {
                if (rankL >= p) np = rankL - p;
                else if (c > L + 1) np = (AL - p) + exL1;
                // the one position of rank p in A_L knows the next queue's length
                if (rankL == p) a.hout->new_qlen = (AL - p) + exL1;
            }
            if (a.deque) {
                deque_finish(a, pos, s, c, L, n_q, c > L && rankL < p, np);
                STAMP(a, SO, 15);
                return;
            }
            // the worker's next {free, queued}: one 8-byte store
            a.free_out[s] = make_int2(raw - (int32_t)n_q, np >= 0 ? 1 : 0);
            if (np >= 0) {
                a.queue_out[np] = s;
                a.qfree_out[np] = raw - (int32_t)n_q;
                a.qhb_out[np] = hbp;
            }
        }
        STAMPR(a, SO, 14);
        STAMP(a, SO, 15);
        return;
    }
    if (bid < a.nbq + a.nbf) {
        // ---- orphan compaction, ascending sequence
        const int b = bid - a.nbq;
        const uint32_t flags = a.ofl[(size_t)b * kBS + threadIdx.x];
        const int64_t off = a.fpre[b];
        uint32_t tot;
        const uint32_t ex = block_excl_scan_u32((uint32_t)__popc(flags), (uint32_t *)misc, tot);
        int64_t o = off + ex;
        const int64_t base = (int64_t)b * kFTile + (int64_t)threadIdx.x * kFItems;
#pragma unroll
        for (int j = 0; j < kFItems; ++j)
            if (flags & (1u << j)) a.orphans[o++] = base + j;
        STAMP(a, SO, 15);
        return;
    }
    // ---- evicted compaction, ascending slot
    const int b = bid - a.nbq - a.nbf;
    const int s = b * kBS + threadIdx.x;
    const uint32_t e = (s < a.W) & ((a.st[min(s, a.W > 0 ? a.W - 1 : 0)] & kStEvicted) != 0);
    const int64_t off = a.wpre[b];
    uint32_t tot;
    const uint32_t ex = block_excl_scan_u32(e, (uint32_t *)misc, tot);
    if (e) a.evicted[off + ex] = s;
    STAMP(a, SO, 15);
}

// ------------------------------------------------------------ k_emit2
// k_emit for the fused path (no k_plan launch).  Every k_scan queue block added
// its round counts into its group's row (atomics, groups of 2^gshift blocks), so
// a queue block reads the group rows (totals A(r), the prefix of earlier groups)
// and the rows of the earlier blocks of its own group: about 2 sqrt(nbq) rows
// instead of the whole nbq x R table.  One block barrier: per-thread partials ->
// barrier; then every wave works alone: S(r) and the fill level L by a wave
// scan, the task index base of each round in one register (lane i: round 64k +
// i) from the round prefix plus the earlier segments' counts that k_scan stored
// per 64-position segment, and the emission.  F / W roles as k_emit's.
// NCH: 64-round chunks kept per lane (rounds 0 .. L+1): 1 for R = 32, 3 up to R = 128.

template <int NCH, typename T>
__device__ __forceinline__ T chunk_pick(const T (&v)[NCH], int k) {
    T x = v[0];
#pragma unroll
    for (int i = 1; i < NCH; ++i) x = k == i ? v[i] : x;
    return x;
}

// Log workgroup of a fused one-GPU tick (f_emit): orphan flags and their compaction.
// The slot purge (k_scan's W role or the apply launch) wrote the died-registration
// bitmap and already counted O for the fill level, so nothing here is on the queue
// role's path.  One workgroup per 2048-entry log tile (many small workgroups spread the
// log reads over the CUs beside the queue blocks): two coalesced 16-byte log loads per
// thread (entry t*2048 + 1024k + 4*tid + j) issued with the bitmap's copy into LDS, the
// died bits from LDS, and the tile's orphans written in ascending order into the
// tile's own segment of the orphan buffer (orphans[t*2048 + i], i < fcnt[t]).  No
// workgroup waits for another: the dense list -- the segments in tile order -- is
// gathered when it is read (k_orph_gather) and the commit walks the segments.
__device__ __forceinline__ void emit_log_tile(const TickArgs &a, int t, unsigned long long *bm) {
    __shared__ uint32_t l4[kWaves];
    const int tid = threadIdx.x;
    const int64_t nlog = a.head_in;
    const int64_t tbase = (int64_t)t * kFTile;
    const int64_t last4 = nlog > 0 ? ((nlog - 1) & ~(int64_t)3) : 0;
    // the previous tick's orphans of this tile (its commit, folded into this tick: an idle
    // tick after an idle tick) leave the log here; their slots died then, so this tick
    // flags none of them whichever value its loads below see
    const uint32_t pc = (a.cm_fold && t < a.cm_tiles) ? a.fcnt[t] : 0u;
    // ... their first 256 log positions loaded with the tile (a tile's previous segment
    // holds ~100 at configs[2]), so the clear below is a store, not a load round
    const int64_t oq0 = (a.cm_fold && t < a.cm_tiles) ? a.orphans[tbase + tid] : 0;
    int32_t v[2][4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int64_t i = tbase + k * 1024 + 4 * tid;
        const int4 x = *reinterpret_cast<const int4 *>(a.log_slot + (i < last4 ? i : last4));
        v[k][0] = i < nlog ? x.x : -1;
        v[k][1] = i + 1 < nlog ? x.y : -1;
        v[k][2] = i + 2 < nlog ? x.z : -1;
        v[k][3] = i + 3 < nlog ? x.w : -1;
    }
    // the died bitmap (<= kLdsBitmapSlots bits) into LDS: <= 4 int4 per thread, all in flight
    {
        const int n4 = ((((a.W + 63) >> 6) + 1) >> 1);
        const uint4 *src = reinterpret_cast<const uint4 *>(a.dmask);
        uint4 t4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = tid + k * kBS;
            t4[k] = src[i < n4 ? i : n4 - 1];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = tid + k * kBS;
            if (i < n4) reinterpret_cast<uint4 *>(bm)[i] = t4[k];
        }
    }
    lds_barrier();
    // (read before the block scans' barriers; the segment is rewritten after them)
    if ((uint32_t)tid < pc) a.log_slot[oq0] = -1;
    for (uint32_t i = tid + kBS; i < pc; i += kBS) a.log_slot[a.orphans[tbase + i]] = -1;
    int64_t o = tbase;  // this tile's segment; entry order within the tile: k, then tid, then j
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        uint32_t m = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int sj = v[k][q], sc = sj < 0 ? 0 : sj;
            m |= (sj >= 0 && ((bm[sc >> 6] >> (sc & 63)) & 1ull)) ? (1u << q) : 0u;
        }
        const int64_t e0 = tbase + k * 1024 + 4 * tid;
        m = drop_completed(a, drop_stale<4>(a, m, v[k], e0), v[k], e0);
        uint32_t tot;
        const uint32_t ex = block_excl_scan_u32((uint32_t)__popc(m), l4, tot);
        int64_t oo = o + ex;
        if (!(kDiagNow & 16))
            for (uint32_t mm = m; mm; mm &= mm - 1) wt_store(a.orphans + oo++, (int64_t)(e0 + __builtin_ctz(mm)));
        o += tot;
    }
    if (tid == 0) a.fcnt[t] = (uint32_t)(o - tbase);
}

// Sum over aligned groups of G adjacent lanes (G = 2 .. 32), every lane of a group left
// with its total: DPP quad permutes (lanes ^1, ^2), then the 8- and 16-lane mirrors (each
// pairs a lane with the other half of its group once the halves are uniform), then the
// 32-lane swizzle
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    if (G >= 4) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    if (G >= 8) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    if (G >= 16) x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);  // row_mirror
    if (G >= 32) x += (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);  // lane ^ 16 within 32
    return x;
}

// XCD-aware order of the queue blocks: workgroups are dealt round-robin over the 8
// XCDs (placement is a speed matter only), so logical block L = (i mod 8) * n/8 + i / 8
// puts consecutive LRU segments on one XCD.  Each round's task range of block L ends
// where block L + 1's begins, in the middle of a 128-byte line: written from one XCD's
// L2 the two halves merge there, from two XCDs each L2 writes back a partial line.
// A bijection on [0, n) for any n.
__device__ __forceinline__ int xcd_block(int i, int n) {
    const int x = i & 7, y = i >> 3, q = n >> 3, r = n & 7;
    return x * q + (x < r ? x : r) + y;
}

// k_emit2's compaction roles (workgroup rel of them): one wave per tile (a k_scan block's
// 2048 log entries or 256 slots), four tiles per workgroup -- a quarter of the blocks of one
// thread per flag byte / slot, so they do not queue behind the queue role.  PLAN: the
// tiles' offsets from k_plan2's scans, else summed here.  NW waves (tiles) per workgroup.
template <bool PLAN, int PEEL, int NW = kWaves>
__device__ __forceinline__ void emit2_compact(const TickArgs &a, int rel, int nbf4, uint32_t (*red)[4]) {
    const int lane = lane_id(), w = wave_id();
    const bool frole = rel < nbf4;
    const int t0 = NW * (frole ? rel : rel - nbf4);
    const int t = t0 + w;
    const int ntile = frole ? a.nbf : a.nbw;
    const uint32_t *cnt = frole ? a.fcnt : a.wcnt;
    int64_t off;  // entries of the tiles before t
    if constexpr (PLAN) {
        const int64_t *pre = frole ? a.fpre : a.wpre;
        off = pre[t < ntile ? t : ntile - 1];
    } else {
        // the workgroup sums the counts of the tiles before its own (PEEL x 256 tiles with
        // every load in flight; a tail loop past that)
        unsigned long long tot, pre;
        peeled_sum<PEEL, 64 * NW>(cnt, t0, t0, tot, pre);
        const uint32_t ws = wave_sum_u32((uint32_t)pre);
        if (lane == 0) red[w][0] = ws;
        lds_barrier();
        off = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) off += red[q][0];
        for (int q = 0; q < w; ++q) off += t0 + q < ntile ? cnt[t0 + q] : 0u;
    }
    if (t >= ntile) return;
    if (frole) {
        // orphans, ascending sequence: lane l holds flag bytes 4l .. 4l+3 of tile t
        // (k_scan's thread j flagged entries t*2048 + 8j .. +8)
        const uint32_t f4 = reinterpret_cast<const uint32_t *>(a.ofl + (size_t)t * kBS)[lane];
        const uint32_t n = (uint32_t)__popc(f4);
        int64_t o = off + (int64_t)(wave_incl_scan_u32(n) - n);
        const int64_t base = (int64_t)t * kFTile + (int64_t)lane * 4 * kFItems;
        for (uint32_t m = f4; m; m &= m - 1) wt_store(a.orphans + o++, (int64_t)(base + __builtin_ctz(m)));
    } else {
        // evicted slots, ascending: lane l holds slots t*256 + 4l .. +4
        const int s0 = t * kBS + 4 * lane;
        const int wl = a.W > 0 ? a.W - 1 : 0;
        uint32_t e = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint8_t sv = a.st[min(s0 + q, wl)];
            e |= ((s0 + q < a.W) && (sv & kStEvicted)) ? (1u << q) : 0u;
        }
        const uint32_t n = (uint32_t)__popc(e);
        int64_t o = off + (int64_t)(wave_incl_scan_u32(n) - n);
        for (uint32_t m = e; m; m &= m - 1) wt_store(a.evicted + o++, (int32_t)(s0 + __builtin_ctz(m)));
    }
}

// k_emit2's queue role from the per-round prefixes on: the fill level, the partial round
// L and the next state of every position (finish), the full rounds' stores.  Lane i holds
// round 64 k + i of chunk k: prev = the tasks of round r taken by earlier blocks, totv =
// A(r), segc = by the earlier waves of this block.
template <int NCH, bool BIG, bool PLAN>
__device__ __forceinline__ void emit2_rounds(const TickArgs &a, int SO, int b, int64_t pos, int32_t raw0, int s0,
                                             double hb0, const uint32_t (&prev)[NCH], const uint32_t (&totv)[NCH],
                                             const uint32_t (&segc)[NCH], int maxc, int64_t O, int64_t nev,
                                             int64_t cap) {
    const int lane = lane_id();
    const int R = a.R;
    const int rlim = maxc < R ? maxc : R;
    // ---- per wave: S(r) (lane i of chunk k: round 64 k + i), capacity, fill level L
    int64_t Sv[NCH], S1v[NCH];
    {
        int64_t carry = 0;
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            const int r = 64 * k + lane;
            const uint32_t v = r < rlim ? totv[k] : 0u;
            const uint32_t incl = wave_incl_scan_u32(v);
            S1v[k] = carry + (int64_t)incl;  // S(r + 1)
            Sv[k] = S1v[k] - (int64_t)v;     // S(r)
            carry += (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        // fused: sum_r A(r) over r < max c = sum of c (PLAN: k_plan's capacity)
        if constexpr (!PLAN) cap = carry;
    }
    if (maxc > R) cap = INT64_MAX;  // capacity beyond the table: only S(R) is known
    const int64_t N = (a.redist ? O : 0) + a.T;  // purge-only ticks report orphans, dispatch none
    const int64_t N_eff = N < cap ? N : cap;
    int L = 0;
#pragma unroll
    for (int k = 0; k < NCH; ++k) L += __popcll(__ballot(64 * k + lane < rlim && S1v[k] <= N_eff));
    const int Lc = L >> 6, Ll = L & 63;
    const int64_t S_L = (int64_t)__builtin_amdgcn_readlane((int)chunk_pick<NCH>(Sv, Lc), Ll);
    int status = 0;
    if (maxc > R && L >= R - 1) status = 1;   // rows beyond the table needed: rerun wider
    else if (a.head_in + N_eff > a.log_cap) status = 2;  // never write past the in-flight log (N_eff exact once R is)
    const int64_t pL = N_eff - S_L;
    const int64_t AL =
        (L < maxc && L < rlim) ? (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)chunk_pick<NCH>(totv, Lc), Ll) : 0;
    if (b == 0 && threadIdx.x == 0) {
        a.hout->O = O;
        a.hout->n_evicted = nev;
        a.hout->cap_total = cap;
        a.hout->maxc = maxc;
        a.hout->L = L;
        a.hout->status = status;
        a.hout->N_eff = status ? 0 : N_eff;
        a.hout->p = pL;
        a.hout->AL = AL;
        if (AL == 0) a.hout->new_qlen = 0;
    }
    if (status) return;
    // ---- rank base (in A_r) and task index base of this wave's segment, per round
    const int32_t raw = pos < a.Qlog ? raw0 : INT32_MIN;
    const int s = s0;
    // free <= 0 still takes one task; deque mode: c_arr holds the token's c itself
    const int c = raw != INT32_MIN ? (a.deque ? raw : (raw > 1 ? raw : 1)) : 0;
    if (a.rb_slot && pos < a.Qlog) compact_out(a, pos, s, c, L);
    int32_t rbv[NCH], basev[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
        const int r = 64 * k + lane;
        rbv[k] = (int32_t)((r < rlim ? prev[k] : 0u) + segc[k]);
        basev[k] = (int32_t)Sv[k] + rbv[k];  // valid for r <= rlim
    }
    STAMP(a, SO, 2);
    int32_t *const out = a.log_slot + a.head_in;
    // ---- round L (partial: ranks < pL) and round L + 1 (ranks for the next queue)
    const int L1 = L + 1, L1c = L1 >> 6, L1l = L1 & 63;
    const int rbL = __builtin_amdgcn_readlane(chunk_pick<NCH>(rbv, Lc), Ll);
    const int rbL1 = __builtin_amdgcn_readlane(chunk_pick<NCH>(rbv, L1c), L1l);
    const uint64_t mL = __ballot(c > L);
    const int64_t rankL = (int64_t)rbL + popc_lt(mL);
    const int64_t exL1 = (int64_t)rbL1 + popc_lt(__ballot(c > L1));
    // round L's stores and the position's next state (free count, next queue)
    auto finish = [&]() {
        if (!(kDiagNow & 32) && c > L && rankL < pL) wt_store(out + S_L + rankL, s);
        if (c > 0) {
            int64_t n_q = c < L ? c : L;
            if (c > L && rankL < pL) n_q += 1;
            int64_t np = -1;
            if (c > L) {
                if (rankL >= pL) np = rankL - pL;
                else if (c > L1) np = (AL - pL) + exL1;
                // the one position of rank pL in A_L knows the next queue's length
                if (rankL == pL) a.hout->new_qlen = (AL - pL) + exL1;
            }
            if (a.deque) {
                deque_finish(a, pos, s, c, L, n_q, c > L && rankL < pL, np);
                return;
            }
            // the worker's next {free, queued}: one 8-byte store, only for the workers served
            // this tick -- the slot role already wrote {free, 1} for every queued one (a
            // streaming tick serves 64 K of 1 M queued workers: 64 K scattered stores, not 1 M)
            // (free_pre: the purge wrote {raw - c, 0}, this position's value when c <= L)
            if (!(kDiagNow & 4) && (a.free_pre ? c > L : (n_q != 0 || np < 0))) {
                wt_store(a.free_out + s, make_int2(raw - (int32_t)n_q, np >= 0 ? 1 : 0));
            }

            if (!(kDiagNow & 8) && np >= 0) {
                wt_store(a.queue_out + np, s);
                wt_store(a.qfree_out + np, raw - (int32_t)n_q);
                wt_store(a.qhb_out + np, hb0);
            }
        }
    };
    // heartbeat loop: issued before the full rounds, so the scattered free-count stores
    // are under way while the rounds store (configs[2]: 10.30 -> 10.16 us per tick; as
    // agent-scope stores no change, as nontemporal stores +0.7 us)
    const bool fin_first = !a.deque;
    if (fin_first) finish();
    // ---- full rounds r < min(L, max c of the wave): every active lane takes one task
    const int wmx = (int)wave_max_u32((uint32_t)c);
    const int rfull = L < wmx ? L : wmx;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
        const int r1 = rfull - 64 * k < 64 ? rfull - 64 * k : 64;
        int i = 0;
        // fused (small) ticks branch-free: every lane stores, inactive ones into the
        // trash words (an `if (act)` store costs an exec save / branch / restore per
        // round; configs[2]: tick 13.4 -> 13.0 us).  (A buffer store predicated by its
        // range check instead -- inactive lanes given an out-of-range offset -- took
        // the 19 rounds from 2.0 K to 3.6 K cycles: rejected.)
        // (one 1 KB trash row per block, 1024 rows: no line shared between blocks)
        int32_t *const tr = a.trash + (size_t)(blockIdx.x & (kTrashRows - 1)) * kBS + threadIdx.x;
        if (kDiagNow & 2) i = r1;
        if (!BIG && a.arena32) {
            // every buffer lies in the context's arena (< 4 GB): 32-bit byte offsets from
            // one scalar base -- a select and a saddr store per round, no 64-bit math
            char *const ab = a.arena;
            const uint32_t oo = (uint32_t)((char *)out - ab), to = (uint32_t)((char *)tr - ab);
            const uint32_t bo = oo + 4u * (uint32_t)basev[k];  // byte offset of each round's first store
            for (; i + 3 < r1; i += 4) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int r = 64 * k + i + u;
                    const bool act = c > r;
                    const uint64_t m = __ballot(act);
                    const uint32_t po = __builtin_amdgcn_readlane(bo, i + u) + 4u * popc_lt(m);
                    const uint32_t off = to + ((po - to) & (0u - (uint32_t)act));
                    if (!(kDiagNow & 1)) wt_store((int32_t *)(ab + off), s);
                    else if (act) wt_store((int32_t *)(ab + po), s);
                }
            }
        }
        for (; i + 3 < r1; i += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int r = 64 * k + i + u;
                const bool act = c > r;
                const uint64_t m = __ballot(act);
                const int base = __builtin_amdgcn_readlane(basev[k], i + u);
                if constexpr (!BIG) {
                    // select by mask arithmetic: a ?: on the pointers becomes an exec-masked block
                    const uint64_t pa = (uint64_t)(out + (base + (int)popc_lt(m))), pt = (uint64_t)tr;
                    wt_store((int32_t *)(pt ^ ((pa ^ pt) & (0ull - (uint64_t)act))), s);
                } else {
                    // large tables (after k_plan): thousands of blocks, where the trash
                    // stores cost more than the branches they save (16M x 1M: +1.2 us)
                    if (act) wt_store(out + base + popc_lt(m), s);
                }
            }
        }
        for (; i < r1; ++i) {
            const int r = 64 * k + i;
            const bool act = c > r;
            const uint64_t m = __ballot(act);
            const int base = __builtin_amdgcn_readlane(basev[k], i);
            if (act) wt_store(out + base + popc_lt(m), s);
        }
    }
    STAMP(a, SO, 3);
    if (!fin_first) finish();
}

// PM 1 (PLAN): large tables (round table beyond the fused limit, R <= 128) -- the same
// emission with this block's prefixes and the totals from k_plan2.  PM 2 (gp): large tables
// without k_plan2 -- the prefixes from the group rows as the fused path (PM 0) reads them,
// the rest as PLAN's (segment counts in LDS, compaction offsets from fpre / wpre).
template <int MODE, int PM, int NCH>
__global__ __launch_bounds__(kBS) void k_emit2(TickArgs a_) {
    constexpr bool PLAN = PM == 1;  // prefixes and totals from k_plan2
    constexpr bool BIG = PM != 0;   // large tables
    STAMP_TOP(a_, a_.nbw + a_.nbf + a_.nbq + (a_.slots_in_scan ? a_.nbw : 0));
    prefetch_args(a_);
    const TickArgs a = specialise<MODE>(a_);
    __shared__ uint32_t gpre[kBS], gtot[kBS];  // per-thread partials of (round, part)
    __shared__ uint32_t red[kWaves][4];
    __shared__ uint32_t pre_c[kRFused];        // PLAN: this block's prefix of round r
    __shared__ uint32_t tot_f[kRFused];        // PLAN: A(r)
    const int SO = a.nbw + a.nbf + a.nbq + (a.slots_in_scan ? a.nbw : 0);
    STAMP(a, SO, 0);
    const int lane = lane_id(), w = wave_id();
    // the other parity's group rows, for the next launch's k_scan atomics
    for (int i = (int)blockIdx.x * kBS + (int)threadIdx.x; i < a.zero_words; i += (int)gridDim.x * kBS)
        a.grp_zero[i] = 0;
    // grid: queue blocks, then compaction blocks -- log workgroups: 4 tiles each (f_emit:
    // one tile each), then the slot tiles 4 per workgroup
    const int nbf4 = a.f_emit ? a.nbf : (a.nbf + 3) >> 2;
    int bid = blockIdx.x;  // the role index
    if (a.cmix) {
        // (fb_set_path("cmix")) the compaction rows of 8 workgroups (one per XCD) spread
        // evenly among the queue rows, so they run beside the queue blocks' load latency
        // instead of after them; a queue block keeps its XCD (role index mod 8 = blockIdx mod 8)
        const int nc = nbf4 + ((a.nbw + 3) >> 2);
        const int x = (int)blockIdx.x & 7, y = (int)blockIdx.x >> 3;
        const int nqr = (a.nbq + 7) >> 3, ncr = (nc + 7) >> 3, nr = nqr + ncr;
        const int cr = (int)((int64_t)y * ncr / nr);
        if ((int)((int64_t)(y + 1) * ncr / nr) > cr) {
            if (8 * cr + x >= nc) return;
            bid = a.nbq + 8 * cr + x;
        } else {
            if (8 * (y - cr) + x >= a.nbq) return;
            bid = 8 * (y - cr) + x;
        }
    }
    const int qb0 = 0, cb0 = a.nbq;
    if (bid >= qb0 && bid < qb0 + a.nbq) {
        const int b = xcd_block(bid - qb0, a.nbq);
        const int64_t pos = (int64_t)b * kBS + threadIdx.x;
        const int R = a.R;       // 32, 64 or 128
        // ---- every load in flight at once (clamped indices, no branches)
        const int64_t pq = pos < a.Qlog ? pos : (a.Qlog > 0 ? a.Qlog - 1 : 0);
        int32_t raw0;
        double hb0;
        if (a.cq_direct) {
            // idle tick: the committed position's free count and heartbeat, k_scan's liveness
            // test repeated (the same bytes k_scan would have copied into c_arr / c_hb)
            const double hq = a.qhb_in[pq];
            const int32_t fq = a.qfree_in[pq];
            hb0 = hq;
            raw0 = ((a.now - hq) > a.tte) ? INT32_MIN : fq;
        } else {
            raw0 = a.c_arr[pq];
            hb0 = a.c_hb[pq];
        }
        const int s0 = a.E == 0 ? a.queue_in[pq] : lq_slot(a, pq);
        // counts of c > r in the earlier segments of this block: lane i, round 64 k + i
        // (all three earlier segments loaded unconditionally, clamped, then masked:
        // a loop bounded by the wave id would issue one load and wait per segment)
        uint32_t segc[NCH];
        // large tables only: on the fused (configs[2]) path the histogram sits on the
        // critical path between the loads and the barrier (11.13 -> 11.45 us per tick)
        constexpr bool kSegLds = BIG;
        __shared__ uint32_t shist[kWaves][kRFused + 1];
        __shared__ uint32_t sseg[kWaves][kRFused];
        if constexpr (kSegLds)
        {
            // ... counted here from this block's own c values: per wave a histogram of
            // min(c, R) in LDS (k_scan's scheme), count(c > r) = 64 - its prefix; summed
            // over the earlier waves after the block barrier below
            const int32_t rw = pos < a.Qlog ? raw0 : INT32_MIN;
            const int cc = rw != INT32_MIN ? (a.deque ? rw : (rw > 1 ? rw : 1)) : 0;
            uint32_t *h = shist[w];
            for (int i = lane; i <= R; i += 64) h[i] = 0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            atomicAdd(&h[cc < R ? cc : R], 1u);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            uint32_t carry = 0;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int r = 64 * k + lane;
                const uint32_t P = carry + wave_incl_scan_u32(r < R ? h[r] : 0u);
                if (r < R) sseg[w][r] = 64u - P;
                carry = (uint32_t)__builtin_amdgcn_readlane((int)P, 63);
            }
        }
        uint32_t sv[NCH][kWaves - 1];
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            segc[k] = 0;
#pragma unroll
            for (int q = 0; q < kWaves - 1; ++q) {
                const int r = min(64 * k + lane, R - 1);
                sv[k][q] = kSegLds ? 0u : a.segcnt[(size_t)(4 * b + q) * R + r];
            }
        }
        int64_t O, nev, cap = 0;
        int maxc;
        uint32_t fo = 0, wo = 0, mo = 0;
        uint32_t prev[NCH], totv[NCH];  // lane i of chunk k, round 64 k + i: this block's prefix, A(r)
        if constexpr (PLAN) {
            STAMPW(a, SO, 5);
            // this block's prefix and the total of every round, scanned by k_plan
            const int64_t *Ar = a.repl ? a.A_rep + (size_t)(b >> a.gshift) * kRFused : a.A;
            const DevTotals *Pr = a.repl ? a.P_rep + (b >> a.gshift) : a.P;
            if ((int)threadIdx.x < R) {
                pre_c[threadIdx.x] = (uint32_t)a.qpre[(size_t)b * R + threadIdx.x];
                tot_f[threadIdx.x] = (uint32_t)Ar[threadIdx.x];
            }
            O = Pr->O;
            nev = Pr->n_evicted;
            cap = Pr->cap_total;
            maxc = Pr->maxc;
#pragma unroll
            for (int k = 0; k < NCH; ++k)
#pragma unroll
                for (int q = 0; q < kWaves - 1; ++q) segc[k] += (q < w && 64 * k + lane < R) ? sv[k][q] : 0u;
            STAMPW(a, SO, 6);
            lds_barrier();
#pragma unroll
            for (int k = 0; k < NCH; ++k) {
                const int rr = min(64 * k + lane, kRFused - 1);
                prev[k] = pre_c[rr];
                totv[k] = tot_f[rr];
            }
        } else {
            // thread t: round r = t / P, part p = t mod P of the rows (a round's parts in
            // adjacent lanes: summed by DPP, no LDS pass over them)
            const int P = kBS / R, r = (int)threadIdx.x / P, p = (int)threadIdx.x & (P - 1);
            const int g = b >> a.gshift, gsz = 1 << a.gshift, ng = a.ngrp;
            const int gs = a.gstride;
            uint32_t pre = 0, tot = 0;
            const int nb_in = b - g * gsz;
            // gp, R = 32, groups of <= 64 blocks: the <= 64 group rows and <= 63 earlier block
            // rows in one load round, 8 + 8 per thread, a column per lane (c = t & 31) and a
            // row class per half wave (rows q + 8 j, q = t >> 5): every wave load covers two
            // whole rows; the 8 row classes of a column are summed by a cross-half shuffle and
            // the 4 waves' partials after the block barrier
            const bool trp = PM == 2 && NCH == 1 && gsz <= 64;
            if (trp) {
                const int cc = (int)threadIdx.x & 31, q = (int)threadIdx.x >> 5;
                uint32_t vg[8], vb[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int i = q + 8 * j;
                    vg[j] = a.grp[min(i, ng - 1) * gs + cc];
                    vb[j] = a.qcnt[(size_t)(g * gsz + min(i, nb_in > 0 ? nb_in - 1 : 0)) * R + cc];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int i = q + 8 * j;
                    tot += i < ng ? vg[j] : 0u;
                    pre += (i < g ? vg[j] : 0u) + (i < nb_in ? vb[j] : 0u);
                }
                pre += (uint32_t)__shfl_xor((int)pre, 32);
                tot += (uint32_t)__shfl_xor((int)tot, 32);
            } else {
            // group rows g' = p + P j: totals, and the prefix of the groups before g
            for (int j0 = 0; j0 * P < ng; j0 += kGrpLd) {
                uint32_t v[kGrpLd];
#pragma unroll
                for (int j = 0; j < kGrpLd; ++j) v[j] = a.grp[min(p + P * (j0 + j), ng - 1) * gs + r];
#pragma unroll
                for (int j = 0; j < kGrpLd; ++j) {
                    const int gg = p + P * (j0 + j);
                    tot += gg < ng ? v[j] : 0u;
                    pre += gg < g ? v[j] : 0u;
                }
            }
            // rows of the blocks of group g before b
            for (int j0 = 0; j0 * P < nb_in; j0 += kGrpLd) {
                uint32_t v[kGrpLd];
#pragma unroll
                for (int j = 0; j < kGrpLd; ++j) {
                    const int jj = min(p + P * (j0 + j), nb_in - 1);
                    v[j] = a.qcnt[(size_t)(g * gsz + jj) * R + r];
                }
#pragma unroll
                for (int j = 0; j < kGrpLd; ++j) pre += p + P * (j0 + j) < nb_in ? v[j] : 0u;
            }
            }
            // max c, orphans and evictions: columns R, R + 1, R + 2 of the group rows
            // (ngrp <= 64: wave 0 holds them)
            const int gi = min((int)threadIdx.x, ng - 1) * gs + R;
            const uint32_t mg = a.grp[gi], og = a.grp[gi + 1], eg = a.grp[gi + 2];
            if (trp) {
                if (lane < 32) {
                    gpre[w * 32 + lane] = pre;
                    gtot[w * 32 + lane] = tot;
                }
            } else {
                if (P == 8) {
                    pre = group_sum<8>(pre);
                    tot = group_sum<8>(tot);
                } else if (P == 4) {
                    pre = group_sum<4>(pre);
                    tot = group_sum<4>(tot);
                } else {
                    pre = group_sum<2>(pre);
                    tot = group_sum<2>(tot);
                }
                if (p == 0) {
                    gpre[r] = pre;
                    gtot[r] = tot;
                }
            }
#pragma unroll
            for (int k = 0; k < NCH; ++k)
#pragma unroll
                for (int q = 0; q < kWaves - 1; ++q) segc[k] += (q < w && 64 * k + lane < R) ? sv[k][q] : 0u;
            STAMP(a, SO, 9);
            const bool gin = (int)threadIdx.x < ng;
            mo = gin ? mg : 0u;
            fo = gin ? og : 0u;
            wo = gin ? eg : 0u;
            fo = wave_sum_u32(fo);
            wo = wave_sum_u32(wo);
            mo = wave_max_u32(mo);
            if (lane == 0) {
                red[w][0] = fo;
                red[w][1] = wo;
                red[w][3] = mo;
            }
            lds_barrier();
            O = (int64_t)red[0][0] + red[1][0] + red[2][0] + red[3][0];
            nev = (int64_t)red[0][1] + red[1][1] + red[2][1] + red[3][1];
            maxc = (int)max(max(red[0][3], red[1][3]), max(red[2][3], red[3][3]));
            // this lane's rounds
#pragma unroll
            for (int k = 0; k < NCH; ++k) {
                const int rr = 64 * k + lane;
                if (trp) {
                    const int rc = rr < 32 ? rr : 31;
                    prev[k] = rr < R ? gpre[rc] + gpre[32 + rc] + gpre[64 + rc] + gpre[96 + rc] : 0u;
                    totv[k] = rr < R ? gtot[rc] + gtot[32 + rc] + gtot[64 + rc] + gtot[96 + rc] : 0u;
                } else {
                    prev[k] = rr < R ? gpre[rr] : 0u;
                    totv[k] = rr < R ? gtot[rr] : 0u;
                }
            }
        }
        STAMP(a, SO, 1);
#ifdef FAASBAL_STAMPS
        if constexpr (PM == 2) {
            // (diagnostic, fb_set_path("gpcheck", 1): k_plan2 ran too; this block's round-0
            // prefix beside k_plan2's)
            if (a.gpcheck && threadIdx.x == 0) {
                unsigned long long *row = a.dbg + (size_t)(3 * (a.nbw + a.nbf + a.nbq) + 1024 + b) * 16;
                row[0] = (unsigned long long)b + 1;
                row[1] = prev[0];
                row[2] = (uint32_t)a.qpre[(size_t)b * R];
                row[3] = (unsigned long long)(b >> a.gshift);
                row[4] = totv[0];
                row[5] = (unsigned long long)a.gshift;
            }
        }
#endif
#pragma unroll
        for (int k = 0; k < NCH && kSegLds; ++k) {
            const int r = min(64 * k + lane, kRFused - 1);
            uint32_t sc = 0;
#pragma unroll
            for (int q = 0; q < kWaves - 1; ++q) sc += (q < w && 64 * k + lane < R) ? sseg[q][r] : 0u;
            segc[k] = sc;
        }
        emit2_rounds<NCH, BIG, PLAN>(a, SO, b, pos, raw0, s0, hb0, prev, totv, segc, maxc, O, nev, cap);
        STAMP(a, SO, 15);
        return;
    }
    // ---- compaction roles (emit2_compact)
    if (a.f_emit && bid >= cb0 && bid < cb0 + a.nbf) {  // f_emit: one log workgroup per tile
        extern __shared__ __attribute__((aligned(16))) unsigned long long dynbm[];
        STAMP(a, SO, 0);
        emit_log_tile(a, bid - cb0, dynbm);
        STAMP(a, SO, 15);
        return;
    }
    STAMP(a, SO, 0);
    if (a.f_emit) emit2_compact<PLAN, PM == 2 ? 16 : kPeel>(a, bid - cb0 - a.nbf, 0, red);
    else emit2_compact<PLAN, PM == 2 ? 16 : kPeel>(a, bid - cb0, nbf4, red);
    STAMP(a, SO, 15);
}

// ------------------------------------------------------------ k_emit_win
// The level-0 emission of a window tick (see win_elem): one workgroup per 1024-element
// chunk, taken in ticket order (back chunks first), thread t holding elements
// i0 + 256 j + t (j < 4) in registers from their classification to their stores.  A
// chunk's counts travel by decoupled look-back along two chains -- the back chunks
// (live backs) and the front / window chunks (live elements, those with c > 1) -- as
// 8-byte granules {state, live, c > 1, max c} written by one agent-scope store each
// (MI355X_MICROARCH.md, visibility: a granule needs no further ordering) and read with
// agent-scope loads, 64 predecessors per wave load.  Live element k < N = O + T takes
// task k (k_emit2's round 0); live backs are appended at the tail in order, then the
// served workers with c > 1 in order (A_0[p:] ++ [served, c > 1]); the element of rank
// N - 1 reports where the next window starts and how long it is.  A tick that is not a
// window tick after all -- an unserved front, or no unserved live element inside the
// scanned prefix -- is flagged (win_ovf) and the host reruns it on the general path.
// the tick cannot finish as a window tick: the host's flag and the device word an eager
// commit reads (device memory; the host-mapped results are too slow to read per block)
__device__ __forceinline__ void win_fail(const TickArgs &a) {
    a.hout->win_ovf = 1;
    a.cw[0] = a.cw_tag;
}
// The window report: the next window [head, head + len) of the queue buffer and the true
// queue length, into the host results and the commit word.  The device checks them with
// fb_tick_wait's bounds (check_lengths) before an eager commit can read them: outside, the
// commit word's failure tag keeps the eager commit from committing, and the host refuses
// the tick with FB_EHIP -- device and host agree the tick is not committed.  (fault_qlen >=
// 0: a test overrides both lengths here, fb_set_path("fault_qlen").)
__device__ __forceinline__ void win_report(const TickArgs &a, int64_t head, int64_t len, int64_t qlen) {
    if (a.fault_qlen >= 0) len = qlen = a.fault_qlen;
    a.hout->win_head = head;
    a.hout->new_qlen = len;
    a.hout->win_qlen = qlen;
    a.cw[1] = head;
    a.cw[2] = len;
    if (head < a.wq_off || len < 0 || head > a.wq_cap || len > a.wq_cap - head || qlen < 0 || qlen > len ||
        qlen > a.q_cap)
        a.cw[0] = a.cw_tag;
}
constexpr uint64_t kGrA = (1ull << 22) - 1, kGrM = (1ull << 18) - 1;
constexpr int kWinStampRow = 8192;  // k_emit_win's diagnostic stamp rows (after k_ev_apply_ll's)
__device__ __forceinline__ uint64_t gr_pack(uint32_t st, uint32_t lv, uint32_t g1, uint32_t mx) {
    return ((uint64_t)st << 62) | ((uint64_t)(mx < kGrM ? mx : kGrM) << 44) | ((uint64_t)g1 << 22) | (uint64_t)lv;
}
__device__ __forceinline__ uint64_t gr_load(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gr_store(unsigned long long *p, uint64_t v) {
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wave 0: publish this chunk's aggregate at chain index i, resolve its exclusive prefix
// from the predecessors (aggregates summed back to the first inclusive one), publish the
// inclusive value.  Returns the exclusive {live, c > 1, max c}; false if a predecessor
// never published (a bound on the wait that only a fault can reach).
__device__ __forceinline__ bool gr_lookback(unsigned long long *g, int i, uint32_t lv, uint32_t g1, uint32_t mx,
                                            uint32_t &elv, uint32_t &eg1, uint32_t &emx) {
    const int lane = lane_id();
    elv = eg1 = emx = 0;
    if (i == 0) {
        if (lane == 0) gr_store(g, gr_pack(2, lv, g1, mx));
        return true;
    }
    if (lane == 0) gr_store(g + i, gr_pack(1, lv, g1, mx));
    int j = i - 1;  // the newest predecessor not yet summed
    for (int spin = 0; spin < (1 << 22);) {
        const int q = j - lane;
        uint64_t v = q >= 0 ? gr_load(g + q) : gr_pack(2, 0, 0, 0);
        // wait until every lane of this window has a published granule
        while (__ballot((v >> 62) == 0) && spin < (1 << 22)) {
            __builtin_amdgcn_s_sleep(1);
            ++spin;
            if ((v >> 62) == 0) v = gr_load(g + q);
        }
        if (__ballot((v >> 62) == 0)) return false;
        const uint64_t incl = __ballot((v >> 62) == 2);
        const int first = incl ? (int)__builtin_ctzll(incl) : 64;  // nearest inclusive predecessor
        const bool take = lane <= first;
        uint32_t a = take ? (uint32_t)(v & kGrA) : 0u, b = take ? (uint32_t)((v >> 22) & kGrA) : 0u;
        uint32_t m = take ? (uint32_t)((v >> 44) & kGrM) : 0u;
        elv += wave_sum_u32(a);
        eg1 += wave_sum_u32(b);
        emx = max(emx, wave_max_u32(m));
        if (first < 64) {
            if (lane == 0) gr_store(g + i, gr_pack(2, elv + lv, eg1 + g1, max(emx, mx)));
            return true;
        }
        j -= 64;
    }
    return false;
}
// The inclusive value of chain index i once published (wave 0); false on the wait bound.
__device__ __forceinline__ bool gr_wait_incl(const unsigned long long *g, int i, uint32_t &lv, uint32_t &mx) {
    uint64_t v = gr_load(g + i);
    for (int spin = 0; (v >> 62) != 2; ++spin) {
        if (spin >= (1 << 22)) return false;
        __builtin_amdgcn_s_sleep(1);
        v = gr_load(g + i);
    }
    lv = (uint32_t)(v & kGrA);
    mx = (uint32_t)((v >> 44) & kGrM);
    return true;
}

__global__ __launch_bounds__(kBS) void k_emit_win(TickArgs a) {
    prefetch_args(a);
    __shared__ uint32_t red[kWaves][4];
    __shared__ uint32_t wt[4][kWaves][2];
    __shared__ uint32_t xs[8];
    const int tid = threadIdx.x, lane = lane_id(), w = wave_id();
    STAMP(a, kWinStampRow, 0);
    // chunk = ticket (predecessors already run), or the workgroup index when every chunk is
    // resident at once (win_direct: no atomic round before the element loads)
    if (!a.win_direct && tid == 0) xs[0] = atomicAdd(a.wticket, 1u);
    // the orphan partials of the log workgroups and the purge's eviction / queued partials
    const uint32_t op = tid < a.n_lpart ? a.lpart[tid] : 0u;
    const uint32_t e0 = tid < 64 ? a.wpart[(size_t)tid * 32] : 0u, q0 = tid < 64 ? a.wpart[(size_t)tid * 32 + 1] : 0u;
    if (!a.win_direct) lds_barrier();
    const int ch = a.win_direct ? (int)blockIdx.x : (int)xs[0];
    int64_t i0, i1;
    const int reg = win_region(a, ch, i0, i1);
    // ---- this chunk's elements: classification (loads in flight), in-chunk ranks
    WinEl e[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = i0 + j * kBS + tid;
        e[j] = win_elem(a, reg, i, i < i1);
    }
    uint64_t ml[4], mg[4];
    uint32_t cmx = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = win_c(e[j].raw);
        ml[j] = __ballot(c > 0);
        mg[j] = __ballot(c > 1);
        cmx = (uint32_t)c > cmx ? (uint32_t)c : cmx;
        if (lane == 0) {
            wt[j][w][0] = (uint32_t)__popcll(ml[j]);
            wt[j][w][1] = (uint32_t)__popcll(mg[j]);
        }
    }
    STAMP(a, kWinStampRow, 1);
    {
        const uint32_t x0 = wave_sum_u32(op), x1 = wave_sum_u32(e0), x2 = wave_sum_u32(q0), x3 = wave_max_u32(cmx);
        if (lane == 0) {
            red[w][0] = x0;
            red[w][1] = x1;
            red[w][2] = x2;
            red[w][3] = x3;
        }
    }
    lds_barrier();
    const uint32_t O = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    const uint32_t nev = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    const uint32_t nq = red[0][2] + red[1][2] + red[2][2] + red[3][2];
    const uint32_t bmx = max(max(red[0][3], red[1][3]), max(red[2][3], red[3][3]));
    uint32_t tl = 0, tg = 0;  // the chunk's live elements / those with c > 1
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int u = 0; u < kWaves; ++u) {
            tl += wt[j][u][0];
            tg += wt[j][u][1];
        }
    const int64_t N = (int64_t)O + a.T;
    const bool logfull = a.head_in + N > a.log_cap;
    const int nfw = a.nchF + a.nchW;
    const int ci = reg == 0 ? ch : ch - a.nchB;  // index in its chain
    unsigned long long *const gch = reg == 0 ? a.wlb : a.wlb + a.nchB;
    // ---- the chains (wave 0), then the totals this chunk needs
    if (w == 0) {
        uint32_t elv, eg1, emx, LB = 0, bmax = 0;
        bool ok = gr_lookback(gch, ci, reg == 0 ? tl : tl, reg == 0 ? 0u : tg, bmx, elv, eg1, emx);
        STAMP(a, kWinStampRow, 4);
        // front / window chunks append after the live backs: the back chain's total
        if (ok && reg != 0) ok = gr_wait_incl(a.wlb, a.nchB - 1, LB, bmax);
        if (lane == 0) {
            xs[1] = elv;
            xs[2] = eg1;
            xs[3] = LB;
            xs[4] = ok ? 1u : 0u;
            if (!ok) win_fail(a);
            if (ch == 0) {
                a.hout->O = O;
                a.hout->n_evicted = nev;
                a.hout->cap_total = -1;  // beyond the scanned prefix (a window tick never needs it)
                a.hout->L = 0;
                a.hout->status = logfull ? 2 : 0;
                if (logfull) win_fail(a);
                a.hout->N_eff = logfull ? 0 : N;
                a.hout->p = N;
            }
            if (ok && reg != 0) {
                const int64_t inc = (int64_t)elv + tl;  // live fronts / window up to this chunk's end
                // every front served: the last front chunk's total may not exceed N
                if (ch == a.nchB + a.nchF - 1 && inc > N) win_fail(a);
                if (ci == nfw - 1) {
                    // the first unserved live element must lie in the scanned prefix
                    if (inc <= N) win_fail(a);
                    a.hout->maxc = (int32_t)max(max(emx, bmx), bmax);
                    a.hout->AL = inc + LB;  // at least
                }
                if (ci == 0 && N == 0) {
                    win_report(a, a.wq_off, a.wq_tail + LB - a.wq_off, nq);
                    if (a.wq_tail + LB - a.wq_off > a.q_cap) win_fail(a);
                }
            }
        }
    }
    lds_barrier();
    STAMP(a, kWinStampRow, 2);
    if (!xs[4] || logfull) {
        STAMP(a, kWinStampRow, 15);
        return;
    }
    if (reg < 2) {
        // a queued slot moved to the front or the back: its committed position (read-only
        // during the tick) is tombstoned by the commit; one entry per list position
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t i = i0 + j * kBS + tid;
            if (i < i1) a.tomb[(reg == 1 ? a.E : 0) + i] = e[j].mv;
        }
    }
    const uint32_t lvx = xs[1], g1x = xs[2], LB = xs[3];
    const uint32_t blx = lvx;  // back chunks: their chain counts live backs
    if (reg != 0 && (int64_t)lvx >= N) {  // every element of the chunk stays put
        STAMP(a, kWinStampRow, 15);
        return;
    }
    uint32_t bl = 0, bg = 0;  // elements of the earlier sub-rounds / waves
    int32_t *const q = a.wq_buf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t rl = bl, rg = bg;
#pragma unroll
        for (int u = 0; u < kWaves; ++u) {
            rl += u < w ? wt[j][u][0] : 0u;
            rg += u < w ? wt[j][u][1] : 0u;
            bl += wt[j][u][0];
            bg += wt[j][u][1];
        }
        rl += (uint32_t)popc_lt(ml[j]);
        rg += (uint32_t)popc_lt(mg[j]);
        const WinEl &x = e[j];
        const int c = win_c(x.raw);
        if (c == 0) continue;
        if (reg == 0) {
            // a live back: appended in order
            const int64_t pq = a.wq_tail + blx + rl;
            if (pq < a.wq_cap) {
                q[pq] = x.s;
                a.wqf_buf[pq] = x.raw;
                a.wqh_buf[pq] = x.hb;
            } else {
                win_fail(a);
            }
            continue;
        }
        const int64_t k = (int64_t)lvx + rl;
        if (k >= N) continue;
        // served: task k, one fewer free process; c > 1 stays queued, appended after the backs
        a.log_slot[a.head_in + k] = x.s;
        a.free_out[x.s] = make_int2(x.raw - 1, c > 1 ? 1 : 0);
        const int64_t G = (int64_t)g1x + rg + (c > 1 ? 1 : 0);  // served workers with c > 1 so far
        if (c > 1) {
            const int64_t pq = a.wq_tail + LB + G - 1;
            if (pq < a.wq_cap) {
                q[pq] = x.s;
                a.wqf_buf[pq] = x.raw - 1;
                a.wqh_buf[pq] = x.hb;
            } else {
                win_fail(a);
            }
        }
        if (k == N - 1) {
            const int64_t head = reg == 2 ? i0 + j * kBS + tid + 1 : a.wq_off;
            win_report(a, head, a.wq_tail + LB + G - head, (int64_t)nq - (N - G));
            // the next window, tombstones included, must fit a general tick's position arrays
            if (a.wq_tail + LB + G - head > a.q_cap) win_fail(a);
        }
    }
    STAMP(a, kWinStampRow, 15);
}

// ------------------------------------------------------------ k_emit_shard
__device__ __forceinline__ void shard_compact(const TickArgs &a, int bid);
constexpr int kRCh = 3;  // 64-round chunks: rounds 0 .. L+1 <= 129
// Phase 2 of a sharded tick.  Every rank computes the global water-filling from
// the exchanged counts (identical on all ranks), writes the whole next LRU queue,
// and appends only its own workers' tasks to its log shard -- in ascending global
// sequence, because own tasks are placed round-major by their own rank.
// k_emit2's scheme with two rank systems: per wave and round, the global task
// index base S(r) + block prefix + earlier segments (for the sequence number)
// and the own-log base So(r) + own block prefix + own earlier segments (for the
// log position), one register per 64 rounds, read with readlane in the round
// loop; block prefixes from k_plan, segment counts from the phase-2 k_scan.
// GRP: no k_plan before this launch -- the totals and this block's prefixes per round come
// from the group rows k_scan's phase-2 blocks added (all / own counts, max c, capacity),
// plus the earlier blocks of its own group; the orphan totals from the exchange records
// and this rank's tile counts.
// XR (with GRP): no phase-2 k_scan either -- every block's counts arrived in the exchange
// as digit rows (phase 1, a.xrows), this rank's in its own rows (ocnt); each block sums the
// rows of all blocks (totals) and of the blocks before it (prefix), and counts its waves'
// rounds itself; max c and the capacity follow from the totals.
// (Large queues, a.xplan: k_emit_shard_xp below.)
template <bool GRP, bool XR>
__global__ __launch_bounds__(kBS) void k_emit_shard(TickArgs a) {
    prefetch_args(a);
    const int bid = blockIdx.x;
    const int lane = lane_id(), w = wave_id();
    const int SO = 3 * (a.nbw + a.nbf + a.nbq);  // diagnostic stamp rows (stamps builds)
    STAMP(a, SO, 0);
    if (XR) {  // the other parity's exchange records, for the next tick's phase 1
        for (int i = bid * kBS + (int)threadIdx.x; i < a.xz_words; i += (int)gridDim.x * kBS) a.xz[i] = 0ull;
    } else if (GRP) {  // the other parity's group rows, for the next launch's k_scan atomics
        for (int i = bid * kBS + (int)threadIdx.x; i < a.zero_words; i += (int)gridDim.x * kBS) a.grp_zero[i] = 0;
    }
    if (bid < a.nbq) {
        const int b = bid;
        const int R = a.R;
        const int64_t pos = (int64_t)b * kBS + threadIdx.x;
        // ---- every load in flight at once (clamped indices, no branches)
        const int64_t pq = pos < a.Qlog ? pos : (a.Qlog > 0 ? a.Qlog - 1 : 0);
        const int cq = xc_get(a, pq);
        const int sq = lq_slot(a, pq);
        const int32_t rawq = a.c_arr[pq];
        int64_t Av[kRCh], oAv[kRCh], pv[kRCh], opv[kRCh];
        int64_t O, cap;
        int maxc;
        uint32_t segc[kRCh] = {0, 0, 0}, osegc[kRCh] = {0, 0, 0};
        if (XR) {
            // ---- the block rows of every block, summed per column: tot over all blocks,
            // pre over the blocks before b.  All positions: the exchanged digit rows (xr_row
            // bytes per block); this rank's: its own count rows (R words).  Thread (load
            // column q, part j) loads the 16-byte column q of rows j, j + Pp, ... (parts the
            // fast index, Pp a power of two), 8 rows per round, both row kinds in flight
            // together; the Pp parts of a column are adjacent lanes and meet by shuffles.
            __shared__ uint32_t xcol[2][kXRowMaxBytes];  // per digit-row byte: tot / pre over the blocks
            __shared__ uint32_t ocol[2][kRFused];        // per own column: tot / pre
            __shared__ uint32_t swc[kWaves][kRFused + 1], sowc[kWaves][kRFused + 1];
            __shared__ uint32_t sred[kWaves][3];
            const int t = threadIdx.x;
            // every rank's orphans and max c (their records; world * 8 <= kBS lines), issued
            // first and consumed after the rows' loads
            const int gx = t < a.world * kXRecLines ? t : 0;
            const unsigned long long xo = a.xrec[(size_t)gx * 16], xm = a.xrec[(size_t)gx * 16 + 1];
            uint32_t orf = 0, mx = 0;
            const int xs = xr_stride(R), nq16 = xr_row(R) >> 4, Pp = xr_parts(R);
            const int nq = R >> 2, Pp2 = kBS / nq;
            const int q = t / Pp, j = t % Pp, q2 = t / Pp2, j2 = t % Pp2;
            const bool xg = a.xgrows != nullptr;  // group rows (R = kXGroupR)
            __shared__ uint32_t gsum[3][kXGroupDigits * 36], osum[3][kXGroupR];  // group tot / pre, block pre
            // (the group path's lane map: 9 + 7 digit-row and 8 + 8 own-row load columns at R = 32)
            static_assert(xg_row(kXGroupR) == 9 * 16 && xr_row(kXGroupR) == 7 * 16 && kXGroupR / 4 == 8,
                          "group-row lane map");
            static_assert(kXRowsMaxBlocks <= kXGroupBlocks * 16, "<= 16 group rows per column");
            if (xg) {
                // ---- lanes 16 i .. 16 i + 15: one 16-byte column of the <= 16 group rows or of
                // the rows of the blocks of b's group before b (lane & 15 = row); pass A the
                // digit rows (9 group + 7 block columns), pass B this rank's rows (8 + 8)
                const int g0 = b / kXGroupBlocks, ng = (a.nbq + kXGroupBlocks - 1) / kXGroupBlocks;
                const int ri = t & 15;
                const bool ga = t < 144, gb = t < 128;
                const int ca = ga ? t >> 4 : (t - 144) >> 4, cb = gb ? t >> 4 : (t - 128) >> 4;
                const int blk = g0 * kXGroupBlocks + ri;
                const bool va = ga ? ri < ng : blk < b, vb = gb ? ri < ng : blk < b;
                // both loads unconditional (clamped rows, one pointer per lane) and masked after:
                // a guarded load would become a branch with its own wait
                const int rg = min(ri, ng - 1), rb = min(blk, a.nbq - 1);
                const uint4 *pa_ = ga ? reinterpret_cast<const uint4 *>(a.xgrows) + (size_t)rg * 9 + ca
                                      : reinterpret_cast<const uint4 *>(a.xrows) + (size_t)rb * 7 + ca;
                const uint4 *pb_ = gb ? reinterpret_cast<const uint4 *>(a.ogrp) + (size_t)rg * 8 + cb
                                      : reinterpret_cast<const uint4 *>(a.ocnt) + (size_t)rb * 8 + cb;
                uint4 v = *pa_, vo = *pb_;
                if (!va) v = make_uint4(0, 0, 0, 0);
                if (!vb) vo = make_uint4(0, 0, 0, 0);
                const bool pa = ga ? ri < g0 : va, pb = gb ? ri < g0 : vb;  // in the prefix
                uint32_t gt[8], gp[8], ot4[4], op4[4];
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w}, o4[4] = {vo.x, vo.y, vo.z, vo.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t e = w4[u] & 0x00ff00ffu, o = (w4[u] >> 8) & 0x00ff00ffu;
                    gt[2 * u] = group_sum<16>(e);
                    gt[2 * u + 1] = group_sum<16>(o);
                    gp[2 * u] = group_sum<16>(pa ? e : 0u);
                    gp[2 * u + 1] = group_sum<16>(pa ? o : 0u);
                    ot4[u] = group_sum<16>(o4[u]);
                    op4[u] = group_sum<16>(pb ? o4[u] : 0u);
                }
                if (ri == 0) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int by = ca * 16 + (u >> 1) * 4 + (u & 1);
                        if (ga) {
                            gsum[0][by] = gt[u] & 0xffffu;
                            gsum[0][by + 2] = gt[u] >> 16;
                            gsum[1][by] = gp[u] & 0xffffu;
                            gsum[1][by + 2] = gp[u] >> 16;
                        } else {
                            gsum[2][by] = gp[u] & 0xffffu;
                            gsum[2][by + 2] = gp[u] >> 16;
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (gb) {
                            osum[0][cb * 4 + u] = ot4[u];
                            osum[1][cb * 4 + u] = op4[u];
                        } else {
                            osum[2][cb * 4 + u] = op4[u];
                        }
                    }
                }
            }
            // packed: bytes two to a word (16-bit halves; <= kXRowsMaxBlocks x 240 each)
            uint32_t tp[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            uint32_t ot[4] = {0, 0, 0, 0}, op[4] = {0, 0, 0, 0};
            if (!xg) {
                const uint4 *src = reinterpret_cast<const uint4 *>(a.xrows) + (q < nq16 ? q : 0);
                const uint4 *ow = reinterpret_cast<const uint4 *>(a.ocnt) + q2;
                const bool xon = q < nq16;
                for (int r0 = 0; r0 < a.nbq; r0 += 8 * Pp) {  // (rounds of 8 rows per thread)
                    uint4 v[8], vo[8];
                    // unconditional loads of clamped rows, masked after (no branch per load)
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int bb = r0 + j + k * Pp, b2 = (r0 / Pp) * Pp2 + j2 + k * Pp2;
                        v[k] = src[(size_t)min(bb, a.nbq - 1) * nq16];
                        vo[k] = ow[(size_t)min(b2, a.nbq - 1) * nq];
                    }
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int bb = r0 + j + k * Pp, b2 = (r0 / Pp) * Pp2 + j2 + k * Pp2;
                        if (!(xon && bb < a.nbq)) v[k] = make_uint4(0, 0, 0, 0);
                        if (b2 >= a.nbq) vo[k] = make_uint4(0, 0, 0, 0);
                    }
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const bool in = r0 + j + k * Pp < b;
                        const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const uint32_t e = w4[u] & 0x00ff00ffu, o = (w4[u] >> 8) & 0x00ff00ffu;
                            tp[2 * u] += e;
                            tp[2 * u + 1] += o;
                            pp[2 * u] += in ? e : 0u;
                            pp[2 * u + 1] += in ? o : 0u;
                        }
                        const bool in2 = (r0 / Pp) * Pp2 + j2 + k * Pp2 < b;
                        const uint32_t o4[4] = {vo[k].x, vo[k].y, vo[k].z, vo[k].w};
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            ot[u] += o4[u];
                            op[u] += in2 ? o4[u] : 0u;
                        }
                    }
                }
            }
            STAMPW(a, SO, 1);
            // this wave's rounds (all / own lanes) from histograms of min(c, R): the in-block
            // bases of the later waves
            {
                const int cw_ = pos < a.Qlog ? cq : 0;
                const int ocw = (cw_ > 0 && sq >= 0 && own_slot(a, sq) >= 0) ? cw_ : 0;
                uint32_t *ha = swc[w], *ho = sowc[w];
                for (int i = lane; i <= R; i += 64) {
                    ha[i] = 0;
                    ho[i] = 0;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                atomicAdd(&ha[cw_ < R ? cw_ : R], 1u);
                atomicAdd(&ho[ocw < R ? ocw : R], 1u);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                uint32_t ca = 0, co = 0;
#pragma unroll
                for (int k = 0; k < 2; ++k) {  // count(c > r) = 64 - #(lanes with min(c, R) <= r)
                    const int r = 64 * k + lane;
                    const uint32_t hv = r < R ? ha[r] : 0u, hw = r < R ? ho[r] : 0u;
                    const uint32_t Pa = ca + wave_incl_scan_u32(hv), Po = co + wave_incl_scan_u32(hw);
                    ca = (uint32_t)__builtin_amdgcn_readlane((int)Pa, 63);
                    co = (uint32_t)__builtin_amdgcn_readlane((int)Po, 63);
                    __builtin_amdgcn_wave_barrier();
                    if (r < R) {
                        ha[r] = 64u - Pa;
                        ho[r] = 64u - Po;
                    }
                }
            }
            // the parts of each column: adjacent lanes (Pp = Pp2, 8 / 16 / 32), DPP sums
            auto psum = [&](auto g) {
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    tp[u] = group_sum<decltype(g)::value>(tp[u]);
                    pp[u] = group_sum<decltype(g)::value>(pp[u]);
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    ot[u] = group_sum<decltype(g)::value>(ot[u]);
                    op[u] = group_sum<decltype(g)::value>(op[u]);
                }
            };
            if (xg) {
            } else if (Pp == 32) psum(std::integral_constant<int, 32>{});
            else if (Pp == 16) psum(std::integral_constant<int, 16>{});
            else psum(std::integral_constant<int, 8>{});
            if (!xg && j == 0 && q < nq16) {
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    // packed word u: int4 word u / 2, even (u even) / odd bytes; halves 2 bytes apart
                    const int by = q * 16 + (u >> 1) * 4 + (u & 1);
                    xcol[0][by] = tp[u] & 0xffffu;
                    xcol[0][by + 2] = tp[u] >> 16;
                    xcol[1][by] = pp[u] & 0xffffu;
                    xcol[1][by + 2] = pp[u] >> 16;
                }
            }
            if (!xg && j2 == 0) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    ocol[0][q2 * 4 + u] = ot[u];
                    ocol[1][q2 * 4 + u] = op[u];
                }
            }
            orf = t < a.world * kXRecLines ? (uint32_t)xo : 0u;
            mx = t < a.world * kXRecLines ? (uint32_t)xm : 0u;
            orf = wave_sum_u32(orf);
            mx = wave_max_u32(mx);
            if (lane == 0) {
                sred[w][1] = orf;
                sred[w][2] = mx;
            }
            __syncthreads();
            STAMP(a, SO, 4);
            // column r's totals and prefixes: from the digits (group rows: 4 digits, block rows 3)
            auto tot_all = [&](int r) -> uint32_t {
                return xg ? gsum[0][r] + (gsum[0][xs + r] << 4) + (gsum[0][2 * xs + r] << 8) + (gsum[0][3 * xs + r] << 12)
                          : xcol[0][r] + (xcol[0][xs + r] << 4) + (xcol[0][2 * xs + r] << 8);
            };
            auto pre_all = [&](int r) -> uint32_t {
                return xg ? gsum[1][r] + (gsum[1][xs + r] << 4) + (gsum[1][2 * xs + r] << 8) + (gsum[1][3 * xs + r] << 12) +
                                gsum[2][r] + (gsum[2][xs + r] << 4) + (gsum[2][2 * xs + r] << 8)
                          : xcol[1][r] + (xcol[1][xs + r] << 4) + (xcol[1][2 * xs + r] << 8);
            };
            // the capacity sum_r<R A(r) = sum of c when max c <= R
            uint32_t cp = t < R ? tot_all(t) : 0u;
            cp = wave_sum_u32(cp);
            if (lane == 0) sred[w][0] = cp;
#pragma unroll
            for (int k = 0; k < kRCh; ++k) {
                const int rr = min(64 * k + lane, R - 1);
                const bool kin = 64 * k < R;  // (chunks past the table: lanes never read)
                Av[k] = kin ? tot_all(rr) : 0u;
                pv[k] = kin ? pre_all(rr) : 0u;
                oAv[k] = !kin ? 0u : (xg ? osum[0][rr] : ocol[0][rr]);
                opv[k] = !kin ? 0u : (xg ? osum[1][rr] + osum[2][rr] : ocol[1][rr]);
                uint32_t sc = 0, osc = 0;
#pragma unroll
                for (int qq = 0; qq < kWaves - 1; ++qq) {
                    const bool in = qq < w && 64 * k + lane < R;
                    sc += in ? swc[qq][rr] : 0u;
                    osc += in ? sowc[qq][rr] : 0u;
                }
                segc[k] = sc;
                osegc[k] = osc;
            }
            __syncthreads();
            // max c (clamped to the byte) from every rank's records
            maxc = (int)max(max(sred[0][2], sred[1][2]), max(sred[2][2], sred[3][2]));
            cap = (int64_t)sred[0][0] + sred[1][0] + sred[2][0] + sred[3][0];
            O = (int64_t)sred[0][1] + sred[1][1] + sred[2][1] + sred[3][1];
            STAMP(a, SO, 5);
        } else if (GRP) {
            // 2R columns (round r of all positions, then of this rank's), tpc consecutive
            // threads per column: each column's total over the group rows and this block's
            // prefix (earlier groups + earlier blocks of its group), every tpc-th row per thread
            __shared__ uint32_t sT[2][kRFused], sP[2][kRFused];
            __shared__ uint32_t smx[kWaves], scap[kWaves], sorf[kWaves];
            int tpc = 1;
            while (tpc * 4 * R <= kBS) tpc *= 2;  // R = 32: 4 threads per column
            const int col = (int)threadIdx.x / tpc, j = (int)threadIdx.x % tpc;
            const int tab = col >= R ? 1 : 0, r = col - tab * R;
            const int g0 = b >> a.gshift, b0 = g0 << a.gshift;
            uint32_t tot = 0, pre = 0;
            if (col < 2 * R) {
                const uint32_t *cg = a.grp + col;
#pragma unroll 4
                for (int g = j; g < a.ngrp; g += tpc) {
                    const uint32_t v = cg[(size_t)g * a.gstride];
                    tot += v;
                    pre += g < g0 ? v : 0u;
                }
                const uint32_t *bc = (tab ? a.ocnt : a.qcnt) + r;
#pragma unroll 4
                for (int bb = b0 + j; bb < b; bb += tpc) pre += bc[(size_t)bb * R];
            }
            if (tpc == 4) {  // the column's tpc threads are adjacent lanes: DPP sums
                tot = group_sum<4>(tot);
                pre = group_sum<4>(pre);
            } else if (tpc == 2) {
                tot = group_sum<2>(tot);
                pre = group_sum<2>(pre);
            }
            if (col < 2 * R && j == 0) {
                sT[tab][r] = tot;
                sP[tab][r] = pre;
            }
            // max c and capacity (threads < ngrp), every rank's orphans (the exchange records)
            // (capacity < Q x 128 and orphans < the 2^31-entry log: 32-bit sums)
            uint32_t mx = 0, cp = 0, orf = 0;
            if ((int)threadIdx.x < a.ngrp) {
                const uint32_t *row = a.grp + (size_t)threadIdx.x * a.gstride;
                mx = row[2 * R];
                cp = row[2 * R + 1];
            }
            for (int g = threadIdx.x; g < a.world * kXRecLines; g += kBS) orf += (uint32_t)a.xrec[(size_t)g * 16];
            mx = wave_max_u32(mx);
            cp = wave_sum_u32(cp);
            orf = wave_sum_u32(orf);
            if (lane == 0) {
                smx[w] = mx;
                scap[w] = cp;
                sorf[w] = orf;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kRCh; ++k) {
                const int rr = min(64 * k + lane, R - 1);
                Av[k] = sT[0][rr];
                oAv[k] = sT[1][rr];
                pv[k] = sP[0][rr];
                opv[k] = sP[1][rr];
            }
            maxc = (int)max(max(smx[0], smx[1]), max(smx[2], smx[3]));
            cap = (int64_t)scap[0] + scap[1] + scap[2] + scap[3];
            O = (int64_t)sorf[0] + sorf[1] + sorf[2] + sorf[3];
        } else {
#pragma unroll
            for (int k = 0; k < kRCh; ++k) {
                const int r = min(64 * k + lane, R - 1);
                Av[k] = a.A[r];
                oAv[k] = a.oA[r];
                pv[k] = a.qpre[(size_t)b * R + r];
                opv[k] = a.opre[(size_t)b * R + r];
            }
            O = a.P->O;
            cap = a.P->cap_total;
            maxc = a.P->maxc;
        }
        if (!XR) {
            uint32_t sv[kRCh][kWaves - 1], osv[kRCh][kWaves - 1];
#pragma unroll
            for (int k = 0; k < kRCh; ++k)
#pragma unroll
                for (int q = 0; q < kWaves - 1; ++q) {
                    const size_t si = (size_t)(4 * b + q) * R + min(64 * k + lane, R - 1);
                    sv[k][q] = a.segcnt[si];
                    osv[k][q] = a.osegcnt[si];
                }
#pragma unroll
            for (int k = 0; k < kRCh; ++k)
#pragma unroll
                for (int q = 0; q < kWaves - 1; ++q) {
                    const bool in = q < w && 64 * k + lane < R;
                    segc[k] += in ? sv[k][q] : 0u;
                    osegc[k] += in ? osv[k][q] : 0u;
                }
        }
        const int rlim = maxc < R ? maxc : R;
        if (maxc > R) cap = INT64_MAX;
        const int64_t N = (a.redist ? O : 0) + a.T;  // purge-only ticks report orphans, dispatch none
        const int64_t N_eff = N < cap ? N : cap;
        // ---- per wave: S(r) and So(r) (lane i of chunk k: round 64 k + i), fill level L
        int64_t Sv[kRCh], Sov[kRCh];
        int L = 0;
        {
            int64_t carry = 0, ocarry = 0;
#pragma unroll
            for (int k = 0; k < kRCh; ++k) {
                const int r = 64 * k + lane;
                const uint32_t v = r < rlim ? (uint32_t)Av[k] : 0u;
                const uint32_t ov = r < rlim ? (uint32_t)oAv[k] : 0u;
                const uint32_t incl = wave_incl_scan_u32(v);
                const uint32_t oincl = wave_incl_scan_u32(ov);
                const int64_t S1 = carry + (int64_t)incl;  // S(r + 1)
                Sv[k] = S1 - (int64_t)v;                   // S(r)
                Sov[k] = ocarry + (int64_t)oincl - (int64_t)ov;
                L += __popcll(__ballot(r < rlim && S1 <= N_eff));
                carry += (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                ocarry += (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)oincl, 63);
            }
        }
        const int Lc = L >> 6, Ll = L & 63;
        const int64_t S_L = (int64_t)__builtin_amdgcn_readlane((int)(Lc == 0 ? Sv[0] : (Lc == 1 ? Sv[1] : Sv[2])), Ll);
        const int64_t oSL =
            (int64_t)__builtin_amdgcn_readlane((int)(Lc == 0 ? Sov[0] : (Lc == 1 ? Sov[1] : Sov[2])), Ll);
        // status 1 (the table is too narrow: every rank sees it, all relaunch) before
        // status 2 (this rank's log shard is full), whose N_eff is exact only once the
        // table is wide enough -- so the ranks never split between a relaunch and a failure
        int status = 0;
        if (maxc > R && L >= R - 1) status = 1;
        else if (a.head_local + N_eff > a.log_cap) status = 2;
        const int64_t p = N_eff - S_L;
        // |A_L| from this wave's totals (lane L & 63 of chunk L >> 6)
        const int64_t ALv = (int64_t)__builtin_amdgcn_readlane((int)(Lc == 0 ? Av[0] : (Lc == 1 ? Av[1] : Av[2])), Ll);
        const int64_t AL = (L < maxc && L < rlim) ? ALv : 0;
        int64_t O_loc = 0, n_ev = 0;
        if (GRP && b == 0) {
            // this rank's orphans and evictions (its phase-1 tile counts) for the host
            __shared__ uint32_t sfo[kWaves], sev[kWaves];
            uint32_t fo = 0, ev = 0;
            for (int t = threadIdx.x; t < a.nbf; t += kBS) fo += a.fcnt[t];
            for (int t = threadIdx.x; t < a.nbw; t += kBS) ev += a.wcnt[t];
            fo = wave_sum_u32(fo);
            ev = wave_sum_u32(ev);
            if (lane == 0) {
                sfo[w] = fo;
                sev[w] = ev;
            }
            __syncthreads();
            O_loc = (int64_t)sfo[0] + sfo[1] + sfo[2] + sfo[3];
            n_ev = (int64_t)sev[0] + sev[1] + sev[2] + sev[3];
        }
        if (b == 0 && threadIdx.x == 0) {
            a.hout->O = O;
            a.hout->O_local = GRP ? O_loc : a.P->O_local;
            a.hout->n_evicted = GRP ? n_ev : a.P->n_evicted;
            a.hout->cap_total = cap;
            a.hout->maxc = maxc;
            a.hout->L = L;
            a.hout->status = status;
            a.hout->N_eff = status ? 0 : N_eff;
            a.hout->p = p;
            a.hout->AL = AL;
            if (!status && AL == 0) {
                a.hout->new_qlen = 0;
                a.hout->n_local = oSL;  // every worker saturated: all own capacity used
            }
        }
        STAMP(a, SO, 6);
        if (status) return;
        const int c = pos < a.Qlog ? cq : 0;
        const int s = sq;
        const int ls = s >= 0 ? own_slot(a, s) : -1;
        const bool own = c > 0 && ls >= 0;
        const int oc = own ? c : 0;
        // rank bases in A_r (global and own) and the task / own-log index bases per round
        int32_t rbv[kRCh], orbv[kRCh], basev[kRCh], obasev[kRCh];
#pragma unroll
        for (int k = 0; k < kRCh; ++k) {
            const int r = 64 * k + lane;
            rbv[k] = (int32_t)((r < rlim ? pv[k] : 0) + segc[k]);
            orbv[k] = (int32_t)((r < rlim ? opv[k] : 0) + osegc[k]);
            basev[k] = (int32_t)Sv[k] + rbv[k];
            obasev[k] = (int32_t)Sov[k] + orbv[k];
        }
        int32_t *const lslot = a.log_slot + a.head_local;
        uint32_t *const lseq = a.lseq_out + a.head_local;
        const uint32_t hin = (uint32_t)a.head_in;
        // ---- full rounds r < min(L, max own c of the wave): own lanes append their task
        // (assign_all: every lane's task into the whole-tick array, rounds < min(L, max c))
        int32_t *const aall = a.assign_all;
        const int owmx = (int)wave_max_u32((uint32_t)(aall ? c : oc));
        const int rfull = L < owmx ? L : owmx;
        // (32-bit byte offsets from the arena base when it spans < 4 GB: a saddr store per
        // array, as k_emit2's rounds; four rounds per step)
        char *const ab = a.arena;
        const uint32_t so = (uint32_t)((char *)lslot - ab), qo = (uint32_t)((char *)lseq - ab);
#pragma unroll
        for (int k = 0; k < kRCh; ++k) {
            const int r1 = rfull - 64 * k < 64 ? rfull - 64 * k : 64;
            int i = 0;
            if (a.arena32) {
                for (; i + 3 < r1; i += 4) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int r = 64 * k + i + u;
                        const uint64_t m = __ballot(c > r);
                        const uint64_t om = __ballot(oc > r);
                        const uint32_t base = (uint32_t)__builtin_amdgcn_readlane(basev[k], i + u);
                        const uint32_t obase = (uint32_t)__builtin_amdgcn_readlane(obasev[k], i + u);
                        if (oc > r) {
                            const uint32_t lp4 = 4u * (obase + popc_lt(om));
                            *reinterpret_cast<int32_t *>(ab + (so + lp4)) = s;
                            *reinterpret_cast<uint32_t *>(ab + (qo + lp4)) = hin + base + popc_lt(m);
                        }
                        if (aall && c > r) aall[base + popc_lt(m)] = s;
                    }
                }
            }
            for (; i < r1; ++i) {
                const int r = 64 * k + i;
                const uint64_t m = __ballot(c > r);
                const uint64_t om = __ballot(oc > r);
                const int base = __builtin_amdgcn_readlane(basev[k], i);
                const int obase = __builtin_amdgcn_readlane(obasev[k], i);
                if (oc > r) {
                    const int lp = obase + popc_lt(om);
                    lslot[lp] = s;
                    lseq[lp] = hin + (uint32_t)(base + popc_lt(m));
                }
                if (aall && c > r) aall[base + popc_lt(m)] = s;
            }
        }
        // ---- round L (partial: ranks < p) and round L + 1 (ranks for the next queue)
        const int L1 = L + 1, L1c = L1 >> 6, L1l = L1 & 63;
        const int rbL = __builtin_amdgcn_readlane(Lc == 0 ? rbv[0] : (Lc == 1 ? rbv[1] : rbv[2]), Ll);
        const int orbL = __builtin_amdgcn_readlane(Lc == 0 ? orbv[0] : (Lc == 1 ? orbv[1] : orbv[2]), Ll);
        const int rbL1 = __builtin_amdgcn_readlane(L1c == 0 ? rbv[0] : (L1c == 1 ? rbv[1] : rbv[2]), L1l);
        const uint64_t mL = __ballot(c > L);
        const uint64_t omL = __ballot(oc > L);
        const int64_t rankL = (int64_t)rbL + popc_lt(mL);
        const int64_t orankL = (int64_t)orbL + popc_lt(omL);
        if (oc > L && rankL < p) {
            const int64_t lp = oSL + orankL;
            lslot[lp] = s;
            lseq[lp] = hin + (uint32_t)(S_L + rankL);
        }
        if (aall && c > L && rankL < p) aall[S_L + rankL] = s;
        const int64_t exL1 = (int64_t)rbL1 + popc_lt(__ballot(c > L1));
        if (c > 0) {
            int64_t n_q = c < L ? c : L;
            if (c > L && rankL < p) n_q += 1;
            int64_t np = -1;
            if (c > L) {
                if (rankL >= p) np = rankL - p;
                else if (c > L1) np = (AL - p) + exL1;
                if (rankL == p) {
                    // first position of round L left without a task: both queue and own-log lengths
                    a.hout->new_qlen = (AL - p) + exL1;
                    a.hout->n_local = oSL + orankL;
                }
            }
            // the owned worker's next {free, queued} in one 8-byte store (the purge wrote {., 0})
            if (own) a.free_out[ls] = make_int2(rawq - (int32_t)n_q, np >= 0 ? 1 : 0);
            if (np >= 0) a.queue_out[np] = s;  // the next queue is replicated on every rank
        }
        STAMP(a, SO, 15);
        return;
    }
    shard_compact(a, bid);
}

// k_emit_shard for xplan ticks (R = kXGroupR, > kXRowsMaxBlocks queue blocks), NSB queue
// blocks per workgroup: every sub-block's loads in one round, the fill level once per
// workgroup, then each sub-block's in-block ranks, emission and next state in turn.  At
// configs[3] the 3 547 blocks of one position per thread made about two generations of
// resident workgroups of ~7 us of dependent phases each (profiles/r05a_stamps_*); NSB = 2
// makes one.
template <int NSB>
__global__ __launch_bounds__(kBS) void k_emit_shard_xp(TickArgs a) {
    prefetch_args(a);
    constexpr int R = kXGroupR;
    static_assert(R < 64, "one 64-round chunk");
    const int t = threadIdx.x, lane = lane_id(), w = wave_id();
    const int nqw = (a.nbq + NSB - 1) / NSB;
    // the compaction workgroups first in the grid (a.xcfirst): they are short, and behind the
    // queue workgroups -- more than fit on the device at once -- they started only as the first
    // queue workgroups left, ~10 us in, and ended the kernel (profiles/r06bb_stamps_shard_*)
    const int ncw = (int)gridDim.x - nqw;
    const int bid = !a.xcfirst ? (int)blockIdx.x
                               : ((int)blockIdx.x < ncw ? nqw + (int)blockIdx.x : (int)blockIdx.x - ncw);
    const int SO = 3 * (a.nbw + a.nbf + a.nbq);  // diagnostic stamp rows (stamps builds)
    STAMP(a, SO, 0);
    // the other parity's exchange records, for the next tick's phase 1
    for (int i = bid * kBS + t; i < a.xz_words; i += (int)gridDim.x * kBS) a.xz[i] = 0ull;
    if (bid >= nqw) {
        shard_compact(a, a.nbq + (bid - nqw));
        return;
    }
    __shared__ uint32_t swc[NSB][kWaves][R + 1], sowc[NSB][kWaves][R + 1];
    __shared__ uint32_t xred[kWaves][2], sfo[kWaves], sev[kWaves];
    const int rr = min(lane, R - 1);
    // ---- every load in flight at once: NSB positions per thread, their blocks' prefix rows
    // (k_xscan: chunk-local + the chunk's), the totals and every rank's records
    int cq[NSB], sq[NSB];
    int32_t rq[NSB];
    uint32_t pre[NSB], opre[NSB];
    // xself (<= 64 chunks): k_xscan left the chunks' raw totals; this workgroup sums them
    // itself -- column col = t & 63 of the 2R, chunks part + 4 i (part = t >> 6), 16 loads in
    // flight per thread -- into its chunks' prefixes and the totals (no ticket, no serial
    // last workgroup in k_xscan)
    __shared__ uint32_t cps[3][4][2 * R];
    const int nch = (a.nbq + kXsBlocks - 1) / kXsBlocks;
    const int ch0 = min(bid * NSB, a.nbq - 1) / kXsBlocks, ch1 = min(bid * NSB + NSB - 1, a.nbq - 1) / kXsBlocks;
    uint32_t xt = 0, xp0 = 0, xp1 = 0;
    if (a.xself) {
        const int col = t & (2 * R - 1), part = t >> 6;
        uint32_t x[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = a.xct[(size_t)min(part + 4 * i, nch - 1) * 2 * R + col];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int k = part + 4 * i;
            xt += k < nch ? x[i] : 0u;
            xp0 += k < ch0 ? x[i] : 0u;
            xp1 += k < ch1 ? x[i] : 0u;
        }
        cps[0][part][col] = xt;
        cps[1][part][col] = xp0;
        cps[2][part][col] = xp1;
    }
#pragma unroll
    for (int j = 0; j < NSB; ++j) {
        const int b = min(bid * NSB + j, a.nbq - 1), ch = b / kXsBlocks;
        const int64_t pos = (int64_t)(bid * NSB + j) * kBS + t;
        const int64_t pq = pos < a.Qlog ? pos : (a.Qlog > 0 ? a.Qlog - 1 : 0);
        cq[j] = xc_get(a, pq);
        sq[j] = lq_slot(a, pq);
        rq[j] = a.c_arr[pq];
        pre[j] = a.xpre[(size_t)b * 2 * R + rr] + (a.xself ? 0u : a.xct[(size_t)ch * 2 * R + rr]);
        opre[j] = a.xpre[(size_t)b * 2 * R + R + rr] + (a.xself ? 0u : a.xct[(size_t)ch * 2 * R + R + rr]);
    }
    uint32_t A0 = a.xself ? 0u : a.xA[rr], oA0 = a.xself ? 0u : a.xA[R + rr];
    const bool rin = t < a.world * kXRecLines;
    const int gx = rin ? t : 0;
    const unsigned long long xo = a.xrec[(size_t)gx * 16], xm = a.xrec[(size_t)gx * 16 + 1];
#pragma unroll
    for (int j = 0; j < NSB; ++j)
        if ((int64_t)(bid * NSB + j) * kBS + t >= a.Qlog) cq[j] = 0;
    {
        const uint32_t orf = wave_sum_u32(rin ? (uint32_t)xo : 0u), mxr = wave_max_u32(rin ? (uint32_t)xm : 0u);
        if (lane == 0) {
            xred[w][0] = orf;
            xred[w][1] = mxr;
        }
    }
    STAMPW(a, SO, 1);
    // ---- per sub-block and wave: counts of c > r (all / own lanes) from histograms of
    // min(c, R) -- the in-block bases of the later waves
#pragma unroll
    for (int j = 0; j < NSB; ++j) {
        const int c = cq[j];
        const int oc = (c > 0 && own_slot(a, sq[j]) >= 0) ? c : 0;
        uint32_t *ha = swc[j][w], *ho = sowc[j][w];
        for (int i = lane; i <= R; i += 64) {
            ha[i] = 0;
            ho[i] = 0;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        atomicAdd(&ha[c < R ? c : R], 1u);
        atomicAdd(&ho[oc < R ? oc : R], 1u);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const uint32_t hv = lane < R ? ha[lane] : 0u, hw = lane < R ? ho[lane] : 0u;
        const uint32_t Pa = wave_incl_scan_u32(hv), Po = wave_incl_scan_u32(hw);
        __builtin_amdgcn_wave_barrier();
        if (lane < R) {
            ha[lane] = 64u - Pa;  // count(c > r) = 64 - #(lanes with min(c, R) <= r)
            ho[lane] = 64u - Po;
        }
    }
    int64_t O_loc = 0, n_ev = 0;
    if (bid == 0) {
        // this rank's orphans and evictions (its phase-1 tile counts) for the host
        uint32_t fo = 0, ev = 0;
        for (int i = t; i < a.nbf; i += kBS) fo += a.fcnt[i];
        for (int i = t; i < a.nbw; i += kBS) ev += a.wcnt[i];
        fo = wave_sum_u32(fo);
        ev = wave_sum_u32(ev);
        if (lane == 0) {
            sfo[w] = fo;
            sev[w] = ev;
        }
    }
    __syncthreads();
    if (bid == 0) {
        O_loc = (int64_t)sfo[0] + sfo[1] + sfo[2] + sfo[3];
        n_ev = (int64_t)sev[0] + sev[1] + sev[2] + sev[3];
    }
    if (a.xself) {
        A0 = cps[0][0][rr] + cps[0][1][rr] + cps[0][2][rr] + cps[0][3][rr];
        oA0 = cps[0][0][R + rr] + cps[0][1][R + rr] + cps[0][2][R + rr] + cps[0][3][R + rr];
#pragma unroll
        for (int j = 0; j < NSB; ++j) {
            const int ch = min(bid * NSB + j, a.nbq - 1) / kXsBlocks;
            const int q = ch == ch0 ? 1 : 2;
            pre[j] += cps[q][0][rr] + cps[q][1][rr] + cps[q][2][rr] + cps[q][3][rr];
            opre[j] += cps[q][0][R + rr] + cps[q][1][R + rr] + cps[q][2][R + rr] + cps[q][3][R + rr];
        }
    }
    STAMP(a, SO, 5);
    // ---- the fill level (every wave alike; lane r = round r, one chunk)
    const int64_t O = (int64_t)xred[0][0] + xred[1][0] + xred[2][0] + xred[3][0];
    const int maxc = (int)max(max(xred[0][1], xred[1][1]), max(xred[2][1], xred[3][1]));
    const int rlim = maxc < R ? maxc : R;
    int64_t cap = (int64_t)wave_sum_u32(lane < R ? A0 : 0u);  // sum of c when max c <= R
    if (maxc > R) cap = INT64_MAX;
    const int64_t N = (a.redist ? O : 0) + a.T;
    const int64_t N_eff = N < cap ? N : cap;
    const uint32_t v = lane < rlim ? A0 : 0u, ov = lane < rlim ? oA0 : 0u;
    const uint32_t incl = wave_incl_scan_u32(v), oincl = wave_incl_scan_u32(ov);
    const int32_t Sv = (int32_t)(incl - v), Sov = (int32_t)(oincl - ov);  // S(r), So(r)
    const int L = __popcll(__ballot(lane < rlim && (int64_t)incl <= N_eff));
    const int64_t S_L = (int64_t)(uint32_t)__builtin_amdgcn_readlane(Sv, L);
    const int64_t oSL = (int64_t)(uint32_t)__builtin_amdgcn_readlane(Sov, L);
    int status = 0;
    if (maxc > R && L >= R - 1) status = 1;
    else if (a.head_local + N_eff > a.log_cap) status = 2;
    const int64_t p = N_eff - S_L;
    const int64_t AL = (L < maxc && L < rlim) ? (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)A0, L) : 0;
    if (bid == 0 && t == 0) {
        a.hout->O = O;
        a.hout->O_local = O_loc;
        a.hout->n_evicted = n_ev;
        a.hout->cap_total = cap;
        a.hout->maxc = maxc;
        a.hout->L = L;
        a.hout->status = status;
        a.hout->N_eff = status ? 0 : N_eff;
        a.hout->p = p;
        a.hout->AL = AL;
        if (!status && AL == 0) {
            a.hout->new_qlen = 0;
            a.hout->n_local = oSL;  // every worker saturated: all own capacity used
        }
    }
    STAMP(a, SO, 6);
    if (status) return;
    int32_t *const lslot = a.log_slot + a.head_local;
    uint32_t *const lseq = a.lseq_out + a.head_local;
    const uint32_t hin = (uint32_t)a.head_in;
    int32_t *const aall = a.assign_all;
    char *const ab = a.arena;
    const uint32_t so = (uint32_t)((char *)lslot - ab), qo = (uint32_t)((char *)lseq - ab);
    const int L1 = L + 1;
#pragma unroll
    for (int j = 0; j < NSB; ++j) {
        if (bid * NSB + j >= a.nbq) break;  // (uniform)
        const int c = cq[j], s = sq[j];
        const int ls = s >= 0 ? own_slot(a, s) : -1;
        const bool own = c > 0 && ls >= 0;
        const int oc = own ? c : 0;
        // rank bases in A_r (global and own) and the task / own-log index bases per round
        uint32_t sc = 0, osc = 0;
#pragma unroll
        for (int qq = 0; qq < kWaves - 1; ++qq) {
            const bool in = qq < w && lane < R;
            sc += in ? swc[j][qq][rr] : 0u;
            osc += in ? sowc[j][qq][rr] : 0u;
        }
        const int32_t rbv = (int32_t)((lane < rlim ? pre[j] : 0u) + sc);
        const int32_t orbv = (int32_t)((lane < rlim ? opre[j] : 0u) + osc);
        const int32_t basev = Sv + rbv, obasev = Sov + orbv;
        // ---- full rounds r < min(L, max own c of the wave) (assign_all: max c)
        const int owmx = (int)wave_max_u32((uint32_t)(aall ? c : oc));
        const int rfull = L < owmx ? L : owmx;
        int i = 0;
        if (a.arena32) {
            for (; i + 3 < rfull; i += 4) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int r = i + u;
                    const uint64_t m = __ballot(c > r);
                    const uint64_t om = __ballot(oc > r);
                    const uint32_t base = (uint32_t)__builtin_amdgcn_readlane(basev, r);
                    const uint32_t obase = (uint32_t)__builtin_amdgcn_readlane(obasev, r);
                    if (oc > r) {
                        const uint32_t lp4 = 4u * (obase + popc_lt(om));
                        *reinterpret_cast<int32_t *>(ab + (so + lp4)) = s;
                        *reinterpret_cast<uint32_t *>(ab + (qo + lp4)) = hin + base + popc_lt(m);
                    }
                    if (aall && c > r) aall[base + popc_lt(m)] = s;
                }
            }
        }
        for (; i < rfull; ++i) {
            const uint64_t m = __ballot(c > i);
            const uint64_t om = __ballot(oc > i);
            const int base = __builtin_amdgcn_readlane(basev, i);
            const int obase = __builtin_amdgcn_readlane(obasev, i);
            if (oc > i) {
                const int lp = obase + popc_lt(om);
                lslot[lp] = s;
                lseq[lp] = hin + (uint32_t)(base + popc_lt(m));
            }
            if (aall && c > i) aall[base + popc_lt(m)] = s;
        }
        // ---- round L (partial: ranks < p) and round L + 1 (ranks for the next queue)
        const int rbL = __builtin_amdgcn_readlane(rbv, L);
        const int orbL = __builtin_amdgcn_readlane(orbv, L);
        const int rbL1 = __builtin_amdgcn_readlane(rbv, L1);
        const uint64_t mL = __ballot(c > L);
        const uint64_t omL = __ballot(oc > L);
        const int64_t rankL = (int64_t)rbL + popc_lt(mL);
        const int64_t orankL = (int64_t)orbL + popc_lt(omL);
        if (oc > L && rankL < p) {
            const int64_t lp = oSL + orankL;
            lslot[lp] = s;
            lseq[lp] = hin + (uint32_t)(S_L + rankL);
        }
        if (aall && c > L && rankL < p) aall[S_L + rankL] = s;
        const int64_t exL1 = (int64_t)rbL1 + popc_lt(__ballot(c > L1));
        if (c > 0) {
            int64_t n_q = c < L ? c : L;
            if (c > L && rankL < p) n_q += 1;
            int64_t np = -1;
            if (c > L) {
                if (rankL >= p) np = rankL - p;
                else if (c > L1) np = (AL - p) + exL1;
                if (rankL == p) {
                    // first position of round L left without a task: both queue and own-log lengths
                    a.hout->new_qlen = (AL - p) + exL1;
                    a.hout->n_local = oSL + orankL;
                }
            }
            // the owned worker's next {free, queued} in one 8-byte store (the purge wrote {., 0})
            if (own) a.free_out[ls] = make_int2(rq[j] - (int32_t)n_q, np >= 0 ? 1 : 0);
            if (np >= 0) a.queue_out[np] = s;  // the next queue is replicated on every rank
        }
    }
    STAMP(a, SO, 15);
}

// ---- compaction roles of k_emit_shard*, as in k_emit2: one wave per tile (a phase-1
// k_scan block's 2048 log entries or 256 slots), four tiles per workgroup
__device__ __forceinline__ void shard_compact(const TickArgs &a, int bid) {
    __shared__ uint32_t cred[kWaves];
    const int lane = lane_id(), w = wave_id();
    const int nbf4 = (a.nbf + 3) >> 2;
    const bool frole = bid < a.nbq + nbf4;
    const int t0 = 4 * (frole ? bid - a.nbq : bid - a.nbq - nbf4);
    const int t = t0 + w;
    const int ntile = frole ? a.nbf : a.nbw;
    // the tile's offset: k_plan's scan of the tile counts, or (no k_plan: group rows) the
    // workgroup's sum of the counts before its first tile -- every load in flight at once
    // (16 per thread up to 4 096 tiles; a wave-serial loop over them put ~t/128 dependent
    // load rounds on the kernel's last workgroups) -- plus its earlier waves' tiles
    int64_t toff = 0;
    if (!a.grp_on && !a.xrows && !a.xplan) {
        if (t < ntile) toff = (frole ? a.fpre : a.wpre)[t];
    } else {
        const uint32_t *cnt = frole ? a.fcnt : a.wcnt;
        unsigned long long tot, pre;
        peeled_sum<16>(cnt, t0 < ntile ? t0 : ntile, t0, tot, pre);
        const uint32_t ws = wave_sum_u32((uint32_t)pre);
        if (lane == 0) cred[w] = ws;
        __syncthreads();
        toff = (int64_t)cred[0] + cred[1] + cred[2] + cred[3];
        for (int q = 0; q < w; ++q) toff += t0 + q < ntile ? cnt[t0 + q] : 0u;
    }
    if (t >= ntile) return;
    auto tile_pre = [&](const uint32_t *, const int64_t *) -> int64_t { return toff; };
    if (frole) {
        // own orphans (global sequence numbers, ascending): lane l holds flag bytes
        // 4l .. 4l+3 of tile t, i.e. local entries t*2048 + 32l .. +32
        const uint32_t f4 = reinterpret_cast<const uint32_t *>(a.ofl + (size_t)t * kBS)[lane];
        const uint32_t n = (uint32_t)__popc(f4);
        int64_t o = tile_pre(a.fcnt, a.fpre) + (int64_t)(wave_incl_scan_u32(n) - n);
        const int64_t base = (int64_t)t * kFTile + (int64_t)lane * 4 * kFItems;
        for (uint32_t m = f4; m; m &= m - 1) a.orphans[o++] = (int64_t)a.lseq[base + __builtin_ctz(m)];
    } else {
        // own evicted slots, as global ids, ascending: lane l holds slots t*256 + 4l .. +4
        const int s0 = t * kBS + 4 * lane;
        const int wl = a.W > 0 ? a.W - 1 : 0;
        uint32_t e = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint8_t sv = a.st[min(s0 + q, wl)];
            e |= ((s0 + q < a.W) && (sv & kStEvicted)) ? (1u << q) : 0u;
        }
        const uint32_t n = (uint32_t)__popc(e);
        int64_t o = tile_pre(a.wcnt, a.wpre) + (int64_t)(wave_incl_scan_u32(n) - n);
        for (uint32_t m = e; m; m &= m - 1) a.evicted[o++] = a.slot_base + s0 + __builtin_ctz(m);
    }
}


// Phase 2 of a sharded tick whose round table is wider than k_emit_shard's three
// 64-round chunks (fill levels of 128 and more: free counts in the hundreds or
// thousands).  The same water-filling, with the rounds walked in 64-round chunks: a
// first pass over the totals finds L, S(L) and So(L) (and keeps every chunk's starting
// S / So in LDS), the emission pass reloads each chunk's block prefixes and segment
// counts, and rounds L and L + 1 read their rank bases directly.
constexpr int kWideMaxCh = 64;  // R <= 4096 rows
__global__ __launch_bounds__(kBS) void k_emit_shard_wide(TickArgs a) {
    prefetch_args(a);
    const int bid = blockIdx.x;
    const int lane = lane_id(), w = wave_id();
    if (bid >= a.nbq) {
        shard_compact(a, bid);
        return;
    }
    __shared__ int64_t chS[kWideMaxCh], chSo[kWideMaxCh];
    const int b = bid;
    const int R = a.R;
    const int64_t pos = (int64_t)b * kBS + threadIdx.x;
    const int64_t pq = pos < a.Qlog ? pos : (a.Qlog > 0 ? a.Qlog - 1 : 0);
    const int cq = xc_get(a, pq);
    const int sq = lq_slot(a, pq);
    const int32_t rawq = a.c_arr[pq];
    const int64_t O = a.P->O;
    int64_t cap = a.P->cap_total;
    const int maxc = a.P->maxc;
    const int rlim = maxc < R ? maxc : R;
    if (maxc > R) cap = INT64_MAX;
    const int64_t N = (a.redist ? O : 0) + a.T;
    const int64_t N_eff = N < cap ? N : cap;
    // ---- pass 1 (every wave alike): S(r), So(r) chunk by chunk until S(r + 1) > N_eff
    int L = 0;
    int64_t S_L = 0, oSL = 0;
    {
        int64_t carry = 0, ocarry = 0;
        bool found = false;
        for (int k = 0; 64 * k < rlim; ++k) {
            const int r = 64 * k + lane;
            const uint32_t v = r < rlim ? (uint32_t)a.A[r] : 0u;
            const uint32_t ov = r < rlim ? (uint32_t)a.oA[r] : 0u;
            if (w == 0 && lane == 0) {
                chS[k] = carry;
                chSo[k] = ocarry;
            }
            const uint32_t incl = wave_incl_scan_u32(v), oincl = wave_incl_scan_u32(ov);
            const int64_t S1 = carry + (int64_t)incl;
            const int nl = __popcll(__ballot(r < rlim && S1 <= N_eff));
            L += nl;
            if (nl < 64) {  // S is non-decreasing: the fill level lies in this chunk
                S_L = carry + (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(incl - v), nl);
                oSL = ocarry + (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(oincl - ov), nl);
                found = true;
                break;
            }
            carry += (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            ocarry += (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)oincl, 63);
        }
        if (!found) {  // every round of the table below the fill level: S(rlim)
            S_L = carry;
            oSL = ocarry;
        }
    }
    lds_barrier();
    int status = 0;  // (precedence as in k_emit_shard)
    if (maxc > R && L >= R - 1) status = 1;  // R <= 64 * kWideMaxCh (the host caps it)
    else if (a.head_local + N_eff > a.log_cap) status = 2;
    const int64_t p = N_eff - S_L;
    const int64_t AL = (L < maxc && L < rlim) ? a.A[L] : 0;
    if (b == 0 && threadIdx.x == 0) {
        a.hout->O = O;
        a.hout->O_local = a.P->O_local;
        a.hout->n_evicted = a.P->n_evicted;
        a.hout->cap_total = cap;
        a.hout->maxc = maxc;
        a.hout->L = L;
        a.hout->status = status;
        a.hout->N_eff = status ? 0 : N_eff;
        a.hout->p = p;
        a.hout->AL = AL;
        if (!status && AL == 0) {
            a.hout->new_qlen = 0;
            a.hout->n_local = oSL;
        }
    }
    if (status) return;
    const int c = pos < a.Qlog ? cq : 0;
    const int s = sq;
    const int ls = s >= 0 ? own_slot(a, s) : -1;
    const bool own = c > 0 && ls >= 0;
    const int oc = own ? c : 0;
    // rank bases of this wave's segment in A_r (all and own) for round r
    auto rank_base = [&](int r, int64_t &rb, int64_t &orb) {
        const int rr = r < R ? r : R - 1;
        rb = r < rlim ? a.qpre[(size_t)b * R + rr] : 0;
        orb = r < rlim ? a.opre[(size_t)b * R + rr] : 0;
        for (int q = 0; q < w; ++q) {
            rb += r < R ? a.segcnt[(size_t)(4 * b + q) * R + rr] : 0u;
            orb += r < R ? a.osegcnt[(size_t)(4 * b + q) * R + rr] : 0u;
        }
    };
    int32_t *const lslot = a.log_slot + a.head_local;
    uint32_t *const lseq = a.lseq_out + a.head_local;
    const uint32_t hin = (uint32_t)a.head_in;
    // ---- full rounds r < min(L, max own c of the wave), a 64-round chunk at a time
    int32_t *const aall = a.assign_all;  // (fb_set_full_assign: every lane's task too)
    const int owmx = (int)wave_max_u32((uint32_t)(aall ? c : oc));
    const int rfull = L < owmx ? L : owmx;
    for (int k = 0; 64 * k < rfull; ++k) {
        const int r = 64 * k + lane;
        int64_t rb, orb;
        rank_base(r, rb, orb);
        const uint32_t v = r < rlim ? (uint32_t)a.A[r] : 0u;
        const uint32_t ov = r < rlim ? (uint32_t)a.oA[r] : 0u;
        const int64_t Sr = chS[k] + (int64_t)(wave_incl_scan_u32(v) - v);
        const int64_t Sor = chSo[k] + (int64_t)(wave_incl_scan_u32(ov) - ov);
        const int32_t basev = (int32_t)(Sr + rb), obasev = (int32_t)(Sor + orb);
        const int r1 = rfull - 64 * k < 64 ? rfull - 64 * k : 64;
        for (int i = 0; i < r1; ++i) {
            const int rr = 64 * k + i;
            const uint64_t m = __ballot(c > rr);
            const uint64_t om = __ballot(oc > rr);
            const int base = __builtin_amdgcn_readlane(basev, i);
            const int obase = __builtin_amdgcn_readlane(obasev, i);
            if (oc > rr) {
                const int lp = obase + popc_lt(om);
                lslot[lp] = s;
                lseq[lp] = hin + (uint32_t)(base + popc_lt(m));
            }
            if (aall && c > rr) aall[base + popc_lt(m)] = s;
        }
    }
    // ---- round L (partial: ranks < p) and round L + 1 (ranks for the next queue)
    int64_t rbL, orbL, rbL1, orbL1;
    rank_base(L, rbL, orbL);
    rank_base(L + 1, rbL1, orbL1);
    const uint64_t mL = __ballot(c > L);
    const uint64_t omL = __ballot(oc > L);
    const int64_t rankL = rbL + popc_lt(mL);
    const int64_t orankL = orbL + popc_lt(omL);
    if (oc > L && rankL < p) {
        const int64_t lp = oSL + orankL;
        lslot[lp] = s;
        lseq[lp] = hin + (uint32_t)(S_L + rankL);
    }
    if (aall && c > L && rankL < p) aall[S_L + rankL] = s;
    const int64_t exL1 = rbL1 + popc_lt(__ballot(c > L + 1));
    if (c > 0) {
        int64_t n_q = c < L ? c : L;
        if (c > L && rankL < p) n_q += 1;
        int64_t np = -1;
        if (c > L) {
            if (rankL >= p) np = rankL - p;
            else if (c > L + 1) np = (AL - p) + exL1;
            if (rankL == p) {
                a.hout->new_qlen = (AL - p) + exL1;
                a.hout->n_local = oSL + orankL;
            }
        }
        // the owned worker's next {free, queued} in one 8-byte store (the purge wrote {., 0})
        if (own) a.free_out[ls] = make_int2(rawq - (int32_t)n_q, np >= 0 ? 1 : 0);
        if (np >= 0) a.queue_out[np] = s;
    }
}

// ------------------------------------------------------------ orphan segments
// A fused one-GPU tick leaves its orphans in per-tile segments (emit_log_tiles): the
// dense list is the segments in tile order.  One workgroup per tile: its offset is the
// sum of the earlier tiles' counts (<= 4 loads per thread), then the copy.  dst may be
// host memory mapped for the device (the readback into pinned memory).
__device__ __forceinline__ void orph_gather_tile(int64_t *__restrict__ dst, const int64_t *__restrict__ src,
                                                 const uint32_t *__restrict__ cnt, int t) {
    __shared__ uint32_t l4[kWaves];
    uint32_t pre = 0;
    for (int i = threadIdx.x; i < t; i += kBS) pre += cnt[i];
    pre = wave_sum_u32(pre);
    if (lane_id() == 0) l4[wave_id()] = pre;
    __syncthreads();
    const int64_t off = (int64_t)l4[0] + l4[1] + l4[2] + l4[3];
    const uint32_t n = cnt[t];
    for (uint32_t i = threadIdx.x; i < n; i += kBS) dst[off + i] = src[(int64_t)t * kFTile + i];
}
__global__ __launch_bounds__(kBS) void k_orph_gather(int64_t *__restrict__ dst, const int64_t *__restrict__ src,
                                                    const uint32_t *__restrict__ cnt, int ntile) {
    orph_gather_tile(dst, src, cnt, blockIdx.x);
}

// pos[queue[p]] = p over the committed window [off, off + n) (tombstones skipped): the
// positions window ticks need, rebuilt once after general ticks (which do not keep them)
__global__ __launch_bounds__(kBS) void k_pos_rebuild(int32_t *__restrict__ pos, const int32_t *__restrict__ queue,
                                                    const int32_t *__restrict__ qfree, int64_t off, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBS + threadIdx.x;
    if (i >= n) return;
    const int32_t s = queue[off + i];
    if (qfree[off + i] != kTomb) pos[s] = (int32_t)(off + i);
}

// Evicted slots in ascending order when the tick did not compact them (window ticks):
// one workgroup scans the per-tile eviction counts, then one block per 256-slot tile
// writes its evicted slots at its offset (dst may be host-mapped memory).
__global__ __launch_bounds__(kBS) void k_wscan(const uint32_t *__restrict__ wcnt, int ntile, int64_t *__restrict__ wpre) {
    __shared__ unsigned long long l4[kWaves];
    run_excl_scan(wcnt, 1, ntile, wpre, 1, l4);
}
__global__ __launch_bounds__(kBS) void k_evict_compact(int32_t *__restrict__ dst, const uint8_t *__restrict__ st,
                                                      const int64_t *__restrict__ wpre, int W) {
    __shared__ uint32_t l4[kWaves];
    const int b = blockIdx.x, s = b * kBS + threadIdx.x;
    const uint32_t e = (s < W) & ((st[min(s, W > 0 ? W - 1 : 0)] & kStEvicted) != 0);
    uint32_t tot;
    const uint32_t ex = block_excl_scan_u32(e, l4, tot);
    if (e) dst[wpre[b] + ex] = s;
}

// ------------------------------------------------------------ readback
// Several word copies in one launch (a tick's outputs into pinned host memory with one
// kernel instead of one per array): copy i takes the blocks [b_i, b_{i+1}) of the grid.
__global__ __launch_bounds__(kBS) void k_copy_multi(CopyMulti m) {
    const int ob = (int)gridDim.x - m.otiles;  // the last otiles blocks gather orphan segments
    if ((int)blockIdx.x >= ob) {
        orph_gather_tile(m.odst, m.osrc, m.ocnt, (int)blockIdx.x - ob);
        return;
    }
    int i = 0;
    while (i + 1 < m.n && (int)blockIdx.x >= m.blk0[i + 1]) ++i;
    uint32_t *__restrict__ dst = m.dst[i];
    const uint32_t *__restrict__ src = m.src[i];
    const int64_t n = m.words[i];
    const int64_t nb = (int64_t)(i + 1 < m.n ? m.blk0[i + 1] : ob) - m.blk0[i];
    const int64_t stride = nb * kBS * 4;
    for (int64_t q0 = ((int64_t)(blockIdx.x - m.blk0[i]) * kBS + threadIdx.x) * 4; q0 < n; q0 += stride) {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = src[q0 + k < n ? q0 + k : n - 1];
        if (((reinterpret_cast<uintptr_t>(dst) & 15) == 0) && q0 + 3 < n) {
            *reinterpret_cast<uint4 *>(dst + q0) = make_uint4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (q0 + k < n) dst[q0 + k] = v[k];
        }
    }
}

// Words to (host-mapped) memory: lane j of a pass moves words 4j .. 4j + 3 -- four
// 4-byte loads (any source alignment), one 16-byte store (dst is 16-byte aligned in
// the callers' pinned buffers; else word stores) -- so a wave store is one 1 KB burst
// across PCIe; two passes per thread in flight.
__global__ __launch_bounds__(kBS) void k_copy_words(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src,
                                                   int64_t n) {
    const bool al = (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
    const int64_t stride = (int64_t)gridDim.x * kBS * 8;
    for (int64_t q0 = ((int64_t)blockIdx.x * kBS * 2 + threadIdx.x) * 4; q0 < n; q0 += stride) {
        uint32_t v[2][4];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int64_t i = q0 + (int64_t)p * kBS * 4 + k;
                v[p][k] = src[i < n ? i : n - 1];
            }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int64_t i = q0 + (int64_t)p * kBS * 4;
            if (al && i + 3 < n) {
                *reinterpret_cast<uint4 *>(dst + i) = make_uint4(v[p][0], v[p][1], v[p][2], v[p][3]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (i + k < n) dst[i + k] = v[p][k];
            }
        }
    }
}

}  // namespace fb

// ------------------------------------------------------------ launchers
namespace fb {
static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
template <int NB>
static void rs_pass(const RsPass &p, Stream h, Stream s) {
    hipExtLaunchKernelGGL(k_rs_hist<NB>, dim3(p.nblk), dim3(kBS), 0, h.s, h.e0, h.e1, 0, p.kin, p.n, p.shift, p.db,
                          p.hist, p.nblk, p.zero0, p.zero1, p.zbits, p.zwords);
    hipEvent_t start = nullptr;
    const uint32_t *tot = nullptr;
    if (p.nblk > kRsScanMin) {
        uint32_t *t = p.hist + (size_t)p.nblk * NB;
        hipExtLaunchKernelGGL(k_rs_scan, dim3(NB / 64), dim3(64 * kRsScanWaves), 0, s.s, start, nullptr, 0, p.hist,
                              p.nblk, NB, t);
        start = nullptr;
        tot = t;
    }
    hipExtLaunchKernelGGL(k_rs_scatter<NB>, dim3(p.nblk), dim3(kBS), 0, s.s, start, s.e1, 0, p.kin, p.vin, p.kout,
                          p.vout, p.n, p.shift, p.db, p.hist, p.nblk, p.identity_vals, tot);
}
void launch_rs_pass(const RsPass &p, Stream h, Stream s) {
    if (p.db <= 8)
        rs_pass<256>(p, h, s);
    else if (p.db <= 10)
        rs_pass<1024>(p, h, s);
    else
        rs_pass<2048>(p, h, s);
}
void launch_ev_apply(const EvArgs &a, Stream st) {
    hipExtLaunchKernelGGL(k_ev_apply, dim3(cdiv(a.E, kBS)), dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
}
void launch_ev_link(const EvArgs &a, Stream st) {
    const int grid = std::max(1, (int)std::max<int64_t>(cdiv(a.E, kBS), std::min<int64_t>(cdiv(a.tbits_words, kBS), 1024)));
    hipExtLaunchKernelGGL(k_ev_link, dim3(grid + a.cm_blocks), dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
}
void launch_ev_apply_ll(const EvArgs &a, Stream st) {
    const int nwb = a.wtiles == 4 ? (a.nbw + 3) / 4 : a.nbw;
    hipExtLaunchKernelGGL(k_ev_apply_ll, dim3(cdiv(a.E, kBS) + nwb), dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
}
void launch_copy_multi(const CopyMulti &m, Stream st) {
    if (m.n <= 0 && m.otiles <= 0) return;
    const int last = m.n - 1;
    const int grid = (m.n > 0 ? m.blk0[last] + (int)std::min<int64_t>(std::max<int64_t>(1, (m.words[last] + 4 * kBS - 1) / (4 * kBS)), 512) : 0) +
                     m.otiles;
    hipExtLaunchKernelGGL(k_copy_multi, dim3(grid), dim3(kBS), 0, st.s, st.e0, st.e1, 0, m);
}
void launch_orph_gather(int64_t *dst, const int64_t *src, const uint32_t *cnt, int ntile, Stream st) {
    if (ntile > 0) hipExtLaunchKernelGGL(k_orph_gather, dim3(ntile), dim3(kBS), 0, st.s, st.e0, st.e1, 0, dst, src, cnt, ntile);
}
void launch_copy_words(uint32_t *dst, const uint32_t *src, int64_t n, Stream st) {
    const int grid = (int)std::min<int64_t>(std::max<int64_t>(1, (n + 8 * kBS - 1) / (8 * kBS)), 2048);
    hipExtLaunchKernelGGL(k_copy_words, dim3(grid), dim3(kBS), 0, st.s, st.e0, st.e1, 0, dst, src, n);
}
// Timing gate (fb_timing_gate): one lane polls a host-mapped word until the host stores
// `want` into it, so the launches queued behind this kernel run back to back, free of
// the host's enqueue pace.  Every exit path is bounded: after `limit` ticks of the
// 100 MHz realtime counter the gate opens by itself and reports it in flag[1].
// Lazy clears: the deferred clears of every entry whose registration died (no record, or
// older than the slot's epoch) -- before a state read, so the log reads as it would had
// every commit cleared its orphans
__global__ __launch_bounds__(kBS) void k_log_normalize(int32_t *__restrict__ log, int64_t n,
                                                       const uint8_t *__restrict__ reg,
                                                       const uint32_t *__restrict__ epoch) {
    for (int64_t q = (int64_t)blockIdx.x * kBS + threadIdx.x; q < n; q += (int64_t)gridDim.x * kBS) {
        const int32_t s = log[q];
        if (s >= 0 && (!reg[s] || (uint64_t)q < (uint64_t)epoch[s])) log[q] = -1;
    }
}

__global__ __launch_bounds__(64) void k_gate(uint32_t *flag, uint32_t want, uint64_t limit) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == want) return;
        if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
            __hip_atomic_store(flag + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}
int emit_win_resident_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_emit_win, kBS, 0) != hipSuccess) return 0;
    return n;
}
void launch_log_normalize(int32_t *log, int64_t n, const uint8_t *reg, const uint32_t *epoch, Stream st) {
    if (n <= 0) return;
    const int grid = (int)std::min<int64_t>(cdiv(n, kBS), 8192);
    hipExtLaunchKernelGGL(k_log_normalize, dim3(grid), dim3(kBS), 0, st.s, st.e0, st.e1, 0, log, n, reg, epoch);
}
void launch_gate(uint32_t *flag, uint32_t want, uint64_t limit, Stream st) {
    hipExtLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, st.s, st.e0, st.e1, 0, flag, want, limit);
}
void launch_selftest(uint32_t *err, uint32_t seed, Stream st) {
    hipExtLaunchKernelGGL(k_selftest, dim3(64), dim3(kBS), 0, st.s, st.e0, st.e1, 0, err, seed);
}
static int tick_mode(const TickArgs &a) { return a.deque ? kModeDeque : (a.E == 0 ? kModeIdle : kModeEvents); }
#define FB_LAUNCH_MODE(K, grid, lds, st, a)                                                              \
    do {                                                                                             \
        switch (tick_mode(a)) {                                                                      \
        case kModeIdle: hipExtLaunchKernelGGL(K<kModeIdle>, grid, dim3(kBS), lds, st.s, st.e0, st.e1, 0, a); break;    \
        case kModeEvents: hipExtLaunchKernelGGL(K<kModeEvents>, grid, dim3(kBS), lds, st.s, st.e0, st.e1, 0, a); break; \
        default: hipExtLaunchKernelGGL(K<kModeDeque>, grid, dim3(kBS), lds, st.s, st.e0, st.e1, 0, a); break;           \
        }                                                                                            \
    } while (0)
void launch_slots(const TickArgs &a, Stream st) {
    FB_LAUNCH_MODE(k_slots, dim3(a.nbw), 0, st, a);
}
template <int WT>
static void launch_scan_t(const TickArgs &a, dim3 g, size_t lds, Stream st) {
    switch (tick_mode(a)) {
    case kModeIdle: hipExtLaunchKernelGGL((k_scan<kModeIdle, WT>), g, dim3(kBS), lds, st.s, st.e0, st.e1, 0, a); break;
    case kModeEvents: hipExtLaunchKernelGGL((k_scan<kModeEvents, WT>), g, dim3(kBS), lds, st.s, st.e0, st.e1, 0, a); break;
    default: hipExtLaunchKernelGGL((k_scan<kModeDeque, WT>), g, dim3(kBS), lds, st.s, st.e0, st.e1, 0, a); break;
    }
}
void launch_scan(const TickArgs &a, Stream st) {
    const size_t lds = (a.lds_bitmap && !a.slots_in_scan) ? (size_t)((a.W + 63) / 64) * 8 : 0;
    const int nbw = (a.shard == 2 || !a.slots_in_scan || a.slots_in_apply) ? 0 : (a.wtiles > 1 ? (a.nbw + a.wtiles - 1) / a.wtiles : a.nbw);
    const int nbf = (a.shard == 2 || a.f_sep || a.f_emit) ? 0 : a.nbf;
    const int wt = nbw ? a.wtiles : 1;
    const int nqb = (wt == 4 && a.qtiles == 4) ? (a.nbq + 3) / 4 : a.nbq;  // (k_scan's own count)
    const dim3 g(nbf + nbw + nqb + (a.cm_fold ? a.cm_blocks : 0));
    if (wt == 4) launch_scan_t<4>(a, g, nbf ? lds : 0, st);
    else if (wt == 2) launch_scan_t<2>(a, g, nbf ? lds : 0, st);
    else launch_scan_t<1>(a, g, nbf ? lds : 0, st);
}
void launch_logscan(const TickArgs &a, int grid, Stream st) {
    const size_t lds = (size_t)(((a.W + 63) / 64 + 1) / 2 + 1) * 16;  // + the spare slot
    hipExtLaunchKernelGGL(k_logscan, dim3(grid), dim3(kLsBS), lds, st.s, st.e0, st.e1, 0, a);
}
void launch_plan(const TickArgs &a, Stream st) {
    if (a.grp_on)
        hipExtLaunchKernelGGL(k_plan2, dim3(a.ngrp + 2), dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
    else
        hipExtLaunchKernelGGL(k_plan, dim3(3 + (a.shard ? 2 : 1) * a.R), dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
}
void launch_xscan(const TickArgs &a, Stream st) {
    hipExtLaunchKernelGGL(k_xscan<kXGroupR>, dim3((a.nbq + kXsBlocks - 1) / kXsBlocks), dim3(kBS), 0, st.s, st.e0,
                          st.e1, 0, a);
}
void launch_emit(const TickArgs &a, Stream st) {
    FB_LAUNCH_MODE(k_emit, dim3(a.nbq + a.nbf + a.nbw), 0, st, a);
}
template <int PM, int NCH>
static void launch_emit2_t(const TickArgs &a, Stream st) {
    const int nc = (a.f_emit ? a.nbf : (a.nbf + 3) / 4) + (a.nbw + 3) / 4;
    const dim3 g(a.cmix ? 8 * ((a.nbq + 7) / 8 + (nc + 7) / 8) : a.nbq + nc);
    // f_emit: the log workgroups stage the died bitmap in LDS (rounded to whole int4)
    const size_t lds = a.f_emit ? (size_t)(((a.W + 63) / 64 + 1) / 2) * 16 : 0;
    switch (tick_mode(a)) {
    case kModeIdle: hipExtLaunchKernelGGL((k_emit2<kModeIdle, PM, NCH>), g, dim3(kBS), lds, st.s, st.e0, st.e1, 0, a); break;
    case kModeEvents: hipExtLaunchKernelGGL((k_emit2<kModeEvents, PM, NCH>), g, dim3(kBS), lds, st.s, st.e0, st.e1, 0, a); break;
    default: hipExtLaunchKernelGGL((k_emit2<kModeDeque, PM, NCH>), g, dim3(kBS), lds, st.s, st.e0, st.e1, 0, a); break;
    }
}
void launch_emit2(const TickArgs &a, Stream st) {
    // one 64-round chunk while rounds 0 .. L+1 <= R+1 fit in a wave's lanes (R = 32)
    if (a.fused) {
        if (a.R <= 32) launch_emit2_t<0, 1>(a, st);
        else launch_emit2_t<0, 3>(a, st);
    } else if (a.gp) {
        if (a.R <= 32) launch_emit2_t<2, 1>(a, st);
        else launch_emit2_t<2, 3>(a, st);
    } else {
        if (a.R <= 32) launch_emit2_t<1, 1>(a, st);
        else launch_emit2_t<1, 3>(a, st);
    }
}
void launch_emit_shard(const TickArgs &a, Stream st) {
    if (a.R > 64 * kRCh - 64) {  // rounds 0 .. L+1 beyond the three register chunks
        hipExtLaunchKernelGGL(k_emit_shard_wide, dim3(a.nbq + (a.nbf + 3) / 4 + (a.nbw + 3) / 4), dim3(kBS), 0, st.s,
                              st.e0, st.e1, 0, a);
        return;
    }
    const dim3 g(a.nbq + (a.nbf + 3) / 4 + (a.nbw + 3) / 4);
    if (a.xplan) {
        // two queue blocks per workgroup (k_emit_shard_xp; four measured no faster, r06f_probe_*)
        const dim3 g2((a.nbq + 1) / 2 + (a.nbf + 3) / 4 + (a.nbw + 3) / 4);
        hipExtLaunchKernelGGL(k_emit_shard_xp<2>, g2, dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
        return;
    }
    if (a.xrows)
        hipExtLaunchKernelGGL(k_emit_shard<true, true>, g, dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
    else if (a.grp_on)
        hipExtLaunchKernelGGL(k_emit_shard<true, false>, g, dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
    else
        hipExtLaunchKernelGGL(k_emit_shard<false, false>, g, dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
}
void launch_evict_gather(int32_t *dst, const uint8_t *st, const uint32_t *wcnt, int64_t *wpre, int W, Stream s) {
    const int nt = cdiv(W, kBS);
    if (nt <= 0) return;
    hipExtLaunchKernelGGL(k_wscan, dim3(1), dim3(kBS), 0, s.s, s.e0, nullptr, 0, wcnt, nt, wpre);
    hipExtLaunchKernelGGL(k_evict_compact, dim3(nt), dim3(kBS), 0, s.s, nullptr, s.e1, 0, dst, st, (const int64_t *)wpre, W);
}
void launch_pos_rebuild(int32_t *pos, const int32_t *queue, const int32_t *qfree, int64_t off, int64_t n, Stream st) {
    if (n > 0)
        hipExtLaunchKernelGGL(k_pos_rebuild, dim3(cdiv(n, kBS)), dim3(kBS), 0, st.s, st.e0, st.e1, 0, pos, queue, qfree,
                              off, n);
}
void launch_emit_win(const TickArgs &a, int grid, Stream st) {
    hipExtLaunchKernelGGL(k_emit_win, dim3(grid), dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
}
void launch_commit(const CommitArgs &a, int grid, Stream st) {
    hipExtLaunchKernelGGL(k_commit, dim3(grid), dim3(kBS), 0, st.s, st.e0, st.e1, 0, a);
}
}  // namespace fb
