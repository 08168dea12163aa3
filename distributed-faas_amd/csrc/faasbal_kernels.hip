// faasbal_kernels.hip -- CDNA4 (gfx950) kernels of one balancer tick.
//
// Tick pipeline, every kernel 256 threads = 4 wave64:
//   [E>0]  k_rs_hist / k_rs_scan / k_rs_scatter   stable LSD radix sort of events by slot
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
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "faasbal_kernels.h"

namespace fb {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
__device__ __forceinline__ int popc_lt(uint64_t m) {
    // number of set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
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
    __syncthreads();
    T pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        T t = lds4[w];
        pre += (w < wave_id()) ? t : (T)0;
        tot += t;
    }
    __syncthreads();
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
    __syncthreads();
    T m = lds4[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) m = m > lds4[w] ? m : lds4[w];
    __syncthreads();
    return m;
}

// ---------------------------------------------------------------- radix sort
// Stable LSD radix sort of (key = slot, val = event index), 8-bit digits.
__global__ __launch_bounds__(kBS) void k_rs_hist(const uint32_t *__restrict__ keys, int n, int shift,
                                                 uint32_t *__restrict__ hist, int nblk) {
    __shared__ uint32_t cnt[256];
    cnt[threadIdx.x] = 0;
    __syncthreads();
    const int base = blockIdx.x * kRsTile;
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) {
        int e = base + j * kBS + threadIdx.x;
        if (e < n) atomicAdd(&cnt[(keys[e] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(size_t)threadIdx.x * nblk + blockIdx.x] = cnt[threadIdx.x];
}

// In-place exclusive scan of n entries by one workgroup.
__global__ __launch_bounds__(kBS) void k_scan_1wg(uint32_t *__restrict__ a, int n) {
    __shared__ uint32_t l4[kWaves];
    uint32_t carry = 0;
    for (int base = 0; base < n; base += kBS) {
        int i = base + threadIdx.x;
        uint32_t v = i < n ? a[i] : 0u, tot;
        uint32_t ex = block_excl_scan<uint32_t>(v, l4, tot);
        if (i < n) a[i] = carry + ex;
        carry += tot;
    }
}

__global__ __launch_bounds__(kBS) void k_rs_scatter(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                    uint32_t *__restrict__ kout, uint32_t *__restrict__ vout, int n,
                                                    int shift, const uint32_t *__restrict__ hist, int nblk,
                                                    int identity_vals) {
    __shared__ uint32_t base[256];
    __shared__ uint32_t wcnt[kWaves][256];
    base[threadIdx.x] = hist[(size_t)threadIdx.x * nblk + blockIdx.x];
    const int tile = blockIdx.x * kRsTile;
    const int lane = lane_id(), w = wave_id();
    for (int j = 0; j < kRsItems; ++j) {
#pragma unroll
        for (int q = 0; q < kWaves; ++q) wcnt[q][threadIdx.x] = 0;
        __syncthreads();
        const int e = tile + j * kBS + threadIdx.x;
        const bool valid = e < n;
        uint32_t key = valid ? kin[e] : 0u;
        uint32_t val = valid ? (identity_vals ? (uint32_t)e : vin[e]) : 0u;
        uint32_t d = (key >> shift) & 255u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            uint64_t m = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        int wrank = popc_lt(peers);
        if (valid && wrank == 0) wcnt[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t off = base[d] + (uint32_t)wrank;
            for (int q = 0; q < w; ++q) off += wcnt[q][d];
            kout[off] = key;
            vout[off] = val;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int q = 0; q < kWaves; ++q) add += wcnt[q][threadIdx.x];
        base[threadIdx.x] += add;
        __syncthreads();
    }
    (void)lane;
}

// ------------------------------------------------------------ event apply
// One thread per slot segment of the slot-sorted events; processes that
// slot's messages in arrival order (task_dispatcher.py:343-390 per message,
// with the purge of the preceding loop iteration at the same clock).
__global__ __launch_bounds__(kBS) void k_ev_apply(EvArgs a) {
    const int j = blockIdx.x * kBS + threadIdx.x;
    if (j >= a.E) return;
    const uint32_t s = a.skeys[j];
    if (j > 0 && a.skeys[j - 1] == s) return;
    int reg = a.reg[s];
    int32_t fr = a.free_in[s];
    double hb = a.hb[s];
    uint32_t epoch = a.epoch[s];
    int inq = a.inq_in[s];
    int qstat = inq ? kQsKeep : kQsOut;
    int qidx = -1;
    int cur_is_start = reg, died_start = 0;
    for (int k = j; k < a.E && a.skeys[k] == s; ++k) {
        const int i = (int)a.svals[k];
        const int kind = a.ev_kind[i];
        const int32_t val = a.ev_val[i];
        const double ts = a.ev_ts[i];
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
            const int64_t q = a.ev_seq[i];
            if (q >= 0 && q < a.head_in && a.log_slot[q] == (int32_t)s) a.log_slot[q] = -1;
            if (fr == 1 && !inq) { inq = 1; qstat = kQsBack; qidx = i; }
        }
        a.ev_status[i] = status;
    }
    a.post_reg[s] = (uint8_t)reg;
    a.post_free[s] = fr;
    a.post_hb[s] = hb;
    a.post_epoch[s] = epoch;
    a.post_flags[s] = (uint8_t)(died_start | (qstat << 1));
    a.touched[s] = a.tick;
    if (qstat == kQsFront) a.front_list[a.E - 1 - qidx] = (int32_t)s;
    if (qstat == kQsBack) a.back_list[qidx] = (int32_t)s;
}

// ------------------------------------------------------------ slot purge
__global__ __launch_bounds__(kBS) void k_slots(SlotArgs a) {
    __shared__ uint32_t l4[kWaves];
    const int s = blockIdx.x * kBS + threadIdx.x;
    uint32_t ev = 0;
    if (s < a.W) {
        const bool t = a.touched[s] == a.tick;
        const int reg0 = a.reg[s];
        int reg = reg0;
        double hb = a.hb[s];
        int32_t fr = a.free_in[s];
        int flags = 0;
        if (t) { reg = a.post_reg[s]; hb = a.post_hb[s]; fr = a.post_free[s]; flags = a.post_flags[s]; }
        // PushWorker.is_alive (:209-212): time.time() - last_heartbeat > time_to_expire
        const bool dead = reg && ((a.now - hb) > a.tte);
        const bool alive = reg && !dead;
        const bool died_start = reg0 && (dead || (flags & kPfDiedStart));
        const bool evicted = (reg0 || t) && !alive;
        a.st[s] = (uint8_t)((alive ? kStAlive : 0) | (died_start ? kStDiedStart : 0) | (evicted ? kStEvicted : 0));
        a.free_out[s] = fr;
        a.inq_out[s] = 0;
        ev = evicted ? 1u : 0u;
    }
    uint32_t tot;
    block_excl_scan<uint32_t>(ev, l4, tot);
    if (threadIdx.x == 0) a.wcnt[blockIdx.x] = tot;
}

// ------------------------------------------------------------ scan
__device__ __forceinline__ int lq_slot(int64_t pos, const ScanArgs &a) {
    if (pos < a.E) return a.front_list[pos];
    pos -= a.E;
    if (pos < a.Qn) return a.queue_in[pos];
    pos -= a.Qn;
    return a.back_list[pos];
}

__device__ __forceinline__ int lq_c(int64_t pos, int s, const ScanArgs &a) {
    if (s < 0) return 0;
    if (!(a.st[s] & kStAlive)) return 0;
    if (pos >= a.E && pos < a.E + a.Qn && a.touched[s] == a.tick && ((a.post_flags[s] >> 1) & 3) != kQsKeep)
        return 0;  // moved to the front, re-appended or removed by this tick's messages
    const int f = a.free_out[s];
    return f > 1 ? f : 1;  // a queued worker with free <= 0 still takes one task (:409-419)
}

__device__ __forceinline__ bool is_orphan(int64_t seq, const int32_t *__restrict__ log_slot,
                                          const uint8_t *__restrict__ st, const uint32_t *__restrict__ epoch) {
    const int32_t s = log_slot[seq];
    return s >= 0 && (st[s] & kStDiedStart) && (uint64_t)seq >= (uint64_t)epoch[s];
}

__global__ __launch_bounds__(kBS) void k_scan(ScanArgs a) {
    __shared__ uint32_t l4[kWaves];
    __shared__ int32_t m4[kWaves];
    __shared__ unsigned long long s4[kWaves];
    __shared__ uint32_t wc[kWaves][kBS];
    if ((int)blockIdx.x < a.nbf) {
        // ---- log role: count orphans in this tile
        const int64_t base = a.log_lo + (int64_t)blockIdx.x * kFTile + (int64_t)threadIdx.x * kFItems;
        uint32_t cnt = 0;
#pragma unroll
        for (int j = 0; j < kFItems; ++j) {
            const int64_t q = base + j;
            if (q < a.head_in && is_orphan(q, a.log_slot, a.st, a.epoch)) ++cnt;
        }
        uint32_t tot;
        block_excl_scan<uint32_t>(cnt, l4, tot);
        if (threadIdx.x == 0) a.fcnt[blockIdx.x] = tot;
        return;
    }
    // ---- queue role
    const int b = (int)blockIdx.x - a.nbf;
    const int64_t pos = (int64_t)b * kBS + threadIdx.x;
    int c = 0;
    if (pos < a.Qlog) {
        const int s = lq_slot(pos, a);
        c = lq_c(pos, s, a);
        a.c_arr[pos] = c;
    }
    const int bm = block_reduce_max<int32_t>(c, m4);
    unsigned long long csum;
    block_excl_scan<unsigned long long>((unsigned long long)c, s4, csum);
    if (threadIdx.x == 0) {
        if (bm > 0) atomicMax(&a.P->maxc, bm);
        if (csum) atomicAdd(&a.P->cap_total, csum);
        a.qbmax[b] = bm < a.R ? bm : a.R;
    }
    // per-round counts of c > r for r < min(bm, R): waves count their part,
    // 256 rounds at a time, then one thread per round sums the four waves.
    const int rmax = bm < a.R ? bm : a.R;
    for (int r0 = 0; r0 < rmax; r0 += kBS) {
        const int rn = (rmax - r0) < kBS ? (rmax - r0) : kBS;
        for (int i = 0; i < rn; ++i) {
            uint64_t m = __ballot(c > r0 + i);
            if (lane_id() == 0) wc[wave_id()][i] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        if ((int)threadIdx.x < rn) {
            uint32_t t = 0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) t += wc[w][threadIdx.x];
            a.qcnt[(size_t)(r0 + threadIdx.x) * a.nbq + b] = t;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------ plan
// wg 0: orphan block offsets; wg 1: evicted block offsets; wg 2+r: row r of the
// round table (exclusive scan across queue blocks) and its total A(r) = |A_r|.
__global__ __launch_bounds__(kBS) void k_plan(PlanArgs a) {
    __shared__ unsigned long long l4[kWaves];
    if (blockIdx.x == 0 || blockIdx.x == 1) {
        const uint32_t *cnt = blockIdx.x == 0 ? a.fcnt : a.wcnt;
        int64_t *pre = blockIdx.x == 0 ? a.fpre : a.wpre;
        const int n = blockIdx.x == 0 ? a.nbf : a.nbw;
        unsigned long long carry = 0;
        for (int base = 0; base < n; base += kBS) {
            const int i = base + threadIdx.x;
            unsigned long long v = i < n ? cnt[i] : 0ull, tot;
            unsigned long long ex = block_excl_scan<unsigned long long>(v, l4, tot);
            if (i < n) pre[i] = (int64_t)(carry + ex);
            carry += tot;
        }
        if (threadIdx.x == 0) {
            if (blockIdx.x == 0) a.P->O = (int64_t)carry;
            else a.P->n_evicted = (int64_t)carry;
        }
        return;
    }
    const int r = (int)blockIdx.x - 2;
    if (r >= a.R) return;
    unsigned long long carry = 0;
    for (int base = 0; base < a.nbq; base += kBS) {
        const int b = base + threadIdx.x;
        unsigned long long v = 0, tot;
        if (b < a.nbq && r < a.qbmax[b]) v = a.qcnt[(size_t)r * a.nbq + b];
        unsigned long long ex = block_excl_scan<unsigned long long>(v, l4, tot);
        if (b < a.nbq) a.qpre[(size_t)r * a.nbq + b] = (int64_t)(carry + ex);
        carry += tot;
    }
    if (threadIdx.x == 0) a.A[r] = (int64_t)carry;
}

// ------------------------------------------------------------ emit
// Fill level: L = max{ r in [0, maxc] : S(r) <= N_eff }, searched 256 rounds at a time.
struct Level {
    int L;
    int status;
    int64_t p, AL, N_eff;
};

__device__ Level find_level(const EmitArgs &a, unsigned long long *l4) {
    Level lv;
    const int64_t O = a.P->O;
    const int64_t N = O + a.T;
    const int64_t cap = (int64_t)a.P->cap_total;
    const int maxc = a.P->maxc;
    lv.N_eff = N < cap ? N : cap;
    lv.status = 0;
    // S(r+1) = S(r) + A(r); count r in [1, min(maxc, R)] with S(r) <= N_eff
    const int rlim = maxc < a.R ? maxc : a.R;
    int64_t carry = 0;  // S(base)
    int Lc = 0;
    for (int base = 0; base < rlim; base += kBS) {
        const int r = base + threadIdx.x;  // computes S(r+1)
        unsigned long long v = r < rlim ? (unsigned long long)a.A[r] : 0ull, tot;
        unsigned long long ex = block_excl_scan<unsigned long long>(v, l4, tot);
        const int64_t S1 = carry + (int64_t)(ex + v);
        const bool ok = r < rlim && S1 <= lv.N_eff;
        uint64_t m = __ballot(ok);
        if (lane_id() == 0) l4[wave_id()] = (unsigned long long)__popcll(m);
        __syncthreads();
        int k = 0;
        for (int w = 0; w < kWaves; ++w) k += (int)l4[w];
        __syncthreads();
        Lc += k;
        carry += (int64_t)tot;
        if (k < kBS) break;  // S is non-decreasing: the first failure ends the search
    }
    lv.L = Lc;
    if (a.head_in + lv.N_eff > a.log_cap) {  // never write past the in-flight log
        lv.status = 2;
        lv.p = lv.AL = 0;
        return lv;
    }
    // exact rows exist for r < R; rounds 0..L+1 (bounded by maxc-1) must be covered
    if (maxc > a.R && lv.L >= a.R - 1) lv.status = 1;
    // S(L) and A(L)
    int64_t SL = 0;
    for (int base = 0; base < lv.L && !lv.status; base += kBS) {
        const int r = base + threadIdx.x;
        unsigned long long v = r < lv.L ? (unsigned long long)a.A[r] : 0ull, tot;
        block_excl_scan<unsigned long long>(v, l4, tot);
        SL += (int64_t)tot;
    }
    lv.p = lv.N_eff - SL;
    lv.AL = (!lv.status && lv.L < a.R && lv.L < maxc) ? a.A[lv.L] : 0;
    return lv;
}

__global__ __launch_bounds__(kBS) void k_emit(EmitArgs a) {
    __shared__ unsigned long long l4[kWaves];
    __shared__ uint32_t l4u[kWaves];
    __shared__ uint32_t rc[2][kWaves];
    const int nq = a.nbq;
    if ((int)blockIdx.x < nq) {
        const int b = blockIdx.x;
        const Level lv = find_level(a, l4);
        if (b == 0 && threadIdx.x == 0) {
            a.P->L = lv.L;
            a.P->status = lv.status;
            a.P->N_eff = lv.status ? 0 : lv.N_eff;
            a.P->p = lv.p;
            a.P->AL = lv.AL;
        }
        if (lv.status) return;
        const int64_t pos = (int64_t)b * kBS + threadIdx.x;
        int c = 0, s = -1;
        if (pos < a.Qlog) {
            c = a.c_arr[pos];
            if (c > 0) {
                const int64_t q = pos;
                if (q < a.E) s = a.front_list[q];
                else if (q < a.E + a.Qn) s = a.queue_in[q - a.E];
                else s = a.back_list[q - a.E - a.Qn];
            }
        }
        const int L = lv.L;
        const int bm = a.qbmax[b];  // rows r < bm carry counts (bm <= R)
        const int rend = (L + 1) < (bm - 1) ? (L + 1) : (bm - 1);
        int64_t S = 0;  // S(r)
        int64_t rankL = -1, rankL1 = -1;
        const int64_t head = a.head_in;
        for (int r = 0; r <= rend; ++r) {
            const bool act = c > r;
            const uint64_t m = __ballot(act);
            if (lane_id() == 0) rc[r & 1][wave_id()] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t wpre = 0;
            for (int w = 0; w < wave_id(); ++w) wpre += rc[r & 1][w];
            if (act) {
                const int64_t rank = a.qpre[(size_t)r * nq + b] + wpre + popc_lt(m);
                if (r < L) {
                    a.log_slot[head + S + rank] = s;
                } else if (r == L) {
                    rankL = rank;
                    if (rank < lv.p) a.log_slot[head + S + rank] = s;
                } else {
                    rankL1 = rank;
                }
            }
            S += a.A[r];
        }
        uint32_t member = 0;
        if (c > 0) {
            int64_t n_q = c < L ? c : L;
            if (c > L && rankL < lv.p) n_q += 1;
            if (n_q) a.free_out[s] = a.free_out[s] - (int32_t)n_q;
            int64_t np = -1;
            if (c > L) {
                if (rankL >= lv.p) np = rankL - lv.p;
                else if (c > L + 1) np = (lv.AL - lv.p) + rankL1;
            }
            if (np >= 0) {
                a.queue_out[np] = s;
                a.inq_out[s] = 1;
                member = 1;
            }
        }
        uint32_t tot;
        block_excl_scan<uint32_t>(member, l4u, tot);
        if (threadIdx.x == 0 && tot) atomicAdd(&a.P->new_qlen, (unsigned long long)tot);
        return;
    }
    if ((int)blockIdx.x < nq + a.nbf) {
        // ---- orphan compaction, ascending sequence
        const int b = blockIdx.x - nq;
        const int64_t base = a.log_lo + (int64_t)b * kFTile + (int64_t)threadIdx.x * kFItems;
        uint32_t flags = 0, cnt = 0;
#pragma unroll
        for (int j = 0; j < kFItems; ++j) {
            const int64_t q = base + j;
            if (q < a.head_in && is_orphan(q, a.log_slot_ro, a.st, a.epoch)) { flags |= 1u << j; ++cnt; }
        }
        uint32_t tot;
        uint32_t ex = block_excl_scan<uint32_t>(cnt, l4u, tot);
        int64_t o = a.fpre[b] + ex;
#pragma unroll
        for (int j = 0; j < kFItems; ++j)
            if (flags & (1u << j)) a.orphans[o++] = base + j;
        return;
    }
    // ---- evicted compaction, ascending slot
    const int b = blockIdx.x - nq - a.nbf;
    const int s = b * kBS + threadIdx.x;
    const uint32_t e = (s < a.W && (a.st[s] & kStEvicted)) ? 1u : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan<uint32_t>(e, l4u, tot);
    if (e) a.evicted[a.wpre[b] + ex] = s;
}

// ------------------------------------------------------------ commit
__global__ __launch_bounds__(kBS) void k_commit(CommitArgs a) {
    const int s = blockIdx.x * kBS + threadIdx.x;
    if (s >= a.W) return;
    const uint8_t stt = a.st[s];
    if (a.touched[s] == a.tick) {
        a.reg[s] = (stt & kStAlive) ? 1 : 0;
        a.hb[s] = a.post_hb[s];
        a.epoch[s] = a.post_epoch[s];
    } else if (stt & kStEvicted) {
        a.reg[s] = 0;
    }
}

}  // namespace fb

// ------------------------------------------------------------ launchers
namespace fb {
static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
void launch_rs_hist(const uint32_t *keys, int n, int shift, uint32_t *hist, int nblk, Stream st) {
    hipLaunchKernelGGL(k_rs_hist, dim3(nblk), dim3(kBS), 0, st, keys, n, shift, hist, nblk);
}
void launch_scan_1wg(uint32_t *a, int n, Stream st) {
    hipLaunchKernelGGL(k_scan_1wg, dim3(1), dim3(kBS), 0, st, a, n);
}
void launch_rs_scatter(const uint32_t *kin, const uint32_t *vin, uint32_t *kout, uint32_t *vout, int n,
                       int shift, const uint32_t *hist, int nblk, int identity_vals, Stream st) {
    hipLaunchKernelGGL(k_rs_scatter, dim3(nblk), dim3(kBS), 0, st, kin, vin, kout, vout, n, shift, hist, nblk,
                       identity_vals);
}
void launch_ev_apply(const EvArgs &a, Stream st) {
    hipLaunchKernelGGL(k_ev_apply, dim3(cdiv(a.E, kBS)), dim3(kBS), 0, st, a);
}
void launch_slots(const SlotArgs &a, int grid, Stream st) {
    hipLaunchKernelGGL(k_slots, dim3(grid), dim3(kBS), 0, st, a);
}
void launch_scan(const ScanArgs &a, int grid, Stream st) {
    hipLaunchKernelGGL(k_scan, dim3(grid), dim3(kBS), 0, st, a);
}
void launch_plan(const PlanArgs &a, int grid, Stream st) {
    hipLaunchKernelGGL(k_plan, dim3(grid), dim3(kBS), 0, st, a);
}
void launch_emit(const EmitArgs &a, int grid, Stream st) {
    hipLaunchKernelGGL(k_emit, dim3(grid), dim3(kBS), 0, st, a);
}
void launch_commit(const CommitArgs &a, int grid, Stream st) {
    hipLaunchKernelGGL(k_commit, dim3(grid), dim3(kBS), 0, st, a);
}
}  // namespace fb
