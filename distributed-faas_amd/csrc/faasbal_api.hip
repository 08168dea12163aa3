// faasbal_api.hip -- C ABI of libfaasbal.so (include/faasbal.h).
//
// Host orchestration of one tick on the context's HIP stream.  No CPU
// fallback exists: every decision is computed by the kernels in
// faasbal_kernels.hip; the host only validates arguments, stages event
// arrays (pinned) and reads back a few scalars.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "faasbal.h"
#include "faasbal_kernels.h"

using namespace fb;

namespace {

// Persistent host workers for the staging pass of large event batches: part i of
// n runs on worker i - 1 (part 0 on the caller).  One pool per context; the ABI
// allows one caller thread per context, so run() is never re-entered.
struct HostPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, done_cv;
    std::function<void(int)> job;
    long gen = 0;
    int pending = 0;
    bool stop = false;

    explicit HostPool(int n) {
        for (int i = 1; i < n; ++i) th.emplace_back([this, i] { loop(i); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : th) t.join();
    }
    int size() const { return (int)th.size() + 1; }
    void loop(int i) {
        long seen = 0;
        for (;;) {
            std::function<void(int)> f;
            {
                std::unique_lock<std::mutex> l(m);
                cv.wait(l, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
                f = job;
            }
            f(i);
            std::lock_guard<std::mutex> g(m);
            if (--pending == 0) done_cv.notify_one();
        }
    }
    void run(const std::function<void(int)> &f) {
        {
            std::lock_guard<std::mutex> g(m);
            job = f;
            pending = (int)th.size();
            ++gen;
        }
        cv.notify_all();
        f(0);
        std::unique_lock<std::mutex> l(m);
        done_cv.wait(l, [&] { return pending == 0; });
    }
};


struct TimedLaunch {
    const char *name;
    hipEvent_t a, b;
};

}  // namespace

struct fb_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int32_t W_cap = 0, E_cap = 0;
    int64_t log_cap = 0;
    // committed state
    int32_t W = 0;
    int cur = 0;  // index of the committed dense buffers
    int2 *free_[2] = {nullptr, nullptr};  // {free_processes, queued} per slot
    int32_t *queue[2] = {nullptr, nullptr};
    int32_t *qfree[2] = {nullptr, nullptr};  // free_processes by LRU position (one-GPU contexts)
    double *qhb[2] = {nullptr, nullptr};     // last_heartbeat by LRU position
    double *c_hb = nullptr;                  // per tick: heartbeat of a live LRU position
    bool qaos = false;                       // qfree/qhb[cur] describe the committed queue
    uint8_t *reg = nullptr;
    double *hb = nullptr;        // last_heartbeat per slot (NaN: no record)
    uint32_t *epoch = nullptr;   // first log sequence of the slot's current registration
    int32_t *log_slot = nullptr;
    // one-GPU heartbeat contexts: in-flight entries per slot (by commit parity), the
    // post-message counts, the entry each event's result completes (cleared by the
    // commit: the log is read-only during a tick), the launch stamp of the last launch
    // whose result completed an entry, and k_emit2's log-workgroup hand-off granules
    int32_t *bud = nullptr;       // in flight + free processes of a registered slot (committed)
    int32_t *bud_next = nullptr;  // touched slots: the budget after the tick (the commit installs it)
    uint32_t *post_infl = nullptr;
    int32_t *ev_clr = nullptr;
    uint32_t *ctag = nullptr;
    uint32_t lstamp = 0;               // per enqueued launch, reruns included (never 0)
    // f_emit ticks leave their orphans in per-tile segments (orphans[t*2048 + i], i < fcnt[t]);
    // the dense list is gathered into orph_dense when something reads it
    bool l_oseg = false, dense_ok = false;
    int l_nbf = 0;
    int64_t *orph_dense = nullptr;
    // compact assignments (fb_set_compact): slot and min(c, L + 1) per LRU position
    int32_t *rb_slot = nullptr;
    uint8_t *rb_c = nullptr;
    int compact = 0, l_compact = 0;    // the setting, and the one the last launch ran with
    // fb_set_compact_out: pinned buffers the ticks write their compact outputs into directly
    // (device views of them, the caller's pointers, capacities); l_cout: the last launch did
    int32_t *cout_slot = nullptr, *cout_ev = nullptr;
    uint8_t *cout_c = nullptr;
    int64_t *cout_orph = nullptr;
    const void *cout_host[4] = {nullptr, nullptr, nullptr, nullptr};
    int64_t cout_cap = 0, cout_ocap = 0, cout_ecap = 0;
    bool l_cout = false;
    HostPool *xpool = nullptr;         // fb_expand_compact's workers (created on first use)
    int32_t *trash = nullptr;  // kTrashRows x kBS words written by inactive lanes (never read)
    int64_t Qn = 0, head = 0;
    // window ticks (one-GPU heartbeat contexts): the committed queue is
    // [qoff, qoff + Qn) of queue[qcur] / qfree[qcur] / qhb[qcur] (qcap entries each; qfree
    // kTomb marks a position whose slot left), pos_of[qcur][s] the position of a queued slot
    int qcur = 0;
    int64_t qoff = 0, qcap = 0, Qtrue = 0;  // Qtrue: the LRU queue's length (tombstones excluded)
    bool win_cap = false;      // the context can run window ticks (buffers allocated)
    int win = -1;              // fb_set_window: -1 auto (large tables), 0 off, 1 on
    bool l_win = false;        // the last launch is a window tick
    int l_nchW = 0;            // ... and the window chunks it scans
    int64_t l_qoff = 0;
    int32_t *pos_of[2] = {nullptr, nullptr};
    bool pos_ok = false;       // pos_of[qcur] is exact for every queued slot (general ticks do not keep it)
    // k_emit_win: per front / back list entry, the committed position of the queued slot it
    // moved (-1: none), read by the tick's commit
    int32_t *tomb = nullptr;
    int32_t *bad_min = nullptr;  // device word: first invalid message of a device-checked batch (0x7f7f7f7f: none)
    unsigned long long *wlb = nullptr;  // k_emit_win's look-back granules
    uint32_t *wticket = nullptr;
    int64_t *cw = nullptr;  // commit word of the launched tick (device; eager commits read it)
    uint32_t *lpart = nullptr, *wpart = nullptr;
    uint32_t *died_tag = nullptr;  // window ticks: the launch stamp of the last tick a registration died in
    int64_t win_slack = 8192;  // window positions scanned beyond the tasks' estimate (grows on a miss)
    int64_t last_O = 0;
    int last_L = -1;
    int64_t win_ticks = 0, win_fallbacks = 0;
    bool evict_ok = false;     // the waited window tick's dense evicted list is built
    bool win_owned = false;    // window buffers allocated by fb_set_window (one allocation)
    void *win_mem = nullptr;
    uint32_t tick = 1;
    // per-tick sparse post-message records
    uint32_t *touched = nullptr;
    uint32_t *tbits = nullptr;   // one GPU, heartbeat loop: touched bitmap of this launch (tbitsb[tick & 1])
    uint32_t *tbitsb[2] = {nullptr, nullptr};  // by launch parity: a deferred commit reads the last tick's
    // fb_tick_commit of a one-GPU heartbeat context is deferred into the next launch's
    // k_ev_link (extra blocks) or flushed as its own launch by the next call that needs it
    bool cm_pending = false;
    CommitArgs cm{};
    int cm_grid = 0;
    int eager = 0;             // fb_set_eager_commit: window ticks commit on the device right behind the tick
    bool l_eager = false;      // the launched tick's eager commit is enqueued (until a rerun cancels it)
    PostRec *post = nullptr;       // post-message records {hb, free, epoch} of touched slots
    uint8_t *post_rf = nullptr, *st = nullptr;
    unsigned long long *dmask = nullptr;
    // events
    uint8_t *ev_kind = nullptr, *ev_status = nullptr;
    int32_t *ev_val = nullptr, *ev_slot = nullptr;
    double *ev_ts = nullptr;
    int64_t *ev_seq = nullptr;
    uint32_t *keys[2] = {nullptr, nullptr}, *vals[2] = {nullptr, nullptr};
    uint32_t *rs_hist[4] = {nullptr, nullptr, nullptr, nullptr};  // per sort pass: [tile][digit] counts
    int32_t *front_list = nullptr, *back_list = nullptr;
    // one GPU, heartbeat loop: messages grouped per slot by linked lists (k_ev_link)
    unsigned long long *ev_head = nullptr;  // per slot {link stamp, last linked message}
    int32_t *ev_next = nullptr;             // per message
    uint32_t link = 0;                      // stamp of the last k_ev_link launch
    int ev_ll = 1;                          // fb_set_path("ev_ll", 0): always the radix sort (test paths)
    bool l_resort = false;                  // this tick reruns through the sort (a slot had > kLinkMax messages)
    bool l_used_ll = false;                 // the last enqueue grouped by linked lists
    void *h_stage = nullptr;  // two pinned halves of E_cap events each (fb_tick_stage)
    // device event arrays, double-buffered like the pinned halves: fb_tick_stage copies
    // half h on its own stream (overlapping a running tick), the launch waits for it
    uint8_t *evk[2] = {nullptr, nullptr};
    int32_t *evsl[2] = {nullptr, nullptr}, *evv[2] = {nullptr, nullptr};
    double *evt[2] = {nullptr, nullptr};
    int64_t *evq[2] = {nullptr, nullptr};
    hipStream_t cp_s = nullptr;                         // H2D copies of staged events
    hipEvent_t stage_ev[2] = {nullptr, nullptr};        // copies of half h done (on cp_s)
    hipEvent_t tick_ev = nullptr;                       // an eagerly committed tick's last kernel done
    bool tick_ev_set = false;                           // ... signalled by that kernel's launch itself
    hipEvent_t use_ev[2] = {nullptr, nullptr};          // the tick reading device half h done
    bool stage_rec[2] = {false, false}, use_rec[2] = {false, false};
    int stage_half = 1;        // half of the last launch's copies
    bool staged = false;       // fb_tick_stage done, fb_tick_launch_staged not yet
    int32_t st_E = 0, st_vmax = 0;
    double st_now = 0.0;
    HostPool *pool = nullptr;  // staging workers (FAASBAL_STAGE_THREADS, default 8; 1 = none)
    // a staged pinned batch k_ev_link checks: the caller's kind / slot / ts arrays (read by
    // the host only to name an offending event), and those of the launched tick
    const void *st_chk[3] = {nullptr, nullptr, nullptr};
    const void *l_chk[3] = {nullptr, nullptr, nullptr};
    // device-resident batches (fb_tick_stage of arrays in this GPU's memory): read in place
    bool st_res = false, l_res = false;
    const void *st_dev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    // scan / plan / emit
    int32_t *c_arr = nullptr, *qbmax = nullptr, *qbm_raw = nullptr;
    unsigned long long *csum = nullptr;
    uint8_t *ofl = nullptr;
    uint32_t *fcnt = nullptr, *wcnt = nullptr;
    int64_t *fpre = nullptr, *wpre = nullptr;
    uint32_t *qcnt = nullptr;
    uint32_t *segcnt = nullptr;  // fused path: per-segment round counts (4 x table)
    uint32_t *grp[2] = {nullptr, nullptr};  // fused path: group rows of round totals, by launch parity
    int gpar = 0;                           // parity of the last fused launch
    int gdirty[2] = {0, 0};                 // words of grp[p] written since it was last zeroed
    int64_t *qpre = nullptr, *A = nullptr;
    int64_t *A_rep = nullptr;     // k_plan2 path: per-group copies of A and the totals
    DevTotals *P_rep = nullptr;
    size_t table_cap = 0;  // entries of qcnt / qpre
    int R_cap = 0;         // entries of A
    int64_t *orphans = nullptr;
    int32_t *evicted = nullptr;
    DevTotals *P = nullptr;
    HostOut *hout = nullptr, *hout_dev = nullptr;  // host-mapped results written by k_emit
    unsigned long long *dbg = nullptr;             // diagnostic stamps
    size_t dbg_n = 0;
    // fb_set_path: the launch sequences of other table sizes on small (oracle-checkable)
    // inputs (test paths)
    int force_plan = 0;    // "plan": 1 the k_plan2 + k_emit2 path, 2 the chunked k_emit (R > 128)
    int rs_wide = 1;       // "rs_wide": 0 8-bit sort digits only (the path past kRsWideMaxBlocks tiles)
    int logscan = -1;      // "logscan": -1 auto (k_logscan for large tables when the bitmap fits in LDS)
    int ncu = 0, max_lds = 0;
    int win_occ = 0;       // k_emit_win workgroups resident per CU (occupancy calculator)
    int split_slots = -1;  // "split_slots": -1 auto (separate k_slots launch once the records outgrow L2)
    // "fault_qlen": the next fb_tick_wait overwrites the device-reported queue length with this
    // value before validating it (tests of check_lengths; -1 = off)
    int64_t fault_qlen = -1;
    // deque contexts (fb_create_deque): PushDispatcher.start, task_dispatcher.py:251-322
    int deque = 0;
    int32_t *tokcnt[2] = {nullptr, nullptr}, *xw[2] = {nullptr, nullptr}, *kl[2] = {nullptr, nullptr};
    uint32_t *qrank[2] = {nullptr, nullptr};
    int32_t *front_rank = nullptr, *back_rank = nullptr, *post_tok = nullptr, *post_nf = nullptr;
    int4 *c_tok = nullptr;
    void *arena = nullptr;    // every fixed-size device buffer, carved from one allocation
    size_t arena_bytes = 0;
    bool table_owned = false; // qcnt/qpre grown beyond the arena's reservation
    bool A_owned = false;
    size_t seg_cap = 0;       // entries (per row of 4) of segcnt and the sharded ocnt/opre/osegcnt
    bool seg_owned = false;
    int oA_cap = 0;
    bool oA_owned = false;
    // last launch
    bool launched = false, waited = false;
    double l_now = 0, l_tte = 0;
    int32_t l_E = 0;
    bool l_purge_only = false;  // fb_purge_launch: orphans reported, not dispatched
    bool next_purge_only = false;
    int64_t l_T = 0, l_head = 0, l_Qn = 0;
    int l_R = 64;
    int32_t maxc_hint = 1;
    int reruns = 0;
    fb_tick_result last{};
    // timing
    bool timing = false;
    std::vector<TimedLaunch> tl;
    std::vector<hipEvent_t> ev_pool;
    // fb_timing_gate: a host-mapped word {open sequence, timed out} the gate kernel polls,
    // the gate's end and the batch's end
    uint32_t *gate_h = nullptr, *gate_d = nullptr;
    uint32_t gate_seq = 0;
    hipEvent_t gate_a = nullptr, gate_b = nullptr;
    int gate_state = 0;  // 1 held, 2 released (span readable)
    std::string err;
    // sharding (fb_create_sharded): this rank owns global slots [slot_base, slot_base + W)
    int shard = 0, rank = 0, world = 1;
    int32_t slot_base = 0, W_global = 0, Wq_cap = 0;  // Wq_cap: LRU queue capacity (global slots)
    int64_t head_local = 0, l_head_local = 0;
    uint32_t *lseq = nullptr;                         // global sequence of each local log entry
    uint32_t *ocnt = nullptr, *osegcnt = nullptr;
    uint32_t *xg_acc = nullptr, *xg_tk = nullptr, *ogrp = nullptr;  // exchanged group rows (phase 1 -> 2)
    uint32_t *xs_tk = nullptr;                        // k_xscan's ticket
    int gp_on = 1;                                    // fb_set_path("gp", 0): large one-GPU tables run k_plan2
    int win_direct = 1;                               // fb_set_path("win_direct", 0): k_emit_win chunks by ticket
    int xself_on = 1;                                 // fb_set_path("xself", 0): k_xscan's last workgroup prefixes the chunks
    int wfirst_on = 1;                                // fb_set_path("wfirst", 0): phase-1 k_scan queue blocks first
    int gpcheck = 0;                                  // fb_set_path("gpcheck", 1): diagnostic (stamps builds)
    int cmix_on = 1;                                  // fb_set_path("cmix"): k_emit2 role interleave
    int wtiles = 0;                                   // fb_set_path("wtiles"): slot tiles per k_scan W workgroup (0 auto)
    int qtiles = 0;                                   // fb_set_path("qtiles"): 1 = one queue block per k_scan Q workgroup (0 auto: 4)
    int lazy_on = 1;                                  // fb_set_path("lazy", 0): commits clear their orphaned log entries
    bool stale_any = false;                           // lazy clears: entries of dead registrations may be in the log
    int xcfirst_on = 1;                               // fb_set_path("xcfirst", 0): k_emit_shard_xp's compaction workgroups last
    int xplan_on = 1;                                 // fb_set_path("xplan", 0): large queues take the phase-2 k_scan path
    int full_assign = 0;                              // fb_set_full_assign: phase 2 writes the whole task -> slot array
    bool l_full = false;                              // ... and the last launch did
    int32_t *assign_all = nullptr;                    // (its own allocation, grown as ticks need)
    int64_t assign_cap = 0;
    int64_t *opre = nullptr, *oA = nullptr;
    uint8_t *xbuf = nullptr;                          // bound exchange buffer (device)
    int64_t xcap = 0;
    // the exchange records' copy the next phase 1 writes (two, by exchange parity: a phase 2
    // with block rows zeroes the other and flips it -- a collective step, so every rank
    // agrees), and whether that copy is known zero (then an idle tick's phase 1 needs no memset)
    int xpar = 0;
    bool xz_ok = false;
    int phase = 0;                                    // 1: phase 1 enqueued; 2: phase 2 enqueued
    int shard_R = 0;                                  // > 0: round rows a relaunch asked for (FB_ERERUN)
    hipStream_t own_s = nullptr;                      // the context's own stream (fb_set_stream may borrow another)
};

namespace {

int fail(fb_ctx *c, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define HIPCHK(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail((ctx), FB_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),    \
                        __FILE__, __LINE__);                                                      \
    } while (0)

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int round_up(int v, int m) { return (v + m - 1) / m * m; }

template <typename T>
int dalloc(fb_ctx *c, T **p, size_t n) {
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void **)p, n * sizeof(T));
    if (e != hipSuccess) return fail(c, FB_ENOMEM, "hipMalloc(%zu B) failed: %s", n * sizeof(T), hipGetErrorString(e));
    return FB_OK;
}

// One device allocation for every fixed-size buffer: random per-slot gathers then
// stay within large, contiguous mappings (fewer GPU TLB misses than many small
// hipMalloc regions).
struct ArenaPlan {
    std::vector<std::pair<void **, size_t>> req;
    template <typename T>
    void add(T **p, size_t n) {
        req.push_back({(void **)p, std::max<size_t>(n, 1) * sizeof(T)});
    }
};

// Buffer i starts (i mod 16) x 4.25 KB after the end of buffer i - 1, so arrays read by
// position side by side (c_arr, c_hb, queue, qfree, qhb: power-of-two sizes at 1 M
// workers) do not start at the same offset modulo the memory channel interleave
size_t arena_skew(int i) { return (size_t)(i % 16) * 4352; }

// The host's wait for the context stream: polled (a tick is tens of microseconds; a
// blocking wait's wake-up was measured at ~20 us per tick, tools/stream_timeline.sh)
static hipError_t stream_wait(fb_ctx *c) {
    for (;;) {
        const hipError_t e = hipStreamQuery(c->stream);
        if (e != hipErrorNotReady) return e;
    }
}

int arena_commit(fb_ctx *c, ArenaPlan &ap) {
    size_t total = 0;
    int i = 0;
    for (auto &r : ap.req) total += ((r.second + 255) & ~(size_t)255) + arena_skew(i++);
    total = (total + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
    hipError_t e = hipMalloc(&c->arena, total);
    if (e != hipSuccess) return fail(c, FB_ENOMEM, "hipMalloc(arena %zu B) failed: %s", total, hipGetErrorString(e));
    c->arena_bytes = total;
    // Every byte written once: some kernels load words no tick has written yet (a
    // round table's rows past the fill level, tail padding) and discard them; zeroing
    // makes those loads deterministic.
    e = hipMemset(c->arena, 0, total);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) return fail(c, FB_EHIP, "hipMemset(arena) failed: %s", hipGetErrorString(e));
    char *p = (char *)c->arena;
    i = 0;
    for (auto &r : ap.req) {
        p += arena_skew(i++);
        *r.first = p;
        p += (r.second + 255) & ~(size_t)255;
    }
    return FB_OK;
}

hipEvent_t pool_event(fb_ctx *c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

// Per-kernel device time: the events ride in the dispatch packets of the timed
// launches (start of the first, end of the last), so they bracket kernel
// execution only -- the same interval rocprofv3's kernel trace reports.
struct Timer {
    fb_ctx *c;
    const char *name;
    hipEvent_t a = nullptr, b = nullptr;
    Timer(fb_ctx *c_, const char *n) : c(c_), name(n) {
        if (c->timing) {
            a = pool_event(c);
            b = pool_event(c);
        }
    }
    Stream st() const { return Stream(c->stream, a, b); }
    Stream first() const { return Stream(c->stream, a, nullptr); }
    Stream mid() const { return Stream(c->stream); }
    Stream last() const { return Stream(c->stream, nullptr, b); }
    ~Timer() {
        if (c->timing) c->tl.push_back({name, a, b});
    }
};

int ensure_table(fb_ctx *c, int R, int nbq) {
    size_t need = (size_t)R * (size_t)nbq;
    if (need > c->table_cap) {
        size_t cap = std::max(need, c->table_cap * 2);
        if (cap > ((size_t)1 << 31))
            return fail(c, FB_ERANGE, "round table of %zu entries (R=%d rows x %d blocks) exceeds the limit", need, R, nbq);
        HIPCHK(c, stream_wait(c));
        if (c->table_owned) {
            hipFree(c->qcnt);
            hipFree(c->qpre);
        }
        c->qcnt = nullptr;
        c->qpre = nullptr;
        int rc;
        if ((rc = dalloc(c, &c->qcnt, cap)) || (rc = dalloc(c, &c->qpre, cap))) return rc;
        HIPCHK(c, hipMemset(c->qcnt, 0, cap * sizeof(uint32_t)));
        HIPCHK(c, hipMemset(c->qpre, 0, cap * sizeof(int64_t)));
        c->table_cap = cap;
        c->table_owned = true;
    }
    if (R > c->R_cap) {
        HIPCHK(c, stream_wait(c));
        if (c->A_owned) hipFree(c->A);
        c->A = nullptr;
        int rc;
        if ((rc = dalloc(c, &c->A, (size_t)R))) return rc;
        c->R_cap = R;
        c->A_owned = true;
    }
    // per-segment round counts (4 rows per block) and, sharded, this rank's tables: the
    // arena holds them for 128 rows; wider sharded tables get their own, grown the same way
    if (c->shard && need > c->seg_cap) {
        const size_t cap = std::max(need, c->seg_cap * 2);
        HIPCHK(c, stream_wait(c));
        if (c->seg_owned) {
            hipFree(c->segcnt);
            hipFree(c->osegcnt);
            hipFree(c->ocnt);
            hipFree(c->opre);
        }
        c->segcnt = c->osegcnt = c->ocnt = nullptr;
        c->opre = nullptr;
        int rc;
        if ((rc = dalloc(c, &c->segcnt, 4 * cap))) return rc;
        if (c->shard && ((rc = dalloc(c, &c->osegcnt, 4 * cap)) || (rc = dalloc(c, &c->ocnt, cap)) ||
                         (rc = dalloc(c, &c->opre, cap))))
            return rc;
        c->seg_cap = cap;
        c->seg_owned = true;
    }
    if (c->shard && R > c->oA_cap) {
        HIPCHK(c, stream_wait(c));
        if (c->oA_owned) hipFree(c->oA);
        c->oA = nullptr;
        int rc;
        if ((rc = dalloc(c, &c->oA, (size_t)R))) return rc;
        c->oA_cap = R;
        c->oA_owned = true;
    }
    return FB_OK;
}

// Exchange buffer of a sharded tick, summed by one uint8 all-reduce: every byte
// has at most one nonzero contributor (the owner of the slot, event or position),
// so the SUM is exact -- except the block rows, whose bytes are 4-bit digits that at
// most kXRowsMaxWorld ranks add (<= 240).  [rec, c8) -- two copies of the per-rank
// records (by launch parity), the event regions -- is zero before phase 1 (a memset, or
// for an idle tick the previous phase 2's zeroing of this parity's records); c8 and the
// rows are written in full.
struct XLayout {
    size_t rec, front, back, evs, c8, rows, grows, total;
};
// The phase-2 form of a sharded tick of this shape: 0 phase 2 re-counts the exchanged c
// values (k_scan) -- > 16 ranks or a table wider than kRFused rows; 1 phase 1 exchanges
// its per-block round counts as digit rows, a one-launch phase 2 sums them (<= kXRowsMaxBlocks
// queue blocks); 2 (xplan; larger queues, R = kXGroupR, configs[3]: 3.5 K blocks) the same
// digit rows, whose per-block prefixes k_xscan scans before k_emit_shard
inline int xrows_mode(int world, int R, int64_t Qlog) {
    const int64_t nbq = std::max<int64_t>(1, cdiv(Qlog, kBS));
    if (world > kXRowsMaxWorld || world * kXRecLines > kBS || R > kRFused) return 0;
    // (the one-launch phase 2 walks the digit rows and this rank's rows in the same rounds:
    // their parts per column must agree, as they do for the 32 / 64 / 128-row tables)
    if (nbq <= kXRowsMaxBlocks && xr_parts(R) == kBS / (R / 4)) return 1;
    return (nbq > kXRowsMaxBlocks && R == kXGroupR) ? 2 : 0;  // (k_xscan decodes 32-round rows)
}
inline size_t xrows_bytes(int world, int R, int64_t Qlog) {
    const int64_t nbq = std::max<int64_t>(1, cdiv(Qlog, kBS));
    return xrows_mode(world, R, Qlog) ? (size_t)nbq * xr_row(R) : 0;
}
// ... and the group rows (one-launch form, R = kXGroupR only)
inline size_t xgrows_bytes(int world, int R, int64_t Qlog) {
    if (R != kXGroupR || xrows_mode(world, R, Qlog) != 1) return 0;
    const int64_t nbq = std::max<int64_t>(1, cdiv(Qlog, kBS));
    return (size_t)cdiv(nbq, kXGroupBlocks) * xg_row(R);
}
// xcw: bytes per exchanged c (1 while the round table has <= kRFused rows, else 2)
XLayout xlayout(int world, int64_t E, int64_t Qlog, int xcw = 1, size_t rows = 0, size_t grows = 0) {
    XLayout x;
    x.rec = 0;
    x.front = (size_t)2 * 8 * kXRecWords * world;
    x.back = x.front + 4 * (size_t)E;
    x.evs = x.back + 4 * (size_t)E;
    x.c8 = (x.evs + (size_t)E + 1) & ~(size_t)1;  // 2-byte aligned for the wide form
    x.rows = (x.c8 + (size_t)xcw * (size_t)Qlog + 15) & ~(size_t)15;
    x.grows = (x.rows + rows + 15) & ~(size_t)15;
    x.total = (x.grows + grows + 15) & ~(size_t)15;
    return x;
}
inline int xc_width(int R) { return R > kRFused ? 2 : 1; }

int choose_R(int32_t maxc) {
    int R = 32;
    while (R < maxc) R <<= 1;
    return R;
}

// The committed window [qoff, qoff + Qn) without its tombstones: slots, free counts and
// (h non-null) heartbeats on the host.  The stream must be idle.
int win_read(fb_ctx *c, std::vector<int32_t> &q, std::vector<int32_t> &f, std::vector<double> *h, int64_t &n) {
    const size_t Qn = (size_t)c->Qn;
    std::vector<int32_t> q0(Qn), f0(Qn);
    std::vector<double> h0(h ? Qn : 0);
    if (Qn) {
        HIPCHK(c, hipMemcpy(q0.data(), c->queue[c->qcur] + c->qoff, Qn * 4, hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(f0.data(), c->qfree[c->qcur] + c->qoff, Qn * 4, hipMemcpyDeviceToHost));
        if (h) HIPCHK(c, hipMemcpy(h0.data(), c->qhb[c->qcur] + c->qoff, Qn * 8, hipMemcpyDeviceToHost));
    }
    q.clear();
    f.clear();
    if (h) h->clear();
    for (size_t i = 0; i < Qn; ++i)
        if (f0[i] != kTomb) {
            q.push_back(q0[i]);
            f.push_back(f0[i]);
            if (h) h->push_back(h0[i]);
        }
    n = (int64_t)q.size();
    if (n != c->Qtrue) return fail(c, FB_EHIP, "window holds %lld live entries, the queue %lld", (long long)n, (long long)c->Qtrue);
    return FB_OK;
}

// Rewrite the committed window densely from position 0 of the other buffers (the state a
// general tick leaves): for readers of the device view.
int win_normalize(fb_ctx *c) {
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    std::vector<int32_t> q, f;
    std::vector<double> h;
    int64_t n = 0;
    if (int rc = win_read(c, q, f, &h, n)) return rc;
    const int o = c->qcur ^ 1;
    if (n) {
        HIPCHK(c, hipMemcpy(c->queue[o], q.data(), (size_t)n * 4, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->qfree[o], f.data(), (size_t)n * 4, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->qhb[o], h.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    }
    if (c->W) {
        std::vector<int32_t> pos((size_t)c->W, 0);
        for (int64_t i = 0; i < n; ++i) pos[q[i]] = (int32_t)i;
        HIPCHK(c, hipMemcpy(c->pos_of[o], pos.data(), (size_t)c->W * 4, hipMemcpyHostToDevice));
    }
    c->qcur = o;
    c->qoff = 0;
    c->Qn = n;
    c->pos_ok = true;
    return FB_OK;
}

// Window buffers for a context created without them (fb_set_window): one allocation,
// the committed queue copied over.
int win_alloc(fb_ctx *c) {
    if (c->win_cap) return FB_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    const size_t W = (size_t)c->W_cap, E = (size_t)c->E_cap, Wq = (size_t)c->Wq_cap;
    const size_t qcap = 2 * Wq + 2 * E + 4096;
    auto r256 = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t bytes = 2 * (r256(qcap * 4) * 2 + r256(qcap * 8) + r256(W * 4)) + r256(2 * E * 4) +
                         r256(kWinMaxCh * 8) +
                         r256(256) + r256(1024 * 4) + r256(256) + r256(64 * 32 * 4);
    void *m = nullptr;
    hipError_t e = hipMalloc(&m, bytes);
    if (e != hipSuccess) return fail(c, FB_ENOMEM, "hipMalloc(window buffers %zu B) failed: %s", bytes, hipGetErrorString(e));
    HIPCHK(c, hipMemset(m, 0, bytes));
    char *p = (char *)m;
    auto take = [&](size_t b) { char *r = p; p += r256(b); return r; };
    int32_t *nq[2], *nf[2];
    double *nh[2];
    for (int i = 0; i < 2; ++i) {
        nq[i] = (int32_t *)take(qcap * 4);
        nf[i] = (int32_t *)take(qcap * 4);
        nh[i] = (double *)take(qcap * 8);
        c->pos_of[i] = (int32_t *)take(W * 4);
    }
    c->tomb = (int32_t *)take(2 * E * 4);
    c->wlb = (unsigned long long *)take(kWinMaxCh * 8);
    c->wticket = (uint32_t *)take(256);
    c->lpart = (uint32_t *)take(1024 * 4);
    c->died_tag = (uint32_t *)take(256);
    c->wpart = (uint32_t *)take(64 * 32 * 4);
    const int k = c->qcur;
    if (c->Qn) {
        HIPCHK(c, hipMemcpy(nq[0], c->queue[k], (size_t)c->Qn * 4, hipMemcpyDeviceToDevice));
        HIPCHK(c, hipMemcpy(nf[0], c->qfree[k], (size_t)c->Qn * 4, hipMemcpyDeviceToDevice));
        HIPCHK(c, hipMemcpy(nh[0], c->qhb[k], (size_t)c->Qn * 8, hipMemcpyDeviceToDevice));
    }
    for (int i = 0; i < 2; ++i) {
        c->queue[i] = nq[i];
        c->qfree[i] = nf[i];
        c->qhb[i] = nh[i];
    }
    c->qcur = 0;
    c->qoff = 0;
    c->qcap = (int64_t)qcap;
    c->win_mem = m;
    c->win_owned = true;
    c->win_cap = true;
    c->pos_ok = true;
    if (c->W && c->Qn) {
        std::vector<int32_t> q((size_t)c->Qn), pos((size_t)c->W, 0);
        HIPCHK(c, hipMemcpy(q.data(), c->queue[0], (size_t)c->Qn * 4, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < c->Qn; ++i) pos[q[i]] = (int32_t)i;
        HIPCHK(c, hipMemcpy(c->pos_of[0], pos.data(), (size_t)c->W * 4, hipMemcpyHostToDevice));
    }
    return FB_OK;
}

// A launched window tick moves the committed window (its commit may already have run on
// the device, eager) while the host's view of it changes only at fb_tick_commit: state
// reads wait for that commit.
int win_uncommitted(fb_ctx *c, const char *what) {
    if (c->launched && c->l_win)
        return fail(c, FB_ESTATE, "%s between the launch and the commit of a window tick: fb_tick_commit first", what);
    return FB_OK;
}

// The deferred commit of the last tick as its own launch (when no k_ev_link takes it).
int flush_commit(fb_ctx *c) {
    if (!c->cm_pending) return FB_OK;
    c->cm_pending = false;
    HIPCHK(c, hipSetDevice(c->device));
    Timer t(c, "commit");
    launch_commit(c->cm, c->cm_grid, t.st());
    HIPCHK(c, hipGetLastError());
    return FB_OK;
}

// Lazy clears (round 6): on one-GPU heartbeat contexts a commit leaves the log entries it
// redistributed; an entry naming slot s is live only if s holds a record and the entry is
// not older than s's registration (epoch), which every kernel that reads the log tests once
// such entries may exist (live_chk).  (configs[3]: the fold's ~380 K scattered clears cost
// 2.9 µs of the committed tick; configs[2]'s 24.6 K, ~0.5 µs.)
bool lazy_ctx(const fb_ctx *c) { return c->lazy_on && !c->shard && !c->deque; }

// Before a state read hands out the log: the deferred clears, all at once (k_log_normalize),
// after the last commit.
int log_settle(fb_ctx *c) {
    if (!c->stale_any) return FB_OK;
    if (int rc_ = flush_commit(c)) return rc_;
    HIPCHK(c, hipSetDevice(c->device));
    launch_log_normalize(c->log_slot, c->head, c->reg, c->epoch, Stream(c->stream, nullptr, nullptr));
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, stream_wait(c));
    c->stale_any = false;
    return FB_OK;
}

// Whether the tick about to launch runs as a window tick, and how much of
// the window it scans: the tasks (T plus about the last tick's orphans), the positions
// between them that are no longer live, a slack that grows whenever a window tick missed
// its first unserved element.  Only level-0 ticks qualify (the last tick was one), with
// messages (the purge rides in k_ev_apply_ll's launch), on the linked-list path.
bool win_plan(fb_ctx *c) {
    const int mode = c->win;
    if (!c->win_cap || mode == 0 || c->l_E <= 0 || !c->ev_head || !c->ev_ll || c->compact ||
        c->l_purge_only || c->deque || c->shard)
        return false;
    if (mode < 0 && c->last_L != 0) return false;  // auto: after a level-0 tick
    if (mode > 0 && c->last_L > 0) return false;
    const int64_t want = (c->l_T + 2 * c->last_O + 256) * 5 / 4 + c->win_slack;
    const int64_t scan = std::min<int64_t>(c->Qn, want);
    if (mode < 0 && scan * 2 > c->Qn) return false;  // auto: only when most of the queue stays put
    const int nchW = (int)cdiv(scan, kWinCh);
    if (nchW == 0) return false;
    if ((size_t)((c->W + 63) / 64 + 2) * 8 > (size_t)c->max_lds) return false;  // k_logscan's bitmap in LDS
    const int nchB = (int)cdiv(c->l_E, kWinCh);
    if (2 * nchB + nchW > kWinMaxCh) return false;
    // room for the appends (backs, served workers with c > 1) behind the window
    // (an underestimate only costs a rerun: k_emit_win flags a store past the buffer)
    if (c->qoff + c->Qn + (int64_t)c->l_E + c->l_T + c->last_O + 1024 > c->qcap) return false;
    c->l_nchW = nchW;
    return true;
}

// Enqueue every kernel of the tick described by c->l_* (events already on device).
int enqueue_tick(fb_ctx *c) {

    const int E = c->l_E;
    const int W = c->W;
    const int R = c->l_R;
    const int64_t head = c->l_head, Qn = c->l_Qn;
    const int64_t Qlog = Qn + 2 * (int64_t)E;
    const int nbw = (int)std::max<int64_t>(1, cdiv(W, kBS));
    // sharded: the log shard holds head_local entries (head is the global sequence)
    const int nbf = (int)cdiv(c->shard ? c->l_head_local : head, kFTile);
    const int nbq = (int)std::max<int64_t>(1, cdiv(Qlog, kBS));
    int rc;
    if ((rc = ensure_table(c, R, nbq))) return rc;
    const int cur = c->cur, nxt = 1 - cur;
    // (fb_set_path("xplan", 0): large queues re-count in a phase-2 k_scan, no rows)
    const bool xoff = !c->xplan_on && xrows_mode(c->world, R, Qlog) == 2;
    const size_t xrb = (c->shard && !xoff) ? xrows_bytes(c->world, R, Qlog) : 0;
    const size_t xgb = c->shard ? xgrows_bytes(c->world, R, Qlog) : 0;
    const XLayout xl = xlayout(c->world, E, Qlog, xc_width(R), xrb, xgb);
    int32_t *front = c->front_list, *back = c->back_list;
    uint8_t *evs = c->ev_status;
    if (c->shard) {
        if (!c->xbuf || c->xcap < (int64_t)xl.total)
            return fail(c, FB_ESTATE, "sharded tick needs an exchange buffer of %zu bytes (bound: %lld)", xl.total,
                        (long long)c->xcap);
        front = (int32_t *)(c->xbuf + xl.front);
        back = (int32_t *)(c->xbuf + xl.back);
        evs = c->xbuf + xl.evs;
        // (an idle tick whose records the last phase 2 zeroed has nothing else to clear)
        if (c->phase != 2 && !(E == 0 && c->xz_ok)) HIPCHK(c, hipMemsetAsync(c->xbuf, 0, xl.c8, c->stream));
    }
    TickArgs a{};
    // lazy clears: the live test once entries of dead registrations may remain
    a.live_chk = (lazy_ctx(c) && c->stale_any) ? 1 : 0;
    a.epoch = c->epoch;
    a.fault_qlen = -1;
    a.W = W;
    a.E = E;
    a.R = R;
    a.nbw = nbw;
    a.nbf = c->deque ? 0 : nbf;  // start(): nobody dies, no log scan
    a.nbq = nbq;
    a.deque = c->deque;
    a.redist = c->l_purge_only ? 0 : 1;
    a.q_cap = c->Wq_cap;
    a.tokcnt_in = c->tokcnt[cur];
    a.xw_in = c->xw[cur];
    a.kl_in = c->kl[cur];
    a.qrank_in = c->qrank[cur];
    a.front_rank = c->front_rank;
    a.back_rank = c->back_rank;
    a.post_tok = c->post_tok;
    a.post_nf = c->post_nf;
    a.c_tok = c->c_tok;
    a.tokcnt_out = c->tokcnt[nxt];
    a.xw_out = c->xw[nxt];
    a.kl_out = c->kl[nxt];
    a.qrank_out = c->qrank[nxt];
    // small round tables: k_emit derives the cross-block prefixes itself (2 launches per tick)
    // fused: k_emit2 reduces the (small) round table in every block, no k_plan launch
    a.fused = (!c->shard && !c->force_plan && R <= kRFused && (int64_t)nbq * R <= (int64_t)kTabLd * kBS * 4) ? 1 : 0;
    // large tables with R <= 128: k_emit2 after k_plan (fb_set_path("plan", 2): the chunked k_emit)
    a.segw = (!c->shard && R <= kRFused && c->force_plan != 2) ? 1 : 0;
    // large tables for k_emit2: group rows too, scanned by k_plan2
    const bool gplan = !a.fused && a.segw && !c->shard;
    // sharded phase 2 with a round table of <= 128 rows: group rows instead of k_plan
    const bool sgrp = c->shard && c->phase == 2 && R <= kRFused && !xrb;
    if ((a.fused || gplan || sgrp) && !c->l_win) {  // (a window tick uses no group rows)
        // group rows: fused / sharded, about sqrt(nbq) groups of 2^gshift queue blocks (the
        // emit reads both); k_plan2, the smallest groups that make at most 64 rows (one
        // workgroup each)
        int gs = 0;
        if (a.fused || sgrp)
            while ((1 << (2 * gs)) < nbq || cdiv(nbq, (int64_t)1 << gs) > 64) ++gs;
        else
            while (cdiv(nbq, (int64_t)1 << gs) > 64) ++gs;
        a.grp_on = 1;
        a.gshift = gs;
        a.gstride = sgrp ? 2 * R + 4 : R + 4;
        a.ngrp = (int)cdiv(nbq, 1 << gs);
        if (a.ngrp > 64 || (int64_t)a.ngrp * a.gstride > kGrpWords)
            return fail(c, FB_ERANGE, "group rows (%d x %d words) exceed the reservation", a.ngrp, a.gstride);
        c->gpar ^= 1;
        a.grp = c->grp[c->gpar];  // zero: its last user's k_emit2 cleared it
        a.grp_zero = c->grp[c->gpar ^ 1];
        a.zero_words = c->gdirty[c->gpar ^ 1];
        c->gdirty[c->gpar ^ 1] = 0;
        c->gdirty[c->gpar] = a.ngrp * a.gstride;
    }
    if (++c->lstamp == 0) c->lstamp = 1;  // every launch (reruns included) stamps its own
    const bool defer = c->bud != nullptr;  // one-GPU heartbeat context
    a.lds_bitmap = W <= kLdsBitmapSlots ? 1 : 0;
    if (defer) {
        a.bud = c->bud;
        a.bud_next = c->bud_next;
        a.post_infl = c->post_infl;
        a.ctag = c->ctag;
        a.lstamp = c->lstamp;
    }
    // the log scan gathers one 16-byte record per in-flight entry; past 128K slots
    // (2 MB of records) those gathers miss L2, so k_slots first writes the
    // died bitmap (W/8 bytes, L2-resident) and the scan tests bits instead
    a.slots_in_scan = (c->split_slots > 0 || (c->split_slots < 0 && W > kLdsBitmapSlots)) ? 0 : 1;
    // ... or better, while the bitmap fits in one workgroup's LDS: the W-role of
    // k_scan writes it and k_logscan tests every entry against an LDS copy
    const size_t bm_bytes = (size_t)(((W + 63) / 64 + 1) / 2 + 1) * 16;
    a.f_sep = (head > 0 && !c->deque && (c->logscan > 0 || (c->logscan < 0 && W > kLdsBitmapSlots)) &&
               bm_bytes <= (size_t)c->max_lds && !(c->shard && c->phase == 2)) ? 1 : 0;
    if (a.f_sep) a.slots_in_scan = 1;
    // fused one-GPU ticks: O from the slot purge's in-flight counts, the orphans flagged
    // and compacted by k_emit2's log workgroups (k_scan without log blocks); not when the
    // log role was asked to run as k_logscan (fb_set_path("logscan", 1))
    const int nbfe = (int)cdiv(nbf, 4);
    const size_t bm16 = (size_t)(((W + 63) / 64 + 1) / 2) * 16;
    a.f_emit = (defer && a.fused && !a.f_sep && W <= kLdsBitmapSlots && nbfe <= kFEmitMaxBlocks &&
                bm16 <= (size_t)c->max_lds && !c->l_win) ? 1 : 0;
    c->l_oseg = a.f_emit != 0 || c->l_win;
    c->l_nbf = nbf;
    c->evict_ok = false;
    c->dense_ok = false;
    const int ls_grid = std::max(1, std::min(c->ncu, (int)cdiv(nbf, kLsBS / 64)));
    c->l_used_ll = false;
    const bool ll = E > 0 && c->ev_head && c->ev_ll && !c->l_resort;
    if (c->l_win && !c->pos_ok) {
        // the first window tick after general ticks: every queued slot's position, once
        launch_pos_rebuild(c->pos_of[c->qcur], c->queue[c->qcur], c->qfree[c->qcur], c->qoff, Qn, Stream(c->stream));
        c->pos_ok = true;
    }
    // the last tick's deferred commit: into this launch's first kernel (k_ev_link below, or
    // k_scan for an idle tick after an idle tick), else as its own launch now
    const bool cm_idle = c->cm_pending && c->cm.E == 0 && !c->cm.win && c->cm.n_clr == 0 && !c->cm.shard;
    if (!ll && !(E == 0 && cm_idle) && (rc = flush_commit(c))) return rc;
    if (ll) {
        // group the messages per slot by linked lists (no sort): two launches
        EvArgs ea{};
        ea.E = E;
        ea.W = W;
        ea.tick = c->tick;
        ea.tte = c->l_tte;
        ea.head_in = head;
        ea.ev_kind = c->ev_kind;
        ea.ev_val = c->ev_val;
        ea.ev_ts = c->ev_ts;
        ea.ev_seq = c->ev_seq;
        ea.ev_status = evs;
        ea.reg = c->reg;
        ea.free_in = c->free_[cur];
        ea.hb = c->hb;
        ea.epoch = c->epoch;
        ea.live_chk = (lazy_ctx(c) && c->stale_any) ? 1 : 0;
        ea.log_slot = c->log_slot;
        ea.post = c->post;
        ea.post_rf = c->post_rf;
        ea.touched = c->touched;
        ea.tbits = c->tbits;
        ea.tbits_words = c->tbits ? (int)cdiv(W, 32) : 0;
        ea.front_list = front;
        ea.back_list = back;
        ea.ev_slot = c->ev_slot;
        ea.ev_head = c->ev_head;
        ea.ev_next = c->ev_next;
        ea.check_ev = c->l_chk[0] != nullptr;
#ifdef FAASBAL_STAMPS
        ea.dbg = c->dbg;
#endif
        ea.bad_min = c->bad_min;
        if (++c->link == 0) c->link = 1;  // a fresh stamp per launch, reruns included
        ea.link = c->link;
        ea.hout = c->hout_dev;
        ea.defer_clr = defer ? 1 : 0;
        ea.ev_clr = c->ev_clr;
        ea.ctag = c->ctag;
        ea.lstamp = c->lstamp;
        ea.bud = c->bud;
        ea.post_infl = c->post_infl;
        ea.bud_next = c->bud_next;
        ea.orph_grp = a.f_emit ? 1 : 0;
        if (c->cm_pending) {  // the previous tick's commit rides in this launch
            ea.cm = c->cm;
            ea.cm_blocks = c->cm_grid;
            c->cm_pending = false;
        }
        // the slot purge (k_scan's W role) runs in k_ev_apply_ll's launch: extra blocks for
        // the untouched slots, each owner thread for its touched slot
        ea.nbw = nbw;
        ea.wtiles = c->wtiles ? c->wtiles : (nbw >= 1024 ? 4 : 1);
        ea.now = c->l_now;
        ea.st = c->st;
        ea.free_out = c->free_[nxt];
        ea.dmask = (!a.slots_in_scan || a.f_sep || a.f_emit || c->l_win) ? c->dmask : nullptr;
        ea.wpart = c->l_win ? c->wpart : nullptr;
        ea.died_tag = c->l_win ? c->died_tag : nullptr;
        if (c->l_win) {  // k_emit_win's look-back granules and ticket start from zero
            ea.wlb = c->wlb;
            ea.wlb_n = 2 * (int)cdiv(E, kWinCh) + c->l_nchW;
            ea.wticket = c->wticket;
            ea.cw = c->cw;
        }
        ea.wcnt = c->wcnt;
        ea.grp = a.grp_on ? a.grp : nullptr;
        ea.ngrp = a.ngrp;
        ea.gstride = a.gstride;
        ea.R = R;
        c->l_used_ll = true;
        {
            Timer t(c, "ev_link");
            launch_ev_link(ea, t.st());
        }
        Timer t(c, "ev_apply");
        launch_ev_apply_ll(ea, t.st());
    } else if (E > 0 && !(c->shard && c->phase == 2)) {

        // stable radix sort of events by slot
        int bits = 1;
        while ((1ll << bits) < (int64_t)(c->shard ? c->W_global : W)) ++bits;
        const int nb = (int)cdiv(E, kRsTile);
        // digits of up to 11 bits while the batch is small enough for the scatter's
        // table walk (1 M workers: two passes of 10 bits instead of three of 8)
        const bool wide = c->rs_wide && nb <= kRsWideMaxBlocks;
        const int passes = wide ? (bits + 10) / 11 : (bits + 7) / 8;
        const int db = wide ? (bits + passes - 1) / passes : 8;
        if (passes > 4) return fail(c, FB_ERANGE, "event sort of %d passes", passes);
        const int NBw = db <= 8 ? 256 : db <= 10 ? 1024 : 2048;
        const uint32_t *kin = (const uint32_t *)c->ev_slot, *vin = nullptr;
        for (int ps = 0; ps < passes; ++ps) {
            Timer t(c, "rs_sort");
            RsPass p{};
            p.kin = kin;
            p.vin = vin;
            p.kout = c->keys[ps & 1];
            p.vout = c->vals[ps & 1];
            p.n = E;
            p.shift = db * ps;
            p.db = db;
            p.nblk = nb;
            p.hist = c->rs_hist[0];
            p.identity_vals = ps == 0 ? 1 : 0;
            if (ps == 0 && !c->shard) {
                // pass 0 also clears the one-GPU front / back lists (sharded: zeroed with the
                // exchange buffer) and the touched bitmap
                p.zero0 = front;
                p.zero1 = back;
                p.zbits = c->tbits;
                p.zwords = c->tbits ? (int)cdiv(W, 32) : 0;
            }
            launch_rs_pass(p, t.first(), t.last());
            kin = p.kout;
            vin = p.vout;
        }
        EvArgs a{};
        a.E = E;
        a.deque = c->deque;
        a.tokcnt_in = c->tokcnt[cur];
        a.front_rank = c->front_rank;
        a.back_rank = c->back_rank;
        a.post_tok = c->post_tok;
        a.post_nf = c->post_nf;
        a.shard = c->shard;
        a.slot_base = c->slot_base;
        a.W = W;
        a.head_local = c->l_head_local;
        a.lseq = c->lseq;
        a.tick = c->tick;
        a.tte = c->l_tte;
        a.head_in = head;
        a.skeys = kin;
        a.svals = vin;
        a.ev_kind = c->ev_kind;
        a.ev_val = c->ev_val;
        a.ev_ts = c->ev_ts;
        a.ev_seq = c->ev_seq;
        a.ev_status = evs;
        a.reg = c->reg;
        a.free_in = c->free_[cur];
        a.hb = c->hb;
        a.epoch = c->epoch;
        a.live_chk = (lazy_ctx(c) && c->stale_any) ? 1 : 0;
        a.log_slot = c->log_slot;
        a.post = c->post;
        a.post_rf = c->post_rf;
        a.touched = c->touched;
        a.tbits = c->tbits;
        a.front_list = front;
        a.back_list = back;
        if (defer) {
            a.defer_clr = 1;
            a.ev_clr = c->ev_clr;
            a.ctag = c->ctag;
            a.lstamp = c->lstamp;
            a.bud = c->bud;
            a.post_infl = c->post_infl;
        }
        Timer t(c, "ev_apply");
        launch_ev_apply(a, t.st());
    }
    a.slots_in_apply = c->l_used_ll ? 1 : 0;
    a.tick = c->tick;
    a.now = c->l_now;
    a.tte = c->l_tte;
    a.Qn = Qn;
    a.Qlog = Qlog;
    a.head_in = head;
    a.T = c->l_T;
    a.log_cap = c->log_cap;
    a.reg = c->reg;
    a.hb = c->hb;
    a.free_in = c->free_[cur];
    // the committed queue: the window [qoff, qoff + Qn) of the current queue buffers
    const int qc = c->qcur, qn = c->qcur ^ 1;
    a.queue_in = c->queue[qc] + c->qoff;
    a.qaos = (!c->shard && c->qaos) ? 1 : 0;
    a.cq_direct = (E == 0 && a.qaos && a.segw && !c->deque) ? 1 : 0;
    a.qfree_in = c->qfree[qc] ? c->qfree[qc] + c->qoff : nullptr;
    a.qhb_in = c->qhb[qc] ? c->qhb[qc] + c->qoff : nullptr;
    a.touched = c->touched;
    a.tbits = c->tbits;
    a.post = c->post;
    a.post_rf = c->post_rf;
    // past the L2-resident sizes the purge is bandwidth-bound: skip untouched post records
    a.post_lazy = W > kLdsBitmapSlots ? 1 : 0;
    a.front_list = front;
    a.back_list = back;
    a.st = c->st;
    a.dmask = c->dmask;
    a.c_arr = c->c_arr;
    a.ofl = c->ofl;
    a.wcnt = c->wcnt;
    a.fcnt = c->fcnt;
    a.qcnt = c->qcnt;
    a.segcnt = c->segcnt;
    a.qbmax = c->qbmax;
    a.qbm_raw = c->qbm_raw;
    a.csum = c->csum;
    a.fpre = c->fpre;
    a.wpre = c->wpre;
    a.qpre = c->qpre;
    a.A = c->A;
    a.P = c->P;
    a.A_rep = c->A_rep;
    a.P_rep = c->P_rep;
    a.repl = gplan ? 1 : 0;  // k_plan2 writes a copy per group
    a.trash = c->trash;
    c->l_compact = c->compact && !c->shard;
    if (c->l_compact) {
        a.rb_slot = c->rb_slot;
        a.rb_c = c->rb_c;
    }
    // registered pinned outputs: the compact form and the evicted slots go straight to the
    // host (fused ticks, whose orphans a gather launch after the emission sends there too)
    c->l_cout = c->l_compact && c->cout_slot && a.fused && a.f_emit && Qlog <= c->cout_cap && W <= c->cout_ecap &&
                head <= c->cout_ocap;
    if (c->l_cout) {
        a.rb_slot = c->cout_slot;
        a.rb_c = c->cout_c;
    }
    a.arena = (char *)c->arena;
    a.arena32 = c->arena_bytes < ((size_t)1 << 32) ? 1 : 0;
    a.log_slot = c->log_slot;
    a.free_out = c->free_[nxt];
    a.queue_out = c->queue[qn];
    a.qfree_out = c->qfree[qn];
    a.qhb_out = c->qhb[qn];

    a.c_hb = c->c_hb;
    a.orphans = c->orphans;
    // (registered pinned outputs: the evicted slots straight into the caller's array)
    a.evicted = c->l_cout ? c->cout_ev : c->evicted;
    a.hout = c->hout_dev;
    if (c->shard) {
        a.shard = c->phase == 2 ? 2 : 1;
        // (only while the log role is fused into k_scan: with k_logscan the slot blocks are
        // the short ones)
        a.wfirst = (a.shard == 1 && !a.f_sep && c->wfirst_on) ? 1 : 0;
        // sharded phase 1: 4 slot tiles per workgroup while the log role has its own launch
        // (N = 2 at configs[3]: scan 18.4 -> 17.8 us), 1 behind wfirst (N = 8: no gain)
        if (a.shard == 1) a.wtiles = c->wtiles ? c->wtiles : (a.wfirst ? 1 : 4);
        a.slot_base = c->slot_base;
        a.rank = c->rank;
        a.world = c->world;
        a.head_local = c->l_head_local;
        a.lseq = c->lseq;
        a.lseq_out = c->lseq;
        a.xc8 = c->xbuf + xl.c8;
        a.xcw = xc_width(R);
        // this tick's copy of the records; phase 2 with block rows zeroes the other
        const size_t xrw = (size_t)c->world * kXRecWords;
        a.xrec = (unsigned long long *)(c->xbuf + xl.rec) + (size_t)c->xpar * xrw;
        a.xrows = xrb ? c->xbuf + xl.rows : nullptr;
        a.xplan = (c->xplan_on && xrows_mode(c->world, R, Qlog) == 2) ? 1 : 0;
        // (<= 64 chunks of kXsBlocks queue blocks: 16 loads per k_emit_shard_xp thread)
        a.xself = (a.xplan && c->xself_on && cdiv(Qlog, kBS) <= 64 * kXsBlocks) ? 1 : 0;
        // k_emit_shard_xp's compaction workgroups first when they are many (configs[3], N = 2:
        // 975 beside 1 774 queue workgroups, emit 30.3 -> 26.9 us; N = 8: 244, no gain)
        a.xcfirst = (a.xplan && c->xcfirst_on &&
                     4 * ((a.nbf + 3) / 4 + (a.nbw + 3) / 4) > (nbq + 1) / 2) ? 1 : 0;
        c->l_full = c->full_assign != 0;
        if (c->l_full && c->phase == 2) {
            // the whole tick's assignments: at most its pending tasks plus every in-flight entry
            const int64_t need = std::max<int64_t>(1, c->l_T + head);
            if (need > c->assign_cap) {
                const int64_t cap = std::max(need, 2 * c->assign_cap);
                HIPCHK(c, stream_wait(c));
                hipFree(c->assign_all);
                c->assign_all = nullptr;
                c->assign_cap = 0;
                if ((rc = dalloc(c, &c->assign_all, (size_t)cap))) return rc;
                c->assign_cap = cap;
            }
            a.assign_all = c->assign_all;
        }
        if (a.xplan) {
            // k_xscan's outputs in the plan tables (unused on this path): per-block prefixes in
            // qpre's words, the chunk prefixes and totals in opre's
            a.xpre = reinterpret_cast<uint32_t *>(c->qpre);
            a.xct = reinterpret_cast<uint32_t *>(c->opre);
            a.xA = a.xct + (size_t)cdiv(nbq, kXsBlocks) * 2 * R;
            a.xtk = c->xs_tk;
        }
        a.xgrows = xgb ? c->xbuf + xl.grows : nullptr;
        a.xg_acc = c->xg_acc;
        a.xg_tk = c->xg_tk;
        a.ogrp = c->ogrp;
        if ((xrb || a.xplan) && c->phase == 2) {
            a.xz = (unsigned long long *)(c->xbuf + xl.rec) + (size_t)(c->xpar ^ 1) * xrw;
            a.xz_words = (int)xrw;
        }
        a.ocnt = c->ocnt;
        a.osegcnt = c->osegcnt;
        a.opre = c->opre;
        a.oA = c->oA;
    }
#ifdef FAASBAL_STAMPS
    {
        // diagnostic stamp rows (stamps builds only); grown geometrically -- hipFree
        // synchronises the device
        // (k_emit_win stamps rows from 8192 on, one per chunk)
        const size_t need = std::max((size_t)4 * (nbw + nbf + nbq) * 16 + 16, (size_t)(8192 + kWinMaxCh) * 16);
        if (need > c->dbg_n) {
            HIPCHK(c, stream_wait(c));
            hipFree(c->dbg);
            c->dbg = nullptr;
            const size_t cap = std::max(need, 2 * c->dbg_n);
            if ((rc = dalloc(c, &c->dbg, cap))) return rc;
            c->dbg_n = cap;
        }
        a.dbg = c->dbg;
    }
#endif
    if (c->l_win) {
        // window tick (E > 0, purge in the apply launch): k_logscan writes the orphans into
        // per-tile segments and a partial count per workgroup (nothing, when no registration
        // died: died_tag); k_emit_win counts the chunks of [backs][fronts][window prefix] by
        // decoupled look-back, serves, appends and reports the window
        a.win = 1;
        a.wseg = 1;
        a.nbf = nbf;
        a.wq_off = c->qoff;
        a.wq_tail = c->qoff + Qn;
        a.wq_cap = c->qcap;
        a.q_cap = c->Wq_cap;  // the next window (tombstones included) must fit the general path
        a.wq_buf = c->queue[qc];
        a.wqf_buf = c->qfree[qc];
        a.wqh_buf = c->qhb[qc];
        a.nchB = (int)cdiv(E, kWinCh);
        a.nchF = a.nchB;
        a.nchW = c->l_nchW;
        a.wlb = c->wlb;
        a.wticket = c->wticket;
        a.cw = c->cw;
        a.cw_tag = c->link;
        a.wpart = c->wpart;
        a.pos_in = c->pos_of[qc];
        a.tomb = c->tomb;
        a.lstamp = c->lstamp;
        // (a test's injected length goes to the device, which checks what an eager commit reads)
        a.fault_qlen = c->fault_qlen;
        const int nch = a.nchB + a.nchF + a.nchW;
        // few enough chunks to be resident together: chunk = workgroup index, no ticket round
        // before the element loads.  A chunk's look-back waits on lower chunks only, so the
        // direct form needs every lower-indexed workgroup resident or done -- guaranteed while
        // the whole grid fits at once (the occupancy calculator's workgroups per CU, context
        // creation), with half of it left to concurrent work on the device
        a.win_direct = (c->win_direct && 2 * (int64_t)nch <= (int64_t)c->win_occ * c->ncu) ? 1 : 0;
        a.lpart = c->lpart;
        a.died_tag = c->died_tag;
        a.n_lpart = head > 0 ? ls_grid : 0;
        if (head > 0) {
            Timer t(c, "logscan");
            launch_logscan(a, ls_grid, t.st());
        }
        {
            Timer t(c, "emit");
            // an eager commit follows: the launch's own completion signal is the event the
            // host waits for (a separate event record between the two kernels cost ~6 us)
            c->tick_ev_set = !c->timing && c->eager && c->reruns == 0;
            launch_emit_win(a, nch, c->tick_ev_set ? Stream(c->stream, nullptr, c->tick_ev) : t.st());
        }
        HIPCHK(c, hipGetLastError());
        return FB_OK;
    }
    if (a.shard == 1) {
        // phase 1: own slots' purge, orphan flags and free counts into the exchange buffer
        if (!a.slots_in_scan) {
            Timer t(c, "slots");
            launch_slots(a, t.st());
        }
        {
            Timer t(c, "scan");
            launch_scan(a, t.st());
        }
        if (a.f_sep) {
            Timer t(c, "logscan");
            launch_logscan(a, ls_grid, t.st());
        }
        HIPCHK(c, hipGetLastError());
        return FB_OK;
    }
    if (a.shard == 2) {
        if (R > kShardMaxR) return fail(c, FB_ERANGE, "sharded tick: round table of %d rows (limit %d)", R, kShardMaxR);
        if (a.xrows || a.xplan) {
            // exchanged block rows: k_emit_shard alone (it also zeroes the other records copy,
            // which the next tick's phase 1 writes); xplan: k_xscan's counts and prefixes of the
            // exchanged c bytes first
            if (a.xplan) {
                Timer t(c, "plan");
                launch_xscan(a, t.st());
            }
            Timer t(c, "emit");
            launch_emit_shard(a, t.st());
            HIPCHK(c, hipGetLastError());
            c->xpar ^= 1;
            c->xz_ok = true;
            return FB_OK;
        }
        c->xz_ok = false;  // the next phase 1 clears the records
        {
            Timer t(c, "scan2");
            launch_scan(a, t.st());
        }
        if (!a.grp_on) {  // wide tables: k_plan's column scans
            Timer t(c, "plan");
            launch_plan(a, t.st());
        }
        Timer t(c, "emit");
        launch_emit_shard(a, t.st());
        HIPCHK(c, hipGetLastError());
        return FB_OK;
    }
    a.free_pre = (a.segw && a.slots_in_scan && !a.slots_in_apply && !c->deque && !c->l_win) ? 1 : 0;
    if (c->cm_pending) {
        // an idle tick's commit (evicted records, orphaned log entries) rides in k_scan when
        // k_scan purges the slots and reads no log entry itself
        // (per-tile orphan segments are cleared by k_emit2's log workgroups, tile by tile)
        const bool seg_ok = !c->cm.oseg || (a.f_emit && c->cm.oseg_tiles <= nbf);
        if (a.slots_in_scan && !a.slots_in_apply && (a.f_emit || a.f_sep) && !c->deque && seg_ok) {
            a.cm_fold = 1;
            a.cm_tiles = c->cm.oseg ? c->cm.oseg_tiles : 0;
            a.cm_n_orph = c->cm.oseg ? 0 : c->cm.n_orph;
            a.cm_blocks = c->cm.oseg ? 0 : std::max(1, (int)cdiv(c->cm.n_orph, kBS));
            c->cm_pending = false;
        } else if ((rc = flush_commit(c))) {
            return rc;
        }
    }
    // large one-GPU tables (<= 64 group rows): no k_plan2 -- k_emit2's queue blocks reduce
    // the group rows, its compaction workgroups the tile counts before theirs
    if (!a.fused && a.segw && a.grp_on && !c->shard && !c->deque && !c->l_win && c->gp_on && nbf <= 4096 * 4 &&
        nbw <= 4096 * 4) {
        a.gp = 1;
        a.gpcheck = c->gpcheck;
    }
    a.cmix = (c->cmix_on && !a.fused && !a.f_emit);
    // slot tiles per k_scan W-role workgroup: unfused (large) tables 4 -- fewer, longer
    // workgroups (configs[3]: scan 16.3 -> 14.8 us with 2, tick 55.4 -> 53.4 us with 4)
    a.wtiles = c->wtiles ? c->wtiles : (a.fused ? 1 : 4);
    // queue blocks per k_scan Q-role workgroup in the same (4-tile) instance: one-GPU unfused
    // tables with ride-along queue records
    a.qtiles = (c->qtiles != 1 && a.wtiles == 4 && !a.fused && !c->shard && !c->deque && a.qaos && a.R <= kRFused)
                   ? 4
                   : 1;
    if (!a.slots_in_scan && !a.slots_in_apply) {
        Timer t(c, "slots");
        launch_slots(a, t.st());
    }
    {
        Timer t(c, "scan");
        launch_scan(a, t.st());
    }
    if (a.f_sep) {
        Timer t(c, "logscan");
        launch_logscan(a, ls_grid, t.st());
    }
    if (!a.fused && (!a.gp || a.gpcheck)) {
        Timer t(c, "plan");
        launch_plan(a, t.st());
    }
    {
        Timer t(c, "emit");
        if (a.segw) launch_emit2(a, t.st());
        else launch_emit(a, t.st());
    }
    if (c->l_cout && head > 0) launch_orph_gather(c->cout_orph, c->orphans, c->fcnt, nbf, Stream(c->stream));
    HIPCHK(c, hipGetLastError());
    return FB_OK;
}

}  // namespace

extern "C" {

const char *fb_last_error(const fb_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

}  // extern "C"

namespace {
int create_ctx(fb_ctx **out, int32_t max_workers, int64_t max_log, int32_t max_events, int device, int shard,
               int rank, int world, int32_t n_workers_global, int64_t max_tokens = 0) {
    if (!out) return FB_EINVAL;
    *out = nullptr;
    if (max_workers < 1 || max_log < 1 || max_events < 0 || max_log >= ((int64_t)1 << 31) ||
        max_workers >= (1 << 30) || max_events >= (1 << 28))
        return FB_EINVAL;
    if (shard && (world < 1 || rank < 0 || rank >= world || n_workers_global < max_workers ||
                  n_workers_global >= (1 << 30)))
        return FB_EINVAL;
    fb_ctx *c = new fb_ctx();
    c->device = device;
    c->shard = shard;
    c->rank = shard ? rank : 0;
    c->world = shard ? world : 1;
    c->W_global = shard ? n_workers_global : max_workers;
    c->deque = max_tokens > 0 ? 1 : 0;
    c->Wq_cap = c->deque ? (int32_t)max_tokens : c->W_global;
    c->W_cap = max_workers;
    c->E_cap = std::max(max_events, 1);
    c->log_cap = max_log;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own_s, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return FB_EHIP;
    }
    c->stream = c->own_s;
    const size_t W = (size_t)max_workers, E = (size_t)c->E_cap, F = (size_t)max_log;
    const size_t Wq = (size_t)c->Wq_cap;  // queue entries are global slots
    const size_t Qlog = Wq + 2 * E;
    // window-capable contexts (one GPU, heartbeat loop): each queue buffer holds a window
    // that slides right by the served prefix and grows at its tail (<= 2 E + tasks per tick)
    // (large tables; fb_set_window allocates them later for others)
    c->win_cap = !shard && !c->deque && W > (size_t)kLdsBitmapSlots;
    c->qcap = c->win_cap ? (int64_t)(2 * Wq + 2 * E + 4096) : (int64_t)Wq;
    const size_t Wqb = (size_t)c->qcap;
    ArenaPlan ap;
    for (int i = 0; i < 2; ++i) {
        ap.add(&c->free_[i], W);
        ap.add(&c->queue[i], Wqb);
        if (!shard) {
            ap.add(&c->qfree[i], Wqb);
            ap.add(&c->qhb[i], Wqb);
        }
        if (c->win_cap) ap.add(&c->pos_of[i], W);
    }
    if (c->win_cap) {
        ap.add(&c->tomb, 2 * E);
        ap.add(&c->wlb, (size_t)kWinMaxCh);
        ap.add(&c->wticket, (size_t)64);
        ap.add(&c->lpart, (size_t)1024);
        ap.add(&c->died_tag, (size_t)64);
        ap.add(&c->wpart, (size_t)64 * 32);
    }
    ap.add(&c->reg, W);
    ap.add(&c->hb, W);
    ap.add(&c->epoch, W);
    ap.add(&c->touched, W);
    if (!shard && !c->deque) {
        ap.add(&c->tbitsb[0], (W + 31) / 32);
        ap.add(&c->tbitsb[1], (W + 31) / 32);
    }
    ap.add(&c->post_rf, W);
    ap.add(&c->st, W);
    ap.add(&c->trash, (size_t)kTrashRows * kBS);
    ap.add(&c->dmask, (W + 63) / 64);
    ap.add(&c->cw, (size_t)8);
    ap.add(&c->bad_min, (size_t)64);
    ap.add(&c->post, W);
    ap.add(&c->ev_status, E);
    for (int i = 0; i < 2; ++i) {
        ap.add(&c->evk[i], E);
        ap.add(&c->evv[i], E);
        ap.add(&c->evsl[i], E);
        ap.add(&c->evt[i], E);
        ap.add(&c->evq[i], E);
    }
    for (int i = 0; i < 2; ++i) {
        ap.add(&c->keys[i], E);
        ap.add(&c->vals[i], E);
    }
    // 8-bit passes: 256 x blocks; wide passes (a tick of <= kRsWideMaxBlocks blocks): 2048 x blocks
    ap.add(&c->rs_hist[0], std::max((size_t)256 * (cdiv(E, kRsTile) + 1),
                                        (size_t)2048 * (size_t)(std::min<int64_t>((int64_t)cdiv(E, kRsTile), kRsWideMaxBlocks) + 1)));
    ap.add(&c->front_list, E);
    ap.add(&c->back_list, E);
    if (!shard && !c->deque) {
        ap.add(&c->ev_head, W);
        ap.add(&c->ev_next, E);
    }
    ap.add(&c->c_arr, Qlog);
    if (!shard) {
        ap.add(&c->rb_slot, Qlog);
        ap.add(&c->rb_c, Qlog);
    }
    if (!shard) {
        ap.add(&c->c_hb, Qlog);
    }
    ap.add(&c->qbmax, (size_t)cdiv(Qlog, kBS));
    ap.add(&c->qbm_raw, (size_t)cdiv(Qlog, kBS));
    ap.add(&c->csum, (size_t)cdiv(Qlog, kBS));
    ap.add(&c->ofl, (size_t)cdiv(F, kFTile) * kBS);
    ap.add(&c->fcnt, (size_t)cdiv(F, kFTile));
    ap.add(&c->fpre, (size_t)cdiv(F, kFTile));
    ap.add(&c->wcnt, (size_t)cdiv(W, kBS));
    ap.add(&c->wpre, (size_t)cdiv(W, kBS));
    ap.add(&c->evicted, W);
    ap.add(&c->P, 1);
    const size_t tab = (size_t)128 * (size_t)cdiv(Qlog, kBS);
    ap.add(&c->qcnt, tab);
    ap.add(&c->segcnt, 4 * tab);
    ap.add(&c->grp[0], kGrpWords);
    ap.add(&c->grp[1], kGrpWords);
    ap.add(&c->qpre, tab);
    ap.add(&c->A, 128);
    ap.add(&c->A_rep, (size_t)64 * kRFused);
    ap.add(&c->P_rep, 64);
    ap.add(&c->log_slot, F);
    ap.add(&c->orphans, (size_t)cdiv(F, kFTile) * kFTile);  // whole tiles: f_emit's per-tile segments
    if (c->deque) {
        for (int i = 0; i < 2; ++i) {
            ap.add(&c->tokcnt[i], W);
            ap.add(&c->xw[i], W);
            ap.add(&c->kl[i], W);
            ap.add(&c->qrank[i], Wq);
        }
        ap.add(&c->front_rank, E);
        ap.add(&c->back_rank, E);
        ap.add(&c->post_tok, W);
        ap.add(&c->post_nf, W);
        ap.add(&c->c_tok, Qlog);
    }
    // in-flight counts only where the fused tick can use them (the died bitmap of the
    // log workgroups fits in LDS); larger tables keep k_logscan and in-place clears
    if (!shard && !c->deque && W <= (size_t)kLdsBitmapSlots) {
        ap.add(&c->bud, W);
        ap.add(&c->bud_next, W);
        ap.add(&c->post_infl, W);
        ap.add(&c->ev_clr, E);
        ap.add(&c->ctag, F);
        ap.add(&c->orph_dense, F);
    }
    // window ticks leave their orphans in per-tile segments too (gathered when read)
    if (c->win_cap && !(!shard && !c->deque && W <= (size_t)kLdsBitmapSlots)) ap.add(&c->orph_dense, F);
    if (shard) {
        ap.add(&c->lseq, F);
        ap.add(&c->ocnt, tab);
        ap.add(&c->osegcnt, 4 * tab);
        ap.add(&c->opre, tab);
        ap.add(&c->oA, 128);
        // exchanged group rows: per group the running sums and ticket (zero between ticks:
        // the arena is zeroed, each group's last block resets them) and this rank's row
        const size_t ng = (size_t)kXRowsMaxBlocks / kXGroupBlocks;
        ap.add(&c->xg_acc, ng * kXgAccStride);
        ap.add(&c->xg_tk, ng);
        ap.add(&c->xs_tk, (size_t)64);  // k_xscan's ticket (zero: the arena is zeroed, the last workgroup resets it)
        ap.add(&c->ogrp, ng * kXGroupR);
    }
    int rc = arena_commit(c, ap);
    if (!rc && hipMemset(c->bad_min, 0x7f, 4) != hipSuccess) rc = fail(c, FB_EHIP, "hipMemset(bad_min) failed");
    if (!rc) {
        c->table_cap = tab;
        c->R_cap = 128;
        c->seg_cap = tab;
        c->oA_cap = 128;
    }
    if (!rc && hipHostMalloc((void **)&c->hout, sizeof(HostOut), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        rc = FB_ENOMEM;
    if (!rc && hipHostGetDevicePointer((void **)&c->hout_dev, c->hout, 0) != hipSuccess) rc = FB_EHIP;
    if (!rc) memset(c->hout, 0, sizeof(HostOut));
    if (!rc && (hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
                hipDeviceGetAttribute(&c->max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess))
        rc = FB_EHIP;
    if (!rc) c->win_occ = emit_win_resident_per_cu();
    if (!rc && hipHostMalloc(&c->h_stage, (size_t)E * 32 * 2, hipHostMallocDefault) != hipSuccess) rc = FB_ENOMEM;
    for (int h = 0; h < 2 && !rc; ++h)
        if (hipEventCreateWithFlags(&c->stage_ev[h], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->use_ev[h], hipEventDisableTiming) != hipSuccess)
            rc = FB_EHIP;
    if (!rc && hipStreamCreateWithFlags(&c->cp_s, hipStreamNonBlocking) != hipSuccess) rc = FB_EHIP;
    if (!rc && hipEventCreateWithFlags(&c->tick_ev, hipEventDisableTiming) != hipSuccess) rc = FB_EHIP;
    if (!rc) {
        int nt = getenv("FAASBAL_STAGE_THREADS") ? atoi(getenv("FAASBAL_STAGE_THREADS")) : 8;
        nt = std::max(1, std::min(nt, 16));
        if (nt > 1 && E >= kStagePar) c->pool = new HostPool(nt);
    }
    if (!rc) {
        c->ev_kind = c->evk[0];
        c->ev_slot = c->evsl[0];
        c->ev_val = c->evv[0];
        c->ev_ts = c->evt[0];
        c->ev_seq = c->evq[0];
    }
    if (!rc && hipMemset(c->touched, 0, W * 4) != hipSuccess) rc = FB_EHIP;
    for (int p = 0; p < 2 && !rc; ++p)
        if (c->tbitsb[p] && hipMemset(c->tbitsb[p], 0, (W + 31) / 32 * 4) != hipSuccess) rc = FB_EHIP;
    if (!rc) c->tbits = c->tbitsb[c->tick & 1];
    for (int p = 0; p < 2 && !rc; ++p)
        if (hipMemset(c->grp[p], 0, kGrpWords * 4) != hipSuccess) rc = FB_EHIP;
    if (!rc && hipMemset(c->reg, 0, W) != hipSuccess) rc = FB_EHIP;
    if (!rc && c->ev_head && hipMemset(c->ev_head, 0, W * 8) != hipSuccess) rc = FB_EHIP;  // stamp 0: never a launch's
    if (rc) {
        fb_destroy(c);
        return rc;
    }
    *out = c;
    return FB_OK;
}
}  // namespace

extern "C" {

int fb_create(fb_ctx **out, int32_t max_workers, int64_t max_log, int32_t max_events, int device) {
    return create_ctx(out, max_workers, max_log, max_events, device, 0, 0, 1, max_workers);
}

int fb_create_deque(fb_ctx **out, int32_t max_workers, int64_t max_tokens, int64_t max_log, int32_t max_events,
                    int device) {
    if (max_tokens < 1 || max_tokens >= (1 << 30)) return FB_EINVAL;
    return create_ctx(out, max_workers, max_log, max_events, device, 0, 0, 1, max_workers, max_tokens);
}

int fb_create_sharded(fb_ctx **out, int32_t max_workers_local, int32_t n_workers_global, int64_t max_log_local,
                      int32_t max_events, int device, int32_t rank, int32_t world) {
    return create_ctx(out, max_workers_local, max_log_local, max_events, device, 1, rank, world, n_workers_global);
}

int fb_destroy(fb_ctx *c) {
    if (!c) return FB_OK;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->table_owned) {
        hipFree(c->qcnt);
        hipFree(c->qpre);
    }
    if (c->A_owned) hipFree(c->A);
    if (c->seg_owned) {
        hipFree(c->segcnt);
        hipFree(c->osegcnt);
        hipFree(c->ocnt);
        hipFree(c->opre);
    }
    if (c->oA_owned) hipFree(c->oA);
    if (c->assign_all) hipFree(c->assign_all);
    if (c->win_owned) hipFree(c->win_mem);
    if (c->dbg) hipFree(c->dbg);
    if (c->arena) hipFree(c->arena);
    if (c->hout) hipHostFree(c->hout);
    if (c->h_stage) hipHostFree(c->h_stage);
    delete c->pool;
    delete c->xpool;
    if (c->cp_s) hipStreamSynchronize(c->cp_s);
    for (int h = 0; h < 2; ++h) {
        if (c->stage_ev[h]) hipEventDestroy(c->stage_ev[h]);
        if (c->use_ev[h]) hipEventDestroy(c->use_ev[h]);
    }
    if (c->tick_ev) hipEventDestroy(c->tick_ev);
    if (c->gate_h) hipHostFree(c->gate_h);
    if (c->gate_a) hipEventDestroy(c->gate_a);
    if (c->gate_b) hipEventDestroy(c->gate_b);
    if (c->cp_s) hipStreamDestroy(c->cp_s);
    for (auto &t : c->tl) {
        hipEventDestroy(t.a);
        hipEventDestroy(t.b);
    }
    for (auto e : c->ev_pool) hipEventDestroy(e);
    if (c->own_s) hipStreamDestroy(c->own_s);
    delete c;
    return FB_OK;
}

int fb_load_state(fb_ctx *c, int32_t n_workers, const uint8_t *registered, const int32_t *free_processes,
                  const double *last_heartbeat, const uint32_t *epoch, const int32_t *queue, int64_t queue_len,
                  const int32_t *log_slot, int64_t log_len) {
    if (!c) return FB_EINVAL;
    if (int rc_ = flush_commit(c)) return rc_;
    c->stale_any = false;  // a loaded log holds only live entries
    if (c->shard) return fail(c, FB_ESTATE, "sharded context: use fb_load_shard");
    if (n_workers < 0 || n_workers > c->W_cap) return fail(c, FB_EINVAL, "n_workers %d outside [0, %d]", n_workers, c->W_cap);
    if (log_len < 0 || log_len > c->log_cap) return fail(c, FB_EINVAL, "log_len %lld exceeds capacity", (long long)log_len);
    if (queue_len < 0 || queue_len > (c->deque ? c->Wq_cap : n_workers))
        return fail(c, FB_EINVAL, "queue_len %lld", (long long)queue_len);
    const size_t W = (size_t)n_workers;
    std::vector<uint8_t> inq(W ? W : 1, 0);
    std::vector<int32_t> tokcnt(c->deque ? (W ? W : 1) : 0, 0);
    std::vector<uint32_t> qrank(c->deque ? (size_t)queue_len : 0);
    int32_t maxc = 1;
    for (int64_t i = 0; i < queue_len; ++i) {
        const int32_t s = queue[i];
        if (s < 0 || s >= n_workers || !registered[s] || (inq[s] && !c->deque))
            return fail(c, FB_EINVAL, "queue[%lld] = %d is out of range, unregistered or duplicated", (long long)i, s);
        inq[s] = 1;
        maxc = std::max(maxc, free_processes[s]);
        if (c->deque) qrank[i] = (uint32_t)(++tokcnt[s]) | kPart2;  // rank among the slot's tokens
    }
    for (int64_t i = 0; i < log_len; ++i)
        if (log_slot[i] < -1 || log_slot[i] >= n_workers)
            return fail(c, FB_EINVAL, "log_slot[%lld] = %d out of range", (long long)i, log_slot[i]);
    std::vector<uint8_t> reg(W ? W : 1, 0);
    std::vector<double> hbv(W ? W : 1);
    std::vector<uint32_t> epv(W ? W : 1);
    for (size_t s = 0; s < W; ++s) {
        reg[s] = registered[s] ? 1 : 0;
        hbv[s] = reg[s] ? last_heartbeat[s] : __builtin_nan("");  // no record: NaN (never "dead")
        epv[s] = epoch ? epoch[s] : 0u;
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    c->cur = 0;
    c->qcur = 0;
    c->qoff = 0;
    if (c->win_cap && W) {
        // a queued slot's position (others: never read)
        std::vector<int32_t> pos(W, 0);
        for (int64_t i = 0; i < queue_len; ++i) pos[queue[i]] = (int32_t)i;
        HIPCHK(c, hipMemcpy(c->pos_of[0], pos.data(), W * 4, hipMemcpyHostToDevice));
    }
    c->pos_ok = c->win_cap;
    if (W) {
        HIPCHK(c, hipMemcpy(c->reg, reg.data(), W, hipMemcpyHostToDevice));
        std::vector<int2> fq(W);
        for (size_t s = 0; s < W; ++s) fq[s] = make_int2(free_processes[s], inq[s]);
        HIPCHK(c, hipMemcpy(c->free_[0], fq.data(), W * sizeof(int2), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->hb, hbv.data(), W * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->epoch, epv.data(), W * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    if (queue_len) {
        HIPCHK(c, hipMemcpy(c->queue[0], queue, (size_t)queue_len * 4, hipMemcpyHostToDevice));
        std::vector<int32_t> qf((size_t)queue_len);
        std::vector<double> qh((size_t)queue_len);
        for (int64_t i = 0; i < queue_len; ++i) {
            qf[i] = free_processes[queue[i]];
            qh[i] = last_heartbeat[queue[i]];
        }
        HIPCHK(c, hipMemcpy(c->qfree[0], qf.data(), (size_t)queue_len * 4, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->qhb[0], qh.data(), (size_t)queue_len * 8, hipMemcpyHostToDevice));
    }
    c->qaos = !c->deque;
    if (c->deque) {
        if (W) {
            HIPCHK(c, hipMemcpy(c->tokcnt[0], tokcnt.data(), W * 4, hipMemcpyHostToDevice));
            HIPCHK(c, hipMemset(c->xw[0], 0, W * 4));
            HIPCHK(c, hipMemset(c->kl[0], 0, W * 4));
        }
        if (queue_len) HIPCHK(c, hipMemcpy(c->qrank[0], qrank.data(), (size_t)queue_len * 4, hipMemcpyHostToDevice));
    }
    if (log_len) {
        // heartbeat contexts keep only live entries of current registrations in the log:
        // an entry of a slot without a record, or older than its registration's epoch,
        // can never be redistributed (build-defined)
        std::vector<int32_t> lg(log_slot, log_slot + log_len);
        if (!c->deque)
            for (int64_t i = 0; i < log_len; ++i)
                if (lg[i] >= 0 && (!reg[lg[i]] || (uint64_t)i < (uint64_t)epv[lg[i]])) lg[i] = -1;
        HIPCHK(c, hipMemcpy(c->log_slot, lg.data(), (size_t)log_len * 4, hipMemcpyHostToDevice));
        if (c->bud) {
            std::vector<int32_t> bud(W ? W : 1, 0);
            for (int64_t i = 0; i < log_len; ++i)
                if (lg[i] >= 0) ++bud[lg[i]];
            for (size_t s = 0; s < W; ++s) bud[s] = reg[s] ? (int32_t)((uint32_t)bud[s] + (uint32_t)free_processes[s]) : 0;
            if (W) HIPCHK(c, hipMemcpy(c->bud, bud.data(), W * 4, hipMemcpyHostToDevice));
        }
    } else if (c->bud && W) {
        std::vector<int32_t> bud(W);
        for (size_t s = 0; s < W; ++s) bud[s] = reg[s] ? free_processes[s] : 0;
        HIPCHK(c, hipMemcpy(c->bud, bud.data(), W * 4, hipMemcpyHostToDevice));
    }
    c->W = n_workers;
    c->Qn = queue_len;
    c->Qtrue = queue_len;
    c->head = log_len;
    c->tick += 1;
    c->maxc_hint = maxc;
    c->last_L = -1;
    c->last_O = 0;
    c->launched = c->waited = false;
    return FB_OK;
}

int fb_read_state(fb_ctx *c, uint8_t *registered, int32_t *free_processes, double *last_heartbeat, uint32_t *epoch,
                  int32_t *queue, int64_t *queue_len, int32_t *log_slot, int64_t *log_len) {
    if (!c) return FB_EINVAL;
    if (int rc_ = win_uncommitted(c, "fb_read_state")) return rc_;
    if (int rc_ = flush_commit(c)) return rc_;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    const size_t W = (size_t)c->W;
    if (W) {
        if (registered) HIPCHK(c, hipMemcpy(registered, c->reg, W, hipMemcpyDeviceToHost));
        if (free_processes) {
            std::vector<int2> fq(W);
            HIPCHK(c, hipMemcpy(fq.data(), c->free_[c->cur], W * sizeof(int2), hipMemcpyDeviceToHost));
            for (size_t s = 0; s < W; ++s) free_processes[s] = fq[s].x;
        }
        if (last_heartbeat) HIPCHK(c, hipMemcpy(last_heartbeat, c->hb, W * sizeof(double), hipMemcpyDeviceToHost));
        if (epoch) HIPCHK(c, hipMemcpy(epoch, c->epoch, W * sizeof(uint32_t), hipMemcpyDeviceToHost));
    }
    if (c->win_cap) {
        // the window without its tombstones
        std::vector<int32_t> q, f;
        int64_t n = 0;
        if (int rc = win_read(c, q, f, nullptr, n)) return rc;
        if (queue && n) memcpy(queue, q.data(), (size_t)n * 4);
        if (queue_len) *queue_len = n;
    } else {
        if (queue && c->Qn) HIPCHK(c, hipMemcpy(queue, c->queue[c->qcur], (size_t)c->Qn * 4, hipMemcpyDeviceToHost));
        if (queue_len) *queue_len = c->Qn;
    }
    const int64_t nlog = c->shard ? c->head_local : c->head;
    if (log_slot && nlog) {
        if (int rc_ = log_settle(c)) return rc_;
        HIPCHK(c, hipMemcpy(log_slot, c->log_slot, (size_t)nlog * 4, hipMemcpyDeviceToHost));
    }
    if (log_len) *log_len = nlog;
    return FB_OK;
}

int fb_load_shard(fb_ctx *c, int32_t slot_base, int32_t n_workers, const uint8_t *registered,
                  const int32_t *free_processes, const double *last_heartbeat, const uint32_t *epoch,
                  const int32_t *queue, int64_t queue_len, const int32_t *log_slot, const uint32_t *log_seq,
                  int64_t log_len, int64_t log_head) {
    if (!c) return FB_EINVAL;
    if (int rc_ = flush_commit(c)) return rc_;
    c->stale_any = false;  // a loaded log holds only live entries
    if (!c->shard) return fail(c, FB_ESTATE, "fb_load_shard on a one-GPU context");
    if (n_workers < 0 || n_workers > c->W_cap || slot_base < 0 || (int64_t)slot_base + n_workers > c->W_global)
        return fail(c, FB_EINVAL, "slot range [%d, %d + %d) outside the %d-slot table", slot_base, slot_base, n_workers,
                    c->W_global);
    if (log_len < 0 || log_len > c->log_cap || log_head < log_len || log_head >= ((int64_t)1 << 31))
        return fail(c, FB_EINVAL, "log_len %lld / log_head %lld", (long long)log_len, (long long)log_head);
    if (queue_len < 0 || queue_len > c->W_global) return fail(c, FB_EINVAL, "queue_len %lld", (long long)queue_len);
    const size_t W = (size_t)n_workers;
    std::vector<uint8_t> inq(W ? W : 1, 0), seen((size_t)c->W_global, 0);
    int32_t maxc = 1;
    for (int64_t i = 0; i < queue_len; ++i) {
        const int32_t s = queue[i];
        if (s < 0 || s >= c->W_global || seen[s])
            return fail(c, FB_EINVAL, "queue[%lld] = %d is out of range or duplicated", (long long)i, s);
        seen[s] = 1;
        const int32_t ls = s - slot_base;
        if (ls >= 0 && ls < n_workers) {
            if (!registered[ls]) return fail(c, FB_EINVAL, "queue[%lld] = %d is not registered", (long long)i, s);
            inq[ls] = 1;
            maxc = std::max(maxc, free_processes[ls]);
        }
    }
    for (int64_t i = 0; i < log_len; ++i) {
        const int32_t s = log_slot[i];
        if (s < -1 || (s >= 0 && (s < slot_base || s >= slot_base + n_workers)))
            return fail(c, FB_EINVAL, "log_slot[%lld] = %d is not one of this rank's slots", (long long)i, s);
        if ((int64_t)log_seq[i] >= log_head || (i && log_seq[i] <= log_seq[i - 1]))
            return fail(c, FB_EINVAL, "log_seq must ascend below log_head (entry %lld)", (long long)i);
    }
    std::vector<uint8_t> reg(W ? W : 1, 0);
    std::vector<double> hbv(W ? W : 1);
    std::vector<uint32_t> epv(W ? W : 1);
    for (size_t s = 0; s < W; ++s) {
        reg[s] = registered[s] ? 1 : 0;
        hbv[s] = reg[s] ? last_heartbeat[s] : __builtin_nan("");  // no record: NaN (never "dead")
        epv[s] = epoch ? epoch[s] : 0u;
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    c->cur = 0;
    c->qcur = 0;
    c->qoff = 0;
    c->qcur = 0;
    c->qoff = 0;
    if (c->win_cap && W) {
        // a queued slot's position (others: never read)
        std::vector<int32_t> pos(W, 0);
        for (int64_t i = 0; i < queue_len; ++i) pos[queue[i]] = (int32_t)i;
        HIPCHK(c, hipMemcpy(c->pos_of[0], pos.data(), W * 4, hipMemcpyHostToDevice));
    }
    if (W) {
        HIPCHK(c, hipMemcpy(c->reg, reg.data(), W, hipMemcpyHostToDevice));
        std::vector<int2> fq(W);
        for (size_t s = 0; s < W; ++s) fq[s] = make_int2(free_processes[s], inq[s]);
        HIPCHK(c, hipMemcpy(c->free_[0], fq.data(), W * sizeof(int2), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->hb, hbv.data(), W * sizeof(double), hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->epoch, epv.data(), W * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    if (queue_len) HIPCHK(c, hipMemcpy(c->queue[0], queue, (size_t)queue_len * 4, hipMemcpyHostToDevice));
    if (log_len) {
        // live entries of current registrations only (see fb_load_state)
        std::vector<int32_t> lg(log_slot, log_slot + log_len);
        for (int64_t i = 0; i < log_len; ++i)
            if (lg[i] >= 0 && (!reg[lg[i] - slot_base] || (uint64_t)log_seq[i] < (uint64_t)epv[lg[i] - slot_base]))
                lg[i] = -1;
        HIPCHK(c, hipMemcpy(c->log_slot, lg.data(), (size_t)log_len * 4, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(c->lseq, log_seq, (size_t)log_len * 4, hipMemcpyHostToDevice));
    }
    c->slot_base = slot_base;
    c->W = n_workers;
    c->Qn = queue_len;
    c->head = log_head;
    c->head_local = log_len;
    c->tick += 1;
    // the first tick's round table from what every rank knows alike (the exchange layout
    // depends on it): its events' values and fb_set_round_hint (the loaded state's global
    // max free count, which the caller knows from the global state); the rank's own max
    // (maxc above) would differ between ranks.  A fill level beyond it relaunches wider.
    (void)maxc;
    c->maxc_hint = 1;
    c->launched = c->waited = false;
    c->phase = 0;
    return FB_OK;
}

int fb_read_inflight(fb_ctx *c, uint32_t *inflight) {
    if (!c || !inflight) return FB_EINVAL;
    if (int rc_ = win_uncommitted(c, "fb_read_inflight")) return rc_;
    if (int rc_ = flush_commit(c)) return rc_;
    if (!c->bud) return fail(c, FB_ESTATE, "in-flight counts exist on one-GPU heartbeat contexts only");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    const size_t W = (size_t)c->W;
    if (!W) return FB_OK;
    std::vector<int32_t> bud(W);
    std::vector<int2> fq(W);
    std::vector<uint8_t> reg(W);
    HIPCHK(c, hipMemcpy(bud.data(), c->bud, W * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(fq.data(), c->free_[c->cur], W * sizeof(int2), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(reg.data(), c->reg, W, hipMemcpyDeviceToHost));
    for (size_t s = 0; s < W; ++s) inflight[s] = reg[s] ? (uint32_t)bud[s] - (uint32_t)fq[s].x : 0u;
    return FB_OK;
}

int fb_read_shard_log(fb_ctx *c, uint32_t *log_seq, int64_t *log_len, int64_t *log_head) {
    if (!c) return FB_EINVAL;
    if (int rc_ = flush_commit(c)) return rc_;
    if (!c->shard) return fail(c, FB_ESTATE, "fb_read_shard_log on a one-GPU context");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    if (log_seq && c->head_local)
        HIPCHK(c, hipMemcpy(log_seq, c->lseq, (size_t)c->head_local * 4, hipMemcpyDeviceToHost));
    if (log_len) *log_len = c->head_local;
    if (log_head) *log_head = c->head;
    return FB_OK;
}

int fb_bind_exchange(fb_ctx *c, void *device_buffer, int64_t bytes) {
    if (!c) return FB_EINVAL;
    if (!c->shard) return fail(c, FB_ESTATE, "fb_bind_exchange on a one-GPU context");
    if (bytes < 0 || (bytes && !device_buffer)) return fail(c, FB_EINVAL, "exchange buffer");
    HIPCHK(c, stream_wait(c));
    c->xbuf = (uint8_t *)device_buffer;
    c->xcap = bytes;
    c->xpar = 0;
    c->xz_ok = false;
    return FB_OK;
}

int fb_exchange_bytes(fb_ctx *c, int32_t n_events, int64_t *bytes) {
    if (!c || !bytes) return FB_EINVAL;
    const int64_t E = n_events < 0 ? c->E_cap : n_events;
    const int64_t Qn = n_events < 0 ? c->Wq_cap : (c->launched ? c->l_Qn : c->Qn);
    // the maximum: room for the wide form or for the block rows of a <= kRFused-row table,
    // whichever is larger; a launched tick: its own width and rows
    const int64_t Qlog = Qn + 2 * E;
    if (n_events < 0) {
        // the largest of: the wide form at the largest queue; a queue of at most
        // kXRowsMaxBlocks blocks with a 128-row table's block rows (the one-launch form; a
        // 32-row table's block + group rows are smaller); the largest queue with a 32-row
        // table's block rows (the k_xscan form)
        const int64_t Qr = std::min<int64_t>(Qlog, (int64_t)kXRowsMaxBlocks * kBS);
        *bytes = (int64_t)std::max({xlayout(c->world, E, Qlog, 2).total,
                                    xlayout(c->world, E, Qr, 1, xrows_bytes(c->world, kRFused, Qr)).total,
                                    xlayout(c->world, E, Qlog, 1, xrows_bytes(c->world, kXGroupR, Qlog),
                                            xgrows_bytes(c->world, kXGroupR, Qlog)).total});
    } else {
        const int R = c->launched ? c->l_R : kRFused;
        const bool xoff = !c->xplan_on && xrows_mode(c->world, R, Qlog) == 2;
        *bytes = (int64_t)xlayout(c->world, E, Qlog, xc_width(R), xoff ? 0 : xrows_bytes(c->world, R, Qlog),
                                  xgrows_bytes(c->world, R, Qlog)).total;
    }
    return FB_OK;
}

int fb_set_stream(fb_ctx *c, void *stream) {
    if (!c) return FB_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    c->stream = stream ? (hipStream_t)stream : c->own_s;
    return FB_OK;
}

int fb_tick_continue(fb_ctx *c) {
    if (!c) return FB_EINVAL;
    if (!c->shard) return fail(c, FB_ESTATE, "fb_tick_continue on a one-GPU context");
    if (!c->launched || c->phase != 1) return fail(c, FB_ESTATE, "fb_tick_continue without fb_tick_launch");
    HIPCHK(c, hipSetDevice(c->device));
    c->phase = 2;
    return enqueue_tick(c);
}

// H2D copies of a staged batch into device half `half` on the copy stream, after the
// last tick that read that half; the launch waits for stage_ev[half].
static int stage_copies(fb_ctx *c, int half, const void *sk, const void *ss, const void *sv, const void *st,
                        const void *sq, int E) {
    if (c->use_rec[half]) HIPCHK(c, hipStreamWaitEvent(c->cp_s, c->use_ev[half], 0));
    HIPCHK(c, hipMemcpyAsync(c->evk[half], sk, E, hipMemcpyHostToDevice, c->cp_s));
    HIPCHK(c, hipMemcpyAsync(c->evsl[half], ss, (size_t)E * 4, hipMemcpyHostToDevice, c->cp_s));
    HIPCHK(c, hipMemcpyAsync(c->evv[half], sv, (size_t)E * 4, hipMemcpyHostToDevice, c->cp_s));
    HIPCHK(c, hipMemcpyAsync(c->evt[half], st, (size_t)E * 8, hipMemcpyHostToDevice, c->cp_s));
    if (sq)
        HIPCHK(c, hipMemcpyAsync(c->evq[half], sq, (size_t)E * 8, hipMemcpyHostToDevice, c->cp_s));
    else
        HIPCHK(c, hipMemsetAsync(c->evq[half], 0xff, (size_t)E * 8, c->cp_s));  // -1 for every event
    HIPCHK(c, hipEventRecord(c->stage_ev[half], c->cp_s));
    c->stage_rec[half] = true;
    return FB_OK;
}

// Validate a tick's events and stage them into the pinned half the next launch
// copies from.  Two halves: staging tick t+1 on the host overlaps tick t on the
// device (the half's previous copies were enqueued two launches ago; its event
// is waited for, not the stream).
int fb_tick_stage(fb_ctx *c, double now, int32_t n_events, const uint8_t *kind, const int32_t *slot,
                  const int32_t *val, const double *ts, const int64_t *seq) {
    if (!c) return FB_EINVAL;
    if (n_events < 0 || n_events > c->E_cap) return fail(c, FB_EINVAL, "n_events %d outside [0, %d]", n_events, c->E_cap);
    if (n_events && (!kind || !slot || !val || !ts))
        return fail(c, FB_EINVAL, "event arrays must be non-NULL");
    const int E = n_events;
    const int half = c->stage_half ^ 1;
    // One pass over the caller's arrays: validate (branch-free; the per-event loop
    // below runs only to name the first offending event) while staging them into
    // pinned memory; fb_tick_launch_staged issues one async copy per array.
    const uint32_t Wv = (uint32_t)(c->shard ? c->W_global : c->W);
    int32_t vmax = 0;
    // Zero-copy: when the caller's arrays are pinned host memory (fb_host_alloc, e.g. a
    // dispatcher that parses messages straight into them) the pass only validates, and
    // the H2D copies read the caller's arrays; they must stay unchanged until the tick
    // that uses them has been waited for.
    bool direct = E > 0, resident = E > 0;
    if (direct) {
        const void *ptrs[5] = {kind, slot, val, ts, seq};
        int nhost = 0, ndev = 0, n = 0;
        for (int j = 0; j < 5; ++j) {
            if (!ptrs[j]) continue;  // seq may be NULL: filled with -1 on the device
            ++n;
            hipPointerAttribute_t at;
            if (hipPointerGetAttributes(&at, ptrs[j]) != hipSuccess) {
                (void)hipGetLastError();
            } else if (at.type == hipMemoryTypeHost) {
                ++nhost;
            } else if (at.type == hipMemoryTypeDevice) {
                if (at.device != c->device)
                    return fail(c, FB_EINVAL, "event array %d is in the memory of GPU %d, the context's is GPU %d", j,
                                at.device, c->device);
                ++ndev;
            }
        }
        direct = nhost == n;
        resident = ndev == n;
        if (ndev && !resident) return fail(c, FB_EINVAL, "event arrays mix this GPU's memory with other memory");
    }
    if (resident) {
        // a batch already in this GPU's memory (e.g. parsed there, or staged ahead): the
        // tick reads it in place and its first kernel checks it (an invalid message is
        // overwritten with a harmless one and fb_tick_wait names it); no host pass
        if (!(c->ev_head && c->ev_ll))
            return fail(c, FB_EINVAL, "device-resident messages need a one-GPU heartbeat context");
        c->st_dev[0] = kind;
        c->st_dev[1] = slot;
        c->st_dev[2] = val;
        c->st_dev[3] = ts;
        c->st_dev[4] = seq;
        c->st_res = true;
        c->st_chk[0] = c->st_chk[1] = c->st_chk[2] = kind;  // device-checked (names come from bad_min)
        c->staged = true;
        c->st_E = E;
        c->st_vmax = 0;
        c->st_now = now;
        return FB_OK;
    }
    c->st_res = false;
    // pinned inputs: their H2D copies go out first and overlap the validation below (a
    // batch that fails validation is never launched, so copying it first is harmless)
    bool copied = false;
    if (E && direct) {
        if (int rc = stage_copies(c, half, kind, slot, val, ts, seq, E)) return rc;
        copied = true;
    }
    if (E) {
        const size_t ecap = (size_t)c->E_cap;
        char *h = (char *)c->h_stage + (size_t)half * ecap * 32;
        uint8_t *hk = (uint8_t *)h;
        int32_t *hs = (int32_t *)(h + ecap);
        int32_t *hv = (int32_t *)(h + ecap * 5);
        double *ht = (double *)(h + ecap * 9);
        int64_t *hq = (int64_t *)(h + ecap * 17);
        HIPCHK(c, hipSetDevice(c->device));
        if (!direct && c->stage_rec[half]) HIPCHK(c, hipEventSynchronize(c->stage_ev[half]));  // staging buffer reuse
        // parts of the batch on the pool's workers when it is large (the pass reads and
        // writes ~25 B per event, mostly cold caller memory: memory-latency bound)
        const int np = (c->pool && E >= kStagePar) ? c->pool->size() : 1;
        uint32_t pbad[16] = {0};
        int32_t pvmax[16] = {0};
        // pinned batches of contexts whose first launch is k_ev_link are checked there
        // (slots, kinds, timestamps; fb_tick_wait names the first offending event and the
        // tick commits nothing): the host does not read them at all.  The round table is
        // then sized from the last tick's free counts (a wider one is a rerun away).
        const bool dev_chk = direct && c->ev_head && c->ev_ll;
        auto part = [&](int pi) {
            if (dev_chk) {
                pbad[pi] = 0;
                pvmax[pi] = 0;
                return;
            }
            const int lo = (int)((int64_t)E * pi / np), hi = (int)((int64_t)E * (pi + 1) / np);
            uint32_t bad = 0;
            int32_t vm = 0;
            double prev = ts[lo > 0 ? lo - 1 : 0];
            for (int i = lo; i < hi; ++i) {
                const uint8_t k = kind[i];
                const int32_t sl = slot[i], v = val[i];
                const double t = ts[i];
                bad |= (uint32_t)((uint32_t)sl >= Wv) | (uint32_t)(k > FB_EV_OTHER) | (uint32_t)!(t <= now) |
                       (uint32_t)(t < prev);
                prev = t;
                vm = std::max(vm, k <= FB_EV_RECONNECT ? v : 0);
                if (!direct) {
                    hk[i] = k;
                    hs[i] = sl;
                    hv[i] = v;
                    ht[i] = t;
                    hq[i] = seq ? seq[i] : -1;
                }
            }
            pbad[pi] = bad;
            pvmax[pi] = vm;
        };
        if (np > 1 && !dev_chk) c->pool->run(part);
        else part(0);
        uint32_t bad = 0;
        for (int pi = 0; pi < np; ++pi) {
            bad |= pbad[pi];
            vmax = std::max(vmax, pvmax[pi]);
        }
        for (int i = 0; bad && i < E; ++i) {
            c->staged = false;
            c->stage_rec[half] = false;  // nothing was copied out of this half
            if ((uint32_t)slot[i] >= Wv) return fail(c, FB_EINVAL, "event %d: slot %d outside [0, %u)", i, slot[i], Wv);
            if (kind[i] > FB_EV_OTHER) return fail(c, FB_EINVAL, "event %d: unknown kind %d", i, kind[i]);
            if (!(ts[i] <= now) || (i && ts[i] < ts[i - 1]))
                return fail(c, FB_EINVAL, "event %d: timestamps must be non-decreasing and <= now", i);
        }
        if (dev_chk) {  // checked by k_ev_link (fb_tick_wait reports)
            c->st_chk[0] = kind;
            c->st_chk[1] = slot;
            c->st_chk[2] = ts;
        } else {
            c->st_chk[0] = nullptr;
        }
    }
    if (E && !copied) {
        const size_t ecap = (size_t)c->E_cap;
        char *h = (char *)c->h_stage + (size_t)half * ecap * 32;
        if (int rc = stage_copies(c, half, h, h + ecap, h + ecap * 5, h + ecap * 9, h + ecap * 17, E)) return rc;
    }
    c->staged = true;
    c->st_E = E;
    c->st_vmax = vmax;
    c->st_now = now;
    return FB_OK;
}

static CommitArgs commit_args(fb_ctx *c, bool eager, int &grid);

int fb_tick_launch_staged(fb_ctx *c, double tte, int64_t n_pending) {
    if (!c) return FB_EINVAL;
    if (!c->staged) return fail(c, FB_ESTATE, "fb_tick_launch_staged without fb_tick_stage");
    if (c->launched && c->l_eager)
        return fail(c, FB_ESTATE, "the last tick was committed eagerly: fb_tick_wait and fb_tick_commit first");
    if (n_pending < 0) return fail(c, FB_EINVAL, "n_pending < 0");
    HIPCHK(c, hipSetDevice(c->device));
    const int E = c->st_E;
    const int half = c->stage_half ^ 1;
    c->l_res = E && c->st_res;
    if (c->l_res) {
        c->ev_kind = (uint8_t *)c->st_dev[0];
        c->ev_slot = (int32_t *)c->st_dev[1];
        c->ev_val = (int32_t *)c->st_dev[2];
        c->ev_ts = (double *)c->st_dev[3];
        c->ev_seq = (int64_t *)c->st_dev[4];
        if (!c->ev_seq) {  // -1 for every message
            HIPCHK(c, hipMemsetAsync(c->evq[half], 0xff, (size_t)E * 8, c->stream));
            c->ev_seq = c->evq[half];
        }
    } else {
        if (E) HIPCHK(c, hipStreamWaitEvent(c->stream, c->stage_ev[half], 0));  // the staged copies
        c->ev_kind = c->evk[half];
        c->ev_slot = c->evsl[half];
        c->ev_val = c->evv[half];
        c->ev_ts = c->evt[half];
        c->ev_seq = c->evq[half];
    }
    c->stage_half = half;
    c->staged = false;
    const double now = c->st_now;
    c->l_now = now;
    c->l_tte = c->deque ? __builtin_inf() : tte;  // start() has no liveness: nobody ever expires
    c->l_E = E;
    c->l_T = n_pending;
    c->l_head = c->head;
    c->l_head_local = c->head_local;
    c->l_Qn = c->Qn;
    c->l_qoff = c->qoff;
    c->phase = 1;
    c->tick += 1;  // per-launch stamp: a relaunch with other messages never sees this launch's marks
    if (c->tbitsb[0]) c->tbits = c->tbitsb[c->tick & 1];  // the last tick's bits stay for its deferred commit
    c->l_R = choose_R(std::max(c->maxc_hint, c->st_vmax));
    // sharded: the round table starts at <= 128 rows (one byte per exchanged c: every
    // round below the table is exact, 255 > 128); a fill level reaching the table makes
    // fb_tick_wait ask for a relaunch, which gets a wider table (two bytes per c)
    if (c->shard) c->l_R = std::min(c->shard_R > 0 ? c->shard_R : std::min(c->l_R, kRFused), kShardMaxR);
    c->reruns = 0;
    c->l_resort = false;
    c->launched = true;
    c->waited = false;
    c->l_purge_only = c->next_purge_only;
    c->next_purge_only = false;
    c->l_win = win_plan(c);
    for (int j = 0; j < 3; ++j) c->l_chk[j] = E ? c->st_chk[j] : nullptr;
    c->hout->bad_ev = 0;  // set by k_ev_link when it finds an invalid message
    // lengths every finished tick writes: a value left unwritten reads back as -1 and fails
    // check_lengths instead of becoming a copy size (a relaunch overwrites them again)
    c->hout->new_qlen = -1;
    c->hout->win_head = -1;
    c->hout->win_qlen = -1;
    const int rc = enqueue_tick(c);
    if (rc) return rc;
    c->l_eager = false;
    if (c->eager && c->l_win) {
        // eager: the window tick's commit right behind it on the stream; it commits only
        // if the tick finished as a window tick (fb_tick_wait reruns it otherwise)
        int grid = 0;
        const CommitArgs a = commit_args(c, true, grid);
        if (!c->tick_ev_set) HIPCHK(c, hipEventRecord(c->tick_ev, c->stream));  // fb_tick_wait waits for the tick, not its commit
        Timer t(c, "commit");
        launch_commit(a, grid, t.st());
        HIPCHK(c, hipGetLastError());
        c->l_eager = true;
    }
    if (E && !c->l_res) {  // (a device-resident batch used no half)
        // the next copy into this device half waits for the tick's reads (a rerun in
        // fb_tick_wait reads it again, but no stage can target this half before then)
        HIPCHK(c, hipEventRecord(c->use_ev[half], c->stream));
        c->use_rec[half] = true;
    }
    return FB_OK;
}

int fb_tick_launch(fb_ctx *c, double now, double tte, int32_t n_events, const uint8_t *kind, const int32_t *slot,
                   const int32_t *val, const double *ts, const int64_t *seq, int64_t n_pending) {
    if (!c) return FB_EINVAL;
    if (n_pending < 0) return fail(c, FB_EINVAL, "n_pending < 0");
    int rc = fb_tick_stage(c, now, n_events, kind, slot, val, ts, seq);
    if (rc) return rc;
    return fb_tick_launch_staged(c, tte, n_pending);
}

int fb_purge_launch(fb_ctx *c, double now, double tte) {
    if (!c) return FB_EINVAL;
    // a tick without messages or pending tasks whose orphans are reported, not dispatched
    int rc = fb_tick_stage(c, now, 0, nullptr, nullptr, nullptr, nullptr, nullptr);
    if (rc) return rc;
    c->next_purge_only = true;
    return fb_tick_launch_staged(c, tte, 0);
}

// Every length a finished tick reports becomes a copy size or a kernel bound later
// (fb_read_state's queue copy, the commit's grids, the readbacks): a value outside its
// buffer is a device fault, reported here with both numbers, before anything uses it.
// (task_dispatcher.py:327: the queue new_qlen describes.)
static int check_lengths(fb_ctx *c) {
    const HostOut &p = *c->hout;
    const int64_t O = p.O, N = p.N_eff;
    if (O < 0 || O > c->l_head)
        return fail(c, FB_EHIP, "device-reported orphans %lld outside [0, %lld] (log head)", (long long)O,
                    (long long)c->l_head);
    if (c->shard && (p.O_local < 0 || p.O_local > c->l_head_local || p.O_local > O))
        return fail(c, FB_EHIP, "device-reported local orphans %lld outside [0, %lld] (local log head)",
                    (long long)p.O_local, (long long)std::min<int64_t>(c->l_head_local, O));
    if (p.n_evicted < 0 || p.n_evicted > c->W)
        return fail(c, FB_EHIP, "device-reported evictions %lld outside [0, %d] (slots)", (long long)p.n_evicted, c->W);
    if (N < 0 || N > c->l_T + O)
        return fail(c, FB_EHIP, "device-reported dispatches %lld outside [0, %lld] (pending + orphans)", (long long)N,
                    (long long)(c->l_T + O));
    if (c->shard && (p.n_local < 0 || p.n_local > N))
        return fail(c, FB_EHIP, "device-reported local dispatches %lld outside [0, %lld]", (long long)p.n_local,
                    (long long)N);
    if (c->l_win) {
        if (p.win_head < c->l_qoff || p.new_qlen < 0 || p.win_head > c->qcap || p.new_qlen > c->qcap - p.win_head)
            return fail(c, FB_EHIP, "device-reported window [%lld, +%lld) outside the queue buffer [%lld, %lld)",
                        (long long)p.win_head, (long long)p.new_qlen, (long long)c->l_qoff, (long long)c->qcap);
        if (p.win_qlen < 0 || p.win_qlen > p.new_qlen || p.win_qlen > c->Wq_cap)
            return fail(c, FB_EHIP, "device-reported queue length %lld outside [0, %lld] (window length)",
                        (long long)p.win_qlen, (long long)std::min<int64_t>(p.new_qlen, c->Wq_cap));
    } else if (p.new_qlen < 0 || (!c->deque && p.new_qlen > c->qcap)) {
        // (deque contexts: a length past the token capacity is FB_ENOSPC below)
        return fail(c, FB_EHIP, "device-reported queue length %lld outside [0, %lld] (queue buffer)",
                    (long long)p.new_qlen, (long long)c->qcap);
    }
    return FB_OK;
}

int fb_tick_wait(fb_ctx *c, fb_tick_result *res) {
    if (!c) return FB_EINVAL;
    if (!c->launched) return fail(c, FB_ESTATE, "fb_tick_wait without fb_tick_launch");
    if (c->shard && c->phase != 2) return fail(c, FB_ESTATE, "sharded tick: exchange, then fb_tick_continue");
    HIPCHK(c, hipSetDevice(c->device));
    for (bool first = true;; first = false) {
        if (first && c->l_eager) {
            // the tick's results are final when its last kernel is: the host goes on while
            // the eager commit runs (the next launch queues behind it)
            hipError_t e;
            while ((e = hipEventQuery(c->tick_ev)) == hipErrorNotReady) {
            }
            HIPCHK(c, e);
        } else {
            HIPCHK(c, stream_wait(c));
        }
        // any rerun below cancels an eager commit (its kernel found the tick unfinished and
        // committed nothing); the rerun's commit is the ordinary one
        if (c->l_chk[0] && c->hout->bad_ev) {
            c->l_eager = false;
            // the batch was left to the device's check: name the first offending event; the
            // tick is not committed (its launch read only committed state)
            c->launched = false;
            // the first offending message's index (k_ev_link atomicMins it for every checked
            // batch): read, and reset for the next checked batch whatever its kind
            int32_t bi = 0x7f7f7f7f;
            const int32_t none = 0x7f7f7f7f;
            HIPCHK(c, hipMemcpy(&bi, c->bad_min, 4, hipMemcpyDeviceToHost));
            HIPCHK(c, hipMemcpy(c->bad_min, &none, 4, hipMemcpyHostToDevice));
            if (c->l_res) {
                // a device-resident batch: the index from the device
                return fail(c, FB_EINVAL, "event %d: invalid message (slot outside [0, %d), unknown kind, or a "
                            "timestamp decreasing or past now)", bi, c->W);
            }
            const uint8_t *k = (const uint8_t *)c->l_chk[0];
            const int32_t *sl = (const int32_t *)c->l_chk[1];
            const double *ts = (const double *)c->l_chk[2];
            for (int i = 0; i < c->l_E; ++i) {
                if ((uint32_t)sl[i] >= (uint32_t)c->W) return fail(c, FB_EINVAL, "event %d: slot %d outside [0, %d)", i, sl[i], c->W);
                if (k[i] > FB_EV_OTHER) return fail(c, FB_EINVAL, "event %d: unknown kind %d", i, k[i]);
                if (!(ts[i] <= c->l_now) || (i && ts[i] < ts[i - 1]))
                    return fail(c, FB_EINVAL, "event %d: timestamps must be non-decreasing and <= now", i);
            }
            return fail(c, FB_EINVAL, "invalid message in the batch");
        }
        if (c->l_used_ll && c->hout->resort) {
            c->l_eager = false;
            // a slot got more messages than k_ev_apply_ll sorts in registers: the same
            // functional tick again, grouped by the radix sort
            if (c->reruns > 4) return fail(c, FB_EHIP, "event regrouping did not converge");
            c->l_resort = true;
            c->l_win = false;  // the sorted path purges in k_scan: a general tick
            c->reruns++;
            int rc = enqueue_tick(c);
            if (rc) return rc;
            continue;
        }
        if (c->l_win && (c->hout->status == 3 || c->hout->win_ovf)) {
            c->l_eager = false;
            // the window tick could not finish inside its window (a fill level above 0, an
            // unserved front, a first unserved element past the scanned prefix, no room at
            // the tail): the same functional tick on the general path
            if (c->hout->status == 3 && (int64_t)c->l_nchW * kWinCh < c->l_Qn)  // the scanned prefix was short
                c->win_slack = std::min<int64_t>(2 * c->win_slack, 1 << 24);
            c->l_win = false;
            c->win_fallbacks++;
            c->reruns++;
            int rc = enqueue_tick(c);
            if (rc) return rc;
            continue;
        }
        if (c->hout->status == 0) break;
        c->l_eager = false;
        if (c->hout->status == 2)
            return fail(c, FB_ENOSPC, "in-flight log full: %lld entries + this tick's dispatches exceed %lld",
                        (long long)c->l_head, (long long)c->log_cap);
        // the queue holds free counts beyond the round table: widen and rerun
        if (c->shard) {
            // the exchange runs between the phases, so the caller relaunches: the same tick
            // with a table sized by the max free count seen (clamped to the exchange width)
            const int R = choose_R(c->hout->maxc);
            if (c->l_R >= kShardMaxR || R <= c->l_R)
                return fail(c, FB_ERANGE, "sharded tick: fill level beyond a %d-round table (max free %d)", c->l_R,
                            c->hout->maxc);
            c->shard_R = std::min(R, kShardMaxR);
            return fail(c, FB_ERERUN, "sharded tick: the fill level reaches the %d-round table; relaunch (%d rows)",
                        c->l_R, c->shard_R);
        }
        const int R = choose_R(c->hout->maxc);
        if (R <= c->l_R || c->reruns > 4)
            return fail(c, FB_ERANGE, "fill level beyond the round table (maxc %d, R %d)", c->hout->maxc, c->l_R);
        c->l_R = R;
        c->reruns++;
        int rc = enqueue_tick(c);
        if (rc) return rc;
    }
    if (c->fault_qlen >= 0) {
        // (a window tick reported the injected length from the device already)
        c->hout->new_qlen = c->fault_qlen;
        c->hout->win_qlen = c->fault_qlen;
        c->fault_qlen = -1;
    }
    if (int rc_ = check_lengths(c)) {
        c->l_eager = false;
        c->launched = false;  // the tick is not committed (its launch read only committed state)
        return rc_;
    }
    const HostOut &p = *c->hout;
    if (c->deque && p.new_qlen > c->Wq_cap)
        return fail(c, FB_ENOSPC, "deque of %lld tokens exceeds the context's capacity %d", (long long)p.new_qlen,
                    c->Wq_cap);
    fb_tick_result r{};
    r.n_assigned = p.N_eff;
    r.n_orphans = p.O;
    r.queue_len = c->l_win ? p.win_qlen : (int64_t)p.new_qlen;
    r.log_head = c->l_head + p.N_eff;
    r.n_evicted = (int32_t)p.n_evicted;
    r.fill_level = p.L;
    r.max_free = p.maxc;
    r.reruns = c->reruns;
    r.n_local = c->shard ? p.n_local : p.N_eff;
    r.n_orphans_local = c->shard ? p.O_local : p.O;
    c->last = r;
    c->waited = true;
    if (res) *res = r;
    return FB_OK;
}

// The commit of the launched tick.  eager: built at launch, before the tick's results
// exist -- the window's head and appended positions are read by the kernel from the
// tick's results, and every orphan tile and appended position gets blocks (grid-stride).
static CommitArgs commit_args(fb_ctx *c, bool eager, int &grid) {
    // lazy clears: the redistributed entries stay in the log (dead to every later tick)
    const bool lazy = lazy_ctx(c);
    const int64_t n_orph = (eager || lazy) ? 0 : c->last.n_orphans_local;
    CommitArgs a{};
    a.W = c->W;
    a.nbw = (int)cdiv(c->W, kBS);
    a.tick = c->tick;
    a.st = c->st;
    a.touched = c->touched;
    a.post = c->post;
    a.tbits = c->tbits;
    a.E = c->l_E;
    a.reg = c->reg;
    a.hb = c->hb;
    a.epoch = c->epoch;
    a.n_orph = n_orph;
    a.orphans = c->orphans;
    a.log_slot = c->log_slot;
    a.lseq = c->lseq;
    a.head_local = c->l_head_local;
    a.shard = c->shard;
    a.nbo = (int)cdiv(n_orph, kBS);
    if (!lazy && c->l_oseg && (n_orph > 0 || eager)) {  // per-tile segments: a wave per log tile
        a.oseg = c->fcnt;
        a.oseg_tiles = c->l_nbf;
        a.nbo = (int)cdiv(c->l_nbf, kWaves);
    }
    a.n_clr = c->ev_clr ? c->l_E : 0;  // one-GPU heartbeat: the results' completed entries
    a.ev_clr = c->ev_clr;
    a.bud = c->bud;
    a.bud_next = c->bud_next;
    if (c->l_win) {
        // the window moves: positions of slots that left become tombstones, kept slots that
        // got messages take their post-message counts, appended slots their positions
        a.win = 1;
        a.wq_tail = c->l_qoff + c->l_Qn;
        if (eager) {
            a.eager = c->cw;
            a.cw_tag = c->link;
            a.nbap = (int)std::min<int64_t>(1024, cdiv(2 * (int64_t)c->l_E + c->l_T, kBS) + 1);
        } else {
            const HostOut &p = *c->hout;
            a.wq_head = p.win_head;
            a.napp = p.win_head + p.new_qlen - a.wq_tail;
            a.nbap = (int)cdiv(a.napp, kBS);
        }
        a.wq_buf = c->queue[c->qcur];
        a.wqf = c->qfree[c->qcur];
        a.wqh = c->qhb[c->qcur];
        a.pos = c->pos_of[c->qcur];
        a.tomb = c->tomb;
        a.n_tomb = 2 * c->l_E;
        a.post_rf = c->post_rf;
    }
    grid = a.nbw + a.nbo + (int)cdiv(a.n_clr, kBS) +
           (a.win ? a.nbap + (int)cdiv(a.n_tomb, kBS) : 0);
    return a;
}

int fb_tick_commit(fb_ctx *c) {
    if (!c) return FB_EINVAL;
    if (!c->waited) return fail(c, FB_ESTATE, "fb_tick_commit without a waited tick");
    HIPCHK(c, hipSetDevice(c->device));
    const int64_t n_orph = c->last.n_orphans_local;
    if (c->l_eager) {
        // the device committed the tick right behind it (fb_tick_launch_staged)
    } else if (c->W > 0 || n_orph > 0 || (c->ev_clr && c->l_E > 0)) {
        int grid = 0;
        const bool defer = c->ev_head && c->ev_ll && !c->l_win;
        const CommitArgs a = commit_args(c, false, grid);
        if (defer) {  // (by default a window tick's commit runs at once)
            // deferred: the next launch's k_ev_link runs it (or flush_commit)
            c->cm = a;
            c->cm_grid = grid;
            c->cm_pending = true;
        } else {
            Timer t(c, "commit");
            launch_commit(a, grid, t.st());
            HIPCHK(c, hipGetLastError());
        }
    }
    c->l_eager = false;
    if (lazy_ctx(c) && c->last.n_orphans > 0) c->stale_any = true;  // its orphans stay in the log
    c->cur = 1 - c->cur;
    // sharded: a tick that needed a wide table keeps it for the next one while the fill
    // level stays beyond the narrow table (no relaunch per tick)
    if (c->shard) c->shard_R = c->last.fill_level + 2 > kRFused ? c->l_R : 0;
    c->head = c->last.log_head;
    c->head_local += c->shard ? c->last.n_local : 0;
    c->Qtrue = c->last.queue_len;
    c->last_L = c->last.fill_level;
    c->last_O = c->last.n_orphans;
    if (c->l_win) {
        // the queue stays in its buffers: the window slid and grew
        c->qoff = c->hout->win_head;
        c->Qn = c->hout->new_qlen;
        c->win_ticks++;
        // the scanned prefix saw only part of the queue: keep the larger hint
        c->maxc_hint = std::max(c->maxc_hint, std::max(1, c->last.max_free));
    } else {
        c->qcur ^= 1;
        c->qoff = 0;
        c->pos_ok = false;  // the new queue's positions are rebuilt by the next window tick
        c->Qn = c->last.queue_len;
        c->maxc_hint = std::max(1, c->last.max_free);
    }
    c->launched = c->waited = false;
    c->phase = 0;
    return FB_OK;
}

int fb_get_local_assignments(fb_ctx *c, int64_t first, int64_t n, int64_t *task, int32_t *slot) {
    if (!c) return FB_EINVAL;
    if (int rc_ = flush_commit(c)) return rc_;
    if (!c->waited) return fail(c, FB_ESTATE, "no waited tick");
    if (first < 0 || n < 0 || first + n > c->last.n_local) return fail(c, FB_EINVAL, "assignment range");
    if (!n) return FB_OK;
    const int64_t base = c->shard ? c->l_head_local : c->l_head;
    if (slot) HIPCHK(c, hipMemcpy(slot, c->log_slot + base + first, (size_t)n * 4, hipMemcpyDeviceToHost));
    if (task) {
        if (c->shard) {
            std::vector<uint32_t> q((size_t)n);
            HIPCHK(c, hipMemcpy(q.data(), c->lseq + base + first, (size_t)n * 4, hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < n; ++i) task[i] = (int64_t)q[i] - c->l_head;
        } else {
            for (int64_t i = 0; i < n; ++i) task[i] = first + i;
        }
    }
    return FB_OK;
}

// Device -> host copy enqueued on the context stream: into pinned host memory by a
// copy kernel whose stores cross PCIe directly (the DMA engine path measured 137 to
// 344 us for 4 MB on different boxes, the kernel path is not tied to it), else by
// hipMemcpyAsync (pageable memory: the runtime stages it).
static int d2h(fb_ctx *c, void *dst, const void *src, size_t bytes) {
    if (!bytes) return FB_OK;
    if ((bytes & 3) == 0) {
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, dst) == hipSuccess && at.type == hipMemoryTypeHost && at.devicePointer) {
            launch_copy_words((uint32_t *)at.devicePointer, (const uint32_t *)src, (int64_t)(bytes / 4), Stream(c->stream));
            HIPCHK(c, hipGetLastError());
            return FB_OK;
        }
        (void)hipGetLastError();
    }
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    return FB_OK;
}
// Device pointer of the waited tick's dense orphan list: an f_emit tick left per-tile
// segments, gathered into orph_dense here (once per tick).
static int64_t *orph_dense_dev(fb_ctx *c) {
    if (!c->l_oseg) return c->orphans;
    if (!c->dense_ok) {
        launch_orph_gather(c->orph_dense, c->orphans, c->fcnt, c->l_nbf, Stream(c->stream));
        c->dense_ok = true;
    }
    return c->orph_dense;
}
// n orphans of the waited tick into dst; the whole list of segments goes straight into
// pinned host memory by the gather kernel
static int orph_out(fb_ctx *c, int64_t *dst, int64_t n) {
    if (!n) return FB_OK;
    if (c->l_oseg && n == c->last.n_orphans_local) {
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, dst) == hipSuccess && at.type == hipMemoryTypeHost && at.devicePointer) {
            launch_orph_gather((int64_t *)at.devicePointer, c->orphans, c->fcnt, c->l_nbf, Stream(c->stream));
            HIPCHK(c, hipGetLastError());
            return FB_OK;
        }
        (void)hipGetLastError();
    }
    return d2h(c, dst, orph_dense_dev(c), (size_t)n * 8);
}
// A window tick leaves its evicted slots to the per-slot status bytes: the ascending list
// is built (once per tick) when something reads it.
static int evict_ready(fb_ctx *c) {
    if (!c->l_win || c->evict_ok || !c->last.n_evicted) return FB_OK;
    launch_evict_gather(c->evicted, c->st, c->wcnt, c->wpre, c->W, Stream(c->stream));
    HIPCHK(c, hipGetLastError());
    c->evict_ok = true;
    return FB_OK;
}
static int copy_out(fb_ctx *c, void *dst, const void *src, size_t bytes) {
    if (!bytes) return FB_OK;
    if (int rc = d2h(c, dst, src, bytes)) return rc;
    HIPCHK(c, stream_wait(c));
    return FB_OK;
}

int fb_get_assignments(fb_ctx *c, int64_t first, int64_t n, int32_t *dst) {
    if (!c || !dst) return FB_EINVAL;
    if (!c->waited) return fail(c, FB_ESTATE, "no waited tick");
    if (c->shard && !c->l_full)
        return fail(c, FB_ESTATE, "sharded context: use fb_get_local_assignments (or fb_set_full_assign)");
    if (first < 0 || n < 0 || first + n > c->last.n_assigned) return fail(c, FB_EINVAL, "assignment range");
    if (c->shard) return copy_out(c, dst, c->assign_all + first, (size_t)n * 4);
    return copy_out(c, dst, c->log_slot + c->l_head + first, (size_t)n * 4);
}

int fb_get_orphans(fb_ctx *c, int64_t n, int64_t *dst) {
    if (!c || !dst) return FB_EINVAL;
    if (!c->waited) return fail(c, FB_ESTATE, "no waited tick");
    if (n < 0 || n > c->last.n_orphans_local) return fail(c, FB_EINVAL, "orphan count");
    HIPCHK(c, hipSetDevice(c->device));
    if (int rc = orph_out(c, dst, n)) return rc;
    HIPCHK(c, stream_wait(c));
    return FB_OK;
}

int fb_get_evicted(fb_ctx *c, int32_t n, int32_t *dst) {
    if (!c || !dst) return FB_EINVAL;
    if (!c->waited) return fail(c, FB_ESTATE, "no waited tick");
    if (n < 0 || n > c->last.n_evicted) return fail(c, FB_EINVAL, "evicted count");
    HIPCHK(c, hipSetDevice(c->device));
    if (c->l_cout) {  // the tick wrote them into the registered pinned buffer
        if (n && dst != c->cout_host[3]) memcpy(dst, c->cout_host[3], (size_t)n * 4);
        return FB_OK;
    }
    if (int rc = evict_ready(c)) return rc;
    return copy_out(c, dst, c->evicted, (size_t)n * 4);
}

int fb_get_outputs(fb_ctx *c, int32_t *assign, int64_t *orphans, int32_t *evicted) {
    if (!c) return FB_EINVAL;
    if (!c->waited) return fail(c, FB_ESTATE, "no waited tick");
    if (assign && c->shard) return fail(c, FB_ESTATE, "sharded context: use fb_get_local_assignments");
    HIPCHK(c, hipSetDevice(c->device));
    // the three copies back to back on the stream, one synchronisation
    int rc;
    if (assign && c->last.n_assigned && (rc = d2h(c, assign, c->log_slot + c->l_head, (size_t)c->last.n_assigned * 4)))
        return rc;
    if (orphans && (rc = orph_out(c, orphans, c->last.n_orphans_local))) return rc;
    if (evicted && (rc = evict_ready(c))) return rc;
    if (evicted && c->last.n_evicted && c->l_cout) {
        if (evicted != c->cout_host[3]) memcpy(evicted, c->cout_host[3], (size_t)c->last.n_evicted * 4);
    } else if (evicted && c->last.n_evicted && (rc = d2h(c, evicted, c->evicted, (size_t)c->last.n_evicted * 4))) {
        return rc;
    }
    HIPCHK(c, stream_wait(c));
    return FB_OK;
}

int fb_set_window(fb_ctx *c, int mode) {
    if (!c) return FB_EINVAL;
    if (c->shard || c->deque) return fail(c, FB_ESTATE, "window ticks exist on one-GPU heartbeat contexts only");
    if (mode < -1 || mode > 1) return fail(c, FB_EINVAL, "window mode %d (-1 auto, 0 off, 1 on)", mode);
    if (c->launched) return fail(c, FB_ESTATE, "fb_set_window between ticks only");
    if (int rc = flush_commit(c)) return rc;
    if (mode > 0) {
        if (int rc = win_alloc(c)) return rc;
    }
    c->win = mode;
    return FB_OK;
}

int fb_set_eager_commit(fb_ctx *c, int enable) {
    if (!c) return FB_EINVAL;
    if (c->launched && !c->waited) return fail(c, FB_ESTATE, "fb_set_eager_commit with a tick in flight");
    c->eager = enable ? 1 : 0;
    return FB_OK;
}

int fb_window_stats(fb_ctx *c, int64_t *window_ticks, int64_t *fallbacks) {
    if (!c) return FB_EINVAL;
    if (window_ticks) *window_ticks = c->win_ticks;
    if (fallbacks) *fallbacks = c->win_fallbacks;
    return FB_OK;
}

int fb_set_compact_out(fb_ctx *c, int32_t *slot, uint8_t *cnt, int64_t cap, int64_t *orphans, int64_t ocap,
                       int32_t *evicted, int64_t ecap) {
    if (!c) return FB_EINVAL;
    if (c->shard) return fail(c, FB_ESTATE, "compact assignments exist on one-GPU contexts only");
    if (c->launched && !c->waited) return fail(c, FB_ESTATE, "fb_set_compact_out with a tick in flight");
    if (!slot) {  // unregister
        c->cout_slot = nullptr;
        return FB_OK;
    }
    if (!cnt || !orphans || !evicted || cap < 0 || ocap < 0 || ecap < 0) return FB_EINVAL;
    void *dv[4];
    const void *hp[4] = {slot, cnt, orphans, evicted};
    for (int j = 0; j < 4; ++j) {
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, hp[j]) != hipSuccess || at.type != hipMemoryTypeHost || !at.devicePointer) {
            (void)hipGetLastError();
            return fail(c, FB_EINVAL, "compact output buffers must be pinned host memory (fb_host_alloc)");
        }
        dv[j] = at.devicePointer;
        c->cout_host[j] = hp[j];
    }
    c->cout_slot = (int32_t *)dv[0];
    c->cout_c = (uint8_t *)dv[1];
    c->cout_orph = (int64_t *)dv[2];
    c->cout_ev = (int32_t *)dv[3];
    c->cout_cap = cap;
    c->cout_ocap = ocap;
    c->cout_ecap = ecap;
    c->compact = 1;
    return FB_OK;
}

int fb_set_compact(fb_ctx *c, int enable) {
    if (!c) return FB_EINVAL;
    if (c->shard) return fail(c, FB_ESTATE, "compact assignments exist on one-GPU contexts only");
    c->compact = enable != 0;
    return FB_OK;
}

int fb_get_outputs_compact(fb_ctx *c, int32_t *slot, uint8_t *cnt, int64_t cap, int64_t *n_pos, int64_t *orphans,
                           int32_t *evicted) {
    if (!c || !n_pos) return FB_EINVAL;
    if (!c->waited) return fail(c, FB_ESTATE, "no waited tick");
    if (!c->l_compact) return fail(c, FB_ESTATE, "the tick was launched without fb_set_compact");
    if (c->last.fill_level + 1 > 255)
        return fail(c, FB_ERANGE, "fill level %d: rounds beyond a byte, read fb_get_outputs", c->last.fill_level);
    const int64_t n = c->l_Qn + 2 * (int64_t)c->l_E;
    *n_pos = n;
    // the tick wrote into the registered buffers: nothing left to copy into those
    if (c->l_cout && (!slot || slot == c->cout_host[0]) && (!cnt || cnt == c->cout_host[1]) &&
        (!orphans || orphans == c->cout_host[2]) && (!evicted || evicted == c->cout_host[3]))
        return FB_OK;
    if ((slot || cnt) && cap < n) return fail(c, FB_EINVAL, "compact buffers of %lld < %lld positions", (long long)cap,
                                              (long long)n);
    HIPCHK(c, hipSetDevice(c->device));
    int rc;
    // into pinned memory: the word copies in one kernel (and the orphan segments gathered
    // straight into their buffer), else one transfer per array
    CopyMulti m{};
    auto mapped = [](void *p) -> uint32_t * {
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost && at.devicePointer)
            return (uint32_t *)at.devicePointer;
        (void)hipGetLastError();
        return nullptr;
    };
    auto add = [&](void *dst, const void *src, int64_t bytes) -> bool {
        uint32_t *d = (bytes & 3) == 0 ? mapped(dst) : nullptr;
        if (!d) return false;
        const int b0 = m.n ? m.blk0[m.n - 1] + (int)std::min<int64_t>(
                                                       std::max<int64_t>(1, (m.words[m.n - 1] + 4 * kBS - 1) / (4 * kBS)), 512)
                           : 0;
        m.dst[m.n] = d;
        m.src[m.n] = (const uint32_t *)src;
        m.words[m.n] = bytes / 4;
        m.blk0[m.n] = b0;
        m.n++;
        return true;
    };
    // the c bytes travel as whole words when the caller's buffer has room for the padding
    const int64_t cw = (n + 3) & ~(int64_t)3;
    if (c->l_cout) {  // the tick wrote the compact form into the registered buffers
        if (slot && n && slot != c->cout_host[0]) memcpy(slot, c->cout_host[0], (size_t)n * 4);
        if (cnt && n && cnt != c->cout_host[1]) memcpy(cnt, c->cout_host[1], (size_t)n);
    } else {
        if (slot && n && !add(slot, c->rb_slot, n * 4) && (rc = d2h(c, slot, c->rb_slot, (size_t)n * 4))) return rc;
        if (cnt && n && !(cw <= cap && add(cnt, c->rb_c, cw)) && (rc = d2h(c, cnt, c->rb_c, (size_t)n))) return rc;
    }
    if (evicted && c->last.n_evicted && c->l_cout) {
        if (evicted != c->cout_host[3]) memcpy(evicted, c->cout_host[3], (size_t)c->last.n_evicted * 4);
    } else if (evicted && c->last.n_evicted && !add(evicted, c->evicted, (int64_t)c->last.n_evicted * 4) &&
               (rc = d2h(c, evicted, c->evicted, (size_t)c->last.n_evicted * 4))) {
        return rc;
    }
    // the orphans' segments gathered by the same launch when they go to pinned memory
    bool orph_done = false;
    if (orphans && c->l_oseg && c->last.n_orphans_local) {
        if (int64_t *od = (int64_t *)mapped(orphans)) {
            m.odst = od;
            m.osrc = c->orphans;
            m.ocnt = c->fcnt;
            m.otiles = c->l_nbf;
            orph_done = true;
        }
    }
    launch_copy_multi(m, Stream(c->stream));
    HIPCHK(c, hipGetLastError());
    if (orphans && !orph_done && (rc = orph_out(c, orphans, c->last.n_orphans_local))) return rc;
    HIPCHK(c, stream_wait(c));
    return FB_OK;
}

// Host: every task's slot from the compact form of the waited tick.  Round r <= L
// serves the positions with c > r in LRU order, task S(r) + j going to the j-th of
// them; S(r) = sum of min(c, r).  The rounds are independent ranges of the output,
// so they are expanded in parallel (FAASBAL_EXPAND_THREADS workers, default 8).
int fb_expand_compact(fb_ctx *c, const int32_t *slot, const uint8_t *cnt, int64_t n_pos, int32_t *assign) {
    if (!c || (n_pos && (!slot || !cnt)) || (!assign && c->last.n_assigned)) return FB_EINVAL;
    if (!c->waited) return fail(c, FB_ESTATE, "no waited tick");
    const int L = c->last.fill_level;
    const int64_t N = c->last.n_assigned;
    if (L + 1 > 255) return fail(c, FB_ERANGE, "fill level %d beyond the compact form", L);
    // A(r) = #{c > r}, S(r + 1) = S(r) + A(r), r <= L
    std::vector<int64_t> hist(L + 3, 0), S(L + 2, 0);
    for (int64_t i = 0; i < n_pos; ++i) hist[std::min<int>(cnt[i], L + 2)]++;
    int64_t above = 0;
    std::vector<int64_t> A(L + 2, 0);
    for (int r = L + 1; r >= 0; --r) {
        above += hist[r + 1];
        A[r] = above;
    }
    for (int r = 0; r <= L; ++r) S[r + 1] = S[r] + A[r];
    if (S[L] > N || N > S[L + 1]) return fail(c, FB_EINVAL, "compact form does not match the waited tick");
    if (!c->xpool) {
        const char *e = getenv("FAASBAL_EXPAND_THREADS");
        c->xpool = new HostPool(std::max(1, std::min(e ? atoi(e) : 8, 64)));
    }
    const int np = c->xpool->size();
    c->xpool->run([&](int t) {
        for (int r = t; r <= L; r += np) {
            int32_t *o = assign + S[r];
            const int64_t lim = std::min<int64_t>(A[r], N - S[r]);
            int64_t k = 0;
            for (int64_t i = 0; i < n_pos && k < lim; ++i)
                if (cnt[i] > r) o[k++] = slot[i];
        }
    });
    return FB_OK;
}

int fb_host_alloc(fb_ctx *c, int64_t bytes, void **ptr) {
    if (!c || !ptr || bytes < 0) return FB_EINVAL;
    *ptr = nullptr;
    HIPCHK(c, hipSetDevice(c->device));
    if (hipHostMalloc(ptr, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault) != hipSuccess)
        return fail(c, FB_ENOMEM, "hipHostMalloc(%lld B) failed", (long long)bytes);
    return FB_OK;
}

int fb_host_free(fb_ctx *c, void *ptr) {
    // pinned host memory belongs to the process, not to the context: ctx may be NULL
    // (a buffer that outlives its context is freed when its last user lets it go)
    if (!c) return (!ptr || hipHostFree(ptr) == hipSuccess) ? FB_OK : FB_EHIP;
    if (ptr) HIPCHK(c, hipHostFree(ptr));
    return FB_OK;
}

int fb_get_event_status(fb_ctx *c, int32_t n, uint8_t *dst) {
    if (!c || !dst) return FB_EINVAL;
    if (!c->waited) return fail(c, FB_ESTATE, "no waited tick");
    if (n < 0 || n > c->l_E) return fail(c, FB_EINVAL, "event count");
    const uint8_t *src = c->shard ? c->xbuf + xlayout(c->world, c->l_E, c->l_Qn + 2 * (int64_t)c->l_E).evs : c->ev_status;
    if (n) HIPCHK(c, hipMemcpy(dst, src, (size_t)n, hipMemcpyDeviceToHost));
    return FB_OK;
}

namespace {
// wait for the launched tick, copy the requested outputs, commit
int finish_tick(fb_ctx *c, int32_t n_events, fb_tick_result *res, uint8_t *ev_status, int32_t *assign,
                int64_t *orphans, int32_t *evicted) {
    int rc;
    fb_tick_result r;
    if ((rc = fb_tick_wait(c, &r))) return rc;
    if (ev_status && (rc = fb_get_event_status(c, n_events, ev_status))) return rc;
    if (assign && (rc = fb_get_assignments(c, 0, r.n_assigned, assign))) return rc;
    if (orphans && (rc = fb_get_orphans(c, r.n_orphans, orphans))) return rc;
    if (evicted && (rc = fb_get_evicted(c, r.n_evicted, evicted))) return rc;
    if (res) *res = r;
    return fb_tick_commit(c);
}
}  // namespace

int fb_apply_events(fb_ctx *c, double tte, int32_t n_events, const uint8_t *kind, const int32_t *slot,
                    const int32_t *val, const double *ts, const int64_t *seq, fb_tick_result *res,
                    uint8_t *ev_status, int64_t *orphans, int32_t *evicted) {
    if (!c) return FB_EINVAL;
    if (c->shard) return fail(c, FB_ESTATE, "fb_apply_events on a sharded context (use the two-phase tick)");
    if (n_events < 0 || (n_events && !ts)) return fail(c, FB_EINVAL, "event arrays");
    if (res) *res = fb_tick_result{};
    if (!n_events) return FB_OK;
    // the messages, each after the purge at its own clock, then the purge that follows
    // the last one (:390) at that clock; nothing dispatched, orphans reported
    int rc = fb_tick_stage(c, ts[n_events - 1], n_events, kind, slot, val, ts, seq);
    if (rc) return rc;
    c->next_purge_only = true;
    if ((rc = fb_tick_launch_staged(c, tte, 0))) return rc;
    return finish_tick(c, n_events, res, ev_status, nullptr, orphans, evicted);
}

int fb_purge(fb_ctx *c, double now, double tte, fb_tick_result *res, int64_t *orphans, int32_t *evicted) {
    if (!c) return FB_EINVAL;
    if (c->shard) return fail(c, FB_ESTATE, "fb_purge on a sharded context (fb_purge_launch + exchange)");
    int rc = fb_purge_launch(c, now, tte);
    if (rc) return rc;
    return finish_tick(c, 0, res, nullptr, nullptr, orphans, evicted);
}

int fb_assign(fb_ctx *c, double now, double tte, int64_t n_tasks, fb_tick_result *res, int32_t *assign,
              int64_t *orphans, int32_t *evicted) {
    if (!c) return FB_EINVAL;
    if (c->shard) return fail(c, FB_ESTATE, "fb_assign on a sharded context (use the two-phase tick)");
    int rc = fb_tick_launch(c, now, tte, 0, nullptr, nullptr, nullptr, nullptr, nullptr, n_tasks);
    if (rc) return rc;
    return finish_tick(c, 0, res, nullptr, assign, orphans, evicted);
}

int fb_tick(fb_ctx *c, double now, double tte, int32_t n_events, const uint8_t *kind, const int32_t *slot,
            const int32_t *val, const double *ts, const int64_t *seq, int64_t n_pending, fb_tick_result *res,
            uint8_t *ev_status, int32_t *assign, int64_t *orphans, int32_t *evicted) {
    int rc = fb_tick_launch(c, now, tte, n_events, kind, slot, val, ts, seq, n_pending);
    if (rc) return rc;
    fb_tick_result r;
    if ((rc = fb_tick_wait(c, &r))) return rc;
    if (ev_status && (rc = fb_get_event_status(c, n_events, ev_status))) return rc;
    if (assign && (rc = fb_get_assignments(c, 0, r.n_assigned, assign))) return rc;
    if (orphans && (rc = fb_get_orphans(c, r.n_orphans, orphans))) return rc;
    if (evicted && (rc = fb_get_evicted(c, r.n_evicted, evicted))) return rc;
    if (res) *res = r;
    return fb_tick_commit(c);
}

int fb_device_view_get(fb_ctx *c, fb_device_view *v) {
    if (!c || !v) return FB_EINVAL;
    if (int rc_ = win_uncommitted(c, "fb_device_view_get")) return rc_;
    if (int rc_ = flush_commit(c)) return rc_;
    v->free_processes = &c->free_[c->cur]->x;
    v->free_processes_stride = (int32_t)sizeof(int2);
    v->last_heartbeat = c->hb;
    v->last_heartbeat_stride = (int32_t)sizeof(double);
    v->registered = c->reg;
    if (c->win_cap && (c->qoff != 0 || c->Qn != c->Qtrue)) {
        if (int rc = win_normalize(c)) return rc;
    }
    v->queue = c->queue[c->qcur];
    if (int rc_ = log_settle(c)) return rc_;
    v->log_slot = c->log_slot;
    v->orphans = orph_dense_dev(c);
    if (c->waited) {
        if (int rc = evict_ready(c)) return rc;
        HIPCHK(c, stream_wait(c));
    }
    v->evicted = c->l_cout ? c->cout_ev : c->evicted;
    v->n_workers = c->W;
    v->queue_len = c->Qn;
    v->log_head = c->head;
    return FB_OK;
}

int fb_set_full_assign(fb_ctx *c, int on) {
    if (!c) return FB_EINVAL;
    if (c->launched) return fail(c, FB_ESTATE, "fb_set_full_assign between ticks only");
    if (!c->shard) return fail(c, FB_ESTATE, "fb_set_full_assign on a one-GPU context (it always has them)");
    c->full_assign = on ? 1 : 0;
    return FB_OK;
}

int fb_set_round_hint(fb_ctx *c, int32_t max_free) {
    if (!c) return FB_EINVAL;
    if (c->launched) return fail(c, FB_ESTATE, "fb_set_round_hint between ticks only");
    c->maxc_hint = std::max<int32_t>(1, max_free);
    return FB_OK;
}

int fb_set_path(fb_ctx *c, const char *name, int value) {
    if (!c || !name) return FB_EINVAL;
    if (c->launched) return fail(c, FB_ESTATE, "fb_set_path between ticks only");
    if (int rc_ = flush_commit(c)) return rc_;
    const std::string n(name);
    if (n == "plan" && value >= 0 && value <= 2) c->force_plan = value;
    else if (n == "logscan" && value >= -1 && value <= 1) c->logscan = value;
    else if (n == "split_slots" && value >= -1 && value <= 1) c->split_slots = value;
    else if (n == "ev_ll" && (value == 0 || value == 1)) c->ev_ll = value;
    else if (n == "rs_wide" && (value == 0 || value == 1)) c->rs_wide = value;
    else if (n == "fault_qlen") c->fault_qlen = value;
    else if (n == "xplan" && (value == 0 || value == 1)) c->xplan_on = value;
    else if (n == "gp" && (value == 0 || value == 1)) c->gp_on = value;
    else if (n == "win_direct" && (value == 0 || value == 1)) c->win_direct = value;
    else if (n == "xself" && (value == 0 || value == 1)) c->xself_on = value;
    else if (n == "wfirst" && (value == 0 || value == 1)) c->wfirst_on = value;
    else if (n == "gpcheck" && (value == 0 || value == 1)) c->gpcheck = value;
    else if (n == "cmix" && (value == 0 || value == 1)) c->cmix_on = value;
    else if (n == "wtiles" && (value == 0 || value == 1 || value == 2 || value == 4)) c->wtiles = value;
    else if (n == "qtiles" && (value == 0 || value == 1 || value == 4)) c->qtiles = value;
    else if (n == "lazy" && (value == 0 || value == 1)) {
        if (!value && c->stale_any) {  // the entries left so far leave the log first
            if (int rc_ = log_settle(c)) return rc_;
        }
        c->lazy_on = value;
    }
    else if (n == "xcfirst" && (value == 0 || value == 1)) c->xcfirst_on = value;
    else return fail(c, FB_EINVAL, "fb_set_path(\"%s\", %d): unknown path or value", name, value);
    return FB_OK;
}

int fb_timing_enable(fb_ctx *c, int enable) {
    if (!c) return FB_EINVAL;
    c->timing = enable != 0;
    return FB_OK;
}

int fb_timing_gate(fb_ctx *c, int hold) {
    if (!c) return FB_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    if (hold) {
        if (c->gate_state == 1) return fail(c, FB_ESTATE, "fb_timing_gate: the gate is already held");
        if (!c->gate_h) {
            if (hipHostMalloc((void **)&c->gate_h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
                return fail(c, FB_ENOMEM, "fb_timing_gate: hipHostMalloc failed");
            memset(c->gate_h, 0, 64);
            HIPCHK(c, hipHostGetDevicePointer((void **)&c->gate_d, c->gate_h, 0));
            HIPCHK(c, hipEventCreate(&c->gate_a));
            HIPCHK(c, hipEventCreate(&c->gate_b));
        }
        // (a pending deferred commit stays pending: it rides in the next gated launch as usual)
        if (++c->gate_seq == 0) c->gate_seq = 1;
        __atomic_store_n(&c->gate_h[1], 0u, __ATOMIC_RELEASE);
        // the gate opens by itself after 0.5 s (5e7 ticks of the 100 MHz counter)
        launch_gate(c->gate_d, c->gate_seq, 50000000ull, Stream(c->stream, nullptr, c->gate_a));
        HIPCHK(c, hipGetLastError());
        c->gate_state = 1;
        return FB_OK;
    }
    if (c->gate_state != 1) return fail(c, FB_ESTATE, "fb_timing_gate(0) without a held gate");
    HIPCHK(c, hipEventRecord(c->gate_b, c->stream));
    __atomic_store_n(&c->gate_h[0], c->gate_seq, __ATOMIC_RELEASE);
    c->gate_state = 2;
    return FB_OK;
}

int fb_timing_mark(fb_ctx *c) {
    if (!c) return FB_EINVAL;
    if (c->gate_state == 1) return fail(c, FB_ESTATE, "fb_timing_mark while the gate is held");
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->gate_h) {
        // (the gate's word, so the mark finds it open)
        if (int rc_ = fb_timing_gate(c, 1)) return rc_;
        return fb_timing_gate(c, 0);
    }
    launch_gate(c->gate_d, c->gate_seq, 50000000ull, Stream(c->stream));
    HIPCHK(c, hipGetLastError());
    return FB_OK;
}

int fb_timing_span(fb_ctx *c, double *ms, int32_t *timed_out) {
    if (!c) return FB_EINVAL;
    if (c->gate_state != 2) return fail(c, FB_ESTATE, "fb_timing_span without a released gate");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    float f = 0;
    HIPCHK(c, hipEventElapsedTime(&f, c->gate_a, c->gate_b));
    if (ms) *ms = f;
    if (timed_out) *timed_out = (int32_t)__atomic_load_n(&c->gate_h[1], __ATOMIC_ACQUIRE);
    return FB_OK;
}

int fb_timing_read(fb_ctx *c, int32_t max_kernels, const char **names, double *total_ms, int64_t *launches,
                   int32_t *n_kernels) {
    if (!c) return FB_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    std::vector<const char *> nm;
    std::vector<double> ms;
    std::vector<int64_t> cnt;
    for (auto &t : c->tl) {
        float f = 0;
        HIPCHK(c, hipEventElapsedTime(&f, t.a, t.b));
        size_t k = 0;
        while (k < nm.size() && strcmp(nm[k], t.name)) ++k;
        if (k == nm.size()) {
            nm.push_back(t.name);
            ms.push_back(0);
            cnt.push_back(0);
        }
        ms[k] += f;
        cnt[k] += 1;
        c->ev_pool.push_back(t.a);
        c->ev_pool.push_back(t.b);
    }
    c->tl.clear();
    const int n = (int)std::min<size_t>(nm.size(), (size_t)std::max(max_kernels, 0));
    for (int i = 0; i < n; ++i) {
        if (names) names[i] = nm[i];
        if (total_ms) total_ms[i] = ms[i];
        if (launches) launches[i] = cnt[i];
    }
    if (n_kernels) *n_kernels = n;
    return FB_OK;
}

// Device self-test of the wave/block primitives (DPP scans); *errors = mismatches.
int fb_selftest(fb_ctx *c, int32_t *errors) {
    if (!c || !errors) return FB_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    uint32_t *d = nullptr;
    int rc = dalloc(c, &d, 1);
    if (rc) return rc;
    HIPCHK(c, hipMemsetAsync(d, 0, 4, c->stream));
    for (uint32_t seed = 1; seed <= 8; ++seed) launch_selftest(d, seed * 7919u, c->stream);
    uint32_t h = 0;
    HIPCHK(c, hipMemcpyAsync(&h, d, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, stream_wait(c));
    hipFree(d);
    *errors = (int32_t)h;
    return FB_OK;
}

// Diagnostic: copy the stamp buffer (meaningful only in FAASBAL_STAMPS builds).
int fb_debug_read(fb_ctx *c, unsigned long long *dst, int64_t n, int64_t *n_total) {
    if (!c) return FB_EINVAL;
    if (int rc_ = flush_commit(c)) return rc_;
    HIPCHK(c, stream_wait(c));
    if (n_total) *n_total = (int64_t)c->dbg_n;
    if (dst && n > 0) HIPCHK(c, hipMemcpy(dst, c->dbg, (size_t)std::min<int64_t>(n, c->dbg_n) * 8, hipMemcpyDeviceToHost));
    return FB_OK;
}

int fb_sync(fb_ctx *c) {
    if (!c) return FB_EINVAL;
    if (int rc_ = flush_commit(c)) return rc_;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, stream_wait(c));
    return FB_OK;
}

}  // extern "C"
