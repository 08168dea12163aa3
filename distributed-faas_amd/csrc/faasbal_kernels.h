// faasbal_kernels.h -- internal: constants and kernel argument blocks.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace fb {

constexpr int kBS = 256;           // threads per workgroup (4 wave64)
constexpr int kWaves = kBS / 64;
constexpr int kTrashRows = 1024;   // k_emit2: trash rows (one per block, modulo) for branch-free stores
constexpr int kStagePar = 16384;   // host: event batches this large are staged by the worker pool
// sharded exchange record: a rank's orphan count as partials on kXRecLines separate
// 128-byte lines (device atomics on one line serialise, ~6 ns each)
constexpr int kXRecLines = 8;
constexpr int kXRecWords = kXRecLines * 16;  // u64 words per rank (1 KB)
// Exchanged block rows (sharded ticks whose round table has <= kRFused rows and whose
// LRU order spans <= kXRowsMaxBlocks queue blocks, <= kXRowsMaxWorld ranks): phase 1
// writes, per queue block, its own positions' counts of c > r for r <= R as three
// 4-bit digits, one byte each ([block][digit][xr_stride(R)] bytes); the SUM all-reduce
// adds at most 16 digits of 15 per byte, so the rows arrive as every rank's counts and
// phase 2 is one launch (no re-count of the exchanged c values, no group rows).
constexpr int kXRowsMaxBlocks = 256;  // packed 16-bit column sums: 256 x 240 < 65536
constexpr int kXRowsMaxWorld = 16;
constexpr int kXRowDigits = 3;  // a block count is <= 256 < 16^3
__host__ __device__ constexpr int xr_stride(int R) { return (R + 1 + 3) & ~3; }
// a block's row: the three digit rows, padded to 16 bytes (phase 2 reads it in int4s)
__host__ __device__ constexpr int xr_row(int R) { return (kXRowDigits * xr_stride(R) + 15) & ~15; }
constexpr int kXRowMaxBytes = (kXRowDigits * ((128 + 1 + 3) & ~3) + 15) & ~15;
// ... and at R = 32 (the configs[2] shapes), per group of 16 queue blocks too: the group's
// last phase-1 block (a ticket per group) writes the group's sums as a 4-digit row (a group
// count is <= 16 x 256 < 16^4) and this rank's own group row, so a phase-2 block reads the
// <= 16 group rows and the rows of the earlier blocks of its group (16 lanes per load column)
constexpr int kXGroupBlocks = 16;
constexpr int kXGroupDigits = 4;
constexpr int kXGroupR = 32;
__host__ __device__ constexpr int xg_row(int R) { return (kXGroupDigits * xr_stride(R) + 15) & ~15; }
constexpr int kXgAccStride = 36;  // words per group accumulator row (R + 1 = 33 columns)
constexpr int kXsBlocks = 64;      // k_xscan: queue blocks per workgroup (chunk): a lane per block
// phase 2: the parts (lanes) per 16-byte load column of the digit rows, a power of two
// with every column's parts in one workgroup; own rows (R / 4 columns) use kBS / (R / 4)
__host__ __device__ constexpr int xr_parts(int R) {
    return (xr_row(R) >> 4) * 32 <= kBS ? 32 : ((xr_row(R) >> 4) * 16 <= kBS ? 16 : 8);
}
constexpr int kFItems = 8;         // log entries per thread in log-role blocks
constexpr int kFTile = kBS * kFItems;
#ifndef FAASBAL_RS_ITEMS
#define FAASBAL_RS_ITEMS 8
#endif
constexpr int kRsItems = FAASBAL_RS_ITEMS;  // radix sort: keys per thread per tile
constexpr int kRsTile = kBS * kRsItems;
constexpr int kRFused = 128;       // fused tick: round table of at most 128 rows ...
constexpr int kTabLd = 16;         // ... read by at most 16 int4 loads per thread
constexpr int kPeel = 4;           // fused tick: block-count arrays of at most 4*256 entries
constexpr int kLdsBitmapSlots = 1 << 17;  // died bitmap staged in LDS up to 128K slots (16 KB)
constexpr int kLsBS = 1024;        // k_logscan: one 16-wave workgroup per CU
// group rows of round totals (<= 64 groups x (R + 4) words; sharded phase 2: x (2 R + 4))
constexpr int kGrpWords = 64 * 260;
constexpr int kShardMaxR = 4096;     // sharded round tables (k_emit_shard_wide: 64 chunks of 64 rounds)

// event kinds / status (include/faasbal.h)
constexpr int kEvRegister = 0, kEvReconnect = 1, kEvHeartbeat = 2, kEvResult = 3, kEvOther = 4;
constexpr uint8_t kEvsApplied = 0, kEvsReconnect = 1;

// deque mode (PushDispatcher.start): a committed token rank with this bit set sat in
// A_L[p:] of the tick that wrote it (final rank = j - x_w), else in A_L[:p] (K_L - x_w + j)
constexpr uint32_t kPart2 = 1u << 30;
constexpr uint8_t kEvsUnknown = 2;  // deque mode: result from an id without a record (KeyError, :291)

// per-slot tick status (st)
constexpr uint8_t kStAlive = 1;      // registered and alive after the final purge
constexpr uint8_t kStDiedStart = 2;  // the registration alive at tick start died this tick
constexpr uint8_t kStEvicted = 4;    // record deleted during the tick and not re-created
// post flags (post_rf >> 1): bit0 died_start, bits 1-2 queue status after the tick's messages
constexpr int kPfDiedStart = 1;
constexpr int kQsKeep = 0, kQsOut = 1, kQsFront = 2, kQsBack = 3;
// post_rf bit 4 (one-GPU heartbeat contexts): a result of this tick completed one of the
// slot's in-flight entries (ctag[q] == the launch stamp names which); the log itself is
// cleared only by the commit, so an orphan test of that slot's entries checks ctag
constexpr uint8_t kRfCleared = 16;
// post_rf bit 5: the slot was in the committed queue at tick start (window ticks: a front /
// back insertion of such a slot leaves a position to tombstone)
constexpr uint8_t kRfQ0 = 32;
// k_emit2's log tiles (one-GPU fused ticks): at most this many log workgroups (4 tiles
// of kFTile entries each; k_orph_gather sums up to 4 x this many tile counts per block)
constexpr int kFEmitMaxBlocks = 1024;
// window ticks (sliding level-0 queue, one GPU): 1024-element chunks of the
// virtual order [backs][fronts][window prefix], one k_emit_win workgroup each (at most
// kWinMaxCh: the look-back granules hold 22-bit prefixes)
constexpr int kWinCh = 1024;
constexpr int kWinMaxCh = 4096;
constexpr int32_t kTomb = INT32_MIN;  // qfree of a window position whose slot left the queue
// st bit: the slot was in the committed queue at tick start (window commits)
constexpr uint8_t kStQ0 = 8;
// Committed per-slot heartbeat: last_heartbeat, NaN when the slot holds no record
// (so the log scan's one 8-byte gather per in-flight entry decides liveness
// without a registered flag); the first log sequence of the current registration
// lives in its own array (epoch).  Log entries of a dead registration are cleared (-1)
// when the tick that redistributed them commits -- except on one-GPU heartbeat contexts
// (round 6, lazy clears): there the commit leaves them, and an entry q naming slot s is
// live only if s holds a record and q >= epoch[s] (entries of a registration that died
// are older than any later registration of the slot).  Kernels test that (live_chk) only
// once such entries may exist; state reads clear them first (k_log_normalize).

// Post-message record of a slot that got messages this tick (k_ev_apply*): one
// 16-byte store per slot; its registered flag and queue flags ride in post_rf
// (bit 0 registered, bit 1 died_start, bits 2-3 queue status: rf >> 1 = post flags).
struct alignas(16) PostRec {
    double hb;
    int32_t free;
    uint32_t epoch;
};

// results of a tick, written by k_emit into host-mapped pinned memory
struct HostOut {
    int64_t O;          // orphans redistributed first
    int64_t n_evicted;
    int64_t N_eff;      // tasks dispatched
    int64_t p;          // tasks of the partial round L
    int64_t AL;         // |A_L|
    int64_t new_qlen;   // next LRU queue length
    int64_t cap_total;  // sum of c over live queued workers
    int32_t L;          // fill level
    int32_t maxc;       // max c
    int32_t status;     // 1 = round table too narrow (rerun wider), 2 = in-flight log full,
                        // 3 = window tick cannot finish in its window (rerun as a general tick)
                        // (deque contexts: new_qlen > token capacity is checked by the host)
    int32_t resort;     // k_ev_apply_ll: a slot got too many messages, rerun through the sort
    int64_t n_local;   // sharded: tasks appended to this rank's log shard
    int64_t O_local;    // sharded: this rank's orphans
    // window ticks: the next window [win_head, win_head + new_qlen) of the queue buffer
    // (tombstones included), the LRU queue's true length, and a store past the buffer
    int64_t win_head;
    int64_t win_qlen;
    int32_t win_ovf;
    int32_t bad_ev;     // k_ev_link: an invalid message (slot, kind, timestamp; cleared by the host)
};

// totals computed by k_plan (large grids only; device memory, no atomics)
struct DevTotals {
    int64_t O, n_evicted, cap_total;  // O: orphans of every rank (tasks dispatched first)
    int32_t maxc, pad;
    int64_t O_local;                  // sharded: this rank's orphans
};

struct CommitArgs {
    int W;
    int slot_base;
    int nbw;            // slot blocks; blocks [nbw, nbw + ceil(n_orph / 256)) clear orphaned log entries
    int32_t *bud;              // one-GPU heartbeat: touched slots get bud_next[s] (budget after the tick)
    const int32_t *bud_next;
    const uint32_t *oseg;  // non-null: orphans in per-tile segments (orphans[t*2048 + i], i < oseg[t]),
                           // blocks [nbw, nbw + nbo) a wave per tile of the oseg_tiles
    int oseg_tiles;
    int nbo;            // ... then blocks [nbw + nbo, + ceil(n_clr / 256)) clear the entries the
    int n_clr;          // committed tick's results completed: log_slot[ev_clr[e]] = -1, e < n_clr
    const int32_t *ev_clr;
    uint32_t tick;
    const uint8_t *st;
    const uint32_t *touched;
    const PostRec *post;
    const uint32_t *tbits;     // one GPU heartbeat loop: slots that got messages (valid when E > 0)
    int E;                     // messages of the committed tick (0: no slot was touched)
    uint8_t *reg;
    double *hb;
    uint32_t *epoch;
    int64_t n_orph;            // orphans of the committed tick (this rank's, sharded)
    const int64_t *orphans;    // their sequence numbers (global, sharded)
    int32_t *log_slot;
    const uint32_t *lseq;      // sharded: global sequence of each local entry (ascending)
    int64_t head_local;        // sharded: local entries
    int shard;
    // window ticks: the committed window keeps [wq_head, wq_tail) of the queue
    // buffer; per slot that was queued at tick start (st & kStQ0) and sits there, its
    // position is tombstoned when the slot died or its messages took it out of the queue,
    // refreshed with the post-message free count / heartbeat when they kept it; the nbap
    // blocks walking [wq_tail, wq_tail + napp) give every appended slot its position, the
    // blocks after them tombstone the positions in k_emit_win's tomb list (n_tomb entries)
    int win;
    int64_t wq_head, wq_tail, napp;
    int nbap;                  // blocks over the appended positions, then over the tomb list
    int32_t *wq_buf, *wqf;
    double *wqh;
    int32_t *pos;
    const int32_t *tomb;       // committed positions of queued slots moved to the front / back
    int n_tomb;                // entries of tomb (-1: nothing to tombstone)
    const uint8_t *post_rf;
    // non-null: an eager commit (enqueued behind its window tick before the host waited):
    // it commits only if the tick finished as a window tick, with wq_head / napp from these
    // results; nbap blocks walk the appended positions grid-stride
    const int64_t *eager;      // the tick's commit word (TickArgs::cw)
    int64_t cw_tag;            // its launch's link stamp: cw[0] == cw_tag means the tick failed
};

struct EvArgs {
    int E;
    int deque;          // 1: PushDispatcher.start semantics (no liveness, deque with repeated ids)
    const int32_t *tokcnt_in;          // deque: committed tokens per slot
    // one-GPU heartbeat contexts: the log is read-only during a tick (so a relaunch of the
    // tick sees the same log); a result that completes entry q records q in ev_clr[e] (the
    // commit clears it) and stamps ctag[q] = lstamp.  bud[s] = in-flight entries + free
    // processes of a registered slot (committed): a dispatch moves one unit from free to
    // in flight, so only messages and deaths change it.  post_infl[s] = the slot's in-flight
    // entries after its messages (bud - free minus the distinct entries its results
    // completed); the purge of a touched slot writes its next budget into bud_next[s],
    // which the commit installs
    int defer_clr;
    int32_t *ev_clr;
    uint32_t *ctag;
    uint32_t lstamp;
    const int32_t *bud;
    uint32_t *post_infl;
    int32_t *bud_next;
    int orph_grp;         // the slot purge adds the orphans of dead registrations to column R + 1
    int live_chk;         // lazy clears: a result completes entry q only if it is live (reg at tick start, q >= epoch)
    int32_t *front_rank, *back_rank;   // deque: rank of a new token among its slot's tokens
    int32_t *post_tok, *post_nf;       // deque: tokens per slot after the messages; new front tokens
    int shard;          // 0: one GPU; else this rank owns global slots [slot_base, slot_base + W)
    int slot_base, W;
    int64_t head_local; // sharded: local log length (entries carry their global seq in lseq)
    const uint32_t *lseq;
    uint32_t tick;
    double tte;
    int64_t head_in;
    const uint32_t *skeys, *svals;
    uint8_t *ev_kind;           // (k_ev_link may neutralise an invalid message of a pinned batch)
    const int32_t *ev_val;
    const double *ev_ts;
    const int64_t *ev_seq;
    uint8_t *ev_status;
    const uint8_t *reg;
    const int2 *free_in;  // {free_processes, queued} per slot
    const double *hb;
    const uint32_t *epoch;
    int32_t *log_slot;
    PostRec *post;
    uint8_t *post_rf;
    uint32_t *touched;  // tick stamp of a slot that got messages (written only without tbits)
    uint32_t *tbits;   // one GPU: bit s = slot s got a message this tick (cleared by the first sort pass)
    int32_t *front_list, *back_list;  // slot + 1 (0 = empty), zeroed before the tick
    // linked-list grouping (k_ev_link / k_ev_apply_ll; one GPU, heartbeat loop)
    int32_t *ev_slot;
    unsigned long long *ev_head;  // per slot: {link stamp, last linked message}
    int32_t *ev_next;             // per message: the message it displaced, -1 = first of its slot
    uint32_t link;                // this launch's stamp (never 0)
    int tbits_words;
    HostOut *hout;                // resort: a slot had more than kLinkMax messages
    // the previous tick's deferred commit, run by k_ev_link's blocks past the link grid
    int cm_blocks;
    CommitArgs cm;
    // the slot purge (k_scan's W role) in k_ev_apply_ll's launch: nbw tiles of 256 slots,
    // wtiles per workgroup, past the apply grid purge the untouched slots, each owner
    // thread its touched slot
    int nbw;
    int wtiles;
    double now;
    uint8_t *st;
    int2 *free_out;
    unsigned long long *dmask;  // died bitmap (null: not needed), zeroed by k_ev_link, atomicOr
    uint32_t *died_tag;         // window ticks: set to lstamp when a registration dies (null: not needed)
    uint32_t *wcnt;             // evictions per 256-slot tile, zeroed by k_ev_link, atomicAdd
    uint32_t *grp;              // group rows (null: none); evictions into column R + 2
    int ngrp, gstride, R;
    // window ticks: evictions and live queued slots as 64 partials (128-byte lines, word 0 /
    // word 1 of each), zeroed by k_ev_link; k_emit_win sums them
    uint32_t *wpart;
    int check_ev;               // k_ev_link checks the messages (host-unchecked pinned batches)
    int32_t *bad_min;           // k_ev_link: the first invalid message's index (atomicMin; reset by the host)
    unsigned long long *wlb;    // k_emit_win's look-back granules (wlb_n of them) and ticket,
    int wlb_n;                  // zeroed here
    uint32_t *wticket;
    int64_t *cw;                // commit word {failed: link stamp, window head, window length} (null: none)
    unsigned long long *dbg;    // diagnostic stamps (FAASBAL_STAMPS builds; null until the first tick allocated them)
};

// one argument block for k_scan / k_plan / k_emit
struct TickArgs {
    int W, E, R, nbw, nbf, nbq;
    int fused;       // 1: k_emit derives the cross-block prefixes itself (no k_plan launch)
    int segw;        // 1: k_scan stores per-64-position segment counts (k_emit2, fused or after k_plan)
    int lds_bitmap;  // 1: F-blocks stage the died-registration bitmap in LDS
    int slots_in_scan;
    int deque;        // 1: PushDispatcher.start semantics (see EvArgs)
    int redist;       // 1: orphans are dispatched first (a tick); 0: reported only (fb_purge_launch)
    int64_t q_cap;    // deque: token capacity of queue_out
    const int32_t *tokcnt_in, *xw_in, *kl_in;  // deque: committed per-slot token count, x_w, K_L
    const uint32_t *qrank_in;                  // deque: committed token rank (+ kPart2) per position
    const int32_t *front_rank, *back_rank, *post_tok, *post_nf;
    int4 *c_tok;                               // deque: {rank j, m, q, k} per position (k_scan -> emit)
    int32_t *tokcnt_out, *xw_out, *kl_out;
    uint32_t *qrank_out;
    // fused path: every k_scan queue block adds its round counts into its group's
    // row (2^gshift blocks per group; row = R counts, then max c), k_emit2 reads the
    // ngrp group rows plus its group's earlier block rows instead of the whole table
    int grp_on, gshift, gstride, ngrp;
    uint32_t *grp;       // this launch's rows (zero before k_scan)
    uint32_t *grp_zero;  // the other parity's rows: k_emit2 zeroes zero_words of them for the next launch
    int zero_words;
    int f_sep;        // 1: log role in its own launch (k_logscan, died bitmap in LDS); k_scan W-role writes the bitmap
    // one-GPU heartbeat contexts: bud / post_infl / bud_next / ctag / lstamp as in EvArgs
    const int32_t *bud;
    int32_t *bud_next;
    const uint32_t *post_infl;
    const uint32_t *ctag;
    uint32_t lstamp;
    // f_emit (fused one-GPU ticks): the orphan count comes from the slot purge (sum of the
    // dead registrations' in-flight counts into column R + 1), k_scan has no log blocks, and
    // k_emit2's log workgroups flag the orphans against the died bitmap in LDS and write
    // them into per-tile segments (orphans[t*2048 + i], i < fcnt[t])
    int f_emit;
    // free_pre (one-GPU ticks on k_emit2 whose slot purge runs in k_scan): the purge writes
    // a queued slot's next free count as if the tick served it c times ({free - c, 0}, what
    // every position with c <= L gets) and k_emit2 rewrites only the positions with c > L --
    // dense stores instead of one scattered 8-byte store per served worker
    int free_pre;
    uint32_t tick;
    double now, tte;
    int64_t Qn, Qlog, head_in, T, log_cap;
    // committed state
    const uint8_t *reg;
    const double *hb;
    const int2 *free_in;  // {free_processes, queued} per slot: one 8-byte record per worker
    const int32_t *queue_in;
    // free_processes / last_heartbeat of the committed queue, by LRU position
    // (written by the previous tick's emit; valid when qaos = 1)
    int qaos;
    const int32_t *qfree_in;
    const double *qhb_in;
    // this tick's message results
    const uint32_t *touched;
    const uint32_t *tbits;  // one GPU, message ticks: touched as a bitmap (L2-resident: 128 KB per 1M slots)
    const PostRec *post;
    const uint8_t *post_rf;
    int slots_in_apply;  // the slot purge ran in k_ev_apply_ll's launch: k_scan has no W blocks
    int cq_direct;  // idle one-GPU tick on k_emit2: the emit recomputes each position's raw free count
                    // and heartbeat from the committed per-position arrays; k_scan stores neither
    int post_lazy;  // 1: the slot purge loads post records only for touched slots (large tables)
    const int32_t *front_list, *back_list;  // slot + 1, 0 = empty
    // intermediates
    uint8_t *st;
    unsigned long long *dmask;  // bit s: the registration alive at tick start died this tick
    int32_t *c_arr;  // raw free_processes of a live LRU position, INT32_MIN otherwise
    uint8_t *ofl;    // orphan flags, one byte per F-thread (8 log entries)
    uint32_t *wcnt, *fcnt, *qcnt;
    uint32_t *segcnt;  // [64-position segment][round] counts of c > r (fused path)
    int32_t *qbmax, *qbm_raw;
    unsigned long long *csum;
    int64_t *fpre, *wpre, *qpre, *A;
    DevTotals *P;
    // k_plan2 path: every group's workgroup writes its own copy of A and the totals, and
    // a k_emit2 queue block reads its group's copy (no line read by every block of the grid)
    int repl;
    int64_t *A_rep;     // [64][128]
    DevTotals *P_rep;   // [64]
    // outputs
    int32_t *log_slot;
    // ---- window ticks (one GPU, heartbeat loop, level 0).  The committed queue
    // is the window [wq_off, wq_tail) of a buffer of wq_cap entries (qfree kTomb: a position
    // whose slot left); k_emit_win takes 1024-element chunks of [backs][fronts][window
    // prefix], serves the first N live elements (fronts, then the window), appends the live
    // backs and then the served workers with c > 1 at the tail
    int win;
    int64_t wq_off, wq_tail, wq_cap;
    int32_t *wq_buf, *wqf_buf;
    double *wqh_buf;
    int nchB, nchF, nchW;
    int win_direct;  // k_emit_win: chunk = workgroup index (every chunk resident at once), else a ticket
    int xself;       // xplan ticks with <= 64 chunks: k_emit_shard_xp prefixes the chunk totals itself
    int wfirst;      // k_scan: log and slot blocks ahead of the queue blocks in the grid (sharded phase 1)
    unsigned long long *wlb;     // look-back granules: [0, nchB) the back chain, then the front / window chain
    uint32_t *wticket;           // chunk tickets (zeroed by k_ev_link)
    int64_t *cw;                 // commit word {failed, window head, window length} (eager commits)
    int64_t cw_tag;              // failures store this launch's link stamp into cw[0]
    uint32_t *lpart;             // k_logscan: orphans per log workgroup
    uint32_t *died_tag;          // window ticks: == lstamp iff the apply's purge saw a registration die
    int n_lpart;
    uint32_t *wpart;             // evictions / live queued slots, 64 partials (EvArgs::wpart)
    const int32_t *pos_in;       // committed position of each queued slot
    int32_t *tomb;               // per back / front list entry: the committed position of a queued slot
                                 // it moved (-1: none), 2 E entries
    int wseg;                    // k_logscan writes per-tile orphan segments (window ticks)
    int64_t fault_qlen;          // >= 0: k_emit_win reports this window / queue length (a test's fault)

    // the previous tick's commit folded into this k_scan (one-GPU heartbeat contexts, an
    // idle tick after an idle tick): the W role deletes the records that tick evicted
    // (st & kStEvicted, read before it writes this tick's st) and the last cm_blocks
    // blocks clear its orphaned log entries -- per-tile segments (cm_tiles tiles of
    // orphans / fcnt) or a dense list of cm_n_orph -- before this tick's log role runs
    int cm_fold, cm_blocks, cm_tiles;
    int64_t cm_n_orph;

    int32_t *trash;     // kTrashRows x kBS words: k_emit2's round stores of inactive lanes land here
    int32_t *rb_slot;   // compact assignments (null: off): slot per LRU position, -1 none
    uint8_t *rb_c;      // ... and min(c, L + 1) (clamped to 255)
    char *arena;        // base of the context's arena (every buffer above)
    int arena32;        // 1: the arena spans < 4 GB (32-bit byte offsets from arena)
    int2 *free_out;     // next {free_processes (INT32_MIN: no live record), queued}
    int32_t *queue_out;
    int32_t *qfree_out;
    double *qhb_out;
    double *c_hb;    // last_heartbeat of a live LRU position (k_scan -> emit)
    int64_t *orphans;
    int32_t *evicted;
    HostOut *hout;
    unsigned long long *dbg;  // diagnostic stamps (FAASBAL_STAMPS builds only)
    // sharding: 0 one GPU; 1 phase 1 (own slots -> exchange); 2 phase 2 (after the
    // exchange all-reduce).  W above is then the local slot count; queue entries are global ids.
    int shard;
    int slot_base, rank, world;
    int64_t head_local;            // local log entries; lseq[i] = global sequence of entry i (ascending)
    const uint32_t *lseq;
    uint32_t *lseq_out;
    uint8_t *xc8;                  // exchange: c per LRU position (single contributor per byte), xcw bytes each:
    int xcw;                       // 1: min(c, 255) while the round table has <= 128 rows, 2: min(c, 65535)
    unsigned long long *xrec;      // exchange: per rank kXRecLines orphan-count partials, one per 128-B line
                                   // (two copies by launch parity: phase 2 zeroes the next tick's)
    uint8_t *xrows;                // exchanged block rows (kXRowsMaxBlocks; null: phase 2 re-counts the c values)
    uint8_t *xgrows;               // exchanged group rows (R = kXGroupR; null: phase 2 sums the block rows)
    int xplan;                     // large queues (> kXRowsMaxBlocks blocks, R = kXGroupR): phase 2 is k_xscan's
                                   // prefix scans of the exchanged digit rows / own rows, then k_emit_shard
    uint32_t *xpre;                // k_xscan: [block][2R] exclusive prefixes inside the block's chunk
                                   // (rounds of all positions, then this rank's)
    uint32_t *xct;                 // [chunk][2R] chunk totals, turned into exclusive prefixes over the chunks
    uint32_t *xA;                  // [2R] totals A(r) (all, then this rank's)
    uint32_t *xtk;                 // k_xscan's ticket (zero between launches)
    // one-GPU large tables with k_logscan (gp): no k_plan2 -- k_emit2's queue blocks reduce the
    // group rows themselves and its compaction workgroups sum the tile counts before theirs
    // (as the fused path does)
    int gp;
    int gpcheck;  // (stamps builds: k_plan2 runs too, k_emit2 records both prefixes)
    int cmix;     // k_emit2: compaction workgroups interleaved with the queue blocks
    int wtiles;   // k_scan: slot tiles per W-role workgroup (1, 2 or 4)
    int qtiles;   // k_scan (one GPU, unfused, 4-tile instance): queue blocks per Q-role workgroup (1 or 4)
    // lazy clears (one-GPU heartbeat contexts): entries of dead registrations may remain in
    // the log; an orphan flag needs q >= epoch[s] (the committed epoch of its died slot)
    int live_chk;
    const uint32_t *epoch;
    int xcfirst;  // k_emit_shard_xp: the compaction workgroups first in the grid
    // sharded phase 2 (fb_set_full_assign): this rank also writes the whole tick's task -> slot
    // array (every rank computes the global water-filling; one rank's copy serves the host)
    int32_t *assign_all;
    uint32_t *xg_acc, *xg_tk;      // phase 1: per group the running sums and the ticket (zero between ticks)
    uint32_t *ogrp;                // phase 1 -> 2: this rank's group rows [group][R]
    unsigned long long *xz;        // phase 2: the other launch parity's exchange records, zeroed for the next tick
    int xz_words;
    uint32_t *ocnt;                // [block][round] counts of this rank's positions
    uint32_t *osegcnt;             // [64-position segment][round] counts of this rank's positions
    int64_t *opre, *oA;
};


// Host-side launchers (defined in faasbal_kernels.hip; grid sizes are the caller's).
// A launch target: the stream, plus optional dispatch-packet timing events
// (hipExtLaunchKernel records them at the kernel's own start and end, the
// interval rocprofv3's kernel trace reports).
struct Stream {
    hipStream_t s;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    Stream(hipStream_t s_) : s(s_) {}
    Stream(hipStream_t s_, hipEvent_t a, hipEvent_t b) : s(s_), e0(a), e1(b) {}
};
// One LSD pass (histogram + scatter launches) over `db`-bit digits at `shift`;
// hist holds (1 << db rounded up to 256 / 1024 / 2048) x (nblk + 1) counts (the
// extra row: digit totals when nblk > kRsScanMin).
// The first pass's histogram launch clears zero0 / zero1 (n words each) and zbits (zwords).
struct RsPass {
    const uint32_t *kin, *vin;
    uint32_t *kout, *vout;
    int n, shift, db, nblk;
    uint32_t *hist;   // this pass's [tile][digit] counts (its histogram launch)
    int identity_vals;
    int32_t *zero0, *zero1;
    uint32_t *zbits;
    int zwords;
};
void launch_rs_pass(const RsPass &p, Stream h, Stream s);
#ifndef FAASBAL_RS_SCAN_MIN
#define FAASBAL_RS_SCAN_MIN 64
#endif
// batches of more tiles than this get a column-prefix launch (k_rs_scan) before the
// scatter instead of every scatter block walking the [tile][digit] table
constexpr int kRsScanMin = FAASBAL_RS_SCAN_MIN;
// wider digits (2 passes for 1 M workers) up to this many tiles: the table is 2048 x tiles words
constexpr int kRsWideMaxBlocks = 4096;
void launch_ev_apply(const EvArgs &a, Stream st);
void launch_ev_link(const EvArgs &a, Stream st);
void launch_ev_apply_ll(const EvArgs &a, Stream st);
void launch_selftest(uint32_t *err, uint32_t seed, Stream st);
// a one-lane kernel that holds the stream until flag[0] == want (host-mapped word) or
// `limit` ticks of the 100 MHz realtime counter pass (then flag[1] = 1)
void launch_gate(uint32_t *flag, uint32_t want, uint64_t limit, Stream st);
void launch_log_normalize(int32_t *log, int64_t n, const uint8_t *reg, const uint32_t *epoch, Stream st);
void launch_slots(const TickArgs &a, Stream st);
void launch_scan(const TickArgs &a, Stream st);
void launch_logscan(const TickArgs &a, int grid, Stream st);
void launch_plan(const TickArgs &a, Stream st);
void launch_xscan(const TickArgs &a, Stream st);
void launch_emit(const TickArgs &a, Stream st);
void launch_emit2(const TickArgs &a, Stream st);
void launch_emit_shard(const TickArgs &a, Stream st);
void launch_emit_win(const TickArgs &a, int grid, Stream st);
// k_emit_win workgroups resident per CU at once (the occupancy calculator; 0 on failure)
int emit_win_resident_per_cu();
void launch_pos_rebuild(int32_t *pos, const int32_t *queue, const int32_t *qfree, int64_t off, int64_t n, Stream st);
// evicted slots in ascending order from the per-slot status bytes and per-tile counts (two
// launches: a one-workgroup scan of the tile counts, then one block per tile)
void launch_evict_gather(int32_t *dst, const uint8_t *st, const uint32_t *wcnt, int64_t *wpre, int W, Stream s);
void launch_commit(const CommitArgs &a, int grid, Stream st);
// dst[i] = src[i], i < n (dst may be host memory mapped for the device: stores cross PCIe)
void launch_copy_words(uint32_t *dst, const uint32_t *src, int64_t n, Stream st);
// up to 4 word copies in one launch; copy i uses blocks [blk0[i], blk0[i + 1]) (the last:
// up to the grid's end), the caller sizes blk0
struct CopyMulti {
    uint32_t *dst[4];
    const uint32_t *src[4];
    int64_t words[4];
    int blk0[4];
    int n;
    // optional: the orphans' per-tile segments gathered into odst, one block per tile after
    // the copies' blocks (k_orph_gather's work in the same launch)
    int64_t *odst;
    const int64_t *osrc;
    const uint32_t *ocnt;
    int otiles;
};
void launch_copy_multi(const CopyMulti &m, Stream st);
// the dense orphan list from per-tile segments (dst may be host-mapped memory): the
// segments concatenated in tile order (each is ascending already, so the list is)
void launch_orph_gather(int64_t *dst, const int64_t *src, const uint32_t *cnt, int ntile, Stream st);

}  // namespace fb
