/*
 * faasbal.h -- C ABI of the MI355X push balancer (libfaasbal.so).
 *
 * Drop-in boundary for the heartbeat push dispatcher of Distributed-FaaS.
 * The reference has no FFI; its seam is the method level of PushDispatcher
 * (reference task_dispatcher.py).  Each entry point below names the reference
 * code it replaces.  Plain pointers and sizes only; no torch types.
 *
 * One tick = inbound events -> heartbeat purge -> orphan redistribution ->
 * LRU water-filling dispatch.  All calls for one context must
 * come from one thread (the reference loop is single-threaded).  Errors are
 * negative return codes; fb_last_error() gives the message.  No exception
 * crosses the ABI.
 */
#ifndef FAASBAL_H
#define FAASBAL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FB_OK 0
#define FB_EINVAL (-1)  /* bad argument or inconsistent state                 */
#define FB_ENOMEM (-2)  /* device or host allocation failed                  */
#define FB_EHIP (-3)    /* HIP runtime error                                  */
#define FB_ERANGE (-4)  /* free counts beyond the supported round range       */
#define FB_ENOSPC (-5)  /* in-flight log full                                 */
#define FB_ESTATE (-6)  /* call out of order (e.g. wait without launch)       */
#define FB_ERERUN (-7)  /* sharded: the fill level reached the round table; launch the
                         * same tick again (a wider table), exchange, continue, wait */

/* Inbound message kinds (task_dispatcher.py:347-387). */
#define FB_EV_REGISTER 0   /* {"type":"register","data":{"num_processes":n}}   */
#define FB_EV_RECONNECT 1  /* {"type":"reconnect","data":{"free_processes":n}} */
#define FB_EV_HEARTBEAT 2  /* {"type":"heartbeat"}                              */
#define FB_EV_RESULT 3     /* {"type":"result", ...}; seq = task's log sequence */
#define FB_EV_OTHER 4      /* any other type: ignored for known workers         */

/* Per-event status written by a tick. */
#define FB_EVS_APPLIED 0
#define FB_EVS_RECONNECT 1 /* sender unknown: reply {"type":"reconnect"}, payload dropped (:356-358) */
#define FB_EVS_UNKNOWN 2   /* deque context: result from an id without a record -- the reference
                            * raises KeyError (:291) and its loop dies; here the message is dropped */

typedef struct fb_ctx fb_ctx;

typedef struct fb_tick_result {
    int64_t n_assigned;  /* tasks dispatched this tick: orphans first, then pending       */
    int64_t n_orphans;   /* in-flight tasks of dead registrations, redistributed first    */
    int64_t queue_len;   /* LRU queue (free_workers) length after the tick                */
    int64_t log_head;    /* log length after the tick: task k got sequence log_head_in+k  */
    int32_t n_evicted;   /* worker records deleted by the tick (purge_workers, :241-249)  */
    int32_t fill_level;  /* water-filling rounds completed (L)                            */
    int32_t max_free;    /* largest effective free count in the queue this tick           */
    int32_t reruns;      /* internal reruns with a wider round table                      */
    int64_t n_local;         /* sharded: tasks dispatched to this rank's workers (else n_assigned) */
    int64_t n_orphans_local; /* sharded: orphans from this rank's log shard (else n_orphans)       */
} fb_tick_result;

/* Device pointers of the context's state (for zero-copy consumers, e.g.
 * torch tensors built from data_ptr).  Valid until the next fb_tick_commit;
 * after a commit, call fb_sync (or fetch the view again) before reading through
 * it, so that the deferred part of the commit has run. */
typedef struct fb_device_view {
    int32_t *free_processes; /* [n_workers]  PushWorker.free_processes (:205), every
                              * free_processes_stride bytes                    */
    double *last_heartbeat;  /* [n_workers]  PushWorker.last_heartbeat (:206), every
                              * last_heartbeat_stride bytes; NaN for empty slots */
    uint8_t *registered;     /* [n_workers]  slot present in self.workers      */
    int32_t *queue;          /* [queue_len]  free_workers in LRU order (:327)  */
    int32_t *log_slot;       /* [log_head]   worker slot per task sequence     */
    int64_t *orphans;        /* last tick's redistributed sequence numbers     */
    int32_t *evicted;        /* last tick's evicted slots                      */
    int32_t n_workers;
    int64_t queue_len, log_head;
    int32_t last_heartbeat_stride; /* bytes between consecutive slots' heartbeats */
    int32_t free_processes_stride; /* bytes between consecutive slots' free counts */
} fb_device_view;

/* Context: owns every device buffer.  device = HIP device ordinal. */
int fb_create(fb_ctx **out, int32_t max_workers, int64_t max_log, int32_t max_events, int device);
int fb_destroy(fb_ctx *ctx);
const char *fb_last_error(const fb_ctx *ctx);

/* Install a worker-table state (replaces building self.workers and the
 * free_workers OrderedDict by hand, task_dispatcher.py:194, :327).
 * queue: slots in LRU order (front first), each registered, no duplicates.
 * log_slot: worker slot per in-flight task sequence number (-1 = completed). */
int fb_load_state(fb_ctx *ctx, int32_t n_workers, const uint8_t *registered,
                  const int32_t *free_processes, const double *last_heartbeat,
                  const uint32_t *epoch, const int32_t *queue, int64_t queue_len,
                  const int32_t *log_slot, int64_t log_len);

/* Read the committed state back (any pointer may be NULL). */
int fb_read_state(fb_ctx *ctx, uint8_t *registered, int32_t *free_processes,
                  double *last_heartbeat, uint32_t *epoch, int32_t *queue, int64_t *queue_len,
                  int32_t *log_slot, int64_t *log_len);

/* One-GPU heartbeat contexts: in-flight log entries per slot of the committed state
 * (n_workers words; build-defined bookkeeping of the redistribution, DESIGN.md §3:
 * the count of the slot's entries that are neither completed nor redistributed). */
int fb_read_inflight(fb_ctx *ctx, uint32_t *inflight);

/* Enqueue one tick on the context's stream (no host sync).
 * Replaces, per tick: the inbound branches (task_dispatcher.py:343-387), the
 * purge (:241-249, called at :390) and the dispatch block (:393-419), plus the
 * build-defined redistribution.  Events are host arrays in arrival order with
 * non-decreasing ts <= now; seq is the log sequence of a result's task or -1.
 * n_pending = tasks waiting in pub/sub (carried-over ones first).
 * Reads the committed state, writes the tick's outputs and the next state into
 * separate buffers: launching again without fb_tick_commit recomputes the same
 * tick (used by the benchmark). */
int fb_tick_launch(fb_ctx *ctx, double now, double tte, int32_t n_events, const uint8_t *kind,
                   const int32_t *slot, const int32_t *val, const double *ts, const int64_t *seq,
                   int64_t n_pending);

/* The same launch in two steps, so that a host can stage tick t+1's events
 * while the device runs tick t (double-buffered pinned staging):
 * fb_tick_stage validates and copies the events (same rules and errors as
 * fb_tick_launch; no device work), fb_tick_launch_staged enqueues the tick on
 * the staged events with the stage's `now`.  fb_tick_launch = stage + launch.
 * Events already in pinned memory (fb_host_alloc) are copied as they are and, on
 * one-GPU heartbeat contexts, checked by the tick's first kernel instead of the
 * host: an invalid message (slot, kind, timestamp) then fails fb_tick_wait with
 * FB_EINVAL naming it, and nothing is committed.  Arrays in this GPU's memory (all of
 * them; seq may be NULL) are not copied at all: the tick reads them in place and its
 * first kernel checks them the same way (overwriting an invalid message with a harmless
 * one); arrays mixing device and host memory are refused.  Pinned arrays must stay
 * unchanged until their tick was waited for, device arrays until it was committed (a
 * window tick's commit reads the slots of its messages). */
int fb_tick_stage(fb_ctx *ctx, double now, int32_t n_events, const uint8_t *kind, const int32_t *slot,
                  const int32_t *val, const double *ts, const int64_t *seq);
int fb_tick_launch_staged(fb_ctx *ctx, double tte, int64_t n_pending);

/* purge_workers (task_dispatcher.py:241-249, called at :390) on its own: a tick at
 * `now` with no messages and no pending tasks.  Records whose heartbeat expired
 * are deleted (fb_get_evicted) and the in-flight tasks of the dead registrations
 * are reported (fb_get_orphans) but NOT dispatched: the caller keeps them pending
 * (the reference drops them, README.md:263-264).  Then fb_tick_wait / outputs /
 * fb_tick_commit as for any tick (sharded contexts: the exchange all-reduce and
 * fb_tick_continue in between, as for a tick). */
int fb_purge_launch(fb_ctx *ctx, double now, double tte);

/* Wait for the last launched tick; fills *res.  Transparently reruns the tick
 * with a wider round table when free counts exceeded the launch's estimate. */
int fb_tick_wait(fb_ctx *ctx, fb_tick_result *res);

/* Make the waited tick's post-state the committed state.  On a one-GPU
 * heartbeat context the device part (registered / last_heartbeat / epoch of the
 * slots the tick touched or evicted, orphaned log entries) is deferred: the
 * next launch's first kernel runs it, and any call that reads or replaces
 * state first (fb_read_state, fb_load_state, fb_device_view_get, fb_sync, ...)
 * enqueues it on its own.  Observably the same as an immediate commit. */
int fb_tick_commit(fb_ctx *ctx);

/* Copy outputs of the waited tick to host memory. */
int fb_get_assignments(fb_ctx *ctx, int64_t first, int64_t n, int32_t *dst); /* slot per task k */
int fb_get_orphans(fb_ctx *ctx, int64_t n, int64_t *dst);   /* old sequence numbers, ascending */
int fb_get_evicted(fb_ctx *ctx, int32_t n, int32_t *dst);   /* slots, ascending                */
int fb_get_event_status(fb_ctx *ctx, int32_t n, uint8_t *dst); /* FB_EVS_* per event          */

/* All three of the waited tick's lists (each may be NULL; sizes res->n_assigned,
 * n_orphans, n_evicted) with one synchronisation: into pinned memory, three DMA
 * transfers back to back. */
int fb_get_outputs(fb_ctx *ctx, int32_t *assign, int64_t *orphans, int32_t *evicted);

/* Compact assignments (one-GPU contexts).  After fb_set_compact(ctx, 1) every tick
 * also writes, per position of its LRU order (fronts ++ queue ++ backs, n_pos of them),
 * the slot and min(c, L + 1) of the worker there (c = effective free count, 0 = no live
 * queued worker): with the fill level L this determines every assignment of the tick
 * (task k of round r <= L goes to the (k - S(r))-th position with c > r), in 5 bytes per
 * position instead of 4 per task (configs[2]: 0.3 MB instead of 4.1 MB to read back).
 * fb_get_outputs_compact copies that form plus the orphans and evicted slots with one
 * synchronisation (cap = entries of slot / c; *n_pos = positions written; FB_ERANGE
 * when L + 1 > 255); fb_expand_compact turns it into fb_get_assignments' array on the
 * host (result->n_assigned slots). */
int fb_set_compact(fb_ctx *ctx, int enable);

/* Window ticks (one-GPU heartbeat contexts).  A tick at fill level 0
 * (fewer tasks than live queued workers, the streaming case) serves a prefix of the LRU
 * queue; as a window tick it leaves the rest of the queue where it is and appends the
 * re-queued workers at its tail, so its work is O(tasks + messages) instead of O(queue).
 * Results are identical either way (the closed form of task_dispatcher.py:393-419);
 * a tick that turns out not to qualify is rerun on the general path.  mode: -1 auto
 * (the default: contexts of more than 128K workers, after a level-0 tick), 0 off, 1
 * whenever the last tick was not above level 0 (allocates the window buffers on contexts
 * created without them).  Between ticks only. */
int fb_set_window(fb_ctx *ctx, int mode);
/* Committed window ticks, and launches that fell back to the general path. */
int fb_window_stats(fb_ctx *ctx, int64_t *window_ticks, int64_t *fallbacks);
/* Eager commits (a streaming loop that commits every tick it waits for): a window tick's
 * commit is enqueued right behind it at launch and commits on the device as soon as the
 * tick finishes -- if the tick finished as a window tick; otherwise it commits nothing and
 * fb_tick_wait reruns the tick on the general path as usual.  The host still calls
 * fb_tick_wait and fb_tick_commit (which then only does the host's bookkeeping) before the
 * next launch; a tick so launched cannot be relaunched uncommitted, and state reads
 * between its wait and commit see the committed state.  Default off.  Between ticks only. */
int fb_set_eager_commit(fb_ctx *ctx, int enable);
int fb_get_outputs_compact(fb_ctx *ctx, int32_t *slot, uint8_t *c, int64_t cap, int64_t *n_pos, int64_t *orphans,
                           int32_t *evicted);
int fb_expand_compact(fb_ctx *ctx, const int32_t *slot, const uint8_t *c, int64_t n_pos, int32_t *assign);
/* Pinned buffers (fb_host_alloc) that ticks write their compact outputs into while they
 * run: slot / c per position (cap entries), orphans (ocap), evicted slots (ecap); turns
 * compact mode on.  A fused tick (the configs[2] shape) whose outputs fit leaves them
 * there by the time fb_tick_wait returns, and fb_get_outputs_compact into the same
 * buffers copies nothing; other ticks fill them through fb_get_outputs_compact as
 * usual.  The buffers must not be touched between a launch and its wait.  slot = NULL
 * unregisters. */
int fb_set_compact_out(fb_ctx *ctx, int32_t *slot, uint8_t *c, int64_t cap, int64_t *orphans, int64_t ocap,
                       int32_t *evicted, int64_t ecap);

/* Pinned host memory: fb_get_* copies into it are single DMA transfers on the
 * context stream (the drop-in's readback of a tick's assignments). */
int fb_host_alloc(fb_ctx *ctx, int64_t bytes, void **ptr);
int fb_host_free(fb_ctx *ctx, void *ptr); /* ctx may be NULL (the memory outlives contexts) */

/* launch + wait + copies + commit.  Output arrays may be NULL. */
int fb_tick(fb_ctx *ctx, double now, double tte, int32_t n_events, const uint8_t *kind,
            const int32_t *slot, const int32_t *val, const double *ts, const int64_t *seq,
            int64_t n_pending, fb_tick_result *res, uint8_t *ev_status, int32_t *assign,
            int64_t *orphans, int32_t *evicted);

/* Per-operation forms (one-GPU contexts; each is one synchronous tick and commits).
 *
 * fb_apply_events: the inbound branches (task_dispatcher.py:343-387) for n messages
 *   in arrival order, each after the purge at its own clock (:390), then the purge
 *   after the last message at ts[n-1]; nothing is dispatched.  Records that expired
 *   are evicted (evicted), their in-flight tasks reported (orphans) for the caller to
 *   keep pending; ev_status as fb_get_event_status.
 * fb_purge: purge_workers at `now` (:241-249) = fb_purge_launch + wait + outputs + commit.
 * fb_assign: the dispatch block (:393-419) for n_tasks pending tasks after the purge at
 *   `now` (:390); orphans of that purge first (build-defined), then the tasks; assign
 *   gets res->n_assigned slots (fewer than requested when capacity runs out: the rest
 *   stay pending, as at :393).
 * Output arrays may be NULL; sizes as fb_get_* (res->n_*). */
int fb_apply_events(fb_ctx *ctx, double tte, int32_t n_events, const uint8_t *kind, const int32_t *slot,
                    const int32_t *val, const double *ts, const int64_t *seq, fb_tick_result *res,
                    uint8_t *ev_status, int64_t *orphans, int32_t *evicted);
int fb_purge(fb_ctx *ctx, double now, double tte, fb_tick_result *res, int64_t *orphans, int32_t *evicted);
int fb_assign(fb_ctx *ctx, double now, double tte, int64_t n_tasks, fb_tick_result *res, int32_t *assign,
              int64_t *orphans, int32_t *evicted);

int fb_device_view_get(fb_ctx *ctx, fb_device_view *view);

/* Per-kernel device timing with HIP events on the context stream.
 * enable=1 starts accumulating; fb_timing_read syncs and returns, per kernel
 * name (static strings), total milliseconds and launch counts. */
int fb_timing_enable(fb_ctx *ctx, int enable);
int fb_timing_read(fb_ctx *ctx, int32_t max_kernels, const char **names, double *total_ms,
                   int64_t *launches, int32_t *n_kernels);

/* Timing gate (measurement only): hold=1 enqueues a one-lane kernel that holds the
 * context stream until hold=0 releases it, so the launches queued in between run back
 * to back on the device whatever the host's enqueue pace (the gate opens by itself
 * after 0.5 s).  fb_timing_span syncs and returns the device time from the gate's end
 * to the release point's event, and whether the gate timed out.  Per-kernel times of
 * the gated launches come from fb_timing_read as usual. */
int fb_timing_gate(fb_ctx *ctx, int hold);
int fb_timing_span(fb_ctx *ctx, double *ms, int32_t *timed_out);
/* A marker launch for profiles: the gate kernel, already open (it returns at once), so a
 * kernel trace can cut a benchmark's timed region out of the run. */
int fb_timing_mark(fb_ctx *ctx);

/* Device self-test of the kernels' wave/block scan primitives; *errors = 0 on success. */
int fb_selftest(fb_ctx *ctx, int32_t *errors);

/* Diagnostic: copy up to n words of the in-kernel stamp buffer (written only by
 * builds compiled with -DFAASBAL_STAMPS); *n_total = buffer length in words. */
int fb_debug_read(fb_ctx *ctx, unsigned long long *dst, int64_t n, int64_t *n_total);

/* Test paths: run the launch sequence another table size would take on small
 * (oracle-checkable) inputs.  Results are identical on every path.  name / value:
 *   "plan"        0 auto, 1 the k_plan2 + k_emit2 sequence of large tables, 2 the
 *                 chunked k_emit of round tables wider than 128 rows;
 *   "logscan"     -1 auto, 0 never, 1 the log role as its own k_logscan launch;
 *   "split_slots" -1 auto, 0 never, 1 the slot purge as its own k_slots launch;
 *   "ev_ll"       1 per-slot linked lists (one GPU), 0 the radix sort of messages;
 *   "rs_wide"     1 digits up to 11 bits while a batch has <= 4096 sort tiles, 0 8-bit;
 *   "xplan"       sharded: 1 large queues exchange digit rows scanned by k_xscan, 0 a
 *                 phase-2 k_scan re-counts them;
 *   "gp"          one GPU, large tables: 1 k_emit2 reduces the group rows itself, 0 k_plan2;
 *   "win_direct"  window ticks: 1 k_emit_win chunk = workgroup index when every chunk is
 *                 resident at once, 0 always by ticket;
 *   "fault_qlen"  test hook: the next waited tick reports this queue length (checked and
 *                 refused by fb_tick_wait when it exceeds the buffer; -1 off);
 *   "xself"       sharded xplan: 1 k_emit_shard_xp sums the chunk totals itself (<= 64
 *                 chunks), 0 k_xscan's last workgroup does behind a ticket;
 *   "wfirst"      sharded phase 1: 1 k_scan's log and slot blocks ahead of its queue blocks
 *                 (while the log role is fused into k_scan), 0 queue blocks first;
 *   "cmix"        k_emit2 on unfused ticks: 1 compaction workgroups interleaved with the queue
 *                 blocks, 0 after them;
 *   "wtiles"      slot tiles (256 slots each) per slot-purge workgroup: 0 auto (k_scan: 4 on
 *                 unfused tables, 1 fused; k_ev_apply_ll: 4 from 1024 tiles), or 1, 2, 4
 *                 (k_ev_apply_ll: 2 runs as 1);
 *   "qtiles"      k_scan's queue role on unfused one-GPU tables: 0 auto (four queue blocks
 *                 per workgroup), 1 one;
 *   "xcfirst"     sharded xplan phase 2: 1 k_emit_shard_xp's compaction workgroups first in
 *                 its grid when they are many (default), 0 after the queue workgroups;
 *   "lazy"        one-GPU heartbeat contexts: 1 commits leave the log entries they
 *                 redistributed, every later reader tests liveness (default), 0 commits clear
 *                 them (the entries left so far are cleared first);
 *   "gpcheck"     diagnostic (stamps builds): k_plan2 runs beside a gp tick for comparison.
 * Between ticks only; FB_EINVAL for an unknown name or value. */
int fb_set_path(fb_ctx *ctx, const char *name, int value);

/* Synchronise the context stream (for wall-clock benchmarking). */
int fb_sync(fb_ctx *ctx);

/* Run the context's work on another HIP stream (e.g. the one a collective
 * library uses), or on its own stream again with stream = NULL. */
int fb_set_stream(fb_ctx *ctx, void *stream);

/* One-GPU contexts: slot per task of the waited tick as (task index, slot)
 * pairs, same content as fb_get_assignments.  Sharded contexts: only the tasks
 * given to this rank's workers, in ascending task index. */
int fb_get_local_assignments(fb_ctx *ctx, int64_t first, int64_t n, int64_t *task, int32_t *slot);

/* ---- Dispatcher without heartbeats (PushDispatcher.start, task_dispatcher.py:251-322) ----
 * A deque context runs the start() loop per tick: no liveness, no purge, no
 * orphans (now / tte are unused); the ready queue is a deque that may hold an id
 * several times.  register(n) creates the record and, for n > 0, inserts the id
 * at the left even if it is queued already (:276-281); result adds one free
 * process and appends the id at the right when that makes exactly 1 (:284-295);
 * other kinds are ignored; dispatch pops the left id, decrements its count and
 * re-appends it while the count stays > 0 (:298-322).  Replaces, per tick, the
 * message branches and the dispatch block of many loop iterations.
 * max_tokens = deque capacity (ids counted with repetition); fb_load_state's
 * queue may repeat slots; fb_tick_wait fails with FB_ENOSPC if a tick's deque
 * would outgrow it.  Everything else as for fb_create. */
int fb_create_deque(fb_ctx **out, int32_t max_workers, int64_t max_tokens, int64_t max_log,
                    int32_t max_events, int device);

/* ---- Sharded worker table (one process per GPU) ----
 * Rank r owns the global slots [slot_base, slot_base + n_workers): their
 * records, their in-flight log entries (global sequence numbers ascending) and
 * the dispatch of tasks to them.  The LRU queue order is replicated.  A tick is
 *   fb_tick_launch (every rank gets the same full event batch)
 *   -> all-reduce(SUM, uint8) of the bound exchange buffer over all ranks
 *   -> fb_tick_continue -> fb_tick_wait -> outputs -> fb_tick_commit.
 * The whole-table result equals the one-GPU tick's: the union of the ranks'
 * local assignments is fb_get_assignments; orphans / evicted are per rank
 * (merge for the global lists); event status and queue are global. */
int fb_create_sharded(fb_ctx **out, int32_t max_workers_local, int32_t n_workers_global,
                      int64_t max_log_local, int32_t max_events, int device, int32_t rank, int32_t world);
/* queue: global slots in LRU order; log_slot: global slot per local entry
 * (-1 completed); log_seq: its global sequence number; log_head: global log length. */
int fb_load_shard(fb_ctx *ctx, int32_t slot_base, int32_t n_workers, const uint8_t *registered,
                  const int32_t *free_processes, const double *last_heartbeat, const uint32_t *epoch,
                  const int32_t *queue, int64_t queue_len, const int32_t *log_slot, const uint32_t *log_seq,
                  int64_t log_len, int64_t log_head);
int fb_read_shard_log(fb_ctx *ctx, uint32_t *log_seq, int64_t *log_len, int64_t *log_head);
/* Between ticks: the largest free count any queued worker of the loaded state has (the
 * GLOBAL maximum, the same on every rank), which sizes the next tick's round table.
 * A sharded context cannot take it from its own shard: the exchange layout depends on
 * the table, so every rank must agree.  Without it the first tick after fb_load_shard
 * starts narrow and a wider fill level costs one FB_ERERUN relaunch.  Replaces nothing in
 * the reference (it sizes a buffer, task_dispatcher.py:393-419 has none). */
int fb_set_round_hint(fb_ctx *ctx, int32_t max_free);
/* Sharded, between ticks: on != 0 makes this rank's phase 2 also write the whole tick's
 * task -> slot array (every rank computes the global water-filling anyway), so
 * fb_get_assignments works on it and the host needs no per-task gather from the other
 * ranks (the rank that serves the dispatcher loop turns it on).  Replaces the gather of
 * task_dispatcher.py:409-413's decisions onto the loop's process. */
int fb_set_full_assign(fb_ctx *ctx, int on);
/* Exchange buffer size for a tick of n_events events (n_events < 0: the maximum). */
int fb_exchange_bytes(fb_ctx *ctx, int32_t n_events, int64_t *bytes);
/* Device buffer (same size on every rank) the ranks all-reduce between phases. */
int fb_bind_exchange(fb_ctx *ctx, void *device_buffer, int64_t bytes);
/* Enqueue phase 2 of a sharded tick, after the exchange all-reduce. */
int fb_tick_continue(fb_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* FAASBAL_H */
