/*
 * push_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C, single-threaded, *sequential* restatement of the reference's
 * heartbeat push dispatcher loop, PushDispatcher.start_heartbeat
 * (reference task_dispatcher.py:324-419), with its helpers
 * PushWorker.is_alive (:209-212) and purge_workers (:241-249).
 *
 * It is NOT a model of the GPU design: it keeps the LRU queue as a doubly
 * linked list (the CPython OrderedDict `free_workers`, :327) and runs the loop
 * iteration by iteration -- in the default mode with the O(W) purge on every
 * iteration exactly as written (:390).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library.
 *
 * Parity is pinned: tests/test_oracle_golden.py checks every output of this
 * file against golden vectors captured from the unmodified reference loop
 * (tests/golden/make_golden.py).
 *
 * Tick model: for every inbound event i the
 * reference runs one iteration with nothing inbound at clock ts_i (purge) and
 * one that handles the event at ts_i (handle, purge); then the dispatch phase
 * at clock `now` pops one task per iteration while the queue is non-empty.
 * Redistribution (build-defined): at the first dispatch
 * iteration, log entries of registrations that died during the tick are
 * prepended, in ascending sequence, to the pending tasks; at the end of the tick
 * those entries leave the log (-1), like completed ones.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { EV_REGISTER = 0, EV_RECONNECT = 1, EV_HEARTBEAT = 2, EV_RESULT = 3, EV_OTHER = 4 };

typedef struct oracle {
    int32_t W;
    uint8_t *reg;      /* slot in self.workers (:194)                   */
    int64_t *free_;    /* PushWorker.free_processes (:205), Python int  */
    double *hb;        /* PushWorker.last_heartbeat (:206)              */
    uint32_t *epoch;   /* first log seq owned by the registration       */
    /* free_workers OrderedDict (:327) as a doubly linked list */
    int32_t *qprev, *qnext;
    uint8_t *inq;
    int32_t qhead, qtail;
    int64_t qlen;
    /* in-flight log: slot per task sequence number, -1 = completed */
    int32_t *log;
    int64_t head, cap;
    /* per-tick scratch */
    uint8_t *cur_is_start, *died_start, *seen;
    uint32_t *start_epoch;
    int purge_mode;    /* 0: purge every iteration (as written), 1: skip when unchanged,
                          2: 1 + a min-heap of heartbeats (large tables, per-event clocks) */
    double last_purge_t;
    int64_t events_since_purge;
    /* purge_mode 2: binary min-heap of (last_heartbeat, slot) entries of registered
     * slots; an entry is stale once the slot's hb changed or its record was deleted */
    double *hkey;
    int32_t *hslot;
    int64_t hn, hcap;
} oracle_t;

/* ------------------------------------------------------------ heartbeat heap */
static int heap_push(oracle_t *o, double key, int32_t s) {
    if (o->hn == o->hcap) {
        int64_t cap = o->hcap ? 2 * o->hcap : 1024;
        double *k2 = (double *)realloc(o->hkey, (size_t)cap * sizeof(double));
        if (!k2) return -1;
        o->hkey = k2;
        int32_t *s2 = (int32_t *)realloc(o->hslot, (size_t)cap * sizeof(int32_t));
        if (!s2) return -1;
        o->hslot = s2;
        o->hcap = cap;
    }
    int64_t i = o->hn++;
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (!(key < o->hkey[p])) break;
        o->hkey[i] = o->hkey[p];
        o->hslot[i] = o->hslot[p];
        i = p;
    }
    o->hkey[i] = key;
    o->hslot[i] = s;
    return 0;
}
static void heap_pop(oracle_t *o) {
    double key = o->hkey[--o->hn];
    int32_t s = o->hslot[o->hn];
    int64_t i = 0;
    for (;;) {
        int64_t c = 2 * i + 1;
        if (c >= o->hn) break;
        if (c + 1 < o->hn && o->hkey[c + 1] < o->hkey[c]) c++;
        if (!(o->hkey[c] < key)) break;
        o->hkey[i] = o->hkey[c];
        o->hslot[i] = o->hslot[c];
        i = c;
    }
    if (o->hn) {
        o->hkey[i] = key;
        o->hslot[i] = s;
    }
}
/* a registered slot's heartbeat changed (or it was just created) */
static void hb_touch(oracle_t *o, int32_t s) {
    if (o->purge_mode == 2 && o->reg[s]) heap_push(o, o->hb[s], s);
}

/* ---------------------------------------------------------------- queue ops */
static void q_unlink(oracle_t *o, int32_t s) {
    int32_t p = o->qprev[s], n = o->qnext[s];
    if (p >= 0) o->qnext[p] = n; else o->qhead = n;
    if (n >= 0) o->qprev[n] = p; else o->qtail = p;
    o->inq[s] = 0;
    o->qlen--;
}
static void q_push_back(oracle_t *o, int32_t s) {          /* od[k] = None, k absent */
    o->qprev[s] = o->qtail; o->qnext[s] = -1;
    if (o->qtail >= 0) o->qnext[o->qtail] = s; else o->qhead = s;
    o->qtail = s; o->inq[s] = 1; o->qlen++;
}
static void q_move_front(oracle_t *o, int32_t s) {         /* od[k]=None; move_to_end(k, last=False) */
    if (o->inq[s]) q_unlink(o, s);
    o->qprev[s] = -1; o->qnext[s] = o->qhead;
    if (o->qhead >= 0) o->qprev[o->qhead] = s; else o->qtail = s;
    o->qhead = s; o->inq[s] = 1; o->qlen++;
}
static int32_t q_pop_front(oracle_t *o) {                  /* popitem(last=False) */
    int32_t s = o->qhead;
    q_unlink(o, s);
    return s;
}

/* ------------------------------------------------------------- lifecycle */
oracle_t *oracle_create(int32_t W, int64_t log_cap) {
    oracle_t *o = (oracle_t *)calloc(1, sizeof(oracle_t));
    if (!o) return NULL;
    o->W = W;
    o->reg = (uint8_t *)calloc(W ? W : 1, 1);
    o->free_ = (int64_t *)calloc(W ? W : 1, 8);
    o->hb = (double *)calloc(W ? W : 1, 8);
    o->epoch = (uint32_t *)calloc(W ? W : 1, 4);
    o->qprev = (int32_t *)calloc(W ? W : 1, 4);
    o->qnext = (int32_t *)calloc(W ? W : 1, 4);
    o->inq = (uint8_t *)calloc(W ? W : 1, 1);
    o->cur_is_start = (uint8_t *)calloc(W ? W : 1, 1);
    o->died_start = (uint8_t *)calloc(W ? W : 1, 1);
    o->seen = (uint8_t *)calloc(W ? W : 1, 1);
    o->start_epoch = (uint32_t *)calloc(W ? W : 1, 4);
    o->cap = log_cap;
    o->log = (int32_t *)calloc(log_cap ? log_cap : 1, 4);
    o->qhead = o->qtail = -1;
    o->last_purge_t = -1.0 / 0.0;
    if (!o->reg || !o->free_ || !o->hb || !o->epoch || !o->qprev || !o->qnext || !o->inq ||
        !o->cur_is_start || !o->died_start || !o->seen || !o->start_epoch || !o->log) return NULL;
    return o;
}

void oracle_destroy(oracle_t *o) {
    if (!o) return;
    free(o->hkey); free(o->hslot);
    free(o->reg); free(o->free_); free(o->hb); free(o->epoch); free(o->qprev); free(o->qnext);
    free(o->inq); free(o->cur_is_start); free(o->died_start); free(o->seen); free(o->start_epoch);
    free(o->log); free(o);
}

void oracle_set_purge_mode(oracle_t *o, int mode) { o->purge_mode = mode; }

/* returns 0, or -1 on inconsistent state (queue entry unregistered/duplicate) */
int oracle_load(oracle_t *o, const uint8_t *reg, const int32_t *free_, const double *hb,
                const uint32_t *epoch, const int32_t *queue, int64_t qlen,
                const int32_t *log, int64_t log_len) {
    if (log_len > o->cap) return -1;
    o->qhead = o->qtail = -1; o->qlen = 0;
    for (int32_t s = 0; s < o->W; s++) {
        o->reg[s] = reg[s] ? 1 : 0; o->free_[s] = free_[s]; o->hb[s] = hb[s];
        o->epoch[s] = epoch[s]; o->inq[s] = 0;
    }
    for (int64_t i = 0; i < qlen; i++) {
        int32_t s = queue[i];
        if (s < 0 || s >= o->W || !o->reg[s] || o->inq[s]) return -1;
        q_push_back(o, s);
    }
    o->hn = 0;
    for (int32_t s = 0; s < o->W; s++) hb_touch(o, s);
    /* The in-flight log (build-defined) holds live entries of current
     * registrations only: an entry of a slot without a record, or older than its
     * registration's epoch, can never be redistributed, so it is dropped here. */
    for (int64_t i = 0; i < log_len; i++) {
        int32_t s = log[i];
        o->log[i] = (s >= 0 && (!o->reg[s] || (uint64_t)i < o->epoch[s])) ? -1 : s;
    }
    o->head = log_len;
    o->events_since_purge = 1;
    return 0;
}

int64_t oracle_export(const oracle_t *o, uint8_t *reg, int32_t *free_, double *hb, uint32_t *epoch,
                      int32_t *queue, int32_t *log, int64_t *head) {
    for (int32_t s = 0; s < o->W; s++) {
        if (reg) reg[s] = o->reg[s];
        if (free_) free_[s] = (int32_t)o->free_[s];
        if (hb) hb[s] = o->hb[s];
        if (epoch) epoch[s] = o->epoch[s];
    }
    int64_t n = 0;
    for (int32_t s = o->qhead; s >= 0; s = o->qnext[s]) { if (queue) queue[n] = s; n++; }
    if (log) memcpy(log, o->log, (size_t)o->head * 4);
    if (head) *head = o->head;
    return n;
}

/* ------------------------------------------------------------ loop pieces */
/* purge_workers (:241-249) with PushWorker.is_alive (:209-212) at clock t */
static void evict(oracle_t *o, int32_t s) {
    o->reg[s] = 0;
    if (o->inq[s]) q_unlink(o, s);                    /* del free_workers[remove_id] (:248-249) */
    if (o->cur_is_start[s]) { o->died_start[s] = 1; o->cur_is_start[s] = 0; }
}

static void purge(oracle_t *o, double t, double tte) {
    if (o->purge_mode >= 1 && t == o->last_purge_t && o->events_since_purge == 0) return;
    if (o->purge_mode == 2) {
        /* the same deletions as the O(W) scan: (t - hb) > tte is monotone in hb (the
         * fp64 subtraction rounds monotonically), so the dead records are exactly the
         * smallest heartbeats -- pop them until the smallest live one survives */
        while (o->hn) {
            int32_t s = o->hslot[0];
            double key = o->hkey[0];
            if (!o->reg[s] || !(o->hb[s] == key)) { heap_pop(o); continue; }  /* stale entry */
            if (!((t - key) > tte)) break;
            heap_pop(o);
            evict(o, s);
        }
        o->last_purge_t = t;
        o->events_since_purge = 0;
        return;
    }
    for (int32_t s = 0; s < o->W; s++) {
        if (o->reg[s] && (t - o->hb[s]) > tte) evict(o, s);  /* time.time() - last_heartbeat > tte */
    }
    o->last_purge_t = t;
    o->events_since_purge = 0;
}

/* one inbound message, :347-387 */
static uint8_t handle(oracle_t *o, uint8_t kind, int32_t s, int32_t val, double t, int64_t seq,
                      int64_t head_in) {
    o->events_since_purge++;
    if (kind == EV_REGISTER) {                                   /* :347-353 */
        if (!o->reg[s]) { o->reg[s] = 1; o->epoch[s] = (uint32_t)head_in; o->seen[s] = 1; }
        o->hb[s] = t;
        hb_touch(o, s);
        o->free_[s] = val;
        if (val > 0) q_move_front(o, s);
        return 0;
    }
    if (!o->reg[s]) {                                            /* :356-358 unknown id */
        o->reg[s] = 1; o->epoch[s] = (uint32_t)head_in; o->seen[s] = 1;
        o->free_[s] = 0; o->hb[s] = t;
        hb_touch(o, s);
        return 1;                                                /* 'reconnect' sent, payload dropped */
    }
    if (kind == EV_RECONNECT) {                                  /* :360-367 */
        o->hb[s] = t;
        o->free_[s] = val;
        if (val > 0) q_move_front(o, s);
    } else if (kind == EV_HEARTBEAT) {                           /* :370-371 */
        o->hb[s] = t;
    } else if (kind == EV_RESULT) {                              /* :374-387 */
        o->free_[s] += 1;
        o->hb[s] = t;
        if (seq >= 0 && seq < o->head && o->log[seq] == s) o->log[seq] = -1;   /* HSET result */
        if (o->free_[s] == 1 && !o->inq[s]) q_push_back(o, s);
    }
    if (kind != EV_OTHER) hb_touch(o, s);
    return 0;
}

/*
 * One tick.  Outputs (caller-allocated):
 *   reconnect_out[E]   1 where the reference answered with {"type":"reconnect"}
 *   orphan_out[...]    old sequence numbers of redistributed tasks, ascending
 *   assign_out[...]    worker slot for dispatched task k (k < n_orphans: orphan k,
 *                      else pending task k - n_orphans); logged at seq head_in + k
 *   evicted_out[...]   slots whose record was deleted and not re-created, ascending
 * dispatch_limit >= 0 stops the dispatch phase after that many tasks (baseline
 * timing of a prefix only).  Returns 0, or -1 if the log would overflow.
 */
int oracle_tick(oracle_t *o, double now, double tte, int32_t E, const uint8_t *kind,
                const int32_t *slot, const int32_t *val, const double *ts, const int64_t *seq,
                int64_t n_pending, int64_t dispatch_limit,
                uint8_t *reconnect_out, int32_t *assign_out, int64_t *n_assigned,
                int64_t *orphan_out, int64_t *n_orphans, int32_t *evicted_out, int32_t *n_evicted) {
    const int64_t head_in = o->head;
    for (int32_t s = 0; s < o->W; s++) {
        o->cur_is_start[s] = o->reg[s];
        o->died_start[s] = 0;
        o->seen[s] = o->reg[s];
        o->start_epoch[s] = o->epoch[s];
    }
    /* event phase: a quiet iteration then a delivering iteration per event */
    for (int32_t i = 0; i < E; i++) {
        purge(o, ts[i], tte);
        reconnect_out[i] = handle(o, kind[i], slot[i], val[i], ts[i], seq ? seq[i] : -1, head_in);
        purge(o, ts[i], tte);
    }
    /* dispatch phase at clock `now` */
    int64_t O = 0, k = 0, N = -1;
    int orphans_done = 0;
    for (;;) {
        purge(o, now, tte);
        if (o->qlen == 0) break;                                 /* `if free_workers:` (:393) */
        if (!orphans_done) {
            for (int64_t q = 0; q < head_in; q++) {
                int32_t s = o->log[q];
                if (s >= 0 && o->died_start[s] && (uint64_t)q >= o->start_epoch[s]) orphan_out[O++] = q;
            }
            N = O + n_pending;
            orphans_done = 1;
        }
        if (k >= N) break;                                       /* get_message() -> None */
        if (dispatch_limit >= 0 && k >= dispatch_limit) break;
        if (head_in + k >= o->cap) return -1;
        int32_t w = q_pop_front(o);                              /* popitem(last=False) (:409) */
        o->log[head_in + k] = w;
        assign_out[k++] = w;
        o->free_[w] -= 1;                                        /* :416 */
        if (o->free_[w] > 0) q_push_back(o, w);                  /* :418-419 */
    }
    if (!orphans_done) {
        for (int64_t q = 0; q < head_in; q++) {
            int32_t s = o->log[q];
            if (s >= 0 && o->died_start[s] && (uint64_t)q >= o->start_epoch[s]) orphan_out[O++] = q;
        }
    }
    o->head = head_in + k;
    /* redistributed entries leave the log: their tasks run under new sequence numbers */
    for (int64_t i = 0; i < O; i++) o->log[orphan_out[i]] = -1;
    int32_t ne = 0;
    for (int32_t s = 0; s < o->W; s++)
        if (o->seen[s] && !o->reg[s]) evicted_out[ne++] = s;
    *n_assigned = k;
    *n_orphans = O;
    *n_evicted = ne;
    return 0;
}
