/*
 * deque_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C, single-threaded, sequential restatement of the reference's push
 * dispatcher loop WITHOUT heartbeats, PushDispatcher.start (reference
 * task_dispatcher.py:251-322).  There is no liveness and no purge; the queue of
 * ready workers is a collections.deque (:254) of worker ids that may hold the
 * same id several times (a register of a queued worker appends it at the left
 * again, :280-281; a result that brings free_processes to 1 appends it at the
 * right, :294-295).  Kept here as a growable ring buffer.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library.  Parity is pinned by tests/test_oracle_golden.py against the
 * deque_*.npz vectors captured from the unmodified reference start() loop
 * (tests/golden/make_golden.py).
 *
 * Tick model (as for start_heartbeat): every inbound event is
 * handled in its own iteration in arrival order with the pub/sub tasks hidden,
 * then one task per iteration is popped while the deque is non-empty (:298-322).
 * Event status: 0 handled (or a kind start() has no branch for: ignored),
 * 2 = result from an id without a record -- the reference raises KeyError at
 * :291 and its loop dies; the drop-in reports it and drops the message.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { DQ_REGISTER = 0, DQ_RESULT = 3 };

typedef struct dq_oracle {
    int32_t W;
    uint8_t *reg;     /* slot in self.workers (:194)                      */
    int64_t *free_;   /* PushWorker.free_processes (:205), a Python int   */
    double *hb;       /* PushWorker.last_heartbeat, set at creation (:206) */
    int32_t *dq;      /* ring buffer: the deque free_workers (:254)        */
    int64_t dq_cap, dq_head, dq_len;
    int32_t *log;     /* in-flight log: slot per task sequence, -1 = completed */
    int64_t head, cap;
} dq_oracle_t;

static int dq_grow(dq_oracle_t *o) {
    int64_t nc = o->dq_cap ? 2 * o->dq_cap : 64;
    int32_t *n = (int32_t *)malloc((size_t)nc * 4);
    if (!n) return -1;
    for (int64_t i = 0; i < o->dq_len; i++) n[i] = o->dq[(o->dq_head + i) % o->dq_cap];
    free(o->dq);
    o->dq = n;
    o->dq_cap = nc;
    o->dq_head = 0;
    return 0;
}
static int dq_append(dq_oracle_t *o, int32_t s) {         /* deque.append */
    if (o->dq_len == o->dq_cap && dq_grow(o)) return -1;
    o->dq[(o->dq_head + o->dq_len) % o->dq_cap] = s;
    o->dq_len++;
    return 0;
}
static int dq_appendleft(dq_oracle_t *o, int32_t s) {     /* deque.appendleft */
    if (o->dq_len == o->dq_cap && dq_grow(o)) return -1;
    o->dq_head = (o->dq_head + o->dq_cap - 1) % o->dq_cap;
    o->dq[o->dq_head] = s;
    o->dq_len++;
    return 0;
}
static int32_t dq_popleft(dq_oracle_t *o) {               /* deque.popleft */
    int32_t s = o->dq[o->dq_head];
    o->dq_head = (o->dq_head + 1) % o->dq_cap;
    o->dq_len--;
    return s;
}

dq_oracle_t *dq_oracle_create(int32_t W, int64_t log_cap) {
    dq_oracle_t *o = (dq_oracle_t *)calloc(1, sizeof(dq_oracle_t));
    if (!o) return NULL;
    o->W = W;
    o->reg = (uint8_t *)calloc(W ? W : 1, 1);
    o->free_ = (int64_t *)calloc(W ? W : 1, 8);
    o->hb = (double *)calloc(W ? W : 1, 8);
    o->cap = log_cap;
    o->log = (int32_t *)calloc(log_cap ? log_cap : 1, 4);
    if (!o->reg || !o->free_ || !o->hb || !o->log || dq_grow(o)) return NULL;
    return o;
}

void dq_oracle_destroy(dq_oracle_t *o) {
    if (!o) return;
    free(o->reg); free(o->free_); free(o->hb); free(o->dq); free(o->log); free(o);
}

/* returns 0, or -1 on inconsistent state (a deque entry without a record) */
int dq_oracle_load(dq_oracle_t *o, const uint8_t *reg, const int32_t *free_, const double *hb,
                   const int32_t *queue, int64_t qlen, const int32_t *log, int64_t log_len) {
    if (log_len > o->cap) return -1;
    for (int32_t s = 0; s < o->W; s++) {
        o->reg[s] = reg[s] ? 1 : 0;
        o->free_[s] = free_[s];
        o->hb[s] = hb[s];
    }
    o->dq_head = o->dq_len = 0;
    for (int64_t i = 0; i < qlen; i++) {
        int32_t s = queue[i];
        if (s < 0 || s >= o->W || !o->reg[s] || dq_append(o, s)) return -1;
    }
    memcpy(o->log, log, (size_t)log_len * 4);
    o->head = log_len;
    return 0;
}

/* queue may be NULL (then only the length is returned) */
int64_t dq_oracle_export(const dq_oracle_t *o, uint8_t *reg, int32_t *free_, double *hb, int32_t *queue,
                         int32_t *log, int64_t *head) {
    for (int32_t s = 0; s < o->W; s++) {
        if (reg) reg[s] = o->reg[s];
        if (free_) free_[s] = (int32_t)o->free_[s];
        if (hb) hb[s] = o->hb[s];
    }
    if (queue)
        for (int64_t i = 0; i < o->dq_len; i++) queue[i] = o->dq[(o->dq_head + i) % o->dq_cap];
    if (log) memcpy(log, o->log, (size_t)o->head * 4);
    if (head) *head = o->head;
    return o->dq_len;
}

/*
 * One tick: E inbound events in arrival order, then up to n_pending dispatches.
 * status_out[E], assign_out[...] (slot of task k, logged at sequence head + k).
 * dispatch_limit >= 0 stops after that many tasks (CPU baseline prefix).
 * Returns 0, -1 if the log would overflow, -2 on allocation failure.
 */
int dq_oracle_tick(dq_oracle_t *o, int32_t E, const uint8_t *kind, const int32_t *slot, const int32_t *val,
                   const double *ts, const int64_t *seq, int64_t n_pending, int64_t dispatch_limit,
                   uint8_t *status_out, int32_t *assign_out, int64_t *n_assigned) {
    const int64_t head_in = o->head;
    for (int32_t i = 0; i < E; i++) {
        const int32_t s = slot[i];
        status_out[i] = 0;
        if (kind[i] == DQ_REGISTER) {                           /* :276-281 */
            o->reg[s] = 1;
            o->hb[s] = ts[i];
            o->free_[s] = val[i];
            if (val[i] > 0 && dq_appendleft(o, s)) return -2;
        } else if (kind[i] == DQ_RESULT) {                      /* :284-295 */
            if (!o->reg[s]) {                                   /* KeyError at :291 */
                status_out[i] = 2;
                continue;
            }
            const int64_t q = seq ? seq[i] : -1;
            if (q >= 0 && q < head_in && o->log[q] == s) o->log[q] = -1;   /* HSET result (:288) */
            o->free_[s] += 1;
            if (o->free_[s] == 1 && dq_append(o, s)) return -2;
        }
        /* any other message type: start() has no branch for it */
    }
    int64_t k = 0;
    while (o->dq_len > 0 && k < n_pending) {                    /* `if free_workers:` (:298) */
        if (dispatch_limit >= 0 && k >= dispatch_limit) break;
        if (head_in + k >= o->cap) return -1;
        const int32_t w = dq_popleft(o);                        /* :313 */
        o->log[head_in + k] = w;
        assign_out[k++] = w;
        o->free_[w] -= 1;                                       /* :318 */
        if (o->free_[w] > 0 && dq_append(o, w)) return -2;      /* :321-322 */
    }
    o->head = head_in + k;
    *n_assigned = k;
    return 0;
}
