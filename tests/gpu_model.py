"""Numpy model of the GPU tick algorithm (faasbal_kernels.hip) -- TEST ONLY.

Mirrors the kernels' decomposition (per-slot event segments, logical queue
fronts ++ queue ++ backs, c = max(free,1), water-filling by rounds with ranks)
so the design can be checked against the sequential oracle on CPU.
"""
import numpy as np

KEEP, OUT, FRONT, BACK = 0, 1, 2, 3


def tick(st, now, tte, ev_kind, ev_slot, ev_val, ev_ts, ev_seq, T):
    reg0 = st["reg"].astype(bool).copy()
    free_in = st["free"].astype(np.int64).copy()
    hb = st["hb"].copy()
    epoch = st["epoch"].copy()
    queue = list(st["queue"])
    log = st["log"].copy()
    head = len(log)
    W = len(reg0)
    # the log holds live entries of current registrations only (entries of slots
    # without a record, or older than their registration's epoch, are dropped at load)
    stale = (log >= 0) & ((~reg0[np.clip(log, 0, None)]) | (np.arange(head) < epoch[np.clip(log, 0, None)]))
    log[stale] = -1
    E = len(ev_kind)
    inq = np.zeros(W, bool)
    inq[queue] = True
    touched = np.zeros(W, bool)
    post = {}
    front = [-1] * E
    back = [-1] * E
    status = np.zeros(E, np.uint8)
    order = np.argsort(ev_slot, kind="stable")
    for s in np.unique(ev_slot):
        idxs = [int(i) for i in order if ev_slot[i] == s]
        reg, fr, h, ep, q = bool(reg0[s]), int(free_in[s]), hb[s], epoch[s], bool(inq[s])
        qs, qi = (KEEP if q else OUT), -1
        cis, ds = reg, False
        for i in idxs:
            k, v, ts = int(ev_kind[i]), int(ev_val[i]), ev_ts[i]
            if reg and (ts - h) > tte:
                reg, q, qs = False, False, OUT
                if cis:
                    ds, cis = True, False
            if k == 0:
                if not reg:
                    reg, ep = True, head
                h, fr = ts, v
                if v > 0:
                    q, qs, qi = True, FRONT, i
            elif not reg:
                reg, ep, h, fr = True, head, ts, 0
                status[i] = 1
            elif k == 1:
                h, fr = ts, v
                if v > 0:
                    q, qs, qi = True, FRONT, i
            elif k == 2:
                h = ts
            elif k == 3:
                fr += 1
                h = ts
                sq = int(ev_seq[i])
                if 0 <= sq < head and log[sq] == s:
                    log[sq] = -1
                if fr == 1 and not q:
                    q, qs, qi = True, BACK, i
        touched[s] = True
        post[s] = (reg, fr, h, ep, ds, qs)
        if qs == FRONT:
            front[E - 1 - qi] = s
        if qs == BACK:
            back[qi] = s
    # k_slots
    cur_reg = reg0.copy()
    cur_hb = hb.copy()
    cur_free = free_in.copy()
    cur_ep = epoch.copy()
    died_mid = np.zeros(W, bool)
    qstat = np.full(W, KEEP)
    for s, (reg, fr, h, ep, ds, qs) in post.items():
        cur_reg[s], cur_free[s], cur_hb[s], cur_ep[s], died_mid[s], qstat[s] = reg, fr, h, ep, ds, qs
    dead = cur_reg & ((now - cur_hb) > tte)
    alive = cur_reg & ~dead
    died_start = reg0 & (dead | died_mid)
    evicted = (reg0 | touched) & ~alive
    # orphans
    orph = [q for q in range(head) if log[q] >= 0 and died_start[log[q]] and q >= epoch[log[q]]]
    O = len(orph)
    # logical queue
    lq = front + queue + back
    c = np.zeros(len(lq), np.int64)
    for pos, s in enumerate(lq):
        if s < 0 or not alive[s]:
            continue
        if E <= pos < E + len(queue) and touched[s] and qstat[s] != KEEP:
            continue
        c[pos] = max(cur_free[s], 1)
    maxc = int(c.max()) if len(c) else 0
    N = O + T
    cap = int(c.sum())
    Neff = min(N, cap)
    S = [0]
    for r in range(maxc):
        S.append(S[-1] + int((c > r).sum()))
    L = max(r for r in range(maxc + 1) if S[r] <= Neff)
    p = Neff - S[L]
    assign = np.full(Neff, -1, np.int64)
    rankL = {}
    rankL1 = {}
    for r in range(min(L + 2, maxc)):
        act = np.nonzero(c > r)[0]
        for rank, pos in enumerate(act):
            if r < L or (r == L and rank < p):
                assign[S[r] + rank] = lq[pos]
            if r == L:
                rankL[pos] = rank
            if r == L + 1:
                rankL1[pos] = rank
    AL = int((c > L).sum())
    newq = {}
    free_out = cur_free.copy()
    for pos in np.nonzero(c > 0)[0]:
        s = lq[pos]
        n = min(c[pos], L) + (1 if c[pos] > L and rankL[pos] < p else 0)
        free_out[s] -= n
        if c[pos] > L:
            if rankL[pos] >= p:
                newq[rankL[pos] - p] = s
            elif c[pos] > L + 1:
                newq[AL - p + rankL1[pos]] = s
    nq = [newq[i] for i in range(len(newq))]
    new_log = np.concatenate([log, assign.astype(np.int32)])
    new_log[np.asarray(orph, np.int64)] = -1  # redistributed entries leave the log at commit
    reg_out = reg0.copy()
    hb_out = hb.copy()
    ep_out = epoch.copy()
    for s in range(W):
        if touched[s]:
            reg_out[s] = alive[s]
            hb_out[s] = cur_hb[s]
            ep_out[s] = cur_ep[s]
        elif evicted[s]:
            reg_out[s] = False
    new_st = dict(reg=reg_out.astype(np.uint8), free=free_out.astype(np.int32), hb=hb_out, epoch=ep_out,
                  queue=np.asarray(nq, np.int32), log=new_log)
    out = dict(reconnect=status, assign=assign.astype(np.int32), orphans=np.asarray(orph, np.int64),
               evicted=np.nonzero(evicted)[0].astype(np.int32))
    return out, new_st


# ---------------------------------------------------------------- deque mode
PART2 = 1 << 30  # qraw flag: the token sat in A_L[p:] (not served in round L)


def deque_load(st):
    """Committed deque-mode state from a plain one (queue may repeat slots):
    per-position rank j of each token among its slot's tokens (encoded as a
    part-2 entry with x_w = 0), per-slot token counts."""
    W = len(st["reg"])
    cnt = np.zeros(W, np.int64)
    qraw = np.zeros(len(st["queue"]), np.int64)
    for i, s in enumerate(st["queue"]):
        cnt[s] += 1
        qraw[i] = cnt[s] | PART2
    return dict(st, qraw=qraw, tokcnt=cnt, xw=np.zeros(W, np.int64), KL=np.zeros(W, np.int64))


def token_c(f, k, j):
    """Rounds served to the j-th (1-based, deque order) of a worker's k tokens
    when the worker has f free processes at dispatch start (start() loop,
    task_dispatcher.py:313-322: every served token decrements the shared count
    and is re-appended while it stays > 0).  Returns (c, m, q): c = m + 1 + (j <= q)."""
    if f <= 0:
        return 1, 0, f - 1  # q = f - m k - 1 with m = 0: j <= q never holds
    m = max(0, -(-f // k) - 1)
    q = f - m * k - 1
    return m + 1 + (1 if j <= q else 0), m, q


def tick_deque(st, ev_kind, ev_slot, ev_val, ev_ts, ev_seq, T):
    reg0 = st["reg"].astype(bool).copy()
    free_in = st["free"].astype(np.int64).copy()
    hb = st["hb"].copy()
    queue = list(st["queue"])
    log = st["log"].copy()
    head = len(log)
    W = len(reg0)
    E = len(ev_kind)
    status = np.zeros(E, np.uint8)
    front, frank = [-1] * E, [0] * E
    back, brank = [-1] * E, [0] * E
    touched = np.zeros(W, bool)
    cur_reg, cur_free, cur_hb = reg0.copy(), free_in.copy(), hb.copy()
    post_tok = st["tokcnt"].copy()
    post_nf = np.zeros(W, np.int64)
    order = np.argsort(ev_slot, kind="stable")
    for s in np.unique(ev_slot):
        idxs = [int(i) for i in order if ev_slot[i] == s]
        k_old = int(st["tokcnt"][s])
        nf = sum(1 for i in idxs if ev_kind[i] == 0 and ev_val[i] > 0)
        reg, fr, h = bool(reg0[s]), int(free_in[s]), hb[s]
        mf = nb = 0
        for i in idxs:
            k, v = int(ev_kind[i]), int(ev_val[i])
            if k == 0:
                reg, h, fr = True, ev_ts[i], v
                if v > 0:
                    mf += 1
                    front[E - 1 - i], frank[E - 1 - i] = s, nf - mf + 1
            elif k == 3:
                if not reg:
                    status[i] = 2
                    continue
                fr += 1
                sq = int(ev_seq[i])
                if 0 <= sq < head and log[sq] == s:
                    log[sq] = -1
                if fr == 1:
                    nb += 1
                    back[i], brank[i] = s, k_old + nf + nb
        touched[s] = True
        cur_reg[s], cur_free[s], cur_hb[s] = reg, fr, h
        post_tok[s] = k_old + nf + nb
        post_nf[s] = nf
    lq = front + queue + back
    c = np.zeros(len(lq), np.int64)
    jj = np.zeros(len(lq), np.int64)
    mq = {}
    for pos, s in enumerate(lq):
        if s < 0:
            continue
        if pos < E:
            j = frank[pos]
        elif pos < E + len(queue):
            raw = int(st["qraw"][pos - E])
            jr = raw & (PART2 - 1)
            j = jr - st["xw"][s] if raw & PART2 else st["KL"][s] - st["xw"][s] + jr
            j += post_nf[s]
        else:
            j = brank[pos - E - len(queue)]
        c[pos], m, q = token_c(int(cur_free[s]), int(post_tok[s]), int(j))
        jj[pos] = j
        mq[s] = (m, q, int(post_tok[s]))
    maxc = int(c.max()) if len(c) else 0
    cap = int(c.sum())
    Neff = min(T, cap)
    S = [0]
    for r in range(maxc):
        S.append(S[-1] + int((c > r).sum()))
    L = max(r for r in range(maxc + 1) if S[r] <= Neff)
    p = Neff - S[L]
    assign = np.full(Neff, -1, np.int64)
    rankL, rankL1 = {}, {}
    for r in range(min(L + 2, maxc)):
        act = np.nonzero(c > r)[0]
        for rank, pos in enumerate(act):
            if r < L or (r == L and rank < p):
                assign[S[r] + rank] = lq[pos]
            if r == L:
                rankL[pos] = rank
            if r == L + 1:
                rankL1[pos] = rank
    AL = int((c > L).sum())
    free_out = cur_free.copy()
    tok_n = np.zeros(W, np.int64)
    xw_n = np.zeros(W, np.int64)
    KL_n = np.zeros(W, np.int64)
    newq = {}
    for pos in np.nonzero(c > 0)[0]:
        s = lq[pos]
        n = min(c[pos], L) + (1 if c[pos] > L and rankL[pos] < p else 0)
        free_out[s] -= n
        if c[pos] > L:
            m, q, k = mq[s]
            KL_n[s] = k if L < m + 1 else (q if L == m + 1 else 0)
            if rankL[pos] < p:
                xw_n[s] = max(xw_n[s], jj[pos])
            npos, part2 = -1, 0
            if rankL[pos] >= p:
                npos, part2 = rankL[pos] - p, PART2
            elif c[pos] > L + 1:
                npos = AL - p + rankL1[pos]
            if npos >= 0:
                newq[npos] = (s, jj[pos] | part2)
                tok_n[s] += 1
    nq = [newq[i][0] for i in range(len(newq))]
    qraw = np.asarray([newq[i][1] for i in range(len(newq))], np.int64)
    new_st = dict(reg=cur_reg.astype(np.uint8), free=free_out.astype(np.int32), hb=cur_hb,
                  epoch=st["epoch"], queue=np.asarray(nq, np.int32), log=np.concatenate([log, assign.astype(np.int32)]),
                  qraw=qraw, tokcnt=tok_n, xw=xw_n, KL=KL_n)
    out = dict(reconnect=status, assign=assign.astype(np.int32), orphans=np.zeros(0, np.int64),
               evicted=np.zeros(0, np.int32))
    return out, new_st
