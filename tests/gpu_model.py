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
