"""Numpy model of the sharded tick protocol (faasbal_api.hip / k_*_shard) -- TEST ONLY.

Reproduces, per rank, what phase 1 writes into the exchange buffer (same byte
layout as ``xlayout`` in faasbal_api.hip: per-rank records of 128 u64 words --
the GPU spreads the orphan count over words 0, 16, .., 112 (one per 128-byte
line); this model puts O in word 0 and also keeps sum c / max c in words 1 / 2,
which the GPU re-derives from the c bytes instead -- front / back lists as int32 slot+1, per-event status bytes, and
min(c, 255) per LRU position), and what phase 2 derives from the summed
buffer.  The CPU tests all-reduce these buffers with torch.distributed (gloo,
world_size 2) and compare the merged result with the sequential oracle.
"""
import numpy as np

KEEP, OUT, FRONT, BACK = 0, 1, 2, 3
R_MAX = 128  # sharded ticks support fill levels below 128 rounds (c8 exchange)
XREC_WORDS = 128  # u64 words of one rank's exchange record (kXRecWords)


def xlayout(world, E, Qlog):
    rec = 0
    front = 8 * XREC_WORDS * world
    back = front + 4 * E
    evs = back + 4 * E
    c8 = evs + E
    total = (c8 + Qlog + 15) & ~15
    return dict(rec=rec, front=front, back=back, evs=evs, c8=c8, total=total)


def shard_range(W, world, rank):
    per = -(-W // world)
    base = min(rank * per, W)
    return base, min(per, W - base)


def split(st, world, rank):
    W = len(st["reg"])
    base, n = shard_range(W, world, rank)
    log = np.asarray(st["log"], np.int64).copy()
    # live entries of current registrations only (fb_load_shard drops the others)
    reg, ep = np.asarray(st["reg"]).astype(bool), np.asarray(st["epoch"], np.int64)
    li = np.clip(log, 0, None)
    log[(log >= 0) & (~reg[li] | (np.arange(len(log)) < ep[li]))] = -1
    seq = np.nonzero((log >= base) & (log < base + n))[0]
    return dict(base=base, n=n, reg=st["reg"][base:base + n].astype(bool).copy(),
                free=st["free"][base:base + n].astype(np.int64).copy(), hb=st["hb"][base:base + n].copy(),
                epoch=st["epoch"][base:base + n].astype(np.int64).copy(), queue=np.asarray(st["queue"], np.int64),
                log_slot=log[seq].copy(), log_seq=seq.astype(np.int64), head=len(log))


def phase1(rs, world, rank, now, tte, ev_kind, ev_slot, ev_val, ev_ts, ev_seq, T):
    base, n, E, head = rs["base"], rs["n"], len(ev_kind), rs["head"]
    lay = xlayout(world, E, len(rs["queue"]) + 2 * E)
    x = np.zeros(lay["total"], np.uint8)
    front = np.zeros(E, np.int32)
    back = np.zeros(E, np.int32)
    evs = np.zeros(E, np.uint8)
    reg0 = rs["reg"].copy()
    inq = np.zeros(n, bool)
    own_q = rs["queue"][(rs["queue"] >= base) & (rs["queue"] < base + n)] - base
    inq[own_q] = True
    cur_reg, cur_free, cur_hb, cur_ep = reg0.copy(), rs["free"].copy(), rs["hb"].copy(), rs["epoch"].copy()
    died_mid = np.zeros(n, bool)
    touched = np.zeros(n, bool)
    qstat = np.full(n, KEEP)
    log_slot = rs["log_slot"].copy()
    seqpos = {int(q): i for i, q in enumerate(rs["log_seq"])}
    order = np.argsort(ev_slot, kind="stable")
    for gs in np.unique(ev_slot):
        if not (base <= gs < base + n):
            continue
        s = gs - base
        reg, fr, h, ep, q = bool(reg0[s]), int(cur_free[s]), cur_hb[s], int(cur_ep[s]), bool(inq[s])
        qs, qi, cis, ds = (KEEP if q else OUT), -1, reg, False
        for i in (int(i) for i in order if ev_slot[i] == gs):
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
                evs[i] = 1
            elif k == 1:
                h, fr = ts, v
                if v > 0:
                    q, qs, qi = True, FRONT, i
            elif k == 2:
                h = ts
            elif k == 3:
                fr, h = fr + 1, ts
                li = seqpos.get(int(ev_seq[i]), -1)
                if 0 <= ev_seq[i] < head and li >= 0 and log_slot[li] == gs:
                    log_slot[li] = -1
                if fr == 1 and not q:
                    q, qs, qi = True, BACK, i
        touched[s] = True
        cur_reg[s], cur_free[s], cur_hb[s], cur_ep[s], died_mid[s], qstat[s] = reg, fr, h, ep, ds, qs
        if qs == FRONT:
            front[E - 1 - qi] = gs + 1
        if qs == BACK:
            back[qi] = gs + 1
    dead = cur_reg & ((now - cur_hb) > tte)
    alive = cur_reg & ~dead
    died_start = reg0 & (dead | died_mid)
    evicted = (reg0 | touched) & ~alive
    if n:
        li = np.clip(log_slot - base, 0, n - 1)
        # the committed epoch: entries of the registration alive at tick start (k_scan F-role)
        orph_mask = (log_slot >= 0) & died_start[li] & (rs["log_seq"] >= rs["epoch"][li])
    else:
        orph_mask = np.zeros(len(log_slot), bool)
    orphans = rs["log_seq"][orph_mask]
    # own LRU positions of fronts ++ queue ++ backs
    lq = np.concatenate([front.astype(np.int64) - 1, rs["queue"], back.astype(np.int64) - 1])
    c = np.zeros(len(lq), np.int64)
    for pos, gs in enumerate(lq):
        if not (base <= gs < base + n) or not alive[gs - base]:
            continue
        if E <= pos < E + len(rs["queue"]) and touched[gs - base] and qstat[gs - base] != KEEP:
            continue
        c[pos] = max(cur_free[gs - base], 1)
    rec = np.zeros(XREC_WORDS * world, np.uint64)
    rec[XREC_WORDS * rank:XREC_WORDS * rank + 3] = [len(orphans), c.sum(), c.max(initial=0)]
    x[lay["rec"]:lay["front"]] = rec.view(np.uint8)
    x[lay["front"]:lay["back"]] = front.view(np.uint8)
    x[lay["back"]:lay["evs"]] = back.view(np.uint8)
    x[lay["evs"]:lay["c8"]] = evs
    x[lay["c8"]:lay["c8"] + len(lq)] = np.minimum(c, 255).astype(np.uint8)
    ctx = dict(lay=lay, E=E, T=T, alive=alive, evicted=evicted, orphans=np.sort(orphans), cur_free=cur_free,
               cur_hb=cur_hb, cur_ep=cur_ep, touched=touched, log_slot=log_slot, raw_c=c, world=world)
    return x, ctx


def phase2(rs, ctx, x, redist=True):
    """Returns (outputs of this rank, next rank state).  redist=False: a purge-only
    tick (fb_purge_launch) -- orphans reported, none dispatched."""
    lay, E, world, base, n, head = ctx["lay"], ctx["E"], ctx["world"], rs["base"], rs["n"], rs["head"]
    rec = x[lay["rec"]:lay["front"]].view(np.uint64).reshape(world, XREC_WORDS).astype(np.int64)
    O, cap, maxc = int(rec[:, 0].sum()), int(rec[:, 1].sum()), int(rec[:, 2].max())
    front = x[lay["front"]:lay["back"]].view(np.int32).astype(np.int64) - 1
    back = x[lay["back"]:lay["evs"]].view(np.int32).astype(np.int64) - 1
    lq = np.concatenate([front, rs["queue"], back])
    c = x[lay["c8"]:lay["c8"] + len(lq)].astype(np.int64)
    own = (lq >= base) & (lq < base + n) & (c > 0)
    N_eff = min((O if redist else 0) + ctx["T"], cap)
    rlim = min(maxc, R_MAX)
    S = [0]
    for r in range(rlim):
        S.append(S[-1] + int((c > r).sum()))
    L = max(r for r in range(rlim + 1) if S[r] <= N_eff)
    assert not (maxc > R_MAX and L >= R_MAX - 1), "fill level beyond the sharded round limit"
    p = N_eff - S[L]
    AL = int((c > L).sum())
    tasks, slots = [], []
    assign_all = np.full(N_eff, -1, np.int32)  # the whole tick's task -> slot (fb_set_full_assign)
    for r in range(L + 1):
        act = np.nonzero(c > r)[0]
        lim = len(act) if r < L else p
        sel = act[:lim]
        sel_own = np.nonzero(own[sel])[0]
        tasks.append(S[r] + sel_own)
        slots.append(lq[sel[sel_own]])
        assign_all[S[r]:S[r] + lim] = lq[sel]
    tasks = np.concatenate(tasks) if tasks else np.zeros(0, np.int64)
    slots = np.concatenate(slots) if slots else np.zeros(0, np.int64)
    rankL = np.cumsum(c > L) - 1
    rankL1 = np.cumsum(c > L + 1) - 1
    free_out = ctx["cur_free"].copy()
    newq = {}
    for pos in np.nonzero(c > 0)[0]:
        nq = min(c[pos], L) + (1 if c[pos] > L and rankL[pos] < p else 0)
        if own[pos]:
            free_out[lq[pos] - base] = ctx["cur_free"][lq[pos] - base] - nq
        if c[pos] > L:
            if rankL[pos] >= p:
                newq[rankL[pos] - p] = lq[pos]
            elif c[pos] > L + 1:
                newq[AL - p + rankL1[pos]] = lq[pos]
    queue = np.asarray([newq[i] for i in range(len(newq))], np.int64)
    alive, touched, evicted = ctx["alive"], ctx["touched"], ctx["evicted"]
    reg = rs["reg"].copy()
    hb, ep = rs["hb"].copy(), rs["epoch"].copy()
    reg[touched] = alive[touched]
    hb[touched], ep[touched] = ctx["cur_hb"][touched], ctx["cur_ep"][touched]
    reg[evicted & ~touched] = False
    assert np.all(np.diff(tasks) > 0)
    log_slot = ctx["log_slot"].copy()
    log_slot[np.isin(rs["log_seq"], ctx["orphans"])] = -1  # redistributed entries leave the log at commit
    nxt = dict(rs, reg=reg, free=free_out, hb=hb, epoch=ep, queue=queue,
               log_slot=np.concatenate([log_slot, slots]),
               log_seq=np.concatenate([rs["log_seq"], head + tasks]), head=head + N_eff)
    out = dict(task=tasks, slot=slots.astype(np.int32), orphans=ctx["orphans"].astype(np.int64),
               evicted=(np.nonzero(evicted)[0] + base).astype(np.int32),
               reconnect=x[lay["evs"]:lay["c8"]].copy(), n_assigned=N_eff, assign_all=assign_all)
    return out, nxt
