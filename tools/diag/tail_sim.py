"""Which tail-team policy should the re-dealt solve use?  List-scheduling simulation (256 CUs, one molecule per CU,
blocks dispatched in order to the first free CU) of the two launches of a re-dealt ALDP solve from per-molecule data
dumped by tools/aldp_tail_probe.py (TP_DUMP: the re-deal key, the NFE at the first launch's end, the final NFE): the
first launch in batch order, then the second with the K longest-key slots as teams of G (an evaluation `speed[G]`
times faster, G CUs each; tools/team_tangent_probe.py) and the rest alone.  Times in units of one evaluation alone.
Usage: python tools/diag/tail_sim.py keys_base.npz [keys_frames.npz ...]"""
import heapq
import sys

import numpy as np

SPEED = {1: 1.0, 2: 1.24, 3: 1.26, 4: 1.43}
NCU = 256


def schedule(jobs, ncu=NCU):
    """jobs: [(cus, duration)] in dispatch order; a job starts when `cus` CUs are free (members dispatched in order)"""
    free = [0.0] * ncu
    heapq.heapify(free)
    end = 0.0
    for cus, dur in jobs:
        starts = [heapq.heappop(free) for _ in range(cus)]
        t0 = max(starts)
        for _ in range(cus):
            heapq.heappush(free, t0 + dur)
        end = max(end, t0 + dur)
    return end


def model_k(keys, G, kmax, ncu=NCU):
    """redeal_kernel's choice (ecnf_hip.hip)"""
    k = np.minimum(keys, 1e6)
    w = k.sum()
    extra = G / SPEED[G] - 1.0
    best, best_k, pre = max(k[0], w / ncu), 0, 0.0
    for K in range(1, min(kmax, len(k)) + 1):
        pre += k[K - 1]
        t = max(k[K] if K < len(k) else 0.0, k[0] / SPEED[G], (w + extra * pre) / ncu)
        if t < best:
            best, best_k = t, K
    return best_k


def run(path):
    d = np.load(path)
    key, nfe1, nfe = d["key"], d["nfe1"], d["nfe"]
    act = key >= 0
    l1 = schedule([(1, float(n)) for n in np.minimum(nfe1, nfe)])
    idx = np.nonzero(act)[0]
    order = idx[np.lexsort((idx, -key[idx]))]
    rem = (nfe - nfe1).astype(float)
    print(f"{path}: {act.sum()} unfinished after launch 1 ({l1:.0f} evals), max NFE {nfe.max()}")

    def l2(G, K):
        return schedule([(G, rem[m] / SPEED[G]) for m in order[:K]] + [(1, rem[m]) for m in order[K:]])
    print(f"  no tail: {l1 + l2(1, 0):.0f}   true-order no tail: "
          f"{l1 + schedule([(1, rem[m]) for m in idx[np.argsort(-rem[idx])]]):.0f}")
    for G in (2, 3, 4):
        row = []
        for K in (8, 16, 24, 32, 48, 64):
            row.append(f"K{K}:{l1 + l2(G, K):.0f}")
        km = model_k(np.sort(key[idx])[::-1], G, min(64, NCU // (2 * G)))
        print(f"  G={G}: " + " ".join(row) + f"   model K={km}: {l1 + l2(G, km):.0f}")


for p in sys.argv[1:]:
    run(p)


def sim_policy(path, Gs=(2, 3, 4), Ks=(0, 8, 16, 24, 32, 40, 48, 56, 64)):
    """the K (and G) that minimise the simulated second launch on the ESTIMATED remaining work (key x NFE per step so
    far), and what that choice gives on the true remaining work"""
    d = np.load(path)
    key, nfe1, nfe, steps1 = d["key"], d["nfe1"], d["nfe"], d["steps1"]
    idx = np.nonzero(key >= 0)[0]
    order = idx[np.lexsort((idx, -key[idx]))]
    est = np.minimum(key, 1e6) * nfe1 / np.maximum(steps1, 1)
    rem = (nfe - nfe1).astype(float)
    l1 = schedule([(1, float(n)) for n in np.minimum(nfe1, nfe)])
    for G in Gs:
        def l2(work, K):
            return schedule([(G, work[m] / SPEED[G]) for m in order[:K]] + [(1, work[m]) for m in order[K:]])
        ests = {K: l2(est, K) for K in Ks if K * G <= NCU // 2 or K == 0}
        kb = min(ests, key=lambda k: (ests[k], k))
        print(f"  {path} G={G}: estimated-best K={kb} -> true {l1 + l2(rem, kb):.0f} (est {l1 + ests[kb]:.0f})")


for p in sys.argv[1:]:
    sim_policy(p)


def sim_stop(path, thresholds=((64, 4),), tail=(2, 64), stop_cost=6.0):
    """launch 2 (optionally with tail teams) stopped when at most `n` molecules remain unfinished, then a launch with
    the survivors as teams of G (G x n <= CUs), possibly again at the next threshold; stop_cost: evaluations lost per
    stop (the molecules finish their current step)"""
    d = np.load(path)
    key, nfe1, nfe = d["key"], d["nfe1"], d["nfe"]
    idx = np.nonzero(key >= 0)[0]
    order = idx[np.lexsort((idx, -key[idx]))]
    rem = {int(m): float(nfe[m] - nfe1[m]) for m in idx}
    l1 = schedule([(1, float(n)) for n in np.minimum(nfe1, nfe)])
    # event simulation of launch 2: (start, end) per molecule on a heap of CUs
    G2, K2 = tail
    jobs = [(G2 if k < K2 else 1, m) for k, m in enumerate(order)]
    free = [0.0] * NCU
    heapq.heapify(free)
    spans = {}
    for cus, m in jobs:
        starts = [heapq.heappop(free) for _ in range(cus)]
        t0 = max(starts)
        dur = rem[m] / SPEED[cus]
        for _ in range(cus):
            heapq.heappush(free, t0 + dur)
        spans[m] = (t0, t0 + dur, cus)
    t = 0.0
    out = []
    ends = sorted(e for _, e, _ in spans.values())
    n_all = len(ends)
    done_rem = {}
    total = l1
    cur = dict(spans)
    prev_t = 0.0
    for n_th, G in thresholds:
        if n_all <= n_th:
            break
        t_stop = ends[n_all - n_th - 1]   # the time the (n_all - n_th)-th molecule finishes
        surv = {}
        for m, (s0, e0, cus) in cur.items():
            if e0 > t_stop:
                done = max(0.0, t_stop - s0) * SPEED[cus]
                surv[m] = rem[m] - done + stop_cost
        total += t_stop
        # next launch: survivors as teams of G, all concurrent
        ends = sorted(v / SPEED[G] for v in surv.values())
        rem = surv
        cur = {m: (0.0, v / SPEED[G], G) for m, v in surv.items()}
        n_all = len(ends)
        out.append((n_th, G, round(t_stop), len(surv)))
    total += max(e for _, e, _ in cur.values())
    print(f"  {path}: tail {tail} stops {thresholds}: {total:.0f}  {out}")


for p in sys.argv[1:]:
    for th in (((64, 4),), ((128, 2),), ((128, 2), (64, 4)), ((96, 2),), ((32, 4),)):
        for tail in ((2, 64), (1, 0)):
            sim_stop(p, th, tail)


def sweep(paths):
    for tail in ((1, 0), (2, 16), (2, 32), (2, 64), (4, 16), (4, 32), (3, 32)):
        for th in (((64, 4),), ((48, 4),), ((80, 3),), ((96, 2), (48, 4))):
            for p in paths:
                sim_stop(p, th, tail)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "--sweep":
    sweep(sys.argv[2:])
