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
