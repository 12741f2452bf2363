"""Maps the Boyar-Peralta S-box circuit onto 3-input LUTs (gfx950
v_bitop3_b32) by cut enumeration + area-flow selection, and checks the mapped
network exhaustively against the S-box.  Used by gen_sbox_hip.py."""
import itertools
from bp_circuit import gates, sbox_ref

K = 3


def build():
    G = gates()
    node = {d: (op, a, b) for d, op, a, b in G}
    order = [d for d, _, _, _ in G]
    return node, order


def fn(op, x, y):
    return x ^ y if op == "+" else (x & y if op == "x" else 1 ^ x ^ y)


def cone_tt(node, root, leaves):
    """Truth table (bit index = leaves[0]<<2 | leaves[1]<<1 | leaves[2])."""
    leaves = list(leaves) + [None] * (K - len(leaves))
    tt = 0
    for j in range(8):
        env = {}
        for i, l in enumerate(leaves):
            if l is not None:
                env[l] = (j >> (K - 1 - i)) & 1

        def ev(n):
            if n in env:
                return env[n]
            op, a, b = node[n]
            v = fn(op, ev(a), ev(b))
            env[n] = v
            return v
        tt |= ev(root) << j
    return tt


def map_lut3():
    node, order = build()
    outs = [f"S{i}" for i in range(8)]
    fanout = {}
    for d, (op, a, b) in node.items():
        for x in (a, b):
            fanout[x] = fanout.get(x, 0) + 1
    cuts = {}
    for i in range(8):
        cuts[f"U{i}"] = [frozenset([f"U{i}"])]
    for d in order:
        op, a, b = node[d]
        cs = set()
        for ca in cuts[a]:
            for cb in cuts[b]:
                u = ca | cb
                if len(u) <= K:
                    cs.add(u)
        cs.add(frozenset([a, b]))
        cuts[d] = [frozenset([d])] + sorted(cs, key=lambda c: (len(c), sorted(c)))
    # area flow
    af = {f"U{i}": 0.0 for i in range(8)}
    best = {}
    for d in order:
        cands = []
        for c in cuts[d][1:]:
            cost = 1.0 + sum(af[x] / max(fanout.get(x, 1), 1) for x in c)
            cands.append((cost, len(c), sorted(c), c))
        cands.sort(key=lambda t: (t[0], t[1], t[2]))
        af[d], _, _, best[d] = cands[0]
    # cover
    used = {}
    stack = list(outs)
    while stack:
        n = stack.pop()
        if n in used or n.startswith("U"):
            continue
        used[n] = best[n]
        stack.extend(best[n])
    # topological order
    topo = [d for d in order if d in used]
    luts = []
    for d in topo:
        leaves = sorted(used[d], key=lambda x: (x[0], int(x[1:]) if x[1:].isdigit() else x))
        luts.append((d, leaves, cone_tt(node, d, leaves)))
    return luts


def map_lut3_ilp(time_limit=600):
    """Area-optimal cover of the same circuit: every 3-feasible cut of every
    gate as a 0/1 variable, a gate is implemented iff one of its cuts is
    chosen, a chosen cut needs its gate leaves implemented, the outputs are
    implemented; minimise the implemented gates (scipy milp / HiGHS).  On the
    Boyar-Peralta circuit: 82 LUTs, proven optimal for this DAG (the area-flow
    cover above: 92)."""
    import numpy as np
    from scipy.optimize import Bounds, LinearConstraint, milp
    node, order = build()
    cuts = {f"U{i}": [frozenset([f"U{i}"])] for i in range(8)}
    for d in order:
        op, a, b = node[d]
        cs = set()
        for ca in cuts[a]:
            for cb in cuts[b]:
                u = ca | cb
                if len(u) <= K:
                    cs.add(u)
        cs.add(frozenset([a, b]))
        cuts[d] = [frozenset([d])] + sorted(cs, key=lambda c: (len(c), sorted(c)))
    var = [(d, c) for d in order for c in cuts[d][1:]]
    yi = {d: i for i, d in enumerate(order)}
    ny, n = len(order), len(order) + len(var)
    rows, lb, ub = [], [], []
    byd = {}
    for j, (d, c) in enumerate(var):
        byd.setdefault(d, []).append(ny + j)
    for d in order:
        r = np.zeros(n)
        r[yi[d]] = 1
        r[byd[d]] = -1
        rows.append(r); lb.append(0); ub.append(0)
    for i in range(8):
        r = np.zeros(n)
        r[yi[f"S{i}"]] = 1
        rows.append(r); lb.append(1); ub.append(1)
    for j, (d, c) in enumerate(var):
        for leaf in c:
            if not leaf.startswith("U"):
                r = np.zeros(n)
                r[yi[leaf]] = 1
                r[ny + j] = -1
                rows.append(r); lb.append(0); ub.append(np.inf)
    cost = np.zeros(n)
    cost[:ny] = 1
    res = milp(cost, constraints=LinearConstraint(np.array(rows), lb, ub),
               integrality=np.ones(n), bounds=Bounds(0, 1),
               options={"time_limit": time_limit})
    assert res.status == 0, res.message
    chosen = {d: c for j, (d, c) in enumerate(var) if res.x[ny + j] > 0.5}
    luts = []
    for d in order:
        if d in chosen:
            leaves = sorted(chosen[d], key=lambda x: (x[0], int(x[1:]) if x[1:].isdigit() else x))
            luts.append((d, leaves, cone_tt(node, d, leaves)))
    return luts


def check(luts):
    ref = sbox_ref()
    for x in range(256):
        env = {f"U{i}": (x >> (7 - i)) & 1 for i in range(8)}
        for d, leaves, tt in luts:
            idx = 0
            for i, l in enumerate(leaves + [None] * (K - len(leaves))):
                idx |= (env[l] if l is not None else 0) << (K - 1 - i)
            env[d] = (tt >> idx) & 1
        y = sum(env[f"S{i}"] << (7 - i) for i in range(8))
        if y != ref[x]:
            return False
    return True


if __name__ == "__main__":
    luts = map_lut3()
    print("area flow: LUT3 count:", len(luts), "exhaustive check:", check(luts))
    luts = map_lut3_ilp()
    print("ILP: LUT3 count:", len(luts), "exhaustive check:", check(luts))
