"""Seeded cases for RelationMultiMap.remove = KeyDeps.without / RangeDeps.without (utils/RelationMultiMap.java:843-905)
and the recovery reduce that uses it (messages/BeginRecovery.java:180-183, coordinate/Recover.java:320-322): one deps
half per group (rmm_cases.gen_groups with one reply each) and per group the TxnId set(s) of the predicate
remove = Deps::contains, plus an independent set-based model of the Java's three returns."""
import numpy as np

import rmm_cases as RC


def one_per_group(seed, n_groups, is_range, **kw):
    """n_groups deps objects in the acc_rmm_in layout (group g = reply g)."""
    _, half = RC.gen_groups(seed, n_groups, 1, is_range=is_range, **kw)
    return half


def group_vals(m, g):
    v0, v1 = int(m["val_off"][g]), int(m["val_off"][g + 1])
    return [(int(m["msb"][v]), int(m["lsb"][v]), int(m["node"][v])) for v in range(v0, v1)]


def make_sets(seed, m, modes=("subset", "single", "all", "empty", "foreign", "flipped")):
    """Per group a remove set split over two sorted sets (set a = `KeyDeps.txnIds`, set b = `RangeDeps.txnIds` of
    the witness): every mode of the Java's returns — a random subset, one TxnId, all of them (-> NONE), none
    (-> from), TxnIds foreign to the group (-> from), identity-equal TxnIds with other raw flag bits (Timestamp.equals
    ignores bits outside IDENTITY_LSB; compareTo == 0)."""
    rng = np.random.default_rng(seed)
    g_n = len(m["val_off"]) - 1
    sets = ([], [])
    for g in range(g_n):
        vals = group_vals(m, g)
        mode = modes[int(rng.integers(0, len(modes)))]
        if mode == "subset":
            pick = [t for t in vals if rng.random() < 0.4]
        elif mode == "single":
            pick = [vals[int(rng.integers(0, len(vals)))]] if vals else []
        elif mode == "all":
            pick = list(vals)
        elif mode == "empty":
            pick = []
        elif mode == "foreign":
            pick = [t for t in RC.txn_pool(rng, 6) if RC.ts_key(*t) not in {RC.ts_key(*v) for v in vals}]
        else:
            pick = [RC.flip_bits(rng, t, 1.0) for t in vals if rng.random() < 0.5]
        a, b = [], []
        for t in pick:
            r = rng.random()
            if r < 0.45:
                a.append(t)
            elif r < 0.9:
                b.append(t)
            else:
                a.append(t); b.append(t)
        # a few foreign TxnIds in every set (never change the result)
        for t in RC.txn_pool(rng, 2, wide=True):
            (a if rng.random() < 0.5 else b).append(t)
        for s, x in zip(sets, (a, b)):
            uniq = {}
            for t in x:
                uniq.setdefault(RC.ts_key(*t), t)
            s.append(sorted(uniq.values(), key=lambda t: RC.ts_key(*t)))
    return pack_sets(sets[0]), pack_sets(sets[1])


def pack_sets(per_group):
    off, msb, lsb, node = [0], [], [], []
    for ts in per_group:
        for t in ts:
            msb.append(t[0]); lsb.append(t[1]); node.append(t[2])
        off.append(len(msb))
    return dict(off=np.array(off, np.uint64), msb=np.array(msb, np.uint64), lsb=np.array(lsb, np.uint64),
                node=np.array(node, np.int32))


def set_keys(s, g):
    if s is None:
        return set()
    return {RC.ts_key(s["msb"][q], s["lsb"][q], s["node"][q]) for q in range(int(s["off"][g]), int(s["off"][g + 1]))}


def model_without(m, g, removed: set):
    """Independent set model of RelationMultiMap.remove for group g: (kind, key_idx, val_idx, k2v)."""
    k0, k1 = int(m["key_off"][g]), int(m["key_off"][g + 1])
    o0, o1 = int(m["k2v_off"][g]), int(m["k2v_off"][g + 1])
    nk, no = k1 - k0, o1 - o0
    vals = group_vals(m, g)
    nv = len(vals)
    h = [int(x) for x in m["k2v"][o0:o1]]
    if no == nk:
        return 0, list(range(nk)), list(range(nv)), h
    kept = [i for i, t in enumerate(vals) if RC.ts_key(*t) not in removed]
    if len(kept) == nv:
        return 0, list(range(nk)), list(range(nv)), h
    if not kept:
        return 1, [], [], []
    remap = {v: q for q, v in enumerate(kept)}
    lists, prev = [], nk
    for k in range(nk):
        end = h[k]
        lists.append([remap[v] for v in h[prev:end] if v in remap])
        prev = end
    hdr, body = [], []
    for lst in lists:
        body.extend(lst)
        hdr.append(nk + len(body))
    return 2, list(range(nk)), kept, hdr + body


def model_batch(m, sa, sb):
    g_n = len(m["key_off"]) - 1
    out = dict(kind=[], key_off=[0], key_idx=[], val_off=[0], val_idx=[], k2v_off=[0], k2v=[])
    for g in range(g_n):
        kd, ki, vi, k2v = model_without(m, g, set_keys(sa, g) | set_keys(sb, g))
        out["kind"].append(kd)
        out["key_idx"].extend(ki); out["val_idx"].extend(vi); out["k2v"].extend(k2v)
        out["key_off"].append(len(out["key_idx"])); out["val_off"].append(len(out["val_idx"]))
        out["k2v_off"].append(len(out["k2v"]))
    return {k: np.array(v, dtype=np.uint8 if k == "kind" else np.uint32 if k.endswith("idx") else
                        np.int32 if k == "k2v" else np.uint64) for k, v in out.items()}


def group_lists(m, res, g):
    """The result of group g as {key position: [TxnId keys]} and its TxnId keys (for the KeyDepsTest property)."""
    vals = group_vals(m, g)
    v0, v1 = int(res["val_off"][g]), int(res["val_off"][g + 1])
    kept = [vals[int(i)] for i in res["val_idx"][v0:v1]]
    k0, k1 = int(res["key_off"][g]), int(res["key_off"][g + 1])
    o0 = int(res["k2v_off"][g])
    nk = k1 - k0
    lists, prev = {}, nk
    for q in range(nk):
        end = int(res["k2v"][o0 + q])
        lists[int(res["key_idx"][k0 + q])] = [RC.ts_key(*kept[int(x)]) for x in res["k2v"][o0 + prev:o0 + end]]
        prev = end
    return lists, [RC.ts_key(*t) for t in kept]


def gen_recovery(seed, n_groups, max_replies, n_keys=6, n_txn=10, p_flip=0.2):
    """Per recovered txn (group) its replies' earlierCommittedWitness and earlierAcceptedNoWitness deps, both halves,
    drawn from one TxnId pool per group so the accepted TxnIds overlap the committed ones (the without removes some,
    all or none of a group). Returns (grp_off, committed dict(key, range), accepted dict(key, range))."""
    rng = np.random.default_rng(seed)
    grp_off = [0]
    reps = {(w, h): [] for w in ("c", "a") for h in (False, True)}
    for _ in range(n_groups):
        nr = int(rng.integers(1, max_replies + 1))
        for is_range in (False, True):
            pool = RC.txn_pool(rng, n_txn, domain=1 if is_range else 0)
            keys = RC.random_keys(rng, n_keys, is_range, False)
            p_c, p_a = float(rng.uniform(0.3, 0.95)), float(rng.uniform(0.3, 0.95))
            for _ in range(nr):
                for w, p in (("c", p_c), ("a", p_a)):
                    out = reps[(w, is_range)]
                    if rng.random() < 0.15:
                        out.append(([], [], {}))   # an empty reply (skipped by the merge)
                        continue
                    ks = sorted(i for i in range(len(keys)) if rng.random() < 0.6) or [0]
                    ent, used = {}, set()
                    for j, _i in enumerate(ks):
                        vs = sorted(v for v in range(n_txn) if rng.random() > p)
                        if vs:
                            ent[j] = vs
                            used.update(vs)
                    if not used:
                        ent[0] = [0]
                        used = {0}
                    vals = sorted(used)
                    idx = {v: q for q, v in enumerate(vals)}
                    ent = {j: [idx[v] for v in vs] for j, vs in ent.items()}
                    out.append(([keys[i] for i in ks], [RC.flip_bits(rng, pool[v], p_flip) for v in vals], ent))
        grp_off.append(len(reps[("c", False)]))
    g = np.array(grp_off, np.uint64)
    return (g, dict(key=RC.build_half(reps[("c", False)], False), range=RC.build_half(reps[("c", True)], True)),
            dict(key=RC.build_half(reps[("a", False)], False), range=RC.build_half(reps[("a", True)], True)))
