"""Seeded synthetic batches for the dependency-calculation path.

Every stream is counter-based SplitMix64 (``x_i = mix64(seed ^ salt + (i+1)*GAMMA)``), so the same
(seed, config) gives the same arrays on every host. Layout matches ``acc_batch_in`` (include/accord_amd.h):
TxnId/executeAt as (msb, lsb, node) columns, InternalStatus ordinals, CSR key offsets and IntKey codes.

TxnId i: epoch=1, hlc=i+1, node=1+(i mod 8), flags = kind<<1 | domain (Timestamp.java:81-89,
TxnId.java:124-137). Committed-class txns get executeAt bumped to hlc+U[1,1000] with node 1000+(i mod 1024)
for 10% of them, so no executeAt compares equal to any TxnId or other executeAt.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)

# InternalStatus ordinals (CommandsForKey.java:194-203)
TRANSITIVELY_KNOWN, HISTORICAL, PREACCEPTED, ACCEPTED, COMMITTED, STABLE, APPLIED, INVALID_OR_TRUNCATED = range(8)
# Txn.Kind ordinals (Txn.java:53-113)
READ, WRITE, EPHEMERAL_READ, SYNC_POINT, EXCLUSIVE_SYNC_POINT, LOCAL_ONLY = range(6)

CONFIG_SEEDS = {
    "1a": 0xACC00101,
    "1b": 0xACC00102,
    "2": 0xACC00002,
    "3u": 0xACC00003,
    "3z": 0xACC00004,
    "4": 0xACC00005,
    "5": 0xACC00006,
}


def mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= M1
        z ^= z >> np.uint64(27)
        z *= M2
        z ^= z >> np.uint64(31)
    return z


def stream(seed: int, salt: int, n: int, offset: int = 0) -> np.ndarray:
    """n SplitMix64 outputs of stream `salt` starting at counter `offset`."""
    base = np.uint64((seed ^ (salt * 0x632BE59BD9B4E019)) & 0xFFFFFFFFFFFFFFFF)
    ctr = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(base + ctr * GAMMA)


def uniform01(seed: int, salt: int, n: int, offset: int = 0) -> np.ndarray:
    return (stream(seed, salt, n, offset) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def stream_at(seed: int, salt: int, idx: np.ndarray) -> np.ndarray:
    """The outputs of stream `salt` at counters idx (stream(seed, salt, n)[idx] without the other counters)."""
    base = np.uint64((seed ^ (salt * 0x632BE59BD9B4E019)) & 0xFFFFFFFFFFFFFFFF)
    ctr = np.asarray(idx, dtype=np.uint64) + np.uint64(1)
    with np.errstate(over="ignore"):
        return mix64(base + ctr * GAMMA)


def uniform01_at(seed: int, salt: int, idx: np.ndarray) -> np.ndarray:
    return (stream_at(seed, salt, idx) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def int_key_code(keys: np.ndarray) -> np.ndarray:
    """IntKey order-preserving code: u32(key ^ 0x80000000) as u64."""
    return (keys.astype(np.int64) + (1 << 31)).astype(np.uint64)


def encode_ts(epoch, hlc, flags, node):
    """Timestamp(epoch, hlc, flags, node) fields (Timestamp.java:81-89)."""
    epoch = np.asarray(epoch, dtype=np.uint64)
    hlc = np.asarray(hlc, dtype=np.uint64)
    flags = np.asarray(flags, dtype=np.uint64)
    msb = (epoch << np.uint64(15)) | (hlc >> np.uint64(48))
    with np.errstate(over="ignore"):
        lsb = (hlc << np.uint64(16)) | flags
    return msb, lsb, np.asarray(node, dtype=np.int32)


@dataclass
class Batch:
    """One CommandsForKey snapshot: the acc_batch_in columns."""
    txn_msb: np.ndarray
    txn_lsb: np.ndarray
    txn_node: np.ndarray
    exe_msb: np.ndarray
    exe_lsb: np.ndarray
    exe_node: np.ndarray
    status: np.ndarray
    key_off: np.ndarray
    key_code: np.ndarray
    meta: dict = field(default_factory=dict)

    @property
    def n_txn(self) -> int:
        return int(self.status.shape[0])

    @property
    def n_pairs(self) -> int:
        return int(self.key_off[-1])

    def permuted(self, perm: np.ndarray) -> "Batch":
        """Same batch with txns reordered: new txn i = old txn perm[i]."""
        counts = np.diff(self.key_off.astype(np.int64))[perm]
        off = np.zeros(len(perm) + 1, dtype=np.uint32)
        np.cumsum(counts, out=off[1:])
        starts = self.key_off[:-1].astype(np.int64)[perm]
        idx = np.repeat(starts - off[:-1].astype(np.int64), counts) + np.arange(int(off[-1]), dtype=np.int64)
        return Batch(self.txn_msb[perm], self.txn_lsb[perm], self.txn_node[perm], self.exe_msb[perm],
                     self.exe_lsb[perm], self.exe_node[perm], self.status[perm], off, self.key_code[idx],
                     dict(self.meta, permuted=True))

    def arrays(self):
        return dict(txn_msb=self.txn_msb, txn_lsb=self.txn_lsb, txn_node=self.txn_node, exe_msb=self.exe_msb,
                    exe_lsb=self.exe_lsb, exe_node=self.exe_node, status=self.status, key_off=self.key_off,
                    key_code=self.key_code)


def _distinct_keys(seed: int, n_txn: int, k: int, sample) -> np.ndarray:
    """n_txn rows of k distinct key ids; duplicates are redrawn from fresh counters until none remain."""
    keys = sample(0, n_txn * k).reshape(n_txn, k)
    offset = n_txn * k
    for _ in range(200):
        keys.sort(axis=1)
        dup = np.zeros_like(keys, dtype=bool)
        dup[:, 1:] = keys[:, 1:] == keys[:, :-1]
        nd = int(dup.sum())
        if nd == 0:
            return keys
        keys[dup] = sample(offset, nd)
        offset += nd
    raise RuntimeError("could not draw distinct keys")


def zipf_sampler(seed: int, salt: int, n_keys: int, s: float, permute: bool):
    w = 1.0 / np.power(np.arange(1, n_keys + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    perm = None
    if permute:
        perm = np.argsort(stream(seed, salt + 7, n_keys), kind="stable").astype(np.int64)

    table = []

    def inverse_cdf(u):
        """searchsorted(cdf, u, 'right') through a 2^24-bucket table of cdf indices (bucket bounds bracket the answer
        within a few ranks; random probes of a 128 MB cdf miss the cache at every level of a plain binary search)."""
        if not table:
            nb = 1 << 24
            table.append(np.searchsorted(cdf, np.arange(nb + 1, dtype=np.float64) / nb, side="right").astype(np.int64))
        idx = table[0]
        b = (u * float(len(idx) - 1)).astype(np.int64)
        lo, hi = idx[b], np.minimum(idx[b + 1], len(cdf))
        act = np.nonzero(lo < hi)[0]
        la, ha, ua = lo[act], hi[act], u[act]
        while len(la):
            mid = (la + ha) >> 1
            c = cdf[mid] <= ua
            la = np.where(c, mid + 1, la)
            ha = np.where(c, ha, mid)
            done = la >= ha
            if done.any():
                lo[act[done]] = la[done]
                keep = ~done
                act, la, ha, ua = act[keep], la[keep], ha[keep], ua[keep]
        return lo

    def sample(offset, n):
        u = uniform01(seed, salt, n, offset)
        r = inverse_cdf(u) if n > (1 << 20) else np.searchsorted(cdf, u, side="right")
        r = np.minimum(r, n_keys - 1)
        return perm[r] if perm is not None else r
    return sample


def uniform_sampler(seed: int, salt: int, n_keys: int):
    def sample(offset, n):
        return (stream(seed, salt, n, offset) % np.uint64(n_keys)).astype(np.int64)
    return sample


def keydeps_batch(n_txn: int, keys_per_txn: int, n_keys: int, seed: int, dist: str = "uniform",
                  zipf_s: float = 0.99, status_model: str = "model", window: int = 10_000,
                  p_write: float = 0.5, p_syncpoint: float = 0.0, permute_keys: bool = True) -> Batch:
    """Synthetic batch per SURVEY.md §8(d).

    status_model: "preaccepted" (config 1a: every txn PREACCEPTED) or "model" (window W of
    PREACCEPTED 70%/ACCEPTED 30%, else APPLIED 80%/STABLE 10%/COMMITTED 10%, plus 0.1%
    INVALID_OR_TRUNCATED and 0.1% TRANSITIVELY_KNOWN).
    """
    i = np.arange(n_txn, dtype=np.int64)
    cols = keydeps_txn_columns(n_txn, i, seed, status_model, window, p_write, p_syncpoint)
    sampler = key_sampler(seed, dist, n_keys, zipf_s, permute_keys)
    keys = _distinct_keys(seed, n_txn, keys_per_txn, sampler)
    key_off = (np.arange(n_txn + 1, dtype=np.int64) * keys_per_txn).astype(np.uint32)
    key_code = int_key_code(keys.reshape(-1))
    meta = dict(n_txn=n_txn, keys_per_txn=keys_per_txn, n_keys=n_keys, seed=seed, dist=dist, zipf_s=zipf_s,
                status_model=status_model, window=window, p_write=p_write)
    return Batch(*cols, key_off, key_code, meta)


def key_sampler(seed: int, dist: str, n_keys: int, zipf_s: float = 0.99, permute_keys: bool = True):
    if dist == "uniform":
        return uniform_sampler(seed, 10, n_keys)
    if dist == "zipf":
        return zipf_sampler(seed, 10, n_keys, zipf_s, permute_keys)
    raise ValueError(dist)


def keydeps_txn_columns(n_txn: int, i: np.ndarray, seed: int, status_model: str = "model", window: int = 10_000,
                        p_write: float = 0.5, p_syncpoint: float = 0.0):
    """The per-txn columns of keydeps_batch (TxnId, executeAt, InternalStatus) at global txn indices i of an n_txn
    batch: every one is a function of i alone (counter-based streams), so any subset is generated on its own."""
    i = np.asarray(i, dtype=np.int64)
    m = len(i)
    u_kind = uniform01_at(seed, 1, i)
    kind = np.where(u_kind < p_write, WRITE, READ).astype(np.int64)
    if p_syncpoint > 0:
        kind = np.where(uniform01_at(seed, 2, i) < p_syncpoint, SYNC_POINT, kind)
    flags = (kind << 1) | 0  # domain Key = 0
    t_msb, t_lsb, t_node = encode_ts(np.ones(m), i + 1, flags, 1 + (i % 8))

    if status_model == "preaccepted":
        status = np.full(m, PREACCEPTED, dtype=np.uint8)
    elif status_model == "model":
        u = uniform01_at(seed, 3, i)
        in_window = i >= n_txn - window
        status = np.where(in_window, np.where(u < 0.7, PREACCEPTED, ACCEPTED),
                          np.where(u < 0.8, APPLIED, np.where(u < 0.9, STABLE, COMMITTED))).astype(np.uint8)
        u2 = uniform01_at(seed, 4, i)
        status = np.where(u2 < 0.001, INVALID_OR_TRUNCATED,
                          np.where(u2 < 0.002, TRANSITIVELY_KNOWN, status)).astype(np.uint8)
    else:
        raise ValueError(status_model)

    committed = (status >= COMMITTED) & (status <= APPLIED)
    bump = committed & (uniform01_at(seed, 5, i) < 0.1)
    bump_by = 1 + (stream_at(seed, 6, i) % np.uint64(1000)).astype(np.int64)
    e_msb, e_lsb_b, e_node_b = encode_ts(np.ones(m), i + 1 + bump_by, np.zeros(m), 1000 + (i % 1024))  # no ties: |i - i' | < 1024
    exe_msb = np.where(bump, e_msb, t_msb).astype(np.uint64)
    exe_lsb = np.where(bump, e_lsb_b, t_lsb).astype(np.uint64)
    exe_node = np.where(bump, e_node_b, t_node).astype(np.int32)
    return t_msb, t_lsb, t_node, exe_msb, exe_lsb, exe_node, status


def distinct_key_rows(n_txn: int, k: int, sample, lo: int, hi: int):
    """Rows [lo, hi) of _distinct_keys(seed, n_txn, k, sample), generated without the other rows: a generator that
    yields this slice's duplicate count of each redraw round and is sent back (duplicates in earlier rows of the
    batch, duplicates in the whole batch) for it; the slices' callers exchange those counts (an all-gather across the
    ranks holding consecutive slices). Returns the rows (StopIteration.value)."""
    keys = sample(lo * k, (hi - lo) * k).reshape(hi - lo, k)
    offset = n_txn * k
    for _ in range(200):
        keys.sort(axis=1)
        dup = np.zeros_like(keys, dtype=bool)
        dup[:, 1:] = keys[:, 1:] == keys[:, :-1]
        nd = int(dup.sum())
        before, total = yield nd
        if total == 0:
            return keys
        if nd:
            keys[dup] = sample(offset + before, nd)
        offset += total
    raise RuntimeError("could not draw distinct keys")


def merge_exec_rank(n_txn: int, seed: int = CONFIG_SEEDS["5"], max_bump: int = 50) -> np.ndarray:
    """executeAt order of config 5's txns: txn t executes at t + U[0, max_bump) (ties by t), as dense ranks; deps on
    txns with a later executeAt are not waited on (Commands.java:804-810)."""
    key = np.arange(n_txn, dtype=np.int64) + (stream(seed, 50, n_txn) % np.uint64(max_bump)).astype(np.int64)
    order = np.lexsort((np.arange(n_txn), key))
    rank = np.empty(n_txn, dtype=np.uint32)
    rank[order] = np.arange(n_txn, dtype=np.uint32)
    return rank


def config(name: str, scale: float = 1.0) -> Batch:
    """BASELINE.json configs 1a/1b (10k x 4 over 1k keys) and 2 (1M x 8, zipf 0.99 over 1M keys)."""
    if name == "1a":
        return keydeps_batch(10_000, 4, 1_000, CONFIG_SEEDS["1a"], "uniform", status_model="preaccepted")
    if name == "1b":
        # status model with a 1,000-txn uncommitted window (an absolute W = 10,000 would cover all 10k txns)
        return keydeps_batch(10_000, 4, 1_000, CONFIG_SEEDS["1b"], "uniform", status_model="model", window=1_000)
    if name == "2":
        n = int(1_000_000 * scale)
        return keydeps_batch(n, 8, max(1000, int(1_000_000 * scale)), CONFIG_SEEDS["2"], "zipf", 0.99,
                             status_model="model")
    raise ValueError(name)


def merge_batch(n_txn: int = 16_384, replies: int = 64, seed: int = CONFIG_SEEDS["5"], n_keys: int = 1_000_000,
                keys_per_txn: int = 8, deps_per_key: int = 4, p_drop: float = 0.1, p_spurious: float = 0.05) -> dict:
    """Config 5 input in the acc_merge_in layout: group t = coordinated txn t, with `replies` KeyDeps replies.

    Each txn gets a base dependency map (keys_per_txn zipf keys, deps_per_key deps on earlier txns of the batch,
    named by batch index = TxnId rank, so the merged deps form the graph that acc_levelise orders),
    standing in for its config-2-style deps; every reply drops each base entry with p_drop and adds
    round(p_spurious * base entries) spurious ones on the txn's keys. Replies are built in the Java layout
    (sorted unique keys / txnId ranks, keysToTxnIds with the end-offset header)."""
    rng_u = lambda salt, n: uniform01(seed, salt, n)  # noqa: E731
    keys = _distinct_keys(seed, n_txn, keys_per_txn, zipf_sampler(seed, 40, n_keys, 0.99, True))
    kc = int_key_code(keys.reshape(-1)).astype(np.int64)
    t_rank = np.arange(n_txn, dtype=np.int64)  # txn t's TxnId rank = its index: deps name earlier txns of the batch
    # base entries (t, key, dep)
    bt = np.repeat(np.arange(n_txn, dtype=np.int64), keys_per_txn * deps_per_key)
    bk = np.repeat(kc, deps_per_key)
    bd = (rng_u(41, len(bt)) * t_rank[bt]).astype(np.int64)
    # replicate per reply, drop, add spurious
    q_base = np.repeat(bt * replies, replies) + np.tile(np.arange(replies, dtype=np.int64), len(bt))
    k_base = np.repeat(bk, replies)
    d_base = np.repeat(bd, replies)
    keep = rng_u(42, len(q_base)) >= p_drop
    q, k, d = q_base[keep], k_base[keep], d_base[keep]
    n_sp = int(round(p_spurious * keys_per_txn * deps_per_key))
    if n_sp:
        sq = np.repeat(np.arange(n_txn * replies, dtype=np.int64), n_sp)
        st = sq // replies
        sk = kc.reshape(n_txn, keys_per_txn)[st, (rng_u(43, len(sq)) * keys_per_txn).astype(np.int64)]
        sd = (rng_u(44, len(sq)) * t_rank[st]).astype(np.int64)
        q, k, d = np.concatenate([q, sq]), np.concatenate([k, sk]), np.concatenate([d, sd])
    order = np.lexsort((d, k, q))
    q, k, d = q[order], k[order], d[order]
    uniq = np.ones(len(q), dtype=bool)
    uniq[1:] = (q[1:] != q[:-1]) | (k[1:] != k[:-1]) | (d[1:] != d[:-1])
    q, k, d = q[uniq], k[uniq], d[uniq]
    nrep = n_txn * replies
    # keys per reply
    kfirst = np.ones(len(q), dtype=bool)
    kfirst[1:] = (q[1:] != q[:-1]) | (k[1:] != k[:-1])
    key_code = k[kfirst].astype(np.uint64)
    key_cnt = np.bincount(q[kfirst], minlength=nrep)
    # values per reply: unique (q, d)
    comb = np.unique((q << 32) | d)
    val_cnt = np.bincount(comb >> 32, minlength=nrep)
    txn_rank = (comb & 0xFFFFFFFF).astype(np.uint32)
    val_off = np.zeros(nrep + 1, dtype=np.uint64)
    np.cumsum(val_cnt, out=val_off[1:])
    key_off = np.zeros(nrep + 1, dtype=np.uint64)
    np.cumsum(key_cnt, out=key_off[1:])
    # index of each entry's dep within its reply's txnIds
    dep_idx = np.searchsorted(comb, (q << 32) | d) - val_off[q].astype(np.int64)
    ent_cnt = np.bincount(q, minlength=nrep)
    k2v_len = key_cnt + ent_cnt
    k2v_off = np.zeros(nrep + 1, dtype=np.uint64)
    np.cumsum(k2v_len, out=k2v_off[1:])
    k2v = np.zeros(int(k2v_off[-1]), dtype=np.int32)
    # entries: after the reply's header
    ent_start = np.zeros(nrep + 1, dtype=np.int64)
    np.cumsum(ent_cnt, out=ent_start[1:])
    pos_in_reply = np.arange(len(q), dtype=np.int64) - ent_start[q]
    k2v[(k2v_off[q].astype(np.int64) + key_cnt[q] + pos_in_reply)] = dep_idx.astype(np.int32)
    # header: end offset of each key = nk + entries up to and including that key
    klast = np.ones(len(q), dtype=bool)
    klast[:-1] = (q[1:] != q[:-1]) | (k[1:] != k[:-1])
    kq = q[klast]
    key_ord = np.arange(len(kq), dtype=np.int64) - key_off[kq].astype(np.int64)
    k2v[k2v_off[kq].astype(np.int64) + key_ord] = (key_cnt[kq] + pos_in_reply[klast] + 1).astype(np.int32)
    grp_off = (np.arange(n_txn + 1, dtype=np.uint64) * np.uint64(replies))
    return dict(grp_off=grp_off, key_off=key_off, key_code=key_code, val_off=val_off, txn_rank=txn_rank,
                k2v_off=k2v_off, k2v=k2v)


def raw_txn_ids(rank: np.ndarray):
    """The TxnIds behind config-5 txn ranks (batch index t = rank t): epoch 1, hlc t+1, Write, node 1 + t mod 8, in
    compareTo order of the rank (Timestamp.java:81-89)."""
    r = np.asarray(rank, dtype=np.uint64)
    return encode_ts(np.ones_like(r), r + np.uint64(1), np.full_like(r, WRITE << 1), (1 + (r % np.uint64(8))).astype(np.int32))


def merge_batch_raw(m: dict) -> dict:
    """A merge_batch (rank-space acc_merge_in layout) as the raw SerializerSupport half of acc_deps_merge: key codes,
    TxnId columns (raw_txn_ids) and the same keysToTxnIds."""
    msb, lsb, node = raw_txn_ids(m["txn_rank"])
    return dict(key_off=m["key_off"], key_a=m["key_code"], val_off=m["val_off"], msb=msb, lsb=lsb, node=node,
                k2v_off=m["k2v_off"], k2v=m["k2v"])


@dataclass
class RangeBatch:
    """A mixed key/range snapshot: `keys` is the acc_batch_in part (key-domain txns
    list their keys; range-domain txns, TxnId domain bit = 1, list none), plus per-txn Ranges
    [rng_off[t], rng_off[t+1]) for range-domain txns (sorted, non-overlapping: Ranges.ofSortedAndDeoverlapped)
    and one Range bound type for the store (end_inclusive: Range.EndInclusive (s, e], else StartInclusive [s, e))."""
    keys: Batch
    rng_off: np.ndarray
    rng_start: np.ndarray
    rng_end: np.ndarray
    end_inclusive: int = 1
    meta: dict = field(default_factory=dict)

    @property
    def n_txn(self) -> int:
        return self.keys.n_txn

    @property
    def n_ranges(self) -> int:
        return int(self.rng_off[-1])

    def is_range(self) -> np.ndarray:
        return (self.keys.txn_lsb & np.uint64(1)).astype(bool)

    def arrays(self):
        return dict(self.keys.arrays(), rng_off=self.rng_off, rng_start=self.rng_start, rng_end=self.rng_end)


def rangedeps_batch(n_txn: int, seed: int, p_range: float = 0.5, keys_per_txn: int = 4, ranges_per_txn: int = 1,
                    key_bits: int = 32, max_width_log2: int = 16, status_model: str = "model", window: int = 10_000,
                    p_write: float = 0.5, p_syncpoint: float = 0.0, end_inclusive: int = 1) -> RangeBatch:
    """Config 4 per SURVEY.md §8(d): txns interleaved in TxnId order, each a range txn with probability p_range
    (`ranges_per_txn` disjoint ranges, start uniform over the 2^key_bits IntKey code space, width log-uniform
    in [1, 2^max_width_log2]) or a key txn (`keys_per_txn` distinct uniform keys). Kinds Read/Write (p_write),
    optional SyncPoint share; statuses and executeAt bumps as keydeps_batch."""
    i = np.arange(n_txn, dtype=np.int64)
    is_range = uniform01(seed, 20, n_txn) < p_range
    kind = np.where(uniform01(seed, 1, n_txn) < p_write, WRITE, READ).astype(np.int64)
    if p_syncpoint > 0:
        kind = np.where(uniform01(seed, 2, n_txn) < p_syncpoint, SYNC_POINT, kind)
    flags = (kind << 1) | is_range.astype(np.int64)
    t_msb, t_lsb, t_node = encode_ts(np.ones(n_txn), i + 1, flags, 1 + (i % 8))
    if status_model == "preaccepted":
        status = np.full(n_txn, PREACCEPTED, dtype=np.uint8)
    else:
        u = uniform01(seed, 3, n_txn)
        in_window = i >= n_txn - window
        status = np.where(in_window, np.where(u < 0.7, PREACCEPTED, ACCEPTED),
                          np.where(u < 0.8, APPLIED, np.where(u < 0.9, STABLE, COMMITTED))).astype(np.uint8)
        u2 = uniform01(seed, 4, n_txn)
        status = np.where(u2 < 0.001, INVALID_OR_TRUNCATED,
                          np.where(u2 < 0.002, TRANSITIVELY_KNOWN, status)).astype(np.uint8)
    committed = (status >= COMMITTED) & (status <= APPLIED)
    bump = committed & (uniform01(seed, 5, n_txn) < 0.1)
    bump_by = 1 + (stream(seed, 6, n_txn) % np.uint64(1000)).astype(np.int64)
    e_msb, e_lsb_b, e_node_b = encode_ts(np.ones(n_txn), i + 1 + bump_by, np.zeros(n_txn), 1000 + (i % 1024))
    exe_msb = np.where(bump, e_msb, t_msb).astype(np.uint64)
    exe_lsb = np.where(bump, e_lsb_b, t_lsb).astype(np.uint64)
    exe_node = np.where(bump, e_node_b, t_node).astype(np.int32)

    space = 1 << key_bits
    n_key_txn = int((~is_range).sum())
    keys = _distinct_keys(seed, n_key_txn, keys_per_txn, lambda off, n: (stream(seed, 21, n, off) % np.uint64(space))
                          .astype(np.int64))
    counts = np.where(is_range, 0, keys_per_txn)
    key_off = np.zeros(n_txn + 1, dtype=np.uint32)
    np.cumsum(counts, out=key_off[1:])
    key_code = keys.reshape(-1).astype(np.uint64)

    n_rt = int(is_range.sum())
    m = n_rt * ranges_per_txn
    width = np.maximum(1, np.floor(np.exp2(uniform01(seed, 22, m) * max_width_log2))).astype(np.int64)
    start = (stream(seed, 23, m) % np.uint64(max(1, space - (1 << max_width_log2) - 1))).astype(np.int64)
    # ranges of one txn: sorted and non-overlapping (shift each past its predecessor's end)
    st = start.reshape(n_rt, ranges_per_txn)
    wd = width.reshape(n_rt, ranges_per_txn)
    order = np.argsort(st, axis=1, kind="stable")
    st = np.take_along_axis(st, order, 1)
    wd = np.take_along_axis(wd, order, 1)
    for j in range(1, ranges_per_txn):
        st[:, j] = np.maximum(st[:, j], st[:, j - 1] + wd[:, j - 1])
    rs = st.reshape(-1).astype(np.uint64)
    re = (st + wd).reshape(-1).astype(np.uint64)
    rcounts = np.where(is_range, ranges_per_txn, 0)
    rng_off = np.zeros(n_txn + 1, dtype=np.uint32)
    np.cumsum(rcounts, out=rng_off[1:])
    kb = Batch(t_msb, t_lsb, t_node, exe_msb, exe_lsb, exe_node, status, key_off, key_code,
               dict(n_txn=n_txn, seed=seed, p_range=p_range))
    meta = dict(n_txn=n_txn, seed=seed, p_range=p_range, keys_per_txn=keys_per_txn, ranges_per_txn=ranges_per_txn,
                key_bits=key_bits, max_width_log2=max_width_log2, status_model=status_model, window=window,
                p_write=p_write, end_inclusive=end_inclusive)
    return RangeBatch(kb, rng_off, rs, re, end_inclusive, meta)


def config4(scale: float = 1.0, **kw) -> RangeBatch:
    """BASELINE config 4: 10M range txns (1 EndInclusive range each) interleaved 50/50 with 10M key txns x 4
    keys over the int32 key space (scale multiplies the txn count)."""
    return rangedeps_batch(int(20_000_000 * scale), CONFIG_SEEDS["4"], **kw)


def cfk_update_stream(n_txn: int, keys_per_txn: int = 8, n_keys: int | None = None, seed: int = CONFIG_SEEDS["2"] + 7,
                      max_deps: int = 16, lag: int = 64, dist: str = "uniform", window: int = 10_000) -> dict:
    """A CommandsForKey update stream of config-2 size (acc_cfk_apply's CFK_UPD layout), for the N4 bench leg: the txns
    of keydeps_batch(n_txn, keys_per_txn, n_keys, uniform keys, status model) as SafeCommandStore.updateCommandsForKey
    sees them (local/SafeCommandStore.java:217-240): an Accept (ACCEPTED, executeAt = TxnId) at time i, then the final
    status (COMMITTED / STABLE / APPLIED with the batch's executeAt, or INVALID_OR_TRUNCATED) at time i + lag; txns whose
    final status is PREACCEPTED / TRANSITIVELY_KNOWN only pre-accept, ACCEPTED ones only accept. The deps of a txn on
    a key (its keyDeps.txnIds(key)) are the latest max_deps txns below it on that key, every one already known to the
    key's CFK. Uniform keys: a zipf hot key's CFK grows with its whole history (CommandsForKey.update copies the key's
    arrays, linear per update), which the reference bounds by pruning, outside the §8 path. dist="zipf": zipf(0.99) keys
    as config 2 (a hot key's updates take acc_cfk_apply's hot-key closed form). window: the status model's
    uncommitted tail (the last `window` txns never reach a final status)."""
    n_keys = n_keys or n_txn
    b = keydeps_batch(n_txn, keys_per_txn, n_keys, seed, dist, status_model="model", window=window)
    st = b.status.astype(np.int64)
    K = keys_per_txn
    # deps per (txn, key) pair: the latest max_deps txns below it on the key (pairs sorted by (key, txn))
    P = b.n_pairs
    pair_txn = np.repeat(np.arange(n_txn, dtype=np.int64), K)
    order = np.lexsort((pair_txn, b.key_code))
    sk = b.key_code[order]
    new = np.ones(P, bool)
    new[1:] = sk[1:] != sk[:-1]
    seg_start = np.maximum.accumulate(np.where(new, np.arange(P), 0))
    r = np.arange(P) - seg_start                       # position within the key
    pos = np.empty(P, np.int64)
    pos[order] = np.arange(P)                          # sorted position of each pair
    ndep_pair = np.minimum(r, max_deps)[pos]           # per pair (txn-major)
    txn_sorted = pair_txn[order]
    # events: (time, txn, kind) kind 0 = first update, 1 = final update
    first = np.where(st == PREACCEPTED, PREACCEPTED, np.where((st == TRANSITIVELY_KNOWN) | (st == INVALID_OR_TRUNCATED),
                                                               PREACCEPTED, ACCEPTED))
    has_final = (st >= COMMITTED) & (st <= INVALID_OR_TRUNCATED)
    ev_txn = np.concatenate([np.arange(n_txn), np.nonzero(has_final)[0]])
    ev_kind = np.concatenate([np.zeros(n_txn, np.int64), np.ones(int(has_final.sum()), np.int64)])
    ev_time = np.where(ev_kind == 0, 2 * ev_txn, 2 * (ev_txn + lag) + 1)
    o = np.argsort(ev_time, kind="stable")
    ev_txn, ev_kind = ev_txn[o], ev_kind[o]
    U = len(ev_txn)
    ust = np.where(ev_kind == 0, first[ev_txn], st[ev_txn]).astype(np.uint8)
    final_exec = (ev_kind == 1) & (ust != INVALID_OR_TRUNCATED)
    xmsb = np.where(final_exec, b.exe_msb[ev_txn], b.txn_msb[ev_txn]).astype(np.uint64)
    xlsb = np.where(final_exec, b.exe_lsb[ev_txn], b.txn_lsb[ev_txn]).astype(np.uint64)
    xnode = np.where(final_exec, b.exe_node[ev_txn], b.txn_node[ev_txn]).astype(np.int32)
    with_deps = (ust >= ACCEPTED) & (ust <= APPLIED)
    # (update, key) pairs in update order
    up_pair = (ev_txn[:, None] * K + np.arange(K)[None, :]).reshape(-1)
    cnt = np.where(np.repeat(with_deps, K), ndep_pair[up_pair], 0).astype(np.int64)
    dep_off = np.zeros(U * K + 1, np.int64)
    np.cumsum(cnt, out=dep_off[1:])
    D = int(dep_off[-1])
    first_src = np.repeat(pos[up_pair] - cnt, cnt)
    dsrc = first_src + (np.arange(D, dtype=np.int64) - np.repeat(dep_off[:-1], cnt))
    dtx = txn_sorted[dsrc]
    return dict(msb=b.txn_msb[ev_txn], lsb=b.txn_lsb[ev_txn], node=b.txn_node[ev_txn], xmsb=xmsb, xlsb=xlsb, xnode=xnode,
                status=ust, flags=np.ones(U, np.uint8), key_off=(np.arange(U + 1, dtype=np.int64) * K).astype(np.uint32),
                key=b.key_code[up_pair], dep_off=dep_off.astype(np.uint32), dmsb=b.txn_msb[dtx], dlsb=b.txn_lsb[dtx],
                dnode=b.txn_node[dtx], time=ev_time[o])


UPD_FIELDS = ("msb", "lsb", "node", "xmsb", "xlsb", "xnode", "status", "flags")


def cfk_slice(u: dict, a: int, b: int) -> dict:
    """Updates [a, b) of a CFK_UPD update list (cfk_update_stream layout), offsets rebased."""
    ko, do = u["key_off"].astype(np.int64), u["dep_off"].astype(np.int64)
    out = {k: u[k][a:b] for k in UPD_FIELDS}
    out["key_off"] = (ko[a:b + 1] - ko[a]).astype(np.uint32)
    out["key"] = u["key"][ko[a]:ko[b]]
    out["dep_off"] = (do[ko[a]:ko[b] + 1] - do[ko[a]]).astype(np.uint32)
    for f in ("dmsb", "dlsb", "dnode"):
        out[f] = u[f][do[ko[a]]:do[ko[b]]]
    return out


def cfk_stream_cuts(u: dict, n_initial: int, batch_txns: int, n_batches: int) -> list:
    """Update-index cuts of a cfk_update_stream for a replica's steady state: [0, cuts[0]) builds the initial store
    (the first n_initial txns' PreAccept / Accept and every final status due by then), then batch b = [cuts[b],
    cuts[b + 1]) brings batch_txns new txns and the final statuses of older ones (time order: txn i's first update at
    2i, its final status at 2(i + lag) + 1)."""
    t = u["time"]
    return [int(np.searchsorted(t, 2 * (n_initial + b * batch_txns))) for b in range(n_batches + 1)]


def preaccept_queries(part: dict) -> dict:
    """The PreAccept queries of an update slice (acc_preaccept_in host layout: TxnId + its keys): one per command
    first seen in it (a cfk_update_stream txn's first update is its only PreAccept / Accept)."""
    sel = np.nonzero((part["status"] == PREACCEPTED) | (part["status"] == ACCEPTED))[0]
    ko = part["key_off"].astype(np.int64)
    cnt = ko[sel + 1] - ko[sel]
    off = np.zeros(len(sel) + 1, np.int64)
    np.cumsum(cnt, out=off[1:])
    src = np.repeat(ko[sel], cnt) + (np.arange(int(off[-1])) - np.repeat(off[:-1], cnt))
    keys = part["key"][src]
    return dict(msb=part["msb"][sel], lsb=part["lsb"][sel], node=part["node"][sel],
                is_range=np.zeros(len(sel), np.uint8), part_off=off.astype(np.uint32), part_start=keys,
                part_end=np.zeros(len(keys), np.uint64))


def conflicts_updates(part: dict, end_inclusive: int = 1) -> dict:
    """An update slice as MaxConflicts updates (CommandStore.updateMaxConflicts: each command's keys with its
    executeAt; acc_conflicts_in host layout)."""
    U = len(part["msb"])
    return dict(end_inclusive=end_inclusive, xmsb=part["xmsb"], xlsb=part["xlsb"], xnode=part["xnode"],
                key_off=part["key_off"], key=part["key"], rng_off=np.zeros(U + 1, np.uint32),
                rng_start=np.zeros(0, np.uint64), rng_end=np.zeros(0, np.uint64))
