"""Model of CommandsForKey.update over batches of commands (local/CommandsForKey.java:652-706, as
SafeCommandStore.updateCommandsForKey calls it, local/SafeCommandStore.java:217-240) — TEST INFRASTRUCTURE: a dict of
TxnId -> entry, exported in TxnId order as the acc_batch_in layout."""
from __future__ import annotations

import numpy as np

from accord_amd import workload as W


class Stale(Exception):
    pass


def _key(m, l, n):
    return (int(m), int(l) >> 16, int(l) & 0x1E, int(n))


def has_info(s):
    return 3 <= s <= 6


class Model:
    def __init__(self):
        self.t = {}   # order key -> [msb, lsb, node, emsb, elsb, enode, status, set(keys)]

    def apply(self, b):
        upd = []
        for i in range(b.n_txn):
            m, l, n = int(b.txn_msb[i]), int(b.txn_lsb[i]), int(b.txn_node[i])
            kind = (l >> 1) & 7
            if (l & 1) or kind in (2, 5):
                continue   # not a CommandsForKey member
            k = _key(m, l, n)
            s = int(b.status[i])
            keys = {int(x) for x in b.key_code[int(b.key_off[i]):int(b.key_off[i + 1])]}
            ex = (int(b.exe_msb[i]), int(b.exe_lsb[i]), int(b.exe_node[i])) if has_info(s) else (m, l, n)
            if k in self.t and s < self.t[k][6]:
                raise Stale()
            upd.append((k, m, l, n, ex, s, keys))
        for k, m, l, n, ex, s, keys in upd:
            if k not in self.t:
                self.t[k] = [m, l, n, *ex, s, set(keys)]
                continue
            e = self.t[k]
            if s > e[6] or has_info(s):
                e[3:7] = [*ex, s]
            e[7] |= keys

    def batch(self):
        ks = sorted(self.t)
        rows = [self.t[k] for k in ks]
        off = np.zeros(len(rows) + 1, np.uint32)
        codes = []
        for i, r in enumerate(rows):
            codes.extend(sorted(r[7]))
            off[i + 1] = len(codes)
        col = lambda j, dt: np.array([r[j] for r in rows], dt)  # noqa: E731
        return W.Batch(col(0, np.uint64), col(1, np.uint64), col(2, np.int32), col(3, np.uint64), col(4, np.uint64),
                       col(5, np.int32), col(6, np.uint8), off, np.array(codes, np.uint64))


def delta(rng, model, n_new, n_upd, n_keys=50, kinds=(0, 1, 3, 4), p_skip=0.05, next_hlc=[1]):
    """a batch of commands: n_new fresh TxnIds (random hlc order) and n_upd updates of stored txns (status never lower)"""
    rows = []
    for _ in range(n_new):
        next_hlc[0] += int(rng.integers(1, 4))
        kind = int(rng.choice([2, 5])) if rng.random() < p_skip else int(rng.choice(kinds))
        m, l, n = (int(x) for x in W.encode_ts(1, next_hlc[0], kind << 1, 1 + int(rng.integers(0, 4))))
        s = int(rng.integers(0, 8))
        rows.append((m, l, n, s, sorted({int(x) for x in rng.integers(0, n_keys, size=int(rng.integers(0, 5)))})))
    stored = list(model.t.values())
    for j in rng.permutation(len(stored))[:n_upd]:
        e = stored[int(j)]
        s = int(rng.integers(e[6], 8))
        keys = sorted({int(x) for x in rng.integers(0, n_keys, size=int(rng.integers(0, 3)))})
        rows.append((e[0], e[1], e[2], s, keys))
    order = rng.permutation(len(rows))
    rows = [rows[int(i)] for i in order]
    off, codes, st, em, el, en = [0], [], [], [], [], []
    for m, l, n, s, keys in rows:
        codes.extend(keys)
        off.append(len(codes))
        st.append(s)
        bump = has_info(s) and rng.random() < 0.5
        e = W.encode_ts(1, ((m & 0x7FFF) << 48 | (l >> 16)) + (int(rng.integers(1, 50)) if bump else 0), 0 if bump else l & 0xFFFF,
                        (100 + n) if bump else n)
        em.append(int(e[0])); el.append(int(e[1])); en.append(int(e[2]))
    return W.Batch(np.array([r[0] for r in rows], np.uint64), np.array([r[1] for r in rows], np.uint64),
                   np.array([r[2] for r in rows], np.int32), np.array(em, np.uint64), np.array(el, np.uint64),
                   np.array(en, np.int32), np.array(st, np.uint8), np.array(off, np.uint32),
                   np.array([W.int_key_code(np.array([c]))[0] for c in codes], np.uint64))
