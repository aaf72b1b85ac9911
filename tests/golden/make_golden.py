"""Generate the committed golden fixtures for BASELINE config 1 (10k txns x 4 keys, 1k uniform keys).

The reference Java cannot be built or run here (no JDK; Gradle needs network), and its own tests hold no
literal vectors for this path. Expected outputs therefore come from the C restatement
(oracle/accord_oracle.c), and this script refuses to write a fixture unless the independent canonical
model (oracle/canonical.py) produces identical arrays for every txn.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle")]

from accord_amd import workload as W  # noqa: E402
import canonical  # noqa: E402
import oracle  # noqa: E402


def main():
    for name in ("1a", "1b"):
        b = W.config(name)
        o = oracle.keydeps_batch(b)
        c = canonical.keydeps_batch(b)
        for t in range(b.n_txn):
            k, d, a = o.txn(t)
            ck, cd, ca = c[t]
            assert list(k) == ck and list(d) == cd and list(a) == ca, f"oracle/canonical mismatch at txn {t}"
        # 4-shard CommandStore evaluation must agree too (PartialDeps.with fold)
        o4 = oracle.keydeps_batch(b, n_shards=4)
        for f in ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn"):
            assert np.array_equal(getattr(o, f), getattr(o4, f)), f
        out = {f"out_{f}": getattr(o, f) for f in ("arena_off", "arena", "kd_off", "key_idx", "u_off", "dep_txn")}
        path = os.path.join(HERE, f"config{name}.npz")
        np.savez_compressed(path, **b.arrays(), **out)
        print(path, os.path.getsize(path), "bytes; edges", o.total_edges)


def config4s():
    """BASELINE config 4 scaled by 1/1000 (20k txns) with the key space scaled by 2^-10 so the stab depth (ranges
    containing a key, ~14) matches the full config: RangeDeps from the C restatement, cross-checked against the
    canonical set model on three query windows (the set model is O(txns x range commands))."""
    rb = W.config4(0.001, key_bits=22)
    o = oracle.rangedeps_batch(rb)
    for lo in (0, 9_000, 19_700):
        ds, de, c = canonical.rangedeps_batch(rb, query_lo=lo, query_hi=lo + 300)
        assert np.array_equal(ds, o.rng_start) and np.array_equal(de, o.rng_end)
        for t in range(lo, lo + 300):
            r, d, a = o.txn(t)
            assert (list(r), list(d), list(a)) == c[t], f"oracle/canonical mismatch at txn {t}"
    out = {f"out_{f}": getattr(o, f) for f in ("rng_start", "rng_end", "arena_off", "arena", "rd_off", "range_id",
                                               "u_off", "dep_txn")}
    path = os.path.join(HERE, "config4s.npz")
    np.savez_compressed(path, **rb.arrays(), end_inclusive=np.int32(rb.end_inclusive), **out)
    print(path, os.path.getsize(path), "bytes; edges", o.total_edges)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "4":
        config4s()
    else:
        main()
        config4s()
