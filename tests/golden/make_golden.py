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


if __name__ == "__main__":
    main()
