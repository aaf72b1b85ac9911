"""Time acc_levelise on the 1M-txn test graph (tests/test_levelise_gpu.py::test_levelise_one_million) per tier:
python tools/lv_time.py [auto|lds|windowed|waves]  (the walk, as acc_opts.lv_tier)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd")]
from accord_amd.deps import Context, levelise  # noqa: E402

rng = np.random.RandomState(2024)
n, k = 1_000_000, 6
er = rng.permutation(n).astype(np.uint32)
pos = np.argsort(er).astype(np.int64)
src = np.repeat(np.arange(n, dtype=np.int64), k)
p = er[src].astype(np.int64)
back = np.minimum(p, rng.randint(1, 3000, size=n * k))
near = pos[np.maximum(p - back, 0)]
far = rng.randint(0, n, size=n * k)
d = np.where(rng.rand(n * k) < 0.9, near, far)
chain = pos[np.maximum(p[::k] - 1, 0)]
allsrc = np.concatenate([src, np.arange(n)])
alld = np.concatenate([d, chain])
o = np.lexsort((alld, allsrc))
allsrc, alld = allsrc[o], alld[o]
keep = np.ones(len(alld), bool)
keep[1:] = (allsrc[1:] != allsrc[:-1]) | (alld[1:] != alld[:-1])
allsrc, alld = allsrc[keep], alld[keep]
off = np.zeros(n + 1, np.uint64)
np.cumsum(np.bincount(allsrc, minlength=n), out=off[1:])
alld = alld.astype(np.uint32)
with Context(0, lv_tier=sys.argv[1] if len(sys.argv) > 1 else "auto") as ctx:
    levelise(ctx, off, alld, er)
    t = time.perf_counter()
    lv, order, nl = levelise(ctx, off, alld, er)
    dt = time.perf_counter() - t
    tier = ctx.stats().get("levelise.lds_tier")
print(f"1M graph: {nl} levels, {dt * 1e3:.1f} ms (host copies included), {dt / nl * 1e6:.3f} us per level, tier {tier}")
