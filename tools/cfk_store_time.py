"""Time acc_cfk_apply_deps on the bench's config-2-sized CommandsForKey update stream (workload.cfk_update_stream:
1M txns x 8 keys, ~2M updates, 16M (update, key) pairs, 63M deps), inputs resident in HBM: acc_cfk_apply alone (the
snapshot API) beside the unified store's update (apply + the txn-major view and missing[] indices rebuilt + copied
into the store). One-off measurement for DESIGN.md §3g."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd")]
import torch  # noqa: E402
from accord_amd import _lib as L  # noqa: E402
from accord_amd import workload as W  # noqa: E402
from accord_amd.deps import Context  # noqa: E402

DIST = os.environ.get("CFK_DIST", "uniform")   # "zipf": the config-2-shaped zipf(0.99) stream (hot keys)
u = W.cfk_update_stream(1_000_000, dist=DIST)
dev = torch.device("cuda", 0)
d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in u.items()}
ptr = lambda k: d[k].data_ptr()  # noqa: E731
ui = L.CfkUpdates(L.ACC_MEM_DEVICE, len(u["msb"]), len(u["key"]), len(u["dmsb"]),
                  L.TsCols(ptr("msb"), ptr("lsb"), ptr("node")), L.TsCols(ptr("xmsb"), ptr("xlsb"), ptr("xnode")),
                  ptr("status"), ptr("flags"), ptr("key_off"), ptr("key"), ptr("dep_off"),
                  L.TsCols(ptr("dmsb"), ptr("dlsb"), ptr("dnode")))
torch.cuda.synchronize()
with Context(0) as c:
    res = {}
    for rep in range(3):
        h = C.c_void_p()
        c.check(c._lib.acc_cfk_create(c.handle, C.byref(h)))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c.check(c._lib.acc_cfk_apply_deps(c.handle, h, C.byref(ui)))
        torch.cuda.synchronize()
        res.setdefault("store_apply_ms", []).append(round((time.perf_counter() - t0) * 1e3, 2))
        v = L.BatchIn()
        c.check(c._lib.acc_cfk_view(c.handle, h, C.byref(v)))
        kv = L.KeydepsView()
        t0 = time.perf_counter()
        c.check(c._lib.acc_keydeps_batch(c.handle, C.byref(v), C.byref(kv)))
        torch.cuda.synchronize()
        res.setdefault("keydeps_on_store_ms", []).append(round((time.perf_counter() - t0) * 1e3, 2))
        c._lib.acc_cfk_destroy(h)
    print({"dist": DIST, "updates": len(u["msb"]), "pairs": len(u["key"]), "deps": len(u["dmsb"]), "store_txns": int(v.n_txn),
           "store_pairs": int(v.n_pairs), **res})
with Context(0, timing=True) as c:   # one more store update with every kernel timed: where its time goes
    h = C.c_void_p()
    c.check(c._lib.acc_cfk_create(c.handle, C.byref(h)))
    c.check(c._lib.acc_cfk_apply_deps(c.handle, h, C.byref(ui)))
    torch.cuda.synchronize()
    c.timing_reset()
    c._lib.acc_cfk_destroy(h)
    c.check(c._lib.acc_cfk_create(c.handle, C.byref(h)))
    c.check(c._lib.acc_cfk_apply_deps(c.handle, h, C.byref(ui)))
    torch.cuda.synchronize()
    t = c.timing()
    top = sorted(t.items(), key=lambda kv: -kv[1][0])[:14]
    print("store update kernels (ms):", {k: round(v[0], 3) for k, v in top}, "sum", round(sum(v[0] for v in t.values()), 3))
    print("paths:", {k: v for k, v in c.stats().items() if k.startswith("cfk.")})
    c._lib.acc_cfk_destroy(h)
