"""GPU parity for a replica's PreAccept path in steady state (messages/PreAccept.java:107-138,
local/CommandStore.java:280-345, local/CommandsForKey.java:652-706): a device store built from the first txns of a
workload.cfk_update_stream, then batches of new txns, each through accord_amd.deps.ReplicaStore — MaxConflicts
proposal, MaxConflicts merge, CommandsForKey.update with deps on the resident store, the KeyDeps scan in place. After
every batch: the proposals equal the C restatement's MaxConflicts over every earlier update, the key-major state equals
the C restatement chained batch by batch (oracle.cfk_apply on its own previous result), the txn-major view and its
missing[] indices equal the host restatement of that state, and the in-place KeyDeps equal the C KeyDeps restatement
of the view."""
import numpy as np
import pytest

import cfk_cases as CC
import oracle
from accord_amd import workload as W

pytestmark = pytest.mark.gpu

FIELDS = ("arena_off", "kd_off", "u_off", "arena", "key_idx", "dep_txn")


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("dist", ["uniform", "zipf"])
def test_replica_preaccept_steady_state(ctx, dist):
    from accord_amd.deps import ReplicaStore, cfk_batch_host
    u = W.cfk_update_stream(24_000, 4, 3_000, dist=dist, window=1_500)
    nb = 5
    cuts = W.cfk_stream_cuts(u, 14_000, 2_000, nb)
    rs = ReplicaStore(ctx)
    try:
        init = W.cfk_slice(u, 0, cuts[0])
        rs.preaccept_batch(init, scan=False)
        o_state = oracle.cfk_apply(CC.empty_snapshot(), init)
        seen_fast = seen_slow = seen_missing = 0
        for b in range(nb):
            part = W.cfk_slice(u, cuts[b], cuts[b + 1])
            q = W.preaccept_queries(part)
            assert len(q["msb"]) == 2_000
            r = rs.preaccept_batch(part, q)
            om = oracle.max_conflicts(W.conflicts_updates(W.cfk_slice(u, 0, cuts[b])), q)
            for k in ("msb", "lsb", "node", "fast"):
                np.testing.assert_array_equal(r["propose"][k], om[k], err_msg=f"{dist} batch {b} propose {k}")
            seen_fast += int(om["fast"].sum())
            seen_slow += int((om["fast"] == 0).sum())
            o_state = oracle.cfk_apply(o_state, part)
            g_state = rs.cfk.state()
            for k in o_state:
                np.testing.assert_array_equal(np.asarray(g_state[k]), np.asarray(o_state[k]),
                                              err_msg=f"{dist} batch {b} state {k}")
            ob, omo, omt = CC.snap_as_batch(o_state)
            gb, gmo, gmt = cfk_batch_host(ctx, rs.cfk.missing_view())
            for f in ("txn_msb", "txn_lsb", "txn_node", "exe_msb", "exe_lsb", "exe_node", "status", "key_off", "key_code"):
                np.testing.assert_array_equal(getattr(gb, f), getattr(ob, f), err_msg=f"{dist} batch {b} view {f}")
            np.testing.assert_array_equal(gmo, omo)
            np.testing.assert_array_equal(gmt, omt)
            seen_missing += len(omt)
            ok = oracle.keydeps_batch(ob)
            for f in FIELDS:
                np.testing.assert_array_equal(getattr(r["keydeps"], f), getattr(ok, f), err_msg=f"{dist} batch {b} keydeps {f}")
        assert seen_fast and seen_slow and seen_missing
    finally:
        rs.close()
