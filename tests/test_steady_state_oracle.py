"""CPU checks of the steady-state stream helpers (workload.cfk_stream_cuts / cfk_slice / preaccept_queries) and of the
chained C restatement the GPU steady-state test compares with: CommandsForKey.update is applied command by command
(local/SafeCommandStore.java:217-240), so applying the batches one after another to the previous result equals one
application of every update so far."""
import numpy as np

import cfk_cases as CC
import oracle
from accord_amd import workload as W


def test_stream_cuts_and_chain():
    u = W.cfk_update_stream(4_000, 4, 1_500, dist="zipf", window=500)
    cuts = W.cfk_stream_cuts(u, 1_500, 300, 4)
    assert cuts[0] > 0 and all(a < b for a, b in zip(cuts, cuts[1:]))
    n_fin = 0
    state = oracle.cfk_apply(CC.empty_snapshot(), W.cfk_slice(u, 0, cuts[0]))
    for b in range(4):
        part = W.cfk_slice(u, cuts[b], cuts[b + 1])
        q = W.preaccept_queries(part)
        assert len(q["msb"]) == 300                      # every new txn of the batch, once
        assert int(q["part_off"][-1]) == 4 * 300
        n_fin += int(((part["status"] >= W.COMMITTED) & (part["status"] <= W.INVALID_OR_TRUNCATED)).sum())
        state = oracle.cfk_apply(state, part)
        whole = oracle.cfk_apply(CC.empty_snapshot(), W.cfk_slice(u, 0, cuts[b + 1]))
        for k in whole:
            np.testing.assert_array_equal(state[k], whole[k], err_msg=f"batch {b} {k}")
    assert n_fin > 0   # the batches carry final statuses of earlier txns too
