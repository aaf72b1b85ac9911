"""CPU: the N4 zipf key-sample fixture (tests/golden/cfk_zipf_sample.npz) re-derived by the C restatement on a part of
its keys (the 3,000 regular keys and the 2K / 1K hot ones; the 5K-50K ones take a few minutes more in make_golden.py)."""
import os
import sys

import numpy as np

import cfk_cases as CC
import oracle

HERE = os.path.dirname(os.path.abspath(__file__))


def test_cfk_zipf_fixture_reproduces():
    from accord_amd import workload as W
    fx = np.load(os.path.join(HERE, "golden", "cfk_zipf_sample.npz"))
    upd = W.cfk_update_stream(1_000_000, 8, 1_000_000, dist="zipf")
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden import cfk_zipf_keys
    keys = cfk_zipf_keys(upd)
    np.testing.assert_array_equal(keys, fx["keys"])
    cnt = np.unique(CC.restrict(upd, keys)["key"], return_counts=True)[1]
    small = keys[cnt <= 2_500]
    o = oracle.cfk_apply(CC.empty_snapshot(), CC.restrict(upd, small))
    kh, ne, nm = CC.key_hashes(o, small)
    sel = np.searchsorted(fx["keys"], small)
    np.testing.assert_array_equal(kh, fx["hash64"][sel])
    np.testing.assert_array_equal(ne, fx["entries"][sel].astype(np.int64))
