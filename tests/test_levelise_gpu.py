"""GPU parity: acc_levelise vs the C restatement and the canonical model."""
import contextlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def random_graph(rng, n, max_deps, exec_perm=True):
    exec_rank = (rng.permutation(n) if exec_perm else np.arange(n)).astype(np.uint32)
    deps = [np.unique(rng.randint(0, n, size=rng.randint(0, max_deps + 1))) for _ in range(n)]
    off = np.concatenate([[0], np.cumsum([len(d) for d in deps])]).astype(np.uint64)
    dep = np.concatenate(deps).astype(np.uint32) if off[-1] else np.zeros(0, np.uint32)
    return off, dep, exec_rank


@pytest.mark.parametrize("n,max_deps", [(1, 0), (100, 5), (5000, 30), (40000, 8)])
def test_levelise_random(ctx, n, max_deps):
    import oracle
    from accord_amd.deps import levelise
    off, dep, er = random_graph(np.random.RandomState(n), n, max_deps)
    lv, order, nl = levelise(ctx, off, dep, er)
    l2, o2, nl2 = oracle.levelise(off, dep, er)
    np.testing.assert_array_equal(lv, l2)
    np.testing.assert_array_equal(order, o2)
    assert nl == nl2


@pytest.mark.parametrize("n", [5000, 30000, 200000])
def test_levelise_long_chain(ctx, n):
    """A hot-key write chain: every txn depends on its predecessor (depth n; 200000 takes the persistent-wave walk)."""
    import oracle
    from accord_amd.deps import levelise
    er = np.arange(n, dtype=np.uint32)[::-1].copy()      # executeAt order reversed vs index
    off = np.concatenate([[0], np.cumsum([1 if t < n - 1 else 0 for t in range(n)])]).astype(np.uint64)
    dep = np.arange(1, n, dtype=np.uint32)              # t depends on t+1 (earlier executeAt)
    lv, order, nl = levelise(ctx, off, dep, er)
    l2, o2, nl2 = oracle.levelise(off, dep, er)
    np.testing.assert_array_equal(lv, l2)
    np.testing.assert_array_equal(order, o2)
    assert nl == n


def test_levelise_ignores_later_and_equal_executeAt(ctx):
    import canonical
    from accord_amd.deps import levelise
    er = np.array([5, 5, 1, 9], dtype=np.uint32)
    off = np.array([0, 1, 3, 4, 6], dtype=np.uint64)
    dep = np.array([1, 0, 2, 3, 0, 2], dtype=np.uint32)   # equal-executeAt and later-executeAt edges ignored
    lv, order, nl = levelise(ctx, off, dep, er)
    l2, o2 = canonical.levelise(off, dep, er)
    np.testing.assert_array_equal(lv, l2)
    np.testing.assert_array_equal(order, o2)


def test_levelise_rejects_bad_dep(ctx):
    from accord_amd.deps import IllegalArgumentException, levelise
    with pytest.raises(IllegalArgumentException):
        levelise(ctx, np.array([0, 1], np.uint64), np.array([7], np.uint32), np.array([0], np.uint32))


@contextlib.contextmanager
def tier_ctx(ctx, tier="auto", chunk=0):
    """The module context for the default walk, else a context whose acc_opts force the tier / chunk cap."""
    from accord_amd.deps import Context
    if tier == "auto" and not chunk:
        yield ctx
        return
    c = Context(0, lv_tier=tier, lv_chunk=chunk)
    try:
        yield c
    finally:
        c.close()


@pytest.mark.parametrize("n,tier", [(1000, "auto"), (70000, "auto"), (1000, "windowed"), (1000, "waves")])
def test_levelise_rejects_decreasing_offsets(ctx, n, tier):
    """Non-monotone offsets with off[n] == E (every range in bounds on its own, but ranges overlap, so the filtered
    counts sum past E): each tier must fail with IllegalArgumentException before writing its lists."""
    with tier_ctx(ctx, tier) as c:
        check_rejects_decreasing(c, n)


def check_rejects_decreasing(ctx, n):
    from accord_amd.deps import IllegalArgumentException, levelise
    E = 10
    off = np.full(n + 1, E, np.uint64)
    off[0] = 0
    off[2] = 0            # txns 0 and 2 both read dep[0:10]: [0, 10, 0, 10, 10, ...]
    er = np.arange(n, dtype=np.uint32)[::-1].copy()
    dep = np.arange(n - E, n, dtype=np.uint32)   # all of them earlier in executeAt order than txns 0 and 2
    with pytest.raises(IllegalArgumentException):
        levelise(ctx, off, dep, er)
    # the context stays usable: a valid graph right after
    off2, dep2, er2 = random_graph(np.random.RandomState(7), 500, 6)
    import oracle
    lv, order, nl = levelise(ctx, off2, dep2, er2)
    l2, o2, nl2 = oracle.levelise(off2, dep2, er2)
    np.testing.assert_array_equal(lv, l2)
    np.testing.assert_array_equal(order, o2)


def test_merge_then_levelise_device(ctx):
    """Config 5 at reduced size through the bench's device chain: merged deps of every coordinated txn
    (KeyDeps.merge) levelised by executeAt, against the oracle merge + oracle levelise."""
    import torch
    import oracle
    from accord_amd import _lib as L
    from accord_amd import workload as W
    from accord_amd.deps import merge_levelise_device
    n = 3000
    m = W.merge_batch(n_txn=n, replies=8, seed=0xACC00006, n_keys=4000)
    er = W.merge_exec_rank(n, 0xACC00006)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in m.items()}
    er_d = torch.from_numpy(er).to(dev)
    level = torch.empty(n, dtype=torch.int32, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    mi = L.MergeIn(L.ACC_MEM_DEVICE, n, len(m["key_off"]) - 1,
                   *(t[k].data_ptr() for k in ("grp_off", "key_off", "key_code", "val_off", "txn_rank", "k2v_off",
                                               "k2v")))
    view, nl = merge_levelise_device(ctx, mi, er_d.data_ptr(), level.data_ptr(), order.data_ptr())
    ctx.sync()
    ref = oracle.keydeps_merge(m)
    assert int(view.total_vals) == len(ref["txn_rank"])
    l2, o2, nl2 = oracle.levelise(ref["val_off"], ref["txn_rank"], er)
    np.testing.assert_array_equal(level.cpu().numpy().view(np.uint32), l2)
    np.testing.assert_array_equal(order.cpu().numpy().view(np.uint32), o2)
    assert nl == nl2 and nl > 1


def test_levelise_one_million(ctx):
    """1M txns, deps mostly on recent txns in executeAt order (a hot-key write chain runs through them), plus random
    far deps and deps executing later (ignored): the windowed walk (pending-set walk, about 1M levels) against the
    oracle."""
    import oracle
    from accord_amd.deps import levelise
    rng = np.random.RandomState(2024)
    n, k = 1_000_000, 6
    er = rng.permutation(n).astype(np.uint32)
    pos = np.argsort(er).astype(np.int64)             # txn at executeAt position p
    src = np.repeat(np.arange(n, dtype=np.int64), k)
    p = er[src].astype(np.int64)
    back = np.minimum(p, rng.randint(1, 3000, size=n * k))
    near = pos[np.maximum(p - back, 0)]
    far = rng.randint(0, n, size=n * k)
    d = np.where(rng.rand(n * k) < 0.9, near, far)
    chain = pos[np.maximum(p[::k] - 1, 0)]            # each txn also depends on its exec predecessor: depth ~n/k... ~n
    allsrc = np.concatenate([src, np.arange(n)])
    alld = np.concatenate([d, chain])
    o = np.lexsort((alld, allsrc))
    allsrc, alld = allsrc[o], alld[o]
    keep = np.ones(len(alld), bool)
    keep[1:] = (allsrc[1:] != allsrc[:-1]) | (alld[1:] != alld[:-1])
    allsrc, alld = allsrc[keep], alld[keep]
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(np.bincount(allsrc, minlength=n), out=off[1:])
    lv, order, nl = levelise(ctx, off, alld.astype(np.uint32), er)
    assert ctx.stats().get("levelise.lds_tier") == 2
    l2, o2, nl2 = oracle.levelise(off, alld.astype(np.uint32), er)
    np.testing.assert_array_equal(lv, l2)
    np.testing.assert_array_equal(order, o2)
    assert nl == nl2 and nl > 1000


@pytest.mark.parametrize("tier,chunk,n,max_deps,stat", [
    ("auto", 0, 2000, 300, 1),             # LDS walk (default below 4,096 txns), default chunks
    ("auto", 64, 2000, 300, 1),            # LDS walk, 64-entry chunks: long lists read from HBM
    ("lds", 256, 20000, 12, 1),            # many rounds, rounds of > 2048 positions
    ("lds", 0, 65535, 6, 1),               # largest LDS-walk graph (u16 levels and positions)
    ("auto", 0, 20000, 12, 1),             # the LDS walk up to 65,535 txns
    ("auto", 0, 65536, 6, 2),              # beyond the LDS tiers: one launch per window
    ("windowed", 0, 2000, 300, 2),         # windowed walk, pending-set walk: two windows
    ("windowed", 0, 5000, 30, 2),          # far deps gathered for windows 2..4
    ("windowed", 0, 1024, 40, 2),          # exactly one window
    ("windowed", 0, 3073, 900, 2),         # a partial last window, long lists
    ("waves", 0, 5000, 30, 0),             # the persistent-wave walk at a size the LDS tier takes
    ("waves", 0, 65536, 6, 0),             # the persistent-wave walk beyond it
])
def test_levelise_tiers(ctx, tier, chunk, n, max_deps, stat):
    import oracle
    from accord_amd.deps import levelise
    off, dep, er = random_graph(np.random.RandomState(n + max_deps), n, max_deps)
    with tier_ctx(ctx, tier, chunk) as c:
        lv, order, nl = levelise(c, off, dep, er)
        assert c.stats().get("levelise.lds_tier") == stat
    l2, o2, nl2 = oracle.levelise(off, dep, er)
    np.testing.assert_array_equal(lv, l2)
    np.testing.assert_array_equal(order, o2)
    assert nl == nl2


@pytest.mark.parametrize("walk", ["windowed", "lds", "waves"])
def test_levelise_config5_graph_both_tiers(ctx, walk):
    """A config-5-shaped merged graph (16,384 txns, deps on recent txns, hundreds of levels) through the windowed walk,
    the LDS walk and the persistent-wave walk: identical levels and order, equal to the oracle."""
    import oracle
    from accord_amd.deps import levelise
    rng = np.random.RandomState(55)
    n = 16384
    er = rng.permutation(n).astype(np.uint32)
    pos = np.argsort(er)
    deps = []
    for t in range(n):
        k = int(er[t])
        lo = max(0, k - 400)
        cand = pos[lo:k]
        deps.append(np.sort(rng.choice(cand, size=min(len(cand), rng.randint(0, 120)), replace=False)) if len(cand) else
                    np.zeros(0, np.int64))
    off = np.concatenate([[0], np.cumsum([len(d) for d in deps])]).astype(np.uint64)
    dep = np.concatenate(deps).astype(np.uint32)
    with tier_ctx(ctx, walk) as c:
        lv, order, nl = levelise(c, off, dep, er)
        assert c.stats().get("levelise.lds_tier") == {"windowed": 2, "lds": 1, "waves": 0}[walk]
    l2, o2, nl2 = oracle.levelise(off, dep, er)
    np.testing.assert_array_equal(lv, l2)
    np.testing.assert_array_equal(order, o2)
    assert nl == nl2 and nl > 100


def test_levelise_dense_prefix_chain(ctx):
    """Every txn depends on all earlier txns by executeAt (depth n, lists up to n - 1 entries spanning chunks)."""
    import oracle
    from accord_amd.deps import levelise
    n = 700
    er = np.random.RandomState(7).permutation(n).astype(np.uint32)
    pos = np.argsort(er)
    deps = [np.sort(pos[:er[t]]) for t in range(n)]
    off = np.concatenate([[0], np.cumsum([len(d) for d in deps])]).astype(np.uint64)
    dep = np.concatenate(deps).astype(np.uint32)
    lv, order, nl = levelise(ctx, off, dep, er)
    l2, o2, nl2 = oracle.levelise(off, dep, er)
    np.testing.assert_array_equal(lv, l2)
    np.testing.assert_array_equal(order, o2)
    assert nl == n
