"""GPU: the Maelstrom Deps JSON (Json.DEPS_ADAPTER, accord-maelstrom/.../Json.java:316-398) parsed and written on device
(acc_deps_from_json / acc_deps_to_json): canonical documents round-trip byte for byte, unsorted documents with
duplicates come back as the Builder result, the parsed keys carry Datum.compareTo order (hash first)."""
import numpy as np
import pytest

import json_cases as JC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from accord_amd.deps import Context
    c = Context(0)
    yield c
    c.close()


def test_json_round_trip_canonical(ctx):
    from accord_amd.deps import deps_from_json, deps_to_json
    rng = np.random.default_rng(1)
    docs = [JC.write_deps(*JC.random_doc(rng, canonical=True)) for _ in range(300)]
    docs.append(b'{"keyDeps":[],"rangeDeps":[]}')
    r = deps_from_json(ctx, docs, with_view=True)
    out = deps_to_json(ctx, r["view"])
    assert out == docs


def test_json_builder_semantics(ctx):
    from accord_amd.deps import deps_from_json, deps_to_json
    rng = np.random.default_rng(2)
    raw = [JC.random_doc(rng) for _ in range(200)]
    docs = [JC.write_deps(*x) for x in raw]
    # whitespace, field order and a missing field are accepted like Gson's JsonReader
    docs.append(b' { "rangeDeps" : [ ] , "keyDeps" : [ [ 5 , [ 1 , 65538 , "n2" ] ] , [ 3 , [ 1 , 65538 , null ] ] ] } ')
    raw.append(([((JC.LONG, False, 5), (1, 65538, 2)), ((JC.LONG, False, 3), (1, 65538, 0))], []))
    docs.append(b'{}')
    raw.append(([], []))
    r = deps_from_json(ctx, docs, with_view=True)
    out = deps_to_json(ctx, r["view"])
    for i, (ke, re_) in enumerate(raw):
        assert out[i] == JC.write_deps(*JC.build(ke, re_)), i
    # dictionary = the batch's distinct datums in Datum.compareTo order
    seen = {JC.datum_order(d) for ke, re_ in raw for d, _ in ke} | \
           {JC.datum_order(x) for ke, re_ in raw for (a, b), _ in re_ for x in (a, b)}
    assert len(r["dict_kind"]) == len(seen)
    got = [JC.datum_order((int(k), bool(nl), int(v) - (1 << 64) if int(v) >= 1 << 63 and int(k) == JC.LONG else
                           (int(np.int32(np.uint32(int(v) & 0xFFFFFFFF))) if int(k) == JC.HASH else int(v))))
           for k, nl, v in zip(r["dict_kind"], r["dict_null"], r["dict_value"])]
    assert got == sorted(seen)
    assert [int(h) for h in r["dict_hash"]] == [g[0] for g in got]


def test_json_errors(ctx):
    from accord_amd.deps import IllegalArgumentException, IllegalStateException, deps_from_json
    bad = [b'{"keyDeps":[[1,[1,2,"n1"]]', b'{"keyDeps":[["s",[1,2,"n1"]]]}', b'{"keyDeps":[[1.5,[1,2,"n1"]]]}',
           b'{"keyDeps":[[1,null]]}', b'{"keyDeps":[[1,[1,2,"x1"]]]}']
    for doc in bad:
        with pytest.raises(IllegalArgumentException):
            deps_from_json(ctx, [doc])
    with pytest.raises(IllegalStateException):
        deps_from_json(ctx, [b'{"other":[]}'])
    # the context stays usable
    r = deps_from_json(ctx, [b'{"keyDeps":[[7,[1,2,"n1"]]],"rangeDeps":[]}'])
    assert int(r["key"]["key_off"][-1]) == 1
