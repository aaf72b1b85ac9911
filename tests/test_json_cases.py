"""CPU: the test-side JSON writer reproduces the reference's byte forms (Datum.write, Json.writeTimestamp, toString(Id))
and Datum.hash; no GPU."""
import json

import json_cases as JC


def test_writer_forms():
    doc = JC.write_deps([((JC.LONG, False, -7), (32768, 327682, 1)), ((JC.HASH, False, -3), (1, 2, 0)),
                         ((JC.HASH, True, 0), (1, 2, -4)), ((JC.LONG, True, 0), ((1 << 64) - 1, 2, 3))],
                        [(((JC.LONG, False, 1), (JC.LONG, False, 9)), (1, 2, 5))])
    assert doc == (b'{"keyDeps":[[-7,[32768,327682,"n1"]],[["HASH",true,-3],[1,2,null]],[["HASH",false],[1,2,"c-4"]],'
                   b'[["LONG"],[-1,2,"n3"]]],"rangeDeps":[[1,9,[1,2,"n5"]]]}')
    json.loads(doc)


def test_datum_hash_and_order():
    # hash(null) = Integer.MAX_VALUE sorts null datums last; a Hash datum's hash is itself
    assert JC.datum_hash(JC.LONG, True, 0) == 0x7FFFFFFF
    assert JC.datum_hash(JC.HASH, False, -5) == -5
    assert JC.datum_order((JC.HASH, False, 0x7FFFFFFF)) < JC.datum_order((JC.HASH, True, 0))
    vals = [JC.datum_hash(JC.LONG, False, v) for v in range(1000)]
    assert len(set(vals)) == 1000 and sorted(vals) != vals   # hash order, not value order
