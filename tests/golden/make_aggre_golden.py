"""Generate tests/golden/aggre_vectors.json: route tables (node and $share
dests), publish topics and their aggre(match_routes(T)) lists from the
oracle's clause-by-clause transcription of emqx_broker:aggre/1
(oracle/pytrie.py; src/emqx_broker.erl:194-206).  Bytes are hex strings.

These vectors are ORACLE-DERIVED: the reference's suites hold no aggre/1
fixture and the reference (Erlang) cannot run here, so they pin the device
path to the transcription, not to the reference (parity unpinned for the
fold's order-dependent tail and Erlang term order beyond the hand-worked
cases of tests/test_aggre.py).  Publish topics are valid MQTT publish
names; wildcard names (rejected at src/emqx_packet.erl:63) are kept apart
under "ood_topics" / "ood_deliveries".

    python tests/golden/make_aggre_golden.py"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pytrie  # noqa: E402

DESTS = [["node", "n1"], ["node", "n2"], ["node", "g1"], ["group", "g1", "n1"], ["group", "g1", "n2"],
         ["group", "g2", "n2"], ["group", "", "n3"]]


def dest_obj(d):
    return (d[1], d[2]) if d[0] == "group" else d[1]


def main():
    rng = random.Random(2024)
    words = [b"a", b"b", b"", b"+", b"#", b"$SYS", b"c"]
    cases = []
    for c in range(6):
        o = pytrie.RouteTable()
        ops = []
        pool = set()
        while len(pool) < 30:
            ws = [rng.choice(words) for _ in range(rng.randint(1, 4))]
            if b"#" not in ws[:-1]:
                pool.add(b"/".join(ws))
        pool = sorted(pool)
        for _ in range(150):
            t, d = rng.choice(pool), rng.choice(DESTS)
            add = rng.random() < 0.75
            (o.add_route if add else o.del_route)(t, dest_obj(d))
            ops.append(["add" if add else "del", t.hex(), d])
        wild = [p for p in pool if any(w in (b"+", b"#") for w in p.split(b"/"))]
        topics = [b"/".join(rng.choice([b"a", b"b", b"", b"$SYS", b"c", b"x"]) for _ in range(rng.randint(1, 5)))
                  for _ in range(40)] + [p for p in pool if p not in wild][:10]
        ood = wild[:10]

        def dl(ts):
            return [[[to.hex(), x[0], x[1].hex()] for to, x in o.match_deliveries(tp)] for tp in ts]
        cases.append({"ops": ops, "topics": [t.hex() for t in topics], "deliveries": dl(topics),
                      "ood_topics": [t.hex() for t in ood], "ood_deliveries": dl(ood)})
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "aggre_vectors.json")
    json.dump({"source": "ORACLE-DERIVED (parity unpinned: no reference fixture for aggre/1): oracle/pytrie.py "
                         "aggre(match_routes(T)), src/emqx_broker.erl:194-206",
               "cases": cases}, open(out, "w"))
    print("wrote", out, sum(len(c["topics"]) for c in cases), "topics")


if __name__ == "__main__":
    main()
