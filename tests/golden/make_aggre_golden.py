"""Generate tests/golden/aggre_vectors.json: route tables (node and $share
dests), publish topics and their aggre(match_routes(T)) lists from the
oracle's clause-by-clause transcription of emqx_broker:aggre/1
(oracle/pytrie.py; src/emqx_broker.erl:194-206).  Bytes are hex strings.

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
        topics = [b"/".join(rng.choice([b"a", b"b", b"", b"$SYS", b"c", b"x"]) for _ in range(rng.randint(1, 5)))
                  for _ in range(40)] + pool[:10]
        want = [[[to.hex(), x[0], x[1].hex()] for to, x in o.match_deliveries(tp)] for tp in topics]
        cases.append({"ops": ops, "topics": [t.hex() for t in topics], "deliveries": want})
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "aggre_vectors.json")
    json.dump({"source": "oracle/pytrie.py aggre(match_routes(T)), src/emqx_broker.erl:194-206",
               "cases": cases}, open(out, "w"))
    print("wrote", out, sum(len(c["topics"]) for c in cases), "topics")


if __name__ == "__main__":
    main()
