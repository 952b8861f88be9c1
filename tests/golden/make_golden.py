"""Generate the golden fixtures under tests/golden/.

Two kinds of vectors:

1. kat_*.json — the reference's own known-answer tests, transcribed BY HAND as
   data (inputs and expected outputs only) from vus520/emqx @ 3.0-rc.3:
     test/emqx_trie_SUITE.erl:45-130     (insert / match order / delete / lookup)
     test/emqx_topic_SUITE.erl:46-211    (match/2, words, triples, join, validate, parse, wildcard)
     test/emqx_router_SUITE.erl:70-122   (match_routes)
     test/emqx_client_SUITE.erl:28-32,190-297 (Paho wildcard sets, '$' topics)
     test/emqx_access_SUITE.erl:360-371  (ACL matching through emqx_topic:match/2)
   The reference cannot run here (no Erlang runtime), so these are pinned as
   written in the suites.

2. o1_vectors.json — ordered match lists and per-topic edge-read counts E
   produced by the C restatement O1 (oracle/o1_trie.c) for randomized small
   tries and hand-built edge cases, each vector cross-checked at generation
   time against the independent pure-Python transcription (oracle/pytrie.py)
   for order and E, and against brute-force emqx_topic:match/2 (O2) for the
   set.

Byte strings are stored as latin-1 decoded JSON strings (1:1 with bytes).
Run:  python tests/golden/make_golden.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import O1, o2_topic_match   # noqa: E402
from oracle import pytrie               # noqa: E402

L1 = "latin-1"


def s(b):
    return b.decode(L1)


# ---------------------------------------------------------------- KATs ------

KAT_TRIE = [
    {"name": "t_insert", "ref": "test/emqx_trie_SUITE.erl:45-58",
     "ops": [["insert", "sensor/1/metric/2"], ["insert", "sensor/+/#"], ["insert", "sensor/#"],
             ["insert", "sensor"], ["insert", "sensor"]],
     "checks": [["lookup", "sensor", [[3, "sensor"]]]]},
    {"name": "t_match", "ref": "test/emqx_trie_SUITE.erl:60-68",
     "ops": [["insert", "sensor/1/metric/2"], ["insert", "sensor/+/#"], ["insert", "sensor/#"]],
     "checks": [["match", "sensor/1", ["sensor/+/#", "sensor/#"]]]},
    {"name": "t_match2", "ref": "test/emqx_trie_SUITE.erl:70-79",
     "ops": [["insert", "#"], ["insert", "+/#"], ["insert", "+/+/#"]],
     "checks": [["match", "a/b/c", ["+/+/#", "+/#", "#"]], ["match", "$SYS/broker/zenmq", []]]},
    {"name": "t_match3", "ref": "test/emqx_trie_SUITE.erl:81-87",
     "ops": [["insert", t] for t in ["d/#", "a/b/c", "a/b/+", "a/#", "#", "$SYS/#"]],
     "checks": [["match_len", "a/b/c", 4], ["match", "$SYS/a/b/c", ["$SYS/#"]]]},
    {"name": "t_delete", "ref": "test/emqx_trie_SUITE.erl:89-103",
     "ops": [["insert", "sensor/1/#"], ["insert", "sensor/1/metric/2"], ["insert", "sensor/1/metric/3"],
             ["delete", "sensor/1/metric/2"], ["delete", "sensor/1/metric"], ["delete", "sensor/1/metric"]],
     "checks": [["lookup", "sensor/1", [[2, None]]]]},
    {"name": "t_delete2", "ref": "test/emqx_trie_SUITE.erl:105-117",
     "ops": [["insert", "sensor"], ["insert", "sensor/1/metric/2"], ["insert", "sensor/1/metric/3"],
             ["delete", "sensor"], ["delete", "sensor/1/metric/2"], ["delete", "sensor/1/metric/3"]],
     "checks": [["lookup", "sensor", []], ["lookup", "sensor/1", []]]},
    {"name": "t_delete3", "ref": "test/emqx_trie_SUITE.erl:119-130",
     "ops": [["insert", "sensor/+"], ["insert", "sensor/+/metric/2"], ["insert", "sensor/+/metric/3"],
             ["delete", "sensor/+/metric/2"], ["delete", "sensor/+/metric/3"], ["delete", "sensor"],
             ["delete", "sensor/+"], ["delete", "sensor/+/unknown"]],
     "checks": [["lookup", "sensor", []], ["lookup", "sensor/+", []]]},
]

# emqx_topic:match/2 truths: [name, filter, expected]
KAT_TOPIC_MATCH = [
    # t_match :52-65
    ["a/b/c", "a/b/+", True], ["a/b/c", "a/#", True], ["abcd/ef/g", "#", True], ["abc/de/f", "abc/de/f", True],
    ["abc", "+", True], ["a/b/c", "a/b/c", True], ["a/b/c", "a/c/d", False], ["$share/x/y", "+", False],
    ["$share/x/y", "+/x/y", False], ["$share/x/y", "#", False], ["$share/x/y", "+/+/#", False],
    ["house/1/sensor/0", "house/+", False], ["house", "house/+", False],
    # t_match2 :67-84
    ["sport/tennis/player1", "sport/tennis/player1/#", True],
    ["sport/tennis/player1/ranking", "sport/tennis/player1/#", True],
    ["sport/tennis/player1/score/wimbledon", "sport/tennis/player1/#", True],
    ["sport", "sport/#", True], ["sport", "#", True], ["/sport/football/score/1", "#", True],
    ["Topic/C", "+/+", True], ["TopicA/B", "+/+", True], ["TopicA/C", "+/+", True], ["abc", "+", True],
    ["a/b/c", "a/b/c", True], ["a/b/c", "a/c/d", False], ["$share/x/y", "+", False],
    ["$share/x/y", "+/x/y", False], ["$share/x/y", "#", False], ["$share/x/y", "+/+/#", False],
    ["house/1/sensor/0", "house/+", False],
    # t_match3 :86-92
    ["device/60019423a83c/fw", "device/60019423a83c/#", True],
    ["device/60019423a83c/$fw", "device/60019423a83c/#", True],
    ["device/60019423a83c/$fw/fw", "device/60019423a83c/$fw/#", True],
    ["device/60019423a83c/fw/checksum", "device/60019423a83c/#", True],
    ["device/60019423a83c/$fw/checksum", "device/60019423a83c/#", True],
    ["device/60019423a83c/dust/type", "device/60019423a83c/#", True],
    # t_sigle_level_match :94-103
    ["sport/tennis/player1", "sport/tennis/+", True], ["sport/tennis/player1/ranking", "sport/tennis/+", False],
    ["sport", "sport/+", False], ["sport/", "sport/+", True], ["/finance", "+/+", True], ["/finance", "/+", True],
    ["/finance", "+", False], ["/devices/$dev1", "/devices/+", True],
    ["/devices/$dev1/online", "/devices/+/online", True],
    # t_sys_match :105-109
    ["$SYS/broker/clients/testclient", "$SYS/#", True], ["$SYS/broker", "$SYS/+", True],
    ["$SYS/broker", "+/+", False], ["$SYS/broker", "#", False],
    # 't_#_match' :111-116
    ["a/b/c", "#", True], ["a/b/c", "+/#", True], ["$SYS/brokers", "#", False], ["a/b/$c", "a/b/#", True],
    ["a/b/$c", "a/#", True],
    # t_match_perf :118-122
    ["a/b/ccc", "a/#", True],
    ["/abkc/19383/192939/akakdkkdkak/xxxyyuya/akakak", "/abkc/19383/+/akakdkkdkak/#", True],
    # emqx_client_SUITE dollar_topics_test :285-297: "$TopicA/B" is not delivered to "+/+"
    ["$TopicA/B", "+/+", False],
    # emqx_access_SUITE match_rule :369: d/e/f/x matches d/e/f/#
    ["d/e/f/x", "d/e/f/#", True],
]

KAT_TOPIC = {
    "ref": "test/emqx_topic_SUITE.erl",
    "match": KAT_TOPIC_MATCH,
    # t_wildcard :46-50
    "wildcard": [["a/b/#", True], ["a/+/#", True], ["", False], ["a/b/c", False]],
    # t_words :158-170 (atoms written as {"atom": ...})
    "words": [["/a/+/#", [{"atom": ""}, "a", {"atom": "+"}, {"atom": "#"}]],
              ["/abkc/19383/+/akakdkkdkak/#", [{"atom": ""}, "abkc", "19383", {"atom": "+"}, "akakdkkdkak",
                                               {"atom": "#"}]]],
    # t_triples :146-150 (parent None = atom root)
    "triples": [["a/b/c", [[None, "a", "a"], ["a", "b", "a/b"], ["a/b", "c", "a/b/c"]]]],
    # t_levels :156
    "levels": [["a/b/c/d", 4]],
    # t_join :180-187 (input word lists)
    "join": [[[], ""], [["x"], "x"], [[{"atom": "#"}], "#"],
             [[{"atom": "+"}, {"atom": ""}, {"atom": "#"}], "+//#"],
             [["x", "y", "z", {"atom": "+"}], "x/y/z/+"]],
    "join_words_roundtrip": ["/ab/cd/ef/", "ab/+/#"],
    # t_validate :128-141, t_sigle_level_validate :143-147: true or an error
    "validate": [[["name", "abc/de/f"], True], [["filter", "abc/+/f"], True], [["filter", "abc/#"], True],
                 [["filter", "x"], True], [["name", "x//y"], True], [["filter", "sport/tennis/#"], True],
                 [["name", ""], "error"], [["name", "abc/#"], False], [["filter", "abc/#/1"], "error"],
                 [["filter", "abc/#xzy/+"], "error"], [["filter", "abc/xzy/+9827"], "error"],
                 [["filter", "sport/tennis#"], "error"], [["filter", "sport/tennis/#/ranking"], "error"],
                 [["filter", "+"], True], [["filter", "+/tennis/#"], True],
                 [["filter", "sport/+/player1"], True], [["filter", "sport+"], "error"]],
    "validate_long_name_error": True,   # validate({name, long_topic()}) :133
    # t_parse :203-211
    "parse": [["a/b/+/#", "a/b/+/#", None], ["$queue/topic", "topic", "$queue"],
              ["$share/group/topic", "topic", "group"], ["$local/topic", "$local/topic", None],
              ["$local/$queue/topic", "$local/$queue/topic", None],
              ["$local/$share/group/a/b/c", "$local/$share/group/a/b/c", None],
              ["$fastlane/topic", "$fastlane/topic", None]],
    # t_feed_var :194-197
    "feed_var": [["$c", "clientId", "$queue/client/$c", "$queue/client/clientId"],
                 ["%u", "test", "username/%u/client/x", "username/test/client/x"],
                 ["%c", "clientId", "username/test/client/%c", "username/test/client/clientId"]],
}

KAT_ROUTER = [
    {"name": "match_routes", "ref": "test/emqx_router_SUITE.erl:70-81",
     "add": [["a/b/c", "node"], ["a/+/c", "node"], ["a/b/#", "node"], ["#", "node"]],
     "topic": "a/b/c", "sorted": [["#", "node"], ["a/+/c", "node"], ["a/b/#", "node"], ["a/b/c", "node"]]},
    {"name": "router_add_del", "ref": "test/emqx_router_SUITE.erl:92-122",
     "add": [["#", "node"], ["a/b/c", "node"], ["+/#", "node"]],
     "topic": "a/b/c", "sorted": [["#", "node"], ["+/#", "node"], ["a/b/c", "node"]],
     "then_del": [["a/b/c", "node"]], "sorted_after": [["#", "node"], ["+/#", "node"]],
     "lookup_after": ["a/b/c", []]},
]

# Paho interop sets (test/emqx_client_SUITE.erl:28-32): subscriptions -> publish -> matched filters
KAT_CLIENT = {
    "ref": "test/emqx_client_SUITE.erl",
    "topics": ["TopicA", "TopicA/B", "Topic/C", "TopicA/C", "/TopicA"],
    "wild_topics": ["TopicA/+", "+/C", "#", "/#", "/+", "+/+", "TopicA/#"],
    "cases": [
        # offline_message_queueing_test :190-212: "+/+" receives TopicA/B, Topic/C, TopicA/C
        {"subs": ["+/+"], "pub": "TopicA/B", "set": ["+/+"]},
        {"subs": ["+/+"], "pub": "Topic/C", "set": ["+/+"]},
        {"subs": ["+/+"], "pub": "TopicA/C", "set": ["+/+"]},
        # overlapping_subscriptions_test :214-235
        {"subs": ["TopicA/#", "TopicA/+"], "pub": "TopicA/C", "set": ["TopicA/#", "TopicA/+"]},
        # redelivery_on_reconnect_test :255-270: "TopicA/#" receives TopicA/B and TopicA/C
        {"subs": ["TopicA/#"], "pub": "TopicA/B", "set": ["TopicA/#"]},
        {"subs": ["TopicA/#"], "pub": "TopicA/C", "set": ["TopicA/#"]},
        # dollar_topics_test :285-297
        {"subs": ["+/+"], "pub": "$TopicA/B", "set": []},
    ],
}


# ------------------------------------------------------------ O1 vectors ----

def rand_filters(rng, n, levels, vocab, p_plus, p_hash, sys_frac=0.0, empty_frac=0.0):
    out = set()
    while len(out) < n:
        k = rng.randint(1, levels)
        ws = []
        for i in range(k):
            if i == 0 and rng.random() < sys_frac:
                ws.append("$SYS")
            elif i == k - 1 and rng.random() < p_hash:
                ws.append("#")
            elif rng.random() < p_plus:
                ws.append("+")
            elif rng.random() < empty_frac:
                ws.append("")
            else:
                ws.append("w%d_%d" % (i, rng.randrange(vocab)))
        out.add("/".join(ws))
    return sorted(out)


def rand_topics(rng, n, levels, vocab, sys_frac=0.0, empty_frac=0.0, var_len=False):
    out = []
    for _ in range(n):
        k = rng.randint(1, levels) if var_len else levels
        ws = []
        for i in range(k):
            if i == 0 and rng.random() < sys_frac:
                ws.append("$SYS")
            elif rng.random() < empty_frac:
                ws.append("")
            else:
                ws.append("w%d_%d" % (i, rng.randrange(vocab)))
        out.append("/".join(ws))
    return out


EDGE_FILTERS = ["#", "+", "+/+", "/#", "/+", "+/#", "a//b", "a/+/", "//", "/", "", "$SYS/#", "$SYS/+",
                "$SYS", "$/#", "$", "a/#", "a/+/#", "a/b/#", "a/b", "+/b/#", "$share/g/a/+", "a/$x/#",
                "+/$x", "#/a", "a/#/b", "+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/#",
                "/".join(["l"] * 40), "/".join(["l"] * 40) + "/#", "/".join(["+"] * 33), "ünï/+/#"]
EDGE_TOPICS = ["", "/", "//", "a", "a/", "a//b", "a/b", "a/b/c", "$SYS", "$SYS/x", "$SYS/x/y", "$", "$/a",
               "a/$x", "a/$x/y", "b/$x", "a/+", "a/#", "+", "#", "+/b", "a/#/b", "$share/g/a/b",
               "/".join(["l"] * 40), "/".join(["l"] * 41), "/".join(["q"] * 33), "/".join(["l"] * 31),
               "/".join(["l"] * 32), "ünï/x", "x" * 300 + "/y"]


def vector(name, filters, topics):
    o1 = O1()
    py = pytrie.Trie()
    fb = [f.encode(L1) if not isinstance(f, bytes) else f for f in filters]
    for f in fb:
        o1.insert(f)
        py.insert(f)
    rows = []
    for t in topics:
        tb = t.encode(L1) if not isinstance(t, bytes) else t
        got, e = o1.match(tb, with_edges=True)
        exp = py.match(tb)
        assert got == exp, (name, t, got, exp)
        assert e == py.edge_reads, (name, t, e, py.edge_reads)
        valid_topic = b"+" not in tb.split(b"/") and b"#" not in tb.split(b"/")
        if valid_topic:
            brute = {f for f in set(fb) if o2_topic_match(tb, f)}
            # O2 (emqx_topic:match/2) agrees with the trie on valid inputs
            # except for invalid filters ('#' not last), which match/2 rejects
            # while the trie may still reach them as intermediate '#' nodes
            brute_valid = {f for f in brute if b"#" not in f.split(b"/")[:-1]}
            got_valid = {f for f in got if b"#" not in f.split(b"/")[:-1]}
            assert got_valid == brute_valid, (name, t, got_valid, brute_valid)
        rows.append({"topic": s(tb), "match": [s(x) for x in got], "edge_reads": e})
    o1.close()
    return {"name": name, "filters": [s(f) for f in fb], "topics": rows}


def main():
    with open(os.path.join(HERE, "kat_trie.json"), "w") as f:
        json.dump(KAT_TRIE, f, indent=1)
    with open(os.path.join(HERE, "kat_topic.json"), "w") as f:
        json.dump(KAT_TOPIC, f, indent=1)
    with open(os.path.join(HERE, "kat_router.json"), "w") as f:
        json.dump(KAT_ROUTER, f, indent=1)
    with open(os.path.join(HERE, "kat_client.json"), "w") as f:
        json.dump(KAT_CLIENT, f, indent=1)

    rng = random.Random(0xE3A1)
    vecs = []
    for kat in KAT_TRIE:
        fl = [op[1] for op in kat["ops"] if op[0] == "insert"]
        if any(op[0] == "delete" for op in kat["ops"]):
            continue
        ts = [c[1] for c in kat["checks"] if c[0] in ("match", "match_len")]
        vecs.append(vector("kat_" + kat["name"], fl, ts))
    vecs.append(vector("edge_cases", EDGE_FILTERS, EDGE_TOPICS))
    vecs.append(vector("c1_mini", rand_filters(rng, 400, 5, 6, 0.2, 0.05, sys_frac=0.02),
                       rand_topics(rng, 300, 5, 6, sys_frac=0.05)))
    vecs.append(vector("dense_plus", rand_filters(rng, 300, 6, 3, 0.45, 0.2),
                       rand_topics(rng, 200, 6, 3)))
    vecs.append(vector("ragged", rand_filters(rng, 300, 7, 4, 0.25, 0.15, empty_frac=0.1),
                       rand_topics(rng, 300, 7, 4, empty_frac=0.1, var_len=True)))
    vecs.append(vector("c5_mini", rand_filters(rng, 500, 16, 2, 0.3, 0.25, sys_frac=0.1),
                       rand_topics(rng, 100, 16, 2, sys_frac=0.1)))
    with open(os.path.join(HERE, "o1_vectors.json"), "w") as f:
        json.dump(vecs, f)
    print("wrote", len(vecs), "O1 vector sets;",
          sum(len(v["topics"]) for v in vecs), "topics")


if __name__ == "__main__":
    main()
