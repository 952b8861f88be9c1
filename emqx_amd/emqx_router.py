"""emqx_router — route table + trie deltas + match_routes/1 (src/emqx_router.erl),
same names and semantics, backed by the MI355X engine: the emqx_route bag
lives in the engine (tm_route_add/del, get_routes), and match_routes/1 runs
on the GPU end to end (trie walk + route expansion, routes.hip).

    add_route(Topic[, Dest])   handle_cast add_route  :148-163, add_trie_route :226-231
    del_route(Topic[, Dest])   handle_cast del_route  :165-187, del_trie_route :252-260
    match_routes(Topic)        :116-118  -> [#route{}]: routes of the literal topic
                               first, then routes of each trie match in trie order
    get_routes / has_routes / topics   :89-90, :107-108, :110-111
    match_deliveries(Topic)    emqx_broker:aggre(match_routes(Topic)) (emqx_broker.erl:152,
                               194-206) -> [{To, Node} | {To, Group}], on the GPU (aggre.hip)

Route = (topic, dest) mirrors #route{topic, dest} (include/emqx.hrl:84-87);
dests are node names or {Group, Node} tuples, passed to the engine as opaque
bytes (the NIF would pass term_to_binary) and decoded back here.
"""
from collections import namedtuple

from .engine import Engine, pack

Route = namedtuple("Route", "topic dest")


def _enc(dest) -> bytes:
    if isinstance(dest, tuple):
        return b"\x01" + b"\x00".join(_enc(x) for x in dest)
    if isinstance(dest, str):
        return b"\x02" + dest.encode()
    return b"\x03" + bytes(dest)


def _key(x) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


class Router:
    def __init__(self, engine: Engine, node=b"emqx@127.0.0.1"):
        self.engine = engine
        self.node = node
        self._dec = {}          # encoded dest -> dest object
        self._topics = {}       # topics with routes (insertion order): mnesia:dirty_all_keys(?ROUTE)

    def _dest(self, dest_id: int):
        return self._dec[self.engine.dest_bytes(dest_id)]

    # get_routes/1 — :89-90
    def get_routes(self, topic: bytes):
        return [Route(topic, self._dest(d)) for d in self.engine.get_routes(topic)]

    def has_routes(self, topic: bytes) -> bool:
        return topic in self._topics

    def topics(self):
        return list(self._topics)

    # handle_cast({add_route, Route}) — :153-163
    def add_route(self, topic: bytes, dest=None):
        dest = self.node if dest is None else dest
        e = _enc(dest)
        if e not in self._dec:
            if isinstance(dest, tuple):      # {Group, Node}: aggre keeps the group
                self.engine.dest_target(e, Engine.TARGET_GROUP, _key(dest[0]))
            else:                            # a node atom
                self.engine.dest_target(e, Engine.TARGET_NODE, _key(dest))
        self._dec[e] = dest
        self.engine.route_add(topic, e)
        self._topics[topic] = True
        return "ok"

    # handle_cast({del_route, Route}) — :165-187 + del_trie_route/1 :252-260
    def del_route(self, topic: bytes, dest=None):
        dest = self.node if dest is None else dest
        self.engine.route_del(topic, _enc(dest))
        if not self.engine.get_routes(topic):
            self._topics.pop(topic, None)
        return "ok"

    # match_routes/1 — :116-118
    def match_routes(self, topic: bytes):
        return self.match_routes_many([topic])[0]

    def match_routes_many(self, topics):
        """batched match_routes/1: one device batch for all topics"""
        topics = list(topics)
        buf, off = pack(topics)
        counts, offs, src, dst = self.engine.match_routes_batch(buf, off)
        names, res = {}, []
        for t, topic in enumerate(topics):
            row = []
            for k in range(int(offs[t]), int(offs[t]) + int(counts[t])):
                s = int(src[k])
                if s == Engine.TOPIC_ROUTE:
                    to = topic
                else:
                    if s not in names:
                        names[s] = self.engine.filter_bytes(s)
                    to = names[s]
                row.append(Route(to, self._dest(int(dst[k]))))
            res.append(row)
        return res

    # emqx_broker:aggre/1 over match_routes/1 — emqx_broker.erl:152, 194-206
    def match_deliveries(self, topic: bytes):
        return self.match_deliveries_many([topic])[0]

    def match_deliveries_many(self, topics, tagged=False):
        """batched aggre(match_routes(T)): [(To, Node) | (To, Group)] per
        topic; tagged=True gives (To, (kind, key bytes)) with kind 0 for a
        node atom and 1 for a group binary (Erlang term order of X)"""
        topics = list(topics)
        buf, off = pack(topics)
        counts, offs, to, tg = self.engine.match_deliveries_batch(buf, off)
        names, tnames, res = {}, {}, []
        for t, topic in enumerate(topics):
            row = []
            for k in range(int(offs[t]), int(offs[t]) + int(counts[t])):
                s = int(to[k])
                if s == Engine.TOPIC_ROUTE:
                    name = topic
                else:
                    if s not in names:
                        names[s] = self.engine.filter_bytes(s)
                    name = names[s]
                g = int(tg[k])
                if g not in tnames:
                    tnames[g] = self.engine.target_bytes(g)
                kind, key = tnames[g]
                row.append((name, (kind, key)) if tagged else (name, key))
            res.append(row)
        return res
