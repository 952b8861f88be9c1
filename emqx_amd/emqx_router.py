"""emqx_router — route table + trie deltas + match_routes/1 (src/emqx_router.erl),
same names and semantics, backed by the MI355X engine for the trie part.

    add_route(Topic[, Dest])   handle_cast add_route  :148-163, add_trie_route :226-231
    del_route(Topic[, Dest])   handle_cast del_route  :165-187, del_trie_route :252-260
    match_routes(Topic)        :116-118  -> [#route{}]: routes of the literal topic
                               first, then routes of each trie match in trie order
    get_routes / has_routes / topics   :89-90, :107-108, :110-111

Route = (topic, dest) mirrors #route{topic, dest} (include/emqx.hrl:84-87);
the emqx_route bag keeps insertion order per topic like an ETS bag.
"""
from collections import namedtuple

from . import emqx_topic
from .engine import Engine

Route = namedtuple("Route", "topic dest")


class Router:
    def __init__(self, engine: Engine, node=b"emqx@127.0.0.1"):
        self.engine = engine
        self.node = node
        self.routes = {}   # emqx_route bag: topic -> [dest]

    # get_routes/1 — :89-90
    def get_routes(self, topic: bytes):
        return [Route(topic, d) for d in self.routes.get(topic, [])]

    def has_routes(self, topic: bytes) -> bool:
        return topic in self.routes

    def topics(self):
        return list(self.routes.keys())

    # handle_cast({add_route, Route}) — :153-163
    def add_route(self, topic: bytes, dest=None):
        dest = self.node if dest is None else dest
        bag = self.routes.get(topic, [])
        if dest in bag:
            return "ok"
        if emqx_topic.wildcard(topic):
            # add_trie_route/1 — :226-231: insert into the trie only when the
            # topic had no route yet
            if not bag:
                self.engine.insert(topic)
        self.routes.setdefault(topic, []).append(dest)
        return "ok"

    # handle_cast({del_route, Route}) — :165-187 + del_trie_route/1 :252-260
    def del_route(self, topic: bytes, dest=None):
        dest = self.node if dest is None else dest
        bag = self.routes.get(topic)
        if not bag or dest not in bag:
            return "ok"
        if emqx_topic.wildcard(topic) and bag == [dest]:
            self.engine.delete(topic)   # last route of the filter: remove it from the trie
        bag.remove(dest)
        if not bag:
            del self.routes[topic]
        return "ok"

    # match_routes/1 — :116-118
    def match_routes(self, topic: bytes):
        matched = self.engine.match([topic])[0]
        out = []
        for to in [topic] + matched:
            out.extend(self.get_routes(to))
        return out

    def match_routes_many(self, topics):
        """batched match_routes/1: one device batch for all topics"""
        rows = self.engine.match(list(topics))
        res = []
        for t, matched in zip(topics, rows):
            out = []
            for to in [t] + matched:
                out.extend(self.get_routes(to))
            res.append(out)
        return res
