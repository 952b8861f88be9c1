"""TEST INFRASTRUCTURE ONLY — an independent, literal pure-Python transcription
of the reference's trie and topic algebra, used to pin the C restatement
(oracle/o1_trie.c) and the HIP path on small cases.  Never imported by the
product package.

Each function mirrors one Erlang function of vus520/emqx @ 3.0-rc.3; mnesia /
ETS set tables become dicts with the same keys:

    ?TRIE       {trie_edge, NodeId, Word} -> #trie{node_id = Child}
    ?TRIE_NODE  NodeId -> #trie_node{edge_count, topic}

Words keep Erlang term identity: the atoms '', '+', '#' are the singletons
EMPTY, PLUS, HASH; binaries are `bytes`; the root node id is ROOT.
"""

class _Atom:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return "'%s'" % self.name


ROOT = _Atom("root")
EMPTY = _Atom("")
PLUS = _Atom("+")
HASH = _Atom("#")


# ---- emqx_topic (src/emqx_topic.erl) ----------------------------------------

def word(w: bytes):
    """word/1 — src/emqx_topic.erl:149-152"""
    if w == b"":
        return EMPTY
    if w == b"+":
        return PLUS
    if w == b"#":
        return HASH
    return w


def words(topic: bytes):
    """words/1 — src/emqx_topic.erl:141-147 (binary:split(T, "/", [global]))"""
    return [word(w) for w in topic.split(b"/")]


def bin_(w):
    """bin/1 — src/emqx_topic.erl:131-134"""
    if w is EMPTY:
        return b""
    if w is PLUS:
        return b"+"
    if w is HASH:
        return b"#"
    return w


def join2(parent, w):
    """join/2 — src/emqx_topic.erl:126-129"""
    if parent is ROOT:
        return bin_(w)
    return bin_(parent) + b"/" + bin_(w)


def triples(topic: bytes):
    """triples/1 — src/emqx_topic.erl:117-124"""
    out, parent = [], ROOT
    for w in words(topic):
        node = join2(parent, w)
        out.append((parent, w, node))
        parent = node
    return out


def wildcard(topic) -> bool:
    """wildcard/1 — src/emqx_topic.erl:41-50"""
    ws = words(topic) if isinstance(topic, bytes) else topic
    return any(w is HASH or w is PLUS for w in ws)


def _weq(a, b):
    return a is b if isinstance(a, _Atom) or isinstance(b, _Atom) else a == b


def match(name, filt) -> bool:
    """match/2 — src/emqx_topic.erl:56-75, clause by clause"""
    if isinstance(name, bytes) and isinstance(filt, bytes):
        if name[:1] == b"$" and filt[:1] in (b"+", b"#"):
            return False
        return match(words(name), words(filt))
    if not name and not filt:                              # match([], [])
        return True
    if name and filt and _weq(name[0], filt[0]):           # match([H|T1], [H|T2])
        return match(name[1:], filt[1:])
    if name and filt and filt[0] is PLUS:                  # match([_H|T1], ['+'|T2])
        return match(name[1:], filt[1:])
    if len(filt) == 1 and filt[0] is HASH:                 # match(_, ['#'])
        return True
    return False


class InvalidTopic(Exception):
    pass


def parse(topic: bytes, options=None):
    """parse/1,2 — src/emqx_topic.erl:180-200"""
    options = dict(options or {})
    if "share" in options and (topic.startswith(b"$queue/") or topic.startswith(b"$share/")):
        raise InvalidTopic(topic)
    if topic.startswith(b"$queue/"):
        options["share"] = b"$queue"
        return parse(topic[len(b"$queue/"):], options)
    if topic.startswith(b"$share/"):
        rest = topic[len(b"$share/"):]
        parts = rest.split(b"/", 1)
        if len(parts) == 1:
            raise InvalidTopic(topic)
        group, inner = parts
        if any(c in group for c in (b"/", b"+", b"#")):
            raise InvalidTopic(topic)
        options["share"] = group
        return inner, options
    return topic, options


# ---- emqx_trie (src/emqx_trie.erl) ------------------------------------------

def _ek(node_id, w):
    wk = ("atom", w.name) if isinstance(w, _Atom) else ("bin", w)
    nk = ("atom", "root") if node_id is ROOT else ("bin", node_id)
    return (nk, wk)


def _nk(node_id):
    return ("atom", "root") if node_id is ROOT else ("bin", node_id)


class Trie:
    def __init__(self, events=None):
        self.trie = {}        # ?TRIE
        self.trie_node = {}   # ?TRIE_NODE: key -> [edge_count, topic or None]
        self.edge_reads = 0   # mnesia:read(?TRIE, ...) calls during match
        # events: a list that records the emqx_trie_node table events a
        # mnesia:subscribe({table, emqx_trie_node, detailed}) subscriber
        # receives, in write order: ("write", "emqx_trie_node", node_id,
        # edge_count, topic) / ("delete", "emqx_trie_node", node_id); node_id
        # is bytes or ROOT (the atom root)
        self.events = events

    def _w(self, key):
        if self.events is not None:
            rec = self.trie_node[key]
            nid = ROOT if key[0] == "atom" else key[1]
            self.events.append(("write", "emqx_trie_node", nid, rec[0], rec[1]))

    def _d(self, key):
        if self.events is not None:
            nid = ROOT if key[0] == "atom" else key[1]
            self.events.append(("delete", "emqx_trie_node", nid))

    # insert/1 — src/emqx_trie.erl:62-73
    def insert(self, topic: bytes):
        rec = self.trie_node.get(_nk(topic))
        if rec is not None and rec[1] == topic:
            return
        if rec is not None and rec[1] is None:
            rec[1] = topic
            self._w(_nk(topic))
            return
        for t in triples(topic):
            self._add_path(t)
        self.trie_node[_nk(topic)] = [0, topic]
        self._w(_nk(topic))

    # add_path/1 — src/emqx_trie.erl:104-117
    def _add_path(self, triple):
        node, w, child = triple
        rec = self.trie_node.get(_nk(node))
        if rec is not None:
            if _ek(node, w) not in self.trie:
                rec[0] += 1
                self._w(_nk(node))
                self.trie[_ek(node, w)] = child
        else:
            self.trie_node[_nk(node)] = [1, None]
            self._w(_nk(node))
            self.trie[_ek(node, w)] = child

    # match/1 — src/emqx_trie.erl:77-79
    def match(self, topic: bytes):
        self.edge_reads = 0
        nodes = self._match_node2(ROOT, words(topic))
        return [r[1] for r in nodes if r[1] is not None]

    # match_node/2 — src/emqx_trie.erl:121-125
    def _match_node2(self, node_id, ws):
        if node_id is ROOT and ws and isinstance(ws[0], bytes) and ws[0][:1] == b"$":
            return self._match_node3(ws[0], ws[1:], [])
        return self._match_node3(node_id, ws, [])

    # match_node/3 — src/emqx_trie.erl:127-136
    def _match_node3(self, node_id, ws, acc):
        if not ws:
            rec = self.trie_node.get(_nk(node_id))
            return ([rec] if rec is not None else []) + self._match_hash(node_id, acc)
        w, rest = ws[0], ws[1:]
        acc = self._match_hash(node_id, acc)
        for warg in (w, PLUS):                        # lists:foldl over [W, '+']
            self.edge_reads += 1
            child = self.trie.get(_ek(node_id, warg))
            if child is not None:
                acc = self._match_node3(child, rest, acc)
        return acc

    # 'match_#'/2 — src/emqx_trie.erl:140-145
    def _match_hash(self, node_id, acc):
        self.edge_reads += 1
        child = self.trie.get(_ek(node_id, HASH))
        if child is not None:
            rec = self.trie_node.get(_nk(child))
            return ([rec] if rec is not None else []) + acc
        return acc

    # lookup/1 — src/emqx_trie.erl:83-84 -> [] or [(edge_count, topic)]
    def lookup(self, node_id: bytes):
        rec = self.trie_node.get(_nk(node_id))
        return [] if rec is None else [(rec[0], rec[1])]

    # delete/1 — src/emqx_trie.erl:88-96
    def delete(self, topic: bytes):
        rec = self.trie_node.get(_nk(topic))
        if rec is None:
            return
        if rec[0] == 0:
            del self.trie_node[_nk(topic)]
            self._d(_nk(topic))
            self._delete_path(list(reversed(triples(topic))))
        else:
            rec[1] = None
            self._w(_nk(topic))

    # delete_path/1 — src/emqx_trie.erl:149-163
    def _delete_path(self, path):
        for node_id, w, _ in path:
            self.trie.pop(_ek(node_id, w), None)
            rec = self.trie_node.get(_nk(node_id))
            if rec is None:
                raise RuntimeError(("node_not_found", node_id))   # mnesia:abort
            if rec[0] == 1 and rec[1] is None:
                del self.trie_node[_nk(node_id)]
                self._d(_nk(node_id))
                continue
            rec[0] -= 1
            self._w(_nk(node_id))
            return


# ---- emqx_router:match_routes/1 (src/emqx_router.erl:116-118) ---------------

def match_routes(trie: Trie, routes: dict, topic: bytes):
    """routes: topic -> list of dests (the emqx_route bag, insertion order)"""
    matched = trie.match(topic)
    out = []
    for to in [topic] + matched:
        out.extend((to, d) for d in routes.get(to, []))
    return out


def _x_term(dest):
    """the X of aggre's {To, X} as an orderable tagged term: a node atom ->
    (0, name), the Group of {Group, Node} -> (1, group); tuple order on
    (tag, bytes) is Erlang term order (atom < binary, then bytewise)"""
    if isinstance(dest, tuple):
        g = dest[0]
        return (1, g.encode() if isinstance(g, str) else bytes(g))
    return (0, dest.encode() if isinstance(dest, str) else bytes(dest))


def _usort(xs):
    """lists:usort/1: sorted in term order, duplicates removed"""
    return sorted(set(xs))


def aggre(routes):
    """emqx_broker:aggre/1 (src/emqx_broker.erl:194-206), clause for clause.
    routes: [(To, Dest)] as match_routes returns them; Dest is a node (bytes /
    str, an atom) or a (Group, Node) tuple.  Result: [(To, (tag, bytes))] with
    _x_term's tagging."""
    if not routes:                                   # aggre([]) -> []
        return []
    if len(routes) == 1:
        to, dest = routes[0]
        if not isinstance(dest, tuple):              # when is_atom(Node) -> [{To, Node}]
            return [(to, _x_term(dest))]
        return [(to, _x_term(dest))]                 # dest = {Group, _Node} -> [{To, Group}]
    acc = []
    for to, dest in routes:                          # lists:foldl(..., [], Routes)
        if not isinstance(dest, tuple):
            acc = [(to, _x_term(dest))] + acc        # [{To, Node} | Acc]
        else:
            acc = _usort([(to, _x_term(dest))] + acc)   # lists:usort([{To, Group} | Acc])
    return acc


class RouteTable:
    """emqx_router's route bag with its trie bookkeeping (TEST ORACLE):
    handle_cast add_route (src/emqx_router.erl:153-163) + add_trie_route/1
    (:226-231), handle_cast del_route (:165-187) + del_trie_route/1
    (:252-260) / del_direct_route/1 (:240-241), get_routes/1 (:89-90)."""

    def __init__(self, events=None):
        # events: a list recording the emqx_trie_node and emqx_route table
        # events (Trie.events; ("write" | "delete_object", "emqx_route",
        # topic, dest)) in the order the transactions write them
        self.events = events
        self.trie = Trie(events)
        self.routes = {}

    def add_route(self, topic: bytes, dest):
        bag = self.routes.get(topic, [])
        if dest in bag:                       # lists:member(Route, get_routes(Topic))
            return
        if wildcard(topic) and not bag:       # mnesia:wread -> [] -> emqx_trie:insert
            self.trie.insert(topic)
        self.routes.setdefault(topic, []).append(dest)
        if self.events is not None:           # mnesia:write(?ROUTE, Route, ...) :231 / :224
            self.events.append(("write", "emqx_route", topic, dest))

    def del_route(self, topic: bytes, dest):
        bag = self.routes.get(topic)
        if not bag or dest not in bag:        # [] -> ok / delete_object of an absent route
            return
        if self.events is not None:           # mnesia:delete_object(?ROUTE, Route, ...) :255 / :257 / :241
            self.events.append(("delete_object", "emqx_route", topic, dest))
        if wildcard(topic) and bag == [dest]:  # [Route] -> delete route and trie path
            self.trie.delete(topic)
        bag.remove(dest)
        if not bag:
            del self.routes[topic]

    def cleanup_routes(self, node):
        """emqx_router_helper:cleanup_routes/1 (src/emqx_router_helper.erl:
        156-160), run on nodedown (:118-124): delete_object of every route
        whose dest is Node or {_, Node} -- routes ONLY, the trie keeps the
        filters (stale filters: match/1 still returns them)"""
        pats = [lambda d: not isinstance(d, tuple) and d == node,      # #route{dest = Node}
                lambda d: isinstance(d, tuple) and d[1] == node]       # #route{dest = {'_', Node}}
        for pat in pats:
            for topic in list(self.routes):
                for dest in [d for d in self.routes[topic] if pat(d)]:
                    self.routes[topic].remove(dest)
                    if self.events is not None:
                        self.events.append(("delete_object", "emqx_route", topic, dest))
                if not self.routes[topic]:
                    del self.routes[topic]

    def get_routes(self, topic: bytes):
        return list(self.routes.get(topic, []))

    def match_routes(self, topic: bytes):
        return match_routes(self.trie, self.routes, topic)

    def match_deliveries(self, topic: bytes):
        """aggre(match_routes(Topic)) — emqx_broker.erl:152"""
        return aggre(self.match_routes(topic))


def rewrite_rule_index(topic: bytes, filters):
    """emqx_mod_rewrite:match_rule/2's rule choice (src/emqx_mod_rewrite.erl:
    52-59): the index of the first rule whose filter match/2 accepts, or None"""
    for i, f in enumerate(filters):
        if match(topic, f):
            return i
    return None
