"""The delta feed — the Python mirror of erlang/emqx_trie_gpu_feed.erl, clause
for clause, over the same C entry points the NIF calls.

The reference keeps two mnesia tables that every broker node matches against
(src/emqx_trie.erl:38-48, src/emqx_router.erl:52-59).  The feed keeps the
engine equal to their committed state from their table events
(mnesia:subscribe({table, Tab, detailed})):

  emqx_trie_node  write with topic =/= undefined   -> tm_insert(topic)
                  write with topic = undefined     -> tm_delete(node_id)
                  delete                           -> tm_delete(node_id)
  emqx_route      write                            -> tm_route_write
                  delete_object                    -> tm_route_delete_object
                  delete (whole key)               -> tm_route_delete_object per old object

Trie membership comes from emqx_trie_node events ONLY and routes from
emqx_route events ONLY, so a node-down cleanup
(emqx_router_helper:cleanup_routes/1, src/emqx_router_helper.erl:156-160),
which deletes route objects and never trie nodes, leaves the stale filters in
the engine's trie exactly as it leaves them in the reference's: match/1 keeps
returning them, match_routes/1 finds no routes for them.

Boot subscribes FIRST and snapshots after: every write committed in between
arrives twice (in the snapshot and as an event), and every handler is an
idempotent set operation, so replaying the events queued since the
subscription over the snapshot ends in the committed state.

Event tuples are those oracle/pytrie.py records: ("write", "emqx_trie_node",
node_id, edge_count, topic), ("delete", "emqx_trie_node", node_id),
("write" | "delete_object", "emqx_route", topic, dest), and the whole-key
delete ("delete", "emqx_route", topic, old_dests) with the Old list mnesia's
detailed event carries.
"""
from .emqx_router import _enc, _key
from .engine import Engine


class TrieFeed:
    def __init__(self, engine: Engine):
        self.engine = engine
        self.targets = set()   # dests whose aggre target is registered
        self.pending = False   # a commit is scheduled (?COMMIT_MS timer)

    # init/1: the committed state so far, after the subscription
    def boot(self, trie_nodes, routes):
        """trie_nodes: [(node_id, edge_count, topic)] (ets:tab2list(emqx_trie_node));
        routes: [(topic, dest)] (ets:tab2list(emqx_route))"""
        for node_id, _count, topic in trie_nodes:
            if topic is not None:
                self.engine.insert(topic)
        for topic, dest in routes:
            self._add_route(topic, dest)
        self.engine.commit()

    # add_route/2: the dest's aggre/1 target, then the bag
    def _add_route(self, topic, dest):
        e = _enc(dest)
        if e not in self.targets:
            if isinstance(dest, tuple):      # {Group, Node}
                self.engine.dest_target(e, Engine.TARGET_GROUP, _key(dest[0]))
            else:                            # a node atom
                self.engine.dest_target(e, Engine.TARGET_NODE, _key(dest))
            self.targets.add(e)
        self.engine.route_write(topic, e)

    # handle_info({mnesia_table_event, ...})
    def handle(self, ev):
        op, tab = ev[0], ev[1]
        if tab == "emqx_trie_node":
            if op == "write":
                _, _, node_id, _count, topic = ev
                if topic is not None:
                    self.engine.insert(topic)
                elif isinstance(node_id, bytes):
                    self.engine.delete(node_id)
                else:
                    return           # the root record: no filter
            elif op == "delete" and isinstance(ev[2], bytes):
                self.engine.delete(ev[2])
            else:
                return
        elif tab == "emqx_route":
            _, _, topic, dest = ev
            if op == "write":
                self._add_route(topic, dest)
            elif op == "delete_object":
                self.engine.route_delete_object(topic, _enc(dest))
            elif op == "delete":   # the whole key: every old object (erl:97-99); dest = the Old list
                for d in dest:
                    self.engine.route_delete_object(topic, _enc(d))
            else:
                return
        else:
            return
        self.pending = True

    # handle_info(commit, ...)
    def commit(self):
        if self.pending:
            self.engine.commit()
            self.pending = False
