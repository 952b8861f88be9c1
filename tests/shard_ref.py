"""Test helpers for the sharded mode: the order key of a match computed on
the host from the filter (the branch the reference's
fold took at each level — 'match_#' 0, topic word 1, '+' 2 — and an end mark
1 for a filter ending at the topic's last level), and a host merge used to
check the exchange logic on CPU ranks.  Valid for in-domain topics (no '+' /
'#' levels) of at most 31 levels."""
import numpy as np


def order_key(filt: bytes, topic_levels: int) -> int:
    key = 0
    ws = filt.split(b"/")
    for i, w in enumerate(ws):
        if w == b"#":
            return key                     # 'match_#' at level i: symbol 0
        key |= (2 if w == b"+" else 1) << (62 - 2 * i)
    assert len(ws) == topic_levels
    return key | (1 << (62 - 2 * len(ws)))   # the node's own filter at the last level


def merge_host(recv_counts, src_base, recv_ids, recv_keys, m, n_shards):
    """reference merge: per topic, all sources' (key, gid) sorted by key descending"""
    counts = np.asarray(recv_counts, dtype=np.int64).reshape(n_shards, m)
    keys = np.asarray(recv_keys).view(np.uint64)
    out = []
    pos = [int(b) for b in src_base]
    for t in range(m):
        items = []
        for s in range(n_shards):
            c = int(counts[s, t])
            for j in range(c):
                items.append((int(keys[pos[s] + j]), int(recv_ids[pos[s] + j]) * n_shards + s))
            pos[s] += c
        items.sort(reverse=True)
        out.append([g for _, g in items])
    return out
