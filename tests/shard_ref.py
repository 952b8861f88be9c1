"""Test helpers for the sharded mode: the order key of a match computed on
the host from the filter (the branch the reference's
fold took at each level — 'match_#' 0, topic word 1, '+' 2 — and an end mark
1 for a filter ending at the topic's last level), packed 2 bits per symbol
position into key_words u64 words (word j = positions 32j..32j+31, as
kernels.hip key_word), and a host merge used to check the exchange logic on
CPU ranks.  Valid for in-domain topics (no '+' / '#' levels)."""
import numpy as np


def order_key(filt: bytes, topic_levels: int, key_words: int = 1):
    """the key as a tuple of key_words ints (an int when key_words == 1)"""
    syms = []
    ws = filt.split(b"/")
    for w in ws:
        if w == b"#":
            syms.append(0)                 # 'match_#' at this level: symbol 0
            break
        syms.append(2 if w == b"+" else 1)
    else:
        assert len(ws) == topic_levels
        syms.append(1)                     # the node's own filter at the last level
    assert len(syms) <= 32 * key_words
    words = [0] * key_words
    for p, x in enumerate(syms):
        words[p // 32] |= x << (62 - 2 * (p % 32))
    return words[0] if key_words == 1 else tuple(words)


def merge_host(recv_counts, src_base, recv_ids, recv_keys, m, n_shards, key_words=1):
    """reference merge: per topic, all sources' (key, gid) sorted by key
    descending; recv_keys holds key_words planes of the received total"""
    counts = np.asarray(recv_counts, dtype=np.int64).reshape(n_shards, m)
    keys = np.asarray(recv_keys).view(np.uint64).reshape(key_words, -1)
    out = []
    pos = [int(b) for b in src_base]
    for t in range(m):
        items = []
        for s in range(n_shards):
            c = int(counts[s, t])
            for j in range(c):
                k = tuple(int(keys[q, pos[s] + j]) for q in range(key_words))
                items.append((k, int(recv_ids[pos[s] + j]) * n_shards + s))
            pos[s] += c
        items.sort(reverse=True)
        out.append([g for _, g in items])
    return out
