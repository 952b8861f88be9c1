"""A workload of 32-64-level topics (MQTT levels are unlimited,
src/emqx_mqtt_caps.erl:110) for the sharded mode's multi-word order keys:
a 2-word vocabulary per level, filters sharing the pattern of their first 34
levels in groups, so each group ties on key word 0 and is ordered only by the
symbols of levels >= 32."""
import numpy as np


def long_case(seed, n_filters=3000, n_topics=400):
    """32-64-level topics over a 2-word vocabulary per level; filters share
    their first 32+ levels' pattern in groups, so whole groups tie on key
    word 0 and are ordered only by the symbols of levels >= 32"""
    rng = np.random.default_rng(seed)
    heads = []
    for _ in range(6):   # shared patterns of the first 34 levels
        heads.append([b"+" if rng.random() < 0.3 else b"w%d_%d" % (i, rng.integers(2)) for i in range(34)])
    filters = set()
    while len(filters) < n_filters:
        h = heads[rng.integers(len(heads))]
        L = int(rng.integers(34, 65))
        lv = list(h) + [b"+" if rng.random() < 0.4 else b"w%d_%d" % (i, rng.integers(2)) for i in range(34, L)]
        if rng.random() < 0.3:
            lv = lv[: int(rng.integers(30, L))] + [b"#"]
        filters.add(b"/".join(lv))
    filters = sorted(filters)
    topics = []
    for k in range(n_topics):
        L = int(rng.integers(32, 65))
        h = heads[k % len(heads)]
        lv = [w if w != b"+" else b"w%d_%d" % (i, rng.integers(2)) for i, w in enumerate(h)][:L]
        lv += [b"w%d_%d" % (i, rng.integers(2)) for i in range(len(lv), L)]
        if k % 17 == 0:
            lv[0] = b"$SYS"
        topics.append(b"/".join(lv))
    return filters, topics
