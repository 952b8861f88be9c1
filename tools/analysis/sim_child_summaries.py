"""Estimate (pure Python, host only) of lever 1 in DESIGN §5.2: visits per topic a
per-child subtree summary would prune after an edge-table probe, beyond the
union summary the walk uses now.  Usage: python tools/analysis/sim_child_summaries.py NFILTERS NTOPICS
(C3 distribution; 2M filters / 20K topics: 4.18 of 63.7 visits per topic)."""
import sys, time
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__)))))
from emqx_amd import workload as W
NF = int(sys.argv[1]); NT = int(sys.argv[2])
fb, fo = W.filters(3, n=NF)
filters = W.unpack(fb, fo)
t0 = time.time()
root = {}
# node: dict word->child, plus key '\0e' end flag
for f in filters:
    ws = f.split(b'/')
    v = root
    for w in ws:
        v = v.setdefault(w, {})
    v[None] = True
print("built", time.time() - t0, file=sys.stderr)
# summaries: ends set as bitmask of relative depth (cap 10), hmin
S = {}
def summ(v):
    ends = 1 if None in v else 0
    hmin = 15
    for w, c in v.items():
        if w is None: continue
        e, h = summ(c)
        if w == b'#':
            # '#' child with a filter fires at v (0 below v)
            if None in c: hmin = 0
        sh = ((e << 1) & 0x7FE) | (0x400 if e & 0x600 else 0)
        ends |= sh
        hmin = min(hmin, h + 1 if h < 15 else 15)
    S[id(v)] = (ends, hmin)
    return ends, hmin
sys.setrecursionlimit(100000)
summ(root)
def useful(s, k):
    e, h = s
    bit = (e >> k) & 1 if k < 10 else (e >> 10) & 1
    return bit or h <= k
tb, to = W.topics(3, n=NT)
topics = W.unpack(tb, to)
tot_vis = 0; table_vis = 0; union_prunable = 0; child_prunable = 0
for t in topics:
    ws = t.split(b'/'); n = len(ws)
    stack = [(root, 0)]
    while stack:
        v, r = stack.pop()
        tot_vis += 1
        if r == n: continue
        lits = [(w, c) for w, c in v.items() if w is not None and w not in (b'+', b'#')]
        k = n - r - 1
        c = v.get(ws[r]) if ws[r] not in (b'+', b'#') else None
        if c is not None:
            union = (0, 15)
            for w2, c2 in lits:
                e, h = S[id(c2)]; union = (union[0] | e, min(union[1], h))
            if not useful(union, k):
                union_prunable += 1
            else:
                if len(lits) >= 2:
                    table_vis += 1
                    if not useful(S[id(c)], k):
                        child_prunable += 1
                        c = None
                if c is not None: stack.append((c, r + 1))
        p = v.get(b'+')
        if p is not None and useful(S[id(p)], k): stack.append((p, r + 1))
print(dict(NF=NF, NT=NT, visits_per_topic=tot_vis / NT, table_visits=table_vis / NT, union_pruned=union_prunable / NT, extra_child_pruned=child_prunable / NT))
