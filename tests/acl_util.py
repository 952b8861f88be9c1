"""Helpers shared by the ACL tests: JSON KAT terms -> oracle terms / the
Python mirror's terms, and random rule sets for the GPU comparison."""
import ipaddress
import random


def who_term(w):
    if w == "all":
        return "all"
    kind, arg = w
    if kind in ("and", "or"):
        return (kind, [who_term(c) for c in arg])
    return (kind, arg)


def rule_term(r):
    if len(r) == 2:
        return (r[0], "all")
    a, w, acc, topics = r
    if isinstance(topics, list):
        topics = [tuple(t) if isinstance(t, list) else t for t in topics]
    return (a, who_term(w), acc, topics)


def oracle_cred(c):
    out = {}
    for k in ("client_id", "username"):
        if k in c:
            out[k] = None if c[k] is None else c[k].encode()
    if "peername" in c:
        p = c["peername"]
        out["peername"] = None if p is None else (ipaddress.ip_address(p[0]).packed, p[1])
    return out


def random_rules(rng: random.Random, k: int):
    words = ["a", "b", "", "+", "#", "%c", "%u", "$SYS", "c"]
    users = ["u1", "u2", "+", ""]
    clients = ["c1", "c2", "+"]

    def who(depth=0):
        x = rng.random()
        if x < 0.3:
            return "all"
        if x < 0.45:
            return ("client", rng.choice(clients + ["all"]))
        if x < 0.6:
            return ("user", rng.choice(users + ["all"]))
        if x < 0.75:
            return ("ipaddr", rng.choice(["10.0.0.1", "10.0.0.0/8", "192.168.1.0/24", "::1", "fe80::/10"]))
        if depth < 2:
            return (rng.choice(["and", "or"]), [who(depth + 1) for _ in range(rng.randint(0, 3))])
        return "all"

    def topic():
        t = "/".join(rng.choice(words) for _ in range(rng.randint(1, 4)))
        return ("eq", t) if rng.random() < 0.15 else t
    rules = []
    for _ in range(k):
        if rng.random() < 0.05:
            rules.append((rng.choice(["allow", "deny"]), "all"))
        else:
            rules.append((rng.choice(["allow", "deny"]), who(), rng.choice(["publish", "subscribe", "pubsub"]),
                          [topic() for _ in range(rng.randint(1, 3))]))
    return rules


def random_checks(rng: random.Random, n: int):
    words = ["a", "b", "", "+", "#", "%c", "%u", "$SYS", "c", "c1", "u1", "x"]
    out = []
    for _ in range(n):
        cred = {}
        if rng.random() < 0.9:
            cred["client_id"] = rng.choice(["c1", "c2", "+", "", "x"]) if rng.random() < 0.9 else None
        if rng.random() < 0.9:
            cred["username"] = rng.choice(["u1", "u2", "+", "", "a"]) if rng.random() < 0.9 else None
        if rng.random() < 0.7:
            cred["peername"] = (rng.choice(["10.1.2.3", "192.168.1.7", "192.168.2.7", "::1", "fe80::5", "127.0.0.1"]),
                                1883) if rng.random() < 0.9 else None
        topic = "/".join(rng.choice(words) for _ in range(rng.randint(1, 5)))
        out.append((cred, rng.choice(["publish", "subscribe"]), topic))
    return out
