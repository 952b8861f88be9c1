"""emqx_mod_rewrite on the GPU (src/emqx_mod_rewrite.erl).

match_rule/2 (:52-59) applies the FIRST rule whose filter
emqx_topic:match/2 accepts (binary clause, '$' rule included), then that
rule's regex (match_regx/3, :61-71): on a regex miss the topic stays as it
is, later rules are never tried.  The device (rewrite.hip) picks the rule for
a whole batch of topics; the regex step runs here on the host with Python's
`re` standing in for Erlang's PCRE-based `re` (same syntax for the common
subset: groups, classes, anchors; `$N` in Dest is the N-th capture,
replaced left to right like the reference's foldl of re:replace/4)."""
import ctypes
import re

import numpy as np

from . import _lib as L
from .engine import pack

NO_RULE = L.TM_NO_RULE


def _b(x):
    return x.encode() if isinstance(x, str) else bytes(x)


class Rewrite:
    """rules: [(filter, regex, dest)] in compile/1 order"""

    def __init__(self, rules, device=0):
        self.lib = L.load()
        h = ctypes.c_void_p()
        rc = self.lib.tm_rewrite_open(device, ctypes.byref(h))
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_rewrite_open(device=%d)" % device)
        self.h = h
        self.rules = []
        for f, rx, dest in rules:
            f = _b(f)
            rc = self.lib.tm_rewrite_rule(self.h, f, len(f))
            if rc != L.TM_OK:
                raise L.TopicMatchError(rc, "tm_rewrite_rule")
            self.rules.append((f, re.compile(_b(rx)), _b(dest)))

    def close(self):
        if self.h:
            self.lib.tm_rewrite_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def rule_index_batch(self, buf, off):
        """u32[n]: index of the first rule whose filter matches, NO_RULE if none"""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) - 1
        out = np.zeros(max(n, 1), dtype=np.uint32)
        rc = self.lib.tm_rewrite_match_batch(self.h, buf.ctypes.data, off.ctypes.data, n, out.ctypes.data)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_rewrite_match_batch")
        return out[:n]

    def rule_index_device(self, d_topics, d_off, n, d_out, stream=None):
        def p(x):
            return None if x is None else ctypes.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))
        st = None if stream is None else ctypes.c_void_p(L.stream_handle(stream))
        rc = self.lib.tm_rewrite_match_batch_device(self.h, p(d_topics), p(d_off), n, p(d_out), st)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_rewrite_match_batch_device")

    def rewrite_many(self, topics):
        """match_rule/2 for every topic: the rewritten topic bytes"""
        idx = self.rule_index_batch(*pack(topics))
        out = []
        for t, k in zip(topics, idx):
            t = _b(t)
            out.append(t if k == NO_RULE else match_regx(t, self.rules[k][1], self.rules[k][2]))
        return out


def _erl_replacement(val: bytes, whole: bytes) -> bytes:
    """the Replacement argument of re:replace/4 expanded for a pattern with
    no subexpressions (OTP re docs: '&' inserts the whole match, \\N
    (N starting 1-9) / \\gN / \\g{N} subexpression N -- none exists here, so
    nothing, except \\g0 / \\g{0}: the whole match; \\0 is an escaped '0'
    (re.erl precomp_repl takes a backslash before a byte outside 1-9 as an
    escape) -- and \\& / \\\\ a literal '&' / backslash; a
    backslash before any other byte keeps that byte).  Parity unpinned: the
    reference holds no vector for it (tests/test_rewrite.py works cases by
    hand)."""
    out, i, n = bytearray(), 0, len(val)
    while i < n:
        c = val[i]
        if c == 0x26:                                   # '&'
            out += whole
            i += 1
        elif c == 0x5C and i + 1 < n:                   # backslash
            d = val[i + 1]
            j = i + 1
            if d == 0x67 and i + 2 < n and val[i + 2] == 0x7B:   # \g{N}
                k = val.find(b"}", i + 3)
                if k > i + 3 and val[i + 3:k].isdigit():
                    out += whole if int(val[i + 3:k]) == 0 else b""
                    i = k + 1
                    continue
            if d == 0x67:                               # \gN
                j = i + 2
            elif d == 0x30:                             # \0: an escaped '0' (precomp_repl: X < $1 ; X > $9)
                out.append(d)
                i += 2
                continue
            k = j
            while k < n and 0x30 <= val[k] <= 0x39:
                k += 1
            if k > j:                                   # \N, \gN
                out += whole if int(val[j:k]) == 0 else b""
                i = k
            else:                                       # \& \\ \x -> the byte
                out.append(d)
                i += 2
        else:
            out.append(c)
            i += 1
    return bytes(out)


def match_regx(topic: bytes, mp, dest: bytes) -> bytes:
    """match_regx/3 (src/emqx_mod_rewrite.erl:61-71): for I = 1..n,
    re:replace(Acc, "\\$I", Val_I, [global]) -- every "$I" of Acc (also the
    "$1" inside "$10"), with Val_I's replacement metacharacters expanded"""
    m = mp.search(topic)
    if m is None:
        return topic
    acc = dest
    for i, val in enumerate(m.groups(), start=1):     # foldl over [{"\\$1", V1}, ...]
        var = b"$%d" % i
        acc = acc.replace(var, _erl_replacement(val if val is not None else b"", var))
    return acc
