"""emqx_amd — MI355X-native topic-routing engine for EMQ X's publish path.

The hot path (emqx_trie:match/1 with emqx_topic:words/1) runs as HIP kernels
for gfx950 in libtopicmatch.so; this package is the host side over its C-ABI:
`Engine` (emqx_trie's insert / delete / match / lookup, batched, and the
route tables), the reference's Erlang modules mirrored where they add logic
(emqx_topic, emqx_router, emqx_access, emqx_mod_rewrite), the micro-batcher,
the multi-GPU modes and the delta feed.  The Erlang side is erlang/ over the
NIF.
"""
from . import _lib
from .engine import Engine, pack

__all__ = ["Engine", "pack", "build_info"]


def build_info():
    return _lib.load().tm_build_info().decode()
