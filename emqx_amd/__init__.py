"""emqx_amd — MI355X-native topic-routing engine for EMQ X's publish path.

The hot path (emqx_trie:match/1 with emqx_topic:words/1) runs as HIP kernels
for gfx950 in libtopicmatch.so; this package is the host-side mirror of the
reference's Erlang API (emqx_topic, emqx_trie, emqx_router) over its C-ABI.
"""
from . import _lib
from .engine import Engine, pack

__all__ = ["Engine", "pack", "build_info"]


def build_info():
    return _lib.load().tm_build_info().decode()
