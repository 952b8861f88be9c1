"""The NIF shim (emqx_amd/csrc/emqx_trie_nif.c) compiles cleanly (-Wall
-Werror, -fsyntax-only) against a declaration stub of erl_nif.h
(tests/nif_stub/: this image has no Erlang/OTP; the stub is test
infrastructure, never linked or run), and registers every Erlang function
the wrapper module erlang/emqx_trie_nif.erl declares, with the upgrade
callback for hot code loading."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NIF = os.path.join(ROOT, "emqx_amd", "csrc", "emqx_trie_nif.c")


def test_nif_compiles_against_erl_nif_api():
    r = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        "-I", os.path.join(ROOT, "tests", "nif_stub"), NIF], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_nif_table_matches_erlang_wrapper():
    src = open(NIF).read()
    table = set(re.findall(r'\{"(\w+)", (\d), nif_\w+', src))
    erl = open(os.path.join(ROOT, "erlang", "emqx_trie_nif.erl")).read()
    exports = re.search(r"-export\(\[(.*?)\]\)", erl, re.S).group(1)
    declared = set(re.findall(r"(\w+)/(\d)", exports))
    assert table == declared, (table ^ declared)
    assert "ERL_NIF_INIT(emqx_trie_nif, funcs, load, NULL, upgrade, NULL)" in src
