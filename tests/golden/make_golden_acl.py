"""Generate tests/golden/kat_acl.json — the reference's own ACL known-answer
tests, transcribed BY HAND as data (inputs and expected outputs only) from
vus520/emqx @ 3.0-rc.3 test/emqx_access_SUITE.erl:
    :81-91    the suite's acl.conf rules (set_acl_config_file/1)
    :141-150  check_acl_1 / check_acl_2 (emqx_access_control:check_acl/3 through
              the internal ACL module)
    :353-371  match_rule (emqx_access_rule:match/3 on compiled rules)
    :332-351  compile_rule (word lists / patterns the compiler produces)

JSON terms: who = "all" | ["client", c] | ["user", u] | ["ipaddr", cidr] |
["and"|"or", [who]]; rule = [A, "all"] | [A, who, access, topics];
credentials = {"client_id", "username", "peername": [ip, port]} (absent key =
absent from the Erlang map).
Run:  python tests/golden/make_golden_acl.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

SUITE_RULES = [                                   # :82-89
    ["allow", ["ipaddr", "127.0.0.1"], "subscribe", ["$SYS/#", "#"]],
    ["allow", ["user", "testuser"], "subscribe", ["a/b/c", "d/e/f/#"]],
    ["allow", ["user", "admin"], "pubsub", ["a/b/c", "d/e/f/#"]],
    ["allow", ["client", "testClient"], "subscribe", ["testTopics/testClient"]],
    ["allow", "all", "subscribe", ["clients/%c"]],
    ["allow", "all", "pubsub", ["users/%u/#"]],
    ["deny", "all", "subscribe", ["$SYS/#", "#"]],
    ["deny", "all"],
]

SELF1 = {"client_id": "client1", "username": "testuser"}      # :142
SELF2 = {"client_id": "client2", "username": "xyz"}           # :149
CHECK_ACL = [                                                  # :143-150
    [SELF1, "subscribe", "users/testuser/1", "allow"],
    [SELF1, "subscribe", "clients/client1", "allow"],
    [SELF1, "subscribe", "clients/client1/x/y", "deny"],
    [SELF1, "publish", "users/testuser/1", "allow"],
    [SELF1, "subscribe", "a/b/c", "allow"],
    [SELF2, "subscribe", "a/b/c", "deny"],
]

USER = {"client_id": "testClient", "username": "TestUser", "peername": ["127.0.0.1", 2948]}      # :354
USER2 = {"client_id": "testClient", "username": "TestUser", "peername": ["192.168.0.10", 3028]}  # :355
MATCH_RULE = [                                                 # :357-371
    [USER, "Test/Topic", ["allow", "all"], "allow"],
    [USER, "Test/Topic", ["deny", "all"], "deny"],
    [USER, "Test/Topic", ["allow", ["ipaddr", "127.0.0.1"], "subscribe", ["$SYS/#", "#"]], "allow"],
    [USER2, "Test/Topic", ["allow", ["ipaddr", "192.168.0.1/24"], "subscribe", ["$SYS/#", "#"]], "allow"],
    [USER, "d/e/f/x", ["allow", ["user", "TestUser"], "subscribe", ["a/b/c", "d/e/f/#"]], "allow"],
    [USER, "d/e/f/x", ["allow", ["user", "admin"], "pubsub", ["d/e/f/#"]], "nomatch"],
    [USER, "testTopics/testClient", ["allow", ["client", "testClient"], "publish", ["testTopics/testClient"]],
     "allow"],
    [USER, "clients/testClient", ["allow", "all", "pubsub", ["clients/%c"]], "allow"],
    [{"username": "user2"}, "users/user2/abc/def", ["allow", "all", "subscribe", ["users/%u/#"]], "allow"],
    [USER, "d/e/f", ["deny", "all", "subscribe", ["$SYS/#", "#"]], "deny"],
    [USER, "Topic", ["allow", ["and", [["ipaddr", "127.0.0.1"], ["user", "WrongUser"]]], "publish", "Topic"],
     "nomatch"],
    [USER, "Topic", ["allow", ["and", [["ipaddr", "127.0.0.1"], ["user", "TestUser"]]], "publish", "Topic"],
     "allow"],
    [USER, "Topic", ["allow", ["or", [["ipaddr", "127.0.0.1"], ["user", "WrongUser"]]], "publish", ["Topic"]],
     "allow"],
]

# compile/1 outputs (:332-351): topic filters as word lists ('+' / '#' / '' as
# atoms written "'+'" etc.), patterns as {"pattern": words}
COMPILE_RULE = [
    [["allow", ["user", "testuser"], "subscribe", ["a/b/c", "d/e/f/#"]], [["a", "b", "c"], ["d", "e", "f", "'#'"]]],
    [["allow", ["user", "admin"], "pubsub", ["d/e/f/#"]], [["d", "e", "f", "'#'"]]],
    [["allow", "all", "pubsub", ["clients/%c"]], [{"pattern": ["clients", "%c"]}]],
    [["allow", "all", "subscribe", ["users/%u/#"]], [{"pattern": ["users", "%u", "'#'"]}]],
    [["deny", "all", "subscribe", ["$SYS/#", "#"]], [["$SYS", "'#'"], ["'#'"]]],
]


def main():
    out = {"ref": "test/emqx_access_SUITE.erl:81-150, 332-371", "suite_rules": SUITE_RULES,
           "check_acl": CHECK_ACL, "match_rule": MATCH_RULE, "compile_rule": COMPILE_RULE}
    with open(os.path.join(HERE, "kat_acl.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
