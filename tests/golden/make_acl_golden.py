"""Writes tests/golden/acl.json — golden vectors for the file-based ACL
plugin (vmq_acl), hand-transcribed from the reference's OWN tests and data
files (file:line relative to /root/reference).  Data only (inputs + expected
outputs), not reference source.  Re-run with
``python tests/golden/make_acl_golden.py``; the JSON is committed.

* pinned   — the eunit test simple_acl/1 (apps/vmq_acl/src/vmq_acl.erl:303-342):
  the six tables after load_from_list/1 and the auth_on_subscribe /
  auth_on_publish answers it asserts.
* unpinned — behaviour read from vmq_acl.erl:128-238 that no reference test
  asserts, each step citing its lines: the shipped ACL files
  (apps/vmq_acl/priv/test.acl, default.acl) as inputs, reload aging,
  a crashing line, the dropped last byte, %u/%c/%m substitution (undefined
  users), subscribe filters checked with vmq_topic:match/2 (vmq_topic.erl:53-65).

Step kinds: {"load": [lines], "ok": bool} ; {"tables": [dump lines]} ;
{"check": [type, words, user|null, mp, client], "expect": 0|1} ;
{"subscribe": [user|null, [mp, client], [[words, qos], ...]], "expect": "ok"|"next"} ;
{"publish": [user|null, [mp, client], words], "expect": "ok"|"next"}.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def W(s):
    return s.split("/")


def sub(user, mp, client, topics, expect):
    return {"subscribe": [user, [mp, client], [[W(t), 0] for t in topics]], "expect": expect}


def pub(user, mp, client, topic, expect):
    return {"publish": [user, [mp, client], W(topic)], "expect": expect}


def chk(ty, topic, user, mp, client, expect):
    return {"check": [ty, W(topic), user, mp, client], "expect": expect}


SIMPLE_ACL = ["# simple comment\n", "topic read a/b/c\n", "# other comment \n", "topic write a/b/c\n", "\n",
              "# ACL for user 'test'\n", "user test\n", "topic x/y/z/#\n", "# some patterns\n",
              "pattern read %m/%u/%c\n", "pattern write %m/%u/%c\n"]

scenarios = [
    {"name": "simple_acl", "pinned": True, "source": "apps/vmq_acl/src/vmq_acl.erl:303-342",
     "steps": [
         {"load": SIMPLE_ACL, "ok": True},
         {"tables": sorted(["read all [a,b,c]", "write all [a,b,c]", "read user test [x,y,z,#]",
                            "write user test [x,y,z,#]", "read pattern [%m,%u,%c]", "write pattern [%m,%u,%c]"])},
         sub("test", "", "my-client-id", ["a/b/c", "x/y/z/#", "/test/my-client-id"], "ok"),
         sub("invalid-user", "", "my-client-id", ["a/b/c", "x/y/z/#", "/test/my-client-id"], "next"),
         pub("test", "", "my-client-id", "a/b/c", "ok"),
         pub("test", "", "my-client-id", "x/y/z/blabla", "ok"),
         pub("test", "", "my-client-id", "/test/my-client-id", "ok"),
         pub("invalid-user", "", "my-client-id", "x/y/z/blabla", "next"),
         pub("invalid-user", "", "my-client-id", "/test/my-client-id", "next"),
     ]},
    {"name": "priv_test_acl", "pinned": False,
     "source": "apps/vmq_acl/priv/test.acl as input; vmq_acl.erl:146-238 (parse, check, subst)",
     "steps": [
         {"load": ["topic read /test/+/nana\n", "topic write /test/1/nana\n", "\n", "user graf\n", "topic /tmp/all\n",
                   "\n", "pattern read /test/%u/user\n", "pattern write /test/%c/user/%u\n",
                   "pattern write /test/graf/user\n"], "ok": True},
         {"tables": sorted(["read all [,test,+,nana]", "write all [,test,1,nana]", "read user graf [,tmp,all]",
                            "write user graf [,tmp,all]", "read pattern [,test,%u,user]",
                            "write pattern [,test,%c,user,%u]", "write pattern [,test,graf,user]"])},
         chk("read", "/test/7/nana", None, "", "c1", 1),             # all table, '+' (:190-192)
         chk("write", "/test/7/nana", "graf", "", "c1", 0),
         chk("write", "/test/1/nana", None, "", "c1", 1),
         chk("read", "/tmp/all", "graf", "", "c1", 1),                # user table (:194-197)
         chk("read", "/tmp/all", "other", "", "c1", 0),
         chk("read", "/tmp/all", None, "", "c1", 0),                  # undefined user: no user rows
         chk("read", "/test/graf/user", "graf", "", "c1", 1),         # %u (:209-210)
         chk("read", "/test/graf/user", "bob", "", "c1", 0),
         chk("read", "/test/graf/user", None, "", "c1", 0),           # %u with undefined: the atom matches nothing
         chk("write", "/test/c9/user/bob", "bob", "", "c9", 1),       # %c and %u (:209-212)
         chk("write", "/test/c9/user/bob", "bob", "", "c8", 0),
         chk("write", "/test/graf/user", None, "", "x", 1),           # a literal pattern applies to anyone
         chk("read", "/test/+/user", "+", "", "c", 1),                # a '+' user name is a wildcard after subst
         chk("read", "/test/x/user", "+", "", "c", 1),
     ]},
    {"name": "default_acl_allows_all", "pinned": False,
     "source": "apps/vmq_acl/priv/default.acl as input; vmq_topic.erl:59-60 (match(_, [#]))",
     "steps": [
         {"load": ["topic #\n"], "ok": True},
         pub(None, "", "c", "a/b", "ok"),
         pub(None, "", "c", "$SYS/x", "ok"),                        # no MQTT-4.7.2-1 '$' rule in vmq_topic:match
         sub(None, "", "c", ["#", "a/+", "$SYS/#"], "ok"),
         sub(None, "", "c", [], "ok"),                              # auth_on_subscribe(_, _, []) -> ok (:78)
     ]},
    {"name": "reload_ages_entries", "pinned": False, "source": "vmq_acl.erl:128-144, :268-276",
     "steps": [
         {"load": ["topic a/b\n", "user u1\n", "topic u/#\n"], "ok": True},
         chk("read", "a/b", None, "", "c", 1),
         {"load": ["topic c/d\n", "user u1\n", "topic u/#\n"], "ok": True},
         {"tables": sorted(["read all [c,d]", "write all [c,d]", "read user u1 [u,#]", "write user u1 [u,#]"])},
         chk("read", "a/b", None, "", "c", 0),                       # aged out
         chk("write", "u/x", "u1", "", "c", 1),
         # a line no parse_acl_line clause takes crashes the load: aged rows
         # stay (del_aged_entries never runs), rows parsed so far are in
         {"load": ["topic e/f\n", "bogus line\n", "topic g/h\n"], "ok": False},
         {"tables": sorted(["read all [c,d]", "write all [c,d]", "read all [e,f]", "write all [e,f]",
                            "read user u1 [u,#]", "write user u1 [u,#]"])},
         chk("read", "c/d", None, "", "c", 1),
         chk("read", "g/h", None, "", "c", 0),
     ]},
    {"name": "parse_edges", "pinned": False, "source": "vmq_acl.erl:146-177, :219-231 (in/3)",
     "steps": [
         # the last byte is always dropped: no trailing newline eats a character;
         # invalid topics are skipped with a warning; "topic read" needs its space
         {"load": ["topic read x/yz", "topic a/#/b\n", "topic readonly/q\n", "topic write w/+\n",
                   "pattern %m/%c/#\n"], "ok": True},
         {"tables": sorted(["read all [x,y]", "read all [readonly,q]", "write all [readonly,q]",
                            "write all [w,+]", "read pattern [%m,%c,#]", "write pattern [%m,%c,#]"])},
         chk("read", "x/y", None, "", "c", 1),
         chk("read", "x/yz", None, "", "c", 0),
         chk("write", "w/anything", None, "", "c", 1),
         chk("read", "w/anything", None, "", "c", 0),
         chk("write", "m1/c7/x/y", None, "m1", "c7", 1),           # %m -> list_to_binary(MP)
         chk("write", "m1/c7", None, "m1", "c7", 1),               # '#' also matches the parent level
         chk("write", "m2/c7/x", None, "m1", "c7", 0),
         chk("write", "/c7/x", None, "", "c7", 1),                 # MP "" -> an empty word
         # subscribe checks run match/2 on the FILTER: its '+'/'#' words meet
         # the rule's by equality first (vmq_topic.erl:55-56)
         chk("read", "readonly/+", None, "", "c", 0),
         chk("write", "w/+", None, "", "c", 1),
         chk("write", "w/#", None, "", "c", 1),                    # [#] vs [+]: the '+' clause (:57-58)
         chk("write", "w/#/x", None, "", "c", 0),
         # "user \n": the dropped byte leaves User = <<>> (a user named ""); a
         # bare "user " has no byte to drop: badmatch, the load crashes
         {"load": ["user \n", "topic z\n"], "ok": True},
         {"tables": ["read user  [z]", "write user  [z]"]},
         chk("read", "z", "", "", "c", 1),
         chk("read", "z", None, "", "c", 0),
         {"load": ["topic k\n", "user "], "ok": False},
         chk("read", "k", None, "", "c", 1),
     ]},
]

with open(os.path.join(HERE, "acl.json"), "w") as f:
    json.dump({"scenarios": scenarios}, f, indent=1, sort_keys=True)
print("acl.json: %d scenarios" % len(scenarios))
