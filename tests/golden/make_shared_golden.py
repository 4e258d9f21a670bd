"""Writes tests/golden/shared_dispatch.json: the reference's shared-subscription
dispatch tests, transcribed by hand (their setup as subscriptions + queue
states, their assertions as the allowed receivers per publish).

Sources (reference checkout):
  vmq_publish_SUITE.erl:653-691   shared_subscription_offline
  vmq_publish_SUITE.erl:693-738   shared_subscription_online_first
  vmq_cluster_SUITE.erl:494-528   shared_subs_prefer_local_policy_test
  vmq_cluster_SUITE.erl:530-575   shared_subs_local_only_policy_test (both phases)
  vmq_cluster_SUITE.erl:577-610   shared_subs_random_policy_test
connect_subscribers/3 (:790-806) picks a random node of the list per
subscriber; the fixture fixes one spread.  Its clients use clean_session
true, so a disconnected local subscriber's subscription is gone (local_only
phase 2).  Hand-derived from the source alone (parity unpinned by a test):
  not_found_skipped  vmq_shared_subscriptions.erl:54-60, 75-78
  draining_is_offline :56-58 (draining is collected like offline)

Run: python tests/golden/make_shared_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
L, N2, N3 = "node1@127.0.0.1", "node2@127.0.0.1", "node3@127.0.0.1"


def cluster_subs(filt, n_local, n_remote, remote_nodes=(N2, N3)):
    subs = [["subscriber-%d-node-local" % i, L, filt, 1] for i in range(n_local)]
    subs += [["subscriber-%d-node-%s" % (i, remote_nodes[i % len(remote_nodes)][:5]),
              remote_nodes[i % len(remote_nodes)], filt, 1] for i in range(n_remote)]
    return subs


def scenarios():
    out = []
    out.append({
        "name": "shared_subscription_offline", "source": "vmq_publish_SUITE.erl:653-691", "pinned": True,
        "node": "nonode@nohost", "nodes": ["nonode@nohost"], "policy": "prefer_local",
        "subs": [["single-offline-sha-sub", "nonode@nohost", "$share/singleofflinesub/shared_sub_topic", 1]],
        "states": {"single-offline-sha-sub": "offline"},
        "publisher": "single-offline-pub", "topic": "shared_sub_topic", "n_publishes": 10,
        "expect": {"singleofflinesub": ["single-offline-sha-sub"]}})
    out.append({
        "name": "shared_subscription_online_first", "source": "vmq_publish_SUITE.erl:693-738", "pinned": True,
        "node": "nonode@nohost", "nodes": ["nonode@nohost"], "policy": "prefer_local",
        "subs": [["shared-sub-sub-offline", "nonode@nohost", "$share/group/shared_sub_topic", 1],
                 ["shared-sub-sub-online", "nonode@nohost", "$share/group/shared_sub_topic", 1]],
        "states": {"shared-sub-sub-offline": "offline", "shared-sub-sub-online": "online"},
        "publisher": "shared-sub-pub", "topic": "shared_sub_topic", "n_publishes": 10,
        "expect": {"group": ["shared-sub-sub-online"]}})
    subs = cluster_subs("$share/share/sharedtopic", 5, 5)
    local = [s[0] for s in subs if s[1] == L]
    out.append({
        "name": "shared_subs_prefer_local_policy_test", "source": "vmq_cluster_SUITE.erl:494-528", "pinned": True,
        "node": L, "nodes": [L, N2, N3], "policy": "prefer_local", "subs": subs, "states": {},
        "publisher": "ss-publisher", "topic": "sharedtopic", "n_publishes": 10, "expect": {"share": local}})
    out.append({
        "name": "shared_subs_local_only_policy_test (locals connected)", "source": "vmq_cluster_SUITE.erl:530-560",
        "pinned": True, "node": L, "nodes": [L, N2, N3], "policy": "local_only", "subs": subs, "states": {},
        "publisher": "ss-publisher", "topic": "sharedtopic", "n_publishes": 10, "expect": {"share": local}})
    out.append({
        "name": "shared_subs_local_only_policy_test (locals gone)", "source": "vmq_cluster_SUITE.erl:562-575",
        "pinned": True, "node": L, "nodes": [L, N2, N3], "policy": "local_only",
        "subs": [s for s in subs if s[1] != L], "states": {},
        "publisher": "ss-publisher", "topic": "sharedtopic", "n_publishes": 10, "expect": {"share": None}})
    subs_r = cluster_subs("$share/share/sharedtopic", 4, 6, (N2, N3))
    out.append({
        "name": "shared_subs_random_policy_test", "source": "vmq_cluster_SUITE.erl:577-610", "pinned": True,
        "node": L, "nodes": [L, N2, N3], "policy": "random", "subs": subs_r, "states": {},
        "publisher": "ss-publisher", "topic": "sharedtopic", "n_publishes": 10,
        "expect": {"share": [s[0] for s in subs_r]}})
    out.append({
        "name": "not_found_skipped", "source": "vmq_shared_subscriptions.erl:54-60, 75-78", "pinned": False,
        "node": "nonode@nohost", "nodes": ["nonode@nohost"], "policy": "random",
        "subs": [["gone", "nonode@nohost", "$share/g/a/+", 0], ["off", "nonode@nohost", "$share/g/a/+", 0],
                 ["also-gone", "nonode@nohost", "$share/h/a/#", 0]],
        "states": {"gone": "not_found", "off": "offline", "also-gone": "not_found"},
        "publisher": "p", "topic": "a/b", "n_publishes": 10, "expect": {"g": ["off"], "h": None}})
    out.append({
        "name": "draining_is_offline", "source": "vmq_shared_subscriptions.erl:46-73", "pinned": False,
        "node": "nonode@nohost", "nodes": ["nonode@nohost"], "policy": "prefer_local",
        "subs": [["d1", "nonode@nohost", "$share/g/t", 0], ["d2", "nonode@nohost", "$share/g/t", 0],
                 ["x", "nonode@nohost", "$share/g/+", 0]],
        "states": {"d1": "draining", "d2": "offline", "x": "not_found"},
        "publisher": "p", "topic": "t", "n_publishes": 10, "expect": {"g": ["d1", "d2"]}})
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "shared_dispatch.json"), "w") as f:
        json.dump({"scenarios": scenarios()}, f, indent=1)
        f.write("\n")
