"""Subscriber-store data model of ``vmq_subscriber`` / ``vmq_subscriber_db``
— the source of the subscription deltas the matcher consumes
(SURVEY.md §3.2).  Host side: these run where the Erlang code runs today
(inside the view's gen_server), and turn a metadata event into the ordered
list of ``{Topic, SubInfo, Node}`` adds and deletes that
``vmq_reg_trie:handle_event/2`` folds over.

Terms: ``subs = [(node, clean_session, [(topic, subinfo), ...]), ...]``
(vmq_subscriber.erl:35-38), topics are tuples of ``bytes``, nodes ``str``.
Node and topic ordering follow Erlang term order, which for ASCII atom text
and lists of binaries is Python's ``str`` / ``tuple-of-bytes`` ordering.
"""
from __future__ import annotations

TOMBSTONE = "$deleted"   # vmq_subscriber_db.erl:27


def new(clean_session: bool, topics=(), node: str = "nonode@nohost"):
    """new/1,2,3 (vmq_subscriber.erl:42-48)."""
    return [(node, clean_session, list(topics))]


def _get_node_subs(node, subs):
    """get_node_subs/2 (:178-182) -> (node_subs, clean_session, present)."""
    for n, c, ns in subs:
        if n == node:
            return list(ns), c, True
    return [], True, False


def _ukeysort(entries):
    """lists:ukeysort(1, L): sort by topic, keep the first of equal keys."""
    out = {}
    for t, si in entries:
        if t not in out:
            out[t] = si
    return sorted(out.items(), key=lambda e: e[0])


def _ukeymerge(a, b):
    """lists:ukeymerge(1, A, B) of two key-sorted lists: on equal keys the
    element of A is kept."""
    keys = {t for t, _ in a}
    return sorted(list(a) + [e for e in b if e[0] not in keys], key=lambda e: e[0])


def add(subs, topics, node: str):
    """add/3 (:60-72) -> (new_subs, changed)."""
    old, clean, present = _get_node_subs(node, subs)
    new_node = _ukeymerge(_ukeysort(topics), old)
    if present:
        return ([(n, c, new_node) if n == node else (n, c, ns) for n, c, ns in subs], old != new_node)
    return (sorted([(node, clean, new_node)] + list(subs), key=lambda e: e[0]), True)


def remove(subs, topics, node: str):
    """remove/3 (:80-95) -> (new_subs, changed)."""
    old, clean, present = _get_node_subs(node, subs)
    if not present:
        return subs, False
    new_node = list(old)
    for t in topics:
        for i, (tt, _) in enumerate(new_node):
            if tt == t:
                del new_node[i]
                break
    return ([(n, c, new_node) if n == node else (n, c, ns) for n, c, ns in subs], old != new_node)


def exists(topic, subs) -> bool:
    """exists/2 (:74-78)."""
    return any(t == topic for _, _, ns in subs for t, _ in ns)


def _list_subtract(a, b):
    """Erlang ``A -- B``: drop the first occurrence of each element of B."""
    a = list(a)
    for x in b:
        try:
            a.remove(x)
        except ValueError:
            pass
    return a


def subtract(s1, s2):
    """subtract/2,3 (:151-169): subscriptions of s1 not in s2, per node."""
    acc = []
    i = j = 0
    while i < len(s1):
        if j < len(s2) and tuple(s1[i]) == tuple(s2[j]):                 # :154-156
            i += 1
            j += 1
            continue
        n1, _, ns1 = s1[i]
        if j < len(s2) and n1 == s2[j][0]:                                # :157-164
            d = _list_subtract(ns1, s2[j][2])
            if d:
                acc.append((n1, d))
            i += 1
            j += 1
            continue
        if j < len(s2) and n1 > s2[j][0]:                                 # :165-166
            j += 1
            continue
        acc.append((n1, list(ns1)))                                       # :167-168
        i += 1
    return acc


def get_changes(old, new=None):
    """get_changes/1 (:50-52) and get_changes/2 (:54-58)."""
    if new is None:
        return [(n, list(ns)) for n, _, ns in old]
    return subtract(old, new), subtract(new, old)


def fold(fun, acc, changes):
    """fold/3 (:184-196) over subs() or changes(): Fun({Topic, SubInfo, Node}, Acc)."""
    for entry in changes:
        node, nsubs = (entry[0], entry[2]) if len(entry) == 3 else entry
        for topic, si in nsubs:
            acc = fun((topic, si, node), acc)
    return acc


def change_node(subs, node, new_node, clean_session):
    """change_node/4 (:97-116)."""
    old_ns, old_clean, _ = _get_node_subs(node, subs)
    existing, new_clean, new_present = _get_node_subs(new_node, subs)
    if new_present and old_clean:
        return [e for e in subs if e[0] != node]
    if new_present:
        merged = _ukeymerge(existing, old_ns)
        rest = [e for e in subs if e[0] != node]
        return [(new_node, clean_session and new_clean, merged) if n == new_node else (n, c, ns)
                for n, c, ns in rest]
    return sorted([(new_node, clean_session, old_ns) if n == node else (n, c, ns) for n, c, ns in subs],
                  key=lambda e: e[0])


def get_nodes(subs):
    """get_nodes/1 (:172-173) — note the reversed fold order."""
    out = []
    for n, _, _ in subs:
        out.insert(0, n)
    return out


def change_node_all(subs, new_node, clean_session):
    """change_node_all/3 (:118-128) -> (subs, changed_nodes)."""
    ch = []
    for n in get_nodes(subs):
        if n == new_node:
            continue
        subs = change_node(subs, n, new_node, clean_session)
        ch.insert(0, n)
    return subs, ch


def check_format(subs, self_node: str = "nonode@nohost"):
    """check_format/1 -> maybe_convert_v0/1,2 (:130-147): the v0 format
    ``[(topic, qos, node), ...]`` is folded into ``new(False)``."""
    if isinstance(subs, tuple) and subs and subs[0] == "v0":
        out = new(False, node=self_node)
        for topic, qos, node in subs[1]:
            out, _ = add(out, [(topic, qos)], node)
        return out
    return subs


def db_event_to_change(event, self_node: str = "nonode@nohost"):
    """The handler fun of vmq_subscriber_db:subscribe_db_events/0
    (vmq_subscriber_db.erl:56-71): ``("updated", sid, old, new)`` /
    ``("deleted", sid, old)`` -> ``("delete", sid, subs)`` |
    ``("update", sid, old, new)`` | ``("ignore",)``."""
    if event[0] == "deleted":
        _, sid, val = event
        if val is None or val == TOMBSTONE:
            return ("ignore",)
        return ("delete", sid, check_format(val, self_node))
    if event[0] == "updated":
        _, sid, old, new_ = event
        if old is None or old == TOMBSTONE:
            return ("update", sid, [], check_format(new_, self_node))
        return ("update", sid, check_format(old, self_node), check_format(new_, self_node))
    return ("ignore",)


def event_ops(event, self_node: str = "nonode@nohost"):
    """handle_event/2 (vmq_reg_trie.erl:240-251): the ordered (op, sid, topic,
    subinfo, node) tuples, op in {"del", "add"}, deletes first."""
    ch = db_event_to_change(event, self_node)
    if ch[0] == "delete":
        _, sid, subs = ch
        return [("del", sid, t, si, n) for n, ns in get_changes(subs) for t, si in ns]
    if ch[0] == "update":
        _, sid, old, new_ = ch
        removed, added = get_changes(old, new_)
        return ([("del", sid, t, si, n) for n, ns in removed for t, si in ns] +
                [("add", sid, t, si, n) for n, ns in added for t, si in ns])
    return []
