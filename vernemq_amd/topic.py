"""Topic rules of ``vmq_topic`` (apps/vmq_commons/src/vmq_topic.erl) used by
the host side: subscription filters and publish topics must be split into
words exactly as the broker splits them, because the matcher works on the
word lists ('interning contract')."""
from __future__ import annotations

MAX_LEN = 65536  # vmq_topic.erl:45


def validate_topic(kind: str, topic: bytes):
    """vmq_topic:validate_topic/2 (vmq_topic.erl:82-133).

    Returns ``("ok", (word, ...))`` or ``("error", atom)``."""
    if topic == b"":
        return ("error", "no_empty_topic_allowed")                    # :82-83
    if len(topic) > MAX_LEN:
        return ("error", "subscribe_topic_too_long")                  # :84-85
    return _publish(topic) if kind == "publish" else _subscribe(topic)


def _segments(topic: bytes):
    return topic.split(b"/")


def _publish(topic: bytes):
    # validate_publish_topic/3 (:97-112): a level that is exactly '+' (:97-98)
    # or a last level '#' (:99) is a publish error; any other '+' / '#' inside
    # a level is a word error (:106-109).
    segs = _segments(topic)
    words = []
    for i, seg in enumerate(segs):
        if seg == b"+":
            return ("error", "no_+_allowed_in_publish")
        if seg == b"#" and i == len(segs) - 1:
            return ("error", "no_#_allowed_in_publish")
        for c in seg:
            if c == 0x2B:
                return ("error", "no_+_allowed_in_word")
            if c == 0x23:
                return ("error", "no_#_allowed_in_word")
        words.append(seg)
    return ("ok", tuple(words))


def _subscribe(topic: bytes):
    # validate_subscribe_topic/3 (:114-129) + validate_shared_subscription/1 (:131-133)
    segs = _segments(topic)
    words = []
    for i, seg in enumerate(segs):
        last = i == len(segs) - 1
        if seg == b"+":
            words.append(seg)
            continue
        if seg == b"#":
            if last:
                words.append(seg)
                continue
            return ("error", "no_#_allowed_in_word")
        for c in seg:
            if c == 0x2B:
                return ("error", "no_+_allowed_in_word")
            if c == 0x23:
                return ("error", "no_#_allowed_in_word")
        words.append(seg)
    if words and words[0] == b"$share" and len(words) < 3:
        return ("error", "invalid_shared_subscription")
    return ("ok", tuple(words))


def contains_wildcard(words) -> bool:
    """vmq_topic:contains_wildcard/1 (vmq_topic.erl:91-95)."""
    for i, w in enumerate(words):
        if w == b"+":
            return True
        if w == b"#" and i == len(words) - 1:
            return True
    return False


def unword(words) -> bytes:
    """vernemq_dev_api:unword_topic/1 as used by vmq_topic:unword/1 (:79-80)."""
    return b"/".join(words)


def is_dollar(words) -> bool:
    """First word starts with '$' (MQTT-4.7.2-1, vmq_reg_trie.erl:283-288)."""
    return bool(words) and words[0][:1] == b"$"
