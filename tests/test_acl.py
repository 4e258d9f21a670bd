"""ACL checks (vmq_acl, include/vmqa.h): the CPU oracle against the
reference's golden vectors (tests/golden/acl.json), the product's host-side
parser/tables against the oracle (no GPU), and — marked gpu — the HIP check
path against the oracle, verdict for verdict."""
import random

import pytest

from oracle import acl_oracle as AO
from tests import scenarios as S

ACL = S.load("acl.json")["scenarios"]


def _w(ws):
    return tuple(w.encode() for w in ws)


def _u(u):
    return None if u is None else u.encode()


class OracleDriver:
    def __init__(self):
        self.o = AO.AclOracle()

    def load(self, lines):
        return self.o.load_from_list([l.encode() for l in lines])

    def tables(self):
        return self.o.dump()

    def check_batch(self, reqs):
        return self.o.check_batch(reqs)

    def auth_on_subscribe(self, user, sid, topics):
        return self.o.auth_on_subscribe(user, sid, topics)

    def auth_on_publish(self, user, sid, topic):
        return self.o.auth_on_publish(user, sid, topic)


class ProductDriver:
    def __init__(self, device=0):
        from vernemq_amd.acl import AclGpu
        self.a = AclGpu(device=device)

    def load(self, lines):
        try:
            self.a.load_from_list([l.encode() for l in lines])
            return True
        except Exception as e:   # the reference's crash: the tables keep what the load did
            from vernemq_amd.acl import AclLoadCrash
            if isinstance(e, AclLoadCrash):
                return False
            raise

    def tables(self):
        return self.a.dump()

    def check_batch(self, reqs):
        return [int(x) for x in self.a.check_batch(reqs)]

    def auth_on_subscribe(self, user, sid, topics):
        return self.a.auth_on_subscribe(user, sid, topics)

    def auth_on_publish(self, user, sid, topic):
        return self.a.auth_on_publish(user, sid, topic)


def run_acl_scenario(scen, drv):
    for i, st in enumerate(scen["steps"]):
        where = "%s step %d" % (scen["name"], i)
        if "load" in st:
            assert drv.load(st["load"]) == st["ok"], where
        elif "tables" in st:
            assert drv.tables() == st["tables"], where
        elif "check" in st:
            ty, t, user, mp, client = st["check"]
            got = drv.check_batch([(ty, _w(t), _u(user), mp, client.encode())])[0]
            assert got == st["expect"], (where, st["check"])
        elif "subscribe" in st:
            user, (mp, client), topics = st["subscribe"]
            got = drv.auth_on_subscribe(_u(user), (mp, client.encode()), [(_w(t), q) for t, q in topics])
            assert got == st["expect"], (where, st["subscribe"])
        else:
            user, (mp, client), t = st["publish"]
            got = drv.auth_on_publish(_u(user), (mp, client.encode()), _w(t))
            assert got == st["expect"], (where, st["publish"])


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("scen", ACL, ids=[s["name"] for s in ACL])
def test_oracle_acl_golden(scen):
    run_acl_scenario(scen, OracleDriver())


def test_pinned_fixture_is_the_eunit_test():
    pinned = [s for s in ACL if s["pinned"]]
    assert [s["name"] for s in pinned] == ["simple_acl"] and len(pinned[0]["steps"]) == 9


def random_acl(seed, n_lines=120):
    """Random ACL text: all/user/pattern rules of every kind, comments, blank
    lines, invalid topics, '+'/'#', %u/%c/%m, several users."""
    rnd = random.Random(seed)
    words = ["a", "b", "c", "", "+", "%u", "%c", "%m", "$SYS"]
    lines = []
    for _ in range(n_lines):
        r = rnd.random()
        if r < 0.05:
            lines.append("# comment\n")
            continue
        if r < 0.08:
            lines.append("\n")
            continue
        if r < 0.18:
            lines.append("user u%d\n" % rnd.randint(0, 4))
            continue
        t = [rnd.choice(words) for _ in range(rnd.randint(1, 4))]
        if rnd.random() < 0.3:
            t.append("#")
        if rnd.random() < 0.03:
            t.insert(0, "#")   # invalid: skipped with a warning
        kind = rnd.choice(["topic read ", "topic write ", "topic ", "pattern read ", "pattern write ", "pattern "])
        lines.append(kind + "/".join(t) + "\n")
    return lines


def random_requests(seed, n=600):
    rnd = random.Random(seed)
    vocab = [b"a", b"b", b"c", b"", b"u1", b"u3", b"c1", b"m1", b"$SYS", b"zz"]
    reqs = []
    for _ in range(n):
        ty = rnd.choice(["read", "write"])
        t = [rnd.choice(vocab) for _ in range(rnd.randint(1, 5))]
        if ty == "read" and rnd.random() < 0.3:   # subscribe filters carry wildcards
            t[rnd.randrange(len(t))] = rnd.choice([b"+", b"#"])
        user = rnd.choice([None, b"u1", b"u3", b"", b"+", b"zz"])
        reqs.append((ty, tuple(t), user, rnd.choice(["", "m1"]), rnd.choice([b"c1", b"a", b"", b"qq"])))
    return reqs


def test_host_tables_match_oracle():
    """The product's host-side parse (vernemq_amd.acl, no GPU) builds the
    oracle's six tables, including reloads and crashing loads."""
    from vernemq_amd.acl import AclGpu
    prod, orc = ProductDriver(device=-1), OracleDriver()
    for seed in range(6):
        lines = random_acl(seed)
        if seed % 3 == 2:
            lines.insert(len(lines) // 2, "garbage\n")
        assert prod.load(lines) == orc.load(lines)
        assert prod.tables() == orc.tables(), seed
    assert isinstance(prod.a, AclGpu)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("scen", ACL, ids=[s["name"] for s in ACL])
def test_acl_golden_on_gpu(scen):
    run_acl_scenario(scen, ProductDriver())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_acl_random_parity(seed):
    prod, orc = ProductDriver(), OracleDriver()
    for k in range(3):   # reloads, one of them crashing half way
        lines = random_acl(seed * 10 + k)
        if k == 1:
            lines.insert(len(lines) // 2, "topic \n" if seed % 2 else "oops\n")
        assert prod.load(lines) == orc.load(lines)
        reqs = random_requests(seed * 10 + k)
        got, want = prod.check_batch(reqs), orc.check_batch(reqs)
        bad = [i for i in range(len(reqs)) if got[i] != want[i]]
        assert not bad, (seed, k, reqs[bad[0]], got[bad[0]], want[bad[0]])


@pytest.mark.gpu
def test_acl_large_tables_skip_lds_staging():
    """All / pattern tables past the 48-KiB LDS budget (the kernel reads them
    from global memory) and a 2,000-rule user: verdicts equal the oracle's."""
    lines = ["topic read r/%d/+/x\n" % k for k in range(3000)] + ["topic write w/%d/#\n" % k for k in range(2000)]
    lines += ["pattern read p/%%c/%d\n" % k for k in range(500)] + ["user big\n"]
    lines += ["topic b/%d/+\n" % k for k in range(2000)]
    prod, orc = ProductDriver(), OracleDriver()
    assert prod.load(lines) and orc.load(lines)
    st = prod.a.stats_raw()
    assert st["rules"] == 3000 + 2000 + 500 + 4000
    rnd = random.Random(3)
    reqs = []
    for _ in range(3000):
        k = rnd.randrange(3500)
        reqs.append(rnd.choice([("read", (b"r", b"%d" % k, b"q", b"x"), None, "", b"c"),
                                ("write", (b"w", b"%d" % k, b"z"), b"big", "", b"c"),
                                ("read", (b"p", b"c%d" % (k % 3), b"%d" % k), None, "", b"c%d" % (k % 2)),
                                ("read", (b"b", b"%d" % k, b"y"), rnd.choice([b"big", b"small"]), "", b"c")]))
    got, want = prod.check_batch(reqs), orc.check_batch(reqs)
    assert got == want and 0 < sum(got) < len(got)
