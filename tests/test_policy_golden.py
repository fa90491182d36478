"""Golden vectors for the reference policy, in both the Python spec and
the native engine, plus the documented quirks Q2-Q5."""
import pytest

from yoda_scheduler_amd.models.labels import parse_gpu_request
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.models.scv import Card, Scv, ScvStatus
from yoda_scheduler_amd.ops.native import core, pod_req, push_scv
from yoda_scheduler_amd.plugins import yoda_policy as P
from yoda_scheduler_amd.utils.gonum import U64, atoi, str_to_uint, uint64_to_int64


def scv(name, cards):
    st = ScvStatus(card_list=cards)
    st.recompute_sums()
    return Scv(name=name, status=st)


def node_a():
    return scv("a", [Card(id=i, bandwidth=384, clock=5705, core=3840, power=250, free_memory=12000,
                          total_memory=12196) for i in range(2)])


def node_b():
    return scv("b", [Card(id=0, bandwidth=352, clock=5505, core=3584, power=250, free_memory=5000,
                          total_memory=11178)])


def view(s: Scv) -> P.NodeView:
    st = s.status
    return P.NodeView(s.name, st.card_list, st.card_number, st.free_memory_sum, st.total_memory_sum)


def engine_with(scvs, compat):
    e = core().Engine(compat, 1)
    for s in scvs:
        i = e.upsert_node(s.name)
        e.set_node_meta(i, False, [], [], 10**6, 10**15, 1000)
        push_scv(e, i, s, compat)
    return e


def pod(labels, name="p"):
    return PodInfo.from_obj({"metadata": {"name": name, "uid": name, "labels": labels}, "spec": {}})


@pytest.mark.parametrize("compat", [True, False])
def test_survey_golden_vector(compat):
    req = parse_gpu_request({"scv/memory": "1000"})
    nodes = [view(node_a()), view(node_b())]
    mv = P.collect_max(req, nodes, compat)
    assert (mv.bandwidth, mv.clock, mv.core, mv.free_memory, mv.power, mv.total_memory) == \
        (384, 5705, 3840, 12000, 250, 12196)
    a, b = (P.calculate_score(mv, req, n, compat) for n in nodes)
    if compat:
        # basic 4170 (2085/card incl. the buggy clock term 1485) + actual 196 + alloc 300
        assert P.card_score(mv, node_a().status.card_list[0], True) == 2085
        assert (a, b) == (4666, 2278)
    else:
        # fixed clock term: 5705*100/5705 = 100 → 700/card
        assert P.card_score(mv, node_a().status.card_list[0], False) == 700
        assert (a, b) == (2 * 700 + 196 + 300, 91 + 96 + 93 + 100 + 82 + 91 + 88 + 300)
    assert P.normalize_scores([a, b]) == [100, 0]


@pytest.mark.parametrize("compat", [True, False])
def test_native_matches_golden(compat):
    e = engine_with([node_a(), node_b()], compat)
    pi = pod({"scv/memory": "1000"})
    r = pod_req(e, pi)
    mx = e.collect_max(r, [0, 1])
    assert mx == (384, 5705, 3840, 12000, 250, 12196)
    raw = [e.yoda_raw_score(r, i, mx) for i in (0, 1)]
    req = parse_gpu_request({"scv/memory": "1000"})
    mv = P.collect_max(req, [view(node_a()), view(node_b())], compat)
    assert raw == [P.calculate_score(mv, req, view(s), compat) for s in (node_a(), node_b())]
    assert e.normalize_yoda(raw) == [100, 0]


def test_q3_filter_conjunction_quirk():
    cards = [Card(id=0, clock=5705, free_memory=2000, total_memory=12000),
             Card(id=1, clock=5505, free_memory=12000, total_memory=12000),
             Card(id=2, clock=5705, free_memory=11000, total_memory=12000)]
    n = view(scv("q3", cards))
    req = parse_gpu_request({"scv/number": "2", "scv/memory": "10000", "scv/clock": "5705"})
    assert P.filter_node(req, n, compat=True)[0] is True      # reference: passes (2 mem-fit, 2 clock-fit)
    assert P.filter_node(req, n, compat=False)[0] is False    # fixed: only card 2 satisfies both
    for compat, want in ((True, 0), (False, 11)):
        e = engine_with([scv("q3", cards)], compat)
        assert e.filter_node(pod_req(e, pod(req_labels := {"scv/number": "2", "scv/memory": "10000",
                                                           "scv/clock": "5705"})), 0) == want, req_labels


def test_q4_zero_total_memory_does_not_panic():
    n = view(scv("z", []))
    assert P.actual_score(n, True) == 0 and P.allocate_score(n, True) == 0
    req = parse_gpu_request({"scv/number": "0"})
    assert P.filter_node(req, n, True)[0] is True               # 0 <= CardNumber(0)
    e = engine_with([scv("z", [])], True)
    pi = pod({"scv/number": "0"})
    r = pod_req(e, pi)
    assert e.yoda_raw_score(r, 0, e.collect_max(r, [0])) == 0


def test_q2_clock_term_uses_max_bandwidth_in_compat_only():
    mv = P.MaxValue(bandwidth=100, clock=2400)
    c = Card(clock=2400, bandwidth=100, core=1, power=1, free_memory=1, total_memory=1)
    assert P.card_score(mv, c, True) - P.card_score(mv, c, False) == 2400 * 100 // 100 - 100


def test_normalize_reference_semantics():
    assert P.normalize_scores([0, 0]) == [100, 100]       # highest == lowest → lowest-1
    assert P.normalize_scores([5]) == [100]
    assert P.normalize_scores([10, 20, 30]) == [0, 50, 100]
    assert core().Engine.normalize_yoda([0, 0]) == [100, 100]
    assert core().Engine.normalize_yoda([10, 20, 30]) == [0, 50, 100]


@pytest.mark.parametrize("s,want", [("5", 5), ("+5", 5), ("-1", U64), ("abc", 0), (" 5", 0), ("", 0),
                                    ("99999999999999999999", 0), ("9223372036854775807", 2**63 - 1),
                                    ("-9223372036854775808", 2**63), ("1_000", 0), ("0x10", 0)])
def test_go_atoi_label_semantics(s, want):
    assert str_to_uint(s) == want


def test_atoi_and_uint64_to_int64():
    assert atoi("007") == (7, True)
    assert atoi("--1") == (0, False)
    assert uint64_to_int64(2**63) == 0 and uint64_to_int64(2**63 - 1) == 2**63 - 1


def test_q5_invalid_number_label_fits_everywhere():
    req = parse_gpu_request({"scv/number": "abc"})
    assert req.number == 0
    assert P.filter_node(req, view(node_b()), True)[0] is True


def test_sort_less_and_fifo_tiebreak():
    from yoda_scheduler_amd.plugins.yoda import Yoda
    y = Yoda()
    hi, lo, bad = pod({"scv/priority": "10"}, "hi"), pod({"scv/priority": "1"}, "lo"), pod({"scv/priority": "x"}, "b")
    assert P.queue_less(10, 1) and not P.queue_less(1, 10)
    assert y.sort_key(hi) < y.sort_key(lo) < y.sort_key(bad)
