"""The oracle (CPU restatement) against the reference's own LoadAware test vectors."""
import numpy as np
import pytest

from koordinator_amd import abi, config, objects
from oracle import oracle as orc
from tests import golden_util as gu

G = gu.load()


@pytest.mark.parametrize("case", G["estimate_pod"], ids=lambda c: c["name"])
def test_estimate_pod(case):
    la = config.loadaware_args(estimatedScalingFactors=case.get("scaling"))
    cpu, mem, mask = orc.estimate_pod(la, objects.make_pod(case["pod"]))
    assert [cpu, mem] == case["want"], case["src"]
    assert mask == abi.GS_USAGE_CPU | abi.GS_USAGE_MEMORY


@pytest.mark.parametrize("case", G["estimate_node"], ids=lambda c: c["name"])
def test_estimate_node(case):
    assert list(orc.estimate_node(objects.make_node(case["node"]))) == case["want"], case["src"]


@pytest.mark.parametrize("case", G["filter_expired"] + G["filter_usage"], ids=lambda c: c["name"])
def test_loadaware_filter(case):
    eng, pod = gu.build(case, orc.Oracle)
    assert eng.loadaware_filter(pod, 0) == case["want_fail"], case["src"]


@pytest.mark.parametrize("case", G["score"], ids=lambda c: c["name"])
def test_loadaware_score(case):
    eng, pod = gu.build(case, orc.Oracle)
    assert eng.loadaware_score(pod, 0) == case["want"], case["src"]


@pytest.mark.parametrize("case", [c for c in G["filter_usage"] if c.get("want_msg")], ids=lambda c: c["name"])
def test_loadaware_filter_reason(case):
    """The failure code's reason text (gs_reason_string over the oracle's code) is the wantStatus message of the
    reference test (load_aware_test.go), and Unschedulable."""
    eng, pod = gu.build(case, orc.Oracle)
    _, codes, _ = eng.evaluate(np.array([pod], abi.POD_DTYPE))
    st, msg = abi.reason_string(int(codes[0, 0]))
    assert (st, msg) == (1, case["want_msg"]), case["src"]
