"""``__graft_entry__.lab_parity`` — the golden check that ``smoke()`` runs on the GPU box — on the
CPU engine: it passes on the real rules and FAILS when a rule constant is perturbed
(``MinimumPriceDataQualityService.java:5``, ``PriceCorrelationDataQualityService.java:6``)."""
import pytest

import __graft_entry__ as entry
from net.jgp.labs.sparkdq4ml_amd.dq import services


def test_lab_parity_passes(cpu_session):
    entry.lab_parity(cpu_session, (("fp64", 1e-9),))


@pytest.mark.parametrize("name,value", [("MIN_PRICE", 25), ("CORRELATION_MAX_GUESTS", 11),
                                        ("CORRELATION_MAX_PRICE", 110)])
def test_lab_parity_catches_perturbed_rule(cpu_session, monkeypatch, name, value):
    monkeypatch.setattr(services, name, value)
    with pytest.raises(AssertionError):
        entry.lab_parity(cpu_session, (("fp64", 1e-9),))

