"""Band layout of the wide Gram's banded fold + all-reduce (ops/device.py ``wide_bands``): the bands
tile the flat WLS layout exactly, in order, each near the bucket size."""
import pytest

from net.jgp.labs.sparkdq4ml_amd.ops.device import wide_bands


@pytest.mark.parametrize("d,bucket,elt", [(4096, 16 << 20, 4), (4096, 4 << 20, 8), (1024, 1 << 18, 4), (300, 1 << 30, 4),
                                          (257, 1 << 16, 8)])
def test_bands_tile_flat_layout(d, bucket, elt):
    P = (d + 255) // 256
    bands = wide_bands(P, d, bucket, elt)
    assert bands[0][:2] == (P, P + 1) and bands[0][2] == 0
    total = 5 + 2 * d + d * (d + 1) // 2
    # real-column bands cover [0, P) contiguously and their flat slices cover the packed part
    js = [(b[0], b[1]) for b in bands[1:]]
    assert js[0][0] == 0 and js[-1][1] == P and all(a[1] == b[0] for a, b in zip(js, js[1:]))
    assert bands[0][3] == bands[1][2] and bands[-1][3] == total
    assert all(a[3] == b[2] for a, b in zip(bands[1:], bands[2:]))
    # every band but the last reaches the bucket size; none exceeds it by more than one panel column
    col_max = (P * 256) * elt * 256
    for b in bands[1:-1]:
        assert bucket <= (b[3] - b[2]) * elt <= bucket + col_max


def test_gang_row_ranges_balance_the_units(monkeypatch):
    # ops/device.py _wide_gang_s: S row ranges per XCD group so the P(P+1)/2 units of a range
    # times S divide evenly over the G blocks of a group (equal-cost units stay in step)
    from net.jgp.labs.sparkdq4ml_amd.ops.device import _wide_gang_s

    monkeypatch.delenv("DQ4ML_WIDE_GANG_S", raising=False)
    nsup = 10_000_000 // 64
    assert _wide_gang_s(16, nsup, 32) == 4  # config 5: 136 x 4 = 544 = 17 x 32
    for P in (2, 3, 5, 16, 40):
        S = _wide_gang_s(P, nsup, 32)
        units = P * (P + 1) // 2 * S
        assert S >= 1 and units / (-(-units // 32) * 32) >= 0.9
        assert nsup >= 8 * S * 16  # >= 16 supersteps per split
    assert _wide_gang_s(16, 100, 32) == 0  # too few rows: the queue schedule instead
    # f32 accumulators count rows exactly only below 2^24 per split
    big = (1 << 30) // 64
    S = _wide_gang_s(16, big, 32)
    assert S and big * 64 / (8 * S) < (1 << 24)
    monkeypatch.setenv("DQ4ML_WIDE_GANG_S", "2")
    assert _wide_gang_s(16, nsup, 32) == 2
