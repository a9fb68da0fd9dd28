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
