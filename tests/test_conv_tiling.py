"""Host-only tiling decisions of the weight-gradient kernel (tb_conv3d_wgrad_config, no GPU): every
C3 U-Net layer has a tiling, rows too wide for the LDS budget at the channel tile report none (the
layer's weight gradient then goes to ATen, texbias/conv.py fast_wgrad_applies)."""
import pytest

from texbias import conv as C

C3_LAYERS = [  # G shape, X shape, stride (scripts/wgrad_bench.py)
    ((2, 16, 120, 120, 80), (2, 16, 120, 120, 80), 1),
    ((2, 16, 120, 120, 80), (2, 4, 240, 240, 160), 2),
    ((2, 32, 60, 60, 40), (2, 16, 120, 120, 80), 2),
    ((2, 3, 240, 240, 160), (2, 3, 240, 240, 160), 1),
    ((2, 32, 120, 120, 80), (2, 3, 240, 240, 160), 2),
]


@pytest.mark.parametrize("g,x,s", C3_LAYERS)
def test_c3_layers_tile(g, x, s):
    assert C._wgrad_tiles(g, x, s)
    cfg = C.wgrad_config(g, x, s)
    assert 1 <= cfg["SEG"] <= 4 and cfg["YB"] >= 1 and cfg["lds_bytes"] <= 160 * 1024


@pytest.mark.parametrize("w", [130, 250])
def test_wide_rows_have_no_tiling(w):
    assert not C._wgrad_tiles((1, 40, 9, 7, w), (1, 24, 9, 7, w), 1)
