"""The analytic conv FLOP count of the bench's ``unet_compute`` key (texbias.train.step_conv_flops): a single
Conv3d / ConvTranspose3d by hand, and the reference U-Net at the C3 bench shape (0.687 TFLOP per step of
2 x 4 x 240 x 240 x 160: 117.1 GFLOP forward per sample, x 3 for training, less the first layer's input gradient)."""
import torch.nn as nn

from texbias.train import reference_model, step_conv_flops


def test_single_layers():
    conv = lambda: nn.Conv3d(4, 8, 3, stride=2, padding=1)  # noqa: E731
    out = 2 * 8 * 4 * 4 * 4  # [2, 8, 4, 4, 4]
    assert step_conv_flops(conv, (2, 4, 8, 8, 8)) == 2 * out * 4 * 27 * 2  # no input gradient
    seq = lambda: nn.Sequential(nn.Conv3d(4, 8, 3, padding=1), nn.ConvTranspose3d(8, 2, 3, stride=2, padding=1,  # noqa: E731
                                                                                 output_padding=1))
    first = 2 * 8 * 8 * 8 * 8 * 4 * 27
    second = 2 * 8 * 8 * 8 * 8 * 2 * 27  # input elements x Cout x k^3
    assert step_conv_flops(seq, (1, 4, 8, 8, 8)) == first * 2 + second * 3


def test_reference_unet_c3():
    f = step_conv_flops(lambda: reference_model(4, 3), (2, 4, 240, 240, 160))
    assert abs(f / 1e12 - 0.6867) < 0.001
    fwd = step_conv_flops(lambda: reference_model(4, 3), (1, 4, 240, 240, 160))
    assert abs(fwd - f / 2) < 1  # linear in the batch
