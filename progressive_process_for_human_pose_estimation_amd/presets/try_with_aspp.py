"""Drop-in for the reference's `try_with_aspp.py` model (BASELINE.json configs[3]).

`creatModel()` (try_with_aspp.py:299-343): the primary stem / hourglass / residual4 / lin trunk,
3 stacks, progressive heads: stack 0 predicts a 2-class background map (`conv2_0`, no bias), which
is concatenated to the lin features and mapped back by `conv4_0` (1x1, 258 -> 256, bias) into the
next stack's input; stack 1 the same with the 20-class skeleton map (`conv2_1` / `conv4_1`, no
biases); stack 2 the 17 keypoint heatmaps (`conv2_2`). The reference trains it with
CrossEntropy(out0, bg) + CrossEntropy(out1, skeleton) + MSE(out2, keypoints) (:356-398).

The reference's hourglass registers four `_ASPPModule`s, a global-average-pool branch and a
1280 -> 256 `conv1` per level (:213-232) and never calls them (:234-250): they are registered here
in the same order (so `torch.manual_seed(s)` gives bit-identical weights and the state_dict keys
match) and, as in the reference, never run and never get a gradient. Module globals (nStack,
nFeats, nModules, nOutChannels_0/1/2, :22-29) are keyword arguments with the reference's values.
"""
import torch.nn as nn

from .. import modules as _m
from ..modules import ResidualBlock, lin  # noqa: F401  (same public names as the reference file)


class _ASPPModule(nn.Module):
    """atrous conv (no bias) + BN + ReLU (try_with_aspp.py:195-207); registered, never run."""

    def __init__(self, inplanes, planes, kernel_size, padding, dilation):
        super().__init__()
        self.atrous_conv = nn.Conv2d(inplanes, planes, kernel_size=kernel_size, stride=1,
                                     padding=padding, dilation=dilation, bias=False)
        self.bn = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU()


class hourglass(_m.hourglass):  # noqa: N801 (reference name)
    """The primary hourglass + the (dead) ASPP registrations of try_with_aspp.py:213-232; the
    innermost level passes low1 straight on (low2 = low1, :245-246: no extra residual chain)."""

    _inner_chain = False

    def __init__(self, n, f, nModules=2, upsample="bilinear"):
        super().__init__(n, f, nModules, upsample)
        inplanes = 256
        dilations = [1, 6, 12, 18]
        self.aspp1 = _ASPPModule(inplanes, 256, 1, padding=0, dilation=dilations[0])
        self.aspp2 = _ASPPModule(inplanes, 256, 3, padding=dilations[1], dilation=dilations[1])
        self.aspp3 = _ASPPModule(inplanes, 256, 3, padding=dilations[2], dilation=dilations[2])
        self.aspp4 = _ASPPModule(inplanes, 256, 3, padding=dilations[3], dilation=dilations[3])
        self.global_avg_pool = nn.Sequential(nn.AdaptiveAvgPool2d((1, 1)),
                                             nn.Conv2d(inplanes, 256, 1, stride=1, bias=False),
                                             nn.BatchNorm2d(256), nn.ReLU())
        self.conv1 = nn.Conv2d(1280, 256, 1, bias=False)


class creatModel(_m.creatModel):  # noqa: N801
    """Progressive 3-stack model; forward returns [bg logits [N,2,h,w], skeleton logits
    [N,20,h,w], keypoint heatmaps [N,17,h,w]] (h, w = H/4, W/4)."""

    _hourglass_cls = hourglass
    _late_heads = False  # stacks i >= 3 emit conv2_2 heatmaps (try_more_layer.py: `elif i >= 2`)

    def __init__(self, nStack=3, nFeats=256, nModules=2, nOutChannels_0=2, nOutChannels_1=20,
                 nOutChannels_2=17, depth=4, upsample="bilinear"):
        _m._EngineModule.__init__(self)
        self._init_trunk(nStack, nFeats, nModules, depth, upsample)
        self.conv2_0 = nn.Conv2d(nFeats, nOutChannels_0, 1, 1, 0, bias=False)
        self.conv4_0 = nn.Conv2d(nFeats + nOutChannels_0, nFeats, 1, 1, 0)
        self.conv2_1 = nn.Conv2d(nFeats, nOutChannels_1, 1, 1, 0, bias=False)
        self.conv4_1 = nn.Conv2d(nFeats + nOutChannels_1, nFeats, 1, 1, 0, bias=False)
        self.conv2_2 = nn.Conv2d(nFeats, nOutChannels_2, 1, 1, 0, bias=False)

    def hg_forward(self, ctx, x):
        inter = self._stem(ctx, x)
        heads = [(self.conv2_0, self.conv4_0), (self.conv2_1, self.conv4_1), (self.conv2_2, None)]
        outs = []
        for i in range(self.nStack):
            a = self._stack_body(ctx, inter)
            if i >= 3 and not self._late_heads:
                # try_with_aspp.py:326-342 (`elif i == 2`): a 4th+ stack runs (BN statistics /
                # running stats) but produces nothing
                continue
            head, back = heads[min(i, 2)]
            tmp = ctx.conv(a, head, stats=False)
            outs.append(tmp)
            if back is not None and i < 2 and i + 1 < self.nStack:
                # ll_ = cat([ll, tmpOut]); inter = conv4_i(ll_): the lin output is materialised
                # (its BN+ReLU applied once) and concatenated on the channel axis
                cat = ctx.concat([ctx.materialize(a), tmp])
                inter = ctx.conv(cat, back)
        return outs
