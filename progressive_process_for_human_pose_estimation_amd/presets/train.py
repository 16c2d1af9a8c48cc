"""Drop-in for the reference's `train.py` model (stride-2 residual blocks).

* `ResidualBlock(numIn, numOut, stride)` (train.py:411-447) is hourglass_compare's block (bn4, the
  always-on BN-ed 1x1 projection per the `stride != 1 | numIn != numOut` precedence quirk) with
  the 3x3 `conv2` and the projection at stride `stride`. Their input-gradients run as stride-1
  convs of the zero-inserted output gradient (`hgk_zero_insert`); forward and weight-gradient
  kernels take the stride directly.
* `ASPP_Block` (:450-494): 1x1 + three dilated 3x3 (6 / 12 / 18) branches with BN+ReLU, the
  image-pool branch (global average pool -> 1x1 -> BN -> ReLU -> bilinear-ac broadcast), concat,
  then `conv1` = 1x1 (1280 -> 256) + BN + ReLU.
* `hourglass(f)` (:497-541): unshared; four stride-2 blocks down, four (f -> f/2) blocks on the
  skip path, ASPP at the bottom, then nearest x2 up-sampling, an (f -> f/2) block and a channel
  concat with the skip per level.
* `creatModel()` (:543-600): stem 7x7/2 + ReLU, RB(64, 128, stride 2), RB(128, 128),
  RB(128, nFeats); 3 unshared stages; re-injection inter = cat[return(out_k) (f/2),
  retuen_2(ll) (f/4), down_feature(inter) (f/4)]. Outputs: [N, 2, h, w], [N, 16, h, w],
  [N, 17, h, w] (MPII: nOutChannels_1 = 15 + 1, nOutChannels_2 = 16 + 1, :25-29).
* `generateMask()` (:603-620): stem + one hourglass + the 2-class head.

Attribute names (including the reference's `downsaple` / `stage1_retuen_2` spellings) and
registration order are the reference's: identical state_dict keys and, under
`torch.manual_seed`, identical initial weights.
"""
import torch.nn as nn

from .. import hgk as H
from .. import modules as _m
from .hourglass_compare import ResidualBlock, run_interleaved  # train.py:411-447 (stride included)
from .try_with_aspp import _ASPPModule


class ASPP_Block(_m._EngineModule):  # noqa: N801 (reference name)
    def __init__(self):
        super().__init__()
        inplanes = 256
        dilations = [1, 6, 12, 18]
        self.aspp1 = _ASPPModule(inplanes, 256, 1, padding=0, dilation=dilations[0])
        self.aspp2 = _ASPPModule(inplanes, 256, 3, padding=dilations[1], dilation=dilations[1])
        self.aspp3 = _ASPPModule(inplanes, 256, 3, padding=dilations[2], dilation=dilations[2])
        self.aspp4 = _ASPPModule(inplanes, 256, 3, padding=dilations[3], dilation=dilations[3])
        self.global_avg_pool = nn.Sequential(nn.AdaptiveAvgPool2d((1, 1)),
                                             nn.Conv2d(inplanes, 256, 1, stride=1, bias=False),
                                             nn.BatchNorm2d(256), nn.ReLU())
        self.conv1 = nn.Sequential(nn.Conv2d(1280, 256, 1, bias=False), nn.BatchNorm2d(256),
                                   nn.ReLU())

    def hg_forward(self, ctx, x):
        x = ctx.materialize(x)
        parts = [ctx.materialize(ctx.bn_relu(ctx.conv(x, m.atrous_conv), m.bn))
                 for m in (self.aspp1, self.aspp2, self.aspp3, self.aspp4)]
        gp = self.global_avg_pool
        pooled = ctx.materialize(ctx.bn_relu(ctx.conv(ctx.spatial_mean(x), gp[1]), gp[2]))
        parts.append(ctx.broadcast(pooled, x.H, x.W))
        return ctx.bn_relu(ctx.conv(ctx.concat(parts), self.conv1[0]), self.conv1[1])


class hourglass(_m._EngineModule):  # noqa: N801 (reference name)
    def __init__(self, f):
        super().__init__()
        self.f = f
        for i in range(1, 5):
            setattr(self, f"downsample{i}", ResidualBlock(f, f, stride=2))
        for i in range(1, 5):
            setattr(self, f"residual{i}", ResidualBlock(f, int(f / 2)))
        for i in range(1, 5):
            setattr(self, f"upsample{i}", ResidualBlock(f, int(f / 2)))
        self.aspp = ASPP_Block()

    def hg_forward(self, ctx, x):
        ups, down = [], x
        for i in range(1, 5):
            res, ds = getattr(self, f"residual{i}"), getattr(self, f"downsample{i}")
            if ctx.pair_blocks:  # independent blocks, interleaved (engine route pair_blocks)
                up, down = run_interleaved(res.hg_steps(ctx, down), ds.hg_steps(ctx, down))
                ups.append(up)
            else:
                ups.append(res.hg_forward(ctx, down))
                down = ds.hg_forward(ctx, down)
        out = ctx.materialize(self.aspp.hg_forward(ctx, down))
        for i in range(4, 0, -1):
            out = ctx.upsample2_add(out, None, H.UP_NEAREST)  # F.interpolate(scale_factor=2)
            out = getattr(self, f"upsample{i}").hg_forward(ctx, out)
            out = ctx.concat([out, ups[i - 1]])
        return out


def _stem(nFeats):
    return nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3), nn.ReLU(), ResidualBlock(64, 128, stride=2),
                         ResidualBlock(128, 128), ResidualBlock(128, nFeats))


def _run_stem(ctx, p, x):
    h = ctx.conv(x, p[0], post_relu=True, stats=False)
    for blk in (p[2], p[3], p[4]):
        h = blk.hg_forward(ctx, h)
    return h


class creatModel(_m._EngineModule):  # noqa: N801
    """3 unshared stages; forward returns [background [N,2,h,w], skeleton [N,16,h,w], keypoints
    [N,17,h,w]] (h, w = H/4, W/4)."""

    _returns_list = True

    def __init__(self, nFeats=256, nOutChannels_0=2, nOutChannels_1=16, nOutChannels_2=17):
        super().__init__()
        self.preprocess1 = _stem(nFeats)
        outs = (nOutChannels_0, nOutChannels_1)
        for k in (1, 2):
            setattr(self, f"stage{k}", hourglass(nFeats))
            setattr(self, f"stage{k}_out", nn.Conv2d(nFeats, outs[k - 1], 1, 1, 0, bias=False))
            setattr(self, f"stage{k}_return",
                    nn.Conv2d(outs[k - 1], int(nFeats / 2), 1, 1, 0, bias=False))
            setattr(self, f"stage{k}_retuen_2", nn.Conv2d(nFeats, int(nFeats / 4), 1, 1, 0, bias=False))
            setattr(self, f"stage{k}_down_feature",
                    nn.Conv2d(nFeats, int(nFeats / 4), 1, 1, 0, bias=False))
        self.stage3 = hourglass(nFeats)
        self.stage3_out = nn.Conv2d(nFeats, nOutChannels_2, 1, 1, 0, bias=False)

    def hg_forward(self, ctx, x):
        inter = _run_stem(ctx, self.preprocess1, x)
        outs = []
        for k in (1, 2, 3):
            ll = getattr(self, f"stage{k}").hg_forward(ctx, inter)
            tmp = ctx.conv(ll, getattr(self, f"stage{k}_out"), stats=False)
            outs.append(tmp)
            if k < 3:
                ret = ctx.conv(tmp, getattr(self, f"stage{k}_return"), stats=False)
                ll_ = ctx.conv(ll, getattr(self, f"stage{k}_retuen_2"), stats=False)
                down = ctx.conv(inter, getattr(self, f"stage{k}_down_feature"), stats=False)
                inter = ctx.concat([ret, ll_, down])
        return outs


class generateMask(_m._EngineModule):  # noqa: N801
    """stem + one hourglass + the 2-class background head (train.py:603-620)."""

    def __init__(self, nFeats=256, nOutChannels_0=2):
        super().__init__()
        self.preprocess1 = _stem(nFeats)
        self.stage1 = hourglass(nFeats)
        self.stage1_out = nn.Conv2d(nFeats, nOutChannels_0, 1, 1, 0, bias=False)

    def hg_forward(self, ctx, x):
        ll = self.stage1.hg_forward(ctx, _run_stem(ctx, self.preprocess1, x))
        return ctx.conv(ll, self.stage1_out, stats=False)
