"""Drop-in for the reference's `hourglass_compare.py` model.

Differences from the primary (`try_with_torch.py`) that this preset reproduces exactly:

* `ResidualBlock` (hourglass_compare.py:405-441) normalises its output branch with `bn4` and adds
  a projected skip `downsaple` = 1x1 conv (no bias) + BN. The reference guards the projection with
  `if self.stride != 1 | self.numIn != self.numOut` — `1 | numIn` binds first, so the chained
  comparison is true for every even channel count and the projection ALWAYS runs; the same
  expression is evaluated here.
* `hourglass(f)` (:492-538) has NO shared residual block: 14 separate blocks (`downsample1..4` =
  maxpool + block, `residual1..5`, `upsample1..4`) and nearest x2 up-sampling + add.
* the stem `preprocess1` (:542-551) has a BatchNorm + ReLU after the 7x7 conv; four UNSHARED
  stages (hourglass, block, 1x1 conv, BN, ReLU) with 16-channel heads (no bias) and the
  re-injection `inter = stage_return(out) + inter + stage_down_feature(ll)` (:598-636).

Every sub-module sits at the reference's attribute name / Sequential index (identical state_dict
keys and, under `torch.manual_seed`, identical initial weights). All ops run on the same libhgk
kernels; the BN-ed sum of the two block branches is ONE pass (Ctx.bn_add: both BN applies, the
add and the sum's statistics; backward both BN reductions in one pass).
"""
import torch.nn as nn

from .. import hgk as H
from .. import modules as _m


class ResidualBlock(_m._EngineModule):
    def __init__(self, numIn, numOut, stride=1):
        super().__init__()
        self.stride = stride
        self.numIn = numIn
        self.numOut = numOut
        self.bn1 = nn.BatchNorm2d(numIn)
        self.relu = nn.ReLU(True)
        self.conv1 = nn.Conv2d(numIn, int(numOut / 2), 1, 1)
        self.bn2 = nn.BatchNorm2d(int(numOut / 2))
        self.conv2 = nn.Conv2d(int(numOut / 2), int(numOut / 2), 3, stride, 1)
        self.bn3 = nn.BatchNorm2d(int(numOut / 2))
        self.conv3 = nn.Conv2d(int(numOut / 2), numOut, 1, 1)
        self.bn4 = nn.BatchNorm2d(numOut)
        self.downsaple = nn.Sequential(nn.Conv2d(numIn, numOut, 1, stride=stride, bias=False),
                                       nn.BatchNorm2d(numOut))

    def hg_forward(self, ctx, x):
        return run_interleaved(self.hg_steps(ctx, x))[0]

    def hg_steps(self, ctx, x):
        """hg_forward as a generator that yields after each BN use is declared and before the
        conv that reads it: run_interleaved advances two independent blocks in turn, so their
        BN finalizes are pending together and go out in one launch (engine route fin_batch)."""
        a = ctx.bn_relu(x, self.bn1)
        yield
        h = ctx.conv(a, self.conv1)
        a = ctx.bn_relu(h, self.bn2)
        yield
        h = ctx.conv(a, self.conv2)
        a = ctx.bn_relu(h, self.bn3)
        yield
        y3 = ctx.conv(a, self.conv3)
        out = ctx.bn_relu(y3, self.bn4, relu=False)
        # the reference's precedence: `stride != (1 | numIn) != numOut` (chained comparison)
        if self.stride != 1 | self.numIn != self.numOut:
            skip = ctx.bn_relu(ctx.conv(x, self.downsaple[0]), self.downsaple[1], relu=False)
            yield
            if ctx.bn_pair:
                # both BN applies + the add in one pass, the sum's statistics included
                return ctx.bn_add(out, skip)
            skip = ctx.materialize(skip)
        else:
            skip = x
        return ctx.add(ctx.materialize(out), skip)


def run_interleaved(*gens):
    """Advance the generators in turn until all are exhausted; their return values, in order."""
    out = [None] * len(gens)
    live = list(range(len(gens)))
    while live:
        nxt = []
        for i in live:
            try:
                next(gens[i])
                nxt.append(i)
            except StopIteration as e:
                out[i] = e.value
        live = nxt
    return out


class hourglass(_m._EngineModule):  # noqa: N801 (reference name)
    def __init__(self, f):
        super().__init__()
        self.f = f
        for i in range(1, 5):
            setattr(self, f"downsample{i}", nn.Sequential(nn.MaxPool2d(2, 2), ResidualBlock(f, f)))
        for i in range(1, 6):
            setattr(self, f"residual{i}", ResidualBlock(f, f))
        for i in range(1, 5):
            setattr(self, f"upsample{i}", ResidualBlock(f, f))

    def _down(self, ctx, i, a):
        seq = getattr(self, f"downsample{i}")
        return seq[1].hg_forward(ctx, ctx.maxpool2(a))

    def _pair(self, ctx, i, x):
        """(residual_i(x), downsample_i(x)): the two blocks are independent"""
        res, seq = getattr(self, f"residual{i}"), getattr(self, f"downsample{i}")
        # engine route pair_blocks: the pair runs interleaved step by step (hourglass_compare.py:
        # 506-520); off = one block after the other (bitwise equal: the same ops, only their
        # order between the two independent blocks changes)
        if not ctx.pair_blocks:
            return res.hg_forward(ctx, x), self._down(ctx, i, x)
        up = res.hg_steps(ctx, x)
        down = seq[1].hg_steps(ctx, ctx.maxpool2(x))
        return tuple(run_interleaved(up, down))

    def hg_forward(self, ctx, x):
        up1, down1 = self._pair(ctx, 1, x)
        up2, down2 = self._pair(ctx, 2, down1)
        up3, down3 = self._pair(ctx, 3, down2)
        up4, down4 = self._pair(ctx, 4, down3)
        out = self.residual5.hg_forward(ctx, down4)
        for i, up in ((4, up4), (3, up3), (2, up2), (1, up1)):
            out = getattr(self, f"upsample{i}").hg_forward(ctx, out)
            out = ctx.upsample2_add(out, up, H.UP_NEAREST)  # F.interpolate(x2) (nearest) + up
        return out


def _stage(nFeats):
    return nn.Sequential(hourglass(nFeats), ResidualBlock(nFeats, nFeats),
                         nn.Conv2d(nFeats, nFeats, 1, 1, 0), nn.BatchNorm2d(nFeats), nn.ReLU())


class creatModel(_m._EngineModule):  # noqa: N801
    """4 unshared stages; forward returns the 4 stage heatmaps [N, 16, H/4, W/4]."""

    _returns_list = True

    def __init__(self, nFeats=256, nOut=16):
        super().__init__()
        self.preprocess1 = nn.Sequential(
            nn.Conv2d(3, 64, 7, 2, 3), nn.BatchNorm2d(64), nn.ReLU(), ResidualBlock(64, 128),
            nn.MaxPool2d(2, 2), ResidualBlock(128, 128), ResidualBlock(128, nFeats))
        for k in range(1, 5):
            setattr(self, f"stage{k}", _stage(nFeats))
            setattr(self, f"stage{k}_out", nn.Conv2d(nFeats, nOut, 1, 1, 0, bias=False))
            if k < 4:
                setattr(self, f"stage{k}_return", nn.Conv2d(nOut, nFeats, 1, 1, 0, bias=False))
                setattr(self, f"stage{k}_down_feature",
                        nn.Conv2d(nFeats, nFeats, 1, 1, 0, bias=False))

    def hg_forward(self, ctx, x):
        p = self.preprocess1
        h = ctx.materialize(ctx.bn_relu(ctx.conv(x, p[0]), p[1], relu=True))
        h = p[3].hg_forward(ctx, h)
        h = ctx.maxpool2(h)
        h = p[5].hg_forward(ctx, h)
        inter = p[6].hg_forward(ctx, h)
        outs = []
        for k in range(1, 5):
            st = getattr(self, f"stage{k}")
            ll = st[0].hg_forward(ctx, inter)
            ll = st[1].hg_forward(ctx, ll)
            a = ctx.bn_relu(ctx.conv(ll, st[2]), st[3], relu=True)
            tmp = ctx.conv(a, getattr(self, f"stage{k}_out"), stats=False)
            outs.append(tmp)
            if k < 4:
                # inter = stage_return(tmpOut) + inter + stage_down_feature(ll)
                ret = ctx.conv(tmp, getattr(self, f"stage{k}_return"), stats=False)
                inter = ctx.conv(a, getattr(self, f"stage{k}_down_feature"),
                                 res=ctx.add(ret, inter), inplace_res=True)
        return outs
