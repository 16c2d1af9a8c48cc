"""Drop-in for the reference's `try_more_layer.py` model (live ASPP).

`try_with_aspp`'s progressive 3-head model (same registrations, same state_dict keys) with the ASPP
block LIVE at the innermost hourglass level (try_more_layer.py:271-292): there
low2 = conv1(cat[aspp1..aspp4(low1), broadcast(GAP branch(low1))]), where

* aspp1 = 1x1 conv + BN + ReLU, aspp2-4 = 3x3 convs dilated (and padded) 6 / 12 / 18 + BN + ReLU
  (try_more_layer.py:234-246) — the dilated implicit-GEMM conv of libhgk;
* the image-pool branch = AdaptiveAvgPool2d((1, 1)) -> 1x1 conv -> BN (over the N pooled rows) ->
  ReLU, then F.interpolate back to the level's size, bilinear with align_corners=True, i.e. a
  broadcast (:266-268,286-287): `hgk_spatial_sum` / `hgk_spatial_broadcast`;
* conv1 = 1x1, 1280 -> 256, no bias, no BN (:269,290).

The outer levels register the same ASPP modules and never run them (no grad, as the reference).
Module globals: nStack = 4 (:25) and `elif i >= 2` (:355): stacks 2 AND 3 both emit conv2_2
heatmaps from the same `inter`; the reference trains on outputs 0-2 only (:398-401).
"""
from . import try_with_aspp as _as
from .try_with_aspp import ResidualBlock, _ASPPModule, lin  # noqa: F401  (reference names)


class hourglass(_as.hourglass):  # noqa: N801 (reference name)
    """try_with_aspp's hourglass with the innermost ASPP block live (try_more_layer.py:271-292)."""

    def _aspp_branch(self, ctx, low, m):
        return ctx.materialize(ctx.bn_relu(ctx.conv(low, m.atrous_conv), m.bn))

    def _inner(self, ctx, low):
        low = ctx.materialize(low)
        parts = [self._aspp_branch(ctx, low, m)
                 for m in (self.aspp1, self.aspp2, self.aspp3, self.aspp4)]
        gp = self.global_avg_pool
        pooled = ctx.materialize(ctx.bn_relu(ctx.conv(ctx.spatial_mean(low), gp[1]), gp[2]))
        parts.append(ctx.broadcast(pooled, low.H, low.W))
        return ctx.conv(ctx.concat(parts), self.conv1)


class creatModel(_as.creatModel):  # noqa: N801
    """4 stacks; forward returns [bg logits [N,2,h,w], skeleton logits [N,20,h,w], keypoint
    heatmaps [N,17,h,w], keypoint heatmaps of the 4th stack [N,17,h,w]]."""

    _hourglass_cls = hourglass
    _late_heads = True

    def __init__(self, nStack=4, nFeats=256, nModules=2, nOutChannels_0=2, nOutChannels_1=20,
                 nOutChannels_2=17, depth=4, upsample="bilinear"):
        super().__init__(nStack, nFeats, nModules, nOutChannels_0, nOutChannels_1, nOutChannels_2,
                         depth, upsample)
