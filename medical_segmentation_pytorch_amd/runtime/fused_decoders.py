"""The smp decoder hub on the fused MI355X kernels (reference ``models/__init__.py:8-10,23-25``).

Unet++, Linknet, FPN, DeepLabV3, DeepLabV3+ and PSPNet decoders over a ResNet encoder run entirely on
the HIP kernels, NHWC bf16 end to end: every conv is the implicit-GEMM / halo conv with the BatchNorm
statistics in its epilogue and the BN(+ReLU) deferred into its consumers' staging; the remaining ops
are the decoder kernels of ``csrc/decoder.hip`` (bilinear resize, GroupNorm, adaptive pooling,
depthwise conv) and the existing elementwise ones (nearest up2 + add / concat, n-way add).  Concats
that feed a conv are read as the conv's input channel groups where the widths allow it (ASPP's five
branches, PSP's pyramid + input, MAnet's gated high-level + skip), so they are never built.  PAN and
MAnet: every conv / BN / pooling / resize on the HIP kernels, and MAnet's position-attention products
+ whole-map softmax on ``csrc/attention.hip`` (``ops.attention``); the remaining attention glue (sigmoid
gates, broadcast products) is torch elementwise ops on the NHWC maps.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.attention import pab_attention
from ..ops.bn import materialize
from ..ops.conv import conv
from ..ops.decoder import adaptive_avgpool, dwconv, group_norm_act, resize_bilinear
from ..ops.elementwise import add_n, from_fm, up2_add
from ..ops.pool import maxpool, up2_cat


def _relu_of(m):
    inner = getattr(m, 'activation', m)
    if isinstance(inner, nn.ReLU):
        return True
    if isinstance(inner, nn.Identity):
        return False
    raise NotImplementedError(f'fused decoders support ReLU/Identity activations, got {inner}')


def _cat(ts):
    """Channel concat of NHWC maps (every width here is a multiple of 8: no padding in between)."""
    ts = [materialize(t) for t in ts]
    return ts[0] if len(ts) == 1 else torch.cat(ts, -1)


def _channel_dropout(x, p, training):
    """nn.Dropout2d on an NHWC map: one keep/scale draw per (image, channel)."""
    if not training or p <= 0:
        return x
    x = materialize(x)
    keep = (torch.rand(x.shape[0], 1, 1, x.shape[-1], device=x.device) >= p).to(x.dtype) * (1.0 / (1.0 - p))
    return x * keep


def _dropout(x, p, training):
    if not training or p <= 0:
        return x
    return F.dropout(materialize(x), p, True)


class SmpDecoders:
    """Mixin of :class:`runtime.fused_model.FusedExecutor`: one method per fused smp decoder."""

    # -- building blocks ------------------------------------------------------------------------------
    def conv_plain(self, conv_mod, xs, training):
        """A conv without a following BN (bias kept): FPN laterals / smoothing convs, PSP's 1x1 pool conv."""
        xs = xs if isinstance(xs, (list, tuple)) else [xs]
        plan = self.plan_conv(conv_mod, gi=len(xs))
        (y,), _ = self._conv(plan, xs, False)
        return y

    def conv_bn_act(self, conv_mod, bn_mod, act_mod, xs, training, single=False):
        """Conv -> BN -> act (BN deferred into the consumers); ``bn_mod`` Identity: conv (+bias) -> act."""
        if isinstance(bn_mod, nn.Identity):
            y = self.conv_plain(conv_mod, xs, training)
            return torch.relu(y) if _relu_of(act_mod) else y
        xs = xs if isinstance(xs, (list, tuple)) else [xs]
        plan = self.plan_conv(conv_mod, gi=len(xs))
        (y,), part = self._conv(plan, xs, training)
        return self._bn_out([y], self.bn(bn_mod), _relu_of(act_mod), training,
                            (part, plan.rows, 0) if training else None, single)

    def separable_bn_act(self, sep, bn_mod, act_mod, x, training):
        """SeparableConv2d (depthwise -> pointwise 1x1) -> BN -> act."""
        dw, pw = sep[0], sep[1]
        y = dwconv(materialize(x), dw)
        return self.conv_bn_act(pw, bn_mod, act_mod, y, training)

    def smp_head(self, model, x):
        """SegmentationHead: conv (+bias) -> NCHW fp32 logits -> optional bilinear upsampling (align_corners,
        nn.UpsamplingBilinear2d) on the C-channel logits."""
        head = model.segmentation_head
        if isinstance(head[1], nn.UpsamplingBilinear2d):
            # the upsampling runs on the NHWC bf16 logits (ops.decoder.resize_bilinear, csrc/decoder.hip)
            # before the one NCHW fp32 conversion: no fp32 NCHW map at 4-8x the head's resolution
            plan = self.plan_conv(head[0])
            (y,), _ = conv(plan, [x], want_stats=False)
            sf = head[1].scale_factor
            sf = sf[0] if isinstance(sf, (tuple, list)) else sf
            return from_fm(resize_bilinear(y, scale_factor=float(sf), align_corners=True), head[0].out_channels)
        return self.head(head[0], x, head[0].out_channels)

    # -- Unet++ (smp UnetPlusPlusDecoder) ---------------------------------------------------------------
    def _unet_block(self, blk, x, cx, skips, training):
        """UnetDecoderBlock: nearest up2 -> concat skips -> 2 x (conv3x3-BN-ReLU); returns (out, channels)."""
        sk = _cat([t for t, _ in skips]) if skips else None
        cs = sum(c for _, c in skips)
        y = up2_cat(materialize(x), sk, cx, cs)
        y = self.cba(blk.conv1, y, training, single=True)
        y = self.cba(blk.conv2, y, training)
        return y, blk.conv2[0].out_channels

    def smp_unetpp(self, model, images, training):
        enc, dec = model.encoder, model.decoder
        feats = self.resnet_encoder(enc, images, training)[::-1]
        chans = list(enc.out_channels[1:])[::-1]
        dense = {}
        depth = dec.depth
        for li in range(len(dec.in_channels) - 1):
            for d in range(depth - li):
                if li == 0:
                    dense[(d, d)] = self._unet_block(dec.blocks[f'x_{d}_{d}'], feats[d], chans[d],
                                                     [(feats[d + 1], chans[d + 1])], training)
                else:
                    top = d + li
                    skips = [dense[(i, top)] for i in range(d + 1, top + 1)] + [(feats[top + 1], chans[top + 1])]
                    x, cx = dense[(d, top - 1)]
                    dense[(d, top)] = self._unet_block(dec.blocks[f'x_{d}_{top}'], x, cx, skips, training)
        x, cx = dense[(0, depth - 1)]
        x, _ = self._unet_block(dec.blocks[f'x_0_{depth}'], x, cx, [], training)
        return self.smp_head(model, x)

    # -- Linknet ----------------------------------------------------------------------------------------
    def smp_linknet(self, model, images, training):
        enc, dec = model.encoder, model.decoder
        feats = self.resnet_encoder(enc, images, training)[::-1]
        x, skips = feats[0], feats[1:]
        for i, blk in enumerate(dec.blocks):
            c1, tr, c2 = blk.block
            y = self.cba(c1, x, training)                       # 1x1 conv-BN-ReLU (read by a transposed conv)
            plan = self.plan_deconv(tr[0])                      # ConvTranspose2d k4 s2 p1 (+bias)
            (u,), part = conv(plan, [y], want_stats=training)
            u = self._bn_out([u], self.bn(tr[1]), _relu_of(tr[2]), training,
                             (part, plan.rows, 0) if training else None, single=True)
            z = self.cba(c2, u, training)                       # 1x1 conv-BN-ReLU
            x = add_n(z, skips[i]) if i < len(skips) else z
        return self.smp_head(model, x)

    # -- FPN --------------------------------------------------------------------------------------------
    def smp_fpn(self, model, images, training):
        enc, dec = model.encoder, model.decoder
        feats = self.resnet_encoder(enc, images, training)
        c2, c3, c4, c5 = feats[-4:]
        p5 = self.conv_plain(dec.p5, c5, training)
        p4 = up2_add(p5, self.conv_plain(dec.p4.skip_conv, c4, training))   # nearest up2 + lateral 1x1
        p3 = up2_add(p4, self.conv_plain(dec.p3.skip_conv, c3, training))
        p2 = up2_add(p3, self.conv_plain(dec.p2.skip_conv, c2, training))
        pyr = []
        for blk, p in zip(dec.seg_blocks, [p5, p4, p3, p2]):
            x = p
            for m in blk.block:                                  # Conv3x3GNReLU (+ bilinear x2, align_corners)
                cv, gn, act = m.block
                x = group_norm_act(self.conv_plain(cv, x, training), gn, relu=_relu_of(act))
                if m.upsample:
                    x = resize_bilinear(x, scale_factor=2, align_corners=True)
            pyr.append(x)
        x = add_n(*pyr) if dec.merge_policy == 'add' else _cat(pyr)
        x = _channel_dropout(x, dec.dropout.p, training)
        return self.smp_head(model, x)

    # -- DeepLabV3 / V3+ --------------------------------------------------------------------------------
    def _aspp(self, aspp, x, training, separable):
        N, H, W, _ = x.shape
        outs = [self.conv_bn_act(aspp.convs[0][0], aspp.convs[0][1], aspp.convs[0][2], x, training)]
        for m in aspp.convs[1:-1]:
            if separable:   # ASPPSeparableConv: SeparableConv2d(dilated depthwise, pointwise) -> BN -> ReLU
                outs.append(self.separable_bn_act(m[0], m[1], m[2], x, training))
            else:           # ASPPConv: dilated 3x3 conv -> BN -> ReLU
                outs.append(self.conv_bn_act(m[0], m[1], m[2], x, training))
        pool = aspp.convs[-1]   # global average pool -> 1x1 conv -> BN -> ReLU -> upsample (from 1x1: broadcast)
        p = adaptive_avgpool(materialize(x), 1)
        p = materialize(self.conv_bn_act(pool[1], pool[2], pool[3], p, training))
        outs.append(p.expand(N, H, W, p.shape[-1]).contiguous())
        pj = aspp.project   # 1x1 over the five branches (read as channel groups: the concat is never built)
        y = self.conv_bn_act(pj[0], pj[1], pj[2], outs, training)
        return _dropout(y, pj[3].p, training)

    def smp_deeplabv3(self, model, images, training):
        enc, dec = model.encoder, model.decoder
        x = self.resnet_encoder(enc, images, training)[-1]
        y = self._aspp(dec[0], x, training, separable=False)
        y = self.conv_bn_act(dec[1], dec[2], dec[3], y, training)
        return self.smp_head(model, y)

    def smp_deeplabv3plus(self, model, images, training):
        enc, dec = model.encoder, model.decoder
        feats = self.resnet_encoder(enc, images, training)
        a = self._aspp(dec.aspp[0], feats[-1], training, separable=True)
        a = self.separable_bn_act(dec.aspp[1], dec.aspp[2], dec.aspp[3], a, training)
        a = resize_bilinear(materialize(a), scale_factor=dec.up.scale_factor, align_corners=True)
        b = self.conv_bn_act(dec.block1[0], dec.block1[1], dec.block1[2], feats[-4], training)
        y = self.separable_bn_act(dec.block2[0], dec.block2[1], dec.block2[2], _cat([a, b]), training)
        return self.smp_head(model, y)

    # -- PSPNet -----------------------------------------------------------------------------------------
    def smp_pspnet(self, model, images, training):
        enc, dec = model.encoder, model.decoder
        x = materialize(self.resnet_encoder(enc, images, training)[-1])
        N, H, W, _ = x.shape
        branches = []
        for b in dec.psp.blocks:   # adaptive pool (1/2/3/6) -> Conv2dReLU 1x1 -> bilinear (align_corners) to H x W
            pool, c = b.pool[0], b.pool[1]
            p = adaptive_avgpool(x, pool.output_size)
            z = materialize(self.conv_bn_act(c[0], c[1], c[2], p, training))
            branches.append(resize_bilinear(z, size=(H, W), align_corners=True))
        # cat([b1..b4, x]) = two equal-width channel groups: the four branches (C) and x (C)
        y = self.conv_bn_act(dec.conv[0], dec.conv[1], dec.conv[2], [_cat(branches), x], training)
        y = _channel_dropout(y, dec.dropout.p, training)
        return self.smp_head(model, y)


    # -- PAN (FPA + GAU attention blocks) ---------------------------------------------------------------
    def _cbr(self, m, x, training):
        """smp ConvBnRelu: conv (+bias) -> BN -> optional ReLU -> optional bilinear x2 (align_corners)."""
        y = materialize(self.conv_bn_act(m.conv, m.bn, m.activation if m.add_relu else nn.Identity(), x, training))
        return resize_bilinear(y, scale_factor=2, align_corners=True) if m.interpolate else y

    def _fpa(self, fpa, x, training):
        x = materialize(x)
        N, h, w, _ = x.shape
        b1 = self._cbr(fpa.branch1[1], adaptive_avgpool(x, 1), training)
        b1 = resize_bilinear(b1, size=(h, w), align_corners=True)
        mid = self._cbr(fpa.mid[0], x, training)
        x1 = self._cbr(fpa.down1[1], maxpool(x, 2, 2, 0), training)           # 1 channel (padded to 8)
        x2 = self._cbr(fpa.down2[1], maxpool(x1, 2, 2, 0), training)
        x3 = self._cbr(fpa.down3[2], self._cbr(fpa.down3[1], maxpool(x2, 2, 2, 0), training), training)
        x3 = resize_bilinear(x3, size=(h // 4, w // 4), align_corners=True)
        t = resize_bilinear(add_n(self._cbr(fpa.conv2, x2, training), x3), size=(h // 2, w // 2), align_corners=True)
        t = resize_bilinear(add_n(t, self._cbr(fpa.conv1, x1, training)), size=(h, w), align_corners=True)
        return t[..., :1] * mid + b1          # the 1-channel attention map broadcast over the channels

    def _gau(self, gau, x, y, training):
        """GAUBlock: up(y) + conv3x3-BN-ReLU(x) * sigmoid(BN(conv1x1(avgpool(y))))."""
        y = materialize(y)
        h, w = x.shape[1], x.shape[2]
        y_up = resize_bilinear(y, size=(h, w), align_corners=True)
        cb = gau.conv1[1]
        g = torch.sigmoid(materialize(self.conv_bn_act(cb.conv, cb.bn, nn.Identity(), adaptive_avgpool(y, 1),
                                                       training)))
        return y_up + self._cbr(gau.conv2, x, training) * g

    def smp_pan(self, model, images, training):
        enc, dec = model.encoder, model.decoder
        feats = self.resnet_encoder(enc, images, training)
        x = self._fpa(dec.fpa, feats[-1], training)
        x = self._gau(dec.gau3, feats[-2], x, training)
        x = self._gau(dec.gau2, feats[-3], x, training)
        x = self._gau(dec.gau1, feats[-4], x, training)
        return self.smp_head(model, x)

    # -- MAnet (position-attention center + multi-scale fusion attention blocks) -------------------------
    def _pab(self, pab, x, training):
        x = materialize(x)
        b, h, w, Cp = x.shape
        hw, P, C = h * w, pab.pab_channels, pab.in_channels
        top = self.conv_plain(pab.top_conv, x, training).reshape(b, hw, -1)[..., :P]
        center = self.conv_plain(pab.center_conv, x, training).reshape(b, hw, -1)[..., :P]
        bottom = self.conv_plain(pab.bottom_conv, x, training).reshape(b, hw, -1)[..., :C]
        sp = pab_attention(center, top, bottom)   # softmax over the whole map, . bottom: [b, hw, C] (HIP)
        # the reference reshapes the [b, hw, C] product straight to [b, C, h, w] (no transpose): same here
        sp = sp.reshape(b, C, h, w).permute(0, 2, 3, 1)
        if Cp != C:
            sp = F.pad(sp, (0, Cp - C))
        return self.conv_plain(pab.out_conv, x + sp.contiguous(), training)

    def _se(self, se, x, training):
        """SE gate: avgpool -> 1x1 (+bias) -> ReLU -> 1x1 (+bias) -> sigmoid, [N, 1, 1, C]."""
        g = self.conv_plain(se[1], adaptive_avgpool(materialize(x), 1), training)
        g = self.conv_plain(se[3], torch.relu(g), training)
        return torch.sigmoid(g)

    def _mfab(self, blk, x, cx, skip, training):
        y = self.cba(blk.hl_conv[0], x, training, single=True)
        y = self.cba(blk.hl_conv[1], y, training)
        cs = blk.hl_conv[1][0].out_channels
        y = up2_cat(materialize(y), None, cs, 0)                               # nearest x2
        att = self._se(blk.SE_hl, y, training)
        if skip is None:
            z = self.cba(blk.conv1, y, training, single=True)
        else:
            att = att + self._se(blk.SE_ll, skip, training)
            z = self.cba(blk.conv1, [y * att, materialize(skip)], training, single=True)   # cat as 2 groups
        return self.cba(blk.conv2, z, training), blk.conv2[0].out_channels

    def smp_manet(self, model, images, training):
        from ..models import smp
        enc, dec = model.encoder, model.decoder
        feats = self.resnet_encoder(enc, images, training)[::-1]
        chans = list(enc.out_channels[1:])[::-1]
        x, cx = self._pab(dec.center, feats[0], training), chans[0]
        skips = feats[1:]
        for i, blk in enumerate(dec.blocks):
            skip = skips[i] if i < len(skips) else None
            if isinstance(blk, smp.MFABBlock):
                x, cx = self._mfab(blk, x, cx, skip, training)
            else:
                x, cx = self._unet_block(blk, x, cx, [(skip, chans[i + 1])] if skip is not None else [], training)
        return self.smp_head(model, x)


def fused_decoder_kind(model):
    """Name of the fused decoder method for an smp model (None: the hybrid eager-decoder path)."""
    from ..models import smp
    dec = getattr(model, 'decoder', None)
    head = getattr(model, 'segmentation_head', None)
    if head is None or not isinstance(head[0], nn.Conv2d) or not isinstance(head[2], nn.Identity):
        return None
    if isinstance(dec, smp.UnetPlusPlusDecoder):
        return 'smp_unetpp' if all(isinstance(b.conv1[1], nn.BatchNorm2d) for b in dec.blocks.values()) else None
    if isinstance(dec, smp.LinknetDecoder):
        return 'smp_linknet' if all(isinstance(b.block[0][1], nn.BatchNorm2d) for b in dec.blocks) else None
    if isinstance(dec, smp.FPNDecoder):
        return 'smp_fpn' if dec.merge_policy in ('add', 'cat') else None
    if isinstance(dec, smp.DeepLabV3Decoder):
        return 'smp_deeplabv3'
    if isinstance(dec, smp.DeepLabV3PlusDecoder):
        return 'smp_deeplabv3plus'
    if isinstance(dec, smp.PSPDecoder):
        return 'smp_pspnet' if isinstance(dec.conv[1], nn.BatchNorm2d) else None
    if isinstance(dec, smp.PANDecoder):
        return 'smp_pan' if dec.gau1.upscale_mode == 'bilinear' else None
    if isinstance(dec, smp.MAnetDecoder):
        return 'smp_manet' if all(isinstance(getattr(b, 'conv1')[1], nn.BatchNorm2d) for b in dec.blocks) else None
    return None
