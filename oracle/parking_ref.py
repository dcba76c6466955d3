"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product package.

CPU (PyTorch fp32) restatement of the reference ParkingModel forward, losses and train step.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this file.

Each class keeps the reference's state-dict key names (861 keys) so a state dict moves
between the reference, this oracle and the product unchanged.  Citations are
reference-relative (file:line under qintonguav/e2e-parking-carla).

Deterministic-train protocol: construct with `dropout=False` to zero every
dropout probability and the EfficientNet drop-connect rate; pass `noise` (B,2 float in
[0,1)) to `forward`/`encoder` to replace the `torch.rand_like` draw of
model/parking_model.py:36.

Pinning: tests/golden/make_golden.py imports the real reference (this container only) and
checks this restatement against it on closed-form weights and inputs; the outputs are
committed under tests/golden/.  The EfficientNet/ResNet trunks (oracle/trunks.py) are a
restatement of third-party packages absent from the image — that part is parity-unpinned.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from oracle import trunks


# ----------------------------------------------------------------------------------------
# configuration (tool/config.py:7-111 + config/training.yaml:1-52)
# ----------------------------------------------------------------------------------------

class Cfg:
    token_nums = 204
    bev_encoder_in_channel = 64
    bev_encoder_out_channel = 258
    bev_x_bound = [-10.0, 10.0, 0.1]
    bev_y_bound = [-10.0, 10.0, 0.1]
    bev_z_bound = [-10.0, 10.0, 20.0]
    d_bound = [0.5, 12.5, 0.25]
    final_dim = [256, 256]
    bev_down_sample = 8
    use_depth_distribution = 1
    backbone = "efficientnet-b4"
    seg_classes = 3
    seg_vehicle_weights = [1.0, 2.0, 2.0]
    tf_en_dim = 258
    tf_en_heads = 6
    tf_en_layers = 4
    tf_en_dropout = 0.05
    tf_en_bev_length = 256
    tf_en_motion_length = 3
    tf_de_dim = 258
    tf_de_heads = 6
    tf_de_layers = 4
    tf_de_dropout = 0.05
    tf_de_tgt_dim = 15
    learning_rate = 1e-4
    weight_decay = 1e-4
    epochs = 155


# ----------------------------------------------------------------------------------------
# geometry (tool/geometry.py:40-59, model/bev_model.py:28-57)
# ----------------------------------------------------------------------------------------

def bev_params(xb, yb, zb):
    rows = (xb, yb, zb)
    res = torch.tensor([r[2] for r in rows])
    start = torch.tensor([r[0] + r[2] / 2.0 for r in rows])
    dim = torch.tensor([(r[1] - r[0]) / r[2] for r in rows], dtype=torch.long)
    return res, start, dim


def frustum(final_dim, down, d_bound):
    H, W = final_dim
    h, w = H // down, W // down
    d = torch.arange(*d_bound, dtype=torch.float)
    D = d.shape[0]
    xs = torch.linspace(0, W - 1, w, dtype=torch.float).view(1, 1, w).expand(D, h, w)
    ys = torch.linspace(0, H - 1, h, dtype=torch.float).view(1, h, 1).expand(D, h, w)
    return torch.stack((xs, ys, d.view(-1, 1, 1).expand(D, h, w)), -1)


def rig_transforms(intrinsics, extrinsics):
    """combine = R(E^-1) K^-1, trans = t(E^-1): model/bev_model.py:46-53 (fp32, CPU)."""
    inv_e = torch.inverse(extrinsics)
    rot, trans = inv_e[..., :3, :3], inv_e[..., :3, 3]
    combine = rot.matmul(torch.inverse(intrinsics))
    return combine, trans


def geometry(frustum_t, intrinsics, extrinsics):
    """model/bev_model.py:45-57 — ego-frame xyz of every frustum point."""
    combine, trans = rig_transforms(intrinsics, extrinsics)
    b, n, _ = trans.shape
    p = frustum_t.unsqueeze(0).unsqueeze(0).unsqueeze(-1)
    p = torch.cat((p[..., :2, :] * p[..., 2:3, :], p[..., 2:3, :]), 5)
    xyz = combine.view(b, n, 1, 1, 1, 3, 3).matmul(p).squeeze(-1)
    return xyz + trans.view(b, n, 1, 1, 1, 3)


def pillar_index(xyz, res, start, dim):
    """model/bev_model.py:85-95 — integer pillar rank per point, -1 where masked.

    Returns int64 (B, N, D, h, w) with rank = x*Y*Z + y*Z + z (z is always 0 here)."""
    B = xyz.shape[0]
    g = ((xyz - (start - res / 2.0)) / res).reshape(B, -1, 3).long()
    ok = ((g[..., 0] >= 0) & (g[..., 0] < dim[0]) & (g[..., 1] >= 0) & (g[..., 1] < dim[1])
          & (g[..., 2] >= 0) & (g[..., 2] < dim[2]))
    rank = g[..., 0] * (dim[1] * dim[2]) + g[..., 1] * dim[2] + g[..., 2]
    rank = torch.where(ok, rank, torch.full_like(rank, -1))
    return rank.view(xyz.shape[:-1])


class _VoxelSum(torch.autograd.Function):
    """tool/geometry.py:285-317 — cumsum-difference segmented sum over rank-sorted points."""

    @staticmethod
    def forward(ctx, x, ranks):
        cs = x.cumsum(0)
        last = torch.ones(x.shape[0], dtype=torch.bool)
        last[:-1] = ranks[1:] != ranks[:-1]
        cs = cs[last]
        out = torch.cat((cs[:1], cs[1:] - cs[:-1]))
        ctx.save_for_backward(last)
        return out, last

    @staticmethod
    def backward(ctx, g, _):
        (last,) = ctx.saved_tensors
        idx = torch.cumsum(last, 0)
        idx[last] -= 1
        return g[idx], None


def splat(xyz, feats, res, start, dim):
    """model/bev_model.py:74-107 — pool (B,N,D,h,w,C) point features into (B,C,X,Y)."""
    B, N, D, h, w, C = feats.shape
    X, Y, Z = (int(v) for v in dim)
    out = torch.zeros((B, C, X, Y), dtype=feats.dtype)
    P = N * D * h * w
    for b in range(B):
        x = feats[b].reshape(P, C)
        g = ((xyz[b] - (start - res / 2.0)) / res).view(P, 3).long()
        keep = ((g[:, 0] >= 0) & (g[:, 0] < X) & (g[:, 1] >= 0) & (g[:, 1] < Y)
                & (g[:, 2] >= 0) & (g[:, 2] < Z))
        x, g = x[keep], g[keep]
        r = g[:, 0] * (Y * Z) + g[:, 1] * Z + g[:, 2]
        order = r.argsort()
        x, g, r = x[order], g[order], r[order]
        s, last = _VoxelSum.apply(x, r)
        g = g[last]
        grid = torch.zeros((Z, X, Y, C), dtype=feats.dtype)
        grid[g[:, 2], g[:, 0], g[:, 1]] = s
        out[b] = grid.permute(0, 3, 1, 2).squeeze(0)
    return out


# ----------------------------------------------------------------------------------------
# camera encoder heads (model/convolutions.py:183-282, model/cam_encoder.py:8-111)
# ----------------------------------------------------------------------------------------

def _cbr(cin, cout, k, pad=0, dil=1, relu_inplace=False):
    return [nn.Conv2d(cin, cout, k, padding=pad, dilation=dil, bias=False), nn.BatchNorm2d(cout),
            nn.ReLU(inplace=relu_inplace)]


class _AsppPool(nn.Sequential):
    def __init__(self, cin, cout):
        super().__init__(nn.AdaptiveAvgPool2d(1), nn.Conv2d(cin, cout, 1, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU())

    def forward(self, x):
        hw = x.shape[-2:]
        return F.interpolate(super().forward(x), size=hw, mode="bilinear", align_corners=False)


class _Aspp(nn.Module):
    def __init__(self, cin, rates, cout, p_drop):
        super().__init__()
        branches = [nn.Sequential(*_cbr(cin, cout, 1))]
        branches += [nn.Sequential(*_cbr(cin, cout, 3, r, r)) for r in rates]
        branches.append(_AsppPool(cin, cout))
        self.convs = nn.ModuleList(branches)
        self.project = nn.Sequential(*_cbr(len(branches) * cout, cout, 1), nn.Dropout(p_drop))

    def forward(self, x):
        return self.project(torch.cat([m(x) for m in self.convs], 1))


class _DeepLab(nn.Sequential):
    def __init__(self, cin, cout, hidden, p_drop):
        super().__init__(_Aspp(cin, (12, 24, 36), hidden, p_drop),
                         nn.Conv2d(hidden, hidden, 3, padding=1, bias=False),
                         nn.BatchNorm2d(hidden), nn.ReLU(), nn.Conv2d(hidden, cout, 1))


class _UpCat(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.upsample = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=False)
        self.conv = nn.Sequential(*_cbr(cin, cout, 3, 1, relu_inplace=True),
                                  *_cbr(cout, cout, 3, 1, relu_inplace=True))

    def forward(self, low, skip):
        return self.conv(torch.cat([skip, self.upsample(low)], 1))


class CamEncoderRef(nn.Module):
    def __init__(self, cfg, D, dropout=True):
        super().__init__()
        self.backbone = trunks.EfficientNet("efficientnet-b4",
                                            drop_connect_rate=0.2 if dropout else 0.0)
        del self.backbone._blocks[22:]
        for k in ("_conv_head", "_bn1", "_avg_pooling", "_dropout", "_fc"):
            delattr(self.backbone, k)
        p = 0.5 if dropout else 0.0
        self.depth_layer_1 = _DeepLab(160, 160, 64, p)
        self.depth_layer_2 = _UpCat(160 + 56, D)
        self.feature_layer_1 = _DeepLab(160, 160, 64, p)
        self.feature_layer_2 = _UpCat(160 + 56, cfg.bev_encoder_in_channel)

    def forward(self, x):
        bb = self.backbone
        x = bb._swish(bb._bn0(bb._conv_stem(x)))
        ends, prev = [], x
        n = len(bb._blocks)
        for i, blk in enumerate(bb._blocks):
            rate = bb._global_params.drop_connect_rate
            if rate:
                rate *= float(i) / n
            x = blk(x, drop_connect_rate=rate)
            if prev.size(2) > x.size(2):
                ends.append(prev)
            prev = x
        ends.append(x)
        deep, skip = ends[3], ends[2]  # reduction_4 (16^2, 160ch), reduction_3 (32^2, 56ch)
        feat = self.feature_layer_2(self.feature_layer_1(deep), skip)
        depth = self.depth_layer_2(self.depth_layer_1(deep), skip)
        return feat, depth


# ----------------------------------------------------------------------------------------
# BEV model / encoder / fusion / heads
# ----------------------------------------------------------------------------------------

class BevModelRef(nn.Module):
    def __init__(self, cfg, dropout=True):
        super().__init__()
        self.cfg = cfg
        res, start, dim = bev_params(cfg.bev_x_bound, cfg.bev_y_bound, cfg.bev_z_bound)
        self.bev_res = nn.Parameter(res, requires_grad=False)
        self.bev_start_pos = nn.Parameter(start, requires_grad=False)
        self.bev_dim = nn.Parameter(dim, requires_grad=False)
        self.frustum = nn.Parameter(frustum(cfg.final_dim, cfg.bev_down_sample, cfg.d_bound),
                                    requires_grad=False)
        self.cam_encoder = CamEncoderRef(cfg, self.frustum.shape[0], dropout)

    def forward(self, images, intrinsics, extrinsics):
        xyz = geometry(self.frustum, intrinsics, extrinsics)
        b, n = images.shape[:2]
        feat, depth = self.cam_encoder(images.reshape(b * n, *images.shape[2:]))
        prob = depth.softmax(1)
        outer = prob.unsqueeze(1) * feat.unsqueeze(2)                 # bev_model.py:66
        outer = outer.view(b, n, *outer.shape[1:]).permute(0, 1, 3, 4, 5, 2)
        bev = splat(xyz, outer, self.bev_res, self.bev_start_pos, self.bev_dim)
        return bev, prob


class BevEncoderRef(nn.Module):
    def __init__(self, cin):
        super().__init__()
        t = trunks.resnet18(zero_init_residual=True)
        self.conv1 = nn.Conv2d(cin + 1, 64, 7, 2, 3, bias=False)
        self.bn1, self.relu, self.max_pool = t.bn1, t.relu, t.maxpool
        self.layer1, self.layer2, self.layer3, self.layer4 = t.layer1, t.layer2, t.layer3, t.layer4

    def forward(self, x):
        x = F.interpolate(x, size=(256, 256), mode="bilinear", align_corners=False)
        x = self.max_pool(self.relu(self.bn1(self.conv1(x))))
        return torch.flatten(self.layer3(self.layer2(self.layer1(x))), 2)


def _xavier_except_pos(mod):
    for name, p in mod.named_parameters():
        if "pos_embed" not in name and p.dim() > 1:
            nn.init.xavier_uniform_(p)
    nn.init.trunc_normal_(mod.pos_embed, std=0.02)


class FeatureFusionRef(nn.Module):
    def __init__(self, cfg, dropout=True):
        super().__init__()
        pd = cfg.tf_en_dropout if dropout else 0.0
        layer = nn.TransformerEncoderLayer(cfg.tf_en_dim, cfg.tf_en_heads,
                                           dropout=0.1 if dropout else 0.0)
        self.tf_encoder = nn.TransformerEncoder(layer, cfg.tf_en_layers, enable_nested_tensor=False)
        self.pos_embed = nn.Parameter(torch.randn(1, cfg.tf_en_bev_length, cfg.tf_en_dim) * 0.02)
        self.pos_drop = nn.Dropout(pd)
        u = cfg.tf_en_bev_length // 4
        self.motion_encoder = nn.Sequential(
            nn.Linear(cfg.tf_en_motion_length, u), nn.ReLU(inplace=True),
            nn.Linear(u, 2 * u), nn.ReLU(inplace=True),
            nn.Linear(2 * u, cfg.tf_en_bev_length), nn.ReLU(inplace=True))
        _xavier_except_pos(self)

    def forward(self, bev, ego_motion):
        m = self.motion_encoder(ego_motion).transpose(1, 2).expand(-1, -1, 2)
        x = self.pos_drop(torch.cat([bev.transpose(1, 2), m], 2) + self.pos_embed)
        return self.tf_encoder(x.transpose(0, 1)).transpose(0, 1)


class ControlPredictRef(nn.Module):
    def __init__(self, cfg, dropout=True):
        super().__init__()
        self.pad_idx = cfg.token_nums - 1
        self.tgt_len = cfg.tf_de_tgt_dim - 1
        self.embedding = nn.Embedding(cfg.token_nums, cfg.tf_de_dim)
        self.pos_drop = nn.Dropout(cfg.tf_de_dropout if dropout else 0.0)
        self.pos_embed = nn.Parameter(torch.randn(1, self.tgt_len, cfg.tf_de_dim) * 0.02)
        layer = nn.TransformerDecoderLayer(cfg.tf_de_dim, cfg.tf_de_heads,
                                           dropout=0.1 if dropout else 0.0)
        self.tf_decoder = nn.TransformerDecoder(layer, cfg.tf_de_layers)
        self.output = nn.Linear(cfg.tf_de_dim, cfg.token_nums)
        _xavier_except_pos(self)

    def _masks(self, tgt):
        L = tgt.shape[1]
        causal = torch.full((L, L), float("-inf")).triu(1)   # control_predict.py:32-37
        return causal, tgt == self.pad_idx

    def _decode(self, memory, emb, tgt):
        causal, padm = self._masks(tgt)
        y = self.tf_decoder(tgt=emb.transpose(0, 1), memory=memory.transpose(0, 1),
                            tgt_mask=causal, tgt_key_padding_mask=padm)
        return self.output(y.transpose(0, 1))

    def forward(self, memory, tgt):
        tgt = tgt[:, :-1]
        return self._decode(memory, self.pos_drop(self.embedding(tgt) + self.pos_embed), tgt)

    def predict(self, memory, tgt):
        L = tgt.size(1)
        pad = torch.full((tgt.size(0), self.tgt_len - L), self.pad_idx, dtype=torch.long)
        tgt = torch.cat([tgt, pad], 1)
        logits = self._decode(memory, self.embedding(tgt) + self.pos_embed, tgt)[:, L - 1, :]
        return logits.softmax(-1).argmax(-1).view(-1, 1)


class SegHeadRef(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        cin, c, k = cfg.bev_encoder_out_channel, cfg.bev_encoder_in_channel, cfg.seg_classes
        self.relu = nn.ReLU(inplace=True)
        self.up_sample = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=False)
        self.c5_conv = nn.Conv2d(cin, c, 1)
        self.up_conv5 = nn.Conv2d(c, c, 1)
        self.up_conv4 = nn.Conv2d(c, c, 1)
        self.up_conv3 = nn.Conv2d(c, c, 1)
        self.segmentation_head = nn.Sequential(nn.Conv2d(c, c, 3, padding=1, bias=False),
                                               nn.BatchNorm2d(c), nn.ReLU(inplace=True),
                                               nn.Conv2d(c, k, 1))

    def forward(self, tokens):
        t = tokens.transpose(1, 2)
        b, c, s = t.shape
        x = t.reshape(b, c, int(math.sqrt(s)), -1)
        x = self.relu(self.c5_conv(x))
        for conv in (self.up_conv5, self.up_conv4, self.up_conv3):
            x = self.relu(conv(self.up_sample(x)))
        x = F.interpolate(x, size=(200, 200), mode="bilinear", align_corners=False)
        return self.segmentation_head(x)


class ParkingModelRef(nn.Module):
    """model/parking_model.py:12-78."""

    def __init__(self, cfg=Cfg, dropout=True):
        super().__init__()
        self.cfg = cfg
        self.bev_model = BevModelRef(cfg, dropout)
        self.bev_encoder = BevEncoderRef(cfg.bev_encoder_in_channel)
        self.feature_fusion = FeatureFusionRef(cfg, dropout)
        self.control_predict = ControlPredictRef(cfg, dropout)
        self.segmentation_head = SegHeadRef(cfg)

    def add_target_bev(self, bev, target_point, noise=None):
        """model/parking_model.py:28-46 (noise = the rand_like draw, (B,2) in [0,1))."""
        b, c, h, w = bev.shape
        tgt = torch.zeros((b, 1, h, w))
        px = (h / 2 + target_point[:, 0] / self.cfg.bev_x_bound[2]).unsqueeze(0).T.int()
        py = (w / 2 + target_point[:, 1] / self.cfg.bev_y_bound[2]).unsqueeze(0).T.int()
        pt = torch.cat([px, py], 1)
        if noise is None:
            noise = torch.rand(pt.shape)
        pt += (noise.float() * 10 - 5).int()
        for i in range(b):
            x0, y0 = int(pt[i, 0]), int(pt[i, 1])
            tgt[i, 0, x0 - 4:x0 + 4, y0 - 4:y0 + 4] = 1.0
        return torch.cat([bev, tgt], 1), tgt

    def encoder(self, data, noise=None):
        bev, depth = self.bev_model(data["image"], data["intrinsics"], data["extrinsics"])
        bev, tgt = self.add_target_bev(bev, data["target_point"], noise)
        fused = self.feature_fusion(self.bev_encoder(bev), data["ego_motion"])
        return fused, self.segmentation_head(fused), depth, tgt

    def forward(self, data, noise=None):
        fused, seg, depth, _ = self.encoder(data, noise)
        return self.control_predict(fused, data["gt_control"]), seg, depth

    def predict(self, data, noise=None):
        fused, seg, depth, tgt = self.encoder(data, noise)
        toks = data["gt_control"]
        for _ in range(3):
            toks = torch.cat([toks, self.control_predict.predict(fused, toks)], 1)
        return toks, seg, depth, tgt


# ----------------------------------------------------------------------------------------
# losses (loss/*.py) and the train step (trainer/pl_trainer.py:55-83,116-121)
# ----------------------------------------------------------------------------------------

def control_loss(pred, gt_control, pad_idx=203):
    return F.cross_entropy(pred.reshape(-1, pred.shape[-1]), gt_control[:, 1:].reshape(-1),
                           ignore_index=pad_idx)


def segmentation_loss(pred, target, weights=(1.0, 2.0, 2.0)):
    if target.shape[-3] != 1:
        raise ValueError("segmentation label must be index label with channel dim = 1")
    b, s, c, h, w = pred.shape
    l = F.cross_entropy(pred.view(b * s, c, h, w), target.view(b * s, h, w), reduction="none",
                        ignore_index=255, weight=torch.tensor(weights, dtype=pred.dtype))
    return l.mean()


def depth_labels(gt, d_bound=(0.5, 12.5, 0.25), down=8):
    """loss/depth_loss.py:31-48 — one-hot (B*N*h*w, D) labels from metric depth."""
    B, N, H, W = gt.shape
    D = int((d_bound[1] - d_bound[0]) / d_bound[2])
    g = gt.view(B * N, H // down, down, W // down, down, 1).permute(0, 1, 3, 5, 2, 4).contiguous()
    g = g.view(-1, down * down)
    g = torch.where(g == 0.0, 1e5 * torch.ones_like(g), g).min(-1).values
    g = (g - (d_bound[0] - d_bound[2])) / d_bound[2]
    g = torch.where((g < D + 1) & (g >= 0.0), g, torch.zeros_like(g))
    return F.one_hot(g.long(), num_classes=D + 1).view(-1, D + 1)[:, 1:].to(gt.dtype)


def depth_loss(prob, gt):
    lab = depth_labels(gt)
    D = lab.shape[1]
    p = prob.permute(0, 2, 3, 1).contiguous().view(-1, D)
    fg = lab.max(1).values > 0.0
    return F.binary_cross_entropy(p[fg], lab[fg], reduction="none").sum() / max(1.0, fg.sum())


def train_losses(model, data, noise=None):
    pc, ps, pd = model(data, noise)
    lc = control_loss(pc, data["gt_control"])
    ls = segmentation_loss(ps.unsqueeze(1), data["segmentation"])
    ld = depth_loss(pd, data["depth"])
    return {"control_loss": lc, "segmentation_loss": ls, "depth_loss": ld,
            "train_loss": lc + ls + ld}, (pc, ps, pd)


def make_optimizer(model, cfg=Cfg):
    return torch.optim.Adam(model.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay)


def train_step(model, opt, data, noise=None):
    losses, outs = train_losses(model, data, noise)
    opt.zero_grad(set_to_none=True)
    losses["train_loss"].backward()
    opt.step()
    return losses, outs
