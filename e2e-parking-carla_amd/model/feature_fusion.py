"""Target/ego fusion: motion MLP + BEV tokens + positional embedding -> 4-layer transformer.

Mirrors reference model/feature_fusion.py:8-51 (keys: tf_encoder.layers.i.*, pos_embed,
motion_encoder.{0,2,4}).  The encoder layers stay `nn.TransformerEncoderLayer` modules so
the closed-loop agent's attention hook (agent/parking_agent.py:71-80,266-268) keeps working;
their arithmetic runs through e2ep_amd.transformer."""
import torch
from torch import nn

from e2ep_amd import nn_ops, transformer


class FeatureFusion(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        det = getattr(cfg, "deterministic", False)
        layer = nn.TransformerEncoderLayer(d_model=cfg.tf_en_dim, nhead=cfg.tf_en_heads,
                                           dropout=0.0 if det else 0.1)
        self.tf_encoder = nn.TransformerEncoder(layer, num_layers=cfg.tf_en_layers,
                                                enable_nested_tensor=False)
        self.pos_embed = nn.Parameter(torch.randn(1, cfg.tf_en_bev_length, cfg.tf_en_dim) * .02)
        self.pos_drop = nn.Dropout(0.0 if det else cfg.tf_en_dropout)
        u = cfg.tf_en_bev_length // 4
        self.motion_encoder = nn.Sequential(
            nn.Linear(cfg.tf_en_motion_length, u), nn.ReLU(inplace=True),
            nn.Linear(u, 2 * u), nn.ReLU(inplace=True),
            nn.Linear(2 * u, cfg.tf_en_bev_length), nn.ReLU(inplace=True))
        for name, p in self.named_parameters():
            if "pos_embed" not in name and p.dim() > 1:
                nn.init.xavier_uniform_(p)
        nn.init.trunc_normal_(self.pos_embed, std=.02)

    def encode_motion(self, ego_motion):
        """motion_encoder (Linear -> ReLU) x 3 with the ReLU in each GEMM's epilogue."""
        x = ego_motion
        for i in (0, 2, 4):
            lin = self.motion_encoder[i]
            x = nn_ops.linear(x, lin.weight, lin.bias, relu=True)
        return x

    def forward(self, bev_feature, ego_motion):
        # cat([bev^T, motion^T expanded]) + pos_embed -> pos_drop as one kernel each way
        # (reference model/feature_fusion.py:41-46)
        motion = self.encode_motion(ego_motion)  # (B, 1, S)
        p = self.pos_drop.p if self.training else 0.0
        tokens = nn_ops.fusion_tokens(bev_feature, motion, self.pos_embed, p)
        return transformer.encoder(self.tf_encoder, tokens)
