"""Control-token decoder: embedding + 4-layer transformer decoder + vocabulary projection.

Mirrors reference model/control_predict.py:8-75 (keys: embedding, pos_embed, tf_decoder.*,
output).  `forward` is the teacher-forced training path, `predict` one autoregressive step
(pads to tf_de_tgt_dim-1 tokens and reads the logits at the last real position)."""
import torch
from torch import nn

from e2ep_amd import _lib, nn_ops, transformer


class ControlPredict(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.pad_idx = cfg.token_nums - 1
        det = getattr(cfg, "deterministic", False)
        self.embedding = nn.Embedding(cfg.token_nums, cfg.tf_de_dim)
        self.pos_drop = nn.Dropout(0.0 if det else cfg.tf_de_dropout)
        self.pos_embed = nn.Parameter(torch.randn(1, cfg.tf_de_tgt_dim - 1, cfg.tf_de_dim) * .02)
        layer = nn.TransformerDecoderLayer(d_model=cfg.tf_de_dim, nhead=cfg.tf_de_heads,
                                           dropout=0.0 if det else 0.1)
        self.tf_decoder = nn.TransformerDecoder(layer, num_layers=cfg.tf_de_layers)
        self.output = nn.Linear(cfg.tf_de_dim, cfg.token_nums)
        for name, p in self.named_parameters():
            if "pos_embed" not in name and p.dim() > 1:
                nn.init.xavier_uniform_(p)
        nn.init.trunc_normal_(self.pos_embed, std=.02)

    def create_mask(self, tgt):
        """Causal float mask (0 on/below the diagonal, -inf above) + PAD key mask."""
        L = tgt.shape[1]
        # built once per (length, device): the fused attention takes causality as a flag, so
        # the tensor only identifies the mask (two kernel launches per step saved)
        if getattr(self, "_causal_key", None) != (L, tgt.device):
            self._causal_mask = torch.full((L, L), float("-inf"), device=tgt.device).triu(1)
            self._causal_key = (L, tgt.device)
        pad = nn_ops.eq_mask(tgt, self.pad_idx) if tgt.is_cuda else tgt == self.pad_idx
        return self._causal_mask, pad

    def decoder(self, encoder_out, tgt_embedding, tgt_mask, tgt_padding_mask):
        # A mask made by create_mask is known to be causal: saying so skips torch's
        # device->host comparison of the mask (a sync that also breaks HIP-graph capture);
        # torch reaches the same decision (causal) by that comparison in the reference.
        causal = True if tgt_mask is getattr(self, "_causal_mask", None) else None
        return transformer.decoder(self.tf_decoder, tgt_embedding, encoder_out, tgt_mask,
                                   tgt_padding_mask, causal)

    def forward(self, encoder_out, tgt):
        tgt = tgt[:, :-1]
        mask, pad = self.create_mask(tgt)
        # embedding + pos_embed -> pos_drop as one kernel each way
        p = self.pos_drop.p if self.training else 0.0
        emb = nn_ops.embed_tokens(tgt, self.embedding.weight, self.pos_embed, p)
        return self.project(self.decoder(encoder_out, emb, mask, pad))

    def project(self, x):
        """self.output (vocabulary projection) on e2ep_gemm."""
        return nn_ops.linear(x, self.output.weight, self.output.bias)

    def predict(self, encoder_out, tgt):
        length = tgt.size(1)
        pad = torch.full((tgt.size(0), self.cfg.tf_de_tgt_dim - length - 1), self.pad_idx,
                         dtype=torch.long, device=tgt.device)
        tgt = torch.cat([tgt, pad], dim=1)
        mask, padm = self.create_mask(tgt)
        emb = nn_ops.embed_tokens(tgt, self.embedding.weight, self.pos_embed)
        logits = self.project(self.decoder(encoder_out, emb, mask, padm))[:, length - 1, :]
        return torch.softmax(logits, dim=-1).argmax(dim=-1).view(-1, 1)

    def predict_tokens(self, encoder_out, toks, steps):
        """`steps` autoregressive predict() calls, each appending its token — the loop of
        reference model/parking_model.py:72-78 over model/control_predict.py:60-75 — on one
        persistent sequence buffer: the PAD padding, softmax, argmax and torch.cat of every
        step are two e2ep launches in all (e2ep_tokens_init once, e2ep_token_argmax_append per
        step), no host sync, HIP-graph capturable.  Returns the (B, L + steps) tokens (a view
        of the buffer)."""
        B, L = toks.shape
        T = self.cfg.tf_de_tgt_dim - 1
        if not (toks.is_cuda and toks.dtype == torch.long and L + steps <= T and steps > 0):
            for _ in range(steps):  # the reference's own loop (it raises where L + steps > T)
                toks = torch.cat([toks, self.predict(encoder_out, toks)], dim=1)
            return toks
        seq = torch.empty((B, T), dtype=torch.long, device=toks.device)
        s = _lib.stream()
        _lib.call("e2ep_tokens_init", _lib.ptr(toks), toks.stride(0), B, L, _lib.ptr(seq), T,
                  self.pad_idx, s)
        mask = None
        for i in range(steps):
            length = L + i
            mask, padm = self.create_mask(seq)
            emb = nn_ops.embed_tokens(seq, self.embedding.weight, self.pos_embed)
            logits = self.project(self.decoder(encoder_out, emb, mask, padm))
            V = logits.shape[-1]
            row = logits[:, length - 1, :]
            if row.stride(1) != 1:
                row = row.contiguous()
            _lib.call("e2ep_token_argmax_append", _lib.ptr(row), row.stride(0), B, V,
                      _lib.ptr(seq), T, length, _lib.stream())
        return seq[:, :L + steps]
