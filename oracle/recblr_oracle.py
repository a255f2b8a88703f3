"""CPU oracle for the RecBLR hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / CPU baseline; the product
(datamining_recblr_amd) never calls it and has no CPU fallback.

This is a plain fp32 PyTorch (CPU) restatement of the reference algorithm,
written functionally over a ``state_dict``-style parameter mapping:

* ``serial_scan`` / ``SerialScan``: the first-order recurrence of
  parallel_scan.py:44-60 (forward) and parallel_scan.py:97-114 (backward:
  shifted gates with a trailing 1, reverse scan, d_gates = [0, h_0..h_{T-2}]
  * d).  Evaluated serially, multiply then add (no FMA, as the reference's
  ``enable_fp_fusion=False``, :92).
* ``grl_forward``: GatedRecurrentLayer.forward, RecBLR.py:170-207, including
  the materialised power-of-two left padding (:176-179), the padded conv via
  F.conv1d + SiLU (:185, the reference's fallback when causal_conv1d is
  absent), the gate formulas (:196-199), the [B, C, T] transposes around the
  scan (:200) and the truncation (:203-204).
* ``ffn_forward`` (RecBLR.py:218-227), ``recurrent_layer_forward`` (:140-145),
  ``model_forward`` (:75-84), ``calculate_loss`` (:86-103), ``predict``
  (:105-112), ``full_sort_predict`` (:114-122).

Pinning: tests/test_oracle_golden.py checks this module against golden
vectors produced by running the reference itself (Triton interpreter scan,
reference RecBLR module) — see tests/golden/make_golden.py.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

__all__ = ["serial_scan", "SerialScan", "oracle_parallel_scan", "grl_forward", "ffn_forward",
           "recurrent_layer_forward", "model_forward", "calculate_loss", "predict",
           "full_sort_predict", "pow2_pad_len"]


def serial_scan(gates: torch.Tensor, tokens: torch.Tensor) -> torch.Tensor:
    """h_t = gates_t * h_{t-1} + tokens_t over the last axis, h_{-1} = 0."""
    T = gates.shape[-1]
    out = torch.empty_like(tokens)
    h = torch.zeros_like(tokens[..., 0])
    for t in range(T):
        h = h * gates[..., t]
        h = h + tokens[..., t]
        out[..., t] = h
    return out


def _serial_scan_reverse(gates: torch.Tensor, grad: torch.Tensor) -> torch.Tensor:
    """d_t = d_{t+1} * gates_t + grad_t running from the end (gates pre-shifted)."""
    T = gates.shape[-1]
    out = torch.empty_like(grad)
    d = torch.zeros_like(grad[..., 0])
    for t in range(T - 1, -1, -1):
        d = d * gates[..., t]
        d = d + grad[..., t]
        out[..., t] = d
    return out


class SerialScan(torch.autograd.Function):
    """Serial-order autograd twin of the reference ``Scan`` (parallel_scan.py:83-114)."""

    @staticmethod
    def forward(ctx, gates, tokens):
        states = serial_scan(gates, tokens)
        ctx.save_for_backward(states, gates)
        return states

    @staticmethod
    def backward(ctx, grad_output):
        states, gates = ctx.saved_tensors
        grad_output = grad_output.contiguous()
        shifted = torch.cat([gates[..., 1:], torch.ones_like(gates[..., :1])], dim=-1)
        d_states = _serial_scan_reverse(shifted, grad_output)
        prev = torch.cat([torch.zeros_like(states[..., :1]), states[..., :-1]], dim=-1)
        return prev * d_states, d_states


def oracle_parallel_scan(gates, tokens):
    return SerialScan.apply(gates, tokens)


def pow2_pad_len(seq_len: int) -> int:
    return 2 ** ((seq_len - 1).bit_length()) - seq_len


def grl_forward(p, prefix: str, x: torch.Tensor, disable_conv1d: bool = False) -> torch.Tensor:
    """GatedRecurrentLayer.forward (RecBLR.py:170-207) on parameters p[prefix + name]."""
    W_in = p[prefix + "input.weight"]
    conv_w = p[prefix + "conv1d.weight"]
    conv_b = p[prefix + "conv1d.bias"]
    W_g = p[prefix + "gates.weight"]
    b_g = p[prefix + "gates.bias"]
    lam = p[prefix + "Lambda"]
    W_out = p[prefix + "output.weight"]
    seq_len = x.shape[1]
    H = lam.shape[0]
    k = conv_w.shape[-1]

    xz = x @ W_in.t()
    u, z = xz[..., :H], xz[..., H:]
    P = pow2_pad_len(seq_len)
    if P:
        u = torch.cat([u.new_zeros(u.shape[0], P, H), u], dim=1)
    T = seq_len + P
    if not disable_conv1d:
        conv = F.conv1d(u.transpose(1, 2), conv_w, conv_b, padding=k - 1, groups=H)
        u = F.silu(conv[..., :T].transpose(1, 2))
    r, i = (u @ W_g.t() + b_g).split(H, dim=-1)
    alpha = torch.exp(-F.softplus(lam) * torch.sigmoid(r))
    beta = torch.sqrt(1 - alpha.pow(2) + 1e-8) * torch.sigmoid(i)
    h = SerialScan.apply(alpha.transpose(1, 2).contiguous(),
                         (beta * u).transpose(1, 2).contiguous()).transpose(1, 2)
    h = h[:, P:]
    return (F.silu(z) * h) @ W_out.t()


def _layer_norm(p, prefix, x):
    return F.layer_norm(x, (x.shape[-1],), p[prefix + "weight"], p[prefix + "bias"], eps=1e-12)


def _drop(x, p_drop):
    """nn.Dropout in train mode (p_drop > 0) or eval (identity)."""
    return F.dropout(x, p_drop, training=True) if p_drop > 0 else x


def ffn_forward(p, prefix: str, x: torch.Tensor, p_drop: float = 0.0) -> torch.Tensor:
    """FeedForward.forward (RecBLR.py:218-227); dropout after the SiLU (:221)
    and after w_2 (:224) when p_drop > 0 (train mode), identity otherwise."""
    h = _drop(F.silu(x @ p[prefix + "w_1.weight"].t() + p[prefix + "w_1.bias"]), p_drop)
    h = _drop(h @ p[prefix + "w_2.weight"].t() + p[prefix + "w_2.bias"], p_drop)
    return _layer_norm(p, prefix + "layer_norm.", h + x)


def recurrent_layer_forward(p, prefix: str, x, disable_conv1d=False, disable_ffn=False,
                            p_drop: float = 0.0):
    """RecurrentLayer.forward (RecBLR.py:140-145); dropout on the GRL output
    (:142) when p_drop > 0."""
    h = _drop(grl_forward(p, prefix + "behavior_modeling.", x, disable_conv1d), p_drop)
    h = _layer_norm(p, prefix + "layer_norm.", h + x)
    return h if disable_ffn else ffn_forward(p, prefix + "ffn.", h, p_drop)


def _flags(cfg):
    dc, df = bool(cfg.get("disable_conv1d", False)), bool(cfg.get("disable_ffn", False))
    if cfg.get("bd_lru_only", False):
        dc = df = True
    return dc, df


def model_forward(p, cfg, item_seq, item_seq_len, p_drop: float = 0.0):
    """RecBLR.forward (RecBLR.py:75-84) -> seq_output [B, d]; eval mode, or
    train-mode dropout at the reference's four sites when p_drop > 0 (used
    only by bench.py's CPU baseline, whose timed step matches the GPU's)."""
    dc, df = _flags(cfg)
    emb = _drop(F.embedding(item_seq, p["item_embedding.weight"], padding_idx=0), p_drop)
    h = _layer_norm(p, "layer_norm.", emb)
    for li in range(cfg["num_layers"]):
        h = recurrent_layer_forward(p, f"recurrent_layers.{li}.", h, dc, df, p_drop)
    idx = (item_seq_len - 1).view(-1, 1, 1).expand(-1, -1, h.shape[-1])
    return h.gather(1, idx).squeeze(1)


def calculate_loss(p, cfg, item_seq, item_seq_len, pos_items, neg_items=None,
                   p_drop: float = 0.0):
    """RecBLR.calculate_loss (RecBLR.py:86-103): CE over all items, or BPR."""
    seq = model_forward(p, cfg, item_seq, item_seq_len, p_drop)
    table = p["item_embedding.weight"]
    if cfg["loss_type"] == "BPR":
        pos = (seq * table[pos_items]).sum(-1)
        neg = (seq * table[neg_items]).sum(-1)
        return -torch.log(1e-10 + torch.sigmoid(pos - neg)).mean()
    return F.cross_entropy(seq @ table.t(), pos_items)


def predict(p, cfg, item_seq, item_seq_len, test_item):
    seq = model_forward(p, cfg, item_seq, item_seq_len)
    return (seq * p["item_embedding.weight"][test_item]).sum(dim=1)


def full_sort_predict(p, cfg, item_seq, item_seq_len):
    return model_forward(p, cfg, item_seq, item_seq_len) @ p["item_embedding.weight"].t()
