"""RecBLR sequential recommender on the MI355X encoder.

Drop-in for the reference's ``RecBLR.py``: same class names, constructor
arguments, config keys (RecBLR.py:22-30), submodule and parameter names
(``item_embedding``, ``recurrent_layers.{i}.behavior_modeling.{input, conv1d,
gates, Lambda, output}``, ``...ffn.{w_1, w_2, layer_norm}``, ...), so RecBole
checkpoints and ``state_dict``s move between the two unchanged.  Modules are
created in the reference's order, so under the same seed the initial weights
are identical too.

What differs is the execution:
* ``GatedRecurrentLayer.forward``: the reference's ~25-kernel chain (pad copy,
  transposes, conv, a dozen elementwise gate ops, Triton scan, truncate,
  merge) is two fused HIP kernels around the gates GEMM (``recurrence.py``);
* embedding -> dropout -> LayerNorm, dropout + residual + LayerNorm and the
  FFN's SiLU + dropout are fused HIP kernels (``blocks.py``), with a
  deterministic sort-based embedding backward;
* projections are MFMA GEMMs with split-K weight gradients (``linear.py``).
Everything needs a ROCm GPU; there is no CPU fallback.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F
from torch import nn

from ._lib import RecBLRNativeError
from .blocks import (ResidualGrad, add_dropout_layer_norm, embed_dropout_layer_norm,
                     feed_forward, linear_add_dropout_layer_norm)
from .kernels import Packed, grl_max_tiles, grl_pieces, pack_plan
from .linear import HipLinearForward, fire_hooks, has_hooks, linear
from .recbole_compat import BPRLoss, SequentialRecommender, install_interaction_hook
from .recurrence import bd_lru, fused_ok, pow2_pad_len, row_pad_lens


from .scoring import full_sort_scores, item_cross_entropy, target_ranks

# RECBLR_CONV_ROWS=0: packed conv forward per sequence instead of per row tile
_CONV_ROWS = os.environ.get("RECBLR_CONV_ROWS", "1") != "0"
class _PinnedRing:
    """A few reusable page-locked staging buffers for the per-batch host ->
    device copy of the packed layout (offsets, order): no pinned allocation
    per step; slot i is reused only after the copy from it has completed
    (its event; only waits if the device runs >= k batches behind).

    Under HIP-graph capture the ring is bypassed: a captured non_blocking
    copy reads its pinned source when the graph is REPLAYED, so a ring slot
    overwritten by a later stage() would change what the graph uploads.  A
    captured stage() therefore copies into a pinned buffer of its own that is
    kept alive (and never rewritten) for the life of the process — the graph
    replays exactly the batch layout it captured."""

    def __init__(self, k: int = 4):
        self.k, self.i = k, 0
        self.bufs = [None] * k
        self.events = [None] * k
        self.captured = []   # pinned sources of captured copies (kept alive)

    def stage(self, host: torch.Tensor, device) -> torch.Tensor:
        if torch.cuda.is_current_stream_capturing():
            buf = torch.empty(host.numel(), dtype=host.dtype, pin_memory=True)
            buf.copy_(host.reshape(-1))
            self.captured.append(buf)
            with torch.cuda.device(device):
                return buf.to(device, non_blocking=True)
        i = self.i
        self.i = (i + 1) % self.k
        n = host.numel()
        buf = self.bufs[i]
        if buf is None or buf.numel() < n or buf.dtype != host.dtype:
            buf = self.bufs[i] = torch.empty(max(n, 4096), dtype=host.dtype, pin_memory=True)
            self.events[i] = None
        if self.events[i] is not None:
            self.events[i].synchronize()
        buf[:n].copy_(host)
        # the copy and its event on the TARGET device's current stream (the
        # current device may be another one)
        with torch.cuda.device(device):
            out = buf[:n].to(device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(device))
        self.events[i] = ev
        return out


_host_ring = _PinnedRing()
_host_ring32 = _PinnedRing()   # int32 staging (the fused kernel's work lists)
_ncus: dict = {}


def _num_cus(dev) -> int:
    n = _ncus.get(dev)
    if n is None:
        n = _ncus[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return n

# RECBLR_LAST_ONLY=0: the last layer's scan writes y at every position
_LAST_ONLY = os.environ.get("RECBLR_LAST_ONLY", "1") != "0"

__all__ = ["RecBLR", "RecurrentLayer", "GatedRecurrentLayer", "FeedForward",
           "softplus_inverse", "lambda_init_range"]


def softplus_inverse(x):
    """log(exp(x) - 1): the Lambda init helper (RecBLR.py:14-15)."""
    return torch.log(torch.exp(x) - 1)


def lambda_init_range(r_min: float = 0.9, r_max: float = 0.999):
    """Lambda endpoints such that exp(-softplus(Lambda)) spans [r_min, r_max]
    (RecBLR.py:153-158), computed in fp32 like the reference."""
    lo = softplus_inverse(torch.tensor(-math.log(r_min))).item()
    hi = softplus_inverse(torch.tensor(-math.log(r_max))).item()
    return lo, hi


class GatedRecurrentLayer(nn.Module):
    """in-proj -> causal conv + SiLU -> BD-LRU gates -> scan -> silu(z)*h -> out-proj.

    Parameters as RecBLR.py:149-167.  ``bd_lru_only`` is stored but, as in the
    reference (:151), does not change this block."""

    def __init__(self, d_model=64, expansion_factor=2, kernel_size=4, bd_lru_only=False,
                 disable_conv1d=False):
        super().__init__()
        self.bd_lru_only = bd_lru_only
        self.disable_conv1d = disable_conv1d
        lo, hi = lambda_init_range()
        hidden = int(d_model * expansion_factor)
        self.hidden = hidden
        self.input = nn.Linear(d_model, 2 * hidden, bias=False)
        self.conv1d = nn.Conv1d(hidden, hidden, kernel_size, groups=hidden,
                                padding=kernel_size - 1, bias=True)
        self.gates = nn.Linear(hidden, 2 * hidden, bias=True)
        self.Lambda = nn.Parameter(torch.linspace(lo, hi, hidden))
        self.output = nn.Linear(hidden, d_model, bias=False)
        # the projections run on the HIP path through their own nn.Linear
        # __call__ (forward hooks fire, the module type stays nn.Linear)
        for m in (self.input, self.output):
            m.forward = HipLinearForward(m)

    def forward(self, x, pad=None, slot=None, rows=None, seq=None, project=True):
        """pad: None (the reference's pow2 pad prefix for x's length) or an
        int64 tensor [B] of per-row pad lengths (see recurrence.bd_lru).
        slot: blocks.ResidualGrad of the enclosing RecurrentLayer.
        rows: flat positions at which the output is needed (the
        out-projection is position-wise, so only those rows are projected;
        returns [len(rows), d]).
        seq: kernels.Packed — x is [ntok, d], the sequences' valid positions
        packed back to back (RecBLR.forward)."""
        if x.device.type != "cuda":
            raise RecBLRNativeError(
                "GatedRecurrentLayer runs only on the MI355X HIP path (ROCm GPU tensors); "
                "move the model to a GPU. The CPU restatement under oracle/ is test-only.")
        self.input._recblr_slot = slot
        xz = self.input(x)
        # the last layer under gather_indexes on packed sequences needs y only
        # at each sequence's last row: the scan kernels keep just those
        last_only = (_LAST_ONLY and rows is not None and seq is not None
                     and rows is seq.last and xz.dtype == torch.float32)
        observe = None
        if has_hooks(self.gates) or has_hooks(self.conv1d):
            def observe(x_, xc, rg):   # hooks of the Linear / Conv1d fused into bd_lru
                if not self.disable_conv1d:
                    fire_hooks(self.conv1d, (x_.transpose(-1, -2),), xc.transpose(-1, -2))
                fire_hooks(self.gates, (xc,), rg + self.gates.bias)
        y = bd_lru(xz, self.conv1d.weight, self.conv1d.bias, self.gates.weight,
                   self.gates.bias, self.Lambda, use_conv=not self.disable_conv1d, pad=pad,
                   seq=seq, last_only=last_only, observe=observe)
        if last_only:
            if seq.order is None:   # packed-sequence order -> batch order
                y = y.index_select(0, seq.inv)
        elif rows is not None:
            y = y.reshape(-1, y.shape[-1]).index_select(0, rows)
        # project=False: y before the out-projection (the caller fuses the
        # projection with its residual LayerNorm, blocks.linear_add_dropout_layer_norm)
        return self.output(y) if project else y

    @staticmethod
    def pad_len(seq_len: int) -> int:
        return pow2_pad_len(seq_len)


class FeedForward(nn.Module):
    """Position-wise FFN with SiLU, residual and LayerNorm (RecBLR.py:210-227)."""

    def __init__(self, d_model, inner_size, dropout=0.2):
        super().__init__()
        self.w_1 = nn.Linear(d_model, inner_size)
        self.w_2 = nn.Linear(inner_size, d_model)
        self.dropout = nn.Dropout(dropout)
        self.layer_norm = nn.LayerNorm(d_model, eps=1e-12)

    def forward(self, input_tensor, in_addend=None, out_addend=None):
        return feed_forward(input_tensor, self, self.training, in_addend, out_addend)


class RecurrentLayer(nn.Module):
    """GRL + dropout + residual LayerNorm, then the FFN (RecBLR.py:124-145)."""

    def __init__(self, d_model, d_conv, expand, dropout, num_layers, bd_lru_only,
                 disable_conv1d, disable_ffn):
        super().__init__()
        self.num_layers = num_layers
        self.disable_ffn = disable_ffn
        self.behavior_modeling = GatedRecurrentLayer(
            d_model=d_model, expansion_factor=expand, kernel_size=d_conv,
            bd_lru_only=bd_lru_only, disable_conv1d=disable_conv1d)
        self.dropout = nn.Dropout(dropout)
        self.layer_norm = nn.LayerNorm(d_model, eps=1e-12)
        self.ffn = FeedForward(d_model=d_model, inner_size=d_model * 4, dropout=dropout)

    def forward(self, input_tensor, pad=None, rows=None, seq=None, slot=None, out_addend=None):
        """rows: evaluate the position-wise tail (out-projection, residual
        LayerNorm, FFN) only at these flat positions -> [len(rows), d].
        seq: kernels.Packed (input_tensor is [ntok, d]).
        slot: blocks.ResidualGrad for the residual branch's gradient (RecBLR
        creates it so that input_tensor's producer can take it);
        out_addend: the next layer's slot (a second gradient of the output)."""
        grad = torch.is_grad_enabled() and input_tensor.requires_grad
        if slot is None and grad:
            slot = ResidualGrad(rows)
        if not grad:
            slot = out_addend = None
        residual = input_tensor
        if rows is not None:
            residual = input_tensor.reshape(-1, input_tensor.shape[-1]).index_select(0, rows)
        out = self.behavior_modeling.output
        # full rows: the out-projection and the residual LayerNorm in one
        # launch where it applies (blocks.linear_add_dropout_layer_norm)
        fuse = rows is None and not has_hooks(out)
        y = self.behavior_modeling(input_tensor, pad, slot, rows, seq, project=not fuse)

        def add_ln(addend):
            if fuse:
                return linear_add_dropout_layer_norm(y, out, residual, self.dropout,
                                                     self.layer_norm, self.training, slot, addend)
            return add_dropout_layer_norm(y, residual, self.dropout, self.layer_norm,
                                          self.training, slot, addend)

        if self.disable_ffn:
            return add_ln(out_addend)
        # the FFN's own residual gradient goes back through h_slot to the
        # LayerNorm that produced h
        h_slot = ResidualGrad() if grad else None
        h = add_ln(h_slot)
        return self.ffn(h, h_slot, out_addend)


# Attribute a data path may set on the item_seq_len device tensor: the same
# lengths as a CPU tensor, so the packed forward needs no device sync to size
# its buffers (distributed.synthetic_interaction, data.SequentialLoader).
HOST_LENGTHS = "_recblr_host_lengths"


def attach_host_lengths(lengths_dev: torch.Tensor, lengths_cpu: torch.Tensor) -> torch.Tensor:
    setattr(lengths_dev, HOST_LENGTHS, lengths_cpu.detach().to("cpu"))
    return lengths_dev


class RecBLR(SequentialRecommender):
    """RecBole sequential recommender with the BD-LRU encoder (RecBLR.py:18-122)."""

    def __init__(self, config, dataset):
        super().__init__(config, dataset)
        self.hidden_size = config["hidden_size"]
        self.loss_type = config["loss_type"]
        self.num_layers = config["num_layers"]
        self.dropout_prob = config["dropout_prob"]
        self.expand = config["expand"]
        self.d_conv = config["d_conv"]
        self.bd_lru_only = config["bd_lru_only"]
        self.disable_conv1d = config["disable_conv1d"]
        self.disable_ffn = config["disable_ffn"]
        if self.bd_lru_only:  # RecBLR.py:33-35
            self.disable_conv1d = True
            self.disable_ffn = True
        # evaluate the last layer's position-wise tail only where gather_indexes
        # reads it (RECBLR_FULL_LAST_LAYER=1: every position, as the reference)
        self.gather_last_layer = os.environ.get("RECBLR_FULL_LAST_LAYER", "0") != "1"
        # run the encoder on each sequence's first item_seq_len positions only,
        # packed back to back (RECBLR_PACKED=0: the dense [B, L] batch, as the
        # reference); identical outputs and gradients, see DESIGN.md
        self.pack_sequences = os.environ.get("RECBLR_PACKED", "1") != "0"

        # run.py's Trainer moves each batch with Interaction.to(device): keep the
        # host lengths on the device tensor (no per-step sync in the packed forward)
        install_interaction_hook(self.ITEM_SEQ_LEN)
        self.item_embedding = nn.Embedding(self.n_items, self.hidden_size, padding_idx=0)
        self.layer_norm = nn.LayerNorm(self.hidden_size, eps=1e-12)
        self.dropout = nn.Dropout(self.dropout_prob)
        self.recurrent_layers = nn.ModuleList(
            RecurrentLayer(d_model=self.hidden_size, d_conv=self.d_conv, expand=self.expand,
                           dropout=self.dropout_prob, num_layers=self.num_layers,
                           bd_lru_only=self.bd_lru_only, disable_conv1d=self.disable_conv1d,
                           disable_ffn=self.disable_ffn)
            for _ in range(self.num_layers))
        if self.loss_type == "BPR":
            self.loss_fct = BPRLoss()
        elif self.loss_type == "CE":
            self.loss_fct = nn.CrossEntropyLoss()
        else:
            raise NotImplementedError("Make sure 'loss_type' in ['BPR', 'CE']!")
        self.apply(self._init_weights)

    @staticmethod
    def _init_weights(module):
        # RecBLR.py:66-73: N(0, 0.02) for Linear/Embedding (every embedding row,
        # padding_idx included), zero Linear biases, LayerNorm (1, 0); the conv
        # keeps PyTorch's default init.
        if isinstance(module, (nn.Linear, nn.Embedding)):
            module.weight.data.normal_(std=0.02)
        elif isinstance(module, nn.LayerNorm):
            module.bias.data.zero_()
            module.weight.data.fill_(1.0)
        if isinstance(module, nn.Linear) and module.bias is not None:
            module.bias.data.zero_()

    def forward(self, item_seq, item_seq_len, exact_lengths: bool = False):
        """RecBLR.py:75-84.  exact_lengths=True makes each row behave as the
        batch-1 forward of its unpadded sequence item_seq[b, :len_b] (its own
        pow2 pad prefix), so users of different lengths batch together
        without changing results (run_with_unseen.py:222-225 runs them one
        by one)."""
        pad = row_pad_lens(item_seq_len) if exact_lengths else None
        if self.pack_sequences:
            return self._forward_packed(item_seq, item_seq_len, pad)
        n = len(self.recurrent_layers)
        rows = None
        if self.gather_last_layer:
            # Everything after the last layer's scan is position-wise and only
            # the positions gather_indexes picks reach the output: evaluate
            # that tail at those B positions (identical results).
            B, L = item_seq.shape
            rows = torch.arange(B, device=item_seq.device) * L + (item_seq_len - 1)
        slots = self._residual_slots(rows)
        h = embed_dropout_layer_norm(item_seq, self.item_embedding, self.dropout, self.layer_norm,
                                     self.training, slots[0])
        for i, layer in enumerate(self.recurrent_layers):
            if i == n - 1 and rows is not None:
                return layer(h, pad, rows, slot=slots[i])
            h = layer(h, pad, slot=slots[i], out_addend=slots[i + 1])
        return self.gather_indexes(h, item_seq_len - 1)

    def _residual_slots(self, last_rows):
        """One blocks.ResidualGrad per layer (+ None): layer i's residual
        gradient, taken by its input's producer (slot i is handed to that
        producer as its out_addend)."""
        n = len(self.recurrent_layers)
        if not torch.is_grad_enabled():
            return [None] * (n + 1)
        return [ResidualGrad(last_rows if i == n - 1 else None) for i in range(n)] + [None]

    def _forward_packed(self, item_seq, item_seq_len, pad):
        """forward() on the valid positions only.  RecBole right-pads every
        sequence to L; the encoder is causal (causal conv, forward scan,
        position-wise projections / LayerNorms / FFN), so position t of row b
        influences only positions >= t of that row, and forward() returns
        position len_b - 1 (gather_indexes, RecBLR.py:84).  Positions >= len_b
        therefore never reach the output or any gradient; they are dropped
        before the embedding and the sequences run packed back to back
        ([ntok, d], ntok = sum of lengths; the recurrence kernels take the
        per-sequence offsets).  The pow2 pad prefix still uses the batch's L."""
        B, L = item_seq.shape
        dev = item_seq.device
        # sequences are packed longest first: the recurrence kernels give one
        # wave per sequence, so the short ones fill in behind the long ones
        host = getattr(item_seq_len, HOST_LENGTHS, None)
        if host is None or host.shape != item_seq_len.shape:
            # lengths only on the device: one sync (RecBole's Trainer path
            # attaches them instead, recbole_compat.install_interaction_hook)
            host = item_seq_len.to("cpu")
        lens_h = host.to(torch.int64).clamp(1, L)
        order_h = torch.argsort(lens_h, descending=True, stable=True)
        offs_h = torch.zeros(B + 1, dtype=torch.int64)
        lens_p = lens_h[order_h]
        torch.cumsum(lens_p, 0, out=offs_h[1:])
        ntok = int(offs_h[-1])
        both = _host_ring.stage(torch.cat([offs_h, order_h]), dev)
        offsets, order = both[:B + 1], both[B + 1:]
        pieces = None
        H = self.hidden_size * self.expand
        if fused_ok(True, H, not self.disable_conv1d, self.d_conv, torch.float32):
            G = _num_cus(dev)
            pieces = _host_ring32.stage(grl_pieces(lens_p, offs_h, G), dev)
            max_tiles = grl_max_tiles(lens_p, G)
        # one launch (rb_pack_plan): the packed item ids, each token's position
        # in its sequence (lets the conv forward tile the packed rows), each
        # batch row's packed index and last token
        ids, pos, inv, last = pack_plan(item_seq.to(torch.int64), offsets, order, ntok)
        seq = Packed(offsets, L, ntok, pos if _CONV_ROWS else None)
        seq.last, seq.inv, seq.order = last, inv, order
        if pieces is not None and pad is None:   # per-row pad prefixes: three-launch path
            seq.pieces, seq.G, seq.max_tiles = pieces, G, max_tiles
        if pad is not None:
            pad = pad.index_select(0, order)
        n = len(self.recurrent_layers)
        slots = self._residual_slots(last if self.gather_last_layer else None)
        h = embed_dropout_layer_norm(ids, self.item_embedding, self.dropout, self.layer_norm,
                                     self.training, slots[0])
        for i, layer in enumerate(self.recurrent_layers):
            if i == n - 1 and self.gather_last_layer:
                return layer(h, pad, last, seq, slot=slots[i])
            h = layer(h, pad, seq=seq, slot=slots[i], out_addend=slots[i + 1])
        return h.index_select(0, last)

    def _scores_all(self, seq_output):
        return full_sort_scores(seq_output, self.item_embedding.weight)

    def calculate_loss(self, interaction):
        seq_output = self.forward(interaction[self.ITEM_SEQ], interaction[self.ITEM_SEQ_LEN])
        pos_items = interaction[self.POS_ITEM_ID]
        if self.loss_type == "BPR":
            neg_items = interaction[self.NEG_ITEM_ID]
            pos_score = (seq_output * self.item_embedding(pos_items)).sum(-1)
            neg_score = (seq_output * self.item_embedding(neg_items)).sum(-1)
            return self.loss_fct(pos_score, neg_score)
        # logits + nn.CrossEntropyLoss fused on MFMA, [B, n_items] never stored
        return item_cross_entropy(seq_output, self.item_embedding.weight, pos_items)

    def predict(self, interaction):
        seq_output = self.forward(interaction[self.ITEM_SEQ], interaction[self.ITEM_SEQ_LEN])
        return (seq_output * self.item_embedding(interaction[self.ITEM_ID])).sum(dim=1)

    def full_sort_predict(self, interaction):
        seq_output = self.forward(interaction[self.ITEM_SEQ], interaction[self.ITEM_SEQ_LEN])
        return self._scores_all(seq_output)

    def full_sort_rank(self, interaction, first_item: int = 1):
        """Rank of each row's target (POS_ITEM_ID) under full_sort_predict's
        scores without materialising them: (n_greater, n_equal) over items
        [first_item, n_items) (item 0 is RecBole's padding id, masked to -inf
        by its full-sort evaluator)."""
        seq_output = self.forward(interaction[self.ITEM_SEQ], interaction[self.ITEM_SEQ_LEN])
        return target_ranks(seq_output, self.item_embedding.weight,
                            interaction[self.POS_ITEM_ID], first_item)
