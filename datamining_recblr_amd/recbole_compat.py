"""RecBole 1.2.0 boundary.

``RecBLR`` subclasses RecBole's ``SequentialRecommender`` (reference
RecBLR.py:4,18).  When RecBole is importable we use its classes unchanged, so
``run.py``'s Trainer, ``get_flops`` and checkpointing see a genuine RecBole
model.  RecBole is not installed in this image, so a minimal stand-in with the
same attributes and ``gather_indexes`` semantics is provided for tests,
benchmarks and direct use.
"""
from __future__ import annotations

from logging import getLogger

import torch
from torch import nn

try:  # pragma: no cover - RecBole is absent in this image
    from recbole.model.abstract_recommender import SequentialRecommender  # type: ignore
    from recbole.model.loss import BPRLoss  # type: ignore
    HAVE_RECBOLE = True
except ImportError:
    HAVE_RECBOLE = False

    def _cfg(config, key, default):
        try:
            v = config[key]
        except (KeyError, TypeError):
            return default
        return default if v is None else v

    class SequentialRecommender(nn.Module):  # type: ignore[no-redef]
        """Stand-in for recbole.model.abstract_recommender.SequentialRecommender.

        Field names follow RecBole's defaults (USER_ID_FIELD, ITEM_ID_FIELD,
        LIST_SUFFIX, ITEM_LIST_LENGTH_FIELD, NEG_PREFIX); ``dataset`` only needs
        ``num(field)``."""

        def __init__(self, config, dataset):
            super().__init__()
            self.logger = getLogger()
            self.USER_ID = _cfg(config, "USER_ID_FIELD", "user_id")
            self.ITEM_ID = _cfg(config, "ITEM_ID_FIELD", "item_id")
            self.ITEM_SEQ = self.ITEM_ID + _cfg(config, "LIST_SUFFIX", "_list")
            self.ITEM_SEQ_LEN = _cfg(config, "ITEM_LIST_LENGTH_FIELD", "item_length")
            self.POS_ITEM_ID = self.ITEM_ID
            self.NEG_ITEM_ID = _cfg(config, "NEG_PREFIX", "neg_") + self.ITEM_ID
            self.max_seq_length = _cfg(config, "MAX_ITEM_LIST_LENGTH", 50)
            self.n_items = dataset.num(self.ITEM_ID)
            self.device = _cfg(config, "device", "cpu")

        def gather_indexes(self, output, gather_index):
            """output[b, gather_index[b], :] for every b."""
            idx = gather_index.view(-1, 1, 1).expand(-1, -1, output.shape[-1])
            return output.gather(dim=1, index=idx).squeeze(1)

        def other_parameter(self):
            return None

        def load_other_parameter(self, para):
            return None

        def __str__(self):
            n = sum(p.numel() for p in self.parameters() if p.requires_grad)
            return super().__str__() + f"\nTrainable parameters: {n}"

    class BPRLoss(nn.Module):  # type: ignore[no-redef]
        """-log(gamma + sigmoid(pos - neg)), averaged (RecBole's BPRLoss)."""

        def __init__(self, gamma: float = 1e-10):
            super().__init__()
            self.gamma = gamma

        def forward(self, pos_score, neg_score):
            return -torch.log(self.gamma + torch.sigmoid(pos_score - neg_score)).mean()


def _attach_lengths(src: dict, out: dict, field: str) -> None:
    """out[field] (a device tensor) gets the host copy src[field] attached
    (model.HOST_LENGTHS): the packed forward then sizes its buffers without
    a device sync."""
    from .model import attach_host_lengths

    s, o = src.get(field), out.get(field)
    if (isinstance(s, torch.Tensor) and isinstance(o, torch.Tensor) and s.device.type == "cpu"
            and o.device.type != "cpu"):
        attach_host_lengths(o, s)


def install_interaction_hook(field: str = "item_length") -> bool:
    """Make RecBole's ``Interaction.to(device)`` keep a host copy of the
    sequence lengths on the device tensor it returns (run.py's Trainer moves
    every CPU batch to the GPU with it right before ``calculate_loss``,
    RecBLR.py:86; recbole/data/interaction.py).  Without it the packed
    forward reads the token count from the device: one sync per step, which
    stops the host from queueing ahead (bench.py's device_lengths: +1.2 ms
    per step).  Idempotent; returns False when RecBole is absent."""
    try:  # pragma: no cover - RecBole is absent in this image
        from recbole.data.interaction import Interaction as _RI  # type: ignore
    except ImportError:
        return False
    if getattr(_RI.to, "_recblr_hooked", False):  # pragma: no cover
        return True
    orig = _RI.to

    def to(self, device, selected_field=None):  # pragma: no cover
        ret = orig(self, device, selected_field)
        _attach_lengths(self.interaction, ret.interaction, field)
        return ret

    to._recblr_hooked = True  # pragma: no cover
    _RI.to = to  # pragma: no cover
    return True  # pragma: no cover


class Interaction:
    """Minimal stand-in for recbole.data.interaction.Interaction: a dict of
    tensors with ``to(device)`` — which, like the installed hook on RecBole's
    own class (install_interaction_hook), attaches the host copy of the
    sequence lengths to the device tensor it creates."""

    LENGTH_FIELD = "item_length"

    def __init__(self, interaction: dict):
        self.interaction = dict(interaction)

    def __getitem__(self, key):
        return self.interaction[key]

    def __contains__(self, key):
        return key in self.interaction

    def keys(self):
        return self.interaction.keys()

    def to(self, device, selected_field=None):
        keys = self.interaction.keys() if selected_field is None else selected_field
        out = {k: (v.to(device) if k in keys and isinstance(v, torch.Tensor) else v)
               for k, v in self.interaction.items()}
        _attach_lengths(self.interaction, out, self.LENGTH_FIELD)
        return Interaction(out)


class SyntheticDataset:
    """Dataset stand-in exposing ``num(field)`` (all the model reads)."""

    def __init__(self, n_items: int, n_users: int = 1):
        self._n = {"item_id": n_items, "user_id": n_users}

    def num(self, field):
        return self._n[field]
