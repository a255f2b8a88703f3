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


class SyntheticDataset:
    """Dataset stand-in exposing ``num(field)`` (all the model reads)."""

    def __init__(self, n_items: int, n_users: int = 1):
        self._n = {"item_id": n_items, "user_id": n_users}

    def num(self, field):
        return self._n[field]
