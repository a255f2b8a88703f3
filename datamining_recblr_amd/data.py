"""Sequential-recommendation data path for real-data runs (RecBole semantics).

The reference trains through RecBole 1.2.0 (run.py:60-80: create_dataset,
data_preparation, Trainer) with config.yaml: atomic ``.inter`` file with
columns user_id / item_id / timestamp, ``user_inter_num_interval`` and
``item_inter_num_interval`` "[5,inf)", ``MAX_ITEM_LIST_LENGTH`` 200,
``train_batch_size`` 2048, leave-one-out evaluation with full ranking.
RecBole is not installable here, so this module restates its published
algorithm (parity unpinned: no RecBole fixtures exist in the reference):

  1. load the atomic file (header ``name:type`` per column, tab separated);
  2. iterative k-core filtering of users and items by interaction count;
  3. token -> id remapping, ids from 1 in order of first appearance
     (0 is ``[PAD]``);
  4. per user, interactions in (timestamp, file order); every prefix
     i_1..i_{k-1} -> i_k (k >= 2) is one sample, the prefix truncated to the
     last MAX_ITEM_LIST_LENGTH items;
  5. leave-one-out by time (RecBole's 'LS': 'valid_and_test'): of a user's
     c samples the last min(2, c-1) are held out - the last -> test, the one
     before -> valid - and the rest train.

Samples are kept as (offset, end) descriptors into one flat item array that
lives in HBM; batches are assembled on the GPU by index arithmetic
(``build_batch``), so the training loop never touches host memory.
Data parallelism: ``SequentialLoader`` deals each epoch's shuffled sample
order round-robin to the ranks (DistributedSampler semantics, identical
permutation on every rank).
"""
from __future__ import annotations

import io
from dataclasses import dataclass

import numpy as np
import torch

__all__ = ["load_atomic", "kcore_filter", "remap_tokens", "SequentialData", "build_sequential",
           "build_batch", "SequentialLoader", "write_atomic", "from_atomic_file"]


def load_atomic(path: str, columns=("user_id", "item_id", "timestamp")) -> dict:
    """RecBole atomic file -> {column name: numpy array}.  Token columns stay
    strings (object arrays), float columns become float64."""
    import pandas as pd

    with open(path, "r", encoding="utf-8") as f:
        header = f.readline().rstrip("\n").split("\t")
    names, types = [], {}
    for h in header:
        name, _, typ = h.partition(":")
        names.append(name)
        types[name] = typ or "token"
    want = [c for c in columns if c in names]
    dtype = {n: (str if types[n].startswith("token") else float) for n in want}
    df = pd.read_csv(path, sep="\t", header=0, names=names, usecols=want, dtype=dtype,
                     engine="c", keep_default_na=False)
    return {c: df[c].to_numpy() for c in want}


def write_atomic(path: str, cols: dict) -> None:
    """Write {name: array} as a RecBole atomic file (token for str/int, float)."""
    names = list(cols)
    typ = ["float" if np.asarray(cols[n]).dtype.kind == "f" else "token" for n in names]
    buf = io.StringIO()
    buf.write("\t".join(f"{n}:{t}" for n, t in zip(names, typ)) + "\n")
    rows = zip(*[np.asarray(cols[n]) for n in names])
    for r in rows:
        buf.write("\t".join(str(x) for x in r) + "\n")
    with open(path, "w", encoding="utf-8") as f:
        f.write(buf.getvalue())


def kcore_filter(users: np.ndarray, items: np.ndarray, min_user: int = 5, min_item: int = 5):
    """Boolean keep-mask of the interactions surviving iterative k-core
    filtering (users with < min_user and items with < min_item interactions
    removed until nothing changes)."""
    keep = np.ones(len(users), dtype=bool)
    _, uinv = np.unique(users, return_inverse=True)
    _, iinv = np.unique(items, return_inverse=True)
    while True:
        ucnt = np.bincount(uinv[keep], minlength=uinv.max() + 1 if len(uinv) else 0)
        icnt = np.bincount(iinv[keep], minlength=iinv.max() + 1 if len(iinv) else 0)
        bad = keep & ((ucnt[uinv] < min_user) | (icnt[iinv] < min_item))
        if not bad.any():
            return keep
        keep &= ~bad


def remap_tokens(tokens: np.ndarray):
    """ids (int64, from 1 in order of first appearance) and id -> token
    (index 0 = "[PAD]")."""
    _, first, inv = np.unique(tokens, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")          # unique tokens by first appearance
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    ids = rank[inv].astype(np.int64) + 1
    id2token = np.concatenate([np.array(["[PAD]"], dtype=object),
                               np.asarray(tokens, dtype=object)[first[order]]])
    return ids, id2token


@dataclass
class SequentialData:
    """Flat per-user item sequences and (offset, end) sample descriptors."""
    items: torch.Tensor          # [N] int64, users' interactions back to back (time order)
    user_of: torch.Tensor        # [N] int64 user id of each position
    train: torch.Tensor          # [S, 2] int64 (start of user's run, target position)
    valid: torch.Tensor
    test: torch.Tensor
    n_items: int                 # including [PAD]
    n_users: int
    max_len: int
    item_tokens: np.ndarray
    user_tokens: np.ndarray

    def to(self, device):
        for f in ("items", "user_of", "train", "valid", "test"):
            setattr(self, f, getattr(self, f).to(device))
        return self


def build_sequential(cols: dict, max_len: int = 200, min_user: int = 5, min_item: int = 5,
                     user_field: str = "user_id", item_field: str = "item_id",
                     time_field: str = "timestamp") -> SequentialData:
    users, items = np.asarray(cols[user_field]), np.asarray(cols[item_field])
    ts = np.asarray(cols[time_field], dtype=np.float64) if time_field in cols else \
        np.arange(len(users), dtype=np.float64)
    keep = kcore_filter(users, items, min_user, min_item)
    users, items, ts = users[keep], items[keep], ts[keep]
    uid, utok = remap_tokens(users)
    iid, itok = remap_tokens(items)
    # per user, by time; ties keep file order
    order = np.lexsort((np.arange(len(uid)), ts, uid))
    uid, iid = uid[order], iid[order]
    n = len(uid)
    starts = np.flatnonzero(np.r_[True, uid[1:] != uid[:-1]]) if n else np.zeros(0, np.int64)
    ends = np.r_[starts[1:], n] if n else np.zeros(0, np.int64)
    pos = np.arange(n)
    run_start = np.repeat(starts, ends - starts)
    k = pos - run_start                                # position inside the user's run
    run_len = np.repeat(ends - starts, ends - starts)
    is_sample = k >= 1
    cnt = run_len - 1                                  # samples of the user
    test = is_sample & (k == run_len - 1) & (cnt >= 2)
    valid = is_sample & (k == run_len - 2) & (cnt >= 3)
    train = is_sample & ~test & ~valid

    def desc(mask):
        return torch.from_numpy(np.stack([run_start[mask], pos[mask]], 1).astype(np.int64))

    return SequentialData(items=torch.from_numpy(iid.astype(np.int64)),
                          user_of=torch.from_numpy(uid.astype(np.int64)),
                          train=desc(train), valid=desc(valid), test=desc(test),
                          n_items=len(itok), n_users=len(utok), max_len=max_len,
                          item_tokens=itok, user_tokens=utok)


def build_batch(data: SequentialData, desc: torch.Tensor) -> dict:
    """RecBole-shaped interaction for samples desc [B, 2] = (run start, target
    position): item_id_list [B, max_len] (the last <= max_len items before
    the target, left-aligned, right-padded with 0), item_length, item_id,
    user_id.  Pure index arithmetic on desc's device."""
    start, tpos = desc[:, 0], desc[:, 1]
    length = torch.clamp(tpos - start, max=data.max_len)
    first = tpos - length
    ar = torch.arange(data.max_len, device=desc.device)
    idx = first[:, None] + ar[None, :]
    inside = ar[None, :] < length[:, None]
    seq = torch.where(inside, data.items[idx.clamp(max=len(data.items) - 1)],
                      torch.zeros((), dtype=torch.int64, device=desc.device))
    return {"item_id_list": seq, "item_length": length, "item_id": data.items[tpos],
            "user_id": data.user_of[tpos]}


class SequentialLoader:
    """Batches of one split.  shuffle: a fresh permutation per epoch from
    (seed, epoch), identical on every rank; rank r takes positions r, r+W, ...
    (DistributedSampler); drop_last keeps per-rank batch counts equal."""

    def __init__(self, data: SequentialData, split: str = "train", batch_size: int = 2048,
                 shuffle: bool = True, seed: int = 2020, rank: int = 0, world: int = 1,
                 drop_last: bool = False):
        self.data, self.desc = data, getattr(data, split)
        self.batch_size, self.shuffle, self.seed = batch_size, shuffle, seed
        self.rank, self.world, self.drop_last = rank, world, drop_last
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def _indices(self):
        n = self.desc.shape[0]
        if self.shuffle:
            g = torch.Generator(device="cpu").manual_seed(self.seed * 1000003 + self.epoch)
            perm = torch.randperm(n, generator=g)
        else:
            perm = torch.arange(n)
        per = n // self.world if self.drop_last else -(-n // self.world)
        if not self.drop_last and per * self.world > n:   # pad by wrapping, as DistributedSampler
            perm = torch.cat([perm, perm[:per * self.world - n]])
        return perm[self.rank:per * self.world:self.world]

    def __len__(self):
        n = len(self._indices())
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        from .model import attach_host_lengths
        idx_h = self._indices()
        idx = idx_h.to(self.desc.device)
        desc_h = self.desc.cpu()
        nb = len(self)
        for b in range(nb):
            sel = idx[b * self.batch_size:(b + 1) * self.batch_size]
            batch = build_batch(self.data, self.desc[sel])
            # the same lengths on the host: the packed forward sizes its buffers
            # from them without a device sync
            dh = desc_h[idx_h[b * self.batch_size:(b + 1) * self.batch_size]]
            attach_host_lengths(batch["item_length"],
                                torch.clamp(dh[:, 1] - dh[:, 0], max=self.data.max_len))
            yield batch


def from_atomic_file(path: str, max_len: int = 200, min_user: int = 5,
                     min_item: int = 5) -> SequentialData:
    return build_sequential(load_atomic(path), max_len=max_len, min_user=min_user,
                            min_item=min_item)

