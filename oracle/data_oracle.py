"""CPU restatement of RecBole 1.2.0's sequential data preparation, loop by
loop (TEST INFRASTRUCTURE ONLY - imported by tests/, never by the package).

RecBole is not part of the reference tree and cannot be installed here, so
this follows its published algorithm as the reference's config.yaml drives
it (parity unpinned: no RecBole fixture exists):
  - Dataset._filter_by_inter_num: users/items below the
    user_inter_num_interval / item_inter_num_interval minimum are removed,
    repeatedly until nothing changes;
  - Dataset._remap: ids from 1 by first appearance, 0 = [PAD];
  - SequentialDataset.data_augmentation: interactions sorted by
    (user, timestamp); each prefix predicts the next item, prefix truncated
    to the last MAX_ITEM_LIST_LENGTH items;
  - Dataset.split_by... leave-one-out 'valid_and_test' per user:
    legal = min(2, count - 1) held-out samples at the end, last -> test.
"""
from collections import Counter, OrderedDict


def kcore(rows, min_user, min_item):
    rows = list(rows)
    while True:
        uc = Counter(r[0] for r in rows)
        ic = Counter(r[1] for r in rows)
        kept = [r for r in rows if uc[r[0]] >= min_user and ic[r[1]] >= min_item]
        if len(kept) == len(rows):
            return kept
        rows = kept


def remap(tokens):
    mp = OrderedDict()
    for t in tokens:
        if t not in mp:
            mp[t] = len(mp) + 1
    return mp


def prepare(rows, max_len, min_user=5, min_item=5):
    """rows: list of (user_token, item_token, timestamp) in file order.
    Returns (train, valid, test): lists of (user_id, item_id_list, target)."""
    rows = kcore(rows, min_user, min_item)
    umap = remap([r[0] for r in rows])
    imap = remap([r[1] for r in rows])
    per_user = OrderedDict()
    for n, (u, i, t) in enumerate(rows):
        per_user.setdefault(umap[u], []).append((t, n, imap[i]))
    train, valid, test = [], [], []
    for u in sorted(per_user):
        seq = [i for _, _, i in sorted(per_user[u])]
        samples = [(u, seq[max(0, k - max_len):k], seq[k]) for k in range(1, len(seq))]
        legal = min(2, len(samples) - 1) if samples else 0
        pr = len(samples) - legal
        train.extend(samples[:pr])
        held = samples[pr:]
        if legal == 2:
            valid.append(held[0])
            test.append(held[1])
        elif legal == 1:
            test.append(held[0])
    return train, valid, test, len(imap) + 1, len(umap) + 1
