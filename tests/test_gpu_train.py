"""Real-data path end to end on the GPU: atomic file -> sequential splits ->
HBM-resident batches -> RecBLR training (fused kernels) -> full-sort
evaluation; plus the evaluator against an explicit score-matrix ranking."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _toy_atomic(tmp_path, cuda):
    from datamining_recblr_amd import data as dp

    g = np.random.default_rng(0)
    users, items, ts = [], [], []
    for u in range(400):            # each user walks a noisy cycle over 60 items
        n = int(g.integers(6, 30))
        s = int(g.integers(0, 60))
        for k in range(n):
            users.append(f"u{u}")
            items.append(f"i{(s + k + int(g.random() < 0.1)) % 60}")
            ts.append(float(k))
    path = str(tmp_path / "toy.inter")
    dp.write_atomic(path, {"user_id": np.array(users, dtype=object),
                           "item_id": np.array(items, dtype=object), "timestamp": np.array(ts)})
    return dp.from_atomic_file(path, max_len=20).to(cuda)


def test_fit_on_synthetic_atomic_file(cuda, tmp_path):
    from datamining_recblr_amd import data as dp
    from datamining_recblr_amd.distributed import DistEnv
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset
    from datamining_recblr_amd.trainer import evaluate_split, fit

    d = _toy_atomic(tmp_path, cuda)
    cfg = {"hidden_size": 32, "loss_type": "CE", "num_layers": 2, "dropout_prob": 0.1,
           "expand": 2, "d_conv": 4, "bd_lru_only": False, "disable_conv1d": False,
           "disable_ffn": False, "MAX_ITEM_LIST_LENGTH": 20}
    torch.manual_seed(0)
    model = RecBLR(cfg, SyntheticDataset(d.n_items, d.n_users)).to(cuda)
    env = DistEnv()
    before = evaluate_split(model, d, "valid", env)
    res = fit(model, d, env, epochs=8, batch_size=256, lr=3e-3, log=None)
    losses = [h["train_loss"] for h in res["history"]]
    assert losses[-1] < losses[0]
    assert res["best_valid"] > before["ndcg@10"] + 0.1     # the cycle is learnable
    assert 0.0 <= res["test"]["hit@10"] <= 1.0
    # evaluator == ranking an explicit score matrix (item 0 masked)
    m = evaluate_split(model, d, "test", env, topk=(10,))
    batch = dp.build_batch(d, d.test)
    with torch.no_grad():
        model.eval()
        sc = model.full_sort_predict(batch)
    sc[:, 0] = -float("inf")
    hit = (sc.topk(10, dim=1).indices == batch["item_id"][:, None]).any(1).double().mean()
    assert abs(m["hit@10"] - hit.item()) < 1e-9


def test_fit_native_adam_matches_torch_adam(cuda, tmp_path, monkeypatch):
    """trainer.fit with the native Adam (default) and with torch.optim.Adam
    (RECBLR_ADAM=torch): the same parameters after two epochs of training
    (fp32 round-off of the same update formula only; dropout off)."""
    from datamining_recblr_amd import optim
    from datamining_recblr_amd.distributed import DistEnv
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.recbole_compat import SyntheticDataset
    from datamining_recblr_amd.trainer import fit

    d = _toy_atomic(tmp_path, cuda)
    cfg = {"hidden_size": 32, "loss_type": "CE", "num_layers": 2, "dropout_prob": 0.0,
           "expand": 2, "d_conv": 4, "bd_lru_only": False, "disable_conv1d": False,
           "disable_ffn": False, "MAX_ITEM_LIST_LENGTH": 20}
    made = []
    orig = optim.make_adam
    monkeypatch.setattr(optim, "make_adam", lambda *a, **k: made.append(orig(*a, **k)) or made[-1])
    models = []
    for kind in ("native", "torch"):
        monkeypatch.setenv("RECBLR_ADAM", kind)
        torch.manual_seed(0)
        m = RecBLR(cfg, SyntheticDataset(d.n_items, d.n_users)).to(cuda)
        fit(m, d, DistEnv(), epochs=2, batch_size=256, lr=3e-3, log=None)
        models.append(m)
    assert isinstance(made[0], optim.Adam) and type(made[1]) is torch.optim.Adam, made
    for (n, a), b in zip(models[0].named_parameters(), models[1].parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5, msg=n)
