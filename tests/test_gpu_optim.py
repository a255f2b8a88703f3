"""rb_adam_step (datamining_recblr_amd.optim.Adam) against torch.optim.Adam
— the training loop's optimizer (run.py: RecBole's Trainer, learner 'adam')
— over tensors of every size class the encoder has (odd tails included),
with and without L2 weight decay, parameters without gradients skipped."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wd", [0.0, 1e-4])
def test_adam_matches_torch(cuda, wd):
    from datamining_recblr_amd.optim import Adam

    g = torch.Generator().manual_seed(3)
    shapes = [(10544, 128), (512, 128), (256,), (4, 256), (7,), (1,), (1023,), (3, 5)]
    base = [torch.randn(s, generator=g) for s in shapes]
    ours = [torch.nn.Parameter(t.clone().to(cuda)) for t in base]
    ref = [torch.nn.Parameter(t.clone().to(cuda)) for t in base]
    skip = torch.nn.Parameter(torch.randn(64, generator=g).to(cuda))   # never gets a grad
    o1 = Adam(ours + [skip], lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)
    o2 = torch.optim.Adam(ref, lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd)
    before = skip.detach().clone()
    for step in range(5):
        for a, b in zip(ours, ref):
            gr = torch.randn(a.shape, generator=g).to(cuda) * (10.0 ** (step - 2))
            a.grad, b.grad = gr.clone(), gr.clone()
        o1.step()
        o2.step()
    # fp32 round-off of the same formula (torch's foreach kernels order a few
    # products differently): parameters of magnitude ~1 moved by ~1e-2 per
    # step agree to a few ulps of 1
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(o1.state[a]["exp_avg_sq"], o2.state[b]["exp_avg_sq"],
                                   rtol=1e-5, atol=0)
    assert torch.equal(skip, before)
    assert o1.state[ours[0]]["step"] == 5


def test_adam_in_a_training_step_matches_torch(cuda):
    """Three RecBLR train steps with the native Adam == with torch's fused
    Adam (fp32 round-off only)."""
    from datamining_recblr_amd.model import RecBLR
    from datamining_recblr_amd.optim import Adam
    from datamining_recblr_amd.distributed import synthetic_interaction
    from datamining_recblr_amd.recbole_compat import SyntheticDataset

    cfg = dict(hidden_size=64, loss_type="CE", num_layers=2, dropout_prob=0.0, expand=2,
               d_conv=4, bd_lru_only=False, disable_conv1d=False, disable_ffn=False,
               MAX_ITEM_LIST_LENGTH=50)
    models, opts = [], []
    for mk in (Adam, lambda ps, lr: torch.optim.Adam(ps, lr=lr, fused=True)):
        torch.manual_seed(0)
        m = RecBLR(cfg, SyntheticDataset(500)).to(cuda).train()
        models.append(m)
        opts.append(mk(m.parameters(), lr=1e-3))
    batches = [synthetic_interaction(64, 50, 500, cuda, seed=i) for i in range(3)]
    for b in batches:
        for m, o in zip(models, opts):
            o.zero_grad(set_to_none=True)
            m.calculate_loss(b).backward()
            o.step()
    for (n, a), b in zip(models[0].named_parameters(), models[1].parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=n)
