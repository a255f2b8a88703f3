"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py: Triton-interpreter scan + reference RecBLR)."""
import pytest
import torch

from conftest import load_golden
from oracle import recblr_oracle as orc


def close(a, b, atol=1e-5, rtol=1e-5, what=""):
    err = (a.detach() - b.detach()).abs()
    assert bool((err <= atol + rtol * b.abs()).all()), f"{what}: {err.max().item():.3e}"


@pytest.mark.parametrize("idx", range(6))
def test_oracle_scan_matches_reference(idx):
    case = load_golden("scan_golden.pt")[idx]
    g = case["gates"].clone().requires_grad_()
    x = case["tokens"].clone().requires_grad_()
    s = orc.oracle_parallel_scan(g, x)
    s.backward(case["grad"])
    # the Triton interpreter evaluates the associative scan in serial order:
    # bit-identical to the serial oracle
    assert torch.equal(s, case["states"])
    assert torch.equal(g.grad, case["d_gates"])
    assert torch.equal(x.grad, case["d_tokens"])


@pytest.mark.parametrize("idx", range(9))
def test_oracle_grl_matches_reference(idx):
    case = load_golden("grl_golden.pt")[idx]
    params = {k: v.clone().requires_grad_() for k, v in case["params"].items()}
    x = case["x"].clone().requires_grad_()
    y = orc.grl_forward(params, "", x, case["disable_conv1d"])
    (y * case["gy"]).sum().backward()
    close(y, case["y"], what="y")
    close(x.grad, case["dx"], what="dx")
    for n, g in case["grads"].items():
        close(params[n].grad, g, what=n, rtol=1e-4)


@pytest.mark.parametrize("idx", range(6))
def test_oracle_model_matches_reference(idx):
    case = load_golden("model_golden.pt")[idx]
    params = {k: v.clone().requires_grad_(v.dtype.is_floating_point)
              for k, v in case["init_state"].items()}
    loss = orc.calculate_loss(params, case["cfg"], case["item_seq"], case["item_seq_len"],
                              case["pos_items"], case["neg_items"])
    loss.backward()
    close(loss, case["loss"], what="loss")
    for n, g in case["grads"].items():
        close(params[n].grad, g, what=n, atol=1e-5, rtol=1e-4)
    with torch.no_grad():
        close(orc.model_forward(params, case["cfg"], case["item_seq"], case["item_seq_len"]),
              case["seq_output"], what="seq_output")
        close(orc.full_sort_predict(params, case["cfg"], case["item_seq"], case["item_seq_len"]),
              case["full_sort"], what="full_sort")
        close(orc.predict(params, case["cfg"], case["item_seq"], case["item_seq_len"],
                          case["pos_items"]), case["predict"], what="predict")
