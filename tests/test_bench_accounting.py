"""bench.py's kernel accounting (CPU, no GPU touched).

Every C-ABI launch is timed under its name with an algorithmic amount: HBM
bytes, or FLOPs for the MFMA kernels listed in kernels.FLOP_KERNELS.  A launch
counted in FLOPs but missing from that set would be reported as bytes per
second (round 3's rb_item_ce_probs_h_both at "12.5x" of 8 TB/s); these tests
tie the two together statically and check the report on a synthetic summary."""
import ast
import glob
import os

from datamining_recblr_amd import kernels

from test_bench_launch import _import_bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch_calls():
    """(file, line, kernel name, counted in FLOPs) for every _launch("...")."""
    out = []
    for path in glob.glob(os.path.join(ROOT, "datamining_recblr_amd", "*.py")):
        tree = ast.parse(open(path).read(), path)
        for node in ast.walk(tree):
            if not (isinstance(node, ast.Call) and getattr(node.func, "id", None) == "_launch"):
                continue
            flops = any(k.arg == "_flops" and isinstance(k.value, ast.Constant) and k.value.value
                        for k in node.keywords)
            name = node.args[0].value if isinstance(node.args[0], ast.Constant) else None
            out.append((os.path.basename(path), node.lineno, name, flops))
    return out


def test_flop_counted_launches_are_exactly_flop_kernels():
    calls = _launch_calls()
    assert len(calls) > 20
    # names built at run time (dtype suffixes) are byte-counted HBM kernels
    assert not [c for c in calls if c[2] is None and c[3]]
    calls = [c for c in calls if c[2] is not None]
    flop_names = {n for _, _, n, f in calls if f}
    byte_names = {n for _, _, n, f in calls if not f}
    assert not flop_names & byte_names, "a kernel counted both ways"
    assert flop_names == set(kernels.FLOP_KERNELS), (flop_names ^ set(kernels.FLOP_KERNELS))
    for name in flop_names:
        assert name.startswith("rb_item_"), name


def test_f16_split_kernel_names():
    for n in ("rb_item_ce_fwd_h", "rb_item_ce_probs_h", "rb_item_ce_probs_h_t",
              "rb_item_ce_probs_h_both"):
        assert kernels.f16_split_kernel(n), n
    for n in ("rb_item_ce_fwd", "rb_item_rank", "rb_item_scores", "rb_gate_scan_bwd"):
        assert not kernels.f16_split_kernel(n), n


def _entry(launches, avg_ms, amount):
    return {"launches": launches, "ms": launches * avg_ms, "bytes": launches * amount,
            "avg_ms": avg_ms, "avg_bytes": amount}


def test_kernel_report_units_and_no_fraction_above_one():
    b = _import_bench()
    steps, ntok, H, layers = 10, 204_000, 256, 2
    N = ntok * H * 4
    summ = {
        "rb_gate_scan_bwd": _entry(20, 0.346, 8.5 * N),
        "rb_gate_scan_fwd": _entry(20, 0.154, 4.5 * N),
        "rb_conv_silu_fwd": _entry(20, 0.075, 2 * N),
        "rb_conv_silu_bwd": _entry(20, 0.160, 4 * N),
        "rb_item_ce_probs_h_both": _entry(10, 0.055, 2 * 2048 * 10544 * 128),
        "rb_item_ce_fwd_h": _entry(10, 0.047, 2 * 2048 * 10544 * 128),
    }
    rep = b.kernel_report(summ, steps, ntok, H, layers)
    assert "anomalies" not in rep
    both = rep["rb_item_ce_probs_h_both"]
    assert "achieved_tflops" in both and "achieved_gbs" not in both
    assert abs(both["peak_tflops"] - b.F16X3_PEAK_TFS) < 0.1
    for name, r in rep.items():
        if "achieved_gbs" in r:
            assert r["frac"] <= 1.0, (name, r)
    path = rep["scan_conv_gate_path"]
    assert path["model_bytes_per_step"] == int(20 * N * layers)
    assert 0 < path["model_frac"] < 1
    # a FLOP count reported as bytes is flagged
    bad = dict(summ, rb_gate_scan_bwd=_entry(20, 0.01, 2 * 2048 * 10544 * 128))
    assert b.kernel_report(bad, steps)["anomalies"] == ["rb_gate_scan_bwd"]
